#!/bin/bash
# r06g: register-weight policy kernel at 2 workgroups per CU as the default build -- phase probe (per-tile phase
# sums), standalone timing, and the headline interleaved against the LDS-staged form and the 3-per-CU variant
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06g
mkdir -p $O
cd $R
timeout -k 10 300 python3 tools/phase_probe.py 131072 > $O/phase_probe.txt 2>&1 || exit $?
for rep in 1 2; do
  USV_POLICY_RW=0 timeout -k 10 120 python3 tools/policy_step_probe.py 131072 lds >> $O/probe.txt 2>&1 || exit $?
  timeout -k 10 120 python3 tools/policy_step_probe.py 131072 rw2 >> $O/probe.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_pol3.so timeout -k 10 120 python3 tools/policy_step_probe.py 131072 rw3 >> $O/probe.txt 2>&1 || exit $?
done
for rep in 1 2 3; do
  for v in 1 0; do
    USV_POLICY_RW=$v timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_rw$v.$rep.json 2> $O/bench_rw$v.$rep.err || exit $?
  done
  USV_HIP_LIB=libusv_hip_pol3.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_rw3.$rep.json 2> $O/bench_rw3.$rep.err || exit $?
done
