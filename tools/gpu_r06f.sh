#!/bin/bash
# r06f: the register-weight policy kernel -- bit identity with the LDS-staged form, standalone timing (variants: 3 / 2
# workgroups per CU, no layer-2 fence), per-kernel medians in the overlapped bench and the headline, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06f
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_headline_gpu.py \
  -k "policy_step" tests/test_overlap_gpu.py > $O/pytest.log 2>&1 || exit $?
for rep in 1 2; do
  USV_POLICY_RW=0 timeout -k 10 120 python3 tools/policy_step_probe.py 131072 lds >> $O/probe.txt 2>&1 || exit $?
  timeout -k 10 120 python3 tools/policy_step_probe.py 131072 rw3 >> $O/probe.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_pol2.so timeout -k 10 120 python3 tools/policy_step_probe.py 131072 rw2 >> $O/probe.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_polnb.so timeout -k 10 120 python3 tools/policy_step_probe.py 131072 rw3nb >> $O/probe.txt 2>&1 || exit $?
done
CASES="rw:USV_POLICY_RW=1 lds:USV_POLICY_RW=0" KERNELS="k_policy_step k_field_stats k_field_wave_pack k_env_step" \
  bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 1 0; do
    USV_POLICY_RW=$v timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_rw$v.$rep.json 2> $O/bench_rw$v.$rep.err || exit $?
  done
  USV_HIP_LIB=libusv_hip_pol2.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_rw2.$rep.json 2> $O/bench_rw2.$rep.err || exit $?
done
