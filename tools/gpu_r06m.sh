#!/bin/bash
# r06m: ppo_value in the register-weight form -- bit identity with the LDS-staged form, value vs oracle, per-kernel
# durations (k_value, k_gae) and the headline against the previous commit's library, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06m
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_headline_gpu.py \
  -k "value or gae or prepare" > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
CASES="new:USV_HIP_LIB= prev:USV_HIP_LIB=libusv_hip_prev.so" KERNELS="k_value k_gae k_prepare_apply k_policy_step" \
  bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
cat $O/kmed.txt
for rep in 1 2; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
    --milestone-seconds 0 > $O/bench_new.$rep.json 2> $O/bench_new.$rep.err || exit $?
  USV_HIP_LIB=libusv_hip_prev.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_prev.$rep.json 2> $O/bench_prev.$rep.err || exit $?
done
