#!/bin/bash
# r06r: sweeps start from the seeded tiles only (the others wait for the front) -- field parity, then per-kernel
# durations and the headline against the previous commit's library, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06r
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_gpu.py \
  tests/test_overlap_gpu.py tests/test_headline_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
CASES="new:USV_HIP_LIB= prev:USV_HIP_LIB=libusv_hip_prev.so" KERNELS="k_field_wave_pack k_field_stats k_env_step k_policy_step" \
  bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
cat $O/kmed.txt
for rep in 1 2 3; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
    --milestone-seconds 0 > $O/bench_new.$rep.json 2> $O/bench_new.$rep.err || exit $?
  USV_HIP_LIB=libusv_hip_prev.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_prev.$rep.json 2> $O/bench_prev.$rep.err || exit $?
done
