#!/bin/bash
# r06o: the exactness fallback inside the sweep kernels (no k_field_exact launch) -- field parity in all three sweep
# kernels, the overlapped step, then the rollout timeline and the headline against the previous commit's library
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06o
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_env_gpu.py \
  tests/test_overlap_gpu.py tests/test_headline_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
    --milestone-seconds 0 > $O/bench_new.$rep.json 2> $O/bench_new.$rep.err || exit $?
  USV_HIP_LIB=libusv_hip_prev.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_prev.$rep.json 2> $O/bench_prev.$rep.err || exit $?
done
bash tools/gpu_r06n.sh > $O/timeline.log 2>&1 || exit $?
