#!/bin/bash
# r06t: tanh as 1 - 2 / (exp(2x) + 1) in the PPO kernels -- PPO parity (reference fixtures, oracle, headline), then
# policy standalone and the headline against the previous commit's library (the odd form), interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06t
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ppo_gpu.py \
  tests/test_headline_gpu.py tests/test_train_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/policy_step_probe.py 131072 new >> $O/probe.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_prev.so timeout -k 10 120 python3 tools/policy_step_probe.py 131072 prev >> $O/probe.txt 2>&1 || exit $?
done
grep envs $O/probe.txt
for rep in 1 2 3; do
  timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
    --milestone-seconds 0 > $O/bench_new.$rep.json 2> $O/bench_new.$rep.err || exit $?
  USV_HIP_LIB=libusv_hip_prev.so timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
    --c2-steps 0 --milestone-seconds 0 > $O/bench_prev.$rep.json 2> $O/bench_prev.$rep.err || exit $?
done
