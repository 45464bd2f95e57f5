#!/bin/bash
# r06u: the gradient kernel's exp(log-sigma) hoisted out of the losses and its KL / entropy / bound terms on wave 7
# during the backward (new) vs the hoist alone (kl0) vs the previous commit (prev) -- PPO parity, headline interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06u
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ppo_gpu.py \
  tests/test_headline_gpu.py tests/test_train_gpu.py tests/test_dist_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2 3; do
  for v in new kl0 prev; do
    if [ $v = new ]; then L=; else L=libusv_hip_$v.so; fi
    USV_HIP_LIB=$L timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
  done
done
