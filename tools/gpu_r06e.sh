#!/bin/bash
# r06e: env-step memory-shape probe (pipelined variant); A/B of the quaternion's 2 / s (fast path vs IEEE division);
# the experience record layout (USV_EXP_REC): parity tests, per-kernel durations and the headline, interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/bin_envstep_mem_probe > $O/probe.txt 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_fast.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_divs.so timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_div.txt 2>&1 || exit $?
done
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ppo_gpu.py \
  tests/test_headline_gpu.py > $O/pytest.log 2>&1 || exit $?
CASES="rec:USV_EXP_REC=1 sep:USV_EXP_REC=0" KERNELS="k_policy_step k_mb_grad k_reduce_partials k_gae k_prepare_apply k_env_step" \
  bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 1 0; do
    USV_EXP_REC=$v timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_rec$v.$rep.json 2> $O/bench_rec$v.$rep.err || exit $?
  done
done
