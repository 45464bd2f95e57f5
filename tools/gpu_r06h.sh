#!/bin/bash
# r06h: the exact branch-free quaternion scale -- parity (env replays / oracle tests), then the env step A/B against
# the IEEE division (variant lib), interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06h
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_env_gpu.py \
  tests/test_overlap_gpu.py tests/test_headline_gpu.py tests/test_ppo_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -2 $O/pytest.log
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_exact.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_div.so timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_div.txt 2>&1 || exit $?
done
grep -h envs $O/ab_exact.txt $O/ab_div.txt
