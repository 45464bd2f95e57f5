#!/bin/bash
# GPU box: PPO parity for the default build and the x3 variant, then the interleaved A/B + probe
set -uo pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_base.log 2>&1 || { tail -30 $O/pytest_base.log; exit 1; }
tail -1 $O/pytest_base.log
USV_HIP_LIB=x3.so timeout -k 10 400 python3 -u -m pytest tests/test_ppo_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_x3.log 2>&1; echo "x3 parity rc=$?"; tail -1 $O/pytest_x3.log
cp gpurun_out/parity_errors.json $O/parity_x3.json 2>/dev/null
VARIANTS="base sync0 prio0 x3 l2f0 l1f1" TAG=r05h bash tools/gpu_ab_probe.sh
