#!/bin/bash
# GPU box: env parity tests + env-step kernel timing at 4096 and 131072 envs
set -uo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/envcheck
cd $R
timeout -k 10 600 python3 -m pytest tests/test_env_gpu.py -x -q > $R/gpurun_out/envcheck/pytest.log 2>&1
rc=$?
tail -5 $R/gpurun_out/envcheck/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 tools/env_step_probe.py 4096 32 2>&1 | grep envs && \
timeout -k 10 200 python3 tools/env_step_probe.py 131072 32 2>&1 | grep envs
