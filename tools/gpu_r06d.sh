#!/bin/bash
# r06d: env-step memory-shape probe (pipelined variant) + A/B of the quaternion's 2 / s (fast path vs IEEE division)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/bin_envstep_mem_probe > $O/probe.txt 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_fast.txt 2>&1 || exit $?
  USV_HIP_LIB=libusv_hip_divs.so timeout -k 10 120 python3 tools/env_step_probe.py 131072 48 >> $O/ab_div.txt 2>&1 || exit $?
done
