#!/bin/bash
# r06v: the multitask peer == collective identity with the new tanh (twice) and with the odd-form tanh (variant lib)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06v
mkdir -p $O
cd $R
T=tests/test_multitask_gpu.py
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread $T > $O/new1.log 2>&1; echo "new1 rc $?"
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread $T > $O/new2.log 2>&1; echo "new2 rc $?"
USV_HIP_LIB=libusv_hip_odd.so timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread $T > $O/odd.log 2>&1; echo "odd rc $?"
grep -h "PASSED\|FAILED" $O/new1.log $O/new2.log $O/odd.log | grep -v "^FAILED"
