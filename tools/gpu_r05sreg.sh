#!/bin/bash
# GPU box: k_field_stats register budget -- env GPU tests on the default build, kernel stats (sequential step) of
# the variants, bench A/B of LIB_B against the default
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05sreg; mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_env_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
CASES="${CASES:-lds:USV_HIP_LIB=,USV_STEP_OVERLAP=0 reg:USV_HIP_LIB=regobst.so,USV_STEP_OVERLAP=0 w5:USV_HIP_LIB=w5.so,USV_STEP_OVERLAP=0 w6:USV_HIP_LIB=w6.so,USV_STEP_OVERLAP=0}" TOP=12 bash tools/gpu_kstats_ab.sh > $O/kstats.txt 2>&1; rc=$?
grep -E "==|k_field_stats|k_policy_step" $O/kstats.txt | grep -v '^"'; rm -rf $R/gpurun_out/kstats_ab; [ $rc -ne 0 ] && exit $rc
[ -z "${LIB_B:-}" ] && exit 0
SKIP_TESTS=1 bash tools/gpu_ab.sh > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
