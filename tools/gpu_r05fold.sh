#!/bin/bash
# GPU box: monotone-fold k_field_stats -- field / env GPU tests, kernel stats of both builds (sequential and
# overlapped rollout), bench A/B against the per-cell build.   FULL=1: the whole GPU suite
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05fold; mkdir -p $O
cd $R
if [ -n "${FULL:-}" ]; then SEL="tests -m gpu"; else SEL="tests/test_env_gpu.py tests/test_headline_gpu.py -m gpu"; fi
timeout -k 10 900 python3 -u -m pytest $SEL -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
CASES="fold_seq:USV_HIP_LIB=,USV_STEP_OVERLAP=0 nofold_seq:USV_HIP_LIB=nofold.so,USV_STEP_OVERLAP=0 fold:USV_HIP_LIB= nofold:USV_HIP_LIB=nofold.so" TOP=12 bash tools/gpu_kstats_ab.sh > $O/kstats.txt 2>&1; rc=$?
grep -E "==|k_field_stats|k_field_wave_pack|k_policy_step" $O/kstats.txt | grep -v '^"'; rm -rf $R/gpurun_out/kstats_ab; [ $rc -ne 0 ] && exit $rc
[ -n "${NOAB:-}" ] && exit 0
SKIP_TESTS=1 LIB_B=nofold.so bash tools/gpu_ab.sh > $O/ab.txt 2>&1; rc=$?; cat $O/ab.txt; exit $rc
