#!/bin/bash
# GPU box: interleaved headline-bench A/B of library variants (tools/gpu_variants.sh), then the phase probe
# of the default build.   VARIANTS="base v1" TAG=r05c bash tools/gpu_ab_probe.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/${TAG:-ab}; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
  tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
BENCH_ARGS="${BENCH_ARGS:---steps 10 --milestone-seconds 0 --extra-steps 0}" bash tools/gpu_variants.sh 2>&1 | tee $O/ab.txt
rc=${PIPESTATUS[0]}; [ $rc -ne 0 ] && exit $rc
if [ "${PROBE:-1}" = "1" ]; then
  timeout -k 10 300 python3 tools/phase_probe.py 131072 > $O/probe.log 2>&1; rc=$?; sed -n 2,24p $O/probe.log; exit $rc
fi
