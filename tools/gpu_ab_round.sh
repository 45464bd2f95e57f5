#!/bin/bash
# GPU box: a pytest selection (TESTS), then the headline bench for each library variant in VARIANTS
# (interleaved, twice each: tools/gpu_variants.sh), then rocprofv3 kernel stats of a short bench of the
# default library (kernel means in $O/prof).     TAG=r03k TESTS="tests/test_ppo_gpu.py" VARIANTS="base old" bash tools/gpu_ab_round.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
if [ -n "${VARIANTS:-}" ]; then
  VARIANTS="$VARIANTS" BENCH_ARGS="${BENCH_ARGS:---steps 10 --milestone-seconds 0}" bash tools/gpu_variants.sh || exit $?
fi
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
  cd $R
  python3 tools/kstats.py $O/prof/trace_kernel_stats.csv 2>/dev/null | head -24 || true
fi
exit 0
