#!/bin/bash
# GPU box: full GPU test suite, then a short bench run (JSON line in gpurun_out/full/bench.json)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/full
mkdir -p $O
cd $R
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?
cat $O/bench.json
exit $rc
