#!/bin/bash
# GPU box: env parity subset (field bit-exactness, fixture replays, Philox vs oracle) + a short bench
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/quick
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_env_gpu.py -x -q --timeout 200 --timeout-method thread \
  -k "${TEST_K:-field or fixture or philox_mode_matches}" > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
rc=$?
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['extra'])"
exit $rc
