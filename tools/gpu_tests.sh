#!/bin/bash
# GPU box: a pytest selection (TESTS, default the whole GPU suite) then, unless BENCH=0, a short bench
# line without the CPU baseline.     TESTS="tests/test_x.py -k y" TAG=r03a bash tools/gpu_tests.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 ${PYTEST_TIMEOUT:-900} python3 -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
cp gpurun_out/parity_errors.json $O/ 2>/dev/null
[ $rc -ne 0 ] && exit $rc
if [ "${BENCH:-1}" != "0" ]; then
  timeout -k 10 600 python3 bench.py --no-cpu-baseline --steps ${STEPS:-10} ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err
  rc=$?
  tail -2 $O/bench.err
  python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['extra'].get('update_us_per_minibatch'),d['roofline']['frac'],d['roofline_ppo']['frac'])"
fi
exit $rc
