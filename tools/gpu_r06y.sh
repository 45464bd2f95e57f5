#!/bin/bash
# r06y: step n's reward store inside step n + 1 after the fields' fork (USV_STORE_DEFER=1, new default) vs after
# each join (0): the overlapped-step / training tests, then the headline interleaved (rollout_ms is the quantity)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06y
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_overlap_gpu.py \
  tests/test_train_gpu.py tests/test_headline_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2 3 4; do
  for v in 1 0; do
    USV_STORE_DEFER=$v timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline \
      --c2-steps 0 --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('store_defer=$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
