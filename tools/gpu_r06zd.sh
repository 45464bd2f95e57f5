#!/bin/bash
# r06zd (repeat of r06zc, order reversed, 5 reps): the deferred reward on the side stream behind part 3 (USV_LATE_ON_JOIN=0) vs on the joining stream (1), with the round-6 schedule
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zd
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_overlap_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2 3 4 5; do
  for v in late base; do
    if [ $v = base ]; then e=USV_DUMMY=0; else e="USV_LATE_ON_JOIN=0"; fi
    env $e timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
