#!/bin/bash
# r06ze: USV_LATE_ON_JOIN=0 vs 1 at 4,096 envs (BASELINE configs[1]), interleaved, 5 reps
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06ze
mkdir -p $O
cd $R
for rep in 1 2 3 4 5; do
  for v in 0 1; do
    USV_LATE_ON_JOIN=$v timeout -k 10 240 python3 bench.py --envs 4096 --steps 30 --warmup 5 --seeds 0 --no-cpu-baseline \
      --c2-steps 0 --extra-steps 0 --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('late_on_join=$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
