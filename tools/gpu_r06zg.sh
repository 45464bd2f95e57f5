#!/bin/bash
# r06zg: the chained step's reset and placement on the side stream (USV_RESET_ON_SIDE=1) with its field kernels
# captured right behind them (side first), vs the defaults; overlap tests, headline interleaved, then its timeline
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zg
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_overlap_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
for rep in 1 2 3 4; do
  for v in base side; do
    if [ $v = base ]; then e=USV_DUMMY=0; else e="USV_RESET_ON_SIDE=1"; fi
    env $e timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
cd /tmp && export TMPDIR=/tmp
export USV_RESET_ON_SIDE=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o t -- python3 $R/bench.py --steps 6 --extra-steps 0 \
  --warmup 2 --seeds 0 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/bench_trace.log 2>&1 || exit $?
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 $R/tools/rollout_timeline.py "$f" $O/rollout_timeline.csv > $O/rollout_timeline.txt 2>&1 || exit $?
rm -rf $O/tr
tail -20 $O/rollout_timeline.txt
