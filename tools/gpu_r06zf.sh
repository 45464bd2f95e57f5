#!/bin/bash
# r06zf: rollout timeline with the round-6 schedule defaults
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o t -- python3 $R/bench.py --steps 6 --extra-steps 0 \
  --warmup 2 --seeds 0 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/bench.log 2>&1 || exit $?
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
python3 $R/tools/rollout_timeline.py "$f" $O/rollout_timeline.csv > $O/rollout_timeline.txt 2>&1 || exit $?
rm -rf $O/tr
tail -30 $O/rollout_timeline.txt
