#!/bin/bash
# GPU box: kernel trace of a short bench run (graph replays included) for timeline/gap analysis
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/trace_${TAG:-x}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 ${BENCH_ARGS:-} > $O/bench.log 2>&1
rc=$?
tail -2 $O/bench.log
ls $O
exit $rc
