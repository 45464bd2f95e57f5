#!/bin/bash
# GPU box: the overlapped rollout's kernel timeline late in training (the last graph-replayed epoch of a 93-epoch
# bench run, ~3,000 resets per step), as tools/gpu_r05w.sh does for the default run
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05late
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05late/raw -o tl -- python3 $R/bench.py --steps 90 --warmup 3 --no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0 > $R/gpurun_out/r05late/bench.json 2> $R/gpurun_out/r05late/bench.err || { tail -5 $R/gpurun_out/r05late/bench.err; exit 1; }
f=$(ls $R/gpurun_out/r05late/raw/*kernel_trace.csv $R/gpurun_out/r05late/raw/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/rollout_timeline.py $f $R/gpurun_out/r05late/timeline.csv > $R/gpurun_out/r05late/summary.txt 2>&1; rc=$?
rm -rf $R/gpurun_out/r05late/raw
cat $R/gpurun_out/r05late/summary.txt; tail -c 600 $R/gpurun_out/r05late/bench.json; exit $rc
