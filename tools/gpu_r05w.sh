set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05w
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r05w/raw -o tl -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0 > $R/gpurun_out/r05w/bench.log 2>&1 || exit 1
f=$(ls $R/gpurun_out/r05w/raw/*kernel_trace.csv $R/gpurun_out/r05w/raw/*/*kernel_trace.csv 2>/dev/null | head -1)
python3 $R/tools/rollout_timeline.py $f $R/gpurun_out/r05w/timeline.csv > $R/gpurun_out/r05w/summary.txt 2>&1; rc=$?
rm -rf $R/gpurun_out/r05w/raw
cat $R/gpurun_out/r05w/summary.txt; exit $rc
