#!/bin/bash
# GPU box: the XCD-group fold A/B -- the headline bench with USV_PPO_FOLD=1 / 0 interleaved (REPS x), then one
# rocprofv3 kernel-stats pass per mode (k_mb_grad / k_reduce_partials means).   TAG=r04c bash tools/gpu_fold_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-r04c}
O=gpurun_out/$TAG/fold_ab
mkdir -p $O
export TMPDIR=/tmp
[ "${SKIP_BENCH:-0}" = "1" ] || CASES="fold1:USV_PPO_FOLD=1 fold0:USV_PPO_FOLD=0" REPS=${REPS:-2} STEPS=${STEPS:-10} bash tools/gpu_envvar_ab.sh || exit $?
cp gpurun_out/envvar_ab/fold*.json $O/ 2>/dev/null
for f in 1 0; do
  USV_PPO_FOLD=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof$f -o k -- \
    python3 bench.py --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 --steps 4 --warmup 2 > $O/prof$f.log 2>&1 || exit $?
  s=$(find $O/prof$f -name '*kernel_stats.csv' | head -1)
  python3 - "$s" $f <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if any(k in r["Name"] for k in ("k_mb_grad", "k_reduce_partials", "k_apply")):
        print("fold%s" % sys.argv[2], r["Name"][:60], "calls", r["Calls"], "mean_us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
done
for f in 1 0; do
  USV_PPO_FOLD=$f timeout -k 10 240 python3 tools/phase_probe.py 131072 > $O/probe$f.log 2>&1 || exit $?
  echo "== probe fold$f"; grep -A30 "k_mb_grad" $O/probe$f.log | head -24
done
