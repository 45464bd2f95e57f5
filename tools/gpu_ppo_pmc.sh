#!/bin/bash
# GPU box: PMC passes (one counter group per run) on the PPO update kernels of a short bench:
# FETCH_SIZE, WRITE_SIZE, TCC_HIT_sum + TCC_MISS_sum.     TAG=r03f bash tools/gpu_ppo_pmc.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03f}
O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 1 --warmup 1 --no-graph --no-cpu-baseline --c2-steps 0 --milestone-seconds 0"
RX=${RX:-k_mb_grad|k_reduce_partials|k_policy_step}
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $O -o p$i -- python3 $B > $O/p$i.log 2>&1 || { tail $O/p$i.log; exit 1; }
  echo "pass $i ($P) done"
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(o + "/p*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()}, "n=", {c: len(v) for c, v in d.items()})
PY
