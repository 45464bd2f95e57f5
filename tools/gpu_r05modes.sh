#!/bin/bash
# GPU box: rollout step orderings at the default bench length and late in training (93 epochs):
# overlapped (default) / sequential step (USV_STEP_OVERLAP=0) / policy after the statistics (USV_STATS_FIRST=1)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05modes; mkdir -p $O
cd $R
B="--no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
for rep in ${REPS:-1}; do
for m in base:X=0 seq:USV_STEP_OVERLAP=0 statsfirst:USV_STATS_FIRST=1; do
  name=${m%%:*}; kv=${m#*:}
  for len in 20 90; do
    env $kv timeout -k 10 300 python3 bench.py --steps $len --warmup 3 $B > $O/$name.$len.$rep.json 2> $O/$name.$len.$rep.err || { tail -3 $O/$name.$len.$rep.err; exit 1; }
    python3 - $O/$name.$len.$rep.json $name $len $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("%-10s epochs %3s rep %s value %.3fM rollout %.2f ms update %.2f ms device-only rollout %.2f ms" % (
    sys.argv[2], sys.argv[3], sys.argv[4], d["value"] / 1e6, e["rollout_ms"], e["update_ms"], e["device_only"]["rollout_ms"]))
PY
  done
done
done
