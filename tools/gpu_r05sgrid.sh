#!/bin/bash
# GPU box: the statistics kernel's grid cap (USV_STATS_GRID) against the rollout, at the default bench length and
# late in training (93 epochs).   GRIDS="4096 1024 512"
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05sgrid; mkdir -p $O
cd $R
B="--no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
for rep in ${REPS:-1}; do
for g in ${GRIDS:-4096 1024 512 256}; do
  for len in 20 90; do
    USV_STATS_GRID=$g timeout -k 10 300 python3 bench.py --steps $len --warmup 3 $B > $O/g$g.$len.$rep.json 2> $O/g$g.$len.$rep.err || { tail -3 $O/g$g.$len.$rep.err; exit 1; }
    python3 - $O/g$g.$len.$rep.json $g $len $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("grid %5s epochs %3s rep %s value %.3fM rollout %.2f ms update %.2f ms device-only rollout %.2f ms" % (
    sys.argv[2], sys.argv[3], sys.argv[4], d["value"] / 1e6, e["rollout_ms"], e["update_ms"], e["device_only"]["rollout_ms"]))
PY
  done
done
done
