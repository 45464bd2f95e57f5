#!/bin/bash
# GPU box: bench A/B of library variants (lib/<name>.so; base = lib/libusv_hip.so) at the default length and late in
# training (93 epochs), REPS reps, interleaved.   VARIANTS="base lds5"
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05libab; mkdir -p $O
cd $R
B="--no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
for rep in ${REPS:-1 2}; do
for v in $VARIANTS; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  for len in 20 90; do
    USV_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps $len --warmup 3 $B > $O/$v.$len.$rep.json 2> $O/$v.$len.$rep.err || { tail -3 $O/$v.$len.$rep.err; exit 1; }
    python3 - $O/$v.$len.$rep.json $v $len $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("%-6s epochs %3s rep %s value %.3fM rollout %.2f ms update %.2f ms device-only rollout %.2f ms" % (
    sys.argv[2], sys.argv[3], sys.argv[4], d["value"] / 1e6, e["rollout_ms"], e["update_ms"], e["device_only"]["rollout_ms"]))
PY
  done
done
done
