#!/bin/bash
# GPU box: statistics-kernel variants late in training -- rocprofv3 kernel trace of a 93-epoch bench with the
# sequential step (USV_STEP_OVERLAP=0), k_field_stats dispatch medians early / mid / late, per library variant;
# then the overlapped bench's rollout per variant.   VARIANTS="base pipe pipe5 lds5"
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05statslate; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="--steps 90 --warmup 3 --no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0"
for v in $VARIANTS; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_HIP_LIB=$lib USV_STEP_OVERLAP=0 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/raw_$v -o t -- python3 $R/bench.py $B > $O/$v.seq.json 2> $O/$v.seq.err || { tail -3 $O/$v.seq.err; exit 1; }
  python3 - $O/raw_$v $v <<'PY'
import csv, glob, statistics, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_field_stats" in r["Kernel_Name"]]
segs = [("epochs ~4-7", d[48:112]), ("~21-24", d[320:384]), ("~90-93", d[-64:])]
print("%-6s k_field_stats sequential medians: " % sys.argv[2] + " | ".join("%s %.1f us" % (n, statistics.median(s)) for n, s in segs))
PY
  rm -rf $O/raw_$v
done
cd $R
for v in $VARIANTS; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_HIP_LIB=$lib timeout -k 10 300 python3 bench.py $B > $O/$v.json 2> $O/$v.err || { tail -3 $O/$v.err; exit 1; }
  python3 - $O/$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("%-6s overlapped 90 epochs value %.3fM rollout %.2f ms device-only rollout %.2f ms" % (
    sys.argv[2], d["value"] / 1e6, e["rollout_ms"], e["device_only"]["rollout_ms"]))
PY
done
