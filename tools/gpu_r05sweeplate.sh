#!/bin/bash
# GPU box: sweep / statistics kernel durations over a 93-epoch bench run with the sequential step
# (USV_STEP_OVERLAP=0: no kernel beside them), early vs late dispatches (rocprofv3 kernel trace)
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05sweeplate; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
USV_STEP_OVERLAP=0 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/raw -o t -- python3 $R/bench.py --steps 90 --warmup 3 --no-cpu-baseline --c2-steps 0 --extra-steps 0 --milestone-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
python3 - $O/raw <<'PY'
import csv, glob, statistics, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for k in ("k_field_wave_pack", "k_field_stats", "k_field_place", "k_env_step<", "k_policy_step", "k_reset"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if k in r["Kernel_Name"]]
    if len(d) < 200:
        continue
    segs = [("dispatches 48-111 (epochs ~4-7)", d[48:112]), ("dispatches 320-383 (~epoch 21-24)", d[320:384]),
            ("last 64 (~epochs 90-93)", d[-64:])]
    print(k, " | ".join("%s median %.1f us" % (n, statistics.median(s)) for n, s in segs))
PY
rm -rf $O/raw
