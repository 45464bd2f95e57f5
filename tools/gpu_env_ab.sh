#!/bin/bash
# GPU box: env-step A/B of library variants in the sequential step (USV_STEP_OVERLAP=0: k_env_step alone on the
# GPU): rocprofv3 kernel-trace stats of a short bench per variant (twice, interleaved), plus one FETCH_SIZE pass
# each.   VARIANTS="base pf0" TAG=r05d bash tools/gpu_env_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-envab}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 --extra-steps 0"
export USV_STEP_OVERLAP=0
for rep in 1 2; do
  for v in $VARIANTS; do
    lib=""; [ "$v" != "base" ] && lib="$v.so"
    USV_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v.$rep -o t -- python3 $B > $O/$v.$rep.log 2>&1 || { tail $O/$v.$rep.log; exit 1; }
    python3 - "$O/$v.$rep/t_kernel_stats.csv" "$v" "$rep" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_env_step<" in r["Name"] and "FixedWin<19>" in r["Name"]:
        print(sys.argv[2], sys.argv[3], "k_env_step calls", r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
    rm -rf $O/$v.$rep   # traces stay on the box (the merge-back cap)
  done
done
for v in $VARIANTS; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_HIP_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_env_step --output-format csv -d $O/$v.fetch -o p -- python3 $B > $O/$v.fetch.log 2>&1 || { tail $O/$v.fetch.log; exit 1; }
  python3 - $O/$v.fetch "$v" <<'PY'
import csv, glob, sys
vals = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "FixedWin<19>" in r.get("Kernel_Name", ""):
            vals.append(float(r["Counter_Value"]))
if vals:
    print(sys.argv[2], "FETCH_SIZE per launch (x1024 x2) MB %.1f over %d" % (sum(vals) / len(vals) * 2048 / 1e6, len(vals)))
PY
  rm -rf $O/$v.fetch
done
