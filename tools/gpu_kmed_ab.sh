#!/bin/bash
# GPU box: per-dispatch durations of chosen kernels under several builds / settings (rocprofv3 kernel trace of a
# short bench): median and mean over the dispatches below 1 ms (the steady-state steps; the all-env reset of the
# first epoch is excluded).   CASES="a:USV_HIP_LIB= b:USV_HIP_LIB=x.so" KERNELS="k_field_stats k_policy_step"
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/kmed; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in $CASES; do
  name=${c%%:*}; vars=${c#*:}
  for kv in ${vars//,/ }; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$name -o t -- python3 $R/bench.py \
    --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/$name.log 2>&1 || exit $?
  for kv in ${vars//,/ }; do unset "${kv%%=*}"; done
  python3 - "$O/$name" "$name" "${KERNELS:-k_field_stats}" <<'PY'
import csv, glob, statistics, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for k in sys.argv[3].split():
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if k in r["Kernel_Name"]]
    s = [x for x in d if x < 1000.0]
    if s:
        print("%-10s %-22s n %4d  steady n %4d  median %8.2f us  mean %8.2f us  p90 %8.2f us" % (
            sys.argv[2], k, len(d), len(s), statistics.median(s), statistics.mean(s), sorted(s)[int(0.9 * len(s))]))
PY
  rm -rf $O/$name
done
