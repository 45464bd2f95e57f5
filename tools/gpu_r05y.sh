set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05y; mkdir -p $O
cd $R
REPS=2 VARIANTS="base noexp" BENCH_ARGS="--extra-steps 0" timeout -k 10 700 bash tools/gpu_variants.sh > $O/ab.txt 2>&1 || { cat $O/ab.txt; exit 1; }
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp
for v in base noexp; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_STEP_OVERLAP=0 USV_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o t -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 --extra-steps 0 > $O/prof_$v.log 2>&1 || exit 1
  python3 - "$O/prof_$v/t_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_policy_step" in r["Name"] or "k_env_step<true, false, false" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], "calls", r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
  rm -rf $O/prof_$v
done
