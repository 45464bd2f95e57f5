set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05t
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_headline_gpu.py tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_overlap_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05t/pytest.log 2>&1 || { tail -30 gpurun_out/r05t/pytest.log; exit 1; }
tail -2 gpurun_out/r05t/pytest.log
REPS=3 VARIANTS="base pol32" BENCH_ARGS="--extra-steps 0" timeout -k 10 900 bash tools/gpu_variants.sh > gpurun_out/r05t/ab.txt 2>&1 || { cat gpurun_out/r05t/ab.txt; exit 1; }
cat gpurun_out/r05t/ab.txt
cd /tmp && export TMPDIR=/tmp
for v in base pol32; do
  lib=""; [ "$v" != "base" ] && lib="$v.so"
  USV_STEP_OVERLAP=0 USV_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05t/prof_$v -o t -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 --extra-steps 0 > $R/gpurun_out/r05t/prof_$v.log 2>&1 || exit 1
  python3 - "$R/gpurun_out/r05t/prof_$v/t_kernel_stats.csv" $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_policy_step" in r["Name"]:
        print(sys.argv[2], "k_policy_step calls", r["Calls"], "avg_us %.2f" % (float(r["AverageNs"]) / 1e3))
PY
  cp $R/gpurun_out/r05t/prof_$v/t_kernel_stats.csv $R/gpurun_out/r05t/stats_$v.csv; rm -rf $R/gpurun_out/r05t/prof_$v
done
