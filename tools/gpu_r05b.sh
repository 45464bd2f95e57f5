set -uo pipefail
R=$GRAFT_REPO_ROOT; cd $R
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_headline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="base bwd1" BENCH_ARGS="--steps 10 --milestone-seconds 0 --extra-steps 0" bash tools/gpu_variants.sh 2>&1 | tee $O/ab.txt; rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/phase_probe.py 131072 > $O/probe.log 2>&1; rc=$?; head -30 $O/probe.log; exit $rc
