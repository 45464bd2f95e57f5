set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r05math
cd $R
timeout -k 10 700 python3 -u -m pytest tests/test_env_gpu.py tests/test_headline_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05math/pytest.log 2>&1 || { grep -E "FAILED|Error|assert" gpurun_out/r05math/pytest.log | head -20; exit 1; }
grep -E "passed|failed" gpurun_out/r05math/pytest.log | tail -1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05math/smoke.log 2>&1 || { tail -20 gpurun_out/r05math/smoke.log; exit 1; }
tail -2 gpurun_out/r05math/smoke.log
VARIANTS="base prevmath" TAG=r05math timeout -k 10 700 bash tools/gpu_env_ab.sh > gpurun_out/r05math/env_ab.txt 2>&1; grep -E "avg_us|FETCH" gpurun_out/r05math/env_ab.txt
