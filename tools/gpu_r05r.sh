set -o pipefail
mkdir -p gpurun_out/r05r
timeout -k 10 600 python3 -u -m pytest tests/test_env_gpu.py tests/test_headline_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05r/pytest_env.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r05r/smoke.log 2>&1
