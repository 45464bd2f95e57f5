set -o pipefail
mkdir -p gpurun_out/r05final
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05final/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r05final/smoke.log 2>&1 && \
timeout -k 10 400 python3 bench.py > gpurun_out/r05final/bench.json 2> gpurun_out/r05final/bench.err
rc=$?; tail -2 gpurun_out/r05final/pytest_gpu.log; tail -3 gpurun_out/r05final/smoke.log; head -c 400 gpurun_out/r05final/bench.json; exit $rc
