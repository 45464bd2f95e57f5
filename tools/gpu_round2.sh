#!/bin/bash
# GPU box: the round's committed evidence in one call -- full GPU test suite (log + parity table),
# rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE passes on the env-step kernel at the
# headline size, condensed into profiles/<tag>_*, the default bench line (with the CPU baseline)
# reading the fresh traffic numbers, and the C3 bf16 line.      bash tools/gpu_round2.sh <tag>
set -uo pipefail
TAG=${1:-r02m}
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/parity_errors.json $O/ 2>/dev/null
bash profiles/run_profiles.sh $TAG 131072 || exit $?
python3 profiles/pmc_traffic.py $TAG 131072 || exit $?
cp profiles/${TAG}_* profiles/env_step_traffic_131072.json $O/ || exit $?
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit $?
cat $O/bench.json
timeout -k 10 300 python3 bench.py --envs 65536 --mixed-precision --no-cpu-baseline --c2-steps 0 > $O/bench_c3_bf16.json 2> $O/bench_c3.err || exit $?
exit 0
