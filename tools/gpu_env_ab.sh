#!/bin/bash
# GPU box: env parity (fixture replays, Philox vs oracle, fields) + bench line + kernel trace/stats and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE) on k_env_step at 131072 envs.     TAG=r03d bash tools/gpu_env_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03d}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests/test_env_gpu.py tests/test_headline_gpu.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
cp gpurun_out/parity_errors.json $O/ 2>/dev/null
timeout -k 10 600 python3 bench.py --no-cpu-baseline --steps 10 --milestone-seconds 0 --c2-steps 0 > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['extra'].get('update_us_per_minibatch'),d['extra'].get('rollout_ms'),d['roofline']['frac'],d['roofline']['launch_ms'],d['roofline_ppo']['frac'])"
bash profiles/run_profiles.sh $TAG 131072 || exit 1
python3 profiles/pmc_traffic.py $TAG 131072 $O/env_step_traffic_131072.json || exit 1
cp profiles/${TAG}_* $O/ || exit 1
cat $O/env_step_traffic_131072.json
exit 0
