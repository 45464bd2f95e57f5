#!/bin/bash
# GPU box: PPO parity subset + bench line + rocprofv3 kernel stats of a short bench (kernel means)
#   TAG=r03c bash tools/gpu_ppo_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03c}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_ppo_gpu.py tests/test_headline_gpu.py} -m gpu -x -q --timeout 300 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python3 bench.py --no-cpu-baseline --steps 10 --milestone-seconds 0 --c2-steps 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['extra'].get('update_us_per_minibatch'),d['extra'].get('rollout_ms'),d['roofline']['frac'],d['roofline_ppo']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
cd $R
python3 tools/kstats.py $O/prof/trace_kernel_stats.csv 2>/dev/null | head -30 || true
exit 0
