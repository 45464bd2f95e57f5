#!/bin/bash
# GPU box: PPO-side GPU tests (gradient/minibatch parity, training, dist), the headline bench
# without the CPU baseline, and a rocprofv3 kernel-stats pass of a short bench.
#   bash tools/gpu_ppo.sh <tag>        (outputs under gpurun_out/<tag>/)
set -uo pipefail
TAG=${1:-ppo}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_ppo_gpu.py tests/test_train_gpu.py tests/test_dist_gpu.py -m gpu -x -q \
  --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 bench.py --no-cpu-baseline --c2-steps 0 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['extra'],d['roofline_ppo'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o trace -- \
  python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --c2-steps 0 > $O/prof.log 2>&1 || exit $?
KS=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 $R/tools/kstats.py "$KS" 20
exit 0
