#!/bin/bash
# GPU box: the headline bench under several environment settings, interleaved, REPS times each.
#   CASES="ov1:USV_STEP_OVERLAP=1 ov0:USV_STEP_OVERLAP=0" bash tools/gpu_envvar_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/envvar_ab
mkdir -p $O
cd $R
for rep in $(seq 1 ${REPS:-2}); do
  for c in $CASES; do
    name=${c%%:*}; vars=${c#*:}
    env ${vars//,/ } timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 \
      --steps ${STEPS:-10} ${BENCH_ARGS:-} > $O/$name.$rep.json 2> $O/$name.$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$O/$name.$rep.json'));e=d['extra'];r=d['roofline'];print('$name', $rep, 'value %.3fM ms/step %.2f rollout %.2f update %.2f us/mb %.2f env %.2f us' % (d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms'], e['update_us_per_minibatch'], r['launch_ms']*1e3))"
  done
done
