#!/bin/bash
# GPU box: the headline bench (no CPU baseline, no C2 line) for each library variant in VARIANTS
# (lib/<name>.so, "base" = lib/libusv_hip.so), twice each, interleaved; prints value and update
# time per minibatch.   VARIANTS="base v1 v2" BENCH_ARGS="--steps 10" bash tools/gpu_variants.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/variants
mkdir -p $O
cd $R
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    lib=""; [ "$v" != "base" ] && lib="$v.so"
    USV_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 ${BENCH_ARGS:-} \
      > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$O/$v.$rep.json'));e=d['extra'];print('$v', $rep, 'value %.3fM ms/step %.2f rollout %.2f update %.2f us/mb %.2f' % (d['value']/1e6, d['ms_per_step'], e['rollout_ms'], e['update_ms'], e['update_us_per_minibatch']))"
  done
done
