#!/bin/bash
# GPU box: the env-step kernel's live launch time (bench roofline.launch_ms, 131072 envs) for each library
# variant in VARIANTS (lib/<name>.so, "base" = lib/libusv_hip.so), interleaved, REPS times each.
#   VARIANTS="base v1 v2" bash tools/gpu_env_variants.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/env_variants
mkdir -p $O
cd $R
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VARIANTS; do
    lib=""; [ "$v" != "base" ] && lib="$v.so"
    USV_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 \
      --steps 2 --warmup 1 ${BENCH_ARGS:-} > $O/$v.$rep.json 2> $O/$v.$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$O/$v.$rep.json'));r=d['roofline'];e=d['extra'];print('$v', $rep, 'env-step %.2f us frac %.3f | rollout %.2f ms value %.2fM' % (r['launch_ms']*1e3, r['frac'], e['rollout_ms'], d['value']/1e6))"
  done
done
