#!/bin/bash
# r06zl: the sweeps' forward pass noting only the tile's edge cells (USV_SWEEP_FNOTE_EDGE=1, new) vs every cell
# (libusv_hip_prev.so, =0): env / field parity (all sweep routes), the sweep kernel's median, the headline interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zl
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_env_gpu.py \
  tests/test_headline_gpu.py tests/test_overlap_gpu.py tests/test_multitask_gpu.py > $O/pytest.log 2>&1 || exit $?
tail -1 $O/pytest.log
CASES="new:USV_DUMMY=0 prev:USV_HIP_LIB=libusv_hip_prev.so" KERNELS="k_field_wave_pack k_field_stats k_policy_step" STEPS=3 \
  bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
cat $O/kmed.txt
for rep in 1 2 3; do
  for v in new prev; do
    if [ $v = new ]; then L=; else L=libusv_hip_prev.so; fi
    USV_HIP_LIB=$L timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
