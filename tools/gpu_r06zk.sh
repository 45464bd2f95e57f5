#!/bin/bash
# r06zk: the statistics kernel's waves at issue priority 2 / 3 (s_setprio; variant libraries) vs 0 (the default):
# its per-dispatch median beside the policy step, then the headline interleaved
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06zk
mkdir -p $O
cd $R
CASES="p0:USV_DUMMY=0 p2:USV_HIP_LIB=libusv_hip_p2.so p3:USV_HIP_LIB=libusv_hip_p3.so" \
  KERNELS="k_field_stats k_policy_step" STEPS=3 bash tools/gpu_kmed_ab.sh > $O/kmed.txt 2>&1 || exit $?
cat $O/kmed.txt
for rep in 1 2 3; do
  for v in p0 p2 p3; do
    if [ $v = p0 ]; then L=; else L=libusv_hip_$v.so; fi
    USV_HIP_LIB=$L timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --seeds 0 --no-cpu-baseline --c2-steps 0 \
      --milestone-seconds 0 > $O/bench_$v.$rep.json 2> $O/bench_$v.$rep.err || exit $?
    python3 -c "import json,sys; d=json.load(open('$O/bench_$v.$rep.json')); e=d['extra']; print('$v rep $rep value %.2f M rollout_ms %.3f update_ms %.3f' % (d['value']/1e6, e['rollout_ms'], e['update_ms']))"
  done
done
