#!/bin/bash
# GPU box: A/B of the peer exchange's memory ordering (USV_DP_ORDER=1 release fence + acquire fence, the
# default library, against lib/libusv_dporder0.so built with -DUSV_DP_ORDER=0: relaxed flag and poll) in
# the two-rank one-device rehearsal (peer mode), A B A B; prints the update time per minibatch of each run.
#   python tools/build_variants.py libusv_dporder0:-DUSV_DP_ORDER=0   (on the CPU host, before the call)
#   TAG=r04b bash tools/gpu_dp2_order_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04b}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo USV_DP_EXCHANGE=peer
for rep in 1 2; do
  for V in order1 order0; do
    LIB=""; [ $V = order0 ] && LIB=libusv_dporder0.so
    USV_HIP_LIB=$LIB timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-5} --warmup 1 --envs ${ENVS:-32768} \
      --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/dp2_${V}_$rep.json 2> $O/dp2_${V}_$rep.err \
      || { tail -30 $O/dp2_${V}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/dp2_${V}_$rep.json'));e=d['extra'];print('$V $rep', 'value %.4gM' % (d['value']/1e6), 'update_us/mb %.2f' % e['update_us_per_minibatch'], 'ppo pair us %.2f' % (d['roofline_ppo']['launch_ms']*1e3))"
  done
done
exit 0
