#!/bin/bash
# GPU box: A/B of the peer exchange's memory ordering in the two-rank one-device rehearsal (peer mode), each
# variant REPS times, interleaved: order3 = the default library (USV_DP_ORDER=3: system-scope release fence
# before the flag + acquire fence after the poll) against lib/libusv_dporder{0,1,2}.so (0: relaxed flag and
# poll, the sc0 sc1 form; 1: release only; 2: acquire only); prints the update time per minibatch of each run.
#   python tools/build_variants.py libusv_dporder0:-DUSV_DP_ORDER=0 libusv_dporder1:-DUSV_DP_ORDER=1 \
#     libusv_dporder2:-DUSV_DP_ORDER=2          (on the CPU host, before the call)
#   TAG=r04b bash tools/gpu_dp2_order_ab.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r04b}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo USV_DP_EXCHANGE=peer
for rep in $(seq 1 ${REPS:-2}); do
  for V in ${VARIANTS:-order3 order0 order1 order2}; do
    LIB=""; [ $V != order3 ] && LIB=libusv_dp$V.so
    USV_HIP_LIB=$LIB timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-5} --warmup 1 --envs ${ENVS:-32768} \
      --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/dp2_${V}_$rep.json 2> $O/dp2_${V}_$rep.err \
      || { tail -30 $O/dp2_${V}_$rep.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/dp2_${V}_$rep.json').read().strip().split('\n')[-1]);e=d['extra'];print('$V $rep', 'value %.4gM' % (d['value']/1e6), 'update_us/mb %.2f' % e['update_us_per_minibatch'], 'ppo pair us %.2f' % (d['roofline_ppo']['launch_ms']*1e3))"
  done
done
exit 0
