#!/bin/bash
# GPU box: the multi-rank bench path as a two-rank rehearsal on one device (gloo process group for the
# handle exchange and the timing reductions; the update's gradient exchange is the in-kernel peer path,
# ppo_minibatch_fused_dp over IPC-mapped memory, captured in the update graph), then the collective path.
#   TAG=r03i bash tools/gpu_dp2_rehearsal.sh
set -uo pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r03i}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
export USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo
for MODE in peer collective; do
  USV_DP_EXCHANGE=$MODE timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps ${STEPS:-3} --warmup 1 --envs ${ENVS:-32768} \
    --no-cpu-baseline --c2-steps 0 --milestone-seconds 0 > $O/dp2_$MODE.json 2> $O/dp2_$MODE.err || { tail -30 $O/dp2_$MODE.err; exit 1; }
  echo "== $MODE"; tail -c 600 $O/dp2_$MODE.json; echo
done
exit 0
