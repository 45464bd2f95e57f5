set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05dp2; mkdir -p $O
cd $R
export USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo
for MODE in peer; do
  USV_DP_EXCHANGE=$MODE timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --c2-steps 5 \
    --no-cpu-baseline --milestone-seconds 0 > $O/dp2_full_$MODE.json 2> $O/dp2_full_$MODE.err || { tail -30 $O/dp2_full_$MODE.err; exit 1; }
  echo "== $MODE"; tail -1 $O/dp2_full_$MODE.json | head -c 300; echo
done
