#!/bin/bash
# GPU box: (1) the multi-rank update's three-launch split measured on one rank (USV_PPO_FUSED=0),
# (2) a two-rank bench rehearsal on the one device (gloo collectives, USV_RANKS_SHARE_DEVICE).
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/splitdp
mkdir -p $O
cd $R
USV_PPO_FUSED=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --c2-steps 0 --steps 10 > $O/split.json 2> $O/split.err || exit $?
python3 -c "import json;d=json.load(open('$O/split.json'));print('split', d['value'], d['ms_per_step'], d['extra']['update_us_per_minibatch'])"
USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --envs 32768 --steps 3 \
  --warmup 2 --no-cpu-baseline --c2-steps 0 > $O/dp2.json 2> $O/dp2.err || exit $?
python3 -c "import json;d=json.load(open('$O/dp2.json'));print('dp2', d['value'], d['ms_per_step'], d['n_gpus'], d['extra']['update_us_per_minibatch'])"
