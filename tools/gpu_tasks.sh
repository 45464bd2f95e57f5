set -o pipefail
mkdir -p gpurun_out/tasks
timeout -k 10 200 python3 bench.py --task GoToPose --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/tasks/pose.json 2> gpurun_out/tasks/pose.err || exit $?
timeout -k 10 200 python3 bench.py --task TrackXYOVelocity --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/tasks/track.json 2> gpurun_out/tasks/track.err || exit $?
USV_RANKS_SHARE_DEVICE=0 USV_DIST_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --task multitask --steps 3 --warmup 2 --no-cpu-baseline --env-only-envs 0 > gpurun_out/tasks/multi.json 2> gpurun_out/tasks/multi.err || exit $?
cat gpurun_out/tasks/*.json
