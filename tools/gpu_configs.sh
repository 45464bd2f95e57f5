#!/bin/bash
# GPU box: bench lines at the other BASELINE configs, one GPU each (per-GPU share of the
# multi-GPU configs): C3 65536 envs CaptureXY SysID (fp32), C4's per-GPU 65536 envs of
# each task (the multitask mix puts GoToPose on even ranks, TrackXYOVelocity on odd ones).  JSON lines in gpurun_out/configs/.
set -uo pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/configs
mkdir -p $O
cd $R
A="--steps 3 --warmup 2 --no-cpu-baseline --c2-steps 0"
timeout -k 10 300 python3 bench.py --envs 65536 $A > $O/c3_65536.json 2> $O/c3.err || exit $?
timeout -k 10 300 python3 bench.py --task GoToPose --envs 65536 $A > $O/c4_pose_65536.json 2> $O/c4p.err || exit $?
timeout -k 10 300 python3 bench.py --task TrackXYOVelocity --envs 65536 $A > $O/c4_track_65536.json 2> $O/c4t.err || exit $?
python3 - <<'PY'
import json, os, glob
for f in sorted(glob.glob(os.path.join(os.environ["GRAFT_REPO_ROOT"], "gpurun_out/configs/*.json"))):
    d = json.load(open(f))
    e = d["extra"]
    print(os.path.basename(f), "value %.4gM ms/step %.2f rollout %.2f update %.2f env_kernel %.1f us (%.1f%% of HBM peak) fps_env %.4gM fps_inf %.4gM" % (
        d["value"] / 1e6, d["ms_per_step"], e.get("rollout_ms", 0), e.get("update_ms", 0),
        d["roofline"]["launch_ms"] * 1e3, 100 * d["roofline"]["frac"], d["fps_step_env_only"] / 1e6, d["fps_step_inference"] / 1e6))
PY
