"""Env-only timing of the fused env-step kernel at a given env count (for rocprofv3
counter passes and kernel A/B runs on the GPU box):

    python tools/env_step_probe.py [envs=131072] [steps=32]

Runs the full env step (reset + fields + env step) with random actions and prints
the mean launch time of usv_env_step (HIP events on the launch stream) and its
algorithmic bandwidth."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from omniisaacgymenvs_loop_amd import _capi  # noqa: E402
from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config  # noqa: E402
from omniisaacgymenvs_loop_amd.tasks.usv_virtual import USVVirtual  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    _capi.build()
    cfg = build_config({"num_envs": envs})
    task = USVVirtual(cfg["task"], num_envs=envs, device="cuda:0", seed=5)
    a = torch.rand((envs, 2), device="cuda:0") * 2 - 1
    for _ in range(3):
        task.env_step(a)
    timer = bench.KernelTimer()
    orig = _capi.call

    def call(name, *aa):
        if name == "usv_env_step":
            timer(lambda: orig(name, *aa))
        else:
            orig(name, *aa)

    _capi.call = call
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        task.env_step(a)
    torch.cuda.synchronize()
    t = time.perf_counter() - t
    _capi.call = orig
    ms = timer.mean_ms()
    gbs = bench.ENV_STEP_BYTES * envs / (ms * 1e-3) / 1e9
    print(f"envs {envs}: env step kernel {ms * 1e3:.2f} us, {gbs:.0f} GB/s algorithmic "
          f"({gbs / bench.HBM_PEAK_GBS:.1%} of peak); full env step {t / steps * 1e3:.3f} ms")


if __name__ == "__main__":
    main()
