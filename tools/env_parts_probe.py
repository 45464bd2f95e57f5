"""Diagnostic: the sequential env-step kernel's launch time at 131,072 envs under configuration changes that
remove parts of its work (not parity runs):  python tools/env_parts_probe.py [envs] [steps]
  base        the headline configuration
  substeps1   controlFrequencyInv 1 (one integrator substep instead of 10)
  nostats     episode sums off (no 25 read-modify-writes)
  both        substeps 1 and no sums"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["USV_STEP_OVERLAP"] = "0"

import torch  # noqa: E402

import bench  # noqa: E402
from omniisaacgymenvs_loop_amd import _capi  # noqa: E402
from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config  # noqa: E402
from omniisaacgymenvs_loop_amd.tasks.usv_virtual import USVVirtual  # noqa: E402


def run(envs, steps, substeps, stats):
    cfg = build_config({"num_envs": envs})
    cfg["task"]["env"]["controlFrequencyInv"] = substeps
    task = USVVirtual(cfg["task"], num_envs=envs, device="cuda:0", seed=5)
    task.cfg.stats_on = int(stats)
    a = torch.rand((envs, 2), device="cuda:0") * 2 - 1
    for _ in range(4):
        task.env_step(a)
    timer = bench.KernelTimer()
    orig = _capi.call

    def call(name, *aa):
        if name == "usv_env_step":
            timer(lambda: orig(name, *aa))
        else:
            orig(name, *aa)

    _capi.call = call
    for _ in range(steps):
        task.env_step(a)
    torch.cuda.synchronize()
    _capi.call = orig
    return timer.mean_ms() * 1e3


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    for rep in range(2):
        for name, sub, st in (("base", 10, True), ("substeps1", 1, True), ("nostats", 10, False), ("both", 1, False)):
            print(f"rep {rep} {name:10s} envs {envs}: env step kernel {run(envs, steps, sub, st):.2f} us", flush=True)


if __name__ == "__main__":
    main()
