"""Fraction of PPO minibatches whose gradient norm exceeds grad_norm (clip_grad_norm_ active) over a
short training run at the bench workload; eager epochs, the norm read back from opt after each apply.
    python tools/grad_norm_stats.py [envs] [epochs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from omniisaacgymenvs_loop_amd import _capi  # noqa: E402


def main():
    os.environ["USV_PPO_FUSED"] = "0"   # the split path: the norm is read back after each ppo_minibatch_apply
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    env, task, agent = bench.build(envs, 0, 1, 42)
    agent.use_graph = False
    norms = []
    orig = _capi.call

    def hook(name, *a):
        orig(name, *a)
        if name == "ppo_minibatch_apply":
            slot = a[6]
            norms.append(agent.opt[8 * (1 - slot) + 3])

    _capi.call = hook
    agent.obs = agent.env_reset()
    per_epoch = []
    for ep in range(epochs):
        n0 = len(norms)
        agent.train_epoch()
        v = torch.stack(norms[n0:]).cpu().numpy()
        per_epoch.append((float(np.mean(v > agent.cfg.grad_norm)), float(np.median(v)), float(v.max())))
        print(f"epoch {ep}: clipped {per_epoch[-1][0]:.3f}  median norm {per_epoch[-1][1]:.3f}  max {per_epoch[-1][2]:.3f}",
              flush=True)
    allv = torch.stack(norms).cpu().numpy()
    print(f"overall: {np.mean(allv > agent.cfg.grad_norm):.3f} of {len(allv)} minibatches clipped (grad_norm "
          f"{agent.cfg.grad_norm}); median {np.median(allv):.3f}")


if __name__ == "__main__":
    main()
