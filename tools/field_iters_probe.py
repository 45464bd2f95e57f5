"""Tile-sweep iterations per reset env as training proceeds: the headline trainer (bench.build, 131,072 envs,
graph-replayed epochs) and, after chosen epochs, the last step's reset count and each of its slots' iteration
count (slot_stats[slot][SS_ITERS] = 10, written by the sweep kernel) and exact-path flag (SS_EXACT = 11).
    python tools/field_iters_probe.py [epoch ...]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from omniisaacgymenvs_loop_amd._abi import DEFINES  # noqa: E402

SS_ITERS, SS_EXACT = 10, 11


def main():
    marks = sorted(int(x) for x in sys.argv[1:]) or [3, 23, 60, 93]
    env, task, agent = bench.build(bench.HEADLINE_ENVS, 0, 1, 42)
    agent.use_graph = True
    agent.obs = agent.env_reset()
    for ep in range(1, marks[-1] + 1):   # as bench.py: the first epoch eager, then graph replays
        agent.update_epoch()
        agent.train_epoch()
        if ep in marks:
            torch.cuda.synchronize()
            k = int(task.ctl[DEFINES["USV_CTL_RESET_COUNT"]].item())
            st = task.slot_stats[:k].cpu().numpy()
            it = st[:, SS_ITERS]
            print("epoch %3d resets %5d iterations mean %.1f p10 %.0f p50 %.0f p90 %.0f max %.0f exact %d  "
                  "rounds of 512 %.2f  iteration-sum / 512 %.1f" % (
                      ep, k, it.mean(), np.percentile(it, 10), np.median(it), np.percentile(it, 90), it.max(),
                      int((st[:, SS_EXACT] != 0).sum()), k / 512, it.sum() / 512), flush=True)


if __name__ == "__main__":
    main()
