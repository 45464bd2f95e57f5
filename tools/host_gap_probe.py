"""Where the per-epoch host gap goes (GPU box): times each host section of A2CAgent.train_epoch at the headline
size over a few graph-replayed epochs.   python tools/host_gap_probe.py [envs]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    envs = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    env, task, agent = bench.build(envs, 0, 1, 42)
    agent.obs = agent.env_reset()
    for _ in range(3):
        agent.train_epoch()
    torch.cuda.synchronize()
    # staged = train_epoch's order (pinned copies enqueued behind the update, read after the sync); "0" = one
    # blocking device read per flag / meter / LR (the round-4 r04s sequence)
    staged = os.getenv("STAGED", "1") != "0"
    names = ["replay_play", "replay_update", "stage", "sync", "check_errors", "check_nan", "meters", "lr_item"]
    acc = {k: [] for k in names}
    for _ in range(6):
        t = [time.perf_counter()]
        agent._graph_play.replay(); agent._advance_host_clocks(); t.append(time.perf_counter())
        agent._graph_update.replay(); t.append(time.perf_counter())
        if staged:
            agent.vec_env.stage_errors()
            agent._stage_tail()
        t.append(time.perf_counter())
        torch.cuda.current_stream().synchronize(); t.append(time.perf_counter())
        agent.vec_env.check_errors(); t.append(time.perf_counter())
        agent._check_nan(); t.append(time.perf_counter())
        agent._replay_meters(); t.append(time.perf_counter())
        float(agent._h_lr[0]) if staged else float(agent.opt[0].item()); t.append(time.perf_counter())
        agent._tail_staged = False
        for i, k in enumerate(names):
            acc[k].append((t[i + 1] - t[i]) * 1e6)
    for k in names:
        v = sorted(acc[k])
        print(f"{k:14s} median {v[len(v) // 2]:9.1f} us  (min {v[0]:.1f}, max {v[-1]:.1f})")


if __name__ == "__main__":
    main()
