"""Wall-clock to a target mean episode reward (the second half of the BASELINE metric):
rl_games PPO on USV_Virtual_CaptureXY (TEST yaml, SysID DR), `rewards/step` = mean unshaped
episode reward over the last 100 episodes (a2c_common.py:1400-1428).

    python tools/train_to_reward.py [--envs 4096 --target 30 --max-seconds 600]
Prints one progress line every --report seconds and a final JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--target", type=float, default=30.0)
    ap.add_argument("--max-seconds", type=float, default=600.0)
    ap.add_argument("--report", type=float, default=20.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--keep-going", action="store_true", help="continue after the target (learning curve)")
    args = ap.parse_args()
    import torch
    import bench
    env, task, agent = bench.build(args.envs, 0, 1, args.seed)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    agent.obs = agent.env_reset()
    last = t0
    epoch = 0
    reached = None
    best = -1e9
    while True:
        agent.train_epoch()
        epoch += 1
        r = float(agent.game_rewards.get_mean()) if agent.game_rewards.current_size else float("nan")
        if r == r:
            best = max(best, r)
        now = time.perf_counter()
        if r == r and r >= args.target and reached is None:
            reached = now - t0
        if now - last >= args.report or (reached is not None and reached == now - t0):
            print(f"t={now - t0:7.1f}s epoch={epoch} frames={epoch * args.envs * agent.horizon_length} "
                  f"reward={r:.2f} best={best:.2f} len={agent.game_lengths.get_mean():.1f} lr={agent.last_lr:.2e}",
                  flush=True)
            last = now
        if (reached is not None and not args.keep_going) or now - t0 > args.max_seconds:
            break
    print(json.dumps({"metric": "wall-clock to reward", "target": args.target, "seconds": reached,
                      "epochs": epoch, "frames": epoch * args.envs * agent.horizon_length, "best_reward": float(best),
                      "envs": args.envs, "elapsed": time.perf_counter() - t0}))


if __name__ == "__main__":
    main()
