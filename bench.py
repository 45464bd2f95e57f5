"""Benchmark: env-steps/s of rl_games PPO training on USV_Virtual_CaptureXY.

One bench "step" = one rl_games train epoch: horizon_length=16 control steps of
num_envs envs (each = reset path + 10 physics substeps + obs/reward/done, on the
GPU) interleaved with the policy forward, then GAE + dataset preparation and
8 mini-epochs of PPO minibatch updates (fwd + bwd + clip + Adam), i.e. the
reference's "fps total" (rl_games a2c_common.py:46-60).  Workload:
BASELINE.json configs[1] = USV_Virtual_CaptureXY num_envs=4096 PPO-MLP fp32 per
GPU; with --gpus N each rank owns 4096 envs (weak scaling) and gradients are
all-reduced over RCCL every minibatch.

    python bench.py [--gpus N --steps K --warmup W --envs 4096]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec USV_CaptureXY at 1/2/4/8 MI355X; wall-clock to reward=30"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
FP32_PEAK_TFS = 157.3          # MI355X fp32 vector / f32-MFMA peak (same table)
# Algorithmic bytes of the fused env-step kernel per env-step:
# SURVEY §8(d) fused figure (476 B: state, lag, DR params, target, obstacles,
# reward history, 4 field texels, obs row, reward, done) + the episode_sums
# read-modify-write the reference performs every step (25 x 8 B) - counted
# exactly from k_env_step's loads/stores: 357 B read + 313 B written.
ENV_STEP_BYTES = 670
# --task: packaged task yamls and the algorithmic bytes per env-step of their step kernels
# (k_env_step_task): GoToPose 221 B read + 309 B written; TrackXYOVelocity
# 221 + 293 in the first launch and 32 + 28 in k_track_finish
TASKS = {"CaptureXY": ("USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST", ENV_STEP_BYTES,
                       "k_env_step (fused 10-substep integrator + obs/reward/done)"),
         "GoToPose": ("USV/USV_Virtual_GoToPose", 530, "k_env_step_task<GoToPose> (integrator + obs/reward/done)"),
         "TrackXYOVelocity": ("USV/USV_Virtual_TrackXYOVelocity", 574,
                              "k_env_step_task<TrackXYO> + k_track_finish (integrator + obs/reward/done)")}
# PPO minibatch gradient kernel: forward (2*(33*128+128*128+128*3)) + backward
# (2x the two hidden GEMMs + heads) = 6 x 21,120 + 2 x 384 flops per row.
PPO_FLOPS_PER_ROW = 2 * (33 * 128 + 128 * 128 + 3 * 128) + 2 * (2 * 128 * 128 + 2 * 33 * 128 + 128 * 128 + 3 * 128)


def _dist_setup(gpus):
    import torch
    import torch.distributed as dist
    from omniisaacgymenvs_loop_amd.rl_games import dist_util
    rank = int(os.getenv("RANK", "0"))
    world = int(os.getenv("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: launch with torch.distributed.run")
    local = int(dist_util.local_device().split(":")[1])
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(dist_util.backend(), rank=rank, world_size=world)
    return rank, world, local


def build(envs, local, world, seed, task_name="CaptureXY"):
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.rl_games import vecenv
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    cfg = build_config({"num_envs": envs, "seed": seed, "multi_gpu": world > 1, "rl_device": f"cuda:{local}",
                        "task": TASKS[task_name][0]})
    cfg["train"]["params"]["config"]["train_dir"] = "/tmp/bench_runs"
    env = VecEnvRLGames(headless=True)
    task = initialize_task(cfg, env)
    vecenv.register("RLGPU", lambda name, n, **kw: vecenv.RLGPUEnv(name, n, **kw))
    vecenv.register_env("rlgpu", {"vecenv_type": "RLGPU", "env_creator": lambda **kw: env})
    params = cfg["train"]["params"]
    params["config"]["print_stats"] = False
    agent = A2CAgent("run", params)
    return env, task, agent


class KernelTimer:
    """HIP events around one C-ABI launch on torch's current stream (the launch stream)."""

    def __init__(self):
        self.pairs = []

    def __call__(self, fn):
        import torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        self.pairs.append((a, b))

    def mean_ms(self):
        if not self.pairs:
            return float("nan")
        return sum(a.elapsed_time(b) for a, b in self.pairs) / len(self.pairs)


def cpu_baseline(envs=256, budget_s=12.0):
    """The oracle (C env restatement + numpy PPO) timed on one host core, on a
    bounded sample of the same workload: repeated train epochs of envs x 16
    control steps (incl. episode resets + potential fields) + 8 mini-epochs of
    PPO on that epoch's batch, until ~budget_s of CPU time has been spent."""
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import oracle as O
    from oracle import ppo_oracle as PO
    from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml, thruster_tables
    yaml_path = os.path.join(ROOT, "omniisaacgymenvs_loop_amd/cfg/task/USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST.yaml")
    task_cfg = load_yaml(yaml_path)
    cfg = build_usv_cfg(task_cfg)
    H = 16
    sw = lambda x: np.ascontiguousarray(np.swapaxes(np.stack(x), 0, 1).reshape(envs * H, *np.stack(x).shape[2:]))
    with threadpool_limits(1):
        E = O.OracleEnv(cfg, envs, O.make_lut(*thruster_tables(task_cfg)))
        rng = np.random.default_rng(0)
        P = PO.unflatten(np.random.default_rng(1).uniform(-0.08, 0.08, PO.NPARAM).astype(np.float32))
        orms, adam, lr = PO.RMS.zeros(33), PO.Adam.zeros(), 1e-4
        E.full_step(np.zeros((envs, 2), np.float32), -0.6, 0, seed=1)     # initial reset of every env: untimed
        obs = E.obs.copy()
        step, epochs = 1, 0
        t0 = time.perf_counter()
        while epochs < 2 or time.perf_counter() - t0 < budget_s:
            obs_buf, act_buf, nlp_buf, val_buf, mu_buf = [], [], [], [], []
            for _ in range(H):
                _, _, mu, v = PO.forward(P, orms.norm(obs).astype(np.float32))
                a = (mu + rng.standard_normal(mu.shape).astype(np.float32)).astype(np.float32)
                obs_buf.append(obs.copy()); act_buf.append(a); val_buf.append(v[:, 0]); mu_buf.append(mu)
                nlp_buf.append(PO.neglogp(a, mu, np.ones_like(mu), np.zeros_like(mu)))
                E.full_step(np.clip(a, -1, 1), -0.6, step, seed=1)
                obs = E.obs.copy()
                step += 1
            ds = {"obs": sw(obs_buf), "actions": sw(act_buf), "old_logp": sw(nlp_buf), "old_values": sw(val_buf),
                  "returns": sw(val_buf) + 0.1, "advantages": rng.standard_normal(envs * H).astype(np.float32),
                  "mu": sw(mu_buf), "sigma": np.ones((envs * H, 2), np.float32)}
            P, lr, _ = PO.train_epoch_update(P, adam, lr, orms, ds, PO.PPOConfig(minibatch=envs * H))
            epochs += 1
        dt = time.perf_counter() - t0
    return {"value": epochs * envs * H / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"{epochs} train epochs of {envs} envs x {H} steps (C oracle env incl. episode resets + "
                      f"potential fields; initial reset untimed) + 8 mini-epochs numpy PPO per epoch; "
                      f"1 thread; {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU (BASELINE configs[1]: 4096)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches (no HIP graph capture)")
    ap.add_argument("--task", default="CaptureXY", choices=sorted(TASKS) + ["multitask"],
                    help="multitask: even ranks GoToPose, odd ranks TrackXYOVelocity, one shared policy (C4)")
    ap.add_argument("--env-only-envs", type=int, default=131072,
                    help="extra env-only throughput probe at the C5 per-GPU size (0 = skip)")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    rank, world, local = _dist_setup(args.gpus)
    task_name = args.task if args.task != "multitask" else ("GoToPose", "TrackXYOVelocity")[rank % 2]
    step_bytes, step_kernel = TASKS[task_name][1], TASKS[task_name][2]
    env, task, agent = build(args.envs, local, world, args.seed + rank, task_name)
    agent.use_graph = not args.no_graph
    from omniisaacgymenvs_loop_amd import _capi

    # live per-launch timing of the fused env-step kernel and the PPO gradient kernel
    env_timer, ppo_timer = KernelTimer(), KernelTimer()
    orig_call, orig_call_rc = _capi.call, _capi.call_rc

    last_env_args = []

    def timed_call(name, *a):
        if timing[0] and name in ("usv_env_step", "usv_env_step_part"):
            if name == "usv_env_step":
                last_env_args[:] = [a]
            env_timer(lambda: orig_call(name, *a))
        elif timing[0] and name == "ppo_minibatch_grad":
            ppo_timer(lambda: orig_call(name, *a))
        else:
            orig_call(name, *a)

    def timed_call_rc(name, *a):
        if timing[0] and name == "ppo_minibatch_fused":
            rc = [0]
            ppo_timer(lambda: rc.__setitem__(0, orig_call_rc(name, *a)))
            return rc[0]
        return orig_call_rc(name, *a)

    timing = [False]
    _capi.call = timed_call
    _capi.call_rc = timed_call_rc

    agent.obs = agent.env_reset()
    # warmup: the first epoch runs eagerly, the second captures the rollout and update HIP graphs
    for _ in range(max(args.warmup, 2)):
        agent.train_epoch()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_t = play_t = 0.0
    for _ in range(args.steps):
        st, pt, ut, tt = agent.train_epoch()
        step_t += st
        play_t += pt
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    frames = world * args.envs * agent.horizon_length * args.steps
    value = frames / elapsed

    # phase split of one epoch with graph replays: rollout (+ GAE/prepare) vs minibatch update
    phase = {}
    if agent._graph_play is not None and agent._graph_update is not None:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tp = tu = 0.0
        nrep = 5
        for _ in range(nrep):
            ev[0].record()
            agent._graph_play.replay()
            ev[1].record()
            agent._graph_update.replay()
            ev[2].record()
            torch.cuda.synchronize()
            agent._advance_host_clocks()
            tp += ev[0].elapsed_time(ev[1])
            tu += ev[1].elapsed_time(ev[2])
        phase = {"rollout_ms": tp / nrep, "update_ms": tu / nrep}

    # per-launch kernel times: the same epochs launched eagerly (graph replays carry no per-kernel events),
    # HIP events on the launch stream around each C-ABI call
    use_graph = agent.use_graph
    agent.use_graph = False
    timing[0] = True
    for _ in range(2):
        agent.train_epoch()
    torch.cuda.synchronize()
    timing[0] = False
    agent.use_graph = use_graph
    # the same env-step launch 32 times back to back between one event pair: the per-launch event
    # pairs above carry ~3 us of event overhead at 4096 envs; this mean (kernel + launch gap) is
    # what rocprofv3's per-kernel average is compared with
    env_b2b_ms = float("nan")
    # only where the step's working set is cache-resident in the training loop too (4096 envs: 2.7 MB);
    # at large env counts back-to-back launches would find the previous launch's state in the MALL
    if last_env_args and args.envs <= 16384:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        nb2b = 32
        e0.record()
        for _ in range(nb2b):
            orig_call("usv_env_step", *last_env_args[0])
        e1.record()
        torch.cuda.synchronize()
        env_b2b_ms = e0.elapsed_time(e1) / nb2b

    # env + inference only (play_steps) and env only (VecEnv.step with fixed actions), same sizes
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(max(2, args.steps // 4)):
        agent.play_steps()
    torch.cuda.synchronize()
    play_fps = args.envs * agent.horizon_length * max(2, args.steps // 4) / (time.perf_counter() - t1)
    acts = torch.zeros((args.envs, 2), device=f"cuda:{local}")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    nenv = 64
    for _ in range(nenv):
        env.step(acts)
    torch.cuda.synchronize()
    env_fps = args.envs * nenv / (time.perf_counter() - t1)

    env_ms_events = env_timer.mean_ms()
    env_ms = env_b2b_ms if env_b2b_ms == env_b2b_ms else env_ms_events
    ppo_ms = ppo_timer.mean_ms()
    achieved = step_bytes * args.envs / (env_ms * 1e-3) / 1e9
    ppo_tfs = PPO_FLOPS_PER_ROW * agent.minibatch_size / (ppo_ms * 1e-3) / 1e12
    extra = {}
    if args.env_only_envs and rank == 0 and world == 1:
        # C5 per-GPU size: env-only throughput and the env-step kernel roofline at scale
        from omniisaacgymenvs_loop_amd.tasks.usv_virtual import USVVirtual
        big = USVVirtual(task._task_cfg, num_envs=args.env_only_envs, device=f"cuda:{local}", seed=5)
        a = torch.rand((args.env_only_envs, 2), device=f"cuda:{local}") * 2 - 1
        for _ in range(3):
            big.env_step(a)
        big_timer = KernelTimer()
        timing_big = []

        def big_call(name, *aa):
            if name == "usv_env_step":
                big_timer(lambda: orig_call(name, *aa))
            else:
                orig_call(name, *aa)

        _capi.call = big_call
        torch.cuda.synchronize()
        tb = time.perf_counter()
        nb = 32
        for _ in range(nb):
            big.env_step(a)
        torch.cuda.synchronize()
        tb = time.perf_counter() - tb
        _capi.call = timed_call
        bms = big_timer.mean_ms()
        extra = {"env_only_envs": args.env_only_envs, "env_only_fps": args.env_only_envs * nb / tb,
                 "env_step_kernel_ms": bms,
                 "env_step_kernel_gbs": step_bytes * args.env_only_envs / (bms * 1e-3) / 1e9,
                 "env_step_kernel_frac": step_bytes * args.env_only_envs / (bms * 1e-3) / 1e9 / HBM_PEAK_GBS}
        tf = os.path.join(ROOT, "profiles", f"env_step_traffic_{args.env_only_envs}.json")
        if os.path.exists(tf) and task_name == "CaptureXY":
            with open(tf) as f:
                tr = json.load(f)
            extra["env_step_kernel_traffic"] = tr.get("bytes_per_launch")
            extra["env_step_kernel_traffic_gbs"] = tr.get("bytes_per_launch") / (bms * 1e-3) / 1e9
        del big
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic (random-init policy, "
            "randomised spawns/obstacles/DR from the reset path)",
            "config": {"workload": (f"USV_Virtual_CaptureXY num_envs={args.envs}/GPU PPO-MLP fp32 (BASELINE configs[1])"
                                    if args.task == "CaptureXY" else
                                    f"USV_Virtual_{args.task} num_envs={args.envs}/GPU PPO-MLP fp32"),
                       "num_envs_per_gpu": args.envs, "horizon_length": agent.horizon_length,
                       "minibatch_size": agent.minibatch_size, "mini_epochs": agent.mini_epochs_num,
                       "parallelism": f"dp{world}"},
            "fps_step_inference": play_fps, "fps_step_env_only": env_fps,
            "roofline": {"bound": "hbm", "kernel": step_kernel,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "bytes_per_env_step": step_bytes, "launch_ms": env_ms,
                         "launch_ms_event_pairs": env_ms_events, "envs_per_launch": args.envs,
                         "launch_ms_method": ("32 back-to-back launches between one HIP event pair on the launch "
                                              "stream" if env_b2b_ms == env_b2b_ms else
                                              "HIP event pair around each launch")},
            "roofline_ppo": {"bound": "mfma",
                             "kernel": ("k_mb_fused (f32 MFMA fwd+bwd + reduction + Adam, one launch)"
                                        if agent.fused_update else
                                        "k_mb_grad + k_reduce_partials (f32 MFMA fwd+bwd, fixed-order reduction)"),
                             "achieved": ppo_tfs,
                             "peak": FP32_PEAK_TFS, "unit": "TFLOP/s", "frac": ppo_tfs / FP32_PEAK_TFS,
                             "launch_ms": ppo_ms, "rows_per_launch": agent.minibatch_size},
            "extra": dict(extra, **phase),
        }
        traffic_file = os.path.join(ROOT, "profiles", "env_step_traffic.json")
        if os.path.exists(traffic_file):
            with open(traffic_file) as f:
                tr = json.load(f)
            if tr.get("envs") == args.envs and task_name == "CaptureXY":
                out["roofline"]["traffic"] = tr.get("bytes_per_launch")
                out["roofline"]["traffic_source"] = tr.get("source")
        if not args.no_cpu_baseline and world == 1 and args.task == "CaptureXY":
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
