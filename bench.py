"""Benchmark: env-steps/s of rl_games PPO training on USV_Virtual_CaptureXY.

One bench "step" = one rl_games train epoch: horizon_length=16 control steps of
num_envs envs (each = reset path + 10 physics substeps + obs/reward/done, on the
GPU) interleaved with the policy forward, then GAE + dataset preparation and
8 mini-epochs of PPO minibatch updates (fwd + bwd + clip + Adam), i.e. the
reference's "fps total" (rl_games a2c_common.py:46-60).  Workload: the north
star's USV_Virtual_CaptureXY at 2^20 envs over 8 GPUs (BASELINE.json configs[4]),
i.e. 131072 envs per GPU, PPO-MLP fp32; with --gpus N each rank owns 131072 envs
(weak scaling) and gradients are all-reduced over RCCL every minibatch.  The
4096-env BASELINE configs[1] line is reported as a secondary field (extra.c2), and on one GPU
configs[2] (65536 envs, bf16 GEMMs: extra.c3) and configs[3]'s per-GPU share of each task (extra.c4_pose,
extra.c4_track) too.

    python bench.py [--gpus N --steps K --warmup W --envs 131072]
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
BF16_PEAK_TFS = 2500.0         # MI355X dense bf16 MFMA peak (same table, no sparsity)
# Algorithmic bytes of the fused env-step kernel per env-step:
# SURVEY §8(d) fused figure (476 B: state, lag, DR params, target, obstacles,
# reward history, 4 field texels, obs row, reward, done) + the episode_sums
# read-modify-write the reference performs every step (25 x 8 B) - counted
# exactly from k_env_step's loads/stores: 389 B read + 313 B written.  The 4 field texels
# are the tiled raw costs (16 B) + the env's 8 normalisation constants (32 B; the field is
# kept as its parts), 357 + 32 = 389 B.
ENV_STEP_BYTES = 702
SURVEY_STEP_BYTES = 476        # SURVEY §8(d)'s algorithmic bytes of the fused env step (the roofline's frac_476)
# --task: packaged task yamls and the algorithmic bytes per env-step of their step kernels
# (k_env_step_task): GoToPose 221 B read + 309 B written; TrackXYOVelocity
# 221 + 293 in the first launch and 32 + 28 in k_track_finish
TASKS = {"CaptureXY": ("USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST", ENV_STEP_BYTES,
                       "k_env_step (fused 10-substep integrator + obs/reward/done)"),
         "GoToPose": ("USV/USV_Virtual_GoToPose", 530, "k_env_step_task<GoToPose> (integrator + obs/reward/done)"),
         "TrackXYOVelocity": ("USV/USV_Virtual_TrackXYOVelocity", 574,
                              "k_env_step_task<TrackXYO> + k_track_finish (integrator + obs/reward/done)")}
# PPO minibatch gradient kernel, algorithmic flops per row (DESIGN.md §4 derives them; elementwise work not
# counted): forward = layer 1 2*33*128 + layer 2 2*128*128 + heads 2*128*3 = 41,984; backward = head weight
# grads 2*3*128 + dh2 = dmu Wmu + dv Wv 2*3*128 + dW2 = dz2^T h1 2*128*128 + dh1 = dz2 W2 2*128*128 +
# dW1 = dz1^T x 2*128*33 = 75,520; total 117,504
PPO_FWD_FLOPS_PER_ROW = 2 * (33 * 128 + 128 * 128 + 128 * 3)
PPO_BWD_FLOPS_PER_ROW = 2 * 3 * 128 + 2 * 3 * 128 + 2 * 128 * 128 + 2 * 128 * 128 + 2 * 128 * 33
PPO_FLOPS_PER_ROW = PPO_FWD_FLOPS_PER_ROW + PPO_BWD_FLOPS_PER_ROW
assert PPO_FLOPS_PER_ROW == 117_504


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


def build(envs, local, world, seed, task_name="CaptureXY", mixed_precision=False):
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.rl_games import vecenv
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    cfg = build_config({"num_envs": envs, "seed": seed, "multi_gpu": world > 1, "rl_device": f"cuda:{local}",
                        "task": TASKS[task_name][0]})
    cfg["train"]["params"]["config"]["train_dir"] = "/tmp/bench_runs"
    cfg["train"]["params"]["config"]["mixed_precision"] = bool(mixed_precision)
    env = VecEnvRLGames(headless=True)
    task = initialize_task(cfg, env)
    vecenv.register("RLGPU", lambda name, n, **kw: vecenv.RLGPUEnv(name, n, **kw))
    vecenv.register_env("rlgpu", {"vecenv_type": "RLGPU", "env_creator": lambda **kw: env})
    params = cfg["train"]["params"]
    params["config"]["print_stats"] = False
    agent = A2CAgent("run", params)
    return env, task, agent


class KernelTimer:
    """HIP events around one C-ABI launch on torch's current stream (the launch stream).  A spin
    kernel (torch.cuda._sleep) keeps the GPU busy while the host enqueues event / launch / event, so
    the pair brackets the launch's own execution, not the host's launch latency (eager epochs are
    host-bound at this size)."""

    def __init__(self, spin_cycles=200_000):
        self.pairs = []
        self.empty = []
        self.spin = spin_cycles

    def _pair(self, fn, into):
        import torch
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        if self.spin:
            torch.cuda._sleep(self.spin)
        a.record()
        if fn is not None:
            fn()
        b.record()
        into.append((a, b))

    def __call__(self, fn):
        self._pair(fn, self.pairs)
        self._pair(None, self.empty)    # the same pair around nothing: the event overhead

    @staticmethod
    def _median(pairs):
        if not pairs:
            return float("nan")
        v = sorted(a.elapsed_time(b) for a, b in pairs)
        m = len(v) // 2
        return v[m] if len(v) % 2 else 0.5 * (v[m - 1] + v[m])

    def raw_ms(self):
        """Median over the launches (a launch that meets a cold cache or a late dispatch does not move it)."""
        return self._median(self.pairs)

    def overhead_ms(self):
        return self._median(self.empty) if self.empty else 0.0

    def mean_ms(self):
        """Launch time: median event-pair time minus the median empty pair (event overhead)."""
        return self.raw_ms() - self.overhead_ms()


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(shapes=((32, 512, 4.0), (4096, 8192, 20.0))):
    """The oracle (C env restatement, OpenMP over envs / reset slots, + numpy PPO with threaded BLAS)
    timed on all host cores, on bounded samples of the same workload at BASELINE's CPU-sized shapes:
    configs[0] (32 envs, minibatch 512 = the whole 32 x 16 batch) and configs[1] (4096 envs, the real
    minibatch 8192).  One sample = whole train epochs: 16 control steps (policy forward, Normal sample,
    env step incl. episode resets + potential fields), GAE on the rewards x 0.01, value / advantage
    preparation, 8 mini-epochs of minibatch updates (fwd + bwd + clip + Adam + adaptive LR), until the
    shape's time budget is spent (at least one epoch).  `value` is the configs[1] rate."""
    os.environ["USV_ORACLE_OMP"] = "1"
    import numpy as np
    from threadpoolctl import threadpool_limits
    from oracle import oracle as O
    from oracle import ppo_oracle as PO
    from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml, thruster_tables
    yaml_path = os.path.join(ROOT, "omniisaacgymenvs_loop_amd/cfg/task/USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST.yaml")
    task_cfg = load_yaml(yaml_path)
    cfg = build_usv_cfg(task_cfg)
    cores = int(O.lib().oracle_threads())
    H = 16
    res = {}
    with threadpool_limits(cores):
        for envs, mb, budget in shapes:
            sw = lambda x: np.ascontiguousarray(np.swapaxes(np.stack(x), 0, 1).reshape(envs * H, *np.stack(x).shape[2:]))
            E = O.OracleEnv(cfg, envs, O.make_lut(*thruster_tables(task_cfg)))
            rng = np.random.default_rng(0)
            P = PO.unflatten(np.random.default_rng(1).uniform(-0.08, 0.08, PO.NPARAM).astype(np.float32))
            orms, vrms, adam, lr = PO.RMS.zeros(33), PO.RMS.zeros(1), PO.Adam.zeros(), 3e-4
            pcfg = PO.PPOConfig(minibatch=mb)
            E.full_step(np.zeros((envs, 2), np.float32), -0.6, 0, seed=1)     # initial reset of every env: untimed
            obs = E.obs.copy()
            dones = np.ones(envs, np.float32)
            step, epochs = 1, 0
            t0 = time.perf_counter()
            while epochs < 1 or time.perf_counter() - t0 < budget:
                obs_b, act_b, nlp_b, val_b, mu_b, rew_b, done_b = [], [], [], [], [], [], []
                for _ in range(H):
                    _, _, mu, v = PO.forward(P, orms.norm(obs).astype(np.float32))
                    a = (mu + rng.standard_normal(mu.shape).astype(np.float32)).astype(np.float32)
                    obs_b.append(obs.copy()); act_b.append(a); val_b.append(v); mu_b.append(mu)
                    nlp_b.append(PO.neglogp(a, mu, np.ones_like(mu), np.zeros_like(mu)))
                    done_b.append(dones.copy())
                    E.full_step(np.clip(a, -1, 1), -0.6, step, seed=1)
                    obs = E.obs.copy()
                    rew_b.append((E.rew * np.float32(0.01))[:, None].astype(np.float32))
                    dones = E.reset_buf.astype(np.float32)
                    step += 1
                _, _, _, last_v = PO.forward(P, orms.norm(obs).astype(np.float32))
                adv = PO.discount_values(0.99, 0.95, dones, last_v, np.stack(done_b), np.stack(val_b), np.stack(rew_b))
                ret = adv + np.stack(val_b)
                vals, rets = sw(val_b)[:, 0], sw([r for r in ret])[:, 0]
                vrms.update(vals[:, None]); vrms.update(rets[:, None])
                a_flat = rets - vals
                a_flat = ((a_flat - a_flat.mean()) / (a_flat.std(ddof=1) + 1e-8)).astype(np.float32)
                ds = {"obs": sw(obs_b), "actions": sw(act_b), "old_logp": sw(nlp_b), "old_values": vals,
                      "returns": rets, "advantages": a_flat, "mu": sw(mu_b),
                      "sigma": np.ones((envs * H, 2), np.float32)}
                P, lr, _ = PO.train_epoch_update(P, adam, lr, orms, ds, pcfg)
                epochs += 1
            dt = time.perf_counter() - t0
            res[envs] = (epochs * envs * H / dt, epochs, dt, mb)
    (v1, e1, t1, m1), (v2, e2, t2, m2) = res[shapes[0][0]], res[shapes[1][0]]
    return {"value": v2, "unit": "env-steps/s", "cores": cores, "kind": "port", "cpu_model": _cpu_model(),
            "value_c1": v1,
            "sample": f"configs[1] shape: {e2} train epochs of {shapes[1][0]} envs x {H} steps in {t2:.1f} s "
                      f"(minibatch {m2}); configs[0] shape: {e1} epochs of {shapes[0][0]} envs in {t1:.1f} s "
                      f"(minibatch {m1}); C oracle env (OpenMP, episode resets + potential fields; initial reset "
                      f"untimed) + numpy PPO (GAE, 8 mini-epochs, clip + Adam + adaptive LR); {cores} threads"}


C2_ENVS = 4096                 # BASELINE configs[1]: secondary line of the same run
HEADLINE_ENVS = 131072         # BASELINE configs[4] per GPU: 2^20 envs over 8 GPUs
REWARD_TARGET = 30.0           # BASELINE metric, half 2: wall-clock to rewards/step >= 30
# the random-init policy's first full 100-episode meter reads about -99 (early collisions), so 30 marks learned
# behaviour; further milestones of the same rewards/step meter are reported beside it
MILESTONES = (30.0, 60.0, 80.0, 100.0)
C3_ENVS = 65536                # BASELINE configs[2]: CaptureXY SysID DR, bf16 (mixed_precision) on one GPU
C4_ENVS = 65536                # BASELINE configs[3]: 262144 envs over 4 GPUs -> 65536 per GPU, per task


def phase_split(timed_events, ms_per_step, minibatches, last_epoch):
    """Rollout / update split of the timed epochs from the (start, rollout end, update end) HIP events each
    recorded on the stream (A2CAgent.phase_events): means over the epochs; host_gap_ms = the rest of the epoch."""
    if not timed_events:
        return {}
    rp = [a.elapsed_time(b) for a, b, _ in timed_events]
    up = [b.elapsed_time(c) for _, b, c in timed_events]
    r, u = sum(rp) / len(rp), sum(up) / len(up)
    return {"rollout_ms": r, "update_ms": u, "update_us_per_minibatch": u * 1e3 / minibatches,
            "host_gap_ms": ms_per_step - (r + u),
            "rollout_ms_min_max": [min(rp), max(rp)], "update_ms_min_max": [min(up), max(up)],
            "phase_method": f"HIP events recorded on the stream inside each of the {len(rp)} timed epochs "
                            f"(epochs {last_epoch - len(rp) + 1}-{last_epoch}) around the rollout (+ GAE / prepare) "
                            "and the update; mean over the timed epochs"}


def rank_record(rank, device, task_name, dp_status, elapsed_local, steps, phase):
    """This rank's part of a multi-rank line: its device, task, the gradient exchange that ran and its start-up
    self-test (A2CAgent.dp_status), its own timed-epoch time and its phase split."""
    from omniisaacgymenvs_loop_amd.rl_games.dist_util import device_identity
    return {"rank": rank, "device": device_identity(device), "task": task_name,
            "exchange": dp_status["exchange"], "selftest": dp_status["selftest"], "exchange_error": dp_status["error"],
            "epoch_ms": elapsed_local / steps * 1e3, "rollout_ms": phase.get("rollout_ms"),
            "update_us_per_minibatch": phase.get("update_us_per_minibatch")}


def rank_records(rec, world):
    """Every rank's record in rank order (all_gather_object over the process group: RCCL or gloo); [rec] alone."""
    if world == 1:
        return [rec]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def dp_fields(records):
    """config.exchange and the per-rank extras of a multi-rank line: which gradient exchange ran (peer: the
    in-kernel IPC exchange of ppo_minibatch_fused_dp; collective: torch.distributed all-reduces), each rank's
    start-up self-test outcome, epoch time and minibatch update time -- so a scaling record says what it measured."""
    ex = sorted({r["exchange"] for r in records})
    return (ex[0] if len(ex) == 1 else "mixed: " + ", ".join(ex)), {
        "dp_selftest": {str(r["rank"]): r["selftest"] for r in records},
        "ranks": records}


def time_epochs(agent, steps, world, local):
    """`steps` train epochs between barrier + synchronize pairs; max over ranks (seconds)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        agent.train_epoch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--envs", type=int, default=HEADLINE_ENVS,
                    help="envs per GPU (default: BASELINE configs[4]'s per-GPU share, 131072 = 2^20 / 8)")
    ap.add_argument("--seeds", default="0,1,2,3,4",
                    help="BASELINE.md's protocol: the headline (W warmup + K timed epochs) once per seed; `value` is "
                         "the median, extra.seeds the per-seed values and min / max.  The first seed's run also "
                         "carries the kernel timings, fps definitions, milestones and the sustained rate")
    ap.add_argument("--seed", type=int, default=None, help="one seed only (same as --seeds <seed>)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="eager launches (no HIP graph capture)")
    ap.add_argument("--task", default="CaptureXY", choices=sorted(TASKS) + ["multitask"],
                    help="multitask: even ranks GoToPose, odd ranks TrackXYOVelocity, one shared policy (C4)")
    ap.add_argument("--mixed-precision", action="store_true",
                    help="bf16 GEMM operands / fp32 accumulation for the policy's 128x128 products (train config "
                         "mixed_precision; BASELINE configs[2] at --envs 65536); physics stays fp32")
    ap.add_argument("--c2-steps", type=int, default=10,
                    help="epochs of the secondary BASELINE configs[1] line (4096 envs/GPU; 0 = skip)")
    ap.add_argument("--extra-steps", type=int, default=10,
                    help="one GPU: epochs of each of the configs[2] / configs[3] lines (extra.c3, extra.c4_pose, "
                         "extra.c4_track; 0 = skip)")
    ap.add_argument("--milestone-seconds", type=float, default=25.0,
                    help="one GPU: keep training after the measurements for this many seconds: wall-clock to the "
                         "learning milestones, and `sustained` = the mean rate over these epochs (0 = skip)")
    args = ap.parse_args()
    seeds = [args.seed] if args.seed is not None else [int(x) for x in args.seeds.split(",") if x.strip()]
    args.seed = seeds[0]
    import torch
    import torch.distributed as dist
    rank, world, local = _dist_setup(args.gpus)
    task_name = args.task if args.task != "multitask" else ("GoToPose", "TrackXYOVelocity")[rank % 2]
    step_bytes, step_kernel = TASKS[task_name][1], TASKS[task_name][2]
    t_start = time.perf_counter()
    # (the task adds LOCAL_RANK to the seed itself on several ranks, task_util.initialize_task)
    env, task, agent = build(args.envs, local, world, args.seed, task_name, args.mixed_precision)
    agent.use_graph = not args.no_graph
    from omniisaacgymenvs_loop_amd import _capi

    # live per-launch timing of the fused env-step kernel and the PPO gradient kernel
    env_timer, ppo_timer = KernelTimer(), KernelTimer()
    orig_call = _capi.call

    resets = []   # the reset count of each timed env step (device control word, read after the launch)

    # USV_BENCH_FLUSH=<MB>: write that many MB ahead of each timed env step (cache-state experiment)
    flush_mb = int(os.getenv("USV_BENCH_FLUSH", "0"))
    flush_buf = torch.empty(flush_mb * 262144, device=f"cuda:{local}") if flush_mb else None

    def timed_call(name, *a):
        if timing[0] and name in ("usv_env_step", "usv_env_step_part"):
            if flush_buf is not None:
                flush_buf.fill_(1.0)
            env_timer(lambda: orig_call(name, *a))
            resets.append(task.ctl[0:1].clone())
        elif timing[0] and name in ("ppo_minibatch_grad", "ppo_minibatch_fused", "ppo_minibatch_fused_dp"):
            ppo_timer(lambda: orig_call(name, *a))
        else:
            orig_call(name, *a)

    timing = [False]
    _capi.call = timed_call

    # training from the random init starts here: the wall clock to reward=30 counts from the first
    # reset (env / agent construction excluded), through warmup and timed epochs alike
    t_train = time.perf_counter()
    to_reward = {"target": REWARD_TARGET, "seconds": None, "epochs": None}
    miles = {str(m): None for m in MILESTONES}
    first_full = {}

    def note_reward():
        gr = agent.game_rewards
        if gr.current_size == 0:
            return
        r = float(gr.get_mean())
        now = time.perf_counter() - t_train
        if not first_full and gr.current_size >= gr.max_size:
            first_full.update(value=r, seconds=now, epochs=agent.epoch_num)
        if to_reward["seconds"] is None and r >= REWARD_TARGET:
            to_reward["seconds"] = now
            to_reward["epochs"] = agent.epoch_num
        for m in MILESTONES:
            if miles[str(m)] is None and r >= m:
                miles[str(m)] = {"seconds": now, "epochs": agent.epoch_num,
                                 "env_steps": agent.epoch_num * args.envs * agent.horizon_length * world}

    agent.obs = agent.env_reset()
    # warmup: the first epoch runs eagerly, the second captures the rollout and update HIP graphs
    for _ in range(max(args.warmup, 2)):
        agent.update_epoch()
        agent.train_epoch()
        note_reward()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    agent.phase_events = []          # (start, rollout end, update end) events recorded inside each timed epoch
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agent.update_epoch()
        agent.train_epoch()          # synchronises the stream at its end (meters, adaptive LR)
        note_reward()                # host-side meter (updated at that sync): the milestones at epoch resolution
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    elapsed_local = elapsed
    t = torch.tensor([elapsed], device=f"cuda:{local}", dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    note_reward()
    timed_events, agent.phase_events = agent.phase_events, None
    epoch_timed_last = agent.epoch_num
    frames = world * args.envs * agent.horizon_length * args.steps
    value = frames / elapsed
    print(f"[bench] rank {rank}: {args.steps} epochs in {elapsed:.3f} s -> {value / 1e6:.2f} M env-steps/s",
          file=sys.stderr, flush=True)

    # phase split of the TIMED epochs: rollout (+ GAE/prepare) vs minibatch update from the HIP events each
    # timed epoch recorded around its two halves on the stream (the intervals hold whatever the GPU did or
    # waited for between the events, host submission included); host_gap_ms = the rest of the timed epoch
    # (the epoch-end synchronisation, meters, the next submission), >= 0 by construction
    phase = phase_split(timed_events, elapsed / args.steps * 1e3, agent.mini_epochs_num * agent.num_minibatches,
                        epoch_timed_last)
    records = rank_records(rank_record(rank, f"cuda:{local}", task_name, agent.dp_status, elapsed_local, args.steps,
                                       phase), world)
    exchange, dp_extra = dp_fields(records)
    # the same two graphs replayed behind a spin kernel after the timed epochs: device time only (no host
    # submission inside the pairs), at a later training state (more resets per step as the policy learns)
    if agent._graph_play is not None and agent._graph_update is not None:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        tp = tu = 0.0
        nrep = 3
        for _ in range(nrep):
            torch.cuda._sleep(int(os.getenv("USV_BENCH_SPIN", "200000000")))
            ev[0].record()
            agent._graph_play.replay()
            ev[1].record()
            agent._graph_update.replay()
            ev[2].record()
            torch.cuda.synchronize()
            agent._advance_host_clocks()
            tp += ev[0].elapsed_time(ev[1])
            tu += ev[1].elapsed_time(ev[2])
        phase["device_only"] = {"rollout_ms": tp / nrep, "update_ms": tu / nrep,
                                "update_us_per_minibatch": tu / nrep * 1e3 / (agent.mini_epochs_num * agent.num_minibatches),
                                "epochs": [epoch_timed_last + 1, epoch_timed_last + nrep],
                                "method": "graph replays behind a spin kernel after the timed epochs (host "
                                          "submission excluded), mean of 3"}

    # per-launch kernel times inside real epochs (eager: graph replays carry no per-kernel events),
    # HIP events on the launch stream around each C-ABI call
    # (the plain sequential step: an overlapped step kernel shares the GPU with the field kernels, so its
    # event pair would time the sharing, not the kernel)
    use_graph = agent.use_graph
    agent.use_graph = False
    overlap_env = os.environ.get("USV_STEP_OVERLAP")
    os.environ["USV_STEP_OVERLAP"] = "0"
    timing[0] = True
    timing_after_epoch = agent.epoch_num
    agent.train_epoch()
    torch.cuda.synchronize()
    timing[0] = False
    if overlap_env is None:
        os.environ.pop("USV_STEP_OVERLAP")
    else:
        os.environ["USV_STEP_OVERLAP"] = overlap_env
    agent.use_graph = use_graph

    # env + inference only (play_steps) and env only (VecEnv.step with fixed actions), same size
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    nplay = 2
    for _ in range(nplay):
        agent.play_steps()
    torch.cuda.synchronize()
    play_fps = args.envs * agent.horizon_length * nplay / (time.perf_counter() - t1)
    acts = torch.zeros((args.envs, 2), device=f"cuda:{local}")
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    nenv = 32
    for _ in range(nenv):
        o_env, _, d_env, _ = env.step(acts)
    torch.cuda.synchronize()
    agent.obs, agent.dones = o_env, d_env   # the agent continues from the env's current state
    env_fps = args.envs * nenv / (time.perf_counter() - t1)

    # wall-clock to learning milestones (one GPU), and the sustained rate: keep training for the budget; the mean
    # env-steps/s over these epochs (resets grow as the policy learns, so late epochs cost more than the early ones
    # the headline times)
    sustained = None
    if world == 1 and args.milestone_seconds > 0:
        torch.cuda.synchronize()
        t_m = time.perf_counter()
        e_m = agent.epoch_num
        while time.perf_counter() - t_m < args.milestone_seconds:
            agent.update_epoch()
            agent.train_epoch()
            note_reward()
        torch.cuda.synchronize()
        dt_m = time.perf_counter() - t_m
        n_m = agent.epoch_num - e_m
        sustained = {"value": args.envs * agent.horizon_length * n_m / dt_m, "unit": "env-steps/s",
                     "epochs": [e_m + 1, agent.epoch_num], "seconds": dt_m,
                     "ms_per_step": dt_m / max(n_m, 1) * 1e3,
                     "method": "graph-replayed train epochs after the measurements, wall clock over all of them"}

    env_ms = env_timer.mean_ms()
    ppo_ms = ppo_timer.mean_ms()
    achieved = step_bytes * args.envs / (env_ms * 1e-3) / 1e9
    ppo_tfs = PPO_FLOPS_PER_ROW * agent.minibatch_size / (ppo_ms * 1e-3) / 1e12
    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32 physics, bf16 GEMM operands / fp32 accumulate" if args.mixed_precision else "fp32",
            "data": "synthetic (random-init policy, "
            "randomised spawns/obstacles/DR from the reset path)",
            "config": {"workload": (f"USV_Virtual_CaptureXY num_envs={args.envs}/GPU PPO-MLP fp32"
                                    + (" (BASELINE configs[4] per GPU: 2^20 envs over 8 GPUs)"
                                       if args.envs == HEADLINE_ENVS else "")
                                    if args.task == "CaptureXY" else
                                    f"USV_Virtual_{args.task} num_envs={args.envs}/GPU PPO-MLP fp32")
                       + (" [mixed_precision: bf16 GEMMs]" if args.mixed_precision else ""),
                       "num_envs_per_gpu": args.envs, "horizon_length": agent.horizon_length,
                       "minibatch_size": agent.minibatch_size, "mini_epochs": agent.mini_epochs_num,
                       "parallelism": f"dp{world}", "exchange": exchange},
            "fps_step_inference": play_fps, "fps_step_env_only": env_fps,
            "roofline": {"bound": "hbm", "kernel": step_kernel,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": None, "bytes_per_env_step": step_bytes,
                         # SURVEY 8(d)'s fused-step figure (no episode-sum read-modify-writes, no field constants)
                         "frac_476": SURVEY_STEP_BYTES * args.envs / (env_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "achieved_476": SURVEY_STEP_BYTES * args.envs / (env_ms * 1e-3) / 1e9,
                         "launch_ms": env_ms, "timed_after_epoch": timing_after_epoch,
                         "launch_ms_raw": env_timer.raw_ms(), "event_overhead_ms": env_timer.overhead_ms(),
                         "resets_per_step": (sorted(int(r.item()) for r in resets) or [None])[len(resets) // 2],
                         "envs_per_launch": args.envs,
                         "launch_ms_method": f"HIP event pair around each of the {len(env_timer.pairs)} env-step "
                                             "launches of one eager training epoch, on the launch stream, behind a "
                                             "spin kernel (host launch latency excluded); median over the launches "
                                             "minus the median of the same pair around no launch (event overhead)"},
            "roofline_ppo": {"bound": "mfma",
                             "kernel": "k_mb_grad + k_reduce_partials (f32 MFMA fwd+bwd, 8 waves per 32-row "
                                       "workgroup, fixed-order reduction)",
                             "achieved": ppo_tfs,
                             "peak": BF16_PEAK_TFS if args.mixed_precision else FP32_PEAK_TFS, "unit": "TFLOP/s",
                             "frac": ppo_tfs / (BF16_PEAK_TFS if args.mixed_precision else FP32_PEAK_TFS),
                             "launch_ms": ppo_ms, "rows_per_launch": agent.minibatch_size,
                             "flops_per_row": PPO_FLOPS_PER_ROW, "flops_per_row_fwd": PPO_FWD_FLOPS_PER_ROW,
                             "flops_per_row_bwd": PPO_BWD_FLOPS_PER_ROW,
                             "launches_timed": len(ppo_timer.pairs),
                             "launch_ms_method": "median HIP event pair around each minibatch's gradient + reduction "
                                                 + (("launches (ppo_minibatch_fused_dp: k_mb_grad + k_reduce_partials "
                                                     "with the in-kernel peer gradient exchange and the Adam step; the "
                                                     "pair includes waiting for the other ranks' chunks)")
                                                    if agent._fused_update() and world > 1 else
                                                    "launches (ppo_minibatch_fused: k_mb_grad + k_reduce_partials with "
                                                    "the Adam step)" if agent._fused_update() else
                                                    "launches (ppo_minibatch_grad: k_mb_grad + k_reduce_partials; the "
                                                    "all-reduce and k_apply follow outside the pair)")
                                                 + " of one eager epoch, minus the empty pair"},
            "wall_clock_to_reward": dict(to_reward, unit="s", since="first env reset of this run (random-init policy)",
                                         note="the BASELINE metric's target on the reference's rewards/step meter "
                                              "(last 100 finished episodes); the random-init policy's first full "
                                              "meter reads first_full_meter (about -99: early collisions), so 30 "
                                              "is learned behaviour; 60 / 80 / 100 are further milestones",
                                         first_full_meter=first_full or None, milestones=miles,
                                         last100_mean_at_end=float(agent.game_rewards.get_mean())),
            "extra": dict(phase, **(dp_extra if world > 1 else {})),
        }
        if sustained is not None:
            out["sustained"] = sustained
        tf = os.path.join(ROOT, "profiles", f"env_step_traffic_{args.envs}.json")
        if not os.path.exists(tf) and args.envs == C2_ENVS:
            tf = os.path.join(ROOT, "profiles", "env_step_traffic.json")
        if os.path.exists(tf) and task_name == "CaptureXY":
            with open(tf) as f:
                tr = json.load(f)
            if tr.get("envs") == args.envs:
                out["roofline"]["traffic"] = tr.get("bytes_per_launch")
                out["roofline"]["traffic_read"] = tr.get("read_bytes_per_launch")
                out["roofline"]["traffic_write"] = tr.get("write_bytes_per_launch")
                out["roofline"]["traffic_source"] = tr.get("source")
    # the other seeds of the protocol: the same build, W warmup and K timed epochs each (the first seed's run
    # above is seed_values[0]); value = the median
    seed_values = [value]
    seed_ms = [elapsed / args.steps * 1e3]
    if len(seeds) > 1:
        if agent._dp is not None:
            torch.cuda.synchronize()
            agent._dp.release()
        del agent, env, task
        torch.cuda.empty_cache()
        for sd in seeds[1:]:
            env_s, task_s, agent_s = build(args.envs, local, world, sd, task_name, args.mixed_precision)
            agent_s.use_graph = not args.no_graph
            agent_s.obs = agent_s.env_reset()
            for _ in range(max(args.warmup, 2)):
                agent_s.update_epoch()
                agent_s.train_epoch()
            el_s = time_epochs(agent_s, args.steps, world, local)
            seed_values.append(world * args.envs * agent_s.horizon_length * args.steps / el_s)
            seed_ms.append(el_s / args.steps * 1e3)
            if agent_s._dp is not None:
                torch.cuda.synchronize()
                agent_s._dp.release()
            del agent_s, env_s, task_s
            torch.cuda.empty_cache()
        agent = env = task = None
    med = sorted(range(len(seeds)), key=lambda i: seed_values[i])[(len(seeds) - 1) // 2]
    if out is not None:
        out["value"] = seed_values[med]
        out["ms_per_step"] = seed_ms[med]
        out["extra"]["seeds"] = {"seeds": seeds, "values": seed_values, "ms_per_step": seed_ms,
                                 "median": seed_values[med], "min": min(seed_values), "max": max(seed_values),
                                 "median_seed": seeds[med],
                                 "note": "value / ms_per_step = the median seed's run (BASELINE.md protocol, seeds "
                                         "0-4); the kernel timings, fps definitions, milestones and `sustained` "
                                         f"come from seed {seeds[0]}'s run"}
    # secondary lines, same code path, graph-replayed epochs: BASELINE configs[1] (4096 envs/GPU) on any number
    # of ranks; on one GPU also configs[2] (65536 envs, bf16 GEMMs) and configs[3]'s per-GPU share of each task
    if args.envs != HEADLINE_ENVS or task_name != "CaptureXY" or args.mixed_precision:
        secondary = []
    else:
        secondary = [("c2", C2_ENVS, "CaptureXY", False, args.c2_steps,
                      f"USV_Virtual_CaptureXY num_envs={C2_ENVS}/GPU PPO-MLP fp32 (BASELINE configs[1])")]
        if world == 1:
            secondary += [
                ("c3", C3_ENVS, "CaptureXY", True, args.extra_steps,
                 f"USV_Virtual_CaptureXY_SysID num_envs={C3_ENVS}/GPU PPO-MLP, bf16 GEMM operands / fp32 "
                 "accumulate (train config mixed_precision; BASELINE configs[2])"),
                ("c4_pose", C4_ENVS, "GoToPose", False, args.extra_steps,
                 f"USV_Virtual_GoToPose num_envs={C4_ENVS}/GPU PPO-MLP fp32 (BASELINE configs[3]'s per-GPU share, "
                 "the GoToPose ranks)"),
                ("c4_track", C4_ENVS, "TrackXYOVelocity", False, args.extra_steps,
                 f"USV_Virtual_TrackXYOVelocity num_envs={C4_ENVS}/GPU PPO-MLP fp32 (BASELINE configs[3]'s "
                 "per-GPU share, the TrackXYOVelocity ranks)")]
    if any(st for *_, st, _ in secondary) and agent is not None:
        if agent._dp is not None:   # every rank: the headline agent's peer buffers, before the next agent maps its own
            torch.cuda.synchronize()
            agent._dp.release()
        del agent, env, task
        torch.cuda.empty_cache()
    for key, n2, task2_name, mixed, st2, workload in secondary:
        if not st2:
            continue
        env2, task2, agent2 = build(n2, local, world, args.seed, task2_name, mixed)
        agent2.use_graph = not args.no_graph
        agent2.obs = agent2.env_reset()
        for _ in range(3):
            agent2.train_epoch()
        el2 = time_epochs(agent2, st2, world, local)
        if out is not None:
            out["extra"][key] = {"workload": workload,
                                 "value": world * n2 * agent2.horizon_length * st2 / el2,
                                 "unit": "env-steps/s", "ms_per_step": el2 / st2 * 1e3, "steps": st2,
                                 "n_gpus": world}
        if agent2._dp is not None:
            torch.cuda.synchronize()
            agent2._dp.release()
        del agent2, env2, task2
        torch.cuda.empty_cache()
    if rank == 0:
        if not args.no_cpu_baseline and world == 1 and args.task == "CaptureXY":
            print("[bench] cpu baseline ...", file=sys.stderr, flush=True)
            out["cpu_baseline"] = cpu_baseline()
        out["extra"]["bench_wall_s"] = time.perf_counter() - t_start
        print(json.dumps(out, default=float))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
