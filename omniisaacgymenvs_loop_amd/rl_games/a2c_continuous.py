"""A2CAgent: rl_games continuous PPO (a2c_continuous + ContinuousA2CBase + A2CBase)
with every per-sample operation in HIP kernels (csrc/ppo.hip).

Reference: rl_games/rl_games/algos_torch/a2c_continuous.py:14-217 and
rl_games/rl_games/common/a2c_common.py:65-1486.  Same constructor
(`A2CAgent(base_name, params)`), same config keys (train yaml `params.config`),
same train() / train_epoch() / play_steps() / prepare_dataset() structure, same
checkpoint dict.  Differences by design:
  * the experience buffer is env-major on the device (the layout
    swap_and_flatten01 produces), written in place by the rollout kernel;
  * the episode meters are accumulated on the device per step and replayed
    into AverageMeter semantics once per epoch (one host sync per epoch,
    instead of per-step .item() calls);
  * the KL and the adaptive learning rate stay on the device;
  * multi-GPU: one process per GPU, flat-gradient all-reduce (+ KL in the same
    buffer) between the gradient and the Adam kernels.
"""
from __future__ import annotations

import copy
import os
import time
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from .. import _capi
from .._abi import DEFINES, PpoAdamBanks, PpoCfg
from . import checkpoint as ckpt
from . import dist_util
from . import vecenv
from ..tasks.usv_config import nan_probe_enabled, raise_nan_flag

NIN, NH, NA = DEFINES["PPO_NIN"], DEFINES["PPO_NH"], DEFINES["PPO_NA"]
NPARAM = DEFINES["PPO_NPARAM"]


class AverageMeter:
    """torch_ext.AverageMeter (torch_ext.py:281-307) fed with (mean, size) pairs."""

    def __init__(self, max_size: int = 100):
        self.max_size = max_size
        self.current_size = 0
        self.mean = 0.0

    def update_stats(self, new_mean: float, size: int) -> None:
        if size == 0:
            return
        size = min(max(int(size), 0), self.max_size)   # np.clip on an int, without its per-call overhead
        old_size = min(self.max_size - size, self.current_size)
        size_sum = old_size + size
        self.current_size = size_sum
        self.mean = (self.mean * old_size + new_mean * size) / size_sum

    def clear(self):
        self.current_size = 0
        self.mean = 0.0

    def get_mean(self) -> float:
        return self.mean

    def __len__(self):
        return self.current_size


class DefaultAlgoObserver:
    """rl_games.common.algo_observer.AlgoObserver hooks (algo_observer.py:6-26)."""

    def before_init(self, base_name, config, experiment_name):
        pass

    def after_init(self, algo):
        self.algo = algo

    def process_infos(self, infos, done_indices):
        pass

    def after_steps(self):
        pass

    def after_clear_stats(self):
        pass

    def after_print_stats(self, frame, epoch_num, total_time):
        pass


def default_linear_init(seed: int, obs_dim: int = NIN) -> torch.Tensor:
    """PyTorch nn.Linear default init in the reference's construction order
    (actor_mlp obs_dim->128, 128->128, value 128->1, mu 128->2), biases zeroed,
    sigma = const 0 (network_builder.py:1520-1575).  obs_dim < NIN: W1's extra
    columns are zero (the padded input of a priv_dim = 4 task)."""
    g = torch.Generator().manual_seed(int(seed))
    parts = {"sigma": torch.zeros(NA)}

    def lin(i, o):
        bound = 1.0 / np.sqrt(i)   # kaiming_uniform(a=sqrt(5)) == U(-1/sqrt(fan_in), 1/sqrt(fan_in))
        w = (torch.rand((o, i), generator=g) * 2 - 1) * bound
        torch.rand((o,), generator=g)   # bias draw (then zeroed by the builder)
        return w, torch.zeros(o)

    W1, b1 = lin(obs_dim, NH)
    W1 = torch.cat([W1, torch.zeros(NH, NIN - obs_dim)], 1)
    W2, b2 = lin(NH, NH)
    Wv, bv = lin(NH, 1)
    Wmu, bmu = lin(NH, NA)
    flat = torch.cat([parts["sigma"], W1.reshape(-1), b1, W2.reshape(-1), b2, Wv.reshape(-1), bv,
                      Wmu.reshape(-1), bmu]).float()
    assert flat.numel() == NPARAM
    return flat


class A2CAgent:
    def __init__(self, base_name: str, params: Dict[str, Any]):
        self.config = config = params["config"]
        self.name = base_name
        self.params = params
        self.seed = int(params.get("seed", 42))
        self.experiment_name = config.get("full_experiment_name") or config["name"]
        self.algo_observer = config.get("features", {}).get("observer") or DefaultAlgoObserver()
        self.algo_observer.before_init(base_name, config, self.experiment_name)
        # ---- distributed (a2c_common.py:87-101): one process per GPU ----
        self.multi_gpu = bool(config.get("multi_gpu", False))
        self.rank, self.rank_size = 0, 1
        if self.multi_gpu:
            self.rank = int(os.getenv("LOCAL_RANK", "0"))
            self.rank_size = int(os.getenv("WORLD_SIZE", "1"))
            if not dist.is_initialized():
                dist.init_process_group(dist_util.backend(), rank=int(os.getenv("RANK", self.rank)),
                                        world_size=self.rank_size)
            config["device"] = dist_util.local_device()
        self.ppo_device = config.get("device", "cuda:0")
        torch.cuda.set_device(torch.device(self.ppo_device))
        self.num_actors = int(config["num_actors"])
        self.env_name = config.get("env_name", "rlgpu")
        self.vec_env = config.get("vec_env", None)
        if self.vec_env is None:
            self.vec_env = vecenv.create_vec_env(self.env_name, self.num_actors, **config.get("env_config", {}))
        self.env_info = config.get("env_info") or self.vec_env.get_env_info()
        # "sim-system need run few step before reset by rlgames" (a2c_common.py:123-127)
        inner = getattr(self.vec_env, "env", None)
        if inner is not None and hasattr(inner, "_world") and hasattr(inner, "_task"):
            for _ in range(5):
                inner._world.step(render=False)
                inner._task.update_state()
        obs_space = self.env_info["observation_space"]
        obs_shape = obs_space.spaces["state"].shape if hasattr(obs_space, "spaces") else obs_space.shape
        if len(obs_shape) != 1 or not (0 < obs_shape[0] <= NIN):
            raise ValueError(f"observation 'state' must be (k,) with k <= {NIN}, got {obs_shape}")
        # k < NIN (priv_dim = 4 tasks: 29): the kernels keep NIN inputs, the extra W1 columns see zero
        # inputs, get zero gradients and stay zero -- exactly the reference's k-input network
        self.obs_dim = int(obs_shape[0])
        self.actions_num = self.env_info["action_space"].shape[0]
        if self.actions_num != NA:
            raise ValueError(f"action space must have {NA} dims")
        self.horizon_length = int(config["horizon_length"])
        self.batch_size = self.horizon_length * self.num_actors
        self.minibatch_size = int(config.get("minibatch_size", self.num_actors * config.get("minibatch_size_per_env", 0)))
        assert self.batch_size % self.minibatch_size == 0, "batch_size % minibatch_size != 0 (a2c_common.py:240)"
        if self.minibatch_size % 32 != 0:
            raise ValueError("minibatch_size must be a multiple of 32 (kernel row block)")
        self.num_minibatches = self.batch_size // self.minibatch_size
        self.mini_epochs_num = int(config["mini_epochs"])
        self.max_epochs = int(config.get("max_epochs", -1))
        self.max_frames = int(config.get("max_frames", -1))
        self.save_freq = int(config.get("save_frequency", 0))
        self.save_best_after = int(config.get("save_best_after", 100))
        self.print_stats = bool(config.get("print_stats", True)) and self.rank == 0
        self.games_to_track = int(config.get("games_to_track", 100))
        self.score_to_win = float(config.get("score_to_win", float("inf")))
        self.normalize_input = bool(config.get("normalize_input", False))
        self.normalize_value = bool(config.get("normalize_value", False))
        self.normalize_advantage = bool(config.get("normalize_advantage", True))
        self.last_lr = float(config["learning_rate"])
        self.is_adaptive_lr = config.get("lr_schedule") == "adaptive"
        if config.get("lr_schedule") not in (None, "adaptive", "None"):
            raise NotImplementedError(f"lr_schedule {config.get('lr_schedule')} is not on the USV hot path")
        if str(config.get("schedule_type", "legacy")) != "legacy":
            raise NotImplementedError("only the legacy (per-minibatch) KL schedule is implemented")
        rs = config.get("reward_shaper", {}) or {}
        if not isinstance(rs, dict):
            rs = {"scale_value": getattr(rs, "scale_value", 1.0), "shift_value": getattr(rs, "shift_value", 0.0)}
        self.cfg = c = PpoCfg()
        c.horizon, c.n_envs, c.minibatch = self.horizon_length, self.num_actors, self.minibatch_size
        c.normalize_input, c.normalize_value = int(self.normalize_input), int(self.normalize_value)
        c.normalize_advantage = int(self.normalize_advantage)
        c.gamma, c.tau = float(config["gamma"]), float(config["tau"])
        c.e_clip, c.critic_coef = float(config["e_clip"]), float(config["critic_coef"])
        c.entropy_coef = float(config["entropy_coef"])
        c.bounds_loss_coef = float(config.get("bounds_loss_coef", 0.0) or 0.0)
        c.clip_value = int(bool(config.get("clip_value", False)))
        c.truncate_grads, c.grad_norm = int(bool(config.get("truncate_grads", False))), float(config["grad_norm"])
        c.adam_b1, c.adam_b2, c.adam_eps = 0.9, 0.999, 1e-8
        c.weight_decay = float(config.get("weight_decay", 0.0))
        c.lr_adaptive = int(self.is_adaptive_lr)
        c.kl_threshold = float(config.get("kl_threshold", 0.008))
        c.lr_min, c.lr_max = 1e-6, 1e-2
        c.reward_scale = float(rs.get("scale_value", 1.0))
        c.reward_shift = float(rs.get("shift_value", 0.0))
        c.rms_eps = 1e-5
        # mixed_precision (a2c_common.py:242-243: torch.cuda.amp autocast + GradScaler in the reference) maps to
        # the MI355X bf16 GEMM mode: bf16 operands / fp32 accumulation for the 128x128 products, fp32
        # elsewhere (no loss scaling needed with bf16's exponent range) -- BASELINE configs[2]
        self.mixed_precision = bool(config.get("mixed_precision", False))
        c.bf16_gemm = int(self.mixed_precision)
        # device NaN probe of the rollout's policy outputs (USV_NAN_PROBE, USV_Virtual.py:57-95)
        c.nan_probe = nan_probe_enabled()
        self._alloc()
        self.frame = 0
        self.epoch_num = 0
        self.mean_rewards = self.last_mean_rewards = -100500
        self.game_rewards = AverageMeter(self.games_to_track)
        self.game_shaped_rewards = AverageMeter(self.games_to_track)
        self.game_lengths = AverageMeter(self.games_to_track)
        self.train_dir = config.get("train_dir", "runs")
        self.experiment_dir = os.path.join(self.train_dir, self.experiment_name)
        self.nn_dir = os.path.join(self.experiment_dir, "nn")
        self.obs = None
        self._step_counter = 0
        # HIP graphs: after one eager epoch, the rollout (+ GAE/prepare) and, on a single GPU, the whole
        # minibatch update are captured once and replayed every epoch (the step / Philox counters live on
        # the device, so a replay continues exactly where the eager loop would)
        self.use_graph = bool(config.get("hip_graph", True))
        self._graph_play = None
        self._graph_update = None
        self._eager_epochs = 0
        self.phase_events = None      # bench: per-epoch (start, rollout end, update end) HIP events
        self.algo_observer.after_init(self)

    def _obs_in(self, obs: torch.Tensor) -> torch.Tensor:
        """The policy kernels' [N, NIN] input: the env rows as they are, or (obs_dim < NIN) copied into
        the zero-padded buffer."""
        if self._obs_pad is None:
            return obs if obs.is_contiguous() else obs.contiguous()
        self._obs_pad[:, :self.obs_dim].copy_(obs)
        return self._obs_pad

    # ------------------------------------------------------------ buffers
    def _alloc(self):
        dev = self.ppo_device
        f32, f64 = dict(device=dev, dtype=torch.float32), dict(device=dev, dtype=torch.float64)
        N, H = self.num_actors, self.horizon_length
        self.model_params = default_linear_init(self.seed, self.obs_dim).to(dev)
        self._obs_pad = torch.zeros((N, NIN), **f32) if self.obs_dim < NIN else None
        if self.multi_gpu:
            dist_util.broadcast_params(self.model_params, 0)   # a2c_common.py:1354 (initial weights from rank 0)
        self.adam_m = torch.zeros(NPARAM, **f32)
        self.adam_v = torch.zeros(NPARAM, **f32)
        # second bank of (params, m, v) for the chained single-GPU update (ppo_minibatch_fused)
        self._bank1 = torch.zeros((3, NPARAM), **f32)
        self._banks = None
        # optimiser scalars, two slots (lr, step, kl, norm): minibatch k reads slot k % 2 and writes the other
        self.opt = torch.zeros(16, **f32)
        self.opt[0] = self.last_lr
        self.obs_rms = torch.zeros(2 * NIN + 1, **f64)
        self.obs_rms[NIN:2 * NIN] = 1.0
        self.obs_rms[2 * NIN] = 1.0
        self.val_rms = torch.tensor([0.0, 1.0, 1.0], **f64)
        self.grad = torch.zeros(_capi.lib().ppo_grad_floats(), **f32)
        self.losses = torch.zeros(8, **f32)
        n_part = _capi.lib().ppo_partials_floats(self.minibatch_size)
        if n_part <= 0:   # the chunk-major partial rows of this many workgroups would overrun the fold words
            raise ValueError(f"minibatch_size {self.minibatch_size}: no partial-gradient layout (ppo_partials_floats)")
        self.partials = torch.zeros(n_part, **f32)
        self.work = torch.zeros(8 + 8 * 4096 + N // 2 + 64, **f64)
        B = N * H
        self.exp_obs = torch.zeros((B, NIN), **f32)
        self.exp_act = torch.zeros((B, NA), **f32)
        self.exp_nlp = torch.zeros(B, **f32)
        self.exp_val = torch.zeros(B, **f32)
        self.exp_ret = torch.zeros(B, **f32)
        self.exp_adv = torch.zeros(B, **f32)
        self.exp_rew = torch.zeros(B, **f32)
        self.exp_mu = torch.zeros((B, NA), **f32)
        self.exp_sigma = torch.zeros((B, NA), **f32)
        self.exp_done = torch.zeros(B, device=dev, dtype=torch.uint8)
        self.actions = torch.zeros((N, NA), **f32)
        self.dones = torch.ones(N, device=dev, dtype=torch.int64)
        self.cur_rew = torch.zeros(N, **f32)
        self.cur_shaped = torch.zeros(N, **f32)
        self.cur_len = torch.zeros(N, **f32)
        # [H][4] per-slot meter sums, then the per-workgroup partials they are folded from
        self.meter_buf = torch.zeros(_capi.lib().ppo_meter_floats(N, H), **f32)
        self.meter = self.meter_buf[:H * 4].view(H, 4)
        self.step_dev = torch.zeros(1, device=dev, dtype=torch.int64)   # rollout Philox step (device clock)
        # running obs statistics after each minibatch of mini-epoch 0 (ppo_obs_rms_epoch)
        nrs = _capi.lib().ppo_rms_seq_doubles(_capi.byref(self.cfg), B) if self.normalize_input else -1
        self.rms_seq = torch.zeros(max(nrs, 1), **f64)
        self.kls = torch.zeros(self.mini_epochs_num * self.num_minibatches, **f32)
        # per minibatch: a_loss, c_loss, entropy, b_loss, kl (this rank), written by the reduce kernel
        self.loss_log = torch.zeros((self.mini_epochs_num * self.num_minibatches, 8), **f32)
        self.nan_flag = torch.zeros(1, device=dev, dtype=torch.int32)
        self.cfg.nan_flag = self.nan_flag.data_ptr()
        # the epoch's host-side tail (meters, LR, NaN flag) as pinned copies enqueued behind the update
        # (_stage_tail): the epoch-end synchronisation covers them, no blocking device read each
        pin = torch.device(dev).type == "cuda"
        self._h_meter = torch.empty(self.meter.shape, dtype=torch.float32, pin_memory=pin)
        self._h_lr = torch.empty(1, dtype=torch.float32, pin_memory=pin)
        self._h_nan = torch.empty(1, dtype=torch.int32, pin_memory=pin)
        self._h_dp_err = None
        self._tail_staged = False
        self.dp_status = {"exchange": "none (one rank)", "selftest": "not run", "error": None}
        # the multi-rank update paths (also at world size 1 with USV_DP_RANK_PATHS=1: the one-GPU tests of the
        # RCCL fallback, whose all-reduce over one rank is the identity)
        self._dp_ranks = self.multi_gpu and (self.rank_size > 1 or os.getenv("USV_DP_RANK_PATHS", "0") == "1")
        self._dp = self._peer_exchange() if self._dp_ranks else None

    def _peer_exchange(self):
        """Several ranks: the one-shot peer exchange of ppo_minibatch_fused_dp (dist_util.PeerExchange) unless
        USV_DP_EXCHANGE=collective; every rank must map every other rank's buffer, otherwise all ranks fall
        back to torch.distributed all-reduces (eager, the three-launch split)."""
        # what ran, for the bench line (config.exchange, extra.ranks): exchange, the start-up self-test's outcome
        self.dp_status = {"exchange": "collective", "selftest": "not run", "error": None}
        if os.getenv("USV_DP_EXCHANGE", "peer") == "collective":
            self.dp_status["error"] = "USV_DP_EXCHANGE=collective"
            return None
        ex, err = None, None
        try:   # every rank succeeds or every rank raises (PeerExchange agrees over the ranks itself)
            ex = dist_util.PeerExchange(self.rank, self.rank_size, self.ppo_device,
                                        timeout_ms=int(os.getenv("USV_DP_TIMEOUT_MS", "20000")))
        except RuntimeError as e:
            err = e
        if not self._ranks_agree(ex is not None):
            if ex is not None:
                ex.close()
            self.dp_status["error"] = str(err) if err is not None else "failed on another rank"
            if err is not None and "start-up exchange test failed" in str(err):
                self.dp_status["selftest"] = "fail"
            if self.rank == 0:
                print(f"peer exchange unavailable ({err or 'on another rank'}); gradients go through "
                      f"torch.distributed all-reduces")
            return None
        self.dp_status.update(exchange="peer", selftest="pass" if ex.selftest_bits == 0 else
                              ("not run" if ex.selftest_bits is None else f"fail (bits {ex.selftest_bits})"))
        return ex

    # ------------------------------------------------------------- rollout
    def env_reset(self):
        obs = self.vec_env.reset()
        return obs

    def play_steps(self) -> Dict[str, Any]:
        """A2CBase.play_steps (a2c_common.py:670-774): H x (policy kernel, env kernels, reward kernel)."""
        if os.getenv("USV_STEP_OVERLAP", "1") != "0" and hasattr(self.vec_env, "step_async"):
            return self._play_steps_overlapped()
        c = _capi
        cfg = c.byref(self.cfg)
        s = c.stream_ptr()
        self.meter.zero_()
        step_time = 0.0
        for n in range(self.horizon_length):
            obs = self._obs_in(self.obs["obs"]["state"] if isinstance(self.obs["obs"], dict) else self.obs["obs"])
            c.call("ppo_policy_step", cfg, c.ptr(self.model_params), c.ptr(self.obs_rms), c.ptr(self.val_rms),
                   c.ptr(obs), n, c.ptr(self.exp_obs), c.ptr(self.exp_act), c.ptr(self.exp_nlp),
                   c.ptr(self.exp_val), c.ptr(self.exp_mu), c.ptr(self.exp_sigma), c.ptr(self.exp_done),
                   c.ptr(self.dones), c.ptr(self.actions), self.seed + 7919 * self.rank, self._step_counter,
                   c.ptr(self.step_dev), None, s)
            t0 = time.time()
            self.obs, rewards, self.dones, infos = self.vec_env.step(self.actions)
            step_time += time.time() - t0
            c.call("ppo_store_reward", cfg, c.ptr(rewards), c.ptr(self.dones), n, c.ptr(self.exp_rew),
                   c.ptr(self.cur_rew), c.ptr(self.cur_shaped), c.ptr(self.cur_len), c.ptr(self.meter_buf),
                   c.ptr(self.step_dev), s)
            self.algo_observer.process_infos(infos, None)
            self._step_counter += 1
        return {"played_frames": self.batch_size, "step_time": step_time}

    def _play_steps_overlapped(self) -> Dict[str, Any]:
        """play_steps with each step's reset-env fields built beside the next policy step: policy(n+1) needs
        only step n's observations and dones, which the overlapped env step (VecEnvRLGames.step_async) makes
        final on this stream while the reset envs' potential fields and deferred rewards finish on a side
        stream; store_reward(n) waits for them (vec_env.join()).  Every kernel sees the inputs it sees in
        the sequential loop, so the experience buffers, meters and env state are the same bits."""
        c = _capi
        cfg = c.byref(self.cfg)
        s = c.stream_ptr()
        self.meter.zero_()
        step_time = 0.0
        base = self._step_counter

        def policy(n):
            obs = self._obs_in(self.obs["obs"]["state"] if isinstance(self.obs["obs"], dict) else self.obs["obs"])
            c.call("ppo_policy_step", cfg, c.ptr(self.model_params), c.ptr(self.obs_rms), c.ptr(self.val_rms),
                   c.ptr(obs), n, c.ptr(self.exp_obs), c.ptr(self.exp_act), c.ptr(self.exp_nlp),
                   c.ptr(self.exp_val), c.ptr(self.exp_mu), c.ptr(self.exp_sigma), c.ptr(self.exp_done),
                   c.ptr(self.dones), c.ptr(self.actions), self.seed + 7919 * self.rank, base + n,
                   c.ptr(self.step_dev), None, s)

        def store(n, rewards, dones):
            c.call("ppo_store_reward", cfg, c.ptr(rewards), c.ptr(dones), n, c.ptr(self.exp_rew),
                   c.ptr(self.cur_rew), c.ptr(self.cur_shaped), c.ptr(self.cur_len), c.ptr(self.meter_buf),
                   c.ptr(self.step_dev), s)

        # USV_STORE_DEFER=1 (default): store_reward(n) runs inside step n + 1 once its fields have forked (the
        # env kernels that overwrite step n's rewards / dones follow it), so it leaves the field chain -- the
        # step's critical path -- that otherwise runs join -> late reward -> store -> next reset; the last step's
        # store follows its join.  0: right after each join
        defer = os.getenv("USV_STORE_DEFER", "1") == "1"
        pending = None
        policy(0)
        for n in range(self.horizon_length):
            t0 = time.time()
            hook = (lambda p=pending: store(*p)) if pending is not None else None
            self.obs, rewards, self.dones, infos = self.vec_env.step_async(self.actions, chain=n > 0,
                                                                           after_fork=hook)
            step_time += time.time() - t0
            if n + 1 < self.horizon_length:
                policy(n + 1)
            self.vec_env.join()
            if defer and n + 1 < self.horizon_length:
                pending = (n, rewards, self.dones)
            else:
                pending = None
                store(n, rewards, self.dones)
            self.algo_observer.process_infos(infos, None)
        self._step_counter = base + self.horizon_length
        return {"played_frames": self.batch_size, "step_time": step_time}

    def prepare_dataset(self) -> None:
        """GAE + returns + value RMS + advantage normalisation (a2c_common.py:525-540, 1257-1332)."""
        c = _capi
        obs = self._obs_in(self.obs["obs"]["state"] if isinstance(self.obs["obs"], dict) else self.obs["obs"])
        c.call("ppo_prepare", c.byref(self.cfg), c.ptr(self.model_params), c.ptr(self.obs_rms),
               c.ptr(self.val_rms), c.ptr(obs), c.ptr(self.dones), c.ptr(self.exp_done), c.ptr(self.exp_val),
               c.ptr(self.exp_rew), c.ptr(self.exp_ret), c.ptr(self.exp_adv), c.ptr(self.work), c.stream_ptr())

    def _allreduce_grad(self) -> float:
        """trancate_gradients_and_step multi-GPU branch (a2c_common.py:309-323): flat SUM / world,
        with the minibatch KL in the same buffer (a2c_common.py:1218-1222)."""
        if not self._dp_ranks:
            return 1.0
        return dist_util.allreduce_grad(self.grad[:NPARAM + 1])

    def _adam_banks(self) -> PpoAdamBanks:
        """ppo_adam_banks_t over (model_params, adam_m, adam_v) and the second bank."""
        ptrs = (self.model_params.data_ptr(), self.adam_m.data_ptr(), self.adam_v.data_ptr(), self.opt.data_ptr())
        if self._banks is None or self._banks[0] != ptrs:
            b = PpoAdamBanks()
            b.params[0], b.m[0], b.v[0], b.opt = ptrs
            b.params[1], b.m[1], b.v[1] = (t.data_ptr() for t in self._bank1)
            self._banks = (ptrs, b)
        return self._banks[1]

    def _fused_update(self) -> bool:
        """Two launches per minibatch (ppo_minibatch_fused; several ranks: ppo_minibatch_fused_dp with the
        peer exchange inside the reduction); USV_PPO_FUSED=0 keeps the three-launch split (grad, reduce,
        [torch.distributed all-reduce], apply), as does a multi-rank run without the peer exchange."""
        dp_ok = not self._dp_ranks or getattr(self, "_dp", None) is not None
        return dp_ok and os.environ.get("USV_PPO_FUSED", "1") != "0"

    def _coll_update(self) -> bool:
        """Several ranks without the peer exchange: the collective chain (ppo_minibatch_coll, two launches + the
        all-reduce per minibatch) unless USV_PPO_FUSED=0 or USV_DP_COLL_CHAIN=0 (the three-launch split)."""
        return (self._dp_ranks and getattr(self, "_dp", None) is None and os.environ.get("USV_PPO_FUSED", "1") != "0"
                and os.environ.get("USV_DP_COLL_CHAIN", "1") != "0")

    def update_epoch_minibatches(self) -> None:
        """The mini-epoch / minibatch loop (a2c_common.py:1190-1245): per minibatch the gradient kernel
        (+ fixed-order partial reduction), [RCCL all-reduce of the flat gradient + KL with several
        ranks], then the clip + Adam + LR kernel.  On one rank the step is taken inside the reduction
        and checked by the next launch (ppo_minibatch_fused / ppo_minibatch_finish)."""
        c = _capi
        cfg = c.byref(self.cfg)
        s = c.stream_ptr()
        dp = self._dp_ranks
        k = 0
        seq = self.normalize_input and self.rms_seq.numel() > 1
        if seq:   # RunningMeanStd.train of mini-epoch 0, all minibatches in two launches
            c.call("ppo_obs_rms_epoch", cfg, c.ptr(self.exp_obs), self.batch_size, c.ptr(self.obs_rms),
                   c.ptr(self.rms_seq), s)
        if self._fused_update():
            banks = c.byref(self._adam_banks())
            dpx = (c.byref(self._dp.desc),) if self._dp is not None else ()
            fn = "ppo_minibatch_fused_dp" if dpx else "ppo_minibatch_fused"
            for mini_ep in range(self.mini_epochs_num):
                for i in range(self.num_minibatches):
                    rms = self.rms_seq[2 * NIN * i:] if seq and mini_ep == 0 else self.obs_rms
                    c.call(fn, cfg, banks, *dpx, k, c.ptr(rms), int(mini_ep == 0 and not seq), i,
                           c.ptr(self.exp_obs), c.ptr(self.exp_act), c.ptr(self.exp_nlp), c.ptr(self.exp_val),
                           c.ptr(self.exp_ret), c.ptr(self.exp_adv), c.ptr(self.exp_mu), c.ptr(self.exp_sigma),
                           c.ptr(self.grad), c.ptr(self.loss_log[k]), c.ptr(self.partials), c.ptr(self.work),
                           c.ptr(self.kls[k - 1:k]) if k else None, s)
                    k += 1
            c.call("ppo_minibatch_finish", cfg, banks, k, c.ptr(self.grad), c.ptr(self.kls[k - 1:k]), s)
            self._bank_back(k)
            return
        if self._coll_update():
            # the RCCL fallback on two launches: minibatch k's gradient kernel takes minibatch k-1's step from the
            # all-reduced [grad, kl] in every workgroup; the in-stream all-reduce sits between the launches
            banks = c.byref(self._adam_banks())
            scale = 1.0 / dist_util.world()
            for mini_ep in range(self.mini_epochs_num):
                for i in range(self.num_minibatches):
                    rms = self.rms_seq[2 * NIN * i:] if seq and mini_ep == 0 else self.obs_rms
                    c.call("ppo_minibatch_coll", cfg, banks, k, float(scale), c.ptr(rms),
                           int(mini_ep == 0 and not seq), i, c.ptr(self.exp_obs), c.ptr(self.exp_act),
                           c.ptr(self.exp_nlp), c.ptr(self.exp_val), c.ptr(self.exp_ret), c.ptr(self.exp_adv),
                           c.ptr(self.exp_mu), c.ptr(self.exp_sigma), c.ptr(self.grad), c.ptr(self.loss_log[k]),
                           c.ptr(self.partials), c.ptr(self.work), c.ptr(self.kls[k - 1:k]) if k else None, s)
                    self._allreduce_grad()
                    k += 1
            c.call("ppo_minibatch_coll_finish", cfg, banks, k, c.ptr(self.grad), float(scale),
                   c.ptr(self.kls[k - 1:k]), s)
            self._bank_back(k)
            return
        for mini_ep in range(self.mini_epochs_num):
            for i in range(self.num_minibatches):
                rms = self.rms_seq[2 * NIN * i:] if seq and mini_ep == 0 else self.obs_rms
                args = (cfg, c.ptr(self.model_params), c.ptr(rms), c.ptr(self.val_rms), int(mini_ep == 0 and not seq), i,
                        c.ptr(self.exp_obs), c.ptr(self.exp_act), c.ptr(self.exp_nlp), c.ptr(self.exp_val),
                        c.ptr(self.exp_ret), c.ptr(self.exp_adv), c.ptr(self.exp_mu), c.ptr(self.exp_sigma),
                        c.ptr(self.grad), c.ptr(self.loss_log[k]), c.ptr(self.partials), c.ptr(self.work))
                c.call("ppo_minibatch_grad", *args, s)
                scale = self._allreduce_grad()
                c.call("ppo_minibatch_apply", cfg, c.ptr(self.model_params), c.ptr(self.grad),
                       c.ptr(self.adam_m), c.ptr(self.adam_v), c.ptr(self.opt), k % 2, float(scale),
                       c.ptr(self.kls[k:k + 1]), int(not dp), s)
                k += 1
        if k % 2:   # the last minibatch wrote slot 1: the epoch ends with the state in slot 0
            self.opt[:8].copy_(self.opt[8:])

    def _bank_back(self, k: int) -> None:
        """A chain of k minibatches ended in bank k % 2: bank 1 / slot 1 is copied back to bank 0 / slot 0."""
        if k % 2:
            self.model_params.copy_(self._bank1[0])
            self.adam_m.copy_(self._bank1[1])
            self.adam_v.copy_(self._bank1[2])
            self.opt[:8].copy_(self.opt[8:])

    def _update_capturable(self) -> bool:
        """The minibatch update goes into a HIP graph: on one GPU, with the peer exchange (kernels only), and with
        the RCCL all-reduces of the collective chain / split path on the nccl backend (USV_GRAPH_COLLECTIVES=0
        keeps those eager; gloo's host-staged collectives are not capturable).  A capture that fails on any rank
        sends every rank to the eager update (train_epoch, _ranks_agree)."""
        if getattr(self, "_graph_update_failed", False):
            return False
        if not self._dp_ranks or (self._dp is not None and self._fused_update()):
            return True   # (the peer exchange is kernels only)
        # the torch.distributed all-reduces (no peer exchange, or USV_PPO_FUSED=0)
        return dist_util.backend() == "nccl" and os.getenv("USV_GRAPH_COLLECTIVES", "1") == "1"

    def _ranks_agree(self, ok: bool) -> bool:
        """All ranks succeeded (MIN over ranks; outside any capture), so no rank replays a graph while another
        falls back to eager collectives."""
        if not self.multi_gpu or self.rank_size == 1:
            return ok
        return dist_util.agree(ok, self.ppo_device)

    def _update_from_graph(self) -> None:
        """Replay the update graph, capturing it first.  The ranks agree on the capture (MIN over ranks, outside any
        capture): if it failed on any rank (a collective the backend cannot capture), every rank runs this epoch's
        update eagerly and stays eager, so no rank replays a graph while another issues eager collectives."""
        if self._graph_update is not None:
            self._graph_update.replay()
            return
        err = None
        try:
            self._graph_update = self._graph_capture(self.update_epoch_minibatches)
        except RuntimeError as e:
            err = e
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if not self._ranks_agree(err is None):   # eager from now on, on every rank
            self._graph_update_failed = True
            self._graph_update = None
            if self.rank == 0:
                print(f"update graph capture failed ({err or 'on another rank'}); the update runs eagerly")
            self.update_epoch_minibatches()
        else:
            self._graph_update.replay()

    def _graph_capture(self, fn):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return g

    def _advance_host_clocks(self):
        """A graph replay advanced the device clocks by one epoch: mirror it on the host counters."""
        self._step_counter += self.horizon_length
        adv = getattr(self.vec_env, "advance_host_clock", None)
        if adv is not None:
            adv(self.horizon_length)

    def _play_and_prepare(self):
        batch = self.play_steps()
        self.prepare_dataset()
        return batch

    def train_epoch(self):
        """ContinuousA2CBase.train_epoch (a2c_common.py:1152-1255)."""
        self.vec_env.set_train_info(self.frame, self)
        play_time_start = time.time()
        # phase_events (bench): a list that receives (start, rollout end, update end) HIP events of this epoch,
        # recorded on the stream in the epoch itself (no extra synchronisation)
        pev = None
        if self.phase_events is not None:
            pev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            pev[0].record()
        graphs = self.use_graph and self._eager_epochs >= 1
        if graphs:
            if self._graph_play is None:
                self._graph_play = self._graph_capture(self._play_and_prepare)   # host clocks advance once here
                self._graph_play.replay()
            else:
                self._graph_play.replay()
                self._advance_host_clocks()
            batch = {"played_frames": self.batch_size, "step_time": float("nan")}
        else:
            batch = self._play_and_prepare()
        play_time_end = time.time()
        if pev is not None:
            pev[1].record()
        self.curr_frames = batch["played_frames"]
        self.algo_observer.after_steps()
        if graphs and self._update_capturable():
            self._update_from_graph()
        else:
            self.update_epoch_minibatches()
        if pev is not None:
            pev[2].record()
            self.phase_events.append(tuple(pev))
        stage = getattr(self.vec_env, "stage_errors", None)
        if stage is not None:
            stage()
        self._stage_tail()
        torch.cuda.current_stream().synchronize()
        update_time_end = time.time()
        try:
            chk = getattr(self.vec_env, "check_errors", None)   # device-flagged env errors (scene replay, NaN probe)
            if chk is not None:
                chk()
            self._check_nan()
            if self._dp is not None:
                self._dp.check(self._h_dp_err if self._tail_staged else None)
            self._eager_epochs += 1
            self._replay_meters()
            self.last_lr = float(self._h_lr[0])
        finally:
            self._tail_staged = False
        step_time = batch["step_time"]
        if step_time != step_time:   # graph replay: no per-step host timing
            step_time = play_time_end - play_time_start
        return (step_time, play_time_end - play_time_start, update_time_end - play_time_end,
                update_time_end - play_time_start)

    def _stage_tail(self):
        """Enqueue the epoch tail's device -> pinned host copies behind the update on the current stream (read
        by _check_nan, _replay_meters and the LR after the epoch-end synchronisation)."""
        self._h_meter.copy_(self.meter, non_blocking=True)
        self._h_lr.copy_(self.opt[:1], non_blocking=True)
        if self.cfg.nan_probe:
            self._h_nan.copy_(self.nan_flag, non_blocking=True)
        if self._dp is not None:
            if self._h_dp_err is None:
                self._h_dp_err = torch.empty(self._dp.err.shape, dtype=self._dp.err.dtype, pin_memory=True)
            self._h_dp_err.copy_(self._dp.err, non_blocking=True)
        self._tail_staged = True

    def _check_nan(self):
        """USV_NAN_PROBE for the policy side: a non-finite mu / value in the rollout's forward."""
        if self.cfg.nan_probe:
            bits = int(self._h_nan[0]) if self._tail_staged else int(self.nan_flag.item())
            if bits:
                self.nan_flag.zero_()
                raise_nan_flag(bits, f"rollout of epoch {self.epoch_num}")

    def _replay_meters(self):
        m = self._h_meter.numpy() if self._tail_staged else self.meter.cpu().numpy()
        for t in range(m.shape[0]):
            cnt = int(round(m[t, 3]))
            if cnt > 0:
                self.game_rewards.update_stats(m[t, 0] / cnt, cnt)
                self.game_shaped_rewards.update_stats(m[t, 1] / cnt, cnt)
                self.game_lengths.update_stats(m[t, 2] / cnt, cnt)

    def init_tensors(self):
        pass

    def train(self):
        """ContinuousA2CBase.train (a2c_common.py:1334-1486) minus TensorBoard."""
        self.init_tensors()
        self.last_mean_rewards = -100500
        start_time = time.time()
        total_time = 0.0
        self.obs = self.env_reset()
        self.curr_frames = self.batch_size
        while True:
            epoch_num = self.update_epoch()
            step_time, play_time, update_time, sum_time = self.train_epoch()
            total_time += sum_time
            frame = self.frame // self.rank_size
            curr_frames = self.curr_frames * self.rank_size if self.multi_gpu else self.curr_frames
            self.frame += curr_frames
            should_exit = False
            if self.rank == 0:
                if self.print_stats:
                    fps_step = curr_frames / max(step_time, 1e-9)
                    fps_si = curr_frames / max(play_time, 1e-9)
                    fps_total = curr_frames / max(sum_time, 1e-9)
                    print(f"fps step: {fps_step:.0f} fps step and policy inference: {fps_si:.0f} fps total: "
                          f"{fps_total:.0f} epoch: {epoch_num}/{self.max_epochs} frames: {self.frame}")
                if self.game_rewards.current_size > 0:
                    mean_rewards = self.game_rewards.get_mean()
                    self.mean_rewards = mean_rewards
                    checkpoint_name = self.config["name"] + "_ep_" + str(epoch_num) + "_rew_" + str(mean_rewards)
                    if self.save_freq > 0 and epoch_num % self.save_freq == 0:
                        self.save(os.path.join(self.nn_dir, "last_" + checkpoint_name))
                    if mean_rewards > self.last_mean_rewards and epoch_num >= self.save_best_after:
                        print("saving next best rewards: ", mean_rewards)
                        self.last_mean_rewards = mean_rewards
                        self.save(os.path.join(self.nn_dir, self.config["name"]))
                        if self.last_mean_rewards > self.score_to_win:
                            print("Maximum reward achieved. Network won!")
                            should_exit = True
                if epoch_num >= self.max_epochs and self.max_epochs != -1:
                    mean_rewards = self.game_rewards.get_mean() if self.game_rewards.current_size else -np.inf
                    self.save(os.path.join(self.nn_dir, "last_" + self.config["name"] + "_ep_" + str(epoch_num) +
                                           "_rew_" + str(mean_rewards)))
                    print("MAX EPOCHS NUM!")
                    should_exit = True
                if self.frame >= self.max_frames and self.max_frames != -1:
                    should_exit = True
            if self.multi_gpu:
                t = torch.tensor([float(should_exit)], device=self.ppo_device)
                dist.broadcast(t, 0)
                should_exit = bool(t.item())
            if should_exit:
                return self.last_mean_rewards, epoch_num

    def update_epoch(self):
        self.epoch_num += 1
        return self.epoch_num

    # ----------------------------------------------------------- checkpoints
    def get_full_state_weights(self) -> Dict[str, Any]:
        step = float(self.opt[1].item())
        # get_weights -> get_stats_weights puts the GradScaler state first under mixed_precision (a2c_common.py:628-631)
        state = {"scaler": ckpt.grad_scaler_state(step)} if self.mixed_precision else {}
        return {**state,
                "model": ckpt.model_state_dict(self.model_params, self.obs_rms, self.val_rms, self.obs_dim),
                "epoch": self.epoch_num,
                "optimizer": ckpt.optimizer_state_dict(self.adam_m, self.adam_v, step, float(self.opt[0].item()),
                                                       self.cfg.weight_decay, self.obs_dim),
                "frame": self.frame,
                "last_mean_rewards": self.last_mean_rewards,
                "env_state": self.vec_env.get_env_state() if self.vec_env is not None else None}

    def set_full_state_weights(self, weights: Dict[str, Any]) -> None:
        ckpt.load_model_state_dict(weights["model"], self.model_params, self.obs_rms, self.val_rms, self.obs_dim)
        self.epoch_num = int(weights["epoch"])
        step, lr = ckpt.load_optimizer_state_dict(weights["optimizer"], self.adam_m, self.adam_v, self.obs_dim)
        self.opt[1] = step
        self.opt[0] = lr
        self.last_lr = lr
        self.frame = int(weights.get("frame", 0))
        self.last_mean_rewards = weights.get("last_mean_rewards", -100500)
        if self.vec_env is not None:
            self.vec_env.set_env_state(weights.get("env_state", None))

    def save(self, fn: str) -> None:
        ckpt.save_checkpoint(fn, self.get_full_state_weights())

    def restore(self, fn: str) -> None:
        self.set_full_state_weights(ckpt.load_checkpoint(fn))

    def get_weights(self):
        return {"model": ckpt.model_state_dict(self.model_params, self.obs_rms, self.val_rms, self.obs_dim)}

    def set_weights(self, weights):
        ckpt.load_model_state_dict(weights["model"], self.model_params, self.obs_rms, self.val_rms, self.obs_dim)
