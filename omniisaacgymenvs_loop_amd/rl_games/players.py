"""PpoPlayerContinuous (rl_games/rl_games/algos_torch/players.py:107-182,
common/player.py:319-423): runs the trained policy, deterministic (mu) by
default, through the same HIP forward used for the rollout."""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from .. import _capi
from .._abi import DEFINES
from . import checkpoint as ckpt
from . import vecenv
from .a2c_continuous import A2CAgent, default_linear_init

NIN, NA, NPARAM = DEFINES["PPO_NIN"], DEFINES["PPO_NA"], DEFINES["PPO_NPARAM"]


class PpoPlayerContinuous:
    def __init__(self, params: Dict[str, Any]):
        self.params = params
        config = params["config"]
        self.config = config
        self.device = config.get("device", "cuda:0")
        self.num_actors = int(config["num_actors"])
        self.env = config.get("vec_env") or vecenv.create_vec_env(config.get("env_name", "rlgpu"), self.num_actors,
                                                                   **config.get("env_config", {}))
        pcfg = params.get("player", {}) or {}
        self.is_deterministic = bool(pcfg.get("deterministic", True))
        self.games_num = int(pcfg.get("games_num", 2000))
        self.max_steps = int(pcfg.get("max_steps", 27000))
        dev = self.device
        info = self.env.get_env_info()
        osp = info["observation_space"]
        self.obs_dim = int((osp.spaces["state"].shape if hasattr(osp, "spaces") else osp.shape)[0])
        self.model_params = default_linear_init(int(params.get("seed", 42)), self.obs_dim).to(dev)
        self.obs_rms = torch.zeros(2 * NIN + 1, device=dev, dtype=torch.float64)
        self.obs_rms[NIN:2 * NIN] = 1.0
        self.obs_rms[2 * NIN] = 1.0
        self.val_rms = torch.tensor([0.0, 1.0, 1.0], device=dev, dtype=torch.float64)
        # reuse the agent's PPO config block and rollout kernel with H=1
        from .._abi import PpoCfg
        self.cfg = PpoCfg()
        self.cfg.horizon, self.cfg.n_envs, self.cfg.minibatch = 1, self.num_actors, 64
        self.cfg.normalize_input = int(bool(config.get("normalize_input", False)))
        self.cfg.normalize_value = int(bool(config.get("normalize_value", False)))
        self.cfg.rms_eps = 1e-5
        N = self.num_actors
        f32 = dict(device=dev, dtype=torch.float32)
        self._scratch = {k: torch.zeros(s, **f32) for k, s in
                         (("obs", (N, NIN)), ("act", (N, NA)), ("nlp", (N,)), ("val", (N,)), ("mu", (N, NA)),
                          ("sigma", (N, NA)))}
        self._done8 = torch.zeros(N, device=dev, dtype=torch.uint8)
        self._dones = torch.zeros(N, device=dev, dtype=torch.int64)
        self._actions = torch.zeros((N, NA), **f32)
        self._step = 0
        self._obs_pad = torch.zeros((N, NIN), **f32) if self.obs_dim < NIN else None

    def restore(self, fn: str) -> None:
        w = ckpt.load_checkpoint(fn)
        ckpt.load_model_state_dict(w["model"], self.model_params, self.obs_rms, self.val_rms, self.obs_dim)

    def get_action(self, obs: torch.Tensor, is_deterministic: bool = True) -> torch.Tensor:
        c = _capi
        sc = self._scratch
        if self._obs_pad is not None:   # k-input network: zero-padded to the kernels' NIN inputs
            self._obs_pad[:, :self.obs_dim].copy_(obs)
            obs = self._obs_pad
        c.call("ppo_policy_step", c.byref(self.cfg), c.ptr(self.model_params), c.ptr(self.obs_rms),
               c.ptr(self.val_rms), c.ptr(obs.contiguous()), 0, c.ptr(sc["obs"]), c.ptr(sc["act"]), c.ptr(sc["nlp"]),
               c.ptr(sc["val"]), c.ptr(sc["mu"]), c.ptr(sc["sigma"]), c.ptr(self._done8), c.ptr(self._dones),
               c.ptr(self._actions), int(self.params.get("seed", 42)), self._step, None, None, c.stream_ptr())
        self._step += 1
        if is_deterministic:
            return torch.clamp(sc["mu"], -1.0, 1.0)     # players.py:139-150: current_action = mu, clamped
        return self._actions

    def run(self):
        obs = self.env.reset()
        steps = torch.zeros(self.num_actors, device=self.device)
        rewards = torch.zeros(self.num_actors, device=self.device)
        sum_rewards, sum_steps, games = 0.0, 0.0, 0
        for _ in range(self.max_steps):
            a = self.get_action(obs["obs"]["state"], self.is_deterministic)
            obs, r, dones, _ = self.env.step(a)
            rewards += r
            steps += 1
            d = dones.bool()
            if bool(d.any()):
                n_done = int(d.sum())
                sum_rewards += float(rewards[d].sum())
                sum_steps += float(steps[d].sum())
                games += n_done
                rewards[d] = 0
                steps[d] = 0
                if games >= self.games_num:
                    break
        if games:
            print(f"av reward: {sum_rewards / games} av steps: {sum_steps / games}")
        return sum_rewards / max(games, 1)
