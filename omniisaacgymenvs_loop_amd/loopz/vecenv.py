"""USVRaisimVecEnv (omniisaacgymenvs/envs/usv_raisim_vecenv.py:43-384): the raisimGymTorch-style
adapter the loopz trainer drives, over this package's VecEnvRLGames.

The reference API is numpy in / numpy out (observe() -> obs, step(action) -> (reward, dones));
observe_device() / step_device() return the device tensors without the host round trip and are
what scripts/loopz_train.py uses.  Observations and rewards are nan_to_num'd as the reference
does after its NaN probe (USV_NAN_PROBE=1 raises on a non-finite value first, :306-384)."""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch


@dataclass
class ScalingState:
    mean: Optional[np.ndarray] = None
    std: Optional[np.ndarray] = None


class USVRaisimVecEnv:
    def __init__(self, base_env: Any, *, reward_info_size: int = 16, device=None) -> None:
        self._env = base_env
        self._task = getattr(base_env, "_task", None)
        if self._task is None:
            raise ValueError("base_env must be a VecEnvRLGames-like env with attribute `_task`.")
        self._device = torch.device(device) if device is not None else torch.device(
            getattr(self._task, "rl_device", self._task.device))
        self.num_envs = int(getattr(self._env, "num_envs", self._task.num_envs))
        self.num_obs = int(self._task.num_observations)
        self.num_acts = int(self._task.num_actions)
        self._reward_info_size = int(reward_info_size)
        self._last_obs: Optional[torch.Tensor] = None
        self._last_rew: Optional[torch.Tensor] = None
        self._last_dones: Optional[torch.Tensor] = None
        self._last_extras: Dict[str, Any] = {}
        self._scaling = ScalingState()

    # ------------------------------------------------------------- device
    def reset_device(self) -> torch.Tensor:
        obs = self._extract(self._env.reset())
        self._probe(obs, "obs(reset)")
        self._last_obs = torch.nan_to_num(obs, nan=0.0, posinf=0.0, neginf=0.0)
        return self._last_obs

    def observe_device(self) -> torch.Tensor:
        if self._last_obs is None:
            self.reset_device()
        return self._last_obs

    def step_device(self, action: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        obs_dict, rew, resets, extras = self._env.step(action.to(self._device, torch.float32))
        obs = self._extract(obs_dict)
        self._probe(obs, "obs(step)")
        self._probe(rew, "reward(step)")
        self._last_obs = torch.nan_to_num(obs, nan=0.0, posinf=0.0, neginf=0.0)
        self._last_rew = torch.nan_to_num(rew, nan=0.0, posinf=0.0, neginf=0.0)
        self._last_dones = resets
        self._last_extras = extras if isinstance(extras, dict) else {"extras": extras}
        return self._last_rew, resets

    # --------------------------------------------------- reference (numpy)
    def reset(self) -> None:
        self.reset_device()

    def observe(self, *_args: Any, **_kwargs: Any) -> np.ndarray:
        return self.observe_device().detach().cpu().numpy().astype(np.float32, copy=False)

    def step(self, action) -> Tuple[np.ndarray, np.ndarray]:
        a = action if torch.is_tensor(action) else torch.from_numpy(np.asarray(action))
        rew, dones = self.step_device(a.float())
        return rew.detach().cpu().numpy().astype(np.float32).reshape(-1), \
            dones.detach().cpu().numpy().reshape(-1).astype(np.bool_)

    def get_reward_info(self) -> np.ndarray:
        info = np.zeros((self.num_envs, self._reward_info_size), np.float32)
        if self._last_rew is not None:
            info[:, 0] = self._last_rew.detach().cpu().numpy().reshape(-1)
        return info

    def get_extras(self) -> Dict[str, Any]:
        return self._last_extras

    def curriculum_callback(self) -> None:
        return None

    def save_scaling(self, directory: str, iteration, *_a, **_k) -> None:
        os.makedirs(directory, exist_ok=True)
        np.savez(os.path.join(directory, f"scaling_{iteration}.npz"),
                 mean=np.array([] if self._scaling.mean is None else self._scaling.mean, np.float32),
                 std=np.array([] if self._scaling.std is None else self._scaling.std, np.float32))

    def load_scaling(self, directory: str, iteration, *_a, **_k) -> None:
        path = os.path.join(directory, f"scaling_{iteration}.npz")
        if not os.path.exists(path):
            self._scaling = ScalingState()
            return
        d = np.load(path)   # allow_pickle=False (numpy default)
        mean, std = d.get("mean"), d.get("std")
        self._scaling = ScalingState(None if mean is None or mean.size == 0 else mean.astype(np.float32),
                                     None if std is None or std.size == 0 else std.astype(np.float32))

    def close(self) -> None:
        fn = getattr(self._env, "close", None)
        if callable(fn):
            fn()

    # ------------------------------------------------------------ helpers
    @staticmethod
    def _extract(obs_dict: Any) -> torch.Tensor:
        if isinstance(obs_dict, dict):
            obs = obs_dict.get("obs")
            if obs is None:
                raise KeyError("obs_dict does not contain key 'obs'.")
            if isinstance(obs, dict):
                if "state" in obs and torch.is_tensor(obs["state"]):
                    return obs["state"]
                vals = [v for v in obs.values() if torch.is_tensor(v)]
                if len(vals) == 1:
                    return vals[0]
                raise TypeError("obs_dict['obs'] is a dict but no single tensor could be inferred")
            if not torch.is_tensor(obs):
                raise TypeError("obs_dict['obs'] must be a torch.Tensor or a dict containing tensors")
            return obs
        if torch.is_tensor(obs_dict):
            return obs_dict
        raise TypeError("Unsupported observation type returned from base_env.reset/step")

    @staticmethod
    def _probe(t, name: str) -> None:
        """USV_NAN_PROBE (default on): raise on non-finite values before they are sanitised."""
        if os.getenv("USV_NAN_PROBE", "1") == "0" or t is None or not torch.is_tensor(t):
            return
        if not bool(torch.isfinite(t).all()):
            raise RuntimeError(f"[USV_NAN_PROBE] non-finite detected: {name}; shape={tuple(t.shape)}")
