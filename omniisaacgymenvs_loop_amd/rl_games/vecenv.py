"""rl_games env registries (rl_games/rl_games/common/vecenv.py:215-232 and
common/env_configurations.py): the names the reference's launcher registers
(scripts/rlgames_train111.py:71-80) resolve here unchanged."""
from __future__ import annotations

from typing import Any, Callable, Dict

configurations: Dict[str, Dict[str, Any]] = {}
vecenv_config: Dict[str, Callable] = {}


def register(config_name: str, func: Callable) -> None:
    """vecenv.register('RLGPU', lambda config_name, num_actors, **kw: RLGPUEnv(...))"""
    vecenv_config[config_name] = func


def register_env(name: str, config: Dict[str, Any]) -> None:
    """env_configurations.register('rlgpu', {'vecenv_type': 'RLGPU', 'env_creator': ...})"""
    configurations[name] = config


def create_vec_env(config_name: str, num_actors: int, **kwargs):
    vec_env_name = configurations[config_name]["vecenv_type"]
    return vecenv_config[vec_env_name](config_name, num_actors, **kwargs)


class RLGPUEnv:
    """IVecEnv adapter (omniisaacgymenvs/utils/rlgames/rlgames_utils.py:102-126)."""

    def __init__(self, config_name: str, num_actors: int, **kwargs):
        self.env = configurations[config_name]["env_creator"](**kwargs)

    def __getattr__(self, name):
        # optional env extensions (advance_host_clock, ...) pass through to the wrapped env
        if name == "env":
            raise AttributeError(name)
        return getattr(self.env, name)

    def step(self, action):
        return self.env.step(action)

    def reset(self):
        return self.env.reset()

    def get_number_of_agents(self):
        return self.env.get_number_of_agents()

    def get_env_info(self):
        info = {"action_space": self.env.action_space, "observation_space": self.env.observation_space}
        if self.env.num_states > 0:
            info["state_space"] = self.env.state_space
        return info

    def set_train_info(self, env_frames, *args, **kwargs):
        if hasattr(self.env, "set_train_info"):
            self.env.set_train_info(env_frames, *args, **kwargs)

    def get_env_state(self):
        return self.env.get_env_state() if hasattr(self.env, "get_env_state") else None

    def set_env_state(self, env_state):
        if hasattr(self.env, "set_env_state"):
            self.env.set_env_state(env_state)
