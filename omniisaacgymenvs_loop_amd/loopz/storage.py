"""RolloutStorage (omniisaacgymenvs/algo/ppo/storage.py:44-148) as device buffers for the loopz
kernels: time-major [T][N] like the reference, so an in-order minibatch is a contiguous row
range; actor and critic observations are one buffer (the trainer feeds both the same
observation, scripts/rlgames_train.py:457-466)."""
from __future__ import annotations

import torch


class RolloutStorage:
    def __init__(self, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape, actions_shape, device):
        if list(actor_obs_shape) != list(critic_obs_shape):
            raise NotImplementedError("the loopz kernels share one observation buffer (actor == critic obs)")
        T, N = int(num_transitions_per_env), int(num_envs)
        f32 = dict(device=device, dtype=torch.float32)
        self.device = device
        self.num_transitions_per_env, self.num_envs = T, N
        self.actor_obs = torch.zeros((T, N, *actor_obs_shape), **f32)
        self.critic_obs = self.actor_obs
        self.rewards = torch.zeros((T, N), **f32)
        self.actions = torch.zeros((T, N, *actions_shape), **f32)
        self.dones = torch.zeros((T, N), device=device, dtype=torch.uint8)
        self.actions_log_prob = torch.zeros((T, N), **f32)
        self.values = torch.zeros((T, N), **f32)
        self.returns = torch.zeros((T, N), **f32)
        self.advantages = torch.zeros((T, N), **f32)
        self.step = 0

    def clear(self):
        self.step = 0
