"""VecEnvRLGames: the omniisaacgymenvs env wrapper contract rl_games drives.

Reference: omniisaacgymenvs/envs/vec_env_rlgames.py:82-230.  step(actions)
returns ({"obs": {"state": [N,33]}, "states": [N,0]}, rew [N] fp32,
resets [N] int64, extras); reset() flags every env and runs one zero-action
step.  The 10 physics substeps, the reset path and the observation / reward /
done computation are one fused sequence of HIP kernels on the current stream
(no host synchronisation inside a step).
"""
from __future__ import annotations

from typing import Any, Dict, Optional

import torch


class VecEnvRLGames:
    def __init__(self, headless: bool = True, sim_device: int = 0, enable_livestream: bool = False,
                 enable_viewport: bool = False, **_: Any):
        self._headless = headless
        self._sim_device = sim_device
        self._render = not headless
        self._task = None
        self._world = None
        self.sim_frame_count = 0
        self._ctl_staged = None   # pinned copy of the task's control words (stage_errors)

    # omni.isaac.gym VecEnvBase.set_task
    def set_task(self, task, backend: str = "torch", sim_params: Optional[dict] = None, init_sim: bool = True) -> None:
        self._task = task
        self._world = task._world
        self._num_envs = task.num_envs
        self.num_envs = task.num_envs
        self.num_states = task.num_states
        self.state_space = task.state_space
        self.observation_space = task.observation_space
        self.action_space = task.action_space

    # ------------------------------------------------------------------ API
    def step(self, actions: torch.Tensor):
        t = self._task
        a = actions
        if a.device != torch.device(t.device):
            a = a.to(t.device)
        # clamp to clipActions happens inside the step kernel (vec_env_rlgames.py:136-140)
        obs, rew, dones = t.env_step(a)
        self.sim_frame_count += t.control_frequency_inv
        obs_dict = {"obs": {"state": obs}, "states": t.states_buf}
        return obs_dict, rew, dones, t.extras

    def step_async(self, actions: torch.Tensor, chain: bool = False, after_fork=None):
        """step() whose rewards are final only after join(): the reset envs' potential fields build on a side
        stream while the caller issues its next policy step (obs and dones are final on return).  chain=True
        when this call follows another step_async of the same rollout (one captured graph) with nothing but
        the caller's own kernels in between: the step's reset then runs on the side stream too.  after_fork:
        a callable issuing the caller's kernels that still read the previous step's rewards and dones; the step
        runs it on the current stream after the reset, the obstacle placement and the fields' fork, before its
        env kernels overwrite those buffers (off the field chain, which bounds the step)."""
        t = self._task
        a = actions if actions.device == torch.device(t.device) else actions.to(t.device)
        obs, rew, dones = t.env_step(a, overlap=True, chain=chain, after_fork=after_fork)
        self.sim_frame_count += t.control_frequency_inv
        return {"obs": {"state": obs}, "states": t.states_buf}, rew, dones, t.extras

    def join(self) -> None:
        join = getattr(self._task, "join_step", None)
        if join is not None:
            join()

    def reset(self):
        """Resets the task and applies zero actions to recompute observations (:219-230)."""
        self._task.reset()
        actions = torch.zeros((self.num_envs, self._task.num_actions), device=self._task.rl_device)
        obs_dict, _, _, _ = self.step(actions)
        return obs_dict

    def check_errors(self) -> None:
        """Raise the errors the device path flags instead of raising mid-step (a host sync; called
        by the trainer after each epoch, outside graph capture): scene replay past its last scene
        with cycle off -> IndexError, as USV_Virtual.py:1386-1390; a non-finite action, state, reward or
        observation -> the USV_NAN_PROBE RuntimeError (USV_Virtual.py:57-95, vec_env_rlgames.py:41-80).
        After stage_errors() and a stream synchronisation the flags come from its pinned host copy."""
        ctl, self._ctl_staged = self._ctl_staged, None
        for name in ("check_scene_replay", "check_nan"):
            chk = getattr(self._task, name, None)
            if chk is not None:
                chk(ctl)

    def stage_errors(self) -> None:
        """Enqueue the error flags' copy to pinned host memory behind the work on the current stream; the next
        check_errors() (after the caller synchronises that stream) reads the copy, not the device."""
        st = getattr(self._task, "stage_ctl", None)
        self._ctl_staged = st() if st is not None else None

    def advance_host_clock(self, steps: int) -> None:
        """A captured rollout graph was replayed: the device step clock advanced by `steps`."""
        self._task.advance_host_clock(steps)
        self.sim_frame_count += steps * self._task.control_frequency_inv

    def get_number_of_agents(self) -> int:
        return 1

    def get_env_info(self) -> Dict[str, Any]:
        info = {"action_space": self.action_space, "observation_space": self.observation_space}
        if self.num_states > 0:
            info["state_space"] = self.state_space
        return info

    def set_train_info(self, env_frames, *args, **kwargs):
        pass

    def get_env_state(self):
        return None

    def set_env_state(self, env_state):
        pass

    def close(self):
        pass
