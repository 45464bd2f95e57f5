"""USVVirtual: the CaptureXY task state on the GPU, stepped by libusv_hip.so.

Mirrors the task object the reference's VecEnvRLGames drives
(omniisaacgymenvs/tasks/USV_Virtual.py:56-1726 + tasks/base/rl_task.py):
same names for the buffers rl_games and the env wrapper touch (obs_buf,
rew_buf, reset_buf, progress_buf, extras, num_envs, num_observations,
num_actions, num_states, clip_obs, clip_actions, observation_space,
action_space, reset(), update_state(), get_states()), but every per-env
quantity is a struct-of-arrays device tensor and one control step is four
kernel launches (reset, potential field, step) with no host synchronisation.
"""
from __future__ import annotations

import ctypes
import os
from typing import Any, Dict, Optional

import numpy as np
import torch

from .. import _capi
from .._abi import DEFINES, UsvBufs, enum_values
from ..utils.spaces import Box, DictSpace
from .usv_config import (action_bias_cfg, build_hydro_cfg, build_usv_cfg, env_origins, has_disturbance,
                         raise_nan_flag, stat_names, thruster_tables)

NOBS = DEFINES["USV_NOBS"]
NOBST = DEFINES["USV_NOBST"]
GRID2 = DEFINES["USV_GRID"] ** 2
FIELD_STRIDE = DEFINES["USV_FIELD_STRIDE"]


NSTAT = DEFINES["USV_NSTAT"]
NU_RESET = DEFINES["USV_NU_RESET"]
NU_STEP = DEFINES["USV_NU_STEP"]
NDIST = enum_values("usv_dist_row")["USV_NDIST"]
TASK_CAPTURE_XY, TASK_TRACK_XYO = DEFINES["USV_TASK_CAPTURE_XY"], DEFINES["USV_TASK_TRACK_XYO"]
TS_ROWS = DEFINES["USV_TS_ROWS"]
CTL_N = DEFINES["USV_CTL_N"]


class _World:
    """Stand-in for omni.isaac.core World: physics runs inside the step kernel."""

    def is_playing(self) -> bool:
        return True

    def step(self, render: bool = False) -> None:
        return None


class USVVirtual:
    """CaptureXY task (USV_capture_xy_static_obs.CaptureXYTask glue) on MI355X."""

    def __init__(self, task_cfg: Dict[str, Any], num_envs: Optional[int] = None, device: str = "cuda:0",
                 seed: int = 42, rl_device: Optional[str] = None):
        if not torch.cuda.is_available():
            raise RuntimeError("USVVirtual needs a ROCm GPU (MI355X); there is no CPU path")
        self._task_cfg = task_cfg
        self._num_envs = int(num_envs if num_envs is not None else task_cfg["env"]["numEnvs"])
        self._device = device
        self.device = device
        self.rl_device = rl_device or device
        self.cfg = build_usv_cfg(task_cfg)
        self._max_episode_length = int(task_cfg["env"]["maxEpisodeLength"])
        # the reference's obs width: 3 + (5 + 5*3) + 2 + priv_dim (USV_core.py:46); the device rows keep
        # NOBS columns (a priv_dim = 4 row ends in 4 zero columns: the policy's padded input)
        self._num_observations = DEFINES["USV_NOBS_BASE"] + int(self.cfg.priv_dim)
        self._num_actions = 2
        self._num_states = 0
        self._num_agents = 1
        self.clip_obs = task_cfg["env"].get("clipObservations", {"state": 12.0})
        self.clip_actions = task_cfg["env"].get("clipActions", 1.0)
        self.control_frequency_inv = int(task_cfg["env"].get("controlFrequencyInv", 10))
        self.randomize_actions = False
        self.randomize_observations = False
        self.observation_space = DictSpace({"state": Box(-np.inf, np.inf, (self._num_observations,))})
        self.action_space = Box(np.array([-1.0, -1.0], np.float32), np.array([1.0, 1.0], np.float32))
        self.state_space = Box(-np.inf, np.inf, (0,))
        self._initial_action_bias, self._initial_action_bias_steps = action_bias_cfg(task_cfg)
        self._action_bias_step_count = 0
        self.seed = int(seed)
        self._step_index = 0
        self.step = 0.0                     # USVVirtual.step (+= 1/horizon per metrics call)
        self._horizon = int(task_cfg["env"].get("horizon_length", 16))
        self.grid_lin: Optional[torch.Tensor] = None
        self._alloc()
        self._env = self
        self._world = _World()

    # ------------------------------------------------------------------ buffers
    def _alloc(self):
        n, dev = self._num_envs, self._device
        f32 = dict(device=dev, dtype=torch.float32)
        i32 = dict(device=dev, dtype=torch.int32)
        Z = lambda *s, **k: torch.zeros(*s, **k)
        # Every per-env array the step kernel touches comes from ONE slab, so they share a < 2 GiB window that the
        # kernel addresses with buffer instructions (one 32-bit lane offset + a per-array offset; include/usv_hip.h,
        # usv_env_step).  With n a multiple of 64 the slab is the canonical layout of include/usv_hip.h (USV_SLAB_*:
        # array X at row USV_SLAB_X of 4 n-byte rows), and for power-of-two 4 n the step kernel takes its
        # constant-offset variant; otherwise the arrays are packed at 256-byte boundaries.
        slab_spec = [("state", (8, n), torch.float32, "STATE"), ("params", (9, n), torch.float32, "PARAMS"),
                     ("damp", (2, 3, n), torch.float32, "LIN_DAMP"), ("tgt", (2, n), torch.float32, "TGT"),
                     ("obst", (NOBST * 2, n), torch.float32, "OBST"), ("prev_cmd", (2, n), torch.float32, "PREV_CMD"),
                     ("hist", (4, n), torch.float32, "HIST"), ("ibuf", (5, n), torch.int32, "IBUF"),
                     ("just_reset", (n,), torch.uint8, "JUST_RESET"), ("stats", (NSTAT, n), torch.float32, "STATS"),
                     ("obs_buf_t", (n, NOBS), torch.float32, "OBS"), ("rew_buf", (n,), torch.float32, "REW"),
                     ("dones", (n,), torch.int64, "DONES"), ("field_old_tgt", (2, n), torch.float32, "FIELD_OLD_TGT"),
                     ("reset_ids", (n,), torch.int32, "RESET_IDS"), ("dist", (NDIST, n), torch.float32, "DIST"),
                     ("env_org", (2, n), torch.float32, "ENV_ORG"), ("tgt_h", (n,), torch.float32, "TGT_H"),
                     ("stale", (DEFINES["USV_STALE_ROWS"], n), torch.float32, "STALE")]
        sizes = [int(np.prod(shape)) * torch.empty((), dtype=dt).element_size() for _, shape, dt, _ in slab_spec]
        if n % 64 == 0:
            rb = 4 * n
            offs = [DEFINES[f"USV_SLAB_{key}"] * rb for _, _, _, key in slab_spec]
            total = DEFINES["USV_SLAB_ROWS"] * rb
            assert all(o + sz <= total for o, sz in zip(offs, sizes))
        else:
            offs = list(np.concatenate([[0], np.cumsum([(sz + 255) // 256 * 256 for sz in sizes])]))
            total = int(offs[-1])
        self._slab = torch.zeros(total, device=dev, dtype=torch.uint8)
        for (name, shape, dt, _), o, sz in zip(slab_spec, offs, sizes):
            setattr(self, name, self._slab[int(o):int(o) + sz].view(dt).view(shape))
        self.params[0] = self.cfg.base_mass
        self.params[4:8] = 1.0
        if self.cfg.drag_rand_on:
            for a in range(3):
                self.damp[0, a] = self.cfg.lin_damp[a]
                self.damp[1, a] = self.cfg.quad_damp[a]
        else:
            self.damp = None
        if not has_disturbance(self.cfg):
            self.dist = None
        # RLTask._env_pos (x, y): only the disturbance sinusoids read world positions
        self.env_org.copy_(torch.from_numpy(env_origins(n)))
        # TrackXYOVelocity's two-phase step: per-env rows + per-256-env-block partial sums
        self.task_scratch = (Z(TS_ROWS * n + (n + 255) // 256, **f32) if self.cfg.task_kind == TASK_TRACK_XYO
                             else None)
        self._has_field = self.cfg.task_kind == TASK_CAPTURE_XY
        self.field = Z((n if self._has_field else 1, FIELD_STRIDE), **f32)   # tiled raw cost of the field
        self.ibuf[2] = 1                               # RLTask.cleanup: reset_buf = ones
        self.just_reset.fill_(1)
        self.ctl = Z(CTL_N, **i32)
        self._ctl_host = None   # pinned copy of ctl (stage_ctl)
        self.fscratch = Z(16, **f32)
        self.extras_buf = Z(NSTAT, **f32)
        self.extras_acc = Z(((n + 255) // 256) * NSTAT, **f32)   # per reset-kernel workgroup (256 envs)
        self.slot_stats = Z((n, DEFINES["USV_FIELD_SLOT_STATS"]), **f32)
        # device step clock (next step, next bias call, current step, current bias call): the kernels take
        # the step index and the action bias from it, so a captured HIP graph replays consecutive steps
        self.clock = Z(DEFINES["USV_CLOCK_WORDS"], device=dev, dtype=torch.int64)
        self.states_buf = Z((n, 0), **f32)
        # the potential field in parts (include/usv_hip.h): .field = cost tiles, .fnorm = per-env constants (the SDF
        # comes from the obstacles), .sdf = the sweeps' raw cost rows
        self.sdf = Z((n if self._has_field else 1, FIELD_STRIDE), **f32)
        self.fnorm = Z((n if self._has_field else 1, DEFINES["USV_FNORM"]), **f32)
        # the overlapped step (env_step(.., overlap=True)): the reset envs' deferred reward terms, a side
        # stream for the field kernels and the fork / join events
        self.rstash = Z((DEFINES["USV_RSTASH_ROWS"], n), **f32) if self._has_field else None
        self._side = None
        self._ev_stats = None
        self._step_pending = False
        self._late_pending = False   # USV_LATE_ON_JOIN: an overlapped step's deferred reward waits for join_step
        self._host_dirty = True   # host-side buffer writes since the last join (the allocation's fills)
        self._side_tail_late = False   # the side stream's last work is an overlapped step's deferred reward
        self.lut = Z((2, 1000), **f32)
        self.hydro = build_hydro_cfg(self._task_cfg)
        tl, tr = thruster_tables(self._task_cfg)
        self._tables = torch.tensor(np.stack([tl, tr]), **f32)
        _capi.call("usv_build_lut", _capi.ptr(self._tables[0]), _capi.ptr(self._tables[1]), int(len(tl)),
                   _capi.ptr(self.lut), _capi.stream_ptr())
        self._init_scene_replay()
        # what step() returns: the reference's obs columns (a strided view of the NOBS-wide rows)
        self.obs_view = self.obs_buf_t[:, :self._num_observations]
        self._bufs = self._make_bufs()
        self.extras: Dict[str, Any] = {}

    def _init_scene_replay(self) -> None:
        """env.scene_replay (USV_Virtual.py:324-341): scenes on the device, per-env counters."""
        sr = self._task_cfg["env"].get("scene_replay", {}) or {}
        self.scene_replay_enabled = bool(sr.get("enabled", False))
        self.scene = self.scene_next = self.scene_last = None
        self.scene_replay_num_scenes = 0
        if not self.scene_replay_enabled:
            return
        from .scene_replay import load_scene_arrays, pack_scenes
        self.scene_replay_npz_path = os.path.abspath(str(sr.get("npz_path", "") or ""))
        self.scene_replay_cycle = bool(sr.get("cycle", True))
        rows = pack_scenes(load_scene_arrays(str(sr.get("npz_path", "") or ""), bool(sr.get("strict_hash", True))))
        self.scene = torch.tensor(rows, device=self._device)
        self.scene_replay_num_scenes = int(rows.shape[0])
        n = self._num_envs
        self.scene_next = torch.full((n,), int(sr.get("start_index", 0) or 0), device=self._device, dtype=torch.int32)
        self.scene_last = torch.full((n,), -1, device=self._device, dtype=torch.int32)

    @property
    def scene_replay_last_scene_idx(self) -> torch.Tensor:
        """Scene index applied at each env's last reset (-1 before the first), on the CPU."""
        if self.scene_last is None:
            return torch.full((self._num_envs,), -1, dtype=torch.long)
        return self.scene_last.long().cpu()

    def stage_ctl(self):
        """Enqueue a copy of the control words into pinned host memory on the current stream (behind the work
        already queued) and return it: after the caller's stream synchronisation the check_* methods read it
        from host memory instead of one blocking device read each."""
        if self._ctl_host is None or self._ctl_host.shape != self.ctl.shape:
            self._ctl_host = torch.empty(self.ctl.shape, dtype=self.ctl.dtype, pin_memory=True)
        self._ctl_host.copy_(self.ctl, non_blocking=True)
        return self._ctl_host

    def check_scene_replay(self, ctl=None) -> None:
        """Raise the reference's IndexError if a reset ran past the scenes with cycle off (host sync, or `ctl`:
        stage_ctl's copy once the stream has been synchronised)."""
        i = DEFINES["USV_CTL_SCENE_ERR"]
        if self.scene is not None and int(ctl[i] if ctl is not None else self.ctl[i].item()):
            raise IndexError(f"scene_replay index out of range: num_scenes={self.scene_replay_num_scenes}")

    def check_nan(self, ctl=None) -> None:
        """The reference's USV_NAN_PROBE fail-fast (USV_Virtual.py:57-95, vec_env_rlgames.py:41-80) for the
        steps since the last check: the step kernels OR the stage of any non-finite clamped action, state,
        reward or observation into ctl[USV_CTL_NAN_FLAG] (no per-step host sync); one read here (or `ctl`, as
        check_scene_replay)."""
        if not self.cfg.nan_probe:
            return
        i = DEFINES["USV_CTL_NAN_FLAG"]
        bits = int(ctl[i] if ctl is not None else self.ctl[i].item())
        if bits:
            self.ctl[i] = 0
            raise_nan_flag(bits, "env step")

    def _make_bufs(self) -> UsvBufs:
        b = UsvBufs()
        b.n = self._num_envs
        p = _capi.ptr
        for i, k in enumerate(("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr")):
            setattr(b, k, p(self.state[i]))
        for i, k in enumerate(("mass", "com_x", "com_y", "com_z", "k_drag", "thr_l", "thr_r", "k_iz", "mass_r")):
            setattr(b, k, p(self.params[i]))
        b.lin_damp = p(self.damp[0]) if self.damp is not None else None
        b.quad_damp = p(self.damp[1]) if self.damp is not None else None
        b.tgt_x, b.tgt_y = p(self.tgt[0]), p(self.tgt[1])
        b.obst = p(self.obst)
        b.field = p(self.field)
        b.prev_cmd = p(self.prev_cmd)
        b.prev_dist, b.prev_head, b.prev_pot, b.prev_wz = (p(self.hist[i]) for i in range(4))
        b.goal_cnt, b.progress, b.reset_buf, b.done_succ, b.done_coll = (p(self.ibuf[i]) for i in range(5))
        b.just_reset = p(self.just_reset)
        b.stats = p(self.stats)
        b.obs, b.rew, b.dones = p(self.obs_buf_t), p(self.rew_buf), p(self.dones)
        b.ctl, b.reset_ids, b.fscratch = p(self.ctl), p(self.reset_ids), p(self.fscratch)
        b.extras, b.extras_acc = p(self.extras_buf), p(self.extras_acc)
        b.field_old_tgt = p(self.field_old_tgt)
        b.slot_stats = p(self.slot_stats)
        b.sdf = p(self.sdf)
        b.fnorm = p(self.fnorm)
        b.clock = p(self.clock)
        b.rstash = p(self.rstash) if self.rstash is not None else None
        b.grid_lin = p(self.grid_lin) if self.grid_lin is not None else None
        b.dist = p(self.dist) if self.dist is not None else None
        b.env_org = p(self.env_org)
        b.tgt_h = p(self.tgt_h)
        b.stale = p(self.stale)
        b.task_scratch = p(self.task_scratch) if self.task_scratch is not None else None
        if self.scene is not None:
            b.scene, b.scene_next, b.scene_last = p(self.scene), p(self.scene_next), p(self.scene_last)
            b.n_scenes, b.scene_cycle = self.scene_replay_num_scenes, int(self.scene_replay_cycle)
        return b

    def field_rowmajor(self, ids=None) -> torch.Tensor:
        """The potential fields of envs `ids` (all by default) as row-major [k, 150 * 150] grids: what
        BatchedMapGPU returns per env, materialised from the parts the device keeps (usv_field_view)."""
        self.join_step()
        ids_t = (torch.arange(self._num_envs, device=self._device) if ids is None
                 else torch.as_tensor(ids, device=self._device).reshape(-1))
        ids_t = ids_t.to(torch.int32).contiguous()
        out = torch.empty((int(ids_t.numel()), GRID2), device=self._device, dtype=torch.float32)
        _capi.call("usv_field_view", _capi.byref(self.cfg), _capi.byref(self._bufs), _capi.ptr(ids_t),
                   int(ids_t.numel()), _capi.ptr(out), _capi.stream_ptr())
        return out

    def _touch(self) -> None:
        """A host-side write to the env buffers on the current stream: the next overlapped step runs its reset on
        that stream again (behind the write) instead of on the side stream (see _step_overlapped)."""
        self.join_step()
        self._host_dirty = True
        self._side_tail_late = False

    def set_env_origins(self, org: torch.Tensor) -> None:
        """World x, y of each env's origin ([2][n]; RLTask._env_pos from the stage)."""
        self._touch()
        self.env_org.copy_(org.to(self._device, torch.float32).reshape(2, self._num_envs))

    def set_grid_lin(self, lin: torch.Tensor) -> None:
        """Override the field grid's cell centres (parity tests vs CPU fixtures)."""
        self._touch()
        self.grid_lin = lin.to(self._device, torch.float32).contiguous()
        self._bufs = self._make_bufs()

    # ------------------------------------------------------------ RLTask API
    @property
    def num_envs(self) -> int:
        return self._num_envs

    @property
    def num_observations(self) -> int:
        return self._num_observations

    @property
    def num_actions(self) -> int:
        return self._num_actions

    @property
    def num_states(self) -> int:
        return self._num_states

    @property
    def num_agents(self) -> int:
        return self._num_agents

    @property
    def reset_buf(self) -> torch.Tensor:
        return self.ibuf[2]

    @property
    def progress_buf(self) -> torch.Tensor:
        return self.ibuf[1]

    @property
    def obs_buf(self) -> Dict[str, torch.Tensor]:
        return {"state": self.obs_view}

    def reset(self) -> None:
        """RLTask.reset: flag every env for reset (rl_task.py:268-270)."""
        self._touch()
        self.ibuf[2].fill_(1)

    def update_state(self) -> None:
        """Physics state lives in the SoA buffers; nothing to read back."""
        return None

    def get_states(self) -> torch.Tensor:
        return self.states_buf

    def advance_host_clock(self, steps: int) -> None:
        """Mirror `steps` device-clock steps (graph replays) on the host counters."""
        self._step_index += steps
        self._action_bias_step_count += steps
        self.step += steps / self._horizon

    def get_extras(self) -> Dict[str, Any]:
        return self.extras

    # -------------------------------------------------------------- stepping
    def current_action_bias(self) -> float:
        if self._initial_action_bias_steps > 0 and self._action_bias_step_count < self._initial_action_bias_steps:
            return float(self._initial_action_bias)
        return 0.0

    def env_step(self, actions: torch.Tensor, u_step: Optional[torch.Tensor] = None,
                 u_reset: Optional[torch.Tensor] = None, post_state: Optional[torch.Tensor] = None,
                 overlap: bool = False, chain: bool = False, after_fork=None):
        """pre_physics_step + 10 substeps + post_physics_step (USV_Virtual.py:1042-1652).

        Returns the device tensors (obs [n,33], rew [n], dones int64 [n]).  u_step / u_reset replay
        recorded uniforms (parity tests) instead of the in-kernel Philox draws.  post_state ([8][n]:
        px, py, yaw, vx, vy, wz, fl, fr) replaces the integrator by a recorded post-integration state:
        the step then runs pre_physics_step and RLTask.post_physics_step (rl_task.py:283-303) on that
        state, as the reference does on whatever PhysX returned (parity of the post-physics path alone).
        overlap: the overlapped step (_step_overlapped); chain: this overlapped step directly follows one in the
        same sequence of calls (a rollout, or one captured graph), so its reset may run on the side stream.
        after_fork: a callable issuing work that reads the previous step's rew / dones, run on the current stream
        before this step's env kernels write them (the default overlapped step: after the fields' fork)."""
        actions = self._f32(actions)
        s = _capi.stream_ptr()
        cfg, b = _capi.byref(self.cfg), _capi.byref(self._bufs)
        overlapped = overlap and self._has_field and post_state is None
        if after_fork is not None and not overlapped:
            after_fork()          # nothing forks: before any kernel of this step
            after_fork = None
        if (overlapped and chain and self._side_tail_late and not self._host_dirty and u_step is None
                and u_reset is None and os.getenv("USV_RESET_ON_SIDE", "0") == "1"):
            # (A/B knob, off: measured slower) the previous overlapped step's side stream ends
            # with its deferred reward; this step's reset and obstacle placement depend on that and on the dones
            # of its part 3 (final on this stream long before), not on this stream's later work (the next policy
            # step, the reward store), so they can run on the side stream right behind it
            bias, k = self._advance()
            if after_fork is not None:
                after_fork()
            return self._step_overlapped(actions, bias, k, u_step, reset_on_side=True)
        self.join_step()
        self._host_dirty = False
        bias, k = self._advance()
        # USV_FOLD_AFTER_FORK=1 (default): the overlapped step folds the episode extras (usv_reset_part 2) on this
        # stream after the side stream has forked for the fields, instead of between the reset and the obstacle
        # placement (the fold feeds nothing of the field chain, which bounds the step); 0: inside usv_reset
        fold_late = overlapped and os.getenv("USV_FOLD_AFTER_FORK", "1") == "1"
        if fold_late:
            _capi.call("usv_reset_part", cfg, b, self.seed, k, _capi.ptr(u_reset), 1, s)
        else:
            _capi.call("usv_reset", cfg, b, self.seed, k, _capi.ptr(u_reset), s)
        if overlapped:
            return self._step_overlapped(actions, bias, k, u_step, fold_late=fold_late, after_fork=after_fork)
        if self._has_field:   # CaptureXY only (GoToPose / TrackXYOVelocity have no obstacles)
            _capi.call("usv_potential_field", cfg, b, s)
        substeps = self.cfg.substeps
        if post_state is not None:
            self.state.copy_(post_state.to(self._device, torch.float32).reshape(8, self._num_envs))
            self.cfg.substeps = 0
        try:
            _capi.call("usv_env_step", cfg, b, _capi.ptr(actions), _capi.ptr(self.lut), ctypes.c_float(bias),
                       self.seed, k, _capi.ptr(u_step), s)
        finally:
            self.cfg.substeps = substeps
        return self.obs_view, self.rew_buf, self.dones

    def _step_overlapped(self, actions, bias, k, u_step, reset_on_side=False, fold_late=False, after_fork=None):
        """The rest of env_step with the reset envs' fields built on a side stream (usv_hip.h, the overlapped
        step): obstacle placement, then the step of every env (part 3) on this stream beside the sweeps /
        statistics / field kernels on the side stream, then the deferred reward of the reset envs there.
        The returned obs and dones are final on this stream; the rewards are final after join_step(), which
        the next env_step (or the caller, before reading rewards) issues.  Same results as the plain step."""
        cfg, b = _capi.byref(self.cfg), _capi.byref(self._bufs)
        main = torch.cuda.current_stream(self._device)
        if self._side is None:
            # USV_SIDE_PRIORITY: the side stream's priority (torch's convention: lower = higher priority)
            self._side = torch.cuda.Stream(device=self._device, priority=int(os.getenv("USV_SIDE_PRIORITY", "0")))
            self._ev_fork, self._ev_early, self._ev_join = (torch.cuda.Event() for _ in range(3))
        side = self._side
        # USV_STATS_FIRST=1: the main stream (the next policy step) waits for the field statistics, which then
        # run alone instead of beside the policy kernel (A/B knob)
        stats_first = os.getenv("USV_STATS_FIRST", "0") == "1"

        def side_fields():
            if stats_first:
                if self._ev_stats is None:
                    self._ev_stats = torch.cuda.Event()
                _capi.call("usv_field_stage", cfg, b, 3, side.cuda_stream)
                self._ev_stats.record(side)
                _capi.call("usv_field_stage", cfg, b, 4, side.cuda_stream)
            else:
                _capi.call("usv_field_stage", cfg, b, 2, side.cuda_stream)

        # USV_SIDE_FIRST=1 (default): the side stream's field kernels are captured right after the fork, before this
        # stream's deferred store and extras fold (a captured graph's launch gives the placement's first dependent
        # its queue, so the sweeps then follow the placement on one queue); 0: after them
        side_first = os.getenv("USV_SIDE_FIRST", "1") == "1" and not reset_on_side
        if reset_on_side:
            # reset + obstacle placement on the side stream behind the previous step's deferred reward; this
            # stream waits for the placement, then folds the episode extras (so what it reads of them between
            # steps is what the plain step leaves) and runs part 3 (every kernel sees the plain step's inputs)
            _capi.call("usv_reset_part", cfg, b, self.seed, k, None, 1, side.cuda_stream)
            _capi.call("usv_field_stage", cfg, b, 1, side.cuda_stream)
            self._ev_fork.record(side)
            main.wait_event(self._ev_fork)
            _capi.call("usv_reset_part", cfg, b, self.seed, k, None, 2, main.cuda_stream)
        else:
            _capi.call("usv_field_stage", cfg, b, 1, main.cuda_stream)
            self._ev_fork.record(main)
            side.wait_event(self._ev_fork)
            if side_first:
                side_fields()
            if after_fork is not None:
                after_fork()
            if fold_late:
                _capi.call("usv_reset_part", cfg, b, self.seed, k, None, 2, main.cuda_stream)
        if not side_first:
            side_fields()
        _capi.call("usv_env_step_part", cfg, b, _capi.ptr(actions), _capi.ptr(self.lut), ctypes.c_float(bias),
                   self.seed, k, _capi.ptr(u_step), 3, main.cuda_stream)
        if stats_first:
            main.wait_event(self._ev_stats)
        # USV_LATE_ON_JOIN=1: the deferred reward runs on the joining stream right after its wait for the fields; 0: on
        # the side stream behind part 3.  Unset: 0 from 32768 envs (the packed-sweep batches: with the round-6
        # schedule the side queue then runs constants -> deferred reward -> next reset back to back, rollout -1.6% at
        # 131072 envs, profiles/r06/r06zd_late_on_side_ab.txt), 1 below (-2% at 4096, r06ze_late_on_join_4096_ab.txt;
        # round 4: profiles/r04/r04z6_late_on_join_ab.txt)
        lj = os.getenv("USV_LATE_ON_JOIN", "")
        late_on_join = lj == "1" if lj in ("0", "1") else self._num_envs < 32768
        if late_on_join:
            self._ev_join.record(side)
            self._late_pending = True
        else:
            self._ev_early.record(main)
            side.wait_event(self._ev_early)
            _capi.call("usv_env_step_late", cfg, b, side.cuda_stream)
            self._ev_join.record(side)
        self._step_pending = True
        self._side_tail_late = not late_on_join
        return self.obs_view, self.rew_buf, self.dones

    def join_step(self) -> None:
        """Make the current stream wait for an overlapped step's side stream (rewards, fields final); with
        USV_LATE_ON_JOIN the step's deferred reward then runs on this stream."""
        if self._step_pending:
            cur = torch.cuda.current_stream(self._device)
            cur.wait_event(self._ev_join)
            self._step_pending = False
            if self._late_pending:
                self._late_pending = False
                _capi.call("usv_env_step_late", _capi.byref(self.cfg), _capi.byref(self._bufs), cur.cuda_stream)

    def _f32(self, actions: torch.Tensor) -> torch.Tensor:
        if actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.to(torch.float32).contiguous()
        return actions

    def _advance(self):
        """Host mirror of the step clock: (action bias, step index) of this step."""
        bias = self.current_action_bias()
        self._action_bias_step_count += 1
        k = self._step_index
        self._step_index += 1
        self.step += 1.0 / self._horizon
        if k == 0 or "episode" not in self.extras:
            # extras["episode"]: 0-d views of the device buffer written at every reset (USV_Virtual.py:1591-1612)
            self.extras = {"episode": {name: self.extras_buf[i] for name, i in stat_names(self.cfg)}}
        return bias, k

    def hydrostatics(self, quat: torch.Tensor, root_z: torch.Tensor):
        """HydrostaticsObject.compute_archimedes_metacentric_local fed as update_state feeds it
        (USV_Virtual.py:785-798, 1105-1109): quat [n][4] (w, x, y, z), root heights [n] ->
        (submerged volume [n], euler [n][3], body-frame wrench [n][6])."""
        quat = quat.to(self._device, torch.float32).contiguous()
        root_z = root_z.to(self._device, torch.float32).contiguous()
        n = int(root_z.shape[0])
        if tuple(quat.shape) != (n, 4):
            raise ValueError(f"quat must be [{n}, 4], got {tuple(quat.shape)}")
        vol = torch.empty(n, device=self._device, dtype=torch.float32)
        eul = torch.empty((n, 3), device=self._device, dtype=torch.float32)
        wr = torch.empty((n, 6), device=self._device, dtype=torch.float32)
        _capi.call("usv_hydrostatics", _capi.byref(self.hydro), n, _capi.ptr(quat), _capi.ptr(root_z),
                   _capi.ptr(vol), _capi.ptr(eul), _capi.ptr(wr), _capi.stream_ptr())
        return vol, eul, wr

    def forces(self) -> torch.Tensor:
        out = torch.empty((self._num_envs, 3), device=self._device, dtype=torch.float32)
        _capi.call("usv_forces", _capi.byref(self.cfg), _capi.byref(self._bufs), _capi.ptr(out), _capi.stream_ptr())
        return out
