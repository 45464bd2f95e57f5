"""ORACLE / TEST INFRASTRUCTURE ONLY.

ctypes front-end of oracle/build/libusv_oracle.so (the C restatement of the
reference env path, oracle/usv_oracle.c) plus helpers shared by the tests,
__graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product package
(omniisaacgymenvs_loop_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# USV_ORACLE_OMP=1: the OpenMP build of the same source (bench.py's cpu_baseline on all host cores;
# bit-identical results, every parallel loop is over independent envs / reset slots)
LIB_PATH = os.path.join(HERE, "build", "libusv_oracle_omp.so" if os.environ.get("USV_ORACLE_OMP") == "1"
                        else "libusv_oracle.so")

NOBS, NOBST, GRID, NSTAT = 33, 16, 150, 28
NU_RESET, NU_STEP = 718, 8
RU_TRIG = 712      # include/usv_hip.h: the recorded reference sin / cos of the reset (cfg.inj_trig)
NDIST = 11
NDBG = 20          # usv_oracle.c USV_ORACLE_NDBG: per-env diagnostics of the last step
CTL_POT_VALID, CTL_PEN_VALID, CTL_REW_VALID = 1, 2, 3

_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", HERE])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        _lib.oracle_step.argtypes = [P, P, P, P, ctypes.c_float, P]
        _lib.oracle_reset.argtypes = [P, P, ctypes.c_int, P, P]
        _lib.oracle_reset_scene.argtypes = [P, P, ctypes.c_int, P, P, P]
        _lib.oracle_potential_field.argtypes = [P, ctypes.c_int, P, P, P, P, P]
        _lib.oracle_step_pre.argtypes = [P, P, P, P, ctypes.c_float, P]
        _lib.oracle_step_physics.argtypes = [P, P]
        _lib.oracle_step_post.argtypes = [P, P, P]
        _lib.oracle_grid_lin.argtypes = [ctypes.c_float, P]
        _lib.oracle_lut.argtypes = [P, ctypes.c_int, ctypes.c_int, P]
        _lib.oracle_forces.argtypes = [P, P, P]
        _lib.oracle_forces_q.argtypes = [P, P, P, P]
        _lib.oracle_sincos_cr.argtypes = [P, ctypes.c_int, P, P]
        _lib.oracle_quat.argtypes = [P, ctypes.c_int, P]
        _lib.oracle_hydrostatics.argtypes = [P, ctypes.c_int, P, P, P, P, P]
        _lib.oracle_compact.argtypes = [P, P]
        _lib.oracle_compact.restype = ctypes.c_int
        _lib.oracle_step_uniforms.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, P]
        _lib.oracle_reset_uniforms.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, P, P]
        _lib.oracle_philox.argtypes = [P, P, P]
        _lib.oracle_sample_field.argtypes = [P, ctypes.c_float, ctypes.c_float, ctypes.c_float]
        _lib.oracle_sample_field.restype = ctypes.c_float
        _lib.oracle_threads.restype = ctypes.c_int
        _lib.oracle_set_skip_field.argtypes = [ctypes.c_int]
    return _lib


def _p(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(ctypes.c_void_p)


_PTR_FIELDS =  ("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr",
                                  "mass", "com_x", "com_y", "com_z", "k_drag", "thr_l", "thr_r", "k_iz", "mass_r",
                                  "lin_damp", "quad_damp", "tgt_x", "tgt_y", "obst", "field", "prev_cmd",
                                  "prev_dist", "prev_head", "prev_pot", "prev_wz", "goal_cnt", "progress",
                                  "reset_buf", "just_reset", "done_succ", "done_coll", "stats", "obs", "rew")


class _OracleEnvC(ctypes.Structure):
    _fields_ = ([("n", ctypes.c_int)] + [(k, ctypes.c_void_p) for k in _PTR_FIELDS] +
                [("ctl", ctypes.c_int32 * 20), ("extras", ctypes.c_float * NSTAT), ("dbg", ctypes.c_void_p),
                 ("tmp", ctypes.c_void_p), ("grid_lin", ctypes.c_void_p), ("dist", ctypes.c_void_p),
                 ("env_org", ctypes.c_void_p), ("tgt_h", ctypes.c_void_p), ("step_f", ctypes.c_double),
                 ("pot_in", ctypes.c_void_p), ("pos_in", ctypes.c_void_p), ("root_cache", ctypes.c_void_p)])


class OracleEnv:
    """Host SoA env state driven by the C oracle (mirrors usv_bufs_t)."""

    F32 = ("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr", "mass", "com_x", "com_y", "com_z", "k_drag",
           "thr_l", "thr_r", "k_iz", "mass_r", "tgt_x", "tgt_y", "tgt_h", "prev_dist", "prev_head", "prev_pot",
           "prev_wz", "rew")
    I32 = ("goal_cnt", "progress", "reset_buf", "done_succ", "done_coll")

    def __init__(self, cfg, n: int, lut: np.ndarray, with_field: bool = True):
        self.cfg, self.n = cfg, n
        self.lut = np.ascontiguousarray(lut, np.float32)
        for k in self.F32:
            setattr(self, k, np.zeros(n, np.float32))
        for k in self.I32:
            setattr(self, k, np.zeros(n, np.int32))
        self.mass[:] = cfg.base_mass
        self.k_drag[:] = 1.0
        self.thr_l[:] = 1.0
        self.thr_r[:] = 1.0
        self.k_iz[:] = 1.0
        self.reset_buf[:] = 1
        self.just_reset = np.ones(n, np.uint8)
        self.obst = np.zeros((NOBST, 2, n), np.float32)
        self.field = np.zeros((n if cfg.task_kind == 0 else 1, GRID * GRID), np.float32)
        self.prev_cmd = np.zeros((2, n), np.float32)
        self.stats = np.zeros((NSTAT, n), np.float32)
        self.obs = np.zeros((n, NOBS), np.float32)
        self.dbg = np.zeros((n, NDBG), np.float32)
        self.tmp = np.zeros((n, 8), np.float32)
        self.grid_lin = None
        self.lin_damp = np.zeros((3, n), np.float32) if cfg.drag_rand_on else None
        self.quad_damp = np.zeros((3, n), np.float32) if cfg.drag_rand_on else None
        if self.lin_damp is not None:
            for a in range(3):
                self.lin_damp[a] = cfg.lin_damp[a]
                self.quad_damp[a] = cfg.quad_damp[a]
        self.c = _OracleEnvC()
        self.c.n = n
        for k in self.F32 + self.I32 + ("just_reset", "obst", "field", "prev_cmd", "stats", "obs"):
            setattr(self.c, k, _p(getattr(self, k)))
        self.c.dbg = _p(self.dbg)
        self.c.tmp = _p(self.tmp)
        # the reference's cached root state (px, py, yaw, vx, vy, wz) at a reset env's first substep (App. C.1)
        self.root_cache = np.zeros((6, n), np.float32)
        self.c.root_cache = _p(self.root_cache)
        self.c.lin_damp = _p(self.lin_damp) if self.lin_damp is not None else None
        self.c.quad_damp = _p(self.quad_damp) if self.quad_damp is not None else None
        # disturbance parameters (zeros until drawn at reset) and env origins
        self.dist = np.zeros((NDIST, n), np.float32) if has_dist(cfg) else None
        self.c.dist = _p(self.dist) if self.dist is not None else None
        self.env_org = None
        self.scenes = None

    def set_env_origins(self, org):
        self.env_org = np.ascontiguousarray(org, np.float32).reshape(2, self.n)
        self.c.env_org = _p(self.env_org)

    @property
    def extras(self):
        return np.array(self.c.extras[:], np.float32)

    def ctl(self, i):
        return self.c.ctl[i]

    def compact(self):
        ids = np.zeros(self.n, np.int32)
        k = lib().oracle_compact(ctypes.byref(self.c), _p(ids))
        return ids[:k].copy()

    def reset(self, ids: np.ndarray, U: np.ndarray):
        ids = np.ascontiguousarray(ids, np.int32)
        U = np.ascontiguousarray(U, np.float32).reshape(len(ids), NU_RESET)
        rows = None
        if self.scenes is not None:
            # USVVirtual._scene_replay_take_scene_indices (USV_Virtual.py:1372-1393)
            idx = self.scene_next[ids].copy()
            self.scene_next[ids] += 1
            if self.scene_cycle:
                idx = idx % len(self.scenes)
            elif (idx < 0).any() or (idx >= len(self.scenes)).any():
                raise IndexError(f"scene_replay index out of range: idx={idx.tolist()}")
            self.scene_last[ids] = idx
            rows = np.ascontiguousarray(self.scenes[idx], np.float32)
        lib().oracle_reset_scene(ctypes.byref(self.cfg), ctypes.byref(self.c), len(ids), _p(ids), _p(U),
                                 _p(rows) if rows is not None else None)

    def set_scenes(self, rows, start_index=0, cycle=True):
        """Scene replay: packed scene rows [S][USV_SCENE_STRIDE] and the per-env counters."""
        self.scenes = np.ascontiguousarray(rows, np.float32)
        self.scene_next = np.full(self.n, start_index, np.int64)
        self.scene_last = np.full(self.n, -1, np.int64)
        self.scene_cycle = cycle

    def step(self, actions: np.ndarray, bias: float, U: np.ndarray):
        actions = np.ascontiguousarray(actions, np.float32)
        U = np.ascontiguousarray(U, np.float32)
        lib().oracle_step(ctypes.byref(self.cfg), ctypes.byref(self.c), _p(actions), _p(self.lut),
                          ctypes.c_float(bias), _p(U))

    def full_step(self, actions, bias, step_idx, seed=0, U_step=None, U_reset=None, pot_in=None, pos_in=None):
        """reset_idx (if any) + step, drawing Philox uniforms unless injected.  pot_in / pos_in: the parity
        harness's device potential samples [n] and post-integration positions [2][n] (see set_device_samples)."""
        ids = self.compact()
        if len(ids):
            if U_reset is None:
                U_reset = reset_uniforms(seed, step_idx, ids)
            self.reset(ids, U_reset)
        if U_step is None:
            U_step = step_uniforms(seed, step_idx, self.n)
        self.set_device_samples(pot_in, pos_in)
        self.step(actions, bias, U_step)
        self.set_device_samples(None, None)
        return ids

    def set_device_samples(self, pot_in=None, pos_in=None):
        """Feed the device's potential samples to the next step's CaptureXY reward (the oracle's own samples go
        to dbg[:, 14]) and have the oracle sample its own field at the device's positions into dbg[:, 15]: the
        reward is then checked at 1e-5 with no potential-sample allowance, the sample itself separately."""
        self._pot_in = None if pot_in is None else np.ascontiguousarray(pot_in, np.float32).reshape(self.n)
        self._pos_in = None if pos_in is None else np.ascontiguousarray(pos_in, np.float32).reshape(2, self.n)
        self.c.pot_in = _p(self._pot_in) if self._pot_in is not None else None
        self.c.pos_in = _p(self._pos_in) if self._pos_in is not None else None

    def set_grid_lin(self, lin):
        self.grid_lin = np.ascontiguousarray(lin, np.float32)
        self.c.grid_lin = _p(self.grid_lin)

    def step_pre(self, actions, bias, U):
        self._a = np.ascontiguousarray(actions, np.float32)
        self._U = np.ascontiguousarray(U, np.float32)
        lib().oracle_step_pre(ctypes.byref(self.cfg), ctypes.byref(self.c), _p(self._a), _p(self.lut),
                              ctypes.c_float(bias), _p(self._U))

    def step_physics(self):
        lib().oracle_step_physics(ctypes.byref(self.cfg), ctypes.byref(self.c))

    def step_post(self, U):
        self._U = np.ascontiguousarray(U, np.float32)
        lib().oracle_step_post(ctypes.byref(self.cfg), ctypes.byref(self.c), _p(self._U))

    def forces(self, quat=None):
        """Planar X, Y, N of the env state; quat [n][4] (w, 0, 0, z): the drag's attitude given as the reference's
        own quaternions instead of the stand-in's quaternion of the yaw."""
        out = np.zeros((self.n, 3), np.float32)
        q = None if quat is None else np.ascontiguousarray(quat, np.float32).reshape(self.n, 4)
        lib().oracle_forces_q(ctypes.byref(self.cfg), ctypes.byref(self.c), _p(q) if q is not None else None, _p(out))
        return out


def hydrostatics(h, quat: np.ndarray, z: np.ndarray):
    """Hydrostatic wrench per env (oracle_hydrostatics): h is a usv_config.UsvHydro."""
    n = len(z)
    quat = np.ascontiguousarray(quat, np.float32)
    z = np.ascontiguousarray(z, np.float32)
    vol, eul, wr = np.zeros(n, np.float32), np.zeros((n, 3), np.float32), np.zeros((n, 6), np.float32)
    lib().oracle_hydrostatics(ctypes.byref(h), n, _p(quat), _p(z), _p(vol), _p(eul), _p(wr))
    return vol, eul, wr


def has_dist(cfg) -> bool:
    return bool(cfg.fdist_on or cfg.tdist_on or cfg.current_on)


def make_lut(table_l, table_r, n_out=1000):
    out = np.zeros((2, n_out), np.float32)
    for i, t in enumerate((table_l, table_r)):
        t = np.ascontiguousarray(t, np.float32)
        row = np.zeros(n_out, np.float32)
        lib().oracle_lut(_p(t), len(t), n_out, _p(row))
        out[i] = row
    return out


def grid_lin(map_size=30.0):
    out = np.zeros(GRID, np.float32)
    lib().oracle_grid_lin(ctypes.c_float(map_size), _p(out))
    return out


def potential_field(cfg, obst: np.ndarray, tgt: np.ndarray, want_cost=False, lin=None):
    lin = None if lin is None else np.ascontiguousarray(lin, np.float32)
    obst = np.ascontiguousarray(obst, np.float32)
    tgt = np.ascontiguousarray(tgt, np.float32)
    k = obst.shape[0]
    field = np.zeros((k, GRID * GRID), np.float32)
    cost = np.zeros((k, GRID * GRID), np.float32) if want_cost else None
    lib().oracle_potential_field(ctypes.byref(cfg), k, _p(obst), _p(tgt), _p(field),
                                 _p(cost) if want_cost else None, _p(lin) if lin is not None else None)
    return (field, cost) if want_cost else field


def step_uniforms(seed, step, n):
    u = np.zeros((n, NU_STEP), np.float32)
    lib().oracle_step_uniforms(seed, step, n, _p(u))
    return u


def reset_uniforms(seed, step, ids):
    ids = np.ascontiguousarray(ids, np.int32)
    u = np.zeros((len(ids), NU_RESET), np.float32)
    lib().oracle_reset_uniforms(seed, step, len(ids), _p(ids), _p(u))
    return u


def sincos(x):
    """The integrator's sin / cos (usv_oracle.c:usv_sincos) of a float32 array."""
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    lib().oracle_sincos(_p(x), ctypes.c_int(x.size), _p(s), _p(c))
    return s, c


def sincos_cr(x):
    """sin / cos where the reference calls torch.sin / torch.cos on the state path (usv_oracle.c:usv_sincos_cr: a
    double evaluation rounded to float)."""
    x = np.ascontiguousarray(x, np.float32)
    s, c = np.empty_like(x), np.empty_like(x)
    lib().oracle_sincos_cr(_p(x), ctypes.c_int(x.size), _p(s), _p(c))
    return s, c


def quat(yaw):
    """Per yaw: (C, S) of quaternion_to_matrix of the stand-in's quaternion, the update_state heading and the yaw
    set_world_poses recovers from that quaternion (usv_oracle.c:oracle_quat) -> [n][4] float32."""
    yaw = np.ascontiguousarray(yaw, np.float32)
    out = np.empty((yaw.size, 4), np.float32)
    lib().oracle_quat(_p(yaw), ctypes.c_int(yaw.size), _p(out))
    return out


def math3(x, y):
    """The observation / reward functions (usv_oracle.c:usv_exp, usv_tanh, usv_atan2) of float32 arrays:
    (exp(x), tanh(x), atan2(y, x))."""
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y, np.float32)
    e, t, a = np.empty_like(x), np.empty_like(x), np.empty_like(x)
    lib().oracle_math(_p(x), _p(y), ctypes.c_int(x.size), _p(e), _p(t), _p(a))
    return e, t, a


def philox(ctr, key):
    c = np.ascontiguousarray(ctr, np.uint32)
    k = np.ascontiguousarray(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib().oracle_philox(_p(c), _p(k), _p(o))
    return o
