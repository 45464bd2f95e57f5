"""Scene-replay NPZ files: deterministic A/B episodes.

Format = the output of the reference's scripts/build_usv_scenes.py:566-736
(keys obstacles_xy [S][M][2] NaN-padded, obstacles_count [S], start_pos [S][2],
start_yaw [S], start_vel [S][2], goal_pos [S][2], plus bookkeeping keys
num_episodes / episode_idx / seed / max_obstacles / generator_cfg / created_at,
and a `<file>.sha1` sidecar holding the SHA-1 of the npz bytes).

The loader follows USVVirtual._scene_replay_load_npz (tasks/USV_Virtual.py:1329-1369)
and packs each scene into one row of include/usv_hip.h's USV_SC_* layout, with the
obstacle list normalised the way CaptureXYTask.apply_scene does it
(USV_capture_xy_static_obs.py:829-842): padded / truncated to 16, entries at or
past obstacles_count sent to limbo (999, 999).  Arrays are read with
allow_pickle=False (the reference passes allow_pickle=True; the format needs no
pickled objects).  When scene_replay.strict_hash is set and the .sha1 sidecar
exists, its checksum must match the file (the reference stores the flag but does
not check it; a mismatch here raises ValueError).
"""
from __future__ import annotations

import datetime
import hashlib
import json
import os
from typing import Dict

import numpy as np

from .._abi import DEFINES

NOBST = DEFINES["USV_NOBST"]
STRIDE = DEFINES["USV_SCENE_STRIDE"]
SC_OBST, SC_START, SC_YAW = DEFINES["USV_SC_OBST"], DEFINES["USV_SC_START"], DEFINES["USV_SC_YAW"]
SC_VEL, SC_GOAL = DEFINES["USV_SC_VEL"], DEFINES["USV_SC_GOAL"]
REQUIRED = ("obstacles_xy", "obstacles_count", "start_pos", "start_yaw", "start_vel", "goal_pos")
LIMBO = 999.0


def sha1_of(path: str) -> str:
    h = hashlib.sha1()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 16), b""):
            h.update(chunk)
    return h.hexdigest()


def load_scene_arrays(npz_path: str, strict_hash: bool = True) -> Dict[str, np.ndarray]:
    """The six required arrays of a scene file (USV_Virtual.py:1334-1364 checks and errors)."""
    if not npz_path:
        raise ValueError("scene_replay.enabled=True but scene_replay.npz_path is empty")
    path = os.path.abspath(npz_path)
    if not os.path.exists(path):
        raise FileNotFoundError(f"scene_replay.npz_path not found: {path}")
    side = path + ".sha1"
    if strict_hash and os.path.exists(side):
        with open(side) as f:
            want = f.read().strip()
        got = sha1_of(path)
        if want != got:
            raise ValueError(f"scene_replay sha1 mismatch for {path}: file {got}, sidecar {want}")
    with np.load(path, allow_pickle=False) as npz:
        missing = [k for k in REQUIRED if k not in npz.files]
        if missing:
            raise KeyError(f"scene_replay npz missing keys={missing}; found={list(npz.files)}")
        data = {k: np.array(npz[k]) for k in REQUIRED}
    if int(data["start_pos"].shape[0]) <= 0:
        raise ValueError(f"scene_replay npz has no scenes: start_pos.shape={data['start_pos'].shape}")
    return data


def pack_scenes(data: Dict[str, np.ndarray]) -> np.ndarray:
    """[S][USV_SCENE_STRIDE] float32 rows for the reset kernel."""
    s = int(data["start_pos"].shape[0])
    rows = np.zeros((s, STRIDE), np.float32)
    obs = np.asarray(data["obstacles_xy"], np.float32)
    if obs.ndim != 3 or obs.shape[-1] < 2:
        raise ValueError(f"obstacles_xy must have shape (S, k, 2), got {obs.shape}")
    obs = obs[..., :2]
    k = obs.shape[1]
    full = np.full((s, NOBST, 2), LIMBO, np.float32)
    full[:, :min(k, NOBST)] = obs[:, :NOBST]
    cnt = np.clip(np.asarray(data["obstacles_count"], np.int64).reshape(-1), 0, NOBST)
    keep = np.arange(NOBST)[None, :] < cnt[:, None]
    full = np.where(keep[..., None], full, np.float32(LIMBO))
    rows[:, SC_OBST:SC_OBST + 2 * NOBST] = full.reshape(s, 2 * NOBST)
    rows[:, SC_START:SC_START + 2] = np.asarray(data["start_pos"], np.float32)[:, :2]
    rows[:, SC_YAW] = np.asarray(data["start_yaw"], np.float32).reshape(-1)
    rows[:, SC_VEL:SC_VEL + 2] = np.asarray(data["start_vel"], np.float32)[:, :2]
    rows[:, SC_GOAL:SC_GOAL + 2] = np.asarray(data["goal_pos"], np.float32)[:, :2]
    return rows


def write_scenes_npz(path: str, obstacles_xy, obstacles_count, start_pos, start_yaw, start_vel, goal_pos,
                     seed: int = 0, generator_cfg=None) -> str:
    """Write a scene file in build_usv_scenes.py's format (+ .sha1 sidecar); returns the sha1."""
    n = int(np.asarray(start_pos).shape[0])
    data = {
        "num_episodes": np.int64(n), "episode_idx": np.arange(n, dtype=np.int32),
        "seed": (seed + np.arange(n)).astype(np.int32), "max_obstacles": np.int64(np.asarray(obstacles_xy).shape[1]),
        "obstacles_xy": np.asarray(obstacles_xy, np.float32), "obstacles_count": np.asarray(obstacles_count, np.int32),
        "start_pos": np.asarray(start_pos, np.float32), "start_yaw": np.asarray(start_yaw, np.float32),
        "start_vel": np.asarray(start_vel, np.float32), "goal_pos": np.asarray(goal_pos, np.float32),
        "generator_cfg": np.array(json.dumps(generator_cfg or {})),
        "created_at": np.array(datetime.datetime(2026, 1, 1).isoformat()),
    }
    np.savez_compressed(path, **data)
    digest = sha1_of(path)
    with open(path + ".sha1", "w") as f:
        f.write(digest)
    return digest
