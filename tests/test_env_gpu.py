"""HIP env kernels (libusv_hip.so via the C ABI) vs the reference fixtures and the C oracle.

* fixture replay: the reference's own recorded draws injected into the kernels;
* Philox mode: kernels draw in-kernel, the oracle replays the same Philox streams;
* potential field: bit-exact against the reference fixture and the oracle;
* full-size properties at BASELINE sizes (determinism, finiteness, resets).
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O
from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml, stat_names, thruster_tables
from tests.test_oracle_golden import GOLDEN_DIR, TEST_YAML, scene_rows

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _task(cfg_d, n):
    from omniisaacgymenvs_loop_amd.tasks.usv_virtual import USVVirtual
    return USVVirtual(cfg_d, num_envs=n, device=DEV, seed=7)


@pytest.mark.parametrize("variant", ["A", "B", "C", "D", "E", "P", "T", "S"])
def test_fixture_replay_on_gpu(golden, variant):
    d = golden(f"episode_{variant}.npz")
    cfg_d = json.loads(bytes(d["config_json"]).decode())
    if cfg_d["env"]["scene_replay"].get("enabled"):
        cfg_d["env"]["scene_replay"]["npz_path"] = os.path.join(GOLDEN_DIR, "scenes_S.npz")
    T, n = d["obs"].shape[:2]
    task = _task(cfg_d, n)
    task.set_grid_lin(torch.tensor(d["grid_lin"]))
    task.set_env_origins(torch.zeros(2, n))   # the fixtures' _env_pos (make_golden.build_usv)
    task.tgt[0] = torch.tensor(d["init_tgt"][:, 0], device=DEV)
    task.tgt[1] = torch.tensor(d["init_tgt"][:, 1], device=DEV)
    ru = 0
    for t in range(T):
        mask = d["reset_mask"][t]
        np.testing.assert_array_equal(task.reset_buf.cpu().numpy().astype(bool), mask)
        ids = np.nonzero(mask)[0]
        U = np.zeros((n, O.NU_RESET), np.float32)
        U[ids] = d["reset_U"][ru:ru + len(ids)]
        ru += len(ids)
        assert task.current_action_bias() == pytest.approx(float(d["bias"][t]))
        obs, rew, dones = task.env_step(torch.tensor(d["actions"][t], device=DEV),
                                        u_step=torch.tensor(d["u_step"][t], device=DEV),
                                        u_reset=torch.tensor(U, device=DEV))
        torch.cuda.synchronize()
        np.testing.assert_allclose(obs.cpu().numpy(), d["obs"][t], rtol=3e-5, atol=3e-5, err_msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), d["rew"][t], rtol=2e-4, atol=2e-4, err_msg=f"rew t={t}")
        np.testing.assert_array_equal(dones.cpu().numpy(), d["reset"][t])
        if len(ids):
            ex = task.extras_buf.cpu().numpy()
            if "extras_names" in d:   # GoToPose / TrackXYOVelocity episode_sums keys
                ex = ex[[slot for _, slot in stat_names(task.cfg)]]
            # episode means of per-step sums: they carry the integrator's ~1e-7 drift vs the reference
            np.testing.assert_allclose(ex, d["extras"][t], rtol=1e-4, atol=1e-5)
        if "scene_last" in d:
            np.testing.assert_array_equal(task.scene_replay_last_scene_idx.numpy(), d["scene_last"][t])
        if "tgt_h" in d:
            np.testing.assert_allclose(task.tgt.cpu().numpy().T, d["tgt"][t], rtol=1e-6, atol=1e-6)
            np.testing.assert_allclose(task.tgt_h.cpu().numpy(), d["tgt_h"][t], rtol=1e-6, atol=1e-6)
        if "dist" in d:   # disturbance parameters drawn by the reset kernel (USV_disturbances.py:327-508)
            np.testing.assert_allclose(task.dist.cpu().numpy(), d["dist"][t], rtol=1e-6, atol=1e-6)


def assert_obs_close(got, want, tol, msg=""):
    """obs parity; a row may differ only by the order of two obstacles whose distances tie to
    within the tolerance (torch.topk on distances that differ in the last bits: many envs of a
    replayed scene sit at the same point, where 1-ulp position differences reorder a near tie)."""
    bad = ~np.isclose(got, want, rtol=tol, atol=tol)
    rows = np.nonzero(bad.any(1))[0]
    for r in rows:
        other = np.r_[0:8, 23:33]
        np.testing.assert_allclose(got[r, other], want[r, other], rtol=tol, atol=tol, err_msg=f"{msg} row {r}")
        dg, dw = got[r, 8:23:3], want[r, 8:23:3]
        np.testing.assert_allclose(np.sort(dg), np.sort(dw), rtol=tol, atol=tol, err_msg=f"{msg} row {r}")
        assert np.min(np.abs(np.diff(np.sort(dw)))) < 10 * tol, f"{msg} row {r}: obstacle order differs without a tie"
    assert len(rows) <= max(1, got.shape[0] // 1000), f"{msg}: {len(rows)} rows differ"


def _oracle_for(cfg, n, task_cfg):
    lut = O.make_lut(*thruster_tables(task_cfg))
    return O.OracleEnv(cfg, n, lut)


def test_philox_mode_matches_oracle():
    """In-kernel Philox draws == the oracle's restatement of the same streams."""
    task_cfg = load_yaml(TEST_YAML)
    n, T = 2048, 24
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    rng = np.random.default_rng(0)
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        E.full_step(a, bias, t, seed=task.seed)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"dones t={t}")
        np.testing.assert_allclose(obs.cpu().numpy(), E.obs, rtol=1e-4, atol=1e-4, err_msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), E.rew, rtol=1e-3, atol=1e-3, err_msg=f"rew t={t}")
    # per-episode parameters drawn by the reset kernel
    np.testing.assert_allclose(task.params[0].cpu().numpy(), E.mass, rtol=1e-6)
    np.testing.assert_allclose(task.obst.cpu().numpy().reshape(16, 2, n), E.obst, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("frame", ["local", "global"])
def test_philox_priv4_matches_oracle(frame):
    """priv_dim 4 (every reference yaml but TEST): 29-column rows, the slab's 4 pad columns stay 0."""
    task_cfg = load_yaml(TEST_YAML)
    task_cfg["env"].pop("mass_dim", None)
    task_cfg["env"]["priv_dim"] = 4
    task_cfg["env"]["observation_frame"] = frame
    n, T = 2048, 16
    task = _task(task_cfg, n)
    assert task.num_observations == 29
    E = _oracle_for(task.cfg, n, task_cfg)
    rng = np.random.default_rng(3)
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        E.full_step(a, bias, t, seed=task.seed)
        torch.cuda.synchronize()
        assert obs.shape == (n, 29)
        assert float(task.obs_buf_t[:, 29:].abs().max()) == 0.0
        np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"dones t={t}")
        np.testing.assert_allclose(obs.cpu().numpy(), E.obs[:, :29], rtol=1e-4, atol=1e-4, err_msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), E.rew, rtol=1e-3, atol=1e-3, err_msg=f"rew t={t}")


def test_philox_mode_disturbances_matches_oracle():
    """Force / torque disturbances + water current, env origins on the reference's
    fallback grid (USV_Virtual.py:1670-1696): kernels vs the oracle on Philox draws."""
    task_cfg = load_yaml(TEST_YAML)
    dist = task_cfg["env"]["disturbances"]
    for key in ("use_force_disturbance", "use_constant_force", "use_sinusoidal_force"):
        dist["forces"][key] = True
    for key in ("use_torque_disturbance", "use_constant_torque", "use_sinusoidal_torque"):
        dist["torques"][key] = True
    task_cfg["env"]["water_current"] = {"use_water_current": True, "flow_velocity": [-0.2, 0.35, 0.0]}
    task_cfg["env"]["maxEpisodeLength"] = 20
    n, T = 1024, 30
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    E.set_env_origins(task.env_org.cpu().numpy())
    assert float(task.env_org.max()) > 0
    rng = np.random.default_rng(5)
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        E.full_step(a, bias, t, seed=task.seed)
        torch.cuda.synchronize()
        np.testing.assert_allclose(task.dist.cpu().numpy(), E.dist, rtol=1e-6, atol=1e-6, err_msg=f"dist t={t}")
        np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"dones t={t}")
        np.testing.assert_allclose(obs.cpu().numpy(), E.obs, rtol=1e-4, atol=1e-4, err_msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), E.rew, rtol=1e-3, atol=1e-3, err_msg=f"rew t={t}")


@pytest.mark.parametrize("name", ["GoToPose", "TrackXYOVelocity"])
def test_philox_mode_pose_tasks_match_oracle(golden, name):
    """SURVEY A20 tasks at 4096 envs with in-kernel draws vs the oracle (TrackXYOVelocity's
    all-env angular sum included)."""
    d = golden("episode_P.npz" if name == "GoToPose" else "episode_T.npz")
    task_cfg = json.loads(bytes(d["config_json"]).decode())
    task_cfg["env"]["maxEpisodeLength"] = 25
    n, T = 4096, 40
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    rng = np.random.default_rng(9)
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        E.full_step(a, bias, t, seed=task.seed)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"dones t={t}")
        np.testing.assert_allclose(obs.cpu().numpy(), E.obs, rtol=1e-4, atol=1e-4, err_msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), E.rew, rtol=1e-4, atol=1e-4, err_msg=f"rew t={t}")
        np.testing.assert_array_equal(task.ibuf[0].cpu().numpy(), E.goal_cnt)
    np.testing.assert_allclose(task.stats.cpu().numpy(), E.stats, rtol=1e-4, atol=1e-3)


def test_philox_mode_scene_replay_matches_oracle():
    """Scene replay at 2048 envs (start_index 5, cycling over 7 scenes) vs the oracle."""
    task_cfg = load_yaml(TEST_YAML)
    task_cfg["env"]["scene_replay"] = {"enabled": True, "npz_path": os.path.join(GOLDEN_DIR, "scenes_S.npz"),
                                       "start_index": 5, "cycle": True, "strict_hash": True}
    task_cfg["env"]["maxEpisodeLength"] = 12
    n, T = 2048, 30
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    E.set_scenes(scene_rows(), 5, True)
    rng = np.random.default_rng(4)
    seen = set()
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        E.full_step(a, bias, t, seed=task.seed)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(task.scene_replay_last_scene_idx.numpy(), E.scene_last)
        np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"dones t={t}")
        assert_obs_close(obs.cpu().numpy(), E.obs, 1e-4, msg=f"obs t={t}")
        np.testing.assert_allclose(rew.cpu().numpy(), E.rew, rtol=1e-3, atol=1e-3, err_msg=f"rew t={t}")
        seen.update(np.unique(E.scene_last).tolist())
    task.check_scene_replay()
    assert {5, 6, 0} <= seen          # start_index 5, cycling over 7 scenes


def _run_field(task, ids, obst, tgt, lin=None):
    from omniisaacgymenvs_loop_amd import _capi
    k = len(ids)
    ids_t = torch.tensor(ids, device=DEV, dtype=torch.int32)
    task.reset_ids[:k] = ids_t
    task.ctl.zero_()
    task.ctl[0] = k
    task.fscratch.zero_()
    o = torch.tensor(obst.reshape(k, 32).T, device=DEV)
    task.obst[:, ids_t.long()] = o
    task.field_old_tgt[:, ids_t.long()] = torch.tensor(tgt.T, device=DEV)
    if lin is not None:
        task.set_grid_lin(torch.tensor(lin))
    _capi.call("usv_potential_field", _capi.byref(task.cfg), _capi.byref(task._bufs), _capi.stream_ptr())
    torch.cuda.synchronize()
    return task.field[ids_t.long()].cpu().numpy()


@pytest.mark.parametrize("pack", ["0", "1"])
def test_potential_field_bit_exact_vs_reference(golden, pack, monkeypatch):
    monkeypatch.setenv("USV_FIELD_PACK", pack)
    g = golden("field.npz")
    task = _task(load_yaml(TEST_YAML), 8)
    for name in ("b1", "b4"):
        k = g[f"{name}_obst"].shape[0]
        ids = list(range(k))[::-1]          # slot order must not matter
        f = _run_field(task, ids, g[f"{name}_obst"][::-1].copy(), g[f"{name}_tgt"][::-1].copy(), g["grid_lin"])
        ref = g[f"{name}_field"].reshape(k, -1)[::-1]
        np.testing.assert_array_equal(f, ref)


@pytest.mark.parametrize("pack", ["0", "1"])
def test_potential_field_random_batches_vs_oracle(pack, monkeypatch):
    """Both launch shapes of the field kernel (one env per CU / two per CU, USV_FIELD_PACK)."""
    monkeypatch.setenv("USV_FIELD_PACK", pack)
    task_cfg = load_yaml(TEST_YAML)
    task = _task(task_cfg, 64)
    rng = np.random.default_rng(3)
    for k in (1, 5, 17):
        obst = (rng.uniform(0, 1, (k, 16, 2)) * 24 - 12).astype(np.float32)
        obst[0, :3] = [[0.3, 0.1], [1.2, -0.4], [-0.9, 0.8]]      # crowd the target
        if k > 2:
            obst[1, :] = 999.0                                      # empty map
        tgt = np.zeros((k, 2), np.float32)
        if k > 3:
            tgt[3] = [0.1, 0.2]                                     # occupied target cell
            obst[3, 0] = [0.1, 0.2]
        ids = rng.choice(64, k, replace=False).astype(np.int32)
        f = _run_field(task, ids, obst, tgt)
        ref = O.potential_field(task.cfg, obst, tgt)
        np.testing.assert_array_equal(f, ref)


def test_forces_vs_reference_drag(golden):
    g = golden("forces.npz")
    task_cfg = load_yaml(TEST_YAML)
    n = len(g["yaw"])
    task = _task(task_cfg, n)
    task.cfg.use_drag_scale = 1
    task.state[2] = torch.tensor(g["yaw"], device=DEV)
    task.state[3] = torch.tensor(g["vel"][:, 0], device=DEV)
    task.state[4] = torch.tensor(g["vel"][:, 1], device=DEV)
    task.state[5] = torch.tensor(g["vel"][:, 5], device=DEV)
    task.state[6:8] = 0
    task.params[4] = torch.tensor(g["k_drag"], device=DEV)
    F = task.forces().cpu().numpy()
    np.testing.assert_allclose(F, g["drag"][:, [0, 1, 5]], rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("n", [65536, 131072])
def test_full_size_properties(n):
    """BASELINE sizes (C3 65536/GPU, C5 131072/GPU): determinism, finiteness, resets, field range."""
    task_cfg = load_yaml(TEST_YAML)
    outs = []
    for rep in range(2):
        task = _task(task_cfg, n)
        g = torch.Generator(device=DEV).manual_seed(1)
        acc_done = 0
        for t in range(12):
            a = torch.rand((n, 2), device=DEV, generator=g) * 2 - 1
            obs, rew, dones = task.env_step(a)
            acc_done += int(dones.sum().item())
        torch.cuda.synchronize()
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
        assert obs.abs().max().item() <= 12.0
        assert acc_done > 0
        f = task.field
        assert float(f.min()) >= 0.0 and float(f.max()) <= 1.5 + 1e-5
        outs.append((obs.clone(), rew.clone(), task.state.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b), "same seed must give bitwise-identical results"
