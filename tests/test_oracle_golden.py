"""The CPU oracle (oracle/usv_oracle.c) against the reference's own outputs.

Golden vectors: tests/golden/*.npz, produced by tests/golden/make_golden.py,
which imports the reference Python (loop-Z/omniisaacgymenvs_loop) in the build
container and records every input, every torch.rand draw and every output.
"""
import json

import numpy as np
import pytest

from oracle import oracle as O
from omniisaacgymenvs_loop_amd.tasks.usv_config import (build_hydro_cfg, build_usv_cfg, load_yaml, parse_penalty_fn,
                                                         stat_names, thruster_tables)
from omniisaacgymenvs_loop_amd._abi import PEN
import os

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
TEST_YAML = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "omniisaacgymenvs_loop_amd",
                         "cfg", "task", "USV", "IROS2024", "USV_Virtual_CaptureXY_SysID-TEST.yaml")


def _cfg_from(d):
    return json.loads(bytes(d["config_json"]).decode())


def test_philox_known_answers():
    # Random123 philox4x32-10 KAT vectors (kat_vectors, Salmon et al. SC'11)
    assert O.philox([0, 0, 0, 0], [0, 0]).tolist() == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2).tolist() == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert O.philox([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0]).tolist() == \
        [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_lut_bit_exact(golden):
    g = golden("lut.npz")
    for name in ("test", "sym"):
        lut = O.make_lut(g[f"{name}_table_l"], g[f"{name}_table_r"])
        np.testing.assert_array_equal(lut[0], g[f"{name}_lut_l"])
        np.testing.assert_array_equal(lut[1], g[f"{name}_lut_r"])


def test_lut_index_and_lag(golden):
    """get_cmd_interpolated index mapping + first-order lag (ThrusterDynamics.py:129-234)."""
    g = golden("lut.npz")
    cfg = build_usv_cfg(load_yaml(TEST_YAML))
    for name in ("test", "sym"):
        lut = O.make_lut(g[f"{name}_table_l"], g[f"{name}_table_r"])
        cmds = g[f"{name}_cmds"]
        idx = np.clip(np.rint(((cmds + np.float32(1)) / np.float32(2)) * np.float32(999)), 0, 999).astype(int)
        tgt = np.stack([lut[0][idx[:, 0]], lut[1][idx[:, 1]]], 1)
        np.testing.assert_array_equal(tgt, g[f"{name}_targets"])
        a = np.float32(cfg.thr_alpha)
        f = np.zeros_like(tgt)
        for k in range(g[f"{name}_lag"].shape[0]):
            f = f * a + (np.float32(1) - a) * tgt
            np.testing.assert_array_equal(f, g[f"{name}_lag"][k])


def test_planar_drag_matches_reference(golden):
    """Surge/sway/yaw drag of HydrodynamicsObject.ComputeHydrodynamicsEffects."""
    g = golden("forces.npz")
    cfg = build_usv_cfg(load_yaml(TEST_YAML))
    cfg.use_drag_scale = 1
    n = len(g["yaw"])
    E = O.OracleEnv(cfg, n, np.zeros((2, 1000), np.float32))
    E.yaw[:] = g["yaw"]
    E.vx[:], E.vy[:], E.wz[:] = g["vel"][:, 0], g["vel"][:, 1], g["vel"][:, 5]
    E.k_drag[:] = g["k_drag"]
    E.fl[:] = 0
    E.fr[:] = 0
    ref = g["drag"][:, [0, 1, 5]]
    # the reference's own quaternions through quaternion_to_matrix and torch.bmm's order: bit for bit
    np.testing.assert_array_equal(E.forces(quat=g["quat"]), ref)
    # the stand-in's quaternion of the same yaws (usv_sincos of yaw / 2 instead of the reference's MKL cos / sin):
    # the drag at 1e-5 of its scale
    np.testing.assert_allclose(E.forces(), ref, rtol=1e-5, atol=1e-5 * float(np.abs(ref).max()))


def test_hydrostatics_matches_reference(golden):
    """Buoyancy + metacentric torques (Hydrostatics.py:63-133) with update_state's submerged volume and
    get_euler_angles (USV_Virtual.py:791-798, 815-835), at random and at level attitudes."""
    g = golden("hydrostatics.npz")
    task_cfg = load_yaml(TEST_YAML)
    assert g["gravity"] == np.float32(task_cfg["sim"]["gravity"][2])
    vol, eul, wr = O.hydrostatics(build_hydro_cfg(task_cfg), g["quat"], g["z"])
    np.testing.assert_allclose(vol, g["volume"], rtol=1e-6, atol=0)
    np.testing.assert_allclose(eul, g["euler"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(wr, g["wrench"], rtol=1e-5, atol=1e-5 * np.abs(g["wrench"]).max())
    # level attitudes (the planar model): surge, sway and yaw contributions are exactly zero
    level = slice(len(g["z"]) // 2, None)
    assert np.all(g["wrench"][level][:, [0, 1, 5]] == 0) and np.all(wr[level][:, [0, 1, 5]] == 0)


def test_potential_field_bit_exact(golden):
    g = golden("field.npz")
    cfg = build_usv_cfg(load_yaml(TEST_YAML))
    for name in ("b1", "b4"):
        field, cost = O.potential_field(cfg, g[f"{name}_obst"], g[f"{name}_tgt"], want_cost=True, lin=g["grid_lin"])
        rc = g[f"{name}_cost"].reshape(cost.shape)
        np.testing.assert_array_equal(cost, rc)
        np.testing.assert_array_equal(field, g[f"{name}_field"].reshape(field.shape))


def test_grid_lin_formula_close(golden):
    """Kernels default to the symmetric linspace formula (the CUDA kernel's);
    the CPU-vectorised torch.linspace that made the fixtures differs by <=1 ulp."""
    g = golden("field.npz")
    np.testing.assert_allclose(O.grid_lin(30.0), g["grid_lin"], rtol=0, atol=2e-6)


def _replay(d, post_only, stale_root=None, inj_trig=1):
    """The fixture's episode through the oracle on the reference's recorded draws.  inj_trig = 1 also takes the
    reference's recorded torch.cos / torch.sin values of the reset path (RU_TRIG: spawn angle and quaternion,
    scene yaw, constant disturbance direction) -- MKL VML HA on the CPU, not restatable bit for bit -- so the
    state follows the reference's exactly; 0 uses the build's own usv_sincos_cr."""
    cfg_d = _cfg_from(d)
    if stale_root is not None:
        cfg_d["env"]["stale_root_after_reset"] = stale_root
    cfg = build_usv_cfg(cfg_d)
    cfg.inj_trig = inj_trig
    lut = O.make_lut(*thruster_tables(cfg_d))
    T, n = d["obs"].shape[:2]
    E = O.OracleEnv(cfg, n, lut)
    E.set_grid_lin(d["grid_lin"])
    if "scene_last" in d:   # scene replay: the fixture's scene file, start_index / cycle of its config
        sr = cfg_d["env"]["scene_replay"]
        E.set_scenes(scene_rows(), int(sr["start_index"]), bool(sr["cycle"]))
    E.tgt_x[:] = d["init_tgt"][:, 0]
    E.tgt_y[:] = d["init_tgt"][:, 1]
    ru = 0
    out = []
    for t in range(T):
        ids = E.compact()
        if stale_root is not None:   # a control run off the fixtures' semantics: follow their reset pattern
            E.reset_buf[:] = d["reset_mask"][t]
            ids = E.compact()
        np.testing.assert_array_equal(ids, np.nonzero(d["reset_mask"][t])[0])
        if len(ids):
            E.reset(ids, d["reset_U"][ru:ru + len(ids)])
            ru += len(ids)
        if len(ids) and stale_root is None:
            ex = d["extras"][t]
            # episode means of per-step sums
            rtol, atol = (1e-5, 1e-6) if post_only or inj_trig else (1e-4, 1e-5)
            if "extras_names" in d:   # task-specific episode_sums keys (USV_Virtual.py:584-601)
                layout = stat_names(cfg)
                assert [k for k, _ in layout] == [str(k) for k in d["extras_names"]]
                ex = np.array([ex[i] for i in range(len(layout))], np.float32)
                np.testing.assert_allclose(E.extras[[sl for _, sl in layout]], ex, rtol=rtol, atol=atol)
            else:
                np.testing.assert_allclose(E.extras, ex, rtol=rtol, atol=atol)
        E.step_pre(d["actions"][t], float(d["bias"][t]), d["u_step"][t])
        E.step_physics()
        if post_only:
            for k in ("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr"):
                getattr(E, k)[:] = d[k][t]
        E.step_post(d["u_step"][t])
        if "scene_last" in d:
            np.testing.assert_array_equal(E.scene_last, d["scene_last"][t])
        if "dist" in d:
            # ForceDisturbance / TorqueDisturbance parameters drawn at reset (USV_disturbances.py:327-508)
            np.testing.assert_allclose(E.dist, d["dist"][t], rtol=1e-6, atol=1e-6, err_msg=f"dist step {t}")
        out.append((E.obs.copy(), E.rew.copy(), E.reset_buf.copy(), E.mass.copy(), E.k_drag.copy(), E.thr_l.copy(),
                    E.thr_r.copy(), E.k_iz.copy(), E.obst.copy(), E.progress.copy(), E.goal_cnt.copy(),
                    np.stack([getattr(E, k).copy() for k in STATE_KEYS])))
    return out


STATE_KEYS = ("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr")


def scene_rows():
    from omniisaacgymenvs_loop_amd.tasks.scene_replay import load_scene_arrays, pack_scenes
    return pack_scenes(load_scene_arrays(os.path.join(GOLDEN_DIR, "scenes_S.npz")))


def test_scene_file_format_and_hash(tmp_path):
    """build_usv_scenes.py format: required keys, NaN padding -> limbo past obstacles_count, sha1 sidecar."""
    from omniisaacgymenvs_loop_amd.tasks import scene_replay as SR
    rows = scene_rows()
    d = np.load(os.path.join(GOLDEN_DIR, "scenes_S.npz"), allow_pickle=False)
    assert rows.shape == (7, 40)
    for i, cnt in enumerate(d["obstacles_count"]):
        ob = rows[i, :32].reshape(16, 2)
        np.testing.assert_array_equal(ob[:cnt], d["obstacles_xy"][i, :cnt])
        assert (ob[cnt:] == 999.0).all()
    np.testing.assert_array_equal(rows[:, 37:39], d["goal_pos"])
    bad = tmp_path / "s.npz"
    SR.write_scenes_npz(str(bad), d["obstacles_xy"], d["obstacles_count"], d["start_pos"], d["start_yaw"],
                        d["start_vel"], d["goal_pos"])
    SR.load_scene_arrays(str(bad))
    (tmp_path / "s.npz.sha1").write_text("0" * 40)
    with pytest.raises(ValueError):
        SR.load_scene_arrays(str(bad))
    SR.load_scene_arrays(str(bad), strict_hash=False)
    with pytest.raises(FileNotFoundError):
        SR.load_scene_arrays(str(tmp_path / "missing.npz"))


def test_episode_c_exercises_disturbances(golden):
    """The disturbance fixture has every generator on and draws non-trivial parameters."""
    d = golden("episode_C.npz")
    cfg = build_usv_cfg(_cfg_from(d))
    assert cfg.fdist_on and cfg.fconst_on and cfg.fsin_on and cfg.tdist_on and cfg.tconst_on and cfg.tsin_on
    assert cfg.current_on and abs(cfg.flow_vel[0] - 0.3) < 1e-7
    assert np.all(np.abs(d["dist"][-1]).sum(0) > 0)
    assert (d["dist"][-1][7] < 0).any() and (d["dist"][-1][7] > 0).any()   # torque sign flip


@pytest.mark.parametrize("variant", ["A", "B", "C", "D", "E", "P", "Q", "T", "S"])
def test_episode_post_physics(golden, variant):
    """obs / reward / done / DR / spawns given the reference's post-integration state."""
    d = golden(f"episode_{variant}.npz")
    w = d["obs"].shape[-1]
    for t, (obs, rew, rb, mass, kd, tl, tr, kiz, obst, prog, gc, _) in enumerate(_replay(d, post_only=True)):
        # rows are 25 + priv_dim wide in the reference; a priv_dim-4 slab row carries 4 zero pad columns
        assert (obs[:, w:] == 0).all()
        np.testing.assert_allclose(obs[:, :w], d["obs"][t], rtol=2e-6, atol=2e-6, err_msg=f"obs step {t}")
        np.testing.assert_allclose(rew, d["rew"][t], rtol=5e-6, atol=5e-6, err_msg=f"rew step {t}")
        np.testing.assert_array_equal(rb, d["reset"][t])
        np.testing.assert_array_equal(prog, d["progress"][t])
        np.testing.assert_array_equal(gc, d["goal_cnt"][t])
        np.testing.assert_allclose(mass, d["mass"][t], rtol=1e-6)
        np.testing.assert_allclose(kd, d["k_drag"][t], rtol=1e-6)
        np.testing.assert_allclose(tl, d["thr_l"][t], rtol=1e-6)
        np.testing.assert_allclose(tr, d["thr_r"][t], rtol=1e-6)
        np.testing.assert_allclose(kiz, d["k_iz"][t], rtol=1e-6)
        np.testing.assert_array_equal(obst.transpose(2, 0, 1), d["obst"][t])


# Episode C's sinusoidal force / torque disturbances call torch.sin (MKL VML HA) at every substep
# (USV_disturbances.py:401-405, 523): the build's usv_sin_cr rounds the same phases to the neighbouring float in a
# few per cent of them, so C's state is within this absolute bound instead of bit-exact (measured 1.5e-8 m/s)
STATE_ATOL = {"C": 1e-7}


@pytest.mark.parametrize("variant", ["A", "B", "C", "D", "E", "P", "Q", "T", "S"])
def test_episode_end_to_end(golden, variant):
    """Full replay incl. this build's integrator (the stand-in for PhysX the fixtures were recorded with), with the
    reference's recorded reset sin / cos: the integrated state is the reference's bit for bit (C: STATE_ATOL), the
    observations, rewards and episode extras within rtol = atol = 1e-5."""
    d = golden(f"episode_{variant}.npz")
    w = d["obs"].shape[-1]
    atol = STATE_ATOL.get(variant, 0.0)
    for t, (obs, rew, rb, *_rest, st) in enumerate(_replay(d, post_only=False)):
        np.testing.assert_allclose(st, np.stack([d[k][t] for k in STATE_KEYS]), rtol=0, atol=atol,
                                   err_msg=f"state step {t}")
        np.testing.assert_allclose(obs[:, :w], d["obs"][t], rtol=1e-5, atol=1e-5, err_msg=f"obs step {t}")
        np.testing.assert_allclose(rew, d["rew"][t], rtol=1e-5, atol=1e-5, err_msg=f"rew step {t}")
        np.testing.assert_array_equal(rb, d["reset"][t])


def _own_trig(d):
    """The build's usv_sincos_cr at the recorded reset sites (the same float32 argument expressions as the reset
    kernel) -> [K][6] like the RU_TRIG columns, NaN where the fixture recorded nothing."""
    U = d["reset_U"]
    rec = U[:, O.RU_TRIG:O.RU_TRIG + 6]
    pi = np.float32(np.pi)
    th = (U[:, 21] * np.float32(2.0)) * pi
    half = (U[:, 22] * pi) * np.float32(0.5)
    tt = (U[:, 705] * pi) * np.float32(2.0)
    out = np.full_like(rec, np.nan)
    s, c = O.sincos_cr(th)
    out[:, 0], out[:, 1] = c, s
    s, c = O.sincos_cr(half)
    out[:, 2], out[:, 3] = c, s
    s, c = O.sincos_cr(tt)
    out[:, 4], out[:, 5] = c, s
    return np.where(np.isnan(rec), np.nan, out), rec


@pytest.mark.parametrize("variant", ["A", "B", "C", "D", "E", "P", "Q", "T"])
def test_episode_end_to_end_own_trig(golden, variant):
    """The same replay with the build's own reset sin / cos (usv_sincos_cr, what training runs): each value
    within 1 ulp of the reference's MKL value and most of them equal; the state then within 1e-5 of the reference
    (a spawn moved by an ulp stays an ulp-scale offset over the episode), the observations within 1e-5."""
    d = golden(f"episode_{variant}.npz")
    own, rec = _own_trig(d)
    ok = ~np.isnan(rec)
    assert ok.any()
    ulps = np.abs(own[ok] - rec[ok]) / np.spacing(np.abs(rec[ok]))
    assert ulps.max() <= 1.0 and (ulps == 0).mean() >= 0.8, (ulps.max(), (ulps == 0).mean())
    w = d["obs"].shape[-1]
    for t, (obs, rew, rb, *_rest, st) in enumerate(_replay(d, post_only=False, inj_trig=0)):
        np.testing.assert_allclose(st, np.stack([d[k][t] for k in STATE_KEYS]), rtol=1e-5, atol=1e-5,
                                   err_msg=f"state step {t}")
        np.testing.assert_allclose(obs[:, :w], d["obs"][t], rtol=1e-5, atol=1e-5, err_msg=f"obs step {t}")
        np.testing.assert_array_equal(rb, d["reset"][t])


@pytest.mark.parametrize("variant", ["A", "C"])
def test_episode_pins_the_cached_root_state(golden, variant):
    """SURVEY App. C.1 is in the fixtures: the reference's first substep after a reset takes its drag (and, in C,
    its disturbances and water current) from the cached pre-reset root state (USV_Virtual.py:1103-1117).  The
    same replay with that substep on the new state (stale_root_after_reset: false) leaves the fixtures'
    observations by far more than the end-to-end tolerance."""
    d = golden(f"episode_{variant}.npz")
    w = d["obs"].shape[-1]
    err = max(float(np.abs(o[0][:, :w] - d["obs"][t]).max()) for t, o in enumerate(_replay(d, False, False)))
    assert err > 1e-2, err


@pytest.mark.parametrize("lo,hi", [(-np.pi, np.pi), (0.0, 2 * np.pi), (-5000.0, 5000.0)])
def test_integrator_sincos_accuracy(lo, hi):
    """The integrator's sin / cos (usv_oracle.c:usv_sincos == csrc/usv_device.h:usv_sincos) against float64 libm:
    within 1e-7 absolute (1.5 ulp of values away from 0) on the yaw range, the spawn-angle range and the
    disturbance phases' range; numpy's float32 sin is within 7e-8 on the same points."""
    x = np.linspace(lo, hi, 1_000_001).astype(np.float32)
    s, c = O.sincos(x)
    xd = x.astype(np.float64)
    assert np.abs(s - np.sin(xd)).max() < 1e-7
    assert np.abs(c - np.cos(xd)).max() < 1e-7
    big = np.abs(np.sin(xd)) > 0.5
    assert (np.abs(s - np.sin(xd))[big] / np.spacing(np.abs(s[big]))).max() <= 1.6
    s0, c0 = O.sincos(np.zeros(1, np.float32))
    assert s0[0] == 0.0 and c0[0] == 1.0


def test_obs_reward_math_accuracy():
    """The observation / reward functions (usv_oracle.c:usv_exp, usv_tanh, usv_atan2 == csrc/usv_device.h) against
    float64 libm: exp within 1 ulp over its whole normal range, tanh within 1.5 ulp, atan2 within 2.6 ulp (3e-7
    absolute) on random and unit-circle arguments; IEEE atan2's signed zeros and pi at the origin."""
    def ulps(got, ref):
        sp = np.spacing(np.abs(ref.astype(np.float32))).astype(np.float64)
        return np.abs(got.astype(np.float64) - ref) / np.maximum(sp, 1e-45)
    x = np.linspace(-87.0, 88.0, 1_000_001).astype(np.float32)
    e, _, _ = O.math3(x, np.ones_like(x))
    ref = np.exp(x.astype(np.float64))
    assert ulps(e[ref > 1.2e-38], ref[ref > 1.2e-38]).max() <= 1.0
    x = np.linspace(-10.0, 10.0, 1_000_001).astype(np.float32)
    _, t, _ = O.math3(x, np.ones_like(x))
    ref = np.tanh(x.astype(np.float64))
    assert ulps(t[ref != 0], ref[ref != 0]).max() <= 1.5
    rng = np.random.default_rng(0)
    xx, yy = rng.normal(0, 10, 1_000_000).astype(np.float32), rng.normal(0, 10, 1_000_000).astype(np.float32)
    th = np.linspace(-np.pi, np.pi, 1_000_001)
    xx = np.concatenate([xx, np.cos(th).astype(np.float32)])
    yy = np.concatenate([yy, np.sin(th).astype(np.float32)])
    _, _, a = O.math3(xx, yy)
    ref = np.arctan2(yy.astype(np.float64), xx.astype(np.float64))
    assert ulps(a, ref).max() <= 2.6 and np.abs(a - ref).max() < 3e-7
    ys = np.array([0.0, -0.0, 0.0, -0.0, 1.0, -1.0], np.float32)
    xs = np.array([0.0, 0.0, -0.0, -0.0, 0.0, 0.0], np.float32)
    np.testing.assert_array_equal(np.signbit(O.math3(xs, ys)[2]), np.signbit(np.arctan2(ys, xs)))
    np.testing.assert_allclose(O.math3(xs, ys)[2], np.arctan2(ys, xs), rtol=1e-7)


def test_penalty_parser():
    c = {"c1": 0.3, "c2": 0.1}
    assert parse_penalty_fn("lambda x,step: -torch.clamp(torch.abs(x) - 0.4, min=0.0) * 0.02", c) == \
        (PEN["PEN_DEADZONE"], 0.02, 0.4, 0.0)
    assert parse_penalty_fn("lambda x,step : -torch.sum(x, dim=-1) * 0.005", c) == (PEN["PEN_SUM"], 0.005, 0.0, 0.0)
    assert parse_penalty_fn("lambda x,step : -torch.abs(x)*c1 + c2", c) == (PEN["PEN_DEADZONE"], 0.3, 0.0, 0.1)
    assert parse_penalty_fn("lambda x,step: -torch.norm(x, dim=-1)*0.01", c) == (PEN["PEN_NORM"], 0.01, 0.0, 0.0)
    assert parse_penalty_fn("lambda x,step: (torch.exp(-0.033 * torch.abs(x)) - 1.0) * 0.2", c)[0] == \
        PEN["PEN_EXPABS"]
    with pytest.raises(ValueError):
        parse_penalty_fn("lambda x,step: torch.sin(x)", c)


def test_packaged_yaml_matches_fixture_config(golden):
    """The packaged TEST yaml resolves to the same kernel constants as the
    reference yaml recorded in the fixture."""
    ref = build_usv_cfg(_cfg_from(golden("episode_A.npz")))
    mine = build_usv_cfg(load_yaml(TEST_YAML))
    for name, _ in ref._fields_:
        a, b = getattr(ref, name), getattr(mine, name)
        if hasattr(a, "__len__"):
            assert list(a) == list(b), name
        else:
            assert a == b, name

