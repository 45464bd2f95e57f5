"""The oracle's device-sample inputs (OracleEnv.full_step(pot_in=, pos_in=)) that the GPU reward checks use in
place of a potential-sample allowance, and the shaping-branch flip counter (tests/test_env_gpu.py): fed its own
samples the oracle reproduces itself bit for bit, fed other samples only the potential-dependent reward terms
move, and the position probe samples the oracle's field where it is told to."""
import numpy as np
import pytest

pytest.importorskip("torch")

from oracle import oracle as O
from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml, thruster_tables
from tests.test_oracle_golden import TEST_YAML


def _env(n):
    task_cfg = load_yaml(TEST_YAML)
    cfg = build_usv_cfg(task_cfg)
    return cfg, O.OracleEnv(cfg, n, O.make_lut(*thruster_tables(task_cfg)))


def test_oracle_fed_its_own_samples_is_itself():
    n, T = 48, 6
    _, A = _env(n)
    _, B = _env(n)
    _, C = _env(n)
    rng = np.random.default_rng(2)
    diff_seen = False
    for t in range(T):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        A.full_step(a, -0.6, t, seed=5)
        own = A.dbg[:, 4].copy()
        assert np.array_equal(own, A.dbg[:, 14])             # no override: the sample used is the own one
        pos = np.stack([A.px, A.py]).copy()
        B.full_step(a, -0.6, t, seed=5, pot_in=own, pos_in=pos)
        for k in ("rew", "px", "py", "yaw", "prev_pot", "goal_cnt", "reset_buf"):
            np.testing.assert_array_equal(getattr(B, k), getattr(A, k), err_msg=f"{k} t={t}")
        np.testing.assert_array_equal(B.obs, A.obs)
        np.testing.assert_array_equal(B.stats, A.stats)
        np.testing.assert_array_equal(B.dbg[:, 15], own)     # sampled at the given (= own) position
        # other samples: only the reward (and its potential-dependent statistics) move
        C.full_step(a, -0.6, t, seed=5, pot_in=np.clip(own + 0.05, 0, 1.5).astype(np.float32), pos_in=pos)
        np.testing.assert_array_equal(C.obs, A.obs)
        np.testing.assert_array_equal(C.reset_buf, A.reset_buf)
        np.testing.assert_array_equal(C.dbg[:, 14], own)
        diff_seen |= bool(np.any(C.rew != A.rew))
        C.rew[:] = A.rew   # keep the three in step (rew is an output only)
        C.stats[:] = A.stats
        C.prev_pot[:] = A.prev_pot
    assert diff_seen
    # the override is cleared after the step
    assert A.c.pot_in is None and B.c.pot_in is None


def test_shaping_branch_flip_counter():
    from tests.test_env_gpu import count_flips, shaping_branches
    br = shaping_branches(np.array([0.005, 0.02, 1.2, -0.2, -0.02], np.float32))
    assert br[0].tolist() == [True, False, False, False, False]        # dead zone
    assert br[1].tolist() == [False, False, True, False, False]        # ppos >= 0.5 (gated)
    assert br[2].tolist() == [False, False, False, True, False]        # worsening
    dbg = np.zeros((3, O.NDBG), np.float32)
    # env 0: device praw inside the dead zone, own praw just outside; env 1: same branch; env 2: a reset env
    dbg[:, 11] = [0.0099, 0.3, 0.0]
    dbg[:, 14] = [0.5, 0.5, 0.7]
    dbg[:, 16] = [0, 0, 1]
    prev_own = np.array([0.5 + 0.000102, 0.5 + 0.003, 0.1], np.float32)
    nflip, own = count_flips(dbg, prev_own)
    assert nflip == 1 and np.array_equal(own, dbg[:, 14])
