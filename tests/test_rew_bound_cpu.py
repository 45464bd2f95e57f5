"""The reward-check allowance for the shaping term's discontinuities (tests/test_env_gpu.py
shaping_flip_allowance): granted exactly where the oracle's own value lies within the potential-sample error
of a discontinuity, sized by that discontinuity's jump, and nowhere else."""
import numpy as np
import pytest

pytest.importorskip("torch")


def _dbg(praw, shaping, ppos):
    d = np.zeros((len(praw), 16), np.float32)
    d[:, 11], d[:, 8], d[:, 12] = praw, shaping, ppos
    return d


def test_allowance_only_near_a_discontinuity():
    from tests.test_env_gpu import shaping_flip_allowance
    dpot = np.array([1e-7, 1e-7, 1e-7, 1e-7, 0.0, 1e-7])
    # praw near the 0.01 dead zone; far from it; ppos near the 0.5 gate; shaping near -0.05; exact (no error); far
    praw = np.array([0.01 + 5e-6, 0.2, 0.3, -0.08, 0.01 + 5e-6, -0.3])
    shaping = np.array([0.02, 0.4, 0.6, -0.05 + 1e-6, 0.02, -0.6])
    ppos = np.array([0.01, 0.2, 0.5 - 1e-6, 0.0, 0.01, 0.0])
    allow, near = shaping_flip_allowance(_dbg(praw, shaping, ppos), dpot, np.zeros_like(dpot))
    assert near.tolist() == [True, False, True, True, False, False]
    d = 100.0 * 1e-7 * 1.001 + 2e-6
    assert allow[0] == pytest.approx(4.0 * np.tanh((0.01 + d) / 2.0))   # 2 x the dead zone's pa1 jump
    assert allow[2] == pytest.approx(2.0 * (0.5 + d))                   # the pass-through gate
    assert allow[3] == pytest.approx(10.0)                              # the turn hazard
    assert allow[1] == allow[4] == allow[5] == 0.0
