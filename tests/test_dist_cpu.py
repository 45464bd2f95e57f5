"""World-size-2 gloo tests of the data-parallel PPO update (CPU, no GPU needed).

The multi-GPU path shards envs across ranks (independent per-rank env blocks,
seeds offset by rank) and all-reduces the flat gradient + KL once per minibatch
(dist_util.allreduce_grad, the RCCL call of A2CAgent on the GPU).  These tests
run exactly that helper on gloo with the numpy PPO oracle as the per-rank
gradient: the averaged gradient of two half-minibatches must equal the
single-process gradient of the whole minibatch (rl_games multi-GPU semantics,
a2c_common.py:308-323), the KL must average the same way, and the initial
broadcast must make every rank start from rank 0's weights (:1354).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ppo_oracle as PO

B = 512          # rows per rank


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rows, seed=3):
    rng = np.random.default_rng(seed)
    f = np.float32
    mu = rng.normal(0, 0.3, (rows, 2)).astype(f)
    return {
        "xn": rng.normal(0, 1, (rows, 33)).astype(f).clip(-5, 5),
        "act": (mu + rng.normal(0, 1, (rows, 2))).astype(f),
        "old_nlp": rng.uniform(1.5, 3.5, rows).astype(f),
        "old_val": rng.normal(0, 1, rows).astype(f),
        "ret": rng.normal(0, 1, rows).astype(f),
        "adv": rng.normal(0, 1, rows).astype(f),
        "old_mu": mu,
        "old_sigma": np.ones((rows, 2), f),
    }


def _params(seed):
    return PO.unflatten(np.random.default_rng(seed).uniform(-0.08, 0.08, PO.NPARAM).astype(np.float32))


def _grad(P, d, sl, rows):
    cfg = PO.PPOConfig(minibatch=rows)
    g, losses, kl, _, _ = PO.minibatch_grad(P, *(d[k][sl] for k in ("xn", "act", "old_nlp", "old_val", "ret", "adv",
                                                                     "old_mu", "old_sigma")), cfg)
    return g, kl


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from omniisaacgymenvs_loop_amd.rl_games import dist_util
        flat = torch.from_numpy(PO.flatten(_params(100 + rank)))      # different on every rank
        dist_util.broadcast_params(flat, 0)
        P = PO.unflatten(flat.numpy().copy())
        d = _data(world * B)
        g, kl = _grad(P, d, slice(rank * B, (rank + 1) * B), B)
        buf = torch.from_numpy(np.concatenate([g, [kl]]).astype(np.float32))
        scale = dist_util.allreduce_grad(buf)
        t = dist_util.max_over_ranks(float(rank) + 0.5, "cpu")
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), flat=flat.numpy(), g=buf.numpy() * np.float32(scale),
                 scale=scale, tmax=t)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_ranks(tmp_path_factory):
    out = tmp_path_factory.mktemp("dist")
    mp.spawn(_worker, args=(2, _port(), str(out)), nprocs=2, join=True)
    return [np.load(out / f"r{r}.npz") for r in range(2)]


def test_initial_broadcast(two_ranks):
    r0, r1 = two_ranks
    np.testing.assert_array_equal(r0["flat"], r1["flat"])
    np.testing.assert_array_equal(r0["flat"], PO.flatten(_params(100)))


def test_allreduced_gradient_equals_full_minibatch(two_ranks):
    r0, r1 = two_ranks
    assert float(r0["scale"]) == 0.5
    np.testing.assert_array_equal(r0["g"], r1["g"])                  # identical on every rank
    g_full, kl_full = _grad(_params(100), _data(2 * B), slice(0, 2 * B), 2 * B)
    np.testing.assert_allclose(r0["g"][:PO.NPARAM], g_full, rtol=2e-4, atol=2e-7)
    np.testing.assert_allclose(r0["g"][PO.NPARAM], kl_full, rtol=1e-5, atol=1e-7)


def test_max_over_ranks(two_ranks):
    assert all(float(r["tmax"]) == 1.5 for r in two_ranks)
