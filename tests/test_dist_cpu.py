"""World-size-2 (and 4) gloo tests of the data-parallel PPO update (CPU, no GPU needed).

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


def test_four_ranks_allreduced_gradient_equals_full_minibatch(tmp_path):
    """The same at world size 4 (BASELINE configs[3] splits over 4 GPUs): rank 0's weights everywhere, scale 1/4,
    identical averaged gradients on every rank equal to the 4 x 512-row minibatch's, the timing max over ranks."""
    mp.spawn(_worker, args=(4, _port(), str(tmp_path)), nprocs=4, join=True)
    rs = [np.load(tmp_path / f"r{r}.npz") for r in range(4)]
    for r in rs:
        np.testing.assert_array_equal(r["flat"], PO.flatten(_params(100)))
        np.testing.assert_array_equal(r["g"], rs[0]["g"])
        assert float(r["scale"]) == 0.25 and float(r["tmax"]) == 3.5
    g_full, kl_full = _grad(_params(100), _data(4 * B), slice(0, 4 * B), 4 * B)
    np.testing.assert_allclose(rs[0]["g"][:PO.NPARAM], g_full, rtol=2e-4, atol=2e-7)
    np.testing.assert_allclose(rs[0]["g"][PO.NPARAM], kl_full, rtol=1e-5, atol=1e-7)


class _FakeDpLib:
    """Stands in for libusv_hip.so's ppo_dp_* calls so the set-up protocol of PeerExchange runs on CPU ranks
    with chosen failures (no device memory is touched)."""

    def __init__(self, rank, fail_alloc, fail_open):
        self.rank, self.fail_alloc, self.fail_open = rank, fail_alloc, fail_open
        self.log = []

    def ppo_dp_alloc(self, pp, handle):
        if self.rank in self.fail_alloc:
            return 7
        pp._obj.value = 0x1000 * (self.rank + 1)
        handle.raw = bytes([self.rank + 1]) * 64
        self.log.append("alloc")
        return 0

    def ppo_dp_open(self, handle, pp):
        if self.rank in self.fail_open:
            return 9
        pp._obj.value = 0x100000 + handle.raw[0]
        self.log.append("open")
        return 0

    def ppo_dp_close(self, p):
        self.log.append("close")
        return 0

    def ppo_dp_free(self, p):
        self.log.append("free")
        return 0


def _pe_worker(rank, world, port, out_dir, fail_alloc, fail_open, shared=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from omniisaacgymenvs_loop_amd import _capi
        from omniisaacgymenvs_loop_amd.rl_games import dist_util
        fake = _FakeDpLib(rank, fail_alloc, fail_open)
        _capi.lib = lambda: fake
        # one device per rank (what torchrun gives on a node), or every rank on one device
        dist_util.device_identity = (lambda d: "host/0000:75:00") if shared else (lambda d: f"host/0000:{rank:02x}:00")
        msg = ""
        try:
            dist_util.PeerExchange(rank, world, "cpu")
        except RuntimeError as e:
            msg = str(e)
        dist.barrier()      # both ranks got here: no rank hangs in a mismatched collective
        np.savez(os.path.join(out_dir, f"pe{rank}.npz"), msg=msg, log=np.array(fake.log))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_alloc,fail_open", [(2, (1,), ()), (2, (), (1,)), (2, (0, 1), ()),
                                                          (4, (), (2,)), (4, (3,), ())])
def test_peer_exchange_setup_failure_is_agreed_and_frees_after_the_barrier(tmp_path, world, fail_alloc, fail_open):
    """A failed allocation or mapping on ONE rank (of two or four): every rank still runs the same collectives
    (handle exchange, agreement), every rank raises, and each frees its own buffer only after unmapping the
    peers' (ADVICE r3)."""
    mp.spawn(_pe_worker, args=(world, _port(), str(tmp_path), fail_alloc, fail_open), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"pe{r}.npz")
        assert "PeerExchange" in str(z["msg"]), (r, z["msg"])
        log = list(z["log"])
        if r not in fail_alloc:
            assert log[0] == "alloc" and log[-1] == "free" and log.count("free") == 1
            if "open" in log:
                assert log.index("close") < log.index("free")
        else:
            assert "free" not in log


@pytest.mark.parametrize("world", [3, 4])
def test_peer_exchange_refuses_more_than_two_ranks_per_device(tmp_path, world, monkeypatch):
    """More ranks on one device than the exchange can make progress with (PEER_MAX_RANKS_PER_DEVICE: the waiting
    ranks' spinning reduction workgroups would starve the last rank's gradient kernel of LDS) is refused on every
    rank with a message naming the device and ranks, before anything is allocated (A2CAgent then falls back to
    collectives); USV_DP_SHARED_DEVICE_SETUP=1 lets the set-up and self-test rehearsal through."""
    from omniisaacgymenvs_loop_amd.rl_games.dist_util import shared_device_refusal
    assert shared_device_refusal(["a", "a"]) is None and shared_device_refusal(["a", "b", "c", "d"]) is None
    assert "ranks [0, 2, 3] share device a" in shared_device_refusal(["a", "b", "a", "a"])
    monkeypatch.delenv("USV_DP_SHARED_DEVICE_SETUP", raising=False)
    mp.spawn(_pe_worker, args=(world, _port(), str(tmp_path), (), (), True), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"pe{r}.npz")
        assert "share device host/0000:75:00" in str(z["msg"]) and "USV_DP_EXCHANGE=collective" in str(z["msg"])
        assert list(z["log"]) == []      # nothing allocated or mapped
    monkeypatch.setenv("USV_DP_SHARED_DEVICE_SETUP", "1")
    mp.spawn(_pe_worker, args=(world, _port(), str(tmp_path), (), (), True), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"pe{r}.npz")
        assert "share device" not in str(z["msg"]) and list(z["log"])[:1] == ["alloc"]


def test_update_capturable_gates_on_the_path_that_runs(monkeypatch):
    """Several ranks: the update graph is captured by default with the peer exchange (kernels only) and, on the
    nccl backend, with the RCCL all-reduces of the collective chain (USV_GRAPH_COLLECTIVES=0 keeps them eager; gloo
    never captures them); the collective chain is the default path without the peer exchange (USV_DP_COLL_CHAIN=0
    or USV_PPO_FUSED=0: the three-launch split)."""
    from types import SimpleNamespace
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    ns = SimpleNamespace(multi_gpu=True, rank_size=2, _dp_ranks=True, _dp=object())
    ns._fused_update = lambda: A2CAgent._fused_update(ns)
    ns._coll_update = lambda: A2CAgent._coll_update(ns)
    for k in ("USV_GRAPH_COLLECTIVES", "USV_DP_COLL_CHAIN"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("USV_DIST_BACKEND", "nccl")
    monkeypatch.setenv("USV_PPO_FUSED", "1")
    assert A2CAgent._update_capturable(ns) and ns._fused_update() and not ns._coll_update()
    ns._dp = None                                   # no peer exchange: the collective chain, captured on nccl
    assert not ns._fused_update() and ns._coll_update() and A2CAgent._update_capturable(ns)
    monkeypatch.setenv("USV_GRAPH_COLLECTIVES", "0")
    assert not A2CAgent._update_capturable(ns)
    monkeypatch.delenv("USV_GRAPH_COLLECTIVES")
    monkeypatch.setenv("USV_DIST_BACKEND", "gloo")
    assert not A2CAgent._update_capturable(ns)
    monkeypatch.setenv("USV_DIST_BACKEND", "nccl")
    monkeypatch.setenv("USV_DP_COLL_CHAIN", "0")
    assert not ns._coll_update()                    # the split path
    monkeypatch.delenv("USV_DP_COLL_CHAIN")
    monkeypatch.setenv("USV_PPO_FUSED", "0")
    assert not ns._coll_update() and not ns._fused_update()
    ns._dp_ranks, ns.rank_size = False, 1
    monkeypatch.setenv("USV_PPO_FUSED", "1")
    assert A2CAgent._update_capturable(ns) and ns._fused_update() and not ns._coll_update()


def _capture_agree_worker(rank, world, port, out_dir, fail_ranks):
    """One rank of A2CAgent._update_from_graph with a capture that raises on `fail_ranks` (a collective the backend
    cannot capture): the ranks agree over gloo and every rank takes the eager update, this epoch and the next."""
    from types import SimpleNamespace
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        log = []
        ns = SimpleNamespace(rank=rank, rank_size=world, multi_gpu=True, ppo_device="cpu", _graph_update=None,
                             _dp_ranks=True, _dp=None)

        class G:
            def replay(self):
                log.append("replay")

        def capture(fn):
            if rank in fail_ranks:
                raise RuntimeError("operation not permitted when stream is capturing")
            return G()
        ns._graph_capture = capture
        ns.update_epoch_minibatches = lambda: log.append("eager")
        ns._ranks_agree = lambda ok: A2CAgent._ranks_agree(ns, ok)
        ns._fused_update = lambda: A2CAgent._fused_update(ns)
        for _ in range(2):   # two epochs: capture (or fall back), then the steady state
            if A2CAgent._update_capturable(ns):
                A2CAgent._update_from_graph(ns)
            else:
                ns.update_epoch_minibatches()
        np.savez(os.path.join(out_dir, f"cap{rank}.npz"), log=np.array(log), failed=getattr(ns, "_graph_update_failed",
                                                                                             False))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_ranks", [(2, ()), (2, (1,)), (2, (0, 1)), (4, ()), (4, (3,))])
def test_graph_capture_agreement_chooses_one_path_on_every_rank(tmp_path, world, fail_ranks, monkeypatch):
    """The update graph with RCCL collectives (the default on nccl): when the capture fails on any rank, every rank
    runs the update eagerly (now and in later epochs); when it succeeds on all, every rank replays the graph.  gloo
    carries the agreement here, as the nccl backend does on the GPUs; 4 ranks rehearse BASELINE configs[3]'s split."""
    monkeypatch.setenv("USV_DIST_BACKEND", "nccl")   # the capture gate of the GPU runs (the agreement still uses gloo)
    monkeypatch.delenv("USV_GRAPH_COLLECTIVES", raising=False)
    mp.spawn(_capture_agree_worker, args=(world, _port(), str(tmp_path), fail_ranks), nprocs=world, join=True)
    logs = [list(np.load(tmp_path / f"cap{r}.npz")["log"]) for r in range(world)]
    want = ["eager", "eager"] if fail_ranks else ["replay", "replay"]
    assert logs == [want] * world, logs
