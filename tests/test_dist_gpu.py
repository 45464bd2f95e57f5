"""Two ranks on ONE GPU (gloo over the device tensors, USV_RANKS_SHARE_DEVICE): A2CAgent's multi-GPU
branch end to end -- the initial weight broadcast (a2c_common.py:1354), the per-minibatch flat
gradient + KL all-reduce and the 1/world scale inside the Adam kernel (a2c_common.py:308-323,
1218-1222), the LR schedule following the all-reduced KL -- against a single rank that trains on
both ranks' rows; and the per-rank env streams (torch_runner.py:74-75 seeds every rank with
seed + LOCAL_RANK before any env draw).
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, H, MB, EPOCHS = 256, 16, 1024, 2     # per rank: 4096 rows, 4 minibatches of 1024


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dataset(rows, seed=5):
    rng = np.random.default_rng(seed)
    f = np.float32
    return {"exp_obs": rng.normal(0, 2, (rows, 33)).astype(f), "exp_act": rng.normal(0, 1, (rows, 2)).astype(f),
            "exp_nlp": rng.uniform(1.5, 3.5, rows).astype(f), "exp_val": rng.normal(0, 1, rows).astype(f),
            "exp_ret": rng.normal(0, 1, rows).astype(f), "exp_adv": rng.normal(0, 1, rows).astype(f),
            "exp_mu": rng.normal(0, 0.3, (rows, 2)).astype(f), "exp_sigma": np.ones((rows, 2), f)}


def _rank_rows(rank, world):
    """Rank r's local batch: minibatch i of rank r = rows [i*MB + r*MB/world .. ) of the union layout
    the single-rank run sees (each union minibatch = rank 0's share, then rank 1's, ...)."""
    half = MB // world
    idx = [np.arange(i * MB + rank * half, i * MB + (rank + 1) * half) for i in range(N * H * world // MB)]
    return np.concatenate(idx)


def _agent(n_envs, minibatch, multi_gpu, params_seed=11):
    import yaml
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from tests.test_ppo_gpu import FakeVecEnv
    with open(os.path.join(ROOT, "omniisaacgymenvs_loop_amd/cfg/train/USV/USV_PPOcontinuous_MLP.yaml")) as f:
        params = yaml.safe_load(f)["params"]
    params["seed"] = params_seed
    # obs RMS is per rank in the reference (never synchronised): off, so the union run is comparable
    params["config"].update(num_actors=n_envs, minibatch_size=minibatch, mini_epochs=EPOCHS, device="cuda:0",
                            vec_env=FakeVecEnv(n_envs), train_dir="/tmp/dist_gpu_runs", multi_gpu=multi_gpu,
                            normalize_input=False, print_stats=False)
    return A2CAgent("run", params)


def _load(ag, data, rows):
    for k, v in data.items():
        getattr(ag, k).copy_(torch.tensor(np.ascontiguousarray(v[rows]), device="cuda:0"))


def _worker(rank, world, port, out_dir, exchange):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), USV_RANKS_SHARE_DEVICE="0", USV_DIST_BACKEND="gloo",
                      USV_DP_EXCHANGE=exchange, USV_DP_TIMEOUT_MS="10000")
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    try:
        # different init seeds per rank: the broadcast must make rank 0's weights everyone's
        ag = _agent(N, MB // world, True, params_seed=11 + 100 * rank)
        assert ag.multi_gpu and ag.rank_size == world
        assert (ag._dp is not None) == (exchange == "peer"), exchange
        _load(ag, _dataset(N * H * world), _rank_rows(rank, world))
        p0 = ag.model_params.cpu().numpy().copy()
        ag.update_epoch_minibatches()
        torch.cuda.synchronize()
        if ag._dp is not None:
            ag._dp.check()
        # env streams: the same config on every rank, seeds offset by LOCAL_RANK
        from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
        from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config
        from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
        cfg = build_config({"num_envs": 64, "seed": 42, "multi_gpu": True})
        task = initialize_task(cfg, VecEnvRLGames(headless=True))
        obs, _, _ = task.env_step(torch.zeros((64, 2), device="cuda:0"))
        torch.cuda.synchronize()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), p0=p0, p=ag.model_params.cpu().numpy(),
                 lr=float(ag.opt[0].item()), kls=ag.kls.cpu().numpy(), env_seed=task.seed, obs=obs.cpu().numpy(),
                 mass=task.params[0].cpu().numpy(), norm=float(ag.opt[3].item()))
        if ag._dp is not None:
            dist.barrier()          # no rank unmaps / frees a buffer another rank may still touch
            ag._dp.close()
    finally:
        dist.destroy_process_group()


_RUNS = {}


def _run_ranks(tmp_path_factory, exchange):
    if exchange not in _RUNS:
        import torch.multiprocessing as mp
        out = tmp_path_factory.mktemp(f"dist_gpu_{exchange}")
        mp.spawn(_worker, args=(2, _port(), str(out), exchange), nprocs=2, join=True)
        _RUNS[exchange] = [np.load(out / f"r{r}.npz") for r in range(2)]
    return _RUNS[exchange]


@pytest.fixture(scope="module", params=["peer", "collective"])
def two_ranks(request, tmp_path_factory):
    """peer: ppo_minibatch_fused_dp's one-shot exchange through IPC-mapped buffers (two processes on one
    device: the same kernels, handles and flags as over xGMI); collective: the gloo all-reduce split."""
    return _run_ranks(tmp_path_factory, request.param)


def test_peer_exchange_equals_collective_path(tmp_path_factory):
    """The peer exchange (rank-order sum / world inside the reduction, speculative Adam step) and the gloo
    all-reduce + k_apply split give bit-identical weights, KLs and LR for two ranks when no step clips
    (x0 + x1 == x1 + x0; / 2 == * 0.5)."""
    a = _run_ranks(tmp_path_factory, "peer")
    b = _run_ranks(tmp_path_factory, "collective")
    assert float(b[0]["norm"]) < 1.0                                 # grad_norm 1.0: no clipping here
    for k in ("p", "kls", "lr"):
        np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=k)
        np.testing.assert_array_equal(a[1][k], b[1][k], err_msg=k)


def test_two_ranks_equal_single_rank_on_the_union(two_ranks):
    r0, r1 = two_ranks
    np.testing.assert_array_equal(r0["p0"], r1["p0"])              # broadcast from rank 0
    np.testing.assert_array_equal(r0["p"], r1["p"])                # identical updates on both ranks
    assert r0["lr"] == r1["lr"]
    single = _agent(2 * N, MB, False, params_seed=11)
    np.testing.assert_array_equal(single.model_params.cpu().numpy(), r0["p0"])
    _load(single, _dataset(N * H * 2), np.arange(2 * N * H))
    single.update_epoch_minibatches()
    torch.cuda.synchronize()
    from tests import errtab as ET
    # the mean of two half-minibatch gradients == the union minibatch's gradient up to summation order
    ET.check("dist_2ranks", "params", r0["p"], single.model_params.cpu().numpy(), 1e-5, 1e-5)
    ET.check("dist_2ranks", "kl", r0["kls"], single.kls.cpu().numpy(), 1e-4, 1e-7)
    assert r0["lr"] == pytest.approx(float(single.opt[0].item()), rel=1e-6)


def _worker_setup_only(rank, world, port, out_dir):
    """The peer exchange's set-up for `world` ranks (handle exchange, mapping, the agreed self-test rounds over
    every sender's flags and payload slots) without training."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), USV_RANKS_SHARE_DEVICE="0", USV_DIST_BACKEND="gloo",
                      USV_DP_EXCHANGE="peer", USV_DP_TIMEOUT_MS="10000", USV_DP_SHARED_DEVICE_SETUP="1")
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    try:
        ag = _agent(N, MB // world, True, params_seed=11 + 100 * rank)
        np.savez(os.path.join(out_dir, f"s{rank}.npz"), peer=ag._dp is not None)
        if ag._dp is not None:
            dist.barrier()
            ag._dp.close()
    finally:
        dist.destroy_process_group()


def test_four_ranks(tmp_path_factory):
    """World size 4: the peer exchange's set-up and self-test pass with four senders per chunk (rank-order sums,
    four flags per chunk), and the multi-rank update (collective path) leaves all four ranks bit-identical and
    equal to a single rank on the union of the four batches up to summation order.  (Training through the peer
    exchange with four processes on ONE device is not a valid rehearsal: the other ranks' spinning reduction
    workgroups hold enough LDS on every CU that a waiting rank's gradient kernel -- 146 KB of LDS per
    workgroup -- cannot be placed; over xGMI every rank has its own device.)"""
    import torch.multiprocessing as mp
    world = 4
    out = tmp_path_factory.mktemp("dist_gpu_4")
    mp.spawn(_worker_setup_only, args=(world, _port(), str(out)), nprocs=world, join=True)
    assert all(bool(np.load(out / f"s{r}.npz")["peer"]) for r in range(world))
    mp.spawn(_worker, args=(world, _port(), str(out), "collective"), nprocs=world, join=True)
    rs = [np.load(out / f"r{r}.npz") for r in range(world)]
    for r in rs[1:]:
        np.testing.assert_array_equal(rs[0]["p0"], r["p0"])
        np.testing.assert_array_equal(rs[0]["p"], r["p"])
        assert rs[0]["lr"] == r["lr"]
    assert len({int(r["env_seed"]) for r in rs}) == world
    single = _agent(world * N, MB, False, params_seed=11)
    _load(single, _dataset(N * H * world), np.arange(world * N * H))
    single.update_epoch_minibatches()
    torch.cuda.synchronize()
    from tests import errtab as ET
    ET.check("dist_4ranks", "params", rs[0]["p"], single.model_params.cpu().numpy(), 1e-5, 1e-5)
    ET.check("dist_4ranks", "kl", rs[0]["kls"], single.kls.cpu().numpy(), 1e-4, 1e-7)
    assert rs[0]["lr"] == pytest.approx(float(single.opt[0].item()), rel=1e-6)


def test_ranks_draw_different_env_streams(two_ranks):
    r0, r1 = two_ranks
    assert int(r0["env_seed"]) == 42 and int(r1["env_seed"]) == 43
    assert not np.array_equal(r0["mass"], r1["mass"])              # SysID domain randomisation
    assert not np.array_equal(r0["obs"], r1["obs"])                # spawns, obstacles, noise


def test_dp_selftest_passes_alone_and_fails_fast_without_the_peer():
    """ppo_dp_selftest, the start-up check PeerExchange runs before training: one rank exchanging with
    itself passes and leaves the minibatch clock at the last test key; with a second "rank" that never
    runs, the first wait times out (bit 0), every later wait sees the error and returns at once, and the
    constructor's path raises -- so the agents fall back to collectives instead of stalling per chunk."""
    import time
    from omniisaacgymenvs_loop_amd.rl_games.dist_util import PeerExchange
    ok = PeerExchange(0, 1, "cuda:0", peers=[0])
    ok._selftest(2000)
    assert int(ok.clock.item()) == PeerExchange.SELFTEST_ROUNDS and int(ok.err.item()) == 0
    ok.close()
    lost = PeerExchange(0, 1, "cuda:0", peers=[0])       # a receive buffer nobody writes into
    ex = PeerExchange(0, 2, "cuda:0", peers=[0, lost.own_ptr])
    t0 = time.time()
    with pytest.raises(RuntimeError, match="flag did not arrive"):
        ex._selftest(300)
    assert time.time() - t0 < 5.0
    lost.close()


def test_bench_two_ranks_on_one_device(tmp_path):
    """The driver's multi-GPU bench path end to end on the one-GPU box: `torch.distributed.run --nproc-per-node 2
    bench.py --gpus 2` with both ranks on cuda:0 (gloo for the host-side collectives), the update's gradient
    exchange through the in-kernel peer path.  Rank 0 prints one line with n_gpus 2, the peer exchange on every
    rank, both start-up self-tests passing, per-rank records and a finite whole-job value."""
    import json
    import subprocess
    import sys
    env = dict(os.environ, USV_RANKS_SHARE_DEVICE="0", USV_DIST_BACKEND="gloo", USV_DP_EXCHANGE="peer",
               USV_DP_TIMEOUT_MS="10000")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_port()),
                          os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--envs", "8192", "--no-cpu-baseline", "--c2-steps", "0", "--milestone-seconds", "0"],
                         capture_output=True, text=True, timeout=240, cwd=str(tmp_path), env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["steps"] == 2
    assert line["config"]["exchange"] == "peer"
    assert line["extra"]["dp_selftest"] == {"0": "pass", "1": "pass"}
    assert [r["rank"] for r in line["extra"]["ranks"]] == [0, 1]
    assert np.isfinite(line["value"]) and line["value"] > 0


def _worker_rccl_one_rank(rank, port, out_dir):
    """The nccl (RCCL) backend on the one GPU a box has: world size 1, the split update path (USV_PPO_FUSED=0)
    with the fallback's collective -- dist_util.allreduce_grad's SUM all-reduce of [grad, kl] -- forced into
    every minibatch, eagerly and captured in the update's HIP graph (the USV_GRAPH_COLLECTIVES form)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
                      USV_DIST_BACKEND="nccl", USV_PPO_FUSED="0")
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import NPARAM
    try:
        data, rows = _dataset(N * H), np.arange(N * H)
        calls = []

        def with_allreduce(ag):
            def allreduce():   # a2c_common.py:309-323 on one rank: SUM over one rank is the identity, scale 1
                dist.all_reduce(ag.grad[:NPARAM + 1], op=dist.ReduceOp.SUM)
                calls.append(1)
                return 1.0
            ag._allreduce_grad = allreduce
            return ag

        eager = with_allreduce(_agent(N, MB, True))
        assert dist.get_backend() == "nccl" and eager.rank_size == 1
        _load(eager, data, rows)
        eager.update_epoch_minibatches()
        torch.cuda.synchronize()
        n_eager = len(calls)
        graph = with_allreduce(_agent(N, MB, True))
        _load(graph, data, rows)
        g = graph._graph_capture(graph.update_epoch_minibatches)   # records the all-reduces, runs nothing
        g.replay()
        torch.cuda.synchronize()
        plain = _agent(N, MB, False)          # the same split path without any collective
        _load(plain, data, rows)
        plain.update_epoch_minibatches()
        torch.cuda.synchronize()
        # the collective chain (ppo_minibatch_coll: two launches + the all-reduce per minibatch, the default
        # fallback of several ranks) on the multi-rank paths at world 1, eager and captured, against the split
        # path of several ranks (clip norm from the all-reduced gradient) without a collective
        os.environ.update(USV_DP_RANK_PATHS="1", USV_DP_EXCHANGE="collective", USV_PPO_FUSED="1")
        n0 = len(calls)
        coll = with_allreduce(_agent(N, MB, True))
        assert coll._dp is None and coll._coll_update() and coll._update_capturable()
        _load(coll, data, rows)
        coll.update_epoch_minibatches()
        torch.cuda.synchronize()
        n_coll = len(calls) - n0
        collg = with_allreduce(_agent(N, MB, True))
        _load(collg, data, rows)
        collg._graph_capture(collg.update_epoch_minibatches).replay()
        torch.cuda.synchronize()
        n_collg = len(calls) - n0 - n_coll
        os.environ["USV_PPO_FUSED"] = "0"
        split = _agent(N, MB, True)           # split path, several-rank semantics, no collective at world 1
        assert split._dp_ranks and not split._coll_update()
        _load(split, data, rows)
        split.update_epoch_minibatches()
        torch.cuda.synchronize()
        st = lambda ag: np.concatenate([ag.model_params.cpu().numpy(), ag.adam_m.cpu().numpy(),
                                        ag.adam_v.cpu().numpy(), ag.opt[:8].cpu().numpy()])
        np.savez(os.path.join(out_dir, "rccl.npz"), eager=eager.model_params.cpu().numpy(),
                 graph=graph.model_params.cpu().numpy(), plain=plain.model_params.cpu().numpy(),
                 kl_eager=eager.kls.cpu().numpy(), kl_graph=graph.kls.cpu().numpy(), kl_plain=plain.kls.cpu().numpy(),
                 n_eager=n_eager, n_capture=n0 - n_eager, minibatches=EPOCHS * N * H // MB,
                 coll=st(coll), collg=st(collg), split=st(split), kl_coll=coll.kls.cpu().numpy(),
                 kl_collg=collg.kls.cpu().numpy(), kl_split=split.kls.cpu().numpy(),
                 loss_coll=coll.loss_log.cpu().numpy(), loss_split=split.loss_log.cpu().numpy(),
                 n_coll=n_coll, n_collg=n_collg)
    finally:
        dist.destroy_process_group()


def test_rccl_fallback_collective_on_one_rank(tmp_path):
    """The RCCL fallback path executes: nccl process group, the flat-gradient SUM all-reduce per minibatch of the
    split update, eager and inside a captured HIP graph; both leave the weights and KLs bit-identical to the same
    update without a collective (one rank: the all-reduce is the identity).  Two ranks cannot share one GPU under
    nccl, so the multi-rank sums stay with the gloo tests above and the driver's multi-GPU run."""
    import torch.multiprocessing as mp
    mp.spawn(_worker_rccl_one_rank, args=(_port(), str(tmp_path)), nprocs=1, join=True)
    r = np.load(tmp_path / "rccl.npz")
    assert int(r["n_eager"]) == int(r["minibatches"]) == int(r["n_capture"])
    np.testing.assert_array_equal(r["eager"], r["plain"])
    np.testing.assert_array_equal(r["graph"], r["plain"])
    np.testing.assert_array_equal(r["kl_eager"], r["kl_plain"])
    np.testing.assert_array_equal(r["kl_graph"], r["kl_plain"])
    assert not np.array_equal(r["plain"], _agent(N, MB, False).model_params.cpu().numpy())   # the update moved them
    # the collective chain: one all-reduce per minibatch, eager and captured, the split path's bits (parameters,
    # Adam moments, optimiser scalars, KLs, losses)
    assert int(r["n_coll"]) == int(r["n_collg"]) == int(r["minibatches"])
    for k in ("coll", "collg"):
        np.testing.assert_array_equal(r[k], r["split"], err_msg=k)
        np.testing.assert_array_equal(r[f"kl_{k}"], r["kl_split"], err_msg=k)
    np.testing.assert_array_equal(r["loss_coll"], r["loss_split"])
