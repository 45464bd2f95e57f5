"""BASELINE configs[3] (C4): GoToPose + TrackXYOVelocity multi-task, one shared policy over task-split ranks.

bench.py --task multitask runs GoToPose on even ranks and TrackXYOVelocity on odd ranks (each rank its own
task instance, USV_go_to_pose.py:31-352 / USV_track_xyo_velocity.py:35-231), with ONE policy kept identical
by the per-minibatch gradient all-reduce (a2c_common.py:308-323, the KL one :1218-1222).  Rehearsed here as
two processes on one GPU (USV_RANKS_SHARE_DEVICE=0, gloo for the handle exchange / the collective path):
  - each rank's env step over its first steps equals the C oracle of its own task (obs at 1e-5, dones and
    goal counts exactly, as test_philox_mode_pose_tasks_match_oracle);
  - after two train epochs (eager, then graph-captured) both ranks hold bit-identical weights, LR and KLs;
  - the in-kernel peer exchange (ppo_minibatch_fused_dp) and the gloo all-reduce split give the same bits.
The runs train with grad_norm = 1e6 (truncate_grads on, never binding): the two paths form the clip norm in
different summation orders (the peer path from the reduction blocks' partial sums, the collective chain in
k_apply's float4 order), so a minibatch whose norm passes the reference's grad_norm 1.0 is stepped with clip
coefficients one ulp apart.  Random-init multi-task minibatches do pass 1.0, and the epoch-last norm the agent
keeps cannot show which did -- the bit comparison is of the exchange, not of the norm's summation order.
"""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, T_ORACLE, EPOCHS = 1024, 12, 2
TASKS = ("GoToPose", "TrackXYOVelocity")        # bench.py --task multitask: rank % 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, exchange):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world), USV_RANKS_SHARE_DEVICE="0", USV_DIST_BACKEND="gloo",
                      USV_DP_EXCHANGE=exchange, USV_DP_TIMEOUT_MS="10000")
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    from oracle import oracle as O
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.rl_games import vecenv
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config
    from omniisaacgymenvs_loop_amd.tasks.usv_config import thruster_tables
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    from tests import errtab as ET
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        name = TASKS[rank % 2]
        cfg = build_config({"num_envs": N, "seed": 42, "multi_gpu": True, "rl_device": "cuda:0",
                            "task": bench.TASKS[name][0]})
        cfg["train"]["params"]["config"].update(train_dir="/tmp/multitask_runs", print_stats=False,
                                                minibatch_size=8192, grad_norm=1e6)
        env = VecEnvRLGames(headless=True)
        task = initialize_task(cfg, env)
        assert task.seed == 42 + rank and task.cfg.task_kind == (1 if name == "GoToPose" else 2)
        # (1) this rank's env against the oracle of its own task, first steps from the initial reset
        E = O.OracleEnv(task.cfg, N, O.make_lut(*thruster_tables(cfg["task"])))
        rng = np.random.default_rng(100 + rank)
        for t in range(T_ORACLE):
            a = rng.uniform(-1, 1, (N, 2)).astype(np.float32)
            bias = task.current_action_bias()
            obs, rew, dones = task.env_step(torch.tensor(a, device="cuda:0"))
            E.full_step(a, bias, t, seed=task.seed)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(dones.cpu().numpy(), E.reset_buf, err_msg=f"{name} dones t={t}")
            ET.check(f"multitask_{name}", "obs", obs.cpu().numpy(), E.obs[:, :obs.shape[1]], 1e-5, 1e-5,
                     ET.obs_cols(obs.shape[1]), f"{name} obs t={t}")
            ET.check(f"multitask_{name}", "rew", rew.cpu().numpy(), E.rew, 1e-5, 1e-5, None, f"{name} rew t={t}")
            np.testing.assert_array_equal(task.ibuf[0].cpu().numpy(), E.goal_cnt, err_msg=f"{name} goals t={t}")
        # (2) one shared policy trained on both tasks' rollouts
        vecenv.register("RLGPU", lambda nm, n, **kw: vecenv.RLGPUEnv(nm, n, **kw))
        vecenv.register_env("rlgpu", {"vecenv_type": "RLGPU", "env_creator": lambda **kw: env})
        ag = A2CAgent("run", cfg["train"]["params"])
        assert ag.multi_gpu and ag.rank_size == world and (ag._dp is not None) == (exchange == "peer")
        ag.obs = ag.env_reset()
        p0 = ag.model_params.cpu().numpy().copy()
        norms = []
        for _ in range(EPOCHS):
            ag.update_epoch()
            ag.train_epoch()
            norms.append(float(ag.opt[3].item()))     # the epoch's last minibatch gradient norm
        torch.cuda.synchronize()
        if ag._dp is not None:
            ag._dp.check()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), p0=p0, p=ag.model_params.cpu().numpy(),
                 m=ag.adam_m.cpu().numpy(), lr=float(ag.opt[0].item()), kls=ag.kls.cpu().numpy(),
                 norm=max(norms), graph=ag._graph_update is not None, rew=ag.exp_rew.cpu().numpy(),
                 task=name)
        if ag._dp is not None:
            dist.barrier()          # no rank unmaps / frees a buffer another rank may still touch
            ag._dp.close()
    finally:
        dist.destroy_process_group()


_RUNS = {}


def _run(tmp_path_factory, exchange):
    if exchange not in _RUNS:
        import torch.multiprocessing as mp
        out = tmp_path_factory.mktemp(f"multitask_{exchange}")
        mp.spawn(_worker, args=(2, _port(), str(out), exchange), nprocs=2, join=True)
        _RUNS[exchange] = [np.load(out / f"r{r}.npz") for r in range(2)]
    return _RUNS[exchange]


@pytest.mark.parametrize("exchange", ["peer", "collective"])
def test_multitask_ranks_share_one_policy(tmp_path_factory, exchange):
    r0, r1 = _run(tmp_path_factory, exchange)
    assert str(r0["task"]) == "GoToPose" and str(r1["task"]) == "TrackXYOVelocity"
    np.testing.assert_array_equal(r0["p0"], r1["p0"])               # rank 0's initial weights everywhere
    assert not np.array_equal(r0["p"], r0["p0"])                    # it trained
    for k in ("p", "m", "kls", "lr"):
        np.testing.assert_array_equal(r0[k], r1[k], err_msg=k)      # one policy: identical bits on both ranks
    assert not np.array_equal(r0["rew"], r1["rew"])                 # ... from two different tasks' rollouts
    if exchange == "peer":
        assert bool(r0["graph"]) and bool(r1["graph"])              # the update replays as one HIP graph


def test_multitask_peer_exchange_equals_collective_path(tmp_path_factory):
    a = _run(tmp_path_factory, "peer")
    b = _run(tmp_path_factory, "collective")
    assert float(b[0]["norm"]) < 1e6                                # no step clipped (see the module doc)
    for k in ("p", "m", "kls", "lr"):
        np.testing.assert_array_equal(a[0][k], b[0][k], err_msg=k)
