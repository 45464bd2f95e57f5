"""End-to-end: rl_games Runner -> A2CAgent -> VecEnvRLGames -> USV kernels, a few epochs."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_runner_trains_usv(tmp_path):
    from omniisaacgymenvs_loop_amd.scripts import rlgames_train as T
    from omniisaacgymenvs_loop_amd.rl_games import vecenv
    from omniisaacgymenvs_loop_amd.rl_games.torch_runner import Runner
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    cfg = T.build_config({"num_envs": 1024, "max_iterations": 3, "minibatch_size": 4096})
    cfg["train"]["params"]["config"]["train_dir"] = str(tmp_path)
    env = VecEnvRLGames(headless=True)
    task = initialize_task(cfg, env)
    vecenv.register("RLGPU", lambda name, n, **kw: vecenv.RLGPUEnv(name, n, **kw))
    vecenv.register_env("rlgpu", {"vecenv_type": "RLGPU", "env_creator": lambda **kw: env})
    runner = Runner()
    runner.load(cfg["train"])
    agent = runner.algo_factory["a2c_continuous"](base_name="run", params=runner.params)
    agent.train()
    assert agent.epoch_num == 3
    assert agent.frame == 3 * 1024 * 16
    assert torch.isfinite(agent.model_params).all()
    assert agent.game_rewards.current_size > 0
    assert os.path.exists(os.path.join(str(tmp_path), agent.experiment_name, "nn"))


def _agent_env(n, minibatch, use_graph, seed=11):
    from omniisaacgymenvs_loop_amd.scripts import rlgames_train as T
    from omniisaacgymenvs_loop_amd.rl_games import vecenv
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    cfg = T.build_config({"num_envs": n, "minibatch_size": minibatch, "seed": seed})
    env = VecEnvRLGames(headless=True)
    task = initialize_task(cfg, env)
    params = cfg["train"]["params"]
    params["config"].update(vec_env=env, train_dir="/tmp/graph_test_runs", hip_graph=use_graph, print_stats=False)
    return env, task, A2CAgent("run", params)


def test_graph_replay_matches_eager():
    """The captured rollout + update graphs replay exactly what the eager loop launches: after 4 epochs
    (1 eager, 1 capture, 2 replays) parameters, optimiser state, env state and episode meters are
    bit-identical."""
    runs = []
    for use_graph in (False, True):
        env, task, ag = _agent_env(512, 2048, use_graph)
        ag.obs = ag.env_reset()
        for _ in range(4):
            ag.train_epoch()
        torch.cuda.synchronize()
        runs.append({"params": ag.model_params.cpu().numpy(), "m": ag.adam_m.cpu().numpy(),
                     "obs_rms": ag.obs_rms.cpu().numpy(), "state": task.state.cpu().numpy(),
                     "obs": task.obs_buf_t.cpu().numpy(), "clock": task.clock.cpu().numpy(),
                     "step_dev": ag.step_dev.cpu().numpy(), "lr": ag.last_lr,
                     "host_step": task._step_index, "meters": ag.game_rewards.get_mean()})
        if use_graph:
            assert ag._graph_play is not None and ag._graph_update is not None
    a, b = runs
    for k in ("params", "m", "obs_rms", "state", "obs", "clock", "step_dev"):
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert a["lr"] == b["lr"] and a["host_step"] == b["host_step"]
    # episode meters: per-workgroup partials folded in a fixed order, so identical too
    assert a["meters"] == b["meters"]
    assert int(b["clock"][0]) == b["host_step"]


def test_priv4_training_keeps_pad_columns_zero(tmp_path):
    """priv_dim 4 -> 29 observation columns: the device net's W1 pad columns get no gradient and
    no Adam moment, so training is exactly the 29-input network's; the checkpoint holds [NH, 29]."""
    from omniisaacgymenvs_loop_amd.scripts import rlgames_train as T
    from omniisaacgymenvs_loop_amd.rl_games import checkpoint as C
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    from omniisaacgymenvs_loop_amd.envs.vec_env_rlgames import VecEnvRLGames
    from omniisaacgymenvs_loop_amd.utils.task_util import initialize_task
    cfg = T.build_config({"num_envs": 512, "minibatch_size": 2048, "seed": 5})
    cfg["task"]["env"].pop("mass_dim", None)
    cfg["task"]["env"]["priv_dim"] = 4
    env = VecEnvRLGames(headless=True)
    task = initialize_task(cfg, env)
    assert task.num_observations == 29
    params = cfg["train"]["params"]
    params["config"].update(vec_env=env, train_dir=str(tmp_path), print_stats=False)
    ag = A2CAgent("run", params)
    ag.obs = ag.env_reset()
    for _ in range(3):
        ag.train_epoch()
    torch.cuda.synchronize()
    for t in (ag.model_params, ag.adam_m, ag.adam_v):
        w1 = C.split_flat(t.detach().cpu())[C.W1_KEY]
        assert float(w1[:, 29:].abs().max()) == 0.0
        assert float(w1[:, :29].abs().max()) > 0.0
    ag.save(str(tmp_path / "ck"))
    ck = C.load_checkpoint(str(tmp_path / "ck.pth"))
    assert tuple(ck["model"][C.W1_KEY].shape) == (C.NH, 29)
    assert tuple(ck["model"]["running_mean_std.running_mean_std.state.running_mean"].shape) == (29,)


def test_nan_probe_raises(monkeypatch):
    """USV_NAN_PROBE (USV_Virtual.py:57-95, vec_env_rlgames.py:41-80): a NaN action reaches the env step
    kernel -> the device flag -> RuntimeError naming the stage at the epoch's check; a NaN in the policy
    weights -> the rollout kernel's flag; USV_NAN_PROBE=0 disables both."""
    env, task, ag = _agent_env(256, 1024, False, seed=2)
    ag.obs = ag.env_reset()
    ag.train_epoch()                                   # finite: no raise
    a = torch.zeros((256, 2), device="cuda:0")
    a[17, 1] = float("nan")
    env.step(a)
    with pytest.raises(RuntimeError, match=r"USV_NAN_PROBE.*actions\(clamped\)"):
        env.check_errors()
    env.check_errors()                                 # the flag was cleared by the raise
    ag.model_params[5] = float("nan")                  # a W1 entry: every mu / value of the rollout is NaN
    with pytest.raises(RuntimeError, match=r"USV_NAN_PROBE.*(policy mu/value|actions)"):
        ag.train_epoch()
    torch.cuda.synchronize()
    monkeypatch.setenv("USV_NAN_PROBE", "0")
    env2, task2, ag2 = _agent_env(256, 1024, False, seed=2)
    ag2.obs = ag2.env_reset()
    ag2.model_params[5] = float("nan")
    ag2.train_epoch()                                  # probe off: no raise
    assert not torch.isfinite(ag2.exp_mu).all()


def test_nan_probe_raises_on_a_nan_episode_extra():
    """USV_Virtual.py:1601-1605: under the probe a NaN episode statistic raises '[USV_NAN_PROBE] episode extra is
    NaN before masking' instead of being zeroed silently (the extras fold ORs USV_NAN_EXTRAS); it is still masked
    to 0 in extras["episode"] as the reference does after the check."""
    from omniisaacgymenvs_loop_amd._abi import STAT_KEYS_ENUM
    env, task, ag = _agent_env(256, 1024, False, seed=2)
    ag.obs = ag.env_reset()
    z = torch.zeros((256, 2), device="cuda:0")
    env.step(z)
    env.check_errors()
    k = STAT_KEYS_ENUM["ST_U_MEAN"]
    task.stats[k, 5] = float("nan")       # a non-reward statistic of env 5 ...
    task.ibuf[2, 5] = 1                   # ... which resets at the start of the next step
    env.step(z)
    torch.cuda.synchronize()
    assert float(task.extras_buf[k]) == 0.0
    with pytest.raises(RuntimeError, match=r"USV_NAN_PROBE.*episode extra is NaN before masking"):
        env.check_errors()
