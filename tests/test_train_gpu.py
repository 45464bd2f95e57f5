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
