"""Training / play entry point (omniisaacgymenvs/scripts/rlgames_train111.py:113-176).

Hydra-style overrides without Hydra:
    python -m omniisaacgymenvs_loop_amd.scripts.rlgames_train \
        task=USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST train=USV/USV_PPOcontinuous_MLP \
        num_envs=4096 seed=42 max_iterations=200 [test=True checkpoint=path.pth] [multi_gpu=True]
        [cfg_dir=/path/to/omniisaacgymenvs/cfg] [task.env.maxEpisodeLength=300 ...]
The yamls are composed and their OmegaConf interpolations resolved as Hydra does (utils/hydra_cfg.py);
cfg_dir points at another cfg tree, e.g. the reference's own (read unmodified).
Launch one process per GPU with torch.distributed.run for multi_gpu.
"""
from __future__ import annotations

import os
import sys
from typing import Any, Dict


PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

from ..utils.hydra_cfg import compose, parse_cli  # noqa: E402


ROOT_KEYS = ("experiment", "num_envs", "seed", "torch_deterministic", "max_iterations", "physics_engine", "pipeline",
             "sim_device", "device_id", "rl_device", "multi_gpu", "num_threads", "solver_type", "test", "checkpoint",
             "evaluation", "headless")
# shorthand keys of this entry point for train.params.config.<key>
TRAIN_SHORTHAND = ("minibatch_size", "horizon_length", "mini_epochs", "learning_rate")


def parse_overrides(argv):
    return parse_cli(argv)


def build_config(ov: Dict[str, Any]) -> Dict[str, Any]:
    """Compose config.yaml + task + train with the overrides and resolve the interpolations
    (rlgames_train111.py:113-124 + omegaconf_to_dict).  cfg_dir=<dir> selects another cfg tree,
    e.g. the reference's own omniisaacgymenvs/cfg (its yamls are read unmodified)."""
    ov = dict(ov)
    cfg_dir = ov.pop("cfg_dir", os.path.join(PKG, "cfg"))
    task_name = ov.pop("task", "USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST")
    train_name = ov.pop("train", "USV/USV_PPOcontinuous_MLP")
    multi_gpu = bool(ov.get("multi_gpu", False))
    from ..rl_games.dist_util import local_device
    if multi_gpu:
        ov["rl_device"] = local_device()
    overrides = {}
    for k, v in ov.items():
        if k in TRAIN_SHORTHAND:
            overrides[f"train.params.config.{k}"] = v
        elif k in ROOT_KEYS or "." in k:
            overrides[k] = v
        else:
            raise SystemExit(f"unknown override {k}")
    cfg = compose(cfg_dir, task_name, train_name, overrides)
    task, train = cfg["task"], cfg["train"]
    num_envs = int(cfg["num_envs"]) if cfg.get("num_envs", "") != "" else int(task["env"]["numEnvs"])
    task["env"]["numEnvs"] = num_envs
    cfg["num_envs"] = num_envs
    cfg["seed"] = int(cfg.get("seed", 42))
    cfg["test"] = bool(cfg.get("test", False))
    cfg["checkpoint"] = cfg.get("checkpoint", "") or ""
    rl_device = cfg.get("rl_device", "cuda:0")
    pc = train["params"]["config"]
    pc["num_actors"] = num_envs
    pc["device"] = pc["device_name"] = rl_device
    pc["multi_gpu"] = multi_gpu    # a2c_common.py:87 reads multi_gpu from the train config
    if cfg.get("max_iterations", "") != "":
        pc["max_epochs"] = int(cfg["max_iterations"])
    train["params"]["seed"] = cfg["seed"]
    return cfg


def main(argv=None):
    ov = parse_overrides(sys.argv[1:] if argv is None else argv)
    cfg = build_config(ov)
    from ..envs.vec_env_rlgames import VecEnvRLGames
    from ..rl_games import vecenv
    from ..rl_games.torch_runner import Runner
    from ..utils.task_util import initialize_task
    env = VecEnvRLGames(headless=True, sim_device=0)
    initialize_task(cfg, env)
    vecenv.register("RLGPU", lambda config_name, num_actors, **kwargs: vecenv.RLGPUEnv(config_name, num_actors,
                                                                                       **kwargs))
    vecenv.register_env("rlgpu", {"vecenv_type": "RLGPU", "env_creator": lambda **kwargs: env})
    runner = Runner()
    runner.load(cfg["train"])
    runner.reset()
    return runner.run({"train": not cfg["test"], "play": cfg["test"], "checkpoint": cfg["checkpoint"] or None})


if __name__ == "__main__":
    main()
