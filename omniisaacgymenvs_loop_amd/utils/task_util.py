"""initialize_task (omniisaacgymenvs/utils/task_util.py:30-90): task map name -> class."""
from __future__ import annotations

import os
from typing import Any, Dict


def initialize_task(config: Dict[str, Any], env, init_sim: bool = True):
    from ..tasks.usv_virtual import USVVirtual
    task_map = {"USVVirtual": USVVirtual}
    task_cfg = config["task"]
    name = task_cfg.get("name", config.get("task_name"))
    if name not in task_map:
        raise NotImplementedError(f"task {name} is not on the MI355X hot path (only USVVirtual/CaptureXY)")
    num_envs = config.get("num_envs") or task_cfg["env"]["numEnvs"]
    device = config.get("rl_device", "cuda:0")
    seed = int(config.get("seed", 42))
    if config.get("multi_gpu", False):
        # the reference reseeds torch with seed + LOCAL_RANK before any training draw
        # (rl_games torch_runner.py:74-75): every rank's envs draw their own streams
        seed += int(os.getenv("LOCAL_RANK", "0"))
    task = task_map[name](task_cfg, num_envs=int(num_envs), device=device, seed=seed, rl_device=device)
    env.set_task(task=task, sim_params=task_cfg.get("sim"), backend="torch", init_sim=init_sim)
    return task
