"""Training / play entry point (omniisaacgymenvs/scripts/rlgames_train111.py:113-176).

Hydra-style overrides without Hydra:
    python -m omniisaacgymenvs_loop_amd.scripts.rlgames_train \
        task=USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST train=USV/USV_PPOcontinuous_MLP \
        num_envs=4096 seed=42 max_iterations=200 [test=True checkpoint=path.pth] [multi_gpu=True]
Launch one process per GPU with torch.distributed.run for multi_gpu.
"""
from __future__ import annotations

import os
import sys
from typing import Any, Dict

import yaml

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(kind: str, name: str) -> Dict[str, Any]:
    path = name if name.endswith(".yaml") and os.path.exists(name) else os.path.join(PKG, "cfg", kind, name + ".yaml")
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)


def parse_overrides(argv):
    ov = {}
    for a in argv:
        if "=" not in a:
            raise SystemExit(f"expected key=value, got {a}")
        k, v = a.split("=", 1)
        k = k.lstrip("+")
        if v.lower() in ("true", "false"):
            v = v.lower() == "true"
        else:
            try:
                v = int(v)
            except ValueError:
                try:
                    v = float(v)
                except ValueError:
                    pass
        ov[k] = v
    return ov


def build_config(ov: Dict[str, Any]) -> Dict[str, Any]:
    task = _load("task", ov.get("task", "USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST"))
    train = _load("train", ov.get("train", "USV/USV_PPOcontinuous_MLP"))
    multi_gpu = bool(ov.get("multi_gpu", False))
    from ..rl_games.dist_util import local_device
    rl_device = local_device() if multi_gpu else ov.get("rl_device", "cuda:0")
    num_envs = int(ov.get("num_envs", task["env"]["numEnvs"]))
    task["env"]["numEnvs"] = num_envs
    cfg = {"task": task, "train": train, "seed": int(ov.get("seed", 42)), "num_envs": num_envs,
           "rl_device": rl_device, "multi_gpu": multi_gpu, "test": bool(ov.get("test", False)),
           "checkpoint": ov.get("checkpoint", "")}
    pc = train["params"]["config"]
    pc["num_actors"] = num_envs
    pc["device"] = pc["device_name"] = rl_device
    pc["multi_gpu"] = multi_gpu
    if "max_iterations" in ov:
        pc["max_epochs"] = int(ov["max_iterations"])
    for k in ("minibatch_size", "horizon_length", "mini_epochs", "learning_rate"):
        if k in ov:
            pc[k] = ov[k]
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
