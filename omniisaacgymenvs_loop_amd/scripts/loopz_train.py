"""loopz training entry: the reference's default trainer (omniisaacgymenvs/scripts/rlgames_train.py)
on the MI355X kernels (csrc/loopz.hip) and this package's USV env.

    python -m omniisaacgymenvs_loop_amd.scripts.loopz_train \
        task=USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST train=USV/USV_MLP \
        num_envs=512 seed=42 max_iterations=100 [checkpoint=runs/USV/nn/full_2000.pt] [cfg_dir=...]

Same loop as the reference (rlgames_train.py:362-558): per update env.reset(), optional checkpoint
(`full_<update>.pt`: actor / distribution / critic state dicts + Adam state + update) every
eval_every_n updates, n_steps = floor(max_time / control_dt) observe / step transitions, ppo.update
(gamma 0.997, lambda 0.95, 4 epochs x 4 in-order minibatches, lr 5e-4, clip 0.5), then
enforce_minimum_std(0.05).  The environment / architecture keys come from
task/USV/IROS2024/cfg.yaml of the cfg tree (num_envs / num_threads not overridden).  The rollout
stays on the GPU (observe_device / step_device); only the per-update statistics are read back.
"""
from __future__ import annotations

import math
import os
import sys
import time

import torch

from .rlgames_train import build_config, parse_overrides
from ..utils.hydra_cfg import load_yaml


# the activation constructors the reference passes (rlgames_train.py:161, 281); the kernels
# implement LeakyReLU(0.01) hidden layers and a tanh / identity output
_LeakyReLU, _Tanh = torch.nn.LeakyReLU, torch.nn.Tanh


def merge_loopz_overrides(cfg, cfg_dir):
    """rlgames_train.py:110-135: environment / architecture of IROS2024/cfg.yaml (num_envs, num_threads dropped)."""
    path = os.path.join(cfg_dir, "task", "USV", "IROS2024", "cfg.yaml")
    try:
        ov = load_yaml(path)
    except (OSError, ValueError) as exc:
        print(f"[loopz] skip legacy overrides (failed to load '{path}'): {exc}")
        return cfg
    env = dict(ov.get("environment", {}) or {})
    env.pop("num_envs", None)
    env.pop("num_threads", None)
    cfg.setdefault("environment", {}).update(env)
    cfg.setdefault("architecture", {}).update(dict(ov.get("architecture", {}) or {}))
    print(f"[loopz] merged legacy overrides: {path}")
    return cfg


def build(cfg):
    from ..envs.vec_env_rlgames import VecEnvRLGames
    from ..loopz import PPO, Actor, Critic, MLPEncode_wrap, SquashedGaussianDiagonalCovariance, USVRaisimVecEnv
    from ..utils.task_util import initialize_task
    env_rlg = VecEnvRLGames(headless=True)
    initialize_task(cfg, env_rlg)
    env = USVRaisimVecEnv(env_rlg)
    env.reset()
    ob_dim, act_dim = env.num_obs, env.num_acts
    ec, ac = cfg["environment"], cfg["architecture"]
    n_steps = math.floor(ec["max_time"] / ec["control_dt"])
    if ec.get("unnormalize_speed_vec"):
        raise NotImplementedError()
    if ac["layer_type"] != "feedforward":
        raise NotImplementedError()
    out_act = {"none": None, "tanh": _Tanh}[ac["activation"]]
    kw = dict(speed_dim=int(ec.get("speed_dim", 3)), mass_dim=int(ec.get("mass_dim", 4)),
              mass_latent_dim=int(ac.get("mass_latent_dim", 8)),
              mass_encoder_shape=tuple(int(v) for v in (ac.get("mass_encoder_shape") or (64, 16))))
    action_scale = float(cfg["task"]["env"].get("clipActions", 1.0))
    seed = int(cfg["seed"])
    device = cfg.get("rl_device", "cuda:0")
    actor = Actor(MLPEncode_wrap(ac["policy_net"], _LeakyReLU, ob_dim, act_dim, out_act, bool(ac["small_init"]),
                                 seed=seed, **kw),
                  SquashedGaussianDiagonalCovariance(act_dim, 0.3, action_scale=action_scale), device)
    critic = Critic(MLPEncode_wrap(ac["value_net"], _LeakyReLU, ob_dim, 1, seed=seed + 1, **kw), device)
    ppo = PPO(actor=actor, critic=critic, num_envs=env.num_envs, num_transitions_per_env=n_steps,
              num_learning_epochs=4, gamma=0.997, lam=0.95, num_mini_batches=4, device=device,
              log_dir=os.path.join("runs", cfg["train"]["params"]["config"]["name"]), mini_batch_sampling="in_order",
              learning_rate=5e-4, seed=seed)
    return env, actor, critic, ppo, n_steps


def save_full(path, actor, critic, ppo, update):
    torch.save({"actor_architecture_state_dict": actor.architecture.state_dict(),
                "actor_distribution_state_dict": actor.distribution.state_dict(),
                "critic_architecture_state_dict": critic.architecture.state_dict(),
                "optimizer_state_dict": ppo.optimizer_state_dict(), "update": update}, path)


def load_full(path, actor, critic, ppo) -> int:
    ckpt = torch.load(path, map_location="cpu", weights_only=True)
    if not (isinstance(ckpt, dict) and "actor_architecture_state_dict" in ckpt):
        print(f"[loopz] Checkpoint not in loopz .pt format, skipping load: {path}")
        return 0
    actor.architecture.load_state_dict(ckpt["actor_architecture_state_dict"])
    if "actor_distribution_state_dict" in ckpt:
        actor.distribution.load_state_dict(ckpt["actor_distribution_state_dict"])
    if "critic_architecture_state_dict" in ckpt:
        critic.architecture.load_state_dict(ckpt["critic_architecture_state_dict"])
    if "optimizer_state_dict" in ckpt:
        ppo.load_optimizer_state_dict(ckpt["optimizer_state_dict"])
    start = int(ckpt.get("update", -1)) + 1 if "update" in ckpt else 0
    print(f"[loopz] Resumed from checkpoint: {path} (start_update={start})")
    return start


def train(cfg, max_updates=None, log=print):
    env, actor, critic, ppo, n_steps = build(cfg)
    exp = cfg["train"]["params"]["config"]["name"]
    ckpt_dir = os.path.join("runs", exp, "nn")
    os.makedirs(ckpt_dir, exist_ok=True)
    start = load_full(cfg["checkpoint"], actor, critic, ppo) if cfg.get("checkpoint") else 0
    ppo.update_rl_coeff(0.3)
    if max_updates is None:
        max_updates = int(cfg["train"]["params"]["config"].get("max_epochs", 500000))
    eval_every = int(cfg["environment"]["eval_every_n"])
    total_steps = n_steps * env.num_envs
    history = []
    dev = ppo.params.device
    for update in range(start, max_updates + 1):
        t0 = time.time()
        env.reset()
        if update % eval_every == 0:
            save_full(os.path.join(ckpt_dir, f"full_{update}.pt"), actor, critic, ppo, update)
            env.reset()
            env.save_scaling(ckpt_dir, str(update))
        rew_sum = torch.zeros((), device=dev, dtype=torch.float64)
        done_sum = torch.zeros((), device=dev, dtype=torch.float64)
        for _ in range(n_steps):
            obs = env.observe_device()
            action = ppo.observe_device(obs)
            rew, dones = env.step_device(action)
            info = env.get_extras()
            # episode infos reach the PPO log only on a step where some env is done (rlgames_train.py:440-456):
            # the step's done flag stays on the device and the log filters on it once per update (no host sync)
            ppo.step_device(rew, dones, infos=[info] if isinstance(info, dict) and info.get("episode") else [],
                            valid=dones.any())
            rew_sum += rew.double().sum()
            done_sum += dones.double().sum()
        env.curriculum_callback()
        obs = env.observe_device()
        ppo.update(actor_obs=obs, value_obs=obs, log_this_iteration=update % 10 == 0, update=update)
        actor.distribution.enforce_minimum_std(torch.ones(env.num_acts) * 0.05)
        dt = time.time() - t0
        avg = float(rew_sum.item()) / total_steps
        history.append({"update": update, "average_ll_reward": avg, "dones": float(done_sum.item()) / total_steps,
                        "lr": ppo.lr, "seconds": dt, "fps": total_steps / dt,
                        "std": actor.distribution.std.detach().cpu().tolist(), "value_loss": ppo.mean_value_loss,
                        "surrogate_loss": ppo.mean_surrogate_loss})
        log('----------------------------------------------------')
        log('{:>6}th iteration'.format(update))
        log('{:<40} {:>6}'.format("average ll reward: ", '{:0.10f}'.format(avg)))
        log('{:<40} {:>6}'.format("dones: ", '{:0.6f}'.format(history[-1]["dones"])))
        log('{:<40} {:>6}'.format("lr: ", '{:.4e}'.format(ppo.lr)))
        log('{:<40} {:>6}'.format("time elapsed in this iteration: ", '{:6.4f}'.format(dt)))
        log('{:<40} {:>6}'.format("fps: ", '{:6.0f}'.format(total_steps / dt)))
        log('std: ' + str(history[-1]["std"]))
    return history, ppo


def main(argv=None):
    ov = parse_overrides(sys.argv[1:] if argv is None else argv)
    ov.setdefault("train", "USV/USV_MLP")
    cfg_dir = ov.get("cfg_dir", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cfg"))
    cfg = build_config(ov)
    cfg = merge_loopz_overrides(cfg, cfg_dir)
    train(cfg)


if __name__ == "__main__":
    main()
