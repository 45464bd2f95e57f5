"""PPO (omniisaacgymenvs/algo/ppo/ppo.py:11-325) on the loopz HIP kernels (csrc/loopz.hip).

Same constructor arguments and methods (observe / step / update / update_scheduler /
update_rl_coeff).  The parameters, the Adam moments, the rollout storage and every step of
observe / step / update live on the GPU; observe() and step() keep the reference's numpy
interface (they copy to / from the host) and observe_device() / step_device() are the
device-resident variants the loopz training loop uses.  mini_batch_sampling 'in_order' is the
trainer's choice (scripts/rlgames_train.py:325); 'shuffle' (the class default) draws a fresh
permutation of the T N storage rows per learning epoch on the device and hands each minibatch's
M rows to the gradient kernel (lz_minibatch_rows)."""
from __future__ import annotations

import math
import os
from datetime import datetime

import numpy as np
import torch

from .. import _capi
from .._abi import LzCfg
from .module import Actor, Critic, check_lib_layout
from .storage import RolloutStorage


class PPO:
    def __init__(self, actor: Actor, critic: Critic, num_envs, num_transitions_per_env, num_learning_epochs,
                 num_mini_batches, clip_param=0.2, gamma=0.998, lam=0.95, value_loss_coef=0.5, entropy_coef=0.0,
                 learning_rate=5e-4, max_grad_norm=0.5, use_clipped_value_loss=True, log_dir='run', device='cpu',
                 mini_batch_sampling='shuffle', log_intervals=10, flat_expert=None, seed=0):
        if mini_batch_sampling not in ("shuffle", "in_order"):
            raise NameError(mini_batch_sampling + ' is not a valid sampling method. Use one of the followings: shuffle, order')
        self.actor, self.critic = actor, critic
        # imitation (ppo.py:93-94, 253-286): any object with evaluate(obs [rows][D]) -> expert actions [rows][2]
        # (module.py Expert / Steps_Expert); frozen, so it is evaluated once per update on the stored
        # observations and the gradient kernel adds (1 - rl_coeff) * sum_a (expert_a - action_mean_a)^2
        self.flat_expert = flat_expert
        self._expert_act = None
        self.device = device if str(device).startswith("cuda") else "cuda:0"
        obs_dim = int(actor.obs_shape[0])
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, [obs_dim], [int(critic.obs_shape[0])],
                                      actor.action_shape, self.device)
        self.num_transitions_per_env, self.num_envs = int(num_transitions_per_env), int(num_envs)
        self.num_learning_epochs, self.num_mini_batches = int(num_learning_epochs), int(num_mini_batches)
        self.clip_param, self.gamma, self.lam = clip_param, gamma, lam
        self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
        self.max_grad_norm, self.use_clipped_value_loss = max_grad_norm, use_clipped_value_loss
        self.learning_rate = learning_rate
        self.rl_coeff = 1
        self.log_dir = os.path.join(log_dir, datetime.now().strftime('%b%d_%H-%M-%S'))
        self.log_intervals = log_intervals
        self.ep_infos = []
        self.tot_timesteps = 0
        self.seed = int(seed)
        self.mini_batch_sampling = mini_batch_sampling
        # shuffle: device permutation stream (the reference draws SubsetRandomSampler's randperm from torch's
        # global CPU generator, storage.py:123-134); inject_batches() replays recorded minibatches instead
        self._perm_gen = None
        self._injected_batches = None
        self._step_counter = 0
        c = LzCfg()
        c.n_envs, c.horizon, c.obs_dim = self.num_envs, self.num_transitions_per_env, obs_dim
        c.mini_batches, c.epochs = self.num_mini_batches, self.num_learning_epochs
        c.use_clipped_value_loss = int(bool(use_clipped_value_loss))
        c.gamma, c.lam, c.clip = float(gamma), float(lam), float(clip_param)
        c.value_loss_coef, c.entropy_coef, c.max_grad_norm = float(value_loss_coef), float(entropy_coef), float(max_grad_norm)
        c.lr, c.adam_b1, c.adam_b2, c.adam_eps = float(learning_rate), 0.9, 0.999, 1e-8
        c.min_std = 0.05
        scale = actor.distribution.action_scale
        c.action_scale[0], c.action_scale[1] = float(scale[0]), float(scale[1])
        self.cfg = c
        if _capi.lib().lz_partials_floats(_capi.byref(c)) < 0:
            raise ValueError("unsupported loopz configuration (obs_dim must be 33..36)")
        n = check_lib_layout(actor, critic)
        f32 = dict(device=self.device, dtype=torch.float32)
        # flat parameters in the optimizer's order (ppo.py:59): actor net | std | critic net
        self.params = torch.cat([actor.architecture.flat(), actor.distribution.std.detach().cpu().float(),
                                 critic.architecture.flat()]).to(**f32).contiguous()
        na = actor.architecture.numel()
        actor.architecture.bind(self.params, 0)
        actor.distribution.bind(self.params, na)
        critic.architecture.bind(self.params, na + actor.distribution.dim)
        self.nparam = n
        self.adam_m = torch.zeros(n, **f32)
        self.adam_v = torch.zeros(n, **f32)
        self.opt = torch.zeros(16, **f32)    # [2][8]: lr, step, value loss, surrogate, norm, applied
        self.opt[0] = float(learning_rate)
        self.partials = torch.zeros(int(_capi.lib().lz_partials_floats(_capi.byref(c))), **f32)
        self.grad = torch.zeros(int(_capi.lib().lz_grad_floats(obs_dim)), **f32)
        self.work = torch.zeros(8 + 2 * ((self.num_envs + 255) // 256) + 8, device=self.device, dtype=torch.float64)
        self.actions_dev = torch.zeros((self.num_envs, 2), **f32)
        self.last_values = torch.zeros(self.num_envs, **f32)
        self._obs_dev = None
        self.mean_value_loss = 0.0
        self.mean_surrogate_loss = 0.0

    # --------------------------------------------------------------- API
    def update_rl_coeff(self, coeffs):
        self.rl_coeff = float(np.clip(coeffs, 0, 1))
        print("Setting RL coeffs to {}".format(self.rl_coeff))

    def observe_device(self, actor_obs: torch.Tensor, eps_inject: torch.Tensor = None) -> torch.Tensor:
        """actor.sample + critic.predict on the device; rows go to storage slot `storage.step`."""
        st = self.storage
        if st.step >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        obs = actor_obs.contiguous()
        if obs.dtype != torch.float32 or obs.device != self.params.device:
            obs = obs.to(self.params.device, torch.float32).contiguous()
        self._obs_dev = obs
        _capi.call("lz_act", _capi.byref(self.cfg), _capi.ptr(self.params), _capi.ptr(obs), st.step,
                   _capi.ptr(st.actor_obs), _capi.ptr(st.actions), _capi.ptr(st.actions_log_prob),
                   _capi.ptr(st.values), _capi.ptr(self.actions_dev), self.seed, self._step_counter,
                   _capi.ptr(eps_inject), _capi.stream_ptr())
        return self.actions_dev

    def observe(self, actor_obs: np.ndarray) -> np.ndarray:
        """ppo.py:102-141 (numpy in, numpy actions out)."""
        return self.observe_device(torch.from_numpy(np.ascontiguousarray(actor_obs, np.float32))).cpu().numpy()

    def step_device(self, rews: torch.Tensor, dones: torch.Tensor, infos=(), valid=None):
        """ppo.py:143-153: values were formed in observe_device; stores rewards / dones.  `valid` (a device
        bool, nullable): the infos count only if it holds -- the trainer passes dones.any() so that the
        reference's "infos only on a step where some env is done" (rlgames_train.py:440-456) is decided at
        log time, once per update, instead of by a host sync every step."""
        st = self.storage
        r = rews.to(self.params.device, torch.float32).contiguous()
        d = dones.to(self.params.device, torch.int64).contiguous()
        _capi.call("lz_store", _capi.byref(self.cfg), _capi.ptr(r), _capi.ptr(d), st.step, _capi.ptr(st.rewards),
                   _capi.ptr(st.dones), _capi.stream_ptr())
        st.step += 1
        self._step_counter += 1
        for info in infos:
            ep = info.get("episode") if isinstance(info, dict) else None
            if ep is not None:
                # the reference's extras["episode"] holds fresh tensors per reset (USV_Virtual.py:1591-1612);
                # here they are views of one device buffer the next reset overwrites: snapshot them (one
                # stack kernel, no host sync)
                keys = list(ep.keys())
                vals = [ep[k] for k in keys]
                if keys and all(torch.is_tensor(v) and v.numel() == 1 for v in vals):
                    self.ep_infos.append((keys, torch.stack([v.reshape(()).float() for v in vals]), valid))
                else:
                    self.ep_infos.append((keys, vals, valid))

    def _valid_ep_infos(self):
        """The episode infos whose step had a done env (one host read of all the step flags)."""
        flags = [v for _, _, v in self.ep_infos if torch.is_tensor(v)]
        got = iter(torch.stack([f.reshape(()).bool() for f in flags]).cpu().tolist()) if flags else iter(())
        return [(k, v) for k, v, f in self.ep_infos if (next(got) if torch.is_tensor(f) else f is None or bool(f))]

    def step(self, value_obs, rews, dones, infos):
        self.step_device(torch.as_tensor(np.asarray(rews, np.float32)), torch.as_tensor(np.asarray(dones).astype(np.int64)),
                         infos)

    def update(self, actor_obs, value_obs, log_this_iteration, update):
        """ppo.py:155-176: last values, compute_returns, _train_step, storage.clear."""
        vo = value_obs if torch.is_tensor(value_obs) else torch.from_numpy(np.ascontiguousarray(value_obs, np.float32))
        vo = vo.to(self.params.device, torch.float32).contiguous()
        s = _capi.stream_ptr()
        st = self.storage
        _capi.call("lz_value", _capi.byref(self.cfg), _capi.ptr(self.params), _capi.ptr(vo), _capi.ptr(self.last_values), s)
        _capi.call("lz_returns", _capi.byref(self.cfg), _capi.ptr(self.last_values), _capi.ptr(st.rewards),
                   _capi.ptr(st.dones), _capi.ptr(st.values), _capi.ptr(st.returns), _capi.ptr(st.advantages),
                   _capi.ptr(self.work), s)
        self._bind_expert()
        self.mean_value_loss, self.mean_surrogate_loss = self._train_step()
        st.clear()
        if log_this_iteration and self.ep_infos:
            self.ep_infos = self._valid_ep_infos()
            if len(self.ep_infos) > 0:
                self.log(update)
        self.ep_infos.clear()

    def inject_batches(self, batches):
        """Replay recorded 'shuffle' minibatches ([epochs * mini_batches][M] row indices into the flattened
        T N storage, e.g. the BatchSampler draws of a reference run) on the next update (tests)."""
        b = torch.as_tensor(np.asarray(batches), dtype=torch.int32)
        m = self.num_transitions_per_env * self.num_envs // self.num_mini_batches
        if b.shape != (self.num_learning_epochs * self.num_mini_batches, m):
            raise ValueError(f"batches shape {tuple(b.shape)} != {(self.num_learning_epochs * self.num_mini_batches, m)}")
        if int(b.min()) < 0 or int(b.max()) >= self.num_transitions_per_env * self.num_envs:
            raise ValueError("batch row index out of range")
        self._injected_batches = b.to(self.params.device).contiguous()

    def _shuffle_rows(self):
        """[epochs * mini_batches][M] int32 rows: per epoch one permutation of range(T N) cut into
        mini_batches chunks of M, the tail dropped (BatchSampler(..., drop_last=True), storage.py:123-134)."""
        if self._injected_batches is not None:
            rows, self._injected_batches = self._injected_batches, None
            return rows
        nt = self.num_transitions_per_env * self.num_envs
        m = nt // self.num_mini_batches
        if self._perm_gen is None:
            self._perm_gen = torch.Generator(device=self.params.device)
            self._perm_gen.manual_seed(self.seed ^ 0x5EED5A11)
        perms = [torch.randperm(nt, device=self.params.device, generator=self._perm_gen)[:m * self.num_mini_batches]
                 for _ in range(self.num_learning_epochs)]
        return torch.stack(perms).view(-1, m).to(torch.int32).contiguous()

    def _bind_expert(self):
        """flat_expert.evaluate of every stored observation row (storage-row order, T N rows) into the buffer the
        gradient kernel reads, with the imitation coefficient 1 - rl_coeff (ppo.py:279-282)."""
        if self.flat_expert is None:
            self.cfg.expert_act = None
            self.cfg.im_coef = 0.0
            return
        st = self.storage
        with torch.no_grad():
            ea = self.flat_expert.evaluate(st.actor_obs.reshape(-1, st.actor_obs.shape[-1]))
        ea = torch.as_tensor(ea).to(self.params.device, torch.float32).reshape(-1, 2).contiguous()
        if ea.shape[0] != self.num_transitions_per_env * self.num_envs:
            raise ValueError(f"flat_expert.evaluate returned {tuple(ea.shape)} for "
                             f"{self.num_transitions_per_env * self.num_envs} rows")
        self._expert_act = ea
        self.cfg.expert_act = ea.data_ptr()
        self.cfg.im_coef = float(np.float32(1.0 - self.rl_coeff))

    def _train_step(self):
        """ppo.py:237-321 on the device: epochs x minibatches (in order, or shuffled rows), each one
        gradient launch, one fixed-order reduction and one clip + Adam launch (skipped on a non-finite loss)."""
        st = self.storage
        s = _capi.stream_ptr()
        k = 0
        logs = torch.zeros((self.num_learning_epochs * self.num_mini_batches, 8), device=self.params.device)
        rows = self._shuffle_rows() if self.mini_batch_sampling == "shuffle" else None
        for _ in range(self.num_learning_epochs):
            for mb in range(self.num_mini_batches):
                _capi.call("lz_minibatch_rows", _capi.byref(self.cfg), _capi.ptr(self.params), _capi.ptr(self.adam_m),
                           _capi.ptr(self.adam_v), _capi.ptr(self.opt), k % 2, mb, _capi.ptr(st.actor_obs),
                           _capi.ptr(st.actions), _capi.ptr(st.actions_log_prob), _capi.ptr(st.values),
                           _capi.ptr(st.returns), _capi.ptr(st.advantages),
                           _capi.ptr(rows[k]) if rows is not None else None, _capi.ptr(self.partials),
                           _capi.ptr(self.grad), s)
                logs[k].copy_(self.opt[8 * ((k + 1) % 2):8 * ((k + 1) % 2) + 8])
                k += 1
        if k % 2:
            self.opt[:8].copy_(self.opt[8:])
        lg = logs.cpu().numpy()
        ok = lg[:, 5] > 0
        if not ok.any():
            return 0.0, 0.0
        return float(lg[ok, 2].mean()), float(lg[ok, 3].mean())

    def update_scheduler(self):
        """LambdaLR(0.9998 ** epoch) (ppo.py:60-61, 323-324)."""
        self._sched_epoch = getattr(self, "_sched_epoch", 0) + 1
        self.opt[0] = float(self.learning_rate) * 0.9998 ** self._sched_epoch

    @property
    def lr(self) -> float:
        return float(self.opt[0].item())

    def adam_step(self) -> int:
        return int(round(float(self.opt[1].item())))

    def log(self, it, pad=28):
        """ppo.py:178-235: per-key 'Mean episode' lines over the episode infos of this update (non-finite
        values skipped, as _to_float / np.isfinite there), then the losses and the action noise."""
        self.tot_timesteps += self.num_transitions_per_env * self.num_envs
        ep_string = ""
        infos = [e[:2] for e in self.ep_infos]
        if infos:
            keys = infos[0][0]
            rows = []
            for ks, v in infos:
                v = v.cpu().numpy() if torch.is_tensor(v) else np.array(
                    [float(x.item()) if torch.is_tensor(x) else float(x) for x in v], np.float64)
                rows.append(dict(zip(ks, v.tolist())))
            for key in keys:
                vals = [r[key] for r in rows if key in r and np.isfinite(r[key])]
                if vals:
                    ep_string += f"{f'Mean episode {key}:':>{pad}} {float(np.mean(vals)):.4f}\n"
        self.last_episode_log = ep_string
        print(f"{'#' * 80}\n{ep_string}{'Value function loss:':>28} {self.mean_value_loss:.4f}\n"
              f"{'Surrogate loss:':>28} {self.mean_surrogate_loss:.4f}\n"
              f"{'Mean action noise std:':>28} {float(self.actor.distribution.std.mean()):.2f}")

    # ------------------------------------------------------ checkpoints
    def optimizer_state_dict(self):
        """torch.optim.Adam.state_dict() of [*actor.parameters(), *critic.parameters()] (ppo.py:59),
        with LambdaLR's initial_lr."""
        shapes = [s for _, s in self.actor.architecture.shapes()] + [(self.actor.distribution.dim,)] + \
                 [s for _, s in self.critic.architecture.shapes()]
        m, v = self.adam_m.detach().cpu(), self.adam_v.detach().cpu()
        step = float(self.opt[1].item())
        state, o = {}, 0
        for i, s in enumerate(shapes):
            n = int(np.prod(s))
            if step > 0:
                state[i] = {"step": torch.tensor(step), "exp_avg": m[o:o + n].reshape(s).clone(),
                            "exp_avg_sq": v[o:o + n].reshape(s).clone()}
            o += n
        group = {"lr": float(self.opt[0].item()), "betas": (0.9, 0.999), "eps": 1e-08, "weight_decay": 0,
                 "amsgrad": False, "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
                 "fused": None, "initial_lr": float(self.learning_rate), "params": list(range(len(shapes)))}
        return {"state": state, "param_groups": [group]}

    def load_optimizer_state_dict(self, osd):
        shapes = [s for _, s in self.actor.architecture.shapes()] + [(self.actor.distribution.dim,)] + \
                 [s for _, s in self.critic.architecture.shapes()]
        ms, vs, step, o = [], [], 0.0, 0
        for i, s in enumerate(shapes):
            n = int(np.prod(s))
            st = osd["state"].get(i)
            if st is None:
                ms.append(torch.zeros(n)); vs.append(torch.zeros(n))
            else:
                if tuple(st["exp_avg"].shape) != tuple(s):
                    raise RuntimeError(f"optimizer state {i}: shape {tuple(st['exp_avg'].shape)} vs {s}")
                ms.append(st["exp_avg"].float().reshape(-1)); vs.append(st["exp_avg_sq"].float().reshape(-1))
                step = float(st["step"])
        self.adam_m.copy_(torch.cat(ms).to(self.adam_m.device))
        self.adam_v.copy_(torch.cat(vs).to(self.adam_v.device))
        self.opt[1] = step
        self.opt[0] = float(osd["param_groups"][0]["lr"])
