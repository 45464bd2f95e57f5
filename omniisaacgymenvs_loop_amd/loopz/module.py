"""Parameter containers of the loopz actor / critic (omniisaacgymenvs/algo/ppo/module.py).

The networks are evaluated and trained by the HIP kernels of csrc/loopz.hip on one flat
parameter vector (optimizer order: actor net | std | critic net, include/usv_hip.h "loopz");
these classes keep the reference's construction arguments, initialisation and state_dict
key names so `full_<update>.pt` checkpoints are interchangeable with the reference's:
  * MLPEncode_wrap (module.py:184-395): `architecture.mass_encoder.{0,2,4}` (mass_dim -> 64 -> 16
    -> mass_latent_dim) and `architecture.action_mlp.{0,2,4}` (speed + task + latent -> shape ->
    output), weights orthogonal with gain sqrt(2) (init_weights :329-334), biases PyTorch's
    nn.Linear default, output layer x 1e-6 when small_init;
  * SquashedGaussianDiagonalCovariance (module.py:517-546): `std` (init_std), buffer `action_scale`.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np
import torch

from .. import _capi

MASS, LAT, NH = 8, 8, 128
ENC = (64, 16)


def _linear_init(out_f: int, in_f: int, gain: float, gen: torch.Generator):
    w = torch.empty(out_f, in_f)
    torch.nn.init.orthogonal_(w, gain=gain, generator=gen)
    bound = 1.0 / math.sqrt(in_f)   # nn.Linear.reset_parameters' bias init (never re-initialised)
    b = torch.empty(out_f).uniform_(-bound, bound, generator=gen)
    return w, b


class MLPEncode_wrap:
    """MLPEncode_wrap(shape, actionvation_fn, input_size, output_size, output_activation_fn,
    small_init, speed_dim, mass_dim, mass_latent_dim, mass_encoder_shape) -- module.py:363-395.
    The kernels implement shape [128, 128], LeakyReLU, mass_dim = mass_latent_dim = 8,
    mass_encoder_shape (64, 16) and input_size 33..36 (checked here)."""

    def __init__(self, shape, actionvation_fn, input_size, output_size, output_activation_fn=None,
                 small_init=False, speed_dim=3, mass_dim=4, mass_latent_dim=8, mass_encoder_shape=(64, 16),
                 seed: int = 0):
        shape = [int(s) for s in shape]
        if shape != [NH, NH] or int(mass_dim) != MASS or int(mass_latent_dim) != LAT or \
                tuple(int(v) for v in mass_encoder_shape) != ENC:
            raise NotImplementedError("the loopz kernels implement policy/value nets [128, 128], mass_dim 8, "
                                      "mass_latent_dim 8, mass_encoder_shape (64, 16) (the IROS2024 cfg.yaml)")
        if not 33 <= int(input_size) <= 36:
            raise NotImplementedError(f"loopz kernels take 33..36 observations, got {input_size}")
        name = getattr(actionvation_fn, "__name__", str(actionvation_fn))
        if "LeakyReLU" not in name:
            raise NotImplementedError(f"loopz kernels implement LeakyReLU hidden layers, got {name}")
        self.speed_dim, self.mass_dim, self.obs_dim = int(speed_dim), MASS, int(input_size)
        self.task_dim = self.obs_dim - self.speed_dim - self.mass_dim
        if self.task_dim <= 0:
            raise ValueError(f"Invalid obs split: input_size={input_size}, speed_dim={speed_dim}, mass_dim={mass_dim}")
        self.output_size = int(output_size)
        self.out_tanh = output_activation_fn is not None
        oname = getattr(output_activation_fn, "__name__", "") if output_activation_fn is not None else ""
        if self.out_tanh and "Tanh" not in oname:
            raise NotImplementedError(f"output activation {oname}: the kernels implement tanh or none")
        self.input_shape = [int(input_size)]
        self.output_shape = [int(output_size)]
        gen = torch.Generator().manual_seed(int(seed))
        g = math.sqrt(2)
        sd: Dict[str, torch.Tensor] = {}
        # module registration order: mass_encoder first (:276), then action_mlp (:313)
        ins = [MASS, ENC[0], ENC[1]]
        outs = [ENC[0], ENC[1], LAT]
        for li, (i_, o_) in enumerate(zip(ins, outs)):
            w, b = _linear_init(o_, i_, g, gen)
            sd[f"architecture.mass_encoder.{2 * li}.weight"], sd[f"architecture.mass_encoder.{2 * li}.bias"] = w, b
        main_in = self.speed_dim + self.task_dim + LAT
        for li, (i_, o_) in enumerate(zip([main_in, NH, NH], [NH, NH, self.output_size])):
            w, b = _linear_init(o_, i_, g, gen)
            if li == 2 and small_init:
                w = w * 1e-6
            sd[f"architecture.action_mlp.{2 * li}.weight"], sd[f"architecture.action_mlp.{2 * li}.bias"] = w, b
        self._sd = sd
        self._bound = None   # (flat device vector, offset) once a PPO owns the parameters

    # ------------------------------------------------------------ state dict
    KEYS = [f"architecture.mass_encoder.{i}.{p}" for i in (0, 2, 4) for p in ("weight", "bias")] + \
           [f"architecture.action_mlp.{i}.{p}" for i in (0, 2, 4) for p in ("weight", "bias")]

    def shapes(self) -> List:
        return [(k, tuple(self._sd[k].shape)) for k in self.KEYS]

    def numel(self) -> int:
        return sum(int(np.prod(s)) for _, s in self.shapes())

    def flat(self) -> torch.Tensor:
        return torch.cat([self._sd[k].reshape(-1) for k in self.KEYS])

    def bind(self, flat: torch.Tensor, offset: int) -> None:
        self._bound = (flat, int(offset))

    def state_dict(self) -> Dict[str, torch.Tensor]:
        if self._bound is None:
            return {k: v.clone() for k, v in self._sd.items()}
        flat, o = self._bound
        host = flat[o:o + self.numel()].detach().cpu()
        out, p = {}, 0
        for k, s in self.shapes():
            n = int(np.prod(s))
            out[k] = host[p:p + n].reshape(s).clone()
            p += n
        return out

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for k, s in self.shapes():
            if tuple(sd[k].shape) != s:
                raise RuntimeError(f"size mismatch for {k}: {tuple(sd[k].shape)} vs {s}")
        self._sd = {k: sd[k].detach().float().cpu().clone() for k in self.KEYS}
        if self._bound is not None:
            flat, o = self._bound
            flat[o:o + self.numel()].copy_(self.flat().to(flat.device))

    def parameters(self):
        return [self._sd[k] for k in self.KEYS]


class SquashedGaussianDiagonalCovariance:
    """module.py:517-546: trainable std (no positivity constraint), buffer action_scale."""

    def __init__(self, dim, init_std, action_scale=1.0, eps: float = 1e-6):
        self.dim = int(dim)
        self.eps = float(eps)
        self._std = float(init_std) * torch.ones(self.dim)
        scale = torch.as_tensor(action_scale, dtype=torch.float32).reshape(-1)
        if scale.numel() == 1:
            scale = scale.repeat(self.dim)
        if scale.numel() != self.dim:
            raise ValueError(f"action_scale must be scalar or shape ({self.dim},), got {tuple(scale.shape)}")
        self.action_scale = scale
        self._bound = None

    def bind(self, flat: torch.Tensor, offset: int) -> None:
        self._bound = (flat, int(offset))

    @property
    def std(self) -> torch.Tensor:
        if self._bound is None:
            return self._std
        flat, o = self._bound
        return flat[o:o + self.dim]

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {"std": self.std.detach().cpu().clone(), "action_scale": self.action_scale.clone()}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        self._std = sd["std"].detach().float().cpu().clone()
        if "action_scale" in sd:
            self.action_scale = sd["action_scale"].detach().float().cpu().clone()
        if self._bound is not None:
            flat, o = self._bound
            flat[o:o + self.dim].copy_(self._std.to(flat.device))

    def enforce_minimum_std(self, min_std) -> None:
        """module.py:649-659 (on the device, csrc/loopz.hip k_lz_min_std, when bound)."""
        if self._bound is None:
            s = torch.where(torch.isfinite(self._std), self._std, torch.as_tensor(min_std).float())
            self._std = torch.maximum(s, torch.as_tensor(min_std).float())
            return
        flat, o = self._bound
        s = flat[o:o + self.dim]
        m = torch.as_tensor(min_std, dtype=torch.float32, device=flat.device).expand(self.dim)
        s.copy_(torch.maximum(torch.where(torch.isfinite(s), s, m), m))


class Actor:
    """module.py:54-96."""

    def __init__(self, architecture: MLPEncode_wrap, distribution: SquashedGaussianDiagonalCovariance, device="cpu"):
        # the actor kernels (lz_act, lz_minibatch: loopz.hip k_lz_forward / k_lz_grad) always take tanh of the
        # mean head, i.e. MLPEncode_wrap(..., output_activation_fn=nn.Tanh); an actor without it would be
        # sampled and trained as if it had one
        if not architecture.out_tanh:
            raise NotImplementedError("loopz actor: the kernels implement a Tanh output activation only "
                                      "(architecture.activation: tanh)")
        self.architecture = architecture
        self.distribution = distribution
        self.device = device

    @property
    def obs_shape(self):
        return self.architecture.input_shape

    @property
    def action_shape(self):
        return self.architecture.output_shape

    def parameters(self):
        return [*self.architecture.parameters(), self.distribution.std]


class Critic:
    """module.py:98-115."""

    def __init__(self, architecture: MLPEncode_wrap, device="cpu"):
        if architecture.out_tanh:   # the critic kernels emit the linear value head
            raise NotImplementedError("loopz critic: the kernels implement a linear value head (no output activation)")
        self.architecture = architecture
        self.device = device

    @property
    def obs_shape(self):
        return self.architecture.input_shape

    def parameters(self):
        return list(self.architecture.parameters())


def check_lib_layout(actor: Actor, critic: Critic) -> int:
    """The flat layout of the kernels == actor net | std | critic net (include/usv_hip.h)."""
    n = actor.architecture.numel() + actor.distribution.dim + critic.architecture.numel()
    want = int(_capi.lib().lz_nparam(actor.architecture.obs_dim))
    if n != want:
        raise RuntimeError(f"loopz parameter layout mismatch: {n} host vs {want} kernels")
    return n
