"""rl_games checkpoint layout (a2c_common.py:590-621, torch_ext.py:54-84).

{'model': state_dict, 'epoch', 'optimizer', 'frame', 'last_mean_rewards',
 'env_state'} with the ModelA2CContinuousLogStd state_dict keys; the flat
device parameter vector maps onto them in model.parameters() order.
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Any, Dict

import numpy as np
import torch

from .._abi import DEFINES

NIN, NH, NA = DEFINES["PPO_NIN"], DEFINES["PPO_NH"], DEFINES["PPO_NA"]
# (state_dict key, shape) in model.parameters() order (network_builder.py:1480-1575)
PARAM_LAYOUT = [
    ("a2c_network.sigma", (NA,)),
    ("a2c_network.actor_mlp.0.weight", (NH, NIN)),
    ("a2c_network.actor_mlp.0.bias", (NH,)),
    ("a2c_network.actor_mlp.2.weight", (NH, NH)),
    ("a2c_network.actor_mlp.2.bias", (NH,)),
    ("a2c_network.value.weight", (1, NH)),
    ("a2c_network.value.bias", (1,)),
    ("a2c_network.mu.weight", (NA, NH)),
    ("a2c_network.mu.bias", (NA,)),
]
NPARAM = sum(int(np.prod(s)) for _, s in PARAM_LAYOUT)
assert NPARAM == DEFINES["PPO_NPARAM"]


W1_KEY = "a2c_network.actor_mlp.0.weight"


def split_flat(flat: torch.Tensor, obs_dim: int = NIN) -> Dict[str, torch.Tensor]:
    """Flat parameter vector -> state_dict tensors; obs_dim < NIN drops W1's zero padding columns
    (the reference's network of a priv_dim = 4 task has obs_dim = 29 inputs)."""
    out, o = OrderedDict(), 0
    for k, s in PARAM_LAYOUT:
        m = int(np.prod(s))
        out[k] = flat[o:o + m].view(*s)
        if k == W1_KEY:
            out[k] = out[k][:, :obs_dim]
        o += m
    return out


def _pad_w1(t: torch.Tensor) -> torch.Tensor:
    """[NH, k] -> [NH, NIN] with zero columns (k <= NIN)."""
    if t.shape[1] == NIN:
        return t
    return torch.cat([t, torch.zeros(t.shape[0], NIN - t.shape[1], dtype=t.dtype)], 1)


def model_state_dict(params: torch.Tensor, obs_rms: torch.Tensor, val_rms: torch.Tensor,
                     obs_dim: int = NIN) -> "OrderedDict":
    """ModelA2CContinuousLogStd.state_dict() key order: value_mean_std, running_mean_std, a2c_network."""
    sd = OrderedDict()
    v = val_rms.detach().cpu()
    o = obs_rms.detach().cpu()
    sd["value_mean_std.running_mean"] = v[0:1].clone()
    sd["value_mean_std.running_var"] = v[1:2].clone()
    sd["value_mean_std.count"] = v[2].clone()
    sd["running_mean_std.running_mean_std.state.running_mean"] = o[0:obs_dim].clone()
    sd["running_mean_std.running_mean_std.state.running_var"] = o[NIN:NIN + obs_dim].clone()
    sd["running_mean_std.running_mean_std.state.count"] = o[2 * NIN].clone()
    for k, t in split_flat(params.detach().cpu(), obs_dim).items():
        sd[k] = t.clone()
    return sd


def load_model_state_dict(sd: Dict[str, torch.Tensor], params: torch.Tensor, obs_rms: torch.Tensor,
                          val_rms: torch.Tensor, obs_dim: int = NIN) -> None:
    for k, s in PARAM_LAYOUT:
        want = (NH, obs_dim) if k == W1_KEY else tuple(s)
        if tuple(sd[k].shape) != want:
            raise ValueError(f"checkpoint tensor {k} has shape {tuple(sd[k].shape)}, expected {want}")
    flat = torch.cat([(_pad_w1(sd[k].float()) if k == W1_KEY else sd[k]).reshape(-1).to(torch.float32)
                      for k, _ in PARAM_LAYOUT])
    params.copy_(flat.to(params.device))
    o = obs_rms.detach().cpu().clone()
    o[0:obs_dim] = sd["running_mean_std.running_mean_std.state.running_mean"].double()
    o[NIN:NIN + obs_dim] = sd["running_mean_std.running_mean_std.state.running_var"].double()
    o[2 * NIN] = sd["running_mean_std.running_mean_std.state.count"].double().reshape(())
    obs_rms.copy_(o.to(obs_rms.device))
    v = torch.cat([sd["value_mean_std.running_mean"].double(), sd["value_mean_std.running_var"].double(),
                   sd["value_mean_std.count"].double().reshape(1)])
    val_rms[:3].copy_(v.to(val_rms.device))


def optimizer_state_dict(adam_m: torch.Tensor, adam_v: torch.Tensor, step: float, lr: float,
                         weight_decay: float = 0.0, obs_dim: int = NIN) -> Dict[str, Any]:
    """torch.optim.Adam.state_dict() layout (one param group, params 0..8)."""
    m = split_flat(adam_m.detach().cpu(), obs_dim)
    v = split_flat(adam_v.detach().cpu(), obs_dim)
    state = {}
    for i, (k, _) in enumerate(PARAM_LAYOUT):
        state[i] = {"step": torch.tensor(float(step)), "exp_avg": m[k].clone(), "exp_avg_sq": v[k].clone()}
    group = {"lr": float(lr), "betas": (0.9, 0.999), "eps": 1e-08, "weight_decay": float(weight_decay),
             "amsgrad": False, "maximize": False, "foreach": None, "capturable": False, "differentiable": False,
             "fused": None, "params": list(range(len(PARAM_LAYOUT)))}
    return {"state": state, "param_groups": [group]}


def load_optimizer_state_dict(osd: Dict[str, Any], adam_m: torch.Tensor, adam_v: torch.Tensor, obs_dim: int = NIN):
    ms, vs, step = [], [], 0.0
    for i, (k, s) in enumerate(PARAM_LAYOUT):
        st = osd["state"].get(i)
        if st is None:
            ms.append(torch.zeros(int(np.prod(s))))
            vs.append(torch.zeros(int(np.prod(s))))
            continue
        fix = (lambda t: _pad_w1(t.reshape(NH, obs_dim))) if k == W1_KEY else (lambda t: t)
        ms.append(fix(st["exp_avg"].float()).reshape(-1))
        vs.append(fix(st["exp_avg_sq"].float()).reshape(-1))
        step = float(st["step"])
    adam_m.copy_(torch.cat(ms).to(adam_m.device))
    adam_v.copy_(torch.cat(vs).to(adam_v.device))
    return step, float(osd["param_groups"][0]["lr"])


def grad_scaler_state(steps: float) -> Dict[str, Any]:
    """torch.cuda.amp.GradScaler().state_dict() as the reference's mixed_precision run leaves it after `steps`
    optimizer steps with finite gradients (a2c_common.py:243, 326-330, 631): init scale 2**16, doubled every
    2000 consecutive finite steps.  The bf16 GEMM mode needs no loss scaling (bf16 keeps fp32's exponent range)
    and its non-finite guard is the NaN probe, so the entry is bookkeeping for checkpoint compatibility.
    The growth is capped at GRAD_SCALE_MAX: a real fp16 run backs off long before (scaled fp16 gradients overflow),
    and an uncapped power would leave the fp32 range after ~224k steps (a reference GradScaler loading it would
    hold an inf scale and skip every step) and raise OverflowError past ~2M steps."""
    steps = max(int(steps), 0)
    doublings = min(steps // 2000, GRAD_SCALE_MAX_DOUBLINGS)
    return {"scale": 65536.0 * 2.0 ** doublings, "growth_factor": 2.0, "backoff_factor": 0.5,
            "growth_interval": 2000, "_growth_tracker": steps % 2000}


GRAD_SCALE_MAX_DOUBLINGS = 8        # 2**16 init -> at most 2**24
GRAD_SCALE_MAX = 65536.0 * 2.0 ** GRAD_SCALE_MAX_DOUBLINGS


def safe_filesystem_op(func, *args, **kwargs):
    """torch_ext.safe_filesystem_op: 5 attempts with exponential back-off (torch_ext.py:54-69)."""
    for attempt in range(5):
        try:
            return func(*args, **kwargs)
        except Exception as exc:  # noqa: BLE001 -- mirror the reference's retry-on-anything
            print(f"Exception {exc} when trying to execute {func}; retrying in {2 ** attempt}s")
            time.sleep(2 ** attempt)
    raise RuntimeError(f"Could not execute {func}, give up after 5 attempts...")


def save_checkpoint(filename: str, state: Dict[str, Any]) -> None:
    print(f"=> saving checkpoint '{filename}.pth'")
    d = os.path.dirname(filename)
    if d:
        os.makedirs(d, exist_ok=True)
    safe_filesystem_op(torch.save, state, filename + ".pth")


def _allow_numpy_globals():
    import codecs
    allow = [np.dtype, codecs.encode]
    try:   # numpy 2 writes numpy._core.multiarray.scalar, numpy 1 wrote numpy.core.multiarray.scalar
        allow.append(np._core.multiarray.scalar)
        allow.append((np._core.multiarray.scalar, "numpy.core.multiarray.scalar"))
    except AttributeError:  # numpy < 2
        allow.append(np.core.multiarray.scalar)
    for name in ("Float64DType", "Float32DType", "Int64DType"):
        if hasattr(np, "dtypes") and hasattr(np.dtypes, name):
            allow.append(getattr(np.dtypes, name))
    torch.serialization.add_safe_globals(allow)


def load_checkpoint(filename: str) -> Dict[str, Any]:
    """Loads with weights_only=True (never unpickles arbitrary objects)."""
    print(f"=> loading checkpoint '{filename}'")
    _allow_numpy_globals()
    return safe_filesystem_op(torch.load, filename, map_location="cpu", weights_only=True)
