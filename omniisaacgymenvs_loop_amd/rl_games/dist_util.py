"""Data-parallel plumbing of the PPO update (one process per GPU, RCCL over xGMI).

Mirrors the multi-GPU branches of rl_games A2CBase (a2c_common.py:87-101,
308-323, 1218-1230, 1354): the initial weights come from rank 0; every
minibatch the flat gradient is all-reduced (SUM) and divided by the world size,
with the minibatch KL riding in the same buffer (one collective instead of
two); the learning rate then follows identically on every rank from the
all-reduced KL, so no LR broadcast is needed.  The same functions run on gloo
(CPU tensors) in the tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def local_device() -> str:
    """The GPU of this rank: cuda:LOCAL_RANK (one process per GPU).  USV_RANKS_SHARE_DEVICE=<i>
    puts every rank on cuda:<i> -- only for rehearsing the multi-process path on a one-GPU box."""
    shared = os.getenv("USV_RANKS_SHARE_DEVICE")
    return f"cuda:{int(shared)}" if shared is not None else f"cuda:{int(os.getenv('LOCAL_RANK', '0'))}"


def backend() -> str:
    """RCCL ("nccl") unless USV_DIST_BACKEND overrides it (gloo for the shared-device rehearsal)."""
    return os.getenv("USV_DIST_BACKEND", "nccl")


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def broadcast_params(flat: torch.Tensor, src: int = 0) -> None:
    """Initial parameter broadcast (a2c_common.py:1354)."""
    if world() > 1:
        dist.broadcast(flat, src)


def allreduce_grad(buf: torch.Tensor) -> float:
    """SUM all-reduce of [grad..., kl] in place; returns the scale (1/world) the
    Adam kernel applies (trancate_gradients_and_step, a2c_common.py:309-323)."""
    w = world()
    if w == 1:
        return 1.0
    dist.all_reduce(buf, op=dist.ReduceOp.SUM)
    return 1.0 / w


def max_over_ranks(x: float, device) -> float:
    """Largest value over ranks (bench timing: the slowest rank defines the step)."""
    if world() == 1:
        return float(x)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
