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


# Ranks per device the peer exchange can train with: the waiting ranks' spinning reduction workgroups (8 KB of
# LDS each, up to one per CU per rank) must leave every CU the 146 KB a gradient workgroup of the last rank needs.
# Two ranks on one device fit (the one-GPU rehearsals); four stall until the exchange timeout.
PEER_MAX_RANKS_PER_DEVICE = 2


def device_identity(device) -> str:
    """Host + PCI location of this rank's GPU (the physical device, whatever HIP_VISIBLE_DEVICES maps it to);
    without a GPU (CPU tests) host + device string."""
    import socket
    host = socket.gethostname()
    try:
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(torch.device(device))
            return f"{host}/{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    except (RuntimeError, AssertionError, AttributeError):
        pass
    return f"{host}/{device}"


def shared_device_refusal(idents, limit: int = PEER_MAX_RANKS_PER_DEVICE):
    """None if no device holds more than `limit` ranks, else the refusal message naming the device and ranks."""
    by_dev = {}
    for r, d in enumerate(idents):
        by_dev.setdefault(d, []).append(r)
    worst = max(by_dev.items(), key=lambda kv: len(kv[1]))
    if len(worst[1]) <= limit:
        return None
    return (f"ranks {worst[1]} share device {worst[0]}: the peer exchange trains with at most {limit} ranks per "
            f"device (the waiting ranks' reduction workgroups would hold the LDS the last rank's gradient kernel "
            f"needs, a stall until the exchange timeout); use one process per GPU, or USV_DP_EXCHANGE=collective")


class PeerExchange:
    """The one-shot gradient all-reduce of ppo_minibatch_fused_dp (include/usv_hip.h ppo_dp_t): every rank
    allocates one receive buffer (ppo_dp_alloc), the 64-byte IPC handles go around once through the process
    group (all_gather_object: gloo or RCCL), every rank maps the others' buffers (ppo_dp_open, lazy peer
    access over xGMI), and from then on the per-minibatch exchange is a pair of stores and flags inside the
    reduction kernel -- no collective call, nothing the host launches between kernels, so the update is one
    HIP graph on every rank.  `peers` (tests) replaces the handle exchange by buffers of this process.

    Set-up is a fixed sequence of collectives that every rank runs whatever fails locally: a rank whose
    allocation failed still takes part in the handle exchange (with an empty handle), the ranks agree (MIN
    all-reduce) after the mapping and again after the start-up self-test, and on any failure every rank
    unmaps the peers' buffers, waits at a barrier (no peer can still write into or hold a mapping of its
    buffer) and only then frees its own -- then every rank raises RuntimeError, and A2CAgent falls back to
    torch.distributed collectives on all of them."""

    SELFTEST_ROUNDS = 4

    def __init__(self, rank: int, world_size: int, device, timeout_ms: int = 20000, peers=None,
                 selftest_ms: int = 5000):
        import ctypes
        from .. import _capi
        from .._abi import DEFINES, PpoDp
        if not 1 <= world_size <= DEFINES["PPO_DP_MAX"]:
            raise RuntimeError(f"PeerExchange: world size {world_size} > PPO_DP_MAX")
        self.selftest_bits = None
        if peers is None and world_size > 1:
            # forward progress needs few enough ranks per device (PEER_MAX_RANKS_PER_DEVICE): every rank sees the
            # same gathered identities, so every rank refuses together, before anything is allocated
            idents = [None] * world_size
            dist.all_gather_object(idents, device_identity(device))
            why = shared_device_refusal(idents)
            if why is not None and os.getenv("USV_DP_SHARED_DEVICE_SETUP") != "1":
                raise RuntimeError(f"PeerExchange: {why}")
            self.shared_device = why is not None
        lib = _capi.lib()
        self.rank, self.world, self.device = rank, world_size, device
        self._lib = lib
        self._own = ctypes.c_void_p()
        self._opened = []
        handle = ctypes.create_string_buffer(64)
        rc = lib.ppo_dp_alloc(ctypes.byref(self._own), handle)
        alloc_ok = rc == 0 and bool(self._own.value)
        if not alloc_ok:
            self._own = None
        ptrs = [None] * world_size
        if peers is not None:       # in-process "ranks" (tests): the other buffers are plain device pointers
            if not alloc_ok:
                raise RuntimeError(f"PeerExchange: ppo_dp_alloc failed (status {rc})")
            ptrs[rank] = self._own.value
            for r, p in enumerate(peers):
                if r != rank:
                    ptrs[r] = int(p)
        else:
            handles = [None] * world_size
            dist.all_gather_object(handles, bytes(handle.raw) if alloc_ok else b"")
            why = None
            if any(h is None or len(h) != 64 for h in handles):
                why = "a rank could not allocate its receive buffer (ppo_dp_alloc)"
            else:
                ptrs[rank] = self._own.value
                for r in range(world_size):
                    if r == rank:
                        continue
                    p = ctypes.c_void_p()
                    rc = lib.ppo_dp_open(ctypes.create_string_buffer(handles[r], 64), ctypes.byref(p))
                    if rc != 0:
                        why = f"cannot map rank {r}'s buffer (ppo_dp_open status {rc})"
                        break
                    self._opened.append(p.value)
                    ptrs[r] = p.value
            if not agree(why is None, device):
                self._fail(why or "another rank could not allocate or map a peer buffer")
        self.clock = torch.zeros(1, device=device, dtype=torch.int32)
        self.err = torch.zeros(1, device=device, dtype=torch.int32)
        d = PpoDp()
        d.rank, d.world, d.timeout_ms = rank, world_size, int(timeout_ms)
        for r, p in enumerate(ptrs):
            d.peer[r] = p
        d.clock, d.err = self.clock.data_ptr(), self.err.data_ptr()
        self.desc = d
        if peers is None and world_size > 1:
            self._selftest(selftest_ms)

    def _fail(self, why: str) -> None:
        """Every rank calls this together (after an agreement): unmap, barrier, free, raise."""
        for p in self._opened:
            self._lib.ppo_dp_close(ctypes_void(p))
        self._opened = []
        if dist.is_available() and dist.is_initialized():
            dist.barrier()          # every rank has unmapped our buffer and finished its kernels on it
        self.close()
        raise RuntimeError(f"PeerExchange: {why}")

    def _selftest(self, timeout_ms: int) -> None:
        """Every rank runs the same exchange kernel on a known payload (ppo_dp_selftest) right after the handles
        went around: a flag that never arrives (no peer access over xGMI) or a payload that arrives wrong or stale
        (a receive buffer whose remote writes the reader does not see) fails the test on some rank, the ranks
        agree on it before any training, and all of them fall back to collectives instead of a run that times out
        per minibatch."""
        import ctypes
        from .. import _capi
        bits = 4
        try:
            _capi.call("ppo_dp_selftest", ctypes.byref(self.desc), 1, self.SELFTEST_ROUNDS, int(timeout_ms),
                       _capi.stream_ptr())
            torch.cuda.synchronize()
            bits = int(self.err.item())
            self.clock.fill_(self.SELFTEST_ROUNDS)  # the flags hold the last test key: real keys continue after it
            self.err.zero_()
            torch.cuda.synchronize()
        except Exception:   # noqa: BLE001 -- a faulted kernel also fails the fills / sync: still reach agree()
            bits |= 4
        self.selftest_bits = bits
        if not agree(bits == 0, self.device):
            what = ("a flag did not arrive" if bits & 1 else "a payload arrived wrong or stale" if bits & 2
                    else "the test kernel failed to launch" if bits & 4 else "it failed on another rank")
            self._fail(f"start-up exchange test failed ({what}, err bits {bits})")

    @property
    def own_ptr(self) -> int:
        return self._own.value

    def check(self, err_host=None) -> None:
        """A peer's chunk missed the kernel's wall-clock bound (a lost or diverged rank): raise.  `err_host`: a
        pinned copy of `err` enqueued behind the update, read after the stream synchronisation."""
        if int(err_host[0] if err_host is not None else self.err.item()):
            raise RuntimeError("[ppo_dp] a peer's gradient chunk did not arrive within the timeout "
                               "(a rank died or the ranks' minibatch sequences diverged)")

    def release(self) -> None:
        """Collective teardown (every rank, kernels finished): unmap the peers' buffers, barrier, free our own."""
        for p in self._opened:
            self._lib.ppo_dp_close(ctypes_void(p))
        self._opened = []
        if dist.is_available() and dist.is_initialized():
            dist.barrier()
        self.close()

    def close(self) -> None:
        for p in self._opened:
            self._lib.ppo_dp_close(ctypes_void(p))
        self._opened = []
        if self._own is not None and self._own.value:
            self._lib.ppo_dp_free(self._own)
            self._own = None


def agree(ok: bool, device) -> bool:
    """True when `ok` holds on every rank (MIN all-reduce; gloo reduces on the host)."""
    if world() == 1:
        return bool(ok)
    flag = torch.tensor([1.0 if ok else 0.0], device="cpu" if dist.get_backend() == "gloo" else device)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item() == 1.0)


def ctypes_void(p):
    import ctypes
    return ctypes.c_void_p(p)
