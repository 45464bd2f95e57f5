"""ctypes binding of libusv_hip.so (include/usv_hip.h) -- the product path.

This module is exactly the FFI a reference maintainer would add:
every entry point takes raw device pointers, sizes and a hipStream_t.  It fails
loudly when the library is missing: there is no CPU fallback anywhere in the
product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  -- load torch's HIP runtime first; the .so binds to it (same SONAME)

from ._abi import PpoCfg, UsvBufs, UsvCfg

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libusv_hip.so")
# instrumented build (per-workgroup phase timestamps, tools/phase_probe.py); selected with USV_HIP_PROBE=1
PROBE_LIB_PATH = os.path.join(LIB_DIR, "libusv_hip_probe.so")
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("usv_env.hip", "usv_field.hip", "ppo.hip", "loopz.hip")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", "usv_device.h"), os.path.join(HERE, "csrc", "usv_layout_gen.h"),
                  os.path.join(ROOT, "include", "usv_hip.h")]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17",
               # no implicit FMA contraction: the arithmetic follows the reference op by op
               "-ffp-contract=off"]

_lib = None


def build(force: bool = False, verbose: bool = False, probe: bool = False) -> str:
    """Compile the HIP kernels for gfx950 into lib/libusv_hip.so (in-tree)."""
    os.makedirs(LIB_DIR, exist_ok=True)
    from ._abi import gen_layout_header
    gen_layout_header()   # csrc/usv_layout_gen.h follows the header (rewritten only when its text changes)
    out = PROBE_LIB_PATH if probe else LIB_PATH
    if not force and os.path.exists(out):
        lib_m = os.path.getmtime(out)
        if all(os.path.getmtime(d) <= lib_m for d in DEPS):
            return out
    cmd = ["hipcc"] + HIPCC_FLAGS + (["-DUSV_PHASE_PROBE"] if probe else []) + ["-o", out] + SOURCES
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return out


def _declare(lib):
    P, I, U64, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_float
    sig = {
        "usv_build_lut": [P, P, I, P, P],
        "usv_reset": [P, P, U64, U64, P, P],
        "usv_reset_part": [P, P, U64, U64, P, I, P],
        "usv_potential_field": [P, P, P],
        "usv_field_stage": [P, P, I, P],
        "usv_field_view": [P, P, P, I, P, P],
        "usv_env_step_late": [P, P, P],
        "usv_env_step": [P, P, P, P, F, U64, U64, P, P],
        "usv_env_step_part": [P, P, P, P, F, U64, U64, P, I, P],
        "usv_forces": [P, P, P, P],
        "usv_hydrostatics": [P, I, P, P, P, P, P, P],
        "lz_act": [P, P, P, I, P, P, P, P, P, U64, U64, P, P],
        "lz_value": [P, P, P, P, P],
        "lz_store": [P, P, P, I, P, P, P],
        "lz_returns": [P, P, P, P, P, P, P, P, P],
        "lz_minibatch": [P, P, P, P, P, I, I, P, P, P, P, P, P, P, P, P],
        "lz_minibatch_rows": [P, P, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P],
        "lz_enforce_min_std": [P, P, P],
        "ppo_policy_step": [P, P, P, P, P, I, P, P, P, P, P, P, P, P, P, U64, U64, P, P, P],
        "ppo_value": [P, P, P, P, P, P, P],
        "ppo_store_reward": [P, P, P, I, P, P, P, P, P, P, P],
        "ppo_prepare": [P, P, P, P, P, P, P, P, P, P, P, P, P],
        "ppo_minibatch_grad": [P, P, P, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P],
        "ppo_minibatch_apply": [P, P, P, P, P, P, I, F, P, I, P],
        "ppo_minibatch_fused": [P, P, I, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
        "ppo_minibatch_finish": [P, P, I, P, P, P],
        "ppo_minibatch_coll": [P, P, I, F, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
        "ppo_minibatch_coll_finish": [P, P, I, P, F, P, P],
        "ppo_minibatch_fused_dp": [P, P, P, I, P, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
        "ppo_dp_alloc": [P, P],
        "ppo_dp_open": [P, P],
        "ppo_dp_close": [P],
        "ppo_dp_free": [P],
        "ppo_dp_selftest": [P, ctypes.c_uint, I, I, P],
        "ppo_partials_floats": [I],
        "ppo_grad_floats": [],
        "ppo_obs_rms_epoch": [P, P, I, P, P, P],
        "ppo_rms_seq_doubles": [P, I],
        "lz_nparam": [I],
        "lz_grad_floats": [I],
        "lz_partials_floats": [P],
        "ppo_meter_floats": [I, I],
        "usv_hip_version": [],
        "usv_hip_layout_key": [],   # (restype long long, below)
    }
    for name, args in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    lib.ppo_dp_buffer_bytes.argtypes = []
    lib.ppo_dp_buffer_bytes.restype = ctypes.c_longlong
    lib.usv_hip_layout_key.argtypes = []
    lib.usv_hip_layout_key.restype = ctypes.c_longlong
    return lib


def layout_key() -> int:
    """usv_hip_layout_key() as this binding's parse of include/usv_hip.h gives it: every integer #define,
    every enumerator, sizeof / offsetof of every ABI struct field (_abi.layout_entries)."""
    from ._abi import layout_entries, layout_key_of
    return layout_key_of(layout_entries())


def lib():
    global _lib
    if _lib is None:
        path = PROBE_LIB_PATH if os.getenv("USV_HIP_PROBE") == "1" else LIB_PATH
        # A/B builds of the same ABI (tools/gpu_ab.sh): lib/<name>.so inside the tree only
        alt = os.getenv("USV_HIP_LIB")
        if alt:
            path = os.path.join(LIB_DIR, os.path.basename(alt))
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; "
                               f"g.build()'` (hipcc --offload-arch=gfx950)")
        loaded = _declare(ctypes.CDLL(path))
        if loaded.usv_hip_layout_key() != layout_key():
            raise RuntimeError(f"{path} was built from another buffer layout than include/usv_hip.h "
                               "(usv_hip_layout_key mismatch): rebuild it")
        _lib = loaded
    return _lib


def call(name: str, *args) -> None:
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def call_rc(name: str, *args) -> int:
    """Like call() but hands the status back (for entry points with a documented fallback code)."""
    return int(getattr(lib(), name)(*args))


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def byref(s):
    return ctypes.byref(s)


__all__ = ["build", "lib", "call", "call_rc", "ptr", "stream_ptr", "byref", "UsvCfg", "UsvBufs", "PpoCfg", "LIB_PATH"]
