"""The C-ABI library loads on a GPU-less host and exports every entry point
include/usv_hip.h declares (no compute calls: there is no device here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "usv_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void)\s+(\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("usv_reset", "usv_potential_field", "usv_env_step", "ppo_policy_step", "ppo_prepare",
                 "ppo_minibatch_grad", "ppo_minibatch_apply"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from omniisaacgymenvs_loop_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libusv_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_capi.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"missing exports: {missing}"
    assert lib.usv_hip_version() >= 1
    assert lib.ppo_partials_floats(8192) > 0


def test_ctypes_signatures_cover_the_header():
    from omniisaacgymenvs_loop_amd import _capi
    src = open(os.path.join(ROOT, "omniisaacgymenvs_loop_amd", "_capi.py")).read()
    for n in declared_functions():
        assert f'"{n}"' in src, f"{n} has no ctypes signature in _capi.py"


def test_library_layout_key_matches_the_header():
    """The library's compiled buffer-layout constants equal the ones the binding allocates with (a library
    built from another layout is refused by _capi.lib() before any call)."""
    from omniisaacgymenvs_loop_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libusv_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_capi.LIB_PATH)
    lib.usv_hip_layout_key.restype = ctypes.c_longlong
    assert lib.usv_hip_layout_key() == _capi.layout_key()
