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


def test_layout_key_covers_every_define_enum_and_struct_of_the_header():
    """usv_hip_layout_key folds EVERY object-like #define of include/usv_hip.h (slab rows, field / PPO / ctl
    constants, ...), every enumerator and sizeof / offsetof of every field of every ABI struct: a library built
    from another header -- e.g. a moved USV_SLAB_* row, the stale library behind round 3's status-800 fault --
    is refused before its first call.  The compiled list (csrc/usv_layout_gen.h) is the header's, current."""
    from omniisaacgymenvs_loop_amd import _abi
    src = re.sub(r"/\*.*?\*/", " ", open(HEADER).read(), flags=re.S)
    defines = set(re.findall(r"^\s*#define\s+(\w+)", src, flags=re.M)) - set(_abi.GUARD_DEFINES)
    names = {name for _, name, _ in _abi.layout_entries()}
    assert defines <= names, f"defines outside the layout key: {sorted(defines - names)}"
    assert {n for n in defines if n.startswith("USV_SLAB_")} and all(
        n in names for n in defines if n.startswith(("USV_SLAB_", "USV_FIELD_", "PPO_", "USV_CTL_", "USV_N")))
    structs = set(re.findall(r"typedef\s+struct\s+(\w+)\s*\{", src))
    assert structs == set(_abi.LAYOUT_STRUCTS), structs ^ set(_abi.LAYOUT_STRUCTS)
    for s in structs:
        cls = _abi._STRUCT_CLASSES[s]
        assert f"sizeof {s}" in names and all(f"{s}.{f}" in names for f, _ in cls._fields_)
    enums = set(re.findall(r"enum\s+(\w+)\s*\{", src))
    assert enums == set(_abi.LAYOUT_ENUMS)
    for e in enums:
        assert set(_abi.enum_values(e)) <= names
    with open(_abi.LAYOUT_GEN) as f:
        assert f.read() == _abi.layout_header_text(), "csrc/usv_layout_gen.h is stale: run _capi.build()"


def test_layout_key_changes_with_any_entry():
    """Moving one slab row, resizing one struct or renaming one define changes the key."""
    from omniisaacgymenvs_loop_amd import _abi
    ent = _abi.layout_entries()
    k0 = _abi.layout_key_of(ent)
    i_slab = next(i for i, e in enumerate(ent) if e[1] == "USV_SLAB_STATS")
    i_size = next(i for i, e in enumerate(ent) if e[1] == "sizeof usv_cfg")
    for i, (expr, name, v) in ((i_slab, (ent[i_slab][0], ent[i_slab][1], ent[i_slab][2] + 1)),
                               (i_size, (ent[i_size][0], ent[i_size][1], ent[i_size][2] + 4)),
                               (0, (ent[0][0], ent[0][1] + "_X", ent[0][2]))):
        mod = list(ent)
        mod[i] = (expr, name, v)
        assert _abi.layout_key_of(mod) != k0


def test_stale_root_needs_its_rows():
    """cfg.stale_root (on by default) without usv_bufs_t.stale: usv_reset and usv_env_step
    refuse the call with status 1 before touching the device (argument checks only: no GPU here)."""
    from omniisaacgymenvs_loop_amd import _capi
    from omniisaacgymenvs_loop_amd._abi import UsvBufs
    from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libusv_hip.so not built (run __graft_entry__.build())")
    cfg = build_usv_cfg(load_yaml(os.path.join(ROOT, "omniisaacgymenvs_loop_amd", "cfg", "task", "USV", "IROS2024",
                                               "USV_Virtual_CaptureXY_SysID-TEST.yaml")))
    assert cfg.stale_root == 1
    b = UsvBufs()
    b.n = 64
    dummy = ctypes.create_string_buffer(64)
    lib = _capi.lib()
    assert lib.usv_reset(_capi.byref(cfg), _capi.byref(b), 0, 0, None, None) == 1
    assert lib.usv_env_step(_capi.byref(cfg), _capi.byref(b), ctypes.addressof(dummy), ctypes.addressof(dummy),
                            ctypes.c_float(0.0), 0, 0, None, None) == 1


def test_partials_layout_for_every_minibatch_and_refused_sizes():
    """ppo_partials_floats covers any positive multiple of 32 rows (the reference yaml's horizon x num_envs minibatch,
    e.g. 65,536 or loopz-sized 76,800 rows, included): the fold control words follow the larger of the chunk-major
    rows (RED_BLOCKS x 128 floats per 32-row block) and the row-major rows + group rows.  Sizes without a layout
    are refused by the minibatch entry points with status 2 before any device work (argument checks only)."""
    from omniisaacgymenvs_loop_amd import _capi
    from omniisaacgymenvs_loop_amd._abi import DEFINES, PpoCfg
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("libusv_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(_capi.LIB_PATH)
    red_blocks = (DEFINES["PPO_NPARAM"] + 5 + 127) // 128
    prev = 0
    for mb in (32, 8192, 48576, 48608, 65536, 76800, 262144):
        f = lib.ppo_partials_floats(mb)
        assert f >= (mb // 32) * red_blocks * 128 + 8 * 64 and f > prev, (mb, f)
        prev = f
    for mb in (0, 16, 8200, 2 ** 31 - 32):
        assert lib.ppo_partials_floats(mb) <= 0, mb
    cfg = PpoCfg()
    buf = ctypes.create_string_buffer(1 << 12)
    p = ctypes.addressof(buf) + (-ctypes.addressof(buf) % 16)   # 16-byte aligned host scratch: never dereferenced
    for mb in (8200, 2 ** 31 - 32):
        cfg.minibatch = mb
        args = [_capi.byref(cfg), p, p, p, 0, 0] + [p] * 9 + [None, p, p, None]   # .., grad, losses, partials, work, stream
        assert _capi.lib().ppo_minibatch_grad(*args) == 2, mb
