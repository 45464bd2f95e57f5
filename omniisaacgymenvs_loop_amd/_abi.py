"""ctypes mirror of the POD structs declared in include/usv_hip.h.

The structs are parsed from the header itself at import time, so the Python
side can never drift from the C ABI (field order, array sizes, pointer
slots).  Used by the product binding (_capi.py) and by the test harness.
"""
from __future__ import annotations

import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(os.path.dirname(_HERE), "include", "usv_hip.h")

_CTYPES = {
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "int": ctypes.c_int,
    "int32_t": ctypes.c_int32,
    "int64_t": ctypes.c_int64,
    "uint8_t": ctypes.c_uint8,
    "uint64_t": ctypes.c_uint64,
}


def _read_header() -> str:
    with open(HEADER, "r", encoding="utf-8") as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", " ", txt, flags=re.S)
    return txt


def _defines(txt: str) -> dict:
    out = {}
    for m in re.finditer(r"#define\s+(\w+)\s+(.+)", txt):
        name, val = m.group(1), m.group(2).strip()
        try:
            out[name] = int(eval(val, {}, dict(out)))  # simple integer expressions only
        except Exception:
            pass
    return out


def _struct_fields(txt: str, name: str, defines: dict):
    m = re.search(r"typedef\s+struct\s+%s\s*\{(.*?)\}\s*%s_t\s*;" % (name, name), txt, flags=re.S)
    if m is None:
        raise RuntimeError(f"struct {name} not found in {HEADER}")
    body = m.group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl.startswith("const "):
            decl = decl[len("const "):]
        if not decl:
            continue
        tm = re.match(r"(\w+)\s+(.*)", decl, flags=re.S)
        base, rest = tm.group(1), tm.group(2)
        for item in rest.split(","):
            item = item.strip()
            ptr = item.startswith("*")
            item = item.lstrip("*").strip()
            am = re.match(r"(\w+)\s*(?:\[(.+)\])?", item)
            fname, arr = am.group(1), am.group(2)
            if ptr:
                ct = ctypes.c_void_p
            else:
                ct = _CTYPES[base]
            if arr is not None:
                ct = ct * int(eval(arr, {}, defines))
            fields.append((fname, ct))
    return fields


_TXT = _read_header()
DEFINES = _defines(_TXT)


class UsvCfg(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "usv_cfg", DEFINES)


class UsvBufs(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "usv_bufs", DEFINES)


class UsvHydro(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "usv_hydro", DEFINES)


class LzCfg(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "lz_cfg", DEFINES)


class PpoCfg(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "ppo_cfg", DEFINES)


class PpoAdamBanks(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "ppo_adam_banks", DEFINES)


class PpoDp(ctypes.Structure):
    _fields_ = _struct_fields(_TXT, "ppo_dp", DEFINES)


def enum_values(enum_name: str) -> dict:
    m = re.search(r"enum\s+%s\s*\{(.*?)\}" % enum_name, _TXT, flags=re.S)
    vals, cur = {}, -1
    for item in m.group(1).split(","):
        item = item.strip()
        if not item:
            continue
        if "=" in item:
            k, v = item.split("=")
            cur = int(v.strip())
            vals[k.strip()] = cur
        else:
            cur += 1
            vals[item] = cur
    return vals


STAT_KEYS_ENUM = enum_values("usv_stat_key")
PEN = enum_values("usv_pen_kind")

# ---- buffer / ABI layout key -------------------------------------------------------------------
# Every object-like integer #define of the header, every enumerator, and sizeof + offsetof of every
# field of every ABI struct, in header order.  libusv_hip.so folds the same list (compiled from
# csrc/usv_layout_gen.h, which gen_layout_header() writes from this function) into
# usv_hip_layout_key(); _capi.lib() refuses a library whose key differs from layout_key() here, so a
# library built from another header -- a moved slab row, a resized buffer, a reordered struct --
# fails loudly before its first call instead of addressing past a buffer.
LAYOUT_STRUCTS = ("usv_cfg", "usv_bufs", "usv_hydro", "ppo_cfg", "ppo_adam_banks", "ppo_dp", "lz_cfg")
LAYOUT_ENUMS = ("usv_stat_key", "usv_pen_kind", "usv_dist_row")
_STRUCT_CLASSES = {"usv_cfg": UsvCfg, "usv_bufs": UsvBufs, "usv_hydro": UsvHydro, "ppo_cfg": PpoCfg,
                   "ppo_adam_banks": PpoAdamBanks, "ppo_dp": PpoDp, "lz_cfg": LzCfg}
GUARD_DEFINES = ("USV_HIP_H",)


def header_int_defines() -> list:
    """(name, value) of every object-like #define of the header with an integer value, in order
    (C integer division for '/'); the include guard excluded."""
    out, env = [], {}
    for line in _TXT.splitlines():
        m = re.match(r"\s*#define\s+(\w+)(?:\s+(.*?))?\s*$", line)
        if not m or m.group(1) in GUARD_DEFINES:
            continue
        name, val = m.group(1), (m.group(2) or "")
        if "(" in name or not val:
            raise RuntimeError(f"{HEADER}: #define {name} has no integer value (layout key)")
        v = int(eval(val.replace("/", "//"), {}, dict(env)))
        env[name] = v
        out.append((name, v))
    return out


def layout_entries() -> list:
    """The layout list as (C expression, name, value) in fold order."""
    ent = [(n, n, v) for n, v in header_int_defines()]
    for e in LAYOUT_ENUMS:
        ent += [(k, k, v) for k, v in enum_values(e).items()]
    for s in LAYOUT_STRUCTS:
        cls = _STRUCT_CLASSES[s]
        ent.append((f"sizeof({s}_t)", f"sizeof {s}", ctypes.sizeof(cls)))
        for fname, _ in cls._fields_:
            ent.append((f"offsetof({s}_t, {fname})", f"{s}.{fname}", getattr(cls, fname).offset))
    return ent


def fnv1a(s: str) -> int:
    h = 1469598103934665603
    for ch in s.encode():
        h = ((h ^ ch) * 1099511628211) % (1 << 64)
    return h


def layout_key_of(entries) -> int:
    """k = k * 1000003 + fnv1a(name), then k = k * 1000003 + value, per entry (mod 2^64), top bit cleared."""
    k = 0
    for _, name, v in entries:
        k = (k * 1000003 + fnv1a(name)) % (1 << 64)
        k = (k * 1000003 + (v % (1 << 64))) % (1 << 64)
    return k & ((1 << 63) - 1)


def layout_header_text() -> str:
    lines = ["/* generated from include/usv_hip.h by omniisaacgymenvs_loop_amd/_abi.py (gen_layout_header): do not edit.",
             " * X(expression, \"name\") for every entry of usv_hip_layout_key() in fold order. */",
             "#define USV_LAYOUT_ENTRIES(X) \\"]
    lines += [f"  X({expr}, \"{name}\") \\" for expr, name, _ in layout_entries()]
    lines.append("")
    return "\n".join(lines) + "\n"


LAYOUT_GEN = os.path.join(_HERE, "csrc", "usv_layout_gen.h")


def gen_layout_header(path: str = LAYOUT_GEN) -> bool:
    """Write csrc/usv_layout_gen.h if its text differs from the header's; True when rewritten."""
    txt = layout_header_text()
    try:
        with open(path, "r", encoding="utf-8") as f:
            if f.read() == txt:
                return False
    except FileNotFoundError:
        pass
    with open(path, "w", encoding="utf-8") as f:
        f.write(txt)
    return True

# episode_sums key names in reference order (USV_Virtual.py:586-601)
STAT_NAMES = [
    "total_reward", "distance_reward", "alignment_reward", "heading_improve_reward",
    "potential_shaping_reward", "speed_reward", "angular_reward", "turn_hazard_penalty",
    "goal_reward", "collision_reward", "time_reward", "success", "collision",
    "position_error", "boundary_penalty", "danger_mean", "danger_hi_rate", "g_gate_mean",
    "g_safe_mean", "angular_vel_penalty", "angular_vel_variation_penalty", "energy_penalty",
    "normed_linear_vel", "normed_angular_vel", "cmd_neg_rate", "u_mean", "u_low_rate", "u_sum",
]
assert len(STAT_NAMES) == DEFINES["USV_NSTAT"]
