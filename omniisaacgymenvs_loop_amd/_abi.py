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
