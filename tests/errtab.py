"""Per-column parity error table for the GPU parity tests.

Every parity assertion records, per named output column, the maximum absolute error, the maximum
relative error (over elements with |want| >= 1e-3) and the ratio
    r = max |got - want| / (ATOL + RTOL * |want|)        with ATOL = RTOL = 1e-5,
i.e. r <= 1 means the column meets the north-star "within 1e-5 fp32" (numpy assert_allclose semantics).
`check()` records and asserts at the tolerance the test states; conftest prints the table at the end of
the session and writes it to gpurun_out/parity_errors.json so the log carries the achieved errors.
"""
from __future__ import annotations

import json
import os

import numpy as np

ATOL = RTOL = 1e-5
_TABLE: dict = {}


def _key(test, qty, col):
    return f"{test}|{qty}|{col}"


def record(test: str, qty: str, got, want, cols=None, tol=None):
    """Fold the error of got vs want into the table (columns along the last axis if `cols` is given)."""
    g = np.asarray(got, np.float64)
    w = np.asarray(want, np.float64)
    assert g.shape == w.shape, (qty, g.shape, w.shape)
    if cols is None:
        g, w, cols = g.reshape(-1, 1), w.reshape(-1, 1), [""]
    else:
        g, w = g.reshape(-1, g.shape[-1]), w.reshape(-1, w.shape[-1])
    d = np.abs(g - w)
    big = np.abs(w) >= 1e-3
    for j, name in enumerate(cols):
        if name is None:
            continue
        dj = d[:, j]
        if dj.size == 0:
            continue
        ab = float(np.nanmax(dj)) if np.isfinite(dj).any() else float("nan")
        rel = float(np.max(dj[big[:, j]] / np.abs(w[big[:, j], j]))) if big[:, j].any() else 0.0
        ratio = float(np.max(dj / (ATOL + RTOL * np.abs(w[:, j]))))
        k = _key(test, qty, name)
        e = _TABLE.get(k, {"test": test, "qty": qty, "col": name, "max_abs": 0.0, "max_rel": 0.0,
                           "tol_ratio_1e5": 0.0, "n": 0, "tol": tol})
        e["max_abs"] = max(e["max_abs"], ab)
        e["max_rel"] = max(e["max_rel"], rel)
        e["tol_ratio_1e5"] = max(e["tol_ratio_1e5"], ratio)
        e["n"] += int(dj.size)
        if tol is not None:
            e["tol"] = tol
        _TABLE[k] = e


def check(test: str, qty: str, got, want, rtol: float, atol: float, cols=None, err_msg=""):
    """record() then numpy's assert_allclose at the stated tolerance."""
    record(test, qty, got, want, cols, tol=(rtol, atol))
    np.testing.assert_allclose(np.asarray(got), np.asarray(want), rtol=rtol, atol=atol, err_msg=err_msg or qty)


def table():
    return sorted(_TABLE.values(), key=lambda e: (e["test"], e["qty"], str(e["col"])))


def format_table() -> str:
    rows = table()
    if not rows:
        return ""
    out = ["parity error table (tol_ratio_1e5 <= 1 means within rtol = atol = 1e-5)",
           f"{'test':38s} {'quantity':12s} {'column':14s} {'max_abs':>10s} {'max_rel':>10s} {'r(1e-5)':>8s}  asserted"]
    for e in rows:
        tol = e.get("tol")
        ts = "" if tol is None else (f"rtol={tol[0]:g} atol={tol[1]:g}" if not isinstance(tol[0], str) else tol[0])
        out.append(f"{e['test'][:38]:38s} {e['qty'][:12]:12s} {str(e['col'])[:14]:14s} {e['max_abs']:10.3g} "
                   f"{e['max_rel']:10.3g} {e['tol_ratio_1e5']:8.3g}  {ts}")
    return "\n".join(out)


def dump(path: str):
    rows = table()
    if not rows:
        return
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(rows, f, indent=1)


OBS_COLS = (["u", "v", "w", "cos_a", "sin_a", "dist", "task6", "task7"]
            + [f"ob{k}_{c}" for k in range(5) for c in ("d", "nx", "ny")]
            + ["cmd_l", "cmd_r", "mass", "com_x", "com_y", "com_z", "k_drag", "thr_l", "thr_r", "k_Iz"])


def obs_cols(width: int):
    return OBS_COLS[:width] if width <= len(OBS_COLS) else [f"c{j}" for j in range(width)]
