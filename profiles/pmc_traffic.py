"""Condense a run_profiles.sh output directory into the committed profile files.

    python profiles/pmc_traffic.py <tag> <envs> [<out_json>]

Reads gpurun_out/prof_<tag>/{trace_kernel_stats,seqtrace_kernel_stats,pmc_fetch_counter_collection,
pmc_write_counter_collection}.csv and writes
  profiles/<tag>_kernel_stats.csv                (rocprofv3 --stats summary, default overlapped step)
  profiles/<tag>_seq_kernel_stats.csv            (the same with USV_STEP_OVERLAP=0: k_env_step alone on the GPU)
  profiles/<tag>_pmc_{fetch,write}_k_env_step.csv (per-dispatch counters)
  <out_json> (default profiles/env_step_traffic_<envs>.json): HBM bytes per
  launch of k_env_step = FETCH_SIZE (KB) x 1024 x 2 (gfx950 half-count
  correction, MI355X_MICROARCH.md) + WRITE_SIZE (KB) x 1024, mean over launches,
  split into reads and writes next to the algorithmic reads / writes, and the
  roofline fractions on both byte counts (702 B: bench ENV_STEP_BYTES, 476 B:
  SURVEY 8(d)) from the sequential trace's k_env_step mean duration -- every
  number of the bench's roofline object recomputable from profiles/ alone.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV_STEP_BYTES = 702   # bench.py ENV_STEP_BYTES
READ_BYTES, WRITE_BYTES = 389, 313   # its split
SURVEY_STEP_BYTES = 476
HBM_PEAK_GBS = 8000.0

KEEP = ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size",
        "VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value"]


def trim(src, dst, envs=None):
    # the fused CaptureXY step at this size only (the grid is one thread per env, rounded to whole 256-thread blocks)
    rows = [r for r in csv.DictReader(open(src)) if "k_env_step" in r["Kernel_Name"] and "task" not in r["Kernel_Name"]
            and (envs is None or int(r["Grid_Size"]) == (envs + 255) // 256 * 256)]
    with open(dst, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=KEEP)
        w.writeheader()
        for r in rows:
            w.writerow({k: r[k] for k in KEEP})
    return [float(r["Counter_Value"]) for r in rows]


def main(tag, envs, out_json=None):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    shutil.copy(os.path.join(src, "trace_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    fetch = trim(os.path.join(src, "pmc_fetch_counter_collection.csv"),
                 os.path.join(dst, f"{tag}_pmc_fetch_k_env_step.csv"), envs)
    write = trim(os.path.join(src, "pmc_write_counter_collection.csv"),
                 os.path.join(dst, f"{tag}_pmc_write_k_env_step.csv"), envs)
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    seq = {}
    sq = os.path.join(src, "seqtrace_kernel_stats.csv")
    if os.path.exists(sq):
        shutil.copy(sq, os.path.join(dst, f"{tag}_seq_kernel_stats.csv"))
        row = next(r for r in csv.DictReader(open(sq)) if "k_env_step" in r["Name"] and "task" not in r["Name"])
        us = float(row["AverageNs"]) / 1e3
        seq = {"seq_kernel_stats": f"profiles/{tag}_seq_kernel_stats.csv", "seq_calls": int(row["Calls"]),
               "seq_mean_us": us,
               "frac_702": ENV_STEP_BYTES * envs / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
               "frac_476": SURVEY_STEP_BYTES * envs / (us * 1e-6) / 1e9 / HBM_PEAK_GBS}
    out = {
        "kernel": "k_env_step<true>",
        "envs": envs,
        "fetch_size_kb_raw_mean": fk,
        "write_size_kb_mean": wk,
        "bytes_per_launch": fk * 1024 * 2 + wk * 1024,
        "read_bytes_per_launch": fk * 1024 * 2,
        "write_bytes_per_launch": wk * 1024,
        "algorithmic_bytes_per_launch": ENV_STEP_BYTES * envs,
        "algorithmic_read_bytes_per_launch": READ_BYTES * envs,
        "algorithmic_write_bytes_per_launch": WRITE_BYTES * envs,
        "survey_bytes_per_launch": SURVEY_STEP_BYTES * envs,
        "read_over_algorithmic": fk * 1024 * 2 / (READ_BYTES * envs),
        "write_over_algorithmic": wk * 1024 / (WRITE_BYTES * envs),
        **seq,
        "source": f"profiles/{tag}_pmc_{{fetch,write}}_k_env_step.csv: mean over launches, FETCH_SIZE x1024 x2 "
                  "(gfx950 half-count correction) + WRITE_SIZE x1024; separate --pmc passes",
    }
    out_json = out_json or os.path.join(dst, f"env_step_traffic_{envs}.json")
    with open(out_json, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
