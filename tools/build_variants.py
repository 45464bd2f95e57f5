"""Build A/B variants of the HIP library (same ABI) into lib/<name>.so for tools/gpu_variants.sh:
    python tools/build_variants.py name1:-DFOO=1 name2:-DFOO=2 ...   (flags separated by ',')"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from omniisaacgymenvs_loop_amd import _capi  # noqa: E402


def one(spec):
    name, _, flags = spec.partition(":")
    out = os.path.join(_capi.LIB_DIR, f"{name}.so")
    cmd = ["hipcc"] + _capi.HIPCC_FLAGS + [f for f in flags.split(",") if f] + ["-o", out] + _capi.SOURCES
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    _capi.build()
    with ThreadPoolExecutor(4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print("built", o)
