"""Every environment variable the product code or the bench reads (getenv / os.environ) and every compile-time
A/B switch of the HIP sources (#ifndef USV_*) is documented in INTEGRATION.md's switches tables."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "omniisaacgymenvs_loop_amd")


def _sources():
    for d, _, files in os.walk(PKG):
        for f in files:
            if f.endswith((".py", ".hip", ".h")):
                yield os.path.join(d, f)
    yield os.path.join(ROOT, "bench.py")


def test_every_switch_is_documented():
    env_re = re.compile(r"""(?:getenv|environ\.get)\(\s*["'](USV_[A-Z0-9_]+)["']""")
    ifndef_re = re.compile(r"^#ifndef (USV_[A-Z0-9_]+)\s*$", re.M)
    names = set()
    for p in _sources():
        text = open(p, encoding="utf-8").read()
        names.update(env_re.findall(text))
        if p.endswith(".hip"):
            names.update(n for n in ifndef_re.findall(text) if not n.endswith("_H"))
    doc = open(os.path.join(ROOT, "INTEGRATION.md"), encoding="utf-8").read()
    assert names, "no switches found: the scan is broken"
    missing = sorted(n for n in names if f"`{n}`" not in doc)
    assert not missing, f"switches missing from INTEGRATION.md: {missing}"
