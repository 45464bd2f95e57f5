"""Hydra / OmegaConf composition of the reference's configs without Hydra or OmegaConf.

The reference composes `cfg/config.yaml` (root keys: seed, num_envs, experiment, rl_device, ...)
with `task=<task yaml>` and `train=<train yaml>` and resolves OmegaConf interpolations
(omniisaacgymenvs/scripts/rlgames_train111.py:113-124, utils/hydra_cfg/hydra_utils.py:36-41,
utils/hydra_cfg/reformat.py:33-41).  The USV yamls use exactly these features:

* relative interpolation: `${...seed}`, `${....task.env.numEnvs}`, `${.name}` -- one dot is the
  node that holds the key, each further dot one level up (OmegaConf 2.1 semantics);
* absolute interpolation: `${task.name}`;
* the four registered resolvers `eq`, `contains`, `if`, `resolve_default` (hydra_utils.py:36-41),
  with nested interpolations and quoted strings as arguments;
* OmegaConf's YAML float rule: `1e-4`, `3e-4` load as floats (plain PyYAML reads them as strings).

`compose()` returns a plain resolved dict, the shape `omegaconf_to_dict(cfg)` gives the reference's
scripts; `python -m omniisaacgymenvs_loop_amd.scripts.rlgames_train cfg_dir=<reference cfg dir> ...`
runs the reference's own unmodified yamls.
"""
from __future__ import annotations

import copy
import os
import re
from typing import Any, Dict, List, Optional, Sequence

import yaml


class _OmegaLoader(yaml.SafeLoader):
    """SafeLoader + OmegaConf's float resolver (exponents without a dot are floats)."""


_OmegaLoader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                  |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                  |\.[0-9_]+(?:[eE][-+][0-9]+)?
                  |[-+]?\.(?:inf|Inf|INF)
                  |\.(?:nan|NaN|NAN))$""", re.X),
    list("-+0123456789."))


def load_yaml(path: str) -> Dict[str, Any]:
    with open(path, "r", encoding="utf-8") as f:
        return yaml.load(f, Loader=_OmegaLoader) or {}


# utils/hydra_cfg/hydra_utils.py:36-41
RESOLVERS = {
    "eq": lambda x, y: str(x).lower() == str(y).lower(),
    "contains": lambda x, y: str(x).lower() in str(y).lower(),
    "if": lambda pred, a, b: a if pred else b,
    "resolve_default": lambda default, arg: default if arg == "" else arg,
}


class InterpolationError(KeyError):
    pass


def _get(root: Dict[str, Any], path: List[str]):
    node: Any = root
    for k in path:
        if isinstance(node, dict) and k in node:
            node = node[k]
        elif isinstance(node, list) and k.isdigit() and int(k) < len(node):
            node = node[int(k)]
        else:
            raise InterpolationError(".".join(path))
    return node


def _split_top(s: str, sep: str = ",") -> List[str]:
    """Split at `sep` outside ${...} and quotes."""
    out, depth, quote, cur = [], 0, None, []
    i = 0
    while i < len(s):
        ch = s[i]
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = None
        elif ch in "'\"":
            quote = ch
            cur.append(ch)
        elif s.startswith("${", i):
            depth += 1
            cur.append("${")
            i += 2
            continue
        elif ch == "}" and depth:
            depth -= 1
            cur.append(ch)
        elif ch == sep and depth == 0:
            out.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
        i += 1
    out.append("".join(cur))
    return out


def _match_close(s: str, start: int) -> int:
    """Index of the `}` closing the `${` at `start`."""
    depth, i = 0, start
    while i < len(s):
        if s.startswith("${", i):
            depth += 1
            i += 2
            continue
        if s[i] == "}":
            depth -= 1
            if depth == 0:
                return i
        i += 1
    raise InterpolationError(f"unterminated interpolation in {s!r}")


class _Resolver:
    def __init__(self, root: Dict[str, Any]):
        self.root = root
        self.active: set = set()

    def value(self, path: List[str]):
        """Fully resolved value at an absolute path."""
        key = tuple(path)
        if key in self.active:
            raise InterpolationError(f"interpolation cycle at {'.'.join(path)}")
        self.active.add(key)
        try:
            return self.node(_get(self.root, path), path)
        finally:
            self.active.discard(key)

    def node(self, v, path: List[str]):
        """v is the value at `path`; interpolations in it are relative to its container."""
        if isinstance(v, dict):
            return {k: self.node(x, path + [k]) for k, x in v.items()}
        if isinstance(v, list):
            return [self.node(x, path + [str(i)]) for i, x in enumerate(v)]
        return self.scalar(v, path[:-1])

    def scalar(self, v, parent: List[str]):
        if not isinstance(v, str) or "${" not in v:
            return v
        s = v.strip()
        if s.startswith("${") and _match_close(s, 0) == len(s) - 1:
            return self.interp(s[2:-1], parent)          # a whole-value interpolation keeps its type
        out, i = [], 0                                    # string interpolation
        while i < len(v):
            j = v.find("${", i)
            if j < 0:
                out.append(v[i:])
                break
            out.append(v[i:j])
            k = _match_close(v, j)
            out.append(str(self.interp(v[j + 2:k], parent)))
            i = k + 1
        return "".join(out)

    def interp(self, body: str, parent: List[str]):
        body = body.strip()
        m = re.match(r"^([A-Za-z_][\w]*):(.*)$", body, re.S)
        if m and m.group(1) in RESOLVERS:
            args = [self.arg(a, parent) for a in _split_top(m.group(2))]
            return RESOLVERS[m.group(1)](*args)
        if body.startswith("."):
            dots = len(body) - len(body.lstrip("."))
            rest = body[dots:]
            up = dots - 1
            if up > len(parent):
                raise InterpolationError(f"${{{body}}} climbs above the root")
            base = parent[:len(parent) - up]
            return self.value(base + (rest.split(".") if rest else []))
        return self.value(body.split("."))

    def arg(self, a: str, parent: List[str]):
        a = a.strip()
        if "${" in a:
            return self.scalar(a, parent)
        if len(a) >= 2 and a[0] == a[-1] and a[0] in "'\"":
            return a[1:-1]
        return yaml.load(a, Loader=_OmegaLoader) if a else ""


def resolve(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """Every interpolation of `cfg` resolved (OmegaConf.to_container(resolve=True))."""
    return _Resolver(cfg).node(cfg, [])


def _set_dotted(d: Dict[str, Any], key: str, value) -> None:
    parts = key.split(".")
    node = d
    for p in parts[:-1]:
        node = node.setdefault(p, {})
    node[parts[-1]] = value


def _find(cfg_dir: str, kind: str, name: str) -> str:
    if name.endswith(".yaml") and os.path.exists(name):
        return name
    path = os.path.join(cfg_dir, kind, name + ".yaml")
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return path


def compose(cfg_dir: str, task: str, train: Optional[str] = None, overrides: Optional[Dict[str, Any]] = None,
            root_yaml: Optional[str] = None) -> Dict[str, Any]:
    """config.yaml + task=<task> + train=<train> + key=value overrides, resolved.

    cfg_dir is a reference-style cfg tree (`task/`, `train/`; config.yaml optional: the package's
    copy of the root keys is used when it has none).  Overrides are root keys (num_envs=, seed=,
    experiment=, checkpoint=, max_iterations=, rl_device=, ...) or dotted paths (task.env.xxx=)."""
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cfg")
    root_path = root_yaml or (os.path.join(cfg_dir, "config.yaml") if os.path.exists(os.path.join(cfg_dir, "config.yaml"))
                              else os.path.join(here, "config.yaml"))
    root = load_yaml(root_path)
    root.pop("defaults", None)
    root.pop("hydra", None)
    root["task"] = load_yaml(_find(cfg_dir, "task", task))
    train = train or f"{root['task'].get('name', task)}PPO"
    root["train"] = load_yaml(_find(cfg_dir, "train", train))
    for k, v in (overrides or {}).items():
        _set_dotted(root, k, copy.deepcopy(v))
    return resolve(root)


def parse_cli(argv: Sequence[str]) -> Dict[str, Any]:
    """Hydra-style `key=value` arguments (values typed by OmegaConf's YAML rules)."""
    ov: Dict[str, Any] = {}
    for a in argv:
        if "=" not in a:
            raise SystemExit(f"expected key=value, got {a}")
        k, v = a.split("=", 1)
        ov[k.lstrip("+")] = yaml.load(v, Loader=_OmegaLoader) if v != "" else ""
    return ov
