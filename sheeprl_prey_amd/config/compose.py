"""Hydra-compatible config composition, written for this framework.

The reference is driven by Hydra 1.3 + OmegaConf (``sheeprl/cli.py:19-84``,
``sheeprl/configs/config.yaml:1-37``).  Neither library is part of the MI355X
image, so this module re-implements the subset of Hydra semantics the
reference's config tree relies on:

* a primary config with a ``defaults`` list (``_self_``, ``group: option``,
  ``exp: ???`` mandatory groups);
* group option files with their own ``defaults`` (``- default``,
  ``- /optim@world_model.optimizer: adam`` package redirection,
  ``- override /env: atari``);
* ``# @package _global_`` headers (experiment presets);
* command-line overrides: ``group=option``, ``a.b.c=value``, ``+a.b=value``,
  ``~a.b`` and ``++a.b=value``;
* interpolations ``${a.b.c}`` (typed when the whole string is one reference,
  textual otherwise) and ``${now:%Y-%m-%d}``.

The result is a plain nested ``dict`` (wrapped in :class:`dotdict` by the CLI).
"""
from __future__ import annotations

import copy
import datetime
import os
import re
from typing import Any, Dict, List, Optional, Sequence, Tuple

import yaml

MISSING = "???"

# --------------------------------------------------------------------------------------
# YAML loading: PyYAML (YAML 1.1) reads ``1e-4`` as a string; OmegaConf reads it as a
# float.  Register the broader float pattern so the reference config values keep types.
# --------------------------------------------------------------------------------------


class _Loader(yaml.SafeLoader):
    pass


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    re.compile(
        r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
        |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
        |\.[0-9_]+(?:[eE][-+][0-9]+)?
        |[-+]?\.(?:inf|Inf|INF)
        |\.(?:nan|NaN|NAN))$""",
        re.X,
    ),
    list("-+0123456789."),
)


def load_yaml_str(text: str) -> Any:
    return yaml.load(text, Loader=_Loader)


def load_yaml(path: str) -> Tuple[Any, Optional[str]]:
    """Return (content, package_header)."""
    with open(path, "r") as f:
        text = f.read()
    package = None
    for line in text.splitlines():
        s = line.strip()
        if s.startswith("# @package"):
            package = s[len("# @package") :].strip()
            break
        if s and not s.startswith("#"):
            break
    data = load_yaml_str(text)
    if data is None:
        data = {}
    return data, package


# --------------------------------------------------------------------------------------
# dict helpers
# --------------------------------------------------------------------------------------


def deep_merge(base: Dict[str, Any], other: Dict[str, Any]) -> Dict[str, Any]:
    """Merge ``other`` into ``base`` in place (dicts recurse, everything else replaces)."""
    for k, v in other.items():
        if isinstance(v, dict) and isinstance(base.get(k), dict):
            deep_merge(base[k], v)
        else:
            base[k] = copy.deepcopy(v)
    return base


def get_path(cfg: Dict[str, Any], path: str, default: Any = KeyError) -> Any:
    node: Any = cfg
    for part in path.split("."):
        if isinstance(node, dict) and part in node:
            node = node[part]
        elif isinstance(node, list) and part.isdigit() and int(part) < len(node):
            node = node[int(part)]
        else:
            if default is KeyError:
                raise KeyError(path)
            return default
    return node


def set_path(cfg: Dict[str, Any], path: str, value: Any, create: bool = True) -> None:
    parts = path.split(".")
    node = cfg
    for part in parts[:-1]:
        if part not in node or not isinstance(node[part], dict):
            if not create:
                raise KeyError(path)
            node[part] = {}
        node = node[part]
    node[parts[-1]] = value


def del_path(cfg: Dict[str, Any], path: str) -> None:
    parts = path.split(".")
    node = cfg
    for part in parts[:-1]:
        node = node[part]
    node.pop(parts[-1], None)


def wrap_package(content: Dict[str, Any], package: str) -> Dict[str, Any]:
    if package in ("", "_global_"):
        return content
    out: Dict[str, Any] = {}
    set_path(out, package, content)
    return out


# --------------------------------------------------------------------------------------
# Overrides
# --------------------------------------------------------------------------------------


class Override:
    __slots__ = ("key", "value", "op", "raw")

    def __init__(self, key: str, value: Any, op: str, raw: str):
        self.key, self.value, self.op, self.raw = key, value, op, raw

    def __repr__(self) -> str:  # pragma: no cover
        return f"Override({self.raw})"


def parse_override(s: str) -> Override:
    op = "set"
    if s.startswith("~"):
        key = s[1:].split("=", 1)[0]
        return Override(key, None, "del", s)
    if s.startswith("++"):
        op, s2 = "force", s[2:]
    elif s.startswith("+"):
        op, s2 = "add", s[1:]
    else:
        s2 = s
    if "=" not in s2:
        raise ValueError(f"Invalid override '{s}': expected key=value")
    key, raw_val = s2.split("=", 1)
    key = key.strip()
    raw_val = raw_val.strip()
    if raw_val == "":
        value: Any = ""
    else:
        try:
            value = load_yaml_str(raw_val)
        except yaml.YAMLError:
            value = raw_val
    if isinstance(value, str) and raw_val.lower() in ("none", "null"):
        value = None
    return Override(key, value, op, s)


# --------------------------------------------------------------------------------------
# Defaults-list processing
# --------------------------------------------------------------------------------------


class _Default:
    """One parsed defaults-list entry."""

    __slots__ = ("group", "option", "package", "is_self", "override", "absolute", "optional")

    def __init__(self, group=None, option=None, package=None, is_self=False, override=False, absolute=False, optional=False):
        self.group = group
        self.option = option
        self.package = package
        self.is_self = is_self
        self.override = override
        self.absolute = absolute
        self.optional = optional


def _parse_default(entry: Any) -> _Default:
    if isinstance(entry, str):
        if entry == "_self_":
            return _Default(is_self=True)
        # a config from the same group, e.g. "- default" inside algo/ppo.yaml
        return _Default(group=None, option=entry)
    if isinstance(entry, dict) and len(entry) == 1:
        (k, v), = entry.items()
        override = False
        optional = False
        k = k.strip()
        if k.startswith("override "):
            override = True
            k = k[len("override ") :].strip()
        if k.startswith("optional "):
            optional = True
            k = k[len("optional ") :].strip()
        package = None
        if "@" in k:
            k, package = k.split("@", 1)
        absolute = k.startswith("/")
        group = k.lstrip("/")
        return _Default(group=group, option=v, package=package, override=override, absolute=absolute, optional=optional)
    raise ValueError(f"Unsupported defaults entry: {entry!r}")


def _strip_ext(name: str) -> str:
    return name[:-5] if name.endswith(".yaml") else name


class Composer:
    """Compose a config from ``config_dir`` the way Hydra would (subset)."""

    GROUP_KEYS_CACHE: Dict[str, List[str]] = {}

    def __init__(self, config_dir: str):
        self.config_dir = config_dir

    # -- filesystem --------------------------------------------------------------------
    def groups(self) -> List[str]:
        out = []
        for root, dirs, _ in os.walk(self.config_dir):
            for d in dirs:
                if d.startswith("_"):
                    continue
                rel = os.path.relpath(os.path.join(root, d), self.config_dir)
                out.append(rel.replace(os.sep, "/"))
        return out

    def options(self, group: str) -> List[str]:
        d = os.path.join(self.config_dir, group)
        if not os.path.isdir(d):
            return []
        return sorted(_strip_ext(f) for f in os.listdir(d) if f.endswith(".yaml"))

    def _file(self, group: Optional[str], option: str) -> str:
        option = _strip_ext(option)
        rel = f"{group}/{option}.yaml" if group else f"{option}.yaml"
        path = os.path.join(self.config_dir, rel)
        if not os.path.isfile(path):
            avail = self.options(group) if group else []
            raise FileNotFoundError(
                f"Could not find '{rel}' in {self.config_dir}." + (f" Available options in '{group}': {avail}" if avail else "")
            )
        return path

    # -- pass 1: gather overrides declared by selected configs -------------------------
    def _collect_overrides(self, group: Optional[str], option: str, acc: Dict[str, str], seen: set) -> None:
        key = (group, option)
        if key in seen:
            return
        seen.add(key)
        content, _ = load_yaml(self._file(group, option))
        defaults = content.get("defaults", []) if isinstance(content, dict) else []
        for entry in defaults:
            d = _parse_default(entry)
            if d.is_self:
                continue
            if d.override:
                acc[d.group] = d.option
                continue
            if d.group is None:
                # same-group parent config: its overrides apply first; ours win afterwards.
                parent_acc: Dict[str, str] = {}
                self._collect_overrides(group, d.option, parent_acc, seen)
                for k, v in parent_acc.items():
                    acc.setdefault(k, v)
        # re-apply own overrides so that child wins over parent
        for entry in defaults:
            d = _parse_default(entry)
            if d.override:
                acc[d.group] = d.option

    # -- pass 2: compose ---------------------------------------------------------------
    def _compose_node(
        self, group: Optional[str], option: str, package: Optional[str], choices: Dict[str, str]
    ) -> Dict[str, Any]:
        content, header = load_yaml(self._file(group, option))
        if not isinstance(content, dict):
            content = {}
        content = dict(content)
        defaults = content.pop("defaults", [])
        if package is None:
            if header is not None:
                package = "" if header == "_global_" else header
            else:
                package = group or ""
        elif header == "_global_" and package == (group or ""):
            package = ""
        parsed = [_parse_default(e) for e in defaults]
        if not any(d.is_self for d in parsed):
            parsed.append(_Default(is_self=True))
        result: Dict[str, Any] = {}
        for d in parsed:
            if d.is_self:
                deep_merge(result, wrap_package(content, package))
                continue
            if d.override:
                # the choice was already resolved globally (pass 1); materialise it here if
                # the group isn't composed by the root defaults list.
                continue
            if d.group is None:
                sub = self._compose_node(group, d.option, package, choices)
                deep_merge(result, sub)
                continue
            sub_group = d.group
            opt = d.option
            if not d.absolute and group is not None and d.group is not None and "/" not in d.group:
                # relative group inside a group dir, e.g. "- default" handled above; a
                # relative "sub: opt" means <group>/sub; the reference only uses absolute ones.
                rel_dir = os.path.join(self.config_dir, group, d.group)
                if os.path.isdir(rel_dir):
                    sub_group = f"{group}/{d.group}"
            opt = choices.get(sub_group, opt)
            if opt is None:
                continue
            if opt == MISSING:
                if d.optional:
                    continue
                raise ValueError(f"You must specify '{sub_group}', e.g, {sub_group}=<OPTION>. Options: {self.options(sub_group)}")
            if d.package is not None:
                sub_pkg = f"{package}.{d.package}" if package else d.package
            else:
                sub_pkg = None  # default: the group path (or header)
            sub = self._compose_node(sub_group, opt, sub_pkg, choices)
            deep_merge(result, sub)
        return result

    def compose(self, config_name: str = "config", overrides: Sequence[str] = ()) -> Dict[str, Any]:
        parsed_ov = [parse_override(o) for o in overrides]
        groups = set(self.groups())
        cli_choices: Dict[str, str] = {}
        value_ov: List[Override] = []
        for ov in parsed_ov:
            gkey = ov.key.lstrip("/")
            if gkey.startswith("hydra/"):
                # hydra/job_logging=disabled & co: logging plumbing we do not have
                continue
            if ov.op in ("set", "add", "force") and gkey in groups and not isinstance(ov.value, dict):
                cli_choices[gkey] = None if ov.value is None else str(ov.value)
            else:
                value_ov.append(ov)
        # root defaults choices
        root, _ = load_yaml(self._file(None, config_name))
        choices: Dict[str, str] = {}
        for entry in root.get("defaults", []):
            d = _parse_default(entry)
            if not d.is_self and d.group:
                choices[d.group] = _strip_ext(str(d.option)) if d.option is not None else None
        choices.update(cli_choices)
        # pass 1: overrides from the selected configs (experiments mostly)
        declared: Dict[str, str] = {}
        seen: set = set()
        for g, opt in list(choices.items()):
            if opt is None or opt == MISSING:
                continue
            self._collect_overrides(g, opt, declared, seen)
        # second round, since an override may pick a config declaring further overrides
        for g, opt in list(declared.items()):
            self._collect_overrides(g, opt, declared, seen)
        for g, opt in declared.items():
            if g not in cli_choices:
                choices[g] = opt
        cfg = self._compose_node(None, config_name, "", choices)
        # value overrides
        for ov in value_ov:
            if ov.op == "del":
                del_path(cfg, ov.key)
                continue
            exists = get_path(cfg, ov.key, default=_SENTINEL) is not _SENTINEL
            if ov.op == "set" and not exists:
                parent = ov.key.rsplit(".", 1)[0] if "." in ov.key else ""
                parent_node = get_path(cfg, parent, default=None) if parent else cfg
                if not isinstance(parent_node, dict):
                    raise KeyError(f"Could not override '{ov.key}': key not found (use '+{ov.raw}' to append)")
                # Hydra is strict here; we are lenient for keys under an existing dict
            if ov.op == "add" and exists:
                raise KeyError(f"Could not append to config. An item is already at '{ov.key}'")
            set_path(cfg, ov.key, ov.value)
        cfg.setdefault("_choices_", {})
        cfg["_choices_"] = {k: v for k, v in choices.items() if k != "hydra"}
        return cfg


_SENTINEL = object()

# --------------------------------------------------------------------------------------
# Interpolation
# --------------------------------------------------------------------------------------

_INTERP = re.compile(r"\$\{([^${}]+)\}")


class InterpolationError(RuntimeError):
    pass


def resolve(cfg: Dict[str, Any], now: Optional[datetime.datetime] = None) -> Dict[str, Any]:
    """Resolve every ``${...}`` in place (with cycle detection)."""
    now = now or datetime.datetime.now()
    resolving: set = set()

    def lookup(path: str) -> Any:
        if path.startswith("now:"):
            return now.strftime(path[4:])
        if path.startswith("oc.env:"):
            name, _, dflt = path[len("oc.env:") :].partition(",")
            return os.environ.get(name.strip(), dflt.strip() or None)
        if path in resolving:
            raise InterpolationError(f"Cyclic interpolation at '{path}'")
        try:
            val = get_path(cfg, path)
        except KeyError:
            raise InterpolationError(f"Interpolation key '{path}' not found")
        if isinstance(val, str) and "${" in val:
            resolving.add(path)
            val = resolve_value(val)
            resolving.discard(path)
            set_path(cfg, path, val)
        elif isinstance(val, (dict, list)):
            resolving.add(path)
            walk(val, path)
            resolving.discard(path)
        return val

    def resolve_value(s: str) -> Any:
        m = _INTERP.fullmatch(s.strip())
        if m:
            return copy.deepcopy(lookup(m.group(1).strip()))
        prev = None
        while prev != s and "${" in s:
            prev = s
            s = _INTERP.sub(lambda mm: str(lookup(mm.group(1).strip())), s)
        return s

    def walk(node: Any, prefix: str) -> None:
        if isinstance(node, dict):
            for k in list(node.keys()):
                v = node[k]
                p = f"{prefix}.{k}" if prefix else str(k)
                if isinstance(v, str) and "${" in v:
                    resolving.add(p)
                    node[k] = resolve_value(v)
                    resolving.discard(p)
                elif isinstance(v, (dict, list)):
                    walk(v, p)
        elif isinstance(node, list):
            for i, v in enumerate(node):
                p = f"{prefix}.{i}"
                if isinstance(v, str) and "${" in v:
                    node[i] = resolve_value(v)
                elif isinstance(v, (dict, list)):
                    walk(v, p)

    walk(cfg, "")
    return cfg


def check_missing(cfg: Any, prefix: str = "", skip: Sequence[str] = ()) -> List[str]:
    out = []
    if isinstance(cfg, dict):
        for k, v in cfg.items():
            p = f"{prefix}.{k}" if prefix else str(k)
            if p in skip:
                continue
            out += check_missing(v, p, skip)
    elif isinstance(cfg, str) and cfg == MISSING:
        out.append(prefix)
    return out


CONFIG_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs")


def compose(
    overrides: Sequence[str] = (),
    config_name: str = "config",
    config_dir: str = CONFIG_DIR,
    resolve_interpolations: bool = True,
) -> Dict[str, Any]:
    """Compose and resolve a config.  Returns ``(job_cfg)`` with ``hydra`` under ``cfg['hydra']``."""
    cfg = Composer(config_dir).compose(config_name, overrides)
    if resolve_interpolations:
        resolve(cfg)
    return cfg
