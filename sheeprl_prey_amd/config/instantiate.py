"""``hydra.utils.instantiate`` / ``get_class`` equivalents for ``_target_`` config nodes."""
from __future__ import annotations

import importlib
from typing import Any, Dict

_ALIASES = {
    # reference targets that have native equivalents here
    "gymnasium.make": "sheeprl_prey_amd.envs.registry.make",
    "gym.make": "sheeprl_prey_amd.envs.registry.make",
    "gymnasium.wrappers.AtariPreprocessing": "sheeprl_prey_amd.envs.atari.AtariPreprocessing",
    "sheeprl.utils.env.get_dummy_env": "sheeprl_prey_amd.utils.env.get_dummy_env",
}


def get_class(path: str) -> Any:
    path = _ALIASES.get(path, path)
    if path.startswith("sheeprl.") and not path.startswith("sheeprl_prey_amd."):
        path = "sheeprl_prey_amd." + path[len("sheeprl.") :]
    module, _, attr = path.rpartition(".")
    if not module:
        raise ImportError(f"invalid target '{path}'")
    try:
        mod = importlib.import_module(module)
        return getattr(mod, attr)
    except (ImportError, AttributeError):
        # nested attribute (Class.method)
        parent, _, cls = module.rpartition(".")
        mod = importlib.import_module(parent)
        return getattr(getattr(mod, cls), attr)


get_method = get_class


def instantiate(cfg: Dict[str, Any], *args, **kwargs) -> Any:
    """Recursively build ``_target_`` nodes; ``kwargs`` override config keys."""
    if cfg is None:
        return None
    if isinstance(cfg, list):
        return [instantiate(c) if isinstance(c, dict) and "_target_" in c else c for c in cfg]
    if not isinstance(cfg, dict) or "_target_" not in cfg:
        return cfg
    params = {}
    for k, v in cfg.items():
        if k in ("_target_", "_recursive_", "_convert_", "_partial_"):
            continue
        if isinstance(v, dict) and "_target_" in v:
            v = instantiate(v)
        elif isinstance(v, dict):
            v = {kk: (instantiate(vv) if isinstance(vv, dict) and "_target_" in vv else vv) for kk, vv in v.items()}
        params[k] = v
    params.update(kwargs)
    target = get_class(cfg["_target_"])
    if cfg.get("_partial_", False):
        import functools

        return functools.partial(target, *args, **params)
    return target(*args, **params)
