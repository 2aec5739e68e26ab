"""Algorithm registry (reference: ``sheeprl/utils/registry.py:8-41``).

``tasks`` maps an algorithm module path to a list of ``{name, entrypoint, decoupled}``;
``@register_algorithm(decoupled=False)`` fills it when the algorithm module is imported.
"""
from __future__ import annotations

import sys
from typing import Any, Callable, Dict, List

tasks: Dict[str, List[Dict[str, Any]]] = {}


def _register(fn: Callable[..., Any], decoupled: bool = False) -> Callable[..., Any]:
    module = sys.modules[fn.__module__]
    module_path = module.__name__
    entry = {"name": module_path.rsplit(".", 1)[-1], "entrypoint": fn.__name__, "decoupled": decoupled}
    bucket = tasks.setdefault(module_path.rsplit(".", 1)[0], [])
    if not any(e["name"] == entry["name"] and e["entrypoint"] == entry["entrypoint"] for e in bucket):
        bucket.append(entry)
    if not hasattr(module, "__all__"):
        module.__all__ = []
    if fn.__name__ not in module.__all__:
        module.__all__.append(fn.__name__)
    return fn


def register_algorithm(decoupled: bool = False) -> Callable[[Callable[..., Any]], Callable[..., Any]]:
    def inner(fn: Callable[..., Any]) -> Callable[..., Any]:
        return _register(fn, decoupled=decoupled)

    return inner


def find_algorithm(name: str):
    """Return (module_path, entry) for the algorithm whose file name is ``name``."""
    for module_path, entries in tasks.items():
        for e in entries:
            if e["name"] == name:
                return module_path, e
    return None, None


def algorithm_names() -> List[str]:
    import sheeprl_prey_amd  # noqa: F401  (importing the package registers every algorithm)

    return [e["name"] for entries in tasks.values() for e in entries]
