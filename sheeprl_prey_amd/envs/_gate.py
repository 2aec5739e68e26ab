"""Import gate for optional third-party simulators (reference ``utils/imports.py``)."""
from __future__ import annotations

import importlib


def require(module: str, hint: str):
    try:
        return importlib.import_module(module)
    except Exception as e:  # noqa: BLE001
        raise ModuleNotFoundError(
            f"`{module}` is required for this environment but is not installed in this image ({e}). {hint}"
        ) from e
