"""GEMM solution selection for the library GEMMs (hipBLASLt / rocBLAS) via PyTorch TunableOp.

The plain GEMMs of the hot path (MLP layers of the Dreamer heads, imagination and actor/critic,
the hoisted RSSM projections) go to hipBLASLt through ``torch.mm`` / ``F.linear``.  Its default
heuristic picks small macro-tiles for the M=1024 imagination shapes (e.g. ``MT64x32x32`` at ~50% of
the fp32 MFMA peak).  TunableOp benchmarks every hipBLASLt and rocBLAS solution for each GEMM shape
once and records the fastest; the results for the MI355X bench shapes are committed under
``configs/tunableop/`` and loaded read-only at start-up, so no run pays the tuning cost.

    mode "use"  : load the committed results (tuning off; unknown shapes keep the default solution)
    mode "tune" : benchmark shapes not in the file; the merged results are written to ``filename``
                  when the process exits (TunableOp writes its file at teardown)
    mode "off"  : library defaults
"""
from __future__ import annotations

import os
from typing import Optional

import torch

RESULTS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "tunableop",
                       "mi355x_gemm_results.csv")


def configure(mode: str = "use", filename: Optional[str] = None) -> bool:
    """Set up TunableOp for this process; returns True when tuned solutions are active."""
    # YAML reads a bare ``off`` / ``on`` as a boolean
    mode = {"false": "off", "none": "off", "no": "off", "0": "off", "true": "use", "on": "use", "yes": "use"}.get(
        str(mode).lower(), str(mode).lower())
    if mode == "off" or not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tun

    src = filename or os.environ.get("SRL_TUNABLEOP_FILE") or RESULTS
    if mode == "use":
        if not os.path.exists(src):
            return False
        tun.enable(True)
        tun.tuning_enable(False)
        # results are written at exit: keep the committed file untouched
        tun.set_filename(os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tunableop_unused_{os.getpid()}.csv"), False)
        tun.read_file(src)
        return True
    if mode == "tune":
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(30)
        tun.set_max_tuning_iterations(50)
        tun.set_filename(src, False)
        if os.path.exists(src):
            tun.read_file(src)
        return True
    raise ValueError(f"unknown gemm tuning mode {mode!r} (use | tune | off)")

