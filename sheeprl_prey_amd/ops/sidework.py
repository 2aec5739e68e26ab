"""Weight-gradient work deferred onto a side stream so it runs beside the persistent RSSM scan backward.

The persistent scan backward (``csrc/rssm_persist.hip``) keeps ``scanp_bwd_grid`` workgroups
resident, one per CU (160 of the 256 CUs at the Atari-100k shapes) for ~2 ms per step; the other
CUs idle.  The decoder's weight gradients do not feed the scan (only its data gradient does), so the
decoder backward (``ops/conv.py``) hands its ``conv_wgrad`` launches to this module instead of
issuing them in line.  The scan backward launches first, then the deferred work goes to a side
stream gated on an event recorded just BEFORE the scan launch: both become ready together and the
wgrad kernels fill the CUs the scan leaves free.  The training step joins the side stream after the
backward (``region`` exit), before anything reads the gradients.

Memory: outputs are allocated by the caller on the main stream (so autograd may steal them as
``.grad`` and nothing reads them before the join); the inputs of deferred work are kept referenced
until the join, so the caching allocator cannot hand their blocks to main-stream work while the side
stream still reads them.  Under hipGraph capture the fork (event wait) and join become graph edges.

Reference counterpart: none (the reference runs the whole backward on one stream,
``dreamer_v3/dreamer_v3.py:179-187``).
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Any, Callable, List, Optional

import torch

_ENABLED = os.environ.get("SRL_SIDE_WGRAD", "0") != "0"


class _State:
    def __init__(self) -> None:
        self.active = False
        self.queue: List[Callable[[], Any]] = []
        self.keep: List[Any] = []
        self.done: Optional[torch.cuda.Event] = None
        self.streams = {}
        self.deferred = 0  # launches handed to the side stream so far (tests check the path is taken)


_S = _State()


def active() -> bool:
    """True inside ``region``: callers may ``defer`` GPU work instead of issuing it in line."""
    return _S.active


def _side(device: torch.device) -> torch.cuda.Stream:
    s = _S.streams.get(device.index)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _S.streams[device.index] = s
    return s


def defer(fn: Callable[[], Any], *keep: Any) -> None:
    """Queue ``fn`` (launches only; it must write into caller-allocated outputs) for the side stream;
    ``keep`` holds its inputs alive until the join."""
    _S.queue.append(fn)
    _S.keep.extend(keep)
    _S.deferred += 1


def deferred_count() -> int:
    return _S.deferred


def launch(gate: Optional[torch.cuda.Event] = None) -> None:
    """Issue the queued work on the side stream, after ``gate`` (default: the current point of the
    calling stream)."""
    if not _S.queue:
        return
    main = torch.cuda.current_stream()
    side = _side(main.device)
    if gate is None:
        gate = torch.cuda.Event()
        gate.record(main)
    side.wait_event(gate)
    with torch.cuda.stream(side):
        for fn in _S.queue:
            fn()
        done = torch.cuda.Event()
        done.record(side)
    _S.queue.clear()
    _S.done = done


def join() -> None:
    """The calling stream waits for the side stream; deferred inputs are released afterwards."""
    if _S.queue:
        launch()
    if _S.done is not None:
        torch.cuda.current_stream().wait_event(_S.done)
        _S.done = None
    _S.keep.clear()


@contextmanager
def region(enabled: bool = True):
    """Scope of a backward whose weight-gradient work may be deferred; joins on exit."""
    on = bool(enabled and _ENABLED and torch.cuda.is_available())
    prev = _S.active
    _S.active = on
    try:
        yield
    finally:
        _S.active = prev
        if on:
            join()
