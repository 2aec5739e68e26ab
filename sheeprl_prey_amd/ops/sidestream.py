"""Side-stream work inside a backward pass: weight gradients nothing downstream of the backward needs.

In the DreamerV3 world-model backward the decoder's weight gradients (``ops/conv.py`` ``DecoderConvFn``) are
off the critical path: the data-gradient chain decoder -> persistent scan backward -> encoder needs only the
decoder's input gradients, and the weight gradients are read first by the optimiser's gradient clip.  The
persistent scan backward holds 160 of the 256 CUs for ~1.7 ms; work on a second stream runs on the other CUs
meanwhile.  hipGraph capture records the fork / join as graph edges and replays the branches concurrently
(``scripts/overlap_probe.py``: ``graph_branch_overlap``).  Reference semantics are unchanged: the same
gradients, joined before anything reads them.

Opt-in per backward: ``with scope(): loss.backward()`` (the DreamerV3 world-model phase does this; the
gradients must be fresh - ``zero_grad(set_to_none=True)`` - so autograd hands them to the parameters without
reading them).  Outside a scope ``on_side`` runs in line, so any other caller of these autograd functions (tests,
gradient accumulation) sees the plain single-stream backward.

Protocol: ``with on_side(dev, *reads):`` forks the side stream off the current stream (it waits for everything
queued so far, e.g. the data gradient a weight gradient consumes), runs the block on it and marks the tensors
the block read as used by the side stream (so the caching allocator does not hand their memory to the main
stream before the side work finishes); the first fork of a backward also queues a join of the branch onto
the forking stream at the end of that backward (autograd final callback), so a captured step always joins the
branch before its capture ends.  ``join()`` makes the current stream wait for all side work; the flat optimiser
also calls it before it reads a gradient (``parallel/flat_optim.py``: ``wait_grads`` / ``_gather`` / the overlap
hooks).

Measured SLOWER, so opt-in: ``SRL_SIDE_WGRAD=1`` (default 0).  On the Atari-100k bench the branch took the
step from 323.4 to 307.4-307.8 env-steps/s (``profiles/r4_side_stream.md``): the side kernels slow the conv
stack (3.74 -> 4.28 ms/step of kernel time) and the scan while they share the chip, and the busy time barely
overlaps (13.63 ms kernel time in a 13.48 ms wall window) - the same verdict as round 2's side-stream weight
gradients in the imagination phase."""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Dict, Iterator

import torch
from torch import Tensor

ENABLED = os.environ.get("SRL_SIDE_WGRAD", "0") == "1"
_streams: Dict[int, "torch.cuda.Stream"] = {}
_pending: Dict[int, bool] = {}
_depth = 0  # open scopes (module-level: autograd runs GPU backward functions on its own device threads)


@contextmanager
def scope() -> Iterator[None]:
    global _depth
    _depth += 1
    try:
        yield
    finally:
        _depth -= 1


def _stream(dev: torch.device) -> "torch.cuda.Stream":
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    s = _streams.get(i)
    if s is None:
        s = _streams[i] = torch.cuda.Stream(device=i)
    return s


def active(dev: torch.device) -> bool:
    return ENABLED and _depth > 0 and dev.type == "cuda"


@contextmanager
def on_side(dev: torch.device, *reads: Tensor) -> Iterator[None]:
    if not active(dev):
        yield
        return
    main = torch.cuda.current_stream(dev)
    s = _stream(dev)
    if not _pending.get(s.device.index):
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _join_one(s.device.index, main))
    s.wait_stream(main)
    with torch.cuda.stream(s):
        yield
    for t in reads:
        if t is not None and t.is_cuda:
            t.record_stream(s)
    _pending[s.device.index] = True


def mark_main(t: Tensor) -> Tensor:
    """A side-allocated result that the main stream will read (after ``join``)."""
    if t.is_cuda and t.device.index in _streams:
        t.record_stream(torch.cuda.current_stream(t.device))
    return t


def _join_one(i: int, main: "torch.cuda.Stream") -> None:
    if _pending.pop(i, False):
        main.wait_stream(_streams[i])


def join(dev=None) -> None:
    """Current stream waits for every pending side branch (of ``dev``, or of every device)."""
    if not _pending:
        return
    for i in list(_pending):
        if dev is not None and torch.device(dev).type == "cuda" and torch.device(dev).index not in (None, i):
            continue
        torch.cuda.current_stream(i).wait_stream(_streams[i])
        del _pending[i]
