"""Deferred parameter gradients: weight-gradient work of the world-model backward run BESIDE the
persistent scan backward instead of in front of it.

In the DreamerV3 world-model backward (reference ``dreamer_v3.py:178-182``: one ``backward`` of the summed
losses through decoder, heads, RSSM scan and encoder) the data-gradient chain is decoder / heads dgrad ->
scan backward (``ops/rssm.py``) -> encoder.  The parameter gradients of the decoder convolutions
(``ops/conv.py`` ``DecoderConvFn``), of the first layers over the latents (``ops/onehot.py``) and of every
``ops.linear`` layer behind them (reward / continue / prior heads) are read first by the optimiser's clip,
so nothing on that chain waits for them.  The persistent scan backward holds ~160 of the 256 CUs for
~1.7 ms while its workgroups mostly wait on each other's hand-offs; the other CUs are idle.

Protocol (``with scope(): loss.backward()``):
* ``param_grads(dev, fn, shapes, *reads)``: inside a scope, the gradient tensors are allocated now (on the
  main stream, so autograd can hand them to the parameters) and ``fn(outs)`` - which fills ``outs`` or
  returns tensors to copy into them - is QUEUED; outside a scope it runs in line and its result is returned.
* ``flush(dev)``: the scan backward calls it right after launching its kernel.  The queue then runs on a
  side stream forked off the main stream (so it sees every data gradient queued so far), behind a short
  spin kernel so that the scan's workgroups are resident before the weight-gradient grids fill the chip (a
  persistent grid needs whole free CUs; the side kernels then run on the CUs the scan leaves idle).
  Reads are marked used by the side stream (``record_stream``) so the caching allocator cannot recycle them.
* the join: the first queued item registers an autograd final callback that flushes whatever is still
  queued (a backward without a scan) and makes the main stream wait for the side stream; the flat
  optimisers also call ``join()`` before they read a gradient (``parallel/flat_optim.py``).  hipGraph
  capture records the fork / join as graph edges (branches replay concurrently:
  ``scripts/overlap_probe.py``).

Same gradients as the in-line backward, joined before anything reads them.  ``SRL_DEFER_WGRAD=0`` runs
everything in line (A/B).  History: round 4 forked each weight gradient onto the side stream as soon as its
output gradient existed; those kernels then competed with the decoder's data-gradient convolutions instead
of filling the scan's idle CUs and the step got slower (``profiles/r4_side_stream.md``)."""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Callable, Dict, Iterator, List, Optional, Sequence

import torch
from torch import Tensor

ENABLED = os.environ.get("SRL_DEFER_WGRAD", "1") != "0"
# cycles of the spin kernel at the head of the side branch (~8 us at the gfx950 shader clock)
DELAY_CYCLES = 20000
_streams: Dict[int, "torch.cuda.Stream"] = {}
_queue: Dict[int, List] = {}
_pending: Dict[int, bool] = {}
_armed: Dict[int, bool] = {}
_depth = 0  # open scopes (module-level: autograd runs GPU backward functions on its own device threads)


@contextmanager
def scope() -> Iterator[None]:
    global _depth
    _depth += 1
    try:
        yield
    finally:
        _depth -= 1


def _stream(i: int) -> "torch.cuda.Stream":
    s = _streams.get(i)
    if s is None:
        s = _streams[i] = torch.cuda.Stream(device=i)
        from sheeprl_prey_amd import ops

        # column-sum launches on this stream rotate through their own half of the ticket workspace (norm.hip)
        ops._ext().set_colsum_side_stream(int(s.cuda_stream))
    return s


def _index(dev: torch.device) -> int:
    return dev.index if dev.index is not None else torch.cuda.current_device()


def active(dev: torch.device) -> bool:
    return ENABLED and _depth > 0 and dev.type == "cuda"


def param_grads(dev: torch.device, fn: Callable[[Optional[List[Optional[Tensor]]]], Sequence[Optional[Tensor]]],
                shapes: Sequence, *reads: Tensor) -> List[Optional[Tensor]]:
    """``fn(outs)`` now (``outs=None``: fn allocates) or, inside a scope, queued until ``flush``; returns the
    gradient tensors (entries of ``shapes`` that are None give None)."""
    if not active(dev):
        return list(fn(None))
    outs = [torch.empty(tuple(s), device=dev, dtype=torch.float32) if s is not None else None for s in shapes]
    i = _index(dev)
    _queue.setdefault(i, []).append((fn, outs, reads))
    if not _armed.get(i):
        _armed[i] = True
        main = torch.cuda.current_stream(dev)
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _finish(i, main))
    return outs


def flush(dev: torch.device, delay: bool = True) -> None:
    """Run the queued parameter-gradient work on the side stream, forked off the current stream now."""
    if dev.type != "cuda":
        return
    i = _index(dev)
    q = _queue.pop(i, None)
    if not q:
        return
    main = torch.cuda.current_stream(dev)
    s = _stream(i)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        if delay and DELAY_CYCLES > 0:
            torch.cuda._sleep(DELAY_CYCLES)
        for fn, outs, _ in q:
            res = fn(outs)
            for o, r in zip(outs, res):
                if o is not None and r is not None and r.data_ptr() != o.data_ptr():
                    o.copy_(r.view_as(o))
    for _, outs, reads in q:
        for t in list(reads) + list(outs):
            if t is not None and t.is_cuda:
                t.record_stream(s)
    _pending[i] = True


def _finish(i: int, main: "torch.cuda.Stream") -> None:
    _armed.pop(i, None)
    if _queue.get(i):
        with torch.cuda.stream(main):
            flush(torch.device("cuda", i), delay=False)
    if _pending.pop(i, False):
        main.wait_stream(_streams[i])


def join(dev=None) -> None:
    """Current stream waits for every pending side branch (of ``dev``, or of every device); queued work not
    flushed yet is flushed first."""
    for i in list(_queue):
        if dev is not None and torch.device(dev).type == "cuda" and torch.device(dev).index not in (None, i):
            continue
        flush(torch.device("cuda", i), delay=False)
    for i in list(_pending):
        if dev is not None and torch.device(dev).type == "cuda" and torch.device(dev).index not in (None, i):
            continue
        torch.cuda.current_stream(i).wait_stream(_streams[i])
        del _pending[i]
