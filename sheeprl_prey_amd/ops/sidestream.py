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
* ``param_grads(dev, fn, params, *reads)``: outside a scope ``fn()`` runs in line and its gradient tensors are
  returned; inside a scope it is QUEUED and None is returned for those parameters (the autograd Function hands
  autograd no gradient for them, so no AccumulateGrad runs - autograd would clone a buffer that is still
  being written on another stream).
* ``fork_point(dev)`` / ``flush(dev, fork=...)``: the scan backward records the fork point on the main stream,
  enqueues its kernel, then flushes.  The queue then runs on a side stream forked off the main stream at that
  point (so it sees every data gradient queued before the scan and does NOT wait for the scan), behind a short
  spin kernel so that the scan's workgroups are resident before the weight-gradient grids fill the chip (a
  persistent grid needs whole free CUs; the side kernels then run on the CUs the scan leaves idle).  Each
  result becomes its parameter's ``.grad`` (or is added to one already there, on the side stream).  Reads
  and results are marked used by the side / main stream (``record_stream``) so the caching allocator cannot
  recycle them early.
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
# microseconds the side branch waits (one-wave delay kernel) before its first weight-gradient grid
DELAY_US = 8.0
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


def param_grads(dev: torch.device, fn: Callable[[], Sequence[Optional[Tensor]]], params: Sequence[Optional[Tensor]],
                *reads: Tensor) -> List[Optional[Tensor]]:
    """``fn()`` -> the gradients of ``params``: computed now and returned, or (inside a scope) queued until
    ``flush`` and None returned."""
    if not active(dev):
        return list(fn())
    i = _index(dev)
    _queue.setdefault(i, []).append((fn, list(params), reads))
    if not _armed.get(i):
        _armed[i] = True
        main = torch.cuda.current_stream(dev)
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _finish(i, main))
    return [None] * len(params)


def fork_point(dev: torch.device) -> Optional["torch.cuda.Event"]:
    """An event on the current stream marking where the side branch forks (recorded BEFORE the kernel it should
    run beside is enqueued: a fork after it would make the branch wait for that kernel to finish)."""
    if dev.type != "cuda" or not _queue.get(_index(dev)):
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return ev


def flush(dev: torch.device, delay: bool = True, fork: Optional["torch.cuda.Event"] = None, inline: bool = False) -> None:
    """Run the queued parameter-gradient work on the side stream, forked off the current stream at ``fork``
    (a ``fork_point`` event) or now.  ``inline``: on the current stream instead - for a scan backward made of
    many short launches (the per-step ``rssm_scan.hip`` / skinny path, e.g. XL): side grids competing with its
    latency-bound kernels measured slower (XL 47.4 vs 48.2 env-steps/s deferred vs in line)."""
    if dev.type != "cuda":
        return
    i = _index(dev)
    q = _queue.pop(i, None)
    if not q:
        return
    main = torch.cuda.current_stream(dev)
    if inline:
        for fn, params, _reads in q:
            for p, r in zip(params, fn()):
                if p is None or r is None:
                    continue
                if p.grad is None:
                    p.grad = r.view_as(p) if r.shape != p.shape else r
                else:
                    p.grad.add_(r.view_as(p))
        _fire_hooks(q)
        return
    s = _stream(i)
    if fork is not None:
        s.wait_event(fork)
    else:
        s.wait_stream(main)
    with torch.cuda.stream(s):
        if delay and DELAY_US > 0:
            from sheeprl_prey_amd import ops

            ops._ext().side_delay(DELAY_US)
        for fn, params, reads in q:
            res = fn()
            for p, r in zip(params, res):
                if p is None or r is None:
                    continue
                if p.grad is None:
                    p.grad = r.view_as(p) if r.shape != p.shape else r
                else:
                    p.grad.add_(r.view_as(p))
                r.record_stream(main)  # read there after the join (flat optimiser gather)
            for t in reads:
                if t is not None and t.is_cuda:
                    t.record_stream(s)
    _pending[i] = True
    _fire_hooks(q)


def _fire_hooks(q) -> None:
    # the post-accumulate-grad hooks autograd did not run for these parameters (the flat optimisers' overlapped
    # all-reduce buckets, parallel/flat_optim.py): they join the side stream before they read the gradient
    for _, params, _ in q:
        for p in params:
            hooks = getattr(p, "_post_accumulate_grad_hooks", None) if p is not None else None
            if hooks and p.grad is not None:
                for h in list(hooks.values()):
                    h(p)


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
