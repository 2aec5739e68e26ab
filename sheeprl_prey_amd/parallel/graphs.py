"""hipGraph capture of whole training steps (torch.cuda.graph == hipGraph on ROCm).

The DreamerV3 Atari-100k step is launch-bound: ~3-4k small kernels (a T=64 sequential RSSM
scan, an H=15 imagination scan, three optimiser updates).  ``GraphedStep`` warms a step function
up on a side stream, captures one invocation into a hipGraph and afterwards replays it: inputs are
copied into static buffers, outputs are the captured static tensors.  Requirements on ``fn``:
no host syncs, no host-value-dependent control flow, persistent state updated in place
(``FlatOptimizer`` scalars, ``Moments`` buffers), RNG from torch's Philox generators.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional

import torch
from torch import Tensor

from sheeprl_prey_amd.parallel.flat_optim import gather_all_pending


def capture_error_mode() -> str:
    """Stream-capture mode of every hipGraph capture here: ``thread_local`` when a process group is up.
    In the default ``global`` mode ANY thread's unsafe HIP call fails during a capture - and the RCCL
    process group's watchdog thread polls the completion events of earlier collectives on its own schedule
    (a query that landed inside a capture aborted a GPU-suite run with hipErrorStreamCaptureUnsupported)."""
    import torch.distributed as dist

    return "thread_local" if dist.is_available() and dist.is_initialized() else "global"


def quiesce_for_capture(settle_s: float = 0.25) -> None:
    """Called right before a capture begins: the device is drained and, with a process group up, the host
    waits ``settle_s`` so the process group's watchdog reaps the (now complete) work of the eager warm-up
    collectives before the capture opens - its next poll (every ~100 ms) then has no event left to query
    while the capture is open.  A few captures per run: the wait costs well under a second in total."""
    import time

    import torch.distributed as dist

    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist.is_available() and dist.is_initialized():
        time.sleep(settle_s)


class GraphedStep:
    def __init__(self, fn: Callable[[Dict[str, Tensor]], Dict[str, Tensor]], warmup: int = 2, enabled: bool = True,
                 name: str = "step"):
        self.fn = fn
        self.warmup = warmup
        self.enabled = enabled and torch.cuda.is_available()
        self.name = name
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_in: Optional[Dict[str, Tensor]] = None
        self.static_out: Optional[Dict[str, Tensor]] = None
        self._calls = 0
        self.pool = None

    def _copy_in(self, data: Dict[str, Tensor]) -> None:
        for k, v in data.items():
            self.static_in[k].copy_(v, non_blocking=v.device.type != "cpu" or v.is_pinned())

    def replay_static(self) -> Optional[Dict[str, Tensor]]:
        """Replay the captured step on whatever the caller wrote into ``static_in`` (no copy-in); None before
        the capture."""
        if self.graph is None:
            return None
        self.graph.replay()
        return self.static_out

    def __call__(self, data: Dict[str, Tensor]) -> Dict[str, Tensor]:
        if not self.enabled:
            return self.fn(data)
        if self.graph is not None:
            self._copy_in(data)
            self.graph.replay()
            return self.static_out
        if self.static_in is None:
            # contiguous static inputs: a permuted replay sample ([B, T] storage viewed as [T, B]) is
            # reordered once by the copy-in instead of by copies inside every replayed step
            self.static_in = {k: v.detach().clone(memory_format=torch.contiguous_format) for k, v in data.items()}
        self._copy_in(data)
        if self._calls < self.warmup:
            # warm-up iterations are real steps, run on a side stream as graph capture requires
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.fn(self.static_in)
            torch.cuda.current_stream().wait_stream(s)
            self._calls += 1
            return out
        g = torch.cuda.CUDAGraph()
        quiesce_for_capture()
        with torch.cuda.graph(g, pool=self.pool, capture_error_mode=capture_error_mode()):
            self.static_out = self.fn(self.static_in)
        self.graph = g
        # capture recorded the work without executing it: run this step for real
        self.graph.replay()
        return self.static_out


class SegmentedGraph:
    """A step made of phases separated by collectives: each phase is captured in its own hipGraph
    (sharing one memory pool, so tensors handed from phase to phase keep their addresses) and the
    collectives run eagerly between replays.  Used for multi-rank training: RCCL calls never enter
    a captured graph, yet ~all kernels of the step are graph-launched.

    ``phases[i](data)`` may stash tensors on the owner for later phases; the last phase returns the
    step outputs.  ``colls[i]()`` runs between ``phases[i]`` and ``phases[i+1]``; ``colls[i](dry=True)``
    must only (re)bind the buffers the next phase reads (it is called between captures)."""

    def __init__(self, phases, colls, warmup: int = 2):
        assert len(colls) == len(phases) - 1
        self.phases, self.colls = phases, colls
        self.warmup = warmup
        self.graphs = None
        self.static_in: Optional[Dict[str, Tensor]] = None
        self.static_out = None
        self._calls = 0
        # opt-in per-phase timing (``enable_timing()``): hipEvents around every phase replay
        self.phase_ms = None
        self._events = None

    def enable_timing(self) -> None:
        self.phase_ms = [0.0] * len(self.phases)
        self.timed_steps = 0

    def _replay_all(self) -> None:
        timing = self.phase_ms is not None
        if timing and self._events is None:
            self._events = [torch.cuda.Event(enable_timing=True) for _ in range(2 * len(self.graphs))]
        for i, g in enumerate(self.graphs):
            if timing:
                self._events[2 * i].record()
            g.replay()
            if timing:
                self._events[2 * i + 1].record()
            if i < len(self.colls):
                self.colls[i]()
        if timing:
            torch.cuda.synchronize()
            for i in range(len(self.graphs)):
                self.phase_ms[i] += self._events[2 * i].elapsed_time(self._events[2 * i + 1])
            self.timed_steps += 1

    def replay_static(self) -> Optional[Dict[str, Tensor]]:
        """Replay the captured phases (and the collectives between them) on whatever the caller wrote into
        ``static_in``; None before the capture."""
        if self.graphs is None:
            return None
        self._replay_all()
        return self.static_out

    def _run_eager(self, data):
        out = None
        for i, ph in enumerate(self.phases):
            out = ph(data)
            if i < len(self.colls):
                self.colls[i]()
        return out

    def __call__(self, data: Dict[str, Tensor]):
        if self.static_in is None:
            self.static_in = {k: v.detach().clone(memory_format=torch.contiguous_format) for k, v in data.items()}
        for k, v in data.items():
            self.static_in[k].copy_(v, non_blocking=v.device.type != "cpu" or v.is_pinned())
        if self.graphs is not None:
            self._replay_all()
            return self.static_out
        if self._calls < self.warmup:
            self._calls += 1
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self._run_eager(self.static_in)
            torch.cuda.current_stream().wait_stream(s)
            return out
        quiesce_for_capture()
        graphs = []
        pool = None
        out = None
        for i, ph in enumerate(self.phases):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=capture_error_mode()):
                out = ph(self.static_in)
                # grads handed over by autograd must reach the flat slabs INSIDE this phase's graph:
                # the collective after it runs eagerly between replays
                gather_all_pending()
            pool = g.pool()
            graphs.append(g)
            if i < len(self.colls):
                self.colls[i](dry=True)  # re-bind hand-off buffers to the captured tensors
        self.graphs = graphs
        self.static_out = out
        # the captures recorded work without running it: execute this step for real
        for i, g in enumerate(self.graphs):
            g.replay()
            if i < len(self.colls):
                self.colls[i]()
        return self.static_out


class PhasedStep:
    """A training step given as ``phases`` separated by ``colls`` (gradient all-reduces etc.).

    * ``graphs`` and one rank: the whole step (phases + the no-op collectives) is ONE hipGraph;
    * ``graphs`` and N ranks: ``SegmentedGraph`` (per-phase graphs, collectives eagerly in between -
      no collective is ever captured);
    * otherwise eager.
    Phase/collective contract as in ``SegmentedGraph``."""

    def __init__(self, runner, phases, colls, graphs: bool = True, warmup: int = 2, name: str = "step",
                 force_segmented: bool = False):
        assert len(colls) == len(phases) - 1
        self.phases, self.colls = list(phases), list(colls)
        use = bool(graphs) and torch.cuda.is_available() and runner.device.type == "cuda"
        if not use:
            self.mode = "eager"
        elif runner.world_size > 1 or force_segmented:
            self.mode = "segmented"
            self._impl = SegmentedGraph(self.phases, self.colls, warmup=warmup)
        else:
            self.mode = "single"
            self._impl = GraphedStep(self._run, warmup=warmup, enabled=True, name=name)

    @property
    def enabled(self) -> bool:
        return self.mode != "eager"

    def _run(self, data):
        out = None
        for i, ph in enumerate(self.phases):
            out = ph(data)
            if i < len(self.colls):
                self.colls[i]()
        return out

    def captured_inputs(self) -> Optional[Dict[str, Tensor]]:
        """The static inputs of the captured single-graph step (write a batch into them, then ``replay()``);
        None before the capture or in the other modes."""
        if self.mode != "single" or self._impl.graph is None:
            return None
        return self._impl.static_in

    def replay(self) -> Optional[Dict[str, Tensor]]:
        """Replay the captured step on what the caller wrote into ``captured_inputs()`` (no copy-in)."""
        return self._impl.replay_static() if self.mode != "eager" else None

    def __call__(self, data: Dict[str, Tensor]):
        if self.mode == "eager":
            return self._run(data)
        return self._impl(data)
