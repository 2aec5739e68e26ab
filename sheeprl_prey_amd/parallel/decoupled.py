"""Decoupled actor-learner topology (reference C10: ``ppo/ppo_decoupled.py:586-633``,
``sac/sac_decoupled.py:501-542``).

rank 0 is the *player* (envs, rollouts/replay, GAE); ranks 1..N-1 are *trainers* that average
gradients over their own ``optimization`` group; trainer rank 1 sends the updated actor weights
back to the player over the ``player_trainer`` {0, 1} group.

Transport (MI355X-first): the reference pickles TensorDicts through ``scatter_object_list``.  Here
only a few-hundred-byte header (keys, shapes, dtypes) travels as an object over a gloo side group;
each trainer's chunk is packed into ONE contiguous byte tensor and sent point-to-point
(``dist.send``/``recv`` - RCCL P2P over xGMI on GPUs), and the actor weights are ONE flat fp32
broadcast.  Stop signal: a ``-1`` header (as in the reference).
"""
from __future__ import annotations

import copy
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

Meta = List[Tuple[str, Tuple[int, ...], str, int]]


def pack(chunk: Dict[str, Tensor]) -> Tuple[Tensor, Meta]:
    meta: Meta = []
    parts = []
    for k, v in chunk.items():
        v = v.contiguous()
        b = v.reshape(-1).view(torch.uint8)
        meta.append((k, tuple(v.shape), str(v.dtype).replace("torch.", ""), b.numel()))
        parts.append(b)
    return (torch.cat(parts) if len(parts) > 1 else parts[0]), meta


def unpack(buf: Tensor, meta: Meta) -> Dict[str, Tensor]:
    out, off = {}, 0
    for k, shape, dtype, n in meta:
        out[k] = buf[off : off + n].clone().view(getattr(torch, dtype)).view(shape)
        off += n
    return out


class DecoupledComm:
    def __init__(self, runner):
        if runner.world_size < 2:
            raise RuntimeError(
                "Please run the script with the number of devices greater than 1: "
                "`python sheeprl.py exp=<algo>_decoupled fabric.devices=2 ...`"
            )
        self.runner = runner
        self.rank = runner.global_rank
        self.world_size = runner.world_size
        backend = runner.backend
        # every rank creates every group, in the same order
        self.player_trainer_group = dist.new_group([0, 1], backend=backend)
        self.optimization_group = dist.new_group(list(range(1, self.world_size)), backend=backend)
        self.world_cpu = runner.cpu_group(None)
        self.pt_cpu = dist.new_group([0, 1], backend="gloo") if backend != "gloo" else self.player_trainer_group
        self.is_player = self.rank == 0

    # ------------------------------------------------------------------ roles
    def trainer_runner(self):
        """The runner trainers use: collectives (gradient all-reduce, metrics) over the
        optimisation group only."""
        r = copy.copy(self.runner)
        r.group = self.optimization_group
        r._loggers = []
        return r

    def _device(self) -> torch.device:
        return self.runner.device if self.runner.backend == "nccl" else torch.device("cpu")

    # ------------------------------------------------------------------ objects
    def broadcast_object_world(self, obj: Any = None, src: int = 0) -> Any:
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.world_cpu)
        return lst[0]

    def player_trainer_object(self, obj: Any = None) -> Any:
        """Trainer rank 1 -> player (metrics, checkpoint state)."""
        lst = [obj]
        dist.broadcast_object_list(lst, src=1, group=self.pt_cpu)
        return lst[0]

    # ------------------------------------------------------------------ data
    def send_chunks(self, chunks: Optional[List[Dict[str, Tensor]]]) -> None:
        """Player: one chunk per trainer (``None`` = stop signal)."""
        n_tr = self.world_size - 1
        if chunks is None:
            dist.scatter_object_list([None], [None] + [-1] * n_tr, src=0, group=self.world_cpu)
            return
        assert len(chunks) == n_tr, f"expected {n_tr} chunks, got {len(chunks)}"
        packed = [pack(c) for c in chunks]
        dist.scatter_object_list([None], [None] + [m for _, m in packed], src=0, group=self.world_cpu)
        dev = self._device()
        works = [dist.isend(buf.to(dev), dst=i + 1) for i, (buf, _) in enumerate(packed)]
        for w in works:
            w.wait()

    def recv_chunk(self) -> Optional[Dict[str, Tensor]]:
        """Trainer: receive this rank's chunk, or ``None`` on the stop signal."""
        out = [None]
        dist.scatter_object_list(out, None, src=0, group=self.world_cpu)
        meta = out[0]
        if isinstance(meta, int) and meta == -1:
            return None
        nbytes = sum(m[3] for m in meta)
        buf = torch.empty(nbytes, dtype=torch.uint8, device=self._device())
        dist.recv(buf, src=0)
        return {k: v.to(self.runner.device) for k, v in unpack(buf, meta).items()}

    # ------------------------------------------------------------------ weights
    def broadcast_params(self, flat: Tensor) -> Tensor:
        """Trainer rank 1 -> player: flat actor parameters (in place on the player)."""
        if self.runner.backend == "nccl":
            dist.broadcast(flat, src=1, group=self.player_trainer_group)
            return flat
        t = flat.detach().cpu() if flat.is_cuda else flat
        dist.broadcast(t, src=1, group=self.player_trainer_group)
        if t is not flat:
            flat.copy_(t)
        return flat


def params_to_vector(params) -> Tensor:
    return torch.cat([p.detach().reshape(-1) for p in params])


@torch.no_grad()
def vector_to_params(vec: Tensor, params) -> None:
    off = 0
    for p in params:
        n = p.numel()
        p.copy_(vec[off : off + n].view_as(p))
        off += n
