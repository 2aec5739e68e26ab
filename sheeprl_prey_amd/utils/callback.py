"""Checkpoint hooks (reference: ``sheeprl/utils/callback.py:9-88``).

Checkpoints are plain ``torch.save`` dicts of state_dicts/ints/tensors (loadable with
``weights_only=True``).  Replay buffers are stored through their ``state_dict()`` - a dict of
tensors - instead of a pickled object; with world_size>1 the per-rank buffers are gathered
to rank 0 as a list (the reference's ``gather_object``), and the write head is temporarily
marked ``done`` so episodes are truncated consistently on resume.
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch


def _mark_truncated(rb) -> list:
    """Set dones=1 at the last written row of every env buffer; return what to restore."""
    restore = []
    for buf in getattr(rb, "buffers_for_checkpoint", lambda: [rb])():
        if buf is None or buf.empty or "dones" not in buf.keys():
            continue
        idx = (buf._pos - 1) % buf.buffer_size
        old = buf["dones"][idx].clone()
        buf["dones"][idx] = torch.ones_like(old)
        restore.append((buf, idx, old))
    return restore


def _to_cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


class CheckpointCallback:
    def __init__(self, keep_last: Optional[int] = None):
        self.keep_last = keep_last

    def on_checkpoint_coupled(self, runner, ckpt_path: str, state: Dict[str, Any], replay_buffer=None) -> None:
        restore = []
        if replay_buffer is not None:
            restore = _mark_truncated(replay_buffer)
            rb_state = replay_buffer.state_dict()
            if runner.world_size > 1:
                gathered = runner.gather_object(rb_state, dst=0)
                state["rb"] = gathered if runner.is_global_zero else None
            else:
                state["rb"] = rb_state
        runner.save(ckpt_path, state)
        for buf, idx, old in restore:
            buf["dones"][idx] = old
        if replay_buffer is not None:
            state.pop("rb", None)
        self._prune(runner, ckpt_path)

    def on_checkpoint_player(self, runner, comm, ckpt_path: str, replay_buffer=None) -> None:
        """Decoupled player (rank 0): receive the trainers' state from trainer rank 1, add the
        replay buffer and write the checkpoint (reference ``callback.py:68-88``)."""
        state = comm.player_trainer_object(None)
        restore = []
        if replay_buffer is not None:
            restore = _mark_truncated(replay_buffer)
            state["rb"] = replay_buffer.state_dict()
        path = ckpt_path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        tmp = path + ".tmp"
        torch.save(state, tmp)
        os.replace(tmp, path)
        for buf, idx, old in restore:
            buf["dones"][idx] = old
        self._prune(runner, ckpt_path)

    def on_checkpoint_trainer(self, runner, comm, state: Dict[str, Any]) -> None:
        """Decoupled trainer rank 1 ships its state to the player, which writes it."""
        comm.player_trainer_object(_to_cpu(state))

    def _prune(self, runner, ckpt_path: str) -> None:
        if not self.keep_last or not runner.is_global_zero:
            return
        d = os.path.dirname(ckpt_path)
        ck = sorted((f for f in os.listdir(d) if f.endswith(".ckpt")), key=lambda f: os.path.getmtime(os.path.join(d, f)))
        for f in ck[: -self.keep_last]:
            try:
                os.remove(os.path.join(d, f))
            except OSError:
                pass
