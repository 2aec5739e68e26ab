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

    def on_checkpoint_player(self, runner, ckpt_path: str, state: Dict[str, Any]) -> None:
        runner.save(ckpt_path, state)
        self._prune(runner, ckpt_path)

    def on_checkpoint_trainer(self, runner, player_trainer_group, ckpt_path: str, state: Dict[str, Any]) -> None:
        # trainer rank 1 ships its state to the player (rank 0), which writes it
        runner.send_object_to_player(state, player_trainer_group)

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
