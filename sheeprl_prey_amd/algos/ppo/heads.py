"""Categorical policy heads: sample / log-prob / entropy for every action head, summed over
heads (reference ``ppo/agent.py:154-178``).  One logits->log_softmax pass per head; sampling by
Gumbel-max on the log-probs (distributionally identical to ``Categorical.sample``)."""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor


def categorical_heads(logits_list: Sequence[Tensor], actions: Optional[Sequence[Tensor]] = None) -> Tuple[Tuple[Tensor, ...], Tensor, Tensor]:
    acts: List[Tensor] = []
    logps: List[Tensor] = []
    ents: List[Tensor] = []
    for i, logits in enumerate(logits_list):
        logp_all = F.log_softmax(logits, dim=-1)
        if actions is None:
            with torch.no_grad():
                g = -torch.log(-torch.log(torch.rand_like(logp_all).clamp_(1e-20, 1.0)))
                idx = (logp_all + g).argmax(-1)
                a = F.one_hot(idx, logits.shape[-1]).to(logits.dtype)
        else:
            a = actions[i]
        acts.append(a)
        logps.append((logp_all * a).sum(-1))
        ents.append(-(logp_all.exp() * logp_all).sum(-1))
    return tuple(acts), torch.stack(logps, -1).sum(-1, keepdim=True), torch.stack(ents, -1).sum(-1, keepdim=True)
