"""DreamerV1 helpers (reference: ``sheeprl/algos/dreamer_v1/utils.py:10-74``)."""
from __future__ import annotations

from torch import Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.algos.dreamer_v1.agent import compute_stochastic_state  # noqa: F401
from sheeprl_prey_amd.algos.dreamer_v2.utils import test  # noqa: F401


def compute_lambda_values(rewards: Tensor, values: Tensor, done_mask: Tensor, last_values: Tensor, horizon: int = 15,
                          lmbda: float = 0.95) -> Tensor:
    """``horizon-1`` TD(lambda) targets bootstrapped on ``last_values`` (= values[horizon-1]):
    ``R_t = r_t + c_t ((1-lambda) v_{t+1} + lambda R_{t+1})`` - the fused reverse scan."""
    next_values = values[1:horizon].clone()
    next_values[-1] = last_values
    return ops.lambda_returns(rewards[: horizon - 1], next_values, done_mask[: horizon - 1], lmbda)
