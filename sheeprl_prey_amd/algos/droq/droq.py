"""DroQ (reference: ``sheeprl/algos/droq/droq.py:34-416``).

Per env step (after ``learning_starts``): ``per_rank_gradient_steps`` (20) critic updates on one
all-gathered sample of ``G*B`` transitions per rank, then one actor + alpha update on a second
all-gathered batch, with the actor maximising the MEAN of the Q ensemble.  Shares the SAC main
loop (``sac.run_sac_family``) and the captured ``SACTrainer`` updates.
"""
from __future__ import annotations

from typing import Any, Dict

from sheeprl_prey_amd.algos.sac.sac import SACTrainer, gather_and_shard, run_sac_family
from sheeprl_prey_amd.utils.registry import register_algorithm
from sheeprl_prey_amd.utils.timer import timer

_KEYS = ("observations", "next_observations", "actions", "rewards", "dones")


def droq_train_update(trainer: SACTrainer, runner, cfg, rb, update: int, learning_starts: int, aggregator) -> bool:
    if update <= learning_starts:
        return False
    B = cfg.per_rank_batch_size
    sample = rb.sample(cfg.algo.per_rank_gradient_steps * B, sample_next_obs=cfg.buffer.sample_next_obs)
    critic_data = gather_and_shard(runner, sample, cfg).to(runner.device)
    actor_data = gather_and_shard(runner, rb.sample(B), cfg).to(runner.device)
    n = trainer.agent.num_critics
    with timer("Time/train_time"):
        for start in range(0, critic_data.shape[0], B):
            batch = critic_data[start : start + B]
            d = {k: batch[k] for k in _KEYS}
            d["ema_w"] = trainer.ema_weight(True, d["rewards"].device)  # EMA after every critic update
            if d["rewards"].shape[0] != B and trainer.critic_step.enabled:
                trainer._critic_fwd_bwd(d)
                trainer._coll_critic()
                out = trainer._critic_apply(d)
            else:
                out = trainer.critic_step(d)
            # the reference logs each critic's own MSE; the ensemble loss is their sum
            aggregator.update("Loss/value_loss", out["Loss/value_loss"] / n)
        obs = actor_data["observations"][:B]
        if obs.shape[0] != B and trainer.actor_step.enabled:
            trainer._actor_fwd_bwd({"observations": obs})
            trainer._coll_actor()
            out = trainer._actor_apply({})
        else:
            out = trainer.actor_step({"observations": obs})
        aggregator.update("Loss/policy_loss", out["Loss/policy_loss"])
        aggregator.update("Loss/alpha_loss", out["Loss/alpha_loss"])
    return True


@register_algorithm()
def main(runner, cfg: Dict[str, Any]):
    run_sac_family(runner, cfg, variant="droq")
