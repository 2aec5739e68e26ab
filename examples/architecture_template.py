"""Three-role distributed RL topology: 1 replay buffer, P players, T trainers (the reference's
``examples/architecture_template.py:35-195``, which moves pickled objects through Lightning
``TorchCollective`` groups).

Here every message is a fixed-shape tensor collective - no pickling on the hot path:

* rank 0            buffer : ``gather`` of the players' rollouts (buffer+players group), samples a
                             batch per trainer and ``scatter``s it (buffer+trainers group)
* ranks 1..P        players: receive the latest policy with ``broadcast`` from the last trainer
                             (players+last-trainer group), play, send their rollout to the buffer
* ranks P+1..P+T    trainers: data-parallel SGD; gradients ``all_reduce``d over the trainers group
                              (on GPUs that group is RCCL over xGMI; the buffer/player traffic stays on gloo)

Run (CPU):   python -m torch.distributed.run --nproc-per-node 5 --master-addr 127.0.0.1 \
                 examples/architecture_template.py --players 2 --trainers 2
"""
from __future__ import annotations

import argparse
import os
from datetime import timedelta

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

OBS, ROLLOUT, BATCH = 4, 8, 6


def player(rank: int, g_play: dist.ProcessGroup, g_params: dist.ProcessGroup, last_trainer: int, iters: int) -> None:
    policy = nn.Linear(OBS, 1)
    flat = torch.nn.utils.parameters_to_vector(policy.parameters()).detach()
    gen = torch.Generator().manual_seed(rank)
    for it in range(iters):
        dist.broadcast(flat, src=last_trainer, group=g_params)  # newest policy from the trainers
        torch.nn.utils.vector_to_parameters(flat, policy.parameters())
        obs = torch.randn(ROLLOUT, OBS, generator=gen)
        with torch.no_grad():
            act = policy(obs)
        rollout = torch.cat((obs, act), -1)  # [ROLLOUT, OBS+1]
        dist.gather(rollout, None, dst=0, group=g_play)
    print(f"[player {rank}] done, last policy norm {flat.norm():.4f}")


def buffer(g_play: dist.ProcessGroup, g_train: dist.ProcessGroup, n_players: int, n_trainers: int,
           iters: int) -> None:
    storage = []
    gen = torch.Generator().manual_seed(0)
    for it in range(iters):
        recv = [torch.empty(ROLLOUT, OBS + 1) for _ in range(n_players + 1)]
        dist.gather(torch.empty(ROLLOUT, OBS + 1), recv, dst=0, group=g_play)
        storage.extend(recv[1:])
        data = torch.cat(storage)
        idx = torch.randint(len(data), (n_trainers, BATCH), generator=gen)
        chunks = [torch.empty(BATCH, OBS + 1)] + [data[i] for i in idx]
        out = torch.empty(BATCH, OBS + 1)
        dist.scatter(out, chunks, src=0, group=g_train)
    print(f"[buffer] stored {sum(len(s) for s in storage)} transitions")


def trainer(rank: int, g_train: dist.ProcessGroup, g_opt: dist.ProcessGroup, g_params: dist.ProcessGroup,
            last_trainer: int, n_trainers: int, iters: int) -> None:
    torch.manual_seed(1)  # identical init on every trainer
    model = nn.Linear(OBS, 1)
    opt = torch.optim.SGD(model.parameters(), lr=0.1)
    for it in range(iters):
        if rank == last_trainer:
            flat = torch.nn.utils.parameters_to_vector(model.parameters()).detach().clone()
            dist.broadcast(flat, src=last_trainer, group=g_params)
        batch = torch.empty(BATCH, OBS + 1)
        dist.scatter(batch, None, src=0, group=g_train)
        loss = F.mse_loss(model(batch[:, :OBS]), batch[:, OBS:].sum(-1, keepdim=True) * 0.5)
        opt.zero_grad()
        loss.backward()
        grads = torch.cat([p.grad.flatten() for p in model.parameters()])  # one bucket
        dist.all_reduce(grads, group=g_opt)
        grads /= n_trainers
        off = 0
        for p in model.parameters():
            p.grad.copy_(grads[off:off + p.numel()].view_as(p))
            off += p.numel()
        opt.step()
    print(f"[trainer {rank}] final loss {loss.item():.4f}")


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--players", type=int, default=2)
    ap.add_argument("--trainers", type=int, default=2)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args(argv)
    P, T = a.players, a.trainers
    dist.init_process_group("gloo", timeout=timedelta(minutes=10))
    world, rank = dist.get_world_size(), dist.get_rank()
    if world != 1 + P + T:
        raise RuntimeError(f"Run with 1 + players + trainers = {1 + P + T} processes (got {world})")
    trainers = list(range(P + 1, P + T + 1))
    last = trainers[-1]
    # every rank creates every group, in the same order
    g_play = dist.new_group(list(range(P + 1)))
    g_train = dist.new_group([0] + trainers)
    g_opt = dist.new_group(trainers)
    g_params = dist.new_group(list(range(1, P + 1)) + [last])
    if rank == 0:
        buffer(g_play, g_train, P, T, a.iters)
    elif rank <= P:
        player(rank, g_play, g_params, last, a.iters)
    else:
        trainer(rank, g_train, g_opt, g_params, last, T, a.iters)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
