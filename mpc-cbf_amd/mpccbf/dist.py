"""Multi-GPU sharding of the swarm: one process per GPU, agents in contiguous blocks.

Each rank owns agents [first, first + count) and solves their QPs; the only exchange is one
all-gather of the 6-double agent states per control step (iteration 1 of the IMPC
loop uses the neighbours' *current* states, ConnectivityIMPCCBF.cpp:174, so no second exchange).
Backend "nccl" is RCCL over xGMI on the MI355X node; "gloo" runs the same code on CPU tensors for
the world-size-2 tests.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block of agents for `rank`: (first, count). Agents must divide evenly."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} / world {world}")
    per = total // world
    if per * world != total:
        raise ValueError(f"{total} agents do not divide over {world} ranks")
    return rank * per, per


class SwarmShard:
    """This rank's slice of the swarm plus the gathered full state table.

    full   (total x 6) every agent's state, refreshed by exchange() — the neighbour source
    local  (count x 6) this rank's agents, written by the solver's closed-loop update
    """

    def __init__(self, full_states: torch.Tensor, world: int = 1, rank: int = 0, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.first, self.count = shard(full_states.shape[0], world, rank)
        self.full = full_states
        self.local = full_states[self.first:self.first + self.count].clone()
        self._gloo = world > 1 and dist.get_backend(group) == "gloo"
        if self._gloo:
            self._parts = list(torch.chunk(self.full, world, dim=0))

    def exchange(self) -> None:
        """All-gather of local states into `full` (one collective per control step)."""
        if self.world == 1:
            self.full.copy_(self.local)
        elif self._gloo:
            # gloo has no all_gather_into_tensor; the chunks are views of `full`
            dist.all_gather(self._parts, self.local, group=self.group)
        else:
            dist.all_gather_into_tensor(self.full, self.local, group=self.group)

    def step(self, solve) -> None:
        """One control step: exchange, then solve(full, first, count) -> next local states."""
        self.exchange()
        nxt = solve(self.full, self.first, self.count)
        self.local.copy_(nxt)
