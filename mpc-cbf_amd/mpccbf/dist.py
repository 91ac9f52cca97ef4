"""Multi-GPU sharding of the swarm: one process per GPU, agents in contiguous blocks.

Each rank owns agents [first, first + count) and solves their QPs; the only exchange is one
all-gather of the 6-double agent states per control step (iteration 1 of the IMPC
loop uses the neighbours' *current* states, ConnectivityIMPCCBF.cpp:174, so no second exchange).
Backend "nccl" is RCCL over xGMI on the MI355X node; "gloo" runs the same code on CPU tensors for
the world-size-2 tests.

Buffers (no copies on the step path):
  world == 1: two full state tables used ping-pong — the solver reads `full` and writes the next
              states straight into `next_out` (the other table); publish() swaps them.
  world  > 1: the solver writes its block's next states into `next_out` (= `local`), publish()
              all-gathers every rank's block into `full`.
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
    """This rank's slice of the swarm plus the full state table the neighbours come from."""

    def __init__(self, full_states: torch.Tensor, world: int = 1, rank: int = 0, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.first, self.count = shard(full_states.shape[0], world, rank)
        if world == 1:
            self._tables = [full_states, full_states.clone()]
            self._cur = 0
        else:
            self._full = full_states
            self.local = full_states[self.first:self.first + self.count].clone()
            self._gloo = dist.get_backend(group) == "gloo"
            if self._gloo:
                self._parts = list(torch.chunk(self._full, world, dim=0))

    @property
    def full(self) -> torch.Tensor:
        """Every agent's current state (total x 6): the solver's input."""
        return self._tables[self._cur] if self.world == 1 else self._full

    @property
    def next_out(self) -> torch.Tensor:
        """Where the solver writes this rank's next states (count x 6)."""
        return self._tables[1 - self._cur] if self.world == 1 else self.local

    def publish(self) -> None:
        """Make the next states current: swap tables, or all-gather the blocks (one collective
        per control step)."""
        if self.world == 1:
            self._cur = 1 - self._cur
        elif self._gloo:
            # gloo has no all_gather_into_tensor; the chunks are views of `full`
            dist.all_gather(self._parts, self.local, group=self.group)
        else:
            dist.all_gather_into_tensor(self._full, self.local, group=self.group)

    def step(self, solve) -> None:
        """One control step: solve(full, first, count, out=next_out) writes this rank's next
        states into next_out (no copy), then publish()."""
        solve(self.full, self.first, self.count, out=self.next_out)
        self.publish()
