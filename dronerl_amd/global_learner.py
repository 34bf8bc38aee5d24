"""One global learner over env shards (the reference's sharded train run).

Reference: train_jax.py:196-212 shards the env state over devices, but the
scan body (:38-115) still has ONE replay ring (jax_impl/buffers.py:57-90,
add_many of all num_envs drone-0 transitions per step, slot = transition
index mod capacity) and ONE train_step per step on batch rows sampled from
it.  Each rank here keeps the learner and a full-capacity image of that
global ring, but writes only its own envs' transitions, at their global slots
(`shard_add_plan`).  Before each learner step every rank draws the same
global slots (drl_dqn_sample_rows: the learner's own counter hash), works out
which rank wrote each slot last (`slot_owner`), and one all_gather of the
`batch` packed rows (8 rows x (2 x 128 B codes + 12 B) ~= 2 KB at train_jax's
defaults; RCCL over xGMI, or gloo) hands every rank the owners' rows, which it
scatters into its image at those slots.  Every rank then runs the identical,
bit-reproducible drl_dqn_train, so every rank's parameters, Adam moments and
counters equal a one-process learner over the concatenated envs, bit for bit.

The exchange is latency-bound (a few KB per step); the env step itself still
has no collective.  This module never reads the oracle.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def shard_add_plan(n_total: int, capacity: int, num_envs_total: int, env_offset: int,
                   shard_envs: int) -> Tuple[int, int]:
    """One global add_many of num_envs_total transitions (env e has global
    transition index n_total + e): of this shard's rows (envs env_offset ..
    env_offset + shard_envs - 1) the rows lo.. land in the ring, row lo at
    slot `cursor` and the rest after it (an add of more rows than capacity
    keeps only its last capacity rows, buffers.py:57-80).  lo == shard_envs:
    none land."""
    first = max(0, num_envs_total - capacity)
    lo = min(shard_envs, max(0, first - env_offset))
    return lo, (n_total + env_offset + lo) % capacity


def slot_owner(slots: torch.Tensor, n_total: int, capacity: int, num_envs_total: int, world: int) -> torch.Tensor:
    """The rank whose env wrote each global slot last: the latest transition
    index i < n_total with i = slot (mod capacity) belongs to env i mod
    num_envs_total, in the contiguous shard (env // (num_envs_total / world))."""
    i = (n_total - 1) - torch.remainder((n_total - 1) - slots, capacity)
    return torch.div(torch.remainder(i, num_envs_total), num_envs_total // world, rounding_mode="floor")


def exchange_rows(packed: torch.Tensor, owner: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """Every rank's packed rows [B, K] (int32 words) -> row b of rank owner[b],
    on every rank (one all_gather; bit-exact whatever the row holds)."""
    if world == 1:
        return packed
    import torch.distributed as dist
    cpu = dist.get_backend(group) == "gloo"
    src = (packed.cpu() if cpu else packed).contiguous()
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    stacked = torch.stack(parts).to(packed.device)
    return stacked[owner.to(packed.device), torch.arange(packed.shape[0], device=packed.device)]


class ShardedReplay:
    """This rank's image of the one global replay ring (see the module
    docstring).  `add_many` takes this shard's rows exactly as
    ReplayBuffer.add_many does; `gather(learner)` runs before each
    `learner.train(self.ring)`."""

    def __init__(self, capacity: int, obs_floats: int, device, num_envs_total: int, env_offset: int,
                 shard_envs: int, rank: int, world: int, code_radius: int = 0, group=None):
        from .dqn import ReplayBuffer
        if world < 1 or num_envs_total % world or shard_envs * world != num_envs_total:
            raise ValueError("shards must split num_envs_total evenly (train_jax.py:401-402)")
        if env_offset != rank * shard_envs:
            raise ValueError("env_offset must be rank * shard_envs (contiguous shards)")
        self.ring = ReplayBuffer(capacity, obs_floats, device, code_radius=code_radius)
        self.capacity, self.E, self.off, self.Er = capacity, num_envs_total, env_offset, shard_envs
        self.rank, self.world, self.group = rank, world, group
        self.n_total = 0
        self.exchanged_bytes = 0  # per gather, for the record

    @property
    def size(self) -> int:
        return self.ring.size

    def add_many(self, obs, actions, rewards, next_obs, dones):
        lo, cur = shard_add_plan(self.n_total, self.capacity, self.E, self.off, self.Er)
        if obs.shape[0] != self.Er:
            raise ValueError(f"a shard's add carries its {self.Er} envs' rows")
        if lo < self.Er:
            self.ring.cursor = cur
            self.ring.add_many(obs[lo:], actions[lo:], rewards[lo:], next_obs[lo:], dones[lo:])
        self.n_total += self.E
        self.ring.cursor = self.n_total % self.capacity
        self.ring.size = min(self.n_total, self.capacity)

    def _pack(self, slots: torch.Tensor) -> torch.Tensor:
        r = self.ring
        B = slots.shape[0]
        o = r.obs[slots].reshape(B, -1).view(torch.int32)
        no = r.next_obs[slots].reshape(B, -1).view(torch.int32)
        return torch.cat([o, no, r.actions[slots].view(B, 1), r.rewards[slots].view(torch.int32).view(B, 1),
                          r.dones[slots].to(torch.int32).view(B, 1)], dim=1)

    def _unpack(self, slots: torch.Tensor, rows: torch.Tensor):
        r = self.ring
        B = slots.shape[0]
        w = r.obs.shape[1] * r.obs.element_size() // 4
        r.obs[slots] = rows[:, :w].contiguous().view(r.obs.dtype).view(B, -1)
        r.next_obs[slots] = rows[:, w:2 * w].contiguous().view(r.obs.dtype).view(B, -1)
        r.actions[slots] = rows[:, 2 * w]
        r.rewards[slots] = rows[:, 2 * w + 1].contiguous().view(torch.float32)
        r.dones[slots] = rows[:, 2 * w + 2].to(torch.uint8)

    def gather(self, learner, slots: Optional[torch.Tensor] = None):
        """Land in this image, at the slots the learner's next step draws,
        the rows their owners hold (nothing when the ring cannot sample yet:
        buffers.py can_sample; nothing to do on one rank)."""
        if self.world == 1 or self.ring.size < learner.hp.batch:
            return
        if slots is None:
            slots = learner.sample_slots(self.ring.size)
        owner = slot_owner(slots, self.n_total, self.capacity, self.E, self.world)
        packed = self._pack(slots)
        self.exchanged_bytes = packed.numel() * 4 * self.world
        self._unpack(slots, exchange_rows(packed, owner, self.world, self.group))
