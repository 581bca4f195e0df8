"""Multi-GPU rollouts: env shards per rank, one gather of transitions per rollout.

The env batch partitions embarrassingly: rank r of G
owns the contiguous env ids [offset_r, offset_r + count_r) (multiples of 32);
because the RNG is keyed by global env id, the union of the shards is
bit-identical to a single-GPU run of all envs.  There is no exchange inside a
step.  The only collective is the hand-off of a rollout's transitions to the
learner: one ``all_gather_into_tensor`` (RCCL over xGMI on MI355X, gloo in
the CPU tests) of the shard's record buffer per rollout of T steps.

Wire format (``TransitionRecords``): one flat byte buffer per shard and rollout,
field-major so that ``pbn_rollout`` writes every field in place (no packing
copies before the collective), (12W + 5) bytes per env-step -- 17 B for
Bittner-28:

    obs     u32 [T][W][n]   state before the step (s)
    action  u32 [T][W][n]   flip mask applied (a)
    next    u32 [T][W][n]   state after the step, before any autoreset (s')
    reward  f32 [T][n]      (r)
    flags   u8  [T][n]      TERMINATED | TRUNCATED | IN_ATTRACTOR | PERTURBED | RESET
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["shard_range", "record_bytes_per_env_step", "TransitionRecords", "ShardedRollout"]


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """(env_offset, count) of rank's contiguous shard; counts are multiples of 32
    and differ by at most 32 between ranks."""
    if n_total % 32:
        raise ValueError("total env count must be a multiple of 32")
    groups = n_total // 32
    base, extra = divmod(groups, world)
    start = rank * base + min(rank, extra)
    count = base + (1 if rank < extra else 0)
    return 32 * start, 32 * count


def record_bytes_per_env_step(words: int) -> int:
    return 12 * words + 5


_FIELDS = (("obs", torch.int32, True), ("flipmask", torch.int32, True), ("final_state", torch.int32, True),
           ("reward", torch.float32, False), ("flags", torch.uint8, False))


class TransitionRecords:
    """The records of one rollout of ``steps`` steps over ``n`` envs (a multiple of 32), as
    typed views into one flat uint8 buffer (the gather's wire format, module docstring)."""

    def __init__(self, steps: int, words: int, n: int, device=None, flat: Optional[torch.Tensor] = None):
        if n % 32:
            raise ValueError("n must be a multiple of 32")
        self.steps, self.words, self.n = int(steps), int(words), int(n)
        nbytes = self.nbytes(self.steps, self.words, self.n)
        if flat is None:
            flat = torch.empty(nbytes, dtype=torch.uint8, device=device)
        if flat.dtype != torch.uint8 or flat.numel() != nbytes or not flat.is_contiguous():
            raise ValueError(f"flat must be a contiguous uint8 tensor of {nbytes} bytes")
        self.flat = flat
        self.fields: Dict[str, torch.Tensor] = {}
        off = 0
        T, W = self.steps, self.words
        for name, dtype, per_word in _FIELDS:
            shape = (T, W, n) if per_word else (T, n)
            size = torch.empty((), dtype=dtype).element_size()
            count = T * (W if per_word else 1) * n
            self.fields[name] = flat[off:off + count * size].view(dtype).view(shape)
            off += count * size

    @staticmethod
    def nbytes(steps: int, words: int, n: int) -> int:
        return steps * n * record_bytes_per_env_step(words)

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.fields[name]

    def rollout_out(self) -> dict:
        """The ``out=`` dict of ``VectorPBNEnv.rollout``: the kernel writes the fields in place."""
        d = dict(self.fields)
        d["_n_steps"] = self.steps
        return d


class ShardedRollout:
    """Drive one env shard per rank and gather (s, a, s', r, flags) every rollout.

    ``env_factory(env_offset, count)`` builds the shard's env (VectorPBNEnv on the
    rank's GPU in production; any object with the same ``rollout`` contract in tests).
    Shards must be equal-sized (all_gather_into_tensor), i.e. n_total / 32 divisible by the
    world size.
    """

    def __init__(self, n_total: int, env_factory: Callable[[int, int], object],
                 group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_total = n_total
        if (n_total // 32) % self.world:
            raise ValueError("equal shards required: (n_total/32) must divide by the world size")
        self.offset, self.count = shard_range(n_total, self.world, self.rank)
        self.env = env_factory(self.offset, self.count)
        self.words = self.env.words
        self._rec: Optional[TransitionRecords] = None
        self._all: Optional[torch.Tensor] = None

    def rollout(self, steps: int, random_actions: bool = True, flipmasks: Optional[torch.Tensor] = None
                ) -> TransitionRecords:
        """``steps`` transitions on the local shard, in one ``rollout`` call whose outputs land
        directly in the record buffer (reused across calls of the same length)."""
        dev = getattr(self.env, "device", None) or self.env.state.device
        if self._rec is None or self._rec.steps != steps:
            self._rec = TransitionRecords(steps, self.words, self.count, device=dev)
        self.env.rollout(steps, flipmasks=flipmasks, random_actions=random_actions, keep_obs=True,
                         keep_final=True, out=self._rec.rollout_out())
        return self._rec

    def gather(self, rec: TransitionRecords) -> List[TransitionRecords]:
        """One ``all_gather_into_tensor`` of the flat record buffers; every rank receives the
        records of every rank (rank r's envs are offset_r + i: rank-major = global order)."""
        if not dist.is_initialized():
            return [rec]
        nbytes = rec.flat.numel()
        if self._all is None or self._all.numel() != self.world * nbytes or self._all.device != rec.flat.device:
            self._all = torch.empty(self.world * nbytes, dtype=torch.uint8, device=rec.flat.device)
        dist.all_gather_into_tensor(self._all, rec.flat, group=self.group)
        return [TransitionRecords(rec.steps, rec.words, rec.n, flat=self._all[r * nbytes:(r + 1) * nbytes])
                for r in range(self.world)]

    @staticmethod
    def to_global(parts: List[TransitionRecords]) -> Dict[str, torch.Tensor]:
        """Per-rank records -> per-field tensors over all envs in global order (env = last axis)."""
        return {name: torch.cat([p[name] for p in parts], dim=-1) for name, _, _ in _FIELDS}
