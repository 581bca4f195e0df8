"""Multi-GPU rollouts: env shards per rank, one gather of transitions per rollout.

The env batch partitions embarrassingly: rank r of G
owns the contiguous env ids [offset_r, offset_r + count_r) (multiples of 32);
because the RNG is keyed by global env id, the union of the shards is
bit-identical to a single-GPU run of all envs.  There is no exchange inside a
step.  The only collective is the hand-off of a rollout's transitions to the
learner: one ``all_gather_into_tensor`` (RCCL over xGMI on MI355X, gloo in
the CPU tests) of a packed int32 record buffer per rollout of T steps.

Record layout per step and env (int32 rows, W = state words):
    obs[W] (state before the step) | action_mask[W] | next_state[W] (s') |
    reward (float32 bits) | flags
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

__all__ = ["shard_range", "record_rows", "ShardedRollout"]


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


def record_rows(words: int) -> int:
    return 3 * words + 2


class ShardedRollout:
    """Drive one env shard per rank and gather (s, a, r, s', flags) every rollout.

    ``env_factory(env_offset, count)`` builds the shard's env (VectorPBNEnv on the
    rank's GPU in production; any object with the same step_flipmask/state/
    flipmask/final_state/words attributes in tests).  Shards must be equal-sized
    (all_gather_into_tensor), i.e. n_total / 32 divisible by the world size.
    """

    def __init__(self, n_total: int, env_factory: Callable[[int, int], object],
                 group: Optional[dist.ProcessGroup] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_total = n_total
        self.offset, self.count = shard_range(n_total, self.world, self.rank)
        if (n_total // 32) % self.world:
            raise ValueError("equal shards required: (n_total/32) must divide by the world size")
        self.env = env_factory(self.offset, self.count)
        self.words = self.env.words

    def rollout(self, steps: int, random_actions: bool = True, policy=None) -> torch.Tensor:
        """Run ``steps`` transitions on the local shard; returns int32 [steps, rows, count]."""
        W, n = self.words, self.count
        env = self.env
        rec = torch.empty((steps, record_rows(W), n), dtype=torch.int32, device=env.state.device)
        if policy is None and hasattr(env, "rollout"):
            # one pbn_rollout launch for the whole rollout (state kept on chip between steps)
            out = env.rollout(steps, random_actions=random_actions, keep_obs=True, keep_final=True)
            rec[:, 0:W] = out["obs"][:, :, :n]
            rec[:, W:2 * W] = out["flipmask"][:, :, :n]
            rec[:, 2 * W:3 * W] = out["final_state"][:, :, :n]
            rec[:, 3 * W] = out["reward"][:, :n].view(torch.int32)
            rec[:, 3 * W + 1] = out["flags"][:, :n].to(torch.int32)
            return rec
        for k in range(steps):
            rec[k, 0:W] = env.state[:, :n]
            if policy is not None:
                fm = policy(env.state[:, :n])
                state, reward, flags = env.step_flipmask(fm)
            else:
                state, reward, flags = env.step_flipmask(None, random_actions=random_actions)
            rec[k, W:2 * W] = env.flipmask[:, :n]
            rec[k, 2 * W:3 * W] = env.final_state[:, :n]
            rec[k, 3 * W] = reward.view(torch.int32)
            rec[k, 3 * W + 1] = flags.to(torch.int32)
        return rec

    def gather(self, rec: torch.Tensor) -> torch.Tensor:
        """All ranks receive [world, steps, rows, count]: env id of [r, :, :, i] is
        offset_r + i (rank-major = global env order)."""
        if self.world == 1:
            return rec[None]
        flat = torch.empty((self.world * rec.shape[0],) + tuple(rec.shape[1:]), dtype=rec.dtype,
                           device=rec.device)
        dist.all_gather_into_tensor(flat, rec.contiguous(), group=self.group)
        return flat.view((self.world,) + tuple(rec.shape))

    @staticmethod
    def to_global(gathered: torch.Tensor) -> torch.Tensor:
        """[world, steps, rows, count] -> [steps, rows, world*count] in global env order."""
        w, s, r, c = gathered.shape
        return gathered.permute(1, 2, 0, 3).reshape(s, r, w * c)
