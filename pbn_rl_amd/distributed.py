"""Multi-GPU rollouts: env shards per rank, one gather of transitions per rollout.

The env batch partitions embarrassingly: rank r of G
owns the contiguous env ids [offset_r, offset_r + count_r) (multiples of 32);
because the RNG is keyed by global env id, the union of the shards is
bit-identical to a single-GPU run of all envs.  There is no exchange inside a
step.  The only collective is the hand-off of a rollout's transitions to the
learner, once per rollout of T steps (RCCL over xGMI on MI355X, gloo in the CPU
tests), in one of two forms:

  * ``dst=r`` (the learner's rank): every other rank sends its record buffer to
    rank r point to point (``batch_isend_irecv``); rank r keeps its own records
    where the kernel wrote them.  Each rank's link to the learner carries its own
    shard only, the 7 x 153 GB/s fan-in SURVEY.md 8(e) prices (17 B per env-step:
    ~6.3e10 env-steps/s delivered across 8 GPUs);
  * ``dst=None``: ``all_gather_into_tensor``, every rank receives every shard.

``ShardedRollout.run`` overlaps the hand-off with the next rollout: records live
in a ring of ``buffers`` slots (two by default), the collective of rollout k is
issued asynchronously behind rollout k on the communicator's own stream, and
rollout k + buffers waits (stream-side, no host sync) only for the collective
that last read its slot.  With one slot there is nothing to overlap: each
rollout is consumed before the next one overwrites the slot.

``gather(rec, dst, copy_own=True)`` also copies the learner's own shard into its
receive slot, so that every shard ends in a learner-owned buffer; at world 1 that
copy is the whole hand-off (bench.py's ``value_with_gather``).  On a GPU env it
rides along the next rollout launch (``pbn_rollout_copy``: a fourth wave per block
of the rollout kernel), overlapped like the collective; CPU tensors or envs without
``copy=`` get a side-stream copy.

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
        if getattr(self, "_out", None) is None:
            self._out = dict(self.fields)
            self._out["_n_steps"] = self.steps
        return self._out


class ShardedRollout:
    """Drive one env shard per rank and hand (s, a, s', r, flags) to the learner every rollout.

    ``env_factory(env_offset, count)`` builds the shard's env (VectorPBNEnv on the
    rank's GPU in production; any object with the same ``rollout`` contract in tests).
    Shards must be equal-sized, i.e. n_total / 32 divisible by the world size.

    Records are a ring of ``buffers`` TransitionRecords per rollout length: the records a
    ``rollout`` returns stay valid until ``buffers`` further rollouts of that length have been
    issued; received records (``gather``) likewise live in a ring of ``buffers`` receive slots.
    Callers that keep records longer copy them out (e.g. into a replay ring).
    """

    def __init__(self, n_total: int, env_factory: Callable[[int, int], object],
                 group: Optional[dist.ProcessGroup] = None, buffers: int = 2):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.n_total = n_total
        if (n_total // 32) % self.world:
            raise ValueError("equal shards required: (n_total/32) must divide by the world size")
        if buffers < 1:
            raise ValueError("buffers must be >= 1")
        self.buffers = int(buffers)
        self.offset, self.count = shard_range(n_total, self.world, self.rank)
        self.env = env_factory(self.offset, self.count)
        self.words = self.env.words
        self._ring: Dict[int, List[TransitionRecords]] = {}
        self._recv: Dict[Tuple[int, Optional[int]], List[torch.Tensor]] = {}
        self._pending: Dict[int, List[Optional[object]]] = {}   # slot -> the collective reading it
        self._issued: Dict[int, int] = {}
        self._gathered: Dict[Tuple[int, Optional[int]], int] = {}

    @property
    def _device(self):
        return getattr(self.env, "device", None) or self.env.state.device

    def _slot(self, steps: int) -> int:
        return self._issued.get(steps, 0) % self.buffers

    def rollout(self, steps: int, random_actions: bool = True, flipmasks: Optional[torch.Tensor] = None
                ) -> TransitionRecords:
        """``steps`` transitions on the local shard, in one ``rollout`` call whose outputs land
        directly in the next record slot of the ring.  If an asynchronous hand-off of that slot
        is still in flight, the rollout is ordered after it on the device (work.wait())."""
        ring = self._ring.setdefault(steps, [])
        k = self._slot(steps)
        if len(ring) <= k:
            ring.append(TransitionRecords(steps, self.words, self.count, device=self._device))
        rec = ring[k]
        pend = self._pending.setdefault(steps, [None] * self.buffers)
        if pend[k] is not None:
            _wait(pend[k])
            pend[k] = None
        ride = self._take_ride(rec)
        kw = {"copy": (ride.dst, ride.src)} if ride is not None else {}
        self.env.rollout(steps, flipmasks=flipmasks, random_actions=random_actions, keep_obs=True,
                         keep_final=True, out=rec.rollout_out(), **kw)
        if ride is not None:   # complete when this launch is (a launch that raised leaves it to
            ride.carried()     # the hand-off's wait())
        self._issued[steps] = self._issued.get(steps, 0) + 1
        rec._slot = k
        return rec

    def gather(self, rec: TransitionRecords, dst: Optional[int] = None, async_op: bool = False,
               copy_own: bool = False, last: bool = False):
        """Hand the records of one rollout to the learner.

        dst = None: ``all_gather_into_tensor``; every rank receives every rank's records
        (rank r's envs are offset_r + i: rank-major = global order).  dst = r: point-to-point
        sends to rank r; rank r receives the other shards and uses its own in place (or, with
        ``copy_own``, copies it into its receive slot too), the other ranks receive nothing (an
        empty list).  Returns the list of per-rank records (valid until ``buffers`` further
        gathers of this shape and form) or, with async_op, (records, work): the records are
        readable on the current stream after ``work.wait()``.

        ``last``: nothing follows this hand-off to overlap with, so the own-shard copy is issued on
        the current stream (no cross-stream wait: the side stream's wait on the rollout's event
        cost ~11 us of idle device time per hand-off, profiles/r05_a_handoff_summary.json).
        """
        if (dst is None or not copy_own) and not dist.is_initialized():
            # one process without a process group: its records are the whole batch
            return ([rec], None) if async_op else [rec]
        if dst is not None and not copy_own and self.world == 1:
            # the learner's own shard: already where the kernel wrote it (all_gather still runs
            # at world 1, so the collective path is exercised on a one-GPU box)
            return ([rec], None) if async_op else [rec]
        nbytes = rec.flat.numel()
        key = (rec.steps, dst, copy_own)
        recv = self._recv.setdefault(key, [])
        k = self._gathered.get(key, 0) % self.buffers
        self._gathered[key] = self._gathered.get(key, 0) + 1
        if dst is None:
            if len(recv) <= k:
                recv.append(torch.empty(self.world * nbytes, dtype=torch.uint8, device=rec.flat.device))
            out = recv[k]
            work = _Works([dist.all_gather_into_tensor(out, rec.flat, group=self.group, async_op=True)])
            parts = [TransitionRecords(rec.steps, rec.words, rec.n, flat=out[r * nbytes:(r + 1) * nbytes])
                     for r in range(self.world)]
        else:
            gdst = (dist.get_global_rank(self.group, dst) if self.group is not None else dst) if self.world > 1 else dst
            works = []
            if self.rank == dst:
                if len(recv) <= k:
                    recv.append(torch.empty(self.world * nbytes, dtype=torch.uint8, device=rec.flat.device))
                out = recv[k]
                ops = [dist.P2POp(dist.irecv, out[r * nbytes:(r + 1) * nbytes],
                                  dist.get_global_rank(self.group, r) if self.group is not None else r, self.group)
                       for r in range(self.world) if r != dst]
                if copy_own:
                    works.append(self._copy_own(out[dst * nbytes:(dst + 1) * nbytes], rec.flat, last))
                parts = [rec if (r == dst and not copy_own) else
                         TransitionRecords(rec.steps, rec.words, rec.n, flat=out[r * nbytes:(r + 1) * nbytes])
                         for r in range(self.world)]
            else:
                ops = [dist.P2POp(dist.isend, rec.flat, gdst, self.group)]
                parts = []
            if ops:
                works.extend(dist.batch_isend_irecv(ops))
            work = _Works(works)
        slot = getattr(rec, "_slot", None)
        if slot is not None:   # the slot's next rollout must wait for this read of it
            self._pending.setdefault(rec.steps, [None] * self.buffers)[slot] = work
        if async_op:
            return parts, work
        _wait(work)
        return parts

    def _copy_own(self, out: torch.Tensor, src: torch.Tensor, last: bool):
        """The learner's own shard into its receive slot.  On a GPU env whose ``rollout`` takes
        ``copy=``, the copy rides along the next rollout launch (``pbn_rollout_copy``: no extra
        kernel, no cross-stream wait); it is issued on the current stream instead if no rollout
        takes it before the hand-off is waited on, or when nothing follows (``last``)."""
        takes = getattr(self, "_env_takes_copy", None)
        if takes is None:
            takes = self._env_takes_copy = _takes_copy(self.env)
        if takes:
            self._flush_ride()
            ride = _Ride(out, src)
            if last:
                ride.flush()
            else:
                self._ride = ride
            return ride
        return self._copy_async(out, src, same_stream=last)

    def _take_ride(self, rec: "TransitionRecords"):
        """The pending own-shard copy for the launch about to write ``rec`` (None: none, or one
        that reads ``rec``'s own buffer, which is then issued first)."""
        ride = getattr(self, "_ride", None)
        if ride is None or ride.done:
            self._ride = None
            return None
        self._ride = None
        if ride.src.data_ptr() == rec.flat.data_ptr():
            ride.flush()
            return None
        return ride

    def _flush_ride(self) -> None:
        ride = getattr(self, "_ride", None)
        if ride is not None:
            ride.flush()
        self._ride = None

    def _copy_async(self, out: torch.Tensor, src: torch.Tensor, same_stream: bool = False):
        """out <- src (pbn_copy_async: 16-byte non-temporal vectors) on a side stream ordered after
        the current stream's work so far, so that it overlaps the next rollout; the returned
        work's wait() orders the current stream after the copy (as a collective's).  With
        ``same_stream`` the copy simply follows on the current stream (nothing to wait for)."""
        if not src.is_cuda:   # (gloo on the CPU: a plain copy)
            out.copy_(src)
            return None
        cur = torch.cuda.current_stream(src.device)
        if same_stream:
            _device_copy(out, src, cur)
            return None
        side = getattr(self, "_side", None)
        if side is None:
            side = self._side = torch.cuda.Stream(device=src.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            _device_copy(out, src, side)
            done = torch.cuda.Event()
            done.record(side)
        return _StreamWork(done, src.device)

    def run(self, n_rollouts: int, steps: int, dst: Optional[int] = None, consume=None,
            random_actions: bool = True, copy_own: bool = False) -> None:
        """``n_rollouts`` rollouts with the hand-off of rollout k overlapped with rollout k + 1
        (two or more record slots; with one slot, rollout k is consumed before rollout k + 1
        overwrites it).  ``consume(k, parts)`` is called on the learner (every rank for dst=None)
        once rollout k's records are readable on the current stream (after the device-side
        wait)."""
        prev = None
        for k in range(n_rollouts):
            rec = self.rollout(steps, random_actions=random_actions)
            parts, work = self.gather(rec, dst=dst, async_op=True, copy_own=copy_own, last=k == n_rollouts - 1)
            if self.buffers < 2:
                _finish((k, parts, work), consume)
                continue
            if prev is not None:
                _finish(prev, consume)
            prev = (k, parts, work)
        if prev is not None:
            _finish(prev, consume)

    @staticmethod
    def to_global(parts: List[TransitionRecords]) -> Dict[str, torch.Tensor]:
        """Per-rank records -> per-field tensors over all envs in global order (env = last axis)."""
        return {name: torch.cat([p[name] for p in parts], dim=-1) for name, _, _ in _FIELDS}


class _Ride:
    """An own-shard copy waiting for the next rollout launch to carry it (a work object: wait()
    issues it on the current stream if no launch has taken it yet, and otherwise orders the
    current stream after the launch that carried it, as a collective's work does)."""

    def __init__(self, dst: torch.Tensor, src: torch.Tensor):
        self.dst, self.src, self.done = dst, src, False
        self.event, self.stream = None, None

    def carried(self) -> None:
        """The rollout launch just issued on the current stream carries the copy (VectorPBNEnv
        launches on the stream current at the call): its completion is an event on that stream."""
        self.done = True
        if self.src.is_cuda:
            self.stream = torch.cuda.current_stream(self.src.device)
            self.event = torch.cuda.Event()
            self.event.record(self.stream)

    def flush(self) -> None:
        if not self.done:
            if self.src.is_cuda:
                self.stream = torch.cuda.current_stream(self.src.device)
                _device_copy(self.dst, self.src, self.stream)
                self.event = torch.cuda.Event()
                self.event.record(self.stream)
            else:
                self.dst.copy_(self.src)
            self.done = True

    def wait(self) -> None:
        self.flush()
        if self.event is not None:
            cur = torch.cuda.current_stream(self.src.device)
            if cur != self.stream:   # a consumer on another stream waits for the carrying launch
                cur.wait_event(self.event)


def _takes_copy(env) -> bool:
    """Whether env.rollout accepts copy= (VectorPBNEnv: pbn_rollout_copy)."""
    import inspect
    try:
        return "copy" in inspect.signature(env.rollout).parameters
    except (TypeError, ValueError):
        return False


def _device_copy(out: torch.Tensor, src: torch.Tensor, stream) -> None:
    """out <- src, both contiguous uint8 device buffers: libpbn_env's pbn_copy_async on ``stream``
    (the record buffers are 16-byte multiples: (12W + 5) B x T x n, n a multiple of 32)."""
    from . import _lib
    _lib.check(_lib.load().pbn_copy_async(out.data_ptr(), src.data_ptr(), out.numel(), stream.cuda_stream),
               "pbn_copy_async")


class _Works:
    """The works of one hand-off, waited together, at most once (a second wait on a finished
    gloo receive blocks)."""

    def __init__(self, works):
        self.works = [w for w in (works or []) if w is not None]

    def wait(self):
        works, self.works = self.works, []
        for w in works:
            w.wait()


class _StreamWork:
    """A side-stream copy's completion as a work object: wait() orders the current stream
    after it (no host synchronisation)."""

    def __init__(self, event, device):
        self.event, self.device = event, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.event)


def _wait(work) -> None:
    if work is not None:
        work.wait()


def _finish(item, consume) -> None:
    k, parts, work = item
    _wait(work)
    if consume is not None and parts:
        consume(k, parts)
