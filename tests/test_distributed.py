"""Env sharding + the per-rollout gather, world_size 2 over gloo on CPU.
The union of the shards' transitions must equal a single-process run."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pbn_rl_amd.distributed import ShardedRollout, TransitionRecords, record_bytes_per_env_step, shard_range


def test_shard_range_partitions():
    for n, w in [(256, 2), (64 * 7, 3), (32, 1), (1 << 20, 8)]:
        parts = [shard_range(n, w, r) for r in range(w)]
        assert parts[0][0] == 0
        for (o, c), (o2, _) in zip(parts, parts[1:]):
            assert o + c == o2 and o % 32 == 0 and c % 32 == 0
        assert sum(c for _, c in parts) == n
    with pytest.raises(ValueError):
        shard_range(100, 2, 0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_total, steps, result_path, form="all"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from tests.oracle_env import OracleVectorEnv

    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05)
    ro = ShardedRollout(n_total, lambda off, cnt: OracleVectorEnv(spec, off, cnt, seed=11),
                        buffers=1 if form == "run1" else 2)
    if form in ("run", "run1", "run_own"):
        # three rollouts, each hand-off to rank 0 overlapped with the next rollout ("run_own": rank 0
        # also copies its own shard into its receive slot, bench.py's value_with_gather form)
        got = {}

        def consume(k, parts):
            if form == "run_own":
                assert all(p.flat.data_ptr() != ro._ring[steps][k % 2].flat.data_ptr() for p in parts)
            got[k] = {n: v.clone() for n, v in ShardedRollout.to_global(parts).items()}
        ro.run(3, steps, dst=0, consume=consume, copy_own=form == "run_own")
        if rank == 0:
            torch.save(got, result_path)
        else:
            assert got == {}
    else:
        rec = ro.rollout(steps)
        parts = ro.gather(rec, dst=0 if form == "dst" else None)
        if form == "dst" and rank != 0:
            assert parts == []
        if rank == 0:
            glob = ShardedRollout.to_global(parts)
            torch.save({k: v.clone() for k, v in glob.items()}, result_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("form", ["all", "dst"])
def test_two_rank_gather_equals_single_run(tmp_path, form):
    """all_gather (every rank receives) and the point-to-point hand-off to the learner (rank 0
    keeps its shard in place, rank 1 sends): the union equals one process's run."""
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from tests.oracle_env import OracleVectorEnv

    n_total, steps = 256, 4
    out = str(tmp_path / "gathered.pt")
    mp.spawn(_worker, args=(2, _free_port(), n_total, steps, out, form), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05)
    single = ShardedRollout(n_total, lambda off, cnt: OracleVectorEnv(spec, off, cnt, seed=11))
    want = single.rollout(steps)
    assert set(got) == {"obs", "flipmask", "final_state", "reward", "flags"}
    for name, t in got.items():
        assert t.shape[-1] == n_total
        assert torch.equal(t, want[name]), name


def test_record_wire_format():
    rec = TransitionRecords(3, 1, 64)
    assert rec.flat.numel() == 3 * 64 * 17 == 3 * 64 * record_bytes_per_env_step(1)
    assert rec["obs"].shape == (3, 1, 64) and rec["reward"].dtype == torch.float32
    rec["flags"].fill_(7)
    assert int(rec.flat[-1]) == 7                       # flags are the last field
    rec2 = TransitionRecords(2, 3, 32)
    assert rec2.flat.numel() == 2 * 32 * (12 * 3 + 5)
    with pytest.raises(ValueError):
        TransitionRecords(1, 1, 48)


@pytest.mark.parametrize("form", ["run", "run1", "run_own"])
def test_two_rank_overlapped_run_equals_single_run(tmp_path, form):
    """ShardedRollout.run: three rollouts with the hand-off of rollout k to rank 0 in flight
    while rollout k + 1 runs (two record slots; "run1": one slot, each rollout consumed before
    the next overwrites it): rank 0 receives all three, equal to three successive rollouts of
    one process."""
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from tests.oracle_env import OracleVectorEnv

    n_total, steps = 256, 3
    out = str(tmp_path / "run.pt")
    mp.spawn(_worker, args=(2, _free_port(), n_total, steps, out, form), nprocs=2, join=True)
    got = torch.load(out, weights_only=True)
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05)
    single = ShardedRollout(n_total, lambda off, cnt: OracleVectorEnv(spec, off, cnt, seed=11), buffers=1)
    assert sorted(got) == [0, 1, 2]
    for k in range(3):
        want = single.rollout(steps)
        for name in ("obs", "flipmask", "final_state", "reward", "flags"):
            assert torch.equal(got[k][name], want[name]), (k, name)


def test_record_ring_keeps_previous_rollout():
    """With two slots the records of rollout k survive rollout k + 1 (and are overwritten by
    rollout k + 2)."""
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from tests.oracle_env import OracleVectorEnv

    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05)
    ro = ShardedRollout(64, lambda off, cnt: OracleVectorEnv(spec, off, cnt, seed=3), buffers=2)
    a = ro.rollout(2)
    snap = a["obs"].clone()
    b = ro.rollout(2)
    assert a.flat.data_ptr() != b.flat.data_ptr() and torch.equal(a["obs"], snap)
    c = ro.rollout(2)
    assert c.flat.data_ptr() == a.flat.data_ptr()


def _spec():
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    return EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05)


class _RideEnv:
    """OracleVectorEnv with VectorPBNEnv's copy= contract (dst <- src once the launch is done),
    logging the copies it carried."""

    def __init__(self, inner):
        self.inner, self.carried = inner, []
        self.words = inner.words

    @property
    def state(self):
        return self.inner.state

    def rollout(self, n_steps, flipmasks=None, random_actions=True, keep_obs=True, keep_final=True, out=None,
                copy=None):
        res = self.inner.rollout(n_steps, flipmasks=flipmasks, random_actions=random_actions, keep_obs=keep_obs,
                                 keep_final=keep_final, out=out)
        if copy is not None:
            dst, src = copy
            dst.copy_(src)
            self.carried.append(src.data_ptr())
        return res


@pytest.mark.parametrize("buffers", [1, 2, 3])
def test_own_shard_copy_rides_along_the_next_rollout(buffers):
    """World 1 without a process group, copy_own: rollout k's records reach the receive slot by
    the copy riding along rollout k + 1 (when k + 1 writes another slot), or on the hand-off's
    wait; the last hand-off is copied at once.  Every received slot equals a single run's records."""
    from pbn_rl_amd.distributed import ShardedRollout
    from tests.oracle_env import OracleVectorEnv
    spec = _spec()
    n, steps, k_total = 64, 3, 5
    env = _RideEnv(OracleVectorEnv(spec, 0, n, seed=9))
    ro = ShardedRollout(n, lambda off, cnt: env, buffers=buffers)
    seen = []
    ro.run(k_total, steps, dst=0, consume=lambda k, parts: seen.append(parts[0].flat.clone()), copy_own=True)
    ref = OracleVectorEnv(spec, 0, n, seed=9)
    from pbn_rl_amd.distributed import TransitionRecords
    assert len(seen) == k_total
    for k in range(k_total):
        want = ref.rollout(steps)
        got = TransitionRecords(steps, env.words, n, flat=seen[k])
        for name in ("obs", "flipmask", "final_state", "flags"):
            assert torch.equal(got[name], want[name]), (k, name)
    # with two or more slots every hand-off but the last rode along the next launch
    assert len(env.carried) == (k_total - 1 if buffers >= 2 else 0)
