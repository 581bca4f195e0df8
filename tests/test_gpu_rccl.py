"""The per-rollout transition hand-off through RCCL ("nccl" backend) on the GPU: a world-1
process group on cuda:0 (the box has one GPU; RCCL refuses two ranks on one device).  The
gathered records must equal the C oracle stepped over the same envs; the
2-rank exchange itself (all_gather and the point-to-point hand-off to the learner) is covered
over gloo in tests/test_distributed.py."""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_world1():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        yield
    finally:
        dist.destroy_process_group()


def _spec(p=0.05):
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    return EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=p)


def _factory(spec, seed, base=0):
    from pbn_rl_amd.vector_env import VectorPBNEnv

    def make(off, cnt):
        env = VectorPBNEnv(spec, cnt, seed=seed, device="cuda:0", env_offset=base + off)
        env.reset()
        return env
    return make


def _check_against_oracle(spec, seed, got, env_offset, n, steps, lo, hi):
    """Records of envs [lo, hi) of the shard (global ids env_offset + lo ..) == the oracle."""
    from tests.oracle_env import OracleVectorEnv
    want = OracleVectorEnv(spec, env_offset + lo, hi - lo, seed=seed).rollout(steps)
    for name in ("obs", "flipmask", "final_state", "reward", "flags"):
        g = got[name][..., lo:hi].cpu()
        w = want[name]
        if name == "reward":
            assert np.array_equal(g.numpy().view(np.uint32), w.numpy().view(np.uint32)), name
        else:
            assert torch.equal(g, w), (name, lo)


def test_rccl_world1_gather_matches_oracle(rccl_world1):
    from pbn_rl_amd.distributed import ShardedRollout
    spec = _spec()
    n_total, steps = 2048, 6
    ro = ShardedRollout(n_total, _factory(spec, 11))
    parts = ro.gather(ro.rollout(steps))
    torch.cuda.synchronize()
    assert len(parts) == 1 and parts[0].flat.data_ptr() != ro._ring[steps][0].flat.data_ptr()   # via RCCL
    _check_against_oracle(spec, 11, ShardedRollout.to_global(parts), 0, n_total, steps, 0, n_total)


def test_rccl_config4_shard_at_size(rccl_world1):
    """BASELINE config 4's per-GPU shard: 1,048,576 Bittner-28 envs at env_offset 3 * 2^20 (rank
    3 of 8), one 16-step rollout (config 4 gathers every T = 16 steps) through the RCCL
    all_gather, then the overlapped hand-off loop of ShardedRollout.run; four 4,096-env windows
    across the shard (start, two interior, end) against the oracle."""
    from pbn_rl_amd.distributed import ShardedRollout
    spec = _spec(0.01)
    n, steps, base = 1 << 20, 16, 3 << 20
    ro = ShardedRollout(n, _factory(spec, 0, base))
    got = ShardedRollout.to_global(ro.gather(ro.rollout(steps)))
    torch.cuda.synchronize()
    for lo in (0, 262144 + 4096, 786432 - 8192, n - 4096):
        _check_against_oracle(spec, 0, got, base, n, steps, lo, lo + 4096)
    # the overlapped loop continues the same envs: rollouts 2 and 3 (steps 17-48), the window of
    # the shard's last 4,096 envs copied out by the learner's consume callback
    from tests.oracle_env import OracleVectorEnv
    seen = []
    ro.run(2, steps, dst=None, consume=lambda k, parts: seen.append(
        {f: v[..., n - 4096:].cpu().clone() for f, v in ShardedRollout.to_global(parts).items()}))
    torch.cuda.synchronize()
    assert len(seen) == 2
    ref = OracleVectorEnv(spec, base + n - 4096, 4096, seed=0)
    ref.rollout(steps)
    for k in range(2):
        want = ref.rollout(steps)
        for name in ("obs", "flipmask", "final_state", "flags"):
            assert torch.equal(seen[k][name], want[name]), (k, name)
        assert np.array_equal(seen[k]["reward"].numpy().view(np.uint32), want["reward"].numpy().view(np.uint32))


def test_world1_own_shard_handoff_copies_records():
    """bench.py's value_with_gather hand-off at world 1 (no process group): the learner's own shard
    copied into its receive slot riding along the next rollout launch (pbn_rollout_copy) or, for
    the last hand-off of a run, by pbn_copy_async on the launch stream.  Three overlapped rollouts;
    every received slot equals the records the kernel wrote, and the oracle."""
    from pbn_rl_amd.distributed import ShardedRollout
    spec = _spec()
    n, steps = 4096, 5
    ro = ShardedRollout(n, _factory(spec, 3))
    seen = []

    def consume(k, parts):
        assert len(parts) == 1 and parts[0].flat.data_ptr() != ro._ring[steps][k % 2].flat.data_ptr()
        seen.append({f: v.cpu().clone() for f, v in ShardedRollout.to_global(parts).items()})
        seen[-1]["_src"] = ro._ring[steps][k % 2].flat.cpu().clone()
        seen[-1]["_dst"] = parts[0].flat.cpu().clone()

    ro.run(3, steps, dst=0, consume=consume, copy_own=True)
    torch.cuda.synchronize()
    assert len(seen) == 3
    for k in range(3):
        assert torch.equal(seen[k]["_src"], seen[k]["_dst"]), k
    from tests.oracle_env import OracleVectorEnv
    ref = OracleVectorEnv(spec, 0, n, seed=3)
    for k in range(3):
        want = ref.rollout(steps)
        for name in ("obs", "flipmask", "final_state", "flags"):
            assert torch.equal(seen[k][name], want[name]), (k, name)


@pytest.mark.parametrize("buffers", [1, 3])
def test_world1_own_shard_handoff_ring_sizes(buffers):
    """The ride-along own-shard copy with one record slot (the next rollout would overwrite the
    copy's source: the copy is issued first, on the launch stream) and with three; the hand-off
    waited on before the next rollout (a plain loop over gather + consume) as well as overlapped."""
    from pbn_rl_amd.distributed import ShardedRollout
    spec = _spec()
    n, steps = 4096, 5
    ro = ShardedRollout(n, _factory(spec, 5), buffers=buffers)
    seen = []

    def consume(k, parts):
        seen.append(parts[0].flat.cpu().clone())

    ro.run(4, steps, dst=0, consume=consume, copy_own=True)
    rec = ro.rollout(steps)   # then one hand-off waited on at once, with no rollout after it
    parts = ro.gather(rec, dst=0, copy_own=True)
    seen.append(parts[0].flat.cpu().clone())
    torch.cuda.synchronize()
    from tests.oracle_env import OracleVectorEnv
    ref = OracleVectorEnv(spec, 0, n, seed=5)
    from pbn_rl_amd.distributed import TransitionRecords
    for k in range(5):
        want = ref.rollout(steps)
        got = TransitionRecords(steps, 1, n, flat=seen[k])
        for name in ("obs", "flipmask", "final_state", "flags"):
            assert torch.equal(got[name], want[name]), (k, name)


def test_world1_ride_consumed_on_another_stream():
    """The hand-off work of a ride-along copy orders a consumer on another stream after the
    launch that carried the copy: gather, the next rollout (it carries the copy),
    then work.wait() and the read on a second stream, with a long kernel queued on the launch
    stream after the carrying launch so that an unordered read would see the slot before the copy."""
    from pbn_rl_amd.distributed import ShardedRollout
    spec = _spec()
    n, steps = 4096, 5
    ro = ShardedRollout(n, _factory(spec, 7))
    rec = ro.rollout(steps)
    want = rec.flat.clone()
    parts, work = ro.gather(rec, dst=0, async_op=True, copy_own=True)
    ro.rollout(steps)   # carries rollout 0's own-shard copy
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        work.wait()
        got = parts[0].flat.clone()
    torch.cuda.synchronize()
    assert torch.equal(got, want)


def test_copy_async_entry_point():
    """pbn_copy_async: ragged sizes (every 16-byte multiple up to a few vectors past the grid's
    stride loop), offsets into a buffer, and its argument checks."""
    import ctypes
    from pbn_rl_amd import _lib
    L = _lib.load()
    src = torch.randint(0, 256, (1 << 22,), dtype=torch.uint8, device="cuda")
    for nbytes in (16, 4096 + 48, (1 << 22) - 16 * 7):
        dst = torch.zeros(1 << 22, dtype=torch.uint8, device="cuda")
        _lib.check(L.pbn_copy_async(dst.data_ptr() + 16, src.data_ptr(), nbytes, None), "copy")
        torch.cuda.synchronize()
        assert torch.equal(dst[16:16 + nbytes], src[:nbytes]) and not dst[:16].any()
        assert not dst[16 + nbytes:].any()
    assert L.pbn_copy_async(src.data_ptr(), src.data_ptr() + 8, 16, None) != 0      # misaligned
    assert L.pbn_copy_async(src.data_ptr() + 16, src.data_ptr(), 64, None) != 0     # overlapping
    assert L.pbn_copy_async(None, src.data_ptr(), 16, None) != 0
    assert L.pbn_copy_async(src.data_ptr(), src.data_ptr(), 0, None) == 0
    del ctypes


@pytest.mark.parametrize("settle", [0, 6])
def test_rollout_copy_entry_point(settle):
    """pbn_rollout_copy: the copy rides along the pipelined launch as its fourth wave (paced by
    the block barriers up to four vectors per lane and iteration, one burst beyond; ragged ends)
    or follows it (the settle kernel, n_steps = 0); either way dst == src with the bytes around dst untouched, and the launch's
    records equal a twin env's plain rollout."""
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.05, settle=settle)
    n, steps = 8192, 5
    cap = (steps + 1) * n * 16   # one vector per env-draw lane (64 envs) and iteration
    envs = [VectorPBNEnv(spec, n, seed=11, device="cuda:0") for _ in range(2)]
    for e in envs:
        e.reset()
    src = torch.randint(0, 256, (4 * cap + 4096,), dtype=torch.uint8, device="cuda")
    # paced at 1, 2 and 4 vectors per lane and iteration, then one burst past 4; no steps: after
    for nbytes, t in ((16, steps), (4096 + 48, steps), (cap, steps), (cap + 16, steps), (2 * cap, steps),
                      (2 * cap + 16, steps), (4 * cap, steps), (4 * cap + 16, steps), (4096, 0)):
        dst = torch.zeros(4 * cap + 4096 + 32, dtype=torch.uint8, device="cuda")
        got = envs[0].rollout(t, keep_obs=True, copy=(dst[16:16 + nbytes], src[:nbytes]))
        want = envs[1].rollout(t, keep_obs=True)
        torch.cuda.synchronize()
        assert torch.equal(dst[16:16 + nbytes], src[:nbytes]), nbytes
        assert not dst[:16].any() and not dst[16 + nbytes:].any(), nbytes
        for name, w in want.items():
            if not isinstance(w, torch.Tensor):
                continue
            g = got[name]
            if g.dtype == torch.float32:
                g, w = g.view(torch.int32), w.view(torch.int32)
            assert torch.equal(g, w), (nbytes, name)
    with pytest.raises(ValueError):
        envs[0].rollout(steps, copy=(dst[:32], src[:16]))
    with pytest.raises(ValueError):   # a strided view: its bytes are not one range
        envs[0].rollout(steps, copy=(dst[:64:2], src[:32]))
    out = envs[0].rollout_buffers(steps, keep_obs=True)
    flat = out["reward"].view(torch.uint8).reshape(-1)
    with pytest.raises(ValueError, match="overlaps"):   # the copy may not touch the launch's own outputs
        envs[0].rollout(steps, keep_obs=True, out=out, copy=(flat[:64], src[:64]))
    with pytest.raises(ValueError, match="overlaps"):
        envs[0].rollout(steps, copy=(dst[:64], envs[0].state.view(torch.uint8).reshape(-1)[:64]))
