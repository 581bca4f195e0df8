"""HIP kernel == CPU oracle, bit for bit, through the C-ABI (libpbn_env.so).

Every output of pbn_step (state_out, final_state, reward, flags, target, t,
and the in-kernel actions) is compared exactly against oracle/pbn_oracle.c on
the same seeded inputs, for every bundled network and configuration axis:
interventions from a buffer / drawn in-kernel, autoreset on / off, selection
resolution (prob_bits), perturbation rate (including a high rate that drives
the rare multi-flip path), env offsets (sharding) and batch sizes up to the
BASELINE sizes.
"""
import numpy as np
import pytest
import torch

from oracle import oracle
from pbn_rl_amd import _lib
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

from .synthetic import random_spec

pytestmark = pytest.mark.gpu

NETS = ["pbn7", "pbn10", "pbn28", "pbn70"]


def make_spec(name, **kw):
    return EnvSpec(load_network(name), load_attractors(name), **kw)


def u32(x: torch.Tensor) -> np.ndarray:
    return x.cpu().numpy().view(np.uint32)


def run_pair(spec, n, steps, *, seed=12345, env_offset=0, mode=3, flip_density=0.1, rng_seed=0,
             start_random=False):
    """Step the GPU env and the oracle side by side; assert equality every step."""
    env = VectorPBNEnv(spec, n, seed=seed, env_offset=env_offset, autoreset=bool(mode & 1))
    env.reset()
    st, tg, t = oracle.reset(spec, seed, 0, env_offset, n)
    assert np.array_equal(u32(env.state), st), "reset state"
    assert np.array_equal(env.target.cpu().numpy(), tg)
    assert np.array_equal(env.t.cpu().numpy(), t)
    rng = np.random.default_rng(rng_seed)
    W = spec.words
    if start_random:
        st = rng.integers(0, 2 ** 32, size=(W, n), dtype=np.uint64).astype(np.uint32)
        if spec.n % 32:
            st[W - 1] &= np.uint32((1 << (spec.n % 32)) - 1)
        env.set_state(torch.from_numpy(st.view(np.int32)).to(env.device))
    for k in range(steps):
        random_actions = bool(mode & _lib.MODE_RANDOM_ACTIONS)
        if random_actions:
            flip = np.zeros((W, n), dtype=np.uint32)
            fm = None
        else:
            bits = (rng.random((W, n, 32)) < flip_density).astype(np.uint64)
            flip = (bits << np.arange(32, dtype=np.uint64)).sum(axis=2).astype(np.uint32)
            fm = torch.from_numpy(flip.view(np.int32)).to(env.device)
        step_idx = env.step_index
        state, reward, flags = env.step_flipmask(fm, random_actions=random_actions)
        ref = oracle.step(spec, seed, step_idx, env_offset, st, flip, tg, t, mode)
        tag = f"step {k}"
        assert np.array_equal(u32(env.final_state), ref["final_state"]), tag + " final_state"
        assert np.array_equal(u32(state), ref["state_out"]), tag + " state_out"
        assert np.array_equal(flags.cpu().numpy(), ref["flags"]), tag + " flags"
        assert np.array_equal(reward.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), tag + " reward"
        assert np.array_equal(env.target.cpu().numpy(), ref["target"]), tag + " target"
        assert np.array_equal(env.t.cpu().numpy(), ref["t"]), tag + " t"
        if random_actions:
            assert np.array_equal(u32(env.flipmask), ref["flipmask"]), tag + " in-kernel actions"
        st, tg, t = ref["state_out"], ref["target"], ref["t"]
    env.close()
    return ref


@pytest.mark.parametrize("name", NETS)
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_step_matches_oracle(name, mode):
    spec = make_spec(name, perturbation=0.02)
    run_pair(spec, 2048, 12, mode=mode, env_offset=0 if mode < 2 else 4096)


@pytest.mark.parametrize("name", ["pbn28", "pbn70"])
def test_high_perturbation_multi_flip_path(name):
    ref = run_pair(make_spec(name, perturbation=0.3), 1024, 6, mode=3)
    assert (ref["flags"] & _lib.FLAG_PERTURBED).mean() > 0.9


@pytest.mark.parametrize("bits", [4, 8, 12, 16])
def test_prob_bits(bits):
    run_pair(make_spec("pbn28", prob_bits=bits, perturbation=0.0), 1024, 6, mode=1, start_random=True)
    run_pair(make_spec("pbn70", prob_bits=bits, perturbation=0.02), 1024, 3, mode=3)


@pytest.mark.parametrize("name", NETS)
def test_from_random_states_no_perturbation(name):
    run_pair(make_spec(name, perturbation=0.0, horizon=0), 2048, 5, mode=0, start_random=True)


def test_no_attractors_autoreset():
    spec = EnvSpec(load_network("pbn28"), [], perturbation=0.01, horizon=3)
    run_pair(spec, 1024, 8, mode=3)


def test_baseline_size_bittner28():
    """BASELINE config 2 size: 65,536 envs, in-kernel actions, autoreset."""
    run_pair(make_spec("pbn28"), 65536, 30, mode=3, seed=0)


def test_baseline_size_pbn70():
    """BASELINE config 3 size: 1,048,576 envs (2-word+ state path)."""
    run_pair(make_spec("pbn70"), 1 << 20, 2, mode=3, seed=1)


def test_shard_invariance():
    """Concatenated shards == one run (env ids keep their RNG streams)."""
    spec = make_spec("pbn28")
    n, steps = 4096, 5
    whole = VectorPBNEnv(spec, n, seed=7)
    whole.reset()
    parts = [VectorPBNEnv(spec, n // 2, seed=7, env_offset=r * (n // 2)) for r in range(2)]
    for p in parts:
        p.step_index = 0
        p.reset()
    for _ in range(steps):
        a = whole.step_flipmask(random_actions=True)
        b = [p.step_flipmask(random_actions=True) for p in parts]
        for i in range(3):
            cat = torch.cat([b[0][i], b[1][i]], dim=-1)
            assert torch.equal(a[i], cat)


def test_abi_rejects_bad_arguments():
    spec = make_spec("pbn28")
    env = VectorPBNEnv(spec, 64)
    L = _lib.load()
    rc = L.pbn_step(env.net.handle, 0, 0, 16, 64, 3, env.state.data_ptr(), env.flipmask.data_ptr(),
                    env.target.data_ptr(), env.t.data_ptr(), env._state_next.data_ptr(), None,
                    env.reward.data_ptr(), env.flags.data_ptr(), None)
    assert rc == -22 and b"of 32" in L.pbn_last_error()
    rc = L.pbn_step(env.net.handle, 0, 0, 0, 64, 3, env.state.data_ptr(), env.flipmask.data_ptr(),
                    env.target.data_ptr(), env.t.data_ptr(), env.state.data_ptr(), None,
                    env.reward.data_ptr(), env.flags.data_ptr(), None)
    assert rc == -22


@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28", "pbn70"])
def test_step_offsets_and_modes(name):
    """pbn_step (one wave per 32-env group) at an env offset, with and without autoreset."""
    run_pair(make_spec(name, perturbation=0.05), 4096, 6, mode=3, env_offset=1024)
    run_pair(make_spec(name, perturbation=0.05), 2048, 4, mode=0)


def run_rollout_pair(spec, n, R, mode, *, seed=4242, env_offset=2048):
    """pbn_rollout (R steps in one launch, state on chip) == R oracle steps, every output."""
    env = VectorPBNEnv(spec, n, seed=seed, env_offset=env_offset, autoreset=bool(mode & 1))
    env.reset()
    st, tg, t = oracle.reset(spec, seed, 0, env_offset, n)
    W = spec.words
    rng = np.random.default_rng(3)
    if mode & 2:
        flips = None
        fm = None
    else:
        flips = rng.integers(0, 2 ** 32, size=(R, W, n), dtype=np.uint64).astype(np.uint32) & np.uint32(0x04010020)
        if spec.n % 32:
            flips[:, W - 1] &= np.uint32((1 << (spec.n % 32)) - 1)
        fm = torch.from_numpy(flips.view(np.int32)).to(env.device)
    out = env.rollout(R, flipmasks=fm, random_actions=bool(mode & 2), keep_obs=True, keep_updates=True)
    for k in range(R):
        flip = np.zeros((W, n), np.uint32) if flips is None else flips[k]
        ref = oracle.step(spec, seed, 1 + k, env_offset, st, flip, tg, t, mode)
        assert np.array_equal(u32(out["obs"][k])[:, :n], st), k
        assert np.array_equal(out["updates"][k].cpu().numpy().view(np.uint16)[:n], ref["updates"]), k
        assert np.array_equal(u32(out["final_state"][k])[:, :n], ref["final_state"]), k
        assert np.array_equal(out["flags"][k].cpu().numpy()[:n], ref["flags"]), k
        assert np.array_equal(out["reward"][k].cpu().numpy()[:n].view(np.uint32), ref["reward"].view(np.uint32)), k
        assert np.array_equal(u32(out["flipmask"][k])[:, :n], ref["flipmask"]), k
        st, tg, t = ref["state_out"], ref["target"], ref["t"]
    assert np.array_equal(u32(env.state)[:, :n], st)
    assert np.array_equal(env.target.cpu().numpy()[:n], tg)
    assert np.array_equal(env.t.cpu().numpy()[:n], t)
    env.close()
    return ref


@pytest.mark.parametrize("variant", ["pipe", "lean"])
@pytest.mark.parametrize("name", ["pbn7", "pbn28", "pbn70"])
@pytest.mark.parametrize("mode", [1, 3])
def test_rollout_matches_oracle(name, mode, variant, monkeypatch):
    monkeypatch.setenv("PBN_ROLL", variant)
    run_rollout_pair(make_spec(name, perturbation=0.05, horizon=7), 4096, 9, mode)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
@pytest.mark.parametrize("n_envs", [32, 96, 2080])
def test_rollout_odd_group_counts(n_envs, variant, monkeypatch):
    """The pipelined kernel pairs groups per block: an odd group count leaves a phantom half."""
    monkeypatch.setenv("PBN_ROLL", variant)
    run_rollout_pair(make_spec("pbn28", perturbation=0.05, horizon=5), n_envs, 7, 3, env_offset=96)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
@pytest.mark.parametrize("bits", [4, 8, 12])
def test_rollout_prob_bits(bits, variant, monkeypatch):
    monkeypatch.setenv("PBN_ROLL", variant)
    run_rollout_pair(make_spec("pbn28", prob_bits=bits, perturbation=0.02), 2048, 6, 3)
    run_rollout_pair(make_spec("pbn70", prob_bits=bits, perturbation=0.02), 2048, 4, 3)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
def test_rollout_high_perturbation_and_no_attractors(variant, monkeypatch):
    monkeypatch.setenv("PBN_ROLL", variant)
    run_rollout_pair(make_spec("pbn28", perturbation=0.3), 2048, 6, 3)
    run_rollout_pair(EnvSpec(load_network("pbn28"), [], perturbation=0.01, horizon=3), 2048, 8, 3)


# ---------------------------------------------------------------- synthetic networks
SYNTH = [(5, 11), (32, 15), (33, 12), (80, 13), (128, 14)]   # 1, 1 (full word), 2, 3, 4 state words


@pytest.mark.parametrize("n_nodes,seed", SYNTH)
def test_synthetic_networks_step(n_nodes, seed):
    """Up to 6 functions per node, arbitrary weights, constant functions (kaban nets have none)."""
    spec = random_spec(n_nodes, seed, perturbation=0.05, horizon=6)
    run_pair(spec, 2048, 5, mode=3, env_offset=1024)
    run_pair(spec, 1024, 3, mode=0)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
@pytest.mark.parametrize("n_nodes,seed", SYNTH)
def test_synthetic_networks_rollout(n_nodes, seed, variant, monkeypatch):
    monkeypatch.setenv("PBN_ROLL", variant)
    spec = random_spec(n_nodes, seed, perturbation=0.05, horizon=6)
    run_rollout_pair(spec, 2080, 6, 3)
    run_rollout_pair(spec, 96, 5, 1)


@pytest.mark.parametrize("n_nodes,seed", [(9, 21), (31, 22), (45, 23), (70, 24), (100, 25)])
@pytest.mark.parametrize("max_funcs", [3, 4])
def test_synthetic_few_functions_rollout(n_nodes, seed, max_funcs):
    """At most kNodeRecs functions per node with per-node weights: the pipelined kernel's
    common instances (no long chains) with per-lane thresholds (the selection's LDS digit-mask
    table at one state word, the per-lane compares above it), where every kaban network takes
    the wave-uniform threshold path."""
    spec = random_spec(n_nodes, seed, max_funcs=max_funcs, perturbation=0.05, horizon=6)
    assert max(len(f) for f in spec.network.nodes) <= 4
    run_rollout_pair(spec, 2080, 7, 3)
    run_rollout_pair(spec, 96, 4, 1)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
def test_rollout_long(variant, monkeypatch):
    """Many steps (horizons, resets, slots wrapping) in one launch: the pipelined kernel and
    the one-wave-per-group rollout against 40 oracle steps, in random-action and given-mask
    modes."""
    monkeypatch.setenv("PBN_ROLL", variant)
    run_rollout_pair(make_spec("pbn28", perturbation=0.03, horizon=9), 4160, 40, 3)
    run_rollout_pair(make_spec("pbn28", perturbation=0.03, horizon=5), 2048, 23, 1)
    run_rollout_pair(make_spec("pbn28", perturbation=0.03, horizon=5), 2048, 3, 0)
    run_rollout_pair(random_spec(5, 11, perturbation=0.05, horizon=6), 1024, 17, 3)


def test_rollout_equals_steps_baseline_size():
    spec = make_spec("pbn28")
    a = VectorPBNEnv(spec, 65536, seed=9)
    b = VectorPBNEnv(spec, 65536, seed=9)
    a.reset(); b.reset()
    out = a.rollout(20)
    for k in range(20):
        state, reward, flags = b.step_flipmask(random_actions=True)
        assert torch.equal(out["flags"][k], flags) and torch.equal(out["reward"][k], reward)
        assert torch.equal(out["final_state"][k], b.final_state)
    assert torch.equal(a.state, b.state) and torch.equal(a.t, b.t) and torch.equal(a.target, b.target)


# ---------------------------------------------------------------- wide functions (gates)
@pytest.mark.parametrize("name", ["bb33", "m47"])
def test_wide_networks(name, monkeypatch):
    """Functions of up to 6 (bb33) and 20 (model_tester's 47-node network) inputs, lowered to
    gates that the wave kernels evaluate level by level before the node functions."""
    spec = make_spec(name, perturbation=0.01, horizon=6)
    assert spec.arrays["n_gates"][0] > 0
    run_pair(spec, 2048, 5, mode=3, start_random=True)
    run_pair(spec, 1024, 3, mode=0, start_random=True)
    for variant in ("auto", "lean"):
        monkeypatch.setenv("PBN_ROLL", variant)
        run_rollout_pair(spec, 2080, 6, 3)


def test_wide_random_network(monkeypatch):
    """Table-only wide functions (Shannon-lowered, 86 gates) with several functions per node."""
    from pbn_rl_amd.attractors import random_state_targets
    from .synthetic import random_network
    net = random_network(12, 7, max_funcs=3, max_arity=7)
    spec = EnvSpec(net, random_state_targets(12, 4, 8), perturbation=0.02, horizon=5)
    run_pair(spec, 1024, 5, mode=3, start_random=True)
    monkeypatch.setenv("PBN_ROLL", "lean")
    run_rollout_pair(spec, 1024, 6, 3)


@pytest.mark.parametrize("name", ["pbn28", "pbn70"])
@pytest.mark.parametrize("settle", [0, 6])
def test_step_ragged_env_counts(name, settle):
    """pbn_reset / pbn_step with n_envs not a multiple of 32 (ABI 9; the scalar facade steps
    n_envs = 1): [W][n] buffers sized exactly, followed by canaries that must stay untouched;
    every output of the n envs equals the oracle's for the same envs of a padded batch (the
    missing envs of the last group change nothing: draws are keyed per env or per group)."""
    spec = make_spec(name, perturbation=0.05, horizon=5, settle=settle)
    env = VectorPBNEnv(spec, 32)
    L, h, W, dev = _lib.load(), env.net.handle, spec.words, env.device
    seed, off = 99, 64
    for n in (1, 5, 33, 70):
        pad = (n + 31) // 32 * 32
        CAN = 64
        def buf(count, dtype):
            return torch.full((count + CAN,), 0x5A, dtype=dtype, device=dev)
        st, tg, tt = buf(W * n, torch.int32), buf(n, torch.uint8), buf(n, torch.uint8)
        _lib.check(L.pbn_reset(h, seed, 0, off, n, st.data_ptr(), tg.data_ptr(), tt.data_ptr(), None), "reset")
        ost, otg, ott = oracle.reset(spec, seed, 0, off, pad)
        torch.cuda.synchronize()
        assert np.array_equal(u32(st[:W * n]).reshape(W, n), ost[:, :n])
        assert np.array_equal(tg[:n].cpu().numpy(), otg[:n]) and np.array_equal(tt[:n].cpu().numpy(), ott[:n])
        rng = np.random.default_rng(n)
        for k, mode in enumerate((3, 1, 0)):
            flip = (rng.integers(0, 2 ** 32, size=(W, pad), dtype=np.uint64).astype(np.uint32) & np.uint32(0x00410020))
            if spec.n % 32:
                flip[W - 1] &= np.uint32((1 << (spec.n % 32)) - 1)
            fm = buf(W * n, torch.int32)
            fm[:W * n] = torch.from_numpy(np.ascontiguousarray(flip[:, :n]).view(np.int32).reshape(-1)).to(dev)
            out, fin = buf(W * n, torch.int32), buf(W * n, torch.int32)
            rew, fl = buf(n, torch.float32), buf(n, torch.uint8)
            _lib.check(L.pbn_step(h, seed, 1 + k, off, n, mode, st.data_ptr(), fm.data_ptr(), tg.data_ptr(),
                                  tt.data_ptr(), out.data_ptr(), fin.data_ptr(), rew.data_ptr(), fl.data_ptr(), None),
                       "pbn_step")
            ref = oracle.step(spec, seed, 1 + k, off, np.pad(ost[:, :n], ((0, 0), (0, pad - n))), flip,
                              np.pad(otg[:n], (0, pad - n)), np.pad(ott[:n], (0, pad - n)), mode)
            torch.cuda.synchronize()
            tag = (n, k)
            assert np.array_equal(u32(out[:W * n]).reshape(W, n), ref["state_out"][:, :n]), tag
            assert np.array_equal(u32(fin[:W * n]).reshape(W, n), ref["final_state"][:, :n]), tag
            assert np.array_equal(fl[:n].cpu().numpy(), ref["flags"][:n]), tag
            assert np.array_equal(rew[:n].cpu().numpy().view(np.uint32), ref["reward"][:n].view(np.uint32)), tag
            assert np.array_equal(tg[:n].cpu().numpy(), ref["target"][:n]), tag
            assert np.array_equal(tt[:n].cpu().numpy(), ref["t"][:n]), tag
            if mode & 2:
                assert np.array_equal(u32(fm[:W * n]).reshape(W, n), ref["flipmask"][:, :n]), tag
            for b in (st, tg, tt, fm, out, fin, rew, fl):   # nothing past the n envs
                tail = b[-CAN:]
                assert torch.equal(tail, torch.full_like(tail, 0x5A)), tag
            st, ost, otg, ott = out, ref["state_out"], ref["target"], ref["t"]
    assert L.pbn_step(h, seed, 0, 16, 1, 0, st.data_ptr(), fm.data_ptr(), tg.data_ptr(), tt.data_ptr(),
                      out.data_ptr(), None, rew.data_ptr(), fl.data_ptr(), None) == -22   # offset not a multiple of 32
    assert L.pbn_rollout(h, seed, 0, 0, 33, 1, 0, st.data_ptr(), fm.data_ptr(), tg.data_ptr(), tt.data_ptr(), None,
                         None, rew.data_ptr(), fl.data_ptr(), None) == -22   # rollouts keep whole groups
