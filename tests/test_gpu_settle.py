"""The settle law on the GPU (include/pbn_env.h "Step law"): kernels == oracle bit for bit, and
the reference's bb33 evaluation replayed through the gym facade on the device.

pbn_rollout runs the pipelined settle kernel (pbn_rollout_settle: one update per iteration, every
env its own update sequence, an env that settles starting its next step) for networks without
gates, and the wave kernel's variant 4 for networks with gates or under PBN_ROLL=lean; pbn_step
runs a one-step launch of the same pipelined kernel on whole groups (the wave kernel's variant 3
for ragged env counts, gates, or PBN_ROLL=lean).  Every output is
compared with oracle/pbn_oracle.c, including the PBN_FLAG_UNSETTLED bit of envs that hit the cap
and the per-env-step update counts (pbn_rollout_ex's d_updates, the settle lengths).
"""
import numpy as np
import pytest

import torch

from oracle import oracle
from pbn_rl_amd import _lib
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.env import PBNEnv
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

from .protocol import load_agent, replay, summary
from .synthetic import random_spec
from .test_bn_pin import reference_result
from .oracle_env import OracleVectorEnv
from .test_gpu_parity import run_pair, run_rollout_pair, u32

pytestmark = pytest.mark.gpu


def settle_spec(name, settle, **kw):
    return EnvSpec(load_network(name), load_attractors(name), settle=settle, **kw)


@pytest.mark.parametrize("variant", ["auto", "lean"])
@pytest.mark.parametrize("name", ["pbn7", "pbn28", "pbn70", "bb33"])
@pytest.mark.parametrize("settle", [2, 9, 64])
def test_settle_step_matches_oracle(name, settle, variant, monkeypatch):
    """pbn_step under the settle law: the one-step launch of the pipelined settle kernel (auto;
    bb33 has gates and takes the wave kernel) and the wave kernel's variant 3 (lean)."""
    monkeypatch.setenv("PBN_ROLL", variant)
    spec = settle_spec(name, settle, perturbation=0.02, horizon=6)
    run_pair(spec, 2048, 6, mode=3, env_offset=1024)
    run_pair(spec, 1024, 4, mode=0, start_random=True)


@pytest.mark.parametrize("variant", ["pipe", "lean"])
@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28", "pbn70", "bb33"])
def test_settle_rollout_matches_oracle(name, variant, monkeypatch):
    monkeypatch.setenv("PBN_ROLL", variant)
    spec = settle_spec(name, 12, perturbation=0.05, horizon=7)
    run_rollout_pair(spec, 2080, 8, 3)
    run_rollout_pair(spec, 1024, 5, 1)


@pytest.mark.parametrize("settle", [2, 3, 64])
@pytest.mark.parametrize("n_envs", [32, 96, 4128])
def test_settle_pipe_caps_and_odd_groups(settle, n_envs):
    """The pipelined settle kernel at caps 2 (every step ends at the cap or earlier), 3 and the
    facade's 64, with an odd group count (a phantom half in the last block) and p = 0 (groups
    that settle early: the speculated update is dropped and re-issued)."""
    for p in (0.0, 0.01):
        spec = settle_spec("pbn28", settle, perturbation=p, horizon=20)
        run_rollout_pair(spec, n_envs, 7, 3, env_offset=0)


def test_settle_pipe_config2_100_steps_at_65536():
    """Config 2 under the facade's default law (settle = 64): pbn28 x 65,536 envs, one 100-step
    pbn_rollout launch (bench.py --settle 64's launch), every output of every step and the
    settle length of every env-step, against the C oracle."""
    spec = settle_spec("pbn28", 64, perturbation=0.01, horizon=20)
    n, T, seed = 65536, 100, 0
    env = VectorPBNEnv(spec, n, seed=seed)
    env.reset()
    out = env.rollout(T, random_actions=True, keep_obs=True, keep_final=True, keep_updates=True)
    torch.cuda.synchronize()
    st, tg, t = oracle.reset(spec, seed, 0, 0, n)
    zero = np.zeros_like(st)
    upd = 0
    for k in range(T):
        ref = oracle.step(spec, seed, 1 + k, 0, st, zero, tg, t, 3)
        assert np.array_equal(u32(out["obs"][k]), st), k
        assert np.array_equal(u32(out["flipmask"][k]), ref["flipmask"]), k
        assert np.array_equal(u32(out["final_state"][k]), ref["final_state"]), k
        assert np.array_equal(out["reward"][k].cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), k
        assert np.array_equal(out["flags"][k].cpu().numpy(), ref["flags"]), k
        assert np.array_equal(out["updates"][k].cpu().numpy().view(np.uint16), ref["updates"]), k
        upd += int(ref["updates"].sum())
        st, tg, t = ref["state_out"], ref["target"], ref["t"]
    assert np.array_equal(u32(env.state), st)
    assert np.array_equal(env.target.cpu().numpy(), tg) and np.array_equal(env.t.cpu().numpy(), t)
    assert upd > 2 * n * T        # the settle law ran (the mean settle length is well above 2)


def test_settle_pipe_config3_pbn70_at_1m():
    """Config 3's size under the settle law: pbn70 x 1,048,576 envs, one 20-step launch, four
    4,096-env windows of every output against the oracle run on those envs."""
    spec = settle_spec("pbn70", 16, perturbation=0.01, horizon=20)
    n, T, seed = 1 << 20, 20, 1
    env = VectorPBNEnv(spec, n, seed=seed)
    env.reset()
    out = env.rollout(T, random_actions=True, keep_obs=True, keep_final=True, keep_updates=True)
    torch.cuda.synchronize()
    for lo in (0, 333 * 1024, 700 * 1024 + 2048, n - 4096):
        hi = lo + 4096
        want = OracleVectorEnv(spec, lo, 4096, seed=seed).rollout(T)
        for name in ("obs", "flipmask", "final_state", "flags", "updates"):
            assert torch.equal(out[name][..., lo:hi].cpu(), want[name]), (name, lo)
        assert np.array_equal(out["reward"][:, lo:hi].cpu().numpy().view(np.uint32),
                              want["reward"].numpy().view(np.uint32)), lo


def test_settle_unsettled_flag_and_high_perturbation():
    """Random targets are almost never hit: every step runs to the cap and is flagged."""
    spec = random_spec(40, 12, perturbation=0.3, horizon=4, settle=5)
    ref = run_pair(spec, 1024, 4, mode=3)
    assert (ref["flags"] & _lib.FLAG_UNSETTLED).mean() > 0.5
    run_rollout_pair(spec, 1024, 5, 3)


@pytest.mark.parametrize("n_nodes,seed", [(5, 11), (80, 13), (128, 14)])
def test_settle_synthetic_networks(n_nodes, seed):
    spec = random_spec(n_nodes, seed, perturbation=0.05, horizon=6, settle=6)
    run_pair(spec, 1024, 4, mode=3)
    run_rollout_pair(spec, 1056, 5, 3)


def test_settle_one_equals_one_update_law():
    """settle = 1 is the one-update law (same kernels' results as settle = 0)."""
    a = run_pair(settle_spec("pbn28", 1, perturbation=0.02), 2048, 4, mode=3)
    b = run_pair(settle_spec("pbn28", 0, perturbation=0.02), 2048, 4, mode=3)
    for k in ("state_out", "flags", "reward"):
        assert np.array_equal(a[k], b[k])


# ------------------------------------------------ the reference's bb33 evaluation, on the GPU
def facade_step_fn(env: PBNEnv, net):
    """model_tester.py:611-625 through the gym facade: graph.setState, step(action), render."""
    def step(words, flip, k):
        out = np.zeros_like(words)
        for i in range(words.shape[1]):
            env.graph.setState(net.unpack([int(w) for w in words[:, i]]))
            acts = [j + 1 for j in range(net.n) if (int(flip[j >> 5, i]) >> (j & 31)) & 1]
            env.step(acts)
            out[:, i] = net.pack(env.render())
        return out
    return step


def test_gpu_bb33_evaluation_reproduces_reference():
    """model_tester.py:587-658 (--mode bn, 3 attractors, 10 runs) with the reference's trained
    bb33 agent, stepping PBNEnv(settle=64, perturbation=0) on the GPU: exactly the per-run
    lengths and the 0/90 failures of data/results/pbn_33_3.pkl."""
    net = load_network("bb33")
    atts = load_attractors("bb33")
    chosen = [atts[i] for i in (0, 2, 1)]
    env = PBNEnv(network=net, attractors=chosen, perturbation=0.0, horizon=0, settle=64, seed=5,
                 grow_attractors=False)
    env.reset()
    res = replay(facade_step_fn(env, net), load_agent("bb33", 33), chosen, n_runs=10)
    mat, same, data = summary(res)
    ref, ref_data = reference_result()
    assert same and np.array_equal(mat / 10, ref)
    assert data == {k: v for k, v in ref_data.items() if k != 101}
    env.close()


def test_gpu_bb33_evaluation_on_default_constructor():
    """The same replay through PBNEnv as the reference builds it (model_tester.py:409-413: no
    step-law argument): the facade's default law (DEFAULT_SETTLE) reproduces the fixture."""
    from pbn_rl_amd.env import DEFAULT_SETTLE
    net = load_network("bb33")
    atts = load_attractors("bb33")
    chosen = [atts[i] for i in (0, 2, 1)]
    env = PBNEnv(N=net.n, genes=net.genes, logic_functions=net.logic_functions, attractors=chosen,
                 perturbation=0.0, horizon=0, seed=5, grow_attractors=False)
    assert env.spec.settle == DEFAULT_SETTLE >= 2
    env.reset()
    res = replay(facade_step_fn(env, net), load_agent("bb33", 33), chosen, n_runs=10)
    mat, same, data = summary(res)
    ref, ref_data = reference_result()
    assert same and np.array_equal(mat / 10, ref)
    assert data == {k: v for k, v in ref_data.items() if k != 101}
    env.close()


def test_gpu_bb33_one_update_law_fails_reference():
    net = load_network("bb33")
    atts = load_attractors("bb33")
    chosen = [atts[i] for i in (0, 2, 1)]
    env = PBNEnv(network=net, attractors=chosen, perturbation=0.0, horizon=0, settle=0, seed=5,
                 grow_attractors=False)
    env.reset()
    res = replay(facade_step_fn(env, net), load_agent("bb33", 33), chosen, n_runs=1)
    ref, _ = reference_result()
    assert not np.array_equal(summary(res)[0], ref)
    env.close()


def test_settle_unpacked_threshold_compare():
    """A node whose last function quantises to weight 0 (weights 0.99 / 0.01 at prob_bits = 4): its
    first threshold is 2^B = 16, which the packed 16-bit compares cannot hold, so the host leaves
    settle_pk = 0 and pbn_rollout_settle's selection wave takes its unpacked compare
    (settle_lt_word on the thresholds in global memory).  Rollouts and pbn_step's
    one-step launches against the oracle."""
    import json
    import os
    from pbn_rl_amd.attractors import find_attractors
    from pbn_rl_amd.network import Network
    d = json.load(open(os.path.join(os.path.dirname(__file__), "..", "pbn_rl_amd", "networks", "pbn7.json")))
    lf = [[(e, w) for e, w in fl] for fl in d["logic_functions"]]
    lf[0] = [(lf[0][0][0], 0.99), (lf[1][0][0], 0.01)]
    net = Network.from_logic_functions(d["genes"], lf, name="pbn7_zero_last")
    assert net.thresholds(4)[0][0] == 16     # == 2^B: not representable in the packed compares
    spec = EnvSpec(net, find_attractors(net, prob_bits=4), prob_bits=4, perturbation=0.05, horizon=6, settle=6)
    run_rollout_pair(spec, 2080, 8, 3)
    run_rollout_pair(spec, 1024, 5, 1)
    run_pair(spec, 2048, 4, mode=3, env_offset=1024)
