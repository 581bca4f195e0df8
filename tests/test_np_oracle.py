"""The batched numpy restatement (oracle/np_oracle.py) against the C oracle: every output of
every env, bit for bit, on the kaban networks, random networks (up to 6 functions per node,
arbitrary weights, 1-3 state words, wide functions) and a network without attractors."""
import numpy as np
import pytest

from oracle import np_oracle, oracle
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec

KEYS = ["state_out", "final_state", "reward", "flags", "target", "t", "flipmask"]


def _compare(spec, n, seed, off, mode, steps=4, flip_mask=0x00100201):
    npo = np_oracle.NpPBN(spec)
    W = spec.words
    st, tg, t = oracle.reset(spec, seed, 0, off, n)
    s2, g2, t2 = npo.reset(seed, 0, off, n)
    assert np.array_equal(st, s2) and np.array_equal(tg, g2) and np.array_equal(t, t2)
    rng = np.random.default_rng(seed)
    for step in range(1, steps + 1):
        flip = rng.integers(0, 2 ** 32, size=(W, n), dtype=np.uint64).astype(np.uint32) & np.uint32(flip_mask)
        if spec.n % 32:
            flip[W - 1] &= np.uint32((1 << (spec.n % 32)) - 1)
        ref = oracle.step(spec, seed, step, off, st, flip, tg, t, mode)
        got = npo.step(seed, step, off, st, flip, tg, t, mode)
        for k in KEYS:
            assert np.array_equal(ref[k], got[k]), (k, step)
        st, tg, t = ref["state_out"], ref["target"], ref["t"]


@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28", "pbn70", "bb33"])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_np_oracle_equals_c_oracle(name, mode):
    spec = EnvSpec(load_network(name), load_attractors(name), perturbation=0.08, horizon=4)
    _compare(spec, 256, 4242, 96, mode)


@pytest.mark.parametrize("n_nodes,seed", [(5, 31), (40, 32), (70, 33)])
def test_np_oracle_equals_c_oracle_synthetic(n_nodes, seed):
    from .synthetic import random_spec
    _compare(random_spec(n_nodes, seed, perturbation=0.1, horizon=3), 128, 555, 32, 3)


def test_np_oracle_wide_random_network():
    from .synthetic import random_network
    from pbn_rl_amd.attractors import random_state_targets
    net = random_network(12, 7, max_funcs=3, max_arity=7)
    spec = EnvSpec(net, random_state_targets(12, 6, 8), perturbation=0.02, horizon=5)
    _compare(spec, 128, 9, 0, 3)


def test_np_oracle_without_attractors():
    spec = EnvSpec(load_network("pbn28"), [], perturbation=0.01, horizon=6)
    _compare(spec, 128, 3, 0, 3, steps=7)


def test_np_oracle_large_perturbation():
    """p = 0.3: many gaps per env, several PERT calls."""
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.3, horizon=20)
    _compare(spec, 256, 11, 0, 3)
