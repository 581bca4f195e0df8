"""The settle law on the GPU (include/pbn_env.h "Step law"): kernels == oracle bit for bit, and
the reference's bb33 evaluation replayed through the gym facade on the device.

pbn_step and pbn_rollout run the wave kernel's settle variants (3, 4) when the descriptor's
settle_max >= 2; every output is compared with oracle/pbn_oracle.c, including the
PBN_FLAG_UNSETTLED bit of envs that hit the cap.
"""
import numpy as np
import pytest

from pbn_rl_amd import _lib
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.env import PBNEnv
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec

from .protocol import load_agent, replay, summary
from .synthetic import random_spec
from .test_bn_pin import reference_result
from .test_gpu_parity import run_pair, run_rollout_pair

pytestmark = pytest.mark.gpu


def settle_spec(name, settle, **kw):
    return EnvSpec(load_network(name), load_attractors(name), settle=settle, **kw)


@pytest.mark.parametrize("name", ["pbn7", "pbn28", "pbn70", "bb33"])
@pytest.mark.parametrize("settle", [2, 9])
def test_settle_step_matches_oracle(name, settle):
    spec = settle_spec(name, settle, perturbation=0.02, horizon=6)
    run_pair(spec, 2048, 6, mode=3, env_offset=1024)
    run_pair(spec, 1024, 4, mode=0, start_random=True)


@pytest.mark.parametrize("name", ["pbn28", "pbn70", "bb33"])
def test_settle_rollout_matches_oracle(name):
    spec = settle_spec(name, 12, perturbation=0.05, horizon=7)
    run_rollout_pair(spec, 2080, 8, 3)
    run_rollout_pair(spec, 1024, 5, 1)


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
