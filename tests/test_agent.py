"""Config 5 (BDQ rollout) host side, CPU: the restated BranchingQNetwork against the
reference module's outputs (tests/golden/bdq_forward.npz, tools/gen_bdq_golden.py), the
reference checkpoint loading into it, and the agent-edge oracle's own pieces.

Tolerance for the Q-network (fp32): |ours - reference| <= 1e-5 + 1e-5 |reference|; the
bilinear layer is summed in a different order (one GEMM over the outer product).
"""
import os

import numpy as np
import pytest
import torch

from oracle import agent_oracle, pyoracle
from pbn_rl_amd.agent import BranchingQNetwork, formula_weights, load_bdq_checkpoint
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "bdq_forward.npz")
ATOL, RTOL = 1e-5, 1e-5


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


def test_qnet_matches_reference_forward(golden):
    net = formula_weights(BranchingQNetwork((28, 28), 29, 3))
    with torch.no_grad():
        q = net(torch.from_numpy(golden["formula_x"].astype(np.float32))).numpy()
    assert q.shape == (96, 3, 29)
    np.testing.assert_allclose(q, golden["formula_q"], atol=ATOL, rtol=RTOL)


def test_qnet_parameter_count_and_names():
    net = BranchingQNetwork((28, 28), 29, 3)
    assert sum(p.numel() for p in net.parameters()) == 258360
    names = set(dict(net.named_parameters()))
    assert "model.0.bilinear.weight" in names and "adv_heads.2.2.bias" in names


def test_reference_checkpoint_loads(reference_dir, golden):
    path = os.path.join(reference_dir, "models", "pbn7", "bdq_final.pt")
    net = load_bdq_checkpoint(BranchingQNetwork((7, 7), 8, 3), path)
    with torch.no_grad():
        q = net(torch.from_numpy(golden["pbn7_x"].astype(np.float32))).numpy()
    np.testing.assert_allclose(q, golden["pbn7_q"], atol=ATOL, rtol=RTOL)


def test_vectorised_philox_matches_scalar():
    rng = np.random.default_rng(3)
    for _ in range(32):
        ctr = rng.integers(0, 2 ** 32, size=4, dtype=np.uint64)
        key = rng.integers(0, 2 ** 32, size=2, dtype=np.uint64)
        got = agent_oracle.philox_vec(*[np.array([c]) for c in ctr], int(key[0]), int(key[1]))
        assert tuple(int(g[0]) for g in got) == pyoracle.philox4x32(ctr, key)
        got10 = agent_oracle.philox_vec(*[np.array([c]) for c in ctr], int(key[0]), int(key[1]), rounds=10)
        assert tuple(int(g[0]) for g in got10) == pyoracle.philox4x32_10(ctr, key)
    w = agent_oracle.explore_words(7, 11, 64, 4)
    for e in range(4):
        assert tuple(int(x[e]) for x in w) == pyoracle.draw(7, 64 + e, 11, agent_oracle.EXPLORE, 0)


def test_argmax_follows_torch():
    q = np.array([[1.0, 3.0, 3.0, 0.0], [np.nan, 1.0, np.nan, 5.0], [2.0, np.nan, 9.0, 9.0], [-1, -1, -1, -1]],
                 dtype=np.float32)
    assert np.array_equal(agent_oracle.argmax_torch(q), torch.argmax(torch.from_numpy(q), dim=1).numpy())


def test_q_to_flipmask_oracle_semantics():
    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"))
    q = np.zeros((64, 3, 8), dtype=np.float32)
    q[:, 0, 3] = 1.0      # branch 0 -> action 3 (node 2)
    q[:, 1, 3] = 1.0      # duplicate of branch 0: flips once
    q[:, 2, 0] = 1.0      # no-op
    flip, act = agent_oracle.q_to_flipmask(spec, q, 1, 2, 0, 0.0)
    assert (act == np.array([3, 3, 0])).all()
    assert (flip == 1 << 2).all()
    _, act1 = agent_oracle.q_to_flipmask(spec, q, 1, 2, 0, 1.0)   # always explore
    assert ((act1 >= 0) & (act1 <= 7)).all() and not (act1 == np.array([3, 3, 0])).all(axis=1).all()


def test_obs_unpack_oracle():
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    st = np.array([[0x1, 0x8000000]], dtype=np.uint32)
    obs = agent_oracle.obs_unpack(spec, st, np.array([0, 0xFF], dtype=np.uint8))
    assert obs.shape == (2, 2, 28)
    assert obs[0, 0, 0] == 1 and obs[0, 0].sum() == 1 and obs[0, 1, 27] == 1
    assert (obs[1, 0] == np.asarray(spec.attractors[0][0], dtype=np.float32)).all()
    assert (obs[1, 1] == 0).all()
