"""model_tester.py:587-648 on the GPU: the trained pbn7 agent steered through pbn_step.

Every (start, target) pair of the reference's four pbn7 attractors runs R times side by side
in one VectorPBNEnv (no autoreset, no horizon): the env starts in the start attractor's first
state ('*' -> 0, :609); each step the agent (tests/golden/pbn7_bdq_final.npz, greedy, :600)
sees (state, target's first state), its three branch argmaxes become a flip mask (distinct
nodes once, bdq_model/__init__.py:176) and pbn_step advances every env; an env's count is the
first step at which its state lies in the target attractor (:616), 101 if none within 100
(:628).  The per-pair mean counts must equal the exact law's (oracle/law.py) within 5
standard errors of the Monte Carlo mean: the kernel's law, driven by the agent, is the
frozen law.  Against the reference's own recorded lengths the comparison is expected to fail
(see tests/test_law_pin.py and DESIGN.md 'Parity status').
"""
import itertools

import numpy as np
import pytest
import torch

from oracle import law
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv, actions_to_flipmask, pack_states, unpack_states
from tests.test_law_pin import pbn7_agent, q_numpy, ref_pbn7_attractors

pytestmark = pytest.mark.gpu

P = 0.01
REPEATS = 2048
MAX_STEPS = 100


def gpu_protocol(seed=5):
    net = load_network("pbn7")
    atts = ref_pbn7_attractors()
    pairs = list(itertools.product(range(len(atts)), repeat=2))
    spec = EnvSpec(net, [[tuple(s) for s in a] for a in atts], perturbation=P, horizon=0)
    n = len(pairs) * REPEATS
    dev = torch.device("cuda:0")
    env = VectorPBNEnv(spec, n, seed=seed, device=dev, autoreset=False, keep_final_state=False)
    env.reset()
    starts = torch.tensor([atts[a][0] for a, t in pairs for _ in range(REPEATS)], dtype=torch.int64, device=dev)
    tid = torch.tensor([t for a, t in pairs for _ in range(REPEATS)], dtype=torch.int64, device=dev)
    env.set_state(pack_states(starts, net.n), target=tid.to(torch.uint8), t=torch.zeros(n, dtype=torch.uint8, device=dev))
    tgt_bits = torch.tensor([atts[t][0] for a, t in pairs for _ in range(REPEATS)], dtype=torch.float32, device=dev)
    q = pbn7_agent().to(dev)
    count = torch.full((n,), MAX_STEPS + 1, dtype=torch.int64, device=dev)
    done = torch.tensor([a == t for a, t in pairs for _ in range(REPEATS)], device=dev)
    count[done] = 0
    with torch.no_grad():
        for k in range(1, MAX_STEPS + 1):
            s = unpack_states(env.state[:, :n], net.n).to(torch.float32)
            acts = q(torch.stack([s, tgt_bits])).argmax(dim=2)           # (n, 3)
            _, _, flags = env.step_flipmask(actions_to_flipmask(acts, net.n, check=False))
            hit = (flags & 1).bool() & ~done                               # FLAG_TERMINATED: s' in target
            count[hit] = k
            done |= hit
            if bool(done.all()):
                break
    torch.cuda.synchronize()
    env.close()
    return pairs, count.view(len(pairs), REPEATS).cpu().numpy()


def test_gpu_agent_protocol_matches_exact_law():
    pairs, counts = gpu_protocol()
    exact = law.evaluate_protocol(load_network("pbn7"), ref_pbn7_attractors(), q_numpy(pbn7_agent()), P)
    for i, pair in enumerate(pairs):
        mean, var, fail = law.pair_statistics(exact[pair])
        mc = counts[i].astype(np.float64)
        se = np.sqrt(var / REPEATS)
        assert abs(mc.mean() - mean) <= 5 * se + 1e-9, (pair, mc.mean(), mean, se)


@pytest.mark.xfail(strict=True, reason="kaban/pbn7.ispl under the frozen law is not the network the pbn7 agent was "
                                        "trained on (DESIGN.md 'Parity status')")
def test_gpu_agent_protocol_matches_reference():
    """The reference recorded a pooled mean of 1.58 steps over its 12 off-diagonal pairs x 10
    runs (data/results/pbn_7_4.pkl); tolerance 3 standard errors of that mean (0.106)."""
    pairs, counts = gpu_protocol()
    off = [i for i, (a, t) in enumerate(pairs) if a != t]
    assert abs(counts[off].mean() - 1.583) < 3 * 0.106
