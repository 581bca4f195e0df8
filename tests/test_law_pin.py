"""The reference's own data against the frozen semantics (CPU).

tests/golden/ref_fixtures.json holds the reference pickles' contents, read by a static opcode
walk (tools/ref_pickles.py: nothing unpickled); tests/golden/pbn7_bdq_final.npz the trained
pbn7 agent (tools/export_pbn7_agent.py, torch.load weights_only).  oracle/law.py is the exact
transition law of DESIGN.md "Step semantics".
"""
import itertools
import json
import os

import numpy as np
import pytest
import torch

from oracle import law, oracle
from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def fixtures():
    with open(os.path.join(GOLD, "ref_fixtures.json")) as f:
        return json.load(f)


def expand(pattern):
    """A '*' pattern -> the states it stands for, its '*' -> 0 state first (model_tester.py:609)."""
    first = [0 if v == "*" else v for v in pattern]
    opts = [[0, 1] if v == "*" else [v] for v in pattern]
    rest = [list(s) for s in itertools.product(*opts) if list(s) != first]
    return [first] + rest


def ref_pbn7_attractors():
    """data/attractors_Bittner-7.pkl in its own order, wildcards expanded (pickle order =
    kaban/pbn7.ispl order)."""
    return [expand(att[0]) for att in fixtures()["attractors_Bittner-7"]["value"]]


def pbn7_agent():
    w = np.load(os.path.join(GOLD, "pbn7_bdq_final.npz"))
    q = BranchingQNetwork((7, 7), 8, 3)
    q.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    return q.eval()


def q_numpy(q):
    def fn(states, targets):
        with torch.no_grad():
            return q(torch.from_numpy(np.stack([states, targets]).astype(np.float32))).numpy()
    return fn


# ------------------------------------------------------------------- fixtures themselves
def test_results_pickle_summary_matches_survey():
    """data/results/pbn_7_4.pkl: SURVEY.md section 6 transcribes it as mean strategy length
    1.58 (excluding 0) and 0 failures of 160."""
    res = fixtures()["results_pbn_7_4"]["value"]
    data = {int(k): v for k, v in res["data"].items()}
    assert sum(data.values()) == 160
    assert data.get(101, 0) == 0
    nz = {k: v for k, v in data.items() if k > 0}
    mean = sum(k * v for k, v in nz.items()) / sum(nz.values())
    assert abs(mean - 1.58) < 0.005
    m = np.array(res["save_matrix"])
    assert m.shape == (4, 4) and np.all(np.diag(m) == 0)
    assert m.sum() == sum(k * v for k, v in data.items())


def test_bundled_attractors_equal_reference_pickles():
    """The bundled attractor sets are the reference pickles' (read statically this round):
    pbn7 in file order, pbn10 in lexicographic gene order, Bittner-28 in numeric gene-ID
    order."""
    fx = fixtures()
    # pbn7: same attractors (as state sets); '*' patterns expand to the multi-state attractor
    ours = {frozenset(map(tuple, a)) for a in load_attractors("pbn7")}
    ref = {frozenset(map(tuple, a)) for a in ref_pbn7_attractors()}
    assert ours == ref
    # Bittner-28: pickle index = rank of the gene's numeric ID; the bundled 14 states are the
    # pickle's (the SURVEY Appendix B transcription)
    net28 = load_network("pbn28")
    num = sorted(range(net28.n), key=lambda i: int(net28.genes[i].lstrip("x")))
    ref28 = [tuple(int(att[0][num.index(i)]) for i in range(net28.n)) for att in fx["attractors_Bittner-28"]["value"]]
    ours28 = [a[0] for a in load_attractors("pbn28")]
    assert sorted(ref28) == sorted(ours28) and len(ref28) == 14


def test_pseudo_attractor_fixtures_are_possible_fixed_points():
    """The pbn10 and Bittner-28 pickles list the fork's *pseudo*-attractors (train_BDQ.py:106
    prints "final pseudo attractors"), not bottom SCCs: every listed state is a possible fixed
    point of the ISPL network (P(s -> s) > 0), but only 3 of pbn10's 6 and 5 of Bittner-28's
    14 lie in bottom SCCs of its transition graph (the bundled pbn10 set and the discovery
    of DESIGN.md 'Next' 2 use the bottom-SCC definition of print_graph.py:15-34)."""
    fx = fixtures()
    net10 = load_network("pbn10")
    lex = sorted(range(net10.n), key=lambda i: net10.genes[i])   # pickle index j = j-th gene, lexicographic
    ref10 = [tuple(int(att[0][lex.index(i)]) for i in range(net10.n)) for att in fx["attractors_pbn10"]["value"]]
    assert all(net10.self_loop_probability(list(s)) > 0 for s in ref10)
    ours10 = {s for a in load_attractors("pbn10") for s in a}
    assert sum(s in ours10 for s in ref10) == 3
    net28 = load_network("pbn28")
    assert all(net28.self_loop_probability(list(a[0])) > 0 for a in load_attractors("pbn28"))


# ------------------------------------------------------------------- law.py vs the C oracle
@pytest.mark.parametrize("p", [0.0, 0.05])
def test_exact_law_matches_oracle_frequencies(p):
    """law.transition_matrix is the law the oracle (hence the kernels) samples: one step of
    65,536 envs from each of three states, chi-square against the exact row."""
    net = load_network("pbn7")
    spec = EnvSpec(net, load_attractors("pbn7"), perturbation=p, horizon=0)
    T = law.transition_matrix(net, p)
    n = 65536
    for s1 in (0b1010001, 0b0110100, 0b1111111):
        st = np.full((1, n), s1, dtype=np.uint32)
        out = oracle.step(spec, 11, 1, 0, st, np.zeros_like(st), np.full(n, 255, np.uint8),
                          np.zeros(n, np.uint8), 0, want_final=False)
        counts = np.bincount(out["state_out"][0], minlength=128)
        expect = T[s1] * n
        assert counts[expect == 0].sum() == 0, "oracle reached a state the law forbids"
        live = expect > 5
        chi2 = (((counts[live] - expect[live]) ** 2) / expect[live]).sum()
        dof = max(int(live.sum()) - 1, 1)
        assert chi2 < dof + 6 * np.sqrt(2 * dof) + 10, (s1, chi2, dof)


# ------------------------------------------------------------------- the trained-agent pin
def exact_protocol(p=0.01):
    net = load_network("pbn7")
    atts = ref_pbn7_attractors()
    return law.evaluate_protocol(net, atts, q_numpy(pbn7_agent()), p)


def pooled_mean(res):
    means = [law.pair_statistics(d)[0] for (a, t), d in res.items() if a != t]
    return float(np.mean(means))


def test_protocol_distribution_is_well_formed():
    res = exact_protocol()
    for (a, t), d in res.items():
        assert abs(d.sum() - 1.0) < 1e-9
        if a == t:
            assert d[0] == 1.0


@pytest.mark.xfail(strict=True, reason="the trained pbn7 agent does not control kaban/pbn7.ispl under the frozen "
                                        "law (exact mean ~30 steps vs the reference's 1.58): the network it was "
                                        "trained on (a BittnerMultiGeneral draw) is not in the reference; "
                                        "DESIGN.md 'Parity status'")
def test_trained_agent_reproduces_reference_strategy_lengths():
    """model_tester.py:587-658 exactly, at p = 0.01: the pooled mean strategy length of the
    12 off-diagonal pairs must lie within 3 standard errors of the reference's 1.58 (SE of
    the reference's own 120-run mean: 0.106)."""
    assert abs(pooled_mean(exact_protocol()) - 1.583) < 3 * 0.106


# ------------------------------------------------------------------- pbn10 under both laws
def pbn10_protocol(settle, order="lex", p=0.01):
    """model_tester.py:587-658 for the trained pbn10 agent (models/pbn10/bdq_final.pt) on
    kaban/pbn10.ispl, exactly, with the six data/attractors pbn10 fixture states as the env's
    attractor set; ``order``: the gene order the agent and the fixture rows are in (the pickle
    is lexicographic)."""
    net = load_network("pbn10")
    perm = (sorted(range(net.n), key=lambda i: net.genes[i]) if order == "lex" else list(range(net.n)))
    fx = fixtures()["attractors_pbn10"]["value"]
    # our node perm[k] is the agent's / fixture's position k
    atts = [[tuple(int(att[0][perm.index(i)]) for i in range(net.n))] for att in fx]
    w = np.load(os.path.join(GOLD, "pbn10_bdq_final.npz"))
    q = BranchingQNetwork((10, 10), 11, 3)
    q.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    q.eval()

    def q_fn(states, targets):   # our order -> the agent's order and back
        with torch.no_grad():
            x = torch.from_numpy(np.stack([states[:, perm], targets[:, perm]]).astype(np.float32))
            out = q(x).numpy()                                   # actions index the agent's order
        mapped = np.zeros_like(out)
        mapped[:, :, 0] = out[:, :, 0]
        for k in range(net.n):                                   # agent action k+1 flips our perm[k]
            mapped[:, :, perm[k] + 1] = out[:, :, k + 1]
        return mapped
    return law.evaluate_protocol(net, atts, q_fn, p, settle=settle)


@pytest.mark.xfail(strict=True, reason="the trained pbn10 agent was not trained on kaban/pbn10.ispl with the "
                                        "fixture's attractors under either law: in lexicographic gene order the "
                                        "settle law brings the expected failures from 56.7 to 3.7 of 360 (the "
                                        "reference: 0), but 80.7 one-step runs against the reference's 213 "
                                        "(DESIGN.md 'Parity status')")
def test_pbn10_agent_reproduces_reference_under_settle_law():
    """data/results/pbn_10_6.pkl: 360 runs, 0 failures, 213 of them one step."""
    res = pbn10_protocol(settle=1000)
    data = sum(d for d in res.values()) * 10
    assert data[101] < 1.0 and abs(data[1] - 213) < 3 * np.sqrt(213)
