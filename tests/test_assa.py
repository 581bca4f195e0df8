"""ASSA-PBN / MATLAB truth-table loader (train_assa_matlab_BQN.py:72-171), CPU."""
import itertools

import pytest

from pbn_rl_amd.assa import parse_assa, write_assa
from pbn_rl_amd.network import Network, load_network

from .synthetic import random_network

SAMPLE = """ASSA-PBN
generated
3
2 1 1
2 1 2 2
0 1 1 1
1 0
0 1 1 0
1 0 0 0
1 2
0
0 2
1 2
0.7 0.3
1.0
1.0
0.001
"""


def test_sample_file_semantics():
    a = parse_assa(SAMPLE)
    assert a.genes == ["x0", "x1", "x2"] and a.perturbation_rate == 0.001
    net = a.network()
    # gene 0, function 0: predictors (x1, x2), outputs over product order (x1 MSB): 0 1 1 1 = OR
    # gene 0, function 1: predictor x0, outputs 1 0 = NOT x0
    # gene 1: predictors (x0, x2): 0 1 1 0 = XOR ; gene 2: (x1, x2): 1 0 0 0 = NOR
    cases = {0: [lambda s: s[1] | s[2], lambda s: 1 - s[0]], 1: [lambda s: s[0] ^ s[2]],
             2: [lambda s: 1 - (s[1] | s[2])]}
    for s in itertools.product([0, 1], repeat=3):
        for node, fns in cases.items():
            assert [f(list(s)) for f in net.nodes[node]] == [g(s) for g in fns]
    w = [f.weight for f in net.nodes[0]]
    assert float(w[0] / sum(w)) == pytest.approx(0.7)


@pytest.mark.parametrize("name", ["pbn7", "pbn10", "pbn28"])
def test_round_trip_bundled_networks(name):
    net = load_network(name)
    back = parse_assa(write_assa(net, 0.02)).network()
    assert [[(f.inputs, f.table) for f in fl] for fl in back.nodes] == \
           [[(f.inputs, f.table) for f in fl] for fl in net.nodes]
    assert back.thresholds(16) == net.thresholds(16)


def test_round_trip_random_network_with_constants():
    net = random_network(8, 5, max_funcs=4)
    back = parse_assa(write_assa(net)).network()
    assert [[(f.inputs, f.table) for f in fl] for fl in back.nodes] == \
           [[(f.inputs, f.table) for f in fl] for fl in net.nodes]


def test_matches_sympy_sop_route():
    """The reference's own route (minterms -> sympy SOPform -> translate) compiles to the same tables."""
    sympy = pytest.importorskip("sympy")
    from sympy.logic import SOPform

    a = parse_assa(SAMPLE)
    ref_lf = {}
    for node, fl in a.logic_functions.items():
        ref_lf[node] = []
    # rebuild the reference expressions from the sample's tables
    rows = SAMPLE.strip().splitlines()
    tables = [[float(x) for x in r.split()] for r in rows[5:9]]
    preds = [r.split() for r in rows[9:13]]
    owner = [0, 0, 1, 2]
    for t, p, node in zip(tables, preds, owner):
        syms = sympy.symbols(",".join(f"x{i}" for i in p))
        syms = syms if isinstance(syms, tuple) else (syms,)
        minterms = [list(st) for st, out in zip(itertools.product([0, 1], repeat=len(p)), t) if out]
        expr = str(SOPform(syms, minterms, [])).replace("~", "not ").replace("|", " or ").replace("&", " and ")
        ref_lf[node].append((expr, 1.0))
    ref = Network.from_logic_functions(a.genes, ref_lf)
    ours = a.network()
    assert [[(f.inputs, f.table) for f in fl] for fl in ref.nodes] == \
           [[(f.inputs, f.table) for f in fl] for fl in ours.nodes]


def test_rejects_inconsistent_counts():
    bad = SAMPLE.replace("2 1 2 2", "2 1 2")
    with pytest.raises(ValueError):
        parse_assa(bad)
