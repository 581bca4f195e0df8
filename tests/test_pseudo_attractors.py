"""Candidate attractor notions against the reference's pseudo-attractor fixtures (VERDICT r04
next 6; tools/pseudo_attractors.py, profiles/r05_pseudo_attractors.json; DESIGN.md "Parity
status").  A documented negative result: no notion computed from the ISPL network alone equals
data/attractors_Bittner-28.pkl or bns_attractors/10_3_attractors.pkl, so PBNEnv keeps growing
its attractor set as bottom SCCs (print_graph.py:15-34).  The one positive structural finding is
checked too: the 14 Bittner-28 states are fixed points of one Boolean network inside the PBN
(one function per node), which random subsets of the possible fixed points never are."""
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "tools"))

import pseudo_attractors as pa  # noqa: E402

TABLE = os.path.join(ROOT, "profiles", "r05_pseudo_attractors.json")


def test_committed_table_has_no_matching_notion():
    d = json.load(open(TABLE))
    for name, size in (("pbn10", 6), ("pbn28", 14)):
        assert d[name]["fixture_size"] == size
        assert not any(v["equals_fixture"] for v in d[name]["notions"].values()), name
    # what PBNEnv grows today (bottom SCCs) holds 3 of 6 and 5 of 14 (tests/test_law_pin.py)
    assert d["pbn10"]["notions"]["bottom_scc"]["hits"] == 3
    assert d["pbn28"]["notions"]["bottom_scc"]["hits"] == 5


def test_pbn10_notions_recomputed():
    d = json.load(open(TABLE))["pbn10"]
    res = pa.score("pbn10")
    for k, v in res["notions"].items():
        assert v == d["notions"][k], k
    assert res["bn_slice"]["consistent"] is False


def test_bittner28_states_are_fixed_points_of_one_boolean_network():
    net, fix = pa.fixture_states("pbn28")
    P = pa.possible_fixed_points(net)
    assert P.size == 218916 and np.isin(fix, P).all()
    sl = pa.slice_consistency(net, fix, P, trials=200, greedy=False)
    assert sl["consistent"] and sl["random_subsets_consistent"] == "0/200"
