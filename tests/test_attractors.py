"""Attractor discovery (bottom SCCs, print_graph.py:15-34 definition) and fixtures."""
from pbn_rl_amd.attractors import clean_state, find_attractors, load_attractors
from pbn_rl_amd.network import load_network


def test_pbn7_attractors():
    atts = find_attractors(load_network("pbn7"))
    # 4 attractors; 3 absorbing fixed points (SURVEY.md 8(c) fixture 2) + one 4-state cycle set
    assert sorted(len(a) for a in atts) == [1, 1, 1, 4]
    assert atts == load_attractors("pbn7")


def test_fixed_points_are_absorbing():
    net = load_network("pbn7")
    for att in find_attractors(net):
        if len(att) == 1:
            s = list(att[0])
            vals = net.function_values(s)
            assert all(all(v == s[i] for v in vals[i]) for i in range(net.n))


def test_pbn10_bundle_consistent():
    assert find_attractors(load_network("pbn10")) == load_attractors("pbn10")


def test_wildcard():
    assert clean_state(["*", 1, "0", 0]) == (0, 1, 0, 0)
