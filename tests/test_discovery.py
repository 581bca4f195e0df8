"""Attractor verification (host half of pbn_rl_amd.discovery), CPU: seeded with every state of a
small network, the bounded successor closure + bottom-SCC filter must return exactly the
exhaustive STG search of attractors.find_attractors (the print_graph.py:15-34 definition)."""
import itertools

import numpy as np
import pytest

from pbn_rl_amd.attractors import find_attractors, load_attractors
from pbn_rl_amd.discovery import bottom_sccs, successor_boxes
from pbn_rl_amd.network import load_network

from .synthetic import random_network


def all_states(n):
    return np.array(list(itertools.product([0, 1], repeat=n)), dtype=np.uint8)[:, ::-1]


@pytest.mark.parametrize("name", ["pbn7", "pbn10"])
def test_bottom_sccs_equal_exhaustive(name):
    net = load_network(name)
    assert bottom_sccs(net, all_states(net.n)) == find_attractors(net)


def test_pbn7_matches_fixture():
    net = load_network("pbn7")
    got = {frozenset(a) for a in bottom_sccs(net, all_states(7))}
    assert got == {frozenset(a) for a in load_attractors("pbn7")}


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_random_networks_equal_exhaustive(seed):
    net = random_network(9, seed, max_funcs=3)
    assert bottom_sccs(net, all_states(9)) == find_attractors(net)


def test_closure_from_one_state_finds_its_attractor():
    """Seeding with a single state inside an attractor closes it (the simulation may visit only
    part of a cyclic attractor)."""
    net = load_network("pbn10")
    for att in find_attractors(net):
        seed = np.array([att[-1]], dtype=np.uint8)
        assert bottom_sccs(net, seed) == [att]


def test_successor_boxes_agree_with_function_values():
    net = load_network("pbn28")
    rng = np.random.default_rng(0)
    bits = rng.integers(0, 2, size=(64, 28)).astype(np.uint8)
    can0, can1 = successor_boxes(net, bits)
    for r in range(64):
        vals = net.function_values(list(bits[r]))
        for i, fv in enumerate(vals):
            assert can1[r, i] == (1 in fv) and can0[r, i] == (0 in fv)


def test_capped_expansion_never_reports_unverified_sets():
    net = load_network("pbn10")
    got = bottom_sccs(net, all_states(10), max_box=1)
    exact = find_attractors(net)
    assert all(a in exact for a in got)


@pytest.mark.parametrize("name", ["bb33", "m47"])
def test_successor_boxes_wide_functions(name):
    """Functions of arity >= 6 (bb33: 6, model_tester.py's 47-node network: 20) have truth
    tables wider than an int64 shift; the boxes must still equal the per-state function values."""
    net = load_network(name)
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2, size=(32, net.n)).astype(np.uint8)
    can0, can1 = successor_boxes(net, bits)
    for r in range(32):
        vals = net.function_values(list(bits[r]))
        for i, fv in enumerate(vals):
            assert can1[r, i] == (1 in fv) and can0[r, i] == (0 in fv)


def test_find_attractors_threads_prob_bits():
    """At prob_bits = 4 a function whose weight quantises to 0 adds no STG edge (the kernel can
    never select it), so the exhaustive search must use the same quantisation."""
    from fractions import Fraction

    from pbn_rl_amd.network import Network, NodeFunction

    f_keep = NodeFunction((0,), 0b10, Fraction(1000))   # x0' = x0
    f_flip = NodeFunction((0,), 0b01, Fraction(1))      # x0' = not x0: weight 0 at 4 bits
    net = Network(["a"], [[f_keep, f_flip]], name="q")
    assert net.thresholds(4)[0][0] == 16        # all mass on f_keep
    assert find_attractors(net, prob_bits=4) == [[(0,)], [(1,)]]
    assert find_attractors(net, prob_bits=16) == [[(0,), (1,)]]


def test_escalating_discovery_keeps_a_callers_burn_in(monkeypatch):
    """a burn_in given by the caller replaces the default ladder (CPU: the GPU
    simulation is replaced by a spy)."""
    from pbn_rl_amd import discovery
    from pbn_rl_amd.network import load_network
    seen = []
    monkeypatch.setattr(discovery, "discover_attractors", lambda net, **kw: seen.append(kw) or [])
    discovery.discover_attractors_escalating(load_network("pbn7"), burn_in=50000, chains=64)
    assert [kw["burn_in"] for kw in seen] == [50000] and seen[0]["chains"] == 64
    seen.clear()
    discovery.discover_attractors_escalating(load_network("pbn7"), burn_ins=(10, 20), burn_in=5)
    assert [kw["burn_in"] for kw in seen] == [10, 20]
    seen.clear()
    discovery.discover_attractors_escalating(load_network("pbn7"))
    assert [kw["burn_in"] for kw in seen] == [1000, 5000, 20000]
