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
