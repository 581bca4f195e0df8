"""Seeded random PBNs for tests: the paths the kaban networks never take.

Every kaban network has 2-3 functions per node with weights 1 (a few merged duplicates).
These networks add nodes with up to 6 distinct functions (the > kNodeRecs chain tail),
arbitrary relative weights (per-node thresholds), constant (arity 0) functions, node counts
that give 1..4 state words, and (max_arity > 4) wide functions that need gates.
"""
from fractions import Fraction

import numpy as np

from pbn_rl_amd.attractors import random_state_targets
from pbn_rl_amd.network import Network, NodeFunction, _reduce
from pbn_rl_amd.spec import EnvSpec


def random_network(n_nodes: int, seed: int, max_funcs: int = 6, max_arity: int = 4) -> Network:
    rng = np.random.default_rng(seed)
    nodes = []
    for i in range(n_nodes):
        nf = int(rng.integers(1, max_funcs + 1))
        funcs, seen = [], set()
        while len(funcs) < nf:
            k = int(rng.integers(0, min(max_arity, n_nodes) + 1))
            ins = [int(x) for x in rng.choice(n_nodes, size=k, replace=False)]
            if (1 << k) <= 32:
                table = int(rng.integers(0, 1 << (1 << k)))
            else:   # wide functions (k >= 6): a random 2^k-bit table
                table = int.from_bytes(rng.bytes((1 << k) // 8), "little")
            key = _reduce(ins, table)
            if key in seen:
                continue
            seen.add(key)
            funcs.append(NodeFunction(key[0], key[1], Fraction(int(rng.integers(1, 10))), []))
        nodes.append(funcs)
    return Network([f"g{i}" for i in range(n_nodes)], nodes, name=f"rand{n_nodes}_{seed}")


def random_spec(n_nodes: int, seed: int, n_targets: int = 8, max_funcs: int = 6, **kw) -> EnvSpec:
    net = random_network(n_nodes, seed, max_funcs=max_funcs)
    return EnvSpec(net, random_state_targets(n_nodes, n_targets, seed + 1), **kw)
