"""Attractor sets: bundled fixtures and exhaustive discovery for small networks.

The reference reads attractor sets from ``env.attracting_states`` /
``env.all_attractors`` (bdq_model/__init__.py:60,182-183) as
``list[attractor] of list[state tuple]``, with ``'*'`` wildcards mapped to 0
by its evaluation loop (model_tester.py:609).  Those sets come from gym-PBN
internals (absent) or from pickles in data/ and bns_attractors/.  This round the
pickles are not loaded: the only permitted safe loader,
``torch.load(weights_only=True)``, refuses them (pickle protocol-4 FRAME opcode),
so:
  * Bittner-28 uses the 14 singleton states transcribed in SURVEY.md
    Appendix B (derived from data/attractors_Bittner-28.pkl); the compiler
    re-checks that each is a possible fixed point with the self-loop
    probabilities the survey lists;
  * small networks (N <= 20) get their attractors by exhaustive search of the
    state-transition graph: the bottom strongly connected components with no
    perturbation and no intervention -- the same definition print_graph.py:15-34
    uses (``genSTG`` + SCC condensation sinks).
"""
from __future__ import annotations

import json
import os
from typing import List, Sequence, Tuple

import numpy as np

from .network import NETWORK_DIR, Network

__all__ = ["find_attractors", "load_attractors", "clean_state", "Attractors"]

Attractors = List[List[Tuple[int, ...]]]


def clean_state(state: Sequence) -> Tuple[int, ...]:
    """'*' wildcard -> 0 (model_tester.py:609), everything else -> int 0/1."""
    return tuple(0 if v == "*" else int(v) for v in state)


def _successor_options(net: Network, s: int, prob_bits: int = 16) -> List[Tuple[int, ...]]:
    """Values each node can take next from state s, over the functions whose quantised weight
    at ``prob_bits`` is non-zero (the functions the kernel can select)."""
    bits = [(s >> i) & 1 for i in range(net.n)]
    opts = []
    thr = net.thresholds(prob_bits)
    for i, fl in enumerate(net.nodes):
        vals = set()
        prev = 0
        for f, c in zip(fl, thr[i]):
            if c > prev:
                vals.add(f(bits))
            prev = c
        opts.append(tuple(sorted(vals)))
    return opts


def find_attractors(net: Network, max_nodes: int = 20, prob_bits: int = 16) -> Attractors:
    """Bottom SCCs of the asynchronous-free synchronous PBN STG (exhaustive)."""
    n = net.n
    if n > max_nodes:
        raise ValueError(f"exhaustive attractor search limited to {max_nodes} nodes (got {n})")
    total = 1 << n
    succ: List[List[int]] = []
    for s in range(total):
        opts = _successor_options(net, s, prob_bits)
        nexts = [0]
        for i, vals in enumerate(opts):
            if len(vals) == 1:
                nexts = [x | (vals[0] << i) for x in nexts]
            else:
                nexts = [x | (v << i) for x in nexts for v in vals]
        succ.append(nexts)
    # iterative Tarjan
    index = [-1] * total
    low = [0] * total
    on = [False] * total
    stack: List[int] = []
    comp = [-1] * total
    comps: List[List[int]] = []
    counter = 0
    for root in range(total):
        if index[root] != -1:
            continue
        work = [(root, 0)]
        while work:
            v, pi = work.pop()
            if pi == 0:
                index[v] = low[v] = counter
                counter += 1
                stack.append(v)
                on[v] = True
            recurse = False
            for k in range(pi, len(succ[v])):
                w = succ[v][k]
                if index[w] == -1:
                    work.append((v, k + 1))
                    work.append((w, 0))
                    recurse = True
                    break
                elif on[w]:
                    low[v] = min(low[v], index[w])
            if recurse:
                continue
            if low[v] == index[v]:
                members = []
                while True:
                    w = stack.pop()
                    on[w] = False
                    comp[w] = len(comps)
                    members.append(w)
                    if w == v:
                        break
                comps.append(members)
            if work:
                u = work[-1][0]
                low[u] = min(low[u], low[v])
    bottoms = []
    for ci, members in enumerate(comps):
        if all(comp[w] == ci for m in members for w in succ[m]):
            bottoms.append(sorted(members))
    bottoms.sort(key=lambda ms: ms[0])
    return [[tuple(net.unpack([m & 0xFFFFFFFF, (m >> 32) & 0xFFFFFFFF][:net.words])) for m in ms]
            for ms in bottoms]


def load_attractors(name: str) -> Attractors:
    """Bundled attractor set ``networks/<name>_attractors.json``."""
    path = os.path.join(NETWORK_DIR, f"{name}_attractors.json")
    with open(path) as f:
        obj = json.load(f)
    return [[clean_state(s) for s in att] for att in obj["attractors"]]


def random_state_targets(n_nodes: int, count: int, seed: int) -> Attractors:
    """Seeded random singleton 'attractors' (target sets for networks with no fixture, e.g. pbn70)."""
    rng = np.random.default_rng(seed)
    seen = set()
    out: Attractors = []
    while len(out) < count:
        s = tuple(int(b) for b in rng.integers(0, 2, size=n_nodes))
        if s not in seen:
            seen.add(s)
            out.append([s])
    return out
