"""Attractor discovery by GPU simulation.

The reference gets attractor sets from gym_PBN internals, from ``graph.genSTG()`` + the sinks
of the SCC condensation (print_graph.py:15-34), or from CABEAN output
(``get_attractors_from_cabean``, model_tester.py:27), and grows ``env.all_attractors`` during
training (bdq_model/__init__.py:182-184).  ``attractors.find_attractors`` restates the STG
definition exhaustively, which is only feasible for about 20 nodes.  Here the search is split:

1. **Simulation (GPU).** ``chains`` copies of the network run without perturbation or
   interventions (``pbn_rollout``, uniform random start states).  Every chain of a finite
   Markov chain is eventually trapped in a bottom SCC of the STG, so the states the chains
   visit after ``burn_in`` steps, over a ``window`` of steps, are the candidates.
2. **Verification (host, exact).**  A state's successors form a box: node i takes any value
   given by one of its functions of non-zero (quantised) weight.  The candidate set is closed
   under successors by a bounded breadth-first expansion.  Tarjan's SCCs on that graph are then
   filtered: a bottom SCC has every successor of every member inside the SCC, and no member
   whose successors were not enumerated.

Every returned set is a bottom SCC, the same definition ``find_attractors`` uses.  Completeness
is probabilistic: an attractor that no chain reached within ``burn_in`` steps is missed.
``tests/test_gpu_discovery.py`` checks the result against the exhaustive search.
"""
from __future__ import annotations

from collections import deque
from typing import Dict, List, Optional, Tuple

import numpy as np

from .attractors import Attractors
from .network import Network

__all__ = ["successor_boxes", "explore", "bottom_sccs", "simulate_visits", "discover_attractors",
           "discover_attractors_escalating", "reached_stg"]


def successor_boxes(net: Network, bits: np.ndarray, prob_bits: int = 16) -> Tuple[np.ndarray, np.ndarray]:
    """bits (S, N) 0/1 -> (can0, can1) bool (S, N): the values node i can take next, over the
    functions with non-zero quantised weight."""
    S, N = bits.shape
    can0 = np.zeros((S, N), dtype=bool)
    can1 = np.zeros((S, N), dtype=bool)
    for i, (fl, thr) in enumerate(zip(net.nodes, net.thresholds(prob_bits))):
        prev = 0
        for f, c in zip(fl, thr):
            if c > prev:
                # the truth table as a byte per row: a Python-int table of arity >= 6 does not
                # fit an int64 shift (bb33, model_tester.py's 47-node network: arity up to 20)
                lut = np.array([(f.table >> m) & 1 for m in range(1 << f.arity)], dtype=np.uint8)
                idx = np.zeros(S, dtype=np.int64)
                for j, g in enumerate(f.inputs):
                    idx |= bits[:, g].astype(np.int64) << j
                v = lut[idx]
                can1[:, i] |= v == 1
                can0[:, i] |= v == 0
            prev = c
    return can0, can1


def _key(bits_row: np.ndarray) -> bytes:
    return np.packbits(bits_row.astype(np.uint8), bitorder="little").tobytes()


def explore(net: Network, candidates: np.ndarray, *, prob_bits: int = 16, max_box: int = 1 << 12,
            max_states: int = 1 << 20) -> Tuple[List[np.ndarray], List[Optional[List[int]]]]:
    """The candidate set ((S, N) 0/1 rows) closed under successors breadth-first: (rows, succ),
    succ[v] = the row indices of v's successors, or None where they were not enumerated (a box
    of more than ``max_box`` states, or ``max_states`` reached)."""
    N = net.n
    index: Dict[bytes, int] = {}
    rows: List[np.ndarray] = []
    for r in np.asarray(candidates, dtype=np.uint8).reshape(-1, N):
        k = _key(r)
        if k not in index:
            index[k] = len(rows)
            rows.append(r.copy())
    succ: List[Optional[List[int]]] = []
    frontier = deque(range(len(rows)))
    while frontier:
        batch = [frontier.popleft() for _ in range(min(len(frontier), 4096))]
        bits = np.stack([rows[v] for v in batch])
        can0, can1 = successor_boxes(net, bits, prob_bits)
        for b, v in enumerate(batch):
            amb = np.nonzero(can0[b] & can1[b])[0]
            while len(succ) <= v:
                succ.append(None)
            if (1 << len(amb)) > max_box or len(index) >= max_states:
                succ[v] = None          # not enumerated: its SCC cannot be certified
                continue
            base = can1[b].astype(np.uint8)
            outs = []
            for m in range(1 << len(amb)):
                t = base.copy()
                for j, node in enumerate(amb):
                    t[node] = (m >> j) & 1
                k = _key(t)
                w = index.get(k)
                if w is None:
                    w = len(rows)
                    index[k] = w
                    rows.append(t)
                    frontier.append(w)
                outs.append(w)
            succ[v] = outs
    while len(succ) < len(rows):
        succ.append(None)
    return rows, succ


def bottom_sccs(net: Network, candidates: np.ndarray, *, prob_bits: int = 16, max_box: int = 1 << 12,
                max_states: int = 1 << 20) -> Attractors:
    """Bottom SCCs reachable from ``candidates`` ((S, N) 0/1 rows), found exactly.

    The candidate set is closed under successors breadth-first (``explore``: at most
    ``max_states`` states; a state with more than ``max_box`` successors is not expanded).  An
    SCC containing a state whose successors were not all enumerated is never reported."""
    rows, succ = explore(net, candidates, prob_bits=prob_bits, max_box=max_box, max_states=max_states)
    total = len(rows)
    # iterative Tarjan over the explored graph
    idx = [-1] * total
    low = [0] * total
    on = [False] * total
    comp = [-1] * total
    stack: List[int] = []
    comps: List[List[int]] = []
    counter = 0
    for root in range(total):
        if idx[root] != -1:
            continue
        work = [(root, 0)]
        while work:
            v, pi = work.pop()
            if pi == 0:
                idx[v] = low[v] = counter
                counter += 1
                stack.append(v)
                on[v] = True
            nxt = succ[v] or []
            recurse = False
            for k in range(pi, len(nxt)):
                w = nxt[k]
                if idx[w] == -1:
                    work.append((v, k + 1))
                    work.append((w, 0))
                    recurse = True
                    break
                if on[w]:
                    low[v] = min(low[v], idx[w])
            if recurse:
                continue
            if low[v] == idx[v]:
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
    def as_int(state):   # bit i = node i, the order find_attractors uses
        return sum(int(b) << i for i, b in enumerate(state))

    out = []
    for ci, members in enumerate(comps):
        if all(succ[m] is not None and all(comp[w] == ci for w in succ[m]) for m in members):
            out.append(sorted((tuple(int(x) for x in rows[m]) for m in members), key=as_int))
    out.sort(key=lambda att: as_int(att[0]))
    return out


def simulate_visits(net: Network, *, chains: int = 65536, burn_in: int = 1000, window: int = 64, seed: int = 0,
                    prob_bits: int = 16, device=None, chunk: int = 250) -> np.ndarray:
    """The distinct states ((S, N) 0/1 rows) that ``chains`` GPU chains of ``net`` (uniform
    random starts, no perturbation or interventions) visit in the ``window`` steps after
    ``burn_in`` steps."""
    import torch

    from .spec import EnvSpec
    from .vector_env import VectorPBNEnv

    spec = EnvSpec(net, [], perturbation=0.0, prob_bits=prob_bits, horizon=0)
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    env = VectorPBNEnv(spec, chains, seed=seed, device=dev, autoreset=False, keep_final_state=False)
    try:
        env.reset()   # no attractors: uniform random start states
        left, buf = burn_in, None   # (burn_in 0: the window starts at the random start states)
        with torch.cuda.device(dev):
            while left > 0:
                k = min(chunk, left)
                buf = env.rollout(k, random_actions=False, keep_obs=False, keep_final=False,
                                  out=buf if buf is not None and buf["_n_steps"] == k else None)
                left -= k
            out = env.rollout(window, random_actions=False, keep_obs=True, keep_final=False)
            words = out["obs"][:, :, :chains].permute(0, 2, 1).reshape(-1, env.words)
            words = torch.unique(words, dim=0).cpu().numpy().view(np.uint32)
    finally:
        env.close()
    shifts = np.arange(32, dtype=np.uint32)
    return ((words[:, :, None] >> shifts) & 1).reshape(len(words), -1)[:, :net.n].astype(np.uint8)


def discover_attractors(net: Network, *, chains: int = 65536, burn_in: int = 1000, window: int = 64, seed: int = 0,
                        prob_bits: int = 16, device=None, chunk: int = 250, max_box: int = 1 << 14,
                        max_states: int = 1 << 20) -> Attractors:
    """Bottom SCCs of ``net``'s STG that ``chains`` GPU chains reach within ``burn_in`` steps."""
    bits = simulate_visits(net, chains=chains, burn_in=burn_in, window=window, seed=seed, prob_bits=prob_bits,
                           device=device, chunk=chunk)
    return bottom_sccs(net, bits, prob_bits=prob_bits, max_box=max_box, max_states=max_states)


def reached_stg(net: Network, *, chains: int = 4096, steps: int = 64, seed: int = 0, prob_bits: int = 16,
                device=None, max_box: int = 1 << 12, max_states: int = 1 << 16) -> Dict[Tuple[int, ...], set]:
    """``graph.genSTG()`` for networks too large to enumerate (print_graph.py:15-34 calls it on
    the reference's networks, bb33 has 33 nodes): the states ``chains`` GPU chains visit in
    their first ``steps`` steps from uniform random starts, closed under successors (at most
    ``max_states`` states), as {state: set of successor states} -- the exact successor relation
    of that region.  States whose successors were not enumerated (past ``max_states`` or a box
    of more than ``max_box``) are left out, as are edges into them."""
    bits = simulate_visits(net, chains=chains, burn_in=0, window=steps, seed=seed, prob_bits=prob_bits,
                           device=device)
    rows, succ = explore(net, bits, prob_bits=prob_bits, max_box=max_box, max_states=max_states)
    keys = [tuple(int(x) for x in r) for r in rows]
    done = {v for v, s in enumerate(succ) if s is not None}
    return {keys[v]: {keys[w] for w in succ[v] if w in done} for v in sorted(done)}


def discover_attractors_escalating(net: Network, *, burn_ins=None, **kwargs) -> Attractors:
    """``discover_attractors`` with a growing burn-in until a bottom SCC is certified: 1,000
    steps suffice for pbn28 but not pbn70 (20,000 certify its bottom SCC).  Returns
    the first non-empty result (empty if every burn-in fails).  A caller's ``burn_in`` (e.g.
    ``PBNEnv(discovery={"burn_in": 50000})``) is used as given, alone; ``burn_ins`` sets the
    ladder; the default ladder is (1000, 5000, 20000)."""
    if burn_ins is None:
        burn_ins = (kwargs.pop("burn_in"),) if "burn_in" in kwargs else (1000, 5000, 20000)
    kwargs.pop("burn_in", None)
    found: Attractors = []
    for b in burn_ins:
        found = discover_attractors(net, burn_in=b, **kwargs)
        if found:
            break
    return found
