"""Score candidate attractor notions against the reference's pseudo-attractor fixtures
(train_BDQ.py:105-106 prints "final pseudo attractors", bdq_model/__init__.py:
182-184 grows env.all_attractors during training).

  python tools/pseudo_attractors.py [--out profiles/r05_pseudo_attractors.json]

Fixtures (tests/golden/ref_fixtures.json, read statically from the reference's pickles):
  * data/attractors_Bittner-28.pkl: 14 single states of kaban/pbn28.ispl (numeric gene-ID order);
  * bns_attractors/10_3_attractors.pkl: 6 single states of kaban/pbn10.ispl (lexicographic order).
Every state of both is a possible fixed point (P(s -> s) > 0 without perturbation).

Notions, each a set of states computed from the ISPL network alone (equal function weights as
the ISPL call sites pass them, duplicates counted twice; a_i(s) = the weight of node i's
functions that keep s_i, in thirds for three equal functions):
  bottom_scc       states of the bottom SCCs of the full transition graph (print_graph.py:15-34,
                   what PBNEnv grows today; pbn28: attractors.discover on the GPU, bundled here
                   from profiles/r01_discovered_attractors_pbn28.json)
  possible_fp      P(s -> s) > 0: every node kept by some function
  majority_fp      every node kept by more than half of its weight (the fixed points of the
                   most probable successor, node by node)
  first_fn_fp      fixed points of the Boolean network of each node's first function (file order)
  self_loop_ge_X   P(s -> s) >= X for X in (1/2, 1/4, 1/9, 2/27)
  top_ssd_k        the k most visited states of long p = 0.01 chains (pbn10: the exact stationary
                   distribution; pbn28: 256 chains x 20,000 steps of the C oracle), k = fixture size
  top_h20_k        the k most frequent end states of 20-step p = 0 chains from uniform random
                   starts (the horizon of train_BDQ.py:50), k = fixture size
Per notion: its size, the fixture states it contains (hits), and whether it equals the fixture.
Also ``bn_slice``: whether some Boolean network inside the PBN (one function per node) has all the
fixture's states as fixed points, the same question for random subsets of the possible fixed
points, and the fewest fixed points among such networks that a greedy search finds.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

from pbn_rl_amd.network import load_network  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "ref_fixtures.json")


def fixture_states(name):
    fx = json.load(open(GOLD))
    if name == "pbn28":
        net = load_network("pbn28")
        num = sorted(range(net.n), key=lambda i: int(net.genes[i].lstrip("x")))
        vals = fx["attractors_Bittner-28"]["value"]
    else:
        net = load_network("pbn10")
        num = sorted(range(net.n), key=lambda i: net.genes[i])
        vals = fx["attractors_pbn10"]["value"]
    out = []
    for att in vals:
        bits = [int(att[0][num.index(i)]) for i in range(net.n)]
        out.append(sum(b << i for i, b in enumerate(bits)))
    return net, out


def keep_fractions(net, S):
    """For states S (int64 array): per node, the fraction of its weight that keeps s_i; shape (n, len(S))."""
    n = net.n
    bits = ((S[None, :] >> np.arange(n)[:, None]) & 1).astype(np.uint8)
    keep = np.zeros((n, S.size))
    for i, fl in enumerate(net.nodes):
        tot = sum(f.weight for f in fl)
        for f in fl:
            m = np.zeros(S.size, dtype=np.int64)
            for j, g in enumerate(f.inputs):
                m |= bits[g].astype(np.int64) << j
            val = (f.table >> m) & 1
            keep[i] += np.where(val == bits[i], float(f.weight / tot), 0.0)
    return keep


def first_fn_fixed(net, S):
    n = net.n
    bits = ((S[None, :] >> np.arange(n)[:, None]) & 1).astype(np.uint8)
    ok = np.ones(S.size, dtype=bool)
    for i, fl in enumerate(net.nodes):
        f = fl[0]
        m = np.zeros(S.size, dtype=np.int64)
        for j, g in enumerate(f.inputs):
            m |= bits[g].astype(np.int64) << j
        ok &= ((f.table >> m) & 1) == bits[i]
    return ok


def possible_fixed_points(net, allowed=None):
    """Every state in which each node is kept by some function (by ``allowed[i]``, the function
    indices node i may use, when given): partial assignments extended one variable at a time,
    filtered as soon as a node and all its inputs are assigned (pbn28: 218,916 of 2^28 in ~7 s)."""
    n = net.n
    need = [set([i]) | set(g for f in fl for g in f.inputs) for i, fl in enumerate(net.nodes)]
    order, assigned, done = [], set(), set()
    while len(order) < n:   # the next variable: the one completing the most constraints
        best = max((v for v in range(n) if v not in assigned),
                   key=lambda v: (sum(1 for i in range(n) if i not in done and need[i] <= assigned | {v}),
                                  -sum(1 for i in range(n) if v in need[i])))
        order.append(best)
        assigned.add(best)
        done |= {i for i in range(n) if need[i] <= assigned}
    states = np.zeros(1, dtype=np.int64)
    assigned, done = set(), set()
    for v in order:
        states = np.concatenate([states, states | (1 << v)])
        assigned.add(v)
        for i in range(n):
            if i in done or not need[i] <= assigned:
                continue
            done.add(i)
            si = (states >> i) & 1
            ok = np.zeros(states.size, dtype=bool)
            for j, f in enumerate(net.nodes[i]):
                if allowed is not None and j not in allowed[i]:
                    continue
                m = np.zeros(states.size, dtype=np.int64)
                for k, g in enumerate(f.inputs):
                    m |= ((states >> g) & 1) << k
                ok |= ((f.table >> m) & 1) == si
            states = states[ok]
    return np.sort(states)


def enumerate_notions(net):
    """The fixed-point notions and the self-loop thresholds: every one is a subset of the
    possible fixed points, so they are computed on those."""
    P = possible_fixed_points(net)
    keep = keep_fractions(net, P)
    p = np.prod(keep, axis=0)
    found = {"possible_fp": P.tolist(), "majority_fp": P[(keep > 0.5).all(0)].tolist(),
             "first_fn_fp": P[first_fn_fixed(net, P)].tolist()}
    for k, x in (("self_loop_ge_1/2", 0.5), ("self_loop_ge_1/4", 0.25), ("self_loop_ge_1/9", 1 / 9),
                 ("self_loop_ge_2/27", 2 / 27)):
        found[k] = P[p >= x - 1e-12].tolist()
    return found, {}, list(zip(p.tolist(), P.tolist()))


def slice_consistency(net, fix, P, trials=2000, seed=0, greedy=True):
    """Whether one Boolean network inside the PBN (one function per node) has every fixture state
    as a fixed point (every node has a function keeping its value in all of them), how often
    random subsets of the possible fixed points of the fixture's size have that property, and the
    fewest fixed points found (greedy) among such networks."""
    n = net.n

    def keeping(S):
        return [[j for j, f in enumerate(fl) if all(f([(s >> k) & 1 for k in range(n)]) == ((s >> i) & 1) for s in S)]
                for i, fl in enumerate(net.nodes)]

    J = keeping(fix)
    rng = np.random.default_rng(seed)
    rand = sum(all(keeping(rng.choice(P, len(fix), replace=False).tolist())) for _ in range(trials))
    out = {"consistent": bool(all(J)), "functions_keeping_all": [len(x) for x in J],
           "random_subsets_consistent": f"{rand}/{trials}"}
    if all(J) and greedy:
        choice = [x[0] for x in J]
        count = lambda ch: possible_fixed_points(net, [{c} for c in ch]).size  # noqa: E731
        best = count(choice)
        improved = True
        while improved:
            improved = False
            for i in range(n):
                for j in J[i]:
                    if j != choice[i]:
                        c2 = list(choice)
                        c2[i] = j
                        v = count(c2)
                        if v < best:
                            best, choice, improved = v, c2, True
        out["fewest_fixed_points_found"] = best
        out["that_network"] = choice
    return out


def ssd_top(net, k, seed=1, chains=256, steps=20000, p=0.01, burn=1000):
    """The k most visited states of long chains, by the C oracle (one-update law)."""
    from oracle import oracle
    from pbn_rl_amd.spec import EnvSpec
    spec = EnvSpec(net, [], perturbation=p, horizon=0)
    rng = np.random.default_rng(seed)
    st = rng.integers(0, 1 << net.n, size=(1, chains), dtype=np.int64).astype(np.uint32)
    tg = np.full(chains, 255, np.uint8)
    t = np.zeros(chains, np.uint8)
    counts = {}
    for s in range(steps):
        out = oracle.step(spec, seed, s, 0, st, np.zeros_like(st), tg, t, 0)
        st = out["state_out"]
        if s >= burn:
            u, c = np.unique(st[0], return_counts=True)
            for a, b in zip(u.tolist(), c.tolist()):
                counts[a] = counts.get(a, 0) + b
    return [s for s, _ in sorted(counts.items(), key=lambda x: -x[1])[:k]]


def h20_top(net, k, seed=2, chains=1 << 16, H=20):
    from oracle import oracle
    from pbn_rl_amd.spec import EnvSpec
    spec = EnvSpec(net, [], perturbation=0.0, horizon=0)
    rng = np.random.default_rng(seed)
    st = rng.integers(0, 1 << net.n, size=(1, chains), dtype=np.int64).astype(np.uint32)
    tg = np.full(chains, 255, np.uint8)
    t = np.zeros(chains, np.uint8)
    for s in range(H):
        st = oracle.step(spec, seed, s, 0, st, np.zeros_like(st), tg, t, 0)["state_out"]
    u, c = np.unique(st[0], return_counts=True)
    return u[np.argsort(-c)[:k]].tolist()


def exact_ssd_top(net, k, p=0.01):
    from oracle import law
    T = law.transition_matrix(net, p)
    w, v = np.linalg.eig(T.T)
    pi = np.abs(np.real(v[:, np.argmin(np.abs(w - 1))]))
    return np.argsort(-pi)[:k].tolist()


def bottom_scc_states(name, net):
    if name == "pbn10":
        from pbn_rl_amd.attractors import find_attractors
        return [s for a in find_attractors(net) for s in (sum(b << i for i, b in enumerate(x)) for x in a)]
    d = json.load(open(os.path.join(ROOT, "profiles", "r01_discovered_attractors_pbn28.json")))
    atts = d["attractors"] if "attractors" in d else d
    out = []
    for a in atts:
        for x in (a["states"] if isinstance(a, dict) else a):
            out.append(int(x) if not isinstance(x, list) else sum(b << i for i, b in enumerate(x)))
    return out


def score(name, quick=False):
    net, fix = fixture_states(name)
    fixset = set(fix)
    found, counts, loops = enumerate_notions(net)
    P = np.array(found["possible_fp"], dtype=np.int64)
    rows = {}

    def add(key, states, size=None):
        st = set(states)
        rows[key] = {"size": size if size is not None else len(st), "hits": len(st & fixset),
                     "equals_fixture": st == fixset}

    add("bottom_scc", bottom_scc_states(name, net))
    for k, v in found.items():
        add(k, v, counts.get(k))
    loops.sort(key=lambda x: -x[0])
    add(f"top_self_loop_{len(fix)}", [s for _, s in loops[:len(fix)]])
    if name == "pbn10":
        add(f"top_ssd_{len(fix)}", exact_ssd_top(net, len(fix)))
    elif not quick:
        add(f"top_ssd_{len(fix)}", ssd_top(net, len(fix)))
    add(f"top_h20_{len(fix)}", h20_top(net, len(fix)))
    pl = {s: p for p, s in loops}
    return {"fixture_size": len(fix), "fixture_self_loop": sorted(round(pl.get(s, 0.0), 4) for s in fix),
            "notions": rows, "bn_slice": slice_consistency(net, fix, P)}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_pseudo_attractors.json"))
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    res = {}
    for name in (["pbn10", "pbn28"] if a.only is None else [a.only]):
        res[name] = score(name)
        print(name, json.dumps(res[name], indent=1))
    if a.only is None:
        json.dump(res, open(a.out, "w"), indent=1)
        print("wrote", a.out)
