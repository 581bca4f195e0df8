"""Which step law do the reference's trained-agent evaluations support?  

Test infrastructure (imports oracle/law.py).  ``python -m tests.law_variants`` scores every
variant of the transition law below against the reference's recorded evaluations of its trained
agents, exactly (oracle/law.py's hitting-time distributions of model_tester.py:587-658), and
writes the table to profiles/r04_law_variants.json:

  data/results/pbn_10_6.pkl  models/pbn10/bdq_final.pt on kaban/pbn10.ispl, the six states of
                             bns_attractors/10_3 (lexicographic gene order), 10 runs x 36 pairs
  data/results/pbn_7_4.pkl   models/pbn7/bdq_final.pt on kaban/pbn7.ispl, the four attractors of
                             data/attractors_Bittner-7.pkl (file order), 10 runs x 16 pairs

Variants (every combination):
  law        one     -- one synchronous update per step (DESIGN.md "Step semantics")
             settle  -- then updates until the state is in ANY attractor of the env's set (the
                        bb33-pinned law, include/pbn_env.h "Step law"), at most CAP = 1025
             target  -- then updates until the state is in the TARGET attractor, at most CAP
  pert       on / off -- Bernoulli(p) perturbation in the settle updates too, or only in the first
  p          0, 0.01
  actions    or  -- each distinct action once (list(action.unique()), bdq_model/__init__.py:176)
             xor -- every entry flips (model_tester.py:624 passes the raw action vector)
  order      pbn10: lex (the fixture's and agent's gene order) or file (kaban order)

Scores, per fixture (higher is better):
  ll_hist    log-likelihood of the recorded count histogram (``data``), every run drawn from the
             pooled per-pair distribution (the pair of a run is not recorded)
  ll_matrix  log-likelihood of the recorded per-pair sums of 10 runs (``save_matrix``): exact, the
             10-fold convolution of each pair's count distribution
  e_fail, e_one   expected failures (101) and one-step runs over the recorded run count
"""
from __future__ import annotations

import itertools
import json
import os
import sys

import numpy as np

from oracle import law

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_STEPS = 100
CAP = 1 + (1 << 10)


def settle_matrix2(T_first: np.ndarray, T_rest: np.ndarray, absorbing, squarings: int = 10) -> np.ndarray:
    """One update by T_first, then updates by T_rest while outside ``absorbing``: at most
    2^squarings further updates (the cap CAP = 1 + 2^10), by repeated squaring of the chain with
    the absorbing states made absorbing (a state outside that never reaches them ends where
    the chain is after the cap, as the capped law does)."""
    A = np.zeros(T_first.shape[0], bool)
    A[list(absorbing)] = True
    P = T_rest.copy()
    P[A, :] = 0.0
    P[A, A] = 1.0
    for _ in range(squarings):
        P = P @ P
    return T_first @ P


_T = {}


def transition(net, p: float) -> np.ndarray:
    key = (net.name, net.n, p)
    if key not in _T:
        _T[key] = law.transition_matrix(net, p)
    return _T[key]


def protocol(net, atts, q_fn, *, law_kind, pert, p, mode):
    """{(a, t): count distribution} of model_tester.py:587-658 under one variant."""
    Tp = transition(net, p)
    T0 = transition(net, 0.0) if (p > 0 and not pert) else Tp
    all_states = [law.state_index(s) for a in atts for s in a]
    if law_kind == "settle":
        M_any = settle_matrix2(Tp, T0, all_states)
    out = {}
    for a, t in itertools.product(range(len(atts)), repeat=2):
        start = law.state_index(atts[a][0])
        tgt = [law.state_index(s) for s in atts[t]]
        if law_kind == "one":
            M = Tp
        elif law_kind == "settle":
            M = M_any
        else:
            M = settle_matrix2(Tp, T0, tgt)
        masks = law.greedy_masks(q_fn, net.n, atts[t][0], mode)
        out[(a, t)] = law.hitting_distribution(M, masks, start, tgt, MAX_STEPS)
    return out


def scores(res, data: dict, matrix, runs: int = 10) -> dict:
    """Log-likelihoods of the recorded histogram and per-pair sums (module docstring)."""
    pairs = list(res)
    pool = sum(res[k] for k in pairs) / len(pairs)
    eps = 1e-300
    ll_hist = 0.0
    for k, c in data.items():
        idx = MAX_STEPS + 1 if int(k) == 101 else int(k)
        ll_hist += c * np.log(max(pool[idx], eps))
    ll_mat = 0.0
    vals = np.arange(MAX_STEPS + 2)
    vals[MAX_STEPS + 1] = 101
    for (a, t), d in res.items():
        # distribution of the per-run value (count, or 101), then its 10-fold sum
        single = np.zeros(102)
        np.add.at(single, vals, d)
        conv = np.array([1.0])
        for _ in range(runs):
            conv = np.convolve(conv, single)
        s = int(round(matrix[a][t]))
        ll_mat += np.log(max(conv[s] if s < len(conv) else 0.0, eps))
    n_runs = sum(data.values())
    return {"ll_hist": ll_hist, "ll_matrix": ll_mat,
            "e_fail": float(pool[MAX_STEPS + 1] * n_runs), "e_one": float(pool[1] * n_runs),
            "e_zero": float(pool[0] * n_runs)}


def fixture_cases():
    """(name, net, attractors, q_fn, data, matrix) of each recorded evaluation, per gene order."""
    import torch

    from pbn_rl_amd.agent import BranchingQNetwork
    from pbn_rl_amd.network import load_network
    from tests.test_law_pin import GOLD, fixtures, pbn7_agent, q_numpy, ref_pbn7_attractors

    fx = fixtures()
    cases = []
    net7 = load_network("pbn7")
    r7 = fx["results_pbn_7_4"]["value"]
    cases.append(("pbn_7_4/file", net7, ref_pbn7_attractors(), q_numpy(pbn7_agent()), r7["data"],
                  r7["save_matrix"]))
    net10 = load_network("pbn10")
    w = np.load(os.path.join(GOLD, "pbn10_bdq_final.npz"))
    q10 = BranchingQNetwork((10, 10), 11, 3)
    q10.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    q10.eval()
    r10 = fx["results_pbn_10_6"]["value"]
    for order in ("lex", "file"):
        perm = sorted(range(net10.n), key=lambda i: net10.genes[i]) if order == "lex" else list(range(net10.n))
        atts = [[tuple(int(att[0][perm.index(i)]) for i in range(net10.n))] for att in fx["attractors_pbn10"]["value"]]

        def q_fn(states, targets, perm=perm):
            with torch.no_grad():
                x = torch.from_numpy(np.stack([states[:, perm], targets[:, perm]]).astype(np.float32))
                out = q10(x).numpy()
            mapped = np.zeros_like(out)
            mapped[:, :, 0] = out[:, :, 0]
            for k in range(net10.n):
                mapped[:, :, perm[k] + 1] = out[:, :, k + 1]
            return mapped
        cases.append((f"pbn_10_6/{order}", net10, atts, q_fn, r10["data"], r10["save_matrix"]))
    return cases


def variants():
    for law_kind in ("one", "settle", "target"):
        for pert in ((True,) if law_kind == "one" else (True, False)):
            for p in (0.0, 0.01):
                if p == 0.0 and not pert:
                    continue   # the same variant as pert=True at p = 0
                for mode in ("or", "xor"):
                    yield {"law": law_kind, "pert_in_settle": pert, "p": p, "actions": mode}


def table():
    rows = []
    for name, net, atts, q_fn, data, matrix in fixture_cases():
        for v in variants():
            res = protocol(net, atts, q_fn, law_kind=v["law"], pert=v["pert_in_settle"], p=v["p"], mode=v["actions"])
            rows.append({"fixture": name, **v, **scores(res, data, matrix),
                         "recorded": {"one": int(data.get("1", 0)), "fail": int(data.get("101", 0)),
                                      "runs": int(sum(data.values()))}})
    return rows


def main(path=os.path.join(ROOT, "profiles", "r04_law_variants.json")):
    rows = table()
    with open(path, "w") as f:
        json.dump({"source": "python -m tests.law_variants (tests/law_variants.py)", "rows": rows}, f, indent=1)
    for r in sorted(rows, key=lambda r: (r["fixture"], -r["ll_hist"])):
        print(f"{r['fixture']:14s} {r['law']:6s} pert={int(r['pert_in_settle'])} p={r['p']:<5} {r['actions']:3s} "
              f"ll_hist={r['ll_hist']:10.1f} ll_matrix={r['ll_matrix']:10.1f} e_fail={r['e_fail']:6.1f} "
              f"e_one={r['e_one']:6.1f} (rec one={r['recorded']['one']} fail={r['recorded']['fail']})")


if __name__ == "__main__":
    sys.exit(main())
