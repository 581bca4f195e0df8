"""Exact transition law of the frozen step semantics, for small networks (test infrastructure).

TEST INFRASTRUCTURE ONLY: imported by tests/ (never by pbn_rl_amd/).  This is a third
restatement of DESIGN.md "Step semantics", as probabilities instead of draws:

  P(s' | s1) = sum over gamma != 0 of [s' = s1 ^ gamma] p^|gamma| (1-p)^(N-|gamma|)
             + (1-p)^N * prod_i P(node i -> s'_i | s1)

with P(node i -> 1 | s1) = sum over the functions f_ij with f_ij(s1) = 1 of their quantised
weight (network.thresholds(prob_bits), the integer thresholds the kernels compare against)
/ 2^prob_bits.  The perturbation is Bernoulli(p) per node exactly (the kernels draw it as
geometric gaps against a 32-bit CDF: the same law to 2^-32 per threshold, except gap 2,
whose uniform is the top word of what the action and reset draws leave of the 64-bit X:
uniform on its own, and within K / 2^64 per threshold of uniform given those draws,
K = (N+1)^3 * A(A-1) * |start attractor| -- 7.5e-9 at N = 128 with 254 single-state
attractors, DESIGN.md "Step semantics").

It is used to pin the law against the one reference artefact that constrains it: the trained
pbn7 agent (models/pbn7/bdq_final.pt) and the strategy lengths model_tester.py:587-658 recorded
for it in data/results/pbn_7_4.pkl.  ``hitting_distribution`` is that evaluation loop done
exactly: start in attractor a's first state ('*' -> 0, :609), act greedily (epsilon 0, :600),
count steps until the state is in the target attractor (:616), fail past 100 steps (:628).
"""
from __future__ import annotations

import itertools
from typing import Callable, Dict, List, Sequence, Tuple

import numpy as np

__all__ = ["transition_matrix", "settle_matrix", "flip_mask", "hitting_distribution", "pair_statistics"]


def _bits(s: int, n: int) -> List[int]:
    return [(s >> i) & 1 for i in range(n)]


def transition_matrix(net, p: float, prob_bits: int = 16) -> np.ndarray:
    """T[s1, s'] for all 2^N states (N <= 14), float64."""
    n = net.n
    if n > 14:
        raise ValueError("exact law limited to 14 nodes")
    S = 1 << n
    thr = net.thresholds(prob_bits)
    scale = float(1 << prob_bits)
    T = np.zeros((S, S))
    # perturbation part: gamma != 0
    pops = np.array([bin(g).count("1") for g in range(S)])
    pg = (p ** pops) * ((1 - p) ** (n - pops))
    pg[0] = 0.0
    idx = np.arange(S)
    for s1 in range(S):
        T[s1, s1 ^ idx] += pg
        bits = _bits(s1, n)
        p1 = np.empty(n)
        for i, (fl, c) in enumerate(zip(net.nodes, thr)):
            prev, acc = 0, 0
            for f, cj in zip(fl, c):
                if f(bits):
                    acc += cj - prev
                prev = cj
            p1[i] = acc / scale
        # product over nodes for every s'
        probs = np.ones(S)
        for i in range(n):
            bit = (idx >> i) & 1
            probs *= np.where(bit == 1, p1[i], 1.0 - p1[i])
        T[s1] += ((1 - p) ** n) * probs
    return T


def settle_matrix(T: np.ndarray, attractor_states: Sequence[int], settle: int) -> np.ndarray:
    """The settle law's step matrix (include/pbn_env.h "Step law"): from s1, one update by T,
    then further updates while the state is outside every attractor, at most ``settle``
    updates in all.  M[s1, s'] = P(the step ends in s')."""
    A = np.zeros(T.shape[0], bool)
    A[list(attractor_states)] = True
    M = np.zeros_like(T)
    cur = T.copy()
    for _ in range(1, max(settle, 1)):
        M[:, A] += cur[:, A]
        cur[:, A] = 0.0
        if not cur.any():
            break
        cur = cur @ T
    return M + cur


def flip_mask(actions: Sequence[int], mode: str = "or") -> int:
    """Flip mask of one action vector (a > 0 flips node a - 1).  "or": each distinct node
    once (``list(action.unique())``, bdq_model/__init__.py:176 -- the frozen semantics);
    "xor": every entry flips, so a repeated action cancels (the alternative reading of
    ``env.step(action)`` with the raw tensor at model_tester.py:624)."""
    m = 0
    for a in actions:
        a = int(a)
        if a > 0:
            m = (m | (1 << (a - 1))) if mode == "or" else (m ^ (1 << (a - 1)))
    return m


def hitting_distribution(T: np.ndarray, policy_mask: np.ndarray, start: int, target_set: Sequence[int],
                         max_steps: int = 100) -> np.ndarray:
    """P(count = k) for k = 0..max_steps+1 (index max_steps + 1 = failure) of the loop
    ``while state not in target: count += 1; act; step; if count > max_steps: fail``.
    policy_mask[s] = the flip mask the greedy agent applies in state s."""
    S = T.shape[0]
    tgt = np.zeros(S, bool)
    tgt[list(target_set)] = True
    out = np.zeros(max_steps + 2)
    if tgt[start]:
        out[0] = 1.0
        return out
    # step matrix with the policy applied: M[s, s'] = T[s ^ m(s), s']
    M = T[np.arange(S) ^ policy_mask]
    dist = np.zeros(S)
    dist[start] = 1.0
    for k in range(1, max_steps + 1):
        dist = dist @ M
        out[k] = dist[tgt].sum()
        dist[tgt] = 0.0
    out[max_steps + 1] = dist.sum()
    return out


def pair_statistics(dist: np.ndarray, max_steps: int = 100) -> Tuple[float, float, float]:
    """(mean, variance, failure probability) of the per-run value model_tester adds to its
    result matrix: the step count, or 101 for a failed run (:635)."""
    k = np.arange(max_steps + 2, dtype=np.float64)
    k[max_steps + 1] = 101.0
    mean = float((dist * k).sum())
    var = float((dist * k * k).sum() - mean * mean)
    return mean, var, float(dist[max_steps + 1])


def greedy_masks(q_fn: Callable[[np.ndarray, np.ndarray], np.ndarray], n: int, target_bits: Sequence[int],
                 mode: str = "or") -> np.ndarray:
    """policy_mask[s] for every state s: argmax per branch of q_fn(states (S, n), targets (S, n))
    -> (S, K, n+1), then flip_mask."""
    S = 1 << n
    states = np.array([_bits(s, n) for s in range(S)], dtype=np.float32)
    targets = np.tile(np.asarray(target_bits, np.float32), (S, 1))
    q = q_fn(states, targets)
    acts = q.argmax(axis=2)
    return np.array([flip_mask(a, mode) for a in acts], dtype=np.int64)


def state_index(bits: Sequence[int]) -> int:
    return sum((int(b) & 1) << i for i, b in enumerate(bits))


def evaluate_protocol(net, attractors: List[List[Sequence[int]]], q_fn, p: float, prob_bits: int = 16,
                      mode: str = "or", max_steps: int = 100, settle: int = 0) -> Dict[Tuple[int, int], np.ndarray]:
    """Exact count distribution of every (start attractor, target attractor) pair of
    model_tester.py:598 (itertools.product over the attractor indices); settle >= 2 uses the
    settle law with ``attractors`` as the env's attractor set."""
    T = transition_matrix(net, p, prob_bits)
    if settle >= 2:
        T = settle_matrix(T, [state_index(s) for a in attractors for s in a], settle)
    out = {}
    for a, t in itertools.product(range(len(attractors)), repeat=2):
        start = state_index(attractors[a][0])
        tgt_states = [state_index(s) for s in attractors[t]]
        masks = greedy_masks(q_fn, net.n, attractors[t][0], mode)
        out[(a, t)] = hitting_distribution(T, masks, start, tgt_states, max_steps)
    return out
