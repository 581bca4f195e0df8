"""numpy restatement of the agent-edge kernels (pbn_obs_unpack, pbn_q_to_flipmask).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of
pbn_rl_amd/csrc/pbn_agent.hip.  Follows the frame loop of the reference:
  - observation = np.stack((state, target)) as float (bdq_model/__init__.py:92-93), batched
    to (2, n, N); target = the first state of the env's target attractor;
  - epsilon-greedy: explore (EXPLORE word 0 < floor(eps * 2^32)) -> uniform ints in [0, N] per
    branch, branch k from EXPLORE word k + 1 by a 32-bit multiply-high (:74-76), else
    argmax of each branch's Q row (:95-96, torch.argmax: first maximum, NaN is the maximum);
  - env actions: list(action.unique()) (:176), a > 0 flips node a-1 (:81-84).
The explore draws follow DESIGN.md (Philox4x32-7, stream EXPLORE = 4); Philox is vectorised
here over envs and checked against oracle/pyoracle.philox4x32 by the tests.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
EXPLORE = 4


PHILOX_ROUNDS = 7   # every stream (DESIGN.md "RNG"); = pyoracle.PHILOX_ROUNDS


def philox_vec(c0, c1, c2, c3, k0: int, k1: int, rounds: int = PHILOX_ROUNDS):
    """Philox4x32-R over arrays of counters (uint32), scalar key (R = 7 for every stream)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & np.uint64(0xFFFFFFFF) for c in (c0, c1, c2, c3))
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(rounds):
        p0 = M0 * c0
        p1 = M1 * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ np.uint64(k0)
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ np.uint64(k1)
        c0, c1, c2, c3 = n0 & mask, p1 & mask, n2 & mask, p0 & mask
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [c.astype(np.uint32) for c in (c0, c1, c2, c3)]


def explore_words(seed: int, step: int, env_offset: int, n: int, calls: int = 1):
    """EXPLORE-stream words of every env: word j = call j >> 2, word j & 3 (4 * calls words)."""
    ge = np.arange(n, dtype=np.uint64) + np.uint64(env_offset)
    c0 = ge & np.uint64(0xFFFFFFFF)
    c1 = np.full(n, step & 0xFFFFFFFF, dtype=np.uint64)
    c3 = ((ge >> np.uint64(32)) & np.uint64(0xFFFF)) | np.uint64(((step >> 32) & 0xFFFF) << 16)
    out = []
    for c in range(calls):
        c2 = np.full(n, (EXPLORE << 28) | c, dtype=np.uint64)
        out += philox_vec(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return out


REPLAY = 7


def replay_rows(seed: int, draw: int, n: int, size: int) -> np.ndarray:
    """The fused learner's replay rows (pbn_replay_advance): row b of draw c is
    floor((x << 32 | y) * size / 2^64) for the REPLAY-stream Philox words (x, y) of (seed, id = b,
    step = c) -- uniform with replacement, as DeviceReplay.sample_indices (the reference draws
    without replacement, random.sample at bdq_model/memory.py:62)."""
    b = np.arange(n, dtype=np.uint64)
    c0 = b & np.uint64(0xFFFFFFFF)
    c1 = np.full(n, draw & 0xFFFFFFFF, dtype=np.uint64)
    c2 = np.full(n, REPLAY << 28, dtype=np.uint64)
    c3 = ((b >> np.uint64(32)) & np.uint64(0xFFFF)) | np.uint64(((draw >> 32) & 0xFFFF) << 16)
    x, y, _, _ = philox_vec(c0, c1, c2, c3, seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return np.array([((int(xi) << 32 | int(yi)) * size) >> 64 for xi, yi in zip(x, y)], dtype=np.int64)


def obs_unpack(spec, state: np.ndarray, target: np.ndarray) -> np.ndarray:
    """state (W, n) uint32, target (n,) uint8 -> (2, n, N) float32."""
    N = spec.n
    W, n = state.shape
    bits = (state.T[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1          # (n, W, 32)
    s = bits.reshape(n, 32 * W)[:, :N].astype(np.float32)
    first = np.zeros((len(spec.attractors) + 1, N), dtype=np.float32)            # last row: no target
    for a, att in enumerate(spec.attractors):
        first[a] = np.asarray(att[0], dtype=np.float32)
    tg = np.asarray(target).astype(np.int64)
    tg = np.where(tg < len(spec.attractors), tg, len(spec.attractors))
    return np.stack([s, first[tg]])


def argmax_torch(q: np.ndarray) -> np.ndarray:
    """argmax over the last axis with torch.argmax's tie and NaN rules."""
    nan = np.isnan(q)
    has_nan = nan.any(axis=-1)
    first_nan = np.argmax(nan, axis=-1)
    plain = np.argmax(np.where(nan, -np.inf, q), axis=-1)   # np.argmax: first maximum
    return np.where(has_nan, first_nan, plain)


def q_to_flipmask(spec, q: np.ndarray, seed: int, step: int, env_offset: int, epsilon: float):
    """q (n, K, N+1) float32 -> (flipmask (W, n) uint32, actions (n, K) int32)."""
    n, K, A = q.shape
    N, W = spec.n, spec.words
    assert A == N + 1
    w = explore_words(seed, step, env_offset, n, calls=(K + 1 + 3) // 4)
    eps_u = int(np.floor(np.float64(np.float32(epsilon)) * 4294967296.0))
    explore = w[0].astype(np.uint64) < np.uint64(eps_u) if eps_u < (1 << 32) else np.ones(n, dtype=bool)
    greedy = argmax_torch(q)                                                     # (n, K)
    rnd = np.zeros((n, K), dtype=np.int64)
    for k in range(K):   # branch k: explore word k + 1, multiply-high onto [0, N] (bias <= (N+1) / 2^32)
        rnd[:, k] = (w[1 + k].astype(np.uint64) * np.uint64(N + 1)) >> np.uint64(32)
    actions = np.where(explore[:, None], rnd, greedy).astype(np.int32)
    flip = np.zeros((W, n), dtype=np.uint32)
    for k in range(K):
        a = actions[:, k].astype(np.int64)
        hit = a > 0
        node = np.where(hit, a - 1, 0)
        for ww in range(W):
            sel = hit & ((node >> 5) == ww)
            flip[ww] |= np.where(sel, np.left_shift(np.uint32(1), (node & 31).astype(np.uint32)), np.uint32(0))
    return flip, actions


def heads_q(heads: np.ndarray) -> np.ndarray:
    """Q (n, K, A) from raw head outputs (K+1, n, A) with pbn_heads_to_flipmask's arithmetic:
    q_a = (v + adv_a) - mean, mean = sequential float32 sum of adv over a / A
    (bdq_model/network.py:59-61; torch's mean reduces in a different order)."""
    h = np.asarray(heads, dtype=np.float32)
    K1, n, A = h.shape
    v = h[0, :, 0]
    adv = h[1:]                                            # (K, n, A)
    s = np.zeros((K1 - 1, n), dtype=np.float32)
    for j in range(A):                                     # left to right, in float32
        s = (s + adv[:, :, j]).astype(np.float32)
    mean = (s / np.float32(A)).astype(np.float32)
    q = ((v[None, :, None] + adv).astype(np.float32) - mean[:, :, None]).astype(np.float32)
    return np.ascontiguousarray(q.transpose(1, 0, 2))
