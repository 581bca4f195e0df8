"""Independence of the draws on the real counter map (Philox4x32-7 has no margin
left over the round count that passes BigCrush, and the counters here are highly structured).

Every stream draws Philox4x32-7 at counter (lo32 id, lo32 step, stream << 28 | idx,
hi16 id | hi16 step << 16) under one fixed key (DESIGN.md "RNG").  Neighbouring counters are
where a marginal round count would fail, so these tests draw the words the kernels actually
use for pairs of neighbours -- env e vs e + 1, step k vs k + 1, call idx vs idx + 1, the SEL vs
the ENV stream at the same id and step, SETTLE_SEL vs SEL, the settle law's per-env selection
calls (update k vs k + 1, call c vs c + 1, and the two 16-bit node fields of one word) -- and
check each pair:
  * joint chi-square of the top 4 bits (256 cells, 2^16 pairs: 256 expected per cell);
  * every one of the 32 x 32 single-bit XOR relations between the two words (a linear
    dependence between bit i of one and bit j of the other shows as a biased XOR): each must
    stay within 6 standard deviations of 1/2;
  * Pearson correlation of the two words as uniforms: |r| < 6 / sqrt(n).
Also the words within one call (x vs y, z vs w).  All bounds are ~6 sigma (false alarm ~1e-9
per statistic).
"""
import numpy as np
import pytest

from oracle.agent_oracle import philox_vec

SEED = 0x0123456789ABCDEF
SEL, ENV, PERT, RESET, EXPLORE, SETTLE_SEL, SETTLE_ENV = 0, 1, 2, 3, 4, 5, 6
N_PAIRS = 1 << 16


def words(ident, step, stream, idx):
    ident = np.asarray(ident, dtype=np.uint64)
    step = np.asarray(step, dtype=np.uint64)
    c0 = ident & np.uint64(0xFFFFFFFF)
    c1 = step & np.uint64(0xFFFFFFFF)
    c2 = (np.uint64(stream) << np.uint64(28)) | (np.asarray(idx, dtype=np.uint64) & np.uint64(0x0FFFFFFF))
    c3 = ((ident >> np.uint64(32)) & np.uint64(0xFFFF)) | (((step >> np.uint64(32)) & np.uint64(0xFFFF)) << np.uint64(16))
    return philox_vec(c0, c1, c2, c3, SEED & 0xFFFFFFFF, SEED >> 32)


def check_pair(a: np.ndarray, b: np.ndarray, what: str, bits: int = 32):
    n = a.size
    # joint top-4-bit chi-square
    top = np.uint32(bits - 4)
    cells = ((a >> top).astype(np.int64) << 4) | (b >> top).astype(np.int64)
    counts = np.bincount(cells, minlength=256)
    expect = n / 256
    chi2 = ((counts - expect) ** 2 / expect).sum()
    assert chi2 < 255 + 6 * np.sqrt(2 * 255) + 10, (what, chi2)
    # single-bit XOR relations, all 32 x 32 bit pairs
    abits = ((a[:, None] >> np.arange(bits, dtype=np.uint32)) & 1).astype(np.uint8)
    bbits = ((b[:, None] >> np.arange(bits, dtype=np.uint32)) & 1).astype(np.uint8)
    ones_a = abits.sum(axis=0).astype(np.int64)
    ones_b = bbits.sum(axis=0).astype(np.int64)
    both = abits.T.astype(np.int32) @ bbits.astype(np.int32)               # (32, 32): count a_i = b_j = 1
    xor1 = ones_a[:, None] + ones_b[None, :] - 2 * both                     # count a_i != b_j
    dev = np.abs(xor1 - n / 2) / np.sqrt(n / 4)
    assert dev.max() < 6.0, (what, float(dev.max()), np.unravel_index(dev.argmax(), dev.shape))
    # linear correlation of the words as uniforms
    r = np.corrcoef(a.astype(np.float64), b.astype(np.float64))[0, 1]
    assert abs(r) < 6.0 / np.sqrt(n), (what, r)


@pytest.mark.parametrize("stream", [ENV, PERT, RESET, EXPLORE, SETTLE_SEL, SETTLE_ENV])
def test_neighbouring_envs(stream):
    e = np.arange(N_PAIRS, dtype=np.uint64) * np.uint64(2)    # pairs (e, e + 1)
    step = np.full(N_PAIRS, 17, dtype=np.uint64)
    A = words(e, step, stream, 0)
    B = words(e + np.uint64(1), step, stream, 0)
    for k in range(4):
        check_pair(A[k], B[k], f"stream {stream} word {k}: env e vs e+1")


@pytest.mark.parametrize("stream", [SEL, ENV])
def test_neighbouring_steps(stream):
    e = np.arange(N_PAIRS, dtype=np.uint64)
    step = np.full(N_PAIRS, 1000, dtype=np.uint64)
    A = words(e, step, stream, 3)
    B = words(e, step + np.uint64(1), stream, 3)
    for k in (0, 3):
        check_pair(A[k], B[k], f"stream {stream} word {k}: step k vs k+1")


def test_neighbouring_steps_vary_along_steps():
    """The same id over consecutive steps (the time series one env sees)."""
    step = np.arange(N_PAIRS, dtype=np.uint64) * np.uint64(2)
    e = np.full(N_PAIRS, 12345, dtype=np.uint64)
    A = words(e, step, ENV, 0)
    B = words(e, step + np.uint64(1), ENV, 0)
    check_pair(A[2], B[2], "one env, step k vs k+1")


def test_neighbouring_selection_calls():
    """SEL idx = 4 node + call: call c vs c + 1 of one node, node i vs i + 1 at the same call."""
    G = np.arange(N_PAIRS, dtype=np.uint64)
    step = np.full(N_PAIRS, 5, dtype=np.uint64)
    A = words(G, step, SEL, 8)
    check_pair(A[0], words(G, step, SEL, 9)[0], "SEL call c vs c+1")
    check_pair(A[1], words(G, step, SEL, 12)[1], "SEL node i vs i+1")


def test_sel_vs_env_and_settle_streams():
    """The group's selection words vs the ENV words of env id == group id (same id, step and
    idx, different stream), and SETTLE_SEL's update 1 vs SEL."""
    ident = np.arange(N_PAIRS, dtype=np.uint64)
    step = np.full(N_PAIRS, 77, dtype=np.uint64)
    S = words(ident, step, SEL, 0)
    E = words(ident, step, ENV, 0)
    T = words(ident, step, SETTLE_SEL, 0)
    for k in range(4):
        check_pair(S[k], E[k], f"SEL vs ENV word {k}")
        check_pair(S[k], T[k], f"SEL vs SETTLE_SEL word {k}")


def test_settle_selection_calls():
    """The settle law's per-env selection draws (SETTLE_SEL idx = k << 8 | call, node i = 16-bit
    field i & 1 of word (i >> 1) & 3 of call i >> 3): update k vs k + 1 and call c vs c + 1 of
    one env, and the two node fields of one word."""
    e = np.arange(N_PAIRS, dtype=np.uint64)
    step = np.full(N_PAIRS, 9, dtype=np.uint64)
    A = words(e, step, SETTLE_SEL, (3 << 8) | 1)
    check_pair(A[2], words(e, step, SETTLE_SEL, (4 << 8) | 1)[2], "SETTLE_SEL update k vs k+1")
    check_pair(A[0], words(e, step, SETTLE_SEL, (3 << 8) | 2)[0], "SETTLE_SEL call c vs c+1")
    for k in range(4):
        check_pair(A[k] & np.uint32(0xFFFF), A[k] >> np.uint32(16), f"SETTLE_SEL word {k}: node 2j vs 2j+1", bits=16)


def test_words_within_one_call():
    ident = np.arange(N_PAIRS, dtype=np.uint64)
    step = np.full(N_PAIRS, 3, dtype=np.uint64)
    x, y, z, w = words(ident, step, ENV, 0)
    check_pair(x, y, "word 0 vs 1")
    check_pair(z, w, "word 2 vs 3")
    check_pair(x, w, "word 0 vs 3")


@pytest.mark.parametrize("rounds", [2, 4, 5])
def test_detector_catches_reduced_round_maps(rounds):
    """The checks have teeth: on the env e vs e + 1 map, Philox4x32 with 5 or fewer rounds
    fails them (5 rounds: words 0 and 3), while 6 and 7 pass -- the streams' 7 rounds sit two
    rounds above what these neighbour tests can detect (measured for this file)."""
    e = np.arange(N_PAIRS, dtype=np.uint64) * np.uint64(2)
    step = np.full(N_PAIRS, 17, dtype=np.uint64)

    def weak(ident):
        c0 = ident & np.uint64(0xFFFFFFFF)
        c3 = np.zeros_like(c0)
        return philox_vec(c0, step, np.full_like(c0, ENV << 28), c3, SEED & 0xFFFFFFFF, SEED >> 32, rounds=rounds)
    A, B = weak(e), weak(e + np.uint64(1))
    failed = 0
    for k in range(4):
        try:
            check_pair(A[k], B[k], f"{rounds}-round map word {k}")
        except AssertionError:
            failed += 1
    assert failed >= 1
