"""The uniform draws of DESIGN.md "Step semantics" against exact uniformity (CPU, C oracle).

Random actions mirror np.random.randint(0, N+1, size=3) (bdq_model/__init__.py:76): three
iid uniform ints on [0, N], so every node is flipped with probability 1 - (N/(N+1))^3 and
no node at all with probability (1/(N+1))^3.  Resets draw (start, target != start)
uniformly over the A(A-1) ordered attractor pairs.  The draws are multiply-shift extractions
from 64-bit Philox values (bias <= (N+1)^3 / 2^64); the round-1 10-bit draws gave 9 of the 29
Bittner-28 actions 36/1024 instead of 35/1024, which the per-node test below resolves at ~7
standard deviations.
"""
import numpy as np

from oracle import oracle
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec


def chi2_bound(dof: int) -> float:
    """A loose upper tail (~6 sigma) of the chi-square distribution with dof degrees."""
    return dof + 6.0 * np.sqrt(2.0 * dof) + 10.0


def test_random_actions_uniform_per_node():
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.0, horizon=0)
    N, n, steps = spec.n, 65536, 24
    st, tg, t = oracle.reset(spec, 3, 0, 0, n)
    counts = np.zeros(N, dtype=np.int64)
    empty = 0
    for k in range(steps):
        out = oracle.step(spec, 3, k + 1, 0, st, np.zeros_like(st), tg, t, 2, want_final=False)
        fm = out["flipmask"][0]
        counts += ((fm[None, :] >> np.arange(N, dtype=np.uint32)[:, None]) & np.uint32(1)).sum(axis=1).astype(np.int64)
        empty += int((fm == 0).sum())
        st, tg, t = out["state_out"], out["target"], out["t"]
    total = n * steps
    p_node = 1.0 - (N / (N + 1)) ** 3
    expect = total * p_node
    # per-node counts are not independent across nodes (a draw flips up to 3), so compare each
    # node with its own binomial spread rather than one pooled chi-square
    z = (counts - expect) / np.sqrt(total * p_node * (1 - p_node))
    assert np.abs(z).max() < 5.0, z
    assert ((counts - expect) ** 2 / (total * p_node * (1 - p_node))).sum() < chi2_bound(N)
    p0 = (1.0 / (N + 1)) ** 3
    assert abs(empty - total * p0) < 6 * np.sqrt(total * p0) + 1


def test_reset_pairs_uniform():
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    A = len(spec.attractors)
    n = 262144
    st, tg, t = oracle.reset(spec, 17, 5, 0, n)
    start = np.array([spec.attractor_id(spec.network.unpack([int(w)])) for w in st[0]])
    assert np.all(start >= 0) and np.all(tg != start)
    pair = start * A + tg.astype(np.int64)
    hist = np.bincount(pair, minlength=A * A).reshape(A, A)
    cells = hist[~np.eye(A, dtype=bool)]
    expect = n / (A * (A - 1))
    chi2 = ((cells - expect) ** 2 / expect).sum()
    assert chi2 < chi2_bound(A * (A - 1) - 1), chi2


def test_autoreset_pairs_uniform_multi_state_attractor():
    """pbn7: one attractor has four states; autoreset start states are uniform within it."""
    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"), perturbation=0.0, horizon=1)
    n = 65536
    st, tg, t = oracle.reset(spec, 2, 0, 0, n)
    out = oracle.step(spec, 2, 1, 0, st, np.zeros_like(st), tg, t, 1, want_final=False)   # every env truncates
    assert np.all(out["flags"] & 16)
    big = next(a for a, att in enumerate(spec.attractors) if len(att) == 4)
    words = [spec.network.pack(s)[0] for s in spec.attractors[big]]
    got = out["state_out"][0]
    counts = np.array([(got == w).sum() for w in words])
    expect = counts.sum() / 4
    assert counts.sum() > 0.2 * n
    assert ((counts - expect) ** 2 / expect).sum() < chi2_bound(3)
