"""The reference's evaluation protocol, model_tester.py:587-658, batched over runs (test helper).

For every ordered (start attractor, target attractor) pair (``itertools.product``, :598) and
every run: start in the start attractor's first state ('*' -> 0, :609), take the target
attractor's first state as the agent's target input (:603), act greedily (epsilon 0, :600; the
argmax per branch of BranchingDQN.predict, bdq_model/__init__.py:91-96), step the env with the
raw action vector (:624), and count steps until the state is in the target attractor (:616),
failing past 100 steps (:628, recorded as 101, :635).

``step_fn(words, flip, k)`` advances a (W, n) uint32 batch of states by one env.step with flip
masks ``flip`` at call k; the runs of all pairs go through it side by side, so a GPU step
kernel or the CPU oracle can stand behind it.
"""
import itertools
import os

import numpy as np
import torch

from pbn_rl_amd.agent import BranchingQNetwork

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_agent(model: str, n: int) -> BranchingQNetwork:
    """tests/golden/<model>_bdq_final.npz: the reference's trained agent (tools/export_agent.py)."""
    w = np.load(os.path.join(GOLD, f"{model}_bdq_final.npz"))
    q = BranchingQNetwork((n, n), n + 1, 3)
    q.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    return q.eval()


def pack(bits_rows: np.ndarray) -> np.ndarray:
    """(n, N) 0/1 -> (W, n) uint32 words (bit i of word w = node 32w + i)."""
    n, N = bits_rows.shape
    W = (N + 31) // 32
    pad = np.zeros((n, 32 * W), np.uint64)
    pad[:, :N] = bits_rows
    words = (pad.reshape(n, W, 32) << np.arange(32, dtype=np.uint64)).sum(axis=2)
    return words.T.astype(np.uint32)


def unpack(words: np.ndarray, N: int) -> np.ndarray:
    W, n = words.shape
    bits = (words.T[:, :, None] >> np.arange(32, dtype=np.uint32)) & 1
    return bits.reshape(n, 32 * W)[:, :N].astype(np.int64)


def greedy_flipmask(q, states: np.ndarray, targets: np.ndarray) -> np.ndarray:
    """(n, N) states and target states -> (W, n) flip masks of the greedy actions (each
    distinct a > 0 flips node a - 1 once)."""
    n, N = states.shape
    with torch.no_grad():
        x = torch.from_numpy(np.stack([states, targets]).astype(np.float32))
        acts = q(x).argmax(dim=2).numpy()                    # (n, branches)
    hit = np.zeros((n, N), np.int64)
    for a in acts.T:
        sel = a > 0
        hit[np.nonzero(sel)[0], a[sel] - 1] = 1
    return pack(hit)


def replay(step_fn, q, attractors, n_runs: int = 10, max_steps: int = 100):
    """Counts of model_tester.py:587-658: {(a, t): int array (n_runs,)}, 101 = failure."""
    A = len(attractors)
    N = len(attractors[0][0])
    pairs = list(itertools.product(range(A), repeat=2))
    runs = [(a, t) for (a, t) in pairs for _ in range(n_runs)]
    n = (len(runs) + 31) // 32 * 32
    start = np.array([list(attractors[a][0]) for a, _ in runs] + [list(attractors[0][0])] * (n - len(runs)))
    target = np.array([list(attractors[t][0]) for _, t in runs] + [list(attractors[0][0])] * (n - len(runs)))
    tsets = [set(map(tuple, attractors[t])) for _, t in runs]
    count = np.zeros(len(runs), np.int64)
    done = np.array([tuple(start[i]) in tsets[i] for i in range(len(runs))])
    words = pack(start)
    for k in range(1, max_steps + 2):
        if done.all():
            break
        bits = unpack(words, N)
        flip = greedy_flipmask(q, bits, target)
        words = step_fn(words, flip, k)
        bits = unpack(words, N)
        for i in np.nonzero(~done)[0]:
            count[i] = k
            if tuple(bits[i]) in tsets[i]:
                done[i] = True
    count[~done] = 101
    return {pair: count[i * n_runs:(i + 1) * n_runs] for i, pair in enumerate(pairs)}


def summary(res):
    """(per-run length matrix or None if runs differ, data histogram {count: runs}) as the
    reference pickles them (data/results/pbn_<n>_<a>.pkl: save_matrix, data)."""
    A = int(round(len(res) ** 0.5))
    mat = np.zeros((A, A))
    same = True
    data = {}
    for (a, t), c in res.items():
        mat[a, t] = c.sum()
        same = same and (c == c[0]).all()
        for v in c:
            data[int(v)] = data.get(int(v), 0) + 1
    return mat, same, data
