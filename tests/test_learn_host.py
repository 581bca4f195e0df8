"""Host side of the fused BDQ update (no GPU): pbn_bdq_layout's segments hold exactly the
reference network's parameters (bdq_model/network.py:24-63) without overlap, the workspace query
validates the batch, and the learner refuses a fused update it cannot run."""
import ctypes

import pytest

from pbn_rl_amd import _lib
from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.replay import _bdq_segments, bdq_layout


@pytest.mark.parametrize("N,K", [(28, 3), (7, 1), (70, 3), (127, 7)])
def test_layout_holds_the_parameters(N, K):
    off = bdq_layout(N, K)
    assert len(off) == 13 and off[0] == 0
    assert all(o % 16 == 0 for o in off)
    assert all(a < b for a, b in zip(off, off[1:]))
    q = BranchingQNetwork((N, N), N + 1, K)
    spans = []
    for p, seg, extra in _bdq_segments(q):
        lo = off[seg] + extra
        hi = lo + p.numel()
        assert off[seg] <= lo and hi <= off[seg + 1], (seg, p.shape)
        spans.append((lo, hi))
    spans.sort()
    assert all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
    assert sum(p.numel() for p in q.parameters()) == sum(h - l for l, h in spans)
    # the value head's second layer is padded to N + 1 outputs: the only gap inside a segment
    H, A = K + 1, N + 1
    assert off[11] - off[10] >= H * A * 64 and off[12] - off[11] >= H * A


def test_layout_and_workspace_reject_bad_shapes():
    L = _lib.load()
    off = (ctypes.c_int64 * 13)()
    assert L.pbn_bdq_layout(0, 3, off) != 0
    assert L.pbn_bdq_layout(128, 3, off) != 0
    assert L.pbn_bdq_layout(28, 8, off) != 0
    b = ctypes.c_int64()
    assert L.pbn_bdq_learn_workspace(28, 3, 256, ctypes.byref(b)) == 0 and b.value > 0
    small = b.value
    assert L.pbn_bdq_learn_workspace(28, 3, 512, ctypes.byref(b)) == 0 and b.value > small
    for bad in (0, 8, 250):
        assert L.pbn_bdq_learn_workspace(28, 3, bad, ctypes.byref(b)) != 0


def test_replay_rows_restatement():
    """agent_oracle.replay_rows (the numpy checker of pbn_replay_advance's rows) against the scalar
    Philox restatement pyoracle.draw, REPLAY stream 7."""
    from oracle import agent_oracle, pyoracle
    rows = agent_oracle.replay_rows(123, 5, 50, 540)
    for b in range(50):
        x, y, _, _ = pyoracle.draw(123, b, 5, 7, 0)
        assert rows[b] == ((x << 32 | y) * 540) >> 64
    assert rows.min() >= 0 and rows.max() < 540


def test_fused_support_query():
    from pbn_rl_amd.replay import fused_update_supported
    assert fused_update_supported(28, 3, 256) and fused_update_supported(70, 3, 64)
    assert not fused_update_supported(28, 3, 100)        # batch not a multiple of 16
    assert not fused_update_supported(127, 7, 256)       # the backward's staged heads exceed one block's LDS
    assert fused_update_supported(127, 3, 256)
