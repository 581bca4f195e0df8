"""bdq_update / soft_update (pbn_rl_amd.replay), CPU: the restated update_policy step
(bdq_model/__init__.py:111-139) against the same arithmetic written out longhand."""
import copy

import torch
import torch.nn.functional as F

from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.replay import bdq_update, soft_update


def batch_for(N, B, K=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    return {"obs": torch.randint(0, 2, (2, B, N), generator=g).float(),
            "next_obs": torch.randint(0, 2, (2, B, N), generator=g).float(),
            "actions": torch.randint(0, N + 1, (B, K, 1), generator=g),
            "rewards": torch.randn(B, 1, generator=g),
            "masks": torch.randint(0, 2, (B, 1), generator=g).float()}


def test_update_matches_longhand():
    torch.manual_seed(0)
    N, B = 7, 64
    q = BranchingQNetwork((N, N), N + 1, 3)
    tgt = copy.deepcopy(q)
    for p in tgt.parameters():
        p.data.add_(0.01)
    q2, tgt2 = copy.deepcopy(q), copy.deepcopy(tgt)
    opt = torch.optim.Adam(q.parameters(), lr=1e-3)
    opt2 = torch.optim.Adam(q2.parameters(), lr=1e-3)
    b = batch_for(N, B)
    loss = bdq_update(q, tgt, opt, b, gamma=0.9)
    # longhand: update_policy lines 111-131
    cur = q2(b["obs"]).gather(2, b["actions"]).squeeze(-1)
    with torch.no_grad():
        am = q2(b["next_obs"]).argmax(dim=2)
        nxt = tgt2(b["next_obs"]).gather(2, am.unsqueeze(2)).squeeze(-1)
    want = F.mse_loss(b["rewards"] + nxt * 0.9 * b["masks"], cur)
    opt2.zero_grad()
    want.backward()
    for p in q2.parameters():
        p.grad.data.clamp_(-1.0, 1.0)
    opt2.step()
    assert torch.allclose(loss, want.detach())
    for a, c in zip(q.parameters(), q2.parameters()):
        assert torch.equal(a, c)


def test_soft_update_halves():
    torch.manual_seed(1)
    q = BranchingQNetwork((5, 5), 6, 3)
    t = BranchingQNetwork((5, 5), 6, 3)
    before = {k: v.clone() for k, v in t.state_dict().items()}
    soft_update(t, q)
    for k, v in t.state_dict().items():
        assert torch.allclose(v, before[k] / 2 + q.state_dict()[k] / 2)


def test_ring_device_position_matches_host_position():
    """store_at / sample_indices(size_t=...) (the graph-captured forms) against store /
    sample_indices with host ints, on CPU tensors."""
    from pbn_rl_amd.replay import DeviceReplay
    a, b = DeviceReplay(100, 2, 3, "cpu"), DeviceReplay(100, 2, 3, "cpu")
    pos_t, size_t = torch.zeros(1, dtype=torch.int64), torch.zeros(1, dtype=torch.int64)
    g = torch.Generator().manual_seed(0)
    for k in range(5):          # 5 x 32 = 160 > 100: wraps
        n = 32
        st = torch.randint(-2 ** 31, 2 ** 31 - 1, (2, n), generator=g, dtype=torch.int32)
        nst = torch.randint(-2 ** 31, 2 ** 31 - 1, (2, n), generator=g, dtype=torch.int32)
        tg = torch.randint(0, 14, (n,), generator=g)
        act = torch.randint(0, 29, (n, 3), generator=g)
        rw, dn = torch.randn(n, generator=g), torch.randint(0, 2, (n,), generator=g)
        a.store(st, tg, act, rw, nst, dn)
        b.store_at(pos_t, size_t, st, tg, act, rw, nst, dn)
        assert int(pos_t) == a.pos and int(size_t) == a.size
    for f in ("state", "next_state", "target", "action", "reward", "done"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
    i1 = a.sample_indices(4096, torch.Generator().manual_seed(3))
    i2 = b.sample_indices(4096, torch.Generator().manual_seed(3), size_t=size_t)
    assert torch.equal(i1, i2) and int(i1.min()) >= 0 and int(i1.max()) == 99


def test_control_to_flipmask():
    """ControlPBNEnv action form: flip exactly the control nodes whose value differs."""
    import pytest
    from pbn_rl_amd.vector_env import control_to_flipmask, pack_states, unpack_states
    g = torch.Generator().manual_seed(5)
    N, n = 40, 64
    bits = torch.randint(0, 2, (n, N), generator=g)
    st = pack_states(bits, N)
    ctrl = [0, 3, 31, 32, 39]
    vals = torch.randint(0, 2, (n, len(ctrl)), generator=g)
    fm = control_to_flipmask(st, vals, ctrl, N)
    s1 = unpack_states(st ^ fm, N).long()
    for k, c in enumerate(ctrl):
        assert torch.equal(s1[:, c], vals[:, k])
    others = [i for i in range(N) if i not in ctrl]
    assert torch.equal(s1[:, others], bits[:, others].long())
    with pytest.raises(ValueError):
        control_to_flipmask(st, vals, [0, 3, 31, 32, 40], N)
