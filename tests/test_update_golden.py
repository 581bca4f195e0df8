"""The learner update pinned to the reference's own update_policy (bdq_model/__init__.py:100-139):
tests/golden/bdq_update.npz holds two calls of that method's source text, executed by
tools/gen_update_golden.py on the reference's BranchingQNetwork (bdq_model/network.py) with a fixed
batch, Adam(lr=1e-3), gamma 0.9 and target_net_update_freq 2 (call 2 ends in the soft update).

CPU: bdq_update (pbn_rl_amd/replay.py, the PyTorch form) + torch.optim.Adam + soft_update from the
fixture's weights and batches.  The GPU form (pbn_bdq_learn) is held to the same fixture in
tests/test_gpu_learn.py.  Tolerances: loss rtol 1e-5, clamped gradients rtol 1e-5 / atol 1e-7
(the same PyTorch arithmetic, the bilinear layer contracted in another order), parameters after
Adam atol 1e-5, 1 % of lr: one Adam step moves a weight by ~lr = 1e-3, and a gradient of the order
of Adam's eps (1e-8) moves it by a fraction of that which its last bits decide."""
import os

import numpy as np
import torch

from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.replay import bdq_update, soft_update

GOLD = os.path.join(os.path.dirname(__file__), "golden", "bdq_update.npz")


def load_fixture():
    d = np.load(GOLD)
    return d, [str(n) for n in d["names"]]


def nets_from(d, names, N=7, K=3):
    q, t = BranchingQNetwork((N, N), N + 1, K), BranchingQNetwork((N, N), N + 1, K)
    q.load_state_dict({n: torch.from_numpy(d["q0." + n]) for n in names})
    t.load_state_dict({n: torch.from_numpy(d["t0." + n]) for n in names})
    return q, t


def batch_of(d, call):
    """The fixture's batch in bdq_update's layout: obs / next_obs (2, B, N) = (state, target)."""
    p = f"b{call}."
    f32 = lambda k: torch.from_numpy(d[p + k].astype(np.float32))  # noqa: E731
    return {"obs": torch.stack([f32("states"), f32("targets")]),
            "next_obs": torch.stack([f32("next_states"), f32("targets")]),
            "actions": torch.from_numpy(d[p + "actions"]).long().unsqueeze(-1),
            "rewards": f32("rewards").reshape(-1, 1),
            "masks": f32("done").reshape(-1, 1)}


def test_fixture_is_the_reference_method():
    d, names = load_fixture()
    assert tuple(d["lines"]) == (100, 139)       # update_policy's span in bdq_model/__init__.py
    assert len(names) == len(list(BranchingQNetwork((7, 7), 8, 3).parameters()))


def test_bdq_update_matches_reference_update_policy():
    d, names = load_fixture()
    q, t = nets_from(d, names)
    opt = torch.optim.Adam(q.parameters(), lr=float(d["lr"]))
    gamma = float(d["gamma"])
    for call in (1, 2):
        loss = float(bdq_update(q, t, opt, batch_of(d, call), gamma=gamma))
        want = float(d["losses"][call - 1])
        assert abs(loss - want) <= 1e-5 * abs(want), (call, loss, want)
        for n, p in q.named_parameters():
            g = torch.from_numpy(d[f"g{call}.{n}"])
            assert torch.allclose(p.grad, g, rtol=1e-5, atol=1e-7), (call, n, (p.grad - g).abs().max().item())
            w = torch.from_numpy(d[f"q{call}.{n}"])
            assert torch.allclose(p.detach(), w, rtol=0, atol=1e-5), (call, n, (p.detach() - w).abs().max().item())
    soft_update(t, q)   # target_net_update_freq 2: the second call ends in the soft update
    for n, p in t.named_parameters():
        w = torch.from_numpy(d["t2." + n])
        assert torch.allclose(p.detach(), w, rtol=0, atol=1e-5), (n, (p.detach() - w).abs().max().item())
