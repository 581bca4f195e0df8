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
GOLD28 = os.path.join(os.path.dirname(__file__), "golden", "bdq_update28.npz")


def formula_params(shapes, seed):
    """Initial online and target weights of the sampled fixture (bdq_update28.npz), computed the
    same way by tools/gen_update_golden.py and the tests: parameter i is seeded normals scaled by
    1/sqrt(fan-in) (0.05 for biases), the target that plus 0.05 x normals of another stream."""
    q, t = {}, {}
    for i, (name, shape) in enumerate(shapes):
        r = np.random.default_rng(seed * 1000 + i)
        fan = int(np.prod(shape[1:])) if len(shape) > 1 else 0
        v = r.standard_normal(shape) * (1.0 / np.sqrt(fan) if fan else 0.05)
        q[name] = v.astype(np.float32)
        t[name] = (v + 0.05 * r.standard_normal(shape)).astype(np.float32)
    return q, t


def load_fixture28():
    d = np.load(GOLD28)
    return d, [str(n) for n in d["names"]]


def nets28_from(d, names, N=28, K=3):
    q, t = BranchingQNetwork((N, N), N + 1, K), BranchingQNetwork((N, N), N + 1, K)
    init_q, init_t = formula_params([(n, tuple(p.shape)) for n, p in q.named_parameters()], int(d["init_seed"]))
    q.load_state_dict({n: torch.from_numpy(v) for n, v in init_q.items()})
    t.load_state_dict({n: torch.from_numpy(v) for n, v in init_t.items()})
    return q, t


def sampled_close(got: torch.Tensor, d, key, n, rtol, atol):
    """got (a whole tensor) against the fixture's norm and sampled entries of ``key``"""
    idx = torch.from_numpy(d["idx." + n]).to(got.device)
    want = torch.from_numpy(d[key]).to(got.device)
    s = got.detach().reshape(-1)[idx]
    norm = float(got.detach().double().norm())
    ok_norm = abs(norm - float(d[key + ".norm"])) <= max(rtol * float(d[key + ".norm"]), atol * np.sqrt(got.numel()))
    return bool(torch.allclose(s, want, rtol=rtol, atol=atol)) and ok_norm, (s - want).abs().max().item(), norm


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


def test_bdq_update_matches_reference_update_policy_benched_shape():
    """The benched shape, BranchingQNetwork((28, 28), 29, 3) (config 5 / the bdq-learn line), held
    to two calls of the reference's update_policy through the sampled fixture (bdq_update28.npz):
    loss rtol 1e-5, per-tensor norms and 4,096 sampled entries of the clamped gradients
    (rtol 1e-4 / atol 1e-6: at 28 nodes the contracted bilinear layer sums 784-term products in
    another order than nn.Bilinear, and call 2 starts from weights that differ in their last bits)
    and of the parameters after Adam and the soft update (atol 1e-5)."""
    d, names = load_fixture28()
    assert tuple(d["lines"]) == (100, 139)
    q, t = nets28_from(d, names)
    opt = torch.optim.Adam(q.parameters(), lr=float(d["lr"]))
    for call in (1, 2):
        loss = float(bdq_update(q, t, opt, batch_of(d, call), gamma=float(d["gamma"])))
        want = float(d["losses"][call - 1])
        assert abs(loss - want) <= 1e-5 * abs(want), (call, loss, want)
        for n, p in q.named_parameters():
            ok, err, _ = sampled_close(p.grad, d, f"g{call}.{n}", n, 1e-4, 1e-6)
            assert ok, (call, n, err)
            ok, err, _ = sampled_close(p, d, f"q{call}.{n}", n, 0, 1e-5)
            assert ok, (call, n, err)
    soft_update(t, q)
    for n, p in t.named_parameters():
        ok, err, _ = sampled_close(p, d, f"t2.{n}", n, 0, 1e-5)
        assert ok, (n, err)
