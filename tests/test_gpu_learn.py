"""The fused BDQ update (pbn_bdq_learn, csrc/pbn_learn.hip; FusedBDQUpdate) against the PyTorch
update it replaces (bdq_update + torch.optim.Adam, itself checked against update_policy's
expressions in test_gpu_replay.py): same nets, same replay rows.

Tolerances: the loss to rtol 1e-5; the clamped gradient to rtol 1e-3 / atol 1e-6 (the bilinear
layer runs as a sum of target-table rows, the other layers as MFMA tiles: fp32 sums in another
order); the Adam step to rtol 1e-5 against torch.optim.Adam's formula applied to the kernel's own
gradient; the target tables bit-exact against pbn_bdq_pack of the new weights."""
import copy

import numpy as np
import pytest
import torch

from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.replay import BDQLearner, DeviceReplay, FusedBDQUpdate, _bdq_segments, bdq_update
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

pytestmark = pytest.mark.gpu


def _filled_replay(spec, K, cap, seed):
    """A ring of random transitions: random states, targets (one in ten without a target), actions
    0..N, rewards, done flags."""
    dev = torch.device("cuda")
    R = DeviceReplay(cap, spec.words, K, dev)
    rng = np.random.default_rng(seed)
    N, W = spec.n, spec.words
    st = rng.integers(0, 2 ** 32, size=(W, cap), dtype=np.uint64).astype(np.uint32)
    nst = rng.integers(0, 2 ** 32, size=(W, cap), dtype=np.uint64).astype(np.uint32)
    if N % 32:
        st[W - 1] &= np.uint32((1 << (N % 32)) - 1)
        nst[W - 1] &= np.uint32((1 << (N % 32)) - 1)
    n_attr = len(spec.attractors)
    tg = rng.integers(0, max(n_attr, 1), size=cap).astype(np.uint8)
    tg[rng.random(cap) < 0.1] = 255
    act = rng.integers(0, N + 1, size=(cap, K)).astype(np.int32)
    rew = rng.standard_normal(cap).astype(np.float32)
    done = (rng.random(cap) < 0.5).astype(np.uint8)
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    R.store(to(st.view(np.int32)), to(tg), to(act), to(rew), to(nst.view(np.int32)), to(done))
    return R


def _nets(N, K, seed):
    torch.manual_seed(seed)
    q = BranchingQNetwork((N, N), N + 1, K).cuda()
    tgt = copy.deepcopy(q)
    with torch.no_grad():
        for p in tgt.parameters():
            p.add_(0.01 * torch.randn_like(p))
    return q, tgt


def _check_image(fused, q, N, K):
    """The image's weight tiles (pbn_learn.hip make_image) restated from the module's weights:
    per dense layer (the three trunk layers, the stacked first head layers, the second head layers
    as (K + 1) x Apad rows, zero past each head's N + 1), tile (ot, kt) of 256 floats in two
    orders; fwd lane g*16 + r holds M[16ot + r][16kt + 4g + v], bwd M[16ot + 4g + v][16kt + r]."""
    A, Ap = N + 1, 16 * ((N + 16) // 16)
    m = q.model
    heads = [q.value_head] + list(q.adv_heads)
    h2 = torch.zeros(len(heads), Ap, 64, device="cuda")
    for h, hd in enumerate(heads):
        h2[h, :hd[2].weight.shape[0]] = hd[2].weight.detach()
    mats = [m[2].weight.detach(), m[4].weight.detach(), m[6].weight.detach(),
            torch.cat([hd[0].weight.detach() for hd in heads]), h2.reshape(-1, 64)]
    o = fused.q_table.numel()
    for M in mats:
        R, C = M.shape
        t = M.reshape(R // 16, 16, C // 16, 16).permute(0, 2, 1, 3)          # [ot][kt][row][col]
        fwd = t.reshape(R // 16, C // 16, 16, 4, 4).permute(0, 1, 3, 2, 4)  # [ot][kt][g][r][v]: M[r][4g + v]
        bwd = t.reshape(R // 16, C // 16, 4, 4, 16).permute(0, 1, 2, 4, 3)  # [ot][kt][g][r][v]: M[4g + v][r]
        for want in (fwd, bwd):
            got = fused.q_image[o:o + R * C]
            assert torch.equal(got, want.reshape(-1)), (M.shape, o)
            o += R * C
    assert o == fused.q_image.numel()


@pytest.mark.parametrize("net,B,K", [("pbn28", 256, 3), ("pbn28", 32, 1), ("pbn28", 96, 7), ("pbn70", 64, 3)])
def test_fused_update_matches_pytorch(net, B, K):
    spec = EnvSpec(load_network(net), load_attractors(net))
    N = spec.n
    env = VectorPBNEnv(spec, 64)
    R = _filled_replay(spec, K, 1024, seed=B + K)
    q, tgt = _nets(N, K, seed=7)
    q_ref, tgt_ref = copy.deepcopy(q), copy.deepcopy(tgt)
    lr, gamma = 1e-3, 0.9
    fused = FusedBDQUpdate(q, tgt, env.net, K, batch_size=B, learning_rate=lr, gamma=gamma, keep_grad=True)
    idx = R.sample_indices(B, torch.Generator(device="cuda").manual_seed(B))
    p0 = [p.detach().clone() for p in q.parameters()]
    loss = float(fused.update(R, idx))
    torch.cuda.synchronize()
    opt = torch.optim.Adam(q_ref.parameters(), lr=lr)
    loss_ref = float(bdq_update(q_ref, tgt_ref, opt, R.gather(idx, env.net), gamma))
    assert abs(loss - loss_ref) <= 1e-5 * abs(loss_ref), (loss, loss_ref)
    names = [n for n, _ in q.named_parameters()]
    for name, g, p in zip(names, fused.grads(), q_ref.parameters()):
        assert torch.allclose(g, p.grad, rtol=1e-3, atol=1e-6), (name, (g - p.grad).abs().max().item())
    # Adam's first step from the kernel's own gradient (torch.optim.Adam's arithmetic)
    b1, b2, eps = 0.9, 0.999, 1e-8
    for name, g, a, b in zip(names, fused.grads(), p0, q.parameters()):
        m, v = (1 - b1) * g, (1 - b2) * g * g
        want = a - (lr / (1 - b1)) * m / (v.sqrt() / (1 - b2) ** 0.5 + eps)
        assert torch.allclose(b, want, rtol=1e-5, atol=1e-7), (name, (b - want).abs().max().item())
    assert float(fused.step) == 1.0
    # the value head's padding (outputs past 0) stays zero in the flat buffer
    o, A = fused.off, N + 1
    assert not fused.q_flat[o[10] + 64:o[10] + A * 64].any() and not fused.q_flat[o[11] + 1:o[11] + A].any()
    # the online image written by the update (table and fragment-ordered weights) = pbn_bdq_pack
    # of the new weights, bit for bit, and the table equal to the PyTorch contraction to rounding
    t_upd = fused.q_image.clone()
    fused.pack("online")
    assert torch.equal(t_upd, fused.q_image)
    _check_image(fused, q, N, K)
    if len(spec.attractors):
        targets = torch.tensor([list(a[0]) for a in spec.attractors], dtype=torch.float32, device="cuda")
        T = q.model[0].target_table(targets)
        assert torch.allclose(fused.q_table.transpose(2, 3).reshape(T.shape), T, rtol=1e-5, atol=1e-6)


def test_fused_update_trajectory_follows_pytorch():
    """Five updates on the same rows: the losses of the fused and the PyTorch updates stay together
    (Adam normalises each step, so weights whose gradient is ~0 may move differently by ~lr)."""
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    env = VectorPBNEnv(spec, 64)
    R = _filled_replay(spec, 3, 2048, seed=3)
    q, tgt = _nets(28, 3, seed=1)
    q_ref, tgt_ref = copy.deepcopy(q), copy.deepcopy(tgt)
    fused = FusedBDQUpdate(q, tgt, env.net, 3, batch_size=256, learning_rate=1e-4, gamma=0.999)
    opt = torch.optim.Adam(q_ref.parameters(), lr=1e-4)
    gen = torch.Generator(device="cuda").manual_seed(0)
    for k in range(5):
        idx = R.sample_indices(256, gen)
        a = float(fused.update(R, idx))
        b = float(bdq_update(q_ref, tgt_ref, opt, R.gather(idx, env.net), 0.999))
        assert abs(a - b) <= 1e-3 * abs(b), (k, a, b)
    fused.soft_update()
    with torch.no_grad():
        for t, o in zip(tgt_ref.parameters(), q_ref.parameters()):
            t.div_(2).add_(o / 2)
    for (n, a), b in zip(tgt.named_parameters(), tgt_ref.parameters()):
        assert torch.allclose(a, b, rtol=1e-3, atol=2e-3), n


def test_fused_layout_views():
    """The networks' parameters are views of the flat buffers in pbn_bdq_layout order, and the
    acting pack's stacked head weights equal head_weights()."""
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    env = VectorPBNEnv(spec, 64)
    q, tgt = _nets(28, 3, seed=2)
    sd = {k: v.clone() for k, v in q.state_dict().items()}
    fused = FusedBDQUpdate(q, tgt, env.net, 3, batch_size=64)
    for k, v in q.state_dict().items():
        assert torch.equal(v, sd[k]), k
    for p, seg, extra in _bdq_segments(q):
        at = fused.off[seg] + extra
        assert p.data_ptr() == fused.q_flat[at:].data_ptr()
    _, bias, hw, _ = fused.acting_pack()
    for a, b in zip(hw, q.head_weights()):
        assert torch.equal(a.reshape(b.shape), b)
    assert torch.equal(bias, q.model[0].bilinear.bias)


def _learner(n, seed, fused, updates_per_frame=1):
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.01)
    env = VectorPBNEnv(spec, n, seed=seed)
    torch.manual_seed(4)
    lr = BDQLearner(env, BranchingQNetwork((28, 28), 29, 3), capacity=8 * n, learning_starts=2 * n,
                    batch_size=256, target_update=4, epsilon_start=1.0, epsilon_final=1.0, seed=11,
                    graphable=True, fused=fused, updates_per_frame=updates_per_frame)
    env.reset()
    return env, lr


@pytest.mark.parametrize("upf", [1, 2])
def test_captured_fused_learner_is_bit_exact(upf):
    """epsilon = 1 and the fused update (no atomics, fixed reduction orders): a captured learner's
    weights, Adam state and losses equal the eager one's bit for bit, soft updates included, with
    one or two updates per frame (both batches of a frame from one draw)."""
    n = 1024
    env_e, eager = _learner(n, 21, True, upf)
    env_g, graph = _learner(n, 21, True, upf)
    assert eager.fused is not None and eager.opt is None
    graph.capture()
    for _ in range(graph.frames):
        eager.frame()
    for k in range(9):
        eager.frame()
        graph.frame()
        torch.cuda.synchronize()
        assert torch.equal(eager.last_loss, graph.last_loss), k
    assert eager.updates == graph.updates
    assert torch.equal(eager.fused.q_flat, graph.fused.q_flat)
    assert torch.equal(eager.fused.t_flat, graph.fused.t_flat)
    assert torch.equal(eager.fused.m, graph.fused.m) and torch.equal(eager.fused.v, graph.fused.v)
    assert torch.equal(eager.fused.q_image, graph.fused.q_image)
    assert float(eager.fused.step) == float(graph.fused.step) == eager.updates


def test_fused_learner_acts_with_its_tables():
    """The acting frame reads the fused update's table and stacked head weights: its flip masks
    equal the ones of an unfused BatchedBDQ on a copy of the trained network."""
    from pbn_rl_amd.agent import BatchedBDQ
    env, lr = _learner(512, 5, True)
    for _ in range(5):
        lr.frame()
    torch.cuda.synchronize()
    q2 = copy.deepcopy(lr.q).eval()
    env2 = VectorPBNEnv(env.spec, 512, seed=5)
    env2.reset()
    env2.state.copy_(env.state)
    env2.target.copy_(env.target)
    env2.step_index = env.step_index
    ref = BatchedBDQ(env2, q2)
    lr.agent.act_q(0.0)
    ref.act_q(0.0)
    torch.cuda.synchronize()
    same = (lr.agent.actions == ref.actions).float().mean().item()
    assert same > 0.999, same   # (argmax ties broken by fp rounding may differ)


def test_fused_learner_loads_a_checkpoint():
    """A reference-style checkpoint (the networks' state_dict, bdq_model/__init__.py:244) loads into
    the fused learner's view parameters; refresh_weights() repacks the tables the acting frame and
    the update read, equal to pbn_bdq_pack of the loaded weights."""
    env, lr = _learner(256, 3, True)
    src = BranchingQNetwork((28, 28), 29, 3).cuda()
    with torch.no_grad():
        for p in src.parameters():
            p.mul_(-1.5)
    lr.q.load_state_dict(src.state_dict())
    lr.target.load_state_dict(src.state_dict())
    lr.refresh_weights()
    torch.cuda.synchronize()
    for (k, a), b in zip(lr.q.named_parameters(), src.parameters()):
        assert torch.equal(a, b), k
    targets = torch.tensor([list(a[0]) for a in env.spec.attractors], dtype=torch.float32, device="cuda")
    T = src.model[0].target_table(targets)
    for table in (lr.fused.q_table, lr.fused.t_table):
        assert torch.allclose(table.transpose(2, 3).reshape(T.shape), T, rtol=1e-5, atol=1e-6)
    for _ in range(3):
        lr.frame()
    torch.cuda.synchronize()
    assert torch.isfinite(lr.last_loss)


def test_fused_update_matches_reference_update_policy():
    """pbn_bdq_learn held to the reference's own update_policy (bdq_model/__init__.py:100-139):
    tests/golden/bdq_update.npz, two calls of that method's source on the reference network
    (tools/gen_update_golden.py; the CPU form is held to it in tests/test_update_golden.py).  The
    fixture's batches go into a DeviceReplay ring (rows 0..255 in order, targets as attractor ids).
    Loss rtol 1e-5; clamped gradients rtol 1e-3 / atol 1e-6; parameters after Adam: atol 1e-5
    where the reference gradient exceeds 1e-4 (one Adam step is ~lr there), else within two steps
    (2 lr: a gradient near 0 may take the other sign); the soft-updated target likewise."""
    from tests.test_update_golden import load_fixture
    d, names = load_fixture()
    N, K, B = 7, 3, 256
    lr, gamma = float(d["lr"]), float(d["gamma"])
    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"))
    env = VectorPBNEnv(spec, 64)
    dev = torch.device("cuda")
    q, tgt = BranchingQNetwork((N, N), N + 1, K).to(dev), BranchingQNetwork((N, N), N + 1, K).to(dev)
    q.load_state_dict({n: torch.from_numpy(d["q0." + n]) for n in names})
    tgt.load_state_dict({n: torch.from_numpy(d["t0." + n]) for n in names})
    fused = FusedBDQUpdate(q, tgt, env.net, K, batch_size=B, learning_rate=lr, gamma=gamma, keep_grad=True)
    bits = (1 << np.arange(N, dtype=np.uint32))
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    idx = torch.arange(B, dtype=torch.int64, device=dev)
    for call in (1, 2):
        p = f"b{call}."
        R = DeviceReplay(B, 1, K, dev)
        st = (d[p + "states"].astype(np.uint32) * bits).sum(1).astype(np.uint32)[None]
        nst = (d[p + "next_states"].astype(np.uint32) * bits).sum(1).astype(np.uint32)[None]
        R.store(to(st.view(np.int32)), to(d[p + "target_ids"]), to(d[p + "actions"].astype(np.int32)),
                to(d[p + "rewards"]), to(nst.view(np.int32)), to(d[p + "done"]))
        loss = float(fused.update(R, idx))
        torch.cuda.synchronize()
        want = float(d["losses"][call - 1])
        assert abs(loss - want) <= 1e-5 * abs(want), (call, loss, want)
        for n, g, w in zip(names, fused.grads(), q.parameters()):
            g_ref = torch.from_numpy(d[f"g{call}.{n}"]).to(dev)
            assert torch.allclose(g, g_ref, rtol=1e-3, atol=1e-6), (call, n, (g - g_ref).abs().max().item())
            w_ref = torch.from_numpy(d[f"q{call}.{n}"]).to(dev)
            err = (w.detach() - w_ref).abs()
            big = g_ref.abs() > 1e-4
            assert err[big].max().item() <= 1e-5 if big.any() else True, (call, n, err[big].max().item())
            assert err.max().item() <= 2.1 * lr * call, (call, n, err.max().item())
    fused.soft_update()
    for n, w in zip(names, tgt.parameters()):
        w_ref = torch.from_numpy(d["t2." + n]).to(dev)
        assert (w.detach() - w_ref).abs().max().item() <= 2.1 * lr, n


def test_fused_update_matches_reference_update_policy_benched_shape():
    """pbn_bdq_learn at the benched shape, BranchingQNetwork((28, 28), 29, 3) (config 5 and the
    bdq-learn line), held to the reference's update_policy through the sampled fixture
    tests/golden/bdq_update28.npz (tools/gen_update_golden.py --shape 28; formula initial weights,
    per-tensor norms and 4,096 sampled entries).  The tolerances of the N = 7 test: loss rtol 1e-5,
    clamped gradients rtol 1e-3 / atol 1e-6, parameters after Adam atol 1e-5 where the reference
    gradient exceeds 1e-4, else within two Adam steps; the soft-updated target likewise."""
    from tests.test_update_golden import load_fixture28, nets28_from, sampled_close
    d, names = load_fixture28()
    N, K, B = 28, 3, 256
    lr, gamma = float(d["lr"]), float(d["gamma"])
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    env = VectorPBNEnv(spec, 64)
    dev = torch.device("cuda")
    q, tgt = nets28_from(d, names)
    q, tgt = q.to(dev), tgt.to(dev)
    fused = FusedBDQUpdate(q, tgt, env.net, K, batch_size=B, learning_rate=lr, gamma=gamma, keep_grad=True)
    bits = (1 << np.arange(N, dtype=np.uint32))
    to = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    idx = torch.arange(B, dtype=torch.int64, device=dev)
    for call in (1, 2):
        p = f"b{call}."
        R = DeviceReplay(B, 1, K, dev)
        st = (d[p + "states"].astype(np.uint32) * bits).sum(1).astype(np.uint32)[None]
        nst = (d[p + "next_states"].astype(np.uint32) * bits).sum(1).astype(np.uint32)[None]
        R.store(to(st.view(np.int32)), to(d[p + "target_ids"]), to(d[p + "actions"].astype(np.int32)),
                to(d[p + "rewards"]), to(nst.view(np.int32)), to(d[p + "done"]))
        loss = float(fused.update(R, idx))
        torch.cuda.synchronize()
        want = float(d["losses"][call - 1])
        assert abs(loss - want) <= 1e-5 * abs(want), (call, loss, want)
        for n, g, w in zip(names, fused.grads(), q.parameters()):
            ok, err, _ = sampled_close(g, d, f"g{call}.{n}", n, 1e-3, 1e-6)
            assert ok, (call, n, err)
            sel = torch.from_numpy(d["idx." + n]).to(dev)
            w_ref = torch.from_numpy(d[f"q{call}.{n}"]).to(dev)
            g_ref = torch.from_numpy(d[f"g{call}.{n}"]).to(dev)
            err = (w.detach().reshape(-1)[sel] - w_ref).abs()
            big = g_ref.abs() > 1e-4
            assert err[big].max().item() <= 1e-5 if big.any() else True, (call, n, err[big].max().item())
            assert err.max().item() <= 2.1 * lr * call, (call, n, err.max().item())
    fused.soft_update()
    for n, w in zip(names, tgt.parameters()):
        sel = torch.from_numpy(d["idx." + n]).to(dev)
        w_ref = torch.from_numpy(d["t2." + n]).to(dev)
        assert (w.detach().reshape(-1)[sel] - w_ref).abs().max().item() <= 2.1 * lr, n
