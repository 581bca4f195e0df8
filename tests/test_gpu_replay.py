"""On-device replay and the batched BDQ learner (pbn_rl_amd.replay) on the GPU: the ring holds
exactly the transitions the oracle produces for the same actions, sampled rows unpack to the
oracle's network inputs, and learning steps run end to end."""
import numpy as np
import pytest
import torch

from oracle import agent_oracle, oracle
from pbn_rl_amd.agent import BranchingQNetwork
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.replay import BDQLearner, DeviceReplay
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

pytestmark = pytest.mark.gpu


def u32(x):
    return x.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("fused,settle,n", [(True, 0, 1024), (False, 0, 1024), (True, 64, 32768)])
def test_learner_transitions_match_oracle(fused, settle, n):
    """settle = 64 at 32,768 envs: BDQLearner's frames under the facade's default law (config 5's
    per-GPU share), every stored transition against the oracle chain."""
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.02, settle=settle)
    seed = 17
    env = VectorPBNEnv(spec, n, seed=seed)
    torch.manual_seed(0)
    learner = BDQLearner(env, BranchingQNetwork((28, 28), 29, 3), capacity=4 * n, learning_starts=2 * n,
                         epsilon_start=0.5, seed=3, fused=fused)
    env.reset()
    st, tg, t = oracle.reset(spec, seed, 0, 0, n)
    for k in range(3):
        step = env.step_index
        learner.frame()
        torch.cuda.synchronize()
        acts = learner.agent.actions.cpu().numpy()
        flip = np.zeros((1, n), dtype=np.uint32)
        for b in range(3):
            a = acts[:, b].astype(np.int64)
            flip[0] |= np.where(a > 0, np.left_shift(np.uint32(1), np.maximum(a - 1, 0).astype(np.uint32)), 0).astype(np.uint32)
        ref = oracle.step(spec, seed, step, 0, st, flip, tg, t, 1)
        sl = slice(k * n, (k + 1) * n)
        R = learner.replay
        assert np.array_equal(u32(R.state[:, sl]), st)
        assert np.array_equal(R.target[sl].cpu().numpy(), tg)
        assert np.array_equal(u32(R.next_state[:, sl]), ref["final_state"])
        assert np.array_equal(R.reward[sl].cpu().numpy(), ref["reward"])
        assert np.array_equal(R.done[sl].cpu().numpy(), ((ref["flags"] & 3) != 0).astype(np.uint8))
        st, tg, t = ref["state_out"], ref["target"], ref["t"]
    # the ring is now 3n of 4n: learning started at 2n
    assert learner.updates == 2 and torch.isfinite(learner.last_loss)
    assert learner.epsilon < 0.5


def test_gather_unpacks_like_the_oracle():
    spec = EnvSpec(load_network("pbn70"), load_attractors("pbn70"))
    env = VectorPBNEnv(spec, 64)
    R = DeviceReplay(512, spec.words, 3, env.device)
    rng = np.random.default_rng(0)
    st = rng.integers(0, 2 ** 32, size=(3, 512), dtype=np.uint64).astype(np.uint32)
    st[2] &= np.uint32((1 << 6) - 1)
    nst = st[:, ::-1].copy()
    tg = rng.integers(0, 16, size=512).astype(np.uint8)
    to = lambda a: torch.from_numpy(a.view(np.int32).copy()).cuda()  # noqa: E731
    R.store(to(st), torch.from_numpy(tg).cuda(), torch.zeros(512, 3, dtype=torch.int32, device="cuda"),
            torch.zeros(512, device="cuda"), to(nst), torch.zeros(512, dtype=torch.uint8, device="cuda"))
    idx = R.sample_indices(96, torch.Generator(device="cuda").manual_seed(1))
    b = R.gather(idx, env.net)
    torch.cuda.synchronize()
    i = idx.cpu().numpy()
    assert np.array_equal(b["obs"].cpu().numpy(), agent_oracle.obs_unpack(spec, st[:, i], tg[i]))
    assert np.array_equal(b["next_obs"].cpu().numpy(), agent_oracle.obs_unpack(spec, nst[:, i], tg[i]))


@pytest.mark.parametrize("fused", [True, False])
def test_learner_many_frames(fused):
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"))
    env = VectorPBNEnv(spec, 4096, seed=1)
    torch.manual_seed(1)
    learner = BDQLearner(env, capacity=1 << 16, learning_starts=4096, updates_per_frame=2, target_update=5,
                         fused=fused)
    env.reset()
    w0 = learner.q.model[0].bilinear.weight.detach().clone()
    for _ in range(12):
        learner.frame()
    torch.cuda.synchronize()
    assert learner.updates == 24 and torch.isfinite(learner.last_loss)   # learning starts after frame 1
    assert not torch.equal(w0, learner.q.model[0].bilinear.weight)
    assert learner.replay.size == 12 * 4096


@pytest.mark.parametrize("B,K", [(256, 3), (512, 3), (32, 1), (40, 7)])
def test_fused_td_loss_matches_pytorch(B, K):
    """pbn_bdq_td_loss (bdq_update's GPU path: both duelings, the double-DQN target, the MSE and
    the backward in one launch) against the same update written in PyTorch, on the same nets and
    batch: the loss to rtol 1e-5 and every parameter gradient to rtol 1e-4 / atol 1e-7 (the
    dueling means and the value head's sum over branches are summed in a different order).
    B = 32 at K = 1 is one block of the row pass."""
    import copy

    import torch.nn.functional as F

    from pbn_rl_amd.replay import _TDLoss
    torch.manual_seed(3)
    N = 28
    q = BranchingQNetwork((N, N), N + 1, K).cuda()
    tgt = copy.deepcopy(q)
    with torch.no_grad():
        for p in tgt.parameters():
            p.add_(0.01 * torch.randn_like(p))
    g = torch.Generator(device="cuda").manual_seed(5)
    obs = torch.randint(0, 2, (2, B, N), device="cuda", generator=g).float()
    nxt = torch.randint(0, 2, (2, B, N), device="cuda", generator=g).float()
    actions = torch.randint(0, N + 1, (B, K, 1), device="cuda", generator=g)
    rewards = torch.randn(B, 1, device="cuda", generator=g)
    masks = torch.randint(0, 2, (B, 1), device="cuda", generator=g).float()
    x = torch.cat([obs, nxt], 1)
    params = list(q.parameters())
    heads = q.forward_heads(q.model[0](x))
    with torch.no_grad():
        t_heads = tgt.forward_heads(tgt.model[0](nxt)).contiguous()
    loss_f = _TDLoss.apply(heads.contiguous(), t_heads, actions.reshape(B, K).contiguous(), rewards.reshape(B).contiguous(),
                           masks.reshape(B).contiguous(), 0.9)
    g_f = torch.autograd.grad(loss_f, params, allow_unused=True)
    q_all = q(x)
    cur = q_all[:B].gather(2, actions).squeeze(-1)
    with torch.no_grad():
        am = q_all[B:].argmax(dim=2)
        mx = tgt(nxt).gather(2, am.unsqueeze(2)).squeeze(-1)
    loss_t = F.mse_loss(rewards + mx * 0.9 * masks, cur)
    g_t = torch.autograd.grad(loss_t, params, allow_unused=True)
    assert torch.allclose(loss_f, loss_t, rtol=1e-5, atol=0), (loss_f.item(), loss_t.item())
    for a, b in zip(g_f, g_t):
        if a is None or b is None:
            assert a is None and b is None
            continue
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-7), (a - b).abs().max().item()


def test_replay_store_kernel_matches_index_copy():
    """store_at's one-launch ring write (pbn_replay_store) equals the six index_copy_ of the
    same transitions, across the ring's wrap-around, and advances the device position and size."""
    dev = torch.device("cuda")
    cap, n, W, K = 100, 64, 2, 3
    g = torch.Generator(device="cuda").manual_seed(1)
    a = DeviceReplay(cap, W, K, dev)
    for step in range(3):   # 64, 128 -> wraps at 100
        st = torch.randint(-2 ** 31, 2 ** 31 - 1, (W, n), device=dev, generator=g, dtype=torch.int64).to(torch.int32)
        nst = torch.randint(-2 ** 31, 2 ** 31 - 1, (W, n), device=dev, generator=g, dtype=torch.int64).to(torch.int32)
        tg = torch.randint(0, 200, (n,), device=dev, generator=g).to(torch.uint8)
        act = torch.randint(0, 29, (n, K), device=dev, generator=g).to(torch.int32)
        rew = torch.randn(n, device=dev, generator=g)
        done = torch.randint(0, 2, (n,), device=dev, generator=g).bool()
        pos_t = torch.full((1,), a.pos, dtype=torch.int64, device=dev)
        size_t = torch.full((1,), a.size, dtype=torch.int64, device=dev)
        want = {k: getattr(a, k).clone() for k in ("state", "next_state", "target", "action", "reward", "done")}
        idx = (torch.arange(n, device=dev) + a.pos) % cap
        want["state"].index_copy_(1, idx, st)
        want["next_state"].index_copy_(1, idx, nst)
        want["target"].index_copy_(0, idx, tg)
        want["action"].index_copy_(0, idx, act)
        want["reward"].index_copy_(0, idx, rew)
        want["done"].index_copy_(0, idx, done.to(torch.uint8))
        a.store_at(pos_t, size_t, st, tg, act, rew, nst, done)
        for k, v in want.items():
            assert torch.equal(getattr(a, k), v), (step, k)
        a.pos = (a.pos + n) % cap
        a.size = min(a.size + n, cap)
        assert int(pos_t.item()) == a.pos and int(size_t.item()) == a.size


def test_replay_advance_counters_and_rows():
    """pbn_replay_advance (a captured frame's counters and the fused learner's rows): position,
    fill level, step index and epsilon as the host arithmetic of BDQLearner.frame, and the rows
    bit-exact against oracle.agent_oracle.replay_rows."""
    from pbn_rl_amd import _lib
    dev = torch.device("cuda")
    i64 = lambda v: torch.tensor([v], dtype=torch.int64, device=dev)  # noqa: E731
    pos, size, step, draw = i64(990), i64(500), i64(7), i64(5)
    eps64 = torch.tensor([0.3], dtype=torch.float64, device=dev)
    eps32 = torch.empty(1, dtype=torch.float32, device=dev)
    idx = torch.empty(300, dtype=torch.int64, device=dev)
    L = _lib.load()
    for k in range(3):
        _lib.check(L.pbn_replay_advance(40, 1000, pos.data_ptr(), size.data_ptr(), step.data_ptr(), eps64.data_ptr(),
                                        eps32.data_ptr(), 0.2, 0.05, 300, 123, draw.data_ptr(), idx.data_ptr(),
                                        torch.cuda.current_stream().cuda_stream), "pbn_replay_advance")
        torch.cuda.synchronize()
        want_size = min(500 + 40 * (k + 1), 1000)
        assert int(pos) == (990 + 40 * (k + 1)) % 1000 and int(size) == want_size and int(step) == 8 + k
        e = 0.3
        for _ in range(k + 1):
            e = max(0.2, e - 0.05)
        assert float(eps64) == e and float(eps32) == float(np.float32(e))
        assert int(draw) == 6 + k
        assert np.array_equal(idx.cpu().numpy(), agent_oracle.replay_rows(123, 5 + k, 300, want_size))


def test_replay_store_done_from_flags():
    """store_at with done_mask: the ring's done (and done_out) = flags & mask != 0."""
    dev = torch.device("cuda")
    n = 96
    a = DeviceReplay(128, 1, 3, dev)
    g = torch.Generator(device=dev).manual_seed(2)
    st = torch.randint(0, 2 ** 31, (1, n), device=dev, generator=g, dtype=torch.int32)
    tg = torch.randint(0, 14, (n,), device=dev, generator=g).to(torch.uint8)
    act = torch.randint(0, 29, (n, 3), device=dev, generator=g, dtype=torch.int32)
    rew = torch.randn(n, device=dev, generator=g)
    flags = torch.randint(0, 64, (n,), device=dev, generator=g).to(torch.uint8)
    out = torch.full((n,), 7, dtype=torch.uint8, device=dev)
    pos_t = torch.tensor([100], dtype=torch.int64, device=dev)
    size_t = torch.tensor([0], dtype=torch.int64, device=dev)
    a.store_at(pos_t, size_t, st, tg, act, rew, st, flags, done_mask=3, done_out=out, advance=False)
    torch.cuda.synchronize()
    want = ((flags & 3) != 0).to(torch.uint8)
    slots = (torch.arange(n, device=dev) + 100) % 128
    assert torch.equal(a.done[slots], want) and torch.equal(out, want)
    assert int(pos_t) == 100 and int(size_t) == 0


def test_replay_store_in_pass_copies():
    """store_at's state_copy / target_copy: the ring gets the values read before the same pass
    overwrites them in place (the captured learner's copy-back of the stepped state)."""
    dev = torch.device("cuda")
    n = 64
    a = DeviceReplay(64, 2, 3, dev)
    g = torch.Generator(device=dev).manual_seed(4)
    st = torch.randint(0, 2 ** 31, (2, n), device=dev, generator=g, dtype=torch.int32)
    nxt = torch.randint(0, 2 ** 31, (2, n), device=dev, generator=g, dtype=torch.int32)
    tg = torch.randint(0, 14, (n,), device=dev, generator=g).to(torch.uint8)
    tg_new = torch.randint(0, 14, (n,), device=dev, generator=g).to(torch.uint8)
    st0, tg0 = st.clone(), tg.clone()
    act = torch.zeros(n, 3, dtype=torch.int32, device=dev)
    rew = torch.zeros(n, device=dev)
    done = torch.zeros(n, dtype=torch.uint8, device=dev)
    pos_t = torch.tensor([0], dtype=torch.int64, device=dev)
    size_t = torch.tensor([0], dtype=torch.int64, device=dev)
    a.store_at(pos_t, size_t, st, tg, act, rew, nxt, done, state_copy=(st, nxt), target_copy=(tg, tg_new))
    torch.cuda.synchronize()
    assert torch.equal(a.state, st0) and torch.equal(a.target, tg0) and torch.equal(a.next_state, nxt)
    assert torch.equal(st, nxt) and torch.equal(tg, tg_new)
    assert int(pos_t) == 0 and int(size_t) == 64


@pytest.mark.parametrize("net,n,pos,cap,done_mask", [("pbn28", 4096, 3000, 5000, 3), ("pbn28", 70, 60, 100, 0),
                                                      ("pbn70", 1024, 0, 1024, 3), ("pbn7", 33, 31, 70, 1)])
def test_step_dev_store_equals_step_then_ring_store(net, n, pos, cap, done_mask):
    """pbn_step_dev_store (the step writing its own transitions into the ring) against
    pbn_step_dev + pbn_replay_store on the same inputs, bit for bit: the stepped env (state in
    place, target, t, final state, reward, flags), every ring field, done_out, and rows outside the
    frame untouched; ring wrap-around, ragged env counts, one and two state words."""
    from pbn_rl_amd import _lib
    spec = EnvSpec(load_network(net), load_attractors(net), perturbation=0.05, horizon=3)
    K = 3
    dev = torch.device("cuda")
    envs = [VectorPBNEnv(spec, n, seed=9) for _ in range(2)]
    g = torch.Generator(device=dev).manual_seed(n)
    for e in envs:
        e.reset()
    for _ in range(2):   # some mid-episode t and a horizon truncation next step
        for e in envs:
            e.step_flipmask(random_actions=True)
    acts = torch.randint(0, spec.n + 1, (envs[0].n_alloc, K), device=dev, generator=g, dtype=torch.int32)
    flip = torch.zeros_like(envs[0].flipmask)
    for b in range(K):
        a = acts[:, b].long()
        on = a > 0
        bit = torch.where(on, a - 1, torch.zeros_like(a))
        w, sh = bit // 32, bit % 32
        for wi in range(envs[0].words):
            flip[wi] |= torch.where(on & (w == wi), torch.ones_like(a) << sh, torch.zeros_like(a)).to(torch.int32)
    step_t = torch.tensor([envs[0].step_index], dtype=torch.int64, device=dev)
    rings = [DeviceReplay(cap, envs[0].words, K, dev) for _ in range(2)]
    for r in rings:   # canaries: rows outside the frame must stay as they were
        r.state.fill_(-7)
        r.next_state.fill_(-7)
        r.target.fill_(0xEE)
        r.action.fill_(-7)
        r.reward.fill_(-7.0)
        r.done.fill_(0xEE)
    pos_t = torch.tensor([pos], dtype=torch.int64, device=dev)
    size_t = torch.tensor([0], dtype=torch.int64, device=dev)
    outs = [torch.full((envs[0].n_alloc,), 0xAB, dtype=torch.uint8, device=dev) for _ in range(2)]
    # reference: the step, then the ring store (pre-step state and target kept aside)
    a = envs[0]
    a.flipmask.copy_(flip)
    st0, tg0 = a.state.clone(), a.target.clone()
    a.step_flipmask_dev(step_t, copy_back=True)
    rings[0].store_at(pos_t, size_t, st0, tg0, acts, a.reward, a.final_state, a.flags, done_mask=done_mask,
                      done_out=outs[0], advance=False)
    # fused
    b = envs[1]
    b.flipmask.copy_(flip)
    r = rings[1]
    ring = _lib.RingStore(cap, pos_t.data_ptr(), r.state.data_ptr(), r.next_state.data_ptr(), r.target.data_ptr(),
                          r.action.data_ptr(), r.reward.data_ptr(), r.done.data_ptr(), acts.data_ptr(), K, done_mask,
                          outs[1].data_ptr())
    b.step_flipmask_dev_store(step_t, ring)
    torch.cuda.synchronize()
    for name in ("state", "target", "t", "final_state", "reward", "flags"):
        assert torch.equal(getattr(a, name), getattr(b, name)), name
    for name in ("state", "next_state", "target", "action", "reward", "done"):
        assert torch.equal(getattr(rings[0], name), getattr(rings[1], name)), name
    assert torch.equal(outs[0], outs[1])
    assert int((rings[1].done != 0xEE).sum()) == envs[0].n_alloc   # exactly the frame's rows written
    assert int(pos_t) == pos


def test_step_dev_store_refuses_the_settle_law():
    from pbn_rl_amd import _lib
    spec = EnvSpec(load_network("pbn7"), load_attractors("pbn7"), settle=8)
    env = VectorPBNEnv(spec, 64)
    env.reset()
    r = DeviceReplay(64, 1, 1, env.device)
    pos_t = torch.zeros(1, dtype=torch.int64, device=env.device)
    acts = torch.zeros(64, 1, dtype=torch.int32, device=env.device)
    ring = _lib.RingStore(64, pos_t.data_ptr(), r.state.data_ptr(), r.next_state.data_ptr(), r.target.data_ptr(),
                          r.action.data_ptr(), r.reward.data_ptr(), r.done.data_ptr(), acts.data_ptr(), 1, 0, None)
    step_t = torch.zeros(1, dtype=torch.int64, device=env.device)
    with pytest.raises(_lib.PbnError, match="one-update law"):
        env.step_flipmask_dev_store(step_t, ring)
