"""Config 5 agent edges on the GPU, through the C-ABI: pbn_obs_unpack and pbn_q_to_flipmask
are bit-exact against oracle/agent_oracle.py, and the batched BDQ frame loop
(BatchedBDQ: unpack -> Q-network -> epsilon-greedy flip masks -> pbn_step) is bit-exact
against the oracle chain fed with the same Q values."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import agent_oracle, oracle
from pbn_rl_amd import _lib
from pbn_rl_amd.agent import BatchedBDQ, BranchingQNetwork
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

pytestmark = pytest.mark.gpu


def make_spec(name, **kw):
    return EnvSpec(load_network(name), load_attractors(name), **kw)


def u32(x):
    return x.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("name,n", [("pbn7", 96), ("pbn28", 4096), ("pbn70", 2080)])
def test_obs_unpack_exact(name, n):
    spec = make_spec(name)
    env = VectorPBNEnv(spec, n, seed=5)
    rng = np.random.default_rng(1)
    W = spec.words
    st = rng.integers(0, 2 ** 32, size=(W, n), dtype=np.uint64).astype(np.uint32)
    if spec.n % 32:
        st[W - 1] &= np.uint32((1 << (spec.n % 32)) - 1)
    tg = rng.integers(0, len(spec.attractors), size=n).astype(np.uint8)
    tg[::7] = 0xFF
    env.set_state(torch.from_numpy(st.view(np.int32)).cuda(), torch.from_numpy(tg).cuda())
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3))
    obs = agent.observe()
    torch.cuda.synchronize()
    assert np.array_equal(obs.cpu().numpy(), agent_oracle.obs_unpack(spec, st, tg))


@pytest.mark.parametrize("name,K,eps", [("pbn28", 3, 0.0), ("pbn28", 3, 0.3), ("pbn28", 3, 1.0),
                                        ("pbn70", 3, 0.25), ("pbn7", 1, 0.5), ("pbn7", 5, 0.1), ("pbn7", 7, 1.0)])
def test_q_to_flipmask_exact(name, K, eps):
    spec = make_spec(name)
    n = 4160
    env = VectorPBNEnv(spec, n, seed=77, env_offset=320)
    env.step_index = 9
    rng = np.random.default_rng(K)
    q = rng.integers(-3, 4, size=(n, K, spec.n + 1)).astype(np.float32)   # many ties
    q[::13, 0, 2] = np.nan
    q[::17, -1, :] = np.nan
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, K), branches=K)
    fm = agent.act(torch.from_numpy(q).cuda(), eps)
    torch.cuda.synchronize()
    flip, act = agent_oracle.q_to_flipmask(spec, q, 77, 9, 320, eps)
    assert np.array_equal(agent.actions.cpu().numpy(), act)
    assert np.array_equal(u32(fm), flip)
    if eps == 0.0:
        assert np.array_equal(act, torch.argmax(torch.from_numpy(q), dim=2).numpy())


def test_q_to_flipmask_rejects_bad_arguments():
    spec = make_spec("pbn28")
    env = VectorPBNEnv(spec, 64)
    L = _lib.load()
    q = torch.zeros(64, 3, 29, device="cuda")
    fm = torch.zeros(1, 64, dtype=torch.int32, device="cuda")
    h = env.net.handle
    assert L.pbn_q_to_flipmask(h, 0, 0, 0, 64, 3, 28, q.data_ptr(), 0.0, fm.data_ptr(), None, None) == -22
    assert L.pbn_q_to_flipmask(h, 0, 0, 0, 64, 10, 29, q.data_ptr(), 0.0, fm.data_ptr(), None, None) == -22
    assert L.pbn_q_to_flipmask(h, 0, 0, 0, 64, 3, 29, q.data_ptr(), ctypes.c_float(1.5), fm.data_ptr(), None,
                               None) == -22
    assert L.pbn_q_to_flipmask(h, 0, 0, 0, 40, 3, 29, q.data_ptr(), 0.0, fm.data_ptr(), None, None) == -22
    assert L.pbn_q_to_flipmask(h, 0, 0, 0, 64, 3, 29, q.data_ptr() + 4, 0.0, fm.data_ptr(), None, None) == -22
    assert L.pbn_obs_unpack(h, 64, None, None, None, None) == -22
    # pbn_heads_to_flipmask: (K+1, n, A) heads, same checks plus device-pointer alignment
    heads = torch.zeros(4, 64, 29, device="cuda")
    st = torch.zeros(8, dtype=torch.int64, device="cuda")
    assert L.pbn_heads_to_flipmask(h, 0, 0, None, 0, 64, 3, 28, heads.data_ptr(), 0.0, None, fm.data_ptr(), None,
                                   None) == -22
    assert L.pbn_heads_to_flipmask(h, 0, 0, st.data_ptr() + 4, 0, 64, 3, 29, heads.data_ptr(), 0.0, None,
                                   fm.data_ptr(), None, None) == -22
    assert L.pbn_heads_to_flipmask(h, 0, 0, None, 0, 64, 3, 29, heads.data_ptr(), 0.0, None, fm.data_ptr(), None,
                                   None) == 0
    # pbn_bilinear_targets: out_dim a multiple of 4 in 4..1024, aligned buffers, non-null
    y = torch.zeros(64, 256, device="cuda")
    b = torch.zeros(256, device="cuda")
    T = torch.zeros(14, 28, 256, device="cuda")
    args = (h, 64, env.state.data_ptr(), env.target.data_ptr(), T.data_ptr(), b.data_ptr())
    assert L.pbn_bilinear_targets(*args, 254, 0, 0.0, y.data_ptr(), None) == -22
    assert L.pbn_bilinear_targets(*args, 2048, 0, 0.0, y.data_ptr(), None) == -22
    assert L.pbn_bilinear_targets(*args, 256, 0, 0.0, y.data_ptr() + 4, None) == -22
    assert L.pbn_bilinear_targets(h, 64, None, env.target.data_ptr(), T.data_ptr(), b.data_ptr(), 256, 0, 0.0,
                                  y.data_ptr(), None) == -22
    assert L.pbn_bilinear_targets(h, 40, *args[2:], 256, 0, 0.0, y.data_ptr(), None) == -22
    assert L.pbn_bilinear_targets(*args, 256, 1, 0.01, y.data_ptr(), None) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("eps", [0.0, 0.2])
def test_bdq_frame_loop_matches_oracle_chain(eps):
    spec = make_spec("pbn28")
    n, seed, frames = 2048, 31, 12
    torch.manual_seed(0)
    env = VectorPBNEnv(spec, n, seed=seed)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3), epsilon=eps)
    env.reset()
    st, tg, t = oracle.reset(spec, seed, 0, 0, n)
    for k in range(frames):
        step = env.step_index
        obs = agent.observe()
        with torch.no_grad():
            q = agent.q(obs)
        agent.act(q)
        state, reward, flags = env.step_flipmask(use_current=True)
        torch.cuda.synchronize()
        assert np.array_equal(obs.cpu().numpy(), agent_oracle.obs_unpack(spec, st, tg)), f"obs frame {k}"
        flip, _ = agent_oracle.q_to_flipmask(spec, q.cpu().numpy(), seed, step, 0, eps)
        ref = oracle.step(spec, seed, step, 0, st, flip, tg, t, 1)
        assert np.array_equal(u32(env.flipmask), flip), f"flipmask frame {k}"
        assert np.array_equal(u32(state), ref["state_out"]), f"state frame {k}"
        assert np.array_equal(reward.cpu().numpy(), ref["reward"])
        assert np.array_equal(flags.cpu().numpy(), ref["flags"])
        st, tg, t = ref["state_out"], ref["target"], ref["t"]


def test_bdq_step_graph_capture():
    """The whole frame (unpack, Q-network, flip masks, step) replays from one hipGraph."""
    spec = make_spec("pbn28")
    env = VectorPBNEnv(spec, 1024, seed=3, keep_final_state=False)
    torch.manual_seed(0)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    env.reset()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        agent.step()
        torch.cuda.synchronize()
        ref_env = VectorPBNEnv(spec, 1024, seed=3, keep_final_state=False)
        ref_env.set_state(env.state.clone(), env.target.clone(), env.t.clone())
        ref_env.step_index = env.step_index
        ref_agent = BatchedBDQ(ref_env, agent.q)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            agent.step()
        g.replay()
        ref_agent.step()
        torch.cuda.synchronize()
    assert torch.equal(env.state, ref_env.state)


@pytest.mark.parametrize("name", ["pbn28", "pbn70", "pbn7"])
def test_bilinear_targets_matches_module(name):
    """pbn_bilinear_targets (from the packed state and a per-target table) against the
    PyTorch fp32 MyBilinear on the unpacked observation; Q of the fast path against the module.
    Tolerance: fp32, different summation order (<= 28 or 70 added rows of |w| < 1)."""
    spec = make_spec(name, perturbation=0.05)
    torch.manual_seed(5)
    env = VectorPBNEnv(spec, 4096, seed=2)
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3))
    env.reset()
    for _ in range(3):
        env.step_flipmask(random_actions=True)
    with torch.no_grad():
        q_fast = agent.q_values().clone()
        agent.bilinear()                    # pbn_bilinear_targets into agent._y
        y_fast = agent._y.clone()
        assert agent._act                   # the kernel applied the LeakyReLU
        obs = agent.observe()
        y_ref = agent.q.model[1](agent.q.model[0](obs))       # bilinear + LeakyReLU
        q_ref = agent.q(obs)
    torch.cuda.synchronize()
    assert torch.allclose(y_fast, y_ref, rtol=1e-5, atol=1e-5), (y_fast - y_ref).abs().max()
    assert torch.allclose(q_fast, q_ref, rtol=1e-4, atol=1e-5), (q_fast - q_ref).abs().max()


def test_bilinear_targets_without_attractors_is_bias():
    spec = EnvSpec(load_network("pbn28"), [], perturbation=0.01)
    env = VectorPBNEnv(spec, 256, seed=1)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    env.reset()
    with torch.no_grad():
        agent.q_values()
        agent.bilinear()
        obs = agent.observe()
        y_ref = agent.q.model[1](agent.q.model[0](obs))
        act_bias = agent.q.model[1](agent.q.model[0].bilinear.bias)
    torch.cuda.synchronize()
    assert torch.equal(agent._y, act_bias.expand_as(agent._y)) and torch.allclose(y_ref, agent._y, atol=1e-6)


@pytest.mark.parametrize("name,K,eps", [("pbn28", 3, 0.0), ("pbn28", 3, 0.3), ("pbn70", 3, 0.25),
                                        ("pbn7", 1, 0.5), ("pbn7", 5, 0.0), ("pbn28", 3, 1.0)])
def test_heads_to_flipmask_exact(name, K, eps):
    """pbn_heads_to_flipmask (dueling combination in the kernel) against the oracle's
    restatement of its arithmetic, bit for bit; and its Q against torch's dueling to fp32."""
    spec = make_spec(name)
    n, A, seed, step = 2080 if name == "pbn70" else 4096, spec.n + 1, 9, 17
    env = VectorPBNEnv(spec, n, seed=seed)
    env.step_index = step
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), A, K), branches=K)
    g = torch.Generator(device="cuda").manual_seed(3)
    heads = torch.randn(K + 1, env.n_alloc, A, device="cuda", generator=g)
    heads[1:, :64, 5] = heads[1:, :64, 2]                    # ties: the first maximum wins
    agent.act_heads(heads, eps)
    torch.cuda.synchronize()
    h = heads.cpu().numpy()
    q = agent_oracle.heads_q(h)
    flip, acts = agent_oracle.q_to_flipmask(spec, q, seed, step, 0, eps)
    assert np.array_equal(u32(env.flipmask), flip)
    assert np.array_equal(agent.actions.cpu().numpy(), acts)
    q_torch = BranchingQNetwork.dueling(heads).cpu().numpy()
    assert np.allclose(q, q_torch, rtol=1e-5, atol=1e-5)
    # device step / epsilon forms
    fm = env.flipmask.clone()
    step_t = torch.full((1,), step, dtype=torch.int64, device="cuda")
    eps_t = torch.full((1,), eps, dtype=torch.float32, device="cuda")
    env.flipmask.zero_()
    agent.act_heads(heads, 0.77, step_t=step_t, epsilon_t=eps_t)
    assert torch.equal(env.flipmask, fm)


def test_bdq_step_uses_fused_heads():
    """BatchedBDQ.step (bilinear kernel + heads kernel) picks the flip masks the module's Q
    gives through pbn_q_to_flipmask, except where fp32 summation order splits a near-tie."""
    spec = make_spec("pbn28")
    torch.manual_seed(7)
    env = VectorPBNEnv(spec, 8192, seed=4)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    env.reset()
    with torch.no_grad():
        q = agent.q(agent.observe())
        agent.act(q, 0.0)
        ref = env.flipmask.clone()
        agent.act_heads(agent.q_heads(), 0.0)
    torch.cuda.synchronize()
    same = (env.flipmask == ref).float().mean().item()
    assert same > 0.999, same


def test_prepacked_weights_follow_in_place_updates():
    """The eval-mode pack (target table, head weights) is rebuilt when a parameter changes."""
    spec = make_spec("pbn28")
    torch.manual_seed(8)
    env = VectorPBNEnv(spec, 1024, seed=6)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    env.reset()
    with torch.no_grad():
        agent.q_values()
        key = agent._pack_key
        agent.q.model[0].bilinear.weight.mul_(1.5)
        agent.q.adv_heads[1][2].bias.add_(0.25)
        q_fast = agent.q_values()
        q_ref = agent.q(agent.observe())
    torch.cuda.synchronize()
    assert agent._pack_key != key
    assert torch.allclose(q_fast, q_ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("name,n", [("pbn28", 32768), ("pbn7", 96), ("pbn70", 2080)])
def test_fused_tail_matches_module(name, n):
    """pbn_qnet_heads (the layers after the bilinear one, one MFMA kernel) against the PyTorch
    layers on the same bilinear output: fp32, rtol 1e-5 / atol 1e-5 (summation order differs
    from hipBLASLt's); and the flip masks it leads to equal the PyTorch tail's except where fp32
    summation order splits a near-tie (> 99.9 %)."""
    spec = make_spec(name)
    torch.manual_seed(11)
    env = VectorPBNEnv(spec, n, seed=2)
    qnet = BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3)
    fused = BatchedBDQ(env, qnet)
    plain = BatchedBDQ(env, qnet, fused_tail=False)
    assert fused.fused_tail and not plain.fused_tail
    env.reset()
    with torch.no_grad():
        hf = fused.q_heads().clone()
        hp = plain.q_heads().clone()
        torch.cuda.synchronize()
        assert torch.allclose(hf, hp, rtol=1e-5, atol=1e-5), (hf - hp).abs().max().item()
        fused.act_heads(hf, 0.0)
        fm_f = env.flipmask.clone()
        plain.act_heads(hp, 0.0)
        same = (env.flipmask == fm_f).float().mean().item()
    assert same > 0.999, same


def test_fused_tail_with_reference_checkpoint():
    """The reference's trained pbn7 agent (models/pbn7/bdq_final.pt via tests/golden): fused
    tail == the module's forward on the unpacked observation, within fp32 tolerance."""
    import os
    w = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pbn7_bdq_final.npz"))
    qnet = BranchingQNetwork((7, 7), 8, 3)
    qnet.load_state_dict({k: torch.from_numpy(w[k]) for k in w.files})
    spec = make_spec("pbn7")
    env = VectorPBNEnv(spec, 256, seed=4)
    agent = BatchedBDQ(env, qnet)
    env.reset()
    with torch.no_grad():
        q_fast = agent.q_values()
        q_ref = agent.q(agent.observe())
    torch.cuda.synchronize()
    assert torch.allclose(q_fast, q_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name,n,K,eps", [("pbn28", 32768, 3, 0.0), ("pbn28", 4096, 3, 0.3), ("pbn70", 2080, 3, 0.25),
                                          ("pbn7", 96, 5, 0.0), ("pbn7", 512, 1, 0.5), ("pbn28", 1024, 3, 1.0)])
def test_qnet_flipmask_equals_heads_path(name, n, K, eps):
    """pbn_qnet_flipmask (the tail + dueling + epsilon-greedy in one launch, act_q) against
    pbn_qnet_heads -> pbn_heads_to_flipmask on the same observations: flip masks and actions bit
    for bit, and both against the oracle's restatement of the heads arithmetic; then the device
    step / epsilon forms."""
    spec = make_spec(name)
    A, seed, step = spec.n + 1, 13, 29
    torch.manual_seed(17)
    env = VectorPBNEnv(spec, n, seed=seed)
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), A, K), branches=K)
    assert agent.fused_tail
    env.reset()
    for _ in range(2):
        env.step_flipmask(random_actions=True)
    env.step_index = step
    with torch.no_grad():
        heads = agent.q_heads().clone()
        agent.act_heads(heads, eps)
        fm_ref, act_ref = env.flipmask.clone(), agent.actions.clone()
        env.flipmask.zero_()
        agent.actions.zero_()
        agent.act_q(eps)
    torch.cuda.synchronize()
    assert torch.equal(env.flipmask, fm_ref)
    assert torch.equal(agent.actions, act_ref)
    flip, acts = agent_oracle.q_to_flipmask(spec, agent_oracle.heads_q(heads.cpu().numpy()), seed, step, 0, eps)
    assert np.array_equal(u32(env.flipmask), flip) and np.array_equal(agent.actions.cpu().numpy(), acts)
    step_t = torch.full((1,), step, dtype=torch.int64, device="cuda")
    eps_t = torch.full((1,), eps, dtype=torch.float32, device="cuda")
    env.flipmask.zero_()
    env.step_index = step + 5          # ignored: the device step wins
    agent.act_q(0.77, step_t=step_t, epsilon_t=eps_t)
    torch.cuda.synchronize()
    assert torch.equal(env.flipmask, fm_ref)


def test_qnet_flipmask_rejects_bad_arguments():
    spec = make_spec("pbn28")
    env = VectorPBNEnv(spec, 64, seed=1)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    L = _lib.load()
    m = agent.q.model
    w1, b1, w2, b2 = agent.q.head_weights()
    ts = [agent._y, m[2].weight, m[2].bias, m[4].weight, m[4].bias, m[6].weight, m[6].bias, w1, b1, w2, b2]
    ptrs = [t.data_ptr() for t in ts]
    fm = env.flipmask.data_ptr()
    h = env.net.handle
    ok = (h, 1, 0, None, 0, 64, *ptrs, 3, 29, 0.01, 0.0, None, fm, None, None)
    assert L.pbn_qnet_flipmask(*ok) == 0
    bad = list(ok); bad[17] = 0                      # n_branches
    assert L.pbn_qnet_flipmask(*bad) == -22
    bad = list(ok); bad[18] = 30                     # n_actions != N + 1
    assert L.pbn_qnet_flipmask(*bad) == -22
    bad = list(ok); bad[20] = 1.5                    # epsilon
    assert L.pbn_qnet_flipmask(*bad) == -22
    bad = list(ok); bad[4] = 16                      # env_offset
    assert L.pbn_qnet_flipmask(*bad) == -22
    bad = list(ok); bad[22] = None                   # flipmask
    assert L.pbn_qnet_flipmask(*bad) == -22
    torch.cuda.synchronize()


@pytest.mark.parametrize("name,n", [("pbn28", 32768), ("pbn7", 4096), ("pbn28", 96)])
def test_bilinear_lds_equals_l2_kernel(name, n, monkeypatch):
    """pbn_bilinear_targets' LDS-staged kernel (the default where the table slices fit) against
    its L2 kernel (PBN_BILINEAR=l2): the same sums in the same order, bit for bit; ragged last
    block, envs without a target (bias only) included."""
    spec = make_spec(name)
    torch.manual_seed(21)
    env = VectorPBNEnv(spec, n, seed=3)
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3))
    env.reset()
    for _ in range(2):
        env.step_flipmask(random_actions=True)
    env.target[::7] = 0xFF
    with torch.no_grad():
        agent.bilinear()
        y_lds = agent._y.clone()
        monkeypatch.setenv("PBN_BILINEAR", "l2")
        agent.bilinear()
        y_l2 = agent._y.clone()
    torch.cuda.synchronize()
    assert torch.equal(y_lds, y_l2)


@pytest.mark.parametrize("name,n", [("pbn28", 32768), ("pbn7", 96), ("pbn70", 2080), ("pbn28", 160)])
def test_qnet_from_state_matches_y_path(name, n):
    """pbn_qnet_heads_from_state (the bilinear layer on the MFMAs inside the tail, envs sorted by
    target per block) against pbn_bilinear_targets -> pbn_qnet_heads on the same state: fp32,
    rtol 1e-5 / atol 1e-5 (the bilinear sums are grouped differently); envs without a target and a
    ragged last block included.  Both acting paths then pick the same flip masks except where
    fp32 rounding splits a near-tie (> 99.9 %)."""
    spec = make_spec(name)
    torch.manual_seed(23)
    env = VectorPBNEnv(spec, n, seed=5)
    qnet = BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3)
    agent = BatchedBDQ(env, qnet)
    env.reset()
    for _ in range(2):
        env.step_flipmask(random_actions=True)
    env.target[::11] = 0xFF
    L = _lib.load()
    with torch.no_grad():
        h_state = agent.q_heads().clone()
        hw = agent.bilinear()                      # y through pbn_bilinear_targets
        m = agent.q.model
        ts = [t.detach().contiguous() for t in (m[2].weight, m[2].bias, m[4].weight, m[4].bias, m[6].weight,
                                                m[6].bias, *hw)]
        h_y = torch.empty_like(h_state)
        _lib.check(L.pbn_qnet_heads(env.net.handle, env.n_alloc, agent._y.data_ptr(), *[t.data_ptr() for t in ts],
                                    4, spec.n + 1, agent._slope, h_y.data_ptr(), None), "pbn_qnet_heads")
        torch.cuda.synchronize()
        assert torch.allclose(h_state, h_y, rtol=1e-5, atol=1e-5), (h_state - h_y).abs().max().item()
        agent.act_q(0.0)
        fm_state = env.flipmask.clone()
        agent.act_heads(h_y, 0.0)
        same = (env.flipmask == fm_state).float().mean().item()
    assert same > 0.999, same


def test_qnet_from_state_rejects_bad_arguments():
    spec = make_spec("pbn28")
    env = VectorPBNEnv(spec, 64, seed=1)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3))
    L = _lib.load()
    ptrs, _keep = agent._tail_operands()             # T, b0, trunk, stacked heads
    st, tg, fm = env.state.data_ptr(), env.target.data_ptr(), env.flipmask.data_ptr()
    h = env.net.handle
    ok = [h, 1, 0, None, 0, 64, st, tg, *ptrs, 3, 29, 0.01, 0.0, None, fm, None, None]
    assert L.pbn_qnet_flipmask_from_state(*ok) == 0
    for idx, val in [(8, None),                       # T with attractors
                     (8, ptrs[0] + 4),                # T misaligned (16-byte loads)
                     (9, ptrs[1] + 4),                # b0 misaligned
                     (6, None),                       # state
                     (20, 0),                         # n_branches
                     (21, 30),                        # n_actions != N + 1
                     (5, 40)]:                        # n_envs not a multiple of 32
        bad = list(ok)
        bad[idx] = val
        assert L.pbn_qnet_flipmask_from_state(*bad) == -22, idx
    heads = torch.empty(4, 64, 29, device="cuda")
    okh = [h, 64, st, tg, *ptrs, 4, 29, 0.01, heads.data_ptr(), None]
    assert L.pbn_qnet_heads_from_state(*okh) == 0
    bad = list(okh); bad[3] = None
    assert L.pbn_qnet_heads_from_state(*bad) == -22
    torch.cuda.synchronize()
