"""Every BASELINE config at its own size, through the kernel that config runs, against the
oracle (VERDICT r02 "Next" 2).  The reference's counterpart is the env step the learner calls
once per frame (bdq_model/__init__.py:177).

  config 2  Bittner-28 x 65,536, pbn_rollout_pipe: one 100-step launch (bench.py's launch
            length), every output of every step
  config 3  pbn70 x 1,048,576, pbn_rollout_pipe<3,16>: one 20-step launch, four 4,096-env
            windows (start, interior, end) of every output against the oracle run on those envs
            (envs are independent and keyed by global id, so a window is exact)
  config 4  its 1,048,576-env shard at env_offset 3 * 2^20 through the RCCL gather:
            tests/test_gpu_rccl.py::test_rccl_config4_shard_at_size
  config 5  the BatchedBDQ frame at 32,768 envs (262,144 over 8 GPUs): six frames, the heads
            the frame consumed replayed through the oracle chain (dueling + epsilon-greedy +
            flip masks + step), every output bit-exact, under the one-update law and under the
            facade's settle law (cap 64)
"""
import numpy as np
import pytest
import torch

from oracle import agent_oracle, oracle
from pbn_rl_amd.agent import BatchedBDQ, BranchingQNetwork
from pbn_rl_amd.attractors import load_attractors
from pbn_rl_amd.network import load_network
from pbn_rl_amd.spec import EnvSpec
from pbn_rl_amd.vector_env import VectorPBNEnv

from .oracle_env import OracleVectorEnv

pytestmark = pytest.mark.gpu


def u32(x):
    return x.cpu().numpy().view(np.uint32)


def spec_for(name, **kw):
    return EnvSpec(load_network(name), load_attractors(name), **kw)


def test_config2_rollout_100_steps_at_65536():
    spec = spec_for("pbn28", perturbation=0.01, horizon=20)
    n, T, seed = 65536, 100, 0
    env = VectorPBNEnv(spec, n, seed=seed)
    env.reset()
    out = env.rollout(T, random_actions=True, keep_obs=True, keep_final=True)
    torch.cuda.synchronize()
    st, tg, t = oracle.reset(spec, seed, 0, 0, n)
    zero = np.zeros_like(st)
    for k in range(T):
        ref = oracle.step(spec, seed, 1 + k, 0, st, zero, tg, t, 3)
        assert np.array_equal(u32(out["obs"][k]), st), k
        assert np.array_equal(u32(out["flipmask"][k]), ref["flipmask"]), k
        assert np.array_equal(u32(out["final_state"][k]), ref["final_state"]), k
        assert np.array_equal(out["reward"][k].cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), k
        assert np.array_equal(out["flags"][k].cpu().numpy(), ref["flags"]), k
        st, tg, t = ref["state_out"], ref["target"], ref["t"]
    assert np.array_equal(u32(env.state), st)
    assert np.array_equal(env.target.cpu().numpy(), tg) and np.array_equal(env.t.cpu().numpy(), t)


def test_config3_pbn70_rollout_at_1m():
    spec = spec_for("pbn70", perturbation=0.01, horizon=20)
    n, T, seed = 1 << 20, 20, 1
    env = VectorPBNEnv(spec, n, seed=seed)
    env.reset()
    out = env.rollout(T, random_actions=True, keep_obs=True, keep_final=True)
    torch.cuda.synchronize()
    for lo in (0, 333 * 1024, 700 * 1024 + 2048, n - 4096):
        hi = lo + 4096
        want = OracleVectorEnv(spec, lo, 4096, seed=seed).rollout(T)
        for name in ("obs", "flipmask", "final_state", "flags"):
            assert torch.equal(out[name][..., lo:hi].cpu(), want[name]), (name, lo)
        assert np.array_equal(out["reward"][:, lo:hi].cpu().numpy().view(np.uint32),
                              want["reward"].numpy().view(np.uint32)), lo


@pytest.mark.parametrize("eps,settle", [(0.0, 0), (0.1, 0), (0.1, 64)])
def test_config5_bdq_frames_at_32768(eps, settle):
    """settle = 64: the gym facade's default law, the one train_BDQ.py:50 -> bdq_model/__init__.py:
    172-220 runs (pbn_step's one-step launch of the pipelined settle kernel)."""
    spec = spec_for("pbn28", perturbation=0.01, horizon=20, settle=settle)
    n, seed, frames = 32768, 0, 6
    torch.manual_seed(0)
    env = VectorPBNEnv(spec, n, seed=seed)
    agent = BatchedBDQ(env, BranchingQNetwork((28, 28), 29, 3), epsilon=eps)
    env.reset()
    st, tg, t = oracle.reset(spec, seed, 0, 0, n)
    with torch.no_grad():
        for f in range(frames):
            step = env.step_index
            heads = agent.q_heads().clone()              # what the frame's flip-mask kernel consumes
            agent.act_heads(heads, eps)
            state, reward, flags = env.step_flipmask(use_current=True)
            torch.cuda.synchronize()
            q = agent_oracle.heads_q(heads.cpu().numpy())
            flip, acts = agent_oracle.q_to_flipmask(spec, q, seed, step, 0, eps)
            assert np.array_equal(u32(env.flipmask), flip), f
            assert np.array_equal(agent.actions.cpu().numpy(), acts), f
            ref = oracle.step(spec, seed, step, 0, st, flip, tg, t, 1)
            assert np.array_equal(u32(state), ref["state_out"]), f
            assert np.array_equal(flags.cpu().numpy(), ref["flags"]), f
            assert np.array_equal(reward.cpu().numpy().view(np.uint32), ref["reward"].view(np.uint32)), f
            st, tg, t = ref["state_out"], ref["target"], ref["t"]
