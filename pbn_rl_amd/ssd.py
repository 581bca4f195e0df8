"""Steady-state distribution (SSD) of a PBN, batched on the GPU.

The reference evaluates every trained agent with ``gym_PBN.utils.eval.compute_ssd_hist(env,
model, resets=300, iters=100_000, multiprocess=True)`` (train_pbn_28.py:257,
train_pbn_10.py:257, train_ddqn.py:156): independent chains of the (optionally controlled)
PBN are run from resets and the visited states are counted.  gym_PBN is not available
(SURVEY.md 8(c)), so the estimator is restated here and its result is parity-unpinned:

* ``resets`` chains, one env each, started by ``pbn_reset`` (a random attractor state);
* no autoreset and no horizon: each chain runs ``burn_in + iters`` steps of the frozen step
  semantics with perturbation; the interventions are the policy's (``model``),
  or none;
* every state s' after step ``burn_in + 1 .. burn_in + iters`` of every chain is counted
  (``pbn_state_histogram`` on the rollout's ``final_state``), and the counts are normalised.

Histogram bins are full states, so networks with at most 32 nodes (2^N bins in HBM: 1 GiB
of 32-bit counters for Bittner-28).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .spec import EnvSpec
from .vector_env import VectorPBNEnv, actions_to_flipmask, unpack_states

__all__ = ["compute_ssd_hist", "state_histogram"]


def state_histogram(states: torch.Tensor, n_cols: int, n_bits: int, hist: torch.Tensor) -> None:
    """hist[states[r, c] & (2^n_bits - 1)] += 1 for every row r and column c < n_cols
    (states: int32 [rows, row_stride] on the GPU, hist: int32 [2^n_bits])."""
    if states.dim() != 2 or not states.is_contiguous():
        raise ValueError("states must be a contiguous [rows, row_stride] tensor")
    L = _lib.load()
    with torch.cuda.device(states.device):
        _lib.check(L.pbn_state_histogram(states.data_ptr(), states.shape[0], n_cols, states.shape[1], n_bits,
                                         hist.data_ptr(), torch.cuda.current_stream(states.device).cuda_stream),
                   "pbn_state_histogram")


def _spec_of(env) -> EnvSpec:
    if isinstance(env, EnvSpec):
        return env
    for obj in (env, getattr(env, "env", None), getattr(getattr(env, "env", None), "env", None)):
        if obj is not None and isinstance(getattr(obj, "spec", None), EnvSpec):
            return obj.spec
    raise TypeError("compute_ssd_hist needs an EnvSpec, a VectorPBNEnv or a PBNEnv")


def compute_ssd_hist(env, model: Optional[Callable] = None, resets: int = 300, iters: int = 100_000,
                     multiprocess: bool = False, *, burn_in: int = 0, seed: int = 0, chunk: int = 200,
                     device=None, graph: bool = True) -> Tuple[np.ndarray, None]:
    """Returns (ssd, plot): ssd[s] = fraction of counted steps spent in state s (float64,
    2^N entries, state s = bit i for node i); plot is None (no plotting backend here).

    ``model``: None (no interventions) or a policy mapping the (resets, N) uint8 state bits on
    the GPU to (resets, k) actions in [0, N] (0 = no-op), called every step.
    ``multiprocess`` is accepted for signature compatibility; chains already run in parallel.
    ``graph``: with a model, capture one policy step (state unpack, model, flip masks,
    pbn_step_dev, histogram) in a hipGraph after a first eager step has validated the
    actions, and replay it; a model that cannot be captured (host syncs) raises, and
    ``graph=False`` runs every step eagerly.  Both give the same histogram.
    """
    spec = _spec_of(env)
    N = spec.n
    if N > 32:
        raise ValueError("the SSD histogram has 2^N bins: networks with at most 32 nodes")
    if resets * iters >= 1 << 32:
        # the histogram's bins are 32-bit counters: a fixed-point attractor could take every count
        raise ValueError(f"resets * iters = {resets * iters} counted steps overflow the 32-bit bins (< 2^32)")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    venv = VectorPBNEnv(spec, resets, seed=seed, device=dev, autoreset=False, keep_final_state=True)
    venv.reset()
    hist = torch.zeros(1 << N, dtype=torch.int32, device=dev)
    n = venv.n_alloc
    with torch.cuda.device(dev):
        if model is None:
            left = burn_in
            buf = None
            while left > 0:
                k = min(chunk, left)
                buf = venv.rollout(k, random_actions=False, keep_final=False)
                left -= k
            left, buf = iters, None
            while left > 0:
                k = min(chunk, left)
                buf = venv.rollout(k, random_actions=False, keep_final=True,
                                   out=buf if buf is not None and buf["_n_steps"] == k else None)
                state_histogram(buf["final_state"].view(k, n), resets, N, hist)
                left -= k
        else:
            step_t = torch.full((1,), venv.step_index, dtype=torch.int64, device=dev)

            def policy_step(count: bool, check: bool) -> None:
                bits = unpack_states(venv.state[:, :resets], N)
                fm = actions_to_flipmask(model(bits).to(dev), N, check=check)
                venv.flipmask[:, :resets].copy_(fm)
                venv.step_flipmask_dev(step_t)
                step_t.add_(1)
                if count:
                    state_histogram(venv.final_state.view(1, n), resets, N, hist)

            venv.flipmask.zero_()      # padding envs (n_alloc > resets) are never intervened on
            total = burn_in + iters
            it = 0
            graphs = {}
            while it < total:
                count = it >= burn_in
                if not graph or it == 0:
                    policy_step(count, check=True)      # eager: the first step validates the actions
                else:
                    g = graphs.get(count)
                    if g is None:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g):
                            policy_step(count, check=False)
                        graphs[count] = g
                    g.replay()
                it += 1
        counts = hist.cpu().numpy().view(np.uint32)
    total = int(counts.sum(dtype=np.uint64))     # the bins are unsigned 32-bit counts
    venv.close()
    # one host pass over the 2^N bins (float64 out), not astype + divide
    ssd = np.empty(counts.shape, dtype=np.float64)
    if total > 0:
        np.divide(counts, total, out=ssd)
    else:
        ssd[:] = 0.0
    return ssd, None
