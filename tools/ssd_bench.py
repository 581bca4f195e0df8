"""Time compute_ssd_hist at the reference's evaluation settings.

    python tools/ssd_bench.py [--network pbn28] [--resets 300] [--iters 100000]

The reference calls compute_ssd_hist(env, model, resets=300, iters=100_000) after every
training run (train_pbn_28.py:257).  Prints one JSON line:
  gpu_chain_s   chains + histogram on the GPU (HIP events around the rollout/histogram loop)
  total_s       the whole call, including the 2^N-bin copy to the host and the normalisation
  cpu_*         the same env-steps priced at the CPU restatements' measured rates (bounded
                samples: the C oracle on host threads over the same number of chains, and
                the per-env pure-Python step), not run to completion
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from pbn_rl_amd.attractors import load_attractors  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402
from pbn_rl_amd.spec import EnvSpec  # noqa: E402
from pbn_rl_amd.ssd import compute_ssd_hist, state_histogram  # noqa: E402
from pbn_rl_amd.vector_env import VectorPBNEnv  # noqa: E402


def gpu_chain_time(spec, resets, iters, chunk=200):
    """The no-policy loop of compute_ssd_hist, timed with HIP events on the current stream."""
    venv = VectorPBNEnv(spec, resets, seed=0, autoreset=False, keep_final_state=True)
    venv.reset()
    hist = torch.zeros(1 << spec.n, dtype=torch.int32, device=venv.device)
    n = venv.n_alloc
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    left, buf = iters, None
    while left > 0:
        k = min(chunk, left)
        buf = venv.rollout(k, random_actions=False, keep_final=True,
                           out=buf if buf is not None and buf["_n_steps"] == k else None)
        state_histogram(buf["final_state"].view(k, n), resets, spec.n, hist)
        left -= k
    b.record()
    torch.cuda.synchronize()
    total = int(hist.sum().item())
    venv.close()
    return a.elapsed_time(b) / 1e3, total


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--resets", type=int, default=300)
    ap.add_argument("--iters", type=int, default=100_000)
    ap.add_argument("--perturbation", type=float, default=0.01)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    args = ap.parse_args()
    spec = EnvSpec(load_network(args.network), load_attractors(args.network), perturbation=args.perturbation)
    steps = args.resets * args.iters

    gpu_chain_time(spec, args.resets, 1000)                      # warm-up (allocator, code objects)
    chain_s, counted = gpu_chain_time(spec, args.resets, args.iters)
    assert counted == steps, (counted, steps)
    t0 = time.perf_counter()
    ssd, _ = compute_ssd_hist(spec, None, resets=args.resets, iters=args.iters)
    total_s = time.perf_counter() - t0
    assert abs(float(ssd.sum()) - 1.0) < 1e-9

    from oracle import oracle, pyoracle
    threads = max(1, min(16, os.cpu_count() or 1))
    st, tg, t = oracle.reset(spec, 1, 0, 0, 320)
    zero = np.zeros_like(st)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_seconds:
        out = oracle.step(spec, 1, k + 1, 0, st, zero, tg, t, 0, want_final=False, n_threads=threads)
        st, tg, t = out["state_out"], out["target"], out["t"]
        k += 1
    c_rate = 320 * k / (time.perf_counter() - t0)
    py = pyoracle.PyPBN(spec)
    s, g, tt = py.reset(1, 0, 0)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        r = py.step(1, k + 1, 0, s, [0] * spec.n, g, tt, 0)
        s, tt = r["final_state"], r["t"]
        k += 1
    py_rate = k / (time.perf_counter() - t0)
    print(json.dumps({
        "what": f"compute_ssd_hist({args.network}, model=None, resets={args.resets}, iters={args.iters}), "
                f"p={args.perturbation}, 2^{spec.n} 32-bit bins in HBM",
        "env_steps": steps, "gpu_chain_s": chain_s, "gpu_env_steps_per_s": steps / chain_s,
        "total_s": total_s,
        "total_note": "includes the 2^N-bin device-to-host copy and float64 normalisation on the host",
        "cpu_c_oracle_env_steps_per_s": c_rate, "cpu_c_oracle_threads": threads,
        "cpu_c_oracle_est_s": steps / c_rate,
        "cpu_python_env_steps_per_s": py_rate, "cpu_python_est_s": steps / py_rate,
        "host": {"cpu_count": os.cpu_count()}}), flush=True)


if __name__ == "__main__":
    main()
