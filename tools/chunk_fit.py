"""Per-launch fixed cost of pbn_rollout: device time of one launch of T steps for several T,
fitted as fixed + T * per_step (HIP events around single-launch graph replays, each gated
by a spin kernel so that the host's launch latency is not timed).

    python tools/chunk_fit.py [--network pbn28] [--envs 65536] [--steps 1,2,5,10,20,50,100]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pbn_rl_amd.attractors import load_attractors  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402
from pbn_rl_amd.spec import EnvSpec  # noqa: E402
from pbn_rl_amd.vector_env import VectorPBNEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", default="1,2,5,10,20,50,100")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--out", default=None)
    ap.add_argument("--mode", choices=["graph", "eager"], default="graph",
                    help="graph: one-launch hipGraph replays; eager: the launch itself")
    a = ap.parse_args()
    spec = EnvSpec(load_network(a.network), load_attractors(a.network))
    env = VectorPBNEnv(spec, a.envs, seed=3, keep_final_state=False)
    env.reset()
    stream = torch.cuda.Stream()
    Ts = [int(x) for x in a.steps.split(",")]
    graphs, bufs = {}, {}
    with torch.cuda.stream(stream):
        for T in Ts:
            bufs[T] = env.rollout_buffers(T, keep_obs=True, keep_final=False)
            env.rollout(T, keep_obs=True, keep_final=False, out=bufs[T])
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=stream):
                env.rollout(T, keep_obs=True, keep_final=False, out=bufs[T])
            graphs[T] = g
        for _ in range(200):   # clock ramp
            graphs[Ts[-1]].replay()
        torch.cuda.synchronize()
        times = {T: [] for T in Ts}
        for _ in range(a.reps):
            for T in Ts:   # interleaved
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda._sleep(100_000)
                e0.record(stream)
                if a.mode == "graph":
                    graphs[T].replay()
                else:
                    env.rollout(T, keep_obs=True, keep_final=False, out=bufs[T])
                e1.record(stream)
                torch.cuda.synchronize()
                times[T].append(e0.elapsed_time(e1) * 1e3)
    med = {T: statistics.median(v) for T, v in times.items()}
    A = np.array([[1.0, T] for T in Ts])
    fixed, per = np.linalg.lstsq(A, np.array([med[T] for T in Ts]), rcond=None)[0]
    # calibration: the same event pair around a one-element fill (launch + event overhead)
    x = torch.zeros(1, device="cuda")
    cal = []
    with torch.cuda.stream(stream):
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(100_000)
            e0.record(stream)
            x.add_(1.0)
            e1.record(stream)
            torch.cuda.synchronize()
            cal.append(e0.elapsed_time(e1) * 1e3)
    rec = {"network": a.network, "envs": a.envs, "mode": a.mode, "tiny_kernel_us": statistics.median(cal),
           "median_us": med, "fit_fixed_us": fixed, "fit_per_step_us": per,
           "per_step_us_at": {T: med[T] / T for T in Ts}}
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
