"""Kernel sweep: time pbn_step ("wave") and pbn_rollout variants (PBN_ROLL) per batch size.

    python tools/sweep.py [--network pbn28] [--envs 65536,1048576] [--kernels wave,rollp,rolll]

Interleaves variants in one process (cdna_hip_programming.md rule 24) and
reports median per-step kernel time from HIP events around graph replays.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from pbn_rl_amd.attractors import load_attractors  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402
from pbn_rl_amd.spec import EnvSpec  # noqa: E402
from pbn_rl_amd.vector_env import VectorPBNEnv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--envs", default="65536,1048576")
    ap.add_argument("--kernels", default="wave,rollp")
    ap.add_argument("--chunk", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--prob-bits", type=int, default=16)
    args = ap.parse_args()
    spec = EnvSpec(load_network(args.network), load_attractors(args.network), prob_bits=args.prob_bits)
    results = []
    stream = torch.cuda.Stream()
    for n in [int(x) for x in args.envs.split(",")]:
        envs = {}
        graphs = {}
        bufs = {}   # a captured graph writes into these: they must outlive it (torch.cuda.graph
                    # empties the allocator cache on entry, unmapping freed >= 20 MB segments)
        for T in args.kernels.split(","):
            os.environ["PBN_ROLL"] = {"rolll": "lean", "rollp": "pipe"}.get(T, "auto")
            env = VectorPBNEnv(spec, n, seed=3, keep_final_state=False)
            env.reset()
            with torch.cuda.stream(stream):
                if T.startswith("roll"):   # one pbn_rollout launch of `chunk` steps
                    bufs[T] = env.rollout(args.chunk)
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=stream):
                        env.rollout(args.chunk, out=bufs[T])
                    envs[T], graphs[T] = env, g
                    continue
                for _ in range(5):
                    env.step_flipmask(random_actions=True)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for _ in range(args.chunk):
                        env.step_flipmask(random_actions=True)
            envs[T], graphs[T] = env, g
        os.environ.pop("PBN_ROLL", None)
        times = {T: [] for T in envs}
        for _ in range(args.rounds):
            for T, g in graphs.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                with torch.cuda.stream(stream):
                    s.record(stream)
                    g.replay()
                    e.record(stream)
                torch.cuda.synchronize()
                times[T].append(s.elapsed_time(e) / args.chunk)
        for T, ts in times.items():
            med = statistics.median(ts)
            rec = {"network": args.network, "envs": n, "kernel": T, "ms_per_step": med,
                   "env_steps_per_s": n / (med * 1e-3), "min_ms": min(ts)}
            results.append(rec)
            print(json.dumps(rec), flush=True)
        for env in envs.values():
            env.close()


if __name__ == "__main__":
    main()
