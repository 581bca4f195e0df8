"""Benchmark: batched PBN env-steps/s (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A "step" is one synchronous PBN transition of every env of the batch (one
``pbn_step`` launch per GPU): in-kernel random interventions (3 uniform actions
per env, the explore policy of bdq_model/__init__.py:76), perturbation,
per-node rule selection + truth-table update, attractor reward, autoreset.
Default workload = BASELINE config 2: Bittner-28 (kaban/pbn28.ispl + the 14
fixture attractors), 65,536 envs per GPU, horizon 20, p = 0.01.  Multi-GPU is
weak scaling: every rank owns its own env range (env_offset = rank * envs), no
data-path collective; the timed region is bracketed by barrier + synchronize
and the max over ranks is reported.  Inputs are resident in HBM before timing.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--network", default="pbn28")
    p.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    p.add_argument("--perturbation", type=float, default=0.01)
    p.add_argument("--prob-bits", type=int, default=16)
    p.add_argument("--horizon", type=int, default=20)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a hipGraph")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    return p.parse_args()


def algorithmic_bytes_per_env(words: int) -> int:
    # read: state 4W, t 1, target 1 ; write: flipmask (in-kernel actions) 4W,
    # state_out 4W, reward 4, flags 1, t 1   (target is rewritten only on reset)
    return 4 * words + 1 + 1 + 4 * words + 4 * words + 4 + 1 + 1


def cpu_baseline(spec, envs: int, seconds: float):
    """Time the C oracle (port of the step) on the host cores for ~`seconds`."""
    import numpy as np

    from oracle import oracle

    threads = max(1, min(16, os.cpu_count() or 1))
    n = min(envs, 65536)
    st, tg, t = oracle.reset(spec, 1, 0, 0, n)
    flip = np.zeros_like(st)
    done_steps, t0 = 0, time.perf_counter()
    while True:
        out = oracle.step(spec, 1, done_steps + 1, 0, st, flip, tg, t, 3, want_final=False, n_threads=threads)
        st, tg, t = out["state_out"], out["target"], out["t"]
        done_steps += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n * done_steps / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pbn_oracle.c (OpenMP, {threads} threads), {n} {spec.network.name} envs x "
                      f"{done_steps} steps ({el:.1f} s), in-kernel-equivalent random actions, autoreset"}


def python_baseline(spec, seconds: float = 3.0):
    """Reference-style per-env, per-node Python step (gym-PBN style), 1 core."""
    from oracle import pyoracle

    py = pyoracle.PyPBN(spec)
    state, tgt, tt = py.reset(5, 0, 0)
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r = py.step(5, k + 1, 0, state, [0] * spec.n, tgt, tt, 3)
        state, tgt, tt = r["state_out"], r["target"], r["t"]
        k += 1
    el = time.perf_counter() - t0
    return {"value": k / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/pyoracle.py single env, {k} steps"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if world > 1 else 0)
    torch.cuda.set_device(dev)

    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    spec = EnvSpec(load_network(args.network), load_attractors(args.network), perturbation=args.perturbation,
                   prob_bits=args.prob_bits, horizon=args.horizon)
    env = VectorPBNEnv(spec, args.envs, seed=args.seed, device=dev, env_offset=rank * args.envs,
                       keep_final_state=False)
    env.reset()

    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)

    def one_step():
        env.step_flipmask(random_actions=True)

    # step_index advances the RNG time coordinate on the host; a replayed graph
    # would reuse one index, so the graph holds a whole chunk of distinct steps.
    use_graph = not args.no_graph
    chunk = 20
    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            one_step()
        torch.cuda.synchronize(dev)

        # per-launch kernel duration with HIP events on the launch stream
        n_ev = 50
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_ev)]
        for s, e in evs:
            s.record(stream)
            one_step()
            e.record(stream)
        torch.cuda.synchronize(dev)
        kernel_ms = sum(s.elapsed_time(e) for s, e in evs) / n_ev

        graphs = []
        if use_graph:
            n_graphs = (args.steps + chunk - 1) // chunk
            for _ in range(n_graphs):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=stream):
                    for _ in range(chunk):
                        one_step()
                graphs.append(g)
            torch.cuda.synchronize(dev)
            graphs[0].replay()  # warm the graph path
            torch.cuda.synchronize(dev)

        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if use_graph:
            full, rem = divmod(args.steps, chunk)
            for i in range(full):
                graphs[i].replay()
            for _ in range(rem):
                one_step()
        else:
            for _ in range(args.steps):
                one_step()
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    total_env_steps = world * args.envs * args.steps
    value = total_env_steps / elapsed

    if rank == 0:
        bytes_env = algorithmic_bytes_per_env(spec.words)
        achieved = env.n_alloc * bytes_env / (kernel_ms * 1e-3) / 1e9
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.network}_{args.envs}.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        out = {
            "metric": "env steps/sec (batched PBN transitions), Bittner-28 at 1/2/4/8 GPUs"
            if args.network == "pbn28" else f"env steps/sec (batched PBN transitions), {args.network}",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": f"{args.network} x {args.envs} envs per GPU, in-kernel random interventions, "
                                   f"autoreset, horizon {args.horizon}, p={args.perturbation}, "
                                   f"prob_bits={args.prob_bits}",
                       "network": args.network, "envs_per_gpu": args.envs, "global_envs": world * args.envs,
                       "parallelism": f"env-shard x{world}", "launch": "hipGraph" if use_graph else "eager"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "pbn_step_kernel", "kernel_ms": kernel_ms,
                         "bytes_per_env_step": bytes_env},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(spec, args.envs, args.cpu_seconds)
            out["cpu_baseline_python"] = python_baseline(spec)
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
