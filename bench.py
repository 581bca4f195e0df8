"""Benchmark: batched PBN env-steps/s (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A "step" is one synchronous PBN transition of every env of the batch:
in-kernel random interventions (3 uniform actions per env, the explore policy
of bdq_model/__init__.py:76), perturbation, per-node rule selection +
truth-table update, attractor reward, autoreset.  By default steps run as
``pbn_rollout`` launches of --chunk (100 = five horizons) steps, state kept on chip
between steps, every step's observation, actions, reward and flags written to
HBM (what a learner consumes); ``--mode step`` times one ``pbn_step`` launch per
step instead.  The launches of the timed run are captured in one hipGraph.
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
FP32_MATRIX_TFLOPS = 157.3  # MI355X FP32 MFMA/vector peak (MI355X_MICROARCH.md)
# VALU issue: 256 CUs x 4 SIMD-32 x 2.4 GHz, one wave64 instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles")
VALU_WAVE_INSTS_PER_S = 256 * 4 * 2.4e9 / 2


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default 2000; bdq workload 200)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default 200; bdq workload 20)")
    p.add_argument("--workload", choices=["env", "bdq", "bdq-learn"], default="env",
                   help="env: BASELINE config 2, the env step alone (in-kernel random interventions); "
                        "bdq: config 5, the full BDQ frame per step (BranchingQNetwork forward: bilinear layer "
                        "by pbn_bilinear_targets, the rest in PyTorch -> pbn_q_to_flipmask -> pbn_step); "
                        "bdq-learn: that frame plus "
                        "storing the transitions in the device replay and one update_policy step of "
                        "batch 256 (one hipGraph per frame: step index, epsilon and ring position live on "
                        "the device; --no-graph launches it eagerly)")
    p.add_argument("--epsilon", type=float, default=0.0, help="bdq workload: exploration rate")
    p.add_argument("--mode", choices=["rollout", "step"], default="rollout",
                   help="rollout: pbn_rollout launches of --chunk steps (state kept on chip); "
                        "step: one pbn_step launch per step")
    p.add_argument("--chunk", type=int, default=100,
                   help="steps per pbn_rollout launch (5 horizons; each launch re-reads the tables and "
                        "refills the wave pipeline: 20 steps/launch runs at ~0.85x the rate of 100, "
                        "profiles/r01_sweep_chunk_pbn28_65536.jsonl)")
    p.add_argument("--network", default="pbn28")
    p.add_argument("--envs", type=int, default=None,
                   help="envs per GPU (default 65,536; bdq workload 32,768 = 262,144 over 8 GPUs)")
    p.add_argument("--perturbation", type=float, default=0.01)
    p.add_argument("--prob-bits", type=int, default=16)
    p.add_argument("--horizon", type=int, default=20)
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--no-graph", action="store_true", help="launch eagerly instead of replaying a hipGraph")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--gather", action="store_true",
                   help="also time rollouts followed by the per-rollout RCCL gather of (s, a, s', r, flags) "
                        "records (SURVEY.md 8(e)); reported as value_with_gather, not the headline")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    a = p.parse_args()
    bdq = a.workload in ("bdq", "bdq-learn")
    a.learn_graph = False
    if a.workload == "bdq-learn":
        a.learn_graph = not a.no_graph   # the learner captures its own one-frame graph
        a.no_graph = True
        a.no_cpu_baseline = True   # the CPU baseline restates acting only
    a.steps = a.steps if a.steps is not None else (200 if bdq else 2000)
    a.warmup = a.warmup if a.warmup is not None else (20 if bdq else 200)
    a.envs = a.envs if a.envs is not None else (32768 if bdq else 65536)
    if bdq:
        a.mode = "step"
    return a


def qnet_flops_per_env(n: int, branches: int = 3) -> int:
    """Multiply-add FLOPs of one BranchingQNetwork forward per env (bdq_model/network.py:24-63):
    bilinear N*N*256, trunk 256-128-64-32, value 32-64-1, branches x (32-64-(N+1))."""
    macs = n * n * 256 + 256 * 128 + 128 * 64 + 64 * 32 + 32 * 64 + 64 + branches * (32 * 64 + 64 * (n + 1))
    return 2 * macs


def algorithmic_bytes_per_env(words: int) -> int:
    # read: state 4W, t 1, target 1 ; write: flipmask (in-kernel actions) 4W,
    # state_out 4W, reward 4, flags 1, t 1   (target is rewritten only on reset)
    return 4 * words + 1 + 1 + 4 * words + 4 * words + 4 + 1 + 1


def rollout_bytes_per_env(words: int, steps: int) -> int:
    # per launch: read + write state 4W, t 1, target 1 once; per step write
    # obs 4W, flipmask (in-kernel actions) 4W, reward 4, flags 1
    return 2 * (4 * words + 1 + 1) + steps * (4 * words + 4 * words + 4 + 1)


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


def numpy_baseline(spec, envs: int, seconds: float = 5.0):
    """The batched numpy restatement (oracle/np_oracle.py, vectorised over envs), 1 process."""
    import numpy as np

    from oracle import np_oracle

    npo = np_oracle.NpPBN(spec)
    n = min(envs, 65536)
    st, tg, t = npo.reset(1, 0, 0, n)
    flip = np.zeros_like(st)
    k, t0 = 0, time.perf_counter()
    while True:
        out = npo.step(1, k + 1, 0, st, flip, tg, t, 3)
        st, tg, t = out["state_out"], out["target"], out["t"]
        k += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n * k / el, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/np_oracle.py (numpy, vectorised over envs), {n} {spec.network.name} envs x {k} steps "
                      f"({el:.1f} s)"}


def host_info() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_count": os.cpu_count(), "cpu_model": model}


def cpu_baseline_bdq(spec, qnet, seconds: float):
    """The BDQ frame on the host cores for ~`seconds`: numpy observation, the same Q-network
    on CPU torch, greedy flip masks and the C oracle step, 4096 envs per frame."""
    import copy

    import numpy as np

    from oracle import agent_oracle, oracle

    threads = max(1, min(16, os.cpu_count() or 1))
    torch.set_num_threads(threads)
    q_cpu = copy.deepcopy(qnet).to("cpu").eval()
    n = 4096
    st, tg, t = oracle.reset(spec, 1, 0, 0, n)
    frames, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            obs = agent_oracle.obs_unpack(spec, st, tg)
            q = q_cpu(torch.from_numpy(obs)).numpy()
            flip, _ = agent_oracle.q_to_flipmask(spec, q, 1, frames + 1, 0, 0.0)
            out = oracle.step(spec, 1, frames + 1, 0, st, flip, tg, t, 1, want_final=False, n_threads=threads)
            st, tg, t = out["state_out"], out["target"], out["t"]
            frames += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return {"value": n * frames / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"BDQ frame on CPU: numpy obs + torch CPU BranchingQNetwork ({threads} threads) + greedy "
                      f"flip masks + oracle/pbn_oracle.c step, {n} envs x {frames} frames ({el:.1f} s)"}


def workload_text(args, chunk: int, rollout_mode: bool) -> str:
    common = (f"horizon {args.horizon}, p={args.perturbation}, prob_bits={args.prob_bits}")
    if args.workload == "bdq":
        return (f"full BDQ rollout (config 5): {args.network} x {args.envs} envs per GPU, per step the "
                f"BranchingQNetwork fp32 forward (random init, seed 0; bilinear layer by pbn_bilinear_targets from "
                f"the packed state) -> epsilon-greedy (eps={args.epsilon}) pbn_q_to_flipmask -> pbn_step, "
                f"autoreset, {common}")
    if args.workload == "bdq-learn":
        return (f"BDQ training frames: {args.network} x {args.envs} envs per GPU, per step the config-5 frame "
                f"(eps={args.epsilon}), the envs' transitions into the device replay, one update_policy step "
                f"(batch 256, Adam, double-DQN target), "
                f"{'one captured hipGraph per frame' if args.learn_graph else 'eager launches'}, {common}")
    return (f"{args.network} x {args.envs} envs per GPU, in-kernel random interventions (3 uniform actions/env/step), "
            f"autoreset, {common}; "
            + (f"pbn_rollout, {chunk} steps/launch, per-step obs/actions/rewards/flags written to HBM"
               if rollout_mode else "pbn_step per step"))


def gather_pass(env, args, world, dev, stream):
    """Env-steps/s (all ranks) when every rollout of --chunk steps is followed by packing its
    (obs, actions, s', reward, flags) records and one all_gather_into_tensor of them
    (pbn_rl_amd.distributed record layout), eager launches."""
    from pbn_rl_amd.distributed import record_rows

    W, n, T = env.words, env.num_envs, args.chunk
    rec = torch.empty((T, record_rows(W), n), dtype=torch.int32, device=dev)
    flat = torch.empty((world * T, record_rows(W), n), dtype=torch.int32, device=dev)
    buf = None
    rounds = max(1, args.steps // T)
    with torch.cuda.stream(stream):
        def one():
            nonlocal buf
            buf = env.rollout(T, random_actions=True, keep_obs=True, keep_final=True, out=buf)
            rec[:, 0:W] = buf["obs"][:, :, :n]
            rec[:, W:2 * W] = buf["flipmask"][:, :, :n]
            rec[:, 2 * W:3 * W] = buf["final_state"][:, :, :n]
            rec[:, 3 * W] = buf["reward"][:, :n].view(torch.int32)
            rec[:, 3 * W + 1] = buf["flags"][:, :n].to(torch.int32)
            if world > 1:
                torch.distributed.all_gather_into_tensor(flat, rec)
        one()
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(rounds):
            one()
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    return world * n * T * rounds / float(el.item())


def launch_plan(steps: int, chunk: int):
    """Rollout launch lengths covering `steps` steps: full chunks, then the remainder."""
    full, rem = divmod(steps, chunk)
    return [chunk] * full + ([rem] if rem else [])


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one GPU per rank over RCCL; more ranks than GPUs (a rehearsal on a smaller box) share
    # them round-robin and synchronise over gloo (RCCL refuses two ranks on one GPU)
    n_dev = max(1, torch.cuda.device_count())
    shared = world > n_dev
    local = local % n_dev
    if world > 1:
        torch.cuda.set_device(local)
        if shared:
            torch.distributed.init_process_group("gloo")
        else:
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
                       keep_final_state=args.workload == "bdq-learn")
    env.reset()
    agent = None
    if args.workload == "bdq":
        from pbn_rl_amd.agent import BatchedBDQ, BranchingQNetwork

        torch.manual_seed(0)   # random-init weights of the reference architecture
        agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3), epsilon=args.epsilon)
    elif args.workload == "bdq-learn":
        from pbn_rl_amd.agent import BranchingQNetwork
        from pbn_rl_amd.replay import BDQLearner

        torch.manual_seed(0)
        learner = BDQLearner(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3), capacity=4 * args.envs,
                             learning_starts=256, epsilon_start=args.epsilon, epsilon_final=args.epsilon,
                             graphable=args.learn_graph)
        agent = learner.agent
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)

    rollout_mode = args.mode == "rollout"
    chunk = args.chunk if rollout_mode else 1
    bufs = {}   # rollout outputs per launch length; captured graphs write into them, so they live
                # as long as the graphs (torch.cuda.graph empties the allocator cache on entry)

    def launch(k: int):
        """One kernel launch covering k steps of every env."""
        if rollout_mode:
            bufs[k] = env.rollout(k, random_actions=True, keep_obs=True, keep_final=False, out=bufs.get(k))
        elif args.workload == "bdq-learn":
            learner.frame()
        elif agent is not None:
            agent.step()
        else:
            env.step_flipmask(random_actions=True)

    plan = launch_plan(args.steps, chunk)
    use_graph = not args.no_graph
    with torch.cuda.stream(stream):
        for k in launch_plan(args.warmup, chunk):
            launch(k)
        if args.learn_graph:
            learner.capture()   # frame() replays the captured frame from here on
        torch.cuda.synchronize(dev)
        graph = None
        if use_graph:
            # step_index (the RNG time coordinate) advances on the host, so the graph holds
            # the whole timed run as distinct launches
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                for k in plan:
                    launch(k)
            torch.cuda.synchronize(dev)
            graph.replay()  # warm the graph path
            torch.cuda.synchronize(dev)

        if world > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        if use_graph:
            graph.replay()
        else:
            for k in plan:
                launch(k)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
    # average launch duration of the step kernel, from HIP events on its own stream over
    # the timed region (launches are back to back inside the graph)
    launch_ms = ev0.elapsed_time(ev1) / len(plan)

    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    total_env_steps = world * args.envs * args.steps
    value = total_env_steps / elapsed

    with_gather = None
    if args.gather:
        with_gather = gather_pass(env, args, world, dev, stream)

    if rank == 0:
        W = spec.words
        if agent is not None:
            bytes_launch = None
            kernel = ("BDQ frame (pbn_bilinear_targets, BranchingQNetwork fp32 layers after the bilinear, "
                      "pbn_q_to_flipmask, pbn_step)")
            if args.workload == "bdq-learn":
                kernel += " + replay store + update_policy (batch 256)"
                kernel += ", one hipGraph replay per frame" if args.learn_graph else ", eager"
        elif rollout_mode:
            bytes_launch = env.n_alloc * rollout_bytes_per_env(W, chunk)
            kernel = "pbn_rollout_pipe (rollout, %d steps/launch)" % chunk
        else:
            bytes_launch = env.n_alloc * algorithmic_bytes_per_env(W)
            kernel = "pbn_step_wave (single step)"
        # the timed plan's launches are full chunks except possibly the last
        full_launch_ms = launch_ms * len(plan) * chunk / args.steps if rollout_mode else launch_ms
        traffic = None
        if agent is not None:
            # the frame is the Q-network: price the reference forward's FLOPs against the
            # FP32 matrix peak (MI355X_MICROARCH.md: 157.3 TFLOP/s), as model-FLOPs utilisation
            flops = env.n_alloc * qnet_flops_per_env(spec.n)
            achieved = flops / (full_launch_ms * 1e-3) / 1e12
            roofline = {"bound": "mfma", "achieved": achieved, "peak": FP32_MATRIX_TFLOPS, "unit": "TFLOP/s",
                        "frac": achieved / FP32_MATRIX_TFLOPS, "traffic": None, "kernel": kernel,
                        "launch_ms": full_launch_ms, "flops_per_launch": flops,
                        "note": "one launch = one whole BDQ frame (~20 kernels); achieved = the reference "
                                "forward's FLOPs (bilinear counted as N*N*256 MACs per env) / frame time, i.e. "
                                "model-FLOPs utilisation. The bilinear layer itself runs as per-target table "
                                "reads (pbn_bilinear_targets), so the executed FLOPs are ~4x lower"}
        else:
            achieved = bytes_launch / (full_launch_ms * 1e-3) / 1e9
            pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.network}_{args.envs}_{args.mode}.json")
            valu_launch = None
            if os.path.exists(pmc_path):
                with open(pmc_path) as f:
                    pmc = json.load(f)
                traffic = pmc.get("hbm_bytes_per_launch")
                valu_launch = pmc.get("valu_insts_per_launch")
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                        "kernel": kernel, "launch_ms": full_launch_ms,
                        "bytes_per_launch": bytes_launch,
                        "note": "VALU-bound (Philox volume), see DESIGN.md 'What bounds it'"}
            if valu_launch:
                # the compute side of the same kernel: wave-level VALU instructions per launch
                # (rocprofv3 SQ_INSTS_VALU, profiles/) over this run's launch time, against the
                # issue rate of one wave64 instruction per 2 cycles per SIMD
                achieved_valu = valu_launch / (full_launch_ms * 1e-3)
                roofline["valu"] = {"achieved": achieved_valu, "peak": VALU_WAVE_INSTS_PER_S,
                                    "unit": "wave-instructions/s", "frac": achieved_valu / VALU_WAVE_INSTS_PER_S,
                                    "insts_per_launch": valu_launch,
                                    "note": "issue slots only: a v_mad_u64_u32 (20 per Philox call) holds its "
                                            "SIMD longer than one slot"}
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
            "dtype": "f32+u32" if agent is not None else "u32",
            "data": "synthetic",
            "config": {"workload": workload_text(args, chunk, rollout_mode),
                       "network": args.network, "envs_per_gpu": args.envs, "global_envs": world * args.envs,
                       "parallelism": f"env-shard x{world}", "launch": "hipGraph" if (use_graph or args.learn_graph) else "eager"},
            "roofline": roofline,
        }
        if with_gather is not None:
            out["value_with_gather"] = with_gather
        if world == 1 and not args.no_cpu_baseline:
            if agent is not None:
                out["cpu_baseline"] = cpu_baseline_bdq(spec, agent.q, args.cpu_seconds)
            else:
                out["cpu_baseline"] = cpu_baseline(spec, args.envs, args.cpu_seconds)
                out["cpu_baseline_python"] = python_baseline(spec)
                out["cpu_baseline_numpy"] = numpy_baseline(spec, args.envs)
            out["host"] = host_info()
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
