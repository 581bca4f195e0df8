"""Benchmark: batched PBN env-steps/s (BASELINE.json metric) on 1..8 MI355X.

    python bench.py [--gpus N --steps K --warmup W]          # N > 1: spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

A "step" is one synchronous PBN transition of every env of the batch:
in-kernel random interventions (3 uniform actions per env, the explore policy
of bdq_model/__init__.py:76), perturbation, per-node rule selection +
truth-table update, attractor reward, autoreset.  Steps run as ``pbn_rollout``
launches of at most --chunk (100 = five horizons) steps, state kept on chip
between steps, every step's observation, actions, reward and flags written to
HBM (what a learner consumes); ``--mode step`` times one ``pbn_step`` launch per
step instead.  The launches of the timed run are captured in one hipGraph.
Default workload = BASELINE config 2: Bittner-28 (kaban/pbn28.ispl + the 14
fixture attractors), 65,536 envs per GPU, horizon 20, p = 0.01.

One process per GPU, RCCL ("nccl") process group over all ranks (world 1 too).
Multi-GPU is weak scaling: every rank owns its own env range (env_offset =
rank * envs).  ``value`` times the steps alone; ``value_with_gather`` times the
same steps with the rollout's (s, a, s', r, flags) records (17 B per env-step for
Bittner-28) handed to the learner (rank 0) after every rollout launch, overlapped
with the next launch (``gather.all_gather`` times the
all-gather form).  Each timed region is bracketed by barrier +
synchronize, timed with HIP events on the launch stream (created without the
system-scope fence: the interval is the device's work; timing.default_events times
the same run between torch's default events), and the max over ranks is reported.  Inputs are resident in HBM before timing.  Before the timed region
the captured run is replayed untimed for at least --clock-warm seconds so the
GPU clocks have ramped (the W warmup steps alone are microseconds of GPU work).
"""
from __future__ import annotations

import argparse
import json
import math
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
                        "bdq: config 5, the full BDQ frame per step (the whole BranchingQNetwork forward, "
                        "dueling and epsilon-greedy in one fp32 MFMA launch from the packed state, "
                        "pbn_qnet_flipmask_from_state -> pbn_step); "
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
    p.add_argument("--graph", action="store_true",
                   help="rollout workload: replay the timed launches as one hipGraph (default: eager launches "
                        "queued behind the spin gate; a graph replay adds ~8 us of device-side overhead per "
                        "replay on this stack, profiles/r02_chunk_fit_pbn28_65536.jsonl)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-final-state", action="store_true",
                   help="rollout workload: do not write s' (final_state) per step; the next step's obs is s' "
                        "except for envs that autoreset, whose s' is then not stored")
    p.add_argument("--no-gather", action="store_true",
                   help="skip the timed hand-off passes (SURVEY.md 8(e)): the rollouts again with their (s, a, "
                        "s', r, flags) records handed to the learner after every launch, point to point to rank "
                        "0 (value_with_gather; at world 1 the learner's shard is copied into its receive slot) "
                        "and as an RCCL all_gather (gather.all_gather)")
    p.add_argument("--settle", type=int, default=0,
                   help="step law of the whole line: 0 = one synchronous update per env step (the headline "
                        "unit, SURVEY.md 8(d)); K >= 2 = the settle law (intervene, then update until an "
                        "attractor state, at most K updates: PBNEnv's default, include/pbn_env.h)")
    p.add_argument("--settle-line", type=int, default=64,
                   help="env workload under the one-update law: also time the same steps under the settle "
                        "law with this cap (PBNEnv's default, 64) and report them as settle_law; 0 = skip")
    p.add_argument("--clock-warm", type=float, default=0.3,
                   help="seconds of untimed replays of the captured run before timing (GPU clock ramp)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    a = p.parse_args()
    bdq = a.workload in ("bdq", "bdq-learn")
    a.learn_graph = False
    if a.workload == "bdq-learn":
        a.learn_graph = not a.no_graph   # the learner captures its own one-frame graph
        a.no_graph = True
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


def qnet_tail_flops_per_env(n: int, branches: int = 3) -> int:
    """FLOPs of the layers after the bilinear one per env (pbn_qnet_flipmask): trunk 256-128-64-32,
    K + 1 first head layers 32-64, value 64-1, K advantage layers 64-(N+1)."""
    macs = 256 * 128 + 128 * 64 + 64 * 32 + (branches + 1) * 32 * 64 + 64 + branches * 64 * (n + 1)
    return 2 * macs


def algorithmic_bytes_per_env(words: int) -> int:
    # read: state 4W, t 1, target 1 ; write: flipmask (in-kernel actions) 4W,
    # state_out 4W, reward 4, flags 1, t 1   (target is rewritten only on reset)
    return 4 * words + 1 + 1 + 4 * words + 4 * words + 4 + 1 + 1


def survey_bytes_per_env_step(n_nodes: int) -> int:
    """SURVEY.md §8(d)'s algorithmic bytes per env-step, the figure roofline.achieved is priced on:
    read s + flip mask + target id u8 + episode step u8, write s' + reward f32 + flags u8 + step u8,
    with s packed in one u32 (N <= 32) or u64 words (N > 32): 20 B for Bittner-28, 56 B for pbn70."""
    s = 4 if n_nodes <= 32 else 8 * ((n_nodes + 63) // 64)
    return 3 * s + 8


def rollout_bytes_per_env(words: int, steps: int, final: bool = False) -> int:
    # per launch: read + write state 4W, t 1, target 1 once; per step write
    # obs 4W, flipmask (in-kernel actions) 4W, reward 4, flags 1 (+ s' 4W with final)
    return 2 * (4 * words + 1 + 1) + steps * (4 * words + 4 * words + 4 + 1 + (4 * words if final else 0))


def usable_cpus() -> dict:
    """Host CPUs this process may run on: the affinity mask, capped by a cgroup v2 CPU quota
    (on the GPU box the job gets a share of a larger host)."""
    total = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = total
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"cpu_count": total, "affinity": aff, "cgroup_quota": quota, "usable": usable}


def cpu_baseline(spec, envs: int, seconds: float, threads: int):
    """Time the C oracle (port of the step) on `threads` host threads for ~`seconds`."""
    import numpy as np

    from oracle import oracle

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
            "sample": f"oracle/pbn_oracle.c (OpenMP, {threads} threads = every CPU this job may use), {n} "
                      f"{spec.network.name} envs x {done_steps} steps ({el:.1f} s), in-kernel-equivalent random "
                      f"actions, autoreset"}


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
            "sample": f"oracle/pyoracle.py single {spec.network.name} env, {k} steps"}


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


def config1_line(dev, seconds: float = 2.0) -> dict:
    """BASELINE config 1: pbn7, ONE env, the gym facade stepped with random interventions
    (3 uniform ints in [0, 7], duplicates once: bdq_model/__init__.py:76,176), reset on done.
    Timed through the GPU facade (PBNEnv -> pbn_step, one launch + one packed copy back per
    step) and through the per-env Python restatement on one host core."""
    import numpy as np

    from pbn_rl_amd.env import PBNEnv

    env = PBNEnv(network="pbn7", seed=7, device=dev)
    rng = np.random.default_rng(7)
    env.reset()
    for _ in range(20):
        env.step(list(np.unique(rng.integers(0, 8, size=3))))
    k, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        _, _, term, trunc, _ = env.step(list(np.unique(rng.integers(0, 8, size=3))))
        if term or trunc:
            env.reset()
        k += 1
    el = time.perf_counter() - t0
    spec7 = env.spec
    env.close()
    return {"workload": f"pbn7 single env through the gym facade (its default step law: settle <= {spec7.settle} "
                        f"updates), random interventions, reset on done",
            "facade_gpu": {"value": k / el, "unit": "env-steps/s", "us_per_step": el / k * 1e6,
                           "sample": f"PBNEnv(network='pbn7').step x {k}"},
            "cpu_python": python_baseline(spec7, seconds)}


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
    info = usable_cpus()
    info["cpu_model"] = model
    return info


def cpu_baseline_bdq(spec, qnet, seconds: float, threads: int):
    """The BDQ frame on the host cores for ~`seconds`: numpy observation, the same Q-network
    on CPU torch, greedy flip masks and the C oracle step, 4096 envs per frame."""
    import copy

    import numpy as np

    from oracle import agent_oracle, oracle

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


def cpu_baseline_bdq_learn(spec, qnet, n: int, seconds: float, threads: int, batch: int = 256,
                          lr: float = 1e-4, gamma: float = 0.999):
    """The BDQ training frame on the host cores for ~`seconds`, at the GPU line's shape: the acting
    frame of cpu_baseline_bdq over the same n envs, their transitions into a host ring, and one
    update_policy step per frame (batch 256, Adam; bdq_update's PyTorch form on CPU tensors, which
    tests/test_update_golden.py pins to the reference's update_policy)."""
    import copy

    import numpy as np

    from oracle import agent_oracle, oracle
    from pbn_rl_amd.replay import bdq_update

    torch.set_num_threads(threads)
    q_cpu = copy.deepcopy(qnet).to("cpu").train()
    target = copy.deepcopy(q_cpu)
    opt = torch.optim.Adam(q_cpu.parameters(), lr=lr)
    N, K = spec.n, q_cpu.n
    cap = 4 * n
    ring = {"obs": np.zeros((2, cap, N), np.float32), "next_obs": np.zeros((2, cap, N), np.float32),
            "actions": np.zeros((cap, K), np.int64), "rewards": np.zeros(cap, np.float32),
            "masks": np.zeros(cap, np.float32)}
    rng = np.random.default_rng(0)
    st, tg, t = oracle.reset(spec, 1, 0, 0, n)
    frames, updates, pos, size, t0 = 0, 0, 0, 0, time.perf_counter()
    while True:
        obs = agent_oracle.obs_unpack(spec, st, tg)
        with torch.no_grad():
            q = q_cpu(torch.from_numpy(obs)).numpy()
        flip, actions = agent_oracle.q_to_flipmask(spec, q, 1, frames + 1, 0, 0.0)
        out = oracle.step(spec, 1, frames + 1, 0, st, flip, tg, t, 1, want_final=True, n_threads=threads)
        rows = (pos + np.arange(n)) % cap
        ring["obs"][:, rows] = obs
        ring["next_obs"][:, rows] = agent_oracle.obs_unpack(spec, out["final_state"], tg)
        ring["actions"][rows] = actions
        ring["rewards"][rows] = out["reward"]
        ring["masks"][rows] = ((out["flags"] & 3) != 0).astype(np.float32)
        pos, size = (pos + n) % cap, min(size + n, cap)
        st, tg, t = out["state_out"], out["target"], out["t"]
        idx = rng.integers(0, size, batch)
        b = {"obs": torch.from_numpy(ring["obs"][:, idx]), "next_obs": torch.from_numpy(ring["next_obs"][:, idx]),
             "actions": torch.from_numpy(ring["actions"][idx]).unsqueeze(-1),
             "rewards": torch.from_numpy(ring["rewards"][idx]).reshape(-1, 1),
             "masks": torch.from_numpy(ring["masks"][idx]).reshape(-1, 1)}
        bdq_update(q_cpu, target, opt, b, gamma)
        frames += 1
        updates += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {"value": n * frames / el, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"BDQ training frame on CPU: numpy obs + torch CPU BranchingQNetwork ({threads} threads) + "
                      f"greedy flip masks + oracle/pbn_oracle.c step + host ring store + one update_policy step "
                      f"(bdq_update on CPU tensors, batch {batch}, Adam), {n} envs x {frames} frames ({el:.1f} s)"}


def update_flops(n: int, batch: int, branches: int = 3) -> int:
    """FLOPs of one update_policy step (bdq_model/__init__.py:111-131) in the reference's
    arithmetic: forwards of the online network over 2B rows (states, next states) and of the
    target over B rows, and the backward over the B rows that carry gradient (weight and input
    gradients: two forwards' worth), 5B row-forwards of qnet_flops_per_env."""
    return 5 * batch * qnet_flops_per_env(n, branches)


def workload_text(args, chunk: int, rollout_mode: bool) -> str:
    common = (f"horizon {args.horizon}, p={args.perturbation}, prob_bits={args.prob_bits}")
    if args.workload == "bdq":
        return (f"full BDQ rollout (config 5): {args.network} x {args.envs} envs per GPU, per step the "
                f"BranchingQNetwork fp32 forward (random init, seed 0; bilinear layer by pbn_bilinear_targets from "
                f"the packed state) -> epsilon-greedy (eps={args.epsilon}) pbn_heads_to_flipmask -> pbn_step, "
                f"autoreset, {common}, "
                + (f"step law: settle (at most {args.settle} updates per env step, the gym facade's default; "
                   f"pbn_step's one-step launch of pbn_rollout_settle)" if args.settle >= 2 else
                   "step law: one synchronous update per env step"))
    if args.workload == "bdq-learn":
        return (f"BDQ training frames: {args.network} x {args.envs} envs per GPU, per step the config-5 frame "
                f"(eps={args.epsilon}), the envs' transitions into the device replay, one update_policy step "
                f"(batch 256, Adam, double-DQN target; the fused update pbn_bdq_learn, three launches), "
                f"{'one captured hipGraph per frame' if args.learn_graph else 'eager launches'}, {common}")
    stored = "obs/actions/rewards/flags" + ("" if args.no_final_state else "/s'")
    return (f"{args.network} x {args.envs} envs per GPU, in-kernel random interventions (3 uniform actions/env/step), "
            f"autoreset, {common}; "
            + (f"pbn_rollout, launches of up to {chunk} steps, per-step {stored} written to HBM"
               + (" (s' of autoreset envs not stored)" if args.no_final_state else "")
               if rollout_mode else "pbn_step per step"))


def settle_stats(updates, elapsed_s: float, env_steps: int, cap: int = 0) -> dict:
    """Settle lengths (pbn_rollout_ex's d_updates) of every env-step of a timed run: the
    synchronous updates applied per second, their distribution, and the kernel's update slots.
    pbn_rollout_settle runs every env's own sequence of updates (per-env plans; DESIGN.md "Step
    law"): an env spends its updates plus one dropped speculation per step that settles before
    the cap, and a launch lasts as long as its busiest env (the launch tail)."""
    u = torch.cat([x.reshape(-1) for x in updates]).to(torch.int64)
    total = int(u.sum().item())
    hist = torch.bincount(u).cpu().tolist()
    n = u.numel()
    cum, q = 0, {}
    for length, c in enumerate(hist):
        cum += c
        for p in (0.5, 0.9, 0.99):
            if p not in q and cum >= p * n:
                q[p] = length
    # iterations per env and launch: updates + the dropped speculation of steps ending before the cap
    slots = []
    for x in updates:   # [T][n] per launch
        x = x.to(torch.int64)
        per_env = (x + (x < cap).to(torch.int64) if cap else x).sum(0).to(torch.float64)
        slots.append((per_env.mean().item(), per_env.max().item(), x.shape[0]))
    T = sum(t for _, _, t in slots)
    mean_it = sum(m for m, _, _ in slots) / T
    launch_it = sum(mx for _, mx, _ in slots) / T
    return {"updates_per_s": total / elapsed_s, "mean_updates_per_env_step": total / n,
            "mean_env_iterations_per_step": mean_it,
            "launch_iterations_per_step": launch_it,
            "launch_tail": launch_it / mean_it,
            "updates_quantiles": {"p50": q.get(0.5), "p90": q.get(0.9), "p99": q.get(0.99), "max": len(hist) - 1},
            "settle_length_histogram": {str(k): c for k, c in enumerate(hist) if c},
            "env_steps_sampled": n, "env_steps_timed": env_steps,
            "note": "updates = synchronous updates applied per env-step (1 + the settle updates), read from "
                    "pbn_rollout_ex's d_updates of every timed launch.  pbn_rollout_settle gives every env its "
                    "own sequence of updates: mean_env_iterations_per_step = an env's updates + one dropped "
                    "speculation per step that settles before the cap; launch_iterations_per_step = the "
                    "busiest env's (a launch lasts as long as its busiest env: launch_tail = their ratio)"}


def launch_plan(steps: int, chunk: int):
    """Rollout launch lengths covering `steps` steps: full chunks, then the remainder."""
    full, rem = divmod(steps, chunk)
    return [chunk] * full + ([rem] if rem else [])


def max_over_ranks(x: float, world: int, dev) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def barrier(world: int, local: int) -> None:
    if world > 1:
        torch.distributed.barrier(device_ids=[local])


# cycles of the spin kernel queued ahead of the start event (~0.1 ms at the shader clock)
GATE_CYCLES = 1_000_000   # ≈ 0.4 ms of spin: the host's enqueue behind it (≈ 0.15 ms for the driver's
                          # one launch, events included) never reaches the start event late


HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000   # hip_runtime_api.h
_HIP = None


class DeviceEvent:
    """A timing HIP event created with hipEventDisableSystemFence: recording it does not
    release device memory to system scope (no write-back of the outputs for the host), so the
    interval between two of them is the device's work on the stream.  The outputs stay in HBM
    for their consumer on the device (the learner); host visibility comes with the
    synchronize after the end event.  torch.cuda.Event records with the system fence, which
    adds ~1.5-2 us to each timed region (tools/event_probe.py, profiles/r03_zh_event_probe.jsonl)."""

    def __init__(self):
        global _HIP
        import ctypes
        if _HIP is None:
            _HIP = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
        self._c = ctypes
        self.ev = ctypes.c_void_p()
        if _HIP.hipEventCreateWithFlags(ctypes.byref(self.ev), HIP_EVENT_DISABLE_SYSTEM_FENCE) != 0:
            raise RuntimeError("hipEventCreateWithFlags failed")

    def record(self, stream):
        if _HIP.hipEventRecord(self.ev, self._c.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end) -> float:
        ms = self._c.c_float()
        if _HIP.hipEventSynchronize(end.ev) != 0 or _HIP.hipEventElapsedTime(self._c.byref(ms), self.ev, end.ev) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)

    def __del__(self):
        if _HIP is not None and self.ev:
            _HIP.hipEventDestroy(self.ev)


def timed(fn, stream, dev, world, local, gate_cycles: int = None, system_fence: bool = False):
    """Device milliseconds of fn() (launches on `stream`), bracketed by barrier + synchronize,
    max over ranks.  A spin kernel is queued on the stream ahead of the start event (the
    "blocking kernel" of nvbench): while it runs the host enqueues the start event, fn's
    launches and the end event, so the events time the GPU work of fn and not the host's
    graph-launch latency in front of it.  The spin itself lies outside the two events.
    Events: DeviceEvent (no system-scope fence), or torch's default events (system_fence)."""
    barrier(world, local)
    torch.cuda.synchronize(dev)
    if system_fence:
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    else:
        ev0, ev1 = DeviceEvent(), DeviceEvent()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(gate_cycles or GATE_CYCLES)
    t0 = time.perf_counter()
    ev0.record(stream)
    fn()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier(world, local)
    host_s = time.perf_counter() - t0
    return max_over_ranks(ev0.elapsed_time(ev1), world, dev), max_over_ranks(host_s, world, dev)


def gather_pass(env, plan, world, local, dev, stream, dst, copy_own=False, clock_warm=0.0):
    """The timed steps again, the records of every rollout launch handed to the learner
    (ShardedRollout: a ring of two record slots the kernel writes in place; the hand-off of
    launch k runs on the communicator's stream while launch k + 1 runs).  dst = 0: point to
    point to rank 0, which keeps its own shard in place, or with copy_own copies it into its
    receive slot inside launch k + 1 (pbn_rollout_copy; world 1: the whole hand-off); dst = None:
    all_gather_into_tensor.  Device ms, max over ranks."""
    from pbn_rl_amd.distributed import ShardedRollout

    ro = ShardedRollout(world * env.n_alloc, lambda off, cnt: env)
    assert ro.offset == env.env_offset and ro.count == env.n_alloc

    def run():
        for j, k in enumerate(plan):
            ro.gather(ro.rollout(k), dst=dst, async_op=True, copy_own=copy_own, last=j == len(plan) - 1)
        for works in ro._pending.values():   # the last hand-offs, before the end event
            for w in works:
                if w is not None:
                    w.wait()

    with torch.cuda.stream(stream):
        for _ in range(2):   # both record slots (and receive slots) allocated before timing
            run()
        torch.cuda.synchronize(dev)
        # the same untimed clock ramp as the rollout-only run's (the passes before this one end
        # on the host, and the GPU clock drops while it idles)
        t_end = time.perf_counter() + clock_warm
        while time.perf_counter() < t_end:
            run()
            torch.cuda.synchronize(dev)
        # the host enqueues every launch and hand-off of the plan while the gate spins (the
        # ring's Python bookkeeping costs more host time per launch than a bare rollout)
        ms, _ = timed(run, stream, dev, world, local, gate_cycles=GATE_CYCLES * (1 + len(plan) // 4))
    wire = sum(env.n_alloc * k * (12 * env.words + 5) for k in plan)
    return ms, wire


def settle_line(args, dev, stream, world, local, plan, K):
    """The timed steps again under the settle law (cap K, PBNEnv's default law): a fresh env
    of the same network, envs and seed, the same launch plan; env-steps/s, the synchronous
    updates applied per second and the settle-length distribution of every timed env-step."""
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    rank = int(os.environ.get("RANK", "0"))
    spec = EnvSpec(load_network(args.network), load_attractors(args.network), perturbation=args.perturbation,
                   prob_bits=args.prob_bits, horizon=args.horizon, settle=K)
    env = VectorPBNEnv(spec, args.envs, seed=args.seed, device=dev, env_offset=rank * args.envs,
                       keep_final_state=False)
    env.reset()
    keep_final = not args.no_final_state
    kw = dict(random_actions=True, keep_obs=True, keep_final=keep_final, keep_updates=True)
    bufs = [env.rollout_buffers(k, keep_obs=True, keep_final=keep_final, keep_updates=True) for k in plan]
    wplan = launch_plan(args.warmup, args.chunk)
    wbufs = {k: env.rollout_buffers(k, keep_obs=True, keep_final=keep_final, keep_updates=True) for k in set(wplan)}

    def run():
        for i, k in enumerate(plan):
            env.rollout(k, out=bufs[i], **kw)

    with torch.cuda.stream(stream):
        for k in wplan:
            env.rollout(k, out=wbufs[k], **kw)
        t_end = time.perf_counter() + args.clock_warm
        while True:
            run()
            torch.cuda.synchronize(dev)
            if time.perf_counter() >= t_end:
                break
        ms, _ = timed(run, stream, dev, world, local)
    elapsed = ms * 1e-3
    total = world * args.envs * args.steps
    stats = settle_stats([b["updates"] for b in bufs], elapsed, total, cap=K)
    if world > 1:   # every rank's updates
        t = torch.tensor([stats["updates_per_s"]], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t)
        stats["updates_per_s"] = float(t.item())
    per_step = survey_bytes_per_env_step(spec.n)
    achieved = env.n_alloc * world * args.steps * per_step / elapsed / 1e9
    hbm = {"achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
           "bytes_per_env_step": per_step,
           "note": "the same per-env-step I/O as the headline; a settle step applies mean_updates_per_env_step "
                   "updates on chip for it"}
    roofline = {"bound": "valu", "achieved": None, "peak": VALU_WAVE_INSTS_PER_S, "unit": "wave-instructions/s",
                "frac": None, "hbm": hbm,
                "note": "the settle kernel is bound by VALU issue and latency (its three waves share one SIMD at "
                        "65,536 envs), so it is priced on SQ_INSTS_VALU of the same launch shape over this run's "
                        "time against the chip's issue rate (256 CU x 4 SIMD x 2.4 GHz / 2 cycles per wave64 "
                        "VALU instruction); none committed for this shape: null"}
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_{args.network}_{args.envs}_rollout_T{plan[0]}_settle{K}.json")
    if len(set(plan)) == 1 and os.path.exists(pmc_path):
        with open(pmc_path) as f:
            pmc = json.load(f)
        if pmc.get("valu_insts_per_launch"):
            v = pmc["valu_insts_per_launch"] * len(plan) / elapsed
            roofline.update(achieved=v, frac=v / VALU_WAVE_INSTS_PER_S, insts_per_launch=pmc["valu_insts_per_launch"],
                            source={"file": os.path.relpath(pmc_path, ROOT), "command": pmc.get("command")})
            roofline["note"] = roofline["note"].rsplit(";", 1)[0]
    line = {"value": total / elapsed, "unit": "env-steps/s", "ms_per_step": ms / args.steps, "settle_max": K,
            "step_law": f"settle: the intervention, then synchronous updates until every state is an attractor "
                        f"state, at most {K} updates (PBNEnv's default; include/pbn_env.h 'Step law')",
            "kernel": "pbn_rollout_settle (%s)" % ", ".join(f"{k} steps" for k in plan),
            "launch_ms": ms / len(plan), "roofline": roofline, **stats}
    env.close()
    return line, spec


def pmc_profile(args, plan):
    """The rocprofv3 PMC summary of the same launch shape, if one is committed under profiles/
    (network, envs, steps per launch, s' stored or not): HBM bytes and VALU instructions per
    launch (tools/pmc_summary.py)."""
    if len(set(plan)) != 1:
        return None, None
    tail = ("_nofinal" if args.no_final_state else "") + (f"_settle{args.settle}" if args.settle >= 2 else "")
    path = os.path.join(ROOT, "profiles", f"pmc_{args.network}_{args.envs}_{args.mode}_T{plan[0]}{tail}.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        return json.load(f), os.path.relpath(path, ROOT)


def kernel_trace(args, plan):
    """The rocprofv3 kernel-trace average of the same launch shape, if committed under profiles/
    (tools/trace_summary.py): the kernel's own device time beside the two event clocks."""
    if len(set(plan)) != 1:
        return None
    tail = ("_nofinal" if args.no_final_state else "") + (f"_settle{args.settle}" if args.settle >= 2 else "")
    path = os.path.join(ROOT, "profiles", f"kernel_trace_{args.network}_{args.envs}_T{plan[0]}{tail}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return {"avg_launch_us": d["avg_us"], "source": d.get("source"), "file": os.path.relpath(path, ROOT),
            "command": d.get("command")}


def visible_gpu_count() -> int:
    """GPUs this process may use, counted without touching HIP: the KFD topology in sysfs
    (nodes with SIMDs are GPUs), narrowed by ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES.  The parent of ``--gpus N`` calls this before it starts the ranks,
    so it must not initialise the GPU (a process that has may not hand the device to children
    cleanly, and on this pool must not exec)."""
    root = "/sys/class/kfd/kfd/topology/nodes"
    n = 0
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "properties")) as f:
                    props = dict(line.split(None, 1) for line in f if line.strip())
            except OSError:
                continue
            if int(props.get("simd_count", "0").strip() or 0) > 0:
                n += 1
    except OSError:
        n = 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        val = os.environ.get(var)
        if val is not None:
            ids = [v for v in val.split(",") if v.strip() != ""]
            n = min(n, len(ids))
    return n


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes (one per GPU) before
    this process touches the GPU, wait for them, return the worst exit code."""
    import socket
    import subprocess

    n_dev = visible_gpu_count()
    if args.gpus > n_dev:
        print(f"bench.py: --gpus {args.gpus} but only {n_dev} GPU(s) visible; refusing to run "
              f"several ranks on one GPU", file=sys.stderr, flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr, flush=True)
        sys.exit(2)
    n_dev = torch.cuda.device_count()
    if world > n_dev or local >= n_dev:
        print(f"bench.py: {world} rank(s) need {world} GPUs, {n_dev} visible", file=sys.stderr, flush=True)
        sys.exit(2)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # one process per GPU, RCCL ("nccl" on ROCm) over xGMI; world 1 too (the per-rollout gather)
    torch.distributed.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    spec = EnvSpec(load_network(args.network), load_attractors(args.network), perturbation=args.perturbation,
                   prob_bits=args.prob_bits, horizon=args.horizon, settle=args.settle)
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

    rollout_mode = args.mode == "rollout" and agent is None
    chunk = args.chunk if rollout_mode else 1
    keep_final = not args.no_final_state
    bufs = {}   # rollout outputs per launch length; captured graphs write into them, so they live
                # as long as the graphs (torch.cuda.graph empties the allocator cache on entry)

    settle_law = rollout_mode and args.settle >= 2
    bufs_t = {}   # settle law: outputs per launch of the timed plan (every launch's settle lengths kept)

    def launch(k: int, i: int = None):
        """One kernel launch covering k steps of every env (i: index in the timed plan)."""
        if rollout_mode:
            if settle_law and i is not None:
                env.rollout(k, random_actions=True, keep_obs=True, keep_final=keep_final, out=bufs_t[i],
                            keep_updates=True)
            else:
                bufs[k] = env.rollout(k, random_actions=True, keep_obs=True, keep_final=keep_final, out=bufs.get(k),
                                      keep_updates=settle_law)
        elif args.workload == "bdq-learn":
            learner.frame()
        elif agent is not None:
            agent.step()
        else:
            env.step_flipmask(random_actions=True)

    plan = launch_plan(args.steps, chunk)
    # rollouts: eager launches (the gate hides the host's enqueue cost; each launch is 35-160 us
    # of GPU work, so the host stays ahead); the BDQ frames are launch-bound chains of small
    # kernels and replay as graphs
    use_graph = (not args.no_graph) and (args.graph or not rollout_mode)
    if rollout_mode:
        # output buffers of every launch length exist before the capture, so the graph holds
        # the rollout launches alone (no allocation or fill kernels in the timed region)
        for k in set(plan) | set(launch_plan(args.warmup, chunk)):
            bufs[k] = env.rollout_buffers(k, keep_obs=True, keep_final=keep_final, keep_updates=settle_law)
        if settle_law:
            for i, k in enumerate(plan):
                bufs_t[i] = env.rollout_buffers(k, keep_obs=True, keep_final=keep_final, keep_updates=True)
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
                for i, k in enumerate(plan):
                    launch(k, i)
            torch.cuda.synchronize(dev)

        def run():
            if use_graph:
                graph.replay()
            else:
                for i, k in enumerate(plan):
                    launch(k, i)

        # untimed clock ramp: replays of the captured run (no timing, no results kept)
        warm_reps, t_end = 0, time.perf_counter() + args.clock_warm
        while True:
            run()
            torch.cuda.synchronize(dev)
            warm_reps += 1
            if time.perf_counter() >= t_end:
                break
        dev_ms, host_s = timed(run, stream, dev, world, local)
        # the same run between torch's default events (system-scope fence at each event)
        fenced_ms, _ = timed(run, stream, dev, world, local, system_fence=True)
        # three more timings of the same K steps on the same clock, reported beside `value` (not
        # in it): a one-launch run is a single sample, and these show whether it is typical
        repeat_ms = [timed(run, stream, dev, world, local)[0] for _ in range(3)]
        # the floor of this timing method: the same gate + event pair around a one-element kernel
        tiny = torch.zeros(1, device=dev)
        floor_ms = min(timed(lambda: tiny.add_(1.0), stream, dev, world, local)[0] for _ in range(5))
        floor_fenced_ms = min(timed(lambda: tiny.add_(1.0), stream, dev, world, local, system_fence=True)[0]
                              for _ in range(5))
    elapsed = dev_ms * 1e-3
    total_env_steps = world * args.envs * args.steps
    value = total_env_steps / elapsed

    settle = None
    if settle_law:
        settle = settle_stats([bufs_t[i]["updates"] for i in range(len(plan))], elapsed, total_env_steps)
    settle_other, settle_spec = None, None
    if rollout_mode and not settle_law and args.workload == "env" and args.settle_line >= 2:
        settle_other, settle_spec = settle_line(args, dev, stream, world, local, plan, args.settle_line)

    with_gather = None
    if rollout_mode and not args.no_gather:
        with_gather = {}
        # the hand-off of launch k overlaps launch k + 1 (at world 1 the own-shard copy rides along
        # launch k + 1); the last one follows its launch on the launch stream.  A one-launch plan
        # (the driver's 20 steps) stays one launch: split in two it paid a second launch's floor
        # for the overlap (68.6 against 59.2 us, profiles/r05_a_handoff_*.json)
        gplan = plan
        own = world == 1
        for key, dst, what in (("learner", 0, "point-to-point sends of every shard to rank 0" +
                                              (" (world 1: the learner's own shard copied into its receive slot, "
                                               "device to device, by a fourth wave of the next rollout "
                                               "launch)" if own else
                                               " (the learner keeps its own shard in place)")),
                               ("all_gather", None, "torch.distributed.all_gather_into_tensor (RCCL): every "
                                                    "rank receives every shard")):
            gms, wire = gather_pass(env, gplan, world, local, dev, stream, dst, copy_own=own and dst == 0,
                                    clock_warm=args.clock_warm)
            with_gather[key] = {"value": total_env_steps / (gms * 1e-3), "ms_per_step": gms / args.steps,
                                "collective": what + "; one hand-off per rollout launch, overlapped with the "
                                              "next launch (two record slots)",
                                "launches": len(gplan), "plan": gplan, "wire_bytes_per_rank": wire,
                                "wire_bytes_per_env_step": wire // (env.n_alloc * args.steps),
                                "records": "s, a, s' (final_state), r, flags of every env-step"}

    tail_ms = None
    if args.workload in ("bdq", "bdq-learn") and agent.fused_tail:
        # the frame's long launch timed alone: 50 back to back, replayed from one hipGraph (eager,
        # the host's ctypes calls would set the pace)
        with torch.cuda.stream(stream):
            agent.act_q(args.epsilon)
            tg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(tg, stream=stream):
                for _ in range(50):
                    agent.act_q(args.epsilon)
            tg.replay()
            tail_ms, _ = timed(tg.replay, stream, dev, world, local)
            tail_ms /= 50
    learn_ms = None
    if args.workload == "bdq-learn" and learner.fused is not None:
        # the fused update (pbn_bdq_learn's three launches) timed alone: 50 back to back on the
        # frame's batch rows, replayed from one hipGraph (after the timed frames), with the
        # learner's parameters, Adam state, tables and loss snapshotted before and restored after,
        # so that the learner leaves the bench as its last frame left it
        fu = learner.fused
        kept = [(t, t.clone()) for t in (fu.q_flat, fu.m, fu.v, fu.step, fu.q_image, fu.loss, fu.grad)
                if t is not None]
        with torch.cuda.stream(stream):
            rows = learner._idx[:learner.batch_size]
            lg = torch.cuda.CUDAGraph()
            with torch.cuda.graph(lg, stream=stream):
                for _ in range(50):
                    fu.update(learner.replay, rows)
            lg.replay()
            learn_ms, _ = timed(lg.replay, stream, dev, world, local)
            learn_ms /= 50
            for t, c in kept:
                t.copy_(c)
            fu.mark_updated()

    if rank == 0:
        W = spec.words
        pmc, pmc_path = (None, None) if agent is not None else pmc_profile(args, plan)
        if agent is not None:
            kernel = ("BDQ frame (pbn_qnet_flipmask_from_state: the whole BranchingQNetwork on fp32 MFMAs from "
                      "the packed state + dueling + epsilon-greedy; pbn_step)")
            if args.workload == "bdq-learn":
                kernel += " + replay store + update_policy (batch 256)"
                kernel += ", one hipGraph replay per frame" if args.learn_graph else ", eager"
        frame_ms = dev_ms / args.steps
        if args.workload in ("bdq", "bdq-learn"):
            # dominant launch: pbn_qnet_flipmask_from_state, MFMA-bound.  Algorithmic FLOPs = the
            # bilinear layer as the target-contracted product (N x 256 MACs per env) + the layers
            # after it (qnet_tail_flops_per_env), fp32 MFMA peak
            n = env.n_alloc
            flops = env.n_alloc * qnet_flops_per_env(spec.n)
            mfu = {"achieved_tflops": flops / (frame_ms * 1e-3) / 1e12, "peak_tflops": FP32_MATRIX_TFLOPS,
                   "note": "the reference forward's FLOPs (bilinear as N*N*256 MACs/env) over the whole frame "
                           "time; the frame executes ~4x fewer"}
            if tail_ms is not None:
                tail_flops = n * (qnet_tail_flops_per_env(spec.n, agent.branches) + 2 * spec.n * 256)
                tf = tail_flops / (tail_ms * 1e-3) / 1e12
                roofline = {"bound": "mfma", "achieved": tf, "peak": FP32_MATRIX_TFLOPS, "unit": "TFLOP/s",
                            "frac": tf / FP32_MATRIX_TFLOPS, "traffic": None,
                            "kernel": "pbn_qnet_flipmask_from_state (the frame's longest launch)",
                            "launch_ms": tail_ms, "flops_per_launch": tail_flops,
                            "note": "v_mfma_f32_16x16x4_f32 (exact f32), one wave per 16 envs; FLOPs = the bilinear "
                                    "layer contracted with the target (N x 256 MACs) + the Linear layers after it "
                                    "(trunk 256-128-64-32, K+1 heads 32-64-A)",
                            "model_flops_utilisation": mfu}
                if args.workload == "bdq-learn":
                    roofline["note"] += ("; the training frame's longest launch, as in the acting line (the frame: "
                                         "Q-network, step, ring store, row draw, the fused update's three launches)")
                    if learn_ms is not None:
                        uf = update_flops(spec.n, learner.batch_size, agent.branches)
                        ut = uf / (learn_ms * 1e-3) / 1e12
                        roofline["update"] = {
                            "bound": "mfma", "achieved": ut, "peak": FP32_MATRIX_TFLOPS, "unit": "TFLOP/s",
                            "frac": ut / FP32_MATRIX_TFLOPS, "kernel": "pbn_bdq_learn (forward, backward, apply)",
                            "update_ms": learn_ms, "flops_per_update": uf,
                            "update_timing_note": "50 updates replayed on the last frame's rows; the learner's "
                                                  "weights, Adam state and tables restored afterwards",
                            "note": "update_policy's FLOPs in the reference's arithmetic (5B row-forwards: online "
                                    "over states and next states, target over next states, backward over B rows, "
                                    "bench.py update_flops) over the fused update's time, 50 replayed back to back"}
            else:
                roofline = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                            "traffic": None, "kernel": "frame (PyTorch tail)", "launch_ms": frame_ms,
                            "model_flops_utilisation": mfu}
        elif rollout_mode:
            per_step = survey_bytes_per_env_step(spec.n)
            bytes_run = env.n_alloc * args.steps * per_step
            moved_run = sum(env.n_alloc * rollout_bytes_per_env(W, k, keep_final) for k in plan)
            achieved = bytes_run / elapsed / 1e9
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS,
                        "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                        "kernel": "pbn_rollout (%s)" % ", ".join(f"{k} steps" for k in plan),
                        "launch_ms": dev_ms / len(plan), "bytes_per_launch": bytes_run / len(plan),
                        "bytes_per_env_step": per_step,
                        "moved_bytes_per_launch": moved_run / len(plan),
                        "moved_bytes_per_env_step": moved_run / (env.n_alloc * args.steps),
                        "note": "achieved = SURVEY.md 8(d)'s algorithmic bytes per env-step (a step kernel's "
                                "minimal packed I/O) x env-steps / HIP-event time.  The rollout keeps the state "
                                "on chip between steps and moves moved_bytes_per_launch, which `traffic` (PMC, "
                                "per launch) measures.  The kernel is VALU-issue / latency bound, see DESIGN.md "
                                "'What bounds it'",
                        # what the counters show bounds the kernel ("bound" is the contract's pricing
                        # axis, the bytes): VALU issue well below its rate, the waves waiting on LDS
                        # round trips and the per-step block barrier (DESIGN.md "What bounds the env
                        # kernel, from counters")
                        "limiter": "latency: VALU issue below its rate, waves parked on s_waitcnt / the "
                                   "per-step block barrier (roofline.valu, traffic_source's wave_state)"}
            if pmc:
                roofline["traffic_source"] = {"file": pmc_path, "command": pmc.get("command")}
                if pmc.get("valu_insts_per_launch"):
                    v = pmc["valu_insts_per_launch"] * len(plan) / elapsed
                    roofline["valu"] = {"achieved": v, "peak": VALU_WAVE_INSTS_PER_S, "unit": "wave-instructions/s",
                                        "frac": v / VALU_WAVE_INSTS_PER_S,
                                        "insts_per_launch": pmc["valu_insts_per_launch"],
                                        "note": "SQ_INSTS_VALU of the same launch shape (traffic_source) over this "
                                                "run's time; issue slots only"}
        else:
            bytes_launch = env.n_alloc * survey_bytes_per_env_step(spec.n)
            achieved = bytes_launch / (frame_ms * 1e-3) / 1e9
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "pbn_step",
                        "launch_ms": frame_ms, "bytes_per_launch": bytes_launch,
                        "bytes_per_env_step": survey_bytes_per_env_step(spec.n),
                        "moved_bytes_per_env_step": algorithmic_bytes_per_env(W)}
        out = {
            "metric": "env steps/sec (batched PBN transitions), Bittner-28 at 1/2/4/8 GPUs"
            if args.network == "pbn28" and not settle_law else
            f"env steps/sec (batched PBN transitions{', settle law' if settle_law else ''}), {args.network}",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dev_ms / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32+u32" if agent is not None else "u32",
            "data": "synthetic",
            "config": {"workload": workload_text(args, chunk, rollout_mode),
                       "network": args.network, "envs_per_gpu": args.envs, "global_envs": world * args.envs,
                       "parallelism": f"env-shard x{world} (RCCL process group)",
                       "launch": "hipGraph" if (use_graph or args.learn_graph) else "eager"},
            "roofline": roofline,
            "timing": {"clock": "HIP events (hipEventDisableSystemFence) on the launch stream behind a spin gate, "
                                "max over ranks",
                       "event_floor_us": floor_ms * 1e3,
                       "default_events": {"value": total_env_steps / (fenced_ms * 1e-3),
                                          "ms_per_step": fenced_ms / args.steps,
                                          "event_floor_us": floor_fenced_ms * 1e3,
                                          "note": "the same run between torch.cuda.Event pairs, whose records "
                                                  "release device memory to system scope (host visibility)"},
                       "note": "event_floor_us: the same gate + event pair around a one-element kernel (dispatch "
                               "and event overhead, part of every timed region)",
                       "host_ms_per_step": host_s * 1e3 / args.steps, "clock_warm_runs": warm_reps,
                       "repeats_ms_per_step": [r / args.steps for r in repeat_ms]},
        }
        if rollout_mode:
            kt = kernel_trace(args, plan)
            out["timing"]["launch_us"] = dev_ms * 1e3 / len(plan)
            out["timing"]["default_events"]["launch_us"] = fenced_ms * 1e3 / len(plan)
            if kt is not None:
                kt["value"] = total_env_steps / (kt["avg_launch_us"] * 1e-6 * len(plan))
                out["timing"]["kernel_trace"] = kt
        if settle is not None:
            out["config"]["step_law"] = f"settle (at most {args.settle} updates per env step)"
            out["settle"] = settle
        elif rollout_mode:
            out["config"]["step_law"] = "one synchronous update per env step (SURVEY.md 8(d)'s unit of work)"
        if settle_other is not None:
            # what one synchronous update costs against one step of the one-update law (this line's
            # own clock): per kernel iteration (the launch's busiest env's iterations) and per update
            # an env needs
            g = settle_other.get("launch_iterations_per_step")
            if g:
                per_it = settle_other["ms_per_step"] / g
                per_env = settle_other["ms_per_step"] / settle_other["mean_updates_per_env_step"]
                settle_other["update_cost_vs_one_update_step"] = {
                    "per_kernel_iteration": per_it / (dev_ms / args.steps),
                    "per_env_update": per_env / (dev_ms / args.steps),
                    "note": "ms per step / (launch iterations, updates) per step, over the headline's ms per step"}
            out["settle_law"] = settle_other
        if with_gather is not None:
            out["value_with_gather"] = with_gather["learner"]["value"]
            out["gather"] = with_gather
        if world == 1 and not args.no_cpu_baseline:
            host = host_info()
            threads = host["usable"]
            if args.workload == "bdq-learn":
                out["cpu_baseline"] = cpu_baseline_bdq_learn(spec, agent.q, args.envs, args.cpu_seconds, threads)
            elif agent is not None:
                out["cpu_baseline"] = cpu_baseline_bdq(spec, agent.q, args.cpu_seconds, threads)
            else:
                out["cpu_baseline"] = cpu_baseline(spec, args.envs, args.cpu_seconds, threads)
                if settle_other is not None:
                    out["settle_law"]["cpu_baseline"] = cpu_baseline(settle_spec, args.envs, args.cpu_seconds / 2,
                                                                     threads)
                out["cpu_baseline_python"] = python_baseline(spec)
                out["cpu_baseline_numpy"] = numpy_baseline(spec, args.envs)
                out["config1"] = config1_line(dev)
            out["host"] = host
        print(json.dumps(out), flush=True)
    env.close()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
