"""The world-1 hand-off pass of bench.py (gather_pass, ShardedRollout.gather with copy_own) alone,
for a kernel-and-copy trace:

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -o run -- \\
      python tools/handoff_trace.py [--steps 20] [--plan 20] [--reps 20]

Each rep: the rollout launches of the plan into the ring's record slots, each followed by the
hand-off of its records (at world 1: the learner's own shard copied into its receive slot by
the next launch's fourth wave, pbn_rollout_copy, the last one by pbn_copy_async on the launch
stream), then a device sync.  The same launches without the hand-off are timed first (bare_*).
Prints one JSON line with the per-rep device time of the pass (HIP events around each rep, after
a 0.3 s clock warm-up), and with --summarize DIR attributes the trace: per rep, the rollout
kernels, the copy (kernel or DMA), and the gaps between them.
"""
import argparse
import glob
import json
import time
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def run(args):
    import torch

    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.distributed import ShardedRollout
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.01, horizon=20)
    env = VectorPBNEnv(spec, args.envs, seed=0, keep_final_state=True)
    env.reset()
    plan = [int(x) for x in args.plan.split(",")]
    ro = ShardedRollout(env.n_alloc, lambda off, cnt: env)
    stream = torch.cuda.current_stream()

    def rep():
        for j, k in enumerate(plan):
            ro.gather(ro.rollout(k), dst=0, async_op=True, copy_own=True, last=j == len(plan) - 1)
        for works in ro._pending.values():
            for w in works:
                if w is not None:
                    w.wait()

    def bare():   # the same launches into the same record slots, no hand-off
        for k in plan:
            ro.rollout(k)

    def clock(fn):
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        t_end = time.perf_counter() + 0.3   # clock ramp, as bench.py's --clock-warm
        while time.perf_counter() < t_end:
            fn()
            torch.cuda.synchronize()
        times = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda._sleep(2_000_000)   # the host enqueues the rep while this spins
            e0.record(stream)
            fn()
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3)
        times.sort()
        return times

    tb = clock(bare)
    times = clock(rep)
    wire = sum(env.n_alloc * k * (12 * env.words + 5) for k in plan)
    print(json.dumps({"what": "world-1 hand-off pass", "plan": plan, "envs": env.n_alloc, "reps": args.reps,
                      "us_median": times[len(times) // 2], "us_min": times[0], "wire_bytes": wire,
                      "bare_us_median": tb[len(tb) // 2], "bare_us_min": tb[0],
                      "with_handoff_over_bare": tb[len(tb) // 2] / times[len(times) // 2]}))


def summarize(d):
    """Attribute the trace: the dispatches and copies between consecutive spin-gate kernels."""
    import csv
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mf = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for f in kf:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"][:60]))
    for f in mf:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "C:" + r.get("Direction", r.get("Operation", "copy"))))
    ev.sort()
    gates = [i for i, e in enumerate(ev) if "sleep" in e[2].lower() or "spin" in e[2].lower()]
    reps = []
    for a, b in zip(gates, gates[1:] + [len(ev)]):
        seg = ev[a + 1:b]
        # the rep: the dispatches queued behind the gate run back to back; the first gap past
        # 20 us ends it (what follows is the next phase's untimed warm-up)
        for i in range(1, len(seg)):
            if seg[i][0] - seg[i - 1][1] > 20_000:
                seg = seg[:i]
                break
        if not seg:
            continue
        t0 = ev[a][1]
        items = [{"what": w, "start_us": (s - t0) / 1e3, "dur_us": (e - s) / 1e3} for s, e, w in seg]
        reps.append({"span_us": (max(e for _, e, _ in seg) - t0) / 1e3, "items": items})
    # the run times the bare launches first, then the hand-off pass (one more dispatch: the last
    # hand-off's copy)
    def median(rs):
        return sorted(rs, key=lambda r: r["span_us"])[len(rs) // 2] if rs else None
    most = max((len(r["items"]) for r in reps), default=0)
    out = {"reps": len(reps), "median_rep": median([r for r in reps if len(r["items"]) == most]),
           "median_bare_rep": median([r for r in reps if len(r["items"]) < most])}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--envs", type=int, default=65536)
    p.add_argument("--plan", default="20")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--summarize", default=None)
    a = p.parse_args()
    if a.summarize:
        summarize(a.summarize)
    else:
        run(a)
