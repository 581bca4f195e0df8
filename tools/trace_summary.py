"""Kernel-trace summary of one bench shape, for bench.py's timing.kernel_trace field.

    python tools/trace_summary.py STATS_CSV --kernel pbn_rollout_pipe --network pbn28 --envs 65536 \
        --steps-per-launch 20 --command "..." [--suffix _settle64]

Reads a rocprofv3 ``--kernel-trace --stats`` summary (``*_kernel_stats.csv``), takes the rows whose
kernel name contains ``--kernel`` and writes
profiles/kernel_trace_{network}_{envs}_T{steps}{suffix}.json with their average duration (the
dispatch-weighted mean over the matching rows).  bench.py puts that figure beside its two event
clocks when a file of its own shape exists.
"""
import argparse
import csv
import json
import os

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps-per-launch", type=int, required=True)
    ap.add_argument("--suffix", default="")
    ap.add_argument("--command", default="")
    a = ap.parse_args()
    calls, total, names = 0, 0.0, []
    with open(a.csv) as f:
        for row in csv.DictReader(f):
            if a.kernel in row["Name"]:
                calls += int(row["Calls"])
                total += float(row["TotalDurationNs"])
                names.append(row["Name"])
    if not calls:
        raise SystemExit(f"no kernel matching {a.kernel!r} in {a.csv}")
    out = {"kernel": names, "dispatches": calls, "avg_us": total / calls / 1e3,
           "source": os.path.relpath(os.path.abspath(a.csv), ROOT), "command": a.command,
           "note": "rocprofv3 --kernel-trace --stats of the same bench command: the average over every "
                   "dispatch of the kernel (warmup, clock-warm replays and the timed launches)"}
    path = os.path.join(ROOT, "profiles",
                        f"kernel_trace_{a.network}_{a.envs}_T{a.steps_per_launch}{a.suffix}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, round(out["avg_us"], 3))


if __name__ == "__main__":
    main()
