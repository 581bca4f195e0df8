"""profiles/kernel_trace_<net>_<envs>_T<steps>.json from a rocprofv3 --kernel-trace run of bench.py
(tools/gpu_bench_profile.sh's trace/ pass): the average dispatch time of the rollout kernel, which
bench.py puts beside its HIP-event clock as timing.kernel_trace.

    python tools/kernel_trace_summary.py gpurun_out/r05_zb/driver/trace --out profiles/kernel_trace_pbn28_65536_T20.json \
        --command "..."

Launches that carry the hand-off's own-shard copy (pbn_rollout_copy: the pipelined kernel with a
fourth wave, 256 threads per block) are left out.
"""
import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--kernel", default="pbn_rollout_pipe")
    ap.add_argument("--out", required=True)
    ap.add_argument("--command", default=None)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    durs, names = [], set()
    for f in files:
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            if "pbn_rollout_pipe" in r["Kernel_Name"] and r.get("Workgroup_Size_X") == "256":
                continue
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
            names.add(r["Kernel_Name"])
    if not durs:
        raise SystemExit(f"no dispatches of {a.kernel} under {a.trace_dir}")
    out = {"kernel": sorted(names), "dispatches": len(durs), "avg_us": sum(durs) / len(durs),
           "source": os.path.normpath(a.trace_dir), "command": a.command,
           "note": "rocprofv3 --kernel-trace of the same bench command: the average over every dispatch of the "
                   "kernel (warmup, clock-warm replays and the timed launches), launches carrying the "
                   "hand-off's copy left out"}
    with open(a.out, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
