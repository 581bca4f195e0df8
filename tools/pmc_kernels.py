"""Per-kernel PMC summary of a multi-kernel workload (the BDQ frame): the mean of every counter
over each kernel's launches, across the PMC pass directories of tools/gpu_session.sh bdqpmc.

    python tools/pmc_kernels.py gpurun_out/r03_g --passes bdq_pmc_l2 bdq_pmc_fetch bdq_pmc_write \
        --kernel-stats gpurun_out/r03_g/bdq_trace/run_kernel_stats.csv --out profiles/pmc_bdq_pbn28_32768.json

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (kB units), MI355X_MICROARCH.md's gfx950 correction.
L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum) (the guide's L2 section).
"""
import argparse
import collections
import csv
import json
import os
import re


def short(name):
    m = re.search(r"(\w+_kernel|\w+_wave|pbn_\w+)", name)
    return m.group(1) if m else name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--passes", nargs="+", required=True)
    ap.add_argument("--kernel-stats", default=None)
    ap.add_argument("--prefix", default="(anonymous namespace)", help="keep kernels whose name contains this")
    ap.add_argument("--command", default=None)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in args.passes:
        with open(os.path.join(args.run_dir, p, "run_counter_collection.csv")) as f:
            for r in csv.DictReader(f):
                if args.prefix in r["Kernel_Name"]:
                    acc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = {}
    if args.kernel_stats:
        with open(args.kernel_stats) as f:
            for r in csv.DictReader(f):
                dur[short(r["Name"])] = float(r["AverageNs"])
    kernels = {}
    for k, cs in acc.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        d["launches"] = max(len(v) for v in cs.values())
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["hbm_bytes_per_launch"] = (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024
        if k in dur:
            d["avg_ns"] = dur[k]
            if "hbm_bytes_per_launch" in d:
                d["hbm_GBps"] = d["hbm_bytes_per_launch"] / dur[k]
        kernels[k] = d
    out = {"run_dir": args.run_dir, "passes": args.passes, "command": args.command,
           "correction": "FETCH_SIZE x2 on gfx950; counter units kB (1024 B)", "kernels": kernels}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    for k, d in kernels.items():
        print(k, {c: round(v, 3) if isinstance(v, float) else v for c, v in d.items()})


if __name__ == "__main__":
    main()
