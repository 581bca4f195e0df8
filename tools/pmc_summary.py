"""Turn the PMC passes of tools/gpu_bench_profile.sh into profiles/pmc_<net>_<envs>_<mode>.json.

    python tools/pmc_summary.py gpurun_out/r01c --envs 65536 --steps-per-launch 100 [--words 1]

HBM bytes per launch of the step kernel = 2 x FETCH_SIZE + WRITE_SIZE (kB units), the gfx950
correction of MI355X_MICROARCH.md's HBM section.  bench.py reads `hbm_bytes_per_launch` as
roofline.traffic.  With the SQ pass (pmc_sq/), also the wave-level VALU / SALU instruction
counts per launch, which bench.py turns into the VALU issue fraction.
"""
import argparse
import csv
import json
import os


def mean_counter(path, counter, kernel="pbn_"):
    """Mean of one counter over the dispatches of the kernel, leaving out the launches that carry
    the hand-off's own-shard copy (pbn_rollout_copy: the pipelined kernel with a fourth wave)."""
    vals, name = [], None
    with open(path) as f:
        for r in csv.DictReader(f):
            ride = "pbn_rollout_pipe" in r["Kernel_Name"] and r.get("Workgroup_Size") == "256"
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"] and "reset" not in r["Kernel_Name"] \
                    and not ride:
                vals.append(float(r["Counter_Value"]))
                name = r["Kernel_Name"]
    return sum(vals) / len(vals), len(vals), name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--mode", default="rollout")
    ap.add_argument("--steps-per-launch", type=int, default=100)
    ap.add_argument("--words", type=int, default=1)
    ap.add_argument("--no-final", action="store_true", help="the run did not store s' (bench.py --no-final-state)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--command", default=None, help="the profiled command, recorded in the summary")
    ap.add_argument("--kernel", default="pbn_",
                    help="kernel-name substring to average (a bench line with a settle_law object runs "
                         "pbn_rollout_pipe and pbn_rollout_settle in one process)")
    ap.add_argument("--suffix", default="", help="file-name suffix (e.g. _settle64)")
    args = ap.parse_args()
    f, n, name = mean_counter(os.path.join(args.run_dir, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE",
                              args.kernel)
    w, _, _ = mean_counter(os.path.join(args.run_dir, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE",
                           args.kernel)
    W, T = args.words, args.steps_per_launch
    if args.mode == "rollout":
        alg = args.envs * (2 * (4 * W + 2) + T * ((8 if args.no_final else 12) * W + 5))
    else:
        alg = args.envs * (12 * W + 8)
    out = {"kernel": name, "mode": args.mode, "envs": args.envs, "launches": n,
           "FETCH_SIZE_kB_per_launch": f, "WRITE_SIZE_kB_per_launch": w,
           "correction": "MI355X_MICROARCH.md HBM section: FETCH_SIZE x2 on gfx950; counter units kB (1024 B)",
           "hbm_read_bytes_per_launch": f * 2 * 1024, "hbm_write_bytes_per_launch": w * 1024,
           "hbm_bytes_per_launch": (2 * f + w) * 1024, "algorithmic_bytes_per_launch": alg,
           "note": "the read side is 4-B and 1-B loads plus table reads, a width the guide leaves uncalibrated",
           "command": args.command, "steps_per_launch": args.steps_per_launch}
    sq = os.path.join(args.run_dir, "pmc_sq", "run_counter_collection.csv")
    if os.path.exists(sq):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_ACTIVE_INST_VALU", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES",
                  "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"):
            try:
                out[c + "_per_launch"] = mean_counter(sq, c, args.kernel)[0]
            except ZeroDivisionError:   # counter not in this pass
                pass
        out["valu_insts_per_launch"] = out["SQ_INSTS_VALU_per_launch"]
        if "SQ_WAVE_CYCLES_per_launch" in out:
            wc = out["SQ_WAVE_CYCLES_per_launch"]
            out["wave_state"] = {
                "note": "fractions of SQ_WAVE_CYCLES (disjoint: MI355X_MICROARCH.md PMC table); quad-cycle units",
                "active_any": out["SQ_ACTIVE_INST_ANY_per_launch"] / wc,
                "active_valu": out["SQ_ACTIVE_INST_VALU_per_launch"] / wc,
                "wait_any (s_waitcnt / barrier)": out["SQ_WAIT_ANY_per_launch"] / wc,
                "wait_inst_any (issue stall)": out["SQ_WAIT_INST_ANY_per_launch"] / wc}
    tail = ("_nofinal" if args.no_final else "") + args.suffix
    path = args.out or os.path.join("profiles",
                                    f"pmc_{args.network}_{args.envs}_{args.mode}_T{args.steps_per_launch}{tail}.json")
    with open(path, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
