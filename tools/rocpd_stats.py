"""Kernel statistics from a rocprofv3 rocpd database (ROCm 7 writes results.db, not CSV).

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [--match rollout] [--csv out.csv]

Per kernel name: launches, average / min / max duration (us), and for --match the
sequence of the last launches with the idle gaps between them.
"""
import argparse
import collections
import csv
import sqlite3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--match", default=None)
    p.add_argument("--csv", default=None)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count "
                     "from kernels order by start").fetchall()
    agg = collections.OrderedDict()
    for name, s, e, gx, wx, lds, vg, sg in rows:
        d = agg.setdefault(name, {"n": 0, "tot": 0, "min": 1e30, "max": 0, "grid": gx, "wg": wx, "lds": lds,
                                  "vgpr": vg, "sgpr": sg})
        d["n"] += 1
        d["tot"] += e - s
        d["min"] = min(d["min"], e - s)
        d["max"] = max(d["max"], e - s)
    out = []
    for name, d in sorted(agg.items(), key=lambda kv: -kv[1]["tot"]):
        out.append({"kernel": name[:120], "calls": d["n"], "avg_us": d["tot"] / d["n"] / 1e3,
                    "min_us": d["min"] / 1e3, "max_us": d["max"] / 1e3, "total_us": d["tot"] / 1e3,
                    "grid": d["grid"], "workgroup": d["wg"], "lds": d["lds"], "vgpr": d["vgpr"], "sgpr": d["sgpr"]})
    for r in out[:15]:
        print(f"{r['calls']:6d} avg {r['avg_us']:9.2f} us  min {r['min_us']:9.2f}  max {r['max_us']:9.2f}  "
              f"grid {r['grid']} wg {r['workgroup']} lds {r['lds']} vgpr {r['vgpr']}  {r['kernel'][:70]}")
    if a.match:
        seq = [(s, e - s) for name, s, e, *_ in rows if a.match in name]
        print("last launches (us):", [round(x[1] / 1e3, 1) for x in seq[-12:]])
        print("gaps before them (us):", [round((seq[i][0] - seq[i - 1][0] - seq[i - 1][1]) / 1e3, 1)
                                         for i in range(max(1, len(seq) - 12), len(seq))])
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0].keys()))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
