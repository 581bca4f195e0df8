"""Host logic of the profile summaries (no GPU): the launches that carry the hand-off's own-shard
copy (pbn_rollout_copy: the pipelined kernel at 256 threads per block) and the standalone copy
kernel stay out of the rollout kernel's averages, and the hand-off trace is cut into reps."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PIPE = "void (anonymous namespace)::pbn_rollout_pipe<1, 16, false>((anonymous namespace)::StepArgs)"


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_pmc_summary_leaves_out_copy_launches(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        import pmc_summary
    finally:
        sys.path.pop(0)
    hdr = ["Kernel_Name", "Workgroup_Size", "Counter_Name", "Counter_Value"]
    rows = [[PIPE, "192", "WRITE_SIZE", "100"], [PIPE, "192", "WRITE_SIZE", "110"],
            [PIPE, "256", "WRITE_SIZE", "300"], ["pbn_copy_kernel", "256", "WRITE_SIZE", "900"]]
    p = str(tmp_path / "c.csv")
    _write(p, hdr, rows)
    mean, n, name = pmc_summary.mean_counter(p, "WRITE_SIZE", "pbn_rollout_pipe")
    assert (mean, n, name) == (105.0, 2, PIPE)


def test_kernel_trace_summary_leaves_out_copy_launches(tmp_path):
    hdr = ["Kernel_Name", "Workgroup_Size_X", "Start_Timestamp", "End_Timestamp"]
    rows = [[PIPE, "192", "0", "20000"], [PIPE, "192", "100000", "124000"], [PIPE, "256", "200000", "260000"],
            ["pbn_copy_kernel", "256", "300000", "310000"]]
    _write(str(tmp_path / "trace" / "run_kernel_trace.csv"), hdr, rows)
    out = str(tmp_path / "kt.json")
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "kernel_trace_summary.py"), str(tmp_path / "trace"),
                    "--out", out], check=True, capture_output=True)
    d = json.load(open(out))
    assert d["dispatches"] == 2 and abs(d["avg_us"] - 22.0) < 1e-9


def test_handoff_summary_cuts_reps_at_gaps(tmp_path):
    """Two gated reps, the second followed (after a gap) by an untimed warm-up's dispatches: each
    rep is its gate's back-to-back dispatches; the rep with the extra copy is the hand-off's."""
    hdr = ["Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    us = 1000
    rows = [["spin_kernel", 0, 100 * us],
            [PIPE, 101 * us, 181 * us], [PIPE, 181 * us, 261 * us],                     # bare rep
            ["spin_kernel", 300 * us, 400 * us],
            [PIPE, 401 * us, 491 * us], [PIPE, 491 * us, 581 * us], ["pbn_copy_kernel", 581 * us, 620 * us],
            [PIPE, 700 * us, 780 * us]]                                                 # next phase's warm-up
    _write(str(tmp_path / "h" / "run_kernel_trace.csv"), hdr, rows)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "handoff_trace.py"), "--summarize",
                        str(tmp_path / "h")], check=True, capture_output=True, text=True)
    d = json.loads(r.stdout)
    assert d["reps"] == 2
    assert len(d["median_rep"]["items"]) == 3 and abs(d["median_rep"]["span_us"] - 220.0) < 1e-6
    assert len(d["median_bare_rep"]["items"]) == 2 and abs(d["median_bare_rep"]["span_us"] - 161.0) < 1e-6
