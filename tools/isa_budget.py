"""Instruction budget of the pipelined one-update kernel, per role and segment, from its ISA
(VERDICT r04 next 2).

  python tools/isa_budget.py [--W 1 --B 16 --K 3] [--json profiles/r05_isa_budget_pbn28.json]

Compiles one instance of pbn_rollout_pipe<W, B, false> to an assembly listing with
-DPBN_ISA_MARKS: every stamp site of the stamps build (tools/stamps.py) becomes a comment line
fenced by scheduling barriers, and each role's loop body is named (`;@loop state_fast K`,
`sel_fast NQ`, `env_fast W`).  Nothing else changes, so the listing is the product's code cut at
the stamps' segment boundaries.  For each role's loop the tool walks ONE iteration along the path
config 2 takes (pbn28: random actions, gap table, single-state attractors, one hash probe,
perturbation gaps below three):
  - a branch (uniform, or an exec-mask skip) is taken when the code it skips enters an inner loop
    and holds no segment mark (the fourth-flip tail, the extra hash probes), or holds only a
    launch-anatomy stamp; otherwise it falls through (an exec-mask skip: the guarded lanes are live);
  - the back edge ends the iteration.
Counts are per block iteration (64 env-steps: two 32-env groups); loops unrolled two steps per
trip are halved.  Classes: VALU (with DPP / SDWA shares), SALU, LDS (with the LDS-array cycles of
MI355X_MICROARCH.md's LDS table), VMEM, SMEM, s_waitcnt, s_nop, branch, barrier.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")

# LDS-array cycles per wave-instruction (MI355X_MICROARCH.md "LDS" table); swizzle / bpermute
# priced as a b32 read
LDS_CYC = {"ds_read_b32": 2, "ds_read_b64": 2, "ds_read_b128": 4, "ds_read_b96": 8,
           "ds_read2_b32": 4, "ds_read2st64_b32": 4, "ds_read2_b64": 8, "ds_read2st64_b64": 8,
           "ds_write_b32": 4, "ds_write_b64": 6, "ds_write2_b32": 6, "ds_write2st64_b32": 6,
           "ds_write_b96": 10, "ds_write_b128": 13, "ds_swizzle_b32": 2, "ds_bpermute_b32": 2,
           "ds_permute_b32": 2, "ds_read_u8": 2, "ds_read_u16": 2, "ds_write_b8": 4, "ds_write_b16": 4}

# segment names of the stamp sites (step_kernels.h pbn_rollout_pipe)
SEGMENTS = {
    "state_fast": {"P0": "slot reads + obs store", "A15": "transpose to bit planes + plane store",
                   "A3": "input gathers + mux chains", "A12": "back-transpose",
                   "A13": "epilogue: perturbation, hash, reward, flags, autoreset, stores",
                   "P1": "barrier", "P2": "loop latch"},
    "env_fast": {"P0": "this step's draws + LDS reads", "A16": "next step's ENV call (Philox)",
                 "A17": "actions, gaps, slot writes, flip-mask store", "P1": "barrier",
                 "P2": "loop latch"},
    "sel_fast": {"P0": "next step's SEL calls (Philox)", "A18": "threshold compares + slot writes",
                 "P1": "barrier", "P2": "loop latch"},
    # pbn_rollout_settle (one update per iteration, per-env plans)
    "settle_state": {"P0": "plan, slot reads, transpose to bit planes + plane store",
                     "A15": "input gathers + mux chains", "A3": "back-transpose, perturbed / idle select",
                     "A12": "attractor lookup, decision C, epilogue (at a step's end), stores",
                     "P1": "barrier", "P2": "loop latch"},
    "settle_env_fast": {"P0": "decision C read, plan", "A16": "ENV / SETTLE_ENV call, draws, gaps, flip-mask store",
                        "A17": "slot writes", "P1": "barrier", "P2": "loop latch"},
    "settle_sel": {"P0": "decision C read, plan, SETTLE_SEL calls (Philox)",
                   "A18": "threshold compares, transposes to planes, slot writes", "P1": "barrier",
                   "P2": "loop latch"},
}
KERNELS = {"pipe": ("pbn_rollout_pipe<%(W)d, %(B)d, false>",
                    lambda a: {"state_fast": a.K, "sel_fast": a.K - 1, "env_fast": a.W}),
           "settle": ("pbn_rollout_settle<%(W)d, %(B)d>",
                      lambda a: {"settle_state": a.K, "settle_sel": 2 * (a.K - 1) + a.pk, "settle_env_fast": a.W})}


def compile_listing(inst, out_s):
    src = os.path.join(tempfile.mkdtemp(prefix="isa_budget_"), "kernel.hip")
    with open(src, "w") as f:
        f.write('#include "%s"\n' % os.path.join(ROOT, "pbn_rl_amd", "csrc", "step_kernels.h"))
        f.write("void* isa_budget_instance() { return reinterpret_cast<void*>(&%s); }\n" % inst)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-DPBN_ISA_MARKS",
                    "--offload-device-only", "-S", "-o", out_s, src], check=True,
                   stderr=subprocess.DEVNULL)


def parse(lines):
    """Basic blocks of the kernel: [{label, depth, header, lines}] in listing order."""
    blocks, cur = [], None
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(\.LBB\d+_\d+):(.*)$", s) or re.match(r"^; (%bb\.\d+):(.*)$", s)
        if m:
            note = m.group(2)
            d = re.search(r"Depth=(\d+)", note)
            hdr = re.search(r"Header=BB(\d+_\d+)", note)
            cur = {"label": m.group(1).replace("%bb.", "bb"), "depth": int(d.group(1)) if d else 0,
                   "header": ("BB" + hdr.group(1)) if hdr else None,
                   "is_header": "This Loop Header" in note or "This Inner Loop Header" in note,
                   "lines": []}
            blocks.append(cur)
            continue
        if cur is None:
            cur = {"label": "entry", "depth": 0, "header": None, "is_header": False, "lines": []}
            blocks.append(cur)
        if not cur["lines"] and s.startswith(";") and "Depth" in s:   # the label's comment lines
            d = re.search(r"Depth[= ](\d+)", s)
            if "Child Loop" not in s and d:
                cur["depth"] = max(cur["depth"], int(d.group(1)))
            cur["is_header"] = cur["is_header"] or "Loop Header" in s
            continue
        cur["lines"].append(s)
    return blocks


def is_insn(s):
    return bool(s) and not s.startswith((";", ".")) and re.match(r"^[a-z_0-9]+", s)


def walk(blocks, start_idx):
    """One iteration of the loop whose header block is blocks[start_idx]: the executed lines."""
    label_idx = {b["label"]: i for i, b in enumerate(blocks)}
    header_label = blocks[start_idx]["label"]
    i, out, steps, path = start_idx, [], 0, []
    while True:
        steps += 1
        path.append(blocks[i]["label"])
        assert steps < 10_000, "walk did not end: " + " ".join(path[:60])
        if steps > 1 and i == start_idx:   # back at the header by a latch block
            return out
        b = blocks[i]
        nxt = i + 1
        ended = False
        for s in b["lines"]:
            out.append(s)
            if not is_insn(s):
                continue
            op = s.split()[0]
            if op == "s_branch":
                tgt = s.split()[1]
                if tgt == header_label:
                    ended = True
                else:
                    nxt = label_idx[tgt]
                break
            if op.startswith("s_cbranch_"):
                tgt = s.split()[1]
                if tgt == header_label:   # conditional back edge (rotated loop): the iteration ends
                    ended = True
                    break
                if op == "s_cbranch_execz":
                    if take_uniform(blocks, i, label_idx[tgt]):   # a divergent rare tail: no lane enters
                        nxt = label_idx[tgt]
                        break
                    continue
                if op == "s_cbranch_execnz":
                    nxt = label_idx[tgt]
                    break
                if take_uniform(blocks, i, label_idx[tgt]):
                    nxt = label_idx[tgt]
                    break
        if ended:
            return out
        i = nxt


ARMS = set()   # the live sides of runtime branches named by PBN_ISA_ARM (main: --arms)


def arms_in(blocks):
    return {re.search(r"@arm (\w+)", s).group(1) for b in blocks for s in b["lines"] if "@arm" in s}


def take_uniform(blocks, i, t):
    """A uniform branch from block i to block t: by the PBN_ISA_ARM names first (taken into a
    live arm, or over dead arms only), else taken iff the code it skips (blocks i+1 .. t-1, a
    forward branch) enters an inner loop or holds a launch-anatomy stamp only."""
    if blocks[t]["depth"] == 0:   # a loop exit: the walked iteration does not leave the loop
        return False
    head = [s for s in blocks[t]["lines"] if "@arm" in s][:1]   # (code sunk into an arm may precede its mark)
    if head:
        return re.search(r"@arm (\w+)", head[0]).group(1) in ARMS
    if t > i:
        named = arms_in(blocks[i + 1:t])
        if named & ARMS:
            return False
        if named:
            return True
    if t > i:
        skipped = blocks[i + 1:t]
    else:   # a join placed above (the listing's last tail): the loop's blocks below this one
        skipped = []
        for b in blocks[i + 1:]:
            if b["depth"] == 0:
                break
            skipped.append(b)
        if not any(b["depth"] >= 2 for b in skipped):
            return False
    marks = [s for b in skipped for s in b["lines"] if "@mark" in s and "@mark R" not in s]
    if any(b["depth"] >= 2 for b in skipped) and not marks:
        return True
    body = [s for b in skipped for s in b["lines"] if is_insn(s) or "@mark" in s]
    return bool(body) and all("@mark R" in s for s in body)


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def budget(lines, role, per_trip):
    segs, order, cur = {}, [], None
    for s in lines:
        m = re.search(r"@mark (\w+)", s)
        if m and m.group(1) in SEGMENTS[role]:
            cur = m.group(1)
            if cur not in order:
                order.append(cur)
            continue
        if cur is None or not is_insn(s):
            continue
        op = s.split()[0]
        c = segs.setdefault(cur, {"valu": 0, "valu_dpp": 0, "valu_sdwa": 0, "salu": 0, "lds": 0,
                                  "lds_cycles": 0, "vmem": 0, "smem": 0, "waitcnt": 0, "nop": 0,
                                  "branch": 0, "barrier": 0, "other": 0})
        k = classify(op)
        c[k] += 1
        if k == "valu" and "_dpp" in op:
            c["valu_dpp"] += 1
        if k == "valu" and "_sdwa" in op:
            c["valu_sdwa"] += 1
        if k == "lds":
            c["lds_cycles"] += LDS_CYC.get(op, 4)
    rows = []
    for key in order:
        c = {k: v / per_trip for k, v in segs.get(key, {}).items()}
        rows.append({"segment": SEGMENTS[role][key], "mark": key, **c})
    return rows


def pmc_launch(run_dirs, kernel="pbn_rollout_pipe"):
    """Per-launch means of every counter in the PMC passes (run_counter_collection.csv under each
    directory) for the kernel's most common grid, and the mean dispatch duration (ns)."""
    import collections
    import csv
    import glob
    vals, durs, grids = collections.defaultdict(list), [], collections.Counter()
    rows = []
    for d in run_dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if kernel in r["Kernel_Name"]]
    for r in rows:
        grids[r["Grid_Size"]] += 1
    grid = grids.most_common(1)[0][0]
    seen = set()
    for r in rows:
        if r["Grid_Size"] != grid:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (r["Dispatch_Id"], r["Start_Timestamp"])
        if key not in seen:
            seen.add(key)
            durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    out["grid"] = int(grid)
    out["dispatch_ns"] = sorted(durs)[len(durs) // 2]
    return out


def issue_model(grand, pmc, steps_per_launch, n_cus=256, simds=4):
    """What the instruction budget predicts for one launch, next to what it measured.  Per block
    iteration (64 env-steps): VALU issue at 2 cycles per wave-instruction on a SIMD-32
    (MI355X_MICROARCH.md, v_fma_f32 row), spread over the CU's 4 SIMDs; LDS-array cycles on the
    CU's one LDS (the table's cycles per instruction).  The shader clock is GRBM_GUI_ACTIVE / 8 XCDs
    over the dispatch time."""
    blocks = pmc["grid"] // 192
    iters = blocks * (steps_per_launch + 1) / n_cus          # block iterations per CU per launch
    clock_ghz = pmc["GRBM_GUI_ACTIVE"] / 8 / pmc["dispatch_ns"]
    wall = pmc["dispatch_ns"] * clock_ghz                    # cycles per launch
    valu_static = grand["valu"] * iters * n_cus
    valu_meas = pmc.get("SQ_INSTS_VALU", valu_static)
    valu_cyc = 2.0 * valu_meas / (n_cus * simds)             # per SIMD
    lds_cyc = grand["lds_cycles"] * iters                     # per CU
    env_steps = blocks * 64 * steps_per_launch
    pred = {
        "shader_clock_ghz": clock_ghz, "cycles_per_launch": wall,
        "block_iterations_per_cu": iters,
        "valu_static_vs_counter": valu_static / valu_meas if valu_meas else None,
        "valu_issue_cycles_per_simd": valu_cyc, "lds_array_cycles_per_cu": lds_cyc,
        "valu_share": valu_cyc / wall, "lds_share": lds_cyc / wall,
        "cycles_per_block_iteration_per_cu": wall / iters,
        "predicted_env_steps_per_s_serial": env_steps / ((valu_cyc + lds_cyc) / clock_ghz * 1e-9),
        "predicted_env_steps_per_s_overlapped": env_steps / (max(valu_cyc, lds_cyc) / clock_ghz * 1e-9),
        "measured_env_steps_per_s": env_steps / (pmc["dispatch_ns"] * 1e-9),
    }
    if "SQ_INSTS_LDS" in pmc:
        pred["lds_static_vs_counter"] = grand["lds"] * iters * n_cus / pmc["SQ_INSTS_LDS"]
    if "SQ_INSTS_SALU" in pmc:
        pred["salu_static_vs_counter"] = grand["salu"] * iters * n_cus / pmc["SQ_INSTS_SALU"]
    return pred


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", choices=sorted(KERNELS), default="pipe")
    ap.add_argument("--W", type=int, default=1)
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--K", type=int, default=3, help="functions per node at most (pbn28: 3)")
    ap.add_argument("--arms", default="sel_all_calls,hash",
                    help="comma-separated live PBN_ISA_ARM names (pbn28: sel_all_calls, N > 24; hash, an attractor table)")
    ap.add_argument("--pk", type=int, default=1, help="settle kernel: the packed two-node compares (settle_pk)")
    ap.add_argument("--listing", default=None, help="reuse this assembly listing")
    ap.add_argument("--json", default=None)
    ap.add_argument("--pmc", action="append", default=[],
                    help="NAME:STEPS:DIR[,DIR] PMC passes of one shape (tools/gpu_session.sh budget) for the "
                         "issue model; repeatable")
    a = ap.parse_args()
    ARMS.update(x for x in a.arms.split(",") if x)
    inst_fmt, roles_of = KERNELS[a.kernel]
    inst = inst_fmt % {"W": a.W, "B": a.B}
    s_path = a.listing or os.path.join(tempfile.mkdtemp(prefix="isa_budget_"), "kernel.s")
    if not a.listing:
        compile_listing(inst, s_path)
    text = open(s_path).read().splitlines()
    blocks = parse(text)
    want = roles_of(a)
    result = {"kernel": inst, "units": "per block iteration (64 env-steps of the one-update law, or 64 "
              "env-updates of the settle law: both 32-env groups)", "roles": {}}
    for role, v in want.items():
        tags = [i for i, b in enumerate(blocks) for s in b["lines"] if s == ";@loop %s %d" % (role, v)]
        assert tags, (role, v)
        bi = tags[0]
        hdr = blocks[bi]
        while not hdr["is_header"]:   # the loop header holding (or preceding) the tag
            bi -= 1
            hdr = blocks[bi]
        lines = walk(blocks, bi)
        per_trip = sum(1 for s in lines if s == ";@loop %s %d" % (role, v))
        rows = budget(lines, role, per_trip)
        tot = {}
        for r in rows:
            for k, x in r.items():
                if isinstance(x, (int, float)):
                    tot[k] = tot.get(k, 0) + x
        result["roles"][role] = {"variant": v, "steps_per_trip": per_trip, "segments": rows, "total": tot}
    grand = {}
    for r in result["roles"].values():
        for k, x in r["total"].items():
            grand[k] = grand.get(k, 0) + x
    result["block_iteration_total"] = grand
    for spec in a.pmc:
        name, steps, dirs = spec.split(":", 2)
        pmc = pmc_launch(dirs.split(","))
        result.setdefault("issue_model", {})[name] = {"counters_per_launch": pmc,
                                                       **issue_model(grand, pmc, int(steps))}
    txt = json.dumps(result, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt + "\n")
    hdr = "%-11s %-62s %5s %4s %4s %5s %4s %4s %4s %4s %4s %4s" % (
        "role", "segment", "VALU", "dpp", "SALU", "LDS", "ldsc", "VMEM", "SMEM", "wait", "nop", "br")
    print(hdr)
    for role, r in result["roles"].items():
        for row in r["segments"] + [dict(r["total"], segment="TOTAL")]:
            print("%-11s %-62s %5.0f %4.0f %4.0f %5.0f %4.0f %4.0f %4.0f %4.0f %4.0f %4.0f" % (
                role, row["segment"][:62], row.get("valu", 0), row.get("valu_dpp", 0), row.get("salu", 0),
                row.get("lds", 0), row.get("lds_cycles", 0), row.get("vmem", 0), row.get("smem", 0),
                row.get("waitcnt", 0), row.get("nop", 0), row.get("branch", 0)))
    g = grand
    print("block iteration: VALU %.0f  SALU %.0f  LDS %.0f (%.0f LDS-array cycles)  VMEM %.0f" % (
        g.get("valu", 0), g.get("salu", 0), g.get("lds", 0), g.get("lds_cycles", 0), g.get("vmem", 0)))
    for name, m in result.get("issue_model", {}).items():
        print(name, json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in m.items()
                                if k != "counters_per_launch"}))


if __name__ == "__main__":
    sys.exit(main())
