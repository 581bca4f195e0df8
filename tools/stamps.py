"""In-kernel phase clocks of the wave kernel (diagnostic build, never the product).

  python tools/stamps.py --build            # here: builds pbn_rl_amd/libpbn_env_stamps.so
  python tools/stamps.py [--envs 65536]     # on the GPU box

Per wave, lane 0 stamps s_memtime at the phase boundaries of pbn_step_wave; we
report the median / p90 over waves of each phase's cycles and the spread of
wave start times.  Read the shares, not the absolute length (stamps cost ~40
cycles each and fence the schedule).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
STAMP_LIB = os.path.join(ROOT, "pbn_rl_amd", "libpbn_env_stamps.so")
PHASES = ["tables+barrier", "philox", "per-env", "transpose+S", "node eval", "back-transpose", "epilogue"]
ROW = 32   # stamp words per block (pipelined kernel) or per wave (wave kernel), step_kernels.h PBN_PSTAMP


def segments(full, it):
    """Critical-path table of iteration 10 of the pipelined kernel's single-word fast paths, per
    role: cycles of each segment between consecutive stamps (medians over blocks), the role's
    wait at the block barrier, and the share of the iteration each accounts for."""
    import numpy as np
    med = lambda x: int(np.median(x))
    c = lambda i: full[:, i]
    roles = {
        "state": [("slot reads + obs store", 0, 15), ("transpose to planes", 15, 3), ("gathers + mux chains", 3, 12),
                  ("back-transpose", 12, 13), ("epilogue (hash, reward, flags, stores)", 13, 1),
                  ("barrier wait", 1, 2)],
        "env draws": [("draws + LDS reads (this step)", 4, 16), ("ENV Philox call (next step)", 16, 17),
                      ("masks, slot writes, flip-mask store", 17, 5), ("barrier wait", 5, 6)],
        "selection": [("SEL Philox calls (next step)", 8, 18), ("threshold compares + slot writes", 18, 9),
                      ("barrier wait", 9, 10)],
    }
    out = {"iteration_median": med(it)}
    for role, segs in roles.items():
        have = all(np.all(c(a) > 0) and np.all(c(b) > 0) for _, a, b in segs)
        if not have:
            continue
        total = med(c(segs[-1][2]) - c(segs[0][1]))
        rows = {name: {"cycles": med(c(b) - c(a)), "share": round(med(c(b) - c(a)) / max(med(it), 1), 3)}
                for name, a, b in segs}
        out[role] = {"segments": rows, "span_median": total,
                     "accounted": round(sum(r["cycles"] for r in rows.values()) / max(med(it), 1), 3)}
    return out


SETTLE_ROLES = {
    "state": [("plan, slot reads, transpose to bit planes + plane store", 0, 15), ("gathers + mux chains", 15, 3),
              ("back-transpose, perturbed / idle select", 3, 12),
              ("attractor lookup, decision C, epilogue at a step's end, stores", 12, 1), ("barrier wait", 1, 2)],
    "env draws": [("decision C read, plan", 4, 16), ("ENV / SETTLE_ENV call, draws, gaps, flip-mask store", 16, 17),
                  ("slot writes", 17, 5), ("barrier wait", 5, 6)],
    "selection": [("decision C read, plan, SETTLE_SEL calls (4 per env)", 8, 18),
                  ("env-major compares, transposes to planes, slot writes", 18, 9), ("barrier wait", 9, 10)],
}


def settle_segments(full, it):
    """pbn_rollout_settle's per-role segments of iteration kSettleStampIt (step_kernels.h)."""
    import numpy as np
    med = lambda x: int(np.median(x))
    c = lambda i: full[:, i]
    out = {"iteration_median": med(it)}
    for role, segs in SETTLE_ROLES.items():
        ok = np.all([(c(a) > 0) & (c(b) > 0) for _, a, b in segs], axis=0)
        rows = {name: {"cycles": med(c(b)[ok] - c(a)[ok]), "share": round(med(c(b)[ok] - c(a)[ok]) / max(med(it), 1), 3)}
                for name, a, b in segs}
        out[role] = {"segments": rows, "blocks": int(ok.sum())}
    return out


def placement(full, it):
    """Where the pipelined kernel's waves ran (HW_ID/XCC_ID words the stamps build stores at
    kernel start: role 0 in column 14, roles 1, 2 in columns 7, 11): the role mix per SIMD and the
    iteration time of blocks by the heaviest role mix among their waves' SIMDs."""
    import numpy as np
    from collections import Counter
    hw = full[:, [14, 7, 11]].astype(np.uint64)
    lo = (hw & np.uint64(0xFFFFFFFF)).astype(np.int64)
    xcc = ((hw >> np.uint64(32)) & np.uint64(0xF)).astype(np.int64)
    simd = (lo >> 4) & 3
    cu = (lo >> 8) & 15
    sh = (lo >> 12) & 1
    se = (lo >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd          # [blocks, role]
    cukey = key // 4
    mix = {}
    for role in range(3):
        for k in key[:, role]:
            mix.setdefault(int(k), [0, 0, 0])[role] += 1
    comp = Counter(tuple(v) for v in mix.values())
    same_cu = float(np.mean((cukey[:, 0] == cukey[:, 1]) & (cukey[:, 0] == cukey[:, 2])))
    distinct = float(np.mean((key[:, 0] != key[:, 1]) & (key[:, 0] != key[:, 2]) & (key[:, 1] != key[:, 2])))
    # per block: the most selection-heavy SIMD among its three waves
    worst = np.array([max(mix[int(k)][2] for k in key[b]) for b in range(len(key))])
    by_worst = {int(w): {"blocks": int((worst == w).sum()), "iteration_median": int(np.median(it[worst == w]))}
                for w in np.unique(worst)}
    return {"simds_used": len(mix), "cus_used": len(set(int(k) // 4 for k in mix)),
            "role_mix_per_simd (state, env, sel): count": {str(k): v for k, v in comp.most_common(12)},
            "block_waves_same_cu": same_cu, "block_waves_distinct_simds": distinct,
            "by_max_selection_waves_on_a_block_simd": by_worst}


def anatomy(r, n_steps, hw=None):
    """Launch anatomy from the state waves' s_memrealtime stamps (100 MHz): entry, image in LDS,
    loop start, after iterations 0 and 1, loop end, final stores landed (columns 0..6)."""
    import numpy as np
    us = lambda x: round(float(x) / 100.0, 3)       # 100 MHz ticks -> us
    med = lambda x: us(np.median(x))
    t0 = r[:, 0].min()
    return {"clock": "s_memrealtime, 100 MHz", "blocks": int(len(r)),
            "entry_spread_us": us(r[:, 0].max() - t0),
            "image_us": med(r[:, 1] - r[:, 0]), "digit_masks_us": med(r[:, 2] - r[:, 1]),
            "iteration0_us": med(r[:, 3] - r[:, 2]), "iteration1_us": med(r[:, 4] - r[:, 3]),
            "loop_us": med(r[:, 5] - r[:, 2]), "per_iteration_us": round(float(np.median(r[:, 5] - r[:, 2])) / 100.0 / (n_steps + 1), 4),
            "final_stores_us": med(r[:, 6] - r[:, 5]),
            "first_entry_to_last_exit_us": us(r[:, 6].max() - t0),
            "loop_start_spread_us": us(r[:, 2].max() - r[:, 2].min()),
            "last_loop_end_minus_first_us": us(r[:, 5].max() - r[:, 5].min()),
            "loop_us_pcts": {p: us(np.percentile(r[:, 5] - r[:, 2], p)) for p in (0, 10, 50, 90, 99, 100)},
            "by_xcc": None if hw is None else {
                int(x): {"blocks": int((xcc == x).sum()), "loop_us_median": med((r[:, 5] - r[:, 2])[xcc == x]),
                         "loop_us_max": us(((r[:, 5] - r[:, 2])[xcc == x]).max()),
                         "loop_end_max_us": us((r[:, 5][xcc == x]).max() - t0)}
                for xcc in [(hw.astype(np.uint64) >> np.uint64(32)).astype(np.int64) & 0xF] for x in np.unique(xcc)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--pipe", action="store_true", help="pipelined rollout kernel: per-role clocks of iteration 10")
    ap.add_argument("--plane", action="store_true", help="plane-resident rollout kernel (4 roles; implies --pipe)")
    ap.add_argument("--lib", default=STAMP_LIB, help="a stamps build (default: the one --build makes)")
    ap.add_argument("--settle", type=int, default=0,
                    help="the settle law with this cap (pbn_rollout_settle; implies --pipe): per-role segments of "
                         "iteration kSettleStampIt")
    ap.add_argument("--rollout", type=int, default=0,
                    help="stamp a pbn_rollout launch of this many steps (phases of its last step)")
    args = ap.parse_args()
    if args.build:
        from pbn_rl_amd import _lib
        _lib.build(out=STAMP_LIB, defines=["PBN_STAMPS"], verbose=True)
        return
    os.environ["PBN_LIB"] = args.lib
    if args.plane or args.pipe:
        os.environ["PBN_ROLL"] = "plane" if args.plane else "pipe"
    import numpy as np
    import torch

    from pbn_rl_amd import _lib
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    L = _lib.load()
    L.pbn_debug_set_stamps.argtypes = [ctypes.c_void_p]
    if args.settle:
        args.pipe = True
    spec = EnvSpec(load_network(args.network), load_attractors(args.network), settle=args.settle)
    env = VectorPBNEnv(spec, args.envs, seed=1, keep_final_state=False)
    env.reset()
    waves = env.n_alloc // 32
    buf = torch.zeros(waves * ROW, dtype=torch.int64, device="cuda")
    for _ in range(10):
        env.step_flipmask(random_actions=True)
    torch.cuda.synchronize()
    out = env.rollout(args.rollout) if args.rollout else None
    torch.cuda.synchronize()
    L.pbn_debug_set_stamps(buf.data_ptr())
    if args.rollout:
        env.rollout(args.rollout, out=out)
    else:
        env.step_flipmask(random_actions=True)
    torch.cuda.synchronize()
    L.pbn_debug_set_stamps(None)
    if args.pipe or args.plane:
        waves = (waves + 1) // 2   # one block per pair of groups
        nr = 4 if args.plane else 3
        t = buf.view(-1, ROW)[:waves, :4 * nr].cpu().numpy().astype(np.int64).reshape(waves, nr, 4)[:, :, :3]
        rep = {"envs": args.envs, "blocks": waves, "rollout_steps": args.rollout}
        names = ["state", "env draws", "selection", "planes+outputs"][:nr]
        for role, name in enumerate(names):
            work = t[:, role, 1] - t[:, role, 0]
            wait = t[:, role, 2] - t[:, role, 1]
            rep[name] = {"work_median": int(np.median(work)), "work_p90": int(np.percentile(work, 90)),
                         "barrier_wait_median": int(np.median(wait))}
        full = buf.view(-1, ROW)[:waves].cpu().numpy().astype(np.int64)
        st0 = full[:, 0]
        if args.settle:
            ok = (t[:, :, 2] > 0).all(axis=1)
            it = t[ok][:, :, 2].max(axis=1) - t[ok][:, :, 0].min(axis=1)
            rep["settle_max"] = args.settle
            rep["iteration_median"] = int(np.median(it))
            rep["critical_path"] = settle_segments(full[ok], it)
            print(json.dumps(rep, indent=1))
            return
        if args.plane:
            it = t[:, :, 2].max(axis=1) - t[:, :, 0].min(axis=1)
            rep["iteration_median"] = int(np.median(it))
            print(json.dumps(rep, indent=1))
            return
        rep["state_phases"] = {
            "slot+transpose": int(np.median(full[:, 3] - st0)),
            "node eval": int(np.median(full[:, 12] - full[:, 3])),
            "back-transpose": int(np.median(full[:, 13] - full[:, 12])),
            "epilogue": int(np.median(full[:, 1] - full[:, 13]))}
        it = t[:, :, 2].max(axis=1) - t[:, :, 0].min(axis=1)
        rep["iteration_median"] = int(np.median(it))
        rep["critical_path"] = segments(full, it)
        rep["placement"] = placement(full, it)
        if args.rollout:
            rep["anatomy"] = anatomy(buf.view(-1, ROW)[waves:2 * waves, :7].cpu().numpy().astype(np.int64),
                                     args.rollout, full[:, 14])
        print(json.dumps(rep, indent=1))
        return
    t = buf.view(waves, ROW)[:, :8].cpu().numpy().astype(np.int64)
    d = np.diff(t, axis=1)
    rep = {"envs": args.envs, "waves": waves, "rollout_steps": args.rollout,
           "start_spread_cycles": int(t[:, 0].max() - t[:, 0].min()),
           "kernel_span_cycles": int(t[:, 7].max() - t[:, 0].min()),
           "wave_total_median": int(np.median(t[:, 7] - t[:, 0])),
           "phases": {PHASES[k]: {"median": int(np.median(d[:, k])), "p90": int(np.percentile(d[:, k], 90))}
                      for k in range(7)}}
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
