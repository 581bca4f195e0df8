"""In-kernel phase clocks of config 5's Q-network launch (diagnostic build, never the product).

  python tools/stamps.py --build              # here: builds pbn_rl_amd/libpbn_env_stamps.so (-DPBN_STAMPS)
  python tools/qnet_stamps.py [--envs 32768]  # on the GPU box

Runs BatchedBDQ frames (bench.py --workload bdq's network and env) on the stamps build and reads
the s_memtime clocks lane 0 of every wave of qnet_tail_kernel stores (pbn_qnet.hip PBN_QSTAMP):
entry, block sort, bilinear layer, then per weight stage the MFMA body and the stage's LDS store +
barrier.  Prints one JSON object: median cycles of each phase over the waves and each phase's
share of the median wave's span.  Read the shares: the stamps fence the schedule.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
STAMP_LIB = os.path.join(ROOT, "pbn_rl_amd", "libpbn_env_stamps.so")
ROW = 64   # kQStampRow


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--network", default="pbn28")
    ap.add_argument("--frames", type=int, default=5)
    args = ap.parse_args()
    os.environ["PBN_LIB"] = STAMP_LIB
    import numpy as np
    import torch

    from pbn_rl_amd import _lib
    from pbn_rl_amd.agent import BatchedBDQ, BranchingQNetwork
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    dev = torch.device("cuda", 0)
    spec = EnvSpec(load_network(args.network), load_attractors(args.network), perturbation=0.01, prob_bits=16,
                   horizon=20, settle=0)
    env = VectorPBNEnv(spec, args.envs, seed=0, device=dev)
    env.reset()
    torch.manual_seed(0)
    agent = BatchedBDQ(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3), epsilon=0.0)
    for _ in range(args.frames):
        agent.step()
    torch.cuda.synchronize()
    L = _lib.load()
    L.pbn_debug_set_qnet_stamps.argtypes = [ctypes.c_void_p]
    waves = args.envs // 16
    buf = torch.zeros(waves * ROW, dtype=torch.int64, device=dev)
    L.pbn_debug_set_qnet_stamps(buf.data_ptr())
    agent.step()
    torch.cuda.synchronize()
    L.pbn_debug_set_qnet_stamps(None)
    s = buf.view(waves, ROW).cpu().numpy().astype(np.int64)
    sub = [57, 58, 59, 60, 61, 62]   # the sort's inner clocks (pbn_qnet.hip PBN_QSTAMP 57-62)
    sort_detail = {}
    if all(np.all(s[:, i] > 0) for i in sub):
        names = ["keys loaded", "barrier", "ballot ranks", "barrier", "chunk prefixes + barrier",
                 "key prefix + barrier", "permutation + barrier"]
        pts = [0] + sub + [1]
        sort_detail = {names[j]: int(np.median(s[:, pts[j + 1]] - s[:, pts[j]])) for j in range(len(pts) - 1)}
    used = [i for i in range(ROW) if np.all(s[:, i] > 0) and i not in sub]
    n_stages = (max(used) - 3) // 3
    med = lambda x: int(np.median(x))
    span = s[:, max(used)] - s[:, 0]
    phases = {"sort": (0, 1), "bilinear": (1, 2), "stage 0 barrier": (2, 3)}
    for st in range(n_stages):
        phases[f"stage {st} body"] = (4 + 3 * st, 5 + 3 * st)
        phases[f"stage {st} store+barrier"] = (5 + 3 * st, 6 + 3 * st)
        if st + 1 < n_stages:
            phases[f"stage {st + 1} fetch issue"] = (6 + 3 * st, 4 + 3 * (st + 1))
    out = {"envs": args.envs, "waves": waves, "n_stages": n_stages, "span_median": med(span),
           "start_spread": med(s[:, 0] - s[:, 0].min()),
           "phases": {k: {"cycles": med(s[:, b] - s[:, a]), "share": round(med(s[:, b] - s[:, a]) / med(span), 3)}
                      for k, (a, b) in phases.items()}}
    tot = {"bodies": sum(v["cycles"] for k, v in out["phases"].items() if k.endswith("body")),
           "store+barrier": sum(v["cycles"] for k, v in out["phases"].items() if k.endswith("barrier")),
           "fetch issue": sum(v["cycles"] for k, v in out["phases"].items() if k.endswith("issue"))}
    out["totals"] = tot
    out["sort_detail"] = sort_detail
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
