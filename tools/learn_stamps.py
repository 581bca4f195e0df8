"""In-kernel phase clocks of the fused BDQ update (diagnostic build, never the product).

  python tools/stamps.py --build                  # here: builds pbn_rl_amd/libpbn_env_stamps.so (-DPBN_STAMPS)
  python tools/learn_stamps.py [--envs 32768]     # on the GPU box

Runs eager BDQ training frames (bench.py --workload bdq-learn's learner) on the stamps build and
reads the s_memtime clocks lane 0 of every wave stores in learn_fwd / learn_bwd / learn_apply
(pbn_learn.hip PBN_LSTAMP), plus each wave's s_memrealtime at entry.  Prints one JSON object: per
kernel, the median cycles from entry to every numbered point over the waves that reached it, and
the spread of the blocks' entry times (100 MHz ticks).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
STAMP_LIB = os.path.join(ROOT, "pbn_rl_amd", "libpbn_env_stamps.so")
ROW, BLOCKS, WAVES = 32, 1024, 8
POINTS = {
    "fwd": ["entry", "rows", "bilinear", "bilinear_sync", "L2", "L2_sync", "L3_sync", "L4_sync", "H1_sync", "end"],
    "bwd": ["entry", "frags_issued", "td_loaded", "td_done", "td_sync", "H2", "H2_sync", "H1_sync", "L3_sync", "end",
            "td_sums", "td_argmax"],
    "apply": ["entry", "bil_loop", "bil_adam", "bil_table", "dense_loop", "dense_end"],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--lib", default=STAMP_LIB, help="a stamps build (default: tools/stamps.py --build's)")
    args = ap.parse_args()
    os.environ["PBN_LIB"] = args.lib
    import numpy as np
    import torch

    from pbn_rl_amd import _lib
    from pbn_rl_amd.agent import BranchingQNetwork
    from pbn_rl_amd.attractors import load_attractors
    from pbn_rl_amd.network import load_network
    from pbn_rl_amd.replay import BDQLearner
    from pbn_rl_amd.spec import EnvSpec
    from pbn_rl_amd.vector_env import VectorPBNEnv

    dev = torch.device("cuda", 0)
    spec = EnvSpec(load_network("pbn28"), load_attractors("pbn28"), perturbation=0.01, prob_bits=16, horizon=20)
    env = VectorPBNEnv(spec, args.envs, seed=0, device=dev, keep_final_state=True)
    env.reset()
    torch.manual_seed(0)
    learner = BDQLearner(env, BranchingQNetwork((spec.n, spec.n), spec.n + 1, 3), capacity=4 * args.envs,
                         learning_starts=256, epsilon_start=0.0, epsilon_final=0.0)
    for _ in range(args.frames):
        learner.frame()
    torch.cuda.synchronize()
    L = _lib.load()
    L.pbn_debug_set_learn_stamps.argtypes = [ctypes.c_void_p]
    buf = torch.zeros(3 * BLOCKS * WAVES * ROW, dtype=torch.int64, device=dev)
    L.pbn_debug_set_learn_stamps(buf.data_ptr())
    learner.frame()
    torch.cuda.synchronize()
    L.pbn_debug_set_learn_stamps(None)
    s = buf.view(3, BLOCKS, WAVES, ROW).cpu().numpy().astype(np.int64)
    out = {"envs": args.envs, "batch": learner.batch_size, "unit": "s_memtime cycles from the wave's entry"}
    for k, name in enumerate(("fwd", "bwd", "apply")):
        st = s[k]
        live = st[:, :, 0] != 0
        rt = st[:, :, 31][live]
        res = {"waves": int(live.sum()), "entry_spread_ticks_100MHz": int(rt.max() - rt.min()) if rt.size else 0}
        for i, p in enumerate(POINTS[name]):
            if i == 0:
                continue
            ok = live & (st[:, :, i] != 0)
            if ok.any():
                d = (st[:, :, i] - st[:, :, 0])[ok]
                res[p] = {"median": int(np.median(d)), "max": int(d.max()), "waves": int(ok.sum())}
        out[name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
