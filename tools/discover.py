"""Discover a network's attractors on the GPU and write them as a networks/*_attractors.json-style file.

  python tools/discover.py pbn28 [--chains 65536 --burn-in 1000 --window 64] [--out gpurun_out/pbn28_discovered.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from pbn_rl_amd.discovery import discover_attractors  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("network")
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--burn-in", type=int, default=1000)
    ap.add_argument("--window", type=int, default=64)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    net = load_network(args.network)
    t0 = time.perf_counter()
    atts = discover_attractors(net, chains=args.chains, burn_in=args.burn_in, window=args.window, seed=args.seed)
    el = time.perf_counter() - t0
    obj = {"network": args.network, "method": "pbn_rl_amd.discovery.discover_attractors",
           "chains": args.chains, "burn_in": args.burn_in, "window": args.window, "seed": args.seed,
           "seconds": el, "sizes": [len(a) for a in atts], "attractors": [[list(s) for s in a] for a in atts]}
    out = args.out or os.path.join("gpurun_out", f"{args.network}_discovered.json")
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(obj, f)
    print(json.dumps({k: v for k, v in obj.items() if k != "attractors"}))


if __name__ == "__main__":
    main()
