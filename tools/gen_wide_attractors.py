"""Regenerate the attractor fixtures of the wide networks (bb33, m47) by GPU discovery
(pbn_rl_amd.discovery: simulation + exact bottom-SCC verification), replacing the seeded random
'synthetic target' states bundled in round 1.  Writes gpurun_out/<name>_attractors.json; copy
into pbn_rl_amd/networks/ after inspection.

    python tools/gen_wide_attractors.py bb33 m47
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pbn_rl_amd.discovery import discover_attractors_escalating  # noqa: E402
from pbn_rl_amd.network import load_network  # noqa: E402


def main(names):
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for name in names:
        net = load_network(name)
        t0 = time.perf_counter()
        atts = discover_attractors_escalating(net, chains=65536, window=64, seed=1)
        el = time.perf_counter() - t0
        obj = {"network": name,
               "source": f"pbn_rl_amd.discovery.discover_attractors_escalating(chains=65536, window=64, seed=1): "
                         f"bottom SCCs of the STG reached by GPU chains, each verified exactly on the host "
                         f"({el:.1f} s on MI355X)",
               "attractors": [["".join(str(b) for b in s) for s in att] for att in atts]}
        path = os.path.join(ROOT, "gpurun_out", f"{name}_attractors.json")
        with open(path, "w") as f:
            json.dump(obj, f, indent=1)
        print(name, len(atts), "attractors, sizes", [len(a) for a in atts][:40], f"{el:.1f}s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["bb33", "m47"])
