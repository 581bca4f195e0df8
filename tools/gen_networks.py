"""Regenerate pbn_rl_amd/networks/*.json from the reference's ISPL files.

Run in the build container (needs /root/reference):  python tools/gen_networks.py
The JSON keeps the parser output (genes + (expression, weight) lists, exactly
what the reference passes to gym.make("gym-PBN/PBNEnv"), train_assa_BQN.py:121-124)
plus the compiled canonical functions, so the GPU box never reads /root/reference.

Attractor sets written alongside (see pbn_rl_amd/attractors.py for provenance):
  pbn28_attractors.json  14 singleton states, SURVEY.md Appendix B (derived from
                         data/attractors_Bittner-28.pkl, which this round's safe
                         loader refused), packed LSB-first in ISPL node order;
  pbn7/pbn10             exhaustive bottom-SCC search of the STG;
  pbn70                  no fixture exists: 16 seeded random states (seed 70).
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from pbn_rl_amd.attractors import find_attractors, random_state_targets  # noqa: E402
from pbn_rl_amd.network import NETWORK_DIR, Network  # noqa: E402

REF = "/root/reference/kaban"

BITTNER28_HEX = [0xeddf7d7, 0xfddf7d7, 0xefdfdc7, 0xffdfdc7, 0xe7df6fb, 0xe7df6ff, 0xe7dfceb,
                 0xf7dfceb, 0xe7dfcef, 0xf7dfcef, 0xe7dfeeb, 0xf7dfeeb, 0xe7dfeef, 0xf7dfeef]


def main():
    os.makedirs(NETWORK_DIR, exist_ok=True)
    for name in ["pbn7", "pbn10", "pbn28", "pbn70"]:
        net = Network.from_ispl(os.path.join(REF, f"{name}.ispl"), name=name)
        obj = net.to_json()
        obj["source"] = f"kaban/{name}.ispl of jakub-zarzycki2022/pbn-rl, parsed by pbn_rl_amd.ispl"
        with open(os.path.join(NETWORK_DIR, f"{name}.json"), "w") as f:
            json.dump(obj, f, indent=1)
        if name == "pbn28":
            atts = [[tuple(net.unpack([h]))] for h in BITTNER28_HEX]
            src = "SURVEY.md Appendix B (data/attractors_Bittner-28.pkl, numeric-ID permutation)"
        elif name == "pbn70":
            atts = random_state_targets(net.n, 16, seed=70)
            src = "no fixture in the reference: 16 seeded random states (numpy default_rng(70))"
        else:
            atts = find_attractors(net)
            src = "exhaustive bottom-SCC search of the synchronous STG (print_graph.py:15-34 definition)"
        with open(os.path.join(NETWORK_DIR, f"{name}_attractors.json"), "w") as f:
            json.dump({"network": name, "source": src,
                       "attractors": [["".join(str(b) for b in s) for s in a] for a in atts]}, f, indent=1)
        print(name, net.n, "nodes,", len(atts), "attractors")


if __name__ == "__main__":
    main()
