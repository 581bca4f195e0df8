"""Regenerate pbn_rl_amd/networks/*.json from the reference's ISPL files.

Run in the build container (needs /root/reference):  python tools/gen_networks.py
The JSON keeps the parser output (genes + (expression, weight) lists, exactly
what the reference passes to gym.make("gym-PBN/PBNEnv"), train_assa_BQN.py:121-124)
plus the compiled canonical functions, so the GPU box never reads /root/reference.

Also bb33 (models/bb33/bb33.ispl, 33 nodes, functions of up to 6 inputs) and the 47-node
inline network of model_tester.py:97-137 (functions of up to 20 inputs, read from the script's
literal lists): the wide-function networks that exercise the gate lowering (lowering.py).

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
    wide = {"bb33": Network.from_ispl("/root/reference/models/bb33/bb33.ispl", name="bb33"),
            "m47": model_tester_network(47)}
    for name, net in wide.items():
        obj = net.to_json()
        obj["source"] = {"bb33": "models/bb33/bb33.ispl of jakub-zarzycki2022/pbn-rl, parsed by pbn_rl_amd.ispl",
                         "m47": "inline 47-node network of model_tester.py:97-137 (its literal gene and "
                                "logic-function lists)"}[name]
        with open(os.path.join(NETWORK_DIR, f"{name}.json"), "w") as f:
            json.dump(obj, f, indent=1)
        atts = random_state_targets(net.n, 8, seed=net.n)
        with open(os.path.join(NETWORK_DIR, f"{name}_attractors.json"), "w") as f:
            json.dump({"network": name, "source": f"no fixture: 8 seeded random states (numpy default_rng({net.n}))",
                       "attractors": [["".join(str(b) for b in s) for s in a] for a in atts]}, f, indent=1)
        print(name, net.n, "nodes, max arity", net.max_arity, ",", len(net.lowered()[0].gates), "gates")


def model_tester_network(n: int) -> Network:
    """The inline gym.make("gym-PBN/PBNEnv", N=n, genes=[...], logic_functions=[...]) of
    model_tester.py, read as literals (ast.literal_eval: nothing is executed)."""
    import ast
    src = open("/root/reference/model_tester.py").read()
    i = src.index(f"N={n}")
    j = src.index("genes=[", i)
    k = src.index("])", src.index("logic_functions=[", j))
    block = src[j:k + 1]
    genes = ast.literal_eval(block[block.index("["):block.index("]") + 1])
    funcs = ast.literal_eval(block[block.index("logic_functions=") + len("logic_functions="):])
    return Network.from_logic_functions(genes, funcs, name=f"m{n}")


if __name__ == "__main__":
    main()
