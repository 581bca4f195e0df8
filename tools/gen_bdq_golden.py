"""Generate tests/golden/bdq_forward.npz: reference BranchingQNetwork outputs (config 5, row A10).

  python tools/gen_bdq_golden.py       (build container only: reads /root/reference)

The reference module is imported from its own file, bdq_model/network.py (the package
__init__ imports the absent gym, so only this file is loaded, by path).  Two cases:
  formula  -- Bittner-28 shape ((28, 28), 29, 3) with pbn_rl_amd.agent.formula_weights
              parameters, 96 seeded binary (state, target) inputs;
  pbn7     -- the reference's trained checkpoint models/pbn7/bdq_final.pt (q network, loaded
              with weights_only=True), 96 seeded binary inputs.  The test re-loads the checkpoint
              from /root/reference, so it runs only where the reference is present.
Stored: inputs (uint8), reference outputs (float32).
"""
import importlib.util
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)

from pbn_rl_amd.agent import formula_weights  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(ROOT, "tests", "golden", "bdq_forward.npz")


def ref_network_module():
    spec = importlib.util.spec_from_file_location("ref_bdq_network", os.path.join(REF, "bdq_model", "network.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    mod = ref_network_module()
    rng = np.random.default_rng(20241016)
    out = {}
    with torch.no_grad():
        net = mod.BranchingQNetwork((28, 28), 29, 3)
        formula_weights(net)
        x = rng.integers(0, 2, size=(2, 96, 28), dtype=np.uint8)
        out["formula_x"] = x
        out["formula_q"] = net(torch.from_numpy(x.astype(np.float32))).numpy()
        net7 = mod.BranchingQNetwork((7, 7), 8, 3)
        sd = torch.load(os.path.join(REF, "models", "pbn7", "bdq_final.pt"), map_location="cpu", weights_only=True)
        net7.load_state_dict({k[2:]: v for k, v in sd.items() if k.startswith("q.")})
        x7 = rng.integers(0, 2, size=(2, 96, 7), dtype=np.uint8)
        out["pbn7_x"] = x7
        out["pbn7_q"] = net7(torch.from_numpy(x7.astype(np.float32))).numpy()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
