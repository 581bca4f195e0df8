"""Export a trained reference agent -> tests/golden/<model>_bdq_final.npz (fp32 tensors).

    python tools/export_agent.py pbn7 bb33 pbn10     (build container only: reads /root/reference)

models/<model>/bdq_final.pt is the BranchingDQN state dict the reference saves at the end of
training (bdq_model/__init__.py:237,240-244) and model_tester.py:548-549 evaluates.  It is
loaded with torch.load(weights_only=True) (tensors only, nothing executed) and the ``q.``
network's tensors are written under their BranchingQNetwork names, so that the GPU box (which
has no /root/reference) can rebuild the agent.  The law pins replay model_tester.py:587-658
with them (tests/test_law_pin.py, tests/test_bn_pin.py, tests/test_gpu_law_pin.py).
"""
import os
import sys

import numpy as np
import torch

REF = "/root/reference"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def export(model: str) -> str:
    sd = torch.load(os.path.join(REF, "models", model, "bdq_final.pt"), map_location="cpu", weights_only=True)
    q = {k[2:]: v.detach().to(torch.float32).numpy() for k, v in sd.items() if k.startswith("q.")}
    out = os.path.join(GOLD, f"{model}_bdq_final.npz")
    np.savez_compressed(out, **q)
    print("wrote", out, sum(v.size for v in q.values()), "floats")
    return out


if __name__ == "__main__":
    for m in sys.argv[1:] or ["pbn7"]:
        export(m)
