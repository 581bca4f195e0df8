"""Export the reference's trained pbn7 agent -> tests/golden/pbn7_bdq_final.npz (fp32 tensors).

    python tools/export_pbn7_agent.py      (build container only: reads /root/reference)

models/pbn7/bdq_final.pt is the BranchingDQN state dict the reference saves at the end of
training (bdq_model/__init__.py:237,240-244) and model_tester.py:548-549 evaluates.  It is
loaded with torch.load(weights_only=True) (tensors only, nothing executed) and the ``q.``
network's tensors are written under their BranchingQNetwork names, so that the GPU box (which
has no /root/reference) can rebuild the agent: the parity pin of the transition law in
tests/test_law_pin.py and tests/test_gpu_law_pin.py replays model_tester.py:587-648 with it.
"""
import os

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "pbn7_bdq_final.npz")


def main():
    sd = torch.load(os.path.join(REF, "models", "pbn7", "bdq_final.pt"), map_location="cpu", weights_only=True)
    q = {k[2:]: v.detach().to(torch.float32).numpy() for k, v in sd.items() if k.startswith("q.")}
    np.savez_compressed(OUT, **q)
    print("wrote", OUT, sum(v.size for v in q.values()), "floats")


if __name__ == "__main__":
    main()
