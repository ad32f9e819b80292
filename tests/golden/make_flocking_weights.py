"""Regenerate tests/golden/flocking_weights.npz: the reference's ten Flocking checkpoints
(data/models/experiment_Flocking-seed_{0..9}.pth — three GATConvs, hidden 8), flattened in
state_dict order (oracle GAT3_PARAM_ORDER), float32 [10, 409].

Loaded with torch.load(weights_only=True) only.  Run from the repo root in a container that
has the reference checkout:  python tests/golden/make_flocking_weights.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import swarm_oracle as O  # noqa: E402

REF = "/root/reference/data/models"


def main():
    W = []
    for s in range(10):
        sd = torch.load(f"{REF}/experiment_Flocking-seed_{s}.pth", weights_only=True)
        assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, s_) for k, s_ in O.GAT3_PARAM_ORDER]
        W.append(torch.cat([sd[k].reshape(-1).float() for k, _ in O.GAT3_PARAM_ORDER]).numpy())
    out = os.path.join(ROOT, "tests", "golden", "flocking_weights.npz")
    np.savez_compressed(out, weights_flocking=np.stack(W).astype(np.float32))
    print("wrote", out)


if __name__ == "__main__":
    main()
