"""Load the committed golden fixtures (tests/golden/*.npz) as torch tensors."""
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def weights(z, prefix="w:", dtype=torch.float32):
    """Weights are stored as raw bf16 bits (int16)."""
    out = {}
    for k in z.files:
        if k.startswith(prefix):
            out[k[len(prefix):]] = torch.from_numpy(z[k].copy()).view(torch.bfloat16).to(dtype)
    return out


def t(z, key, dtype=torch.float32):
    return torch.from_numpy(z[key].copy()).to(dtype)


DT = {"f32": torch.float32, "bf16": torch.bfloat16}
