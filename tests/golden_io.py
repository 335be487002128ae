"""Load the committed golden fixtures (produced by tests/golden/gen_golden.py)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
C0 = 2.998e8
MM = 1e-3


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as fh:
        return json.load(fh)


_CACHE = {}


def arrays(name):
    if name not in _CACHE:
        with np.load(os.path.join(GOLDEN, f"{name}_golden.npz"), allow_pickle=False) as z:
            _CACHE[name] = {k: z[k] for k in z.files}
    return _CACHE[name]


def wavelengths(freqs_ghz, f64=False):
    """The fp32-rounded wavelengths ElectricField makes from floats (DataType/ElectricField.py:85-90)."""
    w = torch.tensor([C0 / (g * 1e9) for g in freqs_ghz], dtype=torch.float32)
    return w.double() if f64 else w


def spacing(dx_mm, dy_mm, f64=False):
    s = torch.tensor([dx_mm * MM, dy_mm * MM], dtype=torch.float32)
    return s.double() if f64 else s


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.complex128)
    b = np.asarray(b, dtype=np.complex128)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
