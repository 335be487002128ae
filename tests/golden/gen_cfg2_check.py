#!/usr/bin/env python3
"""Generate tests/golden/cfg2_check.npz: the REFERENCE's own output on the cfg2 headline workload
(Props/ASM_Prop.py:314-378 on a 4096^2 Gaussian beam, 300 GHz, dx 0.25 mm, padding_scale 1 ->
P = 8192, exact band limit) at the first and the last plane of the bench sweep (z = 20 mm and
120 mm), run in fp64 by the SURVEY.md §8(c) procedure and in fp32 as shipped.

Only a small signature of each 4096^2 plane is kept (bench.py and the GPU tests compare against
it): the energy sum |E|^2, the sub-grid E[::64, ::64] and the full row 2048.  The input is the
oracle's restatement of Guassian_beam (oracle.thz_oracle.gaussian_beam, pinned against the
reference in tests/test_oracle_golden.py) in fp32 -- the beam bench.py generates on the device.

Runs only in the build container (imports /root/reference through ``_refimport``)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_cfg2_check.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from _refimport import import_reference  # noqa: E402

from oracle import thz_oracle as orc  # noqa: E402

C0 = 2.998e8
N, DX, WAIST, FREQ = 4096, 0.25e-3, 50e-3, 300e9
ZS = (20e-3, 120e-3)
SUB = 64
ROW = 2048


def main():
    ref = import_reference()
    torch.set_num_threads(8)
    lam32 = torch.tensor([C0 / FREQ], dtype=torch.float32)
    d = torch.tensor(DX, dtype=torch.float32)
    x = orc.gaussian_beam(N, N, d, d, lam32, WAIST, WAIST).to(torch.complex64)
    arrays = {"lam": lam32.numpy(), "dx": np.float32(DX), "z": np.array(ZS)}
    for f64 in (True, False):
        tag = "64" if f64 else "32"
        old = torch.get_default_dtype()
        torch.set_default_dtype(torch.float64 if f64 else torch.float32)
        try:
            data = x.to(torch.complex128) if f64 else x
            field = ref.ElectricField(data=data, wavelengths=C0 / FREQ, spacing=DX, device="cpu")
            if f64:
                field._wavelengths = field._wavelengths.double()
                field._spacing = field._spacing.double()
            for k, z in enumerate(ZS):
                prop = ref.ASM.ASM_prop(z_distance=z, padding_scale=1, bandlimit_kernel=True,
                                        bandlimit_type="exact", device="cpu")
                with contextlib.redirect_stdout(io.StringIO()):
                    out = prop.forward(field).data.detach()[0, 0].to(torch.complex128).numpy()
                arrays[f"p{k}__energy{tag}"] = np.float64(np.sum(np.abs(out) ** 2))
                arrays[f"p{k}__sub{tag}"] = out[::SUB, ::SUB].copy()
                arrays[f"p{k}__row{tag}"] = out[ROW].copy()
                print(f"z={z} fp{tag}: energy {arrays[f'p{k}__energy{tag}']:.9e}", flush=True)
                del out
        finally:
            torch.set_default_dtype(old)
    np.savez_compressed(os.path.join(HERE, "cfg2_check.npz"), **arrays)


if __name__ == "__main__":
    main()
