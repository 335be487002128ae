#!/usr/bin/env python3
"""Dump the inputs and the HIP gradient of tests/test_loss_fusion_gpu.py::test_loss_near_convergence_vs_fp64_oracle
[separate] (field E, target, loss, dL/dE, the loss statistics) to gpurun_out/diag_loss.npz, for an fp64 analysis on
the CPU of where the fp32 gradient departs from the fp64 one."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from quantizationawarethzdoe_amd import optics, propagation as P  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(8)
shape = (2, 1, 100, 100)
x = (torch.randn(shape, generator=g) + 1j * torch.randn(shape, generator=g)).to(torch.complex64)
wl, sp, z = [2.998e8 / 300e9], (1e-3, 1e-3), 0.12
ph, pw = P.asm_padding(100, 100, (2, 2))
with torch.no_grad():
    E = P.asm_propagate(x.to(dev), wl, sp, [z], ph, pw)[0]
    I = E.abs().double() ** 2
    I = I / I.amax(dim=(1, 2, 3), keepdim=True)
    tgt = (I * (1 + 1e-4 * torch.randn(I.shape, generator=g).to(dev).double())).float()
Ed = E.clone().requires_grad_(True)
loss = optics.intensity_mse(Ed, tgt)
loss.backward()
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/diag_loss.npz", E=E.cpu().numpy(), tgt=tgt.cpu().numpy(), loss=float(loss.detach()),
         gx=Ed.grad.cpu().numpy(), wl=np.array(wl))
print("loss", float(loss.detach()))
