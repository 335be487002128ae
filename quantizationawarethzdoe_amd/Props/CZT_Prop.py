"""Chirp-z (Bluestein) propagation, CZT_prop / VCZT_prop -- drop-in for Props/CZT_Prop.py.

Same constructor (``z_distance, device``; :13-30), ``z`` property (:32-42) and
``forward(field, outputHeight, outputWidth, outputPixel_dx, outputPixel_dy)`` with the same
defaults (output grid = input grid, :280-290) returning a new ElectricField with spacing
[outputPixel_dx, outputPixel_dy] (:308-312).  The data layout of the result is the
reference's [B, C, outW, outH] (square outputs only, as the reference's F0 broadcast at :248
requires; a non-square request raises).  The per-call debug prints of the reference
(:167-176, :217) are not reproduced.  The math runs in libthzdoe's gfx950 kernels
(thz_czt.hip), with the chirp tables generated in double precision on the device; backward runs
the adjoint kernels.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
from quantizationawarethzdoe_amd import propagation as _prop


def _f(v):
    return float(v.detach().cpu()) if torch.is_tensor(v) else float(v)


def _pow2(n):
    return n > 0 and n & (n - 1) == 0


class CZT_prop(nn.Module):
    def __init__(self, z_distance: float = 0.0, device: str = None) -> None:
        super().__init__()
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self._z = torch.tensor(z_distance, device=self.device)
        self._zh = _f(z_distance)

    @property
    def z(self):
        return self._z

    @z.setter
    def z(self, z) -> None:
        if isinstance(z, torch.Tensor) and z.device != torch.device(self.device):
            z = z.to(self.device)
        self._z = z
        self._zh = _f(z)

    @staticmethod
    def compute_np2(x):
        """2**ceil(log2 x) (Props/CZT_Prop.py:120-130)."""
        import numpy as np
        return 2 ** (np.ceil(np.log2(x))).astype(int)

    def RS_kernel(self, z, meshx, meshy, wavelengths):
        """exp(ikr) z / (2 pi r^2) (1/r - ik) on the meshes, [1, C, *mesh] (Props/CZT_Prop.py:44-57),
        evaluated by the HIP kernel thz_rs_kernel (the same device function the CZT passes apply)."""
        return _prop.rs_kernel(meshx, meshy, _f(z), [_f(v) for v in torch.as_tensor(wavelengths).reshape(-1)])

    def build_CZT_grid(self, z, wavelengths, InputHeight, InputWidth, InputPixel_dx, InputPixel_dy,
                       outputHeight, outputWidth, outputPixel_dx, outputPixel_dy):
        """Input / output meshes (linspace(-N d/2, N d/2, N), meshgrid 'ij'), Dm = lambda z / dx_in
        and the zoom ranges f1 = x_out[0] + Dm/2, f2 = x_out[-1] + Dm/2 of both axes
        (Props/CZT_Prop.py:62-118); returns (Inmeshx, Inmeshy, Outmeshx, Outmeshy, Dm, fx_1, fx_2,
        fy_1, fy_2) with Dm and the f's shaped [1, C, 1, 1].  The kernels form these per element
        (thz_czt.hip); this is the reference's grid API for callers that inspect it."""
        dev = self.device

        def grid(n, d):
            e = torch.as_tensor(n * d, dtype=torch.float32) / 2
            return torch.linspace(float(-e), float(e), int(n), device=dev)

        x_in, y_in = grid(InputHeight, InputPixel_dx), grid(InputWidth, InputPixel_dy)
        x_out, y_out = grid(outputHeight, outputPixel_dx), grid(outputWidth, outputPixel_dy)
        Inmeshx, Inmeshy = torch.meshgrid(x_in, y_in, indexing="ij")
        Outmeshx, Outmeshy = torch.meshgrid(x_out, y_out, indexing="ij")
        lam = torch.as_tensor(wavelengths, device=dev).reshape(1, -1, 1, 1)
        Dm = lam * torch.as_tensor(z, device=dev) / torch.as_tensor(InputPixel_dx, device=dev)
        return (Inmeshx, Inmeshy, Outmeshx, Outmeshy, Dm, x_out[0] + Dm / 2, x_out[-1] + Dm / 2,
                y_out[0] + Dm / 2, y_out[-1] + Dm / 2)

    def forward(self, field: ElectricField, outputHeight=None, outputWidth=None, outputPixel_dx=None,
                outputPixel_dy=None) -> ElectricField:
        sp = field.spacing_host
        H, W = field.height, field.width
        outputHeight = H if outputHeight is None else int(outputHeight)
        outputWidth = W if outputWidth is None else int(outputWidth)
        odx = sp[0] if outputPixel_dx is None else _f(outputPixel_dx)
        ody = sp[1] if outputPixel_dy is None else _f(outputPixel_dy)
        data = field.data
        x = _prop.kernel_dtype(data, "CZT_prop", field.wavelengths)
        if outputHeight == outputWidth == 1 and _pow2(W) and not _pow2(H):
            # the reference's second Bluestein pass (m = W, M = 1) has np2 = mp = W: its kept
            # slice b[W:W+1] is empty and it returns a [B, C, 1, 0] field (Props/CZT_Prop.py:206,211;
            # run here).  Every other power-of-two Bluestein length raises there, and the library
            # refuses it (THZ_E_ARG -> RuntimeError).
            # (kept in the autograd graph as the reference's slice is: a zero gradient flows back)
            out = x.new_zeros(x.shape[0], x.shape[1], 1, 0) + 0 * x.sum((-2, -1), keepdim=True)[..., :0]
        else:
            out = _CztFunction.apply(x, tuple(field.wavelengths_host), tuple(sp), self._zh, outputHeight,
                                     outputWidth, odx, ody)
        sp_out = [outputPixel_dx if outputPixel_dx is not None else field.spacing[0],
                  outputPixel_dy if outputPixel_dy is not None else field.spacing[1]]
        if all(torch.is_tensor(v) for v in sp_out):
            sp_out = torch.stack([v.detach().reshape(()) for v in sp_out])
        else:
            sp_out = [_f(v) for v in sp_out]
        return ElectricField(data=out, wavelengths=field.wavelengths, spacing=sp_out, device=field.device)


class _CztFunction(torch.autograd.Function):
    """Forward and adjoint (conjugated chirps, filter and RS kernels, passes reversed) on the
    HIP Bluestein kernels."""

    @staticmethod
    def forward(ctx, data, wavelengths, spacing, z, outH, outW, odx, ody):
        ctx.cfg = (wavelengths, spacing, z, outH, outW, odx, ody, tuple(data.shape))
        return _prop.czt_apply(data, wavelengths, spacing, z, outH, outW, odx, ody)

    @staticmethod
    def backward(ctx, g):
        wavelengths, spacing, z, outH, outW, odx, ody, shape = ctx.cfg
        gin = _prop.czt_apply(g.contiguous(), wavelengths, spacing, z, outH, outW, odx, ody, adjoint=True,
                              field_hw=shape[-2:])
        return gin, None, None, None, None, None, None, None


class VCZT_prop(CZT_prop):
    """Alias of CZT_prop with its own z property (Props/CZT_Prop.py:317-348)."""
