"""Rayleigh-Sommerfeld convolution, RSC_prop / VRS_prop -- drop-in for Props/RSC_Prop.py.

Same constructor (``z_distance, device``; :17-45), ``z`` property (:47-57),
``compute_padding`` (:60-77, padding scale 1), once-per-instance minimum-distance diagnostic
(:89-127) and ``forward(field) -> ElectricField`` (:170-215, :265-321).  As in the
reference, RSC_prop takes a single field (B == 1, :198-200) and the output window is
ifft2(...)[..., H:, W:] (so an odd N returns N-1 samples, :207); VRS_prop forms Ez from the
field's Ex/Ey planes and returns 3 planes.  One documented difference: where the reference's
diagnostic crashes (z_min1 = 0 is an int without ``.detach``, :112-117) this mirror prints
0.000 mm and continues.  The math runs in libthzdoe's gfx950 kernels (the spatial-kernel
FFT and the convolution passes of thz_asm.hip).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
from quantizationawarethzdoe_amd import propagation as _prop

mm = 1e-3


def _f(v):
    return float(v.detach().cpu()) if torch.is_tensor(v) else float(v)


class RSC_prop(nn.Module):
    _vectorial = False

    def __init__(self, z_distance: float = 0.0, device: str = None) -> None:
        super().__init__()
        self.do_padding = True
        self.DEFAULT_PADDING_SCALE = torch.tensor([1, 1])
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self._z = torch.tensor(z_distance, device=self.device)
        self._zh = _f(z_distance)
        self.shape = None
        self.check_Zc = True

    @property
    def z(self):
        return self._z

    @z.setter
    def z(self, z) -> None:
        if isinstance(z, torch.Tensor) and z.device != torch.device(self.device):
            z = z.to(self.device)
        self._z = z
        self._zh = _f(z)

    def compute_padding(self, H, W, return_size_of_padding=False):
        """Props/RSC_Prop.py:60-77."""
        ph, pw = (int(np.floor(H / 2)), int(np.floor(W / 2))) if self.do_padding else (0, 0)
        if return_size_of_padding:
            return ph, pw
        return H + 2 * ph, W + 2 * pw

    def check_RS_minimum_z(self, quality_factor=1, dx=None, dy=None, wavelength=None, Ph=None):
        """Energy-conservation / sampling minimum distances, printed (Props/RSC_Prop.py:89-127)."""
        f32 = np.float32
        dx, dy, lam = f32(dx), f32(dy), f32(wavelength)
        range_x, range_y = f32(self.shape[-2]) * dx, f32(self.shape[-1]) * dy
        dr = np.sqrt(dx ** 2 + dy ** 2)
        rmax = np.sqrt(range_x ** 2 + range_y ** 2)
        factor = (((f32(quality_factor) * dr + rmax) ** 2 - lam ** 2 - rmax ** 2) / (f32(2) * lam)) ** 2 - rmax ** 2
        z_min1 = np.sqrt(factor) if factor > 0 else f32(0)
        print("Minimum propagation distance to satisfy energy conservation: {:.3f} mm".format(z_min1 / mm))
        with np.errstate(invalid="ignore"):
            z_min2 = f32(Ph) * dx ** 2 / lam * np.sqrt(f32(1) - (lam / (f32(2) * dx)) ** 2)
        print("Minimum propagation distance to satisfy sampling for FT: {:.3f} mm".format(z_min2 / mm))
        if self._zh > min(z_min1, z_min2):
            print("The simulation will be accurate !")
        else:
            print("The propagation distance should be larger than minimum propagation distance to keep "
                  "simulation accurate!")

    def create_spatial_grid(self, H, W, dx, dy):
        """linspace(-N dx/2, N dx/2, N) on both axes WITH dx (Props/RSC_Prop.py:79-87, the
        reference's y grid uses dx too), meshgrid 'ij', on the module's device."""
        def grid(n):
            e = (np.float32(-n) * np.float32(_f(dx))) / np.float32(2), (np.float32(n) * np.float32(_f(dx))) / np.float32(2)
            return torch.linspace(float(e[0]), float(e[1]), int(n))
        meshx, meshy = torch.meshgrid(grid(H), grid(W), indexing="ij")
        return meshx.to(device=self.device), meshy.to(device=self.device)

    def create_kernel(self, field: ElectricField) -> torch.Tensor:
        """The spatial RS kernel exp(ikr) z/(2 pi r^2)(1/r - ik) on the padded grid, [1, C, Ph, Pw]
        (Props/RSC_Prop.py:129-167), with the once-per-instance minimum-distance print.  The
        convolution kernels take FFT2 of the same values in-kernel; this materialises them with
        thz_rs_kernel for inspection and sets ``meshx`` / ``meshy`` as the reference does."""
        B, C, H, W = field.shape
        Ph, Pw = self.compute_padding(H, W)
        sp, wl = field.spacing_host, field.wavelengths_host
        self.meshx, self.meshy = self.create_spatial_grid(Ph, Pw, sp[0], sp[1])
        if self.check_Zc:
            self.shape = field.shape
            self.check_RS_minimum_z(1, sp[0], sp[1], min(wl), Ph=Ph)
            self.check_Zc = False
        return _prop.rs_kernel(self.meshx, self.meshy, self._zh, wl)

    def forward(self, field: ElectricField) -> ElectricField:
        data = field.data
        B, C, H, W = self.shape = data.shape
        if not self._vectorial and B != 1:
            raise RuntimeError(f"RSC_prop convolves a single field (B == 1) as the reference does "
                               f"(Props/RSC_Prop.py:198-200); got B={B}")
        sp = field.spacing_host
        wl = field.wavelengths_host
        if self.check_Zc:
            self.check_RS_minimum_z(1, sp[0], sp[1], min(wl), Ph=H + 2 * (H // 2))
            self.check_Zc = False
        x = _prop.kernel_dtype(data, "RSC_prop", field.wavelengths)
        out = _RscFunction.apply(x, tuple(wl), tuple(sp), self._zh, self._vectorial)
        Eout = ElectricField(data=out, wavelengths=field.wavelengths, spacing=field.spacing, device=field.device)
        return Eout._adopt_host(field)


class VRS_prop(RSC_prop):
    """Vectorial RS: Ez = (Ex x + Ey y) / r, then the scalar convolution per component (:218-321)."""
    _vectorial = True


class _RscFunction(torch.autograd.Function):
    """Forward on the HIP convolution; backward = the adjoint convolution (conj FFT2(K), windows
    exchanged).  VRS: out = [RSC(Ex), RSC(Ey), RSC(Ez)], Ez = Ex x/r + Ey y/r, so
    dEx = RSC^H(g0) + x/r RSC^H(g2) and dEy = RSC^H(g1) + y/r RSC^H(g2) on the unpadded grid."""

    @staticmethod
    def forward(ctx, data, wavelengths, spacing, z, vectorial):
        ctx.cfg = (wavelengths, spacing, z, vectorial, tuple(data.shape))
        return _prop.rsc_apply(data, wavelengths, spacing, z, vectorial)

    @staticmethod
    def backward(ctx, g):
        wavelengths, spacing, z, vectorial, shape = ctx.cfg
        B, C, H, W = shape
        adj = _prop.rsc_apply(g.contiguous(), wavelengths, spacing, z, adjoint=True, field_hw=(H, W))
        if not vectorial:
            return adj, None, None, None, None
        # the Ez grid in the field's precision (fp32 for complex64, fp64 for complex128)
        rdt = torch.float64 if adj.dtype == torch.complex128 else torch.float32
        dx = torch.tensor(spacing[0], dtype=rdt)
        x = torch.linspace(float(-dx * H / 2), float(dx * H / 2), H, device=g.device, dtype=rdt)
        y = torch.linspace(float(-dx * W / 2), float(dx * W / 2), W, device=g.device, dtype=rdt)
        X, Y = torch.meshgrid(x, y, indexing="ij")
        r = torch.sqrt(X ** 2 + Y ** 2 + torch.tensor(z, dtype=rdt) ** 2)
        gin = torch.zeros(shape, dtype=adj.dtype, device=g.device)
        gin[0] = adj[0] + adj[2] * (X / r)
        gin[1] = adj[1] + adj[2] * (Y / r)
        return gin, None, None, None, None
