"""Aperture -- drop-in for the reference's Components/Aperture.py (ApertureElement).

'rect' (:93-118, 'xy' grid) and 'circ' (:61-91, 'ij' grid) masks are evaluated inside the
HIP kernel (``thz_aperture``) instead of being built on the host and copied per call.
Reference behaviour kept: rect sizes are clipped to the field; a circ radius not smaller than
the half field size is an error (the reference fails there with an unbound local).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from quantizationawarethzdoe_amd import _lib
from quantizationawarethzdoe_amd import optics as _optics
from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField


def _f32(v):
    return np.float32(v)


class ApertureElement(nn.Module):
    def __init__(self, aperture_type: str = 'circ', aperture_size: float = None, device: torch.device = None):
        super().__init__()
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.aperture_type = aperture_type
        self.aperture_size = aperture_size

    @staticmethod
    def _rect_half(size, d, n):
        full = _f32(d) * _f32(n)  # dx * width as the reference's fp32 tensor
        if size is None:
            size = full / _f32(2)
            return float(size / _f32(2))
        if size < full:
            return float(_f32(size / 2))
        return float(full / _f32(2))

    def forward(self, field: ElectricField) -> ElectricField:
        dx, dy = field.spacing_host
        H, W = field.height, field.width
        if self.aperture_type == 'rect':
            out = _optics.aperture(field.data, _lib.APERTURE_RECT, dx, dy,
                                   half_w=self._rect_half(self.aperture_size, dx, W),
                                   half_h=self._rect_half(self.aperture_size, dy, H))
        elif self.aperture_type == 'circ':
            if self.aperture_size is None:
                raise TypeError("circ aperture needs a radius (the reference fails on torch.tensor(None))")
            if not _f32(self.aperture_size) < min(_f32(dx) * _f32(H), _f32(dy) * _f32(W)) / _f32(2):
                raise ValueError('The radius should not larger than the physical length of E-field ')
            out = _optics.aperture(field.data, _lib.APERTURE_CIRC, dx, dy, radius=self.aperture_size)
        elif self.aperture_type is None:
            out = field.data
        else:
            raise ValueError('No exisiting aperture shape, please define by yourself')
        return ElectricField(data=out, wavelengths=field.wavelengths, spacing=field.spacing)._adopt_host(field)
