"""Thin lens -- drop-in for the reference's Components/Thin_Lens.py (Thin_LensElement).

Goodman eq. (6-10) phase exp(-i pi r^2 / (lambda f)) on the centred integer grid times the
spacing (:31-58), applied by one HIP launch (``thz_thin_lens``) with its adjoint for autograd.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from quantizationawarethzdoe_amd import optics as _optics
from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField


class Thin_LensElement(nn.Module):
    def __init__(self, focal_length, device: torch.device = None):
        super().__init__()
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.focal_length = torch.Tensor([focal_length]).to(self.device)
        self._f = float(torch.Tensor([focal_length])[0])

    def create_lens_phase_shift_kernel(self, field: ElectricField):
        """The [1, C, H, W] lens kernel itself (:31-58), evaluated by the lens kernel on ones."""
        C = len(field.wavelengths_host)
        ones = torch.ones((1, C, field.height, field.width), dtype=torch.complex64, device=field.data.device)
        dx, dy = field.spacing_host
        return _optics.thin_lens(ones, dx, dy, self._f, field.wavelengths_host)

    def forward(self, field: ElectricField) -> ElectricField:
        dx, dy = field.spacing_host
        out = _optics.thin_lens(field.data, dx, dy, self._f, field.wavelengths_host)
        return ElectricField(data=out, wavelengths=field.wavelengths, spacing=field.spacing)._adopt_host(field)
