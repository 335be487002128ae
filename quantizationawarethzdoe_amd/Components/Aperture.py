"""Aperture -- drop-in for the reference's Components/Aperture.py (ApertureElement).

'rect' (:93-118, 'xy' grid) and 'circ' (:61-91, 'ij' grid) masks are evaluated inside the
HIP kernel (``thz_aperture``) instead of being built on the host and copied per call.
Reference behaviour kept: rect sizes are clipped to the field; a circ radius not smaller than
the half field size is an error (the reference fails there with an unbound local).
"""
from __future__ import annotations

import types

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

    def _mask(self, kind, field, **size):
        dx, dy = field.spacing_host
        ones = torch.ones((1, 1, field.height, field.width), dtype=torch.complex64, device=field.device)
        return _optics.aperture(ones, kind, dx, dy, **size).real.to(torch.int64)

    def _circ_radius(self, field, radius):
        dx, dy = field.spacing_host
        if radius is None:
            raise TypeError("circ aperture needs a radius (the reference fails on torch.tensor(None))")
        if not _f32(radius) < min(_f32(dx) * _f32(field.height), _f32(dy) * _f32(field.width)) / _f32(2):
            raise ValueError('The radius should not larger than the physical length of E-field ')
        return radius

    def add_circ_aperture_to_field(self, input_field: ElectricField, radius=None) -> torch.Tensor:
        """The circular mask [1, 1, H, W] (int64: 1 where sqrt(X^2 + Y^2) <= r), Components/Aperture.py:
        44-73, from the HIP aperture kernel applied to a unit field."""
        return self._mask(_lib.APERTURE_CIRC, input_field, radius=self._circ_radius(input_field, radius))

    def add_rect_aperture_to_field(self, input_field: ElectricField, rect_width=None, rect_height=None) -> torch.Tensor:
        """The rectangular mask [1, 1, H, W] (int64), Components/Aperture.py:75-102: sizes default to
        half the field and are clipped to it."""
        dx, dy = input_field.spacing_host
        return self._mask(_lib.APERTURE_RECT, input_field,
                          half_w=self._rect_half(rect_width, dx, input_field.width),
                          half_h=self._rect_half(rect_height, dy, input_field.height))

    @property
    def aperture(self):
        """The mask of the last forward (Components/Aperture.py:112-123 stores it as ``self.aperture``),
        formed on first read instead of on every call."""
        if "_aperture_set" in self.__dict__:  # assigned by the caller, as the reference's attribute can be
            return self.__dict__["_aperture_set"]
        src = self.__dict__.get("_aperture_src")
        if src is None:
            raise AttributeError("'ApertureElement' has no aperture before its first forward")
        kind, field = src  # the last input's geometry (not its data)
        if kind == 'circ':
            return self.add_circ_aperture_to_field(field, radius=self.aperture_size)
        if kind == 'rect':
            return self.add_rect_aperture_to_field(field, rect_height=self.aperture_size, rect_width=self.aperture_size)
        return torch.ones(field.shape, dtype=field.dtype, device=field.device)

    @aperture.setter
    def aperture(self, mask):
        self.__dict__["_aperture_set"] = mask

    def _note_input(self, field, shape=None, dtype=None):
        """The ``.aperture`` attribute's source: the last input's geometry (not its data)."""
        shape = tuple(field.shape) if shape is None else tuple(shape)
        self.__dict__.pop("_aperture_set", None)
        self.__dict__["_aperture_src"] = (self.aperture_type, types.SimpleNamespace(
            spacing_host=field.spacing_host, height=shape[-2], width=shape[-1], shape=shape,
            dtype=field.data.dtype if dtype is None else dtype, device=field.device))

    def window_desc(self, field, H, W):
        """The mask of this aperture on an H x W grid with ``field``'s spacing as a thz_aperture_desc
        (for thz_asm_desc.window_mask: the aperture folded into the propagation before it), or None
        for aperture_type None.  The same sizes, clipping and errors as forward()."""
        dx, dy = field.spacing_host
        if self.aperture_type == 'rect':
            return _lib.ApertureDesc(BC=1, H=H, W=W, kind=_lib.APERTURE_RECT, dx=dx, dy=dy,
                                     half_w=self._rect_half(self.aperture_size, dx, W),
                                     half_h=self._rect_half(self.aperture_size, dy, H), radius=0.0)
        if self.aperture_type == 'circ':
            geo = types.SimpleNamespace(spacing_host=field.spacing_host, height=H, width=W)
            return _lib.ApertureDesc(BC=1, H=H, W=W, kind=_lib.APERTURE_CIRC, dx=dx, dy=dy, half_w=0.0, half_h=0.0,
                                     radius=self._circ_radius(geo, self.aperture_size))
        if self.aperture_type is None:
            return None
        raise ValueError('No exisiting aperture shape, please define by yourself')

    def forward(self, field: ElectricField) -> ElectricField:
        dx, dy = field.spacing_host
        H, W = field.height, field.width
        self._note_input(field)
        if self.aperture_type == 'rect':
            out = _optics.aperture(field.data, _lib.APERTURE_RECT, dx, dy,
                                   half_w=self._rect_half(self.aperture_size, dx, W),
                                   half_h=self._rect_half(self.aperture_size, dy, H))
        elif self.aperture_type == 'circ':
            out = _optics.aperture(field.data, _lib.APERTURE_CIRC, dx, dy,
                                   radius=self._circ_radius(field, self.aperture_size))
        elif self.aperture_type is None:
            out = field.data
        else:
            raise ValueError('No exisiting aperture shape, please define by yourself')
        return ElectricField(data=out, wavelengths=field.wavelengths, spacing=field.spacing)._adopt_host(field)
