"""Helpers of the reference's utils/Helper_Functions.py that sit on the hot path's API.

``ft2`` / ``ift2`` / ``perform_ft`` (:99-160): shifted, 'ortho'-normalised 2-D transforms run
on the LDS Stockham FFT kernel (``thz_fft_rows``) along each axis; the shifts are device rolls.
``normalize`` (:185-193): divide each batch item by its max **in place**, as the reference does.
The propagators themselves never call these (they use the shift-free pipeline).
"""
from __future__ import annotations

import torch

from quantizationawarethzdoe_amd import propagation as _prop


def _fft2(x, inverse):
    y = _prop.fft_rows(x, inverse=inverse)                  # along W
    y = _prop.fft_rows(y.transpose(-1, -2), inverse=inverse)  # along H
    return y.transpose(-1, -2)


def perform_ft(input, delta=1, norm='ortho', pad=False, flag_ifft: bool = False):
    """delta^2 * shift(fft2(shift(x)))  with fftshift (forward) / ifftshift (inverse)."""
    Nx_old, Ny_old = int(input.shape[-2]), int(input.shape[-1])
    if pad:
        px, py = int(Nx_old / 2), int(Ny_old / 2)
        input = torch.nn.functional.pad(input, (py, py, px, px), mode='constant', value=0)
    H, W = input.shape[-2:]
    shift = (lambda t: torch.fft.fftshift(t, dim=(-2, -1))) if not flag_ifft else \
        (lambda t: torch.fft.ifftshift(t, dim=(-2, -1)))
    y = _fft2(shift(input), flag_ifft)
    if norm == 'ortho':
        y = y * (1.0 / (H * W) ** 0.5)
    elif norm == 'backward' or norm is None:
        if flag_ifft:
            y = y * (1.0 / (H * W))
    elif norm == 'forward':
        if not flag_ifft:
            y = y * (1.0 / (H * W))
    else:
        raise ValueError(f"Invalid normalization mode: {norm}")
    out = (delta ** 2) * shift(y)
    if pad:
        pool = torch.nn.AdaptiveAvgPool2d([Nx_old, Ny_old])
        out = pool(out.real) + 1j * pool(out.imag)
    return out


def ft2(input, delta=1, norm='ortho', pad=False):
    return perform_ft(input=input, delta=delta, norm=norm, pad=pad, flag_ifft=False)


def ift2(input, delta=1, norm='ortho', pad=False):
    return perform_ft(input=input, delta=delta, norm=norm, pad=pad, flag_ifft=True)


def normalize(x):
    """normalize to range [0-1]: x /= max over (C, H, W) per batch item, in place (:185-193)."""
    batch_size, num_obj, height, width = x.shape
    x = x.view(batch_size, -1)
    x /= x.max(1, keepdim=True)[0]
    return x.view(batch_size, num_obj, height, width)
