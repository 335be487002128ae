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


def DOE_xyz_cordinates_Generator(height_map, dxy, new_dxy=0.001, origin='center', interp='nearest', for_matlab=True):
    """XYZ point cloud of a height map for the CAD export (utils/Helper_Functions.py:195-251): the
    map is resized by round(dxy / new_dxy) per axis, nearest or bilinear as cv2.resize does (the
    reference's cv2 is absent from this image, so the two resamplings are restated in numpy), put
    on a centred or left-up coordinate grid and written to DOE_xyz_coordinates_<date>.csv.  Off the
    propagation path; kept so the notebooks' import line resolves.  Returns the [N, 3] array."""
    from datetime import datetime

    import numpy as np
    h = np.asarray(height_map.detach().cpu() if torch.is_tensor(height_map) else height_map, dtype=np.float64)
    height, width = h.shape
    print("The physical length of hologram is {} mm".format(height * dxy / 1e-3))
    up_h = int(height * round(dxy / new_dxy))
    up_w = int(width * round(dxy / new_dxy))
    print(up_h)

    def src_index(n_out, n_in, linear):
        # cv2 geometry: source coordinate (dst + 0.5) * n_in / n_out - 0.5 (linear), floor(dst * n_in / n_out) (nearest)
        d = np.arange(n_out, dtype=np.float64)
        if not linear:
            return np.minimum(np.floor(d * n_in / n_out).astype(np.int64), n_in - 1), None
        s = np.clip((d + 0.5) * n_in / n_out - 0.5, 0, n_in - 1)
        i0 = np.floor(s).astype(np.int64)
        return i0, s - i0

    if interp == 'nearest':
        iy, _ = src_index(up_h, height, False)
        ix, _ = src_index(up_w, width, False)
        resized = h[iy][:, ix]
    elif interp == 'linear':
        iy, fy = src_index(up_h, height, True)
        ix, fx = src_index(up_w, width, True)
        iy1, ix1 = np.minimum(iy + 1, height - 1), np.minimum(ix + 1, width - 1)
        top = h[iy][:, ix] * (1 - fx) + h[iy][:, ix1] * fx
        bot = h[iy1][:, ix] * (1 - fx) + h[iy1][:, ix1] * fx
        resized = top * (1 - fy[:, None]) + bot * fy[:, None]
    else:
        raise ValueError(f"interp must be 'nearest' or 'linear', got {interp!r}")
    if origin == 'center':
        xc, yc = np.meshgrid(np.linspace(-up_w / 2 * new_dxy, up_w / 2 * new_dxy, up_w),
                             np.linspace(-up_h / 2 * new_dxy, up_h / 2 * new_dxy, up_h))
    elif origin == 'left-up':
        xc, yc = np.meshgrid(np.linspace(0, up_w * new_dxy, up_w), np.linspace(0, up_h * new_dxy, up_h))
    else:
        raise ValueError(f"origin must be 'center' or 'left-up', got {origin!r}")
    z = resized.T.flatten(order='C') if for_matlab else resized.T.flatten()
    xyz = np.stack([xc.flatten(), yc.flatten(), z], axis=-1).reshape(-1, 3)
    np.savetxt(f"DOE_xyz_coordinates_{datetime.now().strftime('%Y%m%d-%H%M%S')}.csv", xyz, delimiter=",")
    return xyz
