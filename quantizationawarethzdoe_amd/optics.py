"""Device entry points of the optical elements and the QAT loss (thz_optics.hip).

Gaussian source, thin lens, aperture and the fused |E|^2 -> normalize -> MSE loss, each a
single HIP launch (the loss: two forward, one backward) with torch.autograd glue where a
gradient flows.  Physical scalars reach the kernels as fp32 host values computed in the
reference's op order; nothing here has a CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .propagation import _require_device, _stream_handle


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _fptr(arr):
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_float))


def gaussian_beam(H, W, dx, dy, wavelengths, waist_x, waist_y, center=(0.0, 0.0), z_w0=(0.0, 0.0), alpha=0.0,
                  device=None):
    """E [1, C, H, W] complex64 of LightSource/Gaussian_beam.py:88-160 generated on the device."""
    device = torch.device(device) if device is not None else torch.device("cuda")
    if device.type != "cuda":
        raise RuntimeError("gaussian_beam: the MI355X path needs a ROCm device; this framework has no CPU compute path")
    C = len(wavelengths)
    wl, wx, wy = _lib.float_array(wavelengths), _lib.float_array(waist_x), _lib.float_array(waist_y)
    d = _lib.GaussDesc(C=C, H=int(H), W=int(W), dx=float(dx), dy=float(dy), wavelengths=_fptr(wl),
                       waist_x=_fptr(wx), waist_y=_fptr(wy), x0=float(center[0]), y0=float(center[1]),
                       z_w0x=float(z_w0[0]), z_w0y=float(z_w0[1]), alpha=float(alpha))
    out = torch.empty((1, C, int(H), int(W)), dtype=torch.complex64, device=device)
    with torch.cuda.device(device):
        _lib.check(_lib.lib().thz_gaussian_beam(ctypes.byref(d), _p(out), _stream_handle()))
    return out


class _Lens(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dx, dy, f, wavelengths):
        _require_device(x, "thin lens")
        x = x.contiguous()
        out = torch.empty_like(x)
        _lens_launch(x, out, dx, dy, f, wavelengths)
        ctx.cfg = (dx, dy, f, wavelengths)
        return out

    @staticmethod
    def backward(ctx, g):
        dx, dy, f, wavelengths = ctx.cfg
        g = g.contiguous()
        out = torch.empty_like(g)
        _lens_launch(g, out, dx, dy, -f, wavelengths)  # conj(ker): the focal length flips sign
        return out, None, None, None, None


def _lens_launch(x, out, dx, dy, f, wavelengths):
    B, C, H, W = x.shape
    wl = _lib.float_array(wavelengths)
    d = _lib.LensDesc(B=B, C=C, H=H, W=W, dx=float(dx), dy=float(dy), focal_length=float(f), wavelengths=_fptr(wl))
    with torch.cuda.device(x.device):
        _lib.check(_lib.lib().thz_thin_lens(ctypes.byref(d), _p(x), _p(out), _stream_handle()))


def thin_lens(x, dx, dy, focal_length, wavelengths):
    """field * exp(-i pi r^2 / (lambda f)) (Components/Thin_Lens.py:31-85), differentiable."""
    if x.dtype != torch.complex64:
        raise TypeError(f"lens kernel computes in complex64; got {x.dtype}")
    return _Lens.apply(x, float(dx), float(dy), float(focal_length), tuple(float(w) for w in wavelengths))


class _Aperture(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cfg):
        _require_device(x, "aperture")
        x = x.contiguous()
        out = torch.empty_like(x)
        _aperture_launch(x, out, cfg)
        ctx.cfg = cfg
        return out

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        out = torch.empty_like(g)
        _aperture_launch(g, out, ctx.cfg)  # real 0/1 mask: self-adjoint
        return out, None


def _aperture_launch(x, out, cfg):
    kind, dx, dy, half_w, half_h, radius = cfg
    B, C, H, W = x.shape
    d = _lib.ApertureDesc(BC=B * C, H=H, W=W, kind=kind, dx=dx, dy=dy, half_w=half_w, half_h=half_h, radius=radius)
    with torch.cuda.device(x.device):
        _lib.check(_lib.lib().thz_aperture(ctypes.byref(d), _p(x), _p(out), _stream_handle()))


def aperture(x, kind, dx, dy, half_w=0.0, half_h=0.0, radius=0.0):
    """field * mask (Components/Aperture.py:44-136); thresholds are fp32 as the reference compares them."""
    if x.dtype != torch.complex64:
        raise TypeError(f"aperture kernel computes in complex64; got {x.dtype}")
    cfg = (int(kind), float(dx), float(dy), float(np.float32(half_w)), float(np.float32(half_h)),
           float(np.float32(radius)))
    return _Aperture.apply(x, cfg)


class _IntensityMSE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, field, target):
        _require_device(field, "intensity MSE")
        field = field.contiguous()
        target = target.contiguous().float()
        B, C, H, W = field.shape
        t4 = target.reshape((1,) * (4 - target.dim()) + tuple(target.shape))
        d = _lib.LossDesc(B=B, C=C, H=H, W=W, tB=t4.shape[0], tC=t4.shape[1])
        if tuple(t4.shape[-2:]) != (H, W):
            raise ValueError(f"target {tuple(target.shape)} does not broadcast to field {tuple(field.shape)}")
        nbytes = _lib.lib().thz_intensity_mse_workspace_size(ctypes.byref(d))
        stats = torch.empty(nbytes // 4, dtype=torch.float32, device=field.device)
        loss = torch.empty((), dtype=torch.float32, device=field.device)
        with torch.cuda.device(field.device):
            _lib.check(_lib.lib().thz_intensity_mse_forward(ctypes.byref(d), _p(field), _p(t4), _p(loss), _p(stats),
                                                            _stream_handle()))
        ctx.save_for_backward(field, t4, stats)
        ctx.desc = (B, C, H, W, t4.shape[0], t4.shape[1])
        return loss

    @staticmethod
    def backward(ctx, g):
        field, t4, stats = ctx.saved_tensors
        B, C, H, W, tB, tC = ctx.desc
        d = _lib.LossDesc(B=B, C=C, H=H, W=W, tB=tB, tC=tC)
        gf = torch.empty_like(field)
        g = g.detach().float().contiguous()
        with torch.cuda.device(field.device):
            _lib.check(_lib.lib().thz_intensity_mse_backward(ctypes.byref(d), _p(field), _p(t4), _p(stats), _p(g),
                                                             _p(gf), _stream_handle()))
        return gf, None


def intensity_mse(field, target):
    """mean((normalize(|E|^2) - target)^2): the QAT loss of experiment_four_focal_spots.ipynb:336-370
    (normalize = utils/Helper_Functions.py:185-193, per batch item by its max), fused on the device."""
    if field.dtype != torch.complex64:
        raise TypeError(f"loss kernel computes in complex64 fields; got {field.dtype}")
    return _IntensityMSE.apply(field, target)


def field_intensity_mse(field, target):
    """intensity_mse of an ElectricField.  When the field is the deferred output of an ASM_prop
    (propagation.deferred_output), the loss is folded into that propagation's row-inverse pass
    (thz_asm_forward_loss) and the field's data is set from the same pipeline; otherwise this is
    intensity_mse(field.data, target)."""
    pend = field._take_pending_propagation()
    if pend is not None:
        data, loss = pend.run_loss(target)
        field.data = data
        return loss
    return intensity_mse(field.data, target)


class _Resample(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Hout, Wout, dx_in, dy_in, dx_out, dy_out):
        _require_device(x, "field resampler")
        x = x.contiguous()
        B, C, H, W = x.shape
        d = _lib.ResampleDesc(BC=B * C, Hin=H, Win=W, Hout=Hout, Wout=Wout, dx_in=dx_in, dy_in=dy_in, dx_out=dx_out,
                              dy_out=dy_out)
        out = torch.empty((B, C, Hout, Wout), dtype=x.dtype, device=x.device)
        with torch.cuda.device(x.device):
            _lib.check(_lib.lib().thz_resample_forward(ctypes.byref(d), _p(x), _p(out), _stream_handle()))
        ctx.cfg = (d, (B, C, H, W))
        return out

    @staticmethod
    def backward(ctx, g):
        d, shape = ctx.cfg
        g = g.contiguous()
        gin = torch.empty(shape, dtype=g.dtype, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().thz_resample_backward(ctypes.byref(d), _p(g), _p(gin), _stream_handle()))
        return gin, None, None, None, None, None, None


def resample(x, Hout, Wout, dx_in, dy_in, dx_out, dy_out):
    """Bilinear resampling of [B, C, H, W] complex64 onto the centred (Hout, Wout) grid with the
    output pixel pitch (Addons/Field_Resampler.py:74-118), differentiable."""
    if x.dtype != torch.complex64:
        raise TypeError(f"resampler kernel computes in complex64; got {x.dtype}")
    H, W = x.shape[-2:]
    if (H - 1) // 2 == 0 or (W - 1) // 2 == 0:
        # fewer than 3 pixels on an axis: the reference normalises the sampling grid by
        # dx ((H - 1) // 2) = 0 and grid_sample returns NaN everywhere (run here on 1 x 4, 2 x 2 and
        # 2 x 5 fields); the same NaN field, still attached to the input for autograd
        out = torch.full((*x.shape[:-2], int(Hout), int(Wout)), complex(float("nan"), float("nan")),
                         dtype=x.dtype, device=x.device)
        return out + 0 * x.sum(dim=(-2, -1), keepdim=True) if x.requires_grad else out
    return _Resample.apply(x, int(Hout), int(Wout), float(dx_in), float(dy_in), float(dx_out), float(dy_out))
