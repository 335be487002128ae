"""Device entry points for the DOE layers: torch.autograd glue over the C-ABI (thz_doe.hip).

All compute runs in libthzdoe's kernels; torch allocates the buffers and draws the random
numbers the reference draws (``rand_like`` height noise, ``exponential_`` Gumbel noise) so
the same generator state reproduces the reference's RNG stream.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch

from . import _lib
from .propagation import _require_device, _stream_handle


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _doe_desc(B, C, H, W, hs, ws, tol, eps, tand, wavelengths, rng=None):
    """``rng``: None, or (device int32 [2] = (seed, step), stream) -- the height noise is then drawn
    in the kernels (thz_doe_desc.rng) instead of read from a noise array."""
    wl = _lib.float_array(wavelengths)
    d = _lib.DoeDesc(B=B, C=C, H=H, W=W, hs=hs, ws=ws, tolerance=float(tol), epsilon=float(eps), tand=float(tand),
                     wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_float)),
                     rng=rng[0].data_ptr() if rng is not None else None, rng_stream=rng[1] if rng is not None else 0)
    d._keep = wl
    return d


class _Modulate(torch.autograd.Function):
    """field * t(h + noise), nearest-upsampled (Components/QuantizedDOE.py:92-126)."""

    @staticmethod
    def forward(ctx, field, height, noise, tol, eps, tand, wavelengths, rng=None):
        _require_device(field, "DOE modulate")
        field = field.contiguous()
        height = height.detach().contiguous().float()
        B, C, H, W = field.shape
        hs, ws = height.shape
        d = _doe_desc(B, C, H, W, hs, ws, tol, eps, tand, wavelengths, rng if noise is None else None)
        out = torch.empty_like(field)
        hfull = torch.empty((H, W), dtype=torch.float32, device=field.device)
        with torch.cuda.device(field.device):
            _lib.check(_lib.lib().thz_doe_modulate_forward(ctypes.byref(d), _ptr(field), _ptr(height), _ptr(noise),
                                                           _ptr(out), _ptr(hfull), _stream_handle()))
        ctx.save_for_backward(field, height, noise)
        ctx.cfg = (tol, eps, tand, wavelengths, rng)
        ctx.mark_non_differentiable(hfull)
        return out, hfull

    @staticmethod
    def backward(ctx, g, _gh):
        field, height, noise = ctx.saved_tensors
        tol, eps, tand, wavelengths, rng = ctx.cfg
        return modulate_backward(g, field, height, noise, tol, eps, tand, wavelengths, ctx.needs_input_grad[0],
                                 ctx.needs_input_grad[1], rng=rng) + (None, None, None, None, None, None)


def modulate_backward(g, field, height, noise, tol, eps, tand, wavelengths, need_field=True, need_height=True,
                      rng=None):
    """(grad_field, grad_height) of field * t(h + noise) for the output gradient g (one kernel);
    ``rng`` regenerates a device-drawn noise (see _doe_desc)."""
    B, C, H, W = field.shape
    hs, ws = height.shape
    d = _doe_desc(B, C, H, W, hs, ws, tol, eps, tand, wavelengths, rng if noise is None else None)
    g = g.contiguous()
    gf = torch.empty_like(field) if need_field else None
    gh = torch.empty((hs, ws), dtype=torch.float32, device=field.device) if need_height else None
    with torch.cuda.device(field.device):
        _lib.check(_lib.lib().thz_doe_modulate_backward(ctypes.byref(d), _ptr(g), _ptr(field), _ptr(height),
                                                        _ptr(noise), _ptr(gf), _ptr(gh), _stream_handle()))
    return gf, gh


def modulate_quant_backward(g, field, height, noise, tol, eps, tand, wavelengths, link, need_field=True, rng=None):
    """(grad_field, grad_weight) of field * t(q(w) + noise) for the output gradient g, one kernel
    (thz_doe_quant_backward): the modulate backward and the quantizer backward of ``link`` (the
    QuantLink of the quantize() call that produced ``height``) without the height gradient in
    memory.  Requires fusable(link, field)."""
    B, C, H, W = field.shape
    d = _doe_desc(B, C, H, W, H, W, tol, eps, tand, wavelengths, rng if noise is None else None)
    (kind, hq, wq, mirror, lut), kw = link.desc_args()
    q = _quant_desc(kind, hq, wq, mirror, lut, **kw)
    g = g.contiguous()
    gf = torch.empty_like(field) if need_field else None
    gw = grad_slot(link.param, link.w)
    with torch.cuda.device(field.device):
        _lib.check(_lib.lib().thz_doe_quant_backward(ctypes.byref(d), ctypes.byref(q), _ptr(g), _ptr(field),
                                                     _ptr(height), _ptr(noise), _ptr(link.w), _ptr(link.ysoft),
                                                     _ptr(gf), _ptr(gw), _stream_handle()))
    return gf, gw.reshape(link.weight.shape)


def grad_slot(weight, like):
    """A fresh tensor for the gradient of ``weight`` (shape / dtype of ``like``): a view of its slice
    of the trainer's all-reduce bucket when one was registered (qat.GradientAllReduce sets
    ``weight._thz_grad_slot``) -- autograd then adopts it as ``weight.grad`` without a copy and the
    bucket needs no packing -- else a new buffer.  The slice is handed out only while ``weight``
    has no gradient yet and only once per backward (a second contribution, or one onto an existing
    gradient, is accumulated into it by autograd and must not alias it)."""
    slot = getattr(weight, "_thz_grad_slot", None) if weight is not None else None
    if slot is not None and like.dtype == torch.float32 and weight.grad is None and id(weight) not in slot[2]:
        flat, off, used = slot
        used.add(id(weight))
        return flat[off:off + like.numel()].view(like.shape)
    return torch.empty_like(like)


class QuantLink:
    """What a quantized height map remembers of the quantize() call that made it, so the layer's
    backward can run the modulate and quantizer backward as one kernel (modulate_quant_backward):
    the weight tensor it differentiates (``weight``), its fp32 contiguous copy (``w``), the saved
    soft samples (``ysoft``) and the quantizer's configuration."""

    def __init__(self, cfg, weight, w, ysoft, full_shape, param=None):
        self.cfg, self.weight, self.w, self.ysoft, self.full_shape = cfg, weight, w, ysoft, tuple(full_shape)
        self.param = param  # the leaf tensor the weight views (its all-reduce slot: grad_slot)

    def desc_args(self):
        kind, hq, wq, mirror, lut, kw = self.cfg
        return (kind, hq, wq, mirror, lut), kw

    def fusable(self, field, height):
        """The fused backward covers a map of the field's own size (no nearest upsampling)."""
        return (tuple(field.shape[-2:]) == self.full_shape and tuple(height.shape[-2:]) == self.full_shape
                and self.weight.requires_grad)


def _modulate_args(field, height, tolerance, noise, rng=None):
    from quantizationawarethzdoe_amd.propagation import kernel_dtype
    field = kernel_dtype(field, "DOE modulate")
    if field.dtype == torch.complex128:
        # the propagators have fp64 kernels (csrc/thz_f64.hip); the DOE layers compute in complex64
        raise TypeError("DOE modulate: the DOE kernels compute in complex64; got a complex128 field (the "
                        "reference would compute it in fp64, DataType/ElectricField.py:85-90) -- cast the field "
                        "to complex64 before the DOE layer")
    if tolerance is not None and noise is None and rng is None:
        noise = torch.rand_like(height)
    if noise is not None:
        noise = noise.detach().contiguous().float()
    return field, noise, 0.0 if tolerance is None else float(tolerance)


def modulate(field, height, wavelengths, eps, tand, tolerance=None, noise=None, rng=None):
    """Differentiable DOE modulation on the HIP kernel; returns (out, noisy full-size height).
    ``rng`` (see _doe_desc): draw the height noise on the device instead of torch.rand_like."""
    field, noise, tol = _modulate_args(field, height, tolerance, noise, rng)
    return _Modulate.apply(field, height, noise, tol, float(eps), float(tand), tuple(map(float, wavelengths)),
                           rng if tolerance is not None else None)


class PendingModulation:
    """A DOELayer.modulate whose product has not been formed yet.  The noise is drawn
    when the layer runs (the reference's RNG order); the product is formed either by the next
    ASM_prop, inside its row pass (thz_asm_forward_modulated: the modulated field never goes to
    memory), or by ``run()`` -- the plain modulate kernel -- the first time anything reads the
    field's data.  ``hfull`` is the noisy upsampled height map, set by whichever runs first."""
    kind = "modulation"

    def __init__(self, field, height, wavelengths, eps, tand, tolerance=None, noise=None, rng=None, quant=None):
        self.field, self.noise, self.tol = _modulate_args(field, height, tolerance, noise, rng)
        # the QuantLink of the height map, when the layer's backward can run as one kernel
        self.quant = quant if quant is not None and quant.fusable(self.field, height) else None
        self.rng = rng if tolerance is not None and self.noise is None else None
        self.height = height
        self.wavelengths = tuple(map(float, wavelengths))
        self.eps, self.tand = float(eps), float(tand)
        self.out = None
        self.hfull = None

    def run(self):
        if self.out is None:
            self.out, hf = _Modulate.apply(self.field, self.height, self.noise, self.tol, self.eps, self.tand,
                                           self.wavelengths, self.rng)
            if self.hfull is None:
                self.hfull = hf
        return self.out

    def desc(self):
        """The thz_doe_desc of this modulation (+ the arrays it points to kept alive)."""
        B, C, H, W = self.field.shape
        hs, ws = self.height.shape[-2:]
        return _doe_desc(B, C, H, W, hs, ws, self.tol, self.eps, self.tand, self.wavelengths, self.rng)


def _quant_desc(kind, hq, wq, mirror, lut, hmax, clamp, tau=1.0, iter_frac=0.0, c_s=0.0, s=0.0, beta=0.0,
                phase_scale=0.0, dyn=None, rng=None):
    arr = _lib.float_array(lut)
    d = _lib.QuantDesc(kind=kind, hq=hq, wq=wq, mirror=int(bool(mirror)), L=len(lut),
                       lut=ctypes.cast(arr, ctypes.POINTER(ctypes.c_float)), hmax=float(hmax), clamp=float(clamp),
                       tau=float(tau), iter_frac=float(iter_frac), c_s=float(c_s), s=float(s), beta=float(beta),
                       phase_scale=float(phase_scale), dyn=dyn.data_ptr() if dyn is not None else None,
                       rng=rng[0].data_ptr() if rng is not None else None, rng_stream=rng[1] if rng is not None else 0)
    d._keep = arr
    return d


class _Quantize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weight, expo, cfg, expo_shape=None, keep=None):
        kind, hq, wq, mirror, lut, kw = cfg
        d = _quant_desc(kind, hq, wq, mirror, lut, **kw)
        w = weight.detach().contiguous().float()
        Hf, Wf = (2 * hq, 2 * wq) if mirror else (hq, wq)
        out = torch.empty((Hf, Wf), dtype=torch.float32, device=w.device)
        if expo is not None:
            ysoft = torch.empty_like(expo)
        elif expo_shape is not None:  # the Exp(1) noise drawn in the kernel (rng)
            ysoft = torch.empty(expo_shape, dtype=torch.float32, device=w.device)
        else:
            ysoft = None
        with torch.cuda.device(w.device):
            _lib.check(_lib.lib().thz_quant_forward(ctypes.byref(d), _ptr(w), _ptr(expo), _ptr(out), _ptr(ysoft),
                                                    _stream_handle()))
        ctx.save_for_backward(w, ysoft)
        ctx.cfg = cfg
        if keep is not None:  # for the QuantLink
            keep.update(w=w, ysoft=ysoft)
        return out

    @staticmethod
    def backward(ctx, g):
        w, ysoft = ctx.saved_tensors
        kind, hq, wq, mirror, lut, kw = ctx.cfg
        d = _quant_desc(kind, hq, wq, mirror, lut, **kw)
        gw = torch.empty_like(w)
        with torch.cuda.device(w.device):
            _lib.check(_lib.lib().thz_quant_backward(ctypes.byref(d), _ptr(w), _ptr(ysoft), _ptr(g.contiguous()),
                                                     _ptr(gw), _stream_handle()))
        return gw, None, None, None, None


def quantize(kind, weight, lut, hmax, clamp=8.0, mirror=False, expo=None, dyn=None, rng=None, expo_shape=None, **kw):
    """Quantized height map of one of the QAT layers (HIP forward + backward); weight shape kept.

    ``dyn``: optional device float32 [3] = (tau, s, beta) the kernels read instead of the
    keyword values, so a captured graph can be replayed across schedule steps."""
    _require_device(weight, "DOE quantizer")
    shape = weight.shape
    if kind == _lib.Q_NGS:
        hq, wq = shape[-3], shape[-2]  # logits [.., hq, wq, L]
    elif weight.dim() == 1:
        hq, wq = 1, shape[0]  # radial profile
    else:
        hq, wq = shape[-2], shape[-1]
    if len(lut) > _lib.THZ_MAX_LUT:
        raise ValueError(f"at most {_lib.THZ_MAX_LUT} LUT levels")
    if dyn is not None and (dyn.dtype != torch.float32 or not dyn.is_cuda or dyn.numel() != 3):
        raise ValueError("dyn must be a float32 device tensor of 3 values (tau, s, beta)")
    cfg = (kind, int(hq), int(wq), bool(mirror), tuple(float(v) for v in lut),
           dict(hmax=float(hmax), clamp=float(clamp), dyn=dyn, rng=rng if expo is None else None,
                **{k: float(v) for k, v in kw.items()}))
    e = expo.contiguous().float() if expo is not None else None
    wv = weight.reshape(shape)
    keep = {}
    h = _Quantize.apply(wv, e, cfg, tuple(expo_shape) if expo is None and expo_shape else None, keep)
    h._thz_quant = QuantLink(cfg, wv, keep["w"], keep["ysoft"], h.shape, param=weight)
    return h


class _Radial(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prof, R, H, W):
        p = prof.detach().contiguous().float().reshape(-1)
        out = torch.empty((H, W), dtype=torch.float32, device=p.device)
        with torch.cuda.device(p.device):
            _lib.check(_lib.lib().thz_radial_forward(_ptr(p), R, H, W, _ptr(out), _stream_handle()))
        ctx.cfg = (prof.shape, R, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        shape, R, H, W = ctx.cfg
        gp = torch.empty(R, dtype=torch.float32, device=g.device)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().thz_radial_backward(_ptr(g.contiguous()), R, H, W, _ptr(gp), _stream_handle()))
        return gp.reshape(shape), None, None, None


class _RadialQuant(torch.autograd.Function):
    """radial_map of a quantized profile, differentiated straight to the quantizer's weight: the
    backward is one kernel (thz_radial_quant_backward) instead of the radial scatter, its memset
    and the quantizer backward.  ``prof`` enters detached; ``weight`` is the QuantLink's."""

    @staticmethod
    def forward(ctx, weight, prof, link, R, H, W):
        p = prof.detach().contiguous().float().reshape(-1)
        out = torch.empty((H, W), dtype=torch.float32, device=p.device)
        with torch.cuda.device(p.device):
            _lib.check(_lib.lib().thz_radial_forward(_ptr(p), R, H, W, _ptr(out), _stream_handle()))
        ctx.link, ctx.cfg = link, (R, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        link = ctx.link
        R, H, W = ctx.cfg
        (kind, hq, wq, mirror, lut), kw = link.desc_args()
        d = _quant_desc(kind, hq, wq, mirror, lut, **kw)
        gw = grad_slot(link.param, link.w)
        with torch.cuda.device(g.device):
            _lib.check(_lib.lib().thz_radial_quant_backward(ctypes.byref(d), _ptr(g.contiguous()), R, H, W,
                                                            _ptr(link.w), _ptr(link.ysoft), _ptr(gw),
                                                            _stream_handle()))
        return gw.reshape(link.weight.shape), None, None, None, None, None


def radial_map(profile, H, W):
    """Radial profile [.., R] -> [H, W] height map (Components/QuantizedDOE.py:1409-1433).  A profile
    straight from quantize() (its QuantLink, an unmirrored R-pixel map) is differentiated to the
    quantizer's weight in one kernel (_RadialQuant)."""
    _require_device(profile, "radial map")
    R = int(profile.shape[-1])
    link = getattr(profile, "_thz_quant", None)
    if (link is not None and link.weight.requires_grad and not link.cfg[3]
            and int(link.cfg[1]) * int(link.cfg[2]) == R):
        return _RadialQuant.apply(link.weight, profile.detach(), link, R, int(H), int(W))
    return _Radial.apply(profile, R, int(H), int(W))


def f32(x):
    return float(np.float32(x))


def phase_scale(lam_min, eps):
    """fp32 (2 pi / lambda) * (sqrt(eps) - 1), the height->phase factor (QuantizedDOE.py:40-41)."""
    k = np.float32(2 * math.pi) / np.float32(lam_min)
    return float(np.float32(k) * (np.sqrt(np.float32(eps)) - np.float32(1)))
