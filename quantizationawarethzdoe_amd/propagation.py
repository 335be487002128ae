"""Device entry points for the propagators: thin torch glue over the C-ABI.

Each function takes CUDA(HIP) complex64 tensors plus HOST scalars (wavelengths,
spacing, z) and enqueues the hand-written gfx950 kernels of libthzdoe.so on the
current torch stream.  The autograd Functions route backward through the same
kernels (the ASM adjoint == ASM with conj(H)).  There is no CPU
path: a CPU tensor is an error.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import threading

import torch

from . import _lib


def _require_device(t: torch.Tensor, what: str):
    if not t.is_cuda:
        raise RuntimeError(f"{what}: the MI355X path needs a ROCm device tensor (got device {t.device}); "
                           "this framework has no CPU compute path")


def kernel_dtype(data: torch.Tensor, who: str, wavelengths=None) -> torch.Tensor:
    """The field in the precision the reference computes it in (DataType/ElectricField.py:85-90):
    complex128 when the data is complex128 / float64 or the wavelength tensor is float64 (torch's
    promotion; the reference's test_czt.py:12 runs that way), else complex64.  The complex128
    fields run the fp64 kernels (csrc/thz_f64.hip), the rest the fp32 ones; real data is promoted
    as torch's complex products promote it."""
    fp64 = data.dtype in (torch.complex128, torch.float64) or (
        torch.is_tensor(wavelengths) and wavelengths.dtype == torch.float64)
    if data.dtype not in (torch.complex64, torch.complex128, torch.float32, torch.float64, torch.float16,
                          torch.bfloat16):
        raise TypeError(f"{who}: the MI355X kernels compute in complex64 or complex128; got {data.dtype}")
    want = torch.complex128 if fp64 else torch.complex64
    return data if data.dtype == want else data.to(want)


def _stream_handle():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def asm_padding(H, W, padding_scale, do_padding=True):
    """pad = floor(s N / 2), P = N + 2 pad (Props/ASM_Prop.py:119-136)."""
    if not do_padding:
        return 0, 0
    sh, sw = padding_scale
    return int(math.floor(float(sh) * H / 2)), int(math.floor(float(sw) * W / 2))


def _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, adjoint, z_chunk=0,
              mask=None, z_dev=None):
    """thz_asm_desc; ``mask``: an ApertureDesc on the output grid (thz_asm_desc.window_mask);
    ``z_dev``: a float32 device tensor [Z] the kernels read the plane distances from
    (thz_asm_desc.z_dev: graph-replayable planes; ``zs`` then only gives their count)."""
    if z_dev is not None and (z_dev.dtype != torch.float32 or not z_dev.is_contiguous() or z_dev.numel() != len(zs)
                              or z_dev.device.type != "cuda"):
        raise ValueError(f"z_dev: a contiguous float32 device tensor of {len(zs)} planes")
    wl = _lib.float_array(wavelengths)
    zv = _lib.float_array(zs)
    d = _lib.AsmDesc(B=B, C=C, H=H, W=W, pad_h=pad_h, pad_w=pad_w, unpad=int(bool(unpad)),
                     bandlimit=int(bandlimit), Z=len(zs), adjoint=int(adjoint), z_chunk=int(z_chunk),
                     dx=float(spacing[0]), dy=float(spacing[1]),
                     wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_float)),
                     z=ctypes.cast(zv, ctypes.POINTER(ctypes.c_float)),
                     window_mask=ctypes.addressof(mask) if mask is not None else None,
                     z_dev=z_dev.data_ptr() if z_dev is not None else None)
    d._keep = (wl, zv, mask, z_dev)
    return d


def window_mask_fusable(H, W, pad_h, pad_w, unpad, Z=1):
    """True when the library folds an aperture into the propagation (thz_asm_desc.window_mask): the
    300-point layer geometry of the cfg4 / cfg5 systems (100-pixel fields, padding 2, cropped)."""
    return H == W == 100 and pad_h == pad_w == 100 and bool(unpad) and Z == 1


def asm_apply(data, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, adjoint=False, z_chunk=0,
              out=None, mask=None, z_dev=None):
    """Raw launch: forward data [B,C,H,W] -> [Z,B,C,Ho,Wo]; adjoint [Z,B,C,Ho,Wo] -> [B,C,H,W], the sum
    over the Z planes of each plane's adjoint (one pipeline: the column pass sums the planes'
    spectra, thz_asm_forward with adjoint = 1)."""
    _require_device(data, "ASM")
    if mask is not None:
        # the folded aperture exists in the complex64 300-point row passes only, and its adjoint takes
        # one plane: refuse here, in the forward, rather than drop the mask or fail in backward
        if data.dtype != torch.complex64:
            raise TypeError(f"ASM window mask: complex64 fields only, got {data.dtype} (apply the aperture "
                            "separately)")
        if len(zs) != 1:
            raise ValueError(f"ASM window mask: one z-plane per call, got {len(zs)}")
    if data.dtype == torch.complex128:
        if z_dev is not None:
            raise TypeError("ASM z_dev: complex64 fields only (the fp64 kernels take host planes)")
        return _asm64_apply(data, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, adjoint, out)
    if data.dtype != torch.complex64:
        raise TypeError(f"ASM kernels compute in complex64 or complex128; got {data.dtype}")
    L = _lib.lib()
    data = data.contiguous()
    if adjoint:
        Z, B, C, Ho, Wo = data.shape
        if Z != len(zs):
            raise ValueError(f"adjoint: {Z} gradient planes for {len(zs)} z values")
        H = Ho - (0 if unpad else 2 * pad_h)
        W = Wo - (0 if unpad else 2 * pad_w)
        out_shape = (B, C, H, W)
    else:
        B, C, H, W = data.shape
        Ho, Wo = (H, W) if unpad else (H + 2 * pad_h, W + 2 * pad_w)
        out_shape = (len(zs), B, C, Ho, Wo)
    d = _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, adjoint, z_chunk, mask, z_dev)
    nbytes = ctypes.c_size_t(0)
    _lib.check(L.thz_asm_workspace_size(ctypes.byref(d), ctypes.byref(nbytes)))
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=data.device)
    if out is None:
        out = torch.empty(out_shape, dtype=torch.complex64, device=data.device)
    with torch.cuda.device(data.device):
        _lib.check(L.thz_asm_forward(ctypes.byref(d), ctypes.c_void_p(data.data_ptr()),
                                     ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                     ctypes.c_size_t(ws.numel()), _stream_handle()))
    return out


def _asm64_apply(data, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, adjoint=False, out=None):
    """complex128 ASM (thz_asm64_forward): the same shapes as asm_apply; the fp64 adjoint runs one
    launch per plane and sums them."""
    L = _lib.lib()
    data = data.contiguous()
    if adjoint:
        Z, B, C, Ho, Wo = data.shape
        if Z != len(zs):
            raise ValueError(f"adjoint: {Z} gradient planes for {len(zs)} z values")
        H = Ho - (0 if unpad else 2 * pad_h)
        W = Wo - (0 if unpad else 2 * pad_w)
        res = None
        for k, z in enumerate(zs):
            gk = _asm64_launch(data[k:k + 1], (B, C, H, W), wavelengths, spacing, [z], pad_h, pad_w, unpad, bandlimit,
                               True, torch.empty((B, C, H, W), dtype=torch.complex128, device=data.device))
            res = gk if res is None else res + gk
        return res
    B, C, H, W = data.shape
    Ho, Wo = (H, W) if unpad else (H + 2 * pad_h, W + 2 * pad_w)
    if out is None:
        out = torch.empty((len(zs), B, C, Ho, Wo), dtype=torch.complex128, device=data.device)
    return _asm64_launch(data, (B, C, H, W), wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, False, out)


def _asm64_launch(data, shape, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, adjoint, out):
    L = _lib.lib()
    B, C, H, W = shape
    wl = _lib.double_array(wavelengths)
    zv = _lib.double_array(zs)
    d = _lib.AsmDesc64(B=B, C=C, H=H, W=W, pad_h=pad_h, pad_w=pad_w, unpad=int(bool(unpad)), bandlimit=int(bandlimit),
                       Z=len(zs), adjoint=int(adjoint), dx=float(spacing[0]), dy=float(spacing[1]),
                       wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_double)),
                       z=ctypes.cast(zv, ctypes.POINTER(ctypes.c_double)))
    nbytes = ctypes.c_size_t(0)
    _lib.check(L.thz_asm64_workspace_size(ctypes.byref(d), ctypes.byref(nbytes)))
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=data.device)
    with torch.cuda.device(data.device):
        _lib.check(L.thz_asm64_forward(ctypes.byref(d), ctypes.c_void_p(data.data_ptr()),
                                       ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                       ctypes.c_size_t(ws.numel()), _stream_handle()))
    return out


def asm_plan_info(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, z_chunk=0):
    """(kept spectral columns, z-planes per column pass) of the library's plan."""
    d = _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, False, z_chunk)
    n, zc = ctypes.c_int(0), ctypes.c_int(0)
    _lib.check(_lib.lib().thz_asm_band(ctypes.byref(d), ctypes.byref(n), ctypes.byref(zc)))
    return n.value, zc.value


def asm_band_columns(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs):
    return asm_plan_info(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs)[0]


class _AsmFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, z_chunk, mask, z_dev):
        ctx.cfg = (wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, mask, z_dev)
        return asm_apply(data, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, False, z_chunk, mask=mask,
                         z_dev=z_dev)

    @staticmethod
    def backward(ctx, g):
        wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, mask, z_dev = ctx.cfg
        # one adjoint launch for all planes: sum_z A_z^H g_z, the sum taken in the column pass (the
        # window mask, when folded, on the adjoint's input)
        gin = asm_apply(g.contiguous(), wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, True, mask=mask,
                        z_dev=z_dev)
        return gin, None, None, None, None, None, None, None, None, None, None


def asm_transfer_function(wavelengths, spacing, z, H, W, pad_h, pad_w, bandlimit, device):
    """ASM_prop.create_kernel's table (Props/ASM_Prop.py:212-311): [1, C, Ph, Pw] complex64 on the
    centred frequency grid, computed by the HIP kernel the propagators evaluate on the fly."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError(f"ASM transfer function: the MI355X path needs a ROCm device (got {dev}); "
                           "this framework has no CPU compute path")
    bl = _lib.BANDLIMIT[bandlimit] if not isinstance(bandlimit, int) else bandlimit
    d = _asm_desc(1, len(wavelengths), int(H), int(W), int(pad_h), int(pad_w), True, bl, wavelengths, spacing,
                  [float(z)], False)
    out = torch.empty((1, len(wavelengths), H + 2 * pad_h, W + 2 * pad_w), dtype=torch.complex64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().thz_asm_transfer_function(ctypes.byref(d), ctypes.c_void_p(out.data_ptr()),
                                                         _stream_handle()))
    return out


def rs_kernel(meshx, meshy, z, wavelengths):
    """exp(ikr) z/(2 pi r^2) (1/r - ik) on the meshes for each wavelength (Props/CZT_Prop.py:44-57,
    Props/RSC_Prop.py:157-160): [1, C, *mesh.shape] complex64 from the HIP kernel thz_rs_kernel."""
    _require_device(meshx, "RS kernel")
    mx, my = torch.broadcast_tensors(meshx, meshy)
    shape = tuple(mx.shape)
    mx = mx.detach().to(torch.float32).contiguous().reshape(-1)
    my = my.detach().to(device=mx.device, dtype=torch.float32).contiguous().reshape(-1)
    wl = [float(v) for v in wavelengths]
    arr = _lib.float_array(wl)
    out = torch.empty((1, len(wl)) + shape, dtype=torch.complex64, device=mx.device)
    with torch.cuda.device(mx.device):
        _lib.check(_lib.lib().thz_rs_kernel(ctypes.c_void_p(mx.data_ptr()), ctypes.c_void_p(my.data_ptr()),
                                            int(mx.numel()), ctypes.c_float(float(z)), ctypes.cast(arr, ctypes.c_void_p), len(wl),
                                            ctypes.c_void_p(out.data_ptr()), _stream_handle()))
    return out


def asm_propagate(data, wavelengths, spacing, zs, pad_h, pad_w, unpad=True, bandlimit="exact", z_chunk=0,
                  mask=None, z_dev=None):
    """Differentiable ASM over Z planes: [B,C,H,W] -> [Z,B,C,Ho,Wo] (HIP kernels); ``mask``: an
    aperture folded onto the output (window_mask_fusable geometry only); ``z_dev``: the planes in
    device memory (_asm_desc)."""
    bl = _lib.BANDLIMIT[bandlimit] if not isinstance(bandlimit, int) else bandlimit
    return _AsmFunction.apply(data, list(map(float, wavelengths)), tuple(map(float, spacing)),
                              list(map(float, zs)), int(pad_h), int(pad_w), bool(unpad), bl, int(z_chunk), mask, z_dev)


class _AsmModulatedFunction(torch.autograd.Function):
    """ASM forward of DOELayer.modulate(field) in one pipeline (thz_asm_forward_modulated): the row
    pass applies t_c(h + noise) in its loader.  Backward: the ASM adjoint summed over the planes
    (one launch), then the modulate backward kernel (grad_field, grad_height) -- or, when the height
    map comes straight from a quantizer of the field's size (doe.QuantLink), the modulate and
    quantizer backward in one kernel (grad_field, grad_weight)."""

    @staticmethod
    def forward(ctx, field, height, weight, pend, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, mask,
                z_dev):
        _require_device(field, "ASM")
        field = field.contiguous()
        h = height.detach().contiguous().float()
        B, C, H, W = field.shape
        Ho, Wo = (H, W) if unpad else (H + 2 * pad_h, W + 2 * pad_w)
        d = _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, False, mask=mask,
                      z_dev=z_dev)
        m = pend.desc()
        L = _lib.lib()
        nbytes = ctypes.c_size_t(0)
        _lib.check(L.thz_asm_workspace_size(ctypes.byref(d), ctypes.byref(nbytes)))
        ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=field.device)
        out = torch.empty((len(zs), B, C, Ho, Wo), dtype=torch.complex64, device=field.device)
        hfull = torch.empty((H, W), dtype=torch.float32, device=field.device)
        noise = pend.noise
        with torch.cuda.device(field.device):
            _lib.check(L.thz_asm_forward_modulated(
                ctypes.byref(d), ctypes.byref(m), ctypes.c_void_p(field.data_ptr()), ctypes.c_void_p(h.data_ptr()),
                ctypes.c_void_p(noise.data_ptr() if noise is not None else 0), ctypes.c_void_p(hfull.data_ptr()),
                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(ws.numel()),
                _stream_handle()))
        if pend.hfull is None:
            pend.hfull = hfull
        ctx.save_for_backward(field, h)
        ctx.pend = pend
        ctx.cfg = (wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, mask, z_dev)
        return out

    @staticmethod
    def backward(ctx, g):
        field, h = ctx.saved_tensors
        pend = ctx.pend
        wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, mask, z_dev = ctx.cfg
        gm = asm_apply(g.contiguous(), wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, True, mask=mask,
                       z_dev=z_dev)
        gf, gh, gw = _doe_backward(ctx, gm, field, h, pend)
        return (gf, gh, gw) + (None,) * 11


def _doe_inputs(pend):
    """(height, weight) inputs of a fused function for the pending modulation ``pend``: with a
    fusable quantizer link (doe.QuantLink) the weight is differentiated directly, in one kernel with
    the modulate backward (_doe_backward), and the height map enters detached."""
    if pend.quant is None:
        return pend.height, None
    return pend.height.detach(), pend.quant.weight


def _doe_backward(ctx, gm, field, h, pend):
    """(grad_field, grad_height, grad_weight) of the modulation behind a fused function, whose
    inputs 0, 1, 2 are (field, height, weight): one thz_doe_quant_backward when the quantizer is
    linked, else thz_doe_modulate_backward."""
    from . import doe as _doe
    if pend.quant is not None and ctx.needs_input_grad[2]:
        gf, gw = _doe.modulate_quant_backward(gm, field, h, pend.noise, pend.tol, pend.eps, pend.tand,
                                              pend.wavelengths, pend.quant, ctx.needs_input_grad[0], rng=pend.rng)
        return gf, None, gw
    gf, gh = _doe.modulate_backward(gm, field, h, pend.noise, pend.tol, pend.eps, pend.tand, pend.wavelengths,
                                    ctx.needs_input_grad[0], ctx.needs_input_grad[1], rng=pend.rng)
    return gf, gh, None


def asm_propagate_modulated(pend, wavelengths, spacing, zs, pad_h, pad_w, unpad=True, bandlimit="exact", mask=None,
                            z_dev=None):
    """Differentiable fused DOE modulation + ASM over Z planes: [B,C,H,W] -> [Z,B,C,Ho,Wo]; ``mask``
    and ``z_dev`` as asm_propagate."""
    bl = _lib.BANDLIMIT[bandlimit] if not isinstance(bandlimit, int) else bandlimit
    height, weight = _doe_inputs(pend)
    return _AsmModulatedFunction.apply(pend.field, height, weight, pend, list(map(float, wavelengths)),
                                       tuple(map(float, spacing)), list(map(float, zs)), int(pad_h), int(pad_w),
                                       bool(unpad), bl, mask, z_dev)


class _AsmLossFunction(torch.autograd.Function):
    """Z z-planes of ASM (optionally of a pending DOE modulation) whose row-inverse pass also
    accumulates the QAT loss mean((normalize(|E|^2) - target)^2) (thz_asm_forward_loss) -- for
    Z > 1 the sum over the planes of each plane's mean, the multi-plane notebooks' summed MSEs,
    the target [tB, tC, Ho, Wo] broadcast over the Z B plane-major items (tB in {1, Z B}).
    Outputs (out [Z,B,C,Ho,Wo], loss []).  Backward: the ASM adjoint (summed over the planes) of the
    loss gradient of the stored field, formed in the adjoint's row pass (thz_asm_adjoint_loss;
    plus the out cotangent when out is used elsewhere), then the DOE layer's backward when a
    modulation was fused."""

    @staticmethod
    def forward(ctx, field, height, weight, target, pend, wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit,
                z_dev=None):
        ctx.set_materialize_grads(False)
        if field.dtype != torch.complex64:  # thz_asm_forward_loss reads float2 pairs
            raise TypeError(f"fused ASM loss computes in complex64 fields; got {field.dtype}")
        _require_device(field, "ASM")
        field = field.contiguous()
        B, C, H, W = field.shape
        Ho, Wo = (H, W) if unpad else (H + 2 * pad_h, W + 2 * pad_w)
        Z = len(zs)
        t4 = target.detach().float().contiguous()
        t4 = t4.reshape((1,) * (4 - t4.dim()) + tuple(t4.shape))
        if tuple(t4.shape[-2:]) != (Ho, Wo) or t4.shape[0] not in (1, Z * B) or t4.shape[1] not in (1, C):
            raise ValueError(f"target {tuple(target.shape)} does not broadcast to field {(Z * B, C, Ho, Wo)}")
        d = _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, False, z_dev=z_dev)
        ld = _lib.LossDesc(B=Z * B, C=C, H=Ho, W=Wo, tB=t4.shape[0], tC=t4.shape[1])
        L = _lib.lib()
        nbytes = ctypes.c_size_t(0)
        _lib.check(L.thz_asm_workspace_size(ctypes.byref(d), ctypes.byref(nbytes)))
        dev = field.device
        ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
        out = torch.empty((Z, B, C, Ho, Wo), dtype=torch.complex64, device=dev)
        loss = torch.empty((), dtype=torch.float32, device=dev)
        stats = torch.empty(L.thz_intensity_mse_workspace_size(ctypes.byref(ld)) // 4, dtype=torch.float32,
                            device=dev)
        h = hfull = noise = None
        m = None
        if pend is not None:
            h = height.detach().contiguous().float()
            hfull = torch.empty((H, W), dtype=torch.float32, device=dev)
            noise = pend.noise
            m = pend.desc()

        def ptr(t):
            return ctypes.c_void_p(t.data_ptr() if t is not None else 0)

        with torch.cuda.device(dev):
            _lib.check(L.thz_asm_forward_loss(
                ctypes.byref(d), ctypes.byref(m) if m is not None else None, ptr(field), ptr(h), ptr(noise),
                ptr(hfull), ctypes.byref(ld), ptr(t4), ptr(out), ptr(loss), ptr(stats), ptr(ws),
                ctypes.c_size_t(ws.numel()), _stream_handle()))
        if pend is not None and pend.hfull is None:
            pend.hfull = hfull
        ctx.save_for_backward(field, h, out, t4, stats)
        ctx.pend = pend
        ctx.cfg = (wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, z_dev)
        ctx.ldesc = (B, C, Ho, Wo, t4.shape[0], t4.shape[1])
        return out, loss

    @staticmethod
    def backward(ctx, g_out, g_loss):
        field, h, out, t4, stats = ctx.saved_tensors
        wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, z_dev = ctx.cfg
        if g_loss is None and g_out is None:
            return (None,) * 13
        if g_loss is None:
            gm = asm_apply(g_out.contiguous(), wavelengths, spacing, zs, pad_h, pad_w, unpad, bandlimit, True,
                           z_dev=z_dev)
        else:
            # the loss gradient is formed in the adjoint's row pass (thz_asm_adjoint_loss)
            B, C, Ho, Wo, tB, tC = ctx.ldesc
            H, W = field.shape[-2:]
            ld = _lib.LossDesc(B=len(zs) * B, C=C, H=Ho, W=Wo, tB=tB, tC=tC)
            d = _asm_desc(B, C, H, W, pad_h, pad_w, unpad, bandlimit, wavelengths, spacing, zs, True, z_dev=z_dev)
            L = _lib.lib()
            nbytes = ctypes.c_size_t(0)
            _lib.check(L.thz_asm_workspace_size(ctypes.byref(d), ctypes.byref(nbytes)))
            ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=out.device)
            gm = torch.empty((B, C, H, W), dtype=torch.complex64, device=out.device)
            g = g_loss.detach().float().contiguous()
            go = g_out.contiguous() if g_out is not None else None
            with torch.cuda.device(out.device):
                _lib.check(L.thz_asm_adjoint_loss(
                    ctypes.byref(d), ctypes.byref(ld), ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(t4.data_ptr()),
                    ctypes.c_void_p(stats.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                    ctypes.c_void_p(go.data_ptr() if go is not None else 0), ctypes.c_void_p(gm.data_ptr()),
                    ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(ws.numel()), _stream_handle()))
        gh = gw = None
        pend = ctx.pend
        if pend is None:
            gf = gm
        else:
            gf, gh, gw = _doe_backward(ctx, gm, field, h, pend)
        return (gf, gh, gw) + (None,) * 10


def asm_propagate_loss(x, target, wavelengths, spacing, z, pad_h, pad_w, unpad=True, bandlimit="exact", pend=None,
                       z_dev=None):
    """Differentiable ASM fused with the QAT loss: (out [Z,B,C,Ho,Wo], loss []).  ``z``: one
    distance, or a list of Z planes (the loss is then the sum of the planes' means, the target
    broadcast over the Z B plane-major items); ``z_dev`` as asm_propagate.  ``pend``
    (doe.PendingModulation, not yet formed): propagate its modulation of ``pend.field`` (``x`` is
    then ignored), as asm_propagate_modulated."""
    bl = _lib.BANDLIMIT[bandlimit] if not isinstance(bandlimit, int) else bandlimit
    zs = [float(v) for v in z] if isinstance(z, (list, tuple)) else [float(z)]
    if len(zs) > _lib.THZ_MAX_Z:
        raise ValueError(f"the fused loss takes at most {_lib.THZ_MAX_Z} planes per call")
    field, (height, weight) = (pend.field, _doe_inputs(pend)) if pend is not None else (x, (None, None))
    return _AsmLossFunction.apply(field, height, weight, target, pend, list(map(float, wavelengths)),
                                  tuple(map(float, spacing)), zs, int(pad_h), int(pad_w), bool(unpad), bl, z_dev)


class _Deferral(threading.local):
    active = False


_DEFER = _Deferral()


@contextlib.contextmanager
def deferred_output():
    """Inside this block ASM_prop.forward returns its output field unevaluated: the propagation
    runs when the field's ``data`` is first read -- or, when the first reader is the QAT loss
    (optics.field_intensity_mse), as one pipeline with the loss folded into its last pass
    (thz_asm_forward_loss).  The trainers wrap their forward in it; the deferred propagation reads
    its input field when it runs, so the input must not be modified in between."""
    prev = _DEFER.active
    _DEFER.active = True
    try:
        yield
    finally:
        _DEFER.active = prev


def deferring():
    return _DEFER.active


def fft_rows(x, inverse=False):
    """Unnormalised batched 1-D FFT along the last axis with the LDS Stockham kernel (complex128
    input: the fp64 transform)."""
    _require_device(x, "fft_rows")
    x = x.contiguous()
    x = x if x.dtype == torch.complex128 else x.to(torch.complex64)
    out = torch.empty_like(x)
    n = x.shape[-1]
    rows = x.numel() // n
    fn = _lib.lib().thz_fft64_rows if x.dtype == torch.complex128 else _lib.lib().thz_fft_rows
    with torch.cuda.device(x.device):
        _lib.check(fn(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), rows, n, int(inverse),
                      _stream_handle()))
    return out


def czt_apply(data, wavelengths, spacing, z, outH, outW, odx, ody, adjoint=False, field_hw=None):
    """Chirp-z propagation [B,C,H,W] -> [B,C,outW,outH] (Props/CZT_Prop.py:252-314) on the HIP kernels.

    adjoint: the autograd backward, [B,C,outW,outH] -> [B,C,H,W] with (H, W) = field_hw."""
    _require_device(data, "CZT")
    if data.dtype not in (torch.complex64, torch.complex128):
        raise TypeError(f"CZT kernels compute in complex64 or complex128; got {data.dtype}")
    f64 = data.dtype == torch.complex128
    data = data.contiguous()
    B, C = data.shape[:2]
    H, W = (int(v) for v in (field_hw if adjoint else data.shape[-2:]))
    if adjoint and tuple(data.shape[-2:]) != (int(outW), int(outH)):
        raise ValueError(f"CZT adjoint: gradient {tuple(data.shape)} is not [B, C, outW, outH]")
    if f64:
        wl = _lib.double_array(wavelengths)
        d = _lib.CztDesc64(B=B, C=C, H=H, W=W, outH=int(outH), outW=int(outW), dx=float(spacing[0]),
                           dy=float(spacing[1]), odx=float(odx), ody=float(ody), z=float(z),
                           wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_double)), adjoint=int(bool(adjoint)))
    else:
        wl = _lib.float_array(wavelengths)
        d = _lib.CztDesc(B=B, C=C, H=H, W=W, outH=int(outH), outW=int(outW), dx=float(spacing[0]),
                         dy=float(spacing[1]), odx=float(odx), ody=float(ody), z=float(z),
                         wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_float)), adjoint=int(bool(adjoint)))
    L = _lib.lib()
    size_fn, run_fn = (L.thz_czt64_workspace_size, L.thz_czt64_forward) if f64 else \
        (L.thz_czt_workspace_size, L.thz_czt_forward)
    nbytes = ctypes.c_size_t(0)
    _lib.check(size_fn(ctypes.byref(d), ctypes.byref(nbytes)))
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=data.device)
    oshape = (B, C, H, W) if adjoint else (B, C, int(outW), int(outH))
    out = torch.empty(oshape, dtype=data.dtype, device=data.device)
    with torch.cuda.device(data.device):
        _lib.check(run_fn(ctypes.byref(d), ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                          ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(ws.numel()), _stream_handle()))
    return out


def rsc_apply(data, wavelengths, spacing, z, vectorial=False, adjoint=False, field_hw=None):
    """Rayleigh-Sommerfeld convolution (Props/RSC_Prop.py:170-321) on the HIP kernels.

    [B,C,H,W] -> [Bo,C,Ph-H,Pw-W], Ph = H + 2 floor(H/2); vectorial: Ex/Ey planes in, 3 planes out.
    adjoint: the autograd backward of the scalar convolution, [B,C,Ph-H,Pw-W] -> [B,C,H,W] with
    (H, W) = field_hw, the forward field's shape.
    """
    _require_device(data, "RSC")
    if data.dtype not in (torch.complex64, torch.complex128):
        raise TypeError(f"RSC kernels compute in complex64 or complex128; got {data.dtype}")
    f64 = data.dtype == torch.complex128
    data = data.contiguous()
    B, C = data.shape[:2]
    H, W = field_hw if adjoint else data.shape[-2:]
    if f64:
        wl = _lib.double_array(wavelengths)
        d = _lib.RscDesc64(B=B, C=C, H=int(H), W=int(W), vectorial=int(bool(vectorial)), dx=float(spacing[0]),
                           dy=float(spacing[1]), z=float(z),
                           wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_double)), adjoint=int(bool(adjoint)))
    else:
        wl = _lib.float_array(wavelengths)
        d = _lib.RscDesc(B=B, C=C, H=int(H), W=int(W), vectorial=int(bool(vectorial)), dx=float(spacing[0]),
                         dy=float(spacing[1]), z=float(z), wavelengths=ctypes.cast(wl, ctypes.POINTER(ctypes.c_float)),
                         adjoint=int(bool(adjoint)))
    L = _lib.lib()
    size_fn, run_fn = (L.thz_rsc64_workspace_size, L.thz_rsc64_forward) if f64 else \
        (L.thz_rsc_workspace_size, L.thz_rsc_forward)
    nbytes = ctypes.c_size_t(0)
    _lib.check(size_fn(ctypes.byref(d), ctypes.byref(nbytes)))
    ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=data.device)
    if adjoint:
        if tuple(data.shape[-2:]) != (2 * (H // 2), 2 * (W // 2)):
            raise ValueError(f"RSC adjoint: gradient {tuple(data.shape)} does not match field {(H, W)}")
        out = torch.empty((B, C, int(H), int(W)), dtype=data.dtype, device=data.device)
    else:
        Bo = 3 if vectorial else B
        out = torch.empty((Bo, C, 2 * (H // 2), 2 * (W // 2)), dtype=data.dtype, device=data.device)
    if out.numel() == 0 or data.numel() == 0:
        # H or W = 1: the reference's [..., H:, W:] window is empty (Props/RSC_Prop.py:203-207; run
        # here: [B, C, 0, 2 (W // 2)] and the like); the adjoint of an empty output is zero
        return out.zero_()
    with torch.cuda.device(data.device):
        _lib.check(run_fn(ctypes.byref(d), ctypes.c_void_p(data.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                          ctypes.c_void_p(ws.data_ptr()), ctypes.c_size_t(ws.numel()), _stream_handle()))
    return out
