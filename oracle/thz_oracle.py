"""CPU ORACLE for the hot path -- TEST INFRASTRUCTURE ONLY.

This is a PyTorch-CPU restatement of the reference's algorithms for the
propagators and the DOE modulation.  It keeps the
reference's operation sequence (centred ``fftshift`` grids, fully materialised
transfer functions, per-call rebuild) so that it is both

* the parity checker for the HIP kernels (``tests/``, ``__graft_entry__.smoke``), and
* the ``cpu_baseline`` leg of ``bench.py`` (``kind: "port"``).

It is never imported by the product package ``quantizationawarethzdoe_amd``.
Parity status: PINNED -- ``tests/test_oracle_golden.py`` checks every function
here against fixtures produced by running the reference itself
(``tests/golden/gen_golden.py``): fp32 to <=1e-6 rel-L2 against the reference's
fp32 outputs and fp64 to <=1e-12 against the reference's fp64 outputs.

All functions take/return torch tensors; the working precision follows the
input dtype (complex64 -> fp32 math, complex128 -> fp64 math).
"""
from __future__ import annotations

import math

import torch

BASE_PLANE_THICKNESS = 2e-3  # Components/QuantizedDOE.py:23


def _rdt(x: torch.Tensor) -> torch.dtype:
    return torch.float64 if x.dtype in (torch.complex128, torch.float64) else torch.float32


# ---------------------------------------------------------------------------------------------
# ASM  (Props/ASM_Prop.py)
# ---------------------------------------------------------------------------------------------
def asm_padding(H: int, W: int, padding_scale, do_padding: bool = True):
    """pad = floor(s*N/2), P = N + 2 pad  (Props/ASM_Prop.py:119-136)."""
    if not do_padding:
        return 0, 0, H, W
    sh, sw = (padding_scale, padding_scale) if not isinstance(padding_scale, (list, tuple)) else padding_scale
    ph = int(math.floor(float(sh) * H / 2))
    pw = int(math.floor(float(sw) * W / 2))
    return ph, pw, H + 2 * ph, W + 2 * pw


def ft2(x):
    """Centred ortho 2-D FFT (utils/Helper_Functions.py:99-160, core :150)."""
    return torch.fft.fftshift(torch.fft.fft2(torch.fft.fftshift(x, dim=(-2, -1)), norm="ortho"), dim=(-2, -1))


def ift2(x):
    """Centred ortho inverse 2-D FFT (utils/Helper_Functions.py:111-160, ifftshift variant)."""
    return torch.fft.ifftshift(torch.fft.ifft2(torch.fft.ifftshift(x, dim=(-2, -1)), norm="ortho"), dim=(-2, -1))


def asm_transfer_function(Ph, Pw, wavelengths, dx, dy, z, bandlimit=True, bandlimit_type="exact", rdt=torch.float32):
    """Band-limited ASM transfer function on the centred grid, [1, C, Ph, Pw].

    Restates Props/ASM_Prop.py:138-145 (frequency grid: (i - P//2)/P, meshgrid 'ij'),
    :245-262 (H = exp(i z sqrt(k^2 - K^2)), evanescent -> 0) and :288-306 (Matsushima
    2009 band limits; note the reference uses the padded HEIGHT Ph for both axes,
    :274-275 and :290-291).
    """
    kx = (torch.linspace(0, Ph - 1, Ph, dtype=rdt) - (Ph // 2)) / Ph
    ky = (torch.linspace(0, Pw - 1, Pw, dtype=rdt) - (Pw // 2)) / Pw
    KX, KY = torch.meshgrid(kx, ky, indexing="ij")
    lam = wavelengths.to(rdt)[None, :, None, None]
    dx = torch.as_tensor(dx, dtype=rdt)
    dy = torch.as_tensor(dy, dtype=rdt)
    z = torch.as_tensor(z, dtype=rdt)
    Kx = 2 * math.pi * KX[None, None] / dx
    Ky = 2 * math.pi * KY[None, None] / dy
    K2 = Kx ** 2 + Ky ** 2
    k = 2 * torch.tensor(math.pi, dtype=torch.float64) / lam
    k2 = k ** 2
    H = torch.exp(1j * (z * torch.sqrt(k2 - K2)))
    H[(k2 - K2) < 0] = 0
    if bandlimit:
        du = ((2 * math.pi / dx) / (2 * Ph)) / (2 * math.pi)
        dv = ((2 * math.pi / dy) / (2 * Ph)) / (2 * math.pi)
        ulim = 1 / torch.sqrt((2 * du * z) ** 2 + 1) / lam
        vlim = 1 / torch.sqrt((2 * dv * z) ** 2 + 1) / lam
        if bandlimit_type == "exact":
            c1 = ((Kx ** 2) / ((2 * math.pi * ulim) ** 2) + (Ky ** 2) / (k ** 2)) <= 1
            c2 = ((Kx ** 2) / (k ** 2) + (Ky ** 2) / ((2 * math.pi * vlim) ** 2)) <= 1
            H[~(c1 & c2)] = 0
        elif bandlimit_type == "approx":
            Lx = Ph * dx
            Ly = Ph * dy
            kxm = 2 * math.pi / torch.sqrt((2 * (1 / Lx) * z) ** 2 + 1) / lam
            kym = 2 * math.pi / torch.sqrt((2 * (1 / Ly) * z) ** 2 + 1) / lam
            H[(torch.abs(Kx) > kxm) | (torch.abs(Ky) > kym)] = 0
        else:
            raise Exception("Should not be in this state.")
    return H


def asm_critical_distance(Ph, dx, wavelengths):
    """Zc = Ph dx^2 sqrt(1 - (lmax/2dx)^2) / lmax  (Props/ASM_Prop.py:280)."""
    lmax = float(torch.max(torch.as_tensor(wavelengths)))
    dx = float(dx)
    return Ph * dx ** 2 * math.sqrt(1 - (lmax / (2 * dx)) ** 2) / lmax


def asm_forward(data, wavelengths, spacing, z, padding_scale=1, do_padding=True, do_unpad_after_pad=True,
                bandlimit=True, bandlimit_type="exact"):
    """pad -> ft2 -> x H -> ift2 -> centre crop  (Props/ASM_Prop.py:314-378)."""
    rdt = _rdt(data)
    B, C, H, W = data.shape
    ph, pw, Ph, Pw = asm_padding(H, W, padding_scale, do_padding)
    x = torch.nn.functional.pad(data, (pw, pw, ph, ph)) if do_padding else data
    Hf = asm_transfer_function(Ph, Pw, torch.as_tensor(wavelengths), spacing[0], spacing[1], z, bandlimit,
                               bandlimit_type, rdt)
    y = ift2(ft2(x) * Hf)
    if do_padding and do_unpad_after_pad:
        top = int(round((Ph - H) / 2.0))
        left = int(round((Pw - W) / 2.0))
        y = y[..., top:top + H, left:left + W]
    return y


def asm_forward_planes(data, wavelengths, spacing, zs, padding_scale=1, bandlimit_type="exact"):
    """The multi-z sweep of experiment_extend_depth_of_focus.ipynb:229,255-256 (``asm.z = z;
    asm(field)`` per plane): yields (z, asm_forward(data, .., z, ..)) for each z.  ft2(pad x) does not
    depend on z, so it is computed once -- the same operations as the per-plane call, hence the
    same values, at a fraction of the cost for the full-size (P = 8192) parity tests."""
    rdt = _rdt(data)
    B, C, H, W = data.shape
    ph, pw, Ph, Pw = asm_padding(H, W, padding_scale, True)
    spec = ft2(torch.nn.functional.pad(data, (pw, pw, ph, ph)))
    top = int(round((Ph - H) / 2.0))
    left = int(round((Pw - W) / 2.0))
    for z in zs:
        Hf = asm_transfer_function(Ph, Pw, torch.as_tensor(wavelengths), spacing[0], spacing[1], z, True,
                                   bandlimit_type, rdt)
        y = ift2(spec * Hf)[..., top:top + H, left:left + W]
        del Hf
        yield z, y


# ---------------------------------------------------------------------------------------------
# CZT  (Props/CZT_Prop.py)
# ---------------------------------------------------------------------------------------------
def _rs_kernel(z, mx, my, lam):
    """exp(ikr) z/(2 pi r^2) (1/r - ik)  (Props/CZT_Prop.py:44-57)."""
    k = 2 * torch.pi / lam[None, :, None, None]
    r = torch.sqrt(mx ** 2 + my ** 2 + z ** 2)
    return torch.exp(1j * k * r) * (1 / (2 * torch.pi) * z / r ** 2 * (1 / r - 1j * k))


def _bluestein(x, f1, f2, Dm, M):
    """One Bluestein pass along dim -2 with the reference's slicing (Props/CZT_Prop.py:132-225).

    Output is the reference's transposed [.., n, M] layout with the off-by-one slice
    ``[m : m+M]`` and post-chirp ``h[m-1 : m-1+M]`` (:211), then M_shift (:214-224).
    """
    _, _, m, n = x.shape
    D1 = f1 + (M * Dm + f2 - f1) / (2 * M)
    D2 = f2 + (M * Dm + f2 - f1) / (2 * M)
    mp = m + M - 1
    np2 = int(2 ** int(math.ceil(math.log2(mp))))
    A = torch.exp(1j * 2 * torch.pi * D1 / Dm)
    Wc = torch.exp(-1j * 2 * torch.pi * (D1 - D2) / (M * Dm))
    jj = torch.arange(-m + 1, max(M - 1, m - 1) + 1)
    h = Wc ** (jj ** 2 / 2)
    ft = torch.fft.fft(1 / h[: mp + 1], n=np2, dim=-1)
    pre = A ** (-(torch.arange(0, m))) * h[..., torch.arange(m - 1, 2 * m - 1)]
    b = torch.fft.fft(x * torch.tile(pre, (1, 1, n, 1)).transpose(-2, -1), np2, dim=-2)
    b = torch.fft.ifft(b * torch.tile(ft, (1, 1, n, 1)).transpose(-2, -1), dim=-2)
    b = b[..., m:mp + 1, 0:n].transpose(-2, -1) * torch.tile(h[..., m - 1:mp], (1, 1, n, 1))
    ell = torch.linspace(0, M - 1, M)[None, None, None, :]
    ell = ell / M * (D2 - D1) + D1
    shift = torch.tile(torch.exp(-1j * 2 * torch.pi * ell * (-m / 2 + 0.5) / Dm), (1, 1, n, 1))
    return b * shift


def czt_forward(data, wavelengths, spacing, z, outH=None, outW=None, odx=None, ody=None):
    """Chirp-z (Bluestein) RS propagation  (Props/CZT_Prop.py:59-118, 227-314).

    Runs in torch's current default float dtype for the grids (as the reference does);
    callers set ``torch.set_default_dtype(torch.float64)`` for the fp64 oracle.
    """
    _, C, H, W = data.shape
    dxi, dyi = spacing[0], spacing[1]
    outH = H if outH is None else outH
    outW = W if outW is None else outW
    odx = dxi if odx is None else odx
    ody = dyi if ody is None else ody
    lam = torch.as_tensor(wavelengths)
    z = torch.as_tensor(z)
    xi = torch.linspace(-H * dxi / 2, H * dxi / 2, H)
    yi = torch.linspace(-W * dyi / 2, W * dyi / 2, W)
    imx, imy = torch.meshgrid(xi, yi, indexing="ij")
    xo = torch.linspace(-outH * odx / 2, outH * odx / 2, outH)
    yo = torch.linspace(-outW * ody / 2, outW * ody / 2, outW)
    omx, omy = torch.meshgrid(xo, yo, indexing="ij")
    Dm = lam[None, :, None, None] * z / dxi
    fx1, fx2 = xo[0] + Dm / 2, xo[-1] + Dm / 2
    fy1, fy2 = yo[0] + Dm / 2, yo[-1] + Dm / 2
    F0 = _rs_kernel(z, omx, omy, lam)
    F = _rs_kernel(z, imx, imy, lam)
    U = data * F
    U = _bluestein(U, fy1, fy2, Dm, outW)
    U = _bluestein(U, fx1, fx2, Dm, outH)
    return F0 * U * z * odx * ody * lam[None, :, None, None]


# ---------------------------------------------------------------------------------------------
# RSC  (Props/RSC_Prop.py)
# ---------------------------------------------------------------------------------------------
def rsc_forward(data, wavelengths, spacing, z):
    """Rayleigh-Sommerfeld convolution on a 2N grid (Props/RSC_Prop.py:79-87, 129-215).

    Grid: linspace(-P dx/2, P dx/2, P) on BOTH axes with dx (:83-84); B must be 1 (:198-200).
    """
    B, C, H, W = data.shape
    dx, dy = spacing[0], spacing[1]
    Ph, Pw = H + 2 * (H // 2), W + 2 * (W // 2)
    lam = torch.as_tensor(wavelengths)
    z = torch.as_tensor(z)
    x = torch.linspace(-Ph * dx / 2, Ph * dx / 2, Ph)
    y = torch.linspace(-Pw * dx / 2, Pw * dx / 2, Pw)
    mx, my = torch.meshgrid(x, y, indexing="ij")
    k = 2 * torch.pi / lam[:, None, None]
    r = torch.sqrt(mx ** 2 + my ** 2 + z ** 2)
    K = (torch.exp(1j * k * r) * (1 / (2 * torch.pi) * z / r ** 2 * (1 / r - 1j * k)))[None]
    U = torch.zeros_like(K)
    U[..., 0:H, 0:W] = data
    S = torch.fft.fft2(U) * torch.fft.fft2(K) * dx * dy
    return torch.fft.ifft2(S)[..., H:, W:]


# ---------------------------------------------------------------------------------------------
# DOE  (Components/QuantizedDOE.py)
# ---------------------------------------------------------------------------------------------
def doe_transmission(height, wavelengths, eps, tand):
    """t_c(h) = exp(-k/2 (h+b) tand sqrt(eps)) exp(-i k (h+b)(sqrt(eps)-1))  (QuantizedDOE.py:47-79)."""
    lam = torch.as_tensor(wavelengths).reshape(-1)[:, None, None]
    k = 2 * torch.pi / lam
    eps = torch.as_tensor(eps, dtype=height.dtype)
    tand = torch.as_tensor(tand, dtype=height.dtype)
    hb = height[None] + torch.tensor(BASE_PLANE_THICKNESS, dtype=height.dtype)
    loss = torch.exp(-0.5 * k * hb * tand * torch.sqrt(eps))
    delay = torch.exp(-1j * k * hb * (torch.sqrt(eps) - 1))
    return loss * delay


def doe_modulate(field, height, wavelengths, eps, tand, tolerance=None, noise_u01=None):
    """add_height_map_noise -> nearest upsample -> x t  (QuantizedDOE.py:82-126).

    ``noise_u01`` injects the ``rand_like`` draw (U[0,1)) the reference consumes at :85.
    """
    h = height
    if tolerance is not None:
        u = noise_u01 if noise_u01 is not None else torch.rand_like(h)
        h = h + (u - 0.5) * 2 * tolerance
    H, W = field.shape[-2:]
    if h.shape[0] != H or h.shape[1] != W:
        h = torch.nn.functional.interpolate(h[None, None], size=[H, W], mode="nearest")[0, 0]
    return field * doe_transmission(h, wavelengths, eps, tand)[None]


def copy_quad_to_full(q):
    """Mirror a quadrant into the full map (QuantizedDOE.py:28-35), 2-D form."""
    left = torch.cat([torch.flip(q, dims=[0]), q], dim=0)
    return torch.cat([torch.flip(left, dims=[1]), left], dim=1)


def height_to_phase(h, lam, n):
    """QuantizedDOE.py:40-41."""
    return 2 * torch.pi / lam * (n - 1) * h


def sgv3_score(phase, phase_lut, s):
    """score_phase(func='sigmoid')  (QuantizedDOE.py:794-817)."""
    wp = (phase + torch.pi) % (2 * torch.pi) - torch.pi
    lut = (phase_lut[None, :, None, None] + torch.pi) % (2 * torch.pi) - torch.pi
    d = wp - lut
    d = (d + torch.pi) % (2 * torch.pi) - torch.pi
    d = d / torch.pi
    zz = s * d
    return torch.sigmoid(zz) * (1 - torch.sigmoid(zz)) * 4


def sgv3_tau(iter_frac, tau_min, tau_max):
    """Cosine temperature schedule (QuantizedDOE.py:869-871)."""
    return tau_min + 0.5 * (tau_max - tau_min) * (1 + math.cos(iter_frac * math.pi))


def sgv3_height_map(weight, lut, hmax, lam_min, eps, iter_frac, c_s, tau_max, tau_min, expo=None, num_unit=2):
    """SoftGumbelQuantizedDOELayerv3.preprocessed_height_map  (QuantizedDOE.py:819-860).

    ``expo`` injects the Exp(1) draw ``F.gumbel_softmax`` consumes (gumbel = -log(expo)).
    Straight-through forward value: one-hot of argmax((s + g)/tau) over the level axis.
    """
    tau = sgv3_tau(iter_frac, tau_min, tau_max)
    h = hmax * torch.sigmoid(torch.clamp(weight, min=-10.0, max=10.0))[None, None]
    if iter_frac > 0.3:
        n = torch.sqrt(torch.as_tensor(eps, dtype=weight.dtype))
        plut = height_to_phase(lut, lam_min, n)
        qph = height_to_phase(h, lam_min, n)
        sc = sgv3_score(qph, plut, tau_max / tau) * c_s * (tau_max / tau)
        g = -torch.log(expo) if expo is not None else -torch.empty_like(sc).exponential_().log()
        y = torch.softmax((sc + g) / tau, dim=1)
        idx = y.argmax(dim=1, keepdim=True)
        onehot = torch.zeros_like(y).scatter_(1, idx, 1.0)
        q = (lut.reshape(1, -1, 1, 1) * onehot).sum(1, keepdim=True)
        if iter_frac <= 0.8:
            beta = (iter_frac - 0.3) / (0.8 - 0.3)
            h = (1 - beta) * h + beta * q
        else:
            h = q
    h = h[0, 0]
    return copy_quad_to_full(h) if num_unit is not None else h


def ste_quantize(h, lut):
    """Nearest-LUT level (first on ties), identity gradient (QuantizedDOE.py:1239-1255)."""
    idx = torch.argmin(torch.abs(h.unsqueeze(-1) - lut), dim=-1)
    return lut[idx]


def fp_height(weight, hmax, clamp=8.0):
    """h_max * sigmoid(clamp(w)) (QuantizedDOE.py:287, :823 with clamp 10)."""
    return hmax * torch.sigmoid(torch.clamp(weight, min=-clamp, max=clamp))


def gumbel_hard(logits, tau, expo, dim):
    """F.gumbel_softmax(hard=True) with the Exp(1) draw injected: straight-through one-hot."""
    y = torch.softmax((logits + (-torch.log(expo))) / tau, dim=dim)
    idx = y.argmax(dim=dim, keepdim=True)
    hard = torch.zeros_like(y).scatter_(dim, idx, 1.0)
    return hard - y.detach() + y


def psq_height(weight, hmax, L, tau):
    """PSQuantizedDOELayer.preprocessed_height_map (QuantizedDOE.py:1193-1216), before mirroring."""
    h = fp_height(weight, hmax, 8.0)
    delta = (hmax - 0) / (L - 1)
    xn = (h - 0) / delta - 0.5
    levels = torch.arange(L - 1).unsqueeze(0).unsqueeze(2)
    return 0 + delta * torch.sum(torch.sigmoid(tau * (xn.unsqueeze(1) - levels)), dim=1)


def radial_map(profile, R, H, W):
    """Rotationally symmetric expansion (QuantizedDOE.py:1412-1432): bins floor(r) < R-1."""
    x, y = torch.meshgrid(torch.arange(0, R), torch.arange(0, R), indexing="ij")
    r = torch.sqrt(x ** 2 + y ** 2)
    quad = torch.where((r < 1.0) & (r >= 0.0), profile[0], 0)
    for k in range(1, R - 1):
        quad = quad + torch.where((r < float(k + 1)) & (r >= float(k)), profile[k], 0)
    full = copy_quad_to_full(quad)
    sx, sy = R - H // 2, R - W // 2
    return full[sx:sx + H, sy:sy + W]


def _scores(phase, plut, tau, c_s, tau_max):
    return sgv3_score(phase, plut, tau_max / tau) * c_s * (tau_max / tau)


def layer_height_map(cls, weight, lut, hmax, lam_min, eps, iter_frac, optim, num_unit, doe_size, expo=None):
    """preprocessed_height_map of every QAT layer class (QuantizedDOE.py:286-1623), RNG injected.

    ``weight`` is the layer's parameter as the reference shapes it; ``expo`` the Exp(1) draw.
    """
    L = len(lut)
    n = torch.sqrt(torch.as_tensor(eps, dtype=torch.float32))
    tmin, tmax = optim.get("tau_min"), optim.get("tau_max")
    cos_tau = sgv3_tau(iter_frac, tmin, tmax) if iter_frac is not None else None
    mirror = (lambda h: copy_quad_to_full(h)) if num_unit is not None else (lambda h: h)
    rot = cls.startswith("RotationallySymmetric")
    R = int(doe_size[0] * torch.sqrt(torch.tensor(2)) / 2)
    finish = (lambda p: radial_map(p.reshape(-1), R, doe_size[0], doe_size[1])) if rot else None
    if cls in ("FullPrecisionDOELayer", "RotationallySymmetricFullPrecisionDOELayer"):
        h = fp_height(weight, hmax, 8.0)
        return finish(h) if rot else mirror(h.reshape(h.shape[-2:]))
    if cls in ("STEQuantizedDOELayer", "RotationallySymmetricSTEQuantizedDOELayer"):
        h = fp_height(weight, hmax, 8.0)
        h = h if rot else mirror(h.reshape(h.shape[-2:]))
        q = h + (ste_quantize(h, lut) - h).detach()  # identity gradient
        return finish(q) if rot else q
    if cls in ("PSQuantizedDOELayer", "RotationallySymmetricPSQuantizedQuantizedDOELayer"):
        tau = tmin + (tmax - tmin) * iter_frac
        h = psq_height(weight, hmax, L, tau)
        return finish(h) if rot else mirror(h)
    if cls in ("NaiveGumbelQuantizedDOELayer", "RotationallySymmetricNaiveGumbelQuantizedDOELayer"):
        oh = gumbel_hard(weight, cos_tau if cos_tau is not None else 1, expo, -1)
        h = (lut[None, None, :] * oh).sum(dim=-1)
        return finish(h) if rot else mirror(h)
    if cls == "SoftGumbelQuantizedDOELayer":
        oh = gumbel_hard(_scores(weight, height_to_phase(lut, lam_min, n), cos_tau, optim["c_s"], tmax),
                         cos_tau, expo, 1)
        h = (lut.reshape(1, L, 1, 1) * oh).sum(1, keepdim=True)
        if num_unit is not None:
            raise NotImplementedError("v1 with num_unit tiles by the 4-D shape (reference quirk)")
        return h[0, 0]
    if cls in ("SoftGumbelQuantizedDOELayerv2", "SoftGumbelQuantizedDOELayerv3",
               "RotationallySymmetricScoreGumbelSoftQuantizedDOELayer"):
        h = fp_height(weight, hmax, 10.0)
        if weight.dim() == 2:
            h = h[None, None]
        v2 = cls.endswith("v2")
        quant = iter_frac > 0.5 if v2 else iter_frac > 0.3
        if quant:
            oh = gumbel_hard(_scores(height_to_phase(h, lam_min, n), height_to_phase(lut, lam_min, n), cos_tau,
                                     optim["c_s"], tmax), cos_tau, expo, 1)
            q = (lut.reshape(1, L, 1, 1) * oh).sum(1, keepdim=True)
            if not v2 and iter_frac <= 0.8:
                beta = iter_frac if rot else (iter_frac - 0.3) / (0.8 - 0.3)
                h = (1 - beta) * h + beta * q
            else:
                h = q
        if rot:
            return finish(h)
        return mirror(h[0, 0]) if not v2 else h[0, 0]
    raise ValueError(f"unknown layer class {cls}")


# ---------------------------------------------------------------------------------------------
# optical elements and the QAT loss
# ---------------------------------------------------------------------------------------------
WAIST_FIT_E = [2.70171433587848e-13, 3.10350492358753e-10, -6.35088689290759e-07, 0.000322826804965868,
               -0.0665921902050336, 6.08799187520401]
WAIST_FIT_H = [-1.01507121315420e-11, 1.70791445624058e-08, -1.12281052414283e-05, 0.00360605624858374,
               -0.564799749943028, 35.5588926870041]


def waist_fit(wavelengths):
    """BeamWaistCorruagtedTK (LightSource/Gaussian_beam.py:67-85) on f = c / lambda in GHz."""
    f = (2.998e8 / wavelengths) / 1e9
    return [1e-3 * (p[0] * f ** 5 + p[1] * f ** 4 + p[2] * f ** 3 + p[3] * f ** 2 + p[4] * f + p[5])
            for p in (WAIST_FIT_E, WAIST_FIT_H)]


def gaussian_beam(H, W, dx, dy, wavelengths, waist_x=None, waist_y=None, center=(0, 0), z_w0=(0, 0), alpha=0):
    """Guassian_beam.forward (LightSource/Gaussian_beam.py:88-160) -> [1, C, H, W]."""
    lam = torch.as_tensor(wavelengths).reshape(-1)
    if waist_x is None:
        wx0, wy0 = waist_fit(lam)
    else:
        wx0 = torch.full_like(lam, waist_x)
        wy0 = torch.full_like(lam, waist_y)
    dx, dy = torch.as_tensor(dx, dtype=lam.dtype), torch.as_tensor(dy, dtype=lam.dtype)
    x = torch.linspace(-dx * H / 2, dx * H / 2, H, dtype=lam.dtype)
    y = torch.linspace(-dy * W / 2, dy * W / 2, W, dtype=lam.dtype)
    X, Y = torch.meshgrid(x, y, indexing="ij")
    X, Y = X[None], Y[None]
    lam3 = lam[:, None, None]
    k = 2 * torch.pi / lam3
    wx0, wy0 = wx0[:, None, None], wy0[:, None, None]
    zx, zy = torch.tensor(z_w0[0], dtype=lam.dtype), torch.tensor(z_w0[1], dtype=lam.dtype)
    x0, y0 = torch.tensor(center[0], dtype=lam.dtype), torch.tensor(center[1], dtype=lam.dtype)
    a = torch.tensor(alpha, dtype=lam.dtype)
    zrx, zry = torch.pi * wx0 ** 2 / lam3, torch.pi * wy0 ** 2 / lam3
    gx, gy = torch.arctan2(zx, zrx), torch.arctan2(zy, zry)
    wx = wx0 * torch.sqrt(1 + (zx / zrx) ** 2)
    wy = wy0 * torch.sqrt(1 + (zy / zry) ** 2)
    rx = 1e12 if z_w0[0] == 0 else zx * (1 + (zrx / zx) ** 2)
    ry = 1e12 if z_w0[1] == 0 else zy * (1 + (zry / zy) ** 2)
    xr = X * torch.cos(a) + Y * torch.sin(a)
    yr = -X * torch.sin(a) + Y * torch.cos(a)
    phase = torch.exp(-1j * ((k * zx + k * X ** 2 / (2 * rx) - gx) + (k * zy + k * Y ** 2 / (2 * ry) - gy)))
    A = (wx0 / wx) * (wy0 / wy) * torch.exp(-(xr - x0) ** 2 / (wx ** 2) - (yr - y0) ** 2 / (wy ** 2))
    return (A * phase)[None]


def thin_lens(field, dx, dy, focal_length, wavelengths):
    """Thin_LensElement.forward (Components/Thin_Lens.py:31-85)."""
    H, W = field.shape[-2:]
    lam = torch.as_tensor(wavelengths).reshape(-1)[:, None, None]
    xc = torch.linspace(-((H - 1) // 2), (H - 1) // 2, H, dtype=lam.dtype)
    yc = torch.linspace(-((W - 1) // 2), (W - 1) // 2, W, dtype=lam.dtype)
    xg, yg = torch.meshgrid(xc, yc, indexing="ij")
    xg = xg[None, None] * torch.tensor([dx], dtype=lam.dtype)[:, None, None]
    yg = yg[None, None] * torch.tensor([dy], dtype=lam.dtype)[:, None, None]
    f = torch.tensor([focal_length], dtype=lam.dtype)
    ang = -(math.pi / (lam * f)) * (xg ** 2 + yg ** 2)
    return field * torch.exp(1j * ang)


def aperture_mask(H, W, dx, dy, kind, size):
    """ApertureElement masks (Components/Aperture.py:61-118): rect on an 'xy' grid, circ on 'ij'."""
    dx, dy = torch.as_tensor(dx, dtype=torch.float32), torch.as_tensor(dy, dtype=torch.float32)
    if kind == "rect":
        rw = min(size, dx * W) if size is not None else dx * W / 2
        rh = min(size, dy * H) if size is not None else dy * H / 2
        x = torch.linspace(-dx * W / 2, dx * W / 2, W, dtype=dx.dtype)
        y = torch.linspace(-dy * H / 2, dy * H / 2, H, dtype=dy.dtype)
        X, Y = torch.meshgrid(x, y, indexing="xy")
        return torch.where((torch.abs(X) <= rw / 2) & (torch.abs(Y) <= rh / 2), 1, 0)
    r = torch.tensor(size)
    x = torch.linspace(-dx * H / 2, dx * H / 2, H, dtype=dx.dtype)
    y = torch.linspace(-dy * W / 2, dy * W / 2, W, dtype=dy.dtype)
    X, Y = torch.meshgrid(x, y, indexing="ij")
    return torch.where(torch.sqrt(X ** 2 + Y ** 2) <= r, 1, 0)


def intensity_mse(field, target):
    """MSE(normalize(|E|^2), target) of the QAT loop (experiment_four_focal_spots.ipynb:336-370)."""
    amp = normalize(torch.abs(field) ** 2)
    return torch.mean((amp - target.expand_as(amp)) ** 2)


def resample(field, spacing, Hout, Wout, dx_out, dy_out):
    """Field_Resampler.forward (Addons/Field_Resampler.py:56-118): bilinear grid_sample onto the
    centred output grid (generateGrid, Helper_Functions.py:163-182), zeros, align_corners."""
    B, C, H, W = field.shape
    xc = torch.linspace(-((Hout - 1) // 2), (Hout - 1) // 2, Hout) * dx_out
    yc = torch.linspace(-((Wout - 1) // 2), (Wout - 1) // 2, Wout) * dy_out
    gX, gY = torch.meshgrid(xc, yc, indexing="ij")
    dx = torch.tensor([spacing[0]])[:, None, None]
    dy = torch.tensor([spacing[1]])[:, None, None]
    xn = (dx * ((H - 1) // 2))[:, :, None, :]
    yn = (dy * ((W - 1) // 2))[:, :, None, :]
    grid = torch.stack([gY, gX], dim=-1).repeat(B, 1, 1, 1).to(field.real.dtype)
    grid[..., 0] = grid[..., 0] / yn
    grid[..., 1] = grid[..., 1] / xn
    gs = torch.nn.functional.grid_sample
    re = gs(field.real, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    im = gs(field.imag, grid, mode="bilinear", padding_mode="zeros", align_corners=True)
    return re + 1j * im


def normalize(x):
    """Per-batch divide by max (utils/Helper_Functions.py:185-193), out of place."""
    B = x.shape[0]
    v = x.reshape(B, -1)
    return (v / v.max(1, keepdim=True)[0]).reshape(x.shape)
