"""The plane recurrence of the power-of-two column pass (csrc/thz_asm.hip asm_cols_body,
recurrence_step_ok): for a uniform z-sweep (cfg2's linspace, experiment_extend_depth_of_focus.ipynb:229)
the column pass advances G_j = sp H_{z_j} by one complex product per plane instead of one sincos
per element per plane (Props/ASM_Prop.py:257-262 evaluates exp(i z sqrt(k^2 - K^2)) per plane).

Tolerances: each plane vs the fp64 oracle <= max(1e-4, 1.5 x the fp32 oracle's own error on it)
(tests/test_asm_gpu.py's rule), and vs the per-plane sincos form of the same kernel (the
THZ_K2_RECURRENCE=0 switch) <= 2e-5 rel-L2: the recurrence's phase error is <= 4e-6 rad after 64
planes (D rounded once to fp32, 6e-8 per plane) against the sincos form's fp32 rounding of z sq
(<= 3e-5 rad at z sq ~ 750 rad).  The first plane the recurrence runs is bit-identical in both
forms: the chunk's first plane for an increasing sweep (the band narrows with z), its last plane for
a decreasing one (run backwards, so the band still only narrows).
"""
import os

import numpy as np
import pytest
import torch

from oracle import thz_oracle as orc
from tests.golden_io import rel_l2, spacing, wavelengths

pytestmark = pytest.mark.gpu
C0 = 2.998e8


def _run(x, lam, sp, zs, pad, recurrence, **kw):
    from quantizationawarethzdoe_amd.propagation import asm_apply
    old = os.environ.get("THZ_K2_RECURRENCE")
    os.environ["THZ_K2_RECURRENCE"] = "1" if recurrence else "0"
    try:
        out = asm_apply(x, lam, sp, zs, pad, pad, True, 1, **kw)
        torch.cuda.synchronize()
        return out
    finally:
        if old is None:
            del os.environ["THZ_K2_RECURRENCE"]
        else:
            os.environ["THZ_K2_RECURRENCE"] = old


def _narrow_input(N, seed):
    """A white N^2 field at cfg2's sampling (dx 0.25 mm at 300 GHz: the evanescent cut sits at
    |m_x| = P/4, so the recurrence carries 8 of each thread's 16 spectrum values)."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(1, 1, N, N, dtype=torch.complex64, device=dev, generator=g)
    lam = [float(torch.tensor(C0 / 300e9, dtype=torch.float32))]
    sp = [float(torch.tensor(0.25e-3, dtype=torch.float32))] * 2
    return x, lam, sp


@pytest.mark.parametrize("zs", [
    [float(v) for v in torch.linspace(20e-3, 120e-3, 64, dtype=torch.float64)],   # cfg2's sweep
    [float(v) for v in torch.linspace(150e-3, 10e-3, 37, dtype=torch.float64)],   # decreasing
    [0.05 + 0.004 * k for k in range(9)],                                         # short, host floats
], ids=["cfg2_sweep", "decreasing", "nine"])
def test_recurrence_vs_sincos_and_oracle(zs):
    x, lam, sp = _narrow_input(1024, 3)
    a = _run(x, lam, sp, zs, 512, True)
    b = _run(x, lam, sp, zs, 512, False)
    # the recurrence's first plane: the sweep's nearest plane (where the band is widest)
    first = 0 if zs[-1] > zs[0] else len(zs) - 1
    assert torch.equal(a[first], b[first])
    # the two forms really differ elsewhere (the recurrence ran)
    assert not torch.equal(a, b)
    for k in range(len(zs)):
        assert rel_l2(a[k].cpu().numpy(), b[k].cpu().numpy()) <= 2e-5, k
    check = sorted({0, 1, len(zs) // 2, len(zs) - 1})
    xt = x.cpu()
    lt = torch.tensor(lam, dtype=torch.float32)
    st = torch.tensor(sp, dtype=torch.float32)
    with torch.no_grad():
        r64 = orc.asm_forward_planes(xt.to(torch.complex128), lt.double(), st.double(), [zs[k] for k in check], 1)
        r32 = orc.asm_forward_planes(xt, lt, st, [zs[k] for k in check], 1)
    for k, (_, p64), (_, p32) in zip(check, r64, r32):
        floor = rel_l2(p32.numpy(), p64.numpy())
        e = rel_l2(a[k].cpu().numpy(), p64.numpy())
        assert e <= max(1e-4, 1.5 * floor), (k, zs[k], e, floor)


@pytest.mark.parametrize("order", ["increasing", "decreasing"])
def test_recurrence_split_chunks_and_kparts(order):
    """40 planes in z-chunks of 16 (two full chunks and a tail of 8): each chunk restarts the
    recurrence from its own first plane in run order (its first plane, or its last for a decreasing
    sweep), and the last dispatch round's columns split into z-ranges (kparts) restart it from each
    range's own."""
    x, lam, sp = _narrow_input(1024, 4)
    zs = [float(v) for v in torch.linspace(30e-3, 90e-3, 40, dtype=torch.float64)]
    if order == "decreasing":
        zs = zs[::-1]
    a = _run(x, lam, sp, zs, 512, True, z_chunk=16)
    b = _run(x, lam, sp, zs, 512, False, z_chunk=16)
    for k in ((0, 16, 32) if order == "increasing" else (15, 31, 39)):
        assert torch.equal(a[k], b[k]), k
    assert not torch.equal(a, b)
    for k in range(40):
        assert rel_l2(a[k].cpu().numpy(), b[k].cpu().numpy()) <= 2e-5, k


@pytest.mark.parametrize("zs", [
    [0.02, 0.05, 0.06, 0.11],                 # non-uniform steps
    [0.05, 0.05 + 1e-4, 0.05 + 2.3e-4],       # |eps| k above 1e-4 rad
    [0.04, 0.07],                             # two planes
], ids=["nonuniform", "eps_too_large", "two_planes"])
def test_non_uniform_planes_keep_the_sincos_path(zs):
    """recurrence_step_ok refuses these lists: both settings of the switch run the same kernel
    code path and give bit-identical planes."""
    x, lam, sp = _narrow_input(512, 5)
    a = _run(x, lam, sp, zs, 256, True)
    b = _run(x, lam, sp, zs, 256, False)
    assert torch.equal(a, b)
    assert b.abs().amax() > 0


def test_wide_band_columns_keep_the_sincos_path():
    """dx 1 mm at 300 GHz: the band reaches |m_x| >= P/4 in every column, so no column takes the
    recurrence even for a uniform sweep -- bit-identical to the sincos form."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn(1, 1, 512, 512, dtype=torch.complex64, device=dev, generator=g)
    lam = [float(torch.tensor(C0 / 300e9, dtype=torch.float32))]
    sp = [float(torch.tensor(1e-3, dtype=torch.float32))] * 2
    zs = [float(v) for v in torch.linspace(0.05, 0.15, 8, dtype=torch.float64)]
    a = _run(x, lam, sp, zs, 256, True)
    b = _run(x, lam, sp, zs, 256, False)
    assert torch.equal(a, b)
    assert b.abs().amax() > 0


def test_recurrence_two_wavelengths_and_batch():
    """Two wavelengths (the per-channel kmax of the eps bound is the shorter one's) and a batch of
    two: every plane within 2e-5 of the sincos form."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(2, 2, 512, 512, dtype=torch.complex64, device=dev, generator=g)
    lam = [float(torch.tensor(C0 / 300e9, dtype=torch.float32)), float(torch.tensor(C0 / 280e9, dtype=torch.float32))]
    sp = [float(torch.tensor(0.25e-3, dtype=torch.float32))] * 2
    zs = [float(v) for v in torch.linspace(20e-3, 60e-3, 12, dtype=torch.float64)]
    a = _run(x, lam, sp, zs, 256, True)
    b = _run(x, lam, sp, zs, 256, False)
    assert not torch.equal(a, b)
    for k in range(len(zs)):
        assert rel_l2(a[k].cpu().numpy(), b[k].cpu().numpy()) <= 2e-5, k
