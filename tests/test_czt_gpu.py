"""CZT parity on the GPU vs the reference-generated golden fixtures (tests/golden/czt_golden.npz).

Tolerance: rel-L2 vs the fp64 golden <= max(3e-3, 1.25 x the reference's own fp32 error)
(CZT <= 3e-3; the reference's fp32 error is 6e-5 .. 4.1e-3 on these cases,
dominated by its fp32 complex pow chirps, which this build evaluates in double).
"""
import numpy as np
import pytest
import torch

from oracle import thz_oracle as orc
from tests.golden_io import arrays, manifest, rel_l2, wavelengths

pytestmark = pytest.mark.gpu
M = manifest()
C0 = 2.998e8


@pytest.mark.parametrize("case", M["czt"], ids=[c["name"] for c in M["czt"]])
def test_czt_forward_vs_golden(case):
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    A = arrays("czt")
    k = case["name"]
    dev = torch.device("cuda:0")
    wl = [C0 / (f * 1e9) for f in case["f"]]
    field = ElectricField(torch.from_numpy(A[f"{k}__in"]).to(dev), wavelengths=wl if len(wl) > 1 else wl[0],
                          spacing=[case["dx"] * 1e-3, case["dy"] * 1e-3], device=dev)
    prop = CZT_prop(z_distance=case["z"], device=dev)
    out = prop(field, outputHeight=case["oH"], outputWidth=case["oW"], outputPixel_dx=case["odx"] * 1e-3,
               outputPixel_dy=case["ody"] * 1e-3).data.cpu().numpy()
    assert out.shape == A[f"{k}__out64"].shape
    e64 = rel_l2(out, A[f"{k}__out64"])
    assert e64 <= max(3e-3, 1.25 * case["rel32vs64"]), (e64, case["rel32vs64"])
    assert e64 <= 1e-3, f"double-precision chirps should beat the reference's fp32 ({case['rel32vs64']:.1e}): {e64}"


def test_czt_rejects_non_square_output():
    from quantizationawarethzdoe_amd import propagation as P
    x = torch.zeros(1, 1, 32, 32, dtype=torch.complex64, device="cuda:0")
    with pytest.raises(RuntimeError, match="square"):
        P.czt_apply(x, [1e-3], [1e-3, 1e-3], 0.1, 16, 8, 1e-3, 1e-3)


@pytest.mark.parametrize("H,W,M", [(12, 12, 21), (12, 13, 20), (16, 16, 1), (13, 12, 20)])
def test_czt_power_of_two_bluestein_length_raises_like_the_reference(H, W, M):
    """H + M - 1 or W + M - 1 a power of two: the reference's np2 equals mp, its slice b[m:mp+1]
    keeps M - 1 rows and the product with h[m-1:mp] raises RuntimeError (Props/CZT_Prop.py:206,211;
    the reference run here on these four shapes raised RuntimeError every time, MKL's FFT error for
    M = 1).  The build raises RuntimeError (ThzError) before anything is launched, in fp32 and fp64,
    where it used to leave the last output row unset (found by the randomized property sweep)."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    dev = torch.device("cuda:0")
    for dt, wl in ((torch.complex64, 1e-3), (torch.complex128, torch.tensor([1e-3], dtype=torch.float64))):
        f = ElectricField(torch.ones(1, 1, H, W, dtype=dt, device=dev), wavelengths=wl, spacing=[0.5e-3, 0.6e-3],
                          device=dev)
        with pytest.raises(RuntimeError, match="power of two"):
            CZT_prop(z_distance=0.5, device=dev)(f, M, M, 0.4e-3, 0.4e-3)
    # M = 1 with only the second pass's m = W a power of two: the reference returns a [B, C, 1, 0]
    # field (run here: H, W = 5, 2 and 5, 1), so does the build
    for w in (2, 1):
        f = ElectricField(torch.ones(1, 1, 5, w, dtype=torch.complex64, device=dev), wavelengths=1e-3,
                          spacing=[0.5e-3, 0.6e-3], device=dev)
        assert tuple(CZT_prop(z_distance=0.5, device=dev)(f, 1, 1, 0.4e-3, 0.4e-3).data.shape) == (1, 1, 1, 0)
    # one below: a valid length (12 + 20 - 1 = 31) runs and is finite
    f = ElectricField(torch.ones(1, 1, 12, 12, dtype=torch.complex64, device=dev), wavelengths=1e-3,
                      spacing=[0.5e-3, 0.6e-3], device=dev)
    out = CZT_prop(z_distance=0.5, device=dev)(f, 20, 20, 0.4e-3, 0.4e-3).data
    assert out.shape == (1, 1, 20, 20) and bool(torch.isfinite(out).all())


@pytest.mark.parametrize("H,W,out,C", [(48, 64, 24, 2), (64, 64, 16, 1), (40, 36, 40, 1)])
def test_czt_backward_vs_oracle_autograd(H, W, out, C):
    """CZT_prop backward (adjoint Bluestein kernels) vs autograd through the fp64 oracle."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    rng = np.random.default_rng(H + W + out)
    x = (rng.standard_normal((1, C, H, W)) + 1j * rng.standard_normal((1, C, H, W))).astype(np.complex64)
    freqs = [280 + 30 * c for c in range(C)]
    wl = [C0 / (f * 1e9) for f in freqs]
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(x).to(dev).requires_grad_(True)
    field = ElectricField(xd, wavelengths=wl if C > 1 else wl[0], spacing=[0.5e-3, 0.6e-3], device=dev)
    o = CZT_prop(z_distance=0.2, device=dev)(field, out, out, 0.35e-3, 0.35e-3).data
    g = (rng.standard_normal(o.shape) + 1j * rng.standard_normal(o.shape)).astype(np.complex64)
    gx, = torch.autograd.grad(o, xd, grad_outputs=torch.from_numpy(g).to(dev))
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        xo = torch.from_numpy(x).to(torch.complex128).requires_grad_(True)
        sp = torch.tensor([0.5e-3, 0.6e-3], dtype=torch.float32).double()
        ro = orc.czt_forward(xo, wavelengths(freqs, True), sp, 0.2, out, out,
                             float(torch.tensor(0.35e-3, dtype=torch.float32)),
                             float(torch.tensor(0.35e-3, dtype=torch.float32)))
        ro_g, = torch.autograd.grad(ro, xo, grad_outputs=torch.from_numpy(g).to(torch.complex128))
    finally:
        torch.set_default_dtype(old)
    assert gx.shape == xd.shape
    assert rel_l2(gx.cpu().numpy(), ro_g.numpy()) <= 1e-3, rel_l2(gx.cpu().numpy(), ro_g.numpy())


@pytest.mark.parametrize("H,W,out,C", [(2048, 2048, 512, 2), (1800, 2048, 400, 1), (1300, 1100, 256, 3),
                                         (1301, 1100, 256, 1), (1302, 1024, 200, 2)])
def test_czt_overlap_add_vs_oracle(H, W, out, C):
    """cfg3-sized CZT, forward and backward vs the fp64 oracle, rel-L2 <= 1e-3.  The forward passes
    run the overlap-add Bluestein kernels (czt_rows_blk / czt_cols_blk: 512-input blocks, 1024-point
    wave transforms): 4 full blocks per line (2048 -> 512, the cfg3 geometry), a partial last block
    (m = 1800) and 3 blocks with M < 512 over 3 wavelengths; odd H (no mirrored row pairs: each
    wave evaluates its own RS factors) and an odd number of row pairs (the last workgroup's second
    pair idle); the backward runs the np2 adjoint kernels on the same tables."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    rng = np.random.default_rng(H + out)
    x = (rng.standard_normal((1, C, H, W)) + 1j * rng.standard_normal((1, C, H, W))).astype(np.complex64)
    freqs = [240 + 60 * c for c in range(C)]
    wl = [C0 / (f * 1e9) for f in freqs]
    dev = torch.device("cuda:0")
    xd = torch.from_numpy(x).to(dev).requires_grad_(True)
    field = ElectricField(xd, wavelengths=wl if C > 1 else wl[0], spacing=[0.5e-3, 0.5e-3], device=dev)
    o = CZT_prop(z_distance=0.2, device=dev)(field, out, out, 0.35e-3, 0.35e-3).data
    g = (rng.standard_normal(o.shape) + 1j * rng.standard_normal(o.shape)).astype(np.complex64)
    gx, = torch.autograd.grad(o, xd, grad_outputs=torch.from_numpy(g).to(dev))
    old = torch.get_default_dtype()
    torch.set_default_dtype(torch.float64)
    try:
        xo = torch.from_numpy(x).to(torch.complex128).requires_grad_(True)
        sp = torch.tensor([0.5e-3, 0.5e-3], dtype=torch.float32).double()
        ro = orc.czt_forward(xo, wavelengths(freqs, True), sp, 0.2, out, out,
                             float(torch.tensor(0.35e-3, dtype=torch.float32)),
                             float(torch.tensor(0.35e-3, dtype=torch.float32)))
        ro_g, = torch.autograd.grad(ro, xo, grad_outputs=torch.from_numpy(g).to(torch.complex128))
    finally:
        torch.set_default_dtype(old)
    ef = rel_l2(o.detach().cpu().numpy(), ro.detach().numpy())
    eb = rel_l2(gx.cpu().numpy(), ro_g.numpy())
    assert ef <= 1e-3 and eb <= 1e-3, (ef, eb)


@pytest.mark.parametrize("case", M["czt"][:2], ids=[c["name"] for c in M["czt"][:2]])
def test_vczt_alias_propagates_each_component(case):
    """VCZT_prop (Props/CZT_Prop.py:317-348) is CZT_prop on a vectorial (B = 3) field: each component
    plane propagates independently, so (x, 2x, -i x) gives (y, 2y, -i y) with y the reference's
    golden output for x; its z property mirrors CZT_prop's."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import VCZT_prop
    A = arrays("czt")
    k = case["name"]
    dev = torch.device("cuda:0")
    x = torch.from_numpy(A[f"{k}__in"])
    vec = torch.cat([x, 2 * x, -1j * x], 0).to(torch.complex64)
    wl = [C0 / (f * 1e9) for f in case["f"]]
    field = ElectricField(vec.to(dev), wavelengths=wl if len(wl) > 1 else wl[0],
                          spacing=[case["dx"] * 1e-3, case["dy"] * 1e-3], device=dev)
    prop = VCZT_prop(z_distance=case["z"], device=dev)
    assert abs(float(prop.z) - case["z"]) <= 1e-7 * case["z"]  # stored as a float32 tensor, as the reference does
    out = prop(field, outputHeight=case["oH"], outputWidth=case["oW"], outputPixel_dx=case["odx"] * 1e-3,
               outputPixel_dy=case["ody"] * 1e-3).data.cpu().numpy()
    y = A[f"{k}__out64"]
    ref = np.concatenate([y, 2 * y, -1j * y], 0)
    assert out.shape == ref.shape
    assert rel_l2(out, ref) <= 1e-3


def test_czt_cfg3_geometry_vs_reference_signature():
    """cfg3 at its own geometry (2048^2 -> 512^2, dx 0.5 -> 0.25 mm, z = 0.5 m, 32 wavelengths over
    220-330 GHz, all in one call as bench.py times it) vs the REFERENCE's own fp64 output signature
    on the same seeded white inputs (tests/golden/cfg3_check.npz, tests/golden/gen_cfg3_check.py):
    every plane's sub-grid, row 256 and energy within bench.CZT_CHECK_TOL (the reference's own fp32
    output is up to 1.8e-2 off its fp64 here; this build's chirps are double precision)."""
    import bench
    from quantizationawarethzdoe_amd.propagation import czt_apply
    freqs = torch.linspace(220e9, 330e9, 32, dtype=torch.float64)
    lam = [float(torch.tensor(C0 / float(f), dtype=torch.float32)) for f in freqs]
    idx = list(range(32))
    x = torch.stack([bench.cfg3_input(i) for i in idx])[None].to("cuda:0")
    sp = [float(torch.tensor(0.5e-3, dtype=torch.float32))] * 2
    out = czt_apply(x, lam, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
    assert out.shape == (1, 32, 512, 512)
    chk = bench.check_czt(out, idx)
    assert chk["ok"], chk


def test_czt_table_cache_hits_and_graph_capture_match_fresh_tables():
    """The per-device table cache (csrc/thz_czt.hip czt_tables_for): a first call builds a key's
    tables into a cache buffer, later calls with the same key reuse them, a different z or
    wavelength set is its own key, and a call captured into a HIP graph builds its tables in its
    own workspace.  Every route gives bit-identical planes (the same table kernels either way),
    forward and adjoint, on the overlap-add geometry and a np2 one."""
    from quantizationawarethzdoe_amd import propagation as P
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(77)
    for H, M in ((1100, 256), (96, 40)):
        x = torch.randn(1, 2, H, H, dtype=torch.complex64, generator=g).to(dev)
        z1, z2 = 0.2 + 1e-4 * H, 0.31 + 1e-4 * H  # keys no other test uses
        wl = [1.01e-3, 1.2e-3]
        args = ([0.5e-3, 0.5e-3], M, M, 0.35e-3, 0.35e-3)
        a1 = P.czt_apply(x, wl, args[0], z1, *args[1:])          # builds z1's entry
        b1 = P.czt_apply(x, wl, args[0], z2, *args[1:])          # z2's entry
        a2 = P.czt_apply(x, wl, args[0], z1, *args[1:])          # hit
        c1 = P.czt_apply(x, wl[::-1], args[0], z1, *args[1:])    # wavelengths swapped: own key
        assert torch.equal(a1, a2) and not torch.equal(a1, b1)
        assert torch.equal(c1[:, 0], P.czt_apply(x[:, :1].contiguous(), wl[1:], args[0], z1, *args[1:])[:, 0])
        gy = torch.randn(a1.shape, dtype=torch.complex64, generator=g).to(dev)
        adj1 = P.czt_apply(gy, wl, args[0], z1, *args[1:], adjoint=True, field_hw=(H, H))
        adj2 = P.czt_apply(gy, wl, args[0], z1, *args[1:], adjoint=True, field_hw=(H, H))
        assert torch.equal(adj1, adj2)
        # captured: tables built inside the graph, in the call's workspace
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            P.czt_apply(x, wl, args[0], z1, *args[1:])
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = P.czt_apply(x, wl, args[0], z1, *args[1:])
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, a1)
