"""complex128 propagation on the fp64 kernels (csrc/thz_f64.hip) vs the REFERENCE's own fp64 outputs.

The reference computes in the field's precision: a complex128 field or float64 wavelengths make
it compute in fp64 and return complex128 (DataType/ElectricField.py:85-90); its only script,
test_czt.py:12, runs RSC + CZT that way.  The golden ``__out64`` / ``__gin64`` arrays are the
reference run in fp64 (complex128 data, spacing and wavelengths = .double() of the
fp32-rounded values), so the same inputs go in here: complex128 data and float64 wavelength
tensors of the fp32-rounded wavelengths (the spacing is rounded to fp32 by ElectricField either
way).  Tolerances: rel-L2 <= 1e-10 for ASM and RSC (fp64 FFTs and transfer functions in the
reference's operation order; measured ~1e-14), <= 1e-8 for CZT (the reference's chirps are
complex pow W^(j^2/2) in fp64, this build's cis(theta j^2/2): the phases agree to ~1e-10
relative at these lengths).
"""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, example, given, settings
from hypothesis import strategies as st

from tests.golden_io import arrays, manifest, rel_l2

pytestmark = pytest.mark.gpu
M = manifest()
C0 = 2.998e8


def _dev():
    return torch.device("cuda:0")


def _wl64(freqs):
    """float64 tensor of the fp32-rounded wavelengths (the golden procedure)."""
    return torch.tensor([C0 / (f * 1e9) for f in freqs], dtype=torch.float32).double()


def _field(x, case, grad=False):
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    data = torch.from_numpy(np.asarray(x)).to(torch.complex128).to(_dev())
    if grad:
        data.requires_grad_(True)
    f = ElectricField(data, wavelengths=_wl64(case["f"]), spacing=[case["dx"] * 1e-3, case["dy"] * 1e-3],
                      device=_dev())
    return f, data


@pytest.mark.parametrize("case", M["asm"], ids=[c["name"] for c in M["asm"]])
def test_asm_f64_vs_reference_fp64(case):
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    A = arrays("asm")
    k = case["name"]
    field, data = _field(A[f"{k}__in"], case, grad=case["grad"])
    prop = ASM_prop(z_distance=case["z"], do_padding=case.get("do_padding", True),
                    do_unpad_after_pad=case.get("unpad", True), padding_scale=case["s"], bandlimit_kernel=case["bl"],
                    bandlimit_type=case["t"], device=_dev())
    out = prop(field).data
    assert out.dtype == torch.complex128
    e = rel_l2(out.detach().cpu().numpy(), A[f"{k}__out64"])
    assert e <= 1e-10, e
    if case["grad"]:
        out.backward(torch.from_numpy(A[f"{k}__gout"]).to(torch.complex128).to(_dev()))
        eg = rel_l2(data.grad.cpu().numpy(), A[f"{k}__gin64"])
        assert eg <= 1e-10, eg


def test_asm_f64_multi_plane_and_float64_wavelengths_promote():
    """complex64 data with a float64 wavelength tensor promotes to complex128 (torch's rule, as the
    reference's products promote), and propagate_planes in fp64 equals the per-plane forwards."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    A = arrays("asm")
    case = next(c for c in M["asm"] if c["name"] == "n100_s2_p300")
    x = torch.from_numpy(A["n100_s2_p300__in"]).to(_dev())
    field = ElectricField(x, wavelengths=_wl64(case["f"]), spacing=[1e-3, 1e-3], device=_dev())
    prop = ASM_prop(z_distance=case["z"], padding_scale=2, device=_dev())
    out = prop(field).data
    assert out.dtype == torch.complex128
    assert rel_l2(out.cpu().numpy(), A["n100_s2_p300__out64"]) <= 1e-6  # input rounded to complex64
    zs = [0.05, 0.2, 0.31]
    planes = prop.propagate_planes(field, zs)
    for i, z in enumerate(zs):
        prop.z = z
        assert torch.equal(planes[i], prop(field).data)


@pytest.mark.parametrize("case", M["czt"], ids=[c["name"] for c in M["czt"]])
def test_czt_f64_vs_reference_fp64(case):
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    A = arrays("czt")
    k = case["name"]
    field, _ = _field(A[f"{k}__in"], case)
    out = CZT_prop(z_distance=case["z"], device=_dev())(field, outputHeight=case["oH"], outputWidth=case["oW"],
                                                      outputPixel_dx=case["odx"] * 1e-3,
                                                      outputPixel_dy=case["ody"] * 1e-3).data
    assert out.dtype == torch.complex128
    e = rel_l2(out.cpu().numpy(), A[f"{k}__out64"])
    assert e <= 1e-8, e


def test_czt_f64_backward_is_the_adjoint():
    """<CZT x, y> = <x, CZT^H y> in fp64 through autograd (the fp64 adjoint kernels)."""
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.standard_normal((1, 2, 48, 40)) + 1j * rng.standard_normal((1, 2, 48, 40))).to(_dev())
    x.requires_grad_(True)
    field = ElectricField(x, wavelengths=_wl64([280, 320]), spacing=[0.5e-3, 0.6e-3], device=_dev())
    out = CZT_prop(z_distance=0.2, device=_dev())(field, 24, 24, 0.35e-3, 0.35e-3).data
    y = torch.from_numpy(rng.standard_normal(out.shape) + 1j * rng.standard_normal(out.shape)).to(_dev())
    gx, = torch.autograd.grad(out, x, grad_outputs=y)
    lhs = torch.vdot(out.detach().reshape(-1), y.reshape(-1))
    rhs = torch.vdot(x.detach().reshape(-1), gx.reshape(-1))
    assert abs(complex(lhs - rhs)) <= 1e-12 * abs(complex(lhs))


@pytest.mark.parametrize("case", M["rsc"], ids=[c["name"] for c in M["rsc"]])
def test_rsc_f64_vs_reference_fp64(case, capsys):
    from quantizationawarethzdoe_amd.Props.RSC_Prop import RSC_prop
    A = arrays("rsc")
    k = case["name"]
    field, _ = _field(A[f"{k}__in"], case)
    out = RSC_prop(z_distance=case["z"], device=_dev())(field).data
    assert out.dtype == torch.complex128
    e = rel_l2(out.cpu().numpy(), A[f"{k}__out64"])
    assert e <= 1e-10, e
    assert capsys.readouterr().out.strip() == case["stdout"]


@pytest.mark.parametrize("case", M["vrs"], ids=[c["name"] for c in M["vrs"]])
def test_vrs_f64_forward_backward_vs_reference_fp64(case):
    from quantizationawarethzdoe_amd.Props.RSC_Prop import VRS_prop
    A = arrays("vrs")
    k = case["name"]
    field, data = _field(A[f"{k}__in"], case, grad=True)
    out = VRS_prop(z_distance=case["z"], device=_dev())(field).data
    assert out.dtype == torch.complex128
    assert rel_l2(out.detach().cpu().numpy(), A[f"{k}__out64"]) <= 1e-10
    out.backward(torch.from_numpy(A[f"{k}__gout"]).to(torch.complex128).to(_dev()))
    assert rel_l2(data.grad.cpu().numpy(), A[f"{k}__gin64"]) <= 1e-10


def test_reference_smoke_script_in_fp64():
    """test_czt.py (the reference's only script, :12-38): a 200^2 fp64 Gaussian through RSC_prop and
    CZT_prop at 300 GHz-ish (lambda = 1 mm), dx = 1 mm, z = 0.5 m -- complex128 in, complex128 out,
    CZT vs the reference's fp64 output of that case (czt_test_czt_200)."""
    from quantizationawarethzdoe_amd.Props.CZT_Prop import CZT_prop
    from quantizationawarethzdoe_amd.Props.RSC_Prop import RSC_prop
    A = arrays("czt")
    case = next(c for c in M["czt"] if c["name"] == "czt_test_czt_200")
    field, _ = _field(A["czt_test_czt_200__in"], case)
    rsc = RSC_prop(z_distance=0.5, device=_dev())(field)
    assert rsc.data.dtype == torch.complex128 and torch.isfinite(rsc.data.abs()).all()
    out = CZT_prop(z_distance=case["z"], device=_dev())(field, case["oH"], case["oW"], case["odx"] * 1e-3,
                                                      case["ody"] * 1e-3).data
    assert rel_l2(out.cpu().numpy(), A["czt_test_czt_200__out64"]) <= 1e-8


@pytest.mark.parametrize("n", [64, 100, 128, 200, 243, 300, 343, 512, 1000, 1024, 2048, 4096, 6144, 8192, 121, 169])
def test_fft64_rows_vs_numpy(n):
    from quantizationawarethzdoe_amd.propagation import fft_rows
    rng = np.random.default_rng(n)
    x = rng.standard_normal((3, n)) + 1j * rng.standard_normal((3, n))
    xt = torch.from_numpy(x).to(_dev())
    assert rel_l2(fft_rows(xt).cpu().numpy(), np.fft.fft(x, axis=-1)) <= 1e-13
    assert rel_l2(fft_rows(xt, inverse=True).cpu().numpy(), np.fft.ifft(x, axis=-1) * n) <= 1e-13


@settings(max_examples=int(os.environ.get("THZ_PROP_EXAMPLES", "15")), deadline=None, database=None,
          derandomize=os.environ.get("THZ_PROP_RANDOM", "0") != "1",
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(st.fixed_dictionaries({"H": st.integers(1, 900), "W": st.integers(1, 900), "C": st.integers(1, 2),
                              "s": st.sampled_from([1, 1.5, 2]), "z": st.floats(0.01, 0.5),
                              "bl": st.sampled_from(["exact", "approx", "none"]), "f": st.floats(220.0, 380.0),
                              "dx": st.sampled_from([0.5, 1.0]), "seed": st.integers(0, 2 ** 31 - 1)}))
# large prime factors in the padded lengths (2 x 853, 3 x 641): the table-DFT stage
@example({"H": 899, "W": 853, "C": 1, "s": 1, "z": 0.1, "bl": "exact", "f": 300.0, "dx": 0.5, "seed": 1})
@example({"H": 700, "W": 641, "C": 2, "s": 2, "z": 0.3, "bl": "approx", "f": 250.0, "dx": 1.0, "seed": 2})
def test_asm_f64_drawn_sizes_vs_oracle(case):
    """The fp64 ASM at drawn sizes up to P = 2700 (runtime mixed-radix plans: radix 4, 2, 3, 5, 7 in
    registers, any other prime factor by a table DFT) against the fp64 oracle, rel-L2 <= 1e-10, and
    its backward the adjoint to 1e-12."""
    from oracle import thz_oracle as orc
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    rng = np.random.default_rng(case["seed"])
    H, W, C = case["H"], case["W"], case["C"]
    lam = _wl64([case["f"] + 37 * c for c in range(C)])
    x = torch.from_numpy(rng.standard_normal((1, C, H, W)) + 1j * rng.standard_normal((1, C, H, W))).to(_dev())
    prop = ASM_prop(z_distance=case["z"], padding_scale=case["s"], bandlimit_kernel=case["bl"] != "none",
                    bandlimit_type="exact" if case["bl"] == "none" else case["bl"], device=_dev())
    xg = x.clone().requires_grad_(True)
    out = prop(ElectricField(xg, wavelengths=lam, spacing=case["dx"] * 1e-3, device=_dev())).data
    assert out.dtype == torch.complex128
    sp = torch.tensor([case["dx"] * 1e-3] * 2, dtype=torch.float32).double()
    kw = dict(bandlimit=case["bl"] != "none", bandlimit_type="exact" if case["bl"] == "none" else case["bl"])
    ref = orc.asm_forward(x.cpu(), lam, sp, case["z"], case["s"], **kw)
    e = float((out.detach().cpu() - ref).norm() / ref.norm())
    assert e <= 1e-10, e
    g = torch.from_numpy(rng.standard_normal(tuple(out.shape)) + 1j * rng.standard_normal(tuple(out.shape))).to(_dev())
    gx, = torch.autograd.grad(out, xg, grad_outputs=g)
    lhs = torch.vdot(out.detach().reshape(-1), g.reshape(-1))
    rhs = torch.vdot(x.reshape(-1), gx.reshape(-1))
    assert abs(complex(lhs - rhs)) <= 1e-12 * float(out.detach().norm()) * float(g.norm())
