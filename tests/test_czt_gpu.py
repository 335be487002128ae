"""CZT parity on the GPU vs the reference-generated golden fixtures (tests/golden/czt_golden.npz).

Tolerance: rel-L2 vs the fp64 golden <= max(3e-3, 1.25 x the reference's own fp32 error)
(CZT <= 3e-3; the reference's fp32 error is 6e-5 .. 4.1e-3 on these cases,
dominated by its fp32 complex pow chirps, which this build evaluates in double).
"""
import numpy as np
import pytest
import torch

from tests.golden_io import arrays, manifest, rel_l2

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
