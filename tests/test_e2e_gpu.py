"""Deterministic end-to-end golden: designed 4-level height maps through the
whole four-focal-spots system -- Guassian_beam -> ASM 127 mm -> thin lens -> 80 mm aperture ->
FixDOEElement(tolerance = 0) -> ASM 200 mm -> MSE(normalize(|E|^2), nine-PSF target) -- written
with the notebook's own import lines (experiment_four_focal_spots.ipynb:198-260), vs the
REFERENCE's own run of the same system (tests/golden/e2e_golden.npz, gen_e2e_golden.py, fp64 by
the SURVEY §8(c) procedure).

Cases (tests/golden/e2e_manifest.json): the REFERENCE's own trained maps -- edoe_4levels.npy and
plot_data/example_1/splitter_{ours, STE, PSQ, GS, full_precision}.npy, the 80 x 80 crops its
notebook saved, read by a token parser that executes nothing from the file
(tests/golden/refdoe_parse.py) -- zero-padded back to the 100 x 100 DOE (the 80 mm aperture
zeroes the field outside the crop, so this is the trained DOE's detector field) and, for
splitter_ours, upsampled from 80 x 80 as the FixDOE does; plus two splitters designed by the
generator (an 80 x 80 map upsampled to the 100 x 100 field, and a 100 x 100 one).

Tolerances: the field before the DOE and the detector field rel-L2 <= 1e-4 (SURVEY §8(c) ASM
bound; the reference's own fp32 error here is 5e-5), the loss within 1e-4 relative, the height-map
gradient (d loss / d h through the modulation and the ASM adjoint) within 1e-3 rel-L2 of the
reference's fp64 gradient -- for the trained maps, whose symmetric outputs tie the normalize()
maximum, the gradient for the tied pixel this run's maximum picked (see the test).
"""
import json
import os

import numpy as np
import pytest
import torch

from tests.golden_io import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN, "e2e_manifest.json")) as _fh:
    E2E = json.load(_fh)


def _arrays():
    with np.load(os.path.join(GOLDEN, "e2e_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("case", E2E["cases"], ids=[c["name"] for c in E2E["cases"]])
def test_designed_doe_through_four_focal_spots_system(case):
    import quantizationawarethzdoe_amd as pkg
    pkg.install_reference_aliases()
    import torch.nn as nn
    from Components.Aperture import ApertureElement
    from Components.QuantizedDOE import FixDOEElement
    from Components.Thin_Lens import Thin_LensElement
    from LightSource.Gaussian_beam import Guassian_beam
    from Props.ASM_Prop import ASM_prop
    from utils.Helper_Functions import normalize
    from utils.units import m, mm

    A = _arrays()
    k = case["name"]
    eps, tand = E2E["material"]
    wavelengths = 2.998e8 / (E2E["f_ghz"] * 1e9)
    source = Guassian_beam(height=100, width=100, beam_waist_x=None, beam_waist_y=None, wavelengths=wavelengths,
                           spacing=1 * mm)
    asm_prop1 = ASM_prop(z_distance=0.127 * m, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True)
    lens = Thin_LensElement(focal_length=0.127 * m)
    aperture = ApertureElement(aperture_type='rect', aperture_size=0.08)
    field_in = aperture(lens(asm_prop1(source())))
    assert rel_l2(field_in.data.detach().cpu().numpy(), A["field_in64"]) <= 1e-4

    doe = FixDOEElement(height_map=torch.from_numpy(A[f"{k}__h"]), tolerance=0.0, material=[eps, tand])
    asm_prop3 = ASM_prop(z_distance=200 * mm, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True)
    out = asm_prop3(doe(field_in))
    target = torch.from_numpy(A["target32"]).to(out.data.device)
    loss = nn.MSELoss()(normalize(torch.abs(out.data) ** 2), target)
    loss.backward()

    e_out = rel_l2(out.data.detach().cpu().numpy(), A[f"{k}__out64"])
    assert e_out <= 1e-4, e_out
    ref_loss = float(A[f"{k}__loss64"])
    assert abs(float(loss.detach()) - ref_loss) <= 1e-4 * ref_loss, (float(loss.detach()), ref_loss)
    g = doe.height_map.grad.detach().cpu().numpy()
    ref_g = A[f"{k}__grad64"]
    if case.get("tied_max"):
        # The reference's trained maps are mirror-symmetric (num_unit = 2): |E|^2 has four maxima
        # equal to 1e-15, so normalize()'s max -- and the gradient term it routes to that pixel --
        # is a tie-break of rounding (the reference's own fp32 and fp64 runs may differ by 100 %).
        # The fixture holds the fp64 gradient for each tied pixel; grade the one this run's max
        # picked (torch.max: the first index of the maximum, as normalize() takes it).
        inten = (torch.abs(out.data.detach()) ** 2).reshape(-1)
        i, j = divmod(int(torch.argmax(inten)), inten.numel() // 100)
        assert [i, j] in case["tied_max"], (i, j, case["tied_max"])
        ref_g = A[f"{k}__gradtie_{i}_{j}"]
    e_g = rel_l2(g, ref_g)
    assert e_g <= 1e-3, e_g
