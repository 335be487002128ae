"""Drop-in checks on the GPU: the four-focal-spots QAT of experiment_four_focal_spots.ipynb written
as a user of the reference writes it -- the notebook's import lines (after
install_reference_aliases()), its system of source -> ASM -> lens -> aperture -> DOE -> ASM, its
loop of normalize(|E|^2) -> nn.MSELoss -> Adam(lr 0.02) -- reproducing the reference's own 20-step
trace (tests/golden/qat_golden.npz, recorded Gumbel / height-noise draws replayed); and the kept
helpers utils.Helper_Functions.ft2 / ift2 / normalize (:99-193) vs the oracle."""
import numpy as np
import pytest
import torch

from oracle import thz_oracle as orc
from tests.golden_io import arrays, manifest, rel_l2
from tests.test_optics_qat_gpu import replay_draws

pytestmark = pytest.mark.gpu
M = manifest()


def test_four_focal_spots_notebook_style_via_reference_imports():
    import quantizationawarethzdoe_amd as pkg
    pkg.install_reference_aliases()
    import torch.nn as nn
    from Components.Aperture import ApertureElement
    from Components.QuantizedDOE import SoftGumbelQuantizedDOELayerv3 as SoftGumbelQuantizedDOELayer
    from Components.Thin_Lens import Thin_LensElement
    from LightSource.Gaussian_beam import Guassian_beam
    from Props.ASM_Prop import ASM_prop
    from utils.Helper_Functions import normalize
    from utils.units import m, mm

    q = M["qat"]
    A = arrays("qat")

    class Setup(nn.Module):
        """The notebook's system (experiment_four_focal_spots.ipynb cell 6), default devices."""

        def __init__(self, input_dxy, input_field_shape, doe_params, optim_params, wavelengths):
            super().__init__()
            self.source = Guassian_beam(height=input_field_shape[0], width=input_field_shape[1], beam_waist_x=None,
                                        beam_waist_y=None, wavelengths=wavelengths, spacing=input_dxy)
            self.asm_prop1 = ASM_prop(z_distance=0.127 * m, bandlimit_type='exact', padding_scale=2,
                                      bandlimit_kernel=True)
            self.Colli_lens = Thin_LensElement(focal_length=0.127 * m)
            self.aperture = ApertureElement(aperture_type='rect', aperture_size=0.08)
            self.input_field = self.aperture(self.Colli_lens(self.asm_prop1(self.source())))
            self.doe = SoftGumbelQuantizedDOELayer(doe_params, optim_params)
            self.asm_prop3 = ASM_prop(z_distance=200 * mm, bandlimit_type='exact', padding_scale=2,
                                      bandlimit_kernel=True)

        def forward(self, iter_frac):
            return self.asm_prop3(self.doe(self.input_field, iter_frac))

    setup = Setup(1 * mm, [100, 100], q["doe_params"], q["optim_params"], 2.998e8 / (q["f"] * 1e9))
    with torch.no_grad():
        setup.doe.weight_init_phase.copy_(torch.from_numpy(A["w0"]))
    optimizer = torch.optim.Adam(setup.parameters(), lr=q["lr"])
    setup.cuda()
    target = torch.from_numpy(A["target"]).cuda()
    loss_fn = nn.MSELoss()
    losses = []
    with replay_draws(setup.doe, A, q["steps"], q["draws"]):
        for itr in range(q["steps"]):
            out_field = setup.forward(iter_frac=itr / q["steps"])
            out_amp = normalize(torch.abs(out_field.data) ** 2)
            loss = loss_fn(out_amp, target)
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            losses.append(loss.item())
    np.testing.assert_allclose(losses, np.array(q["losses"]), rtol=1e-3)
    assert rel_l2(setup.doe.weight_init_phase.detach().cpu().numpy(), A["w_final"]) <= 1e-3


@pytest.mark.parametrize("shape", [(1, 1, 64, 64), (2, 3, 100, 80), (1, 1, 301, 203), (1, 2, 1024, 1024)])
def test_helper_ft2_ift2_vs_oracle(shape):
    from quantizationawarethzdoe_amd.utils.Helper_Functions import ft2, ift2
    g = torch.Generator().manual_seed(sum(shape))
    x = torch.randn(shape, dtype=torch.complex64, generator=g)
    f = ft2(x.cuda()).cpu()
    b = ift2(x.cuda()).cpu()
    xd = x.to(torch.complex128)
    assert rel_l2(f.numpy(), orc.ft2(xd).numpy()) <= 2e-6 * np.log2(max(shape))
    assert rel_l2(b.numpy(), orc.ift2(xd).numpy()) <= 2e-6 * np.log2(max(shape))
    assert rel_l2(ift2(ft2(x.cuda())).cpu().numpy(), x.numpy()) <= 1e-5


@pytest.mark.parametrize("norm,delta,pad", [("backward", 0.5e-3, False), ("forward", 2.0, False), ("ortho", 1e-3, True)])
def test_helper_perform_ft_options(norm, delta, pad):
    """delta^2 shift(fft2(shift(x), norm)) and the pad -> transform -> adaptive-average-pool branch
    (utils/Helper_Functions.py:121-160), vs the same formula in fp64 torch on the host."""
    from quantizationawarethzdoe_amd.utils.Helper_Functions import ft2, ift2
    g = torch.Generator().manual_seed(3)
    x = torch.randn(1, 2, 48, 40, dtype=torch.complex64, generator=g)
    xd = x.to(torch.complex128)
    for fn, tf, sh in ((ft2, torch.fft.fft2, torch.fft.fftshift), (ift2, torch.fft.ifft2, torch.fft.ifftshift)):
        got = fn(x.cuda(), delta=delta, norm=norm, pad=pad).cpu()
        xi = torch.nn.functional.pad(xd, (20, 20, 24, 24)) if pad else xd
        ref = delta ** 2 * sh(tf(sh(xi, dim=(-2, -1)), dim=(-2, -1), norm=norm), dim=(-2, -1))
        if pad:
            pool = torch.nn.AdaptiveAvgPool2d([48, 40])
            ref = pool(ref.real) + 1j * pool(ref.imag)
        assert got.shape == ref.shape
        assert rel_l2(got.numpy(), ref.numpy()) <= 1e-5


def test_helper_normalize_in_place():
    """normalize divides each batch item by its max over (C, H, W) in place (:185-193)."""
    from quantizationawarethzdoe_amd.utils.Helper_Functions import normalize
    g = torch.Generator().manual_seed(4)
    x = torch.rand(3, 2, 50, 40, generator=g) * torch.tensor([1.0, 5.0, 0.1])[:, None, None, None]
    xc = x.cuda()
    out = normalize(xc)
    ref = orc.normalize(x)
    assert rel_l2(out.cpu().numpy(), ref.numpy()) <= 1e-7
    assert rel_l2(xc.cpu().numpy(), ref.numpy()) <= 1e-7  # the input itself was divided
