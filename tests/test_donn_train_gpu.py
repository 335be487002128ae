"""cfg5 DONN data-parallel training step on the GPU.

The reference notebook's training cells are empty (experiment_DONN_3_layers.ipynb, sections
3-5), so the step's loss (MSE(normalize(|E|^2), per-sample detector target), the reference QAT
loss) and the detector layout are this framework's; the forward pieces are pinned by the DONN
golden fixture (test_optics_qat_gpu.py) and the loss kernel by the QAT fixtures.  Here the
whole step is checked against the same composition of oracle pieces on the host:
loss within 1e-4 relative, weight gradients within 1e-3 rel-L2 (four fp32 ASM propagations and
their adjoints on each side, reductions in a different order).
"""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tests.golden_io import rel_l2

pytestmark = pytest.mark.gpu
C0 = 2.998e8


def _dev():
    return torch.device("cuda:0")


def _oracle_loss(ws, u, target, noises, chained):
    """The DONN step's loss from oracle pieces (FullPrecision layers, height noise injected)."""
    from oracle import thz_oracle as orc
    lam = torch.tensor([C0 / 300e9], dtype=torch.float32)
    sp = torch.tensor([1e-3, 1e-3], dtype=torch.float32)
    d = torch.tensor(1e-3, dtype=torch.float32)
    mask = orc.aperture_mask(100, 100, d, d, "rect", 0.08)[None, None]
    inputs = orc.asm_forward(u.to(torch.complex64), lam, sp, 0.05, padding_scale=2) * mask
    mat = torch.tensor([2.66, 0.003])
    field = inputs
    out = None
    for i in range(3):
        h = orc.fp_height(ws[i], torch.tensor(1e-3), 8.0).reshape(100, 100)
        f = orc.doe_modulate(field if chained else inputs, h, lam, mat[0], mat[1], tolerance=30e-6,
                             noise_u01=noises[i])
        if i < 2:
            field = orc.asm_forward(f, lam, sp, 0.02, padding_scale=2) * mask
        else:
            out = orc.asm_forward(f, lam, sp, 0.05, padding_scale=2)
    return orc.intensity_mse(out, target)


@pytest.mark.parametrize("B", [4, 32, 256], ids=["b4", "b32_cfg5_rank", "b256_cfg5_global"])
@pytest.mark.parametrize("chained", [True, False], ids=["chained", "notebook"])
def test_donn_step_loss_and_grads_vs_oracle(chained, B):
    """B = 32 is cfg5's per-rank batch at 8 GPUs and B = 256 its global batch (the bench's N = 1
    step): both run the modulate backward with 16 batch lanes and its fixed-order LDS reduction
    (csrc/thz_doe.hip), B = 4 runs 4."""
    from quantizationawarethzdoe_amd import donn
    g = torch.Generator().manual_seed(5 + B)
    u = torch.rand(B, 1, 100, 100, generator=g)
    labels = torch.tensor([3, 0, 7, 9]) if B == 4 else torch.randint(0, 10, (B,), generator=g)
    noises = [torch.rand(100, 100, generator=g) for _ in range(3)]
    torch.manual_seed(2)
    model = donn.DONN(device=_dev())
    ws = [next(iter(d.parameters())).detach().cpu().clone() for d in model.does]
    targets = donn.detector_targets(device=_dev())
    tr = donn.DONNTrainer(model, targets, chained=chained)
    it = iter(noises)  # the layers draw rand_like in order 0, 1, 2 in both semantics
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **k: next(it).to(device=t.device, dtype=t.dtype)
    try:
        loss = tr._loss(u.to(_dev()), targets.index_select(0, labels.to(_dev())), None)
        loss.backward()
    finally:
        torch.rand_like = orig
    wo = [w.clone().requires_grad_(True) for w in ws]
    lo = _oracle_loss(wo, u, targets.cpu().index_select(0, labels), noises, chained)
    lo.backward()
    assert abs(float(loss.detach()) - float(lo.detach())) <= 1e-4 * float(lo.detach())
    for i, d in enumerate(model.does):
        gp = next(iter(d.parameters())).grad
        if not chained and i < 2:
            assert gp is None or float(gp.abs().max()) == 0.0  # the notebook discards these branches
            continue
        assert rel_l2(gp.cpu().numpy(), wo[i].grad.numpy()) <= 1e-3


@settings(max_examples=int(os.environ.get("THZ_PROP_EXAMPLES", "12")), deadline=None, database=None,
          derandomize=os.environ.get("THZ_PROP_RANDOM", "0") != "1",
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(st.fixed_dictionaries({"B": st.integers(1, 48), "chained": st.booleans(), "seed": st.integers(0, 2 ** 31 - 1)}))
def test_donn_step_drawn_batches_vs_oracle(case):
    """test_donn_step_loss_and_grads_vs_oracle over drawn batch sizes -- odd ones and ones that do
    not fill the modulate backward's 16 batch lanes -- in both semantics."""
    from quantizationawarethzdoe_amd import donn
    B, chained = case["B"], case["chained"]
    g = torch.Generator().manual_seed(case["seed"])
    u = torch.rand(B, 1, 100, 100, generator=g)
    labels = torch.randint(0, 10, (B,), generator=g)
    noises = [torch.rand(100, 100, generator=g) for _ in range(3)]
    torch.manual_seed(case["seed"] % 1000)
    model = donn.DONN(device=_dev())
    ws = [next(iter(d.parameters())).detach().cpu().clone() for d in model.does]
    targets = donn.detector_targets(device=_dev())
    tr = donn.DONNTrainer(model, targets, chained=chained)
    it = iter(noises)
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **k: next(it).to(device=t.device, dtype=t.dtype)
    try:
        loss = tr._loss(u.to(_dev()), targets.index_select(0, labels.to(_dev())), None)
        loss.backward()
    finally:
        torch.rand_like = orig
    wo = [w.clone().requires_grad_(True) for w in ws]
    lo = _oracle_loss(wo, u, targets.cpu().index_select(0, labels), noises, chained)
    lo.backward()
    assert abs(float(loss.detach()) - float(lo.detach())) <= 1e-4 * float(lo.detach())
    for i, d in enumerate(model.does):
        gp = next(iter(d.parameters())).grad
        if not chained and i < 2:
            assert gp is None or float(gp.abs().max()) == 0.0
            continue
        assert rel_l2(gp.cpu().numpy(), wo[i].grad.numpy()) <= 1e-3


def test_donn_trainer_graph_matches_eager_with_fixed_noise():
    from quantizationawarethzdoe_amd import donn
    g = torch.Generator().manual_seed(11)
    u = torch.rand(8, 1, 100, 100, generator=g)
    labels = torch.randint(0, 10, (8,), generator=g)
    unif = torch.rand(100, 100, generator=g).to(_dev())
    losses, weights = {}, {}
    for graph in (False, True):
        torch.manual_seed(3)
        model = donn.DONN(device=_dev())
        orig = torch.rand_like
        torch.rand_like = lambda t, *a, **k: unif.clone()
        try:
            tr = donn.DONNTrainer(model, donn.detector_targets(device=_dev()), graph=graph, device_rng=False)
            losses[graph] = [float(tr.step(u, labels).detach()) for _ in range(6)]
        finally:
            torch.rand_like = orig
        weights[graph] = torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy()
    np.testing.assert_allclose(losses[True], losses[False], rtol=1e-4)
    assert rel_l2(weights[True], weights[False]) <= 1e-4
    assert losses[False][-1] < losses[False][0]


@pytest.mark.parametrize("chained", [True, False], ids=["chained", "notebook"])
def test_donn_step_b256_vs_reference_step(chained):
    """The cfg5 bench step at its global batch (256) vs the REFERENCE's own fp64 step
    (tests/golden/cfg5_check.npz, tests/golden/gen_cfg5_check.py: the reference's ElectricField,
    ASM_prop, ApertureElement, FullPrecisionDOELayer and normalize, the same weights, batch and
    noise): loss within 1e-4 relative, weight gradients within 1e-3 rel-L2.  bench.py runs this
    check after timing each mode."""
    import bench
    chk = bench.check_donn(_dev(), chained)
    assert chk["ok"], chk


def test_aperture_folded_into_asm_matches_the_modules():
    """donn.propagate_through_aperture (the aperture as thz_asm_desc.window_mask: the 300-point row
    pass multiplies its stores by the mask, the backward's row pass its loads) == ApertureElement
    after ASM_prop, rect and circ, for a plain field and for a DOE layer's unevaluated modulation:
    the same values bit for bit (v or v * 0), forward and gradients, and the same .aperture
    attribute."""
    from quantizationawarethzdoe_amd import donn, propagation
    from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
    from quantizationawarethzdoe_amd.Components.Aperture import ApertureElement
    from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
    from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
    assert propagation.window_mask_fusable(100, 100, 100, 100, True)  # the fold is what runs
    dev = _dev()
    for kind, size in (("rect", 0.08), ("circ", 0.03)):
        for modulated in (False, True):
            g = torch.Generator(device=dev).manual_seed(4)
            x = torch.randn(3, 1, 100, 100, dtype=torch.complex64, device=dev, generator=g)
            cot = torch.randn(3, 1, 100, 100, dtype=torch.complex64, device=dev, generator=g)
            prop = ASM_prop(z_distance=0.02, padding_scale=2, bandlimit_type="exact", device=dev)
            res = []
            for fused in (True, False):
                torch.manual_seed(11)
                xi = x.clone().requires_grad_(True)
                f = ElectricField(data=xi, wavelengths=2.998e8 / 300e9, spacing=1e-3, device=dev)
                doe = None
                if modulated:
                    dp, _ = donn.default_params()
                    doe = Q.FullPrecisionDOELayer(dict(dp, tolerance=0.0), device=dev)
                    f = doe(f, 0.5)
                ap = ApertureElement(aperture_type=kind, aperture_size=size)
                out = donn.propagate_through_aperture(prop, ap, f) if fused else ap(prop(f))
                out.data.backward(cot)
                gw = next(iter(doe.parameters())).grad.clone() if doe is not None else None
                res.append((out.data.detach().clone(), xi.grad.clone(), gw, ap.aperture.clone()))
            (o1, g1, w1, m1), (o2, g2, w2, m2) = res
            assert torch.equal(o1, o2) and torch.equal(g1, g2) and torch.equal(m1, m2), (kind, modulated)
            if modulated:
                assert torch.equal(w1, w2), (kind, modulated)


def test_window_mask_refused_for_complex128_and_several_planes():
    """The folded aperture exists in the complex64 one-plane pipeline only: asm_apply refuses a mask
    with a complex128 field or more than one z-plane in the forward, instead of dropping
    it or failing in the backward."""
    from quantizationawarethzdoe_amd import _lib, propagation
    dev = _dev()
    m = _lib.ApertureDesc(1, 100, 100, _lib.APERTURE_RECT, 1e-3, 1e-3, 0.04, 0.04, 0.0)
    x = torch.randn(1, 1, 100, 100, dtype=torch.complex64, device=dev)
    lam = [2.998e8 / 300e9]
    with pytest.raises(TypeError):
        propagation.asm_apply(x.to(torch.complex128), lam, [1e-3, 1e-3], [0.02], 100, 100, True, 1, mask=m)
    with pytest.raises(ValueError):
        propagation.asm_apply(x, lam, [1e-3, 1e-3], [0.02, 0.03], 100, 100, True, 1, mask=m)
