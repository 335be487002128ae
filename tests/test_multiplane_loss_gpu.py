"""The fused ASM -> loss pipeline over Z planes (thz_asm_forward_loss / thz_asm_adjoint_loss with
Z > 1): the multi-plane notebooks' loss, the sum over the planes of MSE(normalize(|E_z|^2),
target_z) (plot_data/example_2/experiment_dual_plane_hologram.ipynb cell 8,
plot_data/example_3/experiment_extend_depth_of_focus.ipynb cell 24), accumulated in the planes'
row-inverse pass and differentiated in the Z-summing adjoint's row pass.

Against the separate path (propagate_planes, then the loss kernel over the Z B planes as its
batch, times Z): the stored planes bit for bit (same K1 / K2 / K3), the loss within 1e-6 relative
(one-pass fp64 sums reduced in another order), field / weight gradients within 1e-5 rel-L2.
Geometries: P = 300 (the dual-plane system, compile-time plan), P = 500 (the extended-DOF system,
compile-time 5 4 5 5 plan, planes from device memory), a plain field with a per-item and a shared
target; and a hypothesis-drawn sweep over sizes (compile-time, power-of-two and runtime plans),
plane lists, batches and target broadcasts."""
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
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


@pytest.mark.parametrize("H,ps,Z,B,shared", [(100, 2, 2, 1, False), (100, 2, 3, 2, True), (100, 4, 5, 1, True),
                                             (64, 2, 3, 2, False)])
def test_plain_field_multiplane_loss_fused_equals_separate(H, ps, Z, B, shared):
    from quantizationawarethzdoe_amd import optics, propagation as P
    dev = _dev()
    g = torch.Generator().manual_seed(H + Z + B)
    x = torch.view_as_complex(torch.randn(B, 1, H, H, 2, generator=g)).to(dev)
    wl, sp = [C0 / 300e9], (1e-3, 1e-3)
    zs = [0.05 + 0.01 * k for k in range(Z)]
    ph, pw = P.asm_padding(H, H, (ps, ps))
    tgt = torch.rand(1 if shared else Z * B, 1, H, H, generator=g).to(dev)
    xf = x.clone().requires_grad_(True)
    out, loss = P.asm_propagate_loss(xf, tgt, wl, sp, zs, ph, pw)
    loss.backward()
    xs = x.clone().requires_grad_(True)
    ref = P.asm_propagate(xs, wl, sp, zs, ph, pw)
    lref = optics.intensity_mse(ref.reshape((Z * B, 1, H, H)), tgt) * float(Z)
    lref.backward()
    assert torch.equal(out.detach(), ref.detach())
    lv, rv = float(loss.detach()), float(lref.detach())
    assert abs(lv - rv) <= 1e-6 * abs(rv), (lv, rv)
    assert rel_l2(xf.grad.cpu().numpy(), xs.grad.cpu().numpy()) <= 1e-5


@settings(max_examples=int(os.environ.get("THZ_PROP_EXAMPLES", "40")), deadline=None, database=None,
          derandomize=os.environ.get("THZ_PROP_RANDOM", "0") != "1",
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])
@given(st.fixed_dictionaries({"geo": st.sampled_from([(100, 2), (100, 4), (64, 2), (512, 1), (90, 1), (37, 2)]),
                              "Z": st.integers(1, 6), "B": st.integers(1, 4), "shared": st.booleans(),
                              "uniform": st.booleans(), "seed": st.integers(0, 2 ** 31 - 1)}))
def test_multiplane_loss_fused_equals_separate_drawn(case):
    """The fused pipeline against the separate one over drawn geometries (P = 300 / 500 compile-time,
    P = 1024 power of two, runtime plans at P = 128 / 180 / 111), plane counts (Z = 1: the
    single-item loss finish), batches, shared or per-item targets and uniform (the plane recurrence
    at P = 1024) or scattered planes: planes bit-identical, loss 1e-6, gradient 1e-5."""
    from quantizationawarethzdoe_amd import optics, propagation as P
    dev = _dev()
    (H, ps), Z, B = case["geo"], case["Z"], case["B"]
    rng = np.random.default_rng(case["seed"])
    x = torch.from_numpy((rng.standard_normal((B, 1, H, H)) + 1j * rng.standard_normal((B, 1, H, H)))
                         .astype(np.complex64)).to(dev)
    wl, sp = [C0 / 300e9], (1e-3, 1e-3)
    if case["uniform"]:
        zs = [float(v) for v in torch.linspace(0.04, 0.04 + 0.005 * (Z - 1), Z, dtype=torch.float32)]
    else:
        zs = [float(np.float32(v)) for v in rng.uniform(0.02, 0.2, Z)]
    ph, pw = P.asm_padding(H, H, (ps, ps))
    tgt = torch.from_numpy(rng.random((1 if case["shared"] else Z * B, 1, H, H)).astype(np.float32)).to(dev)
    xf = x.clone().requires_grad_(True)
    out, loss = P.asm_propagate_loss(xf, tgt, wl, sp, zs, ph, pw)
    loss.backward()
    xs = x.clone().requires_grad_(True)
    ref = P.asm_propagate(xs, wl, sp, zs, ph, pw)
    lref = optics.intensity_mse(ref.reshape((Z * B, 1, H, H)), tgt) * float(Z)
    lref.backward()
    assert torch.equal(out.detach().reshape(ref.shape), ref.detach())
    lv, rv = float(loss.detach()), float(lref.detach())
    assert abs(lv - rv) <= 1e-6 * abs(rv), (lv, rv)
    assert rel_l2(xf.grad.cpu().numpy(), xs.grad.cpu().numpy()) <= 1e-5


def test_plain_field_multiplane_loss_with_out_cotangent():
    """out used elsewhere too: its cotangent joins the loss gradient in the adjoint's row pass."""
    from quantizationawarethzdoe_amd import optics, propagation as P
    dev = _dev()
    g = torch.Generator().manual_seed(3)
    x = torch.view_as_complex(torch.randn(1, 1, 100, 100, 2, generator=g)).to(dev)
    wl, sp, zs = [C0 / 300e9], (1e-3, 1e-3), [0.06, 0.09]
    ph, pw = P.asm_padding(100, 100, (2, 2))
    tgt = torch.rand(2, 1, 100, 100, generator=g).to(dev)
    xf = x.clone().requires_grad_(True)
    out, loss = P.asm_propagate_loss(xf, tgt, wl, sp, zs, ph, pw)
    (loss + 1e-3 * (out.abs() ** 2).sum()).backward()
    xs = x.clone().requires_grad_(True)
    ref = P.asm_propagate(xs, wl, sp, zs, ph, pw)
    (optics.intensity_mse(ref.reshape((2, 1, 100, 100)), tgt) * 2.0 + 1e-3 * (ref.abs() ** 2).sum()).backward()
    assert rel_l2(xf.grad.cpu().numpy(), xs.grad.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("which", ["dual", "edof"])
def test_multiplane_system_fused_loss_equals_separate(which):
    """The trainers' multi-plane step: forward_planes_loss (fused) == forward_planes + loss kernel
    (separate), same draws: loss and the DOE weight gradient; the extended-DOF planes read from
    device memory (z_dev), as the graph-replayed trainer does."""
    from quantizationawarethzdoe_amd import optics, qat
    dev = _dev()
    res = {}
    for fused in (True, False):
        torch.manual_seed(7)
        system = qat.DualPlaneSystem(device=dev) if which == "dual" else qat.ExtendedDOFSystem(seed=2, device=dev)
        target = qat.logo_targets(device=dev) if which == "dual" else qat.edof_target(device=dev)
        Z = len(system.planes)
        t = target.reshape((-1, 1) + tuple(target.shape[-2:]))
        g = torch.Generator().manual_seed(9)
        param = next(iter(system.doe.parameters()))
        with torch.no_grad():
            param.copy_(torch.randn(param.shape, generator=g))
        expo = {}

        def fixed_expo(shape, like, g=g):
            key = tuple(shape)
            if key not in expo:
                expo[key] = torch.empty(key).exponential_(generator=g).to(like.device)
            return expo[key].clone()
        system.doe._gumbel_noise = fixed_expo
        # (the height-noise draws come from torch's generator, seeded alike for both runs)
        zdev = torch.tensor(system.planes, dtype=torch.float32, device=dev) if which == "edof" else None
        if fused:
            out, loss = system.forward_planes_loss(0.6, t, z_dev=zdev)
        else:
            out = system.forward_planes(0.6, z_dev=zdev)
            loss = optics.intensity_mse(out.reshape((Z,) + tuple(out.shape[2:])), t) * float(Z)
        loss.backward()
        res[fused] = (out.detach().clone(), float(loss.detach()), param.grad.detach().clone())
    assert torch.equal(res[True][0], res[False][0])
    assert abs(res[True][1] - res[False][1]) <= 1e-6 * abs(res[False][1])
    assert rel_l2(res[True][2].cpu().numpy(), res[False][2].cpu().numpy()) <= 1e-5
    assert np.isfinite(res[True][1])
