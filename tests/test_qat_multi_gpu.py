"""The reference's two multi-plane QAT systems on the HIP path (qat.DualPlaneSystem,
qat.ExtendedDOFSystem) against 20-step traces of the REFERENCE itself
(tests/golden/gen_qat_multi.py: plot_data/example_2/experiment_dual_plane_hologram.ipynb cells 2-8
and plot_data/example_3/experiment_extend_depth_of_focus.ipynb cells 1-3, 22-24, every Gumbel /
height-noise draw and every re-drawn plane distance recorded), and the graph-replayed trainer
(planes read from the device step state, thz_asm_desc.z_dev) against the eager one.

The trainer propagates the DOE output to all planes in ONE pipeline (modulation fused into the
shared row pass, one column pass over the Z planes; in backward the Z-summing adjoint, one launch)
and evaluates the loss kernel over the Z planes as its batch (normalize per plane) x Z = the sum of
the per-plane MSEs the notebooks form.  The extended-DOF system runs P = 500, the runtime mixed-radix
plan."""
import contextlib
import json

import numpy as np
import pytest
import torch

from tests.golden_io import GOLDEN, rel_l2

pytestmark = pytest.mark.gpu


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _golden(name):
    with np.load(f"{GOLDEN}/qat_{name}_golden.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


with open(f"{GOLDEN}/qat_multi_manifest.json") as _fh:
    M = json.load(_fh)


@contextlib.contextmanager
def replay(layer, A, steps, kinds):
    """The recorded exponential_ / rand_like draws of each step, fed to the layer in order."""
    expo, unif = [], []
    for s in range(steps):
        for i, k in enumerate(kinds[s]):
            (expo if k == "expo" else unif).append(A[f"step{s}__draw{i}"])
    expo.reverse()
    unif.reverse()
    orig = torch.rand_like

    def fake_unif(t, *a, **kw):
        v = unif.pop()
        assert tuple(t.shape) == v.shape
        return torch.from_numpy(v).to(device=t.device, dtype=t.dtype)

    def fake_expo(shape, like):
        v = expo.pop()
        assert tuple(shape) == v.shape
        return torch.from_numpy(v).to(like.device)

    layer._gumbel_noise = fake_expo
    torch.rand_like = fake_unif
    try:
        yield
    finally:
        torch.rand_like = orig
    assert not expo and not unif, "not every recorded draw was consumed"


def _trace(system, target, A, q, planes=None):
    from quantizationawarethzdoe_amd import qat
    pname = q["param"]
    param = dict(system.doe.named_parameters())[pname]
    with torch.no_grad():
        param.copy_(torch.from_numpy(A["w0"]))
    if planes is not None:
        # the reference's re-drawn planes, in order (step k uses the draw made after step k - 1)
        it = iter(planes[1:])

        def next_planes():
            zs = next(it, None)
            if zs is not None:
                for p, z in zip(system.props, zs):
                    p.z = float(z)
        system.after_forward = next_planes
    trainer = qat.QATTrainer(system, target, lr=q["lr"], max_itrs=q["steps"], optimizer=q["optimizer"])
    losses = []
    with replay(system.doe, A, q["steps"], q["draws"]):
        for _ in range(q["steps"]):
            losses.append(float(trainer.step().detach()))
    return losses, param


def test_dual_plane_trace_vs_reference():
    """Dual-plane hologram, 20 steps of the reference's own trajectory (v3 layer, AdamW lr 0.01,
    planes 100 / 150 mm, P = 300): the targets equal the reference's decoded logos exactly, the input
    field within 1e-5, the first loss within 1e-5, every loss within 1e-3 relative and the final
    weight within 1e-3 rel-L2 (fp32 through 20 Adam steps, as the four-focal-spots trace)."""
    from quantizationawarethzdoe_amd import qat
    A, q = _golden("dual"), M["dual"]
    dev = _dev()
    system = qat.DualPlaneSystem(device=dev)
    assert rel_l2(system.input_field.data.cpu().numpy(), A["field_in"]) <= 1e-5
    target = qat.logo_targets(device=dev)
    np.testing.assert_array_equal(target[:, 0].cpu().numpy(), A["targets"])
    np.testing.assert_allclose(system.planes, [0.1, 0.15], rtol=1e-15)
    losses, param = _trace(system, target, A, q)
    ref = np.array(q["losses"])
    assert abs(losses[0] - ref[0]) <= 1e-5 * ref[0], (losses[0], ref[0])
    np.testing.assert_allclose(losses, ref, rtol=1e-3)
    assert rel_l2(param.detach().cpu().numpy(), A["w_final"]) <= 1e-3


def test_extended_dof_trace_vs_reference():
    """Extended depth of focus, 20 steps of the reference's own trajectory (rotationally symmetric
    v3 layer, AdamW lr 0.02, five planes re-drawn every iteration, P = 500): input field within 1e-5,
    the first loss within 1e-5, every loss within 1e-3 relative, final weight within 1e-3 rel-L2."""
    from quantizationawarethzdoe_amd import qat
    A, q = _golden("edof"), M["edof"]
    dev = _dev()
    system = qat.ExtendedDOFSystem(device=dev)
    assert rel_l2(system.input_field.data.cpu().numpy(), A["field_in"]) <= 1e-5
    target = qat.edof_target(device=dev)
    assert rel_l2(target[0, 0].cpu().numpy(), A["targets"][0]) <= 1e-6
    # the reference's initial planes are fp32 tensors (ASM_prop.__init__); the kernels take fp32 planes
    np.testing.assert_allclose(system.planes, A["zs"][0], rtol=1e-7)
    losses, param = _trace(system, target, A, q, planes=A["zs"])
    ref = np.array(q["losses"])
    assert abs(losses[0] - ref[0]) <= 1e-5 * ref[0], (losses[0], ref[0])
    np.testing.assert_allclose(losses, ref, rtol=1e-3)
    assert rel_l2(param.detach().cpu().numpy(), A["w_final"]) <= 1e-3


@pytest.mark.parametrize("which", ["dual", "edof"])
def test_multi_plane_graph_replay_matches_eager_with_fixed_noise(which):
    """The graph-replayed multi-plane step (one captured graph per schedule phase; the planes read
    from the device step state, so the extended-DOF planes move every replay) == the eager step, with
    the Gumbel / height noise fixed and the same seeded plane draws: 24 steps over the three v3
    phases."""
    from quantizationawarethzdoe_amd import qat
    dev = _dev()
    losses, weights, planes = {}, {}, {}
    for graph in (False, True):
        torch.manual_seed(3)
        system = qat.DualPlaneSystem(device=dev) if which == "dual" else qat.ExtendedDOFSystem(seed=5, device=dev)
        target = qat.logo_targets(device=dev) if which == "dual" else qat.edof_target(device=dev)
        g = torch.Generator().manual_seed(9)
        param = next(iter(system.doe.parameters()))
        with torch.no_grad():
            param.copy_(torch.randn(param.shape, generator=g))
        shapes = {}

        def fixed_expo(shape, like, g=g):
            key = tuple(shape)
            if key not in shapes:
                shapes[key] = torch.empty(key).exponential_(generator=g).to(like.device)
            return shapes[key].clone()
        system.doe._gumbel_noise = fixed_expo
        unif = torch.rand(100, 100, generator=g).to(dev)
        orig = torch.rand_like
        torch.rand_like = lambda t, *a, **k: unif.clone()
        try:
            tr = qat.QATTrainer(system, target, lr=0.01, max_itrs=24, graph=graph, device_rng=False,
                                optimizer="adamw")
            losses[graph] = [float(tr.step().detach()) for _ in range(24)]
        finally:
            torch.rand_like = orig
        weights[graph] = param.detach().cpu().numpy()
        planes[graph] = system.planes
    assert planes[True] == planes[False]
    np.testing.assert_allclose(losses[True], losses[False], rtol=1e-4)
    assert rel_l2(weights[True], weights[False]) <= 1e-4


def test_multi_plane_notebook_forward_equals_one_pipeline():
    """The notebook form of the system (forward: one ASM_prop per plane on the DOE output) and the
    trainer's one-pipeline form (forward_planes) give the same planes with the same draws, and the
    same weight gradient of the summed per-plane loss (dual-plane system, fixed noise)."""
    from quantizationawarethzdoe_amd import optics, qat
    dev = _dev()
    system = qat.DualPlaneSystem(device=dev)
    target = qat.logo_targets(device=dev)
    g = torch.Generator().manual_seed(4)
    expo = torch.empty(1, 4, 100, 100).exponential_(generator=g).to(dev)
    unif = torch.rand(100, 100, generator=g).to(dev)
    system.doe._gumbel_noise = lambda shape, like: expo.clone()
    param = next(iter(system.doe.parameters()))
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **k: unif.clone()
    try:
        outs = system(0.6)
        l1 = sum(optics.intensity_mse(o.data, t[None]) for o, t in zip(outs, target))
        l1.backward()
        g1 = param.grad.clone()
        param.grad = None
        planes = system.forward_planes(0.6)
        l2 = optics.intensity_mse(planes.reshape(2, 1, 100, 100), target) * 2.0
        l2.backward()
        g2 = param.grad.clone()
    finally:
        torch.rand_like = orig
    for k, o in enumerate(outs):
        assert rel_l2(planes[k].detach().cpu().numpy(), o.data.detach().cpu().numpy()) <= 1e-6
    assert abs(float(l1) - float(l2)) <= 1e-6 * float(l1)
    assert rel_l2(g2.cpu().numpy(), g1.cpu().numpy()) <= 1e-5
