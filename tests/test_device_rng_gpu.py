"""Device-drawn noise of the graph-replayed trainers (device_rng): the height noise U[0,1) and the
Gumbel Exp(1) draws are made inside the kernels from a counter-based generator (thz_dev.hpp
rng_*; state [seed, step] on the device), so a captured step holds no torch RNG kernels.

Checked here: the draws are uniform / deterministic per (seed, step) and differ across steps; the
fused DOE -> ASM row pass and the separate modulate kernel draw the same noise; forward and
backward agree with the explicit-noise path fed the same draw; the graph-replayed QAT step with
device noise is deterministic under a seed and trains.  (The reference's own RNG order is kept by
the eager path, which the parity tests use; device_rng only changes which generator a replayed
graph draws from -- same distributions, different samples.)"""
import numpy as np
import pytest
import torch

from tests.golden_io import rel_l2

pytestmark = pytest.mark.gpu
C0 = 2.998e8


def _dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    return torch.device("cuda:0")


def _draw_u(state, stream, hs, ws, dev):
    """The generator's U[0,1) of every height pixel: modulate with h = 0 and tolerance 1 gives
    hfull = (u - 0.5) * 2 exactly, so u = hfull / 2 + 0.5."""
    from quantizationawarethzdoe_amd import doe
    f = torch.ones((1, 1, hs, ws), dtype=torch.complex64, device=dev)
    _, hf = doe.modulate(f, torch.zeros((hs, ws), device=dev), [1e-3], 2.66, 0.03, tolerance=1.0,
                         rng=(state, stream))
    return hf / 2 + 0.5


def test_height_noise_draws():
    dev = _dev()
    state = torch.tensor([12345, 7], dtype=torch.int32, device=dev)
    u = _draw_u(state, 0, 200, 200, dev).cpu().numpy().ravel()
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.01 and abs(u.var() - 1 / 12) < 0.005
    assert np.array_equal(u, _draw_u(state, 0, 200, 200, dev).cpu().numpy().ravel())  # deterministic
    assert not np.allclose(u, _draw_u(state, 2, 200, 200, dev).cpu().numpy().ravel())  # another stream
    state[1] = 8
    assert not np.allclose(u, _draw_u(state, 0, 200, 200, dev).cpu().numpy().ravel())  # the next step


@pytest.mark.parametrize("dsize", [(100, 100), (50, 50)])
def test_device_noise_equals_explicit_noise_fused_and_separate(dsize):
    """Fused DOE -> ASM (K1 loader draws) and the separate modulate kernel (draws) agree with the
    explicit-noise path fed the generator's own draw: outputs and both gradients."""
    from quantizationawarethzdoe_amd import doe, propagation as P
    dev = _dev()
    hs, ws = dsize
    g = torch.Generator().manual_seed(4)
    x = torch.randn((2, 1, 100, 100), dtype=torch.complex64, generator=g).to(dev)
    h = (torch.rand((hs, ws), generator=g) * 1e-3).to(dev)
    gout = torch.randn((1, 2, 1, 100, 100), dtype=torch.complex64, generator=g).to(dev)
    state = torch.tensor([999, 3], dtype=torch.int32, device=dev)
    rng = (state, 4)
    u = _draw_u(state, 4, hs, ws, dev)
    wl, tol = [C0 / 300e9], 1e-5
    ph, pw = P.asm_padding(100, 100, (2, 2))
    res = []
    for mode in ("fused_rng", "separate_rng", "explicit"):
        xd = x.clone().requires_grad_(True)
        hd = h.clone().requires_grad_(True)
        if mode == "explicit":
            pend = doe.PendingModulation(xd, hd, wl, 2.66, 0.03, tolerance=tol, noise=u)
        else:
            pend = doe.PendingModulation(xd, hd, wl, 2.66, 0.03, tolerance=tol, rng=rng)
        if mode == "separate_rng":
            out = P.asm_propagate(pend.run(), wl, (1e-3, 1e-3), [0.2], ph, pw)
        else:
            out = P.asm_propagate_modulated(pend, wl, (1e-3, 1e-3), [0.2], ph, pw)
        out.backward(gout)
        res.append((out.detach().cpu(), pend.hfull.cpu(), xd.grad.cpu(), hd.grad.cpu()))
    for other in res[1:]:
        assert torch.equal(res[0][1], other[1])  # the same noisy height map
        for a, b in zip(res[0][:1] + res[0][2:], other[:1] + other[2:]):
            assert rel_l2(a.numpy(), b.numpy()) <= 1e-6


def test_qat_graph_device_rng_deterministic_and_trains():
    from quantizationawarethzdoe_amd import qat
    dev = _dev()
    runs = []
    for _ in range(2):
        torch.manual_seed(21)
        system = qat.FourFocalSpotsSystem(device=dev)
        tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=60, graph=True)
        assert tr._step_state.device_rng
        runs.append([float(tr.step(f)) for f in np.linspace(0.0, 0.95, 60)])
    a, b = np.array(runs[0]), np.array(runs[1])
    assert np.array_equal(a, b)  # same seed -> same device draws -> same trajectory
    assert np.isfinite(a).all() and a[-10:].mean() < a[:10].mean()


def test_eager_forward_after_graph_training_draws_fresh_noise():
    """The trainer's device generator and schedule buffer sit on the layer only while it captures
    (ADVICE round 2): after graph training, eager forwards draw their tolerance / Gumbel noise
    from torch's generator again -- two calls give different noisy height maps -- and follow the
    iter_frac they are given."""
    from quantizationawarethzdoe_amd import qat
    dev = _dev()
    torch.manual_seed(5)
    system = qat.FourFocalSpotsSystem(device=dev)
    tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=20, graph=True)
    for f in (0.1, 0.5, 0.9):
        tr.step(f)
    assert "_rng" not in system.doe.__dict__ and "_dyn" not in system.doe.__dict__
    with torch.no_grad():
        system(0.9)
        h1 = system.doe.height_map.detach().clone()
        o1 = system(0.9).data.detach().clone()
        o2 = system(0.9).data.detach().clone()
    assert not torch.equal(o1, o2)  # fresh tolerance noise per eager call
    assert torch.isfinite(h1).all()
