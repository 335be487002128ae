"""The gradient all-reduce captured inside the step's HIP graph (``capture_collective``), on a
one-rank RCCL process group with the collective forced on (``force_collective``): the step is
then ONE replay with the RCCL all-reduce kernel inside it, instead of the fwd/bwd replay, an eager
all-reduce and the optimiser replay.  Same trajectory bit for bit as the split form (a one-rank
sum is the identity), for the QAT (cfg4) and DONN (cfg5) trainers; the per-step times of both
forms are printed (-s) for the record.  Multi-rank capture needs more than the one GPU a test box
has; the eager split form stays the default."""
import os
import socket
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def one_rank_rccl():
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    # no event reuse in the PG watchdog (bench.py sets the same): see the note there
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=torch.device("cuda:0"))
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def _time_steps(step, n=200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def test_qat_captured_allreduce_matches_split_graphs(one_rank_rccl):
    from quantizationawarethzdoe_amd import qat
    dev = torch.device("cuda:0")
    res = {}
    for capture in (False, True):
        torch.manual_seed(5)
        system = qat.FourFocalSpotsSystem(device=dev)
        tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), graph=True, force_collective=True,
                            capture_collective=capture)
        assert tr.allreduce.active and tr.allreduce.world == 1
        losses = [float(tr.step(f)) for f in np.linspace(0.0, 0.95, 30)]
        w = next(iter(system.parameters())).detach().clone()
        ms = _time_steps(lambda: tr.step(0.9))
        res[capture] = (losses, w, ms)
        assert all(g is None for _, g, _ in tr._graphs.values()) == capture  # one replay per step
    assert res[False][0] == res[True][0] and torch.equal(res[False][1], res[True][1])
    print(f"\ncfg4 QAT step, one-rank RCCL all-reduce: split graphs + eager collective {res[False][2]:.4f} ms, "
          f"captured {res[True][2]:.4f} ms")


def test_donn_captured_allreduce_matches_split_graphs(one_rank_rccl):
    from quantizationawarethzdoe_amd import donn
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    u = torch.rand(32, 1, 100, 100, generator=g).to(dev)
    labels = torch.randint(0, 10, (32,), generator=g).to(dev)
    targets = donn.detector_targets(device=dev)
    res = {}
    for capture in (False, True):
        torch.manual_seed(7)
        model = donn.DONN(device=dev)
        tr = donn.DONNTrainer(model, targets, graph=True, force_collective=True, capture_collective=capture)
        losses = [float(tr.step(u, labels)) for _ in range(8)]
        ws = [p.detach().clone() for p in tr.params]
        ms = _time_steps(lambda: tr.step(u, labels), n=50)
        res[capture] = (losses, ws, ms)
    assert res[False][0] == res[True][0]
    assert all(torch.equal(a, b) for a, b in zip(res[False][1], res[True][1]))
    print(f"\ncfg5 DONN step (batch 32), one-rank RCCL all-reduce: split {res[False][2]:.4f} ms, "
          f"captured {res[True][2]:.4f} ms")


@pytest.mark.parametrize("trainer", ["qat", "donn"])
def test_capture_collective_refused_without_the_event_cache_setting(one_rank_rccl, monkeypatch, trainer):
    """with TORCH_NCCL_CUDA_EVENT_CACHE not 0 in the process
    (qat.collective_capture_safe) a trainer asked to capture the all-reduce keeps it out of the
    graph: split graphs around the eager collective, a RuntimeWarning naming the variable, and the
    same trajectory as the split form asked for directly."""
    import warnings
    from quantizationawarethzdoe_amd import donn, qat
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(3)
    u = torch.rand(8, 1, 100, 100, generator=g).to(dev)
    labels = torch.randint(0, 10, (8,), generator=g).to(dev)
    res = {}
    for capture in (False, True):
        torch.manual_seed(5)
        if trainer == "qat":
            system = qat.FourFocalSpotsSystem(device=dev)
            tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), graph=True, force_collective=True,
                                capture_collective=capture)
            step = lambda f: tr.step(f)  # noqa: E731
        else:
            model = donn.DONN(device=dev)
            tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True, force_collective=True,
                                  capture_collective=capture)
            step = lambda f: tr.step(u, labels, f)  # noqa: E731
        with monkeypatch.context() as mp_:
            mp_.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")
            with warnings.catch_warnings(record=True) as rec:
                warnings.simplefilter("always")
                losses = [float(step(f)) for f in (0.1, 0.5, 0.9)]
        assert not tr.capture_collective
        assert all(g_opt is not None for _, g_opt, _ in tr._graphs.values())  # split form everywhere
        if capture:
            assert any("TORCH_NCCL_CUDA_EVENT_CACHE" in str(w.message) for w in rec)
        res[capture] = losses
    assert res[True] == res[False]


@pytest.mark.parametrize("which", ["qat", "donn", "qat_full", "donn_eager_first"])
def test_captured_trainers_keep_no_autograd_graph_alive(which):
    """the captured trainers used to keep a step's autograd graph alive (the DOE
    layer's attached ``height_map`` and the returned loss), so the next capture's backward reused
    the weight's AccumulateGrad node made on the warm-up stream and torch warned "AccumulateGrad
    node's stream does not match".  Three schedule phases (three captures) run warning-free, the
    layer's height map carries no grad_fn after a step, and the returned loss is detached."""
    import warnings
    from quantizationawarethzdoe_amd import donn, qat
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        if which.startswith("qat"):
            if which == "qat_full":
                # FullPrecisionDOELayer builds an attached height map in its constructor (the graph
                # the capture's warm-up must not inherit)
                from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
                dp, op = qat.default_params()
                system = qat.FourFocalSpotsSystem(doe_class=Q.FullPrecisionDOELayer, optim_params=op, device=dev)
            else:
                system = qat.FourFocalSpotsSystem(device=dev)
            tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=100, graph=True)
            for frac in (0.1, 0.1, 0.5, 0.5, 0.9, 0.9):
                loss = tr.step(frac)
            layers = [system.doe]
        else:
            model = donn.DONN(device=dev, q_method="sgs")
            u = torch.rand(4, 1, 100, 100, device=dev)
            lab = torch.randint(0, 10, (4,), device=dev)
            if which == "donn_eager_first":
                # eager steps on the default stream first (their graph must not reach the capture)
                eager = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=False)
                eager.step(u, lab, 0.1)
            tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True)
            for frac in (0.1, 0.1, 0.5, 0.5, 0.9, 0.9):
                loss = tr.step(u, lab, frac)
            layers = list(model.does)
        torch.cuda.synchronize()
    bad = [str(w.message) for w in rec if "AccumulateGrad" in str(w.message)]
    assert not bad, bad[:2]
    assert loss.grad_fn is None and torch.isfinite(loss)
    for d in layers:
        assert getattr(d, "height_map").grad_fn is None


@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_fused_backward_writes_gradients_into_the_allreduce_bucket(one_rank_rccl, graph):
    """With an active all-reduce the DOE layers' fused backward kernels write each weight's gradient
    into its slice of the flat bucket (doe.grad_slot), so pack / unpack copy nothing: after a step
    every DONN weight's .grad IS its bucket slice, and the trajectory equals the run without the
    collective (RCCL average over one rank), eager (zero_grad keeps the gradient tensors) and graph."""
    from quantizationawarethzdoe_amd import donn
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(4)
    u = torch.rand(8, 1, 100, 100, generator=g).to(dev)
    labels = torch.randint(0, 10, (8,), generator=g).to(dev)
    targets = donn.detector_targets(device=dev)
    res = {}
    for force in (False, True):
        torch.manual_seed(2)
        model = donn.DONN(device=dev)
        tr = donn.DONNTrainer(model, targets, graph=graph, force_collective=force, device_rng=False)
        losses = [float(tr.step(u, labels, 0.5)) for _ in range(4)]
        res[force] = (losses, [p.detach().clone() for p in tr.params])
        if force:
            flat = tr.allreduce.flat
            for p, off in zip(tr.allreduce.params, tr.allreduce._offsets):
                assert p.grad is not None and p.grad.data_ptr() == flat.data_ptr() + 4 * off
    assert res[True][0] == res[False][0]
    assert all(torch.equal(a, b) for a, b in zip(res[True][1], res[False][1]))
