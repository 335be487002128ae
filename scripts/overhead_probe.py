#!/usr/bin/env python3
"""How much of a graph-replayed small step is its per-step host->device traffic (the step-state
upload, the DONN batch copy and target gather) rather than the captured kernels: the step as
shipped, then (results no longer valid: timing only) with those copies skipped, so only the replay
runs.  python3 scripts/overhead_probe.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantizationawarethzdoe_amd import donn, qat  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda:0")


def timed(name, fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    print(f"{name}: {(time.perf_counter() - t0) / steps * 1e3:.4f} ms per step", flush=True)


torch.manual_seed(0)
tq = qat.QATTrainer(qat.FourFocalSpotsSystem(device=dev), qat.four_focal_spots_target(device=dev), lr=0.02,
                    max_itrs=6000, graph=True, optimizer="adam")
timed("qat shipped", lambda: tq.step(0.9))
up = tq._step_state.upload
tq._step_state.upload = lambda *a, **k: None
timed("qat no upload", lambda: tq.step(0.9))
g = tq._graphs[tq.system.doe._graph_phase(0.9)][0]
timed("qat bare replay", g.replay)
tq._step_state.upload = up

for B in (32, 256):
    model = donn.DONN(device=dev)
    tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True, chained=True)
    u = torch.rand(B, 1, 100, 100, device=dev)
    labels = torch.randint(0, 10, (B,), device=dev)
    timed(f"donn{B} shipped", lambda: tr.step(u, labels, 0.5))
    g = tr._graphs[model.does[0]._graph_phase(0.5)][0]
    timed(f"donn{B} bare replay", g.replay)
