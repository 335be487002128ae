#!/usr/bin/env python3
"""Graph-replayed training steps of one small workload for a rocprofv3 kernel trace (which kernels one
replayed step runs, and for how long):

    python3 scripts/small_prof.py {donn32,donn256,qat,dual,edof} [steps]

donn32 / donn256: the cfg5 DONN step (chained) at batch 32 (one rank's share of an 8-GPU run) or
256; qat: the cfg4 four-focal-spots step; dual / edof: the dual-plane hologram and extended-DOF
steps (plot_data/example_2, example_3).  Each runs 5 warm-up steps (captures included), then
``steps`` replays between two markers printed to stdout with the wall time per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from quantizationawarethzdoe_amd import donn, qat  # noqa: E402

which = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda:0")
torch.manual_seed(0)
if which.startswith("donn"):
    B = int(which[4:])
    model = donn.DONN(device=dev)
    tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True, chained=True)
    u = torch.rand(B, 1, 100, 100, device=dev)
    labels = torch.randint(0, 10, (B,), device=dev)

    def step():
        tr.step(u, labels, 0.5)
else:
    if which == "qat":
        system, target, lr, opt = qat.FourFocalSpotsSystem(device=dev), qat.four_focal_spots_target(device=dev), 0.02, "adam"
    elif which == "dual":
        system, target, lr, opt = qat.DualPlaneSystem(device=dev), qat.logo_targets(device=dev), 0.01, "adamw"
    else:
        system, target, lr, opt = qat.ExtendedDOFSystem(device=dev), qat.edof_target(device=dev), 0.02, "adamw"
    tq = qat.QATTrainer(system, target, lr=lr, max_itrs=6000, graph=True, optimizer=opt)

    def step():
        tq.step(0.9)
for _ in range(5):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / steps
print(f"{which}: {dt * 1e3:.4f} ms per step over {steps} replays")
