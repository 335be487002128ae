#!/usr/bin/env python3
"""Graph-replayed cfg5 DONN training steps (batch 256) and cfg4 QAT steps for a rocprofv3 kernel
trace: which kernels one replayed step runs.  python3 scripts/donn_graph_prof.py [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from quantizationawarethzdoe_amd import donn, qat  # noqa: E402

dev = torch.device("cuda:0")
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for chained in (True, False):
    torch.manual_seed(0)
    model = donn.DONN(device=dev)
    tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True, chained=chained)
    u = torch.rand(256, 1, 100, 100, device=dev)
    labels = torch.randint(0, 10, (256,), device=dev)
    for _ in range(steps):
        tr.step(u, labels)
torch.manual_seed(0)
system = qat.FourFocalSpotsSystem(device=dev)
tq = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=6000, graph=True)
for _ in range(steps):
    tq.step(0.9)
torch.cuda.synchronize()
print("done")
