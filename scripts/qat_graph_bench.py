"""Eager vs graph-replayed QAT step time (cfg4), per schedule phase."""
import sys
import time

import torch

sys.path.insert(0, '.')
from quantizationawarethzdoe_amd import qat  # noqa: E402

dev = torch.device('cuda')
for graph in (False, True):
    torch.manual_seed(0)
    system = qat.FourFocalSpotsSystem(device=dev)
    tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=6000, graph=graph)
    for frac in (0.1, 0.5, 0.9):
        for _ in range(5):
            tr.step(frac)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(200):
            loss = tr.step(frac)
        torch.cuda.synchronize()
        print(f"graph={graph} frac={frac} ms/it={(time.perf_counter() - t0) / 200 * 1e3:.3f} loss={float(loss):.5f}")
