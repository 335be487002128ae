"""Graph-replayed cfg4 QAT steps (quantized phase) for a rocprofv3 kernel trace."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantizationawarethzdoe_amd import qat  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
system = qat.FourFocalSpotsSystem(device=dev)
tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=6000, graph=True)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 100):
    tr.step(0.9)
torch.cuda.synchronize()
print("done")
