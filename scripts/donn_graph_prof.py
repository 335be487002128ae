"""Graph-replayed cfg5 DONN steps (chained, batch 256) for a rocprofv3 kernel trace."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantizationawarethzdoe_amd import donn  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
model = donn.DONN(device=dev)
tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True)
u = torch.rand(256, 1, 100, 100, device=dev)
labels = torch.randint(0, 10, (256,), device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    tr.step(u, labels)
torch.cuda.synchronize()
print("done")
