import torch, time, sys
sys.path.insert(0, '.')
from quantizationawarethzdoe_amd import qat
dev = torch.device('cuda')
torch.manual_seed(0)
system = qat.FourFocalSpotsSystem(device=dev)
tr = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=6000)
for _ in range(10): tr.step(0.9)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(100): tr.step(0.9)
torch.cuda.synchronize()
print("ms/it", (time.perf_counter() - t0) * 10)
