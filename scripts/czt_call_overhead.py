"""cfg3 per-call breakdown on one GPU: host submission time per czt_apply call (no sync), GPU time
per call (HIP events around a batch of calls) and wall time per call; run under rocprofv3
--kernel-trace to see the device timeline between the two passes and between calls."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bench import C0, cfg3_input
from quantizationawarethzdoe_amd.propagation import czt_apply

dev = torch.device("cuda:0")
freqs = torch.linspace(220e9, 330e9, 32, dtype=torch.float64)
lam = [float(torch.tensor(C0 / float(f), dtype=torch.float32)) for f in freqs]
x = torch.stack([cfg3_input(i) for i in range(32)])[None].to(dev)
sp = [float(torch.tensor(0.5e-3, dtype=torch.float32))] * 2
for _ in range(3):
    czt_apply(x, lam, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
torch.cuda.synchronize()
n = 20
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record()
host = []
for _ in range(n):
    h0 = time.perf_counter()
    czt_apply(x, lam, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
    host.append(time.perf_counter() - h0)
e1.record()
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"host submit per call {1e3 * sum(host) / n:.3f} ms (max {1e3 * max(host):.3f}); "
      f"gpu per call {e0.elapsed_time(e1) / n:.3f} ms; wall per call {1e3 * wall / n:.3f} ms")
