#!/usr/bin/env python3
"""Per-kernel cost of graph-replayed launches on this box: a captured graph of N dependent tiny
kernels (ATen add_ on one element; this library's radial map on a 4 x 4 map, small kernel
arguments; the 300-point ASM of a 1-sample 100 x 100 field, three kernels with ~1.5 KB of kernel
arguments each), replayed R times: microseconds per kernel.  Run it under different HIP runtime
environments (the variables are read at process start) to see what the floor depends on.

    python3 scripts/launch_floor.py [N] [R]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes  # noqa: E402

import torch  # noqa: E402

from quantizationawarethzdoe_amd import _lib, propagation as P  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
R = int(sys.argv[2]) if len(sys.argv) > 2 else 50
dev = torch.device("cuda:0")
x = torch.zeros(1, device=dev)
prof = torch.rand(8, device=dev)
hmap = torch.empty(4, 4, device=dev)
field = torch.randn(1, 1, 100, 100, dtype=torch.complex64, device=dev)
ph, pw = P.asm_padding(100, 100, (2, 2))
L = _lib.lib()


def aten():
    for _ in range(N):
        x.add_(1.0)


def radial():
    s = P._stream_handle()
    for _ in range(N):
        _lib.check(L.thz_radial_forward(ctypes.c_void_p(prof.data_ptr()), 8, 4, 4, ctypes.c_void_p(hmap.data_ptr()), s))


def asm():
    for _ in range(N // 3):
        P.asm_apply(field, [2.998e8 / 300e9], (1e-3, 1e-3), [0.02], ph, pw, True, 1)


res = {}
for name, fn, k in (("aten_add", aten, N), ("thz_radial", radial, N), ("thz_asm300", asm, 3 * (N // 3))):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(R):
        g.replay()
    torch.cuda.synchronize()
    res[name] = (time.perf_counter() - t0) / (R * k) * 1e6
env = {k: os.environ[k] for k in sorted(os.environ) if k.startswith(("HIP_", "AMD_", "DEBUG_CLR", "ROC_", "GPU_"))}
print({k: round(v, 3) for k, v in res.items()}, "us/kernel", env, flush=True)
