#!/usr/bin/env python3
"""Host time per graph-replayed QAT / DONN step, split into its parts (schedule values, ring staging,
the graph launch, the slot event) against the wall time per step: is the small step bound by the
host's calls or by the GPU?  python3 scripts/host_probe.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quantizationawarethzdoe_amd import donn, qat  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda:0")
T = {}


def wrap(obj, name, key):
    f = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        T[key] = T.get(key, 0.0) + time.perf_counter() - t0
        return r
    setattr(obj, name, w)


def run(label, step):
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    T.clear()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    host = time.perf_counter() - t0
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    parts = " ".join(f"{k} {v / steps * 1e6:.1f}" for k, v in sorted(T.items()))
    print(f"{label}: wall {wall / steps * 1e6:.1f} us/step, host loop {host / steps * 1e6:.1f} us/step; {parts}",
          flush=True)


torch.manual_seed(0)
tq = qat.QATTrainer(qat.FourFocalSpotsSystem(device=dev), qat.four_focal_spots_target(device=dev), lr=0.02,
                    max_itrs=6000, graph=True, optimizer="adam")
tq.step(0.9)
ss = tq._step_state
wrap(ss, "stage", "stage")
wrap(ss, "launched", "event")
g = tq._graphs[tq.system.doe._graph_phase(0.9)][0]
wrap(g, "replay", "replay")
run("qat", lambda: tq.step(0.9))
g2 = tq._graphs[tq.system.doe._graph_phase(0.9)][0]
run("qat bare replay", g2.replay)

model = donn.DONN(device=dev)
tr = donn.DONNTrainer(model, donn.detector_targets(device=dev), graph=True, chained=True)
u = torch.rand(32, 1, 100, 100, device=dev)
labels = torch.randint(0, 10, (32,), device=dev)
tr.step(u, labels, 0.5)
gd = tr._graphs[model.does[0]._graph_phase(0.5)][0]
wrap(gd, "replay", "replay")
wrap(tr._step_state, "stage", "stage")
run("donn32", lambda: tr.step(u, labels, 0.5))
