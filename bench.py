#!/usr/bin/env python3
"""Headline benchmark: complex-field propagations/s (N x N) + achieved HBM GB/s.

Workload (BASELINE.json configs[1]): band-limited ASM of a 4096^2
Gaussian beam (w = 50 mm, 300 GHz, dx = 0.25 mm, padding_scale 1 -> P = 8192, exact
band limit) to 64 z-planes per GPU, z spread over 20..120 mm (the extend-DOF sweep,
experiment_extend_depth_of_focus.ipynb:229).  One step = all 64 planes of one rank
through the hand-written gfx950 kernels (one shared row pass + per-z column / row
passes).  Multi-GPU: one process per GPU, z-planes sharded across ranks (weak
scaling: 64 planes per rank, the global sweep grows with N), no data-path collective;
a barrier + synchronize bracket the timed region and the max time over ranks counts.

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import contextlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

C0 = 2.998e8
N_FIELD = 4096
DX = 0.25e-3
WAIST = 50e-3
FREQ = 300e9
Z_PER_RANK = 64
Z_MIN, Z_MAX = 20e-3, 120e-3
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
METRIC = "complex-field propagations/sec (N×N) + achieved HBM GB/s at 1/2/4/8 GPU"


def gaussian(N, dx, w, device):
    """Guassian_beam (LightSource/Gaussian_beam.py:88-160) at its waist, generated on the device
    by the thz_gaussian_beam kernel (CPU sample: the oracle's restatement)."""
    lam = C0 / FREQ
    if torch.device(device).type == "cpu":
        from oracle import thz_oracle as orc
        d = torch.tensor(dx, dtype=torch.float32)
        return orc.gaussian_beam(N, N, d, d, torch.tensor([lam], dtype=torch.float32), w, w).to(torch.complex64)
    from quantizationawarethzdoe_amd.optics import gaussian_beam
    return gaussian_beam(N, N, dx, dx, [lam], [w], [w], device=device)


def cfg3_input(i, n=2048):
    """cfg3 input plane of wavelength i, [n, n] complex64: unit-variance white noise from a seeded CPU
    generator.  A white field, not SURVEY §8(d)'s Gaussian beam: for a centred Gaussian the
    reference's CZT returns |E| <= 2e-8 (fp64) from a unit-peak beam, so its output is rounding
    noise that no check can grade (tests/golden/gen_cfg3_check.py); the kernels' work does not
    depend on the data."""
    g = torch.Generator().manual_seed(3000 + i)
    v = torch.randn(2, n, n, generator=g)
    return torch.complex(v[0], v[1]) * (0.5 ** 0.5)


def cfg5_inputs(B=256):
    """The cfg5 check step's data (tests/golden/gen_cfg5_check.py): images u [B, 1, 100, 100] in
    [0, 1), labels [B], the three FullPrecision layers' weights -pi + 2 pi U[0, 1) [1, 1, 100, 100]
    (FullPrecisionDOELayer.build_weight_height_map) and their height-noise planes U[0, 1)
    [100, 100], from one seeded CPU generator."""
    g = torch.Generator().manual_seed(55)
    u = torch.rand(B, 1, 100, 100, generator=g)
    labels = torch.randint(0, 10, (B,), generator=g)
    weights = [-torch.pi + 2 * torch.pi * torch.rand(1, 1, 100, 100, generator=g) for _ in range(3)]
    noises = [torch.rand(100, 100, generator=g) for _ in range(3)]
    return u, labels, weights, noises


def shard_planes(n_planes, rank, world):
    """Contiguous block of plane indices of one rank (every plane exactly once)."""
    base, extra = divmod(n_planes, world)
    start = rank * base + min(rank, extra)
    return list(range(start, start + base + (1 if rank < extra else 0)))


def z_planes(rank, world, split="weak"):
    """This rank's share of the global sweep: weak scaling (the default) gives every rank Z_PER_RANK
    planes of a Z_PER_RANK * world sweep; strong scaling splits the 64-plane cfg2 sweep itself over
    the ranks (8 z per GPU at N = 8)."""
    total = Z_PER_RANK * world if split == "weak" else Z_PER_RANK
    zs = torch.linspace(Z_MIN, Z_MAX, total, dtype=torch.float64)
    return [float(zs[i]) for i in shard_planes(total, rank, world)]


def host_cpu_share():
    """(threads to use, facts): the host cores this process may use -- the smallest of its CPU
    affinity (os.sched_getaffinity), the cgroup CPU quota (cgroup v2 cpu.max / v1 cfs quota, in
    whole CPUs) and OMP_NUM_THREADS when the launcher sets one (the GPU box's lease sets it to its
    CPU share) -- with each figure reported."""
    import math
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
                q = float(fh.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                per = float(fh.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    omp_n = int(omp) if omp and omp.isdigit() and int(omp) > 0 else None
    cands = {"affinity": aff}
    if quota is not None:
        cands["cgroup_quota"] = max(1, int(math.floor(quota)))
    if omp_n is not None:
        cands["OMP_NUM_THREADS"] = omp_n
    limit = min(cands, key=lambda k: cands[k])
    return cands[limit], {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "omp_num_threads": omp_n,
                          "host_cpus": os.cpu_count(), "threads_limited_by": limit}


def cpu_baseline(budget_s=30.0, max_planes=64, progress=False):
    """The oracle (PyTorch-CPU restatement of the reference op sequence, oracle/thz_oracle.py:105-119:
    per-call transfer-function rebuild, four fftshifts, full P x P FFTs) timed on this host's cores
    (host_cpu_share) on a bounded sample of the same workload: whole 4096^2 planes of the 64-plane
    sweep, spread over the sweep, until all 64 planes or the time budget is used."""
    from oracle import thz_oracle as orc
    threads, share = host_cpu_share()
    torch.set_num_threads(threads)
    x = gaussian(N_FIELD, DX, WAIST, "cpu")
    lam = torch.tensor([C0 / FREQ], dtype=torch.float32)
    sp = torch.tensor([DX, DX], dtype=torch.float32)
    zs = z_planes(0, 1)
    # bit-reversed plane order: any prefix of it is spread over the whole 20-120 mm sweep
    order = sorted(range(len(zs)), key=lambda i: int(format(i, "06b")[::-1], 2))
    orc.asm_forward(x[..., :512, :512], lam, sp, zs[0], 1)  # warm MKL
    t0 = time.perf_counter()
    n = 0
    while n < min(max_planes, len(zs)):
        orc.asm_forward(x, lam, sp, zs[order[n]], 1)
        n += 1
        if progress:
            print(f"cpu_baseline: plane {n}/{max_planes} {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return dict({"value": n / dt, "unit": "propagations/s", "cores": threads, "kind": "port",
                 "cpu_model": cpu_model(),
                 "sample": f"{n} of the 64 planes of the cfg2 workload (4096^2 -> P=8192, exact band limit; planes in "
                           f"bit-reversed order, so the sample spreads over the 20-120 mm sweep) through oracle.thz_oracle.asm_forward, torch-CPU "
                           f"fp32, {threads} threads, {dt:.1f} s"}, **share)


def _rel(a, b):
    import numpy as np
    a = np.asarray(a, dtype=np.complex128)
    b = np.asarray(b, dtype=np.complex128)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


CZT_CHECK_TOL = 2e-3  # rel-L2 vs the reference's fp64 signature (its own fp32 output: up to 1.8e-2)


def check_czt(out, idx):
    """Outside the timed region: output planes of the cfg3 call (wavelength indices ``idx`` of the
    32) vs the REFERENCE's own fp64 signature on the same inputs (tests/golden/cfg3_check.npz, made
    by tests/golden/gen_cfg3_check.py): E[::8, ::8], row 256 and the plane energy."""
    import numpy as np
    with np.load(os.path.join(ROOT, "tests", "golden", "cfg3_check.npz"), allow_pickle=False) as G:
        sub, row, en = G["sub64"], G["row64"], G["energy64"]
        st, rw = int(G["sub"]), int(G["row"])
    planes = []
    for j, i in enumerate(idx):
        p = out[0, j]
        e = float((p.abs().double() ** 2).sum())
        r = {"wavelength": i, "rel_sub": _rel(p[::st, ::st].cpu().numpy(), sub[i]),
             "rel_row": _rel(p[rw].cpu().numpy(), row[i]), "rel_energy": abs(e - float(en[i])) / float(en[i])}
        r["ok"] = bool(r["rel_sub"] <= CZT_CHECK_TOL and r["rel_row"] <= CZT_CHECK_TOL and r["rel_energy"] <= CZT_CHECK_TOL)
        planes.append(r)
    return {"ok": all(p["ok"] for p in planes), "tol": CZT_CHECK_TOL,
            "max_rel_sub": max(p["rel_sub"] for p in planes), "max_rel_row": max(p["rel_row"] for p in planes),
            "planes_checked": len(planes), "reference": "tests/golden/cfg3_check.npz (fp64)"}


def bench_czt(dev, rank, world, steps=30, warmup=3, dist=None):
    """cfg3 (secondary line): CZT 2048^2 -> 512^2 zoom (dx 0.5 -> 0.25 mm, z 0.5 m) at 32
    wavelengths c0 / linspace(220, 330 GHz) of seeded white input planes (cfg3_input); the
    wavelengths are sharded over the ranks (strong scaling, no collective).  Every output plane of
    the last timed call is checked against the reference's fp64 signature afterwards."""
    from quantizationawarethzdoe_amd.propagation import czt_apply
    freqs = torch.linspace(220e9, 330e9, 32, dtype=torch.float64)
    lam_all = [float(torch.tensor(C0 / float(f), dtype=torch.float32)) for f in freqs]
    idx = shard_planes(32, rank, world)
    mine = [lam_all[i] for i in idx]
    if not mine:
        return None
    x = torch.stack([cfg3_input(i) for i in idx])[None].to(dev)
    sp = [float(torch.tensor(0.5e-3, dtype=torch.float32))] * 2
    for _ in range(warmup):
        czt_apply(x, mine, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = czt_apply(x, mine, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    check = check_czt(out, idx)
    # per-kernel HIP-event times (separate calls, outside the timed region)
    from quantizationawarethzdoe_amd import _lib
    _lib.timing_reset()
    _lib.timing_enable(True)
    for _ in range(3):
        czt_apply(x, mine, sp, 0.5, 512, 512, 0.25e-3, 0.25e-3)
    torch.cuda.synchronize()
    _lib.timing_enable(False)
    kern = {}
    for k in ("czt_tables", "czt_rows", "czt_cols"):
        ms, n = _lib.timing_read(k)
        if n:
            kern[k] = round(ms / n, 4)
    # SURVEY §8(d) CZT byte model per (b, lambda): 8 (H W + 2 W M1 + M1 M2)
    model = 8 * (2048 * 2048 + 2 * 2048 * 512 + 512 * 512) * len(mine)
    return {"workload": "cfg3: CZT_prop 2048^2 -> 512^2, 32 wavelengths 220-330 GHz sharded over ranks, "
                        "seeded white input planes",
            "value": round(32 * steps / dt, 2), "unit": "propagations/s", "ms_per_call": round(dt / steps * 1e3, 3),
            "kernel_avg_ms": kern, "hbm_gbs_model": round(model / (dt / steps) / 1e9, 1),
            "scaling": "strong", "output_check": check}


def _golden(name):
    import numpy as np
    with np.load(os.path.join(ROOT, "tests", "golden", f"{name}_golden.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def check_qat(dev):
    """Outside the timed region: the reference's own 20-step four-focal-spots QAT trace
    (tests/golden/qat_golden.npz: its initial weights and every Gumbel / height-noise draw,
    replayed in order) through the same system, kernels and Adam; per-step loss within 1e-3
    relative (tests/test_optics_qat_gpu.py's bound).  The schedule runs 0 .. 0.95, so all three
    phases are covered."""
    import numpy as np
    from quantizationawarethzdoe_amd import qat
    A = _golden("qat")
    with open(os.path.join(ROOT, "tests", "golden", "manifest.json")) as fh:
        q = json.load(fh)["qat"]
    system = qat.FourFocalSpotsSystem(device=dev)
    with torch.no_grad():
        system.doe.weight_init_phase.copy_(torch.from_numpy(A["w0"]))
    trainer = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), lr=q["lr"], max_itrs=q["steps"])
    expo, unif = [], []
    for st in range(q["steps"]):
        for i, k in enumerate(q["draws"][st]):
            (expo if k == "expo" else unif).append(A[f"step{st}__draw{i}"])
    expo.reverse()
    unif.reverse()
    system.doe._gumbel_noise = lambda shape, like: torch.from_numpy(expo.pop()).to(like.device)
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **kw: torch.from_numpy(unif.pop()).to(device=t.device, dtype=t.dtype)
    try:
        losses = [float(trainer.step().detach()) for _ in range(q["steps"])]
    finally:
        torch.rand_like = orig
    ref = np.array(q["losses"])
    rel = np.abs(np.array(losses) - ref) / ref
    return {"ok": bool(rel.max() <= 1e-3 and not expo and not unif), "tol": 1e-3, "max_rel_loss": float(rel.max()),
            "steps": q["steps"], "reference": "tests/golden/qat_golden.npz (the reference's own fp32 trace)"}


def bench_qat(dev, rank, world, steps=60, dist=None):
    """cfg4 (secondary line): four-focal-spots QAT iterations/s in each schedule phase (iter_frac
    <= 0.3 continuous, 0.3-0.8 blend, > 0.8 quantized), with the one-bucket gradient all-reduce
    across ranks (each rank its own noise sample; on RCCL captured inside the step's HIP graph, so
    a step is one replay).  Afterwards the reference's 20-step trace is
    replayed through the same kernels (check_qat)."""
    from quantizationawarethzdoe_amd import qat
    torch.manual_seed(1234 + rank)
    system = qat.FourFocalSpotsSystem(device=dev)
    trainer = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), max_itrs=6000, graph=True,
                             capture_collective=True)
    out = {}
    for name, frac in (("continuous", 0.1), ("blend", 0.5), ("quantized", 0.9)):
        for _ in range(5):
            trainer.step(frac)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = trainer.step(frac)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out[name] = {"it_per_s": round(steps / dt, 1), "ms_per_it": round(dt / steps * 1e3, 3),
                     "loss": round(float(loss.detach()), 6)}
    return {"workload": "cfg4: four_focal_spots QAT step (v3 DOE 100^2, ASM P=300, fused loss, Adam), "
                        "HIP-graph replay per schedule phase, gradient all-reduce over ranks (RCCL: inside the graph)",
            "graph_collective": bool(trainer.allreduce.capturable and trainer.capture_collective), "phases": out,
            "output_check": check_qat(dev), "quality_6000": qat_quality_6000(dev)}


def qat_quality_6000(dev, seed=0, iters=6000):
    """Outside the timed region: the notebook's whole v3 run (experiment_four_focal_spots.ipynb
    cells 6-8: 6,000 iterations, iter_frac = itr / 6000, Adam lr 0.02) on this rank's GPU, its
    final / minimum / last-100-mean loss against the reference's own curve
    (plot_data/example_1/loss_curve_Ours.npy via tests/golden/qat_curves.json).  ok: the
    last-100 mean and the minimum within [0.5x, 2x] of the reference's (tests/test_qat_quality_gpu.py;
    scripts/qat_quality.py runs every method with five seeds)."""
    import numpy as np
    from quantizationawarethzdoe_amd import qat
    with open(os.path.join(ROOT, "tests", "golden", "qat_curves.json")) as fh:
        ref = json.load(fh)["methods"]["Ours"]
    torch.manual_seed(seed)
    system = qat.FourFocalSpotsSystem(device=dev)
    trainer = qat.QATTrainer(system, qat.four_focal_spots_target(device=dev), lr=0.02, max_itrs=iters, graph=True)
    curve, dt = trainer.train(iters, log_every=0)
    c = curve.double().numpy()
    st = {"final": float(c[-1]), "min": float(c.min()), "mean_last100": float(c[-100:].mean())}
    ok = bool(np.all(np.isfinite(c)) and all(0.5 * ref[k] <= st[k] <= 2.0 * ref[k] for k in ("min", "mean_last100")))
    return {"iterations": iters, "seconds": round(dt, 2), "ok": ok, **{k: float(f"{v:.4g}") for k, v in st.items()},
            "reference": {k: float(f"{ref[k]:.4g}") for k in ("final", "min", "mean_last100")},
            "reference_source": "plot_data/example_1/loss_curve_Ours.npy (tests/golden/qat_curves.json)"}


def check_qat_multi(dev, which):
    """Outside the timed region: the reference's own 20-step trace of the dual-plane hologram
    (``which`` = "dual") or the extended depth of focus ("edof") -- tests/golden/qat_{which}_golden.npz,
    made by tests/golden/gen_qat_multi.py: its initial weight, every Gumbel / height-noise draw and
    (edof) every re-drawn plane replayed in order -- through the same system, kernels and AdamW;
    per-step loss within 1e-3 relative (tests/test_qat_multi_gpu.py)."""
    import numpy as np
    from quantizationawarethzdoe_amd import qat
    with np.load(os.path.join(ROOT, "tests", "golden", f"qat_{which}_golden.npz"), allow_pickle=False) as z:
        A = {k: z[k] for k in z.files}
    with open(os.path.join(ROOT, "tests", "golden", "qat_multi_manifest.json")) as fh:
        q = json.load(fh)[which]
    if which == "dual":
        system, target = qat.DualPlaneSystem(device=dev), qat.logo_targets(device=dev)
    else:
        system, target = qat.ExtendedDOFSystem(device=dev), qat.edof_target(device=dev)
        nxt = iter(A["zs"][1:])

        def next_planes():
            zs = next(nxt, None)
            if zs is not None:
                for p, zz in zip(system.props, zs):
                    p.z = float(zz)
        system.after_forward = next_planes
    with torch.no_grad():
        dict(system.doe.named_parameters())[q["param"]].copy_(torch.from_numpy(A["w0"]))
    trainer = qat.QATTrainer(system, target, lr=q["lr"], max_itrs=q["steps"], optimizer=q["optimizer"])
    expo, unif = [], []
    for st in range(q["steps"]):
        for i, k in enumerate(q["draws"][st]):
            (expo if k == "expo" else unif).append(A[f"step{st}__draw{i}"])
    expo.reverse()
    unif.reverse()
    system.doe._gumbel_noise = lambda shape, like: torch.from_numpy(expo.pop()).to(like.device)
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **kw: torch.from_numpy(unif.pop()).to(device=t.device, dtype=t.dtype)
    try:
        losses = [float(trainer.step().detach()) for _ in range(q["steps"])]
    finally:
        torch.rand_like = orig
    ref = np.array(q["losses"])
    rel = np.abs(np.array(losses) - ref) / ref
    return {"ok": bool(rel.max() <= 1e-3 and not expo and not unif), "tol": 1e-3, "max_rel_loss": float(rel.max()),
            "steps": q["steps"], "reference": f"tests/golden/qat_{which}_golden.npz (the reference's own fp32 trace)"}


def qat_multi_quality_6000(dev, which, seed=0, iters=6000):
    """Outside the timed region: the notebook's whole "Ours" run of the multi-plane system (6,000
    iterations, iter_frac = itr / 6000, AdamW) on the graph-replayed trainer, final / minimum /
    last-100-mean against the reference's curve (plot_data/example_2 or example_3
    loss_curve_Ours.npy via tests/golden/qat_curves.json); ok: the minimum and the last-100 mean
    within [0.5x, 2x] (tests/test_qat_quality_gpu.py runs three seeds)."""
    import numpy as np
    from quantizationawarethzdoe_amd import qat
    ex = {"dual": "example_2", "edof": "example_3"}[which]
    with open(os.path.join(ROOT, "tests", "golden", "qat_curves.json")) as fh:
        ref = json.load(fh)[ex]["methods"]["Ours"]
    torch.manual_seed(seed)
    if which == "dual":
        system, target, lr = qat.DualPlaneSystem(device=dev), qat.logo_targets(device=dev), 0.01
    else:
        system, target, lr = qat.ExtendedDOFSystem(seed=seed, device=dev), qat.edof_target(device=dev), 0.02
    trainer = qat.QATTrainer(system, target, lr=lr, max_itrs=iters, graph=True, optimizer="adamw")
    curve, dt = trainer.train(iters, log_every=0)
    c = curve.double().numpy()
    st = {"final": float(c[-1]), "min": float(c.min()), "mean_last100": float(c[-100:].mean())}
    ok = bool(np.all(np.isfinite(c)) and all(0.5 * ref[k] <= st[k] <= 2.0 * ref[k] for k in ("min", "mean_last100")))
    return {"iterations": iters, "seconds": round(dt, 2), "ok": ok, **{k: float(f"{v:.4g}") for k, v in st.items()},
            "reference": {k: float(f"{ref[k]:.4g}") for k in ("final", "min", "mean_last100")},
            "reference_source": f"plot_data/{ex}/loss_curve_Ours.npy (tests/golden/qat_curves.json)"}


def bench_qat_multi(dev, rank, world, which, steps=60, dist=None):
    """cfg4 family, secondary lines: the reference's two multi-plane QAT systems -- the dual-plane
    hologram (plot_data/example_2: v3 DOE, planes 100 / 150 mm, P = 300) and the extended depth of
    focus (example_3: rotationally symmetric v3, five planes re-drawn every iteration, P = 500, the
    runtime mixed-radix plan) -- iterations/s per schedule phase on the graph-replayed trainer: every
    plane from one pipeline (modulation fused into the shared row pass, one column pass over the
    planes, the Z-summing adjoint in backward), the planes read from the device step state, the
    one-bucket gradient all-reduce across ranks.  Then the reference's 20-step trace (check_qat_multi)
    and one 6,000-iteration run against the published curve."""
    from quantizationawarethzdoe_amd import qat
    torch.manual_seed(1234 + rank)
    if which == "dual":
        system, target, lr = qat.DualPlaneSystem(device=dev), qat.logo_targets(device=dev), 0.01
    else:
        system, target, lr = qat.ExtendedDOFSystem(seed=rank, device=dev), qat.edof_target(device=dev), 0.02
    trainer = qat.QATTrainer(system, target, lr=lr, max_itrs=6000, graph=True, capture_collective=True,
                             optimizer="adamw")
    out = {}
    for name, frac in (("continuous", 0.1), ("blend", 0.5), ("quantized", 0.9)):
        for _ in range(5):
            trainer.step(frac)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = trainer.step(frac)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out[name] = {"it_per_s": round(steps / dt, 1), "ms_per_it": round(dt / steps * 1e3, 3),
                     "loss": round(float(loss.detach()), 6)}
    desc = {"dual": "dual-plane hologram (example_2: v3 DOE 100^2, planes 100 / 150 mm, ASM P=300)",
            "edof": "extended depth of focus (example_3: rotationally symmetric v3 DOE 100^2, five planes "
                    "re-drawn every iteration, ASM P=500)"}[which]
    return {"workload": f"QAT step of the {desc}: all planes in one pipeline, fused loss over the planes, "
                        "Z-summing adjoint, AdamW, HIP-graph replay per schedule phase, gradient all-reduce "
                        "over ranks", "planes": len(system.planes),
            "graph_collective": bool(trainer.allreduce.capturable and trainer.capture_collective), "phases": out,
            "output_check": check_qat_multi(dev, which), "quality_6000": qat_multi_quality_6000(dev, which)}


def check_donn(dev, chained):
    """Outside the timed region: one cfg5 step at the bench's batch (256) through the same model,
    kernels and loss (eager, the noise injected), vs the REFERENCE's own fp64 loss and weight
    gradients of that step (tests/golden/cfg5_check.npz, made by tests/golden/gen_cfg5_check.py):
    loss within 1e-4 relative, gradients within 1e-3 rel-L2 (tests/test_donn_train_gpu.py)."""
    import numpy as np
    from quantizationawarethzdoe_amd import donn
    mode = "chained" if chained else "notebook"
    with np.load(os.path.join(ROOT, "tests", "golden", "cfg5_check.npz"), allow_pickle=False) as G:
        ref_loss = float(G[f"{mode}__loss64"])
        ref_g = [G[f"{mode}__g{i}_64"] for i in range(3)]
    u, labels, weights, noises = cfg5_inputs()
    model = donn.DONN(device=dev)
    with torch.no_grad():
        for d, w in zip(model.does, weights):
            next(iter(d.parameters())).copy_(w)
    targets = donn.detector_targets(device=dev)
    tr = donn.DONNTrainer(model, targets, chained=chained, device_rng=False)
    it = iter([n.to(dev) for n in noises])
    orig = torch.rand_like
    torch.rand_like = lambda t, *a, **k: next(it).to(dtype=t.dtype)
    try:
        loss = tr._loss(u.to(dev), targets.index_select(0, labels.to(dev)), None)
        loss.backward()
    finally:
        torch.rand_like = orig
    lrel = abs(float(loss.detach()) - ref_loss) / ref_loss
    grel = []
    for d, rg in zip(model.does, ref_g):
        g = next(iter(d.parameters())).grad
        g = np.zeros_like(rg) if g is None else g.detach().double().cpu().numpy()
        grel.append(_rel(g, rg) if np.abs(rg).max() > 0 else float(np.abs(g).max()))
    return {"ok": bool(lrel <= 1e-4 and max(grel) <= 1e-3), "rel_loss": lrel, "grad_rel_l2": grel,
            "batch": int(u.shape[0]), "reference": "tests/golden/cfg5_check.npz (fp64)"}


def bench_donn(dev, rank, world, steps=100, warmup=5, dist=None):
    """cfg5 (secondary line): 3-layer DONN (100^2 fields, ASM P = 300 between layers, the
    FullPrecision DOE layers the notebook instantiates) training step on a global batch of 256
    split over the ranks: forward, detector-target loss, backward, one-bucket gradient all-reduce
    (3 x 100^2 fp32 = 120 KB), Adam; HIP-graph replay.  Synthetic digits: uniform [0, 1) images
    and random labels (seed = rank); identical initial weights on every rank.  Each mode is then
    checked against the reference's own step at batch 256 (check_donn)."""
    from quantizationawarethzdoe_amd import donn
    per = len(shard_planes(256, rank, world))
    g = torch.Generator().manual_seed(rank)
    u = torch.rand(per, 1, 100, 100, generator=g).to(dev)
    labels = torch.randint(0, 10, (per,), generator=g).to(dev)
    targets = donn.detector_targets(device=dev)
    out = {}
    for name, chained in (("chained", True), ("notebook", False)):
        torch.manual_seed(1234)  # same initial weights on every rank
        model = donn.DONN(device=dev)
        torch.manual_seed(1234 + rank)  # per-rank height-noise draws
        tr = donn.DONNTrainer(model, targets, graph=True, chained=chained, capture_collective=True)
        for _ in range(warmup):
            tr.step(u, labels)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            loss = tr.step(u, labels)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out[name] = {"samples_per_s": round(256 * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3),
                     "graph_collective": bool(tr.allreduce.capturable and tr.capture_collective),
                     "loss": round(float(loss.detach()), 6), "output_check": check_donn(dev, chained)}
    return {"workload": "cfg5: 3-layer DONN (100^2, P=300 ASM, FullPrecision DOE layers) training step, global "
                        "batch 256 split over ranks, detector-target loss, gradient all-reduce, Adam, HIP-graph "
                        "replay; synthetic digits", "per_rank_batch": per, "modes": out}


def per_rank_shares(dev, x, lam, sp, world=8):
    """One GPU timing the work ONE rank of an 8-GPU run gets when each workload is split over the
    ranks (strong scaling): cfg2's 64-plane sweep at 8 planes, cfg3's 32 wavelengths at 4, cfg5's
    batch of 256 at 32.  Per-rank times, not a scaling claim: the 8-GPU step takes at least the
    slowest rank's share, so share_time x 8 / full_time is the efficiency a strong split can reach
    (the cfg3 columns pass, e.g., has 8x fewer lines to fill the chip with)."""
    from quantizationawarethzdoe_amd.propagation import asm_apply
    from quantizationawarethzdoe_amd import _lib
    zs = z_planes(0, world, "strong")
    out = torch.empty((len(zs), 1, 1, N_FIELD, N_FIELD), dtype=torch.complex64, device=dev)
    pad = N_FIELD // 2

    def step():
        asm_apply(x, lam, sp, zs, pad, pad, True, 1, out=out)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    _lib.timing_reset()
    _lib.timing_enable(True)
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    _lib.timing_enable(False)
    kern = {}
    for k in ("asm_rows_fwd", "asm_cols", "asm_rows_inv"):
        ms, n = _lib.timing_read(k)
        if n:
            kern[k] = round(ms / n, 4)
    chk = check_plane(out[0, 0, 0], zs[0])
    cfg2 = {"planes": len(zs), "ms_per_step": round(dt * 1e3, 3), "planes_per_s": round(len(zs) / dt, 1),
            "kernel_avg_ms": kern, "output_check": chk}
    czt = bench_czt(dev, 0, world)
    donn = bench_donn(dev, 0, world)
    return {"note": "one GPU timing one rank's share of an 8-GPU strong split; per-rank times, not a scaling "
                    "measurement", "cfg2_8_planes": cfg2,
            "cfg3_4_wavelengths": {k: czt[k] for k in ("ms_per_call", "kernel_avg_ms", "output_check")},
            "cfg5_batch_32": {m: {k: v[k] for k in ("ms_per_step", "output_check")} for m, v in donn["modes"].items()}}


def cpu_model():
    """Host CPU model name (the lscpu "Model name" line, read from /proc/cpuinfo)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def check_plane(plane, z):
    """Outside the timed region: one output plane of the bench vs the REFERENCE's own fp64 output
    signature of the same workload (tests/golden/cfg2_check.npz, made by tests/golden/
    gen_cfg2_check.py in the build container): energy, E[::64, ::64] and row 2048, rel-L2 <= 1e-4."""
    import numpy as np
    path = os.path.join(ROOT, "tests", "golden", "cfg2_check.npz")
    with np.load(path, allow_pickle=False) as G:
        zs = [float(v) for v in G["z"]]
        k = min(range(len(zs)), key=lambda i: abs(zs[i] - z))
        if abs(zs[k] - z) > 1e-9:
            return None
        sub = plane[::64, ::64].cpu().numpy().astype(np.complex128)
        row = plane[2048].cpu().numpy().astype(np.complex128)
        energy = float((plane.abs().double() ** 2).sum())

        def rel(a, b):
            return float(np.linalg.norm(a - b) / np.linalg.norm(b))
        r = {"z_m": z, "rel_sub": rel(sub, G[f"p{k}__sub64"]), "rel_row": rel(row, G[f"p{k}__row64"]),
             "rel_energy": abs(energy - float(G[f"p{k}__energy64"])) / float(G[f"p{k}__energy64"])}
    r["ok"] = bool(r["rel_sub"] <= 1e-4 and r["rel_row"] <= 1e-4 and r["rel_energy"] <= 1e-5)
    return r


class Ranks:
    """One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK / WORLD_SIZE): the barrier and
    the max-over-ranks reduction of the timed region.  ``dry_run``: every rank on the CPU over gloo,
    the propagation stubbed (tests/test_distributed_cpu.py rehearses the orchestration this way)."""

    def __init__(self, dry_run=False):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        self.dry_run = dry_run
        # rehearsing N > 1 on a one-GPU box: every rank on cuda:0 (gloo)
        if os.environ.get("THZ_BENCH_SAME_DEVICE"):
            local = 0
        backend = "gloo" if dry_run else os.environ.get("THZ_BENCH_BACKEND", "nccl")
        if dry_run:
            self.dev = torch.device("cpu")
        else:
            self.dev = torch.device("cuda", local)
            torch.cuda.set_device(self.dev)
        if self.world > 1:
            import torch.distributed as dist
            if backend == "nccl":
                # no event reuse in the PG's watchdog: a captured collective's end event handed back to
                # an eager work made the watchdog's query fail once ("operation not permitted on an
                # event last recorded in a capturing stream", test_collective_capture_gpu, round 5)
                os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(backend)
            self.dist = dist

    def sync(self):
        if not self.dry_run:
            torch.cuda.synchronize()

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, v):
        if self.dist is None:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=self.dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def timed(step, steps, warmup, ranks, on_start=None):
    """W untimed warmup steps, then EXACTLY K timed steps bracketed by a barrier + synchronize on
    both sides; returns the max over ranks of the elapsed wall time."""
    for _ in range(warmup):
        step()
    ranks.sync()
    if on_start:
        on_start()
    ranks.barrier()
    ranks.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ranks.sync()
    ranks.barrier()
    return ranks.max(time.perf_counter() - t0)


def launch_ranks(args):
    """``--gpus N`` without a launcher: start N ranks as a child torch.distributed.run (before anything
    touches the GPU; never an exec) and exit with its code.  Under a launcher, N must equal WORLD_SIZE."""
    if "WORLD_SIZE" in os.environ:
        if int(os.environ["WORLD_SIZE"]) != args.gpus:
            sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}\n")
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def _failed_checks(secondary):
    """The secondaries whose output check ran and failed (a wrong result), as strings: every
    ``output_check`` at any depth of a secondary's result (its modes, the per-rank shares)."""
    failed = []

    def walk(key, d):
        if not isinstance(d, dict) or "error" in d:
            return
        chk = d.get("output_check")
        if isinstance(chk, dict) and not chk.get("ok"):
            failed.append(f"{key}: {chk}")
        for k, v in d.items():
            if k != "output_check" and isinstance(v, dict):
                walk(f"{key}.{k}", v)
    for key, sec in (secondary or {}).items():
        walk(key, sec)
    return failed


WATCHDOG_EXIT = 4  # the secondaries outlived --secondary-timeout: the run did not finish


def _secondary_watchdog(line, keys, rank, timeout_s, snapshot):
    """A timer that, should the secondary measurements outlive ``timeout_s``, completes the JSON line
    with the headline and whatever secondaries finished, marks the rest as timed out, prints it on
    rank 0 and ends the process on every rank with WATCHDOG_EXIT (os._exit: a rank stuck in a GPU
    call or collective cannot be joined; a hang is a failure, not a success).  The headline
    measurement is already done when it starts.  ``snapshot`` is a list the main thread replaces
    with a finished copy of the secondaries after each one, so the timer never reads a dict that
    is being written; any failure inside the timer still ends in os._exit."""
    import threading

    def fire():
        try:
            done = dict(snapshot[0]) if snapshot else {}
            for k in keys:
                done.setdefault(k, {"error": f"timed out after {timeout_s:.0f} s (watchdog)"})
            if rank == 0:
                out = dict(line, secondary=done)
                sys.__stdout__.write(json.dumps(out) + "\n")
                sys.__stdout__.flush()
            failed = _failed_checks(done)
            sys.stderr.write(f"bench.py: secondary measurements exceeded {timeout_s:.0f} s; exiting "
                             f"with status {WATCHDOG_EXIT}\n")
            if failed:
                sys.stderr.write("bench.py: output check FAILED:\n  " + "\n  ".join(failed) + "\n")
            sys.stderr.flush()
        finally:
            os._exit(WATCHDOG_EXIT)

    t = threading.Timer(timeout_s, fire)
    t.daemon = True
    t.start()
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--z-chunk", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-planes", type=int, default=64, help="cpu_baseline sample size (whole 4096^2 planes)")
    ap.add_argument("--cpu-budget", type=float, default=30.0, help="cpu_baseline time budget, seconds")
    ap.add_argument("--headline-only", action="store_true", help="skip the cfg3 / cfg4 / cfg5 secondary measurements")
    ap.add_argument("--secondary-timeout", type=float, default=420.0,
                    help="seconds the cfg3 / cfg4 / cfg5 secondaries may take before the line is printed without them")
    ap.add_argument("--cpu-only", action="store_true",
                    help="time only the cpu_baseline leg (e.g. --cpu-planes 64 --cpu-budget 1e9 for the whole sweep)")
    ap.add_argument("--cfg2-split", choices=("weak", "strong"), default="weak",
                    help="weak: 64 z-planes per rank (the default line); strong: the 64-plane sweep split over the ranks")
    ap.add_argument("--no-shares", action="store_true",
                    help="skip the one-GPU timing of the per-rank shares of an 8-GPU run (world size 1 only)")
    ap.add_argument("--dry-run", action="store_true",
                    help="rehearse the rank orchestration on the CPU (gloo, propagation stubbed, no GPU)")
    args = ap.parse_args()
    if args.cpu_only:
        print(json.dumps({"cpu_baseline": cpu_baseline(args.cpu_budget, args.cpu_planes, progress=True)}))
        return
    launch_ranks(args)
    ranks = Ranks(args.dry_run)
    rank, world, dev = ranks.rank, ranks.world, ranks.dev
    zs = z_planes(rank, world, args.cfg2_split)
    total_planes = Z_PER_RANK * world if args.cfg2_split == "weak" else Z_PER_RANK
    if args.dry_run:
        done = []
        seen = torch.zeros(1, dtype=torch.float64)

        def step():
            done.append(len(zs))
            seen.add_(sum(zs))
        elapsed = timed(step, args.steps, args.warmup, ranks)
        planes = total_planes * args.steps
        cover = sorted(i for r in ranks.gather(shard_planes(total_planes, rank, world)) for i in r)
        lam_cover = sorted(i for r in ranks.gather(shard_planes(32, rank, world)) for i in r)  # cfg3 λ shards
        batch_cover = sorted(i for r in ranks.gather(shard_planes(256, rank, world)) for i in r)  # cfg5 batch
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": round(planes / elapsed, 2), "unit": "propagations/s",
                              "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dry_run": True,
                              "scaling": args.cfg2_split,
                              "planes_per_rank_step": done[-1], "planes_covered": cover,
                              "wavelengths_covered": lam_cover, "samples_covered": batch_cover,
                              "elapsed_max_s": elapsed}), flush=True)
        ranks.close()
        return

    from quantizationawarethzdoe_amd import _lib
    from quantizationawarethzdoe_amd.propagation import asm_apply, asm_plan_info

    x = gaussian(N_FIELD, DX, WAIST, dev)
    lam = [float(torch.tensor(C0 / FREQ, dtype=torch.float32))]
    sp = [float(torch.tensor(DX, dtype=torch.float32))] * 2
    pad = N_FIELD // 2
    out = torch.empty((len(zs), 1, 1, N_FIELD, N_FIELD), dtype=torch.complex64, device=dev)

    def step():
        asm_apply(x, lam, sp, zs, pad, pad, True, 1, z_chunk=args.z_chunk, out=out)

    def start_timing():
        _lib.timing_reset()
        _lib.timing_enable(True)
    elapsed = timed(step, args.steps, args.warmup, ranks, on_start=start_timing)
    _lib.timing_enable(False)
    kern = {k: _lib.timing_read(k) for k in ("asm_rows_fwd", "asm_cols", "asm_rows_inv")}
    # self-check outside the timed region: this rank's first plane (z = 20 mm on rank 0) and, when
    # it is in this rank's share, the sweep's last (120 mm), vs the reference's fp64 signature
    checks = [c for c in (check_plane(out[0, 0, 0], zs[0]), check_plane(out[-1, 0, 0], zs[-1])) if c]
    checks_ok = all(ranks.gather(all(c["ok"] for c in checks)))

    planes = total_planes * args.steps
    value = planes / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    # algorithmic bytes per launch.  SURVEY §8(d)'s figure: per (b, c) slice and plane the 3-pass FFT
    # convolution moves 8*[H*W + H*Pw + Z*(3*H*Pw + H*W)] (row pass reads H*W, writes H*Pw once; per
    # z the column pass reads and writes H*Pw, the row-inverse pass reads H*Pw and writes H*W).  The
    # kernels must move less: only the ncols band columns can be non-zero and the column spectrum
    # stays in registers across the z-chunk.  That minimum ("pruned") grades the roofline; the
    # SURVEY figure is kept under roofline_survey_model.
    ncols, zc = asm_plan_info(1, 1, N_FIELD, N_FIELD, pad, pad, True, 1, lam, sp, zs, args.z_chunk)
    H = W = N_FIELD
    Pw = 2 * N_FIELD
    model = {"asm_rows_fwd": 8 * (H * W + H * Pw), "asm_cols": 16 * zc * H * Pw,
             "asm_rows_inv": 8 * zc * (H * Pw + H * W)}
    pruned = {"asm_rows_fwd": 8 * (H * W + ncols * H), "asm_cols": 8 * (ncols * H + zc * ncols * H),
              "asm_rows_inv": 8 * (zc * ncols * H + zc * H * W)}
    stats = {}
    for k, (ms, n) in kern.items():
        if n:
            avg = ms / n
            stats[k] = {"avg_ms": avg, "launches": n, "alg_bytes": model[k], "pruned_bytes": pruned[k],
                        "gbs": model[k] / (avg * 1e-3) / 1e9, "gbs_pruned": pruned[k] / (avg * 1e-3) / 1e9}
    total_alg = sum(pruned[k] * stats[k]["launches"] for k in stats) / args.steps
    roof = roof_model = roof_step = None
    # roofline: ONE fixed kernel, K2 (asm_cols: the column FFT + transfer function, the kernel
    # north_star grades; K2 and K3 take about the same time, so grading "the dominant" one flipped
    # between them from box to box).  achieved = the bytes K2 must move (the band-pruned minimum:
    # only the ncols spectral columns that can be non-zero, the column spectrum kept in registers
    # across the z-chunk) / its live average launch time (HIP events on the launch stream).
    # traffic = null: PMC counters need rocprofv3 passes of their own, so no HBM byte count is
    # measured inside this run; the counter bytes per launch of the same kernels are in
    # profiles/pmc_traffic.json (a separate profiling run, named there).
    RK = "asm_cols"
    if RK in stats:
        k2 = stats[RK]
        roof = {"bound": "hbm", "kernel": "asm_cols (K2: column FFT + transfer function, north_star's kernel)",
                "achieved": round(k2["gbs_pruned"], 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(k2["gbs_pruned"] / HBM_PEAK_GBS, 4), "traffic": None,
                "traffic_note": "not measured in this run (PMC counters need their own rocprofv3 passes); "
                                "profiles/pmc_traffic.json holds the counter bytes per launch of a separate run",
                "alg_bytes_per_launch": pruned[RK], "avg_launch_ms": round(k2["avg_ms"], 4), "target_frac": 0.40,
                "bytes_model": f"band-pruned minimum per launch ({ncols} of {Pw} spectral columns can be non-zero; "
                               f"K2 keeps each column spectrum in registers across the z-chunk): "
                               f"8 (ncols H + zc ncols H), zc = {zc}"}
        roof_step = {"achieved": round(total_alg / (ms_per_step * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(total_alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_per_step": total_alg}
        # SURVEY §8(d)'s unpruned 3-pass figure, kept for comparison only: it charges K2 a per-z
        # re-read of the column that K2 does not do, so it exceeds 1 for K2
        roof_model = {"kernel": RK, "achieved": round(k2["gbs"], 1), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(k2["gbs"] / HBM_PEAK_GBS, 4),
                      "alg_bytes_per_launch": model[RK],
                      "bytes_model": "SURVEY §8(d) 3-pass model, z_chunk planes per launch"}
    step_model = 8 * (H * W + H * Pw + len(zs) * (3 * H * Pw + H * W))

    line = {
        "metric": METRIC, "value": round(value, 2), "unit": "propagations/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": args.cfg2_split, "vs_baseline": None, "dtype": "complex64 (fp32)",
        "data": "synthetic (Gaussian beam generated on device)",
        "config": {"workload": ("cfg2: ASM_prop 4096x4096 Gaussian_beam -> 64 z-planes/GPU (20-120 mm), "
                                if args.cfg2_split == "weak" else
                                "cfg2: ASM_prop 4096x4096 Gaussian_beam -> 64 z-planes (20-120 mm) split over the GPUs, ")
                               + "300 GHz, dx 0.25 mm, padding_scale 1 (P=8192), exact band limit",
                   "planes_per_step_per_gpu": len(zs), "N": N_FIELD, "P": 2 * N_FIELD,
                   "band_columns": ncols, "z_chunk": zc, "parallelism": f"z-shard x{world}"},
        "hbm_gbs_band_pruned": round(total_alg * args.steps / elapsed / 1e9 * world, 1),
        "hbm_gbs_survey_model": round(step_model * args.steps / elapsed / 1e9 * world, 1),
        "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                    for k, v in stats.items()},
        "roofline": roof,
        # every pass on the same footing (K2 and K3 trade places as the longer kernel box to box)
        "roofline_by_kernel": {k: round(v["gbs_pruned"] / HBM_PEAK_GBS, 4) for k, v in stats.items()},
        "roofline_step": roof_step,
        "roofline_survey_model": roof_model,
        "output_check": {"ok": checks_ok, "planes": checks},
    }
    if not args.headline_only:
        # secondary workloads never take the headline line down with them: an exception is reported
        # in the line, and a secondary still running after --secondary-timeout seconds (a hang, e.g.
        # in a collective) is reported as such by a watchdog that prints the line and ends every rank
        secondary = {}
        snapshot = [{}]
        secs = (("cfg3_czt", bench_czt), ("cfg4_qat", bench_qat),
                ("cfg4_dual_plane", lambda *a, **k: bench_qat_multi(*a, which="dual", **k)),
                ("cfg4_extended_dof", lambda *a, **k: bench_qat_multi(*a, which="edof", **k)),
                ("cfg5_donn", bench_donn))
        watchdog = _secondary_watchdog(line, [k for k, _ in secs], rank, args.secondary_timeout, snapshot)
        # the propagators' own diagnostics (the reference's critical-distance print) go to stderr:
        # stdout carries the one JSON line
        with contextlib.redirect_stdout(sys.stderr):
            for key, fn in secs:
                try:
                    res = fn(dev, rank, world, dist=ranks.dist)
                except Exception as e:  # noqa: BLE001 -- reported in the JSON line
                    res = {"error": f"{type(e).__name__}: {e}"[:300]}
                secondary[key] = res
                snapshot[0] = dict(secondary)  # one reference swap: the watchdog reads a finished copy
            if world == 1 and not args.no_shares:
                try:
                    res = per_rank_shares(dev, x, lam, sp)
                except Exception as e:  # noqa: BLE001 -- reported in the JSON line
                    res = {"error": f"{type(e).__name__}: {e}"[:300]}
                secondary["per_rank_share_n8"] = res
                snapshot[0] = dict(secondary)
            watchdog.cancel()
        line["secondary"] = secondary
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(args.cpu_budget, args.cpu_planes)
    if rank == 0:
        print(json.dumps(line), flush=True)
    ranks.close()
    failed = [] if checks_ok else [f"cfg2 headline: {checks}"]
    for key, sec in (line.get("secondary") or {}).items():
        if isinstance(sec, dict) and "error" in sec:  # reported in the line; only a wrong result fails the run
            sys.stderr.write(f"bench.py: {key} did not run: {sec['error']}\n")
    failed += _failed_checks(line.get("secondary"))
    if failed:
        sys.stderr.write("bench.py: output check FAILED:\n  " + "\n  ".join(failed) + "\n")
        sys.exit(3)


if __name__ == "__main__":
    main()
