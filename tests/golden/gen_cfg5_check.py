#!/usr/bin/env python3
"""Generate tests/golden/cfg5_check.npz: the REFERENCE's own loss and weight gradients for one cfg5
DONN training step at the bench's batch (256 samples of 100^2, FullPrecision layers, ASM P = 300,
80 mm apertures; experiment_DONN_3_layers.ipynb cells 1-3), in fp64 by the SURVEY.md §8(c)
procedure and in fp32 as shipped, for the notebook forward (every layer modulates the encoded
input, nb :194) and the chained one.

The step's loss is the reference's QAT loss, MSE(normalize(|E|^2), target)
(experiment_four_focal_spots.ipynb:336-370, utils/Helper_Functions.py:185-193), against the
per-sample detector target of each label (quantizationawarethzdoe_amd.donn.detector_targets: the
notebook's training cells are empty).  Every module on the path -- ElectricField, ASM_prop,
ApertureElement, FullPrecisionDOELayer and normalize -- is the reference's own; the three layers'
height-noise draws (tolerance 30 um, rand_like) are seeded planes injected in order, and stored.

bench.py's cfg5 line runs the same step through the HIP kernels outside its timed region and
compares against this file; tests/test_donn_train_gpu.py does too.

Runs only in the build container (imports /root/reference through ``_refimport``)::

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_cfg5_check.py
"""
import contextlib
import io
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
from _refimport import import_reference  # noqa: E402

from bench import cfg5_inputs  # noqa: E402  (the batch, labels, weights and noise the check replays)
from quantizationawarethzdoe_amd.donn import detector_targets  # noqa: E402

C0 = 2.998e8
MM = 1e-3
DOE_PARAMS = dict(doe_size=[100, 100], doe_dxy=1 * MM, doe_level=4, look_up_table=None, num_unit=None,
                  height_constraint_max=1 * MM, tolerance=30e-6, material=[2.66, 0.003])


def step(ref, AP, u, target, weights, noises, chained, f64):
    dt = torch.float64 if f64 else torch.float32
    old = torch.get_default_dtype()
    torch.set_default_dtype(dt)
    orig = torch.rand_like
    it = iter(noises)
    torch.rand_like = lambda t, *a, **k: next(it).to(dtype=t.dtype)
    try:
        does = [ref.DOE.FullPrecisionDOELayer(DOE_PARAMS, device="cpu") for _ in range(3)]
        for d, w in zip(does, weights):
            d.weight_height_map = torch.nn.Parameter(w.to(dt).clone())
        asm50 = ref.ASM.ASM_prop(z_distance=50 * MM, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True,
                                 device="cpu")
        asm20 = ref.ASM.ASM_prop(z_distance=20 * MM, bandlimit_type='exact', padding_scale=2, bandlimit_kernel=True,
                                 device="cpu")
        ap = AP.ApertureElement(aperture_type='rect', aperture_size=0.08)
        amp = (torch.ones(1, 1, 100, 100) * u.to(dt)).to(torch.complex128 if f64 else torch.complex64)
        field0 = ref.ElectricField(data=amp, wavelengths=C0 / 300e9, spacing=1 * MM, device="cpu")
        if f64:
            field0._wavelengths = field0._wavelengths.double()
            field0._spacing = field0._spacing.double()
        with contextlib.redirect_stdout(io.StringIO()):
            inputs = ap(asm50(field0))
            field = inputs
            for i in range(2):
                field = ap(asm20(does[i](field if chained else inputs, None)))
            out = asm50(does[2](field if chained else inputs, None))
        amp2 = ref.HF.normalize(torch.abs(out.data) ** 2)
        loss = torch.nn.MSELoss()(amp2, target.to(dt))
        loss.backward()
        grads = [(d.weight_height_map.grad if d.weight_height_map.grad is not None
                  else torch.zeros_like(d.weight_height_map)).detach().double().numpy() for d in does]
        assert next(it, None) is None, "not every injected draw was consumed"
        return float(loss.detach()), grads
    finally:
        torch.rand_like = orig
        torch.set_default_dtype(old)


def main():
    ref = import_reference()
    AP = ref.import_module("Components.Aperture")
    torch.set_num_threads(8)
    u, labels, weights, noises = cfg5_inputs()
    target = detector_targets(device="cpu").index_select(0, labels)
    arrays = {}
    for chained in (False, True):
        mode = "chained" if chained else "notebook"
        for f64 in (True, False):
            tag = "64" if f64 else "32"
            loss, grads = step(ref, AP, u, target, weights, noises, chained, f64)
            arrays[f"{mode}__loss{tag}"] = np.float64(loss)
            for i, g in enumerate(grads):
                arrays[f"{mode}__g{i}_{tag}"] = g
            print(f"{mode} fp{tag}: loss {loss:.9e}, |g2| {np.linalg.norm(grads[2]):.6e}", flush=True)
        for i in range(3):
            a, b = arrays[f"{mode}__g{i}_32"], arrays[f"{mode}__g{i}_64"]
            nb = np.linalg.norm(b)
            print(f"  {mode} layer {i}: reference fp32 vs fp64 grad rel-L2 "
                  f"{np.linalg.norm(a - b) / nb if nb else 0.0:.2e}")
    np.savez_compressed(os.path.join(HERE, "cfg5_check.npz"), **arrays)


if __name__ == "__main__":
    main()
