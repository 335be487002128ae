"""Three-layer diffractive optical neural network (cfg5) -- the model of
experiment_DONN_3_layers.ipynb (cells 1-3), on the HIP propagator / DOE kernels.

``DONN(input_dxy, input_field_shape, doe_params, optim_params, wavelengths, num_layer, d_layer,
q_method)`` keeps the notebook's constructor and ``forward(u, iter_frac)``:
encode (plane wave x u) -> ASM 50 mm -> 80 mm aperture, then per layer DOE -> ASM d_layer ->
aperture, last DOE -> ASM 50 mm to the detector.  The notebook's forward modulates the
encoded INPUT in every layer (``self.does[i](inputs, ...)``, nb :194), so only the last layer
reaches the detector; that is the default here.  ``chained=True``
runs the physically chained network instead (each layer modulates the previous output).
Documented difference: ``q_method='ste'`` works here (the notebook's ``n.ModuleList`` typo
raises NameError).

Data-parallel training: each rank runs its share of the batch and
``qat.GradientAllReduce`` averages the three layers' gradients in one flat all-reduce.
"""
from __future__ import annotations

import gzip
import os

import numpy as np
import torch
import torch.nn as nn

from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
from quantizationawarethzdoe_amd.Components.Aperture import ApertureElement
from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
from quantizationawarethzdoe_amd.utils.units import mm, um

C0 = 2.998e8


def default_params():
    """doe_params / optim_params of the notebook (cell 1)."""
    doe_params = {
        'doe_size': [100, 100], 'doe_dxy': 1 * mm, 'doe_level': 4, 'look_up_table': None, 'num_unit': None,
        'height_constraint_max': 1 * mm, 'tolerance': 30 * um, 'material': [2.66, 0.003],
    }
    optim_params = {'c_s': 100, 'tau_max': 2.5, 'tau_min': 1.5}
    return doe_params, optim_params


class DONN(nn.Module):
    def __init__(self, input_dxy=1 * mm, input_field_shape=(100, 100), doe_params=None, optim_params=None,
                 wavelengths=C0 / 300e9, num_layer=3, d_layer=20 * mm, q_method=None, device=None):
        super().__init__()
        dp, op = default_params()
        self.input_dxy = input_dxy
        self.input_field_shape = list(input_field_shape)
        self.doe_params = doe_params or dp
        self.optim_params = optim_params or op
        self.wavelengths = wavelengths
        self.num_layer = num_layer
        self.d_layer = d_layer
        self.device = device or torch.device('cuda:0' if torch.cuda.is_available() else 'cpu')
        dev = self.device
        self.asm_prop2layer = ASM_prop(z_distance=50 * mm, bandlimit_type='exact', padding_scale=2,
                                       bandlimit_kernel=True, device=dev)
        self.aperture = ApertureElement(aperture_type='rect', aperture_size=0.08)
        if q_method is None:
            make = lambda: Q.FullPrecisionDOELayer(self.doe_params, device=dev)  # noqa: E731
        elif q_method == 'sgs':
            make = lambda: Q.SoftGumbelQuantizedDOELayerv3(self.doe_params, self.optim_params, device=dev)  # noqa
        elif q_method == 'gs':
            make = lambda: Q.NaiveGumbelQuantizedDOELayer(self.doe_params, self.optim_params, device=dev)  # noqa
        elif q_method == 'psq':
            psq = {'c_s': 300, 'tau_max': 800, 'tau_min': 1}
            make = lambda: Q.PSQuantizedDOELayer(self.doe_params, psq, device=dev)  # noqa: E731
        elif q_method == 'ste':
            make = lambda: Q.STEQuantizedDOELayer(self.doe_params, self.optim_params, device=dev)  # noqa
        else:
            raise ValueError(f"unknown q_method {q_method!r}")
        self.does = nn.ModuleList([make() for _ in range(self.num_layer)])
        self.asm_prop_layer = ASM_prop(z_distance=self.d_layer, bandlimit_type='exact', padding_scale=2,
                                       bandlimit_kernel=True, device=dev)
        self.asm_prop2detector = ASM_prop(z_distance=50 * mm, bandlimit_type='exact', padding_scale=2,
                                          bandlimit_kernel=True, device=dev)

    def encode_object(self, u):
        """Plane wave times the object amplitude ``u`` [B, 1, H, W] -> ASM 50 mm -> aperture (nb :171-190)."""
        u = u.to(self.device)
        field = ElectricField(data=u.to(torch.complex64), wavelengths=self.wavelengths, spacing=self.input_dxy,
                              device=self.device)
        return self.aperture(self.asm_prop2layer(field))

    def forward(self, u, iter_frac=None, chained=False):
        inputs = self.encode_object(u)
        field = inputs
        for i in range(self.num_layer - 1):
            field = self.does[i](field if chained else inputs, iter_frac)
            field = self.asm_prop_layer(field)
            field = self.aperture(field)
        field = self.does[-1](field if chained else inputs, iter_frac)
        return self.asm_prop2detector(field)


def read_idx_images(path, count=None):
    """MNIST idx3 images (optionally gzip) -> uint8 [N, 28, 28]; the local t10k file, no download."""
    opener = gzip.open if path.endswith(".gz") else open
    with opener(path, "rb") as fh:
        data = fh.read()
    magic, n, h, w = (int.from_bytes(data[i:i + 4], "big") for i in range(0, 16, 4))
    if magic != 2051:
        raise ValueError(f"{path}: not an idx3 image file")
    n = n if count is None else min(n, count)
    return np.frombuffer(data, dtype=np.uint8, count=n * h * w, offset=16).reshape(n, h, w)


def to_field_batch(images, shape=(100, 100)):
    """uint8 digits -> [B, 1, H, W] float in [0, 1], bilinearly resized (the notebook's
    Resize + ToTensor, with torch's interpolate standing in for torchvision)."""
    x = torch.from_numpy(np.asarray(images, dtype=np.float32) / 255.0)[:, None]
    return torch.nn.functional.interpolate(x, size=list(shape), mode="bilinear", align_corners=False,
                                           antialias=True)
