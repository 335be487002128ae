"""Quantization-aware DOE layers -- drop-in for the reference's Components/QuantizedDOE.py.

Same class names, constructor arguments (``doe_params`` / ``optim_params`` dict keys and
defaults), parameter names and initialisers (so a seeded construction draws the same RNG
stream), temperature schedules, ``forward(field, iter_frac)`` -> new ElectricField,
``.height_map`` / ``._height_map_`` attributes, ``visualize`` and ``save``.

What runs where: the height-map quantizer of every layer (sigmoid parametrisation, LUT
straight-through, PSQ sigmoids, phase-score Gumbel-softmax, mirroring of the unit cell) is
one fused HIP kernel forward and one backward (``thz_quant_*``); the rotationally symmetric
layers' radial expansion is ``thz_radial_*``; the height noise, nearest upsampling,
transmission and field product of ``DOELayer.modulate`` are one pass (``thz_doe_modulate_*``).
torch only allocates and draws the random numbers, in the reference's order
(``exponential_`` of the Gumbel-softmax, then ``rand_like`` of the height noise), so a seeded
run replays the reference's RNG stream.

Documented differences (quirks of the reference that are not reproduced):
  * FixDOEElement stores its height map as float32 (the reference keeps a float64 numpy map
    as float64 and then returns complex128 fields); all layers compute in complex64.
"""
from __future__ import annotations

import math
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn

from quantizationawarethzdoe_amd import _lib
from quantizationawarethzdoe_amd import doe as _doe
from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
from quantizationawarethzdoe_amd.utils.units import mm

BASE_PLANE_THICKNESS = 2 * mm  # :23
LIGHT_SPEED = 2.998e8  # :25


def _copy_quad_to_full(quad_map):
    """Mirror a quadrant into the full map (:28-35); plain data movement on the device."""
    d0, d1 = (2, 3) if quad_map.dim() == 4 else (0, 1)
    half = torch.cat([torch.flip(quad_map, dims=[d0]), quad_map], dim=d0)
    return torch.cat([torch.flip(half, dims=[d1]), half], dim=d1)


def _phase_to_height_with_material_refractive_idx(_phase, _wavelength, _refractive_index):
    return _phase / (2 * torch.pi / _wavelength) / (_refractive_index - 1)  # :37-38


def _height_to_phase_with_material_refractive_idx(_height, _wavelength, _refractive_index):
    return 2 * torch.pi / _wavelength * (_refractive_index - 1) * _height  # :40-41


def _cos_tau(iter_frac, tau_min, tau_max):
    """Cosine temperature schedule of the Gumbel layers (:460-462, :869-871, :1050-1052)."""
    return tau_min + 0.5 * (tau_max - tau_min) * (1 + math.cos(iter_frac * math.pi))


def _linear_tau(iter_frac, tau_min, tau_max):
    """PSQ's linearly increasing temperature (:1219-1223)."""
    return tau_min + (tau_max - tau_min) * iter_frac


class _DeviceNoise:
    """Shape of a noise draw left to the kernel's counter-based generator (see _gumbel_noise)."""

    def __init__(self, shape):
        self.shape = shape


def _scalar(v):
    return float(v.detach().cpu()) if torch.is_tensor(v) else float(v)


class DOELayer(nn.Module):
    """Base of every DOE layer (:44-126)."""

    @staticmethod
    def phase_shift_according_to_height(height_map: torch.Tensor, wavelengths, epsilon, tand) -> torch.Tensor:
        """Transmission t_c(h) [C, H, W] complex64 (:47-79), evaluated by the modulate kernel."""
        h = height_map.reshape(height_map.shape[-2:]).float()
        wl = [_scalar(w) for w in torch.as_tensor(wavelengths).reshape(-1)]
        ones = torch.ones((1, len(wl)) + tuple(h.shape), dtype=torch.complex64, device=h.device)
        out, _ = _doe.modulate(ones, h, wl, _scalar(epsilon), _scalar(tand))
        return out[0]

    @staticmethod
    def add_height_map_noise(height_map, tolerance=None):
        """h + U(-1, 1) * tolerance (:82-87)."""
        if tolerance is not None:
            height_map = height_map + (torch.rand_like(height_map) - 0.5) * 2 * tolerance
        return height_map

    def build_height_map(self):
        return NotImplemented

    def _dyn_values(self, iter_frac):  # layers without a temperature schedule
        return 1.0, 0.0, 0.0

    def _graph_phase(self, iter_frac):
        return 0

    def modulate(self, input_field, preprocessed_height_map, height_tolerance, epsilon, tand) -> ElectricField:
        """Noise + nearest upsampling + transmission + product (:92-126).  The noise is drawn here (the
        reference's RNG order); the product is left pending on the returned field: a following
        ASM_prop forms it inside its row pass (one pipeline), any other reader of
        ``.data`` forms it with the modulate kernel."""
        h = preprocessed_height_map
        link = getattr(h, "_thz_quant", None)  # the quantizer that made h (doe.QuantLink), if any
        if h.dim() != 2:
            h = h.reshape(h.shape[-2:])
        tol = None if height_tolerance is None else self._host_scalar("tol", height_tolerance)
        data = input_field.data
        self._pending_mod = _doe.PendingModulation(data, h, input_field.wavelengths_host,
                                                   self._host_scalar("eps", epsilon), self._host_scalar("tand", tand),
                                                   tolerance=tol, rng=self._rng_spec(0), quant=link)
        out = ElectricField(data=data, wavelengths=input_field.wavelengths,
                            spacing=input_field.spacing)._adopt_host(input_field)
        out._pending = self._pending_mod
        return out

    @property
    def _height_map_(self):
        """The noisy, upsampled height map of the last forward (DOELayer.modulate :102-107)."""
        pend = self.__dict__.get("_pending_mod")
        if pend is None:
            return None
        if pend.hfull is None:
            pend.run()
        return pend.hfull

    # -- shared helpers ------------------------------------------------------------------------
    def _host_scalar(self, key, v):
        """Host value of a (device) scalar, cached per object so a training step does not sync."""
        cache = self.__dict__.setdefault("_host_cache", {})
        hit = cache.get(key)
        if hit is not None and hit[0] is v:
            return hit[1]
        val = _scalar(v)
        cache[key] = (v, val)
        return val

    def _read_doe_params(self, doe_params, device):
        self.device = device if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.doe_size = doe_params.get('doe_size', None)
        self.doe_dxy = doe_params.get('doe_dxy', None)
        self.num_unit = doe_params.get('num_unit', None)
        self.height_constraint_max = torch.tensor(doe_params.get('height_constraint_max', 2 * mm), device=self.device)
        self.tolerance = doe_params.get('tolerance', 0.05 * mm)
        self.material = torch.tensor(doe_params.get('material', None), device=self.device)
        self.epsilon = self.material[0]
        self.tand = self.material[1]
        self._hmax = _scalar(self.height_constraint_max)
        self._eps = _scalar(self.epsilon)

    def look_up_table(self, look_up_table):
        """Manufacturable heights: linspace(0, h_max, L+1)[:-1] or the given list (:374-391)."""
        if look_up_table is None:
            lut = torch.linspace(0, self.height_constraint_max.cpu(), self.doe_level + 1)
            self.lut = lut[:-1].to(self.device)
        else:
            self.lut = torch.tensor(look_up_table, dtype=torch.float32).to(self.device)
            self.doe_level = len(self.lut)
        self._lut_host = [float(v) for v in self.lut.detach().cpu()]

    def _lut_values(self):
        lut = getattr(self, "_lut_host", None)
        if lut is None:  # PSQ / FP never build a LUT (:1068-1100); the kernel only needs L there
            L = getattr(self, "doe_level", 2)
            lut = [self._hmax * i / L for i in range(L)]
        return lut

    def _quantize(self, kind, weight, mirror, clamp, expo=None, **kw):
        # _dyn: device (tau, s, beta) installed by a graph-capturing trainer (qat.QATTrainer)
        if isinstance(expo, _DeviceNoise):  # the Exp(1) draw made in the kernel
            return _doe.quantize(kind, weight, self._lut_values(), self._hmax, clamp=clamp, mirror=mirror, expo=None,
                                 dyn=self.__dict__.get("_dyn"), rng=self._rng_spec(1), expo_shape=expo.shape, **kw)
        return _doe.quantize(kind, weight, self._lut_values(), self._hmax, clamp=clamp, mirror=mirror, expo=expo,
                             dyn=self.__dict__.get("_dyn"), **kw)

    def _gumbel_noise(self, shape, like):
        """The Exp(1) draw F.gumbel_softmax makes (torch.empty_like(logits).exponential_()); with a
        trainer's device generator installed (_rng), a marker: the quantizer kernel draws it."""
        if self.__dict__.get("_rng") is not None:
            return _DeviceNoise(tuple(shape))
        return torch.empty(shape, dtype=torch.float32, device=like.device).exponential_()

    def _rng_spec(self, k):
        """(device [seed, step], stream) of this layer's draw k (0 height noise, 1 Gumbel) or None.
        Installed by a graph-capturing trainer with device_rng (qat.QATTrainer, donn.DONNTrainer)."""
        r = self.__dict__.get("_rng")
        return None if r is None else (r[0], r[1] + k)

    def _score_kw(self, wavelengths, tau):
        if getattr(self, "_wl_hint_src", None) is wavelengths:
            values = self._wl_hint  # the field's host mirror: no device->host copy per step
        else:
            values = _wavelength_values(wavelengths)
        lam_min = min(float(np.float32(w)) for w in values)
        return dict(tau=tau, c_s=self.c_s, s=self.tau_max / tau, phase_scale=_doe.phase_scale(lam_min, self._eps))

    def _radial(self, profile):
        return _doe.radial_map(profile, self.doe_size[0], self.doe_size[1])

    def score_phase(self, phase, lut, s=5.0, func='sigmoid'):
        """Phase-distance scores (:411-434); a torch helper kept for API parity (the layers'
        forward uses the fused kernel)."""
        wrapped_phase = (phase + torch.pi) % (2 * torch.pi) - torch.pi
        lut = (lut[None, :, None, None] + torch.pi) % (2 * torch.pi) - torch.pi
        diff = (wrapped_phase - lut + torch.pi) % (2 * torch.pi) - torch.pi
        diff = diff / torch.pi
        if func == 'sigmoid':
            z = s * diff
            return torch.sigmoid(z) * (1 - torch.sigmoid(z)) * 4
        if func == 'log':
            return -torch.log(diff.abs() + 1e-20) * s
        if func == 'poly':
            return 1 - torch.abs(diff) ** s
        if func == 'sine':
            return torch.cos(torch.pi * (s * diff).clamp(-1., 1.))
        if func == 'chirp':
            return 1 - torch.cos(torch.pi * (1 - diff.abs()) ** s)
        raise ValueError(f"unknown score function {func}")

    def _thickness(self, crop_size):
        thickness = self.height_map.squeeze(0, 1).detach().cpu().numpy() if self.height_map.dim() > 2 \
            else self.height_map.detach().cpu().numpy()
        if crop_size:
            H, W = thickness.shape
            top = int(round(H - crop_size[0]) / 2.0)
            left = int(round(W - crop_size[1]) / 2.0)
            thickness = thickness[top:top + crop_size[0], left:left + crop_size[1]]
        return thickness

    def visualize(self, cmap='viridis', figsize=(4, 4), crop_size=None):
        """Plot the height map (:210-251)."""
        import matplotlib.pyplot as plt
        from quantizationawarethzdoe_amd.utils.Visualization_Helper import add_colorbar, float_to_unit_identifier

        thickness = self._thickness(crop_size)
        size_x = np.array(self.doe_dxy * thickness.shape[0] / 2)
        size_y = np.array(self.doe_dxy * thickness.shape[1] / 2)
        unit_val, unit_axis = float_to_unit_identifier(max(size_x, size_y))
        size_x, size_y = size_x / unit_val, size_y / unit_val
        if figsize is not None:
            plt.figure(figsize=figsize)
        plt.subplot(1, 1, 1)
        im = plt.imshow(thickness, cmap=cmap, extent=[-size_x, size_x, -size_y, size_y])
        plt.title('2D Height Map of DOE')
        plt.xlabel("Position (" + unit_axis + ")")
        plt.ylabel("Position (" + unit_axis + ")")
        add_colorbar(im)
        plt.tight_layout()
        plt.show()

    def save(self, crop_size):
        """Write height_map_<date>.npy with {'thickness', 'dxy'} (:253-267)."""
        height_map = {'thickness': self._thickness(crop_size), 'dxy': np.array(self.doe_dxy)}
        np.save(f"height_map_{datetime.now().strftime('%Y%m%d-%H%M%S')}.npy", height_map)


def _wavelength_values(wavelengths):
    if torch.is_tensor(wavelengths):
        return [float(v) for v in wavelengths.detach().reshape(-1).cpu()]
    return [float(v) for v in np.atleast_1d(wavelengths)]


class FixDOEElement(DOELayer):
    """A fixed (trained or imported) height map (:129-178)."""

    def __init__(self, height_map, tolerance: float = 0.1 * mm, material: list = None,
                 device: torch.device = None) -> None:
        super().__init__()
        self.device = device if device is not None else torch.device("cuda" if torch.cuda.is_available() else "cpu")
        h = height_map.detach().clone() if torch.is_tensor(height_map) else torch.tensor(np.asarray(height_map))
        self.height_map = nn.parameter.Parameter(h.to(device=self.device, dtype=torch.float32))
        self.tolerance = torch.tensor(tolerance, device=self.device)
        self.material = torch.tensor(material, device=self.device)
        self.epsilon = self.material[0]
        self.tand = self.material[1]

    def visualize(self, cmap='viridis', figsize=(4, 4)):
        import matplotlib.pyplot as plt
        from quantizationawarethzdoe_amd.utils.Visualization_Helper import add_colorbar

        if figsize is not None:
            plt.figure(figsize=figsize)
        plt.subplot(1, 1, 1)
        im = plt.imshow(self.height_map.detach().cpu().numpy(), cmap=cmap)
        plt.title('2D Height Map of DOE')
        plt.xlabel('X')
        plt.ylabel('Y')
        add_colorbar(im)
        plt.tight_layout()
        plt.show()

    def forward(self, field: ElectricField) -> ElectricField:
        return self.modulate(field, self.height_map, self.tolerance, self.epsilon, self.tand)


class FullPrecisionDOELayer(DOELayer):
    """h = h_max * sigmoid(clamp(w, -8, 8)) (:181-300)."""

    def __init__(self, doe_params: dict, device: torch.device = None) -> None:
        super().__init__()
        self._read_doe_params(doe_params, device)
        self.build_weight_height_map()

    def build_weight_height_map(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (1, 1, height, width)
        else:
            size = (1, 1, int(height / self.num_unit), int(width / self.num_unit))
        self.weight_height_map = nn.parameter.Parameter(-torch.pi + 2 * torch.pi * torch.rand(*size, device=self.device),
                                                        requires_grad=True)

    def preprocessed_height_map(self):
        self.height_map = self._quantize(_lib.Q_FP, self.weight_height_map, self.num_unit is not None, 8.0)
        return self.height_map

    def forward(self, field: ElectricField, iter_frac=None) -> ElectricField:
        return self.modulate(field, self.preprocessed_height_map(), self.tolerance, self.epsilon, self.tand)


class _ScoreGumbelBase(DOELayer):
    def __init__(self, doe_params: dict, optim_params: dict, device: torch.device = None):
        super().__init__()
        self._read_doe_params(doe_params, device)
        self.doe_level = doe_params.get('doe_level', 6)
        self.c_s = optim_params.get('c_s', 300)
        self.tau_max = optim_params.get('tau_max', 5.5)
        self.tau_min = optim_params.get('tau_min', 2.0)
        self.look_up_table(doe_params.get('look_up_table', None))
        self.build_init_phase()

    def forward(self, field: ElectricField, iter_frac=None) -> ElectricField:
        tau = _cos_tau(iter_frac, self.tau_min, self.tau_max) if iter_frac is not None else None
        self._wl_hint, self._wl_hint_src = field.wavelengths_host, field.wavelengths
        hm = self.preprocessed_height_map(wavelengths=field.wavelengths, tau=tau, iter_frac=iter_frac)
        return self.modulate(field, hm, self.tolerance, self.epsilon, self.tand)

    # -- graph replay support (qat.QATTrainer(graph=True)) -------------------------------------
    def _dyn_values(self, iter_frac):
        """(tau, s, beta) the quantizer kernels read from device memory at this schedule point."""
        tau = _cos_tau(iter_frac, self.tau_min, self.tau_max)
        beta = 0.0
        if 0.3 < iter_frac <= 0.8:
            beta = iter_frac if getattr(self, "_blend_by_iter_frac", False) else (iter_frac - 0.3) / (0.8 - 0.3)
        return tau, self.tau_max / tau, beta

    def _graph_phase(self, iter_frac):
        """Schedule phases with different op sequences (each gets its own captured graph)."""
        return 0 if iter_frac <= 0.3 else (1 if iter_frac <= 0.8 else 2)


class SoftGumbelQuantizedDOELayer(_ScoreGumbelBase):
    """v1: the weight is a phase in [-pi, pi); scores against the LUT phases, Gumbel pick (:303-475)."""

    def _graph_phase(self, iter_frac):
        return 0

    def build_init_phase(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (1, 1, height, width)
        else:
            size = (1, 1, int(height / self.num_unit), int(width / self.num_unit))
        self.init_phase = nn.parameter.Parameter(-torch.pi + 2 * torch.pi * torch.rand(*size, device=self.device),
                                                 requires_grad=True)

    def preprocessed_height_map(self, wavelengths, tau, iter_frac=None):
        height, width = self.doe_size[0], self.doe_size[1]
        w = self.init_phase
        expo = self._gumbel_noise((1, self.doe_level) + tuple(w.shape[-2:]), w)
        hm = self._quantize(_lib.Q_SGV1, w, False, 0.0, expo, **self._score_kw(wavelengths, tau))
        if self.num_unit is None:
            self.height_map = hm
        else:
            # the reference tiles by shape[0] / shape[1] of the 4-D unit map, i.e. by (height, width) (:450-454)
            self.height_map = _copy_quad_to_full(hm).repeat(int(height / 1), int(width / 1))
        return self.height_map


class SoftGumbelQuantizedDOELayerv2(_ScoreGumbelBase):
    """v2: sigmoid height, quantized by score-Gumbel once iter_frac > 0.5 (:478-656)."""

    def _graph_phase(self, iter_frac):
        return int(iter_frac > 0.5)

    def build_init_phase(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            self.weight_init_phase = nn.parameter.Parameter(torch.randn(height, width, device=self.device),
                                                            requires_grad=True)
        else:
            unit = (int(height / self.num_unit), int(width / self.num_unit))
            self.init_phase = nn.parameter.Parameter(
                -torch.pi + 2 * torch.pi * torch.rand(1, 1, unit[0], unit[1], device=self.device), requires_grad=True)

    def preprocessed_height_map(self, wavelengths, tau, iter_frac=None):
        if self.num_unit is not None:  # the reference reads an attribute it never set (:629)
            raise AttributeError("SoftGumbelQuantizedDOELayerv2 with num_unit has no height_map (reference :629)")
        w = self.weight_init_phase
        quant = iter_frac > 0.5
        expo = self._gumbel_noise((1, self.doe_level) + tuple(w.shape[-2:]), w) if quant else None
        kw = self._score_kw(wavelengths, tau)
        self.height_map = self._quantize(_lib.Q_SGV3, w, False, 10.0, expo, iter_frac=1.0 if quant else 0.0, **kw)
        return self.height_map


class SoftGumbelQuantizedDOELayerv3(_ScoreGumbelBase):
    """v3, the paper's method: sigmoid height -> blend -> score-Gumbel quantization (:660-890)."""

    _blend_by_iter_frac = False

    def build_init_phase(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (height, width)
        else:
            size = (int(height / self.num_unit), int(width / self.num_unit))
        self.weight_init_phase = nn.parameter.Parameter(torch.randn(*size, device=self.device), requires_grad=True)

    def _v3_height(self, w, wavelengths, tau, iter_frac, mirror, shape):
        # schedule phase decided in double precision as in the reference (:826, :839)
        if iter_frac > 0.8:
            mode, beta = 1.0, 1.0
        elif iter_frac > 0.3:
            mode = 0.5
            beta = iter_frac if self._blend_by_iter_frac else (iter_frac - 0.3) / (0.8 - 0.3)
        else:
            mode, beta = 0.0, 0.0
        expo = self._gumbel_noise(shape, w) if mode > 0 else None
        kw = self._score_kw(wavelengths, tau) if mode > 0 else dict(tau=1.0)
        return self._quantize(_lib.Q_SGV3, w, mirror, 10.0, expo, iter_frac=mode, beta=beta, **kw)

    def preprocessed_height_map(self, wavelengths, tau, iter_frac=None):
        w = self.weight_init_phase
        self.height_map = self._v3_height(w, wavelengths, tau, iter_frac, self.num_unit is not None,
                                          (1, self.doe_level) + tuple(w.shape[-2:]))
        return self.height_map


class NaiveGumbelQuantizedDOELayer(_ScoreGumbelBase):
    """Gumbel-softmax over free [h, w, L] logits (:892-1065)."""

    def build_init_phase(self):
        self.build_init_logits()

    def build_init_logits(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (height, width, self.doe_level)
        else:
            size = (int(height / self.num_unit), int(width / self.num_unit), self.doe_level)
        self.weight_height_map = nn.parameter.Parameter(torch.rand(*size, device=self.device), requires_grad=True)

    def _ngs(self, tau, mirror):
        w = self.weight_height_map
        expo = self._gumbel_noise(tuple(w.shape), w)
        return self._quantize(_lib.Q_NGS, w, mirror, 0.0, expo, tau=1.0 if tau is None else tau)

    def preprocessed_height_map(self, tau):
        self.height_map = self._ngs(tau, self.num_unit is not None)
        return self.height_map

    def forward(self, field: ElectricField, iter_frac=None) -> ElectricField:
        tau = _cos_tau(iter_frac, self.tau_min, self.tau_max) if iter_frac is not None else None
        return self.modulate(field, self.preprocessed_height_map(tau=tau), self.tolerance, self.epsilon, self.tand)

    def _dyn_values(self, iter_frac):
        return _cos_tau(iter_frac, self.tau_min, self.tau_max), 0.0, 0.0

    def _graph_phase(self, iter_frac):
        return 0


class PSQuantizedDOELayer(DOELayer):
    """Progressive sigmoid quantization: sum of L-1 tempered sigmoids (:1068-1236)."""

    def __init__(self, doe_params: dict, optim_params: dict, device: torch.device = None):
        super().__init__()
        self._read_doe_params(doe_params, device)
        self.doe_level = doe_params.get('doe_level', 6)
        self.tau_max = optim_params.get('tau_max', 400)
        self.tau_min = optim_params.get('tau_min', 1)
        self.build_weight_height_map()

    def build_weight_height_map(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (height, width)
        else:
            unit = int(height / self.num_unit)
            size = (unit, unit)  # the reference uses unit_size[0] twice (:1191)
        self.weight_height_map = nn.parameter.Parameter(torch.randn(*size, device=self.device), requires_grad=True)

    def _psq(self, tau, mirror):
        if tau is None:
            raise TypeError("PSQuantizedDOELayer needs iter_frac (the reference multiplies None, :1206)")
        self.height_constraint_min = 0
        return self._quantize(_lib.Q_PSQ, self.weight_height_map, mirror, 8.0, tau=tau)

    def preprocessed_height_map(self, tau):
        self.height_map = self._psq(tau, self.num_unit is not None)
        return self.height_map

    def forward(self, field: ElectricField, iter_frac=None) -> ElectricField:
        tau = _linear_tau(iter_frac, self.tau_min, self.tau_max) if iter_frac is not None else None
        return self.modulate(field, self.preprocessed_height_map(tau=tau), self.tolerance, self.epsilon, self.tand)

    def _dyn_values(self, iter_frac):
        return _linear_tau(iter_frac, self.tau_min, self.tau_max), 0.0, 0.0

    def _graph_phase(self, iter_frac):
        return 0


class STEQuantizationFunction(torch.autograd.Function):
    """Nearest LUT level forward, identity backward (:1239-1253)."""

    @staticmethod
    def forward(ctx, input, lut):
        idx = torch.argmin(torch.abs(input.unsqueeze(-1) - lut), dim=-1)
        return lut[idx]

    @staticmethod
    def backward(ctx, grad_output):
        return grad_output.clone(), None


ste_quan = STEQuantizationFunction.apply


class STEQuantizedDOELayer(DOELayer):
    """Sigmoid height snapped to the nearest LUT level, straight-through gradient (:1257-1396)."""

    def __init__(self, doe_params: dict, optim_params: dict, device: torch.device = None):
        super().__init__()
        self._read_doe_params(doe_params, device)
        self.doe_level = doe_params.get('doe_level', 6)
        self.build_weight_height_map()
        self.look_up_table(doe_params.get('look_up_table', None))

    def build_weight_height_map(self):
        height, width = self.doe_size[0], self.doe_size[1]
        if self.num_unit is None:
            size = (1, 1, height, width)
        else:
            unit = int(height / self.num_unit)
            size = (1, 1, unit, unit)  # unit_size[0] twice, as the reference (:1377)
        self.weight_height_map = nn.parameter.Parameter(torch.randn(*size, device=self.device), requires_grad=True)

    def preprocessed_height_map(self):
        self.height_map = self._quantize(_lib.Q_STE, self.weight_height_map, self.num_unit is not None, 8.0)
        return self.height_map

    def forward(self, field: ElectricField, iter_frac=None) -> ElectricField:
        return self.modulate(field, self.preprocessed_height_map(), self.tolerance, self.epsilon, self.tand)


# ---------------------------------------------------------------------------------------------
# rotationally symmetric variants (:1399-1623): a radial profile of R = int(H sqrt(2) / 2) bins
# ---------------------------------------------------------------------------------------------
def _radius(height):
    return int(height * torch.sqrt(torch.tensor(2)) / 2)


class RotationallySymmetricFullPrecisionDOELayer(FullPrecisionDOELayer):
    def build_weight_height_map(self):
        self.height_map_shape = _radius(self.doe_size[0])
        self.weight_height_map = nn.parameter.Parameter(
            -torch.pi + 2 * torch.pi * torch.rand(self.height_map_shape, device=self.device), requires_grad=True)

    def preprocessed_height_map(self):
        prof = self._quantize(_lib.Q_FP, self.weight_height_map, False, 8.0)
        self.height_map = self._radial(prof)
        return self.height_map


class RotationallySymmetricScoreGumbelSoftQuantizedDOELayer(SoftGumbelQuantizedDOELayerv3):
    _blend_by_iter_frac = True  # the reference blends with iter_frac, not beta (:1458)

    def build_init_phase(self):
        self.height_map_shape = _radius(self.doe_size[0])
        self.weight_init_phase = nn.parameter.Parameter(
            torch.randn(1, 1, 1, self.height_map_shape, device=self.device), requires_grad=True)

    def preprocessed_height_map(self, wavelengths, tau, iter_frac=None):
        R = self.height_map_shape
        prof = self._v3_height(self.weight_init_phase.reshape(1, R), wavelengths, tau, iter_frac, False,
                               (1, self.doe_level, 1, R))
        self.height_map = self._radial(prof)
        return self.height_map


class RotationallySymmetricSTEQuantizedDOELayer(STEQuantizedDOELayer):
    def build_weight_height_map(self):
        self.height_map_shape = _radius(self.doe_size[0])
        self.weight_height_map = nn.parameter.Parameter(
            -torch.pi + 2 * torch.pi * torch.rand(1, self.height_map_shape, device=self.device), requires_grad=True)

    def preprocessed_height_map(self):
        prof = self._quantize(_lib.Q_STE, self.weight_height_map, False, 8.0)
        self.height_map = self._radial(prof)
        return self.height_map


class RotationallySymmetricNaiveGumbelQuantizedDOELayer(NaiveGumbelQuantizedDOELayer):
    def build_init_logits(self):
        self.height_map_shape = _radius(self.doe_size[0])
        self.weight_height_map = nn.parameter.Parameter(
            torch.rand(1, self.height_map_shape, self.doe_level, device=self.device), requires_grad=True)

    def preprocessed_height_map(self, tau):
        self.height_map = self._radial(self._ngs(tau, False))
        return self.height_map


class RotationallySymmetricPSQuantizedQuantizedDOELayer(PSQuantizedDOELayer):
    def build_weight_height_map(self):
        self.height_map_shape = _radius(self.doe_size[0])
        self.weight_height_map = nn.parameter.Parameter(torch.rand(1, self.height_map_shape, device=self.device),
                                                        requires_grad=True)

    def preprocessed_height_map(self, tau):
        self.height_map = self._radial(self._psq(tau, False))
        return self.height_map
