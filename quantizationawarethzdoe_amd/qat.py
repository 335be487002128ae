"""Quantization-aware training loop of the four-focal-spots DOE (cfg4) and its data-parallel form.

The system is the reference notebook's (experiment_four_focal_spots.ipynb, cells 1-6):
Gaussian source (BeamWaistCorruagtedTK waist) -> ASM 127 mm (padding 2, exact band limit)
-> thin lens f = 127 mm -> 80 mm square aperture -> score-Gumbel DOE (v3) -> ASM 200 mm ->
loss = MSE(normalize(|E|^2), nine-spot target), Adam lr 0.02, iter_frac = itr / max_itrs.

MI355X mapping
  * every stage is a HIP kernel of libthzdoe (source, lens and aperture once at construction;
    per step: fused quantizer, fused modulate, the 3-pass ASM and its adjoint, the fused
    |E|^2 -> normalize -> MSE forward/backward);
  * data parallel: the DOE weight is replicated, each rank evaluates the
    loss on its own noise sample (Gumbel + fabrication tolerance, generator seeded
    base + rank) and the weight gradients are averaged by ONE flat all-reduce (RCCL over
    xGMI on the GPU, gloo in the CPU tests) before the optimiser step -- an N-sample
    estimator per step.
"""
from __future__ import annotations

import contextlib
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from quantizationawarethzdoe_amd import optics as _optics
from quantizationawarethzdoe_amd import propagation as _prop
from quantizationawarethzdoe_amd.Components import QuantizedDOE as Q
from quantizationawarethzdoe_amd.Components.Aperture import ApertureElement
from quantizationawarethzdoe_amd.Components.Thin_Lens import Thin_LensElement
from quantizationawarethzdoe_amd.LightSource.Gaussian_beam import Guassian_beam
from quantizationawarethzdoe_amd.Props.ASM_Prop import ASM_prop
from quantizationawarethzdoe_amd.utils.Helper_Functions import normalize
from quantizationawarethzdoe_amd.utils.units import m, mm, um

# Graph captures restrict unsafe HIP calls to the capturing thread only.  Under the default
# ("global") mode, ProcessGroupNCCL's watchdog thread polling its work events while a step is being
# captured gets hipErrorStreamCaptureUnsupported and aborts the process (seen once in the -m gpu
# suite, tests/test_collective_capture_gpu.py, one-rank RCCL group).  Captured collectives do not
# enqueue watchdog work, so the watchdog only ever polls eager work outside the graph.
_CAPTURE_MODE = "thread_local"

C0 = 2.998e8
FOCI_MM = [(-20, -20), (20, 20), (-20, 20), (20, -20), (0, 0), (0, -20), (-20, 0), (0, 20), (20, 0)]


def default_params():
    """doe_params / optim_params of the notebook (cell 1)."""
    doe_params = {
        'doe_size': [100, 100], 'doe_dxy': 1 * mm, 'doe_level': 4, 'look_up_table': None, 'num_unit': 2,
        'height_constraint_max': 1 * mm, 'tolerance': 10 * um, 'material': [2.66, 0.03],
    }
    optim_params = {'c_s': 100, 'tau_max': 2.5, 'tau_min': 1.5}
    return doe_params, optim_params


def define_FoM(resolution, sampling_size, wavelength, focal_length, position, device=None):
    """Gaussian PSF with the diffraction-limited FWHM at ``position`` (notebook cell 2), max 1."""
    device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    height, width = resolution
    Lx, Ly = sampling_size * width, sampling_size * height
    eff_L = torch.sqrt(torch.tensor(Lx ** 2 + Ly ** 2, device=device))
    NA = torch.sin(torch.atan(eff_L / (2 * focal_length)))
    fwhm = wavelength / (2 * NA)
    xg, yg = torch.meshgrid(torch.linspace(-Lx / 2, Lx / 2, steps=width, device=device),
                            torch.linspace(-Ly / 2, Ly / 2, steps=height, device=device), indexing="ij")
    x0, y0 = torch.tensor(position, device=device)
    psf = torch.exp(-((xg - x0) ** 2 + (yg - y0) ** 2) / ((fwhm * 2) ** 2))
    return normalize(psf.unsqueeze(0).unsqueeze(0))


def four_focal_spots_target(wavelength=C0 / 300e9, resolution=(100, 100), dxy=1 * mm, device=None):
    """Sum of the nine PSFs of notebook cell 3 ([1, 1, H, W])."""
    return sum(define_FoM(list(resolution), dxy, wavelength, 200 * mm, [a * mm, b * mm], device=device)
               for a, b in FOCI_MM)


class FourFocalSpotsSystem(nn.Module):
    """Submm_Setupv2 of the notebook (cell 4): fixed optics before the DOE, DOE, ASM to the target."""

    def __init__(self, input_dxy=1 * mm, input_field_shape=(100, 100), doe_params=None, optim_params=None,
                 wavelengths=C0 / 300e9, doe_class=Q.SoftGumbelQuantizedDOELayerv3, device=None):
        super().__init__()
        dp, op = default_params()
        self.doe_params = doe_params or dp
        self.optim_params = optim_params or op
        self.device = device or torch.device("cuda")
        self.wavelengths = wavelengths
        self.source = Guassian_beam(height=input_field_shape[0], width=input_field_shape[1], beam_waist_x=None,
                                    beam_waist_y=None, wavelengths=wavelengths, spacing=input_dxy, device=self.device)
        self.asm_prop1 = ASM_prop(z_distance=0.127 * m, bandlimit_type='exact', padding_scale=2,
                                  bandlimit_kernel=True, device=self.device)
        self.Colli_lens = Thin_LensElement(focal_length=0.127 * m)
        self.aperture = ApertureElement(aperture_type='rect', aperture_size=0.08)
        with torch.no_grad():
            self.input_field = self.field_before_DOE()
        if doe_class.__name__.endswith("FullPrecisionDOELayer"):
            self.doe = doe_class(self.doe_params, device=self.device)
        else:
            self.doe = doe_class(self.doe_params, self.optim_params, device=self.device)
        self.asm_prop3 = ASM_prop(z_distance=200 * mm, bandlimit_type='exact', padding_scale=2,
                                  bandlimit_kernel=True, device=self.device)

    def field_before_DOE(self):
        field = self.source()
        field = self.asm_prop1(field)
        field = self.Colli_lens(field)
        return self.aperture(field)

    def forward(self, iter_frac):
        return self.asm_prop3(self.doe(self.input_field, iter_frac))


# ---------------------------------------------------------------------------------------------
# The reference's two multi-plane QAT systems (plot_data/example_2 and example_3): one DOE, several
# output planes, loss = sum over the planes of MSE(normalize(|E_z|^2), target_z).
# ---------------------------------------------------------------------------------------------
def dual_plane_params():
    """doe_params / optim_params of experiment_dual_plane_hologram.ipynb cell 2 (high-temp resin:
    tan d 0.003, 50 um tolerance, no unit-cell mirroring)."""
    doe_params = {
        'doe_size': [100, 100], 'doe_dxy': 1 * mm, 'doe_level': 4, 'look_up_table': None, 'num_unit': None,
        'height_constraint_max': 1 * mm, 'tolerance': 0.05 * mm, 'material': [2.66, 0.003],
    }
    return doe_params, {'c_s': 100, 'tau_max': 2.5, 'tau_min': 1.5}


def edof_params():
    """doe_params / optim_params of experiment_extend_depth_of_focus.ipynb cell 1 (the second,
    effective optim_params of the cell)."""
    doe_params = {
        'doe_size': [100, 100], 'doe_dxy': 1 * mm, 'doe_level': 4, 'look_up_table': None, 'num_unit': None,
        'height_constraint_max': 1 * mm, 'tolerance': 10 * um, 'material': [2.66, 0.03],
    }
    return doe_params, {'c_s': 100, 'tau_max': 2.5, 'tau_min': 1.5}


def logo_targets(device=None):
    """The dual-plane notebook's two targets (cells 3-4: the Aalto logos, grayscale, normalised,
    zero-padded 140 / 90 and nearest-resized from round(.) to 100 x 100) as [2, 1, 100, 100].  The
    PNGs are decoded in the build container by tests/golden/gen_qat_multi.py, which writes the
    resulting 0 / 1 maps to data/dual_plane_targets.npz; nothing here needs the image files."""
    import os
    import numpy as np
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "dual_plane_targets.npz")
    with np.load(path, allow_pickle=False) as z:
        t = torch.from_numpy(z["targets"].astype(np.float32))
    return t[:, None].to(device or torch.device("cuda"))


def edof_target(wavelength=C0 / 300e9, device=None):
    """The extended-DOF notebook's target (cells 2-3): define_FoM at f = 100 mm on the axis."""
    return define_FoM([100, 100], 1 * mm, wavelength, 100 * mm, [0 * mm, 0 * mm], device=device)


class MultiPlaneSystem(nn.Module):
    """Submm_Setupv2 of the multi-plane notebooks: Gaussian source (BeamWaistCorruagtedTK waist) ->
    ASM 127 mm -> lens f = 127 mm [-> ASM 127 mm, ``second_prop``] -> 80 mm square aperture -> DOE ->
    one ASM_prop per output plane, all with the same padding and the exact band limit.

    ``forward(iter_frac)`` is the notebook's: a list of ElectricFields, one per plane.
    ``forward_planes(iter_frac)`` is the MI355X path the trainer uses: every plane from ONE
    pipeline (the DOE modulation fused into the shared row pass, one column pass over the Z planes,
    and in backward the Z-summing adjoint: one launch for all planes), [Z, B, C, H, W]."""

    def __init__(self, planes_m, padding_scale, doe_class, doe_params, optim_params, input_dxy=1 * mm,
                 input_field_shape=(100, 100), wavelengths=C0 / 300e9, second_prop=False, device=None):
        super().__init__()
        self.doe_params, self.optim_params = doe_params, optim_params
        self.device = device or torch.device("cuda")
        self.wavelengths = wavelengths
        self.second_prop = second_prop
        kw = dict(bandlimit_type='exact', padding_scale=padding_scale, bandlimit_kernel=True, device=self.device)
        self.source = Guassian_beam(height=input_field_shape[0], width=input_field_shape[1], beam_waist_x=None,
                                    beam_waist_y=None, wavelengths=wavelengths, spacing=input_dxy, device=self.device)
        self.asm_prop1 = ASM_prop(z_distance=0.127 * m, **kw)
        self.Colli_lens = Thin_LensElement(focal_length=0.127 * m)
        if second_prop:
            self.asm_prop2 = ASM_prop(z_distance=0.127 * m, **kw)
        self.aperture = ApertureElement(aperture_type='rect', aperture_size=0.08)
        with torch.no_grad():
            self.input_field = self.field_before_DOE()
        if doe_class.__name__.endswith("FullPrecisionDOELayer"):
            self.doe = doe_class(self.doe_params, device=self.device)
        else:
            self.doe = doe_class(self.doe_params, self.optim_params, device=self.device)
        self.props = nn.ModuleList([ASM_prop(z_distance=z, **kw) for z in planes_m])

    def field_before_DOE(self):
        field = self.asm_prop1(self.source())
        field = self.Colli_lens(field)
        if self.second_prop:
            field = self.asm_prop2(field)
        return self.aperture(field)

    @property
    def planes(self):
        """The current plane distances (m), host floats."""
        return [float(p._zh[0]) for p in self.props]

    def forward(self, iter_frac):
        field = self.doe(self.input_field, iter_frac)
        return [p(field) for p in self.props]

    def forward_planes(self, iter_frac, z_dev=None):
        """[Z, B, C, H, W]; ``z_dev``: the planes read from device memory (graph replay)."""
        field = self.doe(self.input_field, iter_frac)
        return self.props[0].propagate_planes(field, self.planes, z_dev=z_dev)

    def forward_planes_loss(self, iter_frac, target, z_dev=None):
        """forward_planes fused with the notebooks' loss, the sum over the planes of
        MSE(normalize(|E_z|^2), target_z) (``target`` [Z B or 1, 1, H, W]): (out, loss) from one
        pipeline whose row-inverse pass accumulates the loss (ASM_prop.propagate_planes_loss)."""
        field = self.doe(self.input_field, iter_frac)
        return self.props[0].propagate_planes_loss(field, self.planes, target, z_dev=z_dev)

    def after_forward(self):
        """Per-iteration plane update of the notebook's forward (none here; ExtendedDOFSystem)."""


class DualPlaneSystem(MultiPlaneSystem):
    """experiment_dual_plane_hologram.ipynb cell 6 ("Ours"): padding 2, planes 100 and 150 mm, the
    score-Gumbel v3 layer; the full-precision / naive-Gumbel / PSQ / STE cells (16, 39, 46, 53) add
    the second 127 mm propagation before the aperture (``second_prop``)."""

    def __init__(self, doe_class=Q.SoftGumbelQuantizedDOELayerv3, doe_params=None, optim_params=None,
                 second_prop=None, device=None):
        dp, op = dual_plane_params()
        if second_prop is None:
            second_prop = doe_class is not Q.SoftGumbelQuantizedDOELayerv3
        super().__init__([100 * mm, 150 * mm], 2, doe_class, doe_params or dp, optim_params or op,
                         second_prop=second_prop, device=device)


class ExtendedDOFSystem(MultiPlaneSystem):
    """experiment_extend_depth_of_focus.ipynb cell 22 ("Ours"): padding 4 (P = 500), the rotationally
    symmetric score-Gumbel layer, planes at 50 / 60 / 70 / 80 / 90 mm re-drawn after every forward
    (50 + U(0, 5), 60 + U(-5, 5), 70 + U(-5, 5), 80 + U(-5, 5), 90 + U(-5, 0) mm; the notebook uses
    python's unseeded random.uniform, here a random.Random(seed)).  The full-precision cell (6) adds
    the second 127 mm propagation."""
    JITTER_MM = [(50, 0, 5), (60, -5, 5), (70, -5, 5), (80, -5, 5), (90, -5, 0)]

    def __init__(self, doe_class=Q.RotationallySymmetricScoreGumbelSoftQuantizedDOELayer, doe_params=None,
                 optim_params=None, second_prop=None, seed=0, device=None):
        import random
        dp, op = edof_params()
        if second_prop is None:
            second_prop = doe_class is Q.RotationallySymmetricFullPrecisionDOELayer
        super().__init__([c * mm for c, _, _ in self.JITTER_MM], 4, doe_class, doe_params or dp, optim_params or op,
                         second_prop=second_prop, device=device)
        self.rand = random.Random(seed)

    def forward(self, iter_frac):
        outs = super().forward(iter_frac)
        self.after_forward()
        return outs

    def after_forward(self):
        for p, (c, lo, hi) in zip(self.props, self.JITTER_MM):
            p.z = c * mm + self.rand.uniform(lo * mm, hi * mm)


def _optimizer(kind, params, lr, graph):
    """Adam / AdamW: the one-launch HIP optimiser (optim.py) for device parameters, torch's otherwise."""
    from quantizationawarethzdoe_amd import optim
    if params and params[0].is_cuda:
        return {"adam": optim.Adam, "adamw": optim.AdamW}[kind](params, lr=lr)
    return {"adam": torch.optim.Adam, "adamw": torch.optim.AdamW}[kind](params, lr=lr, capturable=graph)


class StepState:
    """The per-step device state of a graph-replayed trainer: int32 [5 + nz] = the float32 bits of
    the layer schedule (tau, s, beta), the device generator's (seed, step), then the float32 bits of
    the nz output-plane distances of a multi-plane system (``zdev``: the ASM kernels read them,
    thz_asm_desc.z_dev, so the extended-DOF planes can move every replay).

    A replayed step gets its state with no host->device copy command: the host fills one slot of a
    pinned ring (``stage``), and the graph's first node (``fetch``, thz_step_fetch, captured) copies
    slot (device counter mod depth) into the state and advances the counter, so the replays of any
    of the trainer's graphs run back to back.  ``launched`` (after each replay) counts the replays and
    records an event after every ``EVERY``-th: a slot is rewritten only once an event recorded after
    the replay that last read it has completed, so the host runs up to ring - EVERY steps ahead of
    the GPU (an event between two replays costs the GPU ~5 us, a per-step one 8 % of a cfg4 step).
    ``upload`` (an asynchronous copy from a second pinned ring) sets the state for the eager warm-up
    steps before a capture.

    ``installed(layers)`` puts the state on the layers (``_dyn``; with device_rng also ``_rng``,
    two draw streams per layer) for the duration of a capture only: the captured kernels keep the
    pointers, while eager forwards after training draw from torch's generator and use their own
    iter_frac, as the reference's layers do."""

    EVERY = 16

    def __init__(self, device, seed, device_rng, depth=8, nz=0, ring=64):
        import numpy as np
        self.width = 5 + nz
        self.state = torch.zeros(self.width, dtype=torch.int32, device=device)
        self.dyn = self.state[:3].view(torch.float32)
        self.zdev = self.state[5:].view(torch.float32) if nz else None
        self.counter = torch.zeros(1, dtype=torch.int32, device=device)
        self.seed = seed
        self.device_rng = device_rng
        self._np = np
        self._pinned = torch.zeros(depth, self.width, dtype=torch.int32).pin_memory()  # eager uploads
        self._host = self._pinned.numpy()
        self._events = [None] * depth
        self._k = 0
        assert ring % self.EVERY == 0 and ring >= 2 * self.EVERY
        self._ring = torch.zeros(ring, self.width, dtype=torch.int32).pin_memory()  # replays (fetch)
        self._ring_host = self._ring.numpy()
        self._ring_events = [None] * (ring // self.EVERY)
        self._fetches = 0  # replays staged so far == the device counter once they have run

    def _fill(self, row, dyn, step, zs):
        row[:3] = self._np.asarray(dyn, dtype=self._np.float32).view(self._np.int32)
        row[3] = int(self.seed)
        row[4] = int(step) & 0x7FFFFFFF
        if zs is not None:
            row[5:] = self._np.asarray(zs, dtype=self._np.float32).view(self._np.int32)

    def upload(self, dyn, step, zs=None):
        k = self._k
        self._k = (k + 1) % len(self._events)
        ev = self._events[k]
        if ev is None:
            ev = self._events[k] = torch.cuda.Event()
        else:
            ev.synchronize()
        self._fill(self._host[k], dyn, step, zs)
        self.state.copy_(self._pinned[k], non_blocking=True)
        ev.record()

    def stage(self, dyn, step, zs=None):
        """Fill the ring slot the next replay's fetch reads."""
        f, n, ev = self._fetches, len(self._ring), self.EVERY
        if f >= n:  # the slot's last reader is replay f - n: wait for the first event at or after it
            c = -(-(f - n + 1) // ev) * ev
            self._ring_events[(c // ev) % len(self._ring_events)].synchronize()
        self._fill(self._ring_host[f % n], dyn, step, zs)

    def launched(self):
        """After a replay (whose graph fetched the staged slot): count it; every EVERY-th, an event."""
        self._fetches += 1
        if self._fetches % self.EVERY == 0:
            i = (self._fetches // self.EVERY) % len(self._ring_events)
            if self._ring_events[i] is None:
                self._ring_events[i] = torch.cuda.Event()
            self._ring_events[i].record()

    def fetch(self):
        """Captured as a step graph's first node: state <- ring[counter % depth], counter += 1."""
        from quantizationawarethzdoe_amd import _lib
        _lib.check(_lib.lib().thz_step_fetch(self._ring.data_ptr(), len(self._ring), self.width,
                                             self.state.data_ptr(), self.counter.data_ptr(),
                                             _prop._stream_handle()))

    @contextlib.contextmanager
    def installed(self, layers):
        for i, d in enumerate(layers):
            d._dyn = self.dyn
            if self.device_rng:
                d._rng = (self.state[3:], 2 * i)
        try:
            yield
        finally:
            for d in layers:
                d.__dict__.pop("_dyn", None)
                d.__dict__.pop("_rng", None)


def _warn_capture(e):
    import warnings
    warnings.warn(f"capturing the gradient all-reduce into the step graph failed ({e}); "
                  "falling back to split graphs around an eager all-reduce", RuntimeWarning)


def release_step_graph(modules):
    """After a step's backward: the DOE layers keep their last quantized ``height_map`` (the
    reference's attribute, read by visualize() / save()) detached.  Attached, it holds the step's
    autograd graph -- down to the weight's AccumulateGrad node -- alive until the next forward, so
    a HIP-graph capture would reuse the node its warm-up made on another stream (torch's
    "AccumulateGrad node's stream does not match" warning).  The values are
    unchanged (a detached view of the same storage, which graph replays keep updating).  The same
    for the layer's last pending modulation (its height, output and upsampled height map)."""
    def _det(t):
        return t.detach() if torch.is_tensor(t) and not isinstance(t, nn.Parameter) and t.grad_fn is not None else t

    for m in modules:
        for layer in m.modules():
            h = layer.__dict__.get("height_map")
            if torch.is_tensor(h):
                layer.height_map = _det(h)
            # the last modulation (DOELayer._height_map_ reads its hfull): its height and product
            # tensors hold the same graph
            pend = layer.__dict__.get("_pending_mod")
            if pend is not None:
                for k in ("field", "height", "out", "hfull"):
                    if k in pend.__dict__:
                        setattr(pend, k, _det(getattr(pend, k)))
                # its quantizer link holds the weight's view (doe.QuantLink.weight): the same graph
                if getattr(pend, "quant", None) is not None:
                    pend.quant = None


def collective_capture_safe():
    """Whether an RCCL collective may be captured into a step graph in this process: only with
    ``TORCH_NCCL_CUDA_EVENT_CACHE=0``.  With torch's default (cached, reused CUDA events) the process
    group's watchdog was seen to abort the process, about once in ten runs, querying an event "last
    recorded in a capturing stream" after a captured all-reduce.  The variable is read
    by ProcessGroupNCCL when the group is created, so the library cannot set it for the caller: it
    must be in the environment before ``init_process_group``; the trainers check it when they
    capture and otherwise keep the collective out of the graph (``agreed_capture``)."""
    return os.environ.get("TORCH_NCCL_CUDA_EVENT_CACHE") == "0"


def agreed_capture(allreduce, capture_fn):
    """Capture the whole step with the collective inside it (``capture_fn() -> (graph, loss)``),
    with every rank agreeing on the outcome: after the attempt, an eager all_reduce(MIN) of a
    success flag outside any capture.  Returns capture_fn's result, or None when the capture failed
    on ANY rank -- every rank then discards its graph and builds the split form (fwd/bwd graph, eager
    all-reduce, optimiser graph), so no rank replays a graph with a captured collective while
    another runs the eager one.  A rank whose environment does not make the capture safe
    (``collective_capture_safe``) does not attempt it and votes for the split form.  Without an
    active collective a capture error is raised as is."""
    ok, res, err = 1, None, None
    if allreduce.active and allreduce.capturable and not collective_capture_safe():
        ok, err = 0, RuntimeError("TORCH_NCCL_CUDA_EVENT_CACHE is not 0 in this process (set it before "
                                  "init_process_group to capture the all-reduce)")
    else:
        try:
            res = capture_fn()
        except RuntimeError as e:
            if not allreduce.active:
                raise
            ok, err = 0, e
    if allreduce.active:
        flag = torch.tensor([ok], dtype=torch.int32, device=allreduce.flat.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=allreduce.group)
        ok = int(flag.item())
    if not ok:
        _warn_capture(err if err is not None else "the capture failed on another rank")
        return None
    return res


class GradientAllReduce:
    """Average the gradients of ``params`` over the process group with ONE flat all-reduce.

    10 KB for cfg4 (50 x 50 fp32): latency-bound, so a single bucket; the flat buffer is
    allocated once and reused every step.  The three phases are separate so the trainers can
    put ``pack`` at the end of the captured forward/backward graph, ``reduce`` (the collective)
    between the graph replays and ``unpack`` at the head of the optimiser graph -- the same
    calls the eager step makes, so the CPU gloo tests run the exact placement the HIP-graph
    path replays.  All three are no-ops at world size 1 unless ``force`` (an initialised process
    group of one rank: the collective still runs, to test and time its capture on one GPU).
    """

    def __init__(self, params, group=None, force=False):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.active = self.world > 1 or (bool(force) and dist.is_available() and dist.is_initialized())
        # the collective can be captured into a HIP graph on RCCL (torch's "nccl" backend) only
        self.capturable = self.active and dist.get_backend(group) == "nccl"
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self._offsets = []
        self._slots_used = set()  # parameters whose slot a backward kernel took this step (doe.grad_slot)
        off = 0
        for p in self.params:
            self._offsets.append(off)
            if self.active and p.dtype == torch.float32:
                # the DOE layers' fused backward kernels write this parameter's gradient straight into
                # its slice of the bucket (doe.grad_slot): pack and unpack then copy nothing
                p._thz_grad_slot = (self.flat, off, self._slots_used)
            off += p.numel()

    def _in_bucket(self, p, off):
        g = p.grad
        return (g is not None and g.dtype == torch.float32 and g.is_contiguous()
                and g.data_ptr() == self.flat.data_ptr() + 4 * off)

    def pack(self):
        """Gradients -> the flat bucket (a parameter without a gradient contributes zeros; one whose
        gradient a fused kernel already wrote into its slice costs nothing)."""
        if not self.active:
            return
        self._slots_used.clear()  # the step's backward is done: the slots are free for the next one
        for p, off in zip(self.params, self._offsets):
            k = p.numel()
            if p.grad is None:
                self.flat[off:off + k].zero_()
            elif not self._in_bucket(p, off):
                self.flat[off:off + k].copy_(p.grad.reshape(-1))

    def reduce(self):
        """The one collective of the step: the mean over ranks (RCCL's average in one kernel; gloo:
        sum, then / world)."""
        if not self.active:
            return
        if dist.get_backend(self.group) == "nccl":
            dist.all_reduce(self.flat, op=dist.ReduceOp.AVG, group=self.group)
        else:
            dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
            self.flat.mul_(1.0 / self.world)

    def unpack(self):
        """The averaged bucket -> every parameter's gradient (nothing to copy for a gradient that
        is the bucket's own slice)."""
        if not self.active:
            return
        for p, off in zip(self.params, self._offsets):
            k = p.numel()
            g = self.flat[off:off + k].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            elif not self._in_bucket(p, off):
                p.grad.copy_(g)

    def __call__(self):
        self.pack()
        self.reduce()
        self.unpack()


class QATTrainer:
    """One QAT iteration = forward, fused loss, backward, gradient all-reduce, Adam step.

    ``graph=True`` captures the iteration as HIP graphs (one per schedule phase of the DOE
    layer: continuous / blend / quantized for v3) and replays them: the step is launch-bound
    at cfg4 sizes (100^2, P = 300; ~30 small kernels), so replay removes the per-kernel host
    overhead.  The schedule values that change every step (tau, s = tau_max / tau, beta) reach
    the quantizer kernels through a 3-float device buffer (thz_quant_desc.dyn), and the
    Gumbel / height-noise draws are graph-safe philox draws, so each replay is a fresh sample.
    On one rank the whole step (forward, loss, backward, Adam) is ONE graph; with N ranks the
    replay is split around the (eager) gradient all-reduce, or, with ``capture_collective``, the
    all-reduce is captured too and the step is again one replay (RCCL kernels inside the graph).
    The random stream differs from the eager path (same distribution, different draws).
    ``force_collective`` runs the collective on a one-rank process group (tests / timing).
    """

    def __init__(self, system, target, lr=0.02, max_itrs=6000, group=None, graph=False, loss_fn=None,
                 device_rng=True, capture_collective=False, force_collective=False, optimizer="adam"):
        self.system = system
        self.target = target.to(system.device).float().contiguous()
        # multi-plane systems (MultiPlaneSystem): ``target`` is [Z, 1, H, W] (one per plane) or
        # [1, 1, H, W] (shared); the loss kernel sees the planes as its batch
        self.multi = hasattr(system, "forward_planes")
        self._zs_graph = None
        if self.multi:
            Z, B = len(system.planes), system.input_field.shape[0]
            t = self.target.reshape((-1, 1) + tuple(self.target.shape[-2:]))
            if t.shape[0] not in (1, Z):
                raise ValueError(f"multi-plane target: {t.shape[0]} maps for {Z} planes")
            self.target = (t.repeat_interleave(B, 0) if t.shape[0] == Z and B > 1 else t).contiguous()
        self.max_itrs = max_itrs
        self.graph = graph
        # loss(out_field_data, target): the fused HIP |E|^2 -> normalize -> MSE by default
        self.loss_fn = loss_fn or _optics.intensity_mse
        params = list(system.parameters())
        # one Adam kernel per step on the GPU, the step counts advanced in it (optim.py; torch's fused
        # capturable path launches a step-count kernel and an update kernel).  "adamw": the notebook's
        # full-precision, naive-Gumbel and STE runs use torch.optim.AdamW with its defaults
        # (weight_decay 0.01; experiment_four_focal_spots.ipynb cells 22, 33, 52)
        self.optimizer = _optimizer(optimizer, params, lr, graph)
        self.allreduce = GradientAllReduce(list(system.parameters()), group=group, force=force_collective)
        self.capture_collective = bool(capture_collective)
        self._one = torch.ones((), dtype=torch.float32, device=system.device)
        self.itr = 0
        self._graphs = {}
        if graph:
            # one device state per step: (tau, s, beta) as float bits, then the generator (seed, step);
            # with device_rng the layer's Gumbel and height-noise draws are made in the kernels from
            # it (no torch RNG kernels, nor their per-replay offset fills, in the captured graph)
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if device_rng else 0
            self._step_state = StepState(system.device, seed, device_rng, nz=len(system.planes) if self.multi else 0)
            self.dyn = self._step_state.dyn
            # multi-plane: the captured propagation reads its planes from the step state
            self._zs_graph = self._step_state.zdev

    def _frac(self, iter_frac):
        return self.itr / self.max_itrs if iter_frac is None else iter_frac

    # The step in two phases around the one collective; the eager step and the captured graphs
    # run the same two functions (fwd/bwd + pack | all-reduce | unpack + Adam).
    def _fb(self, frac):
        if self.multi:
            # every plane from one pipeline ([Z, B, C, H, W]; backward: the Z-summing adjoint), the
            # loss kernel over the Z B planes as its batch (normalize is per plane), x Z: the sum
            # over the planes of each plane's mean
            if self.loss_fn is _optics.intensity_mse:
                # the loss folded into the planes' row-inverse pass, summed over the planes in-kernel
                out, loss = self.system.forward_planes_loss(frac, self.target, z_dev=self._zs_graph)
            else:
                out = self.system.forward_planes(frac, z_dev=self._zs_graph)
                Z, B = out.shape[:2]
                loss = self.loss_fn(out.reshape((Z * B,) + tuple(out.shape[2:])), self.target) * float(Z)
            if self._zs_graph is None:
                self.system.after_forward()  # the notebook's per-iteration plane update (eager)
        elif self.loss_fn is _optics.intensity_mse:
            # the default loss folded into the last propagation
            with _prop.deferred_output():
                out = self.system(frac)
            loss = _optics.field_intensity_mse(out, self.target)
        else:
            out = self.system(frac)
            loss = self.loss_fn(out.data, self.target)
        # d loss / d loss = 1 from a preallocated tensor: no fill kernel per step
        loss.backward(gradient=self._one if loss.dtype == self._one.dtype and loss.device == self._one.device else None)
        release_step_graph([self.system])
        self.allreduce.pack()
        # detached: the returned (graph-static) loss must not hold the step's autograd graph, whose
        # AccumulateGrad nodes -- made on the warm-up stream -- would otherwise outlive the capture and
        # be reused by the next capture's backward on another stream (torch's "AccumulateGrad node's
        # stream does not match" warning)
        return loss.detach()

    def _opt(self):
        self.allreduce.unpack()
        self.optimizer.step()

    def step(self, iter_frac=None):
        frac = self._frac(iter_frac)
        if self.graph:
            loss = self._graph_step(frac)
        else:
            self.optimizer.zero_grad(set_to_none=False)
            loss = self._fb(frac)
            self.allreduce.reduce()
            self._opt()
        self.itr += 1
        return loss

    # -- graph path ----------------------------------------------------------------------------
    def _capture(self, frac):
        # a graph left by construction (the layer's initial height map) or by eager steps would hand
        # the warm-up the weights' AccumulateGrad nodes made on another stream
        release_step_graph([self.system])
        params = self.allreduce.params
        # warm-up steps (allocator, autograd, Adam's lazy state) must not change the training
        # trajectory: snapshot the weights and the optimiser state, restore them afterwards
        p0 = [p.detach().clone() for p in params]
        st0 = {id(p): {k: v.clone() for k, v in self.optimizer.state[p].items() if torch.is_tensor(v)}
               for p in params if p in self.optimizer.state}
        side = torch.cuda.Stream(device=self.system.device)
        side.wait_stream(torch.cuda.current_stream())
        with self._step_state.installed([self.system.doe]):
            with torch.cuda.stream(side):
                for _ in range(2):
                    self.optimizer.zero_grad(set_to_none=True)
                    self._fb(frac)
                    self.allreduce.reduce()  # the communicator is set up outside the capture
                    self._opt()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            with torch.no_grad():
                for p, v in zip(params, p0):
                    p.copy_(v)
                for p in params:
                    saved = st0.get(id(p))
                    for k, v in self.optimizer.state[p].items():
                        if torch.is_tensor(v):
                            v.copy_(saved[k]) if saved is not None else v.zero_()
            self.optimizer.zero_grad(set_to_none=True)
            if not self.allreduce.active or (self.capture_collective and self.allreduce.capturable):
                # no collective, or a captured one: the whole step (fwd/bwd, all-reduce, Adam) is
                # one graph, one replay per step
                def whole():
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                        self._step_state.fetch()
                        loss = self._fb(frac)
                        self.allreduce.reduce()
                        self._opt()
                    return g, loss
                res = agreed_capture(self.allreduce, whole)
                if res is not None:
                    return res[0], None, res[1]
                self.capture_collective = False  # every rank falls back (agreed_capture)
                self.optimizer.zero_grad(set_to_none=True)
            g_fb, g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_fb, capture_error_mode=_CAPTURE_MODE):
                self._step_state.fetch()
                loss = self._fb(frac)
            with torch.cuda.graph(g_opt, capture_error_mode=_CAPTURE_MODE):
                self._opt()
        return g_fb, g_opt, loss

    def _graph_step(self, frac):
        phase = self.system.doe._graph_phase(frac)
        dyn, zs = self.system.doe._dyn_values(frac), (self.system.planes if self.multi else None)
        if phase not in self._graphs:
            self._step_state.upload(dyn, self.itr, zs)  # the capture's eager warm-up steps
            self._graphs[phase] = self._capture(frac)
        g_fb, g_opt, loss = self._graphs[phase]
        self._step_state.stage(dyn, self.itr, zs)
        g_fb.replay()
        self._step_state.launched()
        if g_opt is not None:  # an eager collective between the two captured halves
            self.allreduce.reduce()
            g_opt.replay()
        if self.multi:
            self.system.after_forward()  # the next replay's planes (the notebook's per-iteration update)
        return loss

    def train(self, steps, log_every=200, log=print):
        t0 = time.perf_counter()
        losses = []
        for _ in range(steps):
            loss = self.step()
            # graph replays overwrite the captured loss tensor in place: keep a copy per step
            losses.append(loss.detach().clone())
            if log_every and (self.itr - 1) % log_every == 0:
                log(f"The iteration : {self.itr - 1}, Loss: {float(loss):.6g}")
        torch.cuda.synchronize()
        return torch.stack(losses).cpu(), time.perf_counter() - t0
