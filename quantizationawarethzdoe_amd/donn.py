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

from quantizationawarethzdoe_amd import optics as _optics
from quantizationawarethzdoe_amd.qat import _CAPTURE_MODE, agreed_capture, release_step_graph
from quantizationawarethzdoe_amd import propagation as _prop
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


def propagate_through_aperture(prop, aperture, field):
    """``aperture(prop(field))`` -- an ASM_prop to one plane, then an ApertureElement -- with the
    aperture folded into the propagation when the library carries it (thz_asm_desc.window_mask:
    the 300-point layer geometry): the row-inverse pass stores the masked field and the backward's
    row pass masks the incoming gradient, so no aperture kernel runs either way.  Otherwise (other
    geometries, complex128, a multi-valued z) the two modules run as written."""
    B, C, H, W = field.shape
    ph, pw = prop.compute_padding(H, W, return_size_of_padding=True)
    unpad = (not prop.do_padding) or prop.do_unpad_after_pad
    if field._pending is not None and field._take_pending() is None:  # a deferred propagation's output
        return aperture(prop(field))
    pend = field._take_pending()  # the DOE layer's unevaluated modulation, or None
    data = pend.field if pend is not None else field.data
    dt = _prop.kernel_dtype(data, "ASM_prop", field.wavelengths).dtype
    # (inside the trainers' deferred_output block too: the aperture reads the propagation's output
    # at once either way, so running it here defers nothing the loss fold needs)
    if (dt != torch.complex64 or len(prop._zh) != 1
            or not _prop.window_mask_fusable(H, W, ph, pw, unpad)):
        return aperture(prop(field))
    mask = aperture.window_desc(field, H, W)
    if mask is None:
        return aperture(prop(field))
    out = prop._run(field, prop._zh, out_mask=mask).squeeze(0)
    aperture._note_input(field, shape=out.shape, dtype=out.dtype)
    return ElectricField(data=out, wavelengths=field.wavelengths, spacing=field.spacing,
                         device=field.device)._adopt_host(field)


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
        # wavelength / spacing tensors made once (fp32 casts of ElectricField.check_*): building the
        # input field per step then copies nothing host->device, so a step can be graph-captured
        self._tmpl = ElectricField(data=torch.zeros(1, 1, 1, 1, dtype=torch.complex64), wavelengths=wavelengths,
                                   spacing=input_dxy, device=dev)

    def encode_object(self, u):
        """Plane wave times the object amplitude ``u`` [B, 1, H, W] -> ASM 50 mm -> aperture (nb :171-190)."""
        u = u.to(self.device)
        field = ElectricField(data=u.to(torch.complex64), wavelengths=self._tmpl.wavelengths,
                              spacing=self._tmpl.spacing, device=self.device)._adopt_host(self._tmpl)
        return propagate_through_aperture(self.asm_prop2layer, self.aperture, field)

    def forward(self, u, iter_frac=None, chained=False):
        inputs = self.encode_object(u)
        field = inputs
        for i in range(self.num_layer - 1):
            field = self.does[i](field if chained else inputs, iter_frac)
            field = propagate_through_aperture(self.asm_prop_layer, self.aperture, field)
        field = self.does[-1](field if chained else inputs, iter_frac)
        return self.asm_prop2detector(field)


def detector_targets(num_classes=10, shape=(100, 100), det=10, device=None):
    """Per-class target intensity images [num_classes, 1, H, W] (float32): ones inside the class's
    det x det detector square, zeros elsewhere.  The detectors sit in three rows (3, 4, 3) centred
    in the plane, the usual 10-class DONN readout.

    The reference notebook's label-generator and training cells are empty
    (experiment_DONN_3_layers.ipynb, sections 3-5), so this layout is this framework's choice;
    the loss it feeds is the reference's QAT loss, MSE(normalize(|E|^2), target)
    (experiment_four_focal_spots.ipynb:336-370, utils/Helper_Functions.py:185-193)."""
    H, W = shape
    if num_classes > 10:
        raise ValueError("detector_targets lays out at most 10 detectors")
    rows = [(H * 0.25, 3), (H * 0.5, 4), (H * 0.75, 3)]
    centres = []
    for yc, n in rows:
        for j in range(n):
            centres.append((yc, W * (j + 1) / (n + 1)))
    t = torch.zeros(num_classes, 1, H, W, dtype=torch.float32)
    for k in range(num_classes):
        yc, xc = centres[k]
        y0, x0 = int(round(yc - det / 2)), int(round(xc - det / 2))
        t[k, 0, max(y0, 0):y0 + det, max(x0, 0):x0 + det] = 1.0
    dev = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return t.to(dev)


class DONNTrainer:
    """Data-parallel DONN training step: forward of this rank's share of
    the batch, loss = MSE(normalize(|E|^2), per-sample detector target), backward through the
    HIP adjoint kernels, ONE flat all-reduce of the three layers' weight gradients (120 KB at
    100^2; RCCL over xGMI on the GPU, gloo in the CPU tests), Adam.

    ``chained=False`` keeps the notebook's forward (every layer modulates the encoded input, so
    only the last layer receives a gradient; the others contribute zeros to the all-reduce).
    ``graph=True`` captures the step as HIP graphs per schedule phase (qat.QATTrainer's scheme):
    the batch and its targets are copied into static device buffers before each replay.
    """

    def __init__(self, model, targets, lr=0.02, max_itrs=6000, group=None, graph=False, chained=True, loss_fn=None,
                 device_rng=True, capture_collective=False, force_collective=False):
        from quantizationawarethzdoe_amd.qat import GradientAllReduce, _optimizer
        self.model = model
        self.targets = targets.to(model.device).float().contiguous()
        self.max_itrs = max_itrs
        self.graph = graph
        self.chained = chained
        self.loss_fn = loss_fn
        self.params = [p for p in model.parameters() if p.requires_grad]
        self.optimizer = _optimizer("adam", self.params, lr, graph)
        self.allreduce = GradientAllReduce(self.params, group=group, force=force_collective)
        self.capture_collective = bool(capture_collective)  # qat.QATTrainer's option
        self._one = torch.ones((), dtype=torch.float32, device=model.device)
        self.itr = 0
        self._graphs = {}
        self._static = None
        if graph:
            # (tau, s, beta) bits + the device generator (seed, step): qat.QATTrainer's scheme; each
            # layer draws on its own streams
            from quantizationawarethzdoe_amd.qat import StepState
            seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if device_rng else 0
            self._step_state = StepState(model.device, seed, device_rng)
            self.dyn = self._step_state.dyn

    def _loss(self, u, target, frac):
        if self.loss_fn is None or self.loss_fn is _optics.intensity_mse:
            # the default loss folded into the detector propagation
            with _prop.deferred_output():
                out = self.model(u, frac, chained=self.chained)
            return _optics.field_intensity_mse(out, target)
        out = self.model(u, frac, chained=self.chained)
        return self.loss_fn(out.data, target)

    # the step in two phases around the one collective (qat.QATTrainer's scheme): the eager step
    # and the captured graphs run the same functions
    def _fb(self, u, target, frac):
        loss = self._loss(u, target, frac)
        # preallocated d loss / d loss: no fill kernel per step
        loss.backward(gradient=self._one if loss.dtype == self._one.dtype and loss.device == self._one.device else None)
        release_step_graph([self.model])
        self.allreduce.pack()
        # detached: the returned (graph-static) loss must not hold the step's autograd graph, whose
        # AccumulateGrad nodes -- made on the warm-up stream -- would otherwise outlive the capture and
        # be reused by the next capture's backward on another stream (torch's "AccumulateGrad node's
        # stream does not match" warning)
        return loss.detach()

    def _opt(self):
        self.allreduce.unpack()
        self.optimizer.step()

    def step(self, u, labels, iter_frac=None):
        """One iteration on images ``u`` [B, 1, H, W] (float, this rank's share) and int64 ``labels`` [B]."""
        frac = self.itr / self.max_itrs if iter_frac is None else iter_frac
        labels = labels.to(self.model.device)
        if self.graph:
            loss = self._graph_step(u, labels, frac)
            self.itr += 1
            return loss
        u = u.to(self.model.device, torch.float32)
        target = self.targets.index_select(0, labels)
        self.optimizer.zero_grad(set_to_none=False)
        loss = self._fb(u, target, frac)
        self.allreduce.reduce()
        self._opt()
        self.itr += 1
        return loss

    # -- graph path ----------------------------------------------------------------------------
    def _capture(self, frac):
        # a graph left by construction or by eager steps (the layers' attached height maps) would
        # hand the warm-up the weights' AccumulateGrad nodes made on another stream
        release_step_graph([self.model])
        su, st = self._static
        p0 = [p.detach().clone() for p in self.params]
        st0 = {id(p): {k: v.clone() for k, v in self.optimizer.state[p].items() if torch.is_tensor(v)}
               for p in self.params if p in self.optimizer.state}
        side = torch.cuda.Stream(device=self.model.device)
        side.wait_stream(torch.cuda.current_stream())
        with self._step_state.installed(self.model.does):
            with torch.cuda.stream(side):
                for _ in range(2):  # allocator, autograd, Adam's lazy state, communicator: outside the capture
                    self.optimizer.zero_grad(set_to_none=True)
                    self._fb(su, st, frac)
                    self.allreduce.reduce()
                    self._opt()
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            with torch.no_grad():  # the warm-up must not move the training trajectory
                for p, v in zip(self.params, p0):
                    p.copy_(v)
                for p in self.params:
                    saved = st0.get(id(p))
                    for k, v in self.optimizer.state.get(p, {}).items():
                        if torch.is_tensor(v):
                            v.copy_(saved[k]) if saved is not None else v.zero_()
            self.optimizer.zero_grad(set_to_none=True)
            if not self.allreduce.active or (self.capture_collective and self.allreduce.capturable):
                # no collective, or a captured one: the whole step is one graph, one replay per step

                def whole():
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                        self._step_state.fetch()
                        loss = self._fb(su, st, frac)
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
                loss = self._fb(su, st, frac)
            with torch.cuda.graph(g_opt, capture_error_mode=_CAPTURE_MODE):
                self._opt()
        return g_fb, g_opt, loss

    def _graph_step(self, u, labels, frac):
        # the static inputs: the batch already as the complex64 field the encoder propagates (the copy
        # converts, so the captured step has no conversion kernel) and the targets gathered straight
        # into their buffer (one kernel, no gather + copy)
        shape = (u.shape[0],) + tuple(self.targets.shape[1:])
        if self._static is None or self._static[0].shape != u.shape:
            self._static = (torch.empty(u.shape, dtype=torch.complex64, device=self.model.device),
                            torch.empty(shape, dtype=self.targets.dtype, device=self.model.device))
            self._graphs = {}
        su, st = self._static
        su.copy_(u)
        torch.index_select(self.targets, 0, labels, out=st)
        lead = self.model.does[0]
        phase = lead._graph_phase(frac)
        dyn = lead._dyn_values(frac)
        if phase not in self._graphs:
            self._step_state.upload(dyn, self.itr)  # the capture's eager warm-up steps
            self._graphs[phase] = self._capture(frac)
        g_fb, g_opt, loss = self._graphs[phase]
        self._step_state.stage(dyn, self.itr)
        g_fb.replay()
        self._step_state.launched()
        if g_opt is not None:  # an eager collective between the two captured halves
            self.allreduce.reduce()
            g_opt.replay()
        return loss


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
