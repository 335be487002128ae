"""Band-limited angular-spectrum propagator, ASM_prop -- drop-in for Props/ASM_Prop.py.

Same constructor (``z_distance, do_padding, do_unpad_after_pad, padding_scale,
bandlimit_kernel, bandlimit_type, device``; Props/ASM_Prop.py:19-117), same
``padding_scale`` validation and ``Exception`` text (:75-98), same ``z`` property
(:185-195, including that assigning a non-tensor stores the raw value), same
once-per-instance critical-distance diagnostic (:279-285), same ``forward(field) ->
ElectricField`` (:314-378) and the same OOM hint on ``RuntimeError`` (:363-370).

The math runs in libthzdoe's hand-written gfx950 kernels (thz_asm.hip); the
transfer function is never materialised.  Backward is the adjoint kernel.
MI355X addition (opt-in, additive): ``propagate_planes(field, z_list)`` evaluates
many z-planes with one shared forward row pass (the extend-DOF sweep of
experiment_extend_depth_of_focus.ipynb:229-256) and returns [Z, B, C, H, W].
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField
from quantizationawarethzdoe_amd import propagation as _prop


def _z_host(z):
    if torch.is_tensor(z):
        return [float(v) for v in z.detach().reshape(-1).cpu().tolist()]
    if isinstance(z, (list, tuple, np.ndarray)):
        return [float(v) for v in np.asarray(z).reshape(-1)]
    return [float(z)]


class _PendingAsm:
    """An ASM_prop.forward not yet run (propagation.deferred_output): ``run()`` gives the field
    data as forward would; ``run_loss(target)`` gives (data, QAT loss) from the fused pipeline."""
    kind = "propagation"

    def __init__(self, prop, field, zs):
        self.prop, self.field, self.zs = prop, field, zs

    def run(self):
        return self.prop._run(self.field, self.zs).squeeze(0)

    def run_loss(self, target):
        out, loss = self.prop._run(self.field, self.zs, loss_target=target)
        return out.squeeze(0), loss


class ASM_prop(nn.Module):
    def __init__(self, z_distance: float = 0.0, do_padding: bool = True, do_unpad_after_pad: bool = True,
                 padding_scale=None, bandlimit_kernel: bool = True, bandlimit_type: str = "exact",
                 device: str = None) -> None:
        super().__init__()
        DEFAULT_PADDING_SCALE = torch.tensor([1, 1])
        if do_padding:
            err = False
            if not torch.is_tensor(padding_scale):
                if padding_scale is None:
                    padding_scale = DEFAULT_PADDING_SCALE
                elif np.isscalar(padding_scale):
                    padding_scale = torch.tensor([padding_scale, padding_scale])
                else:
                    padding_scale = torch.tensor(padding_scale)
                    if padding_scale.numel() != 2:
                        err = True
            elif padding_scale.numel() == 1:
                padding_scale = padding_scale.squeeze()
                padding_scale = torch.tensor([padding_scale, padding_scale])
            elif padding_scale.numel() == 2:
                padding_scale = padding_scale.squeeze()
            else:
                err = True
            if err:
                raise Exception("Invalid value for argument 'padding_scale'.  Should be a real-valued non-negative "
                                "scalar number or a two-element tuple/tensor containing real-valued non-negative "
                                "scalar numbers.")
        else:
            padding_scale = None
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self._z = torch.tensor(z_distance, device=self.device)
        self._zh = _z_host(z_distance)
        self.do_padding = do_padding
        self.do_unpad_after_pad = do_unpad_after_pad
        self.padding_scale = padding_scale
        self.bandlimit_kernel = bandlimit_kernel
        self.bandlimit_type = bandlimit_type
        if bandlimit_kernel and bandlimit_type not in ("exact", "approx"):
            self._bad_type = True
        self.shape = None
        self.check_Zc = True

    # -- z property (Props/ASM_Prop.py:185-195) -----------------------------------------------
    @property
    def z(self):
        return self._z

    @z.setter
    def z(self, z) -> None:
        if isinstance(z, torch.Tensor) and z.device != torch.device(self.device):
            z = z.to(self.device)
        self._z = z
        self._zh = _z_host(z)

    # -- frequency grid and transfer function, for inspection (Props/ASM_Prop.py:138-311) ------
    def create_frequency_grid(self, H, W):
        """Normalised centred frequency grids (i - H//2)/H and (j - W//2)/W, meshgrid 'ij'
        (Props/ASM_Prop.py:138-145), as the ``Kx`` / ``Ky`` buffers.  The kernels form the same
        values per element and never read these."""
        with torch.no_grad():
            fx = (torch.arange(H, dtype=torch.float32) - (H // 2)) / H
            fy = (torch.arange(W, dtype=torch.float32) - (W // 2)) / W
            self.Kx, self.Ky = torch.meshgrid(fx, fy, indexing="ij")
        self._grid_shape = self._shape

    @property
    def shape(self):
        return self._shape

    @shape.setter
    def shape(self, shape):
        """The padded field shape of the last call (Props/ASM_Prop.py:151-167).  The reference
        rebuilds Kx / Ky whenever (H, W) changes; here they are built when first read after such a
        change (a P = 8192 grid is 512 MB of host memory that no kernel uses)."""
        self._shape = shape

    def _grid(self):
        shp = self._shape
        if shp is not None and (getattr(self, "_grid_shape", None) is None
                                or tuple(self._grid_shape[-2:]) != tuple(shp[-2:])):
            self.create_frequency_grid(int(shp[-2]), int(shp[-1]))

    @property
    def Kx(self):
        self._grid()
        return self._Kx

    @Kx.setter
    def Kx(self, Kx):
        self.register_buffer("_Kx", Kx)

    @property
    def Ky(self):
        self._grid()
        return self._Ky

    @Ky.setter
    def Ky(self, Ky):
        self.register_buffer("_Ky", Ky)

    def create_kernel(self, field: ElectricField) -> torch.Tensor:
        """The band-limited transfer function [1, C, Ph, Pw] on the centred grid of the padded
        plane (Props/ASM_Prop.py:212-311), with the once-per-instance critical-distance print.
        The propagators never build it (they evaluate H per element); this materialises the same
        values with the HIP kernel thz_asm_transfer_function for inspection."""
        B, C, H, W = field.shape
        ph, pw = self.compute_padding(H, W, return_size_of_padding=True)
        self.shape = torch.Size([B, C, H + 2 * ph, W + 2 * pw])
        sp, wl = field.spacing_host, field.wavelengths_host
        bl = self._bandlimit_code()
        self._zc_diagnostic(H + 2 * ph, sp[0], wl, self._zh[0])
        return _prop.asm_transfer_function(wl, sp, self._zh[0], H, W, ph, pw, bl, field.device)

    def visualize_kernel(self, field: ElectricField):
        """Amplitude and phase of create_kernel(field) (Props/ASM_Prop.py:198-210)."""
        import matplotlib.pyplot as plt
        kernel = self.create_kernel(field=field)
        plt.subplot(121)
        plt.imshow(kernel.abs().cpu().squeeze(), vmin=0)
        plt.title("Amplitude")
        plt.subplot(122)
        plt.imshow(kernel.angle().cpu().squeeze())
        plt.title("Phase")
        plt.tight_layout()

    def compute_padding(self, H, W, return_size_of_padding=False):
        """Props/ASM_Prop.py:119-136."""
        if not self.do_padding:
            ph, pw = 0, 0
        else:
            ph = int(np.floor((float(self.padding_scale[0]) * H) / 2))
            pw = int(np.floor((float(self.padding_scale[1]) * W) / 2))
        if return_size_of_padding:
            return ph, pw
        return H + 2 * ph, W + 2 * pw

    def _bandlimit_code(self):
        if not self.bandlimit_kernel:
            return 0
        if self.bandlimit_type == "exact":
            return 1
        if self.bandlimit_type == "approx":
            return 2
        raise Exception("Should not be in this state.")

    def _zc_diagnostic(self, Ph, dx, wavelengths_host, z):
        """Critical distance print, once per instance (Props/ASM_Prop.py:279-285)."""
        if not (self.bandlimit_kernel and self.check_Zc):
            return
        lmax = np.float32(max(wavelengths_host))
        dx = np.array([dx], dtype=np.float32)
        with np.errstate(invalid="ignore"):  # lambda > 2 dx gives nan, as the reference prints
            zc = (np.float32(Ph) * dx ** 2) * np.sqrt(np.float32(1) - (lmax / (np.float32(2) * dx)) ** 2) / lmax
        if z > zc[0]:
            print("The propagation distance is greater than critical distance {} m, the TF will be undersampled!"
                  .format(zc))
        else:
            print("The critical distance is {} m, the TF will be fine during the sampling !".format(zc))
        self.check_Zc = False

    def _run(self, field: ElectricField, zs, loss_target=None, out_mask=None, z_dev=None):
        """[Z, B, C, Ho, Wo]; with ``loss_target``: (out, QAT loss) from the fused pipeline (Z > 1: the
        sum of the planes' losses, propagation.asm_propagate_loss);
        ``out_mask``: an aperture folded onto the output (propagation.window_mask_fusable geometry);
        ``z_dev``: the planes read from device memory (propagation._asm_desc)."""
        pend = field._take_pending()
        data = pend.field if pend is not None else field.data
        B, C, H, W = data.shape
        ph, pw = self.compute_padding(H, W, return_size_of_padding=True)
        self.shape = torch.Size([B, C, H + 2 * ph, W + 2 * pw])
        bl = self._bandlimit_code()
        wl = field.wavelengths_host
        sp = field.spacing_host
        self._zc_diagnostic(H + 2 * ph, sp[0], wl, zs[0])
        x = _prop.kernel_dtype(data, "ASM_prop", field.wavelengths)
        unpad = (not self.do_padding) or self.do_unpad_after_pad
        if loss_target is not None and x.dtype != torch.complex64:
            # the fused ASM -> loss pipeline and the loss kernel compute in complex64 (the unfused
            # field_intensity_mse refuses a complex128 field the same way, optics.intensity_mse)
            raise TypeError(f"loss kernel computes in complex64 fields; got {x.dtype}")
        try:
            if loss_target is not None:
                fuse = pend is not None and pend.out is None
                x = pend.run() if pend is not None and not fuse else x
                out = _prop.asm_propagate_loss(x, loss_target, wl, sp, list(zs), ph, pw, unpad=unpad, bandlimit=bl,
                                               pend=pend if fuse else None, z_dev=z_dev)
            elif pend is not None and pend.out is None:  # the DOE layer's modulation, fused into the row pass
                out = _prop.asm_propagate_modulated(pend, wl, sp, zs, ph, pw, unpad=unpad, bandlimit=bl,
                                                    mask=out_mask, z_dev=z_dev)
            else:
                x = pend.run() if pend is not None else x
                out = _prop.asm_propagate(x, wl, sp, zs, ph, pw, unpad=unpad, bandlimit=bl, mask=out_mask,
                                          z_dev=z_dev)
        except RuntimeError as err:
            print("##################################################")
            print("An error occurred.  If the error was due to insufficient memory, try decreasing the size of the "
                  "input field or the size of the padding (i.e. decrease 'padding_scale').")
            print("For the best results (e.g. to avoid convolution edge artifacts), the support of the input field "
                  "should be at most 1/2 the size of the input field after padding.")
            print("##################################################")
            raise err
        return out

    def forward(self, field: ElectricField) -> ElectricField:
        """pad -> ft2 -> x H -> ift2 -> crop (Props/ASM_Prop.py:314-378), on the MI355X kernels.
        Inside propagation.deferred_output() the returned field carries the propagation unevaluated
        (_PendingAsm) so the QAT loss can be folded into it.

        One z per call, as the reference: its transfer function exp(i z sqrt(k^2 - K^2)) broadcasts
        a multi-valued z against [1, C, P, P] (:253) and does not give one plane per z.  A z with
        several values raises ValueError naming propagate_planes (all planes in one call) instead of
        propagating only its first value."""
        if len(self._zh) != 1:
            raise ValueError(f"ASM_prop.forward propagates one z-plane; z has {len(self._zh)} values -- use "
                             f"propagate_planes(field, z_list) for [Z, B, C, H, W] in one call")
        if _prop.deferring():
            B, C, H, W = field.shape
            if not (self.do_padding and not self.do_unpad_after_pad):
                Ho, Wo = H, W
            else:
                ph, pw = self.compute_padding(H, W, return_size_of_padding=True)
                Ho, Wo = H + 2 * ph, W + 2 * pw
            # shape-only placeholder (no fill kernel); the data comes from the pending propagation
            holder = torch.empty((), dtype=torch.complex64, device=field.device).expand(B, C, Ho, Wo)
            Eout = ElectricField(data=holder, wavelengths=field.wavelengths, spacing=field.spacing,
                                 device=field.device)._adopt_host(field)
            Eout._pending = _PendingAsm(self, field, self._zh)
            return Eout
        out = self._run(field, self._zh)
        # squeeze, not out[0]: a select's backward materialises a zero [1, B, C, H, W] gradient and
        # copies into it, a squeeze's is a view (one fill and one copy kernel fewer per backward)
        Eout = ElectricField(data=out.squeeze(0), wavelengths=field.wavelengths, spacing=field.spacing,
                             device=field.device)
        return Eout._adopt_host(field)

    def propagate_planes_loss(self, field: ElectricField, z_list, target, z_dev=None):
        """Additive API: propagate_planes fused with the QAT loss of the multi-plane notebooks
        (plot_data/example_2, example_3: the sum over the planes of MSE(normalize(|E_z|^2),
        target_z)) -> (out [Z, B, C, Ho, Wo], loss []).  ``target`` [tB, tC, Ho, Wo] broadcast over
        the Z x B plane-major items (tB in {1, Z B}).  At most THZ_MAX_Z planes."""
        return self._run(field, _z_host(z_list), loss_target=target, z_dev=z_dev)

    def propagate_planes(self, field: ElectricField, z_list, z_dev=None) -> torch.Tensor:
        """Additive API: all planes of ``z_list`` in one call -> [Z, B, C, Ho, Wo].  ``z_dev``
        (float32 device [Z], Z <= THZ_MAX_Z): the kernels read the planes from it instead, so a
        captured graph replays with the values written there before each replay."""
        zs = _z_host(z_list)
        if z_dev is not None:
            return self._run(field, zs, z_dev=z_dev)
        outs = []
        for k in range(0, len(zs), _prop._lib.THZ_MAX_Z):
            outs.append(self._run(field, zs[k:k + _prop._lib.THZ_MAX_Z]))
        return outs[0] if len(outs) == 1 else torch.cat(outs, 0)
