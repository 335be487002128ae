"""ElectricField: the [B, C, H, W] complex field container of the hot path.

API mirror of the reference container (DataType/ElectricField.py:14-440): same
constructor, properties (``data``, ``wavelengths``, ``spacing``, ``shape``,
``height``, ``width``, ``num_wavelengths``, ``Ex/Ey/Ez``), validation rules
(``check_spacing`` :76-83 casts float/list spacing to fp32, ``check_wavelengths``
:85-90 casts float/list wavelengths to fp32 and keeps tensor dtypes, ``check_data``
:92-109 demands 4-D data with C == len(wavelengths) and sets ``field_type`` from B)
and error types (ValueError / AssertionError).

MI355X addition: the container keeps HOST copies of the wavelengths and spacing
(``wavelengths_host`` / ``spacing_host``) so the propagator kernels receive their
physical scalars as kernel arguments without a device->host sync per call.
"""
from __future__ import annotations

from typing import Union

import torch


def _host_values(t: torch.Tensor):
    return [float(v) for v in t.detach().to("cpu").reshape(-1).tolist()]


class ElectricField:
    _BATCH = 0
    _WAVELENGTH = 1
    _HEIGHT = 2
    _WIDTH = 3
    # MI355X addition: a DOE layer's output may carry its modulation unevaluated (doe.PendingModulation);
    # the next ASM_prop then applies it inside its row pass, anything else that reads .data forms it.
    # Inside propagation.deferred_output() an ASM_prop output carries its propagation unevaluated
    # (Props.ASM_Prop._PendingAsm) so the QAT loss can be folded into it (optics.field_intensity_mse).
    _pending = None

    def __init__(self, data: torch.Tensor, wavelengths: Union[torch.Tensor, float] = None,
                 spacing: Union[torch.Tensor, float] = None, requires_grad: bool = None, device=None):
        self.device = device or torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self._spacing = self.check_spacing(spacing)
        self._wavelengths = self.check_wavelengths(wavelengths)
        self.field_type = None
        if data is None:
            data = torch.empty(1, len(self._wavelengths), 1, 1)
        self._data = self.check_data(data)

    # -- properties (DataType/ElectricField.py:48-74) -----------------------------------------
    @property
    def spacing(self) -> torch.Tensor:
        return self._spacing

    @spacing.setter
    def spacing(self, spacing):
        self._spacing = self.check_spacing(spacing)

    @property
    def wavelengths(self):
        return self._wavelengths

    @wavelengths.setter
    def wavelengths(self, wavelengths):
        self._wavelengths = self.check_wavelengths(wavelengths)

    @property
    def requires_grad(self):
        return self.data.requires_grad

    @property
    def data(self) -> torch.Tensor:
        if self._pending is not None:
            pend, self._pending = self._pending, None
            self._data = pend.run()
        return self._data

    @data.setter
    def data(self, data):
        self._pending = None
        self._data = self.check_data(data)

    def _take_pending(self):
        """The unevaluated modulation this field carries (None once its data has been formed)."""
        p = self._pending
        return p if getattr(p, "kind", None) == "modulation" else None

    def _take_pending_propagation(self):
        """The deferred ASM_prop.forward this field is the output of (propagation.deferred_output),
        detached from the field: the caller forms the data (and sets it) itself."""
        p = self._pending
        if getattr(p, "kind", None) != "propagation":
            return None
        self._pending = None
        return p

    # -- host mirrors of the physical scalars (MI355X addition) --------------------------------
    @property
    def wavelengths_host(self):
        if getattr(self, "_wl_host_src", None) is not self._wavelengths:
            self._wl_host = _host_values(self._wavelengths)
            self._wl_host_src = self._wavelengths
        return self._wl_host

    @property
    def spacing_host(self):
        if getattr(self, "_sp_host_src", None) is not self._spacing:
            self._sp_host = _host_values(self._spacing)
            self._sp_host_src = self._spacing
        return self._sp_host

    def _adopt_host(self, other: "ElectricField") -> "ElectricField":
        """Carry the host scalar mirrors over from ``other`` when the tensors are shared."""
        if getattr(other, "_wl_host_src", None) is other._wavelengths and self._wavelengths is other._wavelengths:
            self._wl_host, self._wl_host_src = other._wl_host, self._wavelengths
        if getattr(other, "_sp_host_src", None) is other._spacing and self._spacing is other._spacing:
            self._sp_host, self._sp_host_src = other._sp_host, self._spacing
        return self

    # -- validation (DataType/ElectricField.py:76-109) ----------------------------------------
    def check_spacing(self, spacing):
        host = None
        if isinstance(spacing, (list, tuple)) and len(spacing) == 2:
            spacing = torch.tensor(spacing, dtype=torch.float32)
            host = spacing
        elif isinstance(spacing, (float, int)):
            spacing = torch.tensor([spacing, spacing], dtype=torch.float32)
            host = spacing
        if not torch.is_tensor(spacing) or spacing.numel() != 2:
            raise ValueError("Spacing must be a 2-element tensor.")
        out = spacing.to(self.device)
        if host is not None or spacing.device.type == "cpu":
            self._sp_host = _host_values(spacing)
            self._sp_host_src = out
        return out

    def check_wavelengths(self, wavelengths):
        host = None
        if isinstance(wavelengths, (list, float, int)):
            wavelengths = torch.tensor([wavelengths] if isinstance(wavelengths, (float, int)) else wavelengths,
                                       dtype=torch.float32)
            host = wavelengths
        if not torch.is_tensor(wavelengths):
            raise ValueError("Wavelengths must be a tensor.")
        out = wavelengths.to(self.device)
        if host is not None or wavelengths.device.type == "cpu":
            self._wl_host = _host_values(wavelengths)
            self._wl_host_src = out
        return out

    def check_data(self, data):
        assert torch.is_tensor(data) and data.ndim == 4, \
            "Data must be a 4D torch tensor with BATCH x Channel (Wavelength) x Height x Width"
        if data.shape[self._WAVELENGTH] != len(self._wavelengths):
            raise ValueError("The number of channels in data should be equal to the number of wavelengths")
        if data.shape[self._BATCH] == 1:
            self.field_type = "scalar"
        elif data.shape[self._BATCH] == 3:
            self.field_type = "vectorial"
        else:
            self.field_type = "batch"
        return data.to(self.device)

    # -- derived fields (DataType/ElectricField.py:112-167) -----------------------------------
    def _like(self, data, wavelengths=None, spacing=None):
        f = ElectricField(data=data, wavelengths=self._wavelengths if wavelengths is None else wavelengths,
                          spacing=self._spacing if spacing is None else spacing, device=self.device)
        return f._adopt_host(self)

    def abs(self) -> "ElectricField":
        return self._like(self.data.abs())

    def angle(self) -> "ElectricField":
        return self._like(self.data.angle())

    def detach(self) -> "ElectricField":
        return self._like(self.data.detach(), self._wavelengths.detach(), self._spacing.detach())

    def cpu(self) -> "ElectricField":
        return ElectricField(data=self.data.cpu(), wavelengths=self._wavelengths.detach(),
                             spacing=self._spacing.detach(), device=self.device)

    # -- shape accessors (DataType/ElectricField.py:169-203) ----------------------------------
    @property
    def ndim(self):
        return self._data.ndim

    @property
    def shape(self):
        return self._data.shape

    @property
    def num_batches(self):
        return self.shape[self._BATCH]

    @property
    def num_wavelengths(self):
        return self.shape[self._WAVELENGTH]

    @property
    def height(self):
        return self.shape[self._HEIGHT]

    @property
    def width(self):
        return self.shape[self._WIDTH]

    @property
    def Ex(self):
        return self.data[[0], ...]

    @property
    def Ey(self):
        return self.data[[1], ...]

    @property
    def Ez(self):
        return self.data[[2], ...]

    def _get_data_for_wavelength(self, wavelength):
        idx = (self._wavelengths == wavelength).nonzero()[0]
        return self.data[:, idx, ...]

    def visualize(self, flag_colorbar: bool = True, flag_axis: str = True, cmap="viridis", wavelength=None,
                  figsize=(8, 8), intensity=True):
        """Intensity/amplitude + phase plot for one wavelength (plotting, off the hot path)."""
        assert wavelength is not None, "Wavelength must be specified."
        import matplotlib.pyplot as plt
        data = self._get_data_for_wavelength(wavelength).detach().cpu().squeeze()
        if data.ndim > 2:
            data = data[0]
        fig = plt.figure(figsize=figsize)
        ax1 = fig.add_subplot(1, 2, 1)
        im = ax1.imshow((data.abs() ** 2) if intensity else data.abs(), cmap=cmap)
        ax1.set_title("Intensity" if intensity else "Amplitude")
        if flag_colorbar:
            fig.colorbar(im, ax=ax1)
        ax2 = fig.add_subplot(1, 2, 2)
        im2 = ax2.imshow(data.angle(), cmap=cmap)
        ax2.set_title("Phase")
        if flag_colorbar:
            fig.colorbar(im2, ax=ax2)
        if not flag_axis:
            ax1.axis("off")
            ax2.axis("off")
        plt.tight_layout()
        return fig
