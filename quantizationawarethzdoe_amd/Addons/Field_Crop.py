"""Field cropper -- drop-in for the reference's Addons/Field_Crop.py.

Centre crop [..., top:top+h, left:left+w] with top = int(round(H - h) / 2.0) (:50-67): a
strided view of the device tensor (no data movement, as in the reference), not a kernel.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from quantizationawarethzdoe_amd.DataType.ElectricField import ElectricField


class Field_Cropper(nn.Module):
    def __init__(self, outputHeight: int, outputWidth: int, device: torch.device = None) -> None:
        super().__init__()
        self.device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        if (type(outputHeight) is not int) or (outputHeight <= 0):
            raise Exception("Bad argument: 'outputHeight' should be a positive integer.")
        if (type(outputWidth) is not int) or (outputWidth <= 0):
            raise Exception("Bad argument: 'outputWidth' should be a positive integer.")
        self.outputHeight = outputHeight
        self.outputWidth = outputWidth

    def forward(self, field: ElectricField) -> ElectricField:
        _, _, Hf, Wf = field.data.shape
        top = int(round(Hf - self.outputHeight) / 2.0)
        left = int(round(Wf - self.outputWidth) / 2.0)
        data = field.data[:, :, top:top + self.outputHeight, left:left + self.outputWidth]
        return ElectricField(data=data, wavelengths=field.wavelengths, spacing=field.spacing,
                             device=field.device)._adopt_host(field)
