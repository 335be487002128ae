"""Import the read-only reference tree in-process, for fixture generation ONLY.

This module is used by ``gen_golden.py`` in the build container, never by the
product, the GPU tests, ``smoke()`` or ``bench.py`` (``/root/reference`` does not
exist on the GPU box).  It installs two tiny ``sys.modules`` stand-ins for
third-party packages the reference imports but that are absent from the image
(SURVEY.md §8(c)):

* ``imageio`` -- imported but unused (reference ``utils/Visualization_Helper.py:7``);
* ``torchvision`` -- used only for ``transforms.CenterCrop`` at
  ``Props/ASM_Prop.py:360``.  The stand-in implements torchvision's published
  crop rule ``top = int(round((H - h) / 2))`` on the last two dims.

No reference source is copied; the reference modules are imported from
``/root/reference`` directly with bytecode writing disabled (read-only tree).
"""
import os
import sys
import types

REF = os.environ.get("THZ_REFERENCE", "/root/reference")


def _install_stubs():
    if "imageio" not in sys.modules:
        sys.modules["imageio"] = types.ModuleType("imageio")
    if "torchvision" not in sys.modules:
        tv = types.ModuleType("torchvision")
        tr = types.ModuleType("torchvision.transforms")

        class CenterCrop:
            def __init__(self, size):
                self.size = (size, size) if isinstance(size, int) else tuple(size)

            def __call__(self, x):
                h, w = int(self.size[0]), int(self.size[1])
                H, W = x.shape[-2], x.shape[-1]
                top = int(round((H - h) / 2.0))
                left = int(round((W - w) / 2.0))
                return x[..., top:top + h, left:left + w]

        tr.CenterCrop = CenterCrop
        tv.transforms = tr
        sys.modules["torchvision"] = tv
        sys.modules["torchvision.transforms"] = tr


def import_reference():
    """Return a namespace with the reference modules needed for fixtures."""
    if not os.path.isdir(REF):
        raise SystemExit(f"reference tree {REF} is absent: fixtures are generated only in the build container")
    sys.dont_write_bytecode = True
    _install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib
    ns = types.SimpleNamespace()
    ns.ElectricField = importlib.import_module("DataType.ElectricField").ElectricField
    ns.ASM = importlib.import_module("Props.ASM_Prop")
    ns.CZT = importlib.import_module("Props.CZT_Prop")
    ns.RSC = importlib.import_module("Props.RSC_Prop")
    ns.DOE = importlib.import_module("Components.QuantizedDOE")
    ns.GB = importlib.import_module("LightSource.Gaussian_beam")
    ns.HF = importlib.import_module("utils.Helper_Functions")
    ns.import_module = importlib.import_module
    ns.root = REF
    return ns
