"""MI355X-native hot path of QuantizationAwareTHzDOE.

Sub-packages mirror the reference's module paths (``DataType``, ``Props``,
``Components``, ``LightSource``, ``utils``) so the reference's notebooks can import
this framework unchanged after ``install_reference_aliases()``; the math runs in
the hand-written gfx950 kernels of ``libthzdoe.so`` (``csrc/``) via ``_lib``.
"""
import importlib
import sys

__version__ = "0.4.0"

_ALIASES = ("DataType", "Props", "Components", "LightSource", "utils", "Addons", "VisTools")


_MODULES = ("DataType.ElectricField", "Props.ASM_Prop", "Props.CZT_Prop", "Props.RSC_Prop",
            "Components.QuantizedDOE", "Components.Thin_Lens", "Components.Aperture",
            "LightSource.Gaussian_beam", "Addons.Field_Resampler", "Addons.Field_Crop",
            "utils.units", "utils.Visualization_Helper", "utils.Helper_Functions",
            "VisTools.directions", "VisTools.calc_loss", "VisTools.visualize")


def install_reference_aliases():
    """Make ``from Props.ASM_Prop import ASM_prop`` (the reference's import paths) resolve here.

    Submodules are imported eagerly so every alias names the same module object (one
    ``ElectricField`` class whichever path a caller imports it by).
    """
    for sub in _MODULES:
        try:
            importlib.import_module(f"{__name__}.{sub}")
        except ModuleNotFoundError:
            pass
    for name in _ALIASES:
        mod = importlib.import_module(f"{__name__}.{name}")
        sys.modules[name] = mod
        for sub in list(sys.modules):
            if sub.startswith(f"{__name__}.{name}."):
                sys.modules[sub[len(__name__) + 1:]] = sys.modules[sub]
