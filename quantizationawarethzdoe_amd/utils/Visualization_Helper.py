"""Plot helpers the DOE layers' ``visualize`` uses (reference utils/Visualization_Helper.py:13-49).

Host-side only (matplotlib); imported lazily so the compute path never needs a display stack.
"""
import numpy as np

from .units import m, mm, nm, um


def float_to_unit_identifier(val):
    """(10**(3k), unit name) of the engineering range of ``val`` (e.g. 55 mm -> (1e-3, "mm"))."""
    exponent = np.floor(np.log10(val) / 3)
    unit_val = 10 ** (3 * exponent)
    names = {m: "m", mm: "mm", um: "um", nm: "nm"}
    unit = next((n for v, n in names.items() if np.isclose(unit_val, v, rtol=1e-9, atol=0)), None)
    return unit_val, unit


def add_colorbar(mappable):
    from mpl_toolkits.axes_grid1 import make_axes_locatable
    import matplotlib.pyplot as plt

    last_axes = plt.gca()
    ax = mappable.axes
    cax = make_axes_locatable(ax).append_axes("right", size="5%", pad=0.05)
    cbar = ax.figure.colorbar(mappable, cax=cax)
    plt.sca(last_axes)
    return cbar
