"""Loss-landscape plots -- drop-in for the reference's VisTools/visualize.py:63-121
(``visualize_notebook``, what experiment_vis_loss_landscape.ipynb calls after the sweep).

Reads the surface file calc_loss writes (npz here: h5py is absent from this image, so the sweep
stores xcoordinates / ycoordinates / <surf_name> in ``3d_surface_file.npz``) and draws the same
figures: contour lines, filled contours, a heat map (matplotlib ``imshow``; the reference uses
seaborn, also absent) and the 3-D surface at the reference's four viewing angles.  Host-side
plotting only; nothing here touches the device.
"""
from __future__ import annotations

import os

import numpy as np


def _load_surface(surface_path, surf_name):
    with np.load(surface_path, allow_pickle=False) as f:
        x = np.array(f["xcoordinates"])
        y = np.array(f["ycoordinates"])
        X, Y = np.meshgrid(x, y)
        if surf_name in f.files:
            Z = np.array(f[surf_name])
        else:
            print(f"{surf_name} is not found in {surface_path}")
            Z = np.zeros_like(X)
    return X, Y, Z


def visualize_notebook(args, save_path, surface_path):
    """The reference's notebook figures for ``args.surf_name`` of ``surface_path`` (:63-121); creates
    ``<save_path>/2D_images/`` as the reference does and returns the figures."""
    import matplotlib.pyplot as plt
    os.makedirs(os.path.join(save_path, "2D_images"), exist_ok=True)
    X, Y, Z = _load_surface(surface_path, args.surf_name)
    print(Z.min())
    figs = []
    levels = np.arange(Z.min(), Z.max(), (Z.max() - Z.min()) / 10) if Z.max() > Z.min() else None
    for filled, title in ((False, "Contour Plot"), (True, "Filled Contour Plot")):
        fig = plt.figure()
        if levels is not None:
            CS = (plt.contourf if filled else plt.contour)(X, Y, Z, cmap="summer", levels=levels)
            if not filled:
                plt.clabel(CS, inline=1, fontsize=8)
            plt.colorbar(CS)
        plt.title(title)
        figs.append(fig)
    fig = plt.figure()
    plt.imshow(Z, cmap="viridis")
    plt.colorbar()
    plt.xticks([])
    plt.yticks([])
    plt.title("Heatmap")
    figs.append(fig)
    for elev, azim in [(30, 30), (45, 30), (60, 30), (60, 30)]:
        fig = plt.figure()
        ax = fig.add_subplot(111, projection="3d")
        ax.plot_surface(X, Y, Z, cmap="viridis", linewidth=0, antialiased=True)
        ax.set_title("3D Surface Plot")
        ax.view_init(elev=elev, azim=azim)
        plt.title(f"Elevation: {elev}, Azimuth: {azim}")
        figs.append(fig)
    plt.show()
    return figs
