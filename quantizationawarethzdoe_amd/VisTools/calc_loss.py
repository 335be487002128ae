"""Loss-landscape sweep of a single-DOE system -- drop-in for the reference's
VisTools/calc_loss.py:8-106 (``calulate_single_element_loss_landscape``, the name kept with its
spelling), SURVEY.md §8(f)4.

For every grid point (alpha, beta) of linspace(xmin, xmax, xnum) x linspace(ymin, ymax, ynum) the
weights are set to theta* + alpha d_x + beta d_y (``overwrite_weights``, :96-103) and the system is
evaluated once at iter_frac = 1: loss = loss_f(|E|^2 / max |E|^2, target) (:36-40).  Each grid
point is an independent forward pass on the HIP kernels, so the sweep shards over ranks with no
data-path collective: rank r takes a contiguous block of the unfinished points, keeps its losses on
the device (no per-point host sync, where the reference calls .item() and rewrites the file per
point) and the blocks meet in one all_gather at the end; rank 0 writes the surface file.

Surface file: the reference writes h5 (``3d_surface_file.h5`` with xcoordinates, ycoordinates,
loss; :61-82).  h5py is absent from this image, so the same three arrays go to
``3d_surface_file.npz``.  Index quirk kept: losses has shape (xnum, ynum) but the coordinates of
flat index i come from meshgrid(x, y) (shape (ynum, xnum)), as in get_indices (:85-93).
"""
from __future__ import annotations



import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn


def setup_surface_file(args, save_path):
    """Fresh surface file with loss = -1 everywhere (:61-82); returns its path."""
    surface_path = f"{save_path}/3d_surface_file.npz"
    if _rank() == 0:
        print("Create new 3d_sureface_file.npz")
        x = np.linspace(args.xmin, args.xmax, args.xnum)
        y = np.linspace(args.ymin, args.ymax, args.ynum)
        np.savez(surface_path, xcoordinates=x, ycoordinates=y, loss=-np.ones((len(x), len(y))))
    if _world() > 1:
        dist.barrier()
    return surface_path


def get_indices(vals, xcoordinates, ycoordinates):
    """Flat indices of the unfinished points (loss <= 0) and their (x, y) coordinates (:85-93)."""
    inds = np.array(range(vals.size))
    inds = inds[vals.ravel() <= 0]
    xm, ym = np.meshgrid(xcoordinates, ycoordinates)
    return inds, np.c_[xm.ravel()[inds], ym.ravel()[inds]]


def overwrite_weights(model, init_weights, directions, step):
    """theta = theta* + step[0] d_x + step[1] d_y (:96-103)."""
    dx, dy = directions[0], directions[1]
    changes = [d0 * step[0] + d1 * step[1] for (d0, d1) in zip(dx, dy)]
    for (p, w, d) in zip(model.parameters(), init_weights, changes):
        p.data = w + d


def _world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def _rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def shard(n, rank, world):
    """Contiguous block of range(n) of one rank (every index exactly once)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def calulate_single_element_loss_landscape(args, model, target, loss_f=nn.MSELoss(), directions=None,
                                           save_path=None):
    """Evaluate the loss on the (xnum x ynum) grid around the current weights; returns the path of
    the surface file (rank 0 writes it; every rank gets the path)."""
    surface_path = setup_surface_file(args, save_path)
    init_weights = [p.data for p in model.parameters()]
    with np.load(surface_path) as f:
        x, y, losses = f["xcoordinates"], f["ycoordinates"], f["loss"].copy()
    inds, coords = get_indices(losses, x, y)
    rank, world = _rank(), _world()
    lo, hi = shard(len(inds), rank, world)
    dev = next(model.parameters()).device
    mine = torch.zeros(hi - lo, dtype=torch.float64, device=dev)
    with torch.no_grad():
        for k in range(lo, hi):
            overwrite_weights(model, init_weights, directions, coords[k])
            out = torch.abs(model.forward(iter_frac=1).data) ** 2
            out = out / torch.max(out)
            mine[k - lo] = loss_f(out, target).detach().double()
    got = mine.cpu().numpy()
    if world > 1:
        parts = [None] * world
        dist.all_gather_object(parts, (lo, got))
    else:
        parts = [(lo, got)]
    if rank == 0:
        for start, vals in parts:
            losses.ravel()[inds[start:start + len(vals)]] = vals
        np.savez(surface_path, xcoordinates=x, ycoordinates=y, loss=losses)
    if world > 1:
        dist.barrier()
    return surface_path


def calulate_DONN_loss_landscape(args, model, directions=None, save_path=None):
    """Not implemented in the reference either (:55-61)."""
    pass


def load_surface(surface_path):
    """(xcoordinates, ycoordinates, loss) of a surface file."""
    with np.load(surface_path) as f:
        return f["xcoordinates"], f["ycoordinates"], f["loss"]


__all__ = ["setup_surface_file", "get_indices", "overwrite_weights", "calulate_single_element_loss_landscape",
           "calulate_DONN_loss_landscape", "load_surface", "shard"]

