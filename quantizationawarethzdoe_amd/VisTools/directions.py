"""Random filter-normalised directions in weight space for the loss-landscape sweep -- the part of
the reference's VisTools/directions.py the sweep uses (:73-117): one Gaussian tensor per
parameter, rescaled to that parameter's norm (Li et al. 2018, "Visualizing the Loss Landscape of
Neural Nets"); parameters of dimension <= 1 get a zero direction.  The PCA-direction tooling of the
reference (:165-269, sklearn + h5 files) is not part of the propagation hot path and is not built.
"""
from __future__ import annotations

import torch


def get_weights(model):
    """Parameters of ``model`` as a list of tensors (:84-86)."""
    return [p.data for p in model.parameters()]


def get_random_weights(weights, generator=None):
    """One standard-normal tensor per weight, on the weight's device (:94-99)."""
    return [torch.randn(w.size(), generator=generator).to(w.device) for w in weights]


def normalize_direction(direction, weights):
    """d_i *= |w_i| / (|d_i| + 1e-10) for each pair (:102-104).  The reference calls it with one
    parameter's direction and weight tensors (:111), so the pairs are their slices along dim 0:
    every filter (row) of d is scaled to the norm of the matching row of w (Li et al.'s
    filter-wise normalisation)."""
    for d, w in zip(direction, weights):
        d.mul_(w.norm() / (d.norm() + 1e-10))


def normalize_directions_for_weights(direction, weights):
    """(:106-111): 0- and 1-d parameters get a zero direction, the rest are normalised filter by
    filter (slices along dim 0) as the reference's ``normalize_direction(d, w)`` does."""
    assert len(direction) == len(weights)
    for d, w in zip(direction, weights):
        if d.dim() <= 1:
            d.fill_(0)
            continue
        normalize_direction(d, w)


def create_random_direction(model, generator=None):
    weights = get_weights(model)
    direction = get_random_weights(weights, generator)
    normalize_directions_for_weights(direction, weights)
    return direction


def create_random_directions(model, generator=None):
    """[x_direction, y_direction] (:73-77)."""
    return [create_random_direction(model, generator), create_random_direction(model, generator)]
