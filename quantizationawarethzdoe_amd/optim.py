"""The trainers' optimiser: Adam / AdamW as one HIP kernel per step (thz_adam_step).

The reference's notebooks step ``torch.optim.Adam`` (the score-Gumbel and PSQ runs, the DONN) and
``torch.optim.AdamW`` with its defaults (the full-precision, naive-Gumbel and STE runs;
plot_data/example_1/experiment_four_focal_spots.ipynb cells 22, 33, 52, example_2 / example_3).
These classes take the same constructor arguments and keep the same per-parameter state
(``step`` as a device fp32 tensor -- torch's capturable form -- ``exp_avg``, ``exp_avg_sq``), so a
graph-captured step replays them like torch's capturable optimisers.  The difference is the launch
count: torch's fused capturable path issues a step-count kernel and an update kernel per parameter
group; here every parameter of the optimiser is one launch that also advances the step counts.
The arithmetic is torch's single-tensor (and foreach) Adam's: fp32 element updates (lerp for the
first moment, addcmul for the second, addcdiv for the parameter) with the scalars formed in fp64
and rounded to fp32, as torch forms them in Python -- the bias corrections in fp64 on the device.

Plain fp32 CUDA parameters only (no amsgrad, maximize, or sparse gradients): anything else raises.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .propagation import _stream_handle


class _ThzAdamBase(torch.optim.Optimizer):
    _decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False,
                 maximize=False, foreach=None, fused=None, capturable=None, differentiable=False):
        # foreach / fused / capturable: torch's implementation choices, all the same one launch here
        if amsgrad or maximize or differentiable:
            raise ValueError("thz Adam: amsgrad / maximize / differentiable are not supported")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= weight_decay:
            raise ValueError(f"invalid lr / eps / weight_decay: {lr}, {eps}, {weight_decay}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"invalid betas: {betas}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._done = {}

    def _state(self, p):
        st = self.state[p]
        if not st:
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        else:
            # a loaded state_dict (e.g. torch.optim.Adam's, whose non-capturable step count stays on
            # the host): the kernel reads every state tensor on the parameter's device, fp32, dense
            for k in ("step", "exp_avg", "exp_avg_sq"):
                v = st[k]
                if not torch.is_tensor(v):
                    v = torch.tensor(float(v))
                if v.device != p.device or v.dtype != torch.float32 or not v.is_contiguous():
                    st[k] = v.to(device=p.device, dtype=torch.float32).contiguous()
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            for p in ps:
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous() and p.grad.is_contiguous()
                        and not p.grad.is_sparse and p.grad.dtype == torch.float32):
                    raise ValueError("thz Adam: contiguous fp32 device parameters and gradients only")
            by_dev = {}
            for p in ps:  # one launch reads one device's memory
                by_dev.setdefault(p.device, []).append(p)
            for dps in by_dev.values():
                for k in range(0, len(dps), _lib.THZ_MAX_ADAM_PARAMS):
                    self._launch(group, dps[k:k + _lib.THZ_MAX_ADAM_PARAMS])
        return loss

    def _launch(self, group, ps):
        dev = ps[0].device
        done = self._done.get(dev)
        if done is None:  # the kernel's finished-workgroup count (it leaves it zero)
            done = self._done[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
        arr = (_lib.AdamParam * len(ps))()
        for a, p in zip(arr, ps):
            st = self._state(p)
            a.param, a.grad = p.data_ptr(), p.grad.data_ptr()
            a.exp_avg, a.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            a.step, a.n = st["step"].data_ptr(), p.numel()
        b1, b2 = group["betas"]
        d = _lib.AdamDesc(lr=float(group["lr"]), beta1=float(b1), beta2=float(b2), eps=float(group["eps"]),
                          weight_decay=float(group["weight_decay"]), decoupled=int(self._decoupled),
                          nparams=len(ps), done=done.data_ptr())
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().thz_adam_step(ctypes.byref(d), arr, _stream_handle()))


class Adam(_ThzAdamBase):
    """torch.optim.Adam's update (L2 weight decay added to the gradient), one launch per step."""


class AdamW(_ThzAdamBase):
    """torch.optim.AdamW's update (decoupled weight decay, default 0.01), one launch per step."""
    _decoupled = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, **kw):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, **kw)
