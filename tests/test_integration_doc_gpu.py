"""INTEGRATION.md's ctypes binding (the stub a maintainer adds to the reference) is executable as
written: its asm_forward / asm_adjoint give the package's own results, including the adjoint of
do_unpad_after_pad=False (the padded gradient in, the unpadded field out) and Z > 1 planes."""
import os
import re

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binding():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as fh:
        text = fh.read()
    code = re.search(r"```python\n(# Props/_thzdoe\.py.*?)```", text, re.S).group(1)
    lib = os.path.join(ROOT, "quantizationawarethzdoe_amd", "libthzdoe.so")
    ns = {}
    exec(compile(code.replace('ctypes.CDLL("libthzdoe.so")', f'ctypes.CDLL({lib!r})'), "INTEGRATION.md", "exec"), ns)
    return ns


@pytest.mark.parametrize("unpad", [True, False])
def test_integration_binding_forward_and_adjoint(unpad):
    from quantizationawarethzdoe_amd.propagation import asm_apply
    ns = _binding()
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(7)
    B, C, H, W, ph, pw = 2, 1, 48, 40, 24, 20
    x = torch.from_numpy((rng.standard_normal((B, C, H, W)) + 1j * rng.standard_normal((B, C, H, W)))
                         .astype(np.complex64)).to(dev)
    lam, dx, zs = [1e-3], 1e-3, [0.05, 0.11]
    y = ns["asm_forward"](x, lam, dx, dx, zs, ph, pw, unpad=unpad)
    ref = asm_apply(x, lam, [dx, dx], zs, ph, pw, unpad, 1)
    assert y.shape == ref.shape and torch.equal(y, ref)
    g = torch.randn(y.shape, dtype=torch.complex64, device=dev)
    gx = ns["asm_adjoint"](g, lam, dx, dx, zs, ph, pw, H, W, unpad=unpad)
    assert gx.shape == (B, C, H, W)
    assert torch.equal(gx, asm_apply(g, lam, [dx, dx], zs, ph, pw, unpad, 1, adjoint=True))
    # adjoint identity <A x, g> = <x, A^H g>
    lhs = torch.vdot(y.reshape(-1).to(torch.complex128), g.reshape(-1).to(torch.complex128))
    rhs = torch.vdot(x.reshape(-1).to(torch.complex128), gx.reshape(-1).to(torch.complex128))
    assert abs(complex(lhs - rhs)) <= 1e-5 * abs(complex(lhs))
