"""The C-ABI library builds, loads without a GPU and exports every symbol include/thzdoe.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "thzdoe.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(thz_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    from quantizationawarethzdoe_amd import _lib
    h = _lib.lib()
    names = _declared()
    assert names, "no declarations parsed"
    for n in names:
        assert hasattr(h, n), f"{n} missing from {_lib.LIB_PATH}"
    assert set(names) == set(_lib.EXPORTED)


def test_version_and_errors_without_gpu():
    from quantizationawarethzdoe_amd import _lib
    assert "gfx950" in _lib.version()
    # argument validation runs on the host and reports through thz_last_error
    d = _lib.AsmDesc(B=0, C=1, H=4, W=4, Z=1)
    n = ctypes.c_size_t(0)
    code = _lib.lib().thz_asm_workspace_size(ctypes.byref(d), ctypes.byref(n))
    assert code == _lib.THZ_E_ARG
    assert b"bad shape" in _lib.lib().thz_last_error()


def test_workspace_and_band_host_logic():
    from quantizationawarethzdoe_amd import propagation as P
    # cfg2 geometry: 4096^2, P=8192, dx=0.25 mm, 300 GHz: evanescent cut keeps ~|ky| <= k
    lam = [2.998e8 / 300e9]
    n = P.asm_band_columns(1, 1, 4096, 4096, 2048, 2048, True, 1, lam, [0.25e-3, 0.25e-3], [0.02, 0.12])
    k = 2 * 3.141592653589793 / lam[0]
    dky = 2 * 3.141592653589793 / (8192 * 0.25e-3)
    assert 2 * int(k / dky) + 1 <= n <= 2 * int(k / dky) + 6
    # dx = lambda: all frequencies propagate -> full band
    assert P.asm_band_columns(1, 1, 100, 100, 100, 100, True, 1, lam, [1e-3, 1e-3], [0.2]) == 300


def test_cpu_tensor_is_rejected():
    import torch
    from quantizationawarethzdoe_amd import propagation as P
    with pytest.raises(RuntimeError, match="ROCm device"):
        P.asm_apply(torch.zeros(1, 1, 8, 8, dtype=torch.complex64), [1e-3], [1e-3, 1e-3], [0.1], 4, 4, True, 1)
