"""ctypes binding of libthzdoe.so (include/thzdoe.h).

The shared library is built in-tree by ``quantizationawarethzdoe_amd/csrc/Makefile``
(``__graft_entry__.build()``).  There is NO fallback: if the library is missing or a
symbol is absent, every product entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("THZDOE_LIB", os.path.join(_HERE, "libthzdoe.so"))

THZ_OK = 0
THZ_E_ARG = 1
THZ_E_UNSUPPORTED = 2
THZ_E_WORKSPACE = 3
THZ_E_HIP = 4
THZ_MAX_WAVELENGTHS = 64
THZ_MAX_Z = 256
THZ_ABI_VERSION = 8  # include/thzdoe.h: the descriptor layouts below

BANDLIMIT = {None: 0, False: 0, "none": 0, "exact": 1, "approx": 2}

# every symbol include/thzdoe.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "thz_version", "thz_last_error", "thz_abi_version",
    "thz_asm_workspace_size", "thz_asm_forward", "thz_asm_band", "thz_asm_forward_modulated",
    "thz_asm_forward_loss", "thz_asm_adjoint_loss", "thz_asm_transfer_function", "thz_rs_kernel",
    "thz_czt_workspace_size", "thz_czt_forward",
    "thz_rsc_workspace_size", "thz_rsc_forward",
    "thz_doe_modulate_forward", "thz_doe_modulate_backward", "thz_quant_forward", "thz_quant_backward",
    "thz_doe_quant_backward", "thz_radial_quant_backward",
    "thz_radial_forward", "thz_radial_backward",
    "thz_gaussian_beam", "thz_thin_lens", "thz_aperture",
    "thz_intensity_mse_workspace_size", "thz_intensity_mse_forward", "thz_intensity_mse_backward",
    "thz_resample_forward", "thz_resample_backward",
    "thz_fft_rows",
    "thz_asm64_workspace_size", "thz_asm64_forward", "thz_czt64_workspace_size", "thz_czt64_forward",
    "thz_rsc64_workspace_size", "thz_rsc64_forward", "thz_fft64_rows",
    "thz_step_fetch", "thz_adam_step",
    "thz_timing_enable", "thz_timing_reset", "thz_timing_read",
]


class ThzError(RuntimeError):
    """A libthzdoe call failed; carries the THZ_E_* code."""

    def __init__(self, code, msg):
        super().__init__(f"libthzdoe error {code}: {msg}")
        self.code = code


class AsmDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("pad_h", ctypes.c_int), ("pad_w", ctypes.c_int),
        ("unpad", ctypes.c_int), ("bandlimit", ctypes.c_int), ("Z", ctypes.c_int),
        ("adjoint", ctypes.c_int), ("z_chunk", ctypes.c_int),
        ("dx", ctypes.c_float), ("dy", ctypes.c_float),
        ("wavelengths", ctypes.POINTER(ctypes.c_float)), ("z", ctypes.POINTER(ctypes.c_float)),
        ("window_mask", ctypes.c_void_p),  # const thz_aperture_desc* (ABI 5), NULL = none
        ("z_dev", ctypes.c_void_p),  # const float* device [Z] (ABI 6), NULL = the host z
    ]


class CztDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("outH", ctypes.c_int), ("outW", ctypes.c_int),
        ("dx", ctypes.c_float), ("dy", ctypes.c_float), ("odx", ctypes.c_float), ("ody", ctypes.c_float),
        ("z", ctypes.c_float), ("wavelengths", ctypes.POINTER(ctypes.c_float)), ("adjoint", ctypes.c_int),
    ]


class RscDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("vectorial", ctypes.c_int), ("dx", ctypes.c_float), ("dy", ctypes.c_float), ("z", ctypes.c_float),
        ("wavelengths", ctypes.POINTER(ctypes.c_float)), ("adjoint", ctypes.c_int),
    ]


class AsmDesc64(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("pad_h", ctypes.c_int), ("pad_w", ctypes.c_int),
        ("unpad", ctypes.c_int), ("bandlimit", ctypes.c_int), ("Z", ctypes.c_int), ("adjoint", ctypes.c_int),
        ("dx", ctypes.c_double), ("dy", ctypes.c_double),
        ("wavelengths", ctypes.POINTER(ctypes.c_double)), ("z", ctypes.POINTER(ctypes.c_double)),
    ]


class CztDesc64(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("outH", ctypes.c_int), ("outW", ctypes.c_int),
        ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("odx", ctypes.c_double), ("ody", ctypes.c_double),
        ("z", ctypes.c_double), ("wavelengths", ctypes.POINTER(ctypes.c_double)), ("adjoint", ctypes.c_int),
    ]


class RscDesc64(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("vectorial", ctypes.c_int), ("dx", ctypes.c_double), ("dy", ctypes.c_double), ("z", ctypes.c_double),
        ("wavelengths", ctypes.POINTER(ctypes.c_double)), ("adjoint", ctypes.c_int),
    ]


class DoeDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("hs", ctypes.c_int), ("ws", ctypes.c_int),
        ("tolerance", ctypes.c_float), ("epsilon", ctypes.c_float), ("tand", ctypes.c_float),
        ("wavelengths", ctypes.POINTER(ctypes.c_float)),
        ("rng", ctypes.c_void_p), ("rng_stream", ctypes.c_uint),
    ]


class QuantDesc(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int), ("hq", ctypes.c_int), ("wq", ctypes.c_int), ("mirror", ctypes.c_int),
        ("L", ctypes.c_int), ("lut", ctypes.POINTER(ctypes.c_float)),
        ("hmax", ctypes.c_float), ("clamp", ctypes.c_float), ("tau", ctypes.c_float),
        ("iter_frac", ctypes.c_float), ("c_s", ctypes.c_float), ("s", ctypes.c_float),
        ("beta", ctypes.c_float), ("phase_scale", ctypes.c_float), ("dyn", ctypes.c_void_p),
        ("rng", ctypes.c_void_p), ("rng_stream", ctypes.c_uint),
    ]


class GaussDesc(ctypes.Structure):
    _fields_ = [
        ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("dx", ctypes.c_float), ("dy", ctypes.c_float),
        ("wavelengths", ctypes.POINTER(ctypes.c_float)), ("waist_x", ctypes.POINTER(ctypes.c_float)),
        ("waist_y", ctypes.POINTER(ctypes.c_float)),
        ("x0", ctypes.c_float), ("y0", ctypes.c_float), ("z_w0x", ctypes.c_float), ("z_w0y", ctypes.c_float),
        ("alpha", ctypes.c_float),
    ]


class LensDesc(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
        ("dx", ctypes.c_float), ("dy", ctypes.c_float), ("focal_length", ctypes.c_float),
        ("wavelengths", ctypes.POINTER(ctypes.c_float)),
    ]


class ApertureDesc(ctypes.Structure):
    _fields_ = [
        ("BC", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int), ("kind", ctypes.c_int),
        ("dx", ctypes.c_float), ("dy", ctypes.c_float), ("half_w", ctypes.c_float), ("half_h", ctypes.c_float),
        ("radius", ctypes.c_float),
    ]


class LossDesc(ctypes.Structure):
    _fields_ = [("B", ctypes.c_int), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("tB", ctypes.c_int), ("tC", ctypes.c_int)]


class ResampleDesc(ctypes.Structure):
    _fields_ = [("BC", ctypes.c_int), ("Hin", ctypes.c_int), ("Win", ctypes.c_int), ("Hout", ctypes.c_int),
                ("Wout", ctypes.c_int), ("dx_in", ctypes.c_float), ("dy_in", ctypes.c_float),
                ("dx_out", ctypes.c_float), ("dy_out", ctypes.c_float)]


THZ_MAX_ADAM_PARAMS = 16


class AdamParam(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("step", ctypes.c_void_p), ("n", ctypes.c_longlong)]


class AdamDesc(ctypes.Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("weight_decay", ctypes.c_double), ("decoupled", ctypes.c_int),
                ("nparams", ctypes.c_int),
                ("done", ctypes.c_void_p)]


APERTURE_RECT, APERTURE_CIRC = 1, 2

Q_FP, Q_STE, Q_PSQ, Q_SGV3, Q_NGS, Q_SGV1 = 0, 1, 2, 3, 4, 5
THZ_MAX_LUT = 16

_lib = None
_lock = threading.Lock()


def _declare(lib):
    c_int, c_void_p, c_size_t = ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    lib.thz_version.restype = ctypes.c_char_p
    lib.thz_last_error.restype = ctypes.c_char_p
    lib.thz_asm_workspace_size.argtypes = [ctypes.POINTER(AsmDesc), ctypes.POINTER(c_size_t)]
    lib.thz_asm_forward.argtypes = [ctypes.POINTER(AsmDesc), c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_asm_band.argtypes = [ctypes.POINTER(AsmDesc), ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    lib.thz_asm_forward_modulated.argtypes = [ctypes.POINTER(AsmDesc), ctypes.POINTER(DoeDesc), c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_asm_forward_loss.argtypes = [ctypes.POINTER(AsmDesc), ctypes.POINTER(DoeDesc), c_void_p, c_void_p,
                                         c_void_p, c_void_p, ctypes.POINTER(LossDesc), c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_asm_adjoint_loss.argtypes = [ctypes.POINTER(AsmDesc), ctypes.POINTER(LossDesc), c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_fft_rows.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]
    lib.thz_rsc_workspace_size.argtypes = [ctypes.POINTER(RscDesc), ctypes.POINTER(c_size_t)]
    lib.thz_rsc_forward.argtypes = [ctypes.POINTER(RscDesc), c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_doe_modulate_forward.argtypes = [ctypes.POINTER(DoeDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p]
    lib.thz_doe_modulate_backward.argtypes = [ctypes.POINTER(DoeDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_void_p, c_void_p]
    lib.thz_quant_forward.argtypes = [ctypes.POINTER(QuantDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.thz_quant_backward.argtypes = [ctypes.POINTER(QuantDesc), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.thz_doe_quant_backward.argtypes = [ctypes.POINTER(DoeDesc), ctypes.POINTER(QuantDesc), c_void_p, c_void_p,
                                           c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.thz_radial_quant_backward.argtypes = [ctypes.POINTER(QuantDesc), c_void_p, c_int, c_int, c_int, c_void_p,
                                              c_void_p, c_void_p, c_void_p]
    lib.thz_radial_forward.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]
    lib.thz_radial_backward.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]
    lib.thz_czt_workspace_size.argtypes = [ctypes.POINTER(CztDesc), ctypes.POINTER(c_size_t)]
    lib.thz_czt_forward.argtypes = [ctypes.POINTER(CztDesc), c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]
    lib.thz_gaussian_beam.argtypes = [ctypes.POINTER(GaussDesc), c_void_p, c_void_p]
    lib.thz_thin_lens.argtypes = [ctypes.POINTER(LensDesc), c_void_p, c_void_p, c_void_p]
    lib.thz_aperture.argtypes = [ctypes.POINTER(ApertureDesc), c_void_p, c_void_p, c_void_p]
    lib.thz_asm_transfer_function.argtypes = [ctypes.POINTER(AsmDesc), c_void_p, c_void_p]
    lib.thz_rs_kernel.argtypes = [c_void_p, c_void_p, c_int, ctypes.c_float, c_void_p, c_int, c_void_p, c_void_p]
    lib.thz_intensity_mse_workspace_size.argtypes = [ctypes.POINTER(LossDesc)]
    lib.thz_intensity_mse_forward.argtypes = [ctypes.POINTER(LossDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p]
    lib.thz_intensity_mse_backward.argtypes = [ctypes.POINTER(LossDesc), c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_void_p, c_void_p]
    lib.thz_resample_forward.argtypes = [ctypes.POINTER(ResampleDesc), c_void_p, c_void_p, c_void_p]
    lib.thz_resample_backward.argtypes = [ctypes.POINTER(ResampleDesc), c_void_p, c_void_p, c_void_p]
    for tag, desc in (("asm64", AsmDesc64), ("czt64", CztDesc64), ("rsc64", RscDesc64)):
        getattr(lib, f"thz_{tag}_workspace_size").argtypes = [ctypes.POINTER(desc), ctypes.POINTER(c_size_t)]
        getattr(lib, f"thz_{tag}_forward").argtypes = [ctypes.POINTER(desc), c_void_p, c_void_p, c_void_p, c_size_t,
                                                       c_void_p]
    lib.thz_fft64_rows.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]
    lib.thz_step_fetch.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]
    lib.thz_adam_step.argtypes = [ctypes.POINTER(AdamDesc), ctypes.POINTER(AdamParam), c_void_p]
    lib.thz_timing_enable.argtypes = [c_int]
    lib.thz_timing_reset.argtypes = []
    lib.thz_timing_read.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_long)]
    for name in EXPORTED[2:]:
        getattr(lib, name).restype = c_int
    lib.thz_intensity_mse_workspace_size.restype = c_size_t


def lib():
    """Load (once) and return the ctypes handle; raise loudly if it cannot be loaded."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ThzError(-1, f"{LIB_PATH} not built: run __graft_entry__.build() "
                                       "(make -C quantizationawarethzdoe_amd/csrc)")
                h = ctypes.CDLL(LIB_PATH)
                _declare(h)
                abi = h.thz_abi_version()
                if abi != THZ_ABI_VERSION:
                    raise ThzError(-1, f"{LIB_PATH} has ABI {abi}, these bindings describe ABI {THZ_ABI_VERSION}: "
                                       "rebuild the library (make -C quantizationawarethzdoe_amd/csrc)")
                _lib = h
    return _lib


def check(code):
    if code != THZ_OK:
        raise ThzError(code, lib().thz_last_error().decode())


def version():
    return lib().thz_version().decode()


def timing_enable(on=True):
    check(lib().thz_timing_enable(int(bool(on))))


def timing_reset():
    check(lib().thz_timing_reset())


def timing_read(kernel):
    """(total_ms, launches) of one kernel since the last reset; synchronises pending events."""
    ms, n = ctypes.c_double(0), ctypes.c_long(0)
    check(lib().thz_timing_read(kernel.encode(), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


def double_array(values):
    return (ctypes.c_double * max(1, len(values)))(*[float(v) for v in values])


def float_array(values):
    arr = (ctypes.c_float * max(1, len(values)))(*[float(v) for v in values])
    return arr
