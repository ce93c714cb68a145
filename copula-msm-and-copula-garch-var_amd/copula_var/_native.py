"""ctypes binding of libcvq.so (include/cvq.h).

This is the only door to the compute path.  There is no CPU fallback: if the
shared library is missing or no GPU is visible, every product entry point
raises.  (The CPU restatement under ``oracle/`` is test infrastructure and is
never imported from here.)
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CVQ_LIB", os.path.join(_HERE, "libcvq.so"))

CVQ_OK = 0
CVQ_ERR_INVALID = -1
CVQ_ERR_UNSUPPORTED = -2
CVQ_ERR_HIP = -3
CVQ_ERR_OOM = -4
CVQ_ERR_STATE = -5
CVQ_ERR_RANGE = -6
CVQ_ERR_NUMERIC = -7

MEM_HOST, MEM_DEVICE = 0, 1
GAUSSIAN, STUDENT, PLACKETT = 0, 1, 2
MSM, GARCH, UKF = 0, 1, 2
STRATEGY_PREFIX, STRATEGY_DIRECT, STRATEGY_COMPACT, STRATEGY_SORTED, STRATEGY_SWEEP = 0, 1, 2, 3, 4

COPULA_KIND = {"gaussian": GAUSSIAN, "student": STUDENT, "plackett": PLACKETT}
MODEL_KIND = {"msm": MSM, "garch": GARCH, "mean_reverting": UKF, "ukf": UKF}

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class CvqStatic(C.Structure):
    _fields_ = [
        ("model", C.c_int32), ("copula", C.c_int32), ("dim", C.c_int32), ("n", C.c_int32),
        ("q", C.c_int32), ("n_combos", C.c_int32),
        ("x_values", _dp), ("step", _dp), ("densities", _dp), ("combos", _ip), ("weights", _dp),
        ("vol_states", _dp), ("copula_params", _dp), ("n_copula_params", C.c_int32),
        ("strategy", C.c_int32), ("v_cap", C.c_double),
    ]


class CvqSolveArgs(C.Structure):
    _fields_ = [(name, C.c_double) for name in (
        "obj_var", "first_guess", "second_guess_lo", "second_guess_hi", "min_var", "max_var",
        "lower", "tolerance", "ptf_mean")]


class NativeError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {msg} (cvq status {code})")
        self.code = code


_lib: Optional[C.CDLL] = None


def _declare(lib: C.CDLL) -> None:
    v, i32, i64, d = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    sig = {
        "cvq_last_error": (C.c_char_p, []),
        "cvq_version": (i32, []),
        "cvq_device_count": (i32, [_ip]),
        "cvq_plan_create": (i32, [C.POINTER(CvqStatic), i32, C.POINTER(v)]),
        "cvq_plan_destroy": (i32, [v]),
        "cvq_plan_set_stream": (i32, [v, v]),
        "cvq_plan_info": (i32, [v, C.POINTER(i64), _ip]),
        "cvq_plan_timing": (i32, [v, i32]),
        "cvq_plan_kernel_time": (i32, [v, i32, C.POINTER(d), _ip]),
        "cvq_plan_debug_stamps": (i32, [v, v, i64]),
        "cvq_plan_debug_nodes": (i32, [v, v, i64, v]),
        "cvq_plan_debug_cuts": (i32, [v, v, i64, v]),
        "cvq_plan_count_nodes": (i32, [v, i32]),
        "cvq_plan_nodes_evaluated": (i32, [v, C.POINTER(i64)]),
        "cvq_set_dates": (i32, [v, i64, v, v, i32]),
        "cvq_set_fast_hint": (i32, [v, i32]),
        "cvq_slab": (i32, [v, v, v, i32]),
        "cvq_solve": (i32, [v, C.POINTER(CvqSolveArgs), v, _ip, i32]),
        "cvq_snap_stride": (i32, [C.POINTER(CvqSolveArgs), _ip]),
        "cvq_solve_status": (i32, [v, _ip]),
        "cvq_packed_block_len": (i32, [C.POINTER(CvqSolveArgs), i64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "cvq_solve_finalize_packed": (i32, [v, C.POINTER(CvqSolveArgs), v, i32, i64, i64, v]),
        "cvq_solve_local": (i32, [v, C.POINTER(CvqSolveArgs), v, v]),
        "cvq_solve_finalize": (i32, [v, C.POINTER(CvqSolveArgs), v, i32, v, i64, i64, v]),
        "cvq_msm_filter": (i32, [i32, i32, d, d, d, d, v, i64, i64, v, i32]),
        "cvq_msm_marginals": (i32, [i32, i32, d, d, d, d, v, i64, v, v, i32]),
        "cvq_msm_tables_scratch": (i32, [i32, i32, i64, i64, C.POINTER(C.c_int64)]),
        "cvq_msm_tables": (i32, [i32, v, i32, i32, v, v, i32, v, i64, i64, v, v, v]),
        "cvq_msm_tables_status": (i32, [v, i32, i32, i64, i64, v]),
        "cvq_sigma_tables": (i32, [i32, v, i32, i32, v, v, v, i64, i64, v, v]),
        "cvq_sigma_tables_status": (i32, [v, v]),
        "cvq_garch_forecast": (i32, [i32, d, d, d, v, i64, i64, v, i32]),
        "cvq_ukf_forecast": (i32, [i32, d, d, d, v, i64, i64, v, i32]),
        "cvq_garch_forecast_pq": (i32, [i32, i32, i32, v, v, i64, i64, v, i32]),
        "cvq_msm_loglik": (i32, [i32, i32, v, i64, v, i64, v, i32]),
        "cvq_garch_loglik": (i32, [i32, v, i64, v, i64, v, i32]),
        "cvq_garch_loglik_pq": (i32, [i32, i32, i32, v, i64, v, i64, v, i32]),
        "cvq_ukf_loglik": (i32, [i32, v, i64, v, i64, v, i32]),
        "cvq_ukf_filter": (i32, [i32, v, i64, v, i32, i64, v, v, i32]),
        "cvq_special": (i32, [i32, i32, d, v, i64, v, i32]),
    }
    for name, (res, args) in sig.items():
        if name == "cvq_plan_debug_stamps" and not hasattr(lib, name):
            continue                                   # diagnostic-only symbol (older builds)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args


def lib() -> C.CDLL:
    """Load libcvq.so (raises if it is missing -- there is no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libcvq.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C copula-msm-and-copula-garch-var_amd`; the VaR engine has no CPU fallback")
        # One HIP runtime per process: torch (the device buffers, streams and RCCL around this
        # library) ships its own libamdhip64.  Loaded after libcvq's (/opt/rocm), torch finds no
        # GPU ("No HIP GPUs are available"); loaded first, libcvq binds to it.  So import torch
        # before the library when it is installed.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = C.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def check(code: int, where: str) -> None:
    if code == CVQ_OK:
        return
    msg = (lib().cvq_last_error() or b"").decode(errors="replace")
    if code in (CVQ_ERR_INVALID, CVQ_ERR_UNSUPPORTED, CVQ_ERR_RANGE):
        raise ValueError(f"{where}: {msg}")
    raise NativeError(code, where, msg)


def device_count() -> int:
    n = C.c_int32(0)
    check(lib().cvq_device_count(C.byref(n)), "cvq_device_count")
    return int(n.value)


def require_gpu() -> None:
    if device_count() < 1:
        raise RuntimeError("no HIP device visible: the copula-VaR engine runs on MI355X only (no CPU fallback)")


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


def special(fn: str, x, nu: float = 0.0, device: int = 0) -> np.ndarray:
    """Device t.ppf / norm.ppf / erf (known-answer tests); "tppf6": the solve kernels'
    integer-nu t.ppf (nu = 6)."""
    code = {"tppf": 0, "ndtri": 1, "erf": 2, "tppf6": 3}[fn]
    xx = f64(x).ravel()
    out = np.empty_like(xx)
    check(lib().cvq_special(device, code, float(nu), ptr(xx), xx.size, ptr(out), MEM_HOST), f"cvq_special({fn})")
    return out.reshape(np.shape(x))
