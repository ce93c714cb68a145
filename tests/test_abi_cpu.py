"""The C-ABI boundary without a GPU: libcvq.so loads, exports every function
include/cvq.h declares, the ctypes mirrors match the header's structs, and
argument validation that happens before any device work returns the
documented status codes."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "cvq.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cvq_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_entry_points():
    names = _declared()
    for must in ("cvq_plan_create", "cvq_set_dates", "cvq_slab", "cvq_solve", "cvq_solve_local",
                 "cvq_solve_finalize", "cvq_msm_filter", "cvq_garch_forecast", "cvq_ukf_forecast",
                 "cvq_special", "cvq_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from copula_var import _native as N
    lib = C.CDLL(N.LIB_PATH)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_declares_every_symbol():
    """_native._declare binds exactly the header's entry points."""
    import inspect
    from copula_var import _native as N
    src = inspect.getsource(N._declare)
    bound = set(re.findall(r'"(cvq_[a-z0-9_]+)"', src))
    assert bound == set(_declared())


def test_struct_layouts_match_header():
    from copula_var import _native as N
    # cvq_static: 6 int32, 7 pointers, int32 n_copula_params, int32 strategy, double v_cap
    assert C.sizeof(N.CvqStatic) == 6 * 4 + 7 * 8 + 4 + 4 + 8
    assert N.CvqStatic.v_cap.offset == 6 * 4 + 7 * 8 + 8
    assert C.sizeof(N.CvqSolveArgs) == 9 * 8
    hdr = open(HEADER).read()
    for f, _ in N.CvqStatic._fields_:
        assert re.search(rf"\b{f}\s*;", hdr), f
    for f, _ in N.CvqSolveArgs._fields_:
        assert re.search(rf"\b{f}\b", hdr), f


def test_host_side_validation_without_gpu():
    """Calls that fail argument checks before touching HIP return their status
    codes and set cvq_last_error (no device needed)."""
    from copula_var import _native as N
    lib = N.lib()
    assert lib.cvq_version() >= 1
    # NULL static table -> invalid argument
    h = C.c_void_p()
    rc = lib.cvq_plan_create(None, 0, C.byref(h))
    assert rc == N.CVQ_ERR_INVALID
    assert lib.cvq_last_error()
    # a solve budget beyond 62 bisection steps is rejected on the host
    a = N.CvqSolveArgs(0.05, -3.0, -3.5, -2.0, -7.5, 0.0, -100.0, 1e-30, 0.0)
    s = C.c_int32()
    assert lib.cvq_snap_stride(C.byref(a), C.byref(s)) == N.CVQ_ERR_UNSUPPORTED
    a.tolerance = 1e-6
    assert lib.cvq_snap_stride(C.byref(a), C.byref(s)) == N.CVQ_OK
    assert 20 <= s.value <= 30
    assert lib.cvq_solve_status(None, C.byref(s)) == N.CVQ_ERR_INVALID
    assert lib.cvq_set_fast_hint(None, 1) == N.CVQ_ERR_INVALID


def test_in_sample_entry_points_validate_on_the_host():
    """GARCH(p, q) forecast / likelihood and the UKF E-step reject bad orders, GARCH
    parameters that garch/estimation.py:22-38 rejects, and NULL buffers before any HIP call."""
    import numpy as np
    from copula_var import _native as N
    lib = N.lib()
    r, out = np.zeros(50), np.zeros(50)
    ok = np.array([0.05, 0.1, 0.05, 0.6])                                  # (p, q) = (2, 1)
    bad = np.array([0.05, 0.5, 0.3, 0.4])                                  # sum >= 1
    neg = np.array([0.05, -0.1, 0.05, 0.6])
    f = lambda p, q, prm: lib.cvq_garch_forecast_pq(0, p, q, N.ptr(prm), N.ptr(r), 10, 5, N.ptr(out), N.MEM_HOST)
    assert f(2, 1, bad) == N.CVQ_ERR_INVALID
    assert f(2, 1, neg) == N.CVQ_ERR_INVALID
    assert f(5, 1, np.zeros(7) + 0.01) == N.CVQ_ERR_UNSUPPORTED
    assert lib.cvq_garch_loglik_pq(0, 0, 1, N.ptr(ok), 1, N.ptr(r), 50, N.ptr(out), N.MEM_HOST) == \
        N.CVQ_ERR_UNSUPPORTED
    assert lib.cvq_ukf_filter(0, None, 1, N.ptr(r), 0, 50, N.ptr(out), N.ptr(out), N.MEM_HOST) == N.CVQ_ERR_INVALID
    assert lib.cvq_last_error()


def test_product_path_fails_loudly_without_library(monkeypatch, tmp_path):
    """No CPU fallback: a missing libcvq.so raises instead of computing."""
    import importlib
    from copula_var import _native as N
    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        N.lib()


def test_new_entry_points_validate_on_the_host():
    """Packed finalize layout, solve status and the device MSM tables reject bad arguments
    before any HIP call."""
    from copula_var import _native as N
    lib = N.lib()
    a = N.CvqSolveArgs(0.05, -3.0, -3.5, -2.0, -7.5, 0.0, -100.0, 1e-6, 0.0)
    ln, off = C.c_int64(), C.c_int64()
    assert lib.cvq_packed_block_len(C.byref(a), 1000, C.byref(ln), C.byref(off)) == N.CVQ_OK
    s = C.c_int32()
    lib.cvq_snap_stride(C.byref(a), C.byref(s))
    assert off.value >= 1000 * s.value and off.value % 2 == 0 and ln.value == off.value + 2
    assert lib.cvq_packed_block_len(C.byref(a), 0, C.byref(ln), C.byref(off)) == N.CVQ_ERR_INVALID
    assert lib.cvq_solve_finalize_packed(None, C.byref(a), None, 1, 1, 1, None) == N.CVQ_ERR_INVALID
    n = C.c_int64()
    assert lib.cvq_msm_tables_scratch(2, 4, 1135, 1000, C.byref(n)) == N.CVQ_OK
    # cond, filt, then the scan filter's buffers per asset (window-end prefixes, window-start
    # suffix row sums, 133 block products of 16 steps, 17 superblocks of 8 prefixes + 8 suffixes),
    # err word, then one error flag (int) per asset and block (2 x 134)
    scan = 1000 * 256 + 1000 * 16 + (2134 // 16) * 256 + 2 * 17 * 8 * 256
    assert n.value == 2 * 2134 * 16 + 2 * 1000 * 16 + 2 * scan + 2 + (2 * 134 + 1) // 2
    assert lib.cvq_msm_tables_scratch(4, 4, 1135, 1000, C.byref(n)) == N.CVQ_ERR_INVALID
    prm = np.array([0.45, 1.2, 3.0, 0.3, 0.5, 1.2, 3.0, 0.3])
    smap = np.zeros(32, dtype=np.int32)
    buf = np.zeros(8)
    f = lambda dim, k, q, sm: lib.cvq_msm_tables(0, None, dim, k, N.ptr(prm), sm.ctypes.data_as(C.c_void_p), q,
                                                 N.ptr(buf), 10, 5, N.ptr(buf), N.ptr(buf), N.ptr(buf))
    assert f(1, 4, 5, smap) == N.CVQ_ERR_UNSUPPORTED                      # dim 1 is not a copula
    assert f(2, 8, 5, smap) == N.CVQ_ERR_UNSUPPORTED                      # k > 7
    bad = smap.copy()
    bad[3] = 9
    assert f(2, 4, 5, bad) == N.CVQ_ERR_INVALID                           # state map outside [0, q)
    assert lib.cvq_last_error()



def test_sigma_tables_validate_on_the_host():
    """cvq_sigma_tables (device GARCH / UKF forecast stage) rejects bad arguments before any
    HIP call."""
    from copula_var import _native as N
    lib = N.lib()
    buf = np.zeros(16)
    err = np.zeros(1, dtype=np.int32)
    ok_orders = np.array([1, 1, 2, 1], dtype=np.int32)
    garch = np.array([0.05, 0.08, 0.90, 0.05, 0.04, 0.04, 0.90])
    f = lambda model, dim, orders, prm: lib.cvq_sigma_tables(
        0, None, model, dim, orders.ctypes.data_as(C.c_void_p) if orders is not None else None, N.ptr(prm),
        N.ptr(buf), 10, 5, err.ctypes.data_as(C.c_void_p), N.ptr(buf))
    assert f(N.MSM, 2, None, garch) == N.CVQ_ERR_UNSUPPORTED               # MSM has cvq_msm_tables
    assert f(N.GARCH, 1, None, garch) == N.CVQ_ERR_UNSUPPORTED             # dim 1
    assert f(N.GARCH, 2, np.array([1, 5, 1, 1], dtype=np.int32), garch) == N.CVQ_ERR_UNSUPPORTED   # q > 4
    nonstat = garch.copy()
    nonstat[6] = 0.95                                                      # alpha_1 + alpha_2 + beta >= 1
    assert f(N.GARCH, 2, ok_orders, nonstat) == N.CVQ_ERR_INVALID
    assert lib.cvq_sigma_tables(0, None, N.UKF, 2, None, None, N.ptr(buf), 10, 5,
                                err.ctypes.data_as(C.c_void_p), N.ptr(buf)) == N.CVQ_ERR_INVALID
    assert lib.cvq_sigma_tables_status(None, None) == N.CVQ_ERR_INVALID
    assert lib.cvq_last_error()
