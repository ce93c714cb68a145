"""Host-side handle on the HIP quadrature engine (libcvq.so).

``QuadraturePlan`` is the device replacement for the reference's quadrature
stack: ``compute_integral`` replaces ValueAtRiskCalcualtion.compute_integral
(utils/calc_var_class.py:179-212 -> utils/calc_integral/calc_integral.py:8-225)
and ``calc_var`` replaces calc_var + bisection_algorithm
(utils/calc_var_class.py:95-177, 250-309) with one device solve.
The forecast-stage functions replace the per-date filters
(msm_estimation.py:140-202, garch_estimation.py:190-231,
mean_reverting_estimation.py:192-232).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _native as N

DEFAULT_SOLVE = dict(obj_var=0.05, first_guess=-3.0, second_guess=(-3.5, -2.0), min_var=-7.5,
                     max_var=0.0, lower=-100.0, tolerance=1e-6)


def solve_args(ptf_mean: float = 0.0, obj_var=0.05, first_guess=-3.0, second_guess=(-3.5, -2.0),
               min_var=-7.5, max_var=0.0, lower=-100.0, tolerance=1e-6) -> N.CvqSolveArgs:
    """calc_var arguments (calc_var_class.py:95) + its constants (:111-114, :257)."""
    return N.CvqSolveArgs(float(obj_var), float(first_guess), float(second_guess[0]), float(second_guess[1]),
                          float(min_var), float(max_var), float(lower), float(tolerance), float(ptf_mean))


MAX_N = 512                           # num_points limit of every strategy but 2-D SORTED (cvq_plan_create)
SORTED_MAX_N = {2: 1024, 3: 255}     # sorted_max_n (cvq_sorted_kernels.h): 2-D n > 512 runs 1024-thread dates;
                                      # 3-D: the 32-bit node word (a0 = i0 + n [i1 == 0] < 2n in 9 bits,
                                      # i1 in 8); its LDS (9 n doubles + a 16-KB tail) is not the bound
PREFIX_MAX_N_3D = 64                  # PREFIX solves at most 4096 rows (cvq_plan.hip pick_solve_shape)
MATERIALISED = ("prefix", "sorted", "sweep")   # strategies that hold only nodes with level <= v_cap


def general_power(copula: Optional[str], copula_params=None) -> bool:
    """A Student copula whose node power -(nu + 2)/2 is not a half-integer (an IFM-fitted nu):
    every node takes the general power exp(ex log b) (cvq_special.h pow_node)."""
    if copula != "student" or copula_params is None:
        return False
    nu = float(np.atleast_1d(np.asarray(copula_params, dtype=np.float64))[0])
    return (nu + 2.0) != np.floor(nu + 2.0)


def auto_strategy(model: str, dim: int, n: Optional[int] = None, copula: Optional[str] = None,
                  copula_params=None) -> str:
    """The measured-fastest strategy per workload (cfg 1-5 on one MI355X)
    among those that run it: COMPACT for 2-asset MSM (cfg 2: 20.3M vs SORTED 16.4M
    VaR-dates/s) and for 2-asset GARCH / UKF with an integer-power Student copula (cfg 5:
    25.2M vs 22.5M since r05's grid-edge fast records), SORTED for the other 2-asset
    GARCH / UKF copulas (cfg 3 Plackett: 8.1M vs 6.3M; cfg 1 Gaussian: 33.8M vs 26.9M) and
    for 3 assets (the only strategy that runs the 128^3 grid of cfg 4).  n (num_points)
    bounds the choice: every 2-D strategy takes n <= 512 (the plan's limit, so a 2-D
    rule never picks a strategy that fails later), 3-D SORTED n <= 255, 3-D PREFIX n <= 64; no 3-D strategy
    takes n > 255.  A 2-D grid with 512 < n <= 1024 (the reference takes any num_points,
    calc_var_class.py:16; main.py:50 suggests raising it) runs on SORTED, whose 1024-thread
    instance holds it.  SORTED and PREFIX hold the nodes with level <= v_cap only;
    QuadraturePlan(strategy="auto") routes a query above v_cap to an unrestricted
    sibling plan (COMPACT in 2-D, SORTED with v_cap at the grid's top in 3-D and for
    2-D n > 512)."""
    if dim == 2:
        if n is not None and n > MAX_N:
            if n > SORTED_MAX_N[2]:
                raise ValueError(f"2-asset grids support num_points <= {SORTED_MAX_N[2]} (SORTED), got {n}")
            return "sorted"
        # a fitted (non-integer) Student nu: SORTED (r06, nu = 5.364, in flight: cfg 2 10.7-11.0 M vs
        # COMPACT 9.2 M VaR-dates/s, cfg 5 12.2 M vs 9.4 M; COMPACT's general-power instance needs 98 VGPRs)
        if general_power(copula, copula_params):
            return "sorted"
        return "compact" if model == "msm" or copula == "student" else "sorted"
    if n is None or n <= SORTED_MAX_N[3]:
        return "sorted"
    raise ValueError(f"3-asset grids support num_points <= {SORTED_MAX_N[3]} (SORTED), got {n}")


class QuadraturePlan:
    """One device plan: static grid tables + copula + per-date inputs on one GPU."""

    def __init__(self, model: str, copula: str, dim: int, x_values, step, densities, combos, weights,
                 copula_params, vol_states=None, v_cap: float = 0.0, device: int = 0,
                 strategy: str = "auto"):
        N.require_gpu()
        self._ctor = (model, copula, dim, x_values, step, densities, combos, weights, copula_params, vol_states,
                      device)
        self.model, self.copula, self.dim = model, copula, int(dim)
        self.device = int(device)
        self._x = N.f64(x_values)
        self._step = N.f64(step)
        self._dens = N.f64(densities)
        self._combos = np.ascontiguousarray(np.asarray(combos).astype(np.int32))
        self._w = N.f64(weights)
        self._cp = N.f64(np.atleast_1d(np.asarray(copula_params, dtype=np.float64)))
        self._vs = N.f64(vol_states) if vol_states is not None else None
        q = self._dens.shape[1]
        st = N.CvqStatic()
        st.model = N.MODEL_KIND[model]
        st.copula = N.COPULA_KIND[copula]
        st.dim = self.dim
        st.n = self._x.size
        st.q = q
        st.n_combos = self._combos.shape[0]
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
        st.x_values, st.step, st.densities = dp(self._x), dp(self._step), dp(self._dens)
        st.combos = self._combos.ctypes.data_as(C.POINTER(C.c_int32))
        st.weights = dp(self._w)
        st.vol_states = dp(self._vs) if self._vs is not None else None
        st.copula_params = dp(self._cp)
        st.n_copula_params = self._cp.size
        self._auto = strategy == "auto"
        self._wide: Optional["QuadraturePlan"] = None       # unrestricted sibling (auto, level > v_cap)
        self._dates = None                                  # last set_dates / set_dates_device arguments
        self._stream, self._timing, self._counting = None, False, False   # forwarded to the sibling
        self._last: Optional["QuadraturePlan"] = None       # plan of the last device solve (solve_status)
        self._counted: Optional["QuadraturePlan"] = None    # plan that ran the last solve / slab (node counts)
        if strategy == "auto":
            strategy = auto_strategy(model, self.dim, self._x.size, copula, self._cp)
        st.strategy = {"prefix": N.STRATEGY_PREFIX, "direct": N.STRATEGY_DIRECT,
                       "compact": N.STRATEGY_COMPACT, "sorted": N.STRATEGY_SORTED,
                       "sweep": N.STRATEGY_SWEEP}[strategy]
        self.strategy = strategy
        st.v_cap = float(v_cap)
        self.v_cap = float(v_cap)
        self._static = st
        h = C.c_void_p()
        N.check(N.lib().cvq_plan_create(C.byref(st), self.device, C.byref(h)), "cvq_plan_create")
        self._h = h
        self.T = 0
        reach, rows = C.c_int64(), C.c_int32()
        N.check(N.lib().cvq_plan_info(self._h, C.byref(reach), C.byref(rows)), "cvq_plan_info")
        self.reach_nodes, self.rows = int(reach.value), int(rows.value)

    # ------------------------------------------------------------ lifecycle
    def close(self) -> None:
        if getattr(self, "_wide", None) is not None:
            self._wide.close()
            self._wide = None
        if getattr(self, "_h", None):
            N.lib().cvq_plan_destroy(self._h)
            self._h = None

    # ------------------------------------------------------------ auto: levels above v_cap
    def _route(self, top: float) -> "QuadraturePlan":
        """The plan that serves a query reaching level `top`: this one, or (strategy
        "auto" on a materialised strategy, top > v_cap) an unrestricted sibling --
        COMPACT in 2-D (its slabs run k_direct, any bounds), SORTED in 3-D with v_cap
        at the grid's top level -- holding the same per-date inputs."""
        if not self._auto or self.strategy not in MATERIALISED or not (top > self.v_cap):
            return self
        if self._wide is not None and self._wide.strategy in MATERIALISED and top > self._wide.v_cap:
            self._wide.close()                  # a higher level than the 3-D sibling holds: rebuild it
            self._wide = None
        if self._wide is None:
            model, copula, dim, x, step, dens, combos, w, cp, vs, dev = self._ctor
            if self.dim == 2 and self._x.size <= MAX_N:
                self._wide = QuadraturePlan(model, copula, dim, x, step, dens, combos, w, cp, vol_states=vs,
                                            device=dev, strategy="compact")
            else:
                grid_top = float(np.sum(np.abs(self._w)) * np.max(np.abs(self._x)))
                self._wide = QuadraturePlan(model, copula, dim, x, step, dens, combos, w, cp, vol_states=vs,
                                            v_cap=max(grid_top, float(top)), device=dev, strategy="sorted")
            if self._stream is not None:          # else the sibling keeps its own non-blocking stream
                self._wide.set_stream(self._stream)
            if self._dates is not None:
                kind, args = self._dates
                (self._wide.set_dates if kind == "host" else self._wide.set_dates_device)(*args)
            self._wide.enable_timing(self._timing)
            self._wide.count_nodes(self._counting)
        return self._wide._route(top)

    @staticmethod
    def _top(args: N.CvqSolveArgs) -> float:
        """The highest level a solve with these arguments can query."""
        return max(args.first_guess, args.second_guess_lo, args.second_guess_hi, args.max_var, args.min_var,
                   args.lower)

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: Optional[int]) -> None:
        """Launch on this HIP stream from now on (0 / None = the null stream, torch's default)."""
        N.check(N.lib().cvq_plan_set_stream(self._h, C.c_void_p(stream_handle or 0)), "cvq_plan_set_stream")
        self._stream = stream_handle
        if self._wide is not None:
            self._wide.set_stream(stream_handle)

    KERNELS = {"tables": 0, "mass": 1, "solve": 2, "finalize": 3, "slab": 4}

    def enable_timing(self, on=True) -> None:
        """Record HIP events around kernel launches on the plan's stream: True = every
        kind, False = off, or an iterable of kind names (e.g. ("solve",))."""
        if on is True or on is False:
            mask = 0x1F if on else 0
        else:
            mask = 0
            for k in on:
                mask |= 1 << self.KERNELS[k]
        N.check(N.lib().cvq_plan_timing(self._h, mask), "cvq_plan_timing")
        self._timing = on if (on is True or on is False) else tuple(on)
        if self._wide is not None:
            self._wide.enable_timing(self._timing)

    def kernel_time(self, kind: str) -> Tuple[float, int]:
        """(total milliseconds, launches) of one kernel kind since enable_timing(), summed over
        this plan and its auto-routed sibling (solves above v_cap run there)."""
        ms, n = C.c_double(), C.c_int32()
        N.check(N.lib().cvq_plan_kernel_time(self._h, self.KERNELS[kind], C.byref(ms), C.byref(n)),
                "cvq_plan_kernel_time")
        tot, cnt = float(ms.value), int(n.value)
        if self._wide is not None:
            wm, wn = self._wide.kernel_time(kind)
            tot, cnt = tot + wm, cnt + wn
        return tot, cnt

    def count_nodes(self, on: bool = True) -> None:
        """Record, in the following solves, how many quadrature nodes each date evaluates
        (COMPACT / SORTED / SWEEP; measurement aid, slower -- never in a timed run)."""
        N.check(N.lib().cvq_plan_count_nodes(self._h, 1 if on else 0), "cvq_plan_count_nodes")
        self._counting = bool(on)
        if self._wide is not None:
            self._wide.count_nodes(on)

    def nodes_evaluated(self) -> int:
        """Nodes evaluated by the last counted solve, summed over its dates (read from the
        sibling plan when the auto rule routed that solve there)."""
        if self._counted is not None and self._counted is not self:
            return self._counted.nodes_evaluated()
        n = C.c_int64()
        N.check(N.lib().cvq_plan_nodes_evaluated(self._h, C.byref(n)), "cvq_plan_nodes_evaluated")
        return int(n.value)

    # ------------------------------------------------------------ per-date inputs
    def set_dates(self, integrations_params_t) -> None:
        """integrations_params_t as the reference builds it: MSM (forecasts_by_states
        (T,dim,q), forecasts (T,Q)); GARCH/UKF [sigma (T,dim)] (garch_estimation.py:231)."""
        if self.model == "msm":
            fbs, pi = integrations_params_t
            a, b = N.f64(fbs), N.f64(pi)
            T = a.shape[0]
            N.check(N.lib().cvq_set_dates(self._h, T, N.ptr(a), N.ptr(b), N.MEM_HOST), "cvq_set_dates")
        else:
            sig = integrations_params_t[0] if isinstance(integrations_params_t, (list, tuple)) else integrations_params_t
            a = N.f64(sig)
            T = a.shape[0]
            N.check(N.lib().cvq_set_dates(self._h, T, N.ptr(a), None, N.MEM_HOST), "cvq_set_dates")
        self.T = int(T)
        if self._auto:
            self._dates = ("host", (integrations_params_t,))
            if self._wide is not None:
                self._wide.set_dates(integrations_params_t)

    def set_dates_device(self, T: int, a_ptr: int, b_ptr: Optional[int] = None, fast: bool = False) -> None:
        """Per-date inputs already resident in device memory (e.g. torch tensors' data_ptr()).
        They are read in place by the following launches (no copy): keep them alive and
        unchanged until the next set_dates.  fast=True asserts that every date takes
        COMPACT's fast node path (MSM: pi_t is the outer product of the per-asset
        forecasts, as the reference and cvq_msm_tables build it; GARCH/UKF: finite
        marginal tables) -- cvq_set_fast_hint; a violating date fails the solve."""
        N.check(N.lib().cvq_set_dates(self._h, int(T), C.c_void_p(a_ptr), C.c_void_p(b_ptr or 0), N.MEM_DEVICE),
                "cvq_set_dates")
        if fast:
            N.check(N.lib().cvq_set_fast_hint(self._h, 1), "cvq_set_fast_hint")
        self.T = int(T)
        if self._auto:
            self._dates = ("device", (T, a_ptr, b_ptr, fast))
            if self._wide is not None:
                self._wide.set_dates_device(T, a_ptr, b_ptr, fast)

    # ------------------------------------------------------------ quadrature
    def compute_integral(self, bounds) -> np.ndarray:
        """Drop-in for ValueAtRiskCalcualtion.compute_integral(bounds) -> (T,)."""
        b = N.f64(bounds)
        if b.shape != (self.T, 2):
            raise ValueError(f"bounds must have shape ({self.T}, 2)")
        top = float(np.nanmax(b)) if b.size else 0.0
        target = self._route(top)
        self._counted = target
        if target is not self:
            return target.compute_integral(b)
        out = np.empty(self.T)
        N.check(N.lib().cvq_slab(self._h, N.ptr(b), N.ptr(out), N.MEM_HOST), "cvq_slab")
        return out

    def calc_var(self, ptf_mean: float = 0.0, obj_var=0.05, first_guess=-3.0, second_guess=(-3.5, -2.0),
                 **consts) -> Tuple[np.ndarray, int]:
        """Drop-in for calc_var (calc_var_class.py:95-177): returns (VaR (T,), iterations)."""
        args = solve_args(ptf_mean, obj_var, first_guess, second_guess, **consts)
        target = self._route(self._top(args))
        self._last = self._counted = target
        if target is not self:
            return target.calc_var(ptf_mean, obj_var, first_guess, second_guess, **consts)
        out = np.empty(self.T)
        it = C.c_int32(0)
        N.check(N.lib().cvq_solve(self._h, C.byref(args), N.ptr(out), C.byref(it), N.MEM_HOST), "cvq_solve")
        return out, int(it.value)

    # ------------------------------------------------------------ device-resident solve
    def solve_device(self, args: N.CvqSolveArgs, var_ptr: int, check: bool = False) -> Optional[int]:
        """calc_var into a device buffer.  check=False: in stream order, no host
        synchronisation and no convergence check (call solve_status() to check);
        check=True: synchronises, widens the bisection budget if a date needed more
        iterations (non-dyadic guesses) and returns the iteration count.  A plan built with
        strategy "auto" routes levels above v_cap to its unrestricted sibling, as calc_var does."""
        target = self._route(self._top(args))
        self._last = self._counted = target
        if target is not self:
            return target.solve_device(args, var_ptr, check)
        if not check:
            N.check(N.lib().cvq_solve(self._h, C.byref(args), C.c_void_p(var_ptr), None, N.MEM_DEVICE), "cvq_solve")
            return None
        it = C.c_int32(0)
        N.check(N.lib().cvq_solve(self._h, C.byref(args), C.c_void_p(var_ptr), C.byref(it), N.MEM_DEVICE),
                "cvq_solve")
        return int(it.value)

    def solve_status(self) -> int:
        """Synchronise and check the last device-mode solve / finalize: raises NativeError
        (CVQ_ERR_NUMERIC) if a date did not converge within the bisection budget; returns
        the reference's bisection iteration count."""
        if self._last is not None and self._last is not self:
            return self._last.solve_status()
        it = C.c_int32(0)
        N.check(N.lib().cvq_solve_status(self._h, C.byref(it)), "cvq_solve_status")
        return int(it.value)

    @staticmethod
    def snap_stride(args: N.CvqSolveArgs) -> int:
        s = C.c_int32()
        N.check(N.lib().cvq_snap_stride(C.byref(args), C.byref(s)), "cvq_snap_stride")
        return int(s.value)

    def solve_local(self, args: N.CvqSolveArgs, header_ptr: int, snaps_ptr: int) -> None:
        target = self._route(self._top(args))
        self._last = None                        # the finalize (on this plan) reports the status
        self._counted = target
        if target is not self:
            return target.solve_local(args, header_ptr, snaps_ptr)
        N.check(N.lib().cvq_solve_local(self._h, C.byref(args), C.c_void_p(header_ptr), C.c_void_p(snaps_ptr)),
                "cvq_solve_local")

    @staticmethod
    def packed_block_len(args: N.CvqSolveArgs, dates_per_rank: int) -> Tuple[int, int]:
        """(block length, header offset) in doubles of one rank's packed block."""
        ln, off = C.c_int64(), C.c_int64()
        N.check(N.lib().cvq_packed_block_len(C.byref(args), int(dates_per_rank), C.byref(ln), C.byref(off)),
                "cvq_packed_block_len")
        return int(ln.value), int(off.value)

    def solve_finalize_packed(self, args: N.CvqSolveArgs, blocks_ptr: int, n_ranks: int, dates_per_rank: int,
                              T_total: int, var_ptr: int) -> None:
        N.check(N.lib().cvq_solve_finalize_packed(self._h, C.byref(args), C.c_void_p(blocks_ptr), int(n_ranks),
                                                  int(dates_per_rank), int(T_total), C.c_void_p(var_ptr)),
                "cvq_solve_finalize_packed")

    def solve_finalize(self, args: N.CvqSolveArgs, headers_ptr: int, n_ranks: int, snaps_ptr: int,
                       dates_per_rank: int, T_total: int, var_ptr: int) -> None:
        N.check(N.lib().cvq_solve_finalize(self._h, C.byref(args), C.c_void_p(headers_ptr), int(n_ranks),
                                           C.c_void_p(snaps_ptr), int(dates_per_rank), int(T_total),
                                           C.c_void_p(var_ptr)), "cvq_solve_finalize")


# ====================================================================== forecasts
def msm_filter(returns_c, n_in: int, k: int, m0: float, sig: float, b: float, gamma: float,
               device: int = 0) -> np.ndarray:
    """Filtered state probabilities at each window end, (T, 2**k).  returns_c: centred
    returns of one asset, length n_in + T - 1 (windows returns_c[t:t+n_in])."""
    r = N.f64(returns_c)
    T = r.size - n_in + 1
    out = np.empty((T, 1 << k))
    N.check(N.lib().cvq_msm_filter(device, k, m0, sig, b, gamma, N.ptr(r), n_in, T, N.ptr(out), N.MEM_HOST),
            "cvq_msm_filter")
    return out


def msm_marginals(returns, k: int, m0: float, sig: float, b: float, gamma: float, device: int = 0):
    """In-sample MSM marginals and densities of one return series on the device
    (cvq_msm_marginals; calc_marginals.py:7-30): two arrays of length N - 1."""
    r = N.f64(returns)
    m = np.empty(r.size - 1)
    d = np.empty(r.size - 1)
    N.check(N.lib().cvq_msm_marginals(device, k, m0, sig, b, gamma, N.ptr(r), r.size, N.ptr(m), N.ptr(d),
                                      N.MEM_HOST), "cvq_msm_marginals")
    return m, d


class MsmTables:
    """Device-resident MSM forecast stage (cvq_msm_tables): every asset's rolling-window
    Hamilton filters, the per-state collapse onto unique vols and the forecast
    combinations, written straight into device buffers that a QuadraturePlan reads in
    place (set_dates_device).  Replaces the host assembly of
    msm_estimation.integration_params_retrieval (msm_estimation.py:123-418) in the
    timed end-to-end path; buffers are torch tensors on `device`."""

    def __init__(self, params, k: int, state_map, q: int, n_in: int, T: int, device: int = 0):
        import torch
        self.k, self.q, self.n_in, self.T = int(k), int(q), int(n_in), int(T)
        self.params = np.ascontiguousarray(np.asarray(params, dtype=np.float64).reshape(-1, 4))
        self.dim = self.params.shape[0]
        self.state_map = np.ascontiguousarray(np.asarray(state_map, dtype=np.int32).reshape(self.dim, -1))
        self.device = int(device)
        n = C.c_int64()
        N.check(N.lib().cvq_msm_tables_scratch(self.dim, self.k, self.n_in, self.T, C.byref(n)),
                "cvq_msm_tables_scratch")
        dev = torch.device("cuda", self.device)
        self.scratch = torch.empty(int(n.value), dtype=torch.float64, device=dev)
        self.fbs = torch.empty((self.T, self.dim, self.q), dtype=torch.float64, device=dev)
        self.pi = torch.empty((self.T, self.q ** self.dim), dtype=torch.float64, device=dev)

    def run(self, returns_c_dev, stream: Optional[int] = None) -> None:
        """returns_c_dev: device tensor [dim][n_in + T - 1] of centred returns (C-contiguous)."""
        N.check(N.lib().cvq_msm_tables(self.device, C.c_void_p(stream or 0), self.dim, self.k, N.ptr(self.params),
                                       self.state_map.ctypes.data_as(C.c_void_p), self.q,
                                       C.c_void_p(returns_c_dev.data_ptr()), self.n_in, self.T,
                                       C.c_void_p(self.scratch.data_ptr()), C.c_void_p(self.fbs.data_ptr()),
                                       C.c_void_p(self.pi.data_ptr())), "cvq_msm_tables")

    def status(self, stream: Optional[int] = None) -> None:
        N.check(N.lib().cvq_msm_tables_status(C.c_void_p(self.scratch.data_ptr()), self.dim, self.k, self.n_in,
                                              self.T, C.c_void_p(stream or 0)), "cvq_msm_tables_status")


class SigmaTables:
    """Device-resident GARCH / UKF forecast stage (cvq_sigma_tables): every asset's
    rolling-window sigma forecast written straight into a device [T][dim] buffer that a
    QuadraturePlan reads in place (set_dates_device).  Replaces the host assembly of
    Garch/MeanRevertingEstimation.integration_params_retrieval (garch_estimation.py:133-145,
    mean_reverting_estimation.py:135-147) in the timed end-to-end path.

    model 'garch': params = per-asset dicts {'omega','alpha','beta'} or {'pq': (p, q),
    'params': (omega, alpha_1..p, beta_1..q)}; 'mean_reverting' (UKF): {'a','l','q'}."""

    def __init__(self, model: str, params: Sequence[dict], n_in: int, T: int, device: int = 0):
        import torch
        self.n_in, self.T, self.device = int(n_in), int(T), int(device)
        self.dim = len(params)
        if model == "garch":
            self.kind = N.GARCH
            orders, flat = [], []
            for p in params:
                if "pq" in p:
                    pq = (int(p["pq"][0]), int(p["pq"][1]))
                    row = list(np.asarray(p["params"], dtype=np.float64).ravel())
                    if len(row) != 1 + pq[0] + pq[1]:
                        raise ValueError(f"GARCH{pq} needs {1 + sum(pq)} parameters, got {len(row)}")
                else:
                    pq, row = (1, 1), [p["omega"], p["alpha"], p["beta"]]
                orders += pq
                flat += row
            self.orders = np.ascontiguousarray(orders, dtype=np.int32)
        elif model in ("mean_reverting", "ukf"):
            self.kind = N.UKF
            self.orders = None
            flat = [v for p in params for v in (p["a"], p["l"], p["q"])]
        else:
            raise ValueError(f"SigmaTables: model must be 'garch' or 'mean_reverting', got {model!r}")
        self.params = np.ascontiguousarray(flat, dtype=np.float64)
        dev = torch.device("cuda", self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.sig = torch.empty((self.T, self.dim), dtype=torch.float64, device=dev)

    def run(self, returns_c_dev, stream: Optional[int] = None) -> None:
        """returns_c_dev: device tensor [dim][n_in + T - 1] of centred returns (C-contiguous)."""
        orders = self.orders.ctypes.data_as(C.c_void_p) if self.orders is not None else None
        N.check(N.lib().cvq_sigma_tables(self.device, C.c_void_p(stream or 0), self.kind, self.dim, orders,
                                         N.ptr(self.params), C.c_void_p(returns_c_dev.data_ptr()), self.n_in,
                                         self.T, C.c_void_p(self.err.data_ptr()), C.c_void_p(self.sig.data_ptr())),
                "cvq_sigma_tables")

    def status(self, stream: Optional[int] = None) -> None:
        N.check(N.lib().cvq_sigma_tables_status(C.c_void_p(self.err.data_ptr()), C.c_void_p(stream or 0)),
                "cvq_sigma_tables_status")


def garch_forecast(returns_c, n_in: int, omega: float, alpha: float, beta: float, device: int = 0) -> np.ndarray:
    r = N.f64(returns_c)
    T = r.size - n_in + 1
    out = np.empty(T)
    N.check(N.lib().cvq_garch_forecast(device, omega, alpha, beta, N.ptr(r), n_in, T, N.ptr(out), N.MEM_HOST),
            "cvq_garch_forecast")
    return out


def garch_forecast_pq(returns_c, n_in: int, p: int, q: int, params, device: int = 0) -> np.ndarray:
    """GARCH(p, q) sigma forecasts per window; params = (omega, alpha_1..p, beta_1..q)."""
    r, prm = N.f64(returns_c), N.f64(params).ravel()
    if prm.size != 1 + p + q:
        raise ValueError(f"GARCH({p},{q}) needs {1 + p + q} parameters, got {prm.size}")
    T = r.size - n_in + 1
    out = np.empty(T)
    N.check(N.lib().cvq_garch_forecast_pq(device, int(p), int(q), N.ptr(prm), N.ptr(r), n_in, T, N.ptr(out),
                                          N.MEM_HOST), "cvq_garch_forecast_pq")
    return out


def ukf_forecast(returns_c, n_in: int, a: float, l: float, q: float, device: int = 0) -> np.ndarray:
    r = N.f64(returns_c)
    T = r.size - n_in + 1
    out = np.empty(T)
    N.check(N.lib().cvq_ukf_forecast(device, a, l, q, N.ptr(r), n_in, T, N.ptr(out), N.MEM_HOST),
            "cvq_ukf_forecast")
    return out


def msm_loglik(returns, k: int, params, device: int = 0) -> np.ndarray:
    """params (B, 4) rows (m0, sigma, b, gamma) -> (B,) log-likelihoods."""
    r, p = N.f64(returns), N.f64(np.atleast_2d(params))
    out = np.empty(p.shape[0])
    N.check(N.lib().cvq_msm_loglik(device, k, N.ptr(p), p.shape[0], N.ptr(r), r.size, N.ptr(out), N.MEM_HOST),
            "cvq_msm_loglik")
    return out


def garch_loglik(returns, params, device: int = 0) -> np.ndarray:
    """params (B, 3) rows (omega, alpha, beta)."""
    r, p = N.f64(returns), N.f64(np.atleast_2d(params))
    out = np.empty(p.shape[0])
    N.check(N.lib().cvq_garch_loglik(device, N.ptr(p), p.shape[0], N.ptr(r), r.size, N.ptr(out), N.MEM_HOST),
            "cvq_garch_loglik")
    return out


def garch_loglik_pq(returns, p: int, q: int, params, device: int = 0) -> np.ndarray:
    """params (B, 1 + p + q) rows (omega, alpha_1..alpha_p, beta_1..beta_q) -> (B,) log-likelihoods
    (numba_garch_log_likelihood, garch/estimation.py:91-125)."""
    r, pp = N.f64(returns), N.f64(np.atleast_2d(params))
    if pp.shape[1] != 1 + p + q:
        raise ValueError(f"GARCH({p},{q}) parameter rows have {1 + p + q} entries, got {pp.shape[1]}")
    out = np.empty(pp.shape[0])
    N.check(N.lib().cvq_garch_loglik_pq(device, int(p), int(q), N.ptr(pp), pp.shape[0], N.ptr(r), r.size,
                                        N.ptr(out), N.MEM_HOST), "cvq_garch_loglik_pq")
    return out


def ukf_loglik(returns, params, device: int = 0) -> np.ndarray:
    """params (B, 3) rows (a, l, q)."""
    r, p = N.f64(returns), N.f64(np.atleast_2d(params))
    out = np.empty(p.shape[0])
    N.check(N.lib().cvq_ukf_loglik(device, N.ptr(p), p.shape[0], N.ptr(r), r.size, N.ptr(out), N.MEM_HOST),
            "cvq_ukf_loglik")
    return out


def ukf_filter(returns, params, device: int = 0):
    """params (B, 3) rows (a, l, q); returns (N,) shared or (B, N) one series per row
    -> (LL (B,), state paths (B, N)); a failed pass has LL -1e10 and a NaN path
    (estimate.py:270-271: state_estimation None)."""
    r, p = N.f64(returns), N.f64(np.atleast_2d(params))
    B = p.shape[0]
    per = int(r.ndim == 2)
    if per and r.shape[0] != B:
        raise ValueError(f"returns has {r.shape[0]} series for {B} parameter rows")
    n = r.shape[-1]
    ll, states = np.empty(B), np.empty((n, B))
    N.check(N.lib().cvq_ukf_filter(device, N.ptr(p), B, N.ptr(r), per, n, N.ptr(ll), N.ptr(states), N.MEM_HOST),
            "cvq_ukf_filter")
    return ll, np.ascontiguousarray(states.T)
