"""ValueAtRiskCalcualtion -- the reference's VaR driver (utils/calc_var_class.py:8-309)
with the quadrature and the bisection on the GPU.

Same constructor, same pipeline order, same ``calc_var(obj_var, first_guess,
second_guess) -> np.ndarray (T,)`` and ``compute_integral(bounds) -> (T,)``
(the seam SURVEY.md §8b names).  Underneath:

* ``compute_integral`` is one device slab launch (cvq_slab) instead of
  np.unique + nested-grid build + joblib over dates (calc_var_class.py:179-212);
* ``calc_var`` is one device solve (cvq_solve: one k_compact launch for 2 assets,
  one k_sorted launch for 3, each with the finalize fused in) that reproduces
  calc_var + bisection_algorithm (:95-177, :250-309) with quirks Q1-Q4 -- results
  bit-identical to the reference on the golden cases (tests/test_gpu_parity.py,
  tests/test_driver_gpu.py);
* ``bisection_algorithm`` / ``adjust_integral`` keep the reference's host loop
  over device slabs, for callers that drive the bisection themselves.

The in-sample stage runs as the reference's does (model fits, marginals, the IFM
copula fit of calc_copula_params, :77-82) on the device likelihoods.

Keyword-only additions: ``copula_params`` (packed copula parameters that override
the IFM fit), ``device``, ``strategy`` ("auto" = COMPACT for 2-asset MSM, SORTED for
3 assets and for 2-asset GARCH / UKF, engine.auto_strategy; or "direct", "prefix", "sorted", "compact").
"""
from __future__ import annotations

import time

import numpy as np

from ..data_loader.load_data import IndexReturnsRetriever
from ..engine import QuadraturePlan


DEVICE_MODELS = ("msm", "garch", "mean_reverting")
DEVICE_COPULAS = ("student", "gaussian", "plackett")


def check_device_adapter(method) -> None:
    """The device evaluates the integrand itself (integrated_function is not a per-node
    callback here), so an adapter must name a device model and copula: `model_kind` in
    DEVICE_MODELS and `copula_kind` in DEVICE_COPULAS, as the factory's adapters do.  A
    user-written VaRCalculationMethod without them fails here, before any in-sample work."""
    model = getattr(method, "model_kind", None)
    copula = getattr(method, "copula_kind", None)
    bad = []
    if model not in DEVICE_MODELS:
        bad.append(f"model_kind={model!r} (one of {DEVICE_MODELS})")
    if copula not in DEVICE_COPULAS:
        bad.append(f"copula_kind={copula!r} (one of {DEVICE_COPULAS})")
    if bad:
        raise ValueError(
            f"{type(method).__name__} cannot run on the device engine: it needs " + " and ".join(bad)
            + ". The integrand is evaluated inside the HIP quadrature (cvq_slab / cvq_solve), so a "
              "VaRCalculationMethod must be one of the factory's (copula x model) adapters or "
              "declare those two attributes; a Python integrated_function is not called "
              "(INTEGRATION.md, 'Plug-in adapters').")


class ValueAtRiskCalcualtion:
    def __init__(self, tickers, start_date, in_sample_data_num, VaRCalculationMethod, end_date=None,
                 num_points=100, weights=np.array([0.5, 0.5]), *args, copula_params=None, device=0,
                 strategy="auto", **kwargs):
        check_device_adapter(VaRCalculationMethod)
        self.num_points = num_points
        self.tickers = tickers
        self.start_date = start_date
        self.in_sample_data_num = in_sample_data_num
        self.VaRCalculationMethod = VaRCalculationMethod
        self.end_date = end_date
        self.weights = weights
        self.device = int(device)
        if hasattr(VaRCalculationMethod, "set_device"):
            VaRCalculationMethod.set_device(self.device)

        (self.in_sample_dict, self.rolling_windows_dict, self.mean_returns, self.end_date, self.out_sample_data,
         self.out_sample_N, self.dim, self.ptf_mean) = self.get_in_sample_data()

        self.in_sample_params = self.retrieve_param_in_sample(*args, **kwargs)
        self.marginals, self.densities, self.vol_states_array = self.calc_marg_and_densities(*args, **kwargs)
        self.copula_params = np.atleast_1d(np.asarray(
            copula_params if copula_params is not None else self.calc_copula_params(), dtype=np.float64))
        self.integrations_params_t, self.integrations_params_static, self.grids_generations_params = (
            self.integration_params_retrieval())

        self.copula_function = VaRCalculationMethod.copula_density
        self.unpack_copula_params = VaRCalculationMethod.unpack_copula_params
        self.integrated_function = VaRCalculationMethod.integrated_function

        densities, x_values, step_size, combos = self.grids_generations_params
        self.plan = QuadraturePlan(VaRCalculationMethod.model_kind, VaRCalculationMethod.copula_kind, self.dim,
                                   x_values, step_size, densities, combos, self.weights, self.copula_params,
                                   vol_states=self.integrations_params_static, device=self.device,
                                   strategy=strategy)
        self.plan.set_dates(self.integrations_params_t)

    # ----------------------------------------------------------- pipeline (:47-93)
    def get_in_sample_data(self):
        retriever = IndexReturnsRetriever(tickers=self.tickers, start_date=self.start_date,
                                          N=self.in_sample_data_num, weights=self.weights, end_date=self.end_date)
        return retriever.get_insample_data()

    def retrieve_param_in_sample(self, *args, **kwargs):
        return self.VaRCalculationMethod.model_params_insample(self.in_sample_dict, *args, **kwargs)

    def calc_marg_and_densities(self, *args, **kwargs):
        return self.VaRCalculationMethod.calculate_marginals_and_densities_in_sample(
            self.in_sample_dict, self.in_sample_params, *args, **kwargs)

    def calc_copula_params(self):
        best_fit = self.VaRCalculationMethod.copula_or_correl_params_insample(self.marginals, self.densities)
        return self.VaRCalculationMethod.copula_integrations_params(best_fit)

    def integration_params_retrieval(self):
        return self.VaRCalculationMethod.integration_params_retrieval(
            self.dim, self.rolling_windows_dict, self.in_sample_params, self.num_points, self.vol_states_array)

    # ----------------------------------------------------------- VaR (:95-177)
    def calc_var(self, obj_var=0.05, first_guess=-3, second_guess=(-3.5, -2)):
        """Per-date VaR (T,) = solved quantile + ptf_mean, one device solve."""
        start_time = time.time()
        var, self.last_iterations = self.plan.calc_var(self.ptf_mean, obj_var, first_guess, second_guess)
        print(f"calc_var function execution time: {time.time() - start_time:.4f} seconds")
        return var

    def compute_integral(self, bounds):
        """I_t(a, b] for every date t (calc_var_class.py:179-212), one device launch."""
        return self.plan.compute_integral(np.asarray(bounds, dtype=np.float64))

    def adjust_integral(self, new_result, prev_results, bounds, prev_upper):
        """calc_var_class.py:214-248 (exact float equality)."""
        return np.where(bounds[:, 0] == prev_upper, prev_results + new_result, prev_results - new_result)

    def bisection_algorithm(self, obj_var, bisection_bounds, prev_result, upper_stack, prev_upper,
                            tolerance=1e-6):
        """calc_var_class.py:250-309 on the host, each slab integral on the device."""
        lower, upper = bisection_bounds[:, 0].copy(), bisection_bounds[:, 1].copy()
        while np.any(upper - lower > tolerance):
            mid = (lower + upper) / 2
            b = np.where(upper_stack[:, None], np.column_stack((lower, mid)), np.column_stack((mid, upper)))
            result = self.adjust_integral(self.compute_integral(b), prev_result, b, prev_upper)
            if np.all(result == 0):
                break
            upper_stack = result < obj_var
            lower = np.where(~upper_stack, lower, mid)
            upper = np.where(upper_stack, upper, mid)
            prev_result = result
            prev_upper = mid
        return (lower + upper) / 2

    def close(self):
        self.plan.close()
