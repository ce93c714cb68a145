"""Oracle: nested-grid copula quadrature and the bisection VaR solve, numpy.

Test infrastructure only (see oracle/__init__.py).  Restates
utils/calc_integral/* + copulas/* + utils/calc_var_class.py of the reference.

The reference evaluates its integrand node by node on a freshly built nested
grid per unique bounds row.  This restatement evaluates the same integrand on
the whole box once per date (the special functions depend only on the 1-D grid
index, SURVEY.md finding 3) and sums it under the reference's exact membership
rule for each slab, so per-call values agree to rounding and every bisection
decision -- hence the VaR -- is identical.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import special, stats

BOX_LO, BOX_HI = -5, 5          # calc_var_class.py:201-202


def norm_cdf(x):
    """utils/utils.py:4-22 -- erf form (Q16)."""
    z = (x - 0) / 1
    return 0.5 * (1 + special.erf(z / np.sqrt(2)))


def norm_pdf(x):
    """utils/utils.py:24-42."""
    z = (x - 0) / 1
    return (1 / (1 * np.sqrt(2 * np.pi))) * np.exp(-0.5 * z ** 2)


def unpack_copula(copula: str, params):
    """unpack_copula_params of student_estimation.py:40-56, gaussian_estimation.py:13-23,
    plackett_estimation.py:12-16 -> (nu_or_theta, corr)."""
    if copula == "plackett":
        return float(np.asarray(params).reshape(-1)[0]), None
    p = np.asarray(params, dtype=np.float64).reshape(-1)
    if copula == "student":
        nu, rho = float(p[0]), p[1:]
    else:
        nu, rho = None, p
    n = int((1 + np.sqrt(1 + 8 * len(rho))) / 2)
    R = np.eye(n)
    R[np.triu_indices(n, k=1)] = rho
    R[np.tril_indices(n, k=-1)] = rho
    return nu, R


class Problem:
    """Static + per-date inputs of one calc_var, in the reference's own layout.

    MSM:  per_date = (forecasts_by_states (T,dim,q), forecasts (T,Q)), static = unique_vol_states
    GARCH/UKF: per_date = sigma forecasts (T,dim)."""

    def __init__(self, model, copula, dim, x_values, step, densities, combos, weights,
                 copula_params, per_date, unique_vol_states=None):
        self.model, self.copula, self.dim = model, copula, int(dim)
        self.x = np.asarray(x_values, dtype=np.float64)
        self.step = np.asarray(step, dtype=np.float64)
        self.n = self.x.size
        self.dens = np.asarray(densities, dtype=np.float64)
        self.combos = np.asarray(combos).astype(np.int64)
        self.w = np.asarray(weights, dtype=np.float64)
        self.copula_params = copula_params
        self.nu, self.R = unpack_copula(copula, copula_params)
        if model == "msm":
            self.fbs, self.pi = (np.asarray(a, dtype=np.float64) for a in per_date)
            self.uvs = np.asarray(unique_vol_states, dtype=np.float64)
            self.T = self.fbs.shape[0]
        else:
            self.sigma = np.asarray(per_date, dtype=np.float64)
            self.T = self.sigma.shape[0]
        self._mass = {}

    # ---------------------------------------------------------------- integrand
    def axis_cdf(self, t):
        """Per-axis marginal CDF tables u[d, i] (msm_integration_function.py:34-36;
        garch_integration_function.py:31-33) and GARCH pdf tables."""
        if self.model == "msm":
            xs = self.x[None, :, None] / self.uvs[:, None, :]           # (dim, n, q)
            u = np.sum(self.fbs[t][:, None, :] * norm_cdf(xs), axis=2)
            return u, None
        s = self.sigma[t]
        xs = self.x[None, :] / s[:, None]
        return norm_cdf(xs), norm_pdf(xs) / s[:, None]

    def _broadcast(self, tab):
        d = self.dim
        return [tab[c].reshape([self.n if a == c else 1 for a in range(d)]) for c in range(d)]

    def copula_density(self, u):
        """Copula density on the full box from per-axis u tables (copulas/*)."""
        d, cop = self.dim, self.copula
        if cop == "plackett":                                        # plackett.py:46-71 (Q11)
            U, V = self._broadcast(u)[:2]
            th = self.nu
            num = th * (1 + (th - 1) * (U + V - 2 * U * V))
            den = ((1 + (th - 1) * (U + V)) * (1 + (th - 1) * (1 - U - V))) ** 2
            return num / den
        if cop == "student":
            z = stats.t.ppf(u, df=self.nu)                           # student.py:100-102
        else:
            z = stats.norm.ppf(u)                                    # gaussian.py:43-44
        Z = self._broadcast(z)
        Ri = np.linalg.inv(self.R)
        det = np.linalg.det(self.R)
        y = [sum(Z[i] * Ri[i, j] for i in range(d)) for j in range(d)]
        qf = sum(y[j] * Z[j] for j in range(d))
        if cop == "student":
            nu = self.nu
            term1 = math.gamma((nu + d) / 2) / (math.gamma(nu / 2) * ((nu * np.pi) ** (d / 2)) * np.sqrt(det))
            finite = np.ones(qf.shape, dtype=bool)
            for c in range(d):
                finite = finite & np.isfinite(Z[c])
            with np.errstate(invalid="ignore", over="ignore"):
                mv = np.where(finite, term1 * (1 + qf / nu) ** (-(nu + d) / 2), 0.0)   # student.py:133-141
            g = math.gamma((nu + 1) / 2) / (np.sqrt(nu * np.pi) * math.gamma(nu / 2))
            with np.errstate(invalid="ignore", over="ignore"):
                uni = np.where(np.isfinite(z), g * (1 + (z ** 2 / nu)) ** (-(nu + 1) / 2), 0.0)
        else:
            term1 = 1 / (np.sqrt((2 * np.pi) ** d * det))
            with np.errstate(invalid="ignore", over="ignore"):
                mv = term1 * np.exp(-0.5 * qf)                       # gaussian.py:107-113
            uni = (1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * z ** 2)   # gaussian.py:82
        U = self._broadcast(uni)
        prod = U[0]
        for c in range(1, d):
            prod = prod * U[c]
        with np.errstate(invalid="ignore", divide="ignore"):
            return mv / prod                                         # student.py:77 / gaussian.py:59

    def delta_weights(self, t):
        """sum_l pi_t[l] * Delta[node, l], with the Delta-product of create_grids.py:102-171:
        axis c uses densities[(c-1) mod dim] (Q5); in 3-D the axis-0 factor survives only
        where i1 == 0 (Q6)."""
        d, n = self.dim, self.n
        Q = self.combos.shape[0]
        pi = self.pi[t] if self.model == "msm" else np.ones(1)
        W = np.zeros([n] * d)
        for l in range(Q):
            f = [self.dens[(c - 1) % d, self.combos[l, c], :] * self.step for c in range(d)]
            F = self._broadcast(np.array(f))
            if d == 3:
                F0 = np.where(np.arange(n)[None, :, None] == 0, F[0], 1.0)
                term = (F0 * F[1]) * F[2]
            else:
                term = F[0]
                for c in range(1, d):
                    term = term * F[c]
            W += pi[l] * term
        return W

    def mass(self, t):
        """Integrand x Delta on every node of the box for date t
        (msm_integration_function.py:45 / garch_integration_function.py:38-50)."""
        if t in self._mass:
            return self._mass[t]
        u, pdf = self.axis_cdf(t)
        c = self.copula_density(u)
        W = self.delta_weights(t)
        if self.model == "msm":
            m = c * W                                                # no NaN guard (Q15)
        else:
            P = self._broadcast(pdf)
            dp = P[0]
            for k in range(1, self.dim):
                dp = dp * P[k]
            m = np.nan_to_num(c * dp) * W                            # garch_integration_function.py:45-50
        self._mass[t] = m
        return m

    # ---------------------------------------------------------------- membership
    def inner_mask(self, a, b):
        """Nested-grid membership for bounds (a, b] (create_grids.py:102-108, 127;
        var_function integration_algo.py:20 (Q10); strict clamped lower edge (Q9))."""
        d, x, w = self.dim, self.x, self.w
        if d == 2:
            s = x * w[1]
            shape_prev = (self.n, 1)
        else:
            s = (x[:, None] * w[1]) + (x[None, :] * w[2])
            shape_prev = (self.n, self.n, 1)
        g_hi = (b - s) / w[0]
        g_lo = (a - s) / w[0]
        g_lo = np.where(BOX_LO > g_lo, BOX_LO, g_lo)                # Python max(g, -5)
        xi = x.reshape([1] * (d - 1) + [self.n])
        return (xi > g_lo.reshape(shape_prev)) & (xi <= g_hi.reshape(shape_prev))

    def slab(self, t, a, b):
        """One date's compute_integral value for bounds (a, b]."""
        return float(np.sum(self.mass(t)[self.inner_mask(a, b)]))

    def compute_integral(self, bounds):
        """calc_var_class.py:179-212 (dedupe is a performance detail only)."""
        bounds = np.asarray(bounds, dtype=np.float64)
        return np.array([self.slab(t, bounds[t, 0], bounds[t, 1]) for t in range(self.T)])


# ------------------------------------------------------------------ control flow
def adjust_integral(new_result, prev_results, bounds, prev_upper):
    """calc_var_class.py:214-248 (exact float equality)."""
    return np.where(bounds[:, 0] == prev_upper, prev_results + new_result, prev_results - new_result)


def calc_var(compute_integral, T, ptf_mean, obj_var=0.05, first_guess=-3, second_guess=(-3.5, -2),
             tolerance=1e-6, trace=None):
    """ValueAtRiskCalcualtion.calc_var (calc_var_class.py:95-177) + bisection_algorithm
    (:250-309), quirks Q1-Q4 included.  np.empty brackets (Q3) are NaN here.
    Returns (var (T,), n_iterations, broke_all_zero)."""
    min_var_value, max_var_value = -7.5, 0
    lower, upper = -100, first_guess
    bounds = np.column_stack((lower * np.ones(T), upper * np.ones(T)))
    results = compute_integral(bounds)
    new_lower = np.where(results >= obj_var, second_guess[0], first_guess)
    new_upper = np.where(results < obj_var, second_guess[1], first_guess)
    bounds = np.column_stack((new_lower, new_upper))
    prev_upper = np.where(new_lower == second_guess[0], second_guess[0], first_guess)   # Q1
    new_result = compute_integral(bounds)
    result_current = adjust_integral(new_result, results, bounds, upper * np.ones(T))
    upper = bounds[:, 1]
    bb = np.full((T, 2), np.nan)                                                       # Q3
    m = result_current > obj_var
    bb[m, 0], bb[m, 1] = min_var_value, second_guess[0]
    m = (result_current < obj_var) & (upper == first_guess)
    bb[m, 0], bb[m, 1] = second_guess[0], first_guess
    m = (result_current < obj_var) & (upper == second_guess[1])
    bb[m, 0], bb[m, 1] = second_guess[1], max_var_value
    m = (result_current > obj_var) & (upper == second_guess[1])
    bb[m, 0], bb[m, 1] = first_guess, second_guess[1]
    upper_stack = ~np.isin(bb[:, 1], list(second_guess))
    if trace is not None:
        trace["brackets"] = bb.copy()
    lo, hi = bb[:, 0].copy(), bb[:, 1].copy()
    prev_result = result_current
    iters, broke = 0, False
    while np.any(hi - lo > tolerance):                                                 # Q2
        mid = (lo + hi) / 2
        b = np.where(upper_stack[:, None], np.column_stack((lo, mid)), np.column_stack((mid, hi)))
        mid_result = compute_integral(b)
        rc = adjust_integral(mid_result, prev_result, b, prev_upper)
        if np.all(rc == 0):                                                            # Q4
            broke = True
            break
        upper_stack = rc < obj_var
        lo = np.where(~upper_stack, lo, mid)
        hi = np.where(upper_stack, hi, mid)
        prev_result = rc
        prev_upper = mid
        iters += 1
    return (lo + hi) / 2 + ptf_mean, iters, broke
