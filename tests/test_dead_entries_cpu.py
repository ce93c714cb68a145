"""The premise of the r05 dead-entry fast records (cvq_sorted_kernels.h / cvq_compact_kernels.h
table phases): for GARCH / UKF with a Student copula, every node through a grid entry whose
marginal u is 0 or 1 (t.ppf = -inf / +inf) has integrand exactly 0 in the reference -- the
multivariate and univariate t pdfs are 0 for a non-finite z (student.py:130-131, :166-167),
0 / 0 = NaN and nan_to_num gives 0 (garch_integration_function.py:48) -- so the device may
evaluate those nodes as +0 on the fast path.  Checked on the pinned oracle (CPU)."""
import numpy as np
import pytest

from conftest import load_golden


@pytest.mark.parametrize("nu", [1.0, 6.0])
def test_nodes_through_dead_entries_are_zero(nu):
    from oracle.quadrature import Problem
    z = load_golden("garch_student_n64")
    x = z["x_values"]
    sig = np.array(z["sigma_forecasts"], dtype=np.float64)[:6]
    xmax = float(np.max(np.abs(x)))
    sig[0::2] = xmax / 70.0                                  # grid edges at |x| / sigma ~ 70: u in {0, 1}
    sig[1, 0] = xmax / 8.0                                    # u down to ~1e-16, still inside (0, 1)
    P = Problem("garch", "student", 2, x, z["step"], z["densities"], z["combos"], z["weights"],
                np.array([nu, 0.5]), sig)
    seen_dead = 0
    for t in range(P.T):
        u, _ = P.axis_cdf(t)
        dead = (u == 0.0) | (u == 1.0)                       # (dim, n)
        m = P.mass(t)
        through = dead[0][:, None] | dead[1][None, :]
        seen_dead += int(through.sum())
        assert np.all(m[through] == 0.0), t
        assert np.all(np.isfinite(m)), t                     # no node becomes +-inf (nan_to_num's DBL_MAX)
        live = ~through
        assert np.all(m[live] >= 0.0)
        # u strictly inside (0, 1) is >= 2^-54: 1 + erf rounds to 0 or to >= 2^-53
        inside = u[(u > 0.0) & (u < 1.0)]
        assert inside.size == 0 or inside.min() >= 2.0 ** -54
    assert seen_dead > 0
