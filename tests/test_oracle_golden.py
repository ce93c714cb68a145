"""The CPU oracle vs the reference's golden vectors (CPU only, no GPU).

The goldens (tests/golden/*.npz) were produced by running the reference itself
in the build container (tests/golden/gen_golden.py).  Pinning the oracle to
them is what lets the GPU parity tests use the oracle as their checker.

Bars: every golden VaR reproduced bit-for-bit with the reference's iteration
count; every recorded compute_integral call within 1e-10 relative + 1e-15
absolute (the oracle sums in a different order than the reference's
np.sum over the nested grid); forecast tables within 1e-12 relative.
"""
import numpy as np
import pytest

from conftest import GOLDEN_CASES, golden_calls, golden_kwargs, load_golden

SLAB_RTOL, SLAB_ATOL = 1e-10, 1e-15
TABLE_RTOL = 1e-12

# n=256 / n=128 3-D goldens take a few seconds each through the numpy oracle
FAST = [c for c in GOLDEN_CASES if c not in ("cfg2_n256", "cfg3_n128")]


def _problem(z):
    from oracle.quadrature import Problem
    model = str(z["model"])
    per = (z["forecasts_by_states"], z["forecasts"]) if model == "msm" else z["sigma_forecasts"]
    return Problem(model, str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                   z["combos"], z["weights"], z["copula_params"], per, z.get("unique_vol_states"))


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_oracle_calc_var_bit_exact(case):
    from oracle.quadrature import calc_var
    z = load_golden(case)
    P = _problem(z)
    var, iters, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]), **golden_kwargs(z))
    assert np.array_equal(var, z["var"]), f"{case}: {np.max(np.abs(var - z['var']))}"
    assert iters == int(z["n_calls"]) - 2


@pytest.mark.parametrize("case", FAST)
def test_oracle_slabs_match_every_recorded_call(case):
    z = load_golden(case)
    P = _problem(z)
    for i, (b, ref) in enumerate(golden_calls(z)):
        np.testing.assert_allclose(P.compute_integral(b), ref, rtol=SLAB_RTOL, atol=SLAB_ATOL,
                                   err_msg=f"{case} call {i}")


@pytest.mark.parametrize("case", [c for c in GOLDEN_CASES if c != "cfg1_kwargs"])
def test_oracle_forecast_tables(case):
    from oracle import forecast as F
    z = load_golden(case)
    n_in, model = int(z["n_in"]), str(z["model"])
    mp = [dict(zip(list(z["model_param_names"]), row)) for row in z["model_params"]]
    mean, ptf, win = F.insample_split(z["returns"], n_in, z["weights"])
    assert ptf == float(z["ptf_mean"])
    if model == "msm":
        k = int(z["k"])
        got = F.msm_integration_params(win, mp, k, int(z["num_points"]))
        for key in ("forecasts_by_states", "forecasts", "unique_vol_states", "densities"):
            np.testing.assert_allclose(got[key], z[key], rtol=TABLE_RTOL * 100, atol=1e-300, err_msg=key)
        for key in ("x_values", "step"):
            assert np.array_equal(got[key], z[key]), key
        assert np.array_equal(got["combos"], z["combos"])
    else:
        got = F.sigma_forecasts(win, model, mp)
        np.testing.assert_allclose(got, z["sigma_forecasts"], rtol=TABLE_RTOL)


def test_joblib_port_matches_oracle_on_a_golden_case():
    """The CPU baseline (joblib, scalar t.ppf) is the same algorithm: same VaR."""
    from oracle.joblib_port import JoblibPath
    z = load_golden("cfg2_n64")
    P = _problem(z)
    J = JoblibPath(P, n_jobs=2)
    var, iters, _ = J.calc_var(float(z["ptf_mean"]))
    assert np.array_equal(var, z["var"])
    assert iters == int(z["n_calls"]) - 2


def test_q1_case_is_covered():
    """The goldens must exercise Q1 (second bracket (-3,-2] -> prev_upper -3) and
    its [-2, 0] bisection bracket (calc_var_class.py:132, :151-155)."""
    seen = set()
    for case in GOLDEN_CASES:
        z = load_golden(case)
        b1 = z["call01_bounds"]
        seen |= {tuple(r) for r in np.round(b1, 6)}
    assert (-3.0, -2.0) in seen and (-3.5, -3.0) in seen


def test_fullbatch_fixtures_are_consistent():
    """The full-batch fixtures (gen_fullbatch.py) hold what the GPU tests compare against:
    the whole batch, finite VaRs, the global iteration count of a solve without a Q4 break,
    and the oracle's forecast tables for the first dates (re-derived here on the CPU)."""
    import os
    from conftest import GOLDEN
    from copula_var import synthetic
    from oracle import forecast as F
    for cfg, T in ((2, 1000), (5, 5000), (3, 5000), (4, 250)):
        path = os.path.join(GOLDEN, f"fullbatch_cfg{cfg}.npz")
        z = dict(np.load(path, allow_pickle=False))
        assert int(z["T"]) == T and z["var"].shape == (T,) and not np.isnan(z["var"]).any()
        assert 19 <= int(z["iterations"]) <= 22 and not bool(z["broke"])
        c = synthetic.baseline_configs()[cfg]
        rets = synthetic.simulate_returns(c)
        # the stored returns (the e2e GPU test's input) are the BASELINE batch's, cut to T dates
        np.testing.assert_array_equal(z["returns"], rets[: c.n_in + T])
        assert int(z["n_in"]) == c.n_in
        # first dates' windows (cfg 4, k = 6: all of its 250, as generated -- the batched filter's
        # 64-state matmuls round differently per batch shape)
        m4 = T if cfg == 4 else 4
        _, ptf, windows = F.insample_split(rets[:c.n_in + m4], c.n_in, c.weights)
        assert ptf == float(z["ptf_mean"])
        if c.model == "msm":
            m = F.msm_integration_params(windows, c.msm_params, c.k, c.num_points)
            np.testing.assert_array_equal(m["forecasts_by_states"], z["forecasts_by_states"][:m4])
        else:
            np.testing.assert_array_equal(F.sigma_forecasts(windows, c.model, c.model_params()),
                                          z["sigma_forecasts"][:m4])


def test_q4_zero_case_oracle():
    """The constructed Q4 case (tests/q4_zero_case.py): the oracle breaks on the all-zero
    iteration with the bracket midpoint, as the reference's loop does (calc_var_class.py:293)."""
    from oracle.quadrature import Problem, calc_var
    from q4_zero_case import CASES, build
    for l22, (var_ref, it_ref) in CASES.items():
        z = build(l22)
        P = Problem(z["model"], z["copula"], 2, z["x_values"], z["step"], z["densities"], z["combos"],
                    z["weights"], z["copula_params"], (z["forecasts_by_states"], z["forecasts"]),
                    z["unique_vol_states"])
        m = P.mass(0)
        assert np.count_nonzero(m) == 4 and np.all(m[m != 0] == 2.0 ** -8)
        var, it, broke = calc_var(P.compute_integral, P.T, z["ptf_mean"])
        assert broke and it == it_ref
        np.testing.assert_array_equal(var, np.full(P.T, var_ref))
