"""HIP path vs the reference's golden vectors (and the oracle) -- needs an MI355X.

Bars (north_star): VaR within 1e-9 relative of the reference (in practice
bit-identical: every bisection decision matches); per-call slab integrals within
1e-10 relative + 1e-15 absolute (summation order differs; slabs are differences of
row prefix sums, and each one is added to an F of order 0.05, so an absolute floor
far below F's own rounding is the meaningful bar); forecast tables within 1e-12
relative.
"""
import numpy as np
import pytest

from conftest import GOLDEN_CASES, golden_calls, golden_kwargs, load_golden

pytestmark = pytest.mark.gpu

VAR_RTOL = 1e-9
SLAB_RTOL = 1e-10
SLAB_ATOL = 1e-15
TABLE_RTOL = 1e-12


def _plan(z, **kw):
    from copula_var.engine import QuadraturePlan
    model = str(z["model"])
    p = QuadraturePlan(model, str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"],
                       vol_states=z.get("unique_vol_states"), **kw)
    if model == "msm":
        p.set_dates((z["forecasts_by_states"], z["forecasts"]))
    else:
        p.set_dates([z["sigma_forecasts"]])
    return p


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def test_special_functions_vs_scipy_and_mpmath():
    """Device t.ppf / norm.ppf / erf vs scipy (the reference's own special functions)
    where scipy is accurate, and vs mpmath ground truth over the full range
    (scipy's stdtrit is clamped at |t| = 1e100 and loses accuracy below u ~ 1e-150)."""
    from copula_var import _native as N
    k = np.load(__import__("conftest").GOLDEN + "/kat_special.npz")
    u = k["u"]
    for nu in k["tppf_nus"]:
        ref = k[f"tppf_nu{nu:g}"]
        got = N.special("tppf", u, nu=nu)
        assert np.array_equal(np.isfinite(got), np.isfinite(ref)), nu
        ok = np.isfinite(ref) & (u >= 1e-150) & (u <= 1 - 1e-16) & (np.abs(ref) < 1e99) & (np.abs(ref) > 1e-6)
        rel = np.abs(got[ok] - ref[ok]) / np.abs(ref[ok])
        assert rel.max() < 1e-10, (nu, rel.max())           # scipy itself is ~1e-11 accurate
        near = np.abs(ref) <= 1e-6                            # p ~ 0.5: absolute accuracy
        assert np.max(np.abs(got[near] - ref[near]), initial=0) < 1e-15
    ut = k["truth_u"]
    for nu in (1.0, 3.0, 6.0, 30.0):
        tr = k[f"truth_tppf_nu{nu:g}"]
        got = N.special("tppf", ut, nu=nu)
        rel = np.abs(got - tr) / np.abs(tr)
        assert rel.max() < 1e-13, (nu, rel.max())
    got = N.special("ndtri", u)
    ref = k["ndtri"]
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    assert np.all(np.abs(got[fin] - ref[fin]) <= 1e-13 * np.abs(ref[fin]) + 1e-16)
    # the device norm.ppf restates scipy's own (Cephes) ndtri: within 4 ulp of it everywhere
    assert np.all(np.abs(got[fin] - ref[fin]) <= 4 * np.spacing(np.abs(ref[fin]))), \
        np.max(np.abs(got[fin] - ref[fin]) / np.spacing(np.abs(ref[fin])))
    # the solve kernels' t.ppf for nu = 6 (float-seeded root p^(1/6), no exp/log): same tables,
    # ~1e-14 relative vs mpmath (far inside the 1e-8 node noise the VaR tolerates)
    tr = k["truth_tppf_nu6"]
    got = N.special("tppf6", ut, nu=6.0)
    rel = np.abs(got - tr) / np.abs(tr)
    assert rel.max() < 1e-13, rel.max()
    ref6 = N.special("tppf", u, nu=6.0)
    ok = np.isfinite(ref6) & (np.abs(ref6) > 1e-6)
    assert np.array_equal(np.isfinite(N.special("tppf6", u, nu=6.0)), np.isfinite(ref6))
    assert np.max(np.abs(N.special("tppf6", u, nu=6.0)[ok] - ref6[ok]) / np.abs(ref6[ok])) < 1e-13
    got = N.special("erf", k["erf_x"])
    assert np.max(np.abs(got - k["erf"])) <= 2.3e-16


STRATEGIES = ["prefix", "direct", "compact", "sorted", "sweep"]


def _skip_unsupported(z, strategy):
    if strategy in ("direct", "compact", "sweep") and int(z["dim"]) != 2:
        pytest.skip("DIRECT, COMPACT and SWEEP strategies are built for dim == 2")


@pytest.mark.parametrize("strategy", STRATEGIES)
@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_slab_integrals_match_reference(case, strategy):
    z = load_golden(case)
    _skip_unsupported(z, strategy)
    p = _plan(z, strategy=strategy)
    try:
        for i, (b, ref) in enumerate(golden_calls(z)):
            got = p.compute_integral(b)
            np.testing.assert_allclose(got, ref, rtol=SLAB_RTOL, atol=SLAB_ATOL, err_msg=f"{case} call {i}")
    finally:
        p.close()


@pytest.mark.parametrize("strategy", STRATEGIES)
@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_calc_var_matches_reference(case, strategy):
    z = load_golden(case)
    _skip_unsupported(z, strategy)
    p = _plan(z, strategy=strategy)
    try:
        var, iters = p.calc_var(float(z["ptf_mean"]), **golden_kwargs(z))
    finally:
        p.close()
    ref = z["var"]
    np.testing.assert_allclose(var, ref, rtol=VAR_RTOL, atol=0)
    assert np.array_equal(var, ref), f"{case}: not bit-identical (max diff {np.max(np.abs(var - ref))})"
    # bisection iterations the reference ran = compute_integral calls - 2
    assert iters == int(z["n_calls"]) - 2


@pytest.mark.parametrize("case", [c for c in GOLDEN_CASES if not c.startswith("cfg1_kwargs")])
def test_forecast_stage_matches_reference(case):
    from copula_var import engine
    from oracle import forecast as F
    z = load_golden(case)
    n_in = int(z["n_in"])
    names = list(z["model_param_names"])
    mp = [dict(zip(names, row)) for row in z["model_params"]]
    mean, ptf, win = F.insample_split(z["returns"], n_in, z["weights"])
    rc = (z["returns"] - mean)[:-1]          # windows i:i+n_in, i < T  (load_data.py:131-132)
    for d in range(int(z["dim"])):
        p = mp[d]
        if str(z["model"]) == "msm":
            got = engine.msm_filter(rc[:, d], n_in, int(z["k"]), p["m_0"], p["sig"], p["b"], p["gamma"])
            ref = z["filtered_probs"][d]
            np.testing.assert_allclose(got, ref, rtol=TABLE_RTOL * 100, atol=1e-300)
        elif str(z["model"]) == "garch":
            got = engine.garch_forecast(rc[:, d], n_in, p["omega"], p["alpha"], p["beta"])
            np.testing.assert_allclose(got, z["sigma_forecasts"][:, d], rtol=TABLE_RTOL)
        else:
            got = engine.ukf_forecast(rc[:, d], n_in, p["a"], p["l"], p["q"])
            np.testing.assert_allclose(got, z["sigma_forecasts"][:, d], rtol=TABLE_RTOL)


@pytest.mark.parametrize("strategy", ["compact", "sorted"])
def test_node_count_measurement(strategy):
    """cvq_plan_count_nodes (bench.py's FP64 roofline basis): a counted solve returns the same
    VaR, and every date evaluates at least its first fixed slab and at most ~the reachable set
    (COMPACT's block tail evaluates its whole last cell once, so a little above the path)."""
    z = load_golden("cfg2_n64")
    p = _plan(z, strategy=strategy)
    ptf = float(z["ptf_mean"])
    v0, _ = p.calc_var(ptf)
    p.count_nodes(True)
    v1, _ = p.calc_var(ptf)
    nodes = p.nodes_evaluated()
    p.count_nodes(False)
    assert np.array_equal(v0, v1, equal_nan=True)
    T = v0.size
    assert 0.2 * p.reach_nodes * T < nodes <= 1.2 * p.reach_nodes * T, (nodes, p.reach_nodes, T)
    p.calc_var(ptf)
    with pytest.raises(RuntimeError):
        p.nodes_evaluated()                 # the last solve was not counted
    with pytest.raises(ValueError):
        _plan(z, strategy="prefix").count_nodes(True)
