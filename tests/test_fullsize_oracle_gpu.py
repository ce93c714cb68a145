"""Full-size parity against the oracle, independent of the plan's host v* tables.

Every device strategy consumes host-computed geometry (COMPACT's v* and cut tables,
SORTED's v*-sorted node list), so a full-size device-vs-device check cannot see an
error in that shared geometry.  Here the HIP solve is compared with
``oracle.quadrature`` -- whole-box masses + boolean membership masks
(create_grids.py:102-108, integration_algo.py:20), no v* anywhere -- on a few dates
taken from each BASELINE workload at its full grid size:

* cfg 2 (MSM Student, n = 256): 8 dates of the 1000-date workload, COMPACT (auto);
* cfg 3 (GARCH Plackett, n = 512): 4 dates of the 5000-date workload, SORTED (auto);
* cfg 5 (UKF Student, n = 256): 4 dates of the 5000-date workload, COMPACT (auto);
* cfg 1 (GARCH Gaussian, n = 64): all 50 dates.

The dates are spread over the VaR range of the full batch (so every bracket class
that occurs is sampled).  Bars: VaR bit-identical with the same bisection count,
slabs (-100, -3] and (-3, -2] within 1e-10 relative + 1e-15 absolute.

Also: strategy "auto" above the v_cap of a materialised strategy (SORTED holds the
nodes with level <= 0) routes to an unrestricted sibling plan instead of failing.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SLAB_RTOL, SLAB_ATOL = 1e-10, 1e-15

FULL = [(2, 1000, 8), (3, 5000, 4), (5, 5000, 4), (1, 50, 50)]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _workload(cfg_no, T, **kw):
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[cfg_no].with_(T=T, **kw)
    rets = synthetic.simulate_returns(c)
    _, ptf_mean, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    return c, ipt, uvs, ggp, ptf_mean


def _subset(c, ipt, idx):
    return (ipt[0][idx], ipt[1][idx]) if c.model == "msm" else [ipt[0][idx]]


def _plan(c, ipt, uvs, ggp, strategy="auto"):
    from copula_var.engine import QuadraturePlan
    dens, x, step, combos = ggp
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                       vol_states=uvs, strategy=strategy)
    p.set_dates(ipt)
    return p


def _problem(c, ipt, uvs, ggp):
    from oracle.quadrature import Problem
    dens, x, step, combos = ggp
    per = ipt if c.model == "msm" else ipt[0]
    return Problem(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(), per, uvs)


@pytest.mark.parametrize("cfg,T,S", FULL)
def test_full_size_dates_match_oracle(cfg, T, S):
    from oracle.quadrature import calc_var
    c, ipt, uvs, ggp, ptf = _workload(cfg, T)
    p = _plan(c, ipt, uvs, ggp)
    try:
        full, _ = p.calc_var(ptf)
    finally:
        p.close()
    assert not np.isnan(full).any()
    # S dates spread over the full batch's VaR range (sorted order, evenly spaced ranks)
    order = np.argsort(full, kind="stable")
    idx = np.sort(order[np.linspace(0, T - 1, S).round().astype(int)])
    sub = _subset(c, ipt, idx)
    P = _problem(c, sub, uvs, ggp)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, ptf)
    p = _plan(c, sub, uvs, ggp)
    try:
        var, it = p.calc_var(ptf)
        for b in ([-100.0, -3.0], [-3.0, -2.0]):
            bounds = np.tile(b, (P.T, 1))
            np.testing.assert_allclose(p.compute_integral(bounds), P.compute_integral(bounds), rtol=SLAB_RTOL,
                                       atol=SLAB_ATOL, err_msg=f"cfg {cfg} slab {b}")
    finally:
        p.close()
    assert it == ref_it, (it, ref_it)
    assert np.array_equal(var, ref), (cfg, float(np.max(np.abs(var - ref))))


@pytest.mark.parametrize("case", ["cfg1", "ukf_plackett_n64", "cfg4_k4_n16"])
def test_auto_routes_levels_above_v_cap(case):
    """auto = SORTED for 2-D GARCH / UKF with a Gaussian or Plackett copula and for 3-D;
    SORTED holds nodes up to v_cap = 0:
    slabs and a solve that reach above 0 go to an unrestricted sibling (COMPACT in 2-D,
    SORTED with v_cap at the grid's top in 3-D) and still match the oracle."""
    from conftest import load_golden
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden(case)
    msm = str(z["model"]) == "msm"
    vs = z.get("unique_vol_states")
    per = (z["forecasts_by_states"], z["forecasts"]) if msm else z["sigma_forecasts"]
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=vs, strategy="auto")
    P = Problem(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                z["combos"], z["weights"], z["copula_params"], per, vs)
    try:
        assert p.strategy == "sorted"
        p.set_dates(per if msm else [per])
        for b in ([-1.0, 0.5], [0.25, 3.0], [-100.0, 100.0]):
            bounds = np.tile(b, (P.T, 1))
            np.testing.assert_allclose(p.compute_integral(bounds), P.compute_integral(bounds), rtol=SLAB_RTOL,
                                       atol=SLAB_ATOL, err_msg=str(b))
        ref, ref_it, _ = calc_var(P.compute_integral, P.T, 0.0, first_guess=0.25)
        var, it = p.calc_var(0.0, first_guess=0.25)
        assert it == ref_it
        assert np.array_equal(var, ref)
        # below v_cap the plan itself serves (no sibling needed for the default solve)
        var0, _ = p.calc_var(0.0)
        ref0, _, _ = calc_var(P.compute_integral, P.T, 0.0)
        assert np.array_equal(var0, ref0)
    finally:
        p.close()


def test_explicit_sorted_still_refuses_above_v_cap():
    """An explicit strategy keeps the documented CVQ_ERR_RANGE contract."""
    from conftest import load_golden
    from copula_var import _native as N
    from copula_var.engine import QuadraturePlan
    z = load_golden("cfg1")
    p = QuadraturePlan("garch", "gaussian", 2, z["x_values"], z["step"], z["densities"], z["combos"], z["weights"],
                       z["copula_params"], strategy="sorted")
    try:
        p.set_dates([z["sigma_forecasts"]])
        with pytest.raises((ValueError, N.NativeError)):
            p.compute_integral(np.tile([-1.0, 0.5], (p.T, 1)))
    finally:
        p.close()


def test_fast_path_proof_boundary_sigma_xmax_over_6_nu1():
    """cvq_set_dates proves COMPACT's fast path for GARCH / UKF host inputs when
    |x| / sigma <= 6 (u >= Phi(-6) ~ 9.87e-10, finite t.ppf even at nu = 1).  At the
    boundary sigma = xmax / 6 exactly, with Student nu = 1, the solve must succeed on
    the fast path and match the oracle."""
    from conftest import load_golden
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("garch_student_n64")
    x = z["x_values"]
    sig = np.array(z["sigma_forecasts"], dtype=np.float64)
    xmax = float(np.max(np.abs(x)))
    sig[: max(1, sig.shape[0] // 2)] = xmax / 6.0                 # boundary dates
    cp = np.array([1.0, 0.5])
    args = ("garch", "student", 2, x, z["step"], z["densities"], z["combos"], z["weights"], cp)
    P = Problem(*args, sig)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, 0.0)
    p = QuadraturePlan(*args, strategy="compact")
    try:
        p.set_dates([sig])
        var, it = p.calc_var(0.0)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref, equal_nan=True)


@pytest.mark.parametrize("nu", [1.0, 6.0])
@pytest.mark.parametrize("strategy", ["compact", "sorted"])
def test_fast_path_dead_entries_small_sigma(strategy, nu):
    """GARCH / UKF Student dates whose grid reaches |x| / sigma ~ 70 (u = 0 or 1 at the grid
    edges: z = +-inf, the reference zeroes those nodes) and ~ 8 (u down to ~1e-16: the
    largest finite quantiles) take the fast path with dead records (r05; cfg 5 has such
    dates): VaR bit-identical to the oracle, with the host's fast-path proof (COMPACT skips
    its generic kernel) and in SORTED's per-date check."""
    from conftest import load_golden
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("garch_student_n64")
    x = z["x_values"]
    sig = np.array(z["sigma_forecasts"], dtype=np.float64)
    xmax = float(np.max(np.abs(x)))
    sig[0::3] = xmax / 70.0
    sig[1::3, 0] = xmax / 8.0
    cp = np.array([nu, 0.5])
    args = ("garch", "student", 2, x, z["step"], z["densities"], z["combos"], z["weights"], cp)
    P = Problem(*args, sig)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, 0.0)
    p = QuadraturePlan(*args, strategy=strategy)
    try:
        p.set_dates([sig])
        var, it = p.calc_var(0.0)
        b = np.tile([-3.0, -2.0], (P.T, 1))
        np.testing.assert_allclose(p.compute_integral(b), P.compute_integral(b), rtol=SLAB_RTOL, atol=SLAB_ATOL)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref, equal_nan=True)


@pytest.mark.parametrize("case", ["cfg1", "cfg5_n64", "cfg4_k4_n16", "cfg3_n128"])
@pytest.mark.parametrize("strategy", ["sorted", "prefix", "compact"])
def test_slabs_ending_at_zero(case, strategy):
    """Slabs whose upper bound is 0 (the default v_cap): the nodes on the anti-diagonal have
    v* ~ -ulp(level) / 2, found by the host's ordered-integer bisection (vstar_exact); a
    signed overflow there once sent them to +inf, so SORTED dropped them from every slab
    ending at 0 (a solve never reaches them)."""
    from conftest import load_golden
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem
    z = load_golden(case)
    if strategy == "compact" and int(z["dim"]) != 2:
        pytest.skip("COMPACT is 2-D")
    msm = str(z["model"]) == "msm"
    vs = z.get("unique_vol_states")
    per = (z["forecasts_by_states"], z["forecasts"]) if msm else z["sigma_forecasts"]
    P = Problem(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                z["combos"], z["weights"], z["copula_params"], per, vs)
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=vs, strategy=strategy)
    try:
        p.set_dates(per if msm else [per])
        for b in ([-1e-15, 0.0], [-0.1, 0.0], [-2.0, 0.0], [-100.0, 0.0]):
            bounds = np.tile(b, (P.T, 1))
            np.testing.assert_allclose(p.compute_integral(bounds), P.compute_integral(bounds), rtol=SLAB_RTOL,
                                       atol=SLAB_ATOL, err_msg=f"{case} {strategy} {b}")
    finally:
        p.close()


@pytest.mark.parametrize("strategy", ["auto", "compact", "sorted", "direct", "prefix"])
def test_2d_grid_above_512_refused_at_creation(strategy):
    """2-D num_points in (512, 1024] runs on SORTED only (r06; auto picks it): every other strategy
    refuses it when the plan is created, and every strategy refuses n > 1024 there (ADVICE r03
    feared an 'auto' plan that builds and then fails every solve).  The SORTED solves at n = 700 /
    1024 are checked against the oracle in tests/test_large_grid_gpu.py."""
    from copula_var import synthetic, tables
    for n, ok in ((600, strategy in ("auto", "sorted")), (1025, False)):
        c = synthetic.baseline_configs()[1].with_(T=4, num_points=n)
        rets = synthetic.simulate_returns(c)
        _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
        if ok:
            p = _plan(c, ipt, uvs, ggp, strategy=strategy)
            try:
                assert p.strategy == "sorted"
                var, it = p.calc_var(ptf)
                assert np.all(np.isfinite(var))
            finally:
                p.close()
        else:
            with pytest.raises(ValueError, match="512|1024"):
                _plan(c, ipt, uvs, ggp, strategy=strategy)


@pytest.mark.parametrize("case", ["cfg1", "cfg4_k4_n16"])
def test_auto_routes_device_solves_above_v_cap(case):
    """solve_device / solve_local on an 'auto' SORTED plan with a guess above v_cap = 0 route to
    the unrestricted sibling, on the plan's stream (only the host entry points did)."""
    import torch
    from conftest import load_golden
    from copula_var.engine import QuadraturePlan, solve_args
    from oracle.quadrature import Problem, calc_var
    z = load_golden(case)
    msm = str(z["model"]) == "msm"
    vs = z.get("unique_vol_states")
    per = (z["forecasts_by_states"], z["forecasts"]) if msm else z["sigma_forecasts"]
    P = Problem(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                z["combos"], z["weights"], z["copula_params"], per, vs)
    ref, _, _ = calc_var(P.compute_integral, P.T, 0.0, first_guess=0.25)
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=vs, strategy="auto")
    s = torch.cuda.Stream()
    try:
        assert p.strategy == "sorted"
        p.set_stream(s.cuda_stream)
        p.set_dates(per if msm else [per])
        args = solve_args(0.0, first_guess=0.25)
        out = torch.empty(P.T, dtype=torch.float64, device="cuda")
        with torch.cuda.stream(s):
            p.solve_device(args, out.data_ptr())
        p.solve_status()
        s.synchronize()
        assert p._wide is not None and p._wide._stream == s.cuda_stream
        assert np.array_equal(out.cpu().numpy(), ref)
        # the sharded entry points: local solve on the sibling, finalize on this plan
        ln, hoff = QuadraturePlan.packed_block_len(args, P.T)
        blk = torch.zeros(ln, dtype=torch.float64, device="cuda")
        with torch.cuda.stream(s):
            p.solve_local(args, blk[hoff:].data_ptr(), blk.data_ptr())
            p.solve_finalize_packed(args, blk.data_ptr(), 1, P.T, P.T, out.data_ptr())
        p.solve_status()
        assert np.array_equal(out.cpu().numpy(), ref)
    finally:
        p.close()


@pytest.mark.parametrize("strategy", ["auto", "compact", "sorted"])
@pytest.mark.parametrize("cfg,T,S", [(2, 1000, 4), (5, 5000, 4)])
def test_fitted_nu_full_size_matches_oracle(cfg, T, S, strategy):
    """A fitted (non-integer) Student nu -- 5.364, SURVEY.md's measured scipy case -- takes the
    general node power b^-(nu+2)/2 = exp(ex log b) (cvq_special.h pow_node: log_node /
    exp_node) and the general t.ppf tables: full-size cfg 2 / cfg 5 workloads, S dates spread
    over the VaR range against the oracle (VaR bit-identical, same bisection count), and the
    whole batch free of NaN."""
    from oracle.quadrature import calc_var
    c, ipt, uvs, ggp, ptf = _workload(cfg, T, nu=5.364)
    p = _plan(c, ipt, uvs, ggp, strategy=strategy)
    try:
        full, _ = p.calc_var(ptf)
    finally:
        p.close()
    assert not np.isnan(full).any()
    order = np.argsort(full, kind="stable")
    idx = np.sort(order[np.linspace(0, T - 1, S).round().astype(int)])
    sub = _subset(c, ipt, idx)
    P = _problem(c, sub, uvs, ggp)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, ptf)
    p = _plan(c, sub, uvs, ggp, strategy=strategy)
    try:
        var, it = p.calc_var(ptf)
        bounds = np.tile([-3.0, -2.0], (P.T, 1))
        np.testing.assert_allclose(p.compute_integral(bounds), P.compute_integral(bounds), rtol=SLAB_RTOL,
                                   atol=SLAB_ATOL)
    finally:
        p.close()
    assert it == ref_it, (it, ref_it)
    assert np.array_equal(var, ref), (cfg, strategy, float(np.max(np.abs(var - ref))))


@pytest.mark.parametrize("strategy", ["sorted", "sweep", "compact"])
@pytest.mark.parametrize("theta", [1.0, 1.5, 6.0])
def test_plackett_theta_range_matches_oracle(theta, strategy):
    """The Plackett node (plackett.py:66-69) across its parameter: theta = 1 (independence,
    a1 = 0), 1.5 (denominator bounded away from 0) and 6 (its zero line u + v = 1 + 1/a1
    crosses the square) on cfg 3's 512^2 geometry.  SORTED / SWEEP evaluate it from
    precomputed records (-2 u, theta s), ((theta - 1) v, s) with one Newton step on the
    reciprocal, COMPACT from its row constants: S = 3 dates spread over the VaR range of a
    200-date batch against the oracle, VaR bit-identical with the same bisection count."""
    from oracle.quadrature import calc_var
    c, ipt, uvs, ggp, ptf = _workload(3, 200, theta=theta)
    p = _plan(c, ipt, uvs, ggp, strategy=strategy)
    try:
        full, _ = p.calc_var(ptf)
    finally:
        p.close()
    assert not np.isnan(full).any()
    order = np.argsort(full, kind="stable")
    idx = np.sort(order[np.linspace(0, 199, 3).round().astype(int)])
    sub = _subset(c, ipt, idx)
    P = _problem(c, sub, uvs, ggp)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, ptf)
    p = _plan(c, sub, uvs, ggp, strategy=strategy)
    try:
        var, it = p.calc_var(ptf)
    finally:
        p.close()
    assert it == ref_it, (it, ref_it)
    assert np.array_equal(var, ref), (theta, strategy, float(np.max(np.abs(var - ref))))
