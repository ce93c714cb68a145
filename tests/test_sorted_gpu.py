"""SORTED strategy on the GPU (reachable nodes sorted by their exact membership
threshold v*; a slab is one contiguous range of the sorted list).

* BASELINE config 4's full geometry (3 assets, n = 128, MSM k = 6, Q = 343) against
  the oracle on a few dates -- the shape no other strategy supports;
* against PREFIX (an independent device strategy) where PREFIX fits (3-D, n = 64),
  over many dates, bit-identical VaR;
* against COMPACT at config 2's full size (1000 dates);
* the generic node path (a non-rank-1 pi, reference-semantics W contraction);
* the sharded entry points (solve_local / finalize across R plans).
Bars: VaR bit-identical, bisection count equal; slabs within 1e-10 rel + 1e-15 abs.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu

SLAB_RTOL, SLAB_ATOL = 1e-10, 1e-15


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _workload(cfg_no, T, n=None):
    """Synthetic per-date tables of a BASELINE config (device forecast filters)."""
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[cfg_no]
    c = c.with_(T=T, num_points=n or c.num_points)
    rets = synthetic.simulate_returns(c)
    _, ptf_mean, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    return c, ipt, uvs, ggp, ptf_mean


def _plan(c, ipt, uvs, ggp, strategy, sl=slice(None)):
    from copula_var.engine import QuadraturePlan
    dens, x, step, combos = ggp
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                       vol_states=uvs, strategy=strategy)
    if c.model == "msm":
        p.set_dates((ipt[0][sl], ipt[1][sl]))
    else:
        p.set_dates([ipt[0][sl]])
    return p


def _problem(c, ipt, uvs, ggp, sl=slice(None)):
    from oracle.quadrature import Problem
    dens, x, step, combos = ggp
    per = (ipt[0][sl], ipt[1][sl]) if c.model == "msm" else ipt[0][sl]
    return Problem(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(), per, uvs)


def test_cfg4_full_geometry_matches_oracle():
    from oracle.quadrature import calc_var
    c, ipt, uvs, ggp, ptf = _workload(4, 3)
    P = _problem(c, ipt, uvs, ggp)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, ptf)
    p = _plan(c, ipt, uvs, ggp, "sorted")
    try:
        assert p.reach_nodes == 1049622                     # SURVEY.md §8 geometry table, cfg 4
        var, it = p.calc_var(ptf)
        for b in ([-100.0, -3.0], [-3.0, -2.0], [-2.0, -1.0], [-1.25, -1.0]):
            bounds = np.tile(b, (P.T, 1))
            np.testing.assert_allclose(p.compute_integral(bounds), P.compute_integral(bounds), rtol=SLAB_RTOL,
                                       atol=SLAB_ATOL)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref), (var, ref)


def test_3d_sorted_matches_prefix_many_dates():
    c, ipt, uvs, ggp, ptf = _workload(4, 400, n=64)
    out = {}
    for strategy in ("prefix", "sorted"):
        p = _plan(c, ipt, uvs, ggp, strategy)
        try:
            out[strategy] = p.calc_var(ptf)
        finally:
            p.close()
    (vp, ip), (vs, is_) = out["prefix"], out["sorted"]
    assert ip == is_
    assert np.array_equal(vp, vs), float(np.nanmax(np.abs(vp - vs)))


def test_cfg2_full_size_sorted_matches_compact():
    c, ipt, uvs, ggp, ptf = _workload(2, 1000)
    out = {}
    for strategy in ("compact", "sorted", "sweep"):
        p = _plan(c, ipt, uvs, ggp, strategy)
        try:
            out[strategy] = p.calc_var(ptf)
        finally:
            p.close()
    for strategy in ("sorted", "sweep"):
        assert out["compact"][1] == out[strategy][1]
        assert np.array_equal(out["compact"][0], out[strategy][0]), strategy


@pytest.mark.parametrize("cfg,T", [(1, 50), (3, 1000), (5, 1000)])
def test_full_size_sweep_matches_sorted(cfg, T):
    """SWEEP (one pass per bisection cell, slabs as prefix differences) against SORTED
    (one strided range sum per level) at the BASELINE geometries: bit-identical VaR."""
    c, ipt, uvs, ggp, ptf = _workload(cfg, T)
    out = {}
    for strategy in ("sorted", "sweep"):
        p = _plan(c, ipt, uvs, ggp, strategy)
        try:
            out[strategy] = p.calc_var(ptf)
        finally:
            p.close()
    assert out["sorted"][1] == out["sweep"][1]
    assert np.array_equal(out["sorted"][0], out["sweep"][0])


@pytest.mark.parametrize("case,strategy", [("cfg4_k4_n16", "sorted"), ("cfg2_n64", "sorted"), ("cfg2_n64", "sweep"),
                                           ("cfg2_n64", "compact")])
def test_generic_path_non_rank1_pi(case, strategy):
    """A pi that is not the product of per-asset forecasts forces the generic node
    path (full W contraction, create_grids.py:121-171); VaR must follow the oracle."""
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden(case)
    fbs = z["forecasts_by_states"]
    pi = z["forecasts"].copy()
    rng = np.random.default_rng(7)
    pi[::2] *= rng.uniform(0.9, 1.1, size=pi[::2].shape)          # every other date: not rank 1
    args = (str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
            z["combos"], z["weights"], z["copula_params"])
    P = Problem(*args, (fbs, pi), z["unique_vol_states"])
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
    p = QuadraturePlan(*args, vol_states=z["unique_vol_states"], strategy=strategy)
    try:
        p.set_dates((fbs, pi))
        var, it = p.calc_var(float(z["ptf_mean"]))
        b = np.tile([-3.0, -2.0], (P.T, 1))
        np.testing.assert_allclose(p.compute_integral(b), P.compute_integral(b), rtol=SLAB_RTOL, atol=SLAB_ATOL)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref)


@pytest.mark.parametrize("case,ranks,strategy", [("cfg4_k6_n16", 2, "sorted"), ("cfg2_n64", 3, "sorted"),
                                                 ("cfg1", 2, "sorted"), ("cfg2_n64", 3, "sweep"),
                                                 ("cfg1", 2, "sweep")])
def test_sharded_sorted(case, ranks, strategy):
    from copula_var import engine
    from copula_var.distributed import shard
    from copula_var.engine import QuadraturePlan
    z = load_golden(case)
    T = z["var"].size
    args = engine.solve_args(float(z["ptf_mean"]))
    stride = QuadraturePlan.snap_stride(args)
    dev = torch.device("cuda", 0)
    per = shard(T, 0, ranks)[2]
    hdr_all = torch.zeros(2 * ranks, dtype=torch.int64, device=dev)
    snaps_all = torch.full((ranks * per, stride), float("nan"), dtype=torch.float64, device=dev)
    plans = []
    try:
        for r in range(ranks):
            lo, hi, _ = shard(T, r, ranks)
            if hi <= lo:
                continue
            p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"],
                               z["densities"], z["combos"], z["weights"], z["copula_params"],
                               vol_states=z.get("unique_vol_states"), strategy=strategy)
            p.set_stream(torch.cuda.current_stream().cuda_stream)
            if str(z["model"]) == "msm":
                p.set_dates((z["forecasts_by_states"][lo:hi], z["forecasts"][lo:hi]))
            else:
                p.set_dates([z["sigma_forecasts"][lo:hi]])
            plans.append(p)
            p.solve_local(args, hdr_all[2 * r: 2 * r + 2].data_ptr(), snaps_all[r * per: r * per + hi - lo].data_ptr())
        var = torch.empty(T, dtype=torch.float64, device=dev)
        plans[-1].solve_finalize(args, hdr_all.data_ptr(), ranks, snaps_all.data_ptr(), per, T, var.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(var.cpu().numpy(), z["var"])
    finally:
        for p in plans:
            p.close()


@pytest.mark.parametrize("kw", [dict(), dict(first_guess=-2.5, second_guess=(-4.0, -1.5)),
                                dict(first_guess=-1.0, second_guess=(-2.0, -0.5), min_var=-5.0),
                                dict(first_guess=-3.0, second_guess=(-2.0, -3.5)),      # unordered: SORTED path
                                dict(obj_var=0.01), dict(obj_var=0.2)])
@pytest.mark.parametrize("cfg", [2, 5])
def test_sweep_matches_sorted_solve_arguments(cfg, kw):
    """SWEEP against SORTED for non-default calc_var arguments (other brackets, other
    objectives; unordered guesses fall back to the per-level loop): bit-identical."""
    c, ipt, uvs, ggp, ptf = _workload(cfg, 300, n=96)
    out = {}
    for strategy in ("sorted", "sweep"):
        p = _plan(c, ipt, uvs, ggp, strategy)
        try:
            out[strategy] = p.calc_var(ptf, **kw)
        finally:
            p.close()
    assert out["sorted"][1] == out["sweep"][1]
    np.testing.assert_array_equal(out["sorted"][0], out["sweep"][0])


def test_sorted_rejects_levels_above_v_cap():
    z = load_golden("cfg2_n64")
    from copula_var.engine import QuadraturePlan
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), 2, z["x_values"], z["step"], z["densities"], z["combos"],
                       z["weights"], z["copula_params"], vol_states=z["unique_vol_states"], strategy="sorted")
    try:
        p.set_dates((z["forecasts_by_states"], z["forecasts"]))
        with pytest.raises(ValueError):                     # CVQ_ERR_RANGE
            p.compute_integral(np.tile([-1.0, 0.5], (z["var"].size, 1)))
    finally:
        p.close()


@pytest.mark.parametrize("copula", ["student", "gaussian"])
def test_3d_general_layout_n_above_128(copula):
    """3-D with n in (128, 255] takes the general node-word layout (kLay3G); GARCH
    margins (Q = 1) keep the oracle cheap at n = 136."""
    from copula_var import synthetic, tables
    from oracle.quadrature import calc_var
    R3 = np.array([[1.0, 0.5, 0.4], [0.5, 1.0, 0.3], [0.4, 0.3, 1.0]])
    c = synthetic.Config("g3_136", "garch", copula, 3, 136, 3, garch_params=[{"omega": 0.05, "alpha": 0.08,
                                                                             "beta": 0.90}] * 3,
                         nu=6.0, corr=R3, innov_copula="gaussian", innov_corr=R3)
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    P = _problem(c, ipt, uvs, ggp)
    ref, ref_it, _ = calc_var(P.compute_integral, P.T, ptf)
    p = _plan(c, ipt, uvs, ggp, "sorted")
    try:
        var, it = p.calc_var(ptf)
        b = np.tile([-3.0, -2.0], (P.T, 1))
        np.testing.assert_allclose(p.compute_integral(b), P.compute_integral(b), rtol=SLAB_RTOL, atol=SLAB_ATOL)
    finally:
        p.close()
    assert it == ref_it
    assert np.array_equal(var, ref)


def _perturbed_pi(z, every):
    pi = z["forecasts"].copy()
    rng = np.random.default_rng(11)
    pi[::every] *= rng.uniform(0.9, 1.1, size=pi[::every].shape)
    return pi


def test_compact_deferral_reuse():
    """COMPACT's fast kernel defers the dates that need the generic node path (pi not
    rank 1) to a second kernel, which also finalizes.  One plan solves a mixed batch,
    an all-fast batch and an all-generic batch in turn: every VaR follows the oracle,
    so the deferral count and the tickets are reset between solves."""
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("cfg2_n64")
    fbs = z["forecasts_by_states"]
    args = (str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
            z["combos"], z["weights"], z["copula_params"])
    p = QuadraturePlan(*args, vol_states=z["unique_vol_states"], strategy="compact")
    try:
        for pi in (_perturbed_pi(z, 3), z["forecasts"], _perturbed_pi(z, 1), z["forecasts"]):
            P = Problem(*args, (fbs, pi), z["unique_vol_states"])
            ref, ref_it, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
            p.set_dates((fbs, pi))
            var, it = p.calc_var(float(z["ptf_mean"]))
            assert it == ref_it
            assert np.array_equal(var, ref)
    finally:
        p.close()


def test_compact_deferral_sharded():
    """The deferral in the sharded (unfused) solve: per-rank cvq_solve_local with some
    generic dates in each block, then every rank finalizes the whole vector."""
    import torch
    from copula_var import engine
    from copula_var.distributed import shard
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("cfg2_n64")
    fbs, pi = z["forecasts_by_states"], _perturbed_pi(z, 4)
    cargs = (str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
             z["combos"], z["weights"], z["copula_params"])
    P = Problem(*cargs, (fbs, pi), z["unique_vol_states"])
    ref, _, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
    T, ranks = P.T, 3
    args = engine.solve_args(float(z["ptf_mean"]))
    stride = engine.QuadraturePlan.snap_stride(args)
    dev = torch.device("cuda", 0)
    per = shard(T, 0, ranks)[2]
    hdr_all = torch.zeros(2 * ranks, dtype=torch.int64, device=dev)
    snaps_all = torch.full((ranks * per, stride), float("nan"), dtype=torch.float64, device=dev)
    plans = []
    try:
        for r in range(ranks):
            lo, hi, _ = shard(T, r, ranks)
            p = QuadraturePlan(*cargs, vol_states=z["unique_vol_states"], strategy="compact")
            plans.append(p)
            p.set_stream(torch.cuda.current_stream().cuda_stream)
            p.set_dates((fbs[lo:hi], pi[lo:hi]))
            p.solve_local(args, hdr_all[2 * r: 2 * r + 2].data_ptr(), snaps_all[r * per: r * per + (hi - lo)].data_ptr())
        var = torch.empty(T, dtype=torch.float64, device=dev)
        plans[0].solve_finalize(args, hdr_all.data_ptr(), ranks, snaps_all.data_ptr(), per, T, var.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(var.cpu().numpy(), ref)
    finally:
        for p in plans:
            p.close()


def test_compact_fast_hint_violation_fails_loudly():
    """set_dates_device(fast=True) skips the deferred-date kernel; a date whose pi is not
    rank 1 then fails the solve (CVQ_ERR_NUMERIC) instead of returning a VaR.  The same
    inputs without the hint solve to the oracle's VaR."""
    import torch
    from copula_var import engine
    from copula_var.engine import QuadraturePlan
    from oracle.quadrature import Problem, calc_var
    z = load_golden("cfg2_n64")
    fbs, pi = z["forecasts_by_states"], _perturbed_pi(z, 5)
    cargs = (str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
             z["combos"], z["weights"], z["copula_params"])
    P = Problem(*cargs, (fbs, pi), z["unique_vol_states"])
    ref, _, _ = calc_var(P.compute_integral, P.T, float(z["ptf_mean"]))
    dev = torch.device("cuda", 0)
    d_a = torch.tensor(np.ascontiguousarray(fbs), dtype=torch.float64, device=dev)
    d_b = torch.tensor(np.ascontiguousarray(pi), dtype=torch.float64, device=dev)
    args = engine.solve_args(float(z["ptf_mean"]))
    p = QuadraturePlan(*cargs, vol_states=z["unique_vol_states"], strategy="compact")
    try:
        p.set_stream(torch.cuda.current_stream().cuda_stream)
        var = torch.empty(P.T, dtype=torch.float64, device=dev)
        p.set_dates_device(P.T, d_a.data_ptr(), d_b.data_ptr(), fast=True)
        p.solve_device(args, var.data_ptr())
        with pytest.raises(RuntimeError, match="generic node path"):
            p.solve_status()
        p.set_dates_device(P.T, d_a.data_ptr(), d_b.data_ptr())
        p.solve_device(args, var.data_ptr())
        p.solve_status()
        assert np.array_equal(var.cpu().numpy(), ref)
    finally:
        p.close()
