"""Device-resident MSM forecast stage (cvq_msm_tables): filters of every asset in one
launch, states collapsed onto unique vols and the forecast combinations formed on the
device, read in place by the solve.  Checked against the reference's own tables
(golden cases: forecasts_by_states / forecasts computed by msm_estimation.py) and
against the host assembly (copula_var/tables.py), with the VaR bit-identical."""
import numpy as np
import pytest
import torch

from conftest import golden_kwargs, load_golden

pytestmark = pytest.mark.gpu

TABLE_RTOL = 1e-10          # the filter sums in another order than calc_prob.py (butterflies)


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _device_tables(rc, n_in, k, params, dev=0):
    """rc: centred returns (n_in + T - 1, dim) on the host -> MsmTables after one run."""
    from copula_var import engine, tables
    dim = rc.shape[1]
    vsa = np.array([tables.msm_vol_states(k, p["m_0"], p["sig"]) for p in params])
    state_map, uvs = tables.unique_vol_map(vsa)
    T = rc.shape[0] - n_in + 1
    mt = engine.MsmTables([[p["m_0"], p["sig"], p["b"], p["gamma"]] for p in params], k, state_map, uvs.shape[1],
                          n_in, T, dev)
    r_dev = torch.tensor(np.ascontiguousarray(rc.T), dtype=torch.float64, device=f"cuda:{dev}")
    mt.run(r_dev)
    mt.status()
    return mt, uvs, r_dev


@pytest.mark.parametrize("case", ["cfg2_n64", "cfg2_n256", "cfg4_k4_n16", "cfg4_k6_n16", "msm_gauss_n64"])
def test_device_tables_match_reference(case):
    from copula_var.engine import QuadraturePlan, solve_args
    from oracle import forecast as F
    z = load_golden(case)
    n_in, k = int(z["n_in"]), int(z["k"])
    names = list(z["model_param_names"])
    params = [dict(zip(names, row)) for row in z["model_params"]]
    mean, _, _ = F.insample_split(z["returns"], n_in, z["weights"])
    rc = (z["returns"] - mean)[:-1]
    mt, uvs, _ = _device_tables(rc, n_in, k, params)
    np.testing.assert_allclose(uvs, z["unique_vol_states"], rtol=0, atol=0)
    np.testing.assert_allclose(mt.fbs.cpu().numpy(), z["forecasts_by_states"], rtol=TABLE_RTOL, atol=1e-300)
    np.testing.assert_allclose(mt.pi.cpu().numpy(), z["forecasts"], rtol=TABLE_RTOL, atol=1e-300)
    # the solve reads the device tables in place
    p = QuadraturePlan("msm", str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z["unique_vol_states"])
    try:
        p.set_stream(torch.cuda.current_stream().cuda_stream)
        p.set_dates_device(mt.T, mt.fbs.data_ptr(), mt.pi.data_ptr())
        var = torch.empty(mt.T, dtype=torch.float64, device="cuda")
        it = p.solve_device(solve_args(float(z["ptf_mean"]), **golden_kwargs(z)), var.data_ptr(), check=True)
    finally:
        p.close()
    assert it == int(z["n_calls"]) - 2
    assert np.array_equal(var.cpu().numpy(), z["var"])


@pytest.mark.parametrize("cfg_no,T", [(2, 300), (4, 40)])
def test_device_tables_match_host_assembly(cfg_no, T):
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[cfg_no].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, _, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    (fbs, pi), uvs, _ = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    mt, uvs_d, _ = _device_tables(centred[:-1], c.n_in, c.k, c.msm_params)
    np.testing.assert_array_equal(uvs_d, uvs)
    np.testing.assert_allclose(mt.fbs.cpu().numpy(), fbs, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(mt.pi.cpu().numpy(), pi, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("cfg_no,T", [(1, 50), (3, 400), (5, 300)])
def test_device_sigma_tables_match_host_path(cfg_no, T):
    """cvq_sigma_tables (all assets, stream-ordered, [T][dim] in place) equals the per-asset
    forecast kernels behind tables.sigma_integration_params bit for bit, and the solve
    reading it in place returns the same VaR."""
    from copula_var import engine, synthetic, tables
    from copula_var.engine import QuadraturePlan, solve_args
    c = synthetic.baseline_configs()[cfg_no].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf_mean, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    ipt, uvs, (dens, x, step, combos) = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(),
                                                                        c.num_points)
    st = engine.SigmaTables(c.model, c.model_params(), c.n_in, T)
    r_dev = torch.tensor(np.ascontiguousarray(centred[:-1].T), dtype=torch.float64, device="cuda:0")
    st.run(r_dev)
    st.status()
    np.testing.assert_array_equal(st.sig.cpu().numpy(), ipt[0])
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params())
    try:
        p.set_stream(torch.cuda.current_stream().cuda_stream)
        var_h = torch.empty(T, dtype=torch.float64, device="cuda")
        p.set_dates(ipt)
        p.solve_device(solve_args(ptf_mean), var_h.data_ptr(), check=True)
        var_d = torch.empty(T, dtype=torch.float64, device="cuda")
        p.set_dates_device(T, st.sig.data_ptr())
        p.solve_device(solve_args(ptf_mean), var_d.data_ptr(), check=True)
    finally:
        p.close()
    assert np.array_equal(var_d.cpu().numpy(), var_h.cpu().numpy())


def test_device_sigma_tables_garch_pq_per_asset():
    """Per-asset GARCH orders in one call (GarchOptimizer picks (p, q) per ticker): each
    column equals cvq_garch_forecast_pq of that asset."""
    from copula_var import engine
    rng = np.random.default_rng(7)
    n_in, T = 300, 64
    rc = rng.standard_normal((n_in + T - 1, 3)) * 1.3
    params = [{"pq": (2, 1), "params": (0.05, 0.05, 0.03, 0.88)},
              {"omega": 0.04, "alpha": 0.07, "beta": 0.91},
              {"pq": (1, 3), "params": (0.06, 0.08, 0.3, 0.3, 0.3)}]
    st = engine.SigmaTables("garch", params, n_in, T)
    st.run(torch.tensor(np.ascontiguousarray(rc.T), dtype=torch.float64, device="cuda:0"))
    st.status()
    sig = st.sig.cpu().numpy()
    np.testing.assert_array_equal(sig[:, 0], engine.garch_forecast_pq(rc[:, 0], n_in, 2, 1, params[0]["params"]))
    np.testing.assert_array_equal(sig[:, 1], engine.garch_forecast(rc[:, 1], n_in, 0.04, 0.07, 0.91))
    np.testing.assert_array_equal(sig[:, 2], engine.garch_forecast_pq(rc[:, 2], n_in, 1, 3, params[2]["params"]))


def test_device_sigma_tables_ukf_failure_is_reported():
    """An extreme return makes the UKF normaliser underflow (estimate.py:219-220): the
    stage flags it and status() raises, as the host forecast does."""
    from copula_var import _native as N, engine
    n_in, T = 200, 16
    rc = np.random.default_rng(3).standard_normal((n_in + T - 1, 2)) * 0.8
    rc[150, 1] = 1e6
    st = engine.SigmaTables("mean_reverting", [{"a": 0.97, "l": 0.05, "q": 0.15}] * 2, n_in, T)
    st.run(torch.tensor(np.ascontiguousarray(rc.T), dtype=torch.float64, device="cuda:0"))
    with pytest.raises(N.NativeError):
        st.status()


def test_device_tables_zero_normaliser_is_reported():
    """A return so extreme that every state's density underflows to 0 makes the reference's
    Bayes normaliser 0 (calc_prob.py:64-65): the device stage flags it (blocked filter:
    in the block products and the window steps) and status() raises."""
    from copula_var import _native as N
    c_params = [{"m_0": 0.45, "sig": 1.2, "b": 3.0, "gamma": 0.3}, {"m_0": 0.5, "sig": 1.2, "b": 3.0, "gamma": 0.3}]
    n_in, T = 300, 40
    rc = np.random.default_rng(5).standard_normal((n_in + T - 1, 2))
    rc[170, 0] = 1e4
    with pytest.raises(N.NativeError):
        _device_tables(rc, n_in, 4, c_params)


@pytest.mark.parametrize("n_in,T", [(33, 7), (64, 100), (1135, 1000), (3000, 50)])
def test_blocked_filter_matches_stepwise(n_in, T):
    """The blocked filter (block products + partial-block steps) against the step-by-step
    device filter on every window, across block-length regimes (n_in just above one
    block, several, the cfg-2 geometry, and long windows that double the block)."""
    from copula_var import engine
    p = {"m_0": 0.45, "sig": 1.2, "b": 3.0, "gamma": 0.3}
    rc = np.random.default_rng(11).standard_normal((n_in + T - 1, 2)) * 1.1
    mt, _, _ = _device_tables(rc, n_in, 4, [p, p])
    fbs = mt.fbs.cpu().numpy()
    for d in range(2):
        seq = engine.msm_filter(rc[:, d], n_in, 4, p["m_0"], p["sig"], p["b"], p["gamma"])
        from copula_var import tables
        vs = tables.msm_vol_states(4, p["m_0"], p["sig"])
        smap, _ = tables.unique_vol_map(vs[None, :])
        ref = np.stack([seq[:, smap[0] == u].sum(axis=1) for u in range(fbs.shape[2])], axis=1)
        np.testing.assert_allclose(fbs[:, d, :], ref, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("n_in,T", [(65, 1), (70, 50), (100, 17), (600, 300), (1135, 1000), (1135, 7)])
def test_scan_filter_window_shapes(n_in, T):
    """cvq_msm_tables' transfer-matrix scan (block prefixes / suffixes, superblock scans, <= 5
    mat-vecs per window) against the step-by-step filter behind the host assembly, over window
    lengths that hit every middle-block case (none, a superblock prefix or suffix alone, loose
    blocks inside one superblock, several superblocks) and T from 1 to 1000."""
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[2].with_(T=T, n_in=n_in)
    rets = synthetic.simulate_returns(c)
    _, _, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    (fbs, pi), uvs, _ = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    mt, uvs_d, _ = _device_tables(centred[:-1], c.n_in, c.k, c.msm_params)
    np.testing.assert_array_equal(uvs_d, uvs)
    np.testing.assert_allclose(mt.fbs.cpu().numpy(), fbs, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(mt.pi.cpu().numpy(), pi, rtol=1e-12, atol=1e-300)


@pytest.mark.parametrize("cfg_no,k,n_in,T", [(4, 6, 1135, 200), (4, 6, 70, 50), (4, 6, 600, 300), (4, 6, 1135, 1),
                                             (2, 5, 1135, 300), (2, 5, 100, 17), (2, 6, 300, 64)])
def test_wide_scan_filter_k5_k6(cfg_no, k, n_in, T):
    """k = 5, 6 (BASELINE config 4's 64 states): the wide transfer-matrix scan (block products,
    superblock scans over 64 x 64 matrices, the window's last partial block as filter steps)
    against the step-by-step filter behind the host assembly, 2 and 3 assets, window lengths
    hitting each middle-block case."""
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[cfg_no].with_(T=T, n_in=n_in, k=k)
    rets = synthetic.simulate_returns(c)
    _, _, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    (fbs, pi), uvs, _ = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    mt, uvs_d, _ = _device_tables(centred[:-1], c.n_in, c.k, c.msm_params)
    np.testing.assert_array_equal(uvs_d, uvs)
    np.testing.assert_allclose(mt.fbs.cpu().numpy(), fbs, rtol=1e-12, atol=1e-300)
    np.testing.assert_allclose(mt.pi.cpu().numpy(), pi, rtol=1e-12, atol=1e-300)
