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
