"""The end-to-end device path at full BASELINE batch size against the pinned oracle
(VERDICT r05 #1).

bench.py's e2e leg runs: centred returns resident in HBM -> the device forecast stage
(cvq_msm_tables: every asset's rolling-window Hamilton filters as transfer-matrix scans, the
state collapse (Q14) and the forecast combinations (Q7); cvq_sigma_tables: GARCH(1, 1)
recursions or the closed-form UKF pass) -> the solve reading those tables in place.  Its own
check compares device with device.  Here the same stage runs on each fixture's returns
(tests/golden/fullbatch_cfg{2,5,3,4}.npz: the synthetic returns and the pinned oracle's host
forecast stage + calc_var over the whole batch; cfg 4: its first 250 of 2000 dates) and

* the device tables must equal the oracle's within 1e-12 relative (forecasts_by_states and
  forecasts for MSM; sigma for GARCH / UKF -- msm_estimation.py:123-418,
  garch/forecast.py:5-19, kalman_mean_reverting/estimate.py:230-281, forecast.py:12);
* the VaR solved from the device tables must equal the oracle's VaR bit for bit, with the same
  global iteration count (Q2, calc_var_class.py:278) -- the tables' last-ulp differences never
  flip a bisection decision."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

TABLE_RTOL = 1e-12


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


def _run_stage(cfg_no, z):
    """The device forecast stage on the fixture's returns: (per-date device tensors, fast hint)."""
    from copula_var import engine, synthetic, tables
    c = synthetic.baseline_configs()[cfg_no].with_(T=int(z["T"]))
    n_in = int(z["n_in"])
    _, ptf_mean, centred, T = tables.insample_split(z["returns"], n_in, c.weights)
    assert T == int(z["T"]) and ptf_mean == float(z["ptf_mean"])
    r_dev = torch.tensor(np.ascontiguousarray(centred[:-1].T), dtype=torch.float64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    if c.model == "msm":
        vsa = np.array([tables.msm_vol_states(c.k, p["m_0"], p["sig"]) for p in c.msm_params])
        smap, uvs = tables.unique_vol_map(vsa)
        np.testing.assert_array_equal(uvs, z["unique_vol_states"])
        mt = engine.MsmTables([[p["m_0"], p["sig"], p["b"], p["gamma"]] for p in c.msm_params], c.k, smap,
                              uvs.shape[1], n_in, T, 0)
        mt.run(r_dev, s)
        mt.status(s)
        return mt, (mt.fbs, mt.pi), True
    st = engine.SigmaTables(c.model, c.model_params(), n_in, T, 0)
    st.run(r_dev, s)
    st.status(s)
    return st, (st.sig, None), c.copula == "student" and c.dim == 2


@pytest.mark.parametrize("cfg_no", [2, 5, 3, 4])
def test_device_forecast_stage_then_solve_matches_oracle(cfg_no):
    from copula_var.engine import QuadraturePlan, solve_args
    path = os.path.join(GOLDEN, f"fullbatch_cfg{cfg_no}.npz")
    z = dict(np.load(path, allow_pickle=False))
    T = int(z["T"])
    holder, (ta, tb), fast = _run_stage(cfg_no, z)
    if str(z["model"]) == "msm":
        np.testing.assert_allclose(ta.cpu().numpy(), z["forecasts_by_states"], rtol=TABLE_RTOL, atol=1e-300)
        np.testing.assert_allclose(tb.cpu().numpy(), z["forecasts"], rtol=TABLE_RTOL, atol=1e-300)
    else:
        np.testing.assert_allclose(ta.cpu().numpy(), z["sigma_forecasts"], rtol=TABLE_RTOL, atol=0)
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=z.get("unique_vol_states"))
    try:
        p.set_stream(torch.cuda.current_stream().cuda_stream)
        p.set_dates_device(T, ta.data_ptr(), tb.data_ptr() if tb is not None else None, fast=fast)
        var = torch.empty(T, dtype=torch.float64, device="cuda")
        it = p.solve_device(solve_args(float(z["ptf_mean"])), var.data_ptr(), check=True)
    finally:
        p.close()
    got = var.cpu().numpy()
    assert it == int(z["iterations"]), (it, int(z["iterations"]))
    assert np.array_equal(got, z["var"]), (cfg_no, int((got != z["var"]).sum()))
