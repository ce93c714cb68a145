"""Device UKF forecasts in the update's cancelling regime (estimate.py:214-229,
custom_cholesky :54-78).

tests/ukf_spike_case.py builds windows whose update puts nearly all the weight on one sigma
point, where a variance formed as Syy / Z - mu^2 can round below 0 and take the var <= 0
branch the reference never takes (tests/test_ukf_variance_cpu.py shows the regime on the
CPU).  Both device forecast kernels that run ukf_forecast_pass -- cvq_ukf_forecast
(k_ukf_forecast) and the end-to-end stage cvq_sigma_tables (k_ukf_sigma) -- must match the
reference's filter (oracle.forecast.ukf_run, pinned to reference-run goldens) within 1e-12
relative on every window, as the step-by-step pass (cvq_ukf_filter) does."""
import numpy as np
import pytest
import torch

import ukf_spike_case as U
from oracle.forecast import ukf_run

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


@pytest.fixture(scope="module")
def cases():
    W = U.windows()
    ref, _, _, failed = ukf_run(W, *U.PARAMS)
    assert not failed.any()
    return W, ref


def test_ukf_forecast_kernel(cases):
    from copula_var import engine
    W, ref = cases
    a, l, q = U.PARAMS
    got = np.array([engine.ukf_forecast(w, U.N_IN, a, l, q)[0] for w in W])
    rel = np.abs(got - ref) / ref
    assert float(rel.max()) < 1e-12, (float(rel.max()), int(np.argmax(rel)))


def test_sigma_tables_kernel(cases):
    """cvq_sigma_tables (the e2e stage): two assets per launch, each window its own launch of T = 1."""
    from copula_var import engine
    W, ref = cases
    a, l, q = U.PARAMS
    prm = [{"a": a, "l": l, "q": q}] * 2
    st = engine.SigmaTables("mean_reverting", prm, U.N_IN, 1, 0)
    m = W.shape[0] - W.shape[0] % 2
    got = np.empty(m)
    s = torch.cuda.current_stream().cuda_stream
    for k in range(0, m, 2):                      # asset 0: window k, asset 1: window k + 1
        r = torch.tensor(np.stack([W[k], W[k + 1]]), dtype=torch.float64, device="cuda")
        st.run(r, s)
        st.status(s)
        got[k: k + 2] = st.sig.cpu().numpy()[0]
    rel = np.abs(got - ref[:m]) / ref[:m]
    assert float(rel.max()) < 1e-12, (float(rel.max()), int(np.argmax(rel)))


def test_step_by_step_filter(cases):
    """cvq_ukf_filter (the EM E-step's pass, sigma-point arithmetic as the reference) agrees too."""
    from copula_var import engine
    W, ref = cases
    a, l, q = U.PARAMS
    ll, _ = engine.ukf_filter(W, np.tile([a, l, q], (W.shape[0], 1)))
    _, ll_ref, _, _ = ukf_run(W, a, l, q)
    np.testing.assert_allclose(ll, ll_ref, rtol=1e-11, atol=1e-11)
