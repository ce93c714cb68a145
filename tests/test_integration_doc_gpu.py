"""INTEGRATION.md's ctypes binding (the stub a maintainer would add to the
reference) is executable documentation: run it against the golden cases."""
import os
import re
import types

import numpy as np
import pytest

from conftest import REPO, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def binding(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")
    from copula_var import _native
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, flags=re.S)
    src = next(b for b in blocks if "class CvqPlan" in b)
    src = src.replace("/path/to/copula_var/libcvq.so", _native.LIB_PATH)
    mod = types.ModuleType("cvq_binding")
    exec(compile(src, "INTEGRATION.md", "exec"), mod.__dict__)
    return mod


@pytest.mark.parametrize("case", ["cfg1", "cfg2_n64", "cfg3_n128", "cfg5_n64", "cfg4_k4_n16"])
def test_integration_stub_reproduces_reference(binding, case):
    z = load_golden(case)
    model = str(z["model"])
    ipt = (z["forecasts_by_states"], z["forecasts"]) if model == "msm" else [z["sigma_forecasts"]]
    ggp = (z["densities"], z["x_values"], z["step"], z["combos"])
    plan = binding.CvqPlan(model, str(z["copula"]), int(z["dim"]), ggp, z.get("unique_vol_states"), ipt,
                           z["copula_params"], z["weights"])
    var = plan.calc_var(float(z["ptf_mean"]))
    assert np.array_equal(var, z["var"])
    b, ref = z["call00_bounds"], z["call00_result"]
    np.testing.assert_allclose(plan.compute_integral(b), ref, rtol=1e-10, atol=1e-15)


@pytest.mark.parametrize("cfg,T", [(4, 3), (5, 4), (3, 3), (2, 4)])
def test_integration_stub_full_baseline_geometry(binding, cfg, T):
    """The stub at each BASELINE config's full grid (cfg 4: 128^3, k = 6, Q = 343; cfg 5:
    UKF 256^2; cfg 3: Plackett 512^2; cfg 2: MSM 256^2) on a few dates against the oracle
    -- VaR bit-identical -- plus a compute_integral bound above 0 (the stub's SORTED plan
    holds the whole grid)."""
    from copula_var import synthetic, tables
    from oracle.quadrature import Problem, calc_var
    c = synthetic.baseline_configs()[cfg].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
        per = ipt
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
        per = ipt[0]
    dens, x, step, combos = ggp
    P = Problem(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(), per, uvs)
    ref, _, _ = calc_var(P.compute_integral, P.T, ptf)
    plan = binding.CvqPlan(c.model, c.copula, c.dim, ggp, uvs, ipt, c.copula_params(), c.weights)
    var = plan.calc_var(ptf)
    assert np.array_equal(var, ref), (var, ref)
    for b in ([-100.0, -3.0], [-1.0, 0.5]):
        bounds = np.tile(b, (T, 1))
        np.testing.assert_allclose(plan.compute_integral(bounds), P.compute_integral(bounds), rtol=1e-10,
                                   atol=1e-15)
