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
