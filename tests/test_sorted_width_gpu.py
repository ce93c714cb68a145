"""SORTED at 256, 384, 512 and 1024 threads per date (cvq_sorted.hip sorted_threads).

A strong-scaling block of a few hundred dates per GPU takes the wider workgroups (the
launch is latency bound there); a full batch takes 256.  The width changes only how a
date's range sums are strided over its lanes (summation order), never which nodes a slab
holds or the control flow (calc_var_class.py:95-177, 250-309), so the VaR must be the
same bit for bit at every width -- against the reference goldens, and at full BASELINE
geometry between the widths (cfg 3 / cfg 5: 625 dates = 5000 over 8 GPUs; cfg 4: 250 =
2000 over 8).  Slabs within 1e-10 relative (summation order)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

WIDTHS = ["256", "384", "512", "1024"]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu(gpu_available):
    if not gpu_available:
        pytest.fail("GPU tests were selected but no HIP device / libcvq.so is available")


@pytest.mark.parametrize("width", WIDTHS)
@pytest.mark.parametrize("case", ["cfg1", "cfg3_n128", "cfg5_n64", "cfg2_n64", "cfg4_k4_n16", "cfg4_k6_n16",
                                  "garch_student_n64", "ukf_plackett_n64", "garch3d_student_n16", "q1_lowvol"])
def test_width_matches_golden(case, width, monkeypatch):
    from copula_var.engine import QuadraturePlan
    monkeypatch.setenv("CVQ_SORT_NT", width)
    z = load_golden(case)
    msm = str(z["model"]) == "msm"
    vs = z.get("unique_vol_states")
    per = (z["forecasts_by_states"], z["forecasts"]) if msm else [z["sigma_forecasts"]]
    p = QuadraturePlan(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                       z["combos"], z["weights"], z["copula_params"], vol_states=vs, strategy="sorted")
    try:
        p.set_dates(per)
        var, _ = p.calc_var(float(z["ptf_mean"]))
        b, ref = z["call00_bounds"], z["call00_result"]
        slab = p.compute_integral(b)
    finally:
        p.close()
    assert np.array_equal(var, z["var"]), (case, width)
    np.testing.assert_allclose(slab, ref, rtol=1e-10, atol=1e-15)


def _workload(cfg_no, T):
    from copula_var import synthetic, tables
    c = synthetic.baseline_configs()[cfg_no].with_(T=T)
    rets = synthetic.simulate_returns(c)
    _, ptf, centred, _ = tables.insample_split(rets, c.n_in, c.weights)
    if c.model == "msm":
        ipt, uvs, ggp = tables.msm_integration_params(centred, c.n_in, c.msm_params, c.k, c.num_points)
    else:
        ipt, uvs, ggp = tables.sigma_integration_params(centred, c.n_in, c.model, c.model_params(), c.num_points)
    return c, ipt, uvs, ggp, ptf


@pytest.mark.parametrize("cfg,T", [(3, 625), (5, 625), (4, 250)])
def test_width_full_geometry_identical(cfg, T, monkeypatch):
    from copula_var.engine import QuadraturePlan
    c, ipt, uvs, ggp, ptf = _workload(cfg, T)
    dens, x, step, combos = ggp
    p = QuadraturePlan(c.model, c.copula, c.dim, x, step, dens, combos, c.weights, c.copula_params(),
                       vol_states=uvs, strategy="sorted")
    out = {}
    try:
        p.set_dates(ipt)
        for w in WIDTHS:
            monkeypatch.setenv("CVQ_SORT_NT", w)
            out[w] = p.calc_var(ptf)
        monkeypatch.delenv("CVQ_SORT_NT")
        out["auto"] = p.calc_var(ptf)
    finally:
        p.close()
    v0, it0 = out["256"]
    assert not np.isnan(v0).any()
    for w, (v, it) in out.items():
        assert it == it0, (w, it, it0)
        assert np.array_equal(v, v0), (cfg, w, float(np.max(np.abs(v - v0))))

