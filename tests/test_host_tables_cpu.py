"""Host-side table assembly (copula_var/tables.py) vs the reference goldens, CPU only.

These are the small, non-iterative pieces of integration_params_retrieval
(msm_estimation.py:123-418, garch_estimation.py:133-188) that stay on the host;
the filters that feed them run on the GPU and are covered by test_gpu_parity.py.
"""
import numpy as np
import pytest

from conftest import GOLDEN_CASES, load_golden

MSM_CASES = [c for c in GOLDEN_CASES if str(load_golden(c)["model"]) == "msm"]


@pytest.mark.parametrize("case", GOLDEN_CASES)
def test_insample_split_and_grid(case):
    from copula_var import tables
    z = load_golden(case)
    mean, ptf, centred, T = tables.insample_split(z["returns"], int(z["n_in"]), z["weights"])
    assert ptf == float(z["ptf_mean"])                         # load_data.py:113, bit-exact
    assert T == z["var"].size
    x, step = tables.x_grid(int(z["num_points"]), str(z["model"]))
    assert np.array_equal(x, z["x_values"]) and np.array_equal(step, z["step"])


@pytest.mark.parametrize("case", MSM_CASES)
def test_msm_host_tables(case):
    from copula_var import tables
    z = load_golden(case)
    k = int(z["k"])
    names = list(z["model_param_names"])
    mp = [dict(zip(names, row)) for row in z["model_params"]]
    vsa = np.array([tables.msm_vol_states(k, p["m_0"], p["sig"]) for p in mp])
    np.testing.assert_allclose(vsa, z["vol_states_array"], rtol=1e-15)
    fbs, uvs = tables.sum_forecast_by_state(z["vol_states_array"], z["filtered_probs"])
    np.testing.assert_allclose(fbs, z["forecasts_by_states"], rtol=1e-13, atol=1e-300)
    assert np.array_equal(uvs, z["unique_vol_states"])
    pi = tables.forecast_combinations(z["forecasts_by_states"])
    np.testing.assert_allclose(pi, z["forecasts"], rtol=1e-15, atol=1e-300)
    combos = tables.vol_combinations(int(z["dim"]), uvs.shape[1])
    assert np.array_equal(combos, z["combos"])
    dens = tables.msm_densities(z["unique_vol_states"], z["x_values"])
    np.testing.assert_allclose(dens, z["densities"], rtol=1e-15)


def test_3d_forecast_combination_permutation_q7():
    """In 3-D the reference's xy-meshgrid product permutes the combos (Q7,
    msm_estimation.py:413 vs :384): combo (ia, ib, ic) gets f0[ib] f1[ic] f2[ia]."""
    from copula_var import tables
    rng = np.random.default_rng(1)
    fbs = rng.random((2, 3, 4))
    pi = tables.forecast_combinations(fbs)
    combos = tables.vol_combinations(3, 4)
    for t in range(2):
        for l, (ia, ib, ic) in enumerate(combos):
            assert pi[t, l] == pytest.approx(fbs[t, 0, ib] * fbs[t, 1, ic] * fbs[t, 2, ia], rel=1e-15)


def test_insample_split_rejects_short_series():
    from copula_var import tables
    with pytest.raises(ValueError, match="Not enough returns"):
        tables.insample_split(np.zeros((10, 2)), 10, np.array([0.5, 0.5]))
