"""engine.auto_strategy: the measured-fastest strategy among those that run a workload
(no GPU needed)."""
import pytest


def test_auto_strategy_rules():
    from copula_var.engine import auto_strategy
    assert auto_strategy("msm", 2, 256) == "compact"
    assert auto_strategy("msm", 2, 512) == "compact"
    for m in ("garch", "mean_reverting"):
        assert auto_strategy(m, 2, 64) == "sorted"
        assert auto_strategy(m, 2, 512) == "sorted"
        assert auto_strategy(m, 2, 513) == "sorted"         # 512 < n <= 1024: SORTED's 1024-thread dates
        assert auto_strategy(m, 2, 1024) == "sorted"
        with pytest.raises(ValueError, match="1024"):
            auto_strategy(m, 2, 1025)                       # no plan takes n > 1024: fail at the rule
    assert auto_strategy("msm", 2, 1000, "student", [6.0, 0.5]) == "sorted"
    assert auto_strategy("msm", 3, 128) == "sorted"
    assert auto_strategy("garch", 3, 255) == "sorted"
    assert auto_strategy("msm", 2) == "compact"            # n unknown: the 2-D rule
    # a fitted Student nu (general node power): SORTED for MSM too; nu = 6 or any integer: COMPACT
    assert auto_strategy("msm", 2, 256, "student", [5.364, 0.5]) == "sorted"
    assert auto_strategy("msm", 2, 256, "student", [6.0, 0.5]) == "compact"
    assert auto_strategy("msm", 2, 256, "student", [5.0, 0.5]) == "compact"   # nu + 2 integer: no log / exp
    assert auto_strategy("msm", 2, 256, "student", [4.5, 0.5]) == "sorted"
    assert auto_strategy("msm", 2, 256, "gaussian", [0.5]) == "compact"
    # GARCH / UKF: COMPACT for an integer-power Student copula (cfg 5), SORTED otherwise
    assert auto_strategy("mean_reverting", 2, 256, "student", [6.0, 0.5]) == "compact"
    assert auto_strategy("garch", 2, 256, "student", [5.364, 0.5]) == "sorted"
    assert auto_strategy("garch", 2, 512, "plackett", [3.0]) == "sorted"
    assert auto_strategy("garch", 2, 64, "gaussian", [0.6]) == "sorted"
    with pytest.raises(ValueError):
        auto_strategy("msm", 3, 256)                        # no 3-D strategy takes n > 255


def test_plugin_adapter_without_device_kinds_fails_early():
    """A user-written VaRCalculationMethod (the reference's plug-in seam) cannot supply a
    Python integrand here: ValueAtRiskCalcualtion names the missing model_kind /
    copula_kind before any in-sample work (data loading, fits) runs."""
    from copula_var.utils.calc_var_ABC import VaRCalculationMethod
    from copula_var.utils.calc_var_class import ValueAtRiskCalcualtion

    calls = []

    class Mine(VaRCalculationMethod):
        def model_params_insample(self, *a, **k):
            calls.append("model_params_insample")

        def calculate_marginals_and_densities_in_sample(self, *a, **k):
            calls.append("marginals")

        def copula_or_correl_params_insample(self, *a, **k):
            calls.append("copula")

        def integration_params_retrieval(self, *a, **k):
            calls.append("integration")

        def integrated_function(self, *a, **k):
            return 0.0

    with pytest.raises(ValueError, match="model_kind=None.*copula_kind=None"):
        ValueAtRiskCalcualtion(["A", "B"], "2001-01-01", 100, Mine(), "2002-01-01")
    assert calls == []

    class Half(Mine):
        model_kind = "garch"
        copula_kind = "clayton"

    with pytest.raises(ValueError, match="copula_kind='clayton'"):
        ValueAtRiskCalcualtion(["A", "B"], "2001-01-01", 100, Half(), "2002-01-01")


def test_factory_adapters_pass_device_check():
    from copula_var.utils.calc_var_class import check_device_adapter
    from copula_var.utils.factory import ValueAtRiskCalculationFactory
    for est in ("msm", "garch", "mean_reverting"):
        for cop in ("student", "gaussian", "plackett"):
            check_device_adapter(ValueAtRiskCalculationFactory.create_var_calculator(cop, est))
