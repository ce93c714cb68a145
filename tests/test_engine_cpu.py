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
    assert auto_strategy("msm", 3, 128) == "sorted"
    assert auto_strategy("garch", 3, 255) == "sorted"
    assert auto_strategy("msm", 2) == "compact"            # n unknown: the 2-D rule
    with pytest.raises(ValueError):
        auto_strategy("msm", 3, 256)                        # no 3-D strategy takes n > 255
