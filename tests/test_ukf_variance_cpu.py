"""The UKF update's cancelling regime, on the CPU (estimate.py:214-229).

The constructed windows of tests/ukf_spike_case.py put nearly all of one update's weight on
one sigma point.  A numpy restatement of the device forecast pass shows that there the
shortcut variance Syy / Z - mu^2 goes negative on many windows and moves the forecast by
~1e-8 relative, while the variance about the updated mean -- the form the reference uses
(:226) and cvq_forecast.hip's ukf_forecast_pass now computes -- never does and stays within
1e-13 of the reference's filter (oracle.forecast.ukf_run).  The GPU side is
tests/test_ukf_variance_gpu.py."""
import numpy as np

import ukf_spike_case as U
from oracle.forecast import ukf_run


def test_constructed_windows_reach_the_cancelling_regime():
    W = U.windows()
    assert W.shape[0] >= 200
    ref, _, _, failed = ukf_run(W, *U.PARAMS)
    assert not failed.any()
    neg_short, worst_short, worst_mean = 0, 0.0, 0.0
    for k in range(W.shape[0]):
        fs, ns = U.restate(W[k], "shortcut")
        fm, nm = U.restate(W[k], "about_mean")
        assert nm == 0                                   # sum of non-negative terms
        neg_short += int(ns > 0)
        worst_short = max(worst_short, abs(fs - ref[k]) / ref[k])
        worst_mean = max(worst_mean, abs(fm - ref[k]) / ref[k])
    assert neg_short >= 20, neg_short                    # the regime is reached ...
    assert worst_short > 1e-9, worst_short               # ... and the shortcut is visibly off there
    assert worst_mean < 1e-13, worst_mean
