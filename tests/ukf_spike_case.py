"""Constructed UKF windows whose update puts nearly all the weight on one sigma point
(kalman_mean_reverting/estimate.py:214-229): one return of 6-13 standard deviations a few
days before the window's end.

With eta = r_t / e^{X2} large at every point, h = phi(eta)|eta| is ~1e-40 or smaller at two of
the three sigma points, so the updated mean sits on the third and the reference's variance
sum_i wm2_i (h_i / Z)(X2_i - mean)^2 (:226) is a tiny positive number.  The algebraically
equal shortcut Syy / Z - (Sy / Z)^2 cancels there and rounds to +-1 ulp of (X2 - x)^2: when
it lands below 0, custom_cholesky's var <= 0 -> +1e-8 branch (:72-74) fires where the
reference's does not, and the forecast moves by ~1e-8 relative.

`windows()` returns the cases on which the reference's own filter (oracle.forecast.ukf_run,
pinned to reference-run goldens) does not fail (Z >= 1e-10); `restate()` is a numpy
restatement of the device forecast pass's step (cvq_forecast.hip ukf_forecast_pass) with
either variance form, used by the CPU test to show that the set reaches the cancelling
regime.  Test infrastructure."""
import numpy as np

PARAMS = (0.97, 0.05, 0.15)            # a, l, q of BASELINE cfg 5
N_IN = 64


def windows(seeds=range(24)):
    from oracle.forecast import ukf_run
    a, l, q = PARAMS
    out = []
    for seed in seeds:
        rng = np.random.default_rng(1000 + seed)
        base = rng.standard_normal(N_IN)
        for amp in np.linspace(6.0, 13.0, 15):
            for pos in (N_IN - 4, N_IN - 3, N_IN - 2):
                w = base.copy()
                w[pos] = amp * (1.0 if rng.random() < 0.5 else -1.0)
                _, _, _, failed = ukf_run(w[None], a, l, q)
                if not failed[0]:
                    out.append(w)
    return np.array(out)


def restate(w, form, alpha=1.6, beta=2.0, kappa=1.75):
    """(forecast, number of steps whose variance came out negative) of one window, with the
    device pass's closed-form prediction and the variance as `form`: "shortcut"
    (Syy / Z - mu^2) or "about_mean" (sum w_i (y_i - mu)^2 / Z)."""
    a, l, q = PARAMS
    L = 2
    lam = alpha ** 2 * (L + kappa) - L
    wm0, wm1 = lam / (L + lam), 1 / (2 * (L + lam))
    phi = np.sqrt(L + lam)
    kP = 2 * wm1 * phi * phi
    x, var, neg, xm = l, q, 0, 0.0
    for t in range(w.size):
        dvar = var + 1e-8 if var <= 0 else var
        xm = a * (x - l) + l
        sP = np.sqrt(kP * (a * a * dvar + q * q))
        y = np.array([0.0, phi * sP, -(phi * sP)])
        eta = w[t] * np.exp(-(xm + y))
        wi = np.array([wm0, wm1, wm1]) * ((1 / np.sqrt(2 * np.pi)) * np.exp(-0.5 * eta * eta) * np.abs(eta))
        Z = wi.sum()
        mu = (wi * y).sum() / Z
        if form == "shortcut":
            v2 = (wi * y * y).sum() / Z - mu * mu
        else:
            v2 = (wi[0] * mu * mu + wi[1] * (y[1] - mu) ** 2 + wi[2] * (y[2] - mu) ** 2) / Z
        neg += int(v2 < 0)
        x, var = xm + mu, v2
    return float(np.exp(xm)), neg
