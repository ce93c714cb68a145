"""A constructed Q4 case (calc_var_class.py:293): F passes exactly through 0.0 after the
reference's first bisection level subtracted a slab it never added (Q1, :132).

MSM model with one vol state, Plackett copula at theta = 1 (plackett.py:66-69 gives c = 1
exactly), a 21-point grid of step 0.5 and static densities that are zero except at two
indices per axis (value 2^-3, so every nonzero node mass is (2^-3 * 0.5)^2 = 2^-8 and every
sum below is exact in any order).  The four nonzero nodes lie at levels -2.5, -1.75, -1.5
and L22.  Per date:
  r0 = F(-3) = 0 < 0.05          -> second slab (-3, -2]: F(-2) = m    (prev_upper -3, Q1)
  bracket (-2, 0]; level 0: mid -1, slab (-2, -1] (2 m) subtracted -> F = -m < 0
  then F(v) = -m for v < L22 and exactly 0 from L22 on: the first mid >= L22 makes every
  date's F == 0 and the reference breaks (Q4) with VaR = the bracket's midpoint.
L22 = -0.75 breaks at iteration 1 (VaR -0.5), L22 = -0.25 at iteration 2 (VaR -0.25).
Whole brackets fit the solve kernels' tails (n = 21), so these levels run in the tails'
closed-form walk (zero_interval): the round-3 rule ("F just above lo < 0: no zeros")
would miss the break."""
import numpy as np

N = 21


def build(l22: float, T: int = 3):
    x = np.linspace(-5, 5, N)
    step = np.diff(x, prepend=x[0])
    step[0] = step[1]
    dens = np.zeros((2, 1, N))
    xj2 = 2 * l22 + 1.5                                  # x_i2 + x_j2 = 2 L22, x_i2 = -1.5
    ia = [int(np.argmin(np.abs(x - v))) for v in (-3.0, -1.5)]
    jb = [int(np.argmin(np.abs(x - v))) for v in (-2.0, xj2)]
    dens[1, 0, ia] = 0.125                               # axis 0 (Q5: densities[(c - 1) mod dim])
    dens[0, 0, jb] = 0.125                               # axis 1
    return dict(model="msm", copula="plackett", dim=2, x_values=x, step=step, densities=dens,
                combos=np.zeros((1, 2), dtype=np.int64), weights=np.array([0.5, 0.5]),
                copula_params=np.array([1.0]), unique_vol_states=np.ones((2, 1)),
                forecasts_by_states=np.ones((T, 2, 1)), forecasts=np.ones((T, 1)), ptf_mean=0.0)


CASES = {-0.75: (-0.5, 1), -0.25: (-0.25, 2)}            # L22 -> (VaR, iterations at the break)
