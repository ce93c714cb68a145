"""Host check of log_node_fast's truncation (cvq_special.h): the fdlibm-form log(b) with one Newton step
on a 2^-24.4 reciprocal and the minimax polynomial with / without its Lg7 term, against numpy's log
over b in [1, 1e31] (the Student node power's base).  numpy has no FMA, so the evaluation rounds a
little differently; the truncation error (~5e-13 absolute) is what this measures."""
import numpy as np

LG = [1.479819860511658591e-01, 1.531383769920937332e-01, 1.818357216161805012e-01, 2.222219843214978396e-01,
      2.857142874366239149e-01, 3.999999999940941908e-01, 6.666666666666735130e-01]


def log_fdlibm(b, drop7, rng):
    m, e = np.frexp(b)
    lo = m < 0.70710678118654752440
    m = np.where(lo, m + m, m)
    k = np.where(lo, e - 1, e).astype(float)
    f = m - 1.0
    d = 2.0 + f
    y = (1.0 / d) * (1 + 2.0 ** -24.4 * rng.choice([-1, 1], len(d)))     # v_rcp_f64's error, either sign
    y = y + y * (1.0 - d * y)                                             # one Newton step
    s = f * y
    z = s * s
    coef = LG[1:] if drop7 else LG
    R = np.full_like(z, coef[0])
    for c in coef[1:]:
        R = z * R + c
    R = R * z
    hfsq = 0.5 * f * f
    return k * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + k * 1.90821492927058770002e-10)) - f)


if __name__ == "__main__":
    rng = np.random.default_rng(1)
    b = np.concatenate([1 + rng.random(20000) * 1e-3, 10 ** rng.uniform(0, 31, 200000), 1 + rng.random(20000)])
    for drop7 in (False, True):
        err = np.abs(log_fdlibm(b, drop7, rng) - np.log(b))
        print(f"{'without Lg7' if drop7 else 'full polynomial'}: max |error| {err.max():.3g}")
