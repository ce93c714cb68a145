"""Fit exp's polynomial on |r| <= ln2/2 with (near-)equioscillating relative error (cvq_special.h
exp_node7).  Weighted Chebyshev least squares, reweighted by the current error; prints the max
relative error of the double Horner evaluation and the coefficients (r^0 first).  --base2: the same
polynomial in t = r / ln2 (2^t on |t| <= 1/2, exp2_node7: coefficient k times ln2^k)."""
import sys

import numpy as np
from numpy.polynomial import chebyshev as C, polynomial as P


def fit(deg, iters=30, n=4000):
    h = np.log(2) / 2
    x = np.cos(np.pi * (np.arange(n) + 0.5) / n) * h
    w = np.exp(-x)
    for _ in range(iters):
        pc = C.cheb2poly(C.chebfit(x / h, np.exp(x), deg, w=w))
        coef = [pc[k] / h ** k for k in range(deg + 1)]
        e = np.abs(P.polyval(x, coef) / np.exp(x) - 1)
        w = np.exp(-x) * (e / e.max()) ** 0.5 + 1e-3
    xs = np.linspace(-h, h, 200001)
    return coef, float(np.max(np.abs(P.polyval(xs, coef) / np.exp(xs) - 1)))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    deg = int(args[0]) if args else 7
    coef, err = fit(deg)
    if "--base2" in sys.argv:
        coef = [c * np.log(2) ** k for k, c in enumerate(coef)]
        ts = np.linspace(-0.5, 0.5, 200001)
        err = float(np.max(np.abs(P.polyval(ts, coef) / np.exp2(ts) - 1)))
    print(f"degree {deg}{' (2^t)' if '--base2' in sys.argv else ''}: max relative error {err:.3g}")
    for k, v in enumerate(coef):
        print(k, repr(float(v)))
