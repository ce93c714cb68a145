"""The SORTED strategy's premise, checked on the CPU against the oracle's membership
rule (create_grids.py:102-108 + integration_algo.py:20, Q9 / Q10):

a node (row r, inner index j >= 1) lies in the slab (a, b] iff a < v*(r, j) <= b,
v*(r, j) = the smallest double v with x_j <= (v - lev_r) / w0.

So every slab is one contiguous range of the nodes sorted by v*, and its value is a
difference of two positions.  The exact v* restated here mirrors vstar_exact in
csrc/cvq_plan.hip (start at x_j w0 + lev, walk ulps to the boundary)."""
import numpy as np
import pytest

from conftest import load_golden


def vstar(x, lev, w0):
    xj = np.broadcast_to(x, np.broadcast_shapes(x.shape, lev.shape))
    v = xj * w0 + lev
    pred = lambda v: xj <= (v - lev) / w0
    for _ in range(64):                       # walk down while the predecessor still qualifies
        d = np.nextafter(v, -np.inf)
        m = pred(v) & pred(d)
        if not m.any():
            break
        v = np.where(m, d, v)
    for _ in range(64):                       # walk up until the predicate holds
        m = ~pred(v)
        if not m.any():
            break
        v = np.where(m, np.nextafter(v, np.inf), v)
    bad = ~(pred(v) & ~pred(np.nextafter(v, -np.inf)))
    if bad.any():                             # cancellation near v = 0: bisect on the ordered-integer view
        v = np.array(v)
        for k in zip(*np.nonzero(bad)):
            xk, lk = float(xj[k]), float(np.broadcast_to(lev, v.shape)[k])
            p = lambda o: xk <= (_o2d(o) - lk) / w0
            lo, hi = _d2o(-np.inf), _d2o(np.inf)
            while hi - lo > 1:
                m = lo + (hi - lo) // 2
                if p(m):
                    hi = m
                else:
                    lo = m
            v[k] = _o2d(hi)
    assert (pred(v) & ~pred(np.nextafter(v, -np.inf))).all()
    return v


def _d2o(d):
    b = int(np.float64(d).view(np.int64))
    return b if b >= 0 else ~(b & 0x7FFFFFFFFFFFFFFF)


def _o2d(o):
    b = o if o >= 0 else (~o) | -0x8000000000000000
    return float(np.int64(b).view(np.float64))


def _geometry(z):
    from oracle.quadrature import Problem
    per = (z["forecasts_by_states"], z["forecasts"]) if str(z["model"]) == "msm" else z["sigma_forecasts"]
    P = Problem(str(z["model"]), str(z["copula"]), int(z["dim"]), z["x_values"], z["step"], z["densities"],
                z["combos"], z["weights"], z["copula_params"], per, z.get("unique_vol_states"))
    x, w = P.x, P.w
    if P.dim == 2:
        lev = (x * w[1])[:, None]
    else:
        lev = ((x[:, None] * w[1]) + (x[None, :] * w[2]))[:, :, None]
    vs = vstar(x.reshape([1] * (P.dim - 1) + [-1]), lev, w[0])
    inner = np.zeros(vs.shape, dtype=bool)
    inner[..., 1:] = True                     # x_0 = -5 is never inside (strict, clamped lower edge, Q9)
    return P, vs, inner


@pytest.mark.parametrize("case", ["cfg1", "cfg2_n64", "cfg3_n128", "cfg4_k6_n16", "garch3d_student_n16"])
def test_membership_is_a_vstar_interval(case):
    z = load_golden(case)
    P, vs, inner = _geometry(z)
    rng = np.random.default_rng(3)
    # the solve's fixed levels, dyadic bisection points, the golden calls' own bounds and random levels
    levels = [-100.0, -7.5, -3.5, -3.0, -2.0, 0.0, -2.75, -1.0, -0.5, -0.25]
    for i in range(int(z["n_calls"])):
        levels += list(np.unique(z[f"call{i:02d}_bounds"]))
    levels += list(rng.uniform(-8, 0.5, 40))
    levels = np.array(levels)
    for _ in range(200):
        a, b = rng.choice(levels, 2)
        got = inner & (vs > a) & (vs <= b)
        assert np.array_equal(got, P.inner_mask(a, b)), (case, a, b)


@pytest.mark.parametrize("case", ["cfg2_n64", "cfg4_k6_n16"])
def test_slab_is_a_sorted_range(case):
    """slab value = sum over sorted positions [ub(a), ub(b)) (np.searchsorted 'right' = ub)."""
    z = load_golden(case)
    P, vs, inner = _geometry(z)
    keep = inner & (vs <= 0.0)                # reachable nodes (v_cap = 0)
    order = np.argsort(vs[keep], kind="stable")
    svs = vs[keep][order]
    for i in range(int(z["n_calls"])):
        bounds, ref = z[f"call{i:02d}_bounds"], z[f"call{i:02d}_result"]
        for t in range(P.T):
            m = P.mass(t)[keep][order]
            a, b = bounds[t]
            p0, p1 = np.searchsorted(svs, [a, b], side="right")
            got = m[p0:p1].sum() if p1 > p0 else 0.0
            np.testing.assert_allclose(got, ref[t], rtol=1e-10, atol=1e-15)
