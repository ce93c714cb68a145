"""CPU oracle for the copula-VaR hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, in numpy/scipy, the reference algorithm
(Nassim-cha/copula-MSM-and-copula-Garch-VaR @ 2024-11-25) for the path that
BASELINE.json's north_star names: the per-date forecast tables (MSM Hamilton
filter, GARCH recursion, UKF), the nested-grid copula quadrature
(utils/calc_integral) and the per-date bisection VaR solve
(utils/calc_var_class.py:95-309).  Every function cites the reference
file:line it follows.

Parity status: PINNED.  tests/test_oracle_golden.py checks this oracle against
golden vectors produced by running the reference itself in the build
container (tests/golden/gen_golden.py).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this package, and only as the checker /
baseline -- never as the product path.  The product path
(copula-msm-and-copula-garch-var_amd/copula_var) runs on the HIP library and
fails loudly when it is missing.
"""
