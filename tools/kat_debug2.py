import sys, numpy as np
sys.path.insert(0, 'copula-msm-and-copula-garch-var_amd')
from copula_var import _native as N
k = np.load('tests/golden/kat_special.npz')
u = k['u']
for nu in k['tppf_nus']:
    ref = k[f'tppf_nu{nu:g}']
    got = N.special('tppf', u, nu=nu)
    ok = np.isfinite(ref) & (u >= 1e-150) & (u <= 1 - 1e-16) & (np.abs(ref) < 1e99) & (np.abs(ref) > 1e-6)
    rel = np.where(ok, np.abs(got - ref) / np.abs(np.where(ok, ref, 1)), 0)
    bad = np.argsort(-rel)[:3]
    print(f'nu={nu:g} maxrel={rel.max():.3e} n>1e-10: {(rel>1e-10).sum()}')
    for i in bad:
        print(f'    u={u[i]:.17e} ref={ref[i]:.17e} got={got[i]:.17e} rel={rel[i]:.2e}')
