import sys, numpy as np
sys.path.insert(0, 'copula-msm-and-copula-garch-var_amd')
from copula_var import _native as N
k = np.load('tests/golden/kat_special.npz')
u = k['u']
for nu in k['tppf_nus']:
    ref = k[f'tppf_nu{nu:g}']
    got = N.special('tppf', u, nu=nu)
    fin = np.isfinite(ref) & np.isfinite(got)
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300)
    rel = np.where(np.abs(ref) < 1e-6, 0, rel)
    bad = np.argsort(-np.where(fin, rel, np.inf))[:4]
    print(f'nu={nu:g} maxrel(fin)={np.max(np.where(fin, rel, 0)):.3e} nonfinite_mismatch={np.sum(np.isfinite(ref)!=np.isfinite(got))}')
    for i in bad:
        print(f'    u={u[i]:.6e} ref={ref[i]:.17e} got={got[i]:.17e} rel={rel[i]:.2e}')
got = N.special('ndtri', u); ref = k['ndtri']
fin = np.isfinite(ref)
rel = np.abs(got[fin]-ref[fin])/np.maximum(np.abs(ref[fin]),1e-300)
print('ndtri maxrel', rel.max(), 'abs where |ref|<1e-12', np.max(np.abs(got[fin]-ref[fin])[np.abs(ref[fin])<1e-12], initial=0))
got = N.special('erf', k['erf_x'])
print('erf maxabs', np.max(np.abs(got-k['erf'])), 'n diff', np.sum(got != k['erf']))
ut = k['truth_u']
for nu in (1.0, 3.0, 6.0, 30.0):
    tr = k[f'truth_tppf_nu{nu:g}']
    got = N.special('tppf', ut, nu=nu)
    rel = np.abs(got - tr)/np.abs(tr)
    i = np.argmax(rel)
    print('truth nu', nu, 'maxrel', rel.max(), 'at u', ut[i], got[i], tr[i])
