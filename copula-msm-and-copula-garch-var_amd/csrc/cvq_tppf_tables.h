// cvq_tppf_tables.h -- host-side construction of the stdtrit initial-guess tables.
#pragma once
#include <algorithm>
#include <cmath>
#include <vector>

#include "cvq_special.h"

namespace cvq {

// stdtrit initial-guess tables (TConst::tab_c / tab_v), built and checked on the
// host with the same refinement the device runs.  Returns false if the guess is
// not accurate enough for a single Halley step at any interval midpoint.
inline bool build_tppf_tables(TConst& hk, int n_c, int n_v, std::vector<double>& tab) {
    const double ps = hk.p_split, hc = (0.5 - ps) / n_c;
    const double vmax = std::exp(std::log(ps) / hk.nu), hv = vmax / n_v;
    tab.assign(2 * (n_c + 1) + 2 * (n_v + 1), 0.0);
    double* tc = tab.data();
    double* tv = tc + 2 * (n_c + 1);
    for (int i = 0; i <= n_c; ++i) {                 // t(p), dt/dp = 1 / pdf
        const double p = (i == n_c) ? 0.5 : ps + i * hc;
        const double t = (i == n_c) ? 0.0 : stdtrit(hk, p);
        double lnF, lpdf;
        t_lower_logs(hk, t, &lnF, &lpdf);
        tc[2 * i] = t;
        tc[2 * i + 1] = std::exp(-lpdf);
    }
    tv[0] = 0.0;                                     // g = -1/t ~ v exp(-ln_tail / nu)
    tv[1] = std::exp(-hk.ln_tail / hk.nu);
    for (int i = 1; i <= n_v; ++i) {                 // g(v), dg/dv = nu v^(nu-1) / (t^2 pdf)
        const double v = i * hv, lp = hk.nu * std::log(v);
        const double t = tppf_refine(hk, tppf_tail_guess(hk, lp), lp);
        double lnF, lpdf;
        t_lower_logs(hk, t, &lnF, &lpdf);
        tv[2 * i] = -1.0 / t;
        tv[2 * i + 1] = std::exp(std::log(hk.nu) + (hk.nu - 1.0) * std::log(v) - 2.0 * std::log(-t) - lpdf);
    }
    hk.tab_c = tc;
    hk.tab_v = tv;
    hk.n_c = n_c;
    hk.n_v = n_v;
    hk.inv_hc = 1.0 / hc;
    hk.inv_hv = 1.0 / hv;
    double worst = 0.0;
    for (int i = 0; i < n_c; ++i) {
        const double p = ps + (i + 0.5) * hc;
        const double g = tppf_table_guess(hk, p);
        TConst plain = hk;
        plain.tab_c = nullptr;
        const double t = stdtrit(plain, p);
        worst = std::max(worst, std::fabs(g - t) / std::fabs(t));
    }
    for (int i = 0; i < n_v; ++i) {
        const double v = (i + 0.5) * hv, lp = hk.nu * std::log(v);
        if (lp < -700.0) continue;                   // exp(lp) would underflow the check
        const double p = std::exp(lp);
        const double g = tppf_table_guess(hk, p);
        const double t = tppf_refine(hk, tppf_tail_guess(hk, lp), lp);
        worst = std::max(worst, std::fabs(g - t) / std::fabs(t));
    }
    return worst < 2e-7;
}

// Degree-5 polynomial through (s_i, f_i), i < 6 (the Chebyshev points of [0,1]
// up to input rounding), as power-basis coefficients in s (long double solve).
inline void cheb5_fit(const double* sx, const double* f, double* c) {
    long double A[6][7];
    for (int i = 0; i < 6; ++i) {
        const long double s = sx[i];
        long double pw = 1.0L;
        for (int j = 0; j < 6; ++j) { A[i][j] = pw; pw *= s; }
        A[i][6] = f[i];
    }
    for (int col = 0; col < 6; ++col) {                  // Gaussian elimination, partial pivoting
        int piv = col;
        for (int r = col + 1; r < 6; ++r) if (std::fabs((double)A[r][col]) > std::fabs((double)A[piv][col])) piv = r;
        for (int j = 0; j < 7; ++j) std::swap(A[col][j], A[piv][j]);
        for (int r = 0; r < 6; ++r) {
            if (r == col) continue;
            const long double m = A[r][col] / A[col][col];
            for (int j = col; j < 7; ++j) A[r][j] -= m * A[col][j];
        }
    }
    for (int j = 0; j < 6; ++j) c[j] = (double)(A[j][6] / A[j][j]);
}

inline double cheb_node(int i) { return 0.5 - 0.5 * std::cos((2 * i + 1) * M_PI / 12.0); }

// Direct-evaluation tables (TConst::q_c / q_v), degree-5 piecewise polynomials of
// functions bounded away from 0, so relative accuracy carries over to t:
//   centre: r(d) = t(1/2 - d) / d on d in [0, 1/2 - p_split]      (t = d r)
//   tail:   q(v) = -1 / (v t(v^nu)) on v in [0, p_split^(1/nu)]    (t = -1 / (v q))
// Reference values come from the refined quantile (hk must carry working cubic
// tables).  Verified at 5 points per interval (ends included); false if any is
// off by more than tol relative.
inline bool build_tppf_quintic(TConst& hk, int n_c, int n_v, std::vector<double>& q, double tol = 4e-14) {
    const double nu = hk.nu, dmax = 0.5 - hk.p_split, hc = dmax / n_c;
    const double vmax = std::exp(std::log(hk.p_split) / nu), hv = vmax / n_v;
    // reference quantiles refined in long double from the double result (noise ~1e-18)
    using LD = long double;
    auto t_of_p = [&](double p) {
        const LD lp = std::log((LD)p);
        return (double)tppf_refine<LD>(hk, (LD)stdtrit(hk, p), lp);
    };
    auto t_of_lp = [&](double lp) {
        const double t0 = tppf_refine(hk, tppf_tail_guess(hk, lp), lp);
        return (double)tppf_refine<LD>(hk, (LD)t0, (LD)lp);
    };
    q.assign(6 * (n_c + n_v), 0.0);
    double* qc = q.data();
    double* qv = qc + 6 * n_c;
    double f[6], sx[6];
    for (int i = 0; i < n_c; ++i) {
        for (int m = 0; m < 6; ++m) {
            // the device sees p, not d: fit r at d = 1/2 - p of the rounded p
            const double p = 0.5 - (i + cheb_node(m)) * hc;
            const double d = 0.5 - p;
            sx[m] = d / hc - i;
            f[m] = t_of_p(p) / d;
        }
        cheb5_fit(sx, f, qc + 6 * i);
    }
    for (int i = 0; i < n_v; ++i) {
        for (int m = 0; m < 6; ++m) {
            const double v = (i + cheb_node(m)) * hv;
            sx[m] = cheb_node(m);
            f[m] = -1.0 / (v * t_of_lp(nu * std::log(v)));
        }
        cheb5_fit(sx, f, qv + 6 * i);
    }
    TConst tk = hk;
    tk.q_c = qc;
    tk.q_v = qv;
    tk.n_qc = n_c;
    tk.n_qv = n_v;
    tk.inv_qc = 1.0 / hc;
    tk.inv_qv = 1.0 / hv;
    double worst = 0.0;
    for (int i = 0; i < n_c; ++i)
        for (double fr : {0.0, 0.1, 0.5, 0.9, 0.999999}) {
            const double d = (i + fr) * hc;
            if (d <= 0.0) continue;
            const double p = 0.5 - d, t = t_of_p(p);
            worst = std::max(worst, std::fabs(tppf_quintic(tk, p) - t) / std::fabs(t));
        }
    for (int i = 0; i < n_v; ++i)
        for (double fr : {0.0, 0.1, 0.5, 0.9, 0.999999}) {
            const double v = (i + fr) * hv, lp = nu * std::log(v);
            if (v <= 0.0 || lp < -700.0) continue;
            const double p = std::exp(lp), t = t_of_lp(std::log(p));
            worst = std::max(worst, std::fabs(tppf_quintic(tk, p) - t) / std::fabs(t));
        }
    if (!(worst <= tol)) return false;
    hk.n_qc = n_c;
    hk.n_qv = n_v;
    hk.inv_qc = tk.inv_qc;
    hk.inv_qv = tk.inv_qv;
    return true;
}

}  // namespace cvq
