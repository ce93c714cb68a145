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

}  // namespace cvq
