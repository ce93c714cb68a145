// cvq_special.h -- FP64 special functions for gfx950 used on the VaR hot path.
//
// The reference evaluates these through scipy on the host:
//   t.ppf   -> scipy.special.stdtrit   (copulas/student/student.py:100-102)
//   norm.ppf-> scipy.special.ndtri     (copulas/gaussian/gaussian.py:43-44)
//   erf     -> scipy.special.erf       (utils/utils.py:20)
// They are restated here as device code.  Accuracy target ~1e-14 relative
// (scipy's own stdtrit is 1e-11..1e-16); the VaR is decided by
// F(v) < obj_var comparisons and is insensitive far below 1e-8 (§8c).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace cvq {

// Host-precomputed constants of the Student-t distribution for one nu.
struct TConst {
    double nu;          // degrees of freedom
    double a;           // nu / 2
    double ln_nu;       // log(nu)
    double lbeta;       // lgamma(nu/2) + lgamma(1/2) - lgamma(nu/2 + 1/2)
    double ln_k;        // log of Gamma((nu+1)/2) / (sqrt(nu pi) Gamma(nu/2))
    double ln_tail;     // log(k_nu) + (nu-1)/2 log(nu): F(t) ~ exp(ln_tail) |t|^-nu as t -> -inf
    double split;       // (a + 1) / (a + 1/2 + 2): continued-fraction branch point
    double ln_a;        // log(a)
    const double* cf_dir;   // CF coefficients c_k of I_x(a, 1/2)   (d_k = c_k x), device
    const double* cf_cmp;   // CF coefficients c_k of I_y(1/2, a),  device
    int cf_terms;           // table length
    // Initial-guess tables for stdtrit (cubic Hermite, {value, derivative} pairs;
    // nullptr = use the Cornish-Fisher / power-tail guess):
    //   centre: t(p) on p in [p_split, 1/2], uniform in p;
    //   tail:   g(v) = -1/t on v = p^(1/nu) in [0, p_split^(1/nu)], uniform in v
    //           (1/|t| is analytic in v near 0: F ~ C |t|^-nu).
    const double* tab_c;
    const double* tab_v;
    int n_c, n_v;           // intervals
    double p_split, inv_hc, inv_hv, inv_nu;
    // Direct evaluation tables (quintic Hermite in power form, 6 coefficients per
    // interval in the local coordinate s in [0,1)), same variables as above;
    // host-verified to 4e-14 relative, so stdtrit needs no refinement.  nullptr:
    // not built (then the cubic guess + one Halley step is used).
    const double* q_c;
    const double* q_v;
    int n_qc, n_qv;
    double inv_qc, inv_qv;
};

// Host: continued-fraction coefficients of the regularised incomplete beta
// I_x(a, b) = x^a (1-x)^b / (a B(a,b)) * 1/(1 + d1/(1 + d2/(1 + ...))), d_k = c_k x:
//   c_{2m+1} = -(a+m)(a+b+m) / ((a+2m)(a+2m+1)),   c_{2m} = m(b-m) / ((a+2m-1)(a+2m)).
inline void ibeta_cf_coeffs(double a, double b, double* c, int terms) {
    for (int k = 1; k <= terms; ++k) {
        const int m = k / 2;
        if (k & 1) c[k - 1] = -(a + m) * (a + b + m) / ((a + 2.0 * m) * (a + 2.0 * m + 1.0));
        else c[k - 1] = m * (b - m) / ((a + 2.0 * m - 1.0) * (a + 2.0 * m));
    }
}

__host__ __device__ __forceinline__ double pos_inf() { return __builtin_huge_val(); }

// 1/(1 + d1/(1 + d2/(1 + ...))), d_k = c[k-1] x, by the forward recurrence of
// the convergents A_k / B_k (no division per term; the coefficient index is
// wave-uniform, so c[] comes through the scalar cache).  R = double on the
// device; the host also runs it in long double to build the quantile tables.
template <class R = double>
__host__ __device__ inline R ibeta_cf(const double* __restrict__ c, int terms, R x) {
    constexpr R tol = sizeof(R) > 8 ? (R)1e-19L : (R)1e-16;
    R Am = 1, Bm = 1;               // A_1, B_1
    R Ap = 0, Bp = 1;               // A_0, B_0
    for (int k = 1; k < terms; k += 2) {
        R An = fma((R)c[k - 1] * x, Ap, Am), Bn = fma((R)c[k - 1] * x, Bp, Bm);
        Ap = Am; Bp = Bm; Am = An; Bm = Bn;
        An = fma((R)c[k] * x, Ap, Am); Bn = fma((R)c[k] * x, Bp, Bm);
        Ap = Am; Bp = Bm; Am = An; Bm = Bn;
        // |A_k/B_k - A_{k-1}/B_{k-1}| <= tol |A_k/B_k|
        if (fabs(fma(Am, Bp, -Ap * Bm)) <= tol * fabs(Am * Bp)) break;
        if (fabs(Bm) > (R)1e150) {
            const R s = 1 / Bm;
            Am *= s; Ap *= s; Bp *= s; Bm = 1;
        }
    }
    return Am / Bm;
}

// log F_nu(t) and log pdf_nu(t) for t <= 0.
template <class R = double>
__host__ __device__ inline void t_lower_logs(const TConst& k, R t, R* lnF, R* lpdf) {
    const R nu = k.nu, at = fabs(t);
    R L;                                        // log(nu + t^2)
    R ln_t2;                                    // log(t^2)
    if (at > (R)1e100) {
        const R la = log(at);
        ln_t2 = 2 * la;
        L = ln_t2 + log1p((nu / at) / at);
    } else {
        const R t2 = at * at;
        ln_t2 = log(t2);
        L = log(nu + t2);
    }
    *lpdf = (R)k.ln_k - (R)0.5 * (nu + 1) * (L - (R)k.ln_nu);
    const R lnx = (R)k.ln_nu - L;               // x = nu / (nu + t^2)
    const R x = exp(lnx);
    if (x < (R)k.split) {
        // F = 0.5 * I_x(a, 1/2) = 0.5 * x^a (1-x)^(1/2) / (a B) * cf
        const R ln1mx = ln_t2 - L;
        *lnF = (R)-0.693147180559945309417232121458176568L + (R)k.a * lnx + (R)0.5 * ln1mx - (R)k.lbeta -
               (R)k.ln_a + log(ibeta_cf<R>(k.cf_dir, k.cf_terms, x));
    } else {
        // F = 0.5 * (1 - I_y(1/2, a)),  y = t^2 / (nu + t^2) small
        const R y = (at * at) / (nu + at * at);
        R front = 0;
        if (y > 0) front = exp((R)0.5 * log(y) + (R)k.a * log1p(-y) - (R)k.lbeta) * 2 * ibeta_cf<R>(k.cf_cmp, k.cf_terms, y);
        *lnF = log((R)0.5 * (1 - front));
    }
}

// Acklam's rational approximation of the lower-half normal quantile (0 < pp <= 0.5),
// relative error ~1e-9.
__host__ __device__ __forceinline__ double ndtri_approx(double pp) {
    if (pp < 0.02425) {
        const double q = sqrt(-2.0 * log(pp));
        return (((((-7.784894002430293e-03 * q - 3.223964580411365e-01) * q - 2.400758277161838e+00) * q -
                  2.549732539343734e+00) * q + 4.374664141464968e+00) * q + 2.938163982698783e+00) /
               ((((7.784695709041462e-03 * q + 3.224671290700398e-01) * q + 2.445134137142996e+00) * q +
                 3.754408661907416e+00) * q + 1.0);
    }
    const double q = pp - 0.5, r = q * q;
    return (((((-3.969683028665376e+01 * r + 2.209460984245205e+02) * r - 2.759285104469687e+02) * r +
              1.383577518672690e+02) * r - 3.066479806614716e+01) * r + 2.506628277459239e+00) * q /
           (((((-5.447609879822406e+01 * r + 1.615858368580409e+02) * r - 1.556989798598866e+02) * r +
              6.680131188771972e+01) * r - 1.328068155288572e+01) * r + 1.0);
}

// Standard normal quantile, scipy.special.ndtri (gaussian.py:43-44 via norm.ppf): the
// Cephes ndtri algorithm scipy itself ships (rational approximations, no iteration) --
// centre |p - 1/2| < 1/2 - e^-2 in y = p - 1/2; tails in z = 1 / sqrt(-2 log p), split at
// sqrt(-2 log p) = 8.  Restated here; host-checked against scipy 1.15.3's ndtri: 99.996% of
// 2.8e6 points bit-identical, max 4 ulp (tests/test_gpu_parity.py KATs: <= 1e-13 vs mpmath).
__host__ __device__ __forceinline__ double ndtri_poly(double x, const double* c, int deg) {
    double a = c[0];
    for (int i = 1; i <= deg; ++i) a = a * x + c[i];        // Cephes polevl (no fused multiply-add)
    return a;
}
__host__ __device__ __forceinline__ double ndtri_poly1(double x, const double* c, int deg) {   // leading 1
    double a = x + c[0];
    for (int i = 1; i < deg; ++i) a = a * x + c[i];         // Cephes p1evl
    return a;
}
__device__ inline double ndtri(double p) {
    constexpr double P0[5] = {-5.99633501014107895267E1, 9.80010754185999661536E1, -5.66762857469070293439E1,
                              1.39312609387279679503E1, -1.23916583867381258016E0};
    constexpr double Q0[8] = {1.95448858338141759834E0, 4.67627912898881538453E0, 8.63602421390890590575E1,
                              -2.25462687854119370527E2, 2.00260212380060660359E2, -8.20372256168333339912E1,
                              1.59056225126211695515E1, -1.18331621121330003142E0};
    constexpr double P1[9] = {4.05544892305962419923E0, 3.15251094599893866154E1, 5.71628192246421288162E1,
                              4.40805073893200834700E1, 1.46849561928858024014E1, 2.18663306850790267539E0,
                              -1.40256079171354495875E-1, -3.50424626827848203418E-2, -8.57456785154685413611E-4};
    constexpr double Q1[8] = {1.57799883256466749731E1, 4.53907635128879210584E1, 4.13172038254672030440E1,
                              1.50425385692907503408E1, 2.50464946208309415979E0, -1.42182922854787788574E-1,
                              -3.80806407691578277194E-2, -9.33259480895457427372E-4};
    constexpr double P2[9] = {3.23774891776946035970E0, 6.91522889068984211695E0, 3.93881025292474443415E0,
                              1.33303460815807542389E0, 2.01485389549179081538E-1, 1.23716634817820021358E-2,
                              3.01581553508235416007E-4, 2.65806974686737550832E-6, 6.23974539184983293730E-9};
    constexpr double Q2[8] = {6.02427039364742014255E0, 3.67983563856160859403E0, 1.37702099489081330271E0,
                              2.16236993594496635890E-1, 1.34204006088543189037E-2, 3.28014464682127739104E-4,
                              2.89247864745380683936E-6, 6.79019408009981274425E-9};
    constexpr double kExpM2 = 0.13533528323661269189;   // e^-2
    if (!(p >= 0.0 && p <= 1.0)) return __builtin_nan("");
    if (p == 0.0) return -pos_inf();
    if (p == 1.0) return pos_inf();
    double y = p;
    bool lower = true;
    if (y > 1.0 - kExpM2) {                       // upper tail: 1 - p exact
        y = 1.0 - y;
        lower = false;
    }
    if (y > kExpM2) {                             // centre
        y = y - 0.5;
        const double y2 = y * y;
        const double x = y + y * (y2 * ndtri_poly(y2, P0, 4) / ndtri_poly1(y2, Q0, 8));
        return x * 2.50662827463100050242;
    }
    const double x = sqrt(-2.0 * log(y));
    const double x0 = x - log(x) / x;
    const double z = 1.0 / x;
    const double x1 = x < 8.0 ? z * ndtri_poly(z, P1, 8) / ndtri_poly1(z, Q1, 8)
                              : z * ndtri_poly(z, P2, 8) / ndtri_poly1(z, Q2, 8);
    const double r = x0 - x1;
    return lower ? -r : r;
}

// Cubic Hermite on uniform nodes: tab[2k] = y_k, tab[2k+1] = dy/dx_k, x in node units.
__host__ __device__ __forceinline__ double hermite(const double* __restrict__ tab, int n, double x, double h) {
    int k = (int)x;
    k = k < 0 ? 0 : (k > n - 1 ? n - 1 : k);
    const double s = x - k;
    const double y0 = tab[2 * k], d0 = tab[2 * k + 1] * h, y1 = tab[2 * k + 2], d1 = tab[2 * k + 3] * h;
    const double s2 = s * s, s3 = s2 * s;
    return (2.0 * s3 - 3.0 * s2 + 1.0) * y0 + (s3 - 2.0 * s2 + s) * d0 + (3.0 * s2 - 2.0 * s3) * y1 + (s3 - s2) * d1;
}

// Initial guess for t.ppf at pp in (0, 1/2): the plan's Hermite tables (~1e-7
// relative, so one Halley step of stdtrit lands at rounding level), else NaN.
__host__ __device__ __forceinline__ double tppf_table_guess(const TConst& k, double pp) {
    if (k.tab_c == nullptr) return __builtin_nan("");
    if (pp >= k.p_split) return hermite(k.tab_c, k.n_c, (pp - k.p_split) * k.inv_hc, 1.0 / k.inv_hc);
    const double v = exp(log(pp) * k.inv_nu);
    const double g = hermite(k.tab_v, k.n_v, v * k.inv_hv, 1.0 / k.inv_hv);
    return g > 0.0 ? -1.0 / g : __builtin_nan("");
}

// Halley on g(t) = log F(t) - lp for t < 0 (cubic convergence; stop once a step
// is below 1e-6 relative: the next error is then ~1e-18).  Bisection fallback
// whenever a step leaves the bracket F(lo) < p < F(hi).
template <class R = double>
__host__ __device__ inline R tppf_refine(const TConst& k, R t, R lp) {
    constexpr R step_done = sizeof(R) > 8 ? (R)1e-7 : (R)1e-6;
    const R nu = k.nu, inf = (R)pos_inf();
    R lo = -inf, hi = 0;
    for (int it = 0; it < 60; ++it) {
        R lnF, lpdf;
        t_lower_logs<R>(k, t, &lnF, &lpdf);
        const R g = lnF - lp;
        if (g > 0) hi = t; else lo = t;
        if (g == 0) break;
        const R h = exp(lpdf - lnF);                        // g'  = pdf / F
        const R dl = -(nu + 1) * t / (nu + t * t);           // pdf'/pdf
        const R gn = g / h;
        const R den = 1 - (R)0.5 * gn * (dl - h);            // 1 - g g'' / (2 g'^2)
        R tn = (den > (R)0.5 && den < 2) ? t - gn / den : t - gn;
        if (tn == t) break;                                  // correction below one ulp
        bool fallback = false;
        if (!(tn >= lo && tn <= hi)) {                        // outside the bracket: bisect
            fallback = true;
            if (lo == -inf) tn = 2 * t - 1;
            else tn = (R)0.5 * (lo + hi);
        }
        const bool done = !fallback && fabs(tn - t) <= step_done * fabs(tn);
        t = tn;
        if (done) break;
    }
    return t;
}

// Power-tail guess for log p = lp: F = exp(ln_tail)|t|^-nu (1 - A / t^2 + ...),
// A = nu^2 (nu+1) / (2 (nu+2)), inverted to first order: t0 (1 - A / (nu t0^2)).
template <class R = double>
__host__ __device__ __forceinline__ R tppf_tail_guess(const TConst& k, R lp) {
    const R nu = k.nu;
    R t = -exp(((R)k.ln_tail - lp) / nu);
    return t * (1 - nu * (nu + 1) / (2 * (nu + 2) * t * t));
}

__host__ __device__ __forceinline__ double quintic(const double* __restrict__ tab, int n, double x) {
    int k = (int)x;
    k = k < 0 ? 0 : (k > n - 1 ? n - 1 : k);
    const double s = x - k;
    const double* c = tab + 6 * k;
    return fma(fma(fma(fma(fma(c[5], s, c[4]), s, c[3]), s, c[2]), s, c[1]), s, c[0]);
}

// t.ppf at pp in (0, 1/2) straight from the plan's degree-5 tables (see
// build_tppf_quintic): centre t = d r(d), d = 1/2 - pp; tail t = -1 / (v q(v)).
__host__ __device__ __forceinline__ double tppf_quintic(const TConst& k, double pp) {
    if (pp >= k.p_split) {
        const double d = 0.5 - pp;
        return d * quintic(k.q_c, k.n_qc, d * k.inv_qc);
    }
    const double v = exp(log(pp) * k.inv_nu);
    return -1.0 / (v * quintic(k.q_v, k.n_qv, v * k.inv_qv));
}

// t.ppf for pp in (0, 1/2) without the direct tables: Cornish-Fisher / power-tail
// or cubic-table guess, then Halley.
__host__ __device__ inline double tppf_lower_refined(const TConst& k, double pp) {
    const double nu = k.nu;
    double t = tppf_table_guess(k, pp);        // the plan's cubic tables: one Halley step
    if (!(t < 0.0)) {
        // Cornish-Fisher around the normal quantile, or the power tail.
        const double z = ndtri_approx(pp);
        const double z2 = z * z;
        const double tcf = z + (z2 * z + z) / (4.0 * nu) +
                           (((5.0 * z2 + 16.0) * z2 + 3.0) * z) / (96.0 * nu * nu) +
                           ((((3.0 * z2 + 19.0) * z2 + 17.0) * z2 - 15.0) * z) / (384.0 * nu * nu * nu);
        if (nu > 1e5) return tcf;
        const double ttail = tppf_tail_guess(k, log(pp));
        t = (ttail < tcf && z2 > nu) ? ttail : tcf;
        if (!(t < 0.0)) t = -1e-3;
    }
    return tppf_refine(k, t, log(pp));
}

// stdtrit for plans whose direct tables exist (k.q_c != nullptr): no refinement
// code at all, so kernels that inline it keep a small register budget.
__host__ __device__ __forceinline__ double stdtrit_tabulated(const TConst& k, double p) {
    if (!(p >= 0.0 && p <= 1.0)) return __builtin_nan("");
    if (p == 0.0) return -pos_inf();
    if (p == 1.0) return pos_inf();
    if (p == 0.5) return 0.0;
    const bool upper = p > 0.5;
    const double t = tppf_quintic(k, upper ? (1.0 - p) : p);
    return upper ? -t : t;
}

// stdtrit_tabulated without data-dependent branches: the same arithmetic (both
// table variables evaluated, one selected), so a thread can keep two
// evaluations' table gathers in flight together.
__device__ __forceinline__ double log_node(double b);
__device__ __forceinline__ double exp_node(double x);
__device__ __forceinline__ double stdtrit_tab_bf(const TConst& k, double p) {
    const bool upper = p > 0.5;
    const double pp = upper ? (1.0 - p) : p;                   // exact
    const bool centre = pp >= k.p_split;
    const double d = 0.5 - pp;
    // tail variable pp^(1/nu) without library calls (log_node / exp_node, ~1e-14; pp = 0 and NaN
    // are replaced below)
    const double v = exp_node(log_node(pp) * k.inv_nu);
    const double q = centre ? quintic(k.q_c, k.n_qc, d * k.inv_qc) : quintic(k.q_v, k.n_qv, v * k.inv_qv);
    double t = centre ? d * q : -1.0 / (v * q);
    t = upper ? -t : t;
    if (p == 0.5) t = 0.0;
    if (p == 0.0) t = -pos_inf();
    if (p == 1.0) t = pos_inf();
    return (p >= 0.0 && p <= 1.0) ? t : __builtin_nan("");
}

// p^(1/NU) for p in (0, 1] and an integer NU: an exact power-of-two reduction p = w 2^(NU k),
// w in [1/2, 2^(NU-1)), a float seed 2^(log2(w) / NU) (v_log_f32 / v_exp_f32, ~1e-7) and two
// Newton steps on v^NU = w (~1e-14, then ~1 ulp) -- instead of exp(log(p) / nu) (two FP64
// library calls, ~110 VALU).  p = 0 gives NaN (callers select their own value there).
template <int N>
__device__ __forceinline__ double ipow_pos(double v) {
    if constexpr (N == 1) return v;
    else if constexpr (N % 2 == 0) { const double h = ipow_pos<N / 2>(v); return h * h; }
    else return ipow_pos<N - 1>(v) * v;
}
__device__ __forceinline__ double fast_rcp(double r);
template <int NU>
__device__ __forceinline__ double root_nu(double p) {
    int e;
    const double m = frexp(p, &e);                              // p = m 2^e, m in [1/2, 1)
    const int k = e >= 0 ? e / NU : -((NU - 1 - e) / NU);       // floor(e / NU)
    const double w = ldexp(m, e - NU * k);
    double v = (double)__builtin_amdgcn_exp2f(__builtin_amdgcn_logf((float)w) * (1.0f / (float)NU));
#pragma unroll
    for (int it = 0; it < 2; ++it) {                            // v <- v + (w / v^(NU-1) - v) / NU
        const double t = fma(w, fast_rcp(ipow_pos<NU - 1>(v)), -v);
        v = fma(t, 1.0 / NU, v);
    }
    return ldexp(v, k);
}

// stdtrit_tab_bf for an integer nu = NU: the tail variable p^(1/nu) by root_nu and the tail's
// -1 / (v q) by a Newton-refined reciprocal (~1 ulp; the VaR tolerates ~1e-8)
template <int NU>
__device__ __forceinline__ double stdtrit_tab_int(const TConst& k, double p) {
    const bool upper = p > 0.5;
    const double pp = upper ? (1.0 - p) : p;                   // exact
    const bool centre = pp >= k.p_split;
    const double d = 0.5 - pp;
    const double v = root_nu<NU>(pp);
    const double q = centre ? quintic(k.q_c, k.n_qc, d * k.inv_qc) : quintic(k.q_v, k.n_qv, v * k.inv_qv);
    double t = centre ? d * q : -fast_rcp(v * q);
    t = upper ? -t : t;
    if (p == 0.5) t = 0.0;
    if (p == 0.0) t = -pos_inf();
    if (p == 1.0) t = pos_inf();
    return (p >= 0.0 && p <= 1.0) ? t : __builtin_nan("");
}

// Student-t quantile t.ppf(p, nu) (scipy semantics: 0 -> -inf, 1 -> +inf, outside -> nan).
__host__ __device__ inline double stdtrit(const TConst& k, double p) {
    if (!(p >= 0.0 && p <= 1.0) || !(k.nu > 0.0)) return __builtin_nan("");
    if (p == 0.0) return -pos_inf();
    if (p == 1.0) return pos_inf();
    if (p == 0.5) return 0.0;
    const bool upper = p > 0.5;
    const double pp = upper ? (1.0 - p) : p;   // exact
    const double t = (k.q_c != nullptr) ? tppf_quintic(k, pp)      // the plan's verified direct tables
                                        : tppf_lower_refined(k, pp);
    return upper ? -t : t;
}

// 1/r for r > 0: hardware reciprocal + two Newton steps (~1 ulp; no IEEE div sequence).
__device__ __forceinline__ double fast_rcp(double r) {
    double y = __builtin_amdgcn_rcp(r);
    y = fma(y, fma(-r, y, 1.0), y);
    y = fma(y, fma(-r, y, 1.0), y);
    return y;
}

// exp(x): 2^k e^r, |r| <= ln2 / 2, degree-9 polynomial fitted to exp's relative error on that
// interval (max 1.4e-14; the solve's decisions are unchanged by 1e-8 node noise).
// For finite |x| < 1e9; x < -1075 underflows to 0, NaN stays NaN.
__device__ __forceinline__ double exp_node(double x) {
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, x);      // ln2 hi (exact k * hi for |k| < 2^20)
    r = fma(-k, 1.90821492927058770002e-10, r);             // ln2 lo
    double p = 2.747468209548047e-06;
    p = fma(p, r, 2.488396512173419e-05);
    p = fma(p, r, 0.00019841616545137992);
    p = fma(p, r, 0.001388880293639777);
    p = fma(p, r, 0.008333332984833044);
    p = fma(p, r, 0.041666667031658604);
    p = fma(p, r, 0.1666666666788623);
    p = fma(p, r, 0.499999999994599);
    p = fma(p, r, 0.9999999999998875);
    p = fma(p, r, 1.0000000000000127);
    return __builtin_amdgcn_ldexp(p, (int)k);
}

// exp(x) as exp_node with a degree-7 polynomial (relative error 4.0e-11 on |r| <= ln2 / 2, fitted
// to equioscillate; tools/exp_fit.py), two FMAs shorter -- node noise 2.5 decades under the 1e-8
// the decisions tolerate and under the 1e-10 the slab (compute_integral) tests hold.  Same domain
// as exp_node.  The SORTED Gaussian node's exp with CVQ_SORT_EXP2=0 (default: exp2_node7 below).
__device__ __forceinline__ double exp_node7(double x) {
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, x);
    r = fma(-k, 1.90821492927058770002e-10, r);
    double p = 0.00019772555637949558;
    p = fma(p, r, 0.0013948167915837227);
    p = fma(p, r, 0.00833356655115887);
    p = fma(p, r, 0.04166622570210699);
    p = fma(p, r, 0.16666665093713834);
    p = fma(p, r, 0.5000000104412344);
    p = fma(p, r, 1.0000000002478642);
    p = fma(p, r, 0.9999999999617687);
    return __builtin_amdgcn_ldexp(p, (int)k);
}

// 2^x as exp_node7 in t = r / ln2 (coefficient k times ln2^k; tools/exp_fit.py --base2): k = rint(x),
// t = x - k exact, no ln2 reduction -- for arguments already scaled by log2(e) (the SORTED Gaussian
// records).  4.0e-11 relative; x < -1075 underflows to 0, NaN stays NaN; finite |x| < 1e9.
__device__ __forceinline__ double exp2_node7(double x) {
    const double k = __builtin_rint(x);
    const double t = x - k;
    double p = 1.5199910599689e-05;
    p = fma(p, t, 0.000154692740464984);
    p = fma(p, t, 0.001333393130124095);
    p = fma(p, t, 0.009618027317530873);
    p = fma(p, t, 0.055504103426500875);
    p = fma(p, t, 0.24022651197562325);
    p = fma(p, t, 0.6931471807317516);
    p = fma(p, t, 0.9999999999617687);
    return __builtin_amdgcn_ldexp(p, (int)k);
}

// log(b) for finite b > 0 (the node power base, the quantile tail pp): b = 2^k m, m in [sqrt(1/2), sqrt(2)),
// log(1 + f) from s = f / (2 + f) and the published fdlibm e_log.c minimax polynomial in s^2
// (< 1 ulp there; the reciprocal here is v_rcp_f64 + two Newton steps, ~1 ulp more), no
// branches or library calls.
__device__ __forceinline__ double log_node(double b) {
    double m = __builtin_amdgcn_frexp_mant(b);             // [1/2, 1)
    int k = __builtin_amdgcn_frexp_exp(b);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;
    k = lo ? k - 1 : k;
    const double f = m - 1.0;
    const double s = f * fast_rcp(2.0 + f);
    const double z = s * s;
    // R = Lg1 z + ... + Lg7 z^7 as one Horner chain (fewer live values than fdlibm's even / odd split)
    double R = fma(z, 1.479819860511658591e-01, 1.531383769920937332e-01);
    R = fma(z, R, 1.818357216161805012e-01);
    R = fma(z, R, 2.222219843214978396e-01);
    R = fma(z, R, 2.857142874366239149e-01);
    R = fma(z, R, 3.999999999940941908e-01);
    R = fma(z, R, 6.666666666666735130e-01);
    R *= z;
    const double hfsq = 0.5 * f * f, dk = (double)k;
    return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

// log_node for the quadrature nodes' general power (b >= 1, then scaled by ex ~ -3.7 and exponentiated at
// 4e-11): one Newton step on v_rcp_f64 (2^-48 relative in s) and the minimax polynomial without its Lg7
// term (s^15 Lg7 < 5e-13): within 5e-13 absolute of log b (host check: tools/log_fit_check.py), three
// FMAs fewer than log_node
__device__ __forceinline__ double log_node_fast(double b) {
    double m = __builtin_amdgcn_frexp_mant(b);
    int k = __builtin_amdgcn_frexp_exp(b);
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;
    k = lo ? k - 1 : k;
    const double f = m - 1.0;
    const double d = 2.0 + f;
    double y = __builtin_amdgcn_rcp(d);
    y = fma(y, fma(-d, y, 1.0), y);
    const double s = f * y;
    const double z = s * s;
    double R = fma(z, 1.531383769920937332e-01, 1.818357216161805012e-01);
    R = fma(z, R, 2.222219843214978396e-01);
    R = fma(z, R, 2.857142874366239149e-01);
    R = fma(z, R, 3.999999999940941908e-01);
    R = fma(z, R, 6.666666666666735130e-01);
    R *= z;
    const double hfsq = 0.5 * f * f, dk = (double)k;
    return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + dk * 1.90821492927058770002e-10)) - f);
}

__device__ __forceinline__ double pow_gen(double b, double ex);
// b^ex for b >= 1 with ex = -m/2 (m = node_m >= 0): squarings + one reciprocal;
// m < 0 (non-integer nu: an IFM-fitted copula) selects exp(ex log b) from log_node / exp_node
// (~1e-14 relative; the OCML pair cost ~210 instructions per node in the solve kernels' node
// loops, ~10x the integer-nu node); b = inf -> 0 and NaN -> NaN, as pow gives them.
// Used once per quadrature node.
__device__ __forceinline__ double pow_node(double b, int m, double ex) {
    if (m >= 0) {
        double r = 1.0, s = b;
        int k = m >> 1;
        while (k) { if (k & 1) r *= s; s *= s; k >>= 1; }
        if (m & 1) r *= sqrt(b);
        if (!(r < 1.0e300)) return r == r ? 0.0 : r;     // overflow -> 0, NaN stays NaN
        return fast_rcp(r);
    }
    return pow_gen(b, ex);                                   // ex <= -1/2: +inf -> 0, NaN stays NaN
}

// b^ex for b >= 1 from log_node / exp_node (~1e-14 relative, no library calls); b = +inf gives
// 0 (ex < 0) or +inf, NaN stays NaN
__device__ __forceinline__ double pow_gen(double b, double ex) {
    const double y = exp_node(ex * log_node(b));
    return (b < 1.0e300) ? y : (b == b ? (ex < 0.0 ? 0.0 : b) : b);
}

// b^(-m/2) for b >= 1, general m >= 0 (m < 0: b^ex, ex = -(nu+1)/2); no loop for m <= 16.
__device__ __forceinline__ double pow_half_neg(double b, int m, double ex) {
    if (m < 0 || m > 16) return pow_gen(b, ex);
    const double b2 = b * b, b4 = b2 * b2, b8 = b4 * b4;
    const int k = m >> 1;
    double r = (k & 1) ? b : 1.0;
    if (k & 2) r *= b2;
    if (k & 4) r *= b4;
    if (k & 8) r *= b8;
    if (m & 1) r *= sqrt(b);
    if (!(r < 1.0e300)) return r == r ? 0.0 : r;
    return 1.0 / r;
}

// b^(M/2) for a compile-time M >= 0 (the integer-nu tables: M = nu + 1)
template <int M>
__device__ __forceinline__ double pow_half_pos_c(double b) {
    double r = 1.0, s = b;
#pragma unroll
    for (int k = M >> 1; k; k >>= 1) {
        if (k & 1) r *= s;
        s *= s;
    }
    if constexpr (M & 1) r *= sqrt(b);
    return r;
}

// b^(m/2) for b >= 1, general m >= 0 (m < 0: exp(ex log b)), the reciprocal of pow_half_neg
// without its division (ex = +(nu+1)/2 here)
__device__ __forceinline__ double pow_half_pos(double b, int m, double ex) {
    if (m < 0 || m > 16) return pow_gen(b, ex);
    const double b2 = b * b, b4 = b2 * b2, b8 = b4 * b4;
    const int k = m >> 1;
    double r = (k & 1) ? b : 1.0;
    if (k & 2) r *= b2;
    if (k & 4) r *= b4;
    if (k & 8) r *= b8;
    if (m & 1) r *= sqrt(b);
    return r;
}

__device__ __forceinline__ double nan_to_num(double v) {
    // numpy.nan_to_num defaults: nan -> 0, +inf -> DBL_MAX, -inf -> -DBL_MAX
    if (v != v) return 0.0;
    if (v == pos_inf()) return 1.7976931348623157e308;
    if (v == -pos_inf()) return -1.7976931348623157e308;
    return v;
}

}  // namespace cvq
