// cvq_quad_kernels.h -- gfx950 kernels of the copula quadrature + VaR solve.
//
// Reference path (Nassim-cha/copula-MSM-and-copula-Garch-VaR @ 2024-11-25):
//   calc_var            utils/calc_var_class.py:95-177, bisection :250-309, adjust :214-248
//   compute_integral    utils/calc_var_class.py:179-212 -> utils/calc_integral/calc_integral.py:8-225
//   nested grid         utils/calc_integral/create_grids.py:6-240 (membership :102-108, :127; Q5/Q6)
//   integrands          utils/calc_integral/integration_functions/{msm,garch}_integration_function.py
//   copula densities    copulas/{student,gaussian,plackett}/*.py
//
// MI355X design: the special functions depend only on (date, axis,
// 1-D grid index), so k_tables evaluates them once per table entry; a node of
// the nested grid then costs a quadratic form, one power and a short W
// contraction.  Rows of the innermost axis are processed one wavefront per
// row with an in-register inclusive scan; the solve walks the bisection with
// per-row binary searches on an LDS copy of the grid.
#pragma once
#include "cvq_common.h"

namespace cvq {

constexpr double kInvSqrt2 = 1.4142135623730951;      // np.sqrt(2): divided by, as utils.py:20
constexpr double kInvSqrt2Pi = 0.3989422804014327;    // 1 / np.sqrt(2 * np.pi)

// ------------------------------------------------------------------ wave helpers
// DPP lane exchange of a double (two 32-bit halves); CTRL is a gfx9 dpp_ctrl code.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}

// Wave-wide sum, identical (bitwise) in every lane: symmetric DPP exchanges within
// rows of 16 (xor 1, xor 2, half-mirror, mirror), then the four row sums combined
// in a fixed order.  No LDS traffic.
// unrolled vol-state loops (MSM q = k + 1 <= 8: k <= 7) issue their table loads together
constexpr int kQUnroll = 8;

__device__ __forceinline__ double wave_sum(double v) {
    v += dpp_f64<0xB1>(v);      // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);      // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);     // row_half_mirror
    v += dpp_f64<0x140>(v);     // row_mirror
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// -------------------------------------------------------- static Phi (MSM only)
// phi[d][s][i] = 0.5 * (1 + erf((x_i / sigma_{d,s}) / sqrt 2))  (msm_integration_function.py:32-36)
#ifndef CVQ_NO_PLAN_KERNELS    // non-template kernels live in cvq_plan.hip only
__global__ void k_phi(StaticDev S, const double* __restrict__ uvs, double* __restrict__ phi) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    const int total = S.dim * S.q * S.n;
    if (idx >= total) return;
    const int i = idx % S.n;
    const int ds = idx / S.n;
    const double xs = S.x[i] / uvs[ds];
    phi[idx] = 0.5 * (1.0 + erf(xs / kInvSqrt2));
}
#endif

// ---------------------------------------------------------------- k_tables
// One thread per (date t, axis d, grid index i):
//   u   = marginal CDF  (MSM: sum_s f_t[d,s] Phi(x/sigma_{d,s}); GARCH/UKF: Phi(x/sigma_t,d))
//   A   = z = t.ppf(u, nu) | norm.ppf(u)        (Plackett: A = u)
//   B   = pdf / univariate-copula-margin-pdf      (MSM: pdf = 1; Plackett: B = pdf)
// Layout [T][dim][n], coalesced along i.
// TAB: the plan has verified direct t.ppf tables (Student only; see stdtrit_tabulated).
// Marginal CDF value u and density factor of grid index i on axis d, date row td.
template <bool MSM>
__device__ __forceinline__ void marginal_u(const StaticDev& S, const double* __restrict__ a, long long td, int d, int i,
                                           double* u_out, double* pdf_out) {
    if (MSM) {
        const double* f = a + td * S.q;
        // 32-bit element offsets into the static table (dim q n <= 12288 entries): the loads take
        // the SGPR base + VGPR offset form, no 64-bit address arithmetic per load
        const unsigned ph0 = (unsigned)(d * S.q * S.n + i);
        double acc;
        if (S.q <= kQUnroll) {                                   // every load issued before the sum
            // the weights of states s >= q are 0 (their Phi loads repeat state q - 1's finite
            // values), so acc + 0 * pv[s] leaves the sum bit for bit unchanged and no scalar
            // load waits behind a branch on s < q
            double pv[kQUnroll], fv[kQUnroll];
#pragma unroll
            for (int s = 0; s < kQUnroll; ++s) fv[s] = f[min(s, S.q - 1)];
#pragma unroll
            for (int s = 0; s < kQUnroll; ++s) pv[s] = ld32(S.phi, ph0 + (unsigned)(min(s, S.q - 1) * S.n));
            acc = fv[0] * pv[0];
#pragma unroll
            for (int s = 1; s < kQUnroll; ++s) acc = acc + (s < S.q ? fv[s] : 0.0) * pv[s];
        } else {
            acc = f[0] * ld32(S.phi, ph0);
            for (int s = 1; s < S.q; ++s) acc += f[s] * ld32(S.phi, ph0 + (unsigned)(s * S.n));
        }
        *u_out = acc;                                            // msm_integration_function.py:34-36
        *pdf_out = 1.0;
    } else {
        const double sig = a[td];
        const double xs = S.x[i] / sig;                         // garch_integration_function.py:31
        *u_out = 0.5 * (1.0 + erf(xs / kInvSqrt2));              // :33
        *pdf_out = (kInvSqrt2Pi * exp(-0.5 * (xs * xs))) / sig;  // :38
    }
}

// NUI > 0 (with TAB): the Student nu is the integer NUI -- quantile tail variable by root_nu,
// B = pdf (1 + z^2/nu)^((nu+1)/2) / g_uni without divisions (~1 ulp from the reference's
// arithmetic; the VaR tolerates ~1e-8 relative node noise)
template <int COP, bool MSM, bool TAB = false, int NUI = 0>
__device__ __forceinline__ void table_entry(const StaticDev& S, const double* __restrict__ a, long long td, int d,
                                            int i, double* A_out, double* B_out) {
    double u, pdf;
    marginal_u<MSM>(S, a, td, d, i, &u, &pdf);
    if constexpr (COP == CVQ_STUDENT && TAB && NUI > 0) {
        const double z = stdtrit_tab_int<NUI>(S.tk, u);                              // student.py:102
        const double pw = pow_half_pos_c<NUI + 1>(fma(z * z, S.inv_nu, 1.0));            // :164-172, uni_m = nu + 1
        *A_out = z;
        *B_out = isfinite(z) ? (pdf * pw) * S.inv_g_uni : pdf * pos_inf();
        return;
    }
    if (COP == CVQ_PLACKETT) {
        *A_out = u;
        *B_out = pdf;
    } else {
        double z, uni;
        if (COP == CVQ_STUDENT) {
            z = TAB ? stdtrit_tab_bf(S.tk, u) : stdtrit(S.tk, u);   // student.py:102
            uni = isfinite(z) ? S.g_uni * pow_half_neg(1.0 + (z * z) / S.nu, S.uni_m, S.uni_ex) : 0.0;   // :164-172
        } else {
            z = ndtri(u);                                        // gaussian.py:44
            uni = kInvSqrt2Pi * exp(-0.5 * (z * z));             // gaussian.py:82
        }
        *A_out = z;
        *B_out = (1.0 / uni) * pdf;
    }
}

template <int COP, bool MSM>
__global__ __launch_bounds__(256) void k_tables(StaticDev S, long long T, const double* __restrict__ a,
                                                double* __restrict__ tA, double* __restrict__ tB, Header* zero_hdr) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx == 0 && zero_hdr) {                     // the following solve's header (saves a memset launch)
        zero_hdr->iters = 0;
        zero_hdr->error = 0;
        zero_hdr->nonzero = 0;
    }
    const long long total = T * S.dim * S.n;
    if (idx >= total) return;
    const int i = (int)(idx % S.n);
    const long long td = idx / S.n;
    const int d = (int)(td % S.dim);
    double A, B;
    table_entry<COP, MSM>(S, a, td, d, i, &A, &B);
    tA[idx] = A;
    tB[idx] = B;
}

// ---------------------------------------------------------------- node value
// Row context: everything about a node that depends only on its outer indices.
struct RowCtx {
    double z0, z1;      // outer-axis table values (z, or u for Plackett)
    double p0, p1, p2;  // outer part of y = z^T R^-1 (student.py:136 order)
    double B;           // product of outer B factors
    bool fin;           // all outer z finite (student.py:133)
};

template <int COP, bool MSM, int DIM>
__device__ __forceinline__ double node_value(const StaticDev& S, const RowCtx& r, double zc, double Bc,
                                             double W) {
    double c;
    if (COP == CVQ_PLACKETT) {
        const double u = r.z0, v = zc, th = S.theta;               // plackett.py:66-69 (Q11)
        const double num = th * (1.0 + (th - 1.0) * (u + v - 2.0 * u * v));
        double den = (1.0 + (th - 1.0) * (u + v)) * (1.0 + (th - 1.0) * (1.0 - u - v));
        den = den * den;
        c = (num / den) * (r.B * Bc);
    } else {
        double qf;
        // z^T R^-1 z in the order of student.py:136 (rounding differences ~1e-16)
        if (DIM == 2) {
            const double y0 = fma(zc, S.Ri[2], r.p0);
            const double y1 = fma(zc, S.Ri[3], r.p1);
            qf = fma(y1, zc, y0 * r.z0);
        } else {
            const double y0 = fma(zc, S.Ri[6], r.p0);
            const double y1 = fma(zc, S.Ri[7], r.p1);
            const double y2 = fma(zc, S.Ri[8], r.p2);
            qf = fma(y2, zc, fma(y1, r.z1, y0 * r.z0));
        }
        double mv;
        if (COP == CVQ_STUDENT) {
            const bool fin = r.fin && isfinite(zc);
            mv = fin ? S.term1 * pow_node(fma(qf, S.inv_nu, 1.0), S.node_m, S.node_ex) : 0.0;   // :133-141
        } else {
            mv = S.term1 * exp(-0.5 * qf);                         // gaussian.py:105-113
        }
        c = mv * (r.B * Bc);                                       // c / prod(uni) [* prod(pdf)]
    }
    if (MSM) return c * W;                                          // no NaN guard (Q15)
    return nan_to_num(c) * W;                                       // garch_integration_function.py:45-50
}

template <int COP, int DIM>
__device__ __forceinline__ RowCtx make_row(const StaticDev& S, double z0, double z1, double B) {
    RowCtx r;
    r.z0 = z0;
    r.z1 = z1;
    r.B = B;
    if (COP == CVQ_PLACKETT) {
        r.p0 = r.p1 = r.p2 = 0.0;
        r.fin = true;
    } else if (DIM == 2) {
        r.p0 = z0 * S.Ri[0];
        r.p1 = z0 * S.Ri[1];
        r.p2 = 0.0;
        r.fin = isfinite(z0);
    } else {
        r.p0 = z0 * S.Ri[0] + z1 * S.Ri[3];
        r.p1 = z0 * S.Ri[1] + z1 * S.Ri[4];
        r.p2 = z0 * S.Ri[2] + z1 * S.Ri[5];
        r.fin = isfinite(z0) && isfinite(z1);
    }
    return r;
}

// ------------------------------------------------------------------ k_mass
// PREFIX strategy: C[t][off[r] + j - 1] = sum_{j' <= j} node(t, r, j') for every
// reachable node (level <= v_cap) of date t.
//
// Mapping: one 64-lane wavefront per (date, group of 64 rows); lane = row.
// All lanes walk the inner (column) axis together, so every column-table
// operand is wave-uniform (scalar loads, SGPR operands) and each lane keeps its
// row's running prefix in a register -- no cross-lane scan.  Blocks of 16
// columns are transposed through LDS so the global stores are 4 rows x 128 B
// contiguous per instruction.
//
// W(node) = sum_l pi_t[l] Delta[node, l], Delta = prod_c F_c(combo_c, i_c)
// (create_grids.py:121,143; Q5 rotation baked into F; Q6: in 3-D the axis-0
// factor only where i1 == 0), contracted per row as G[b] and per column as F_inner(b, j).
template <int COP, bool MSM, int DIM, int QT>
__global__ __launch_bounds__(64) void k_mass(StaticDev S, const double* __restrict__ tA,
                                             const double* __restrict__ tB, const double* __restrict__ pi,
                                             double* __restrict__ C) {
    constexpr int CB = 16;                       // columns per transpose block
    constexpr int LD = CB + 1;                   // padded LDS row (conflict-free b64 access)
    __shared__ double tile[64 * LD];
    const int lane = threadIdx.x;
    const long long t = blockIdx.x;
    const int n = S.n, q = QT;
    const int r = blockIdx.y * 64 + lane;
    const bool live = r < S.nrows;
    const double* At = tA + t * S.dim * n;
    const double* Bt = tB + t * S.dim * n;
    const double* pit = pi + t * S.Q;
    const int inner = DIM - 1;
    const double* Ac = At + inner * n;           // inner-axis tables (wave-uniform reads)
    const double* Bc = Bt + inner * n;
    const double* Fc = S.F + (size_t)inner * q * n;

    const int rr_ = live ? r : 0;
    const int i0 = (DIM == 2) ? rr_ : rr_ / n;
    const int i1 = (DIM == 2) ? 0 : rr_ % n;

    // ---- row weights G[b] (outer axes contracted with pi_t)
    double G[QT];
    if (DIM == 2) {
#pragma unroll
        for (int b = 0; b < QT; ++b) {
            double g = 0.0;
#pragma unroll
            for (int a = 0; a < QT; ++a) g = fma(pit[a * q + b], S.F[(size_t)a * n + i0], g);
            G[b] = g;
        }
    } else {
        double f0[QT], f1[QT];
#pragma unroll
        for (int a = 0; a < QT; ++a) {
            f0[a] = (i1 == 0) ? S.F[(size_t)a * n + i0] : 1.0;     // Q6: axis-0 factor only at i1 == 0
            f1[a] = S.F[((size_t)q + a) * n + i1];
        }
#pragma unroll
        for (int c = 0; c < QT; ++c) {
            double g = 0.0;
#pragma unroll
            for (int b = 0; b < QT; ++b) {
                double h = 0.0;
#pragma unroll
                for (int a = 0; a < QT; ++a) h = fma(pit[(a * q + b) * q + c], f0[a], h);
                g = fma(h, f1[b], g);
            }
            G[c] = g;
        }
    }
    // ---- row context
    RowCtx ctx;
    if (DIM == 2) ctx = make_row<COP, DIM>(S, At[i0], 0.0, Bt[i0]);
    else ctx = make_row<COP, DIM>(S, At[i0], At[n + i1], Bt[i0] * Bt[n + i1]);   // prod over axes in order
    const int km = live ? S.kmax[r] : 0;
    const long long off = live ? S.off[r] : 0;
    int maxlen = km;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) maxlen = max(maxlen, __shfl_xor(maxlen, o, 64));
    double* Cd = C + t * S.G;

    double acc = 0.0;
    for (int jb = 1; jb <= maxlen; jb += CB) {
#pragma unroll
        for (int c = 0; c < CB; ++c) {
            const int j = jb + c;                 // wave-uniform
            if (j < n) {
                double W = 0.0;
#pragma unroll
                for (int b = 0; b < QT; ++b) W = fma(G[b], Fc[(size_t)b * n + j], W);
                const double v = node_value<COP, MSM, DIM>(S, ctx, Ac[j], Bc[j], W);
                if (j <= km) acc += v;
            }
            tile[lane * LD + c] = acc;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int rr = 0; rr < 64; rr += 4) {
            const int row = rr + (lane >> 4), col = lane & 15;
            const int krow = __shfl(km, row, 64);
            const long long orow = __shfl(off, row, 64);
            const int j = jb + col;
            if (j <= krow) Cd[orow + j - 1] = tile[row * LD + col];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// ------------------------------------------------------------------ solve
// Team of TPD threads per date; thread owns rows r = tid + i*TPD (i < RPT).
template <int TPD>
struct TeamReduce {
    // red: 2 * (TPD / 64) doubles; parity alternates the half used, so one
    // barrier per reduction suffices (a half is rewritten only after every wave
    // has passed the next reduction's barrier, i.e. finished reading it).
    __device__ static double sum(double v, double* red, int& parity) {
        v = wave_sum(v);
        if (TPD == 64) return v;
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
        double* r = red + parity * (TPD / 64);
        parity ^= 1;
        if (lane == 0) r[wave] = v;
        __syncthreads();
        double s = r[0];
#pragma unroll
        for (int w = 1; w < TPD / 64; ++w) s += r[w];
        return s;
    }
};

// count of inner nodes j in [1, kmax] with x_j <= g, searched in [klo, khi]
// (x_{klo} <= g is known true, or klo == 0).  create_grids.py:104-108.
__device__ __forceinline__ int count_le(const double* sx, double g, int klo, int khi) {
    int lo = klo, hi = khi;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sx[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ double row_level(const StaticDev& S, const double* sx, int r) {
    // np.sum(previous_points * weights[1:]) (integration_algo.py:20)
    if (S.dim == 2) return sx[r] * S.w1;
    const int i0 = r / S.n, i1 = r % S.n;
    return sx[i0] * S.w1 + sx[i1] * S.w2;
}

template <int TPD, int RPT>
struct SolveTeam {
    const StaticDev& S;
    const double* sx;
    const double* Cd;      // this date's prefix block
    double* red;
    int parity = 0;
    double s[RPT];
    int kmx[RPT];
    long long off[RPT];
    int nrows_here;

    __device__ SolveTeam(const StaticDev& S_, const double* sx_, const double* Cd_, double* red_)
        : S(S_), sx(sx_), Cd(Cd_), red(red_) {
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            const int r = threadIdx.x + i * TPD;
            if (r < S.nrows) {
                s[i] = row_level(S, sx, r);
                kmx[i] = S.kmax[r];
                off[i] = S.off[r];
            } else {
                s[i] = 0.0;
                kmx[i] = 0;
                off[i] = 0;
            }
        }
    }
    __device__ __forceinline__ int count(int i, double v, int klo, int khi) const {
        const double g = (v - s[i]) / S.w0;                     // var_function (Q10)
        return count_le(sx, g, klo, khi);
    }
    __device__ __forceinline__ double pref(int i, int k) const { return k > 0 ? Cd[off[i] + k - 1] : 0.0; }
    // Full slab (a, b] for this date.
    __device__ double slab(double a, double b) {
        double part = 0.0;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            if (kmx[i] == 0) continue;
            const int ka = count(i, a, 0, kmx[i]);
            const int kb = count(i, b, 0, kmx[i]);
            if (kb > ka) part += pref(i, kb) - pref(i, ka);
        }
        return TeamReduce<TPD>::sum(part, red, parity);
    }
};

// Steps (i)-(iii) of calc_var + K bisection iterations.  Writes snaps[t][0..K]
// (= (lo+hi)/2 after k updates) and folds iterations-needed / nonzero masks
// into the rank header.
template <int TPD, int RPT>
__global__ __launch_bounds__(TPD) void k_solve_prefix(StaticDev S, SolveConst P, const double* __restrict__ C,
                                                      double* __restrict__ snaps, Header* hdr) {
    __shared__ double sx[512];
    __shared__ double red[2 * (TPD / 64 > 0 ? TPD / 64 : 1)];
    for (int j = threadIdx.x; j < S.n; j += TPD) sx[j] = S.x[j];
    __syncthreads();
    const long long t = blockIdx.x;
    SolveTeam<TPD, RPT> tm(S, sx, C + t * S.G, red);

    // (i) r0 = I(lower, first_guess]                            calc_var_class.py:114-121
    const double r0 = tm.slab(P.lower, P.fg);
    // (ii) second bracket                                        :125-142
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;                          // Q1
    const double nr = tm.slab(nl, nu);
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;                           // adjust_integral
    // (iii) bracket classification                                :147-160 (Q3 -> NaN)
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    if (F > P.obj) { lo = P.vmin; hi = P.sg0; }
    if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; }
    if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; }
    if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; }
    bool ustack = !(hi == P.sg0 || hi == P.sg1);

    int kLo[RPT], kHi[RPT];
    double cLo[RPT], cHi[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        kLo[i] = tm.kmx[i] ? tm.count(i, lo, 0, tm.kmx[i]) : 0;
        kHi[i] = tm.kmx[i] ? tm.count(i, hi, kLo[i], tm.kmx[i]) : 0;
        cLo[i] = tm.pref(i, kLo[i]);
        cHi[i] = tm.pref(i, kHi[i]);
    }
    // (iv) bisection                                              :250-309
    double prev = F, prevU = prevU0;
    int nt = -1;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    for (int k = 0; k < P.K; ++k) {
        const double mid = (lo + hi) / 2;
        if (threadIdx.x == 0) sn[k] = mid;
        if (nt < 0 && !(hi - lo > P.tol)) nt = k;
        int kM[RPT];
        double cM[RPT];
        double part = 0.0;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            kM[i] = tm.kmx[i] ? tm.count(i, mid, kLo[i], kHi[i]) : 0;
            cM[i] = tm.pref(i, kM[i]);
            if (ustack) { if (kM[i] > kLo[i]) part += cM[i] - cLo[i]; }   // slab (lo, mid]
            else        { if (kHi[i] > kM[i]) part += cHi[i] - cM[i]; }   // slab (mid, hi]
        }
        const double val = TeamReduce<TPD>::sum(part, red, tm.parity);
        const double slab_lower = ustack ? lo : mid;
        const double Fn = (slab_lower == prevU) ? prev + val : prev - val;     // adjust_integral
        if (Fn != 0.0) mask |= (1ull << k);                                      // Q4
        ustack = Fn < P.obj;
        if (ustack) lo = mid; else hi = mid;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            if (ustack) { kLo[i] = kM[i]; cLo[i] = cM[i]; }
            else        { kHi[i] = kM[i]; cHi[i] = cM[i]; }
        }
        prev = Fn;
        prevU = mid;
    }
    if (threadIdx.x == 0) {
        sn[P.K] = (lo + hi) / 2;
        if (nt < 0 && !(hi - lo > P.tol)) nt = P.K;
        if (nt < 0) atomicOr(&hdr->error, 1);
        else atomicMax(&hdr->iters, nt);
        atomicOr((unsigned long long*)&hdr->nonzero, (unsigned long long)mask);
    }
}

// Drop-in compute_integral: out[t] = I_t(bounds[t][0], bounds[t][1]].
template <int TPD, int RPT>
__global__ __launch_bounds__(TPD) void k_slab_prefix(StaticDev S, const double* __restrict__ C,
                                                     const double* __restrict__ bounds, double* __restrict__ out) {
    __shared__ double sx[512];
    __shared__ double red[2 * (TPD / 64 > 0 ? TPD / 64 : 1)];
    for (int j = threadIdx.x; j < S.n; j += TPD) sx[j] = S.x[j];
    __syncthreads();
    const long long t = blockIdx.x;
    SolveTeam<TPD, RPT> tm(S, sx, C + t * S.G, red);
    const double v = tm.slab(bounds[2 * t], bounds[2 * t + 1]);
    if (threadIdx.x == 0) out[t] = v;
}

// Finalise: combine rank headers (Q2 global iteration count, Q4 global break)
// and pick each date's snapshot; var = mid + ptf_mean (calc_var_class.py:171).
#ifndef CVQ_NO_PLAN_KERNELS
__global__ void k_finalize(const Header* __restrict__ hdrs, int nranks, const double* __restrict__ snaps,
                           long long T_total, int stride, int K, double ptf_mean, double* __restrict__ var,
                           int* __restrict__ err) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int N = 0, e = 0;
    unsigned long long nz = 0;
    for (int r = 0; r < nranks; ++r) {
        N = max(N, hdrs[r].iters);
        e |= hdrs[r].error;
        nz |= hdrs[r].nonzero;
    }
    if (N > K) e |= 2;
    int kstop = min(N, K);
    for (int k = 0; k < kstop; ++k)
        if (!((nz >> k) & 1ull)) { kstop = k; break; }
    if (t == 0) { err[0] = e; err[1] = kstop; err[2] = N; }
    if (t >= T_total) return;
    var[t] = snaps[t * stride + kstop] + ptf_mean;
}

// Same, from ONE all-gathered buffer of per-rank blocks (cvq_solve_finalize_packed):
// block r = blocks + r * rstride holds the rank's [per][stride] snapshots, then its
// 16-B header at offset hoff (doubles, 16-B aligned).
__global__ void k_finalize_packed(const double* __restrict__ blocks, int nranks, long long per, long long rstride,
                                  long long hoff, long long T_total, int stride, int K, double ptf_mean,
                                  double* __restrict__ var, int* __restrict__ err) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    int N = 0, e = 0;
    unsigned long long nz = 0;
    for (int r = 0; r < nranks; ++r) {
        const Header* h = (const Header*)(blocks + r * rstride + hoff);
        N = max(N, h->iters);
        e |= h->error;
        nz |= h->nonzero;
    }
    if (N > K) e |= 2;
    int kstop = min(N, K);
    for (int k = 0; k < kstop; ++k)
        if (!((nz >> k) & 1ull)) { kstop = k; break; }
    if (t == 0) { err[0] = e; err[1] = kstop; err[2] = N; }
    if (t >= T_total) return;
    const long long r = t / per;
    var[t] = blocks[r * rstride + (t - r * per) * stride + kstop] + ptf_mean;
}
#endif

}  // namespace cvq
