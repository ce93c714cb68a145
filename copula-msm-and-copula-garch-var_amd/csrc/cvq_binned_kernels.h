// cvq_binned_kernels.h -- BINNED strategy: every node of a date evaluated once,
// the bisection resolved from bin sums four levels at a time.
//
// Reference: calc_var + bisection_algorithm (utils/calc_var_class.py:95-177,
// :250-309) call compute_integral on 2 + K slabs (a, b] per date; a slab is, per
// outer row r, the contiguous inner-index range (cnt_r(a), cnt_r(b)] with
// cnt_r(v) = #{x_j <= (v - x_r w1) / w0} (create_grids.py:102-108, Q9/Q10).
// Every slab the reference can issue is a union of "bins" whose edges are known
// before the solve starts:
//   * (lower, sg0], (sg0, fg], (fg, sg1] -- steps (i)/(ii) (:114-142);
//   * the 16 leaves of the depth-4 bisection tree of each bracket (:147-160):
//     the tree's midpoints are the (lo + hi) / 2 the reference will compute,
//     whichever way its comparisons go (:279-305).
// So one pass over the date's reachable nodes (key <= vmax) fills 19 bin sums,
// from which r0, the second slab, the bracket and (for the (sg1, vmax] bracket,
// 91% of cfg-2 dates) four bisection levels follow with no further node work.
// Later levels repeat this on the chosen 1/16 of the bracket (a "block"):
// 16 bins whose edges are the next four levels' midpoints.  Each node is thus
// evaluated once per block that contains it -- the same node count as the
// slab-by-slab walk of k_direct -- but with one workgroup reduction per four
// levels instead of one per level, and no binary searches in pass 1 (the
// pass-1 and bracket cut columns are date-independent: host tables).
//
// W factorisation.  The MSM weight of node (r, j) is sum_l pi_l Delta_l =
// sum_{a,b} pi[a][b] F0_a(r) F1_b(j) (msm_integration_function.py:45,
// create_grids.py:121,143 with Q5's rotation in F).  The reference's pi is the
// outer product of the per-asset forecasts (compute_forecast_combinations,
// msm_estimation.py:392-418), so W = wr(r) * wc(j) with wr = sum_a p_a F0_a(r),
// wc = sum_b q_b F1_b(j).  Each workgroup checks pi[a q + b] == p_a * q_b bitwise;
// otherwise it uses the general rank-Q contraction.  GARCH/UKF: Q = 1, pi = 1.
//
// Fast node.  With finite tables (always for MSM, whose reference path has no
// NaN guard and propagates NaN the same way; Plackett's u is always finite), a
// node is scale_r * f(row consts, z_j) * B'_j with B'_j = B_j wc(j):
//   Student  f = (R_r + z (P_r + C z))^-(nu+2)/2   (student.py:133-141; 7 FP64 + rcp for nu = 6)
//   Gaussian f = exp(-(R_r + z (P_r + Ri11 z)) / 2) (gaussian.py:105-113)
//   Plackett f = (N_r + M_r v) / ((D_r + a1 v)(E_r - a1 v))^2   (plackett.py:66-69, Q11)
// GARCH/UKF dates with a non-finite table entry (u in {0, 1}) take the generic
// per-node path with node_value's nan_to_num (garch_integration_function.py:45-50).
//
// Mapping: one 256-thread workgroup per date, thread = outer row (rows of a wave
// are consecutive, so their bin ranges differ by about one column: the per-bin
// loops stay converged); the row block of each wave is rotated by date so the
// long rows of the triangle do not all land on the same SIMD.
#pragma once
#include <utility>

#include "cvq_direct_kernels.h"

namespace cvq {

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>): guaranteed unrolling
// (bin accumulators must stay statically indexed registers).
template <class F, int... Es>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, Es...>) {
    (f(std::integral_constant<int, Es>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

constexpr int kBinLevels = 4;                 // bisection levels per block
constexpr int kBins = 1 << kBinLevels;        // 16 leaves
constexpr int kE1 = 3 + kBins;                // pass-1 bins
constexpr int kRedW = 32;                     // reduction slots per wave
// interior tree edges in the order the bisection creates them (parents first)
constexpr int kTreeOrder[kBins - 1] = {8, 4, 12, 2, 6, 10, 14, 1, 3, 5, 7, 9, 11, 13, 15};

// Host-built, date-independent cut columns for one (plan, solve arguments).
struct BinGeom {
    const int16_t* cut1;      // [n][kE1 + 1]: edges lower, sg0, fg, sg1, 15 tree mids of (sg1, vmax], vmax
    const int16_t* cutB;      // [3][n][kBins + 1]: tree edges of (vmin, sg0], (sg0, fg], (fg, sg1]
};

// Full-wave sum landing in lane 63 (row reductions, then row_bcast15/31); fixed
// order, so every workgroup thread that recombines the partials agrees bitwise.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_f64_rows(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWMASK, 0xF, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_total63(double v) {
    v += dpp_f64<0xB1>(v);            // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);            // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);           // row_half_mirror
    v += dpp_f64<0x140>(v);           // row_mirror: every lane holds its row's sum
    v += dpp_f64_rows<0x142, 0xA>(v); // row_bcast:15 -> rows 1, 3
    v += dpp_f64_rows<0x143, 0xC>(v); // row_bcast:31 -> rows 2, 3
    return v;                          // lane 63: the wave's total
}

// Workgroup sums of NB per-thread values -> tot[0..NB) in LDS (two barriers).
template <int NB>
__device__ __forceinline__ void team_sums(const double (&v)[NB], double* red, double* tot) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double s = wave_total63(v[b]);
        if (lane == 63) red[wave * kRedW + b] = s;
    }
    __syncthreads();
    if (threadIdx.x < NB) {
        const int b = threadIdx.x;
        tot[b] = (red[b] + red[kRedW + b]) + (red[2 * kRedW + b] + red[3 * kRedW + b]);
    }
    __syncthreads();
}

// Fast-path row constants (see header) and node kernel f(row, z_j).
struct FastRow {
    double c0, c1, c2, c3;
    double scale;
};

template <int COP>
__device__ __forceinline__ FastRow fast_row(const StaticDev& S, double z0, double B0, double wr) {
    FastRow f;
    if constexpr (COP == CVQ_STUDENT) {
        f.c0 = fma(S.Ri[0] * S.inv_nu, z0 * z0, 1.0);
        f.c1 = (S.Ri[1] + S.Ri[2]) * S.inv_nu * z0;
        f.c2 = f.c3 = 0.0;
        f.scale = S.term1 * B0 * wr;
    } else if constexpr (COP == CVQ_GAUSSIAN) {
        f.c0 = S.Ri[0] * (z0 * z0);
        f.c1 = (S.Ri[1] + S.Ri[2]) * z0;
        f.c2 = f.c3 = 0.0;
        f.scale = S.term1 * B0 * wr;
    } else {
        const double th = S.theta, a1 = th - 1.0, u = z0;
        f.c0 = th * fma(a1, u, 1.0);                   // num = c0 + c1 v
        f.c1 = th * a1 * fma(-2.0, u, 1.0);
        f.c2 = fma(a1, u, 1.0);                        // d1 = c2 + a1 v
        f.c3 = fma(a1, 1.0 - u, 1.0);                  // d2 = c3 - a1 v
        f.scale = B0 * wr;
    }
    return f;
}

template <int COP, int PM>
__device__ __forceinline__ double fast_node(const StaticDev& S, const FastRow& f, double zc) {
    if constexpr (COP == CVQ_STUDENT) {
        const double b = fma(zc, fma(zc, S.Ri[3] * S.inv_nu, f.c1), f.c0);
        if constexpr (PM == 8) {
            double y = __builtin_amdgcn_rcp(b);
            y = fma(y, fma(-b, y, 1.0), y);
            const double y2 = y * y;
            return y2 * y2;
        } else {
            return pow_node_t<PM>(b, S.node_m, S.node_ex);
        }
    } else if constexpr (COP == CVQ_GAUSSIAN) {
        const double qf = fma(zc, fma(zc, S.Ri[3], f.c1), f.c0);
        return exp(-0.5 * qf);
    } else {
        const double a1 = S.theta - 1.0;
        const double num = fma(f.c1, zc, f.c0);
        const double d = fma(a1, zc, f.c2) * fma(-a1, zc, f.c3);
        const double den = d * d;
        double y = __builtin_amdgcn_rcp(den);
        y = fma(y, fma(-den, y, 1.0), y);
        y = fma(y, fma(-den, y, 1.0), y);
        return num * y;
    }
}

// mode 0: calc_var solve (snapshots + header, fused finalize when P.fin_var).
template <int COP, bool MSM, int RPT, int PM>
__global__ __launch_bounds__(256, 4) void k_binned(StaticDev S, SolveConst P, BinGeom BG, const double* __restrict__ a,
                                                   const double* __restrict__ pi, double* __restrict__ stamps_out,
                                                   double* __restrict__ snaps, Header* hdr) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int NT = 256;
    const int n = S.n, tid = threadIdx.x, lane = tid & 63;
    const long long t = blockIdx.x;
    double* col = lds;                       // [n][4]: z_j, B'_j = B_j wc_j, B_j, wc_j
    double* sx = col + 4 * n;                // [n]
    double* red = sx + n;                    // [4][kRedW]
    double* tot = red + 4 * kRedW;           // [kRedW]
    int16_t* c1s = (int16_t*)(tot + kRedW);  // [256 * RPT][kE1 + 1]: this workgroup's threads' pass-1 cuts
    __shared__ int flags;                    // bit 0: non-finite table entry, bit 1: pi not rank 1

    unsigned long long* stamps = stamps_out ? (unsigned long long*)stamps_out + t * 32 : nullptr;
    auto stamp = [&](int idx) {              // diagnostic only (never in a timed run)
        if (stamps && tid == 0 && idx < 32) stamps[idx] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    // rows of this thread: wave block rotated by date (see header)
    const int wb = ((tid >> 6) + (int)(t & 3)) & 3;
    int row[RPT];
    bool has[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        row[k] = wb * 64 + lane + 256 * k;
        has[k] = row[k] < n;
    }
    // this thread's pass-1 cut columns (date independent, L2-resident) -> LDS
    auto c1 = [&](int k, int e) -> int { return c1s[(k * NT + tid) * (kE1 + 1) + e]; };
    {
        const int* src = (const int*)BG.cut1;                    // rows of kE1 + 1 = 20 int16
        int* dst = (int*)c1s;
        for (int w = tid; w < RPT * NT * (kE1 + 1) / 2; w += NT) {
            const int slot = w / ((kE1 + 1) / 2), k = slot / NT, th = slot % NT;
            const int r = (((th >> 6) + (int)(t & 3)) & 3) * 64 + (th & 63) + 256 * k;
            dst[w] = r < n ? src[(size_t)r * ((kE1 + 1) / 2) + w % ((kE1 + 1) / 2)] : 0;
        }
    }
    if (tid == 0) flags = 0;
    __syncthreads();

    // ---- tables: axis 1 -> LDS column records, axis 0 -> this thread's rows
    const int q = MSM ? S.q : 1;
    const double* fb = MSM ? a + t * 2 * q : nullptr;          // forecasts_by_states[t] (2, q)
    int bad = 0;
    for (int i = tid; i < n; i += NT) {
        sx[i] = S.x[i];
        double A, B;
        table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * 2 + 1, 1, i, &A, &B);
        double wc;
        if constexpr (MSM) {
            wc = 0.0;
            for (int b = 0; b < q; ++b) wc = fma(fb[q + b], S.F[((size_t)q + b) * n + i], wc);
        } else {
            wc = S.F[n + i];
        }
        double* c = col + 4 * i;
        c[0] = A;
        c[1] = B * wc;
        c[2] = B;
        c[3] = wc;
        if (!isfinite(A) || !isfinite(B)) bad |= 1;
    }
    if constexpr (MSM) {                                         // rank-1 check of pi_t
        const double* pit = pi + t * S.Q;
        for (int l = tid; l < S.Q; l += NT)
            if (!(pit[l] == fb[l / q] * fb[q + l % q])) bad |= 2;
    }
    double z0[RPT], B0[RPT], wr[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int rr = has[k] ? row[k] : 0;
        table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * 2, 0, rr, &z0[k], &B0[k]);
        if constexpr (MSM) {
            double g = 0.0;
            for (int b = 0; b < q; ++b) g = fma(fb[b], S.F[(size_t)b * n + rr], g);
            wr[k] = g;
        } else {
            wr[k] = S.F[rr];
        }
        if (has[k] && (!isfinite(z0[k]) || !isfinite(B0[k]))) bad |= 1;
    }
    if (bad) atomicOr(&flags, bad);
    __syncthreads();
    stamp(1);
    const int fl = flags;
    // fast folded path: rank-1 W and (MSM / Plackett: any tables; GARCH/UKF: finite tables)
    const bool fast = !(fl & 2) && (MSM || COP == CVQ_PLACKETT || !(fl & 1));

    FastRow fr[RPT];
    double lev[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        fr[k] = fast_row<COP>(S, z0[k], B0[k], wr[k]);
        lev[k] = S.x[has[k] ? row[k] : 0] * S.w1;                  // integration_algo.py:20 (2-D)
    }

    // ---- node sums over the columns (j0, j1] of row k
    auto sum_fast = [&](int k, int j0, int j1) {
        double s0 = 0.0, s1 = 0.0;
        int j = j0 + 1;
        for (; j + 1 <= j1; j += 2) {
            const double2 ca = *(const double2*)(col + 4 * j);
            const double2 cb = *(const double2*)(col + 4 * (j + 1));
            s0 = fma(fast_node<COP, PM>(S, fr[k], ca.x), ca.y, s0);
            s1 = fma(fast_node<COP, PM>(S, fr[k], cb.x), cb.y, s1);
        }
        if (j <= j1) {
            const double2 ca = *(const double2*)(col + 4 * j);
            s0 = fma(fast_node<COP, PM>(S, fr[k], ca.x), ca.y, s0);
        }
        return s0 + s1;
    };
    // generic path: per-node reference semantics (node_value), rank-1 or rank-Q W
    auto sum_generic = [&](int k, int j0, int j1, const RowCtx& ctx) {
        double s = 0.0;
        for (int j = j0 + 1; j <= j1; ++j) {
            const double* c = col + 4 * j;
            double W;
            if (!(fl & 2)) {
                W = wr[k] * c[3];
            } else {                                    // sum_ab pi[a][b] F0_a(r) F1_b(j)
                const double* pit = pi + t * S.Q;
                W = 0.0;
                for (int b = 0; b < q; ++b) {
                    double g = 0.0;
                    for (int a2 = 0; a2 < q; ++a2) g = fma(pit[a2 * q + b], S.F[(size_t)a2 * n + row[k]], g);
                    W = fma(g, S.F[((size_t)q + b) * n + j], W);
                }
            }
            s += node_value<COP, MSM, 2>(S, ctx, c[0], c[2], W);
        }
        return s;
    };
    // NB bins of this thread's rows, bin e = columns (cut(k, e), cut(k, e + 1)]
    auto eval_bins = [&](auto nbc, auto&& cut, double* part) {
        constexpr int NB = decltype(nbc)::value;
        static_for<NB>([&](auto e) { part[e] = 0.0; });
        static_for<RPT>([&](auto k) {
            if (!has[k] || cut(k, NB) <= cut(k, 0)) return;
            if (fast) {
                static_for<NB>([&](auto e) {
                    const int j0 = cut(k, e), j1 = cut(k, e + 1);
                    if (j1 > j0) part[e] = fma(fr[k].scale, sum_fast(k, j0, j1), part[e]);
                });
            } else {                                       // rare: one code copy, select-add
                const RowCtx ctx = make_row<COP, 2>(S, z0[k], 0.0, B0[k]);
                for (int e = 0; e < NB; ++e) {
                    const int j0 = cut(k, e), j1 = cut(k, e + 1);
                    const double v = (j1 > j0) ? sum_generic(k, j0, j1, ctx) : 0.0;
                    static_for<NB>([&](auto ee) {
                        if (ee == e) part[ee] += v;
                    });
                }
            }
        });
    };

    // ---- pass 1: every node with key in (lower, vmax]
    double p1[kE1];
    eval_bins(std::integral_constant<int, kE1>{}, c1, p1);
    stamp(2);
    team_sums<kE1>(p1, red, tot);
    stamp(3);

    // ---- (i)-(iii): calc_var_class.py:114-160 (Q1, Q3) from the pass-1 bins
    const double r0 = tot[0] + tot[1];                          // I(lower, fg]
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;
    const double nr = (nl == P.sg0 && nu == P.fg) ? tot[1] : (nl == P.fg && nu == P.sg1) ? tot[2] : 0.0;
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    if (F > P.obj) { lo = P.vmin; hi = P.sg0; }
    if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; }
    if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; }
    if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; }
    bool ustack = !(hi == P.sg0 || hi == P.sg1);

    // (iv) bisection (:250-309); Q2 / Q4 are resolved across dates by the finalize
    double prev = F, prevU = prevU0;
    int nt = -1, it = 0;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    // up to four levels from 16 bins tot[b0 .. b0 + 16); returns the chosen bin
    auto levels = [&](int b0, bool zero) {
        int base = 0, w = kBins;
        const int nlev = min(kBinLevels, P.K - it);
        for (int l = 0; l < nlev; ++l) {
            const double mid = (lo + hi) / 2;
            if (tid == 0) sn[it] = mid;
            if (nt < 0 && !(hi - lo > P.tol)) nt = it;
            const int h = w >> 1;
            const int s0 = b0 + (ustack ? base : base + h);
            double val = 0.0;
            if (!zero)
                for (int e = 0; e < h; ++e) val += tot[s0 + e];
            const double slab_lower = ustack ? lo : mid;
            const double Fn = (slab_lower == prevU) ? prev + val : prev - val;   // adjust_integral
            if (Fn != 0.0) mask |= (1ull << it);
            ustack = Fn < P.obj;
            if (ustack) { lo = mid; base += h; } else { hi = mid; }
            w = h;
            prev = Fn;
            prevU = mid;
            ++it;
        }
        return base;
    };

    int kLo[RPT], kHi[RPT];
    bool empty = !(lo == lo);                                    // Q3 bracket: every later slab is empty
    if (!empty) {
        int cb[RPT][kBins + 1];
        int b0 = 3;                                              // (sg1, vmax]: pass-1 bins 3..18
        int which = -1;
        if (lo == P.vmin && hi == P.sg0) which = 0;
        else if (lo == P.sg0 && hi == P.fg) which = 1;
        else if (lo == P.fg && hi == P.sg1) which = 2;
        if (which >= 0) {                                        // static block over the bracket
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                const int16_t* cr = BG.cutB + ((size_t)which * n + (has[k] ? row[k] : 0)) * (kBins + 1);
#pragma unroll
                for (int e = 0; e <= kBins; ++e) cb[k][e] = has[k] ? (int)cr[e] : 0;
            }
            double pb[kBins];
            eval_bins(std::integral_constant<int, kBins>{}, [&](int k, int e) { return cb[k][e]; }, pb);
            team_sums<kBins>(pb, red, tot);
            b0 = 0;
        }
        const int sel = levels(b0, false);
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            int l0 = 0, l1 = 0;
#pragma unroll
            for (int e = 0; e < kBins; ++e)
                if (e == sel) {
                    l0 = which >= 0 ? cb[k][e] : c1(k, 3 + e);
                    l1 = which >= 0 ? cb[k][e + 1] : c1(k, 4 + e);
                }
            kLo[k] = l0;
            kHi[k] = l1;
        }
    }
    stamp(4);
    // ---- dynamic blocks: the next four levels' midpoints cut the current bracket
    int blk = 0;
    while (it < P.K) {
        if (empty) { levels(0, true); continue; }
        double ed[kBins + 1];
        ed[0] = lo;
        ed[kBins] = hi;
        static_for<kBins - 1>([&](auto i) {                      // tree order: 8, 4, 12, 2, 6, ...
            constexpr int e = kTreeOrder[i], s = e & -e;
            ed[e] = (ed[e - s] + ed[e + s]) / 2;
        });
        int cd[RPT][kBins + 1];
        double pd[kBins + 1];
        static_for<RPT>([&](auto k) {
            cd[k][0] = kLo[k];
            cd[k][kBins] = kHi[k];
            const bool live = has[k] && kHi[k] > kLo[k];
            static_for<kBins - 1>([&](auto i) {                  // parents first: narrowed searches
                constexpr int e = kTreeOrder[i], s = e & -e;
                cd[k][e] = live ? count_le(sx, (ed[e] - lev[k]) / S.w0, cd[k][e - s], cd[k][e + s]) : kLo[k];
            });
        });
        eval_bins(std::integral_constant<int, kBins>{}, [&](int k, int e) { return cd[k][e]; }, pd);
        pd[kBins] = 0.0;
        static_for<RPT>([&](auto k) { pd[kBins] += has[k] ? (double)(kHi[k] - kLo[k]) : 0.0; });
        team_sums<kBins + 1>(pd, red, tot);
        empty = !(tot[kBins] > 0.0);
        const int sel = levels(0, empty);
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            int l0 = kLo[k], l1 = kHi[k];
#pragma unroll
            for (int e = 0; e < kBins; ++e)
                if (e == sel) { l0 = cd[k][e]; l1 = cd[k][e + 1]; }
            kLo[k] = l0;
            kHi[k] = l1;
        }
        stamp(5 + (blk++));
    }

    __shared__ int last;
    if (tid == 0) {
        sn[P.K] = (lo + hi) / 2;
        if (nt < 0 && !(hi - lo > P.tol)) nt = P.K;
        if (nt < 0) atomicOr(&hdr->error, 1);
        else atomicMax(&hdr->iters, nt);
        atomicOr((unsigned long long*)&hdr->nonzero, (unsigned long long)mask);
        if (P.fin_var) {
            __threadfence();                             // release: this date's snapshots + header bits
            last = atomicAdd(&P.fin_err[3], 1) == (int)gridDim.x - 1;
        }
    }
    if (!P.fin_var) return;
    __syncthreads();
    if (!last) return;
    // k_finalize for a single rank, run by the last workgroup (calc_var_class.py:278, :293, :171)
    __threadfence();                                     // acquire: every workgroup's stores
    const int N = __hip_atomic_load(&hdr->iters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int err = __hip_atomic_load(&hdr->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (N > P.K ? 2 : 0);
    const unsigned long long nz = __hip_atomic_load((unsigned long long*)&hdr->nonzero, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    int kstop = min(N, P.K);
    for (int k = 0; k < kstop; ++k)
        if (!((nz >> k) & 1ull)) { kstop = k; break; }
    for (long long d = tid; d < (long long)gridDim.x; d += NT)
        P.fin_var[d] = snaps[d * P.stride + kstop] + P.ptf_mean;
    __syncthreads();                                     // every thread has read the header
    if (tid == 0) {
        P.fin_err[0] = err;
        P.fin_err[1] = kstop;
        P.fin_err[2] = N;
        P.fin_err[3] = 0;                                // ticket reset for the next launch
        hdr->iters = 0;                                  // header reset for the next launch
        hdr->error = 0;
        hdr->nonzero = 0;
    }
}

}  // namespace cvq
