// cvq_sorted_kernels.h -- SORTED strategy (2 or 3 assets): every slab of the
// bisection is a contiguous range of one date-independent list of nodes.
//
// Reference: calc_var + bisection_algorithm (utils/calc_var_class.py:95-177,
// :250-309) integrate 2 + K slabs (a, b] per date over the nested grid of
// create_grids.py:102-171.  A node (outer indices r, inner index j >= 1) lies in
// (a, b] iff x_j > max(g_r(a), -5) and x_j <= g_r(b), g_r(v) = (v - lev_r) / w0
// (Q9, Q10).  g_r is non-decreasing in v, so each node has an exact threshold
// v*(r, j) = the smallest double v with x_j <= g_r(v), and membership is
// a < v* <= b.  The plan sorts the reachable nodes (v* <= v_cap) by v* once:
// slab (a, b] = sorted positions [ub(a), ub(b)), ub(v) = #{v* <= v}.
//
// Every position the solve can ask for is date-independent: the fixed levels
// (lower, first / second guesses, min / max VaR) and the bisection mids, which
// form one binary tree per bracket ((lo + hi) / 2 from the bracket's ends).  The
// host tabulates ub() of the fixed levels and of the tree's mids down to the
// depth where every cell holds <= kSortTailCap nodes, so a level costs one
// table read, the slab's node evaluations spread evenly over the workgroup, and
// one reduction.  Beyond that depth the bracket's nodes go to LDS and one wave
// finishes the remaining levels with masked wave sums (COMPACT's tail).
//
// One NT-thread workgroup per date.  Node values (fast path, the date's pi is
// rank 1 -- the reference builds it as the product of per-asset forecasts,
// msm_estimation.py:392-418 -- and its tables are finite):
//   Gaussian  exp(E), E = g0 + g1 + g2 + cross terms of -z^T R^-1 z / 2, with the
//             per-axis log factors g_c = log(B_c w_c) - Ri_cc z_c^2 / 2 tabulated
//             in LDS (gaussian.py:105-113 divided by the margins, :56-59)
//   Student   S0 B'1 B'2 (1 + z^T R^-1 z / nu)^-(nu+d)/2   (student.py:133-141)
// and otherwise the reference-semantics node (node_value, full W contraction,
// garch_integration_function.py:45-50 nan_to_num).  3-D: the axis-0 weight
// factor survives only on the plane i1 == 0 (create_grids.py:169-171, Q6) and
// pi pairs combo (L0, L1, L2) with f0[L1] f1[L2] f2[L0] (msm_estimation.py:413, Q7).
#pragma once
#include "cvq_compact_kernels.h"

namespace cvq {

constexpr int kSortTailPerLane = 4;
constexpr int kSortTailCap = 64 * kSortTailPerLane;   // bracket size that switches to the one-wave tail
constexpr int kSortMaxDepth = 16;                     // deepest tabulated bisection level
constexpr int kSortIlp = 4;                           // nodes in flight per thread

// Date-independent device tables of a SORTED plan.
struct SortedGeom {
    const uint32_t* idx;   // [G] packed node indices, sorted by v* (2-D: i0 | j << 16; 3-D: i0 | i1 << 8 | i2 << 16)
    const double* vs;      // [G] the sorted v*
    const int* tree;       // [4][1 << depth]: ub(mid) of heap node h (1 <= h < 2^depth) of each bracket's tree
    int G;
    int depth;
    int fix[6];            // ub() of lower, sg0, fg, sg1, vmin, vmax
};

// exp(x): 2^k e^r, |r| <= ln2 / 2, degree-11 Taylor polynomial (relative error
// ~1e-15; the solve's decisions are unchanged by 1e-8 node noise).
// x < -800 underflows to 0, NaN stays NaN.
__device__ __forceinline__ double exp_node(double x) {
    x = x < -800.0 ? -800.0 : x;
    const double k = __builtin_rint(x * 1.4426950408889634);
    double r = fma(-k, 6.93147180369123816490e-01, x);      // ln2 hi (exact k * hi for |k| < 2^20)
    r = fma(-k, 1.90821492927058770002e-10, r);             // ln2 lo
    double p = 2.505210838544172e-08;                        // 1 / 11!
    p = fma(p, r, 2.755731922398589e-07);
    p = fma(p, r, 2.7557319223985893e-06);
    p = fma(p, r, 2.48015873015873e-05);
    p = fma(p, r, 0.0001984126984126984);
    p = fma(p, r, 0.001388888888888889);
    p = fma(p, r, 0.008333333333333333);
    p = fma(p, r, 0.041666666666666664);
    p = fma(p, r, 0.16666666666666666);
    p = fma(p, r, 0.5);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return __builtin_amdgcn_ldexp(p, (int)k);
}

// upper bound: first position p in [lo, hi) with vs[p] > v (hi if none); NaN v -> lo.
__device__ __forceinline__ int sorted_ub(const double* __restrict__ vs, int lo, int hi, double v) {
    if (!(v == v)) return lo;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (vs[m] <= v) lo = m + 1; else hi = m;
    }
    return lo;
}

template <int DIM>
__device__ __forceinline__ void unpack_node(uint32_t c, int* i0, int* i1, int* j) {
    if constexpr (DIM == 2) {
        *i0 = (int)(c & 0xFFFFu);
        *i1 = 0;
        *j = (int)(c >> 16);
    } else {
        *i0 = (int)(c & 0xFFu);
        *i1 = (int)((c >> 8) & 0xFFu);
        *j = (int)(c >> 16);
    }
}

// LDS doubles per grid point: generic z / B / w of 3 axes (9), fast records (8);
// arrays are laid out with an even stride so every double2 is 16-B aligned.
constexpr int kSortLdsPerPoint = 17;
inline int sorted_stride(int n) { return (n + 1) & ~1; }
inline size_t sorted_lds_bytes(int n, int nt) {
    return sizeof(double) * (size_t)kSortLdsPerPoint * sorted_stride(n) + sizeof(double2) * kSortTailCap +
           sizeof(double) * 6 * (nt / 64);
}

// mode 0: calc_var solve (snapshots + header, fused finalize when P.fin_var);
// mode 1: one slab per date (compute_integral): out[t] = I_t(bounds[2t], bounds[2t+1]].
template <int COP, bool MSM, int DIM, int NT, int PM, bool FUSED>
__global__ __launch_bounds__(NT) void k_sorted(StaticDev S, SolveConst P, SortedGeom G, const double* __restrict__ a,
                                               const double* __restrict__ tA, const double* __restrict__ tB,
                                               const double* __restrict__ pi, int mode,
                                               const double* __restrict__ bounds, double* __restrict__ out,
                                               double* __restrict__ snaps, Header* hdr) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int n = S.n, tid = threadIdx.x, lane = tid & 63;
    const int ns = (n + 1) & ~1;                   // sorted_stride(n)
    const long long t = blockIdx.x;
    // generic tables (reference semantics): z, B, w per axis (axis 0 of 3-D: w = the i1 == 0 weight)
    double* zg = lds;                              // [3][ns] (row ax at zg + ax * n, n <= ns)
    double* Bg = zg + 3 * ns;                      // [3][ns]
    double* wg = Bg + 3 * ns;                      // [3][ns]
    double* fr0 = wg + 3 * ns;                     // [ns][2] fast axis 0
    double* fd0 = fr0 + 2 * ns;                    // [ns]    fast axis 0, plane i1 == 0 (3-D)
    double* fr1 = fd0 + ns;                        // [ns][2] fast axis 1 (3-D)
    double* fg1 = fr1 + 2 * ns;                    // [ns]    fast axis 1, third value (3-D)
    double* fr2 = fg1 + ns;                        // [ns][2] fast inner axis
    double2* tail = (double2*)(fr2 + 2 * ns);      // [kSortTailCap] (v*, value)
    double* red = (double*)(tail + kSortTailCap);  // [2][3][NT / 64]
    __shared__ int flags;                          // bit 0: non-finite table entry, bit 1: pi not rank 1
    __shared__ double s_arest;                     // 3-D: the axis-0 weight off the plane i1 == 0

    if (tid == 0) flags = 0;
    __syncthreads();
    // ---- tables: grid index i of every axis (table_entry; W factors of the rank-1 pi)
    const int q = MSM ? S.q : 1;
    const double* fb = MSM ? a + t * DIM * q : nullptr;     // forecasts_by_states[t] (DIM, q)
    int bad = 0;
    for (int i = tid; i < n; i += NT) {
#pragma unroll
        for (int ax = 0; ax < DIM; ++ax) {
            double A, B;
            if constexpr (FUSED) {
                table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * DIM + ax, ax, i, &A, &B);
            } else {
                A = tA[(t * DIM + ax) * n + i];
                B = tB[(t * DIM + ax) * n + i];
            }
            // 2-D: pi[a][b] = f0[a] f1[b]; 3-D: pi[L0][L1][L2] = f0[L1] f1[L2] f2[L0] (Q7)
            const int fax = DIM == 2 ? ax : (ax + 2) % 3;
            double w;
            if constexpr (MSM) {
                w = 0.0;
                for (int s = 0; s < q; ++s) w = fma(fb[fax * q + s], S.F[((size_t)ax * q + s) * n + i], w);
            } else {
                w = S.F[(size_t)ax * n + i];
            }
            if (!isfinite(A) || !isfinite(B)) bad |= 1;
            zg[ax * n + i] = A;
            Bg[ax * n + i] = B;
            wg[ax * n + i] = w;
        }
    }
    const double* pit = pi + t * S.Q;
    if constexpr (MSM) {                                   // rank-1 check of pi_t, bitwise
        for (int l = tid; l < S.Q; l += NT) {
            double v;
            if constexpr (DIM == 2) v = fb[l / q] * fb[q + l % q];
            else v = (fb[(l / q) % q] * fb[q + l % q]) * fb[2 * q + l / (q * q)];
            if (!(pit[l] == v)) bad |= 2;
        }
    }
    if (DIM == 3 && tid == 0) {                            // sum over L0 of pi's axis-0 factor off the plane
        double s = 1.0;
        if constexpr (MSM) {
            s = 0.0;
            for (int L = 0; L < q; ++L) s += fb[2 * q + L];
        }
        s_arest = s;
    }
    if (bad) atomicOr(&flags, bad);
    __syncthreads();
    const int fl = flags;
    const bool rank1 = !(fl & 2);
    const bool fast = rank1 && !(fl & 1) && COP != CVQ_PLACKETT;
    const double arest = DIM == 3 ? s_arest : 1.0;
    if (fast) {                                            // fast records from the generic tables
        for (int i = tid; i < n; i += NT) {
            const double z0 = zg[i], zi = zg[(DIM - 1) * n + i];
            const double B0 = Bg[i], Bi = Bg[(DIM - 1) * n + i];
            const double w0 = wg[i], wi = wg[(DIM - 1) * n + i];
            if constexpr (COP == CVQ_GAUSSIAN) {
                const double s0 = DIM == 3 ? arest : w0;
                fr0[2 * i] = DIM == 2 ? -(S.Ri[1] + S.Ri[2]) * 0.5 * z0 : z0;
                fr0[2 * i + 1] = log(S.term1 * B0 * s0) - 0.5 * S.Ri[0] * (z0 * z0);
                fr2[2 * i] = zi;
                fr2[2 * i + 1] = log(Bi * wi) - 0.5 * S.Ri[DIM * DIM - 1] * (zi * zi);
                if constexpr (DIM == 3) {
                    const double z1 = zg[n + i];
                    fd0[i] = log(w0) - log(arest);
                    fr1[2 * i] = -(S.Ri[1] + S.Ri[3]) * 0.5 * z1;                    // c01 z1
                    fr1[2 * i + 1] = -(S.Ri[5] + S.Ri[7]) * 0.5 * z1;                // c12 z1
                    fg1[i] = log(Bg[n + i] * wg[n + i]) - 0.5 * S.Ri[4] * (z1 * z1);
                }
            } else {                                       // Student
                const double s0 = DIM == 3 ? arest : w0;
                fr0[2 * i] = z0;
                fr0[2 * i + 1] = S.term1 * B0 * s0;
                fr2[2 * i] = zi;
                fr2[2 * i + 1] = Bi * wi;
                if constexpr (DIM == 3) {
                    fd0[i] = w0 / arest;
                    fr1[2 * i] = zg[n + i];
                    fr1[2 * i + 1] = Bg[n + i] * wg[n + i];
                }
            }
        }
    }
    __syncthreads();

    // Gaussian cross coefficients (-z^T R^-1 z / 2), Student y = z^T R^-1 z / nu coefficients
    const double c02 = -(S.Ri[2] + S.Ri[6]) * 0.5;
    const double a00 = S.Ri[0] * S.inv_nu, a11 = S.Ri[DIM + 1] * S.inv_nu, a22 = S.Ri[DIM * DIM - 1] * S.inv_nu;
    const double a01 = (S.Ri[1] + S.Ri[DIM]) * S.inv_nu;
    const double a02 = DIM == 2 ? a01 : (S.Ri[2] + S.Ri[6]) * S.inv_nu;
    const double a12 = DIM == 3 ? (S.Ri[5] + S.Ri[7]) * S.inv_nu : 0.0;

    auto node_fast = [&](uint32_t c) -> double {
        int i0, i1, j;
        unpack_node<DIM>(c, &i0, &i1, &j);
        const double2 A = *(const double2*)(fr0 + 2 * i0);
        const double2 C = *(const double2*)(fr2 + 2 * j);
        if constexpr (COP == CVQ_GAUSSIAN) {
            if constexpr (DIM == 2) {
                return exp_node(fma(A.x, C.x, A.y + C.y));
            } else {
                const double2 Bv = *(const double2*)(fr1 + 2 * i1);
                double E = fma(A.x, fma(c02, C.x, Bv.x), fma(Bv.y, C.x, (A.y + fg1[i1]) + C.y));
                if (i1 == 0) E += fd0[i0];
                return exp_node(E);
            }
        } else {                                           // Student
            double y, sc;
            if constexpr (DIM == 2) {
                y = fma(A.x, fma(a00, A.x, a02 * C.x), a22 * (C.x * C.x));
                sc = A.y * C.y;
            } else {
                const double2 Bv = *(const double2*)(fr1 + 2 * i1);
                y = fma(A.x, fma(a00, A.x, fma(a01, Bv.x, a02 * C.x)), Bv.x * fma(a11, Bv.x, a12 * C.x));
                y = fma(a22, C.x * C.x, y);
                sc = (A.y * Bv.y) * C.y;
                if (i1 == 0) sc *= fd0[i0];
            }
            return sc * pow_node_t<PM>(1.0 + y, S.node_m, S.node_ex);
        }
    };
    auto node_generic = [&](uint32_t c) -> double {
        int i0, i1, j;
        unpack_node<DIM>(c, &i0, &i1, &j);
        const double zi = zg[(DIM - 1) * n + j], Bi = Bg[(DIM - 1) * n + j];
        double W;
        if (rank1) {
            if constexpr (DIM == 2) W = wg[i0] * wg[n + j];
            else W = ((i1 == 0 ? wg[i0] : arest) * wg[n + i1]) * wg[2 * n + j];
        } else if constexpr (DIM == 2) {                   // sum_ab pi[a][b] F0_a(i0) F1_b(j)
            W = 0.0;
            for (int b = 0; b < q; ++b) {
                double g = 0.0;
                for (int a2 = 0; a2 < q; ++a2) g = fma(pit[a2 * q + b], S.F[(size_t)a2 * n + i0], g);
                W = fma(g, S.F[((size_t)q + b) * n + j], W);
            }
        } else {                                           // sum_l pi[l] F0'(L0) F1(L1) F2(L2)   (k_mass order)
            W = 0.0;
            for (int L2 = 0; L2 < q; ++L2) {
                double g = 0.0;
                for (int L1 = 0; L1 < q; ++L1) {
                    double h = 0.0;
                    for (int L0 = 0; L0 < q; ++L0)
                        h = fma(pit[(L0 * q + L1) * q + L2], i1 == 0 ? S.F[(size_t)L0 * n + i0] : 1.0, h);
                    g = fma(h, S.F[((size_t)q + L1) * n + i1], g);
                }
                W = fma(g, S.F[((size_t)2 * q + L2) * n + j], W);
            }
        }
        RowCtx ctx;
        if constexpr (DIM == 2) ctx = make_row<COP, 2>(S, zg[i0], 0.0, Bg[i0]);
        else ctx = make_row<COP, 3>(S, zg[i0], zg[n + i1], Bg[i0] * Bg[n + i1]);
        return node_value<COP, MSM, DIM>(S, ctx, zi, Bi, W);
    };
    // sum of the nodes at sorted positions [p0, p1), strided over the workgroup
    auto range_sum = [&](int p0, int p1) -> double {
        double acc[kSortIlp];
#pragma unroll
        for (int u = 0; u < kSortIlp; ++u) acc[u] = 0.0;
        int p = p0 + tid;
        if (fast) {
            for (; p + (kSortIlp - 1) * NT < p1; p += kSortIlp * NT) {
                uint32_t c[kSortIlp];
#pragma unroll
                for (int u = 0; u < kSortIlp; ++u) c[u] = G.idx[p + u * NT];
#pragma unroll
                for (int u = 0; u < kSortIlp; ++u) acc[u] += node_fast(c[u]);
            }
            for (; p < p1; p += NT) acc[0] += node_fast(G.idx[p]);
        } else {
            for (; p < p1; p += NT) acc[0] += node_generic(G.idx[p]);
        }
        return (acc[0] + acc[1]) + (acc[2] + acc[3]);
    };
    int parity = 0;
    double sums[3];
    auto team_sum = [&](double v) {
        team_sum3<NT>(v, 0.0, 0.0, red, parity, sums);
        return sums[0];
    };

    if (mode == 1) {                                       // compute_integral of bounds[t]
        const int pa = sorted_ub(G.vs, 0, G.G, bounds[2 * t]);
        const int pb = sorted_ub(G.vs, 0, G.G, bounds[2 * t + 1]);
        const double v = team_sum(range_sum(pa, pb));
        if (tid == 0) out[t] = v;
        return;
    }

    auto fixpos = [&](double v) {
        return v == P.lower ? G.fix[0] : v == P.sg0 ? G.fix[1] : v == P.fg ? G.fix[2]
             : v == P.sg1 ? G.fix[3] : v == P.vmin ? G.fix[4] : G.fix[5];
    };
    // ---- (i)-(iii): calc_var_class.py:114-160 (Q1, Q3)
    const double r0 = team_sum(range_sum(G.fix[0], G.fix[2]));                 // (lower, fg]
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;
    const double nr = team_sum(range_sum(fixpos(nl), fixpos(nu)));
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    int br = -1;                                           // bracket (tree) index; -1: NaN bracket (Q3)
    if (F > P.obj) { lo = P.vmin; hi = P.sg0; br = 0; }
    if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; br = 1; }
    if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; br = 2; }
    if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; br = 3; }
    bool ustack = !(hi == P.sg0 || hi == P.sg1);
    int plo = br >= 0 ? fixpos(lo) : 0, phi = br >= 0 ? max(fixpos(hi), plo) : 0;
    int h = 1;                                             // heap index of (lo, hi) in the bracket's tree

    // ---- (iv) bisection (:250-309); Q2 / Q4 are resolved across dates by the finalize
    double prev = F, prevU = prevU0;
    int nt = -1, it = 0;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    for (; it < P.K && phi - plo > kSortTailCap; ++it) {
        const double mid = (lo + hi) / 2;
        if (tid == 0) sn[it] = mid;
        if (nt < 0 && !(hi - lo > P.tol)) nt = it;
        const bool tab = h < (1 << G.depth);               // tabulated; deeper: search (only if ties pile up)
        const int pm = tab ? G.tree[(br << G.depth) + h] : sorted_ub(G.vs, plo, phi, mid);
        const double val = team_sum(ustack ? range_sum(plo, pm) : range_sum(pm, phi));
        const double slab_lower = ustack ? lo : mid;
        const double Fn = (slab_lower == prevU) ? prev + val : prev - val;   // adjust_integral
        if (Fn != 0.0) mask |= (1ull << it);
        ustack = Fn < P.obj;
        if (ustack) { lo = mid; plo = pm; }
        else        { hi = mid; phi = pm; }
        if (tab) h = 2 * h + (ustack ? 1 : 0);             // children: (lo, mid) = 2h, (mid, hi) = 2h + 1
        prev = Fn;
        prevU = mid;
    }

    // ---- tail: the bracket's <= kSortTailCap nodes -> LDS, wave 0 finishes the levels
    if (it < P.K) {
        const int tot = phi - plo;
        for (int e = tid; e < tot; e += NT) {
            const uint32_t c = G.idx[plo + e];
            tail[e] = make_double2(G.vs[plo + e], fast ? node_fast(c) : node_generic(c));
        }
        __syncthreads();
        if (tid < 64) {
            double tx[kSortTailPerLane], ty[kSortTailPerLane];
#pragma unroll
            for (int m = 0; m < kSortTailPerLane; ++m) {
                const bool ok = lane + 64 * m < tot;
                const double2 e = ok ? tail[lane + 64 * m] : make_double2(__builtin_nan(""), 0.0);
                tx[m] = e.x;
                ty[m] = e.y;
            }
            for (; it < P.K; ++it) {
                const double mid = (lo + hi) / 2;
                if (tid == 0) sn[it] = mid;
                if (nt < 0 && !(hi - lo > P.tol)) nt = it;
                const double a0 = ustack ? lo : mid, b0 = ustack ? mid : hi;   // slab (a0, b0]
                double p = 0.0;
#pragma unroll
                for (int m = 0; m < kSortTailPerLane; ++m) p += (tx[m] > a0 && tx[m] <= b0) ? ty[m] : 0.0;
                const double val = wave_sum(p);
                const double slab_lower = ustack ? lo : mid;
                const double Fn = (slab_lower == prevU) ? prev + val : prev - val;
                if (Fn != 0.0) mask |= (1ull << it);
                ustack = Fn < P.obj;
                if (ustack) lo = mid; else hi = mid;
                prev = Fn;
                prevU = mid;
            }
        }
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
    fused_finalize<NT>(P, hdr, snaps, (long long)gridDim.x);
}

}  // namespace cvq
