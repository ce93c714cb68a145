// cvq_direct_kernels.h -- DIRECT strategy: one workgroup per date does it all.
//
// The reference (utils/calc_var_class.py:95-309) evaluates 2 + K slab integrals
// per date; each slab (a, b] is a set of contiguous inner-axis index ranges,
// one per outer row (create_grids.py:102-108).  Here one 256-thread workgroup
// per date
//   1. evaluates the date's marginal / quantile tables straight into LDS
//      (same code as k_tables),
//   2. walks calc_var's control flow (Q1-Q4) exactly as k_solve_prefix does,
//      but sums each slab's nodes on the fly instead of reading prefix sums:
//      thread = outer row, serial loop over that row's column range, node
//      operands from LDS, one workgroup reduction per slab.
// Nothing but the tables' inputs and the per-date snapshots touch HBM, so the
// kernel is bound by FP64 issue and LDS latency, not by memory.
#pragma once
#include "cvq_quad_kernels.h"

namespace cvq {

__device__ __forceinline__ double pow_node_fast(double b, int m, double ex) {
    // -(nu+d)/2 = -4 (nu=6, d=2) and -4.5 (nu=6, d=3) are the common cases
    if (m == 8) { const double b2 = b * b; const double r = b2 * b2; return r < 1e300 ? fast_rcp(r) : 0.0; }
    if (m == 9) { const double b2 = b * b; const double r = b2 * b2 * sqrt(b); return r < 1e300 ? fast_rcp(r) : 0.0; }
    return pow_node(b, m, ex);
}

template <int COP, bool MSM, int DIM>
__device__ __forceinline__ double node_value_d(const StaticDev& S, const RowCtx& r, double zc, double Bc, double W) {
    if (COP != CVQ_STUDENT) return node_value<COP, MSM, DIM>(S, r, zc, Bc, W);
    const double y0 = fma(zc, S.Ri[2], r.p0);
    const double y1 = fma(zc, S.Ri[3], r.p1);
    const double qf = fma(y1, zc, y0 * r.z0);
    const bool fin = r.fin && isfinite(zc);
    const double mv = fin ? S.term1 * pow_node_fast(fma(qf, S.inv_nu, 1.0), S.node_m, S.node_ex) : 0.0;
    const double c = mv * (r.B * Bc);
    if (MSM) return c * W;
    return nan_to_num(c) * W;
}

// mode 0: calc_var solve (snapshots + header);  mode 1: one slab per date (compute_integral)
template <int COP, bool MSM, int QT, int RPT>
__global__ __launch_bounds__(256) void k_direct2(StaticDev S, SolveConst P, const double* __restrict__ a,
                                                 const double* __restrict__ pi, int mode,
                                                 const double* __restrict__ bounds, double* __restrict__ out,
                                                 double* __restrict__ snaps, Header* hdr) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int n = S.n, tid = threadIdx.x;
    const long long t = blockIdx.x;
    double* sx = lds;
    double* cA = sx + n;
    double* cB = cA + n;
    double* cF = cB + n;              // [QT][n] inner-axis Delta factors
    double* rA = cF + QT * n;
    double* rB = rA + n;
    double* red = rB + n;             // [4]

    // 1. this date's tables (axis 0 -> rows, axis 1 -> columns)
    for (int e = tid; e < 2 * n; e += 256) {
        const int d = e / n, i = e - d * n;
        double A, B;
        table_entry<COP, MSM>(S, a, t * S.dim + d, d, i, &A, &B);
        if (d == 0) { rA[i] = A; rB[i] = B; } else { cA[i] = A; cB[i] = B; }
    }
    for (int i = tid; i < n; i += 256) {
        sx[i] = S.x[i];
#pragma unroll
        for (int b = 0; b < QT; ++b) cF[b * n + i] = S.F[((size_t)QT + b) * n + i];
    }
    __syncthreads();

    // 2. row contexts (row = outer index i0 = tid + 256 k)
    const double* pit = pi + t * S.Q;
    RowCtx ctx[RPT];
    double G[RPT][QT];
    double lev[RPT];
    bool has[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = tid + 256 * k;
        has[k] = r < n;
        const int i0 = has[k] ? r : 0;
        ctx[k] = make_row<COP, 2>(S, rA[i0], 0.0, rB[i0]);
#pragma unroll
        for (int b = 0; b < QT; ++b) {
            double g = 0.0;
#pragma unroll
            for (int a2 = 0; a2 < QT; ++a2) g = fma(pit[a2 * QT + b], S.F[(size_t)a2 * n + i0], g);
            G[k][b] = g;
        }
        lev[k] = sx[i0] * S.w1;                       // integration_algo.py:20 (2-D)
    }
    auto cnt = [&](int k, double v, int klo, int khi) {
        const double g = (v - lev[k]) / S.w0;         // var_function (Q10), exact FP64
        return count_le(sx, g, klo, khi);
    };
    auto rowsum = [&](int k, int k0, int k1) {
        double s = 0.0;
        for (int j = k0 + 1; j <= k1; ++j) {
            double W = 0.0;
#pragma unroll
            for (int b = 0; b < QT; ++b) W = fma(G[k][b], cF[b * n + j], W);
            s += node_value_d<COP, MSM, 2>(S, ctx[k], cA[j], cB[j], W);
        }
        return s;
    };
    auto slab = [&](double lo_v, double hi_v) {
        double part = 0.0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (!has[k]) continue;
            const int ka = cnt(k, lo_v, 0, n - 1);
            const int kb = cnt(k, hi_v, ka, n - 1);
            if (kb > ka) part += rowsum(k, ka, kb);
        }
        return TeamReduce<256>::sum(part, red);
    };

    if (mode == 1) {
        const double v = slab(bounds[2 * t], bounds[2 * t + 1]);
        if (tid == 0) out[t] = v;
        return;
    }
    // (i)-(iii): calc_var_class.py:114-160 (Q1, Q3)
    const double r0 = slab(P.lower, P.fg);
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;
    const double nr = slab(nl, nu);
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    if (F > P.obj) { lo = P.vmin; hi = P.sg0; }
    if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; }
    if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; }
    if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; }
    bool ustack = !(hi == P.sg0 || hi == P.sg1);
    int kLo[RPT], kHi[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        kLo[k] = has[k] ? cnt(k, lo, 0, n - 1) : 0;
        kHi[k] = has[k] ? cnt(k, hi, kLo[k], n - 1) : 0;
    }
    // (iv) bisection (:250-309), Q2 / Q4 resolved across dates by k_finalize
    double prev = F, prevU = prevU0;
    int nt = -1;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    for (int it = 0; it < P.K; ++it) {
        const double mid = (lo + hi) / 2;
        if (tid == 0) sn[it] = mid;
        if (nt < 0 && !(hi - lo > P.tol)) nt = it;
        int kM[RPT];
        double part = 0.0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            kM[k] = has[k] ? cnt(k, mid, kLo[k], kHi[k]) : 0;
            if (ustack) { if (kM[k] > kLo[k]) part += rowsum(k, kLo[k], kM[k]); }   // (lo, mid]
            else        { if (kHi[k] > kM[k]) part += rowsum(k, kM[k], kHi[k]); }   // (mid, hi]
        }
        const double val = TeamReduce<256>::sum(part, red);
        const double slab_lower = ustack ? lo : mid;
        const double Fn = (slab_lower == prevU) ? prev + val : prev - val;       // adjust_integral
        if (Fn != 0.0) mask |= (1ull << it);
        ustack = Fn < P.obj;
        if (ustack) lo = mid; else hi = mid;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (ustack) kLo[k] = kM[k]; else kHi[k] = kM[k];
        }
        prev = Fn;
        prevU = mid;
    }
    if (tid == 0) {
        sn[P.K] = (lo + hi) / 2;
        if (nt < 0 && !(hi - lo > P.tol)) nt = P.K;
        if (nt < 0) atomicOr(&hdr->error, 1);
        else atomicMax(&hdr->iters, nt);
        atomicOr((unsigned long long*)&hdr->nonzero, (unsigned long long)mask);
    }
}

}  // namespace cvq
