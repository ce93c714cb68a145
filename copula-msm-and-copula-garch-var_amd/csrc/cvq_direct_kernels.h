// cvq_direct_kernels.h -- DIRECT strategy: one workgroup per date does it all.
//
// The reference (utils/calc_var_class.py:95-309) evaluates 2 + K slab integrals
// per date; each slab (a, b] is a set of contiguous inner-axis index ranges,
// one per outer row (create_grids.py:102-108).  Here one 256-thread workgroup
// per date
//   1. stages the date's inner-axis tables (k_tables output) into LDS and its
//      outer-axis row constants into registers,
//   2. walks calc_var's control flow (Q1-Q4) exactly as k_solve_prefix does,
//      but sums each slab's nodes on the fly instead of reading prefix sums:
//      thread = outer row, serial loop over that row's column range, node
//      operands from LDS, one workgroup reduction per slab.
// Nothing but the tables' inputs and the per-date snapshots touch HBM, so the
// kernel is bound by FP64 issue and LDS latency, not by memory.
#pragma once
#include "cvq_quad_kernels.h"

namespace cvq {

// b^-(m/2) for b >= 1 with a compile-time m (PM > 0): squarings, hardware
// reciprocal + one Newton step (v_rcp_f64 seeds >= 26 bits, so the step gives
// ~1e-15 relative; the node tolerance is 1e-9); PM == 0: runtime m.
// b = inf or NaN -> 0, exactly as pow_node's overflow rule.
template <int PM>
__device__ __forceinline__ double pow_node_t(double b, int m, double ex) {
    if constexpr (PM == 0) {
        return pow_node(b, m, ex);
    } else {
        constexpr int k = PM >> 1;
        double r = 1.0, s = b;
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {
            if ((k >> bit) & 1) r *= s;
            if ((k >> (bit + 1)) == 0) break;
            s *= s;
        }
        if constexpr (PM & 1) r *= sqrt(b);
        double y = __builtin_amdgcn_rcp(r);
        y = fma(y, fma(-r, y, 1.0), y);
        return (r < 1.0e300) ? y : 0.0;
    }
}

// mode 0: calc_var solve (snapshots + header);  mode 1: one slab per date (compute_integral);
//
// Thread `slot` of the 256-thread block owns rows slot + 256 k (k < RPT) for the
// whole solve.  Row constants (outer table values, row weights G) live in
// registers; per node only the column operands come from LDS, and the lanes of
// a wave (consecutive rows) read near-consecutive columns along the slab's
// anti-diagonal edge, so the reads are conflict-free.  Two independent node
// chains per iteration give the FP64 pipe instruction-level parallelism.
#ifndef CVQ_DIRECT_ILP
#define CVQ_DIRECT_ILP 2
#endif
// FUSED: evaluate the date's tables here (table_entry; Student only with the
// plan's direct t.ppf tables); else read k_tables' output tA / tB [T][2][n].
template <int COP, bool MSM, int QT, int RPT, int PM, bool FUSED, int ILP = CVQ_DIRECT_ILP>
__global__ __launch_bounds__(256, 4) void k_direct(StaticDev S, SolveConst P, const double* __restrict__ a,
                                                        const double* __restrict__ tA, const double* __restrict__ tB,
                                                        const double* __restrict__ pi,
                                                        int mode, const double* __restrict__ bounds,
                                                        double* __restrict__ out, double* __restrict__ snaps,
                                                        Header* hdr) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int NT = 256;
    const long long t = blockIdx.x;
    const int n = S.n, tid = threadIdx.x, slot = tid;
    // Column records, one per inner index j, CS doubles each (16-B aligned):
    //   [0] z_j, [1..QT] F'_b[j], then B_j for the non-folded paths.
    // A lane's operands for a node are CS contiguous doubles (ds_read_b128 x CS/2);
    // lanes at consecutive j are CS*8 bytes apart, conflict-free for CS = 6.
    constexpr bool FOLD = (COP == CVQ_STUDENT) && MSM;
    constexpr int CS = ((1 + QT + (FOLD ? 0 : 1)) + 1) & ~1;
    double* col = lds;                // [n][CS]
    double* sx = col + CS * n;        // [n] grid
    double* red = sx + n;             // [2][NT / 64]
    int parity = 0;

    unsigned long long* stamps = (mode == 0 && out) ? (unsigned long long*)out + t * 32 : nullptr;
    auto stamp = [&](int idx) {                      // diagnostic only (never in a timed run)
        if (stamps && tid == 0) stamps[idx] = __builtin_amdgcn_s_memtime();
    };
    stamp(0);
    // Student + MSM folds every per-node factor that is constant along a row or a
    // column: node = b^-(nu+2)/2 * sum_b G'_b[r] F'_b[j] with F' = F * B_col and
    // G' = G * term1 * B_row, and b = 1 + q/nu = R_r + z_j (P_r + C z_j).  A non-
    // finite z makes b non-finite (pow -> 0) and its B infinite, so the node is
    // 0 * inf = NaN exactly where student.py's 0/0 gives NaN (Q15, no guard on MSM).
    // This date's marginal / quantile tables (k_tables' table_entry, evaluated
    // here): axis 1 -> LDS column records, axis 0 -> this thread's row constants.
    for (int i = tid; i < n; i += NT) {
        sx[i] = S.x[i];
        double* c = col + i * CS;
        double Ac, Bc;
        if constexpr (FUSED) {
            table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * 2 + 1, 1, i, &Ac, &Bc);
        } else {
            Ac = tA[(t * 2 + 1) * n + i];
            Bc = tB[(t * 2 + 1) * n + i];
        }
        c[0] = Ac;
#pragma unroll
        for (int b = 0; b < QT; ++b) {
            const double f = S.F[((size_t)QT + b) * n + i];
            c[1 + b] = FOLD ? f * Bc : f;
        }
        if constexpr (!FOLD) c[1 + QT] = Bc;
    }
    // this thread's rows: context + row weights G[b] = sum_a pi[a][b] F0[a][r]
    const double* pit = pi + t * S.Q;
    RowCtx ctx[RPT];
    double G[RPT][QT];
    double lev[RPT], Rr[RPT], Pr[RPT], Kr[RPT];
    bool has[RPT];
    const double Cq = S.Ri[3] * S.inv_nu;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int r = slot + 256 * k;
        has[k] = r < n;
        const int rr = has[k] ? r : 0;
        double Ar, Br;
        if constexpr (FUSED) {
            table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * 2, 0, rr, &Ar, &Br);
        } else {
            Ar = tA[t * 2 * n + rr];
            Br = tB[t * 2 * n + rr];
        }
        ctx[k] = make_row<COP, 2>(S, Ar, 0.0, Br);
        lev[k] = S.x[rr] * S.w1;                      // integration_algo.py:20 (2-D)
        const double z0 = ctx[k].z0;
        Rr[k] = fma(S.Ri[0] * S.inv_nu, z0 * z0, 1.0);
        Pr[k] = (S.Ri[1] + S.Ri[2]) * S.inv_nu * z0;
        Kr[k] = S.term1 * ctx[k].B;
#pragma unroll
        for (int b = 0; b < QT; ++b) {
            double g = 0.0;
#pragma unroll
            for (int a2 = 0; a2 < QT; ++a2) g = fma(pit[a2 * QT + b], S.F[(size_t)a2 * n + rr], g);
            G[k][b] = FOLD ? g * Kr[k] : g;
        }
    }
    __syncthreads();
    stamp(1);
    auto cnt = [&](int k, double v, int klo, int khi) {
        const double g = inner_coord(S, v, lev[k]);   // var_function (Q10), exact FP64
        return count_le(sx, g, klo, khi);
    };
    auto node = [&](int k, int j) {
        const double* c = col + j * CS;
        double W = 0.0;
#pragma unroll
        for (int b = 0; b < QT; ++b) W = fma(G[k][b], c[1 + b], W);
        const double zc = c[0];
        if constexpr (COP == CVQ_STUDENT) {
            const double pw = pow_node_t<PM>(fma(zc, fma(zc, Cq, Pr[k]), Rr[k]), S.node_m, S.node_ex);
            if constexpr (MSM) return pw * W;                                 // msm_integration_function.py:45
            return nan_to_num(pw * Kr[k] * c[1 + QT]) * W;                    // garch_integration_function.py:45-50
        } else {
            return node_value<COP, MSM, 2>(S, ctx[k], zc, c[1 + QT], W);
        }
    };
    // Folded Student/MSM path: per row, acc_b = sum_j pw_j F'_b[j] and the row's
    // sum is sum_b G'_b acc_b -- 12 FP64 ops per node (2 FMA quadratic form,
    // RCP + 2 FMA Newton + 2 MUL for b^-4, QT FMA), no select: 1/b of an infinite
    // or NaN b is NaN, which is what the node must be there (see above).
    auto pw_fold = [&](int k, double zc) {
        const double b = fma(zc, fma(zc, Cq, Pr[k]), Rr[k]);
        if constexpr (PM == 8) {
            double y = __builtin_amdgcn_rcp(b);
            y = fma(y, fma(-b, y, 1.0), y);
            const double y2 = y * y;
            return y2 * y2;
        } else {
            return pow_node_t<PM>(b, S.node_m, S.node_ex);
        }
    };
    auto range_sum_fold = [&](const int (&ka)[RPT], const int (&kb)[RPT]) {
        double part = 0.0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int len = has[k] ? kb[k] - ka[k] : 0;
            if (len <= 0) continue;
            double acc[ILP][QT];
#pragma unroll
            for (int u = 0; u < ILP; ++u)
#pragma unroll
                for (int b = 0; b < QT; ++b) acc[u][b] = 0.0;
            int j = ka[k] + 1;
            const int j1 = j + len;
            for (; j + ILP - 1 < j1; j += ILP) {
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    const double* c = col + (j + u) * CS;
                    const double pw = pw_fold(k, c[0]);
#pragma unroll
                    for (int b = 0; b < QT; ++b) acc[u][b] = fma(pw, c[1 + b], acc[u][b]);
                }
            }
            for (; j < j1; ++j) {
                const double* c = col + j * CS;
                const double pw = pw_fold(k, c[0]);
#pragma unroll
                for (int b = 0; b < QT; ++b) acc[0][b] = fma(pw, c[1 + b], acc[0][b]);
            }
#pragma unroll
            for (int b = 0; b < QT; ++b) {
                double a = acc[0][b];
#pragma unroll
                for (int u = 1; u < ILP; ++u) a += acc[u][b];
                part = fma(G[k][b], a, part);
            }
        }
        return TeamReduce<NT>::sum(part, red, parity);
    };
    auto range_sum = [&](const int (&ka)[RPT], const int (&kb)[RPT]) {
        if constexpr (FOLD) return range_sum_fold(ka, kb);
        // ILP independent node chains per thread (the slab's longest row is the
        // workgroup's critical path, so per-row latency matters more than issue)
        double p[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) p[u] = 0.0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int len = has[k] ? kb[k] - ka[k] : 0;
            if (len <= 0) continue;
            int j = ka[k] + 1;
            const int j1 = j + len;
            for (; j + ILP - 1 < j1; j += ILP) {
#pragma unroll
                for (int u = 0; u < ILP; ++u) p[u] += node(k, j + u);
            }
            for (; j < j1; ++j) p[ILP - 1] += node(k, j);
        }
#pragma unroll
        for (int h = 1; h < ILP; h <<= 1)
#pragma unroll
            for (int u = 0; u + h < ILP; u += 2 * h) p[u] += p[u + h];
        return TeamReduce<NT>::sum(p[0], red, parity);
    };
    auto slab = [&](double lo_v, double hi_v) {
        int ka[RPT], kb[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            ka[k] = has[k] ? cnt(k, lo_v, 0, n - 1) : 0;
            kb[k] = has[k] ? cnt(k, hi_v, ka[k], n - 1) : 0;
        }
        return range_sum(ka, kb);
    };

    if (mode == 1) {
        const double v = slab(bounds[2 * t], bounds[2 * t + 1]);
        if (tid == 0) out[t] = v;
        return;
    }
    // (i)-(iii): calc_var_class.py:114-160 (Q1, Q3)
    stamp(2);
    const double r0 = slab(P.lower, P.fg);
    stamp(3);
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;
    const double nr = slab(nl, nu);
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
    stamp(4);
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
    stamp(5);
    // (iv) bisection (:250-309), Q2 / Q4 resolved across dates by k_finalize
    double prev = F, prevU = prevU0;
    int nt = -1;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    for (int it = 0; it < P.K; ++it) {
        const double mid = (lo + hi) / 2;
        if (tid == 0) sn[it] = mid;
        if (nt < 0 && !(hi - lo > P.tol)) nt = it;
        int kM[RPT], ka[RPT], kb[RPT];
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            kM[k] = has[k] ? cnt(k, mid, kLo[k], kHi[k]) : 0;
            ka[k] = ustack ? kLo[k] : kM[k];               // (lo, mid]  or  (mid, hi]
            kb[k] = ustack ? kM[k] : kHi[k];
        }
        const double val = range_sum(ka, kb);
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
        if (it < 24) stamp(6 + it);
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
    const int e = __hip_atomic_load(&hdr->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (N > P.K ? 2 : 0);
    const unsigned long long nz = __hip_atomic_load((unsigned long long*)&hdr->nonzero, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    int kstop = min(N, P.K);
    for (int k = 0; k < kstop; ++k)
        if (!((nz >> k) & 1ull)) { kstop = k; break; }
    // every load in flight before the first store: one memory latency for T <= 4 NT
    for (long long d0 = tid; d0 < (long long)gridDim.x; d0 += 4 * NT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long d = d0 + (long long)u * NT;
            v[u] = d < (long long)gridDim.x ? snaps[d * P.stride + kstop] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long d = d0 + (long long)u * NT;
            if (d < (long long)gridDim.x) P.fin_var[d] = v[u] + P.ptf_mean;
        }
    }
    __syncthreads();                                     // every thread has read the header
    if (tid == 0) {
        P.fin_err[0] = e;
        P.fin_err[1] = kstop;
        P.fin_err[2] = N;
        P.fin_err[3] = 0;                                // ticket reset for the next launch
        hdr->iters = 0;                                  // header reset for the next launch
        hdr->error = 0;
        hdr->nonzero = 0;
    }
}

}  // namespace cvq
