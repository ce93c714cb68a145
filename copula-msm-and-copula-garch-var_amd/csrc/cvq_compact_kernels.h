// cvq_compact_kernels.h -- COMPACT strategy (2 assets): the DIRECT control flow
// with a rank-1 node weight, one barrier per bisection level, O(1) grid lookups,
// and the last bisection levels compacted into one wavefront.
//
// Reference: calc_var + bisection_algorithm (utils/calc_var_class.py:95-177,
// :250-309) integrate 2 + K slabs (a, b] per date; a slab is, per outer row r,
// the inner-index range (cnt_r(a), cnt_r(b)] with cnt_r(v) = largest j with
// x_j <= (v - x_r w1) / w0, else 0 (create_grids.py:102-108, Q9/Q10).
//
// One NT-thread workgroup per date (NT = 256 by default, CVQ_COMPACT_NT; NT = 64
// -- one wavefront, no LDS reduction or barrier -- measured slower for lack of
// latency hiding); thread tid owns the outer rows tid + NT k.
//  1. Tables: thread i evaluates the table entries of grid index i on both axes
//     (table_entry's arithmetic, the Student quantile written without
//     data-dependent branches so the two entries' memory latencies overlap) ->
//     LDS column records (z_j, B'_j) and LDS row records.
//  2. r0, nr and the bracket take their per-row cuts from a date-independent
//     table of the solve's fixed levels (lower, sg0, fg, sg1, vmin, vmax).
//  3. Each bisection level: kM = cnt_r(mid) by a bucket lookup into the grid and
//     an exact probe (count_le's result in O(1) LDS reads); the row owner sums
//     its slab columns with kIlp independent node chains; ONE workgroup
//     reduction returns (slab sum, slab nodes, bracket nodes).
//  4. Block tail (host cell tables present, the default): once the bisection cell
//     holds <= NT * kBlkPerThread nodes, the workgroup evaluates the cell's nodes
//     once in the host's v*-sorted order (v*(r, j): the smallest level with node
//     (r, j) inside, the exact FP64 membership rule), one block prefix scan gives F
//     at every node threshold, and the first thresholds where F >= obj and F != 0
//     decide every remaining level (one lane, no sums).  Without cell tables: the
//     bracket's (v*, value) pairs go to LDS once it holds <= kTailCap nodes and one
//     wave runs the remaining levels with masked wave sums.
//
// Phase stamps of the DIRECT kernel showed the per-level workgroup steps --
// binary searches, reductions, barriers -- and the single-row critical paths,
// not the node arithmetic, set a date's time; this kernel cuts each of them.
//
// Node values (fast path).  The MSM weight of node (r, j) is
// sum_{a,b} pi[a][b] F0_a(r) F1_b(j) (msm_integration_function.py:45 with Q5's
// rotation in F); the reference's pi is the outer product of the per-asset
// forecasts (compute_forecast_combinations, msm_estimation.py:392-418), so W =
// wr(r) wc(j), checked bitwise per date.  Then a node is
// scale_r * f(row consts, z_j) * B'_j, B'_j = B_j wc(j):
//   Student  f = (R_r + z (P_r + C z))^-(nu+2)/2   (student.py:133-141)
//   Gaussian f = exp(-(R_r + z (P_r + Ri11 z)) / 2) (gaussian.py:105-113)
//   Plackett f = (N_r + M_r v) / ((D_r + a1 v)(E_r - a1 v))^2   (plackett.py:66-69, Q11)
// A date whose pi is not rank 1, or a GARCH/UKF date with a non-finite table
// entry (nan_to_num semantics, garch_integration_function.py:45-50), takes the
// generic per-node path (node_value, full W contraction) for the whole solve.
#pragma once
#include "cvq_direct_kernels.h"

namespace cvq {

#ifndef CVQ_TAIL_PER_LANE
#define CVQ_TAIL_PER_LANE 4
#endif
constexpr int kTailPerLane = CVQ_TAIL_PER_LANE;     // tail nodes per lane of the tail wave
constexpr int kTailCap = 64 * kTailPerLane;         // bracket size that switches to the tail
// LDS row record (doubles): the generic kernel's [c0 c1 c2 c3 scale | z0 B0 wr]; the fast
// kernel keeps only the fast constants, [c0 c1 scale -] (Plackett [c0 c1 c2 c3 scale -])
template <int COP, bool GEN>
constexpr int kRowRec = GEN ? 8 : (COP == CVQ_PLACKETT ? 6 : 4);
template <int COP, bool GEN>
constexpr int kScaleAt = (GEN || COP == CVQ_PLACKETT) ? 4 : 2;
constexpr int kColRec = 2;                          // doubles per LDS column record (16 B: lanes at
                                                    // consecutive columns read conflict-free)
constexpr int kCutFixed = 8;                        // int16 per row in the fixed-level cut table (HBM)
constexpr int kCutLds = 6;                          // int16 per row of its LDS copy (the 6 used columns)
constexpr int kBucketsPerPoint = 4;                 // grid lookup buckets per grid point
// LDS budget: <= 32 KB per workgroup at n = 256 so five dates share a CU (160 KB):
// the generic path's column words (B_j, wc_j) live in the row records' unused
// Plackett slots [2], [3] for the Student / Gaussian kernels, and the LDS cut
// table keeps 6 of the HBM table's 8 columns.
template <int COP>
constexpr bool kColgInRow = COP != CVQ_PLACKETT;      // (generic kernel only)
#ifndef CVQ_COMPACT_WAVES
#define CVQ_COMPACT_WAVES 0                         // min waves per SIMD (0: compiler default)
#endif
#ifndef CVQ_COMPACT_ILP
#define CVQ_COMPACT_ILP 2
#endif
constexpr int kIlp = CVQ_COMPACT_ILP;               // independent node chains per row range
#ifndef CVQ_COMPACT_EXP2
#define CVQ_COMPACT_EXP2 1                          // fitted-nu power and Gaussian node by exp2_node7
#endif
constexpr double kGaussQ = CVQ_COMPACT_EXP2 ? -0.5 * 1.4426950408889634 : -0.5;   // Gaussian exponent scale
#ifndef CVQ_COMPACT_ILP0
#define CVQ_COMPACT_ILP0 1                          // node chains of the general (non-integer nu) power
#endif

// Fixed-level cut table columns: lower, sg0, fg, sg1, vmin, vmax (then padding).
enum { kCutLower = 0, kCutSg0, kCutFg, kCutSg1, kCutVmin, kCutVmax };

// Block tail (host cell tables present): once the bisection cell holds <= kBlkPerThread
// nodes per thread, the whole workgroup evaluates the cell's nodes once, in the host's
// v*-sorted order, and one block prefix scan gives F at every node threshold; the
// remaining levels then follow from two crossing thresholds with no further sums.
#ifndef CVQ_BLK_PER_THREAD
#define CVQ_BLK_PER_THREAD 12
#endif
constexpr int kBlkPerThread = CVQ_BLK_PER_THREAD;
// tail list word: row (bits 0-10) | column (bits 11-21) | last node of a tie group (bit 31)
constexpr uint32_t kTlRowMask = 0x7FFu;
constexpr int kTlColShift = 11;
constexpr uint32_t kTlGroupEnd = 1u << 31;
constexpr int kNoPos = 0x7FFFFFFF;                  // "no such position" in the crossing search

// Date-independent device tables of a COMPACT plan.
struct CompactGeom {
    const int16_t* cutfix;    // [n][kCutFixed] cut columns of the fixed levels (per solve arguments)
    const double* vstar;      // [n][n] v*(r, j): smallest level with node (r, j) inside (Q9/Q10)
    const int16_t* bucket;    // [nb] largest j with x_j <= bx0 + b / binv (0 if none): a start guess
    double bx0, binv;         // bucket of a grid coordinate g: floor((g - bx0) * binv)
    int nb;
    // [4][2 << cdepth] node counts of the bisection cells (heap node h of bracket b's tree at
    // (b << (cdepth + 1)) + h, 1 <= h < 2^(cdepth+1); every depth-cdepth cell holds <= the
    // block tail's NT * kBlkPerThread nodes); nullptr: the levels reduce the bracket's node
    // count on the device and finish with the one-wave tail
    const int* ccount;
    int cdepth;
    // with ccount: every node (r, j >= 1) sorted by v* (tail list words) and their v*; bracket
    // b's cells are contiguous ranges starting at bstart[b] (the cell tree's positions)
    const uint32_t* tlist;
    const double* tvs;
    int bstart[4];
    // with ccount: [4][2^cdepth][n] per-row cuts cnt_r(mid) of every bisection cell the levels split
    // (heap nodes 1 .. 2^cdepth - 1; date-independent, host-built); nullptr: the levels search the grid
    const int16_t* kcut;
    // [3][NT RPT][2] the fixed slabs' schedule: slot tid + NT k sums two half-rows of slab (lower, fg],
    // (sg0, fg] or (fg, sg1], each given as its column range row | j0 << 10 | len << 20 (0: none),
    // host-paired longest with shortest (ensure_cutfix); nullptr: slot k of thread tid takes the
    // first half of row r and the second half of row n - 1 - r
    const int* fpair;
};

// ------------------------------------------------------------------ reductions
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, ROWMASK, 0xF, true);
}

// Inclusive prefix sum over the 64 lanes: row_shr 1, 2, 4, 8 inside rows of 16,
// then row_bcast:15 (rows 1, 3) and row_bcast:31 (rows 2, 3).
__device__ __forceinline__ int wave_incl_scan(int v) {
    v += dpp_i32<0x111>(v);
    v += dpp_i32<0x112>(v);
    v += dpp_i32<0x114>(v);
    v += dpp_i32<0x118>(v);
    v += dpp_i32<0x142, 0xA>(v);
    v += dpp_i32<0x143, 0xC>(v);
    return v;
}

template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ double dpp_f64z(double v) {          // out-of-row / masked lanes read 0
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWMASK, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWMASK, 0xF, true);
    return __hiloint2double(hi, lo);
}

// Inclusive prefix sum of a double over the 64 lanes (same DPP pattern as wave_incl_scan).
__device__ __forceinline__ double wave_incl_scan_f64(double v) {
    v += dpp_f64z<0x111>(v);
    v += dpp_f64z<0x112>(v);
    v += dpp_f64z<0x114>(v);
    v += dpp_f64z<0x118>(v);
    v += dpp_f64z<0x142, 0xA>(v);
    v += dpp_f64z<0x143, 0xC>(v);
    return v;
}

// The zeros of the tail cell's F (non-decreasing in v: node values >= 0, a NaN makes every later F
// NaN) as the interval [vza, vzb) of mids, from F just above lo (Flo) and the thresholds of the first
// tie-group end with F == 0 (za, +inf if none) and the first with !(F <= 0) (zb, +inf if none):
// Flo > 0 or NaN: no zeros; Flo == 0: F is zero up to zb; Flo < 0 (the reference's first level can
// leave F at the CDF minus a constant, Q1): F may pass through exactly 0 from za up to zb.
__device__ __forceinline__ void zero_interval(double Flo, double za, double zb, double& vza, double& vzb) {
    const double inf = __builtin_inf();
    vza = (Flo == 0.0) ? -inf : (Flo < 0.0 ? za : inf);
    vzb = zb;
}

// The remaining R = K - it bisection levels of a date in closed form (P.exact_walk: every bracket's
// bisection points are exact dyadics, host-checked by dyadic_walk_ok).  Every decision is "mid >=
// v_c" (hi = mid), so after R levels the bracket is the cell (lo + c wR, lo + (c + 1) wR] holding v_c
// (kc 0: every mid decides high, c = 0; kc 1: none does, c = 2^R - 1), and level l's bracket is that
// cell's ancestor c >> (R - l): mid_l = lo + (2 (c >> (R - l)) + 1) w 2^-(l+1), all exact.  The Q4
// bit of level l is "F(mid_l) != 0": F is non-decreasing, so its zeros are one v-interval and the
// bit is !(v_za <= mid_l < v_zb) (zero_interval).  Called by all 64 lanes of one wave (lane l =
// level it + l); lo, hi, it, nt, mask come out identical in every lane.
__device__ __forceinline__ void dyadic_walk(const SolveConst& P, int kc, double vcs, double vza, double vzb,
                                            double& lo, double& hi, int& it, int& nt, uint64_t& mask, double* sn) {
    const int lane = threadIdx.x & 63;
    const int R = P.K - it;                                    // 1 <= R <= 52
    const double w = hi - lo, wR = ldexp(w, -R), top = ldexp(1.0, R) - 1.0;
    double c = kc == 0 ? 0.0 : top;
    if (kc == 2) {
        c = fmin(fmax(ceil((vcs - lo) / wR) - 1.0, 0.0), top);   // within 1 of the cell
        if (c > 0.0 && !(fma(c, wR, lo) < vcs)) c -= 1.0;
        else if (c < top && !(vcs <= fma(c + 1.0, wR, lo))) c += 1.0;
    }
    const bool act = lane < R;
    const double cl = floor(ldexp(c, lane - R));
    const double mid = fma(2.0 * cl + 1.0, ldexp(w, -(lane + 1)), lo);
    if (act) sn[it + lane] = mid;
    const unsigned long long bz = __ballot(act && !(mid >= vza && mid < vzb));
    const unsigned long long bt = __ballot(act && !(ldexp(w, -lane) > P.tol));
    if (nt < 0 && bt) nt = it + (int)__builtin_ctzll(bt);
    mask |= bz << it;
    const double lo0 = lo;
    lo = fma(c, wR, lo0);
    hi = fma(c + 1.0, wR, lo0);
    it = P.K;
}

// Block-wide exclusive scan of v; *total = sum over the block.  One barrier.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int v, int* wtot, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if constexpr (NT == 64) {
        *total = __builtin_amdgcn_readlane(incl, 63);
        return incl - v;
    }
    if (lane == 63) wtot[wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        const int s = wtot[w];
        base += (w < wave) ? s : 0;
        tot += s;
    }
    *total = tot;
    return base + incl - v;
}

// Workgroup sums of three values, identical in every thread (fixed order), one
// barrier; red: 2 x 3 x NT / 64 doubles, parity alternates the half used.
template <int NT>
__device__ __forceinline__ void team_sum3(double a, double b, double c, double* red, int& parity, double* out) {
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    if constexpr (NT == 64) {                                   // one wave: no LDS, no barrier
        out[0] = a;
        out[1] = b;
        out[2] = c;
        return;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double* rr = red + parity * (3 * (NT / 64));
    parity ^= 1;
    if (lane == 0) {
        rr[3 * wave] = a;
        rr[3 * wave + 1] = b;
        rr[3 * wave + 2] = c;
    }
    __syncthreads();
    double s0 = rr[0], s1 = rr[1], s2 = rr[2];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) {
        s0 += rr[3 * w];
        s1 += rr[3 * w + 1];
        s2 += rr[3 * w + 2];
    }
    out[0] = s0;
    out[1] = s1;
    out[2] = s2;
}

// Workgroup sum of one value, identical in every thread (fixed order), one barrier;
// shares team_sum3's slots (parity alternates the half used).
template <int NT>
__device__ __forceinline__ double team_sum1(double a, double* red, int& parity) {
    a = wave_sum(a);
    if constexpr (NT == 64) return a;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double* rr = red + parity * (3 * (NT / 64));
    parity ^= 1;
    if (lane == 0) rr[wave] = a;
    __syncthreads();
    double s = rr[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) s += rr[w];
    return s;
}

// count_le(sx, g, klo, khi) -- the largest j in [klo, khi] with x_j <= g, else klo
// (x_klo <= g or klo == 0; create_grids.py:104-108) -- from a bucket guess and an
// exact probe instead of a binary search.
__device__ __forceinline__ int grid_count(const double* sx, const int16_t* bk, const CompactGeom& G, double g, int klo,
                                          int khi) {
    if (!(g == g) || khi <= klo) return klo;                    // NaN level: nothing is <= g
    if (sx[khi] <= g) return khi;
    const double fb = (g - G.bx0) * G.binv;
    int j = fb < 0.0 ? 0 : (fb >= (double)(G.nb - 1) ? (int)bk[G.nb - 1] : (int)bk[(int)fb]);
    j = min(max(j, klo), khi - 1);
    while (j > klo && sx[j] > g) --j;
    while (sx[j + 1] <= g) ++j;                                 // stops at khi - 1: x_khi > g
    return j;
}

// ------------------------------------------------------------------ node values
struct FastRow {
    double c0, c1, c2, c3, scale;
};

template <int COP, int SI>
__device__ __forceinline__ void fast_row_consts(const StaticDev& S, double z0, double B0, double wr, double* rec) {
    if constexpr (COP == CVQ_STUDENT) {
        rec[0] = fma(S.Ri[0] * S.inv_nu, z0 * z0, 1.0);                 // R_r  (k_direct's Rr)
        rec[1] = (S.Ri[1] + S.Ri[2]) * S.inv_nu * z0;                   // P_r
        rec[SI] = S.term1 * B0 * wr;
    } else if constexpr (COP == CVQ_GAUSSIAN) {
        // the exponent -qf / 2 scaled by log2(e) (kGaussQ): the node is 2^E' (fast_f)
        rec[0] = (kGaussQ * S.Ri[0]) * (z0 * z0);
        rec[1] = (kGaussQ * (S.Ri[1] + S.Ri[2])) * z0;
        rec[SI] = S.term1 * B0 * wr;
    } else {
        static_assert(SI == 4, "Plackett row records hold four constants before the scale");
        const double th = S.theta, a1 = th - 1.0, u = z0;
        rec[0] = th * fma(a1, u, 1.0);                                   // num = c0 + c1 v
        rec[1] = th * a1 * fma(-2.0, u, 1.0);
        rec[2] = fma(a1, u, 1.0);                                        // d1 = c2 + a1 v
        rec[3] = fma(a1, 1.0 - u, 1.0);                                  // d2 = c3 - a1 v
        rec[4] = B0 * wr;
    }
}

template <int COP, int SI>
__device__ __forceinline__ FastRow load_fast_row(const double* rec) {
    FastRow f;
    const double2 a = *(const double2*)rec;
    f.c0 = a.x;
    f.c1 = a.y;
    if constexpr (COP == CVQ_PLACKETT) {
        const double2 b = *(const double2*)(rec + 2);
        f.c2 = b.x;
        f.c3 = b.y;
    } else {
        f.c2 = f.c3 = 0.0;
    }
    f.scale = rec[SI];
    return f;
}

template <int COP, int PM>
__device__ __forceinline__ double fast_f(const StaticDev& S, const FastRow& f, double zc) {
    if constexpr (COP == CVQ_STUDENT) {
        const double b = fma(zc, fma(zc, S.Ri[3] * S.inv_nu, f.c1), f.c0);
        if constexpr (PM == 8) {                      // nu = 6: b^-4; 1/inf = 0, 1/NaN = NaN
            double y = __builtin_amdgcn_rcp(b);
            y = fma(y, fma(-b, y, 1.0), y);
            const double y2 = y * y;
            return y2 * y2;
        } else {
#if CVQ_COMPACT_EXP2
            if (PM == 0 && S.node_m < 0) {               // fitted nu: 2^(ex log2(e) log b), 4e-11 (cvq_sorted_kernels.h pow_fast)
                const double y = exp2_node7((S.node_ex * 1.4426950408889634) * log_node_fast(b));
                return b < 1.0e300 ? y : (b == b ? 0.0 : b);   // ex < 0: +inf -> 0, NaN stays NaN
            }
#endif
            return pow_node_t<PM>(b, S.node_m, S.node_ex);
        }
    } else if constexpr (COP == CVQ_GAUSSIAN) {
        // exp(-qf / 2) = 2^E', E' = -log2(e) qf / 2 from the scaled row records (exp2_node7: 4e-11 relative;
        // CVQ_COMPACT_EXP2=0: kGaussQ = -1/2 and the library exp)
        const double E = fma(zc, fma(zc, kGaussQ * S.Ri[3], f.c1), f.c0);
        return CVQ_COMPACT_EXP2 ? exp2_node7(E) : exp(E);
    } else {
        const double a1 = S.theta - 1.0;
        const double num = fma(f.c1, zc, f.c0);
        const double d = fma(a1, zc, f.c2) * fma(-a1, zc, f.c3);
        const double den = d * d;
        double y = __builtin_amdgcn_rcp(den);
        y = fma(y, fma(-den, y, 1.0), y);
        y = fma(y, fma(-den, y, 1.0), y);
        // num / 0 as IEEE division gives it (the Newton steps would give NaN)
        return den == 0.0 ? (num == 0.0 ? __builtin_nan("") : __builtin_copysign(__builtin_inf(), num)) : num * y;
    }
}

// Generic node: reference semantics (node_value); cg = (B_j, wc_j); W = wr * wc
// (rank 1) or the full sum_ab pi[a][b] F0_a(r) F1_b(j).
template <int COP, bool MSM>
__device__ __forceinline__ double generic_node(const StaticDev& S, const double* rrec, double zc, const double* cg, int r,
                                               int j, bool rank1, const double* pit) {
    const RowCtx ctx = make_row<COP, 2>(S, rrec[5], 0.0, rrec[6]);
    double W;
    if (rank1) {
        W = rrec[7] * cg[1];
    } else {
        const int q = S.q, n = S.n;
        W = 0.0;
        for (int b = 0; b < q; ++b) {
            double g = 0.0;
            for (int a2 = 0; a2 < q; ++a2) g = fma(pit[a2 * q + b], S.F[(size_t)a2 * n + r], g);
            W = fma(g, S.F[((size_t)q + b) * n + j], W);
        }
    }
    return node_value<COP, MSM, 2>(S, ctx, zc, cg[0], W);
}

// table_entry of grid index i on axis 0 (row) and axis 1 (column) at once: the
// same arithmetic, with the Student quantile free of data-dependent branches so
// the two entries' table gathers are in flight together.
// NUI > 0: the copula's nu is the integer NUI (the nu = 6 node instances, PM = 8): the quantile's
// tail variable by root_nu and B = pdf (1 + z^2/nu)^((nu+1)/2) / g_uni without divisions
template <int COP, bool MSM, bool FUSED, int NUI = 0>
__device__ __forceinline__ void table_pair(const StaticDev& S, const double* __restrict__ a,
                                           const double* __restrict__ tA, const double* __restrict__ tB, long long t,
                                           int i, double* A, double* B) {
    if constexpr (!FUSED) {
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) {
            A[ax] = tA[(t * 2 + ax) * S.n + i];
            B[ax] = tB[(t * 2 + ax) * S.n + i];
        }
    } else if constexpr (COP == CVQ_STUDENT) {
        double u[2], pdf[2];
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) marginal_u<MSM>(S, a, t * 2 + ax, ax, i, &u[ax], &pdf[ax]);
        double z[2];
        if constexpr (NUI > 0) {
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) z[ax] = stdtrit_tab_int<NUI>(S.tk, u[ax]);   // student.py:102
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {                                            // :164-172
                const double pw = pow_half_pos_c<NUI + 1>(fma(z[ax] * z[ax], S.inv_nu, 1.0));   // uni_m = nu + 1
                A[ax] = z[ax];
                B[ax] = isfinite(z[ax]) ? (pdf[ax] * pw) * S.inv_g_uni : pdf[ax] * pos_inf();
            }
        } else {
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) z[ax] = stdtrit_tab_bf(S.tk, u[ax]);      // student.py:102
#pragma unroll
            for (int ax = 0; ax < 2; ++ax) {
                const double uni = isfinite(z[ax])
                    ? S.g_uni * pow_half_neg(1.0 + (z[ax] * z[ax]) / S.nu, S.uni_m, S.uni_ex) : 0.0;   // :164-172
                A[ax] = z[ax];
                B[ax] = (1.0 / uni) * pdf[ax];
            }
        }
    } else {
#pragma unroll
        for (int ax = 0; ax < 2; ++ax) table_entry<COP, MSM, COP == CVQ_STUDENT>(S, a, t * 2 + ax, ax, i, &A[ax], &B[ax]);
    }
}

template <int NT>
constexpr int kWtotInts = ((NT / 64) + 3) & ~3;

// k_finalize for a single rank, run by the last workgroup of a solve launch over
// T dates (calc_var_class.py:278, :293, :171): Q2 / Q4 from the header, VaR =
// snapshot + ptf_mean, status words to P.fin_err, header and ticket reset for
// the next launch.
template <int NT>
__device__ __forceinline__ void fused_finalize(const SolveConst& P, Header* hdr, const double* __restrict__ snaps,
                                               long long T) {
    const int tid = threadIdx.x;
    __threadfence();                                     // acquire: every workgroup's stores
    const int Nit = __hip_atomic_load(&hdr->iters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int err = __hip_atomic_load(&hdr->error, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (Nit > P.K ? 2 : 0);
    const unsigned long long nz = __hip_atomic_load((unsigned long long*)&hdr->nonzero, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
    int kstop = min(Nit, P.K);
    for (int k = 0; k < kstop; ++k)
        if (!((nz >> k) & 1ull)) { kstop = k; break; }
    // every load in flight before the first store: one memory latency for T <= 4 NT
    for (long long d0 = tid; d0 < T; d0 += 4 * NT) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long d = d0 + (long long)u * NT;
            v[u] = d < T ? snaps[d * P.stride + kstop] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const long long d = d0 + (long long)u * NT;
            if (d < T) P.fin_var[d] = v[u] + P.ptf_mean;
        }
    }
    __syncthreads();                                     // every thread has read the header
    if (tid == 0) {
        P.fin_err[0] = err;
        P.fin_err[1] = kstop;
        P.fin_err[2] = Nit;
        P.fin_err[3] = 0;                                // ticket reset for the next launch
        hdr->iters = 0;                                  // header reset for the next launch
        hdr->error = 0;
        hdr->nonzero = 0;
    }
}

// ------------------------------------------------------------------ the kernel
// calc_var solve: snapshots + header, fused finalize when P.fin_var.
// Thread tid owns rows tid + NT k (k < RPT, RPT = ceil(n / NT)); NT = 64 makes the
// whole solve one wavefront: no barriers, no LDS round trips in the reductions.
// FUSED: evaluate the date's tables here; else read k_tables' tA / tB.
#if CVQ_COMPACT_WAVES > 0
#define CVQ_COMPACT_BOUNDS(NT) __launch_bounds__(NT, CVQ_COMPACT_WAVES)
#else
#define CVQ_COMPACT_BOUNDS(NT) __launch_bounds__(NT)
#endif
// One date's solve by the whole workgroup: snapshots + this date's header bits.  GEN =
// false compiles the fast node path only (63 instead of 107 VGPRs at cfg 2: five
// workgroups per CU instead of four, +8.5%); a date that needs the generic path (pi not
// rank 1, or a non-finite GARCH / UKF table entry) is appended to defer[2 ..] (count in
// defer[0]) and left to the GEN = true kernel.  defer == nullptr: the caller asserted
// that no date needs the generic path (cvq_set_fast_hint, or the host's proof in
// cvq_set_dates) and no generic kernel follows -- such a date sets error bit 4 of the
// header instead (the solve fails with CVQ_ERR_NUMERIC).  Returns true when deferred.
template <int COP, bool MSM, int NT, int RPT, int PM, bool FUSED, bool GEN>
__device__ __forceinline__ bool compact_date(const StaticDev& S, const SolveConst& P, const CompactGeom& G,
                                             const double* __restrict__ a, const double* __restrict__ tA,
                                             const double* __restrict__ tB, const double* __restrict__ pi,
                                             double* __restrict__ stamps_out, double* __restrict__ snaps, Header* hdr,
                                             int* defer, const long long t) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int n = S.n, tid = threadIdx.x, lane = tid & 63;
    double* col = lds;                              // [n][kColRec]: z_j, B'_j = B_j wc_j
    // [n][2]: B_j, wc_j (generic path), stride cgs; Student / Gaussian: row record slots [2], [3]
    // (generic kernel only; the fast kernel has no such words)
    constexpr int RR = kRowRec<COP, GEN>, SI = kScaleAt<COP, GEN>;
    constexpr bool cg_in_row = GEN && kColgInRow<COP>, cg_own = GEN && !kColgInRow<COP>;
    constexpr int cgs = cg_in_row ? RR : 2;
    double* rowr = col + kColRec * n + (cg_own ? 2 * n : 0);   // [n][RR] row records
    double* colg = cg_in_row ? rowr + 2 : col + kColRec * n;
    double* sx = rowr + RR * n;                     // [n] grid
    double2* tail = (double2*)(sx + n);             // [kTailCap] tail nodes: (v*, value)
    double* red = (double*)(tail + kTailCap);       // [2][3][NT / 64] reduction slots
    int* wtot = (int*)(red + 6 * (NT / 64));        // [NT / 64] scan slots (padded to 16 B)
    int16_t* cfx = (int16_t*)(wtot + kWtotInts<NT>);   // [n][kCutLds] fixed-level cuts
    int16_t* bk = cfx + (size_t)kCutLds * n;        // [nb] grid lookup buckets

    unsigned long long* stamps = stamps_out ? (unsigned long long*)stamps_out + t * 32 : nullptr;
    auto stamp = [&](int idx) {                     // diagnostic only (never in a timed run)
        if (stamps && tid == 0 && idx < 32) stamps[idx] = __builtin_amdgcn_s_memtime();
    };
    // nodes this thread evaluated (stamps only: added to stamps[28] per date, zeroed by the host)
    int nev = 0;
    stamp(0);
    if (stamps && tid == 0) {
        stamps[25] = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
        stamps[30] = blockIdx.x;                         // dispatch position (placement analysis)
        // placement: HW_ID (wave, SIMD, CU, SH, SE fields) and XCC_ID of this workgroup's first wave
        stamps[27] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                     ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    }
    if (stamps && lane == 0 && (tid >> 6) < 4)     // placement of every wave (SIMD in bits 5:4)
        stamps[20 + (tid >> 6)] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    int row[RPT];
    bool own[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        row[k] = tid + NT * k;
        own[k] = row[k] < n;
    }
    // static LDS images (grid, lookup buckets, fixed-level cuts): every load issued here,
    // the stores after the tables phase, so their latency hides behind the tables' own
    // loads (n <= NT RPT, nb = kBucketsPerPoint n; clamped indices stay in bounds)
    static_assert(kCutLds % 2 == 0 && kCutFixed % 2 == 0, "cut rows copied as int pairs");
    constexpr int kBkPer = kBucketsPerPoint * RPT, kCutPer = (kCutLds / 2) * RPT;
    double xv[RPT];
    int bv[kBkPer], cv[kCutPer];

#pragma unroll
    for (int k = 0; k < RPT; ++k) xv[k] = S.x[min(tid + NT * k, n - 1)];
#pragma unroll
    for (int k = 0; k < kBkPer; ++k) bv[k] = G.bucket[min(tid + NT * k, G.nb - 1)];
#pragma unroll
    for (int k = 0; k < kCutPer; ++k) {
        const int w = min(tid + NT * k, (kCutLds / 2) * n - 1);
        cv[k] = ((const int*)G.cutfix)[(w / (kCutLds / 2)) * (kCutFixed / 2) + w % (kCutLds / 2)];
    }
    // the fixed slabs' half-row column ranges (host schedule G.fpair): (lower, fg], (sg0, fg], (fg, sg1]
    // (plain ints, selected with compile-time indices: an int2 array selected by slab went to scratch)
    int fpx[3][RPT], fpy[3][RPT];
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int2 w2 = G.fpair ? ((const int2*)G.fpair)[s3 * NT * RPT + tid + NT * k] : make_int2(0, 0);
            fpx[s3][k] = w2.x;
            fpy[s3][k] = w2.y;
        }
    // the first bisection level's per-row cuts of all four brackets (host table G.kcut, heap node 1)
    int krt[4][RPT];
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int k = 0; k < RPT; ++k)
            krt[b][k] = (G.kcut && G.ccount) ? ld32(G.kcut, (unsigned)((((b << G.cdepth) + 1) * n) + min(tid + NT * k, n - 1))) : 0;

    // ---- tables: index i -> row record i (axis 0) and column record i (axis 1)
    const int q = MSM ? S.q : 1;
    const double* fb = MSM ? a + t * 2 * q : nullptr;          // forecasts_by_states[t] (2, q)
    int bad = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        if (!own[k]) continue;
        const int i = row[k];
        double A[2], B[2];
        table_pair<COP, MSM, FUSED, (COP == CVQ_STUDENT && PM == 8) ? 6 : 0>(S, a, tA, tB, t, i, A, B);
        double wr, wc;                                             // row / column weight factors
        if constexpr (MSM) {
            wr = wc = 0.0;
            if (q <= kQUnroll) {                                   // every load issued before the chains
                double fr[kQUnroll], fc[kQUnroll], wa[kQUnroll], wb[kQUnroll];
#pragma unroll
                for (int b = 0; b < kQUnroll; ++b) {
                    const int bb = min(b, q - 1);
                    wa[b] = fb[bb];
                    wb[b] = fb[q + bb];
                    fr[b] = ld32(S.F, (unsigned)(bb * n + i));
                    fc[b] = ld32(S.F, (unsigned)((q + bb) * n + i));
                }
                // states b >= q: weight 0 (F finite: fma(0, F, w) == w), so no load waits
                // behind a branch on b < q
#pragma unroll
                for (int b = 0; b < kQUnroll; ++b) {
                    wr = fma(b < q ? wa[b] : 0.0, fr[b], wr);
                    wc = fma(b < q ? wb[b] : 0.0, fc[b], wc);
                }
            } else {
                for (int b = 0; b < q; ++b) {
                    wr = fma(fb[b], ld32(S.F, (unsigned)(b * n + i)), wr);
                    wc = fma(fb[q + b], ld32(S.F, (unsigned)((q + b) * n + i)), wc);
                }
            }
        } else {
            wr = S.F[i];
            wc = ld32(S.F, (unsigned)(n + i));
        }
        // GARCH / UKF Student: a dead entry (z = +-inf or NaN: u in {0, 1}) zeroes its nodes in the
        // reference (k_sorted's table phase, student.py:130-131, :166-167, nan_to_num): record
        // (0, scale 0) on the fast path rather than deferring the date to the generic kernel
        const bool d0 = COP == CVQ_STUDENT && !MSM && !isfinite(A[0]);
        const bool d1 = COP == CVQ_STUDENT && !MSM && !isfinite(A[1]);
        if ((!d0 && (!isfinite(A[0]) || !isfinite(B[0]))) || (!d1 && (!isfinite(A[1]) || !isfinite(B[1])))) bad |= 1;
        col[kColRec * i] = d1 ? 0.0 : A[1];
        col[kColRec * i + 1] = d1 ? 0.0 : B[1] * wc;
        double* rr = rowr + RR * i;
        fast_row_consts<COP, SI>(S, d0 ? 0.0 : A[0], d0 ? 0.0 : B[0], wr, rr);
        if constexpr (GEN) {
            colg[cgs * i] = B[1];                                  // may share rr[2..3] (Student / Gaussian)
            colg[cgs * i + 1] = wc;
            rr[5] = A[0];
            rr[6] = B[0];
            rr[7] = wr;
        }
    }
    const double* pit = pi + t * S.Q;
    if constexpr (MSM) {                                          // rank-1 check of pi_t
        for (int l = tid; l < S.Q; l += NT)
            if (!(pit[l] == fb[l / q] * fb[q + l % q])) bad |= 2;
    }
#pragma unroll
    for (int k = 0; k < RPT; ++k)
        if (tid + NT * k < n) sx[tid + NT * k] = xv[k];
#pragma unroll
    for (int k = 0; k < kBkPer; ++k)
        if (tid + NT * k < G.nb) bk[tid + NT * k] = (int16_t)bv[k];
#pragma unroll
    for (int k = 0; k < kCutPer; ++k)
        if (tid + NT * k < (kCutLds / 2) * n) ((int*)cfx)[tid + NT * k] = cv[k];
    // MSM: only bit 1 (pi not rank 1) decides the path; GARCH / UKF: only bit 0 (a
    // non-finite table entry, whose pi is rank 1 by construction)
    const bool flag = __syncthreads_or(MSM ? (bad & 2) : (bad & 1)) != 0;
    stamp(1);
    const bool rank1 = !(MSM && flag);
    const bool fast = rank1 && (MSM || !flag);
    if constexpr (!GEN) {
        if (!fast) {                                             // uniform: the whole workgroup leaves
            if (tid == 0) {
                if (defer) defer[2 + atomicAdd(&defer[0], 1)] = (int)t;
                else atomicOr(&hdr->error, 4);
            }
            return true;
        }
    }
    double lev[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) lev[k] = sx[own[k] ? row[k] : 0] * S.w1;   // integration_algo.py:20 (2-D)
    int parity = 0;

    // sum of row rr's nodes j in [j0, j1] (fast path: row scale included, kIlp
    // independent chains; generic: node values)
    auto range_sum = [&](int rr, int j0, int j1) -> double {
        if constexpr (GEN) {
            if (!fast) {
                double acc = 0.0;
                for (int j = j0; j <= j1; ++j)
                    acc += generic_node<COP, MSM>(S, rowr + RR * rr, col[kColRec * j], colg + cgs * j, rr, j,
                                                  rank1, pit);
                return acc;
            }
        }
        const FastRow fr = load_fast_row<COP, SI>(rowr + RR * rr);
        constexpr int IL = (COP == CVQ_STUDENT && PM == 0) ? CVQ_COMPACT_ILP0 : kIlp;   // general pow: register bound
        double acc[IL];
#pragma unroll
        for (int u = 0; u < IL; ++u) acc[u] = 0.0;
        int j = j0;
        for (; j + IL - 1 <= j1; j += IL) {
#pragma unroll
            for (int u = 0; u < IL; ++u) {
                const double2 cz = *(const double2*)(col + kColRec * (j + u));
                acc[u] = fma(fast_f<COP, PM>(S, fr, cz.x), cz.y, acc[u]);
            }
        }
        for (; j <= j1; ++j) {
            const double2 cz = *(const double2*)(col + kColRec * j);
            acc[0] = fma(fast_f<COP, PM>(S, fr, cz.x), cz.y, acc[0]);
        }
#pragma unroll
        for (int h = 1; h < IL; h <<= 1)
#pragma unroll
            for (int u = 0; u + h < IL; u += 2 * h) acc[u] += acc[u + h];
        return fr.scale * acc[0];
    };
    // one node (r, j) (the block tail): range_sum(r, j, j) without its loops, same arithmetic
    auto node1 = [&](int rr, int j) -> double {
        if constexpr (GEN) {
            if (!fast) return generic_node<COP, MSM>(S, rowr + RR * rr, col[kColRec * j], colg + cgs * j, rr, j, rank1, pit);
        }
        const FastRow fr = load_fast_row<COP, SI>(rowr + RR * rr);
        const double2 cz = *(const double2*)(col + kColRec * j);
        return fr.scale * fma(fast_f<COP, PM>(S, fr, cz.x), cz.y, 0.0);
    };
    // one level's workgroup sums: slab (ka, kb] sum, its node count, bracket (blo, bhi] nodes
    double sums[3];
    auto level_sums = [&](const int (&ka)[RPT], const int (&kb)[RPT], const int (&blo)[RPT], const int (&bhi)[RPT]) {
        double part = 0.0;
        int ns = 0, nb = 0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int len = own[k] ? max(kb[k] - ka[k], 0) : 0;
            if (len > 0) part += range_sum(row[k], ka[k] + 1, ka[k] + len);
            nev += len;
            ns += len;
            nb += own[k] ? max(bhi[k] - blo[k], 0) : 0;
        }
        team_sum3<NT>(part, (double)ns, (double)nb, red, parity, sums);
    };
    auto fixcut = [&](int k, double v) {                         // one of the solve's fixed levels
        const int16_t* c = cfx + (size_t)(own[k] ? row[k] : 0) * kCutLds;
        return v == P.lower ? c[kCutLower] : v == P.sg0 ? c[kCutSg0] : v == P.fg ? c[kCutFg]
             : v == P.sg1 ? c[kCutSg1] : v == P.vmin ? c[kCutVmin] : v == P.vmax ? c[kCutVmax]
             : grid_count(sx, bk, G, inner_coord(S, v, lev[k]), 0, n - 1);
    };
    int ka[RPT], kb[RPT];
    // slab (va, vb] between two fixed levels: these are triangles and corner bands
    // whose row lengths run from 0 to ~n, so the owner of row r sums the first half
    // of row r and the second half of row n - 1 - r (long rows pair with short ones)
    // sl: the slab's host schedule (0 = (lower, fg], 1 = (sg0, fg], 2 = (fg, sg1]; -1: none)
    // this thread's part of the slab (va, vb]
    auto fixed_part = [&](double va, double vb, int sl) -> double {
        double part = 0.0;
        if (G.fpair && sl >= 0) {
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                const int wx = sl == 0 ? fpx[0][k] : sl == 1 ? fpx[1][k] : fpx[2][k];
                const int wy = sl == 0 ? fpy[0][k] : sl == 1 ? fpy[1][k] : fpy[2][k];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const unsigned w = (unsigned)(e == 0 ? wx : wy);
                    const int len = (int)(w >> 20);
                    if (len == 0) continue;
                    const int j0 = (int)__builtin_amdgcn_ubfe(w, 10, 10);
                    part += range_sum((int)(w & 0x3FFu), j0, j0 + len - 1);
                    nev += len;
                }
            }
            return part;
        }
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (!own[k]) continue;
            const int r1 = row[k], r2 = n - 1 - row[k];
            const int16_t* c1 = cfx + (size_t)r1 * kCutLds;
            const int16_t* c2 = cfx + (size_t)r2 * kCutLds;
            auto cut = [&](const int16_t* c, double v) {
                return v == P.lower ? c[kCutLower] : v == P.sg0 ? c[kCutSg0] : v == P.fg ? c[kCutFg]
                     : v == P.sg1 ? c[kCutSg1] : v == P.vmin ? c[kCutVmin] : c[kCutVmax];
            };
            const int a1 = cut(c1, va), b1 = max((int)cut(c1, vb), a1);
            const int a2 = cut(c2, va), b2 = max((int)cut(c2, vb), a2);
            const int m1 = a1 + (b1 - a1 + 1) / 2, m2 = a2 + (b2 - a2 + 1) / 2;
            if (m1 > a1) part += range_sum(r1, a1 + 1, m1);
            if (b2 > m2) part += range_sum(r2, m2 + 1, b2);
            nev += max(m1 - a1, 0) + max(b2 - m2, 0);
        }
        return part;
    };

    // ---- (i)-(iii): calc_var_class.py:114-160 (Q1, Q3)
    const double r0 = team_sum1<NT>(fixed_part(P.lower, P.fg, 0), red, parity);
    stamp(2);
    const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
    const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
    const double prevU0 = (nl == P.sg0) ? P.sg0 : P.fg;
    const double nr = team_sum1<NT>(fixed_part(nl, nu, (nl == P.sg0 && nu == P.fg) ? 1 : (nl == P.fg && nu == P.sg1) ? 2 : -1),
                                    red, parity);
    const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
    stamp(3);
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    int bsel = -1;                                               // bracket: the host cell tables' index
    if (F > P.obj) { lo = P.vmin; hi = P.sg0; bsel = 0; }
    if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; bsel = 1; }
    if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; bsel = 2; }
    if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; bsel = 3; }
    bool ustack = !(hi == P.sg0 || hi == P.sg1);
    int kLo[RPT], kHi[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k) {                              // NaN bracket (Q3): empty
        kLo[k] = (own[k] && lo == lo) ? fixcut(k, lo) : 0;
        kHi[k] = (own[k] && lo == lo) ? max((int)fixcut(k, hi), kLo[k]) : 0;
    }
    stamp(4);

    // ---- (iv) bisection (:250-309); Q2 / Q4 are resolved across dates by the finalize
    double prev = F, prevU = prevU0;
    int nt = -1, it = 0;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    // the tail runs on wave 0; its lane 0 owns the header (rotating the tail wave
    // by date, to spread the tails of a CU's dates over its SIMDs, measured slower)
    const int leader = 0;
    // bracket nodes: the host's cell table (heap node hc of bracket bsel's tree), else
    // reduced with the level's sum; a NaN bracket (Q3) holds none
    const bool tabc = G.ccount != nullptr;
    const int* cc = tabc ? G.ccount + ((size_t)max(bsel, 0) << (G.cdepth + 1)) : nullptr;
    const int hend = tabc ? 2 << G.cdepth : 0;                   // heap nodes 1 .. 2^(cdepth+1) - 1
    // the levels' per-row cuts from the host table (tabulated cells: heap nodes < 2^cdepth), the
    // two children's loaded one level ahead; the first level's loaded with the bracket
    const bool tcut = tabc && G.kcut != nullptr && bsel >= 0;
    const int16_t* kc0 = tcut ? G.kcut + ((size_t)bsel << G.cdepth) * n : nullptr;
    const int kcn = tcut ? 1 << G.cdepth : 0;
    int kmt[RPT];
#pragma unroll
    for (int k = 0; k < RPT; ++k)
        kmt[k] = bsel == 0 ? krt[0][k] : bsel == 1 ? krt[1][k] : bsel == 2 ? krt[2][k] : krt[3][k];
    int hc = 1;
    int nbr_next = !tabc ? 1 << 30 : (bsel < 0 || hc >= hend) ? 0 : cc[hc];
    int ps = (tabc && bsel >= 0) ? G.bstart[bsel] : 0;           // the cell's first sorted position
    // the block tail (host tables) needs one bisection level first: the reference's first
    // level may subtract a slab it never added (Q1), after which F is the CDF plus a constant
    const int cap = tabc ? NT * kBlkPerThread : kTailCap;
    for (; it < P.K && (nbr_next > cap || (tabc && it == 0 && bsel >= 0)); ++it) {
        const double mid = (lo + hi) / 2;
        if (tid == 0) sn[it] = mid;
        if (nt < 0 && !(hi - lo > P.tol)) nt = it;
        // the children's counts, loaded while the level runs (depth cdepth: all <= kTailCap)
        const int c_lo = (tabc && 2 * hc < hend) ? cc[2 * hc] : 0;
        const int c_hi = (tabc && 2 * hc + 1 < hend) ? cc[2 * hc + 1] : 0;
        int kM[RPT], kml[RPT], kmh[RPT];
        const bool tnext = tcut && 2 * hc + 1 < kcn;               // both children tabulated: fetch now
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int rr = own[k] ? row[k] : 0;
            kml[k] = tnext ? ld32(kc0, (unsigned)(2 * hc * n + rr)) : 0;
            kmh[k] = tnext ? ld32(kc0, (unsigned)((2 * hc + 1) * n + rr)) : 0;
        }
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            kM[k] = !own[k] ? 0 : (tcut && hc < kcn) ? kmt[k]
                  : grid_count(sx, bk, G, inner_coord(S, mid, lev[k]), kLo[k], kHi[k]);   // Q10
            ka[k] = ustack ? kLo[k] : kM[k];
            kb[k] = ustack ? kM[k] : kHi[k];
        }

        double val;
        int Nlow = 0, Nbr = 0;
        if (tabc) {
            double part = 0.0;
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                const int len = own[k] ? max(kb[k] - ka[k], 0) : 0;
                if (len > 0) part += range_sum(row[k], ka[k] + 1, ka[k] + len);
                nev += len;
            }
            val = team_sum1<NT>(part, red, parity);
        } else {
            level_sums(ka, kb, kLo, kHi);
            val = sums[0];
            const int Ns = (int)sums[1];
            Nbr = (int)sums[2];
            Nlow = ustack ? Ns : Nbr - Ns;                       // nodes of (lo, mid]
        }
        const double slab_lower = ustack ? lo : mid;
        const double Fn = (slab_lower == prevU) ? prev + val : prev - val;   // adjust_integral
        if (Fn != 0.0) mask |= (1ull << it);
        ustack = Fn < P.obj;
#pragma unroll
        for (int k = 0; k < RPT; ++k) kmt[k] = ustack ? kmh[k] : kml[k];
        if (ustack) {
            lo = mid;
            nbr_next = tabc ? c_hi : Nbr - Nlow;
            ps += tabc ? c_lo : 0;
            hc = 2 * hc + 1;
#pragma unroll
            for (int k = 0; k < RPT; ++k) kLo[k] = kM[k];
        } else {
            hi = mid;
            nbr_next = tabc ? c_lo : Nlow;
            hc = 2 * hc;
#pragma unroll
            for (int k = 0; k < RPT; ++k) kHi[k] = kM[k];
        }
        prev = Fn;
        prevU = mid;
        if (it < 15) stamp(5 + it);
    }

    // ---- block tail (host cell tables): the cell (lo, hi] = sorted positions [ps, ps + cnt).
    // Thread tid evaluates positions tid * NPT + m in order; a block scan turns the values
    // into F at every node threshold (F = prev + prefix when the last level moved lo, else
    // prev - (cell total - prefix): the reference's adjust_integral chain after its first
    // level).  F is non-decreasing in v (node values >= 0; a NaN makes every later F NaN),
    // so each remaining level's decision "F(mid) < obj" is "mid < v_c" with v_c the first
    // tie-group end where !(F < obj), and its nonzero bit is "mid >= v_z", v_z the first
    // where F != 0 -- one lane then walks the remaining levels without sums.
    if (tabc && it < P.K) {
        constexpr int NPT = kBlkPerThread;
        const int cnt = max(nbr_next, 0);
        const uint32_t* tl = G.tlist + ps;
        uint32_t wd[NPT];
        double pre[NPT];                                          // local inclusive prefix
        double run = 0.0;
        nev += min(max(cnt - tid * NPT, 0), NPT);
#pragma unroll
        for (int m = 0; m < NPT; ++m) wd[m] = (tid * NPT + m < cnt) ? tl[tid * NPT + m] : 0u;
#pragma unroll
        for (int m = 0; m < NPT; ++m) {
            const int r = (int)(wd[m] & kTlRowMask), j = (int)((wd[m] >> kTlColShift) & kTlRowMask);
            const double v = (tid * NPT + m < cnt) ? node1(r, j) : 0.0;
            run += v;
            pre[m] = run;
        }
        // block exclusive scan of the thread totals (one barrier)
        const double incl = wave_incl_scan_f64(run);
        double* wt = red + parity * (3 * (NT / 64));
        parity ^= 1;
        if (lane == 63) wt[tid >> 6] = incl;
        __syncthreads();
        double base = incl - run, Stot = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) {
            const double x = wt[w];
            base += (w < (tid >> 6)) ? x : 0.0;
            Stot += x;
        }
        const double Flo = ustack ? prev : prev - Stot;           // F just above lo
        // first crossing / first zero / first positive (or NaN) group end (zero_interval)
        int mc = NPT, ma = NPT, mz = NPT;
#pragma unroll
        for (int m = NPT - 1; m >= 0; --m) {
            if (!(wd[m] & kTlGroupEnd) || tid * NPT + m >= cnt) continue;
            const double pa = base + pre[m];
            const double Fv = ustack ? prev + pa : prev - (Stot - pa);
            if (!(Fv < P.obj)) mc = m;
            if (Fv == 0.0) ma = m;
            if (!(Fv <= 0.0)) mz = m;
        }
        // first thread (lowest positions) holding each: wave ballots, then the block's waves
        const unsigned long long bc = __ballot(mc < NPT), ba = __ballot(ma < NPT), bz = __ballot(mz < NPT);
        int* ew = (int*)(red + parity * (3 * (NT / 64)));         // the other reduction half: 3 ints / wave
        parity ^= 1;
        // the first flagged thread of the wave holds the wave's first crossing; its position goes
        // to LDS, and the walk compares each mid with that node's v* from the plan's sorted list
        // (measured faster than re-evaluating the membership test x_j <= (mid - x_r w1) / w0)
        const int lc = bc ? (int)__builtin_ctzll(bc) : 0, la = ba ? (int)__builtin_ctzll(ba) : 0,
                  lz = bz ? (int)__builtin_ctzll(bz) : 0;
        const int mcl = __shfl(mc, lc, 64), mal = __shfl(ma, la, 64), mzl = __shfl(mz, lz, 64);
        if (lane == 0) {
            int* e = ew + 4 * (tid >> 6);
            e[0] = bc ? ((tid >> 6) * 64 + lc) * NPT + mcl : kNoPos;
            e[1] = ba ? ((tid >> 6) * 64 + la) * NPT + mal : kNoPos;
            e[2] = bz ? ((tid >> 6) * 64 + lz) * NPT + mzl : kNoPos;
        }
        __syncthreads();
        stamp(29);
        // exact dyadic bisection points (host check, P.exact_walk): wave 0 walks the remaining
        // levels in closed form, lane l = level it + l; else lane 0 walks them one by one
        const bool exact = P.exact_walk != 0;
        if (exact ? tid < 64 : tid == leader) {
            int ec = kNoPos, ea = kNoPos, ez = kNoPos;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) {                   // waves in position order: first wins
                const int* e = ew + 4 * w;
                if (ec == kNoPos && e[0] != kNoPos) ec = e[0];
                if (ea == kNoPos && e[1] != kNoPos) ea = e[1];
                if (ez == kNoPos && e[2] != kNoPos) ez = e[2];
            }
            // kind: 0 = every mid (F just above lo already decides), 1 = no mid, 2 = mids at or
            // above the node's threshold (v* loaded from the plan's sorted list)
            const int kc = !(Flo < P.obj) ? 0 : (ec == kNoPos ? 1 : 2);
            const double vcs = kc == 2 ? G.tvs[ps + ec] : 0.0;
            const double inf = __builtin_inf();
            double vza, vzb;
            zero_interval(Flo, (Flo < 0.0 && ea != kNoPos) ? G.tvs[ps + ea] : inf,
                          (!(Flo > 0.0) && ez != kNoPos) ? G.tvs[ps + ez] : inf, vza, vzb);
            if (exact) {
                dyadic_walk(P, kc, vcs, vza, vzb, lo, hi, it, nt, mask, sn);
            } else {
                for (; it < P.K; ++it) {
                    const double mid = (lo + hi) / 2;
                    sn[it] = mid;
                    if (nt < 0 && !(hi - lo > P.tol)) nt = it;
                    const bool geq = kc == 0 || (kc == 2 && mid >= vcs);
                    const bool nz = !(mid >= vza && mid < vzb);
                    if (nz) mask |= (1ull << it);
                    ustack = !geq;
                    if (ustack) lo = mid; else hi = mid;
                }
            }
        }
    } else if (it < P.K) {
    // ---- tail: the bracket's nodes -> LDS, wave 0 finishes the levels
        int len = 0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) len += own[k] ? kHi[k] - kLo[k] : 0;
        int total;
        int off = block_excl_scan<NT>(len, wtot, &total);
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            if (!own[k]) continue;
            for (int j = kLo[k] + 1; j <= kHi[k] && off < kTailCap; ++j, ++off) {  // total <= kTailCap
                tail[off] = make_double2(G.vstar[(size_t)row[k] * n + j], range_sum(row[k], j, j));
                ++nev;
            }
        }
        __syncthreads();
        stamp(29);
        if ((tid >> 6) == (leader >> 6)) {
            // this lane's entries lane + 64 m: (v*, value); padding v* = NaN is in no interval
            const int tot = min(total, kTailCap);
            double tx[kTailPerLane], ty[kTailPerLane];
#pragma unroll
            for (int m = 0; m < kTailPerLane; ++m) {
                const bool ok = lane + 64 * m < tot;
                const double2 e = ok ? tail[lane + 64 * m] : make_double2(__builtin_nan(""), 0.0);
                tx[m] = e.x;
                ty[m] = e.y;
            }
            for (; it < P.K; ++it) {
                const double mid = (lo + hi) / 2;
                if (tid == leader) sn[it] = mid;
                if (nt < 0 && !(hi - lo > P.tol)) nt = it;
                const double a0 = ustack ? lo : mid, b0 = ustack ? mid : hi;   // slab (a0, b0]
                double p = 0.0;
#pragma unroll
                for (int m = 0; m < kTailPerLane; ++m) p += (tx[m] > a0 && tx[m] <= b0) ? ty[m] : 0.0;
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
    stamp(31);
    if (stamps && tid == 0) stamps[26] = __builtin_amdgcn_s_memrealtime();
    if (stamps) {
        const int w = (int)wave_sum((double)nev);                  // exact in a double
        if (lane == 0 && w) atomicAdd(&stamps[28], (unsigned long long)w);
    }

    if (tid == leader) {
        sn[P.K] = (lo + hi) / 2;
        if (nt < 0 && !(hi - lo > P.tol)) nt = P.K;
        if (nt < 0) atomicOr(&hdr->error, 1);
        else atomicMax(&hdr->iters, nt);
        atomicOr((unsigned long long*)&hdr->nonzero, (unsigned long long)mask);
    }
    return false;
}

// The solve over T dates: GEN = false, one workgroup per date (grid T); GEN = true, a
// small grid working through the dates the fast kernel deferred (none: every workgroup
// leaves at once).  Fused finalize (P.fin_var) by the last workgroup of the launch that
// completes the solve: the fast kernel when it deferred nothing, else the generic one.
// defer[0] = deferred count, defer[1] = the generic kernel's ticket; both reset there.
template <int COP, bool MSM, int NT, int RPT, int PM, bool FUSED, bool GEN>
__global__ CVQ_COMPACT_BOUNDS(NT) void k_compact(StaticDev S, SolveConst P, CompactGeom G, const double* __restrict__ a,
                                                const double* __restrict__ tA, const double* __restrict__ tB,
                                                const double* __restrict__ pi, double* __restrict__ stamps_out,
                                                double* __restrict__ snaps, Header* hdr, int* defer, long long T) {
    const int tid = threadIdx.x;
    __shared__ int last;
    if constexpr (!GEN) {
        compact_date<COP, MSM, NT, RPT, PM, FUSED, false>(S, P, G, a, tA, tB, pi, stamps_out, snaps, hdr, defer,
                                                          (long long)blockIdx.x);
        if (!P.fin_var) return;
        if (tid == 0) {
            __threadfence();                             // release: this date's snapshots + header bits / deferral
            last = atomicAdd(&P.fin_err[3], 1) == (int)gridDim.x - 1;
        }
        __syncthreads();
        if (!last) return;
        __threadfence();
        if (!defer || __hip_atomic_load(&defer[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            fused_finalize<NT>(P, hdr, snaps, T);
        } else if (tid == 0) {
            P.fin_err[3] = 0;                            // the generic kernel finalizes
        }
    } else {
        const int cnt = __hip_atomic_load(&defer[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int k = blockIdx.x; k < cnt; k += gridDim.x) {
            const long long t = defer[2 + k];
            compact_date<COP, MSM, NT, RPT, PM, FUSED, true>(S, P, G, a, tA, tB, pi, stamps_out, snaps, hdr, defer, t);
            __syncthreads();                             // LDS reused by the next date
        }
        if (tid == 0) {
            __threadfence();
            last = atomicAdd(&defer[1], 1) == (int)gridDim.x - 1;
        }
        __syncthreads();
        if (!last) return;
        __threadfence();
        if (cnt > 0 && P.fin_var) fused_finalize<NT>(P, hdr, snaps, T);
        __syncthreads();
        if (tid == 0) {
            defer[0] = 0;                                // reset for the next solve
            defer[1] = 0;
        }
    }
}

// LDS bytes of one k_compact workgroup (cfg 2, n = 256, Student: fast 23,760 B -- six dates per CU --,
// generic 31,952 B)
template <int COP, bool GEN>
inline size_t compact_lds_bytes(int n, int nt, int nb) {
    constexpr int cg = (GEN && !kColgInRow<COP>) ? 2 : 0;
    return sizeof(double) * ((size_t)(kColRec + cg + kRowRec<COP, GEN> + 1) * n) + sizeof(double2) * kTailCap +
           sizeof(double) * 6 * (nt / 64) + sizeof(int) * (((nt / 64) + 3) & ~3) +
           sizeof(int16_t) * ((size_t)kCutLds * n + nb);
}

}  // namespace cvq
