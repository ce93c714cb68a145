// cvq_forecast.hip -- per-date forecast stage + batched in-sample likelihoods (gfx950).
//
// Reference:
//   MSM   markov_switching_multifractal/calc_prob.py:8-142, calc_marginals.py:33-38,
//         utils/model_estimation/model/msm_estimation.py:140-202
//   GARCH garch/estimation.py:40-125, garch/forecast.py:5-19
//   UKF   kalman_mean_reverting/estimate.py:53-281, forecast.py:5-12
//
// Each rolling window restarts its filter (load_data.py:130-137), so windows are
// independent: the batch axis is (window) for forecasts and (parameter candidate)
// for likelihoods.  The MSM transition matrix is a Kronecker product of k 2x2
// blocks (calc_prob.py:91-101), so A.pi is applied as k butterflies instead of an
// S x S mat-vec: a quad of lanes holds one window's 2^k states, low state bits
// in registers, the top two bits across the quad (__shfl_xor 1, 2).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "cvq_common.h"

using namespace cvq;

namespace {

constexpr double kInvSqrt2Pi = 0.3989422804014327;

struct MsmParams {
    double p[8];       // stay probabilities p_c = 1 - gamma_c / 2 (calc_prob.py:93-95)
    double qv[8];      // 1 - p_c
    double vs[128];    // vol states sqrt(prod M_s) * sigma (calc_prob.py:103-108)
};

struct MsmParamsN {
    MsmParams a[3];                                // per asset (dim <= 3), passed by value
};

struct StateMap {
    uint8_t u[3][128];                             // unique-vol index of state s of asset d
};

struct StateMapQ {                                 // unique-vol index of each of <= 16 states, per asset
    uint8_t u[3][16];
    int q;
};

MsmParams msm_params(int k, double m0, double sigma, double b, double gamma) {
    MsmParams P{};
    for (int c = 0; c < k; ++c) {
        const double gk = 1 - std::pow(1 - gamma, std::pow(b, (double)c));
        P.p[c] = 1 - gk / 2;
        P.qv[c] = 1 - P.p[c];
    }
    const int S = 1 << k;
    for (int s = 0; s < S; ++s) {
        double prod = 1.0;
        for (int c = 0; c < k; ++c) {            // itertools.product order: component c <-> bit k-1-c
            const int bit = (s >> (k - 1 - c)) & 1;
            prod = (c == 0) ? (bit ? 2 - m0 : m0) : prod * (bit ? 2 - m0 : m0);
        }
        P.vs[s] = std::sqrt(prod) * sigma;
    }
    return P;
}

__device__ __forceinline__ double cond_prob(double r, double vs) {
    const double z = r / vs;
    return (1 / (vs * 2.5066282746310002)) * exp(-0.5 * (z * z));   // calc_prob.py:116-117
}

// Quad-local lane exchange of a double by DPP (xor 1: quad_perm [1,0,3,2]; xor 2:
// [2,3,0,1]): a VALU move with no LDS round trip, unlike __shfl_xor's ds_bpermute --
// the filter's per-step chain is latency-bound, so this sets its speed.
template <int M>
__device__ __forceinline__ double quad_xor(double v) {
    constexpr int ctrl = M == 1 ? 0xB1 : 0x4E;
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// Lane exchanges for a state vector spread one state per lane over a wavefront: v of lane
// (l xor M).  M = 1, 2: quad_perm; M = 4, 8: row_shl / row_shr by M selected by lane bit M (DPP,
// VALU moves with no LDS round trip); M = 16, 32: ds_bpermute (__shfl_xor).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int M>
__device__ __forceinline__ double lane_xor(double v) {
    if constexpr (M == 1) return dpp_f64<0xB1>(v);
    else if constexpr (M == 2) return dpp_f64<0x4E>(v);
    else if constexpr (M == 4 || M == 8) {
        const double up = dpp_f64<0x100 | M>(v), dn = dpp_f64<0x110 | M>(v);   // row_shl:M / row_shr:M
        return (threadIdx.x & M) ? dn : up;
    } else {
        // v_permlane16_swap / v_permlane32_swap (gfx950, VALU): with both operands v, lane l of the
        // swapped src (lanes below the half) or of vdst (lanes above) holds v of lane l xor M
        const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
        const bool up = (threadIdx.x & M) != 0;
        unsigned nlo, nhi;
        if constexpr (M == 16) {
            const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
            const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
            nlo = up ? a[0] : a[1];
            nhi = up ? b[0] : b[1];
        } else {
            const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
            const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
            nlo = up ? a[0] : a[1];
            nhi = up ? b[0] : b[1];
        }
        return __hiloint2double((int)nhi, (int)nlo);
    }
}
// sum over the 64 lanes, in every lane: DPP inclusive scan (row_shr 1, 2, 4, 8, row_bcast 15, 31),
// then lane 63's total broadcast
template <int CTRL, int RM>
__device__ __forceinline__ double dpp_f64z(double v) {         // bound_ctrl: out-of-row lanes read 0
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, RM, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, RM, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_total(double v) {
    v += dpp_f64z<0x111, 0xF>(v);
    v += dpp_f64z<0x112, 0xF>(v);
    v += dpp_f64z<0x114, 0xF>(v);
    v += dpp_f64z<0x118, 0xF>(v);
    v += dpp_f64z<0x142, 0xA>(v);
    v += dpp_f64z<0x143, 0xC>(v);
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), 63),
                            __builtin_amdgcn_readlane(__double2loint(v), 63));
}

template <int K>
struct Quad {
    static constexpr int S = 1 << K;
    static constexpr int L = S < 4 ? S : 4;        // lanes per window
    static constexpr int SL = S / L;               // states per lane
    static constexpr int LB = (SL == 1) ? 0 : __builtin_ctz(SL);
};

// One Hamilton-filter step (calc_bayes_upd_numba, calc_prob.py:51-69) for a
// quad-resident state vector.  v: this lane's SL states (state s = lane_q*SL + j),
// cv: the matching conditional densities.  Returns the normaliser.  IEEE: normalise
// by IEEE division, v / tot as calc_prob.py does (the reference-facing filter
// cvq_msm_filter); else by a hardware reciprocal + two Newton steps (~1 ulp; the
// blocked end-to-end filter and the likelihoods, where ~1e-16 is far below the 1e-8
// node noise the VaR tolerates).
template <int K, bool IEEE = false>
__device__ __forceinline__ double msm_step(double (&v)[Quad<K>::SL], const double (&cv)[Quad<K>::SL],
                                           const MsmParams& P, bool* zero) {
    constexpr int SL = Quad<K>::SL, L = Quad<K>::L, LB = Quad<K>::LB;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const int pos = K - 1 - c;                 // component c <-> state bit k-1-c
        const double pc = P.p[c], qc = P.qv[c];
        if (pos < LB) {
            double nv[SL];
#pragma unroll
            for (int j = 0; j < SL; ++j) nv[j] = pc * v[j] + qc * v[j ^ (1 << pos)];
#pragma unroll
            for (int j = 0; j < SL; ++j) v[j] = nv[j];
        } else {
            const int m = 1 << (pos - LB);
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                const double o = m == 1 ? quad_xor<1>(v[j]) : quad_xor<2>(v[j]);
                v[j] = pc * v[j] + qc * o;
            }
        }
    }
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < SL; ++j) {
        v[j] = v[j] * cv[j];
        part += v[j];
    }
    double tot = part;
    if (L >= 2) tot += quad_xor<1>(tot);
    if (L >= 4) tot += quad_xor<2>(tot);
    *zero = !(tot != 0.0);
    if constexpr (IEEE) {
#pragma unroll
        for (int j = 0; j < SL; ++j) v[j] = v[j] / tot;
        return tot;
    }
    double inv = __builtin_amdgcn_rcp(tot);
    inv = fma(inv, fma(-tot, inv, 1.0), inv);
    inv = fma(inv, fma(-tot, inv, 1.0), inv);
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = v[j] * inv;
    return tot;
}

// cond[d][i][s] for every return of each asset's series (shared by all windows containing i);
// blockIdx.y = asset, its returns at r + d * N.
__global__ void k_msm_cond(MsmParamsN PN, int S, const double* __restrict__ r, long long N, double* __restrict__ cond) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= N * S) return;
    const int d = blockIdx.y;
    cond[d * N * S + idx] = cond_prob(r[d * N + idx / S], PN.a[d].vs[idx % S]);
}

// Filtered state probabilities at the end of each window (calc_forecasts), every asset
// of the batch in one launch (blockIdx.y = asset; cond / out strides per asset).  The
// window's N_in steps are a dependent chain, so the conditional densities of the next
// kPrefetch steps are loaded ahead in a register ring: the chain waits on the FP64
// math, not on an L2 round trip per step.
constexpr int kPrefetch = 8;

template <int K>
__global__ __launch_bounds__(256) void k_msm_filter(MsmParamsN PN, const double* __restrict__ cond, long long cstride,
                                                    long long n_in, long long T, double* __restrict__ out,
                                                    long long ostride, int* err) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    const MsmParams& P = PN.a[blockIdx.y];
    cond += blockIdx.y * cstride;
    out += blockIdx.y * ostride;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long t = gid / L;
    const int lane_q = (int)(gid % L);
    const bool active = t < T;
    const long long tt = active ? t : T - 1;
    double v[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = 1.0 / S;               // equi_prob (calc_prob.py:12-13)
    bool bad = false;
    const double* base = cond + tt * S + lane_q * SL;          // row i of this window: base + i * S
    double ring[kPrefetch][SL];
#pragma unroll
    for (int d = 0; d < kPrefetch; ++d)
#pragma unroll
        for (int j = 0; j < SL; ++j) ring[d][j] = d < n_in ? base[(long long)d * S + j] : 0.0;
    for (long long i0 = 0; i0 < n_in; i0 += kPrefetch) {
#pragma unroll
        for (int d = 0; d < kPrefetch; ++d) {
            const long long i = i0 + d;
            if (i < n_in) {
                double cv[SL];
#pragma unroll
                for (int j = 0; j < SL; ++j) cv[j] = ring[d][j];
                const long long nx = i + kPrefetch;
#pragma unroll
                for (int j = 0; j < SL; ++j) ring[d][j] = nx < n_in ? base[nx * S + j] : 0.0;
                bool z;
                msm_step<K, true>(v, cv, P, &z);
                bad |= z;
            }
        }
    }
    if (!active) return;
    if (bad) atomicOr(err, 1);
#pragma unroll
    for (int j = 0; j < SL; ++j) out[t * S + lane_q * SL + j] = v[j];
}

// ------------------------------------------------------- blocked (time-parallel) filter
// The filter is linear up to its per-step normalisation: window t's filtered vector is
// normalise(M_{t+n-1} ... M_t u), M_i = diag(c_i) A, u uniform (calc_prob.py:12-13,
// :51-69).  Rolling windows share all but one of their steps, so the series is cut into
// blocks of kBlk steps whose products G_b = M_{(b+1)B-1} ... M_{bB} are formed once
// (k_msm_gblocks, every block in parallel); window t then runs only its partial first and
// last blocks as filter steps and crosses the full blocks in between with one dense
// G_b mat-vec each (k_msm_windows): <= 2B + n/B dependent steps instead of n.  All terms
// are non-negative, so the reordering is benign (no cancellation): the forecasts agree
// with the step-by-step filter to ~1e-14 relative.
//
// k_msm_gblocks: column j of G_b is the un-normalised filter run from e_j over the block;
// every step is scaled by the common factor 1 / max_s c_i[s] (the same for all columns,
// so it cancels on the final normalisation) to keep entries <= 1.  One quad per column.
template <int K>
__global__ __launch_bounds__(256) void k_msm_gblocks(MsmParamsN PN, const double* __restrict__ cond,
                                                     long long cstride, int B, int nfull, double* __restrict__ G,
                                                     long long gstride, int* err) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    const MsmParams& P = PN.a[blockIdx.y];
    cond += blockIdx.y * cstride;
    G += blockIdx.y * gstride;
    const int col = threadIdx.x / L, lane_q = threadIdx.x % L;
    const int b = blockIdx.x;
    if (b >= nfull || col >= S) return;
    double v[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = (lane_q * SL + j == col) ? 1.0 : 0.0;
    const double* base = cond + (long long)b * B * S + lane_q * SL;
    bool bad = false;
    for (int i = 0; i < B; ++i) {
        double cv[SL], m = 0.0;
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            cv[j] = base[(long long)i * S + j];
            m = fmax(m, cv[j]);
        }
        if (L >= 2) m = fmax(m, quad_xor<1>(m));
        if (L >= 4) m = fmax(m, quad_xor<2>(m));
        bad |= !(m > 0.0);                             // every state's density is 0: calc_prob.py:64-65
        const double s = 1.0 / m;
#pragma unroll
        for (int c = 0; c < K; ++c) {
            const int pos = K - 1 - c;
            const double pc = P.p[c], qc = P.qv[c];
            if (pos < Quad<K>::LB) {
                double nv[SL];
#pragma unroll
                for (int j = 0; j < SL; ++j) nv[j] = pc * v[j] + qc * v[j ^ (1 << pos)];
#pragma unroll
                for (int j = 0; j < SL; ++j) v[j] = nv[j];
            } else {
                const int mm = 1 << (pos - Quad<K>::LB);
#pragma unroll
                for (int j = 0; j < SL; ++j) {
                    const double o = mm == 1 ? quad_xor<1>(v[j]) : quad_xor<2>(v[j]);
                    v[j] = pc * v[j] + qc * o;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < SL; ++j) v[j] = v[j] * (cv[j] * s);
    }
    if (bad && col == 0 && lane_q == 0) atomicOr(err, 1);
    double* g = G + (long long)b * S * S;                       // G_b[r][c], row-major
#pragma unroll
    for (int j = 0; j < SL; ++j) g[(lane_q * SL + j) * S + col] = v[j];
}

// k_msm_windows: one quad per window, kWinPerWG windows per workgroup; the full blocks any
// of the workgroup's windows crosses are staged in LDS once.
constexpr int kWinPerWG = 16;

template <int K>
__device__ __forceinline__ void msm_steps(double (&v)[Quad<K>::SL], const double* __restrict__ base, long long i0,
                                          long long i1, const MsmParams& P, bool* bad) {
    constexpr int SL = Quad<K>::SL;
    constexpr int S = Quad<K>::S;
    constexpr int PF = 4;                                       // rows in flight ahead of the chain
    double ring[PF][SL];
#pragma unroll
    for (int d = 0; d < PF; ++d)
#pragma unroll
        for (int j = 0; j < SL; ++j) ring[d][j] = (i0 + d < i1) ? base[(i0 + d) * S + j] : 0.0;
    for (long long i = i0; i < i1; i += PF) {
#pragma unroll
        for (int d = 0; d < PF; ++d) {
            if (i + d < i1) {
                double cv[SL];
#pragma unroll
                for (int j = 0; j < SL; ++j) cv[j] = ring[d][j];
                const long long nx = i + d + PF;
#pragma unroll
                for (int j = 0; j < SL; ++j) ring[d][j] = nx < i1 ? base[nx * S + j] : 0.0;
                bool z;
                msm_step<K>(v, cv, P, &z);
                *bad |= z;
            }
        }
    }
}

template <int K>
__global__ __launch_bounds__(64) void k_msm_windows(MsmParamsN PN, const double* __restrict__ cond, long long cstride,
                                                    const double* __restrict__ G, long long gstride, int B,
                                                    long long n_in, long long T, double* __restrict__ out,
                                                    long long ostride, int* err) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    static_assert(L == 4 && SL * L == S, "blocked filter: a quad holds the states (2 <= k <= 4)");
    extern __shared__ __attribute__((aligned(16))) double gl[];       // [nb][S][S]
    const MsmParams& P = PN.a[blockIdx.y];
    cond += blockIdx.y * cstride;
    G += blockIdx.y * gstride;
    out += blockIdx.y * ostride;
    const long long t0 = (long long)blockIdx.x * kWinPerWG;
    const long long tl = min(t0 + kWinPerWG, T) - 1;                  // last window of the workgroup
    const long long blo = t0 / B + 1, bhi = (tl + n_in - 1) / B - 1;  // full blocks crossed by any window
    const long long nb = bhi >= blo ? bhi - blo + 1 : 0;
    {
        const double2* src = (const double2*)(G + blo * S * S);
        double2* dst = (double2*)gl;
        for (long long w = threadIdx.x; w < nb * S * S / 2; w += blockDim.x) dst[w] = src[w];
    }
    __syncthreads();
    const long long t = t0 + threadIdx.x / L;
    const int lane_q = threadIdx.x % L;
    const bool active = t < T;
    const long long tt = active ? t : T - 1;
    const long long b0 = tt / B, b1 = (tt + n_in - 1) / B;            // b1 >= b0 + 1 (host: n_in > B)
    double v[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = 1.0 / S;                      // equi_prob (calc_prob.py:12-13)
    bool bad = false;
    const double* base = cond + lane_q * SL;
    msm_steps<K>(v, base, tt, (b0 + 1) * B, P, &bad);                 // first partial block
    for (long long b = b0 + 1; b < b1; ++b) {                         // full blocks: dense mat-vec
        // the window's whole vector: src[x] = the states of quad lane lane_q ^ x
        double src[4][SL];
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            src[0][j] = v[j];
            src[1][j] = quad_xor<1>(v[j]);
            src[2][j] = quad_xor<2>(v[j]);
            src[3][j] = quad_xor<1>(src[2][j]);
        }
        const double* g = gl + (b - blo) * S * S + lane_q * SL * S;   // this lane's SL rows
        double part = 0.0;
#pragma unroll
        for (int j = 0; j < SL; ++j) {
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int x = 0; x < 4; ++x) {
                const double* gp = g + j * S + (lane_q ^ x) * SL;     // columns of lane lane_q ^ x
                if constexpr (SL == 1) {
                    a0 = fma(gp[0], src[x][0], a0);
                } else {
#pragma unroll
                    for (int jj = 0; jj < SL; jj += 2) {
                        const double2 gg = *(const double2*)(gp + jj);
                        a0 = fma(gg.x, src[x][jj], a0);
                        a1 = fma(gg.y, src[x][jj + 1], a1);
                    }
                }
            }
            v[j] = a0 + a1;
            part += v[j];
        }
        double tot = part + quad_xor<1>(part);
        tot += quad_xor<2>(tot);
        bad |= !(tot > 0.0);
        const double inv = 1.0 / tot;
#pragma unroll
        for (int j = 0; j < SL; ++j) v[j] *= inv;
    }
    msm_steps<K>(v, base, b1 * B, tt + n_in, P, &bad);                // last partial block
    if (!active) return;
    if (bad) atomicOr(err, 1);
#pragma unroll
    for (int j = 0; j < SL; ++j) out[t * S + lane_q * SL + j] = v[j];
}

// ------------------------------------------------------- transfer-matrix scan filter
// Window t's filtered vector is normalise(M_{t+n-1} ... M_t u), M_i = diag(c_i) A, u uniform
// (calc_prob.py:12-13, :51-69).  The steps are cut into blocks of B and the blocks into
// superblocks of C; every window is then ONE product of at most four stored factors
//     Pre_{b1}(e) x SGfull ... x PG/SG (superblock pieces) x Suf_{b0}(t) u,   e = t + n - 1,
// with Pre_b(i) = M_i ... M_{bB} (prefix of i's block), Suf_b(i) = M_{bB+B-1} ... M_i
// (suffix of i's block), PG_s / SG_s the prefix / suffix products of superblock s's block
// products G_b = Pre_b(bB + B - 1).  The prefixes and suffixes are B- and C-step recursions
// run once for all windows (every block / superblock in parallel), so a window costs four
// 2^k x 2^k mat-vecs instead of n filter steps.  All factors are non-negative; each is kept
// at a common scale of its own (a positive factor cancels in the final normalisation), so
// the forecasts agree with the step-by-step filter to ~1e-14 relative.
// B = 16, C = 8 (r03): e2e 16.7-16.8 M -> 18.1-18.4 M VaR-dates/s vs B = 32, C = 16 (profiles/r03p); a
// n_in = 1135 window then takes up to ~10 factors instead of 5, but both serial chains halve
#ifndef CVQ_SCAN_B
#define CVQ_SCAN_B 16
#endif
#ifndef CVQ_SCAN_C
#define CVQ_SCAN_C 8
#endif
constexpr int kScanB = CVQ_SCAN_B;   // steps per block (the block scan's serial chain)
constexpr int kScanC = CVQ_SCAN_C;   // blocks per superblock (the superblock scan's serial chain)

// k = 5, 6 (32 / 64 states, BASELINE config 4's k = 6): the same factorisation with the block
// prefixes left out -- a window runs its last partial block (<= B steps) as filter steps on the
// vector instead of reading a stored S x S prefix per window end (T S^2 doubles: 196 MB at cfg 4)
// -- and the matrices stored column-major so a window's lanes (one state each) read a factor
// column in one coalesced load (k_msm_supscan_w, k_msm_scanwin_w).
template <int K>
constexpr bool kWideScan = K >= 5;

// v <- A v for a quad-resident state vector (the transition of calc_prob.py:91-101 as k
// Kronecker butterflies; A is symmetric, so this is also v^T A for a row vector)
template <int K>
__device__ __forceinline__ void apply_A(double (&v)[Quad<K>::SL], const MsmParams& P) {
    constexpr int SL = Quad<K>::SL, LB = Quad<K>::LB;
#pragma unroll
    for (int c = 0; c < K; ++c) {
        const int pos = K - 1 - c;
        const double pc = P.p[c], qc = P.qv[c];
        if (pos < LB) {
            double nv[SL];
#pragma unroll
            for (int j = 0; j < SL; ++j) nv[j] = pc * v[j] + qc * v[j ^ (1 << pos)];
#pragma unroll
            for (int j = 0; j < SL; ++j) v[j] = nv[j];
        } else {
            const int m = 1 << (pos - LB);
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                const double o = m == 1 ? quad_xor<1>(v[j]) : quad_xor<2>(v[j]);
                v[j] = pc * v[j] + qc * o;
            }
        }
    }
}

template <int K>
__device__ __forceinline__ double quad_max(double m) {
    m = fmax(m, quad_xor<1>(m));
    return fmax(m, quad_xor<2>(m));
}

// Block prefixes (blockIdx.z = 0: quad q = column q of Pre_b(i), forward from e_q) and block
// suffix row sums (z = 1: quad q = row q of Suf_b(i), backward from e_q^T; only Suf_b(i) u is
// ever used, so only its row sums are stored).  The block's conditional densities
// (calc_prob.py:116-117) are computed once into LDS.  Stored: Pre at window ends i >= n_in - 1
// (Pre[(i - n_in + 1)][S][S], row-major), Suf1 at window starts i < T (Suf1[i][S]), the full
// blocks' products G_b (Gf[b][S][S]).  Each step is scaled by 1 / max_s c_i (common to every
// column / row of the block).
template <int K>
__global__ __launch_bounds__(4 << K) void k_msm_blkscan(MsmParamsN PN, const double* __restrict__ r,
                                                        long long N, long long n_in, long long T,
                                                        double* __restrict__ Pre, long long pstride,
                                                        double* __restrict__ Suf1, long long ustride,
                                                        double* __restrict__ Gf, long long gstride, int* flags) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    __shared__ double cl[kScanB * S];                           // c_i[s] of the block's steps
    __shared__ double cm[kScanB];                               // 1 / max_s c_i
    const MsmParams& P = PN.a[blockIdx.y];
    r += blockIdx.y * N;
    const int q = threadIdx.x / L, lane_q = threadIdx.x % L;
    const long long b0 = (long long)blockIdx.x * kScanB;
    const long long b1 = min(b0 + kScanB, N);                    // steps [b0, b1)
    const int nb = (int)(b1 - b0);
    {
        // entry k = tid + 4 S m is step tid / S + 4 m, state tid % S: every return of the block
        // loaded before the first density (one memory latency instead of kScanB / 4)
        constexpr int PER = kScanB / 4;
        const int s = threadIdx.x % S, o0 = threadIdx.x / S;
        double rv[PER];
#pragma unroll
        for (int m = 0; m < PER; ++m) rv[m] = (o0 + 4 * m < nb) ? r[b0 + o0 + 4 * m] : 0.0;
        const double vs = P.vs[s];
#pragma unroll
        for (int m = 0; m < PER; ++m)
            if (o0 + 4 * m < nb) cl[(o0 + 4 * m) * S + s] = cond_prob(rv[m], vs);
    }
    __syncthreads();
    bool bad = false;
    for (int o = threadIdx.x; o < nb; o += blockDim.x) {
        double m = 0.0;
        for (int s2 = 0; s2 < S; ++s2) m = fmax(m, cl[o * S + s2]);
        bad |= !(m > 0.0);                                       // every state's density is 0: calc_prob.py:64-65
        cm[o] = 1.0 / m;
    }
    // this block's error flag, overwritten by every run (no reset launch between runs)
    const int badb = __syncthreads_or(bad);
    if (blockIdx.z == 0 && threadIdx.x == 0) flags[blockIdx.y * gridDim.x + blockIdx.x] = badb ? 1 : 0;
    double v[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = (lane_q * SL + j == q) ? 1.0 : 0.0;
    if (blockIdx.z == 0) {                                       // Pre: columns, forward
        double* pre = Pre + blockIdx.y * pstride;
        for (int o = 0; o < nb; ++o) {
            const long long i = b0 + o;
            const double sc = cm[o];
            apply_A<K>(v, P);
#pragma unroll
            for (int j = 0; j < SL; ++j) v[j] = v[j] * (cl[o * S + lane_q * SL + j] * sc);
            if (!kWideScan<K> && i >= n_in - 1) {
                double* dst = pre + ((i - (n_in - 1)) * S + lane_q * SL) * S + q;
#pragma unroll
                for (int j = 0; j < SL; ++j) dst[j * S] = v[j];
            }
            if (o == kScanB - 1) {                               // a full block's product G_b
                if constexpr (kWideScan<K>) {                    // column-major: column q is contiguous
                    double* dst = Gf + blockIdx.y * gstride + (blockIdx.x * (long long)S + q) * S + lane_q * SL;
#pragma unroll
                    for (int j = 0; j < SL; ++j) dst[j] = v[j];
                } else {
                    double* dst = Gf + blockIdx.y * gstride + (blockIdx.x * (long long)S + lane_q * SL) * S + q;
#pragma unroll
                    for (int j = 0; j < SL; ++j) dst[j * S] = v[j];
                }
            }
        }
    } else {                                                     // Suf: rows, backward
        double* suf = Suf1 + blockIdx.y * ustride;
        for (int o = nb - 1; o >= 0; --o) {
            const long long i = b0 + o;
            const double sc = cm[o];
#pragma unroll
            for (int j = 0; j < SL; ++j) v[j] = v[j] * (cl[o * S + lane_q * SL + j] * sc);
            apply_A<K>(v, P);                                    // row q of Suf_b(i) = row q of Suf_b(i+1) diag(c_i) A
            if (i < T) {
                double rs = 0.0;
#pragma unroll
                for (int j = 0; j < SL; ++j) rs += v[j];
                rs += quad_xor<1>(rs);
                rs += quad_xor<2>(rs);
                if (lane_q == 0) suf[i * S + q] = rs;
            }
        }
    }
}

// Superblock prefixes PG_s(beta) = G_{sC+beta} ... G_{sC} (z = 0, quad = column, forward) and
// suffixes SG_s(beta) = G_{last} ... G_{sC+beta} (z = 1, quad = row, backward) of the block
// products G_b (k_msm_blkscan's Gf), staged in LDS.  One wavefront per (superblock, asset,
// direction) for K = 4 (16 quads): the common scale of each stored matrix is its maximum over
// the wave.
template <int K>
__global__ __launch_bounds__(4 << K) void k_msm_supscan(const double* __restrict__ Gf, long long gstride,
                                                        long long nfull, double* __restrict__ PG,
                                                        double* __restrict__ SG, long long sstride) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    static_assert((4 << K) <= 64, "one wavefront per scan");
    __shared__ __attribute__((aligned(16))) double gl[kScanC * S * S];
    const int q = threadIdx.x / L, lane_q = threadIdx.x % L;
    const long long s0 = (long long)blockIdx.x * kScanC;
    const long long s1 = min(s0 + kScanC, nfull);
    Gf += blockIdx.y * gstride;
    {
        // the superblock's block products (kScanC S^2 doubles, 2 S double2 per thread): every
        // load issued before the first LDS store (one memory latency instead of 2 S in a row)
        constexpr int PER = kScanC * S * S / 2 / (4 * S);
        const double2* src = (const double2*)(Gf + s0 * S * S);
        double2* dst = (double2*)gl;
        const int nv = (int)((s1 - s0) * S * S / 2);
        double2 tmp[PER];
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = threadIdx.x + m * 4 * S;
            tmp[m] = k < nv ? src[k] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int m = 0; m < PER; ++m) {
            const int k = threadIdx.x + m * 4 * S;
            if (k < nv) dst[k] = tmp[m];
        }
    }
    __syncthreads();
    double v[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) v[j] = (lane_q * SL + j == q) ? 1.0 : 0.0;
    auto wave_max = [](double m) {
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) m = fmax(m, __shfl_xor(m, o, 64));
        return m;
    };
    if (blockIdx.z == 0) {                                       // columns: x <- G_b x
        double* dst0 = PG + blockIdx.y * sstride + blockIdx.x * (long long)kScanC * S * S;
        for (long long b = s0; b < s1; ++b) {
            const double* G = gl + (b - s0) * S * S;
            double nv[SL];
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                const double* row = G + (lane_q * SL + j) * S;
                double acc = 0.0;
#pragma unroll
                for (int c = 0; c < S; ++c) {
                    const double xc = __shfl(v[c % SL], (threadIdx.x & ~(L - 1)) + c / SL, 64);
                    acc = fma(row[c], xc, acc);
                }
                nv[j] = acc;
            }
            double m = 0.0;
#pragma unroll
            for (int j = 0; j < SL; ++j) m = fmax(m, nv[j]);
            const double sc = 1.0 / wave_max(m);
            double* dst = dst0 + (b - s0) * S * S;
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                v[j] = nv[j] * sc;
                dst[(lane_q * SL + j) * S + q] = v[j];
            }
        }
    } else {                                                     // rows: y^T <- y^T G_b
        double* dst0 = SG + blockIdx.y * sstride + blockIdx.x * (long long)kScanC * S * S;
        for (long long b = s1 - 1; b >= s0; --b) {
            const double* G = gl + (b - s0) * S * S;
            double nv[SL];
#pragma unroll
            for (int j = 0; j < SL; ++j) {                       // y_c = sum_r y_r G[r][c], c = lane_q*SL + j
                const int c = lane_q * SL + j;
                double acc = 0.0;
#pragma unroll
                for (int rr = 0; rr < S; ++rr) {
                    const double yr = __shfl(v[rr % SL], (threadIdx.x & ~(L - 1)) + rr / SL, 64);
                    acc = fma(yr, G[rr * S + c], acc);
                }
                nv[j] = acc;
            }
            double m = 0.0;
#pragma unroll
            for (int j = 0; j < SL; ++j) m = fmax(m, nv[j]);
            const double sc = 1.0 / wave_max(m);
            double* dst = dst0 + (b - s0) * S * S;
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                v[j] = nv[j] * sc;
                dst[q * S + lane_q * SL + j] = v[j];
            }
        }
    }
}

// Windows: 16 lanes per window (one matrix row each; the whole vector in every lane) ->
// filtered vector -> collapsed onto the asset's unique vols (sum_forecast_by_state,
// msm_estimation.py:205-248, Q14: states in order) straight into fbs[t][d][u].  The window's
// factors (<= 4 for n_in >> B C, their addresses known up front) are loaded one ahead.
template <int K>
__global__ __launch_bounds__(256) void k_msm_scanwin(const double* __restrict__ Pre, long long pstride,
                                                     const double* __restrict__ Suf1, long long ustride,
                                                     const double* __restrict__ Gf, long long gstride,
                                                     const double* __restrict__ PG, const double* __restrict__ SG,
                                                     long long sstride, long long nfull, long long n_in, long long T,
                                                     StateMapQ M, int dim, double* __restrict__ fbs) {
    constexpr int S = 1 << K;
    static_assert(S <= 16, "one matrix row per lane of a 16-lane group");
    const int g = threadIdx.x % 16;
    const long long t = (long long)blockIdx.x * (blockDim.x / 16) + threadIdx.x / 16;
    const bool active = t < T;
    const long long tt = active ? t : T - 1;
    const int d = blockIdx.y;
    Pre += d * pstride;
    Suf1 += d * ustride;
    Gf += d * gstride;
    PG += d * sstride;
    SG += d * sstride;
    const int row = g < S ? g : 0;
    const long long e = tt + n_in - 1;
    const long long lo_b = tt / kScanB + 1, hi_b = e / kScanB - 1;   // full blocks strictly between
    const long long sa = lo_b / kScanC, sb = hi_b / kScanC;
    // the chain of factors applied to Suf_{b0}(t) u, first to last
    int kind;                                                    // 0 none, 1 PG only, 2 SG only, 3 loose, 4 spread
    long long cnt;
    if (lo_b > hi_b) { kind = 0; cnt = 1; }
    else if (sa == sb) {
        const long long send = min(sa * kScanC + kScanC, nfull) - 1;
        kind = lo_b == sa * kScanC ? 1 : (hi_b == send ? 2 : 3);
        cnt = kind == 3 ? hi_b - lo_b + 2 : 2;
    } else { kind = 4; cnt = (sb - sa + 1) + 1; }
    auto mat = [&](long long k) -> const double* {
        if (k == cnt - 1) return Pre + (e - (n_in - 1)) * S * S;
        switch (kind) {
            case 1: return PG + (sa * kScanC + (hi_b - sa * kScanC)) * S * S;
            case 2: return SG + (sa * kScanC + (lo_b - sa * kScanC)) * S * S;
            case 3: return Gf + (lo_b + k) * S * S;
            default:
                if (k == 0) return SG + (sa * kScanC + (lo_b - sa * kScanC)) * S * S;
                if (k == cnt - 2) return PG + (sb * kScanC + (hi_b - sb * kScanC)) * S * S;
                return SG + ((sa + k) * kScanC) * S * S;      // full superblock sa + k
        }
    };
    // the first kPre factors' rows and Suf_{b0}(t) u are loaded together (one memory latency;
    // n_in = 1135 windows take 3-4 factors), later factors one ahead of their use
    constexpr int kPre = 4;
    double x[S], fm[kPre][S];
#pragma unroll
    for (int c = 0; c < S; ++c) x[c] = Suf1[tt * S + c];         // Suf_{b0}(t) u, up to a factor
#pragma unroll
    for (int k = 0; k < kPre; ++k) {
        const double* m = mat(k < cnt ? k : 0) + row * S;
#pragma unroll
        for (int c = 0; c < S; ++c) fm[k][c] = m[c];
    }
    {
        double tot = 0.0;
#pragma unroll
        for (int c = 0; c < S; ++c) tot += x[c];
        const double inv = 1.0 / tot;
#pragma unroll
        for (int c = 0; c < S; ++c) x[c] *= inv;
    }
    auto apply = [&](const double (&cur)[S]) {                   // x <- normalise(F x)
        double y = 0.0;
#pragma unroll
        for (int c = 0; c < S; ++c) y = fma(cur[c], x[c], y);
        double tot = 0.0;
#pragma unroll
        for (int c = 0; c < S; ++c) {
            x[c] = __shfl(y, (threadIdx.x & ~15) + c, 64);
            tot += x[c];
        }
        const double inv = 1.0 / tot;
#pragma unroll
        for (int c = 0; c < S; ++c) x[c] *= inv;
    };
#pragma unroll
    for (int k = 0; k < kPre; ++k)
        if (k < cnt) apply(fm[k]);
    if (cnt > kPre) {
        double cur[S], nxt[S];
        {
            const double* m0 = mat(kPre) + row * S;
#pragma unroll
            for (int c = 0; c < S; ++c) cur[c] = m0[c];
        }
        for (long long k = kPre; k < cnt; ++k) {
            if (k + 1 < cnt) {
                const double* m1 = mat(k + 1) + row * S;
#pragma unroll
                for (int c = 0; c < S; ++c) nxt[c] = m1[c];
            }
            apply(cur);
#pragma unroll
            for (int c = 0; c < S; ++c) cur[c] = nxt[c];
        }
    }
    if (!active || g >= M.q) return;
    double f = 0.0;
#pragma unroll
    for (int c = 0; c < S; ++c) f += M.u[d][c] == g ? x[c] : 0.0;
    fbs[(t * dim + d) * M.q + g] = f;
}

// Superblock prefix / suffix products for 32 or 64 states: the running product X (S x S, a
// (S/16) x (S/16) block per thread of 256) times the next block product G_b staged in LDS
// (rows padded by one double: a column read by the 16 block-rows of a wave hits 16 banks),
// then scaled by its maximum over the workgroup.  z = 0: PG_s(beta) = G_{sC+beta} ... G_{sC}
// (X <- G X); z = 1: SG_s(beta) = G_{last} ... G_{sC+beta} (X <- X G).  Column-major I/O.
template <int K>
__global__ __launch_bounds__(256) void k_msm_supscan_w(const double* __restrict__ Gf, long long gstride,
                                                       long long nfull, double* __restrict__ PG,
                                                       double* __restrict__ SG, long long sstride) {
    constexpr int S = 1 << K, SP = S + 2, RB = S / 16;      // RB x RB block of X per thread
    static_assert(RB % 2 == 0, "16-B LDS reads of pairs");
    __shared__ __attribute__((aligned(16))) double Gs[S * SP], Xs[S * SP];
    __shared__ double wmax[4];
    const int tid = threadIdx.x, br = tid / 16, bc = tid % 16;
    const long long s0 = (long long)blockIdx.x * kScanC, s1 = min(s0 + kScanC, nfull);
    Gf += blockIdx.y * gstride;
    double* out = (blockIdx.z == 0 ? PG : SG) + blockIdx.y * sstride;
    double x[RB][RB];
#pragma unroll
    for (int a = 0; a < RB; ++a)
#pragma unroll
        for (int b = 0; b < RB; ++b) x[a][b] = (br * RB + a == bc * RB + b) ? 1.0 : 0.0;
    const bool fwd = blockIdx.z == 0;
    constexpr int GE = S * S / 256;
    double gn[GE];                                               // the next block product, loaded a step ahead
    const long long nst = s1 - s0;
    auto gload = [&](long long it) {
        const double* G = Gf + (fwd ? s0 + it : s1 - 1 - it) * S * S;   // column-major: G[c * S + r] = G_b(r, c)
#pragma unroll
        for (int m = 0; m < GE; ++m) gn[m] = G[tid + 256 * m];
    };
    if (nst > 0) gload(0);
    for (long long it = 0; it < nst; ++it) {
        const long long bidx = fwd ? s0 + it : s1 - 1 - it;
#pragma unroll
        for (int m = 0; m < GE; ++m) {
            const int e = tid + 256 * m, c = e / S, r = e % S;
            Gs[r * SP + c] = gn[m];
        }
        if (it + 1 < nst) gload(it + 1);
#pragma unroll
        for (int a = 0; a < RB; ++a)
#pragma unroll
            for (int b = 0; b < RB; ++b) Xs[(br * RB + a) * SP + bc * RB + b] = x[a][b];
        __syncthreads();
        double y[RB][RB];
#pragma unroll
        for (int a = 0; a < RB; ++a)
#pragma unroll
            for (int b = 0; b < RB; ++b) y[a][b] = 0.0;
        // forward Y = G X: u = G(i, c), w = X(c, j); backward Y = X G: u = X(i, c), w = G(c, j);
        // two c per round, every operand a 16-B LDS read (rows padded to S + 2: aligned pairs,
        // the 4 block-rows of a wave on distinct banks)
        const double* U = fwd ? Gs : Xs;
        const double* W = fwd ? Xs : Gs;
#pragma unroll 2
        for (int c = 0; c < S; c += 2) {
            double2 u[RB], w0[RB / 2], w1[RB / 2];
#pragma unroll
            for (int a = 0; a < RB; ++a) u[a] = *(const double2*)&U[(br * RB + a) * SP + c];
#pragma unroll
            for (int b = 0; b < RB / 2; ++b) {
                w0[b] = *(const double2*)&W[c * SP + bc * RB + 2 * b];
                w1[b] = *(const double2*)&W[(c + 1) * SP + bc * RB + 2 * b];
            }
#pragma unroll
            for (int a = 0; a < RB; ++a)
#pragma unroll
                for (int b = 0; b < RB / 2; ++b) {
                    y[a][2 * b] = fma(u[a].x, w0[b].x, y[a][2 * b]);
                    y[a][2 * b + 1] = fma(u[a].x, w0[b].y, y[a][2 * b + 1]);
                    y[a][2 * b] = fma(u[a].y, w1[b].x, y[a][2 * b]);
                    y[a][2 * b + 1] = fma(u[a].y, w1[b].y, y[a][2 * b + 1]);
                }
        }
        double m = 0.0;
#pragma unroll
        for (int a = 0; a < RB; ++a)
#pragma unroll
            for (int b = 0; b < RB; ++b) m = fmax(m, y[a][b]);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) m = fmax(m, __shfl_xor(m, o, 64));
        if ((tid & 63) == 0) wmax[tid >> 6] = m;
        __syncthreads();                                         // also: every read of Gs / Xs is done
        const double sc = 1.0 / fmax(fmax(wmax[0], wmax[1]), fmax(wmax[2], wmax[3]));
        double* dst = out + bidx * S * S;
#pragma unroll
        for (int a = 0; a < RB; ++a)
#pragma unroll
            for (int b = 0; b < RB; ++b) {
                x[a][b] = y[a][b] * sc;
                dst[(bc * RB + b) * S + br * RB + a] = x[a][b];
            }
        __syncthreads();                                         // wmax is rewritten by the next step
    }
}

// Windows for 32 or 64 states, 16 consecutive windows per workgroup (t0 = 16 g: one start
// block b0, so one lo_b, and ends in at most two blocks).  Lane s of each wave = state s, a wave
// holds 4 windows.  Per window: its first partial block [t, (b0 + 1) B) as filter steps from the
// uniform prior (calc_prob.py:12-13, 51-69: butterflies by lane xor, c_i from the returns), the
// full blocks lo_b .. H shared by the group (H = the group's smallest hi_b; each factor staged
// once in LDS, column-major, and applied to all 16 vectors), one more block product G_{H+1} for
// the windows whose hi_b = H + 1, then its last partial block [b1 B, e] as filter steps, and the
// collapse onto the asset's unique vols in state order (Q14) into fbs.  Every vector normalised
// after each factor / step (positive factors cancel).
constexpr int kWinGroup = 16;                                    // windows per workgroup = kScanB
#ifndef CVQ_SCAN_STEP_NORM
#define CVQ_SCAN_STEP_NORM 4       // partial-block filter steps between normalisations (1: every step)
#endif
template <int K>
__global__ __launch_bounds__(256) void k_msm_scanwin_w(MsmParamsN PN, const double* __restrict__ r, long long N,
                                                       const double* __restrict__ Gf, long long gstride,
                                                       const double* __restrict__ PG, const double* __restrict__ SG,
                                                       long long sstride, long long nfull, long long n_in,
                                                       long long T, StateMap M, int q, int dim,
                                                       double* __restrict__ fbs) {
    constexpr int S = 1 << K, WPW = 4;                           // states, windows per wave
    static_assert(S <= 64 && kWinGroup == 4 * WPW && kWinGroup == kScanB, "16 windows, one start block");
    __shared__ __attribute__((aligned(16))) double Fs[S * S];    // the factor, column-major
    __shared__ __attribute__((aligned(16))) double xs[4][S][WPW];   // per wave: x_m[c] of its 4 windows
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, s = lane < S ? lane : 0;
    const bool act = lane < S;
    const int d = blockIdx.y;
    const MsmParams& P = PN.a[d];
    r += d * N;
    Gf += d * gstride;
    PG += d * sstride;
    SG += d * sstride;
    const long long t0 = (long long)blockIdx.x * kWinGroup;
    long long tw[WPW];
    bool live[WPW];
#pragma unroll
    for (int m = 0; m < WPW; ++m) {
        tw[m] = t0 + wv * WPW + m;
        live[m] = tw[m] < T;
    }
    double x[WPW];
    auto wsum = [&](double v) { return wave_total(act ? v : 0.0); };   // over the wave's S state lanes
    // filter steps i in [i0, i1) (i1 - i0 <= 64) for window m when i lies in its range [a_m, b_m);
    // the returns r[i0 ..] are loaded once, one per lane, and broadcast by readlane.  A vector is
    // normalised every kStepNorm steps and at its range's last step (positive scale factors cancel,
    // as between the block products; four unnormalised steps stay far inside the double range), so
    // three of four steps skip the wave-wide sum that otherwise closes every step's chain
    constexpr int kStepNorm = CVQ_SCAN_STEP_NORM;
    auto steps = [&](long long i0, long long i1, const long long (&a)[WPW], const long long (&b)[WPW]) {
        const double rl = (i0 + lane < i1) ? r[i0 + lane] : 0.0;
#pragma unroll 1
        for (long long i = i0; i < i1; ++i) {
            const int li = (int)(i - i0);
            const double ri = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(rl), li),
                                               __builtin_amdgcn_readlane(__double2loint(rl), li));
            const double ci = act ? cond_prob(ri, P.vs[s]) : 0.0;
#pragma unroll
            for (int m = 0; m < WPW; ++m) {
                const bool on = i >= a[m] && i < b[m];           // wave-uniform
                double v = x[m];
                auto bfly = [&](auto cc) {                       // component c <-> state bit K-1-c
                    constexpr int c = decltype(cc)::value;
                    const double o = lane_xor<(1 << (K - 1 - c))>(v);
                    v = P.p[c] * v + P.qv[c] * o;
                };
                bfly(std::integral_constant<int, 0>{});
                bfly(std::integral_constant<int, 1>{});
                bfly(std::integral_constant<int, 2>{});
                bfly(std::integral_constant<int, 3>{});
                bfly(std::integral_constant<int, 4>{});
                if constexpr (K == 6) bfly(std::integral_constant<int, 5>{});
                v *= ci;
                if ((li % kStepNorm) == kStepNorm - 1 || i == b[m] - 1) {   // wave-uniform
                    const double tot = wsum(v);
                    v = v * (1.0 / tot);
                }
                if (on) x[m] = v;
            }
        }
    };
    // 1. first partial block: [t, (b0 + 1) B) from the uniform prior
    const long long b0 = t0 / kScanB, bend = (b0 + 1) * kScanB;
    {
        long long a[WPW], b[WPW];
#pragma unroll
        for (int m = 0; m < WPW; ++m) {
            x[m] = 1.0 / S;
            a[m] = tw[m];
            b[m] = bend;
        }
        steps(a[0], bend, a, b);       // this wave's first window starts at a[0]
    }
    // 2. full blocks lo_b .. H (shared), then G_{H+1} for the windows with hi_b = H + 1
    const long long lo_b = b0 + 1, H = (t0 + n_in - 1) / kScanB - 1;
    long long hib[WPW];
#pragma unroll
    for (int m = 0; m < WPW; ++m) hib[m] = (tw[m] + n_in - 1) / kScanB - 1;
    const long long sa = lo_b / kScanC, sb = H / kScanC;
    int kind;                                                    // as k_msm_scanwin, for (lo_b, H)
    long long cnt;
    if (lo_b > H) { kind = 0; cnt = 0; }
    else if (sa == sb) {
        const long long send = min(sa * kScanC + kScanC, nfull) - 1;
        kind = lo_b == sa * kScanC ? 1 : (H == send ? 2 : 3);
        cnt = kind == 3 ? H - lo_b + 1 : 1;
    } else { kind = 4; cnt = sb - sa + 1; }
    auto mat = [&](long long k) -> const double* {
        if (k == cnt) return Gf + (H + 1) * S * S;               // the extra block (some windows)
        switch (kind) {
            case 1: return PG + (sa * kScanC + (H - sa * kScanC)) * S * S;
            case 2: return SG + (sa * kScanC + (lo_b - sa * kScanC)) * S * S;
            case 3: return Gf + (lo_b + k) * S * S;
            default:
                if (k == 0) return SG + (sa * kScanC + (lo_b - sa * kScanC)) * S * S;
                if (k == cnt - 1) return PG + (sb * kScanC + (H - sb * kScanC)) * S * S;
                return SG + ((sa + k) * kScanC) * S * S;          // full superblock sa + k
        }
    };
    bool extra = false;                                          // any window of the group needs G_{H+1}
#pragma unroll
    for (int m = 0; m < WPW; ++m) extra |= live[m] && hib[m] == H + 1;
    extra = __syncthreads_or(extra);
    const long long nf = cnt + (extra ? 1 : 0);
    constexpr int FE = S * S / 256;                              // factor entries per thread
    double fn[FE];                                               // the next factor, loaded a factor ahead
    if (nf > 0) {
        const double* F = mat(0);
#pragma unroll
        for (int e = 0; e < FE; ++e) fn[e] = F[tid + 256 * e];
    }
    for (long long k = 0; k < nf; ++k) {
#pragma unroll
        for (int e = 0; e < FE; ++e) Fs[tid + 256 * e] = fn[e];
        if (k + 1 < nf) {
            const double* F = mat(k + 1);
#pragma unroll
            for (int e = 0; e < FE; ++e) fn[e] = F[tid + 256 * e];
        }
        if (act) {
#pragma unroll
            for (int m = 0; m < WPW; ++m) xs[wv][s][m] = x[m];
        }
        __syncthreads();
        double y[WPW] = {};
#pragma unroll 4
        for (int c = 0; c < S; ++c) {
            const double f = Fs[c * S + s];
            const double2 x01 = *(const double2*)&xs[wv][c][0];  // broadcast reads
            const double2 x23 = *(const double2*)&xs[wv][c][2];
            y[0] = fma(f, x01.x, y[0]);
            y[1] = fma(f, x01.y, y[1]);
            y[2] = fma(f, x23.x, y[2]);
            y[3] = fma(f, x23.y, y[3]);
        }
#pragma unroll
        for (int m = 0; m < WPW; ++m) {
            const double tot = wsum(y[m]);
            if (k < cnt || hib[m] == H + 1) x[m] = y[m] * (1.0 / tot);
        }
        __syncthreads();                                         // Fs / xs rewritten by the next factor
    }
    // 3. last partial block [b1 B, e] of each window
    {
        long long a[WPW], b[WPW], lo = 1LL << 62, hi = 0;
#pragma unroll
        for (int m = 0; m < WPW; ++m) {
            const long long e = tw[m] + n_in - 1;
            a[m] = (e / kScanB) * kScanB;
            b[m] = live[m] ? e + 1 : a[m];
            lo = min(lo, a[m]);
            hi = max(hi, b[m]);
        }
        if (hi > lo) steps(lo, hi, a, b);
    }
    // 4. collapse onto unique vols, states in order (Q14): lane u < q of the wave sums its
    // windows' states mapped to u (the vectors through LDS; the last barrier freed xs)
    if (act) {
#pragma unroll
        for (int m = 0; m < WPW; ++m) xs[wv][s][m] = x[m];
    }
    __syncthreads();
    if (lane < q) {
        double f[WPW] = {};
#pragma unroll 1
        for (int c = 0; c < S; ++c) {
            if (M.u[d][c] != lane) continue;
#pragma unroll
            for (int m = 0; m < WPW; ++m) f[m] += xs[wv][c][m];
        }
#pragma unroll
        for (int m = 0; m < WPW; ++m)
            if (live[m]) fbs[(tw[m] * dim + d) * q + lane] = f[m];
    }
}

// sum_forecast_by_state (msm_estimation.py:205-248, Q14) + compute_forecast_combinations
// (:392-418, Q7) on the device.  filt [dim][T][S] -> fbs [T][dim][q]
// (states collapsed onto their unique 1e-6-rounded vol, summed in state order) and
// pi [T][q^dim] in the reference's xy-meshgrid product order (2-D: f0[a] f1[b];
// 3-D: (f0[L1] f1[L2]) f2[L0]).
// One thread per output: k_msm_fbs, thread per (date, asset), the
// states of its filtered vector summed onto their unique vols in state order; k_msm_pi,
// thread per (date, combination), the product in the reference's meshgrid order.
__global__ void k_msm_fbs(StateMap M, int dim, int S, int q, const double* __restrict__ filt, long long T,
                          double* __restrict__ fbs) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T * dim) return;
    const long long t = idx / dim;
    const int d = (int)(idx % dim);
    double f[8];
    for (int u = 0; u < q; ++u) f[u] = 0.0;
    const double* row = filt + ((long long)d * T + t) * S;
    for (int s2 = 0; s2 < S; ++s2) f[M.u[d][s2]] += row[s2];
    for (int u = 0; u < q; ++u) fbs[(t * dim + d) * q + u] = f[u];
}

__global__ void k_msm_pi(int dim, int q, const double* __restrict__ fbs, long long T, double* __restrict__ pi) {
    const int Q = dim == 2 ? q * q : q * q * q;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= T * Q) return;
    const long long t = idx / Q;
    const int l = (int)(idx % Q);
    const double* f = fbs + t * dim * q;
    if (dim == 2) {
        pi[idx] = f[l / q] * f[q + l % q];
    } else {
        const int L0 = l / (q * q), L1 = (l / q) % q, L2 = l % q;
        pi[idx] = (f[L1] * f[q + L2]) * f[2 * q + L0];
    }
}

// Batched MSM log-likelihood (calc_prob.py:134-142 -> :36-47): one quad per candidate.
template <int K>
__global__ __launch_bounds__(256) void k_msm_loglik(const MsmParams* __restrict__ Ps, long long B,
                                                    const double* __restrict__ r, long long N, double* __restrict__ out) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long bi = gid / L;
    const int lane_q = (int)(gid % L);
    const bool active = bi < B;
    const MsmParams& P = Ps[active ? bi : B - 1];
    double v[SL], vs[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) { v[j] = 1.0 / S; vs[j] = P.vs[lane_q * SL + j]; }
    double LL = 0.0;
    bool dead = false;
    for (long long i = 0; i < N; ++i) {
        double cv[SL];
        const double ri = r[i];
#pragma unroll
        for (int j = 0; j < SL; ++j) cv[j] = cond_prob(ri, vs[j]);
        bool z;
        const double tot = msm_step<K>(v, cv, P, &z);
        if (i >= 1) {
            if (!(tot > 0.0)) dead = true; else LL += log(tot);
        }
        if (z) dead = true;
    }
    if (active && lane_q == 0) out[bi] = dead ? -__builtin_huge_val() : LL;
}

// scipy.special.ndtr (norm.cdf, calc_prob.py:128): the erf form near 0, the erfc tail beyond
// |x| / sqrt 2 >= 1 / sqrt 2, as cephes' ndtr evaluates it (relative accuracy in both tails).
__device__ __forceinline__ double ndtr_dev(double a) {
    const double x = a * 0.70710678118654752440, z = fabs(x);
    if (z < 0.70710678118654752440) return 0.5 + 0.5 * erf(x);
    const double y = 0.5 * erfc(z);
    return x > 0.0 ? 1.0 - y : y;
}

// In-sample MSM marginals and densities (calc_marginals.py:7-30, the copula fit's inputs):
// the filtered state probabilities of every step (calc_prob.py:51-69, normalised by IEEE
// division as the reference does) weighted by the conditional CDF / pdf of the PREVIOUS return,
//   marg[i - 1] = sum_s prob[i][s] ndtr(r[i-1] / vs_s),  dens[i - 1] = sum_s prob[i][s] pdf(r[i-1]; vs_s),
// i = 1 .. N - 1 (state_prob_t[1:] * cond_marg_vect[:-1]).  One quad (L lanes) per series
// (blockIdx.x): the steps are a dependent chain; the state sums reduce by quad DPP.
template <int K>
__global__ void k_msm_marginals(MsmParams P, const double* __restrict__ r, long long N, double* __restrict__ marg,
                                double* __restrict__ dens, int* err) {
    constexpr int S = Quad<K>::S, L = Quad<K>::L, SL = Quad<K>::SL;
    const int lane_q = threadIdx.x;                    // blockDim.x == L
    double v[SL], vs[SL];
#pragma unroll
    for (int j = 0; j < SL; ++j) {
        v[j] = 1.0 / S;                                // equi_prob (calc_prob.py:12-13)
        vs[j] = P.vs[lane_q * SL + j];
    }
    bool bad = false;
    double rprev = 0.0;
    for (long long i = 0; i < N; ++i) {
        const double ri = r[i];
        double cv[SL];
#pragma unroll
        for (int j = 0; j < SL; ++j) cv[j] = cond_prob(ri, vs[j]);
        bool z;
        msm_step<K, true>(v, cv, P, &z);
        bad |= z;
        if (i >= 1) {
            double pm = 0.0, pd = 0.0;
#pragma unroll
            for (int j = 0; j < SL; ++j) {
                pm += v[j] * ndtr_dev(rprev / vs[j]);
                pd += v[j] * cond_prob(rprev, vs[j]);
            }
            if (L >= 2) { pm += quad_xor<1>(pm); pd += quad_xor<1>(pd); }
            if (L >= 4) { pm += quad_xor<2>(pm); pd += quad_xor<2>(pd); }
            if (lane_q == 0) {
                marg[i - 1] = pm;
                dens[i - 1] = pd;
            }
        }
        rprev = ri;
    }
    if (bad && lane_q == 0) atomicOr(err, 1);
}

// ----------------------------------------------------------------- GARCH(1,1)
__global__ void k_garch_forecast(double omega, double alpha, double beta, const double* __restrict__ r,
                                 long long n_in, long long T, double* __restrict__ out) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const double* w = r + t;
    double s2 = omega / (1 - alpha - beta);                     // estimation.py:52
    for (long long i = 1; i < n_in; ++i) {
        double v = omega + alpha * (w[i - 1] * w[i - 1]);
        v = v + beta * s2;
        s2 = (1e-7 > v) ? 1e-7 : v;                             // max(sigma2, epsilon)
    }
    const double rl = w[n_in - 1];
    out[t] = sqrt(omega + alpha * (rl * rl) + beta * s2);      // forecast.py:14-19
}

__global__ void k_garch_loglik(const double* __restrict__ prm, long long B, const double* __restrict__ r, long long N,
                               double* __restrict__ out) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const double omega = prm[3 * b], alpha = prm[3 * b + 1], beta = prm[3 * b + 2];
    double s2 = omega / (1 - alpha - beta);
    double acc = 0.0;
    for (long long i = 1; i < N; ++i) {
        double v = omega + alpha * (r[i - 1] * r[i - 1]);
        v = v + beta * s2;
        s2 = (1e-7 > v) ? 1e-7 : v;
        acc += log(2 * M_PI * s2) + (r[i] * r[i]) / s2;          // estimation.py:118-123
    }
    out[b] = -0.5 * acc;
}

// GARCH(p, q) log-likelihood of numba_garch_log_likelihood (garch/estimation.py:91-125)
// for a batch of parameter rows [omega, alpha_1..alpha_p, beta_1..beta_q], one
// thread per row: sigma2[0] = omega / (1 - sum(alpha) - sum(beta)); sigma2[t] =
// max(omega + sum_{i < min(p,t)} alpha_i r[t-i-1]^2 + sum_{j < min(q,t)} beta_j
// sigma2[t-j-1], 1e-7); LL = -0.5 sum_{t >= max(p,q)} log(2 pi sigma2_t) + r_t^2 / sigma2_t.
// The last q variances live in a register ring (P, Q <= kGarchMaxPQ).
constexpr int kGarchMaxPQ = 4;
template <int P, int Q>
__global__ void k_garch_loglik_pq(const double* __restrict__ prm, long long B, const double* __restrict__ r,
                                  long long N, double* __restrict__ out) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const double* pr = prm + b * (1 + P + Q);
    const double omega = pr[0];
    double alpha[P], beta[Q], sa = 0.0, sb = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) { alpha[i] = pr[1 + i]; sa += alpha[i]; }
#pragma unroll
    for (int j = 0; j < Q; ++j) { beta[j] = pr[1 + P + j]; sb += beta[j]; }
    double hist[Q];                                   // hist[j] = sigma2[t - 1 - j]
#pragma unroll
    for (int j = 0; j < Q; ++j) hist[j] = 0.0;
    hist[0] = omega / (1 - sa - sb);                  // estimation.py:106 (np.sum order)
    constexpr int M = P > Q ? P : Q;                  // extra_size: chopped prefix (:119-121)
    double acc = 0.0;
    for (long long t = 1; t < N; ++t) {
        double v = omega;
#pragma unroll
        for (int i = 0; i < P; ++i)
            if (i < t) v += alpha[i] * (r[t - i - 1] * r[t - i - 1]);
#pragma unroll
        for (int j = 0; j < Q; ++j)
            if (j < t) v += beta[j] * hist[j];
        const double s2 = (v < 1e-7) ? 1e-7 : v;      // max(sigma2[t], epsilon)
#pragma unroll
        for (int j = Q - 1; j > 0; --j) hist[j] = hist[j - 1];
        hist[0] = s2;
        if (t >= M) acc += log(2 * M_PI * s2) + (r[t] * r[t]) / s2;
    }
    out[b] = -0.5 * acc;
}

// GARCH(p, q) calc_forecast (garch/forecast.py:5-19) per window t of n_in returns
// (one thread per window): the variance recursion above, then
// sqrt((omega + sum_i alpha_i r[n-p+i]^2) + sum_j beta_j sigma2[n-q+j]) -- note the
// reference pairs alpha_1 with the OLDEST of the last p returns (returns[-p:]).
template <int P, int Q>
__global__ void k_garch_forecast_pq(const double* __restrict__ prm, const double* __restrict__ r, long long n_in,
                                    long long T, double* __restrict__ out) {
    const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 >= T) return;
    const double* w = r + t0;
    const double omega = prm[0];
    double alpha[P], beta[Q], sa = 0.0, sb = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) { alpha[i] = prm[1 + i]; sa += alpha[i]; }
#pragma unroll
    for (int j = 0; j < Q; ++j) { beta[j] = prm[1 + P + j]; sb += beta[j]; }
    double hist[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) hist[j] = 0.0;
    hist[0] = omega / (1 - sa - sb);
    for (long long t = 1; t < n_in; ++t) {
        double v = omega;
#pragma unroll
        for (int i = 0; i < P; ++i)
            if (i < t) v += alpha[i] * (w[t - i - 1] * w[t - i - 1]);
#pragma unroll
        for (int j = 0; j < Q; ++j)
            if (j < t) v += beta[j] * hist[j];
        const double s2 = (v < 1e-7) ? 1e-7 : v;
#pragma unroll
        for (int j = Q - 1; j > 0; --j) hist[j] = hist[j - 1];
        hist[0] = s2;
    }
    double s_a = 0.0, s_b = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const double ri = w[n_in - P + i];
        s_a = (i == 0) ? alpha[i] * (ri * ri) : s_a + alpha[i] * (ri * ri);
    }
#pragma unroll
    for (int j = 0; j < Q; ++j) s_b = (j == 0) ? beta[j] * hist[Q - 1] : s_b + beta[j] * hist[Q - 1 - j];
    out[t0] = sqrt((omega + s_a) + s_b);
}

// Device-resident sigma stage (cvq_sigma_tables): the same recursion for one asset of a
// batch, parameters by value, the forecast written straight into the solve's
// integrations_params_t layout out[t * ostride] (ostride = dim).
struct GarchPrm {
    double v[1 + 2 * 4];
};

template <int P, int Q>
__global__ void k_garch_sigma(GarchPrm G, const double* __restrict__ r, long long n_in, long long T,
                              double* __restrict__ out, int ostride) {
    const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t0 >= T) return;
    const double* w = r + t0;
    const double omega = G.v[0];
    double alpha[P], beta[Q], sa = 0.0, sb = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) { alpha[i] = G.v[1 + i]; sa += alpha[i]; }
#pragma unroll
    for (int j = 0; j < Q; ++j) { beta[j] = G.v[1 + P + j]; sb += beta[j]; }
    double hist[Q];
#pragma unroll
    for (int j = 0; j < Q; ++j) hist[j] = 0.0;
    hist[0] = omega / (1 - sa - sb);
    for (long long t = 1; t < n_in; ++t) {
        double v = omega;
#pragma unroll
        for (int i = 0; i < P; ++i)
            if (i < t) v += alpha[i] * (w[t - i - 1] * w[t - i - 1]);
#pragma unroll
        for (int j = 0; j < Q; ++j)
            if (j < t) v += beta[j] * hist[j];
        const double s2 = (v < 1e-7) ? 1e-7 : v;
#pragma unroll
        for (int j = Q - 1; j > 0; --j) hist[j] = hist[j - 1];
        hist[0] = s2;
    }
    double s_a = 0.0, s_b = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const double ri = w[n_in - P + i];
        s_a = (i == 0) ? alpha[i] * (ri * ri) : s_a + alpha[i] * (ri * ri);
    }
#pragma unroll
    for (int j = 0; j < Q; ++j) s_b = (j == 0) ? beta[j] * hist[Q - 1] : s_b + beta[j] * hist[Q - 1 - j];
    out[t0 * ostride] = sqrt((omega + s_a) + s_b);
}

template <int P>
void launch_garch_sigma(int q, const GarchPrm& G, const double* r, long long n_in, long long T, double* o, int os,
                        hipStream_t st) {
    const dim3 g((unsigned)((T + 255) / 256)), blk(256);
    switch (q) {
        case 1: hipLaunchKernelGGL((k_garch_sigma<P, 1>), g, blk, 0, st, G, r, n_in, T, o, os); break;
        case 2: hipLaunchKernelGGL((k_garch_sigma<P, 2>), g, blk, 0, st, G, r, n_in, T, o, os); break;
        case 3: hipLaunchKernelGGL((k_garch_sigma<P, 3>), g, blk, 0, st, G, r, n_in, T, o, os); break;
        default: hipLaunchKernelGGL((k_garch_sigma<P, 4>), g, blk, 0, st, G, r, n_in, T, o, os); break;
    }
}

template <int P>
void launch_garch_forecast_pq(int q, const double* prm, const double* r, long long n_in, long long T, double* o) {
    const dim3 g((unsigned)((T + 255) / 256)), blk(256);
    switch (q) {
        case 1: hipLaunchKernelGGL((k_garch_forecast_pq<P, 1>), g, blk, 0, 0, prm, r, n_in, T, o); break;
        case 2: hipLaunchKernelGGL((k_garch_forecast_pq<P, 2>), g, blk, 0, 0, prm, r, n_in, T, o); break;
        case 3: hipLaunchKernelGGL((k_garch_forecast_pq<P, 3>), g, blk, 0, 0, prm, r, n_in, T, o); break;
        default: hipLaunchKernelGGL((k_garch_forecast_pq<P, 4>), g, blk, 0, 0, prm, r, n_in, T, o); break;
    }
}

template <int P>
void launch_garch_pq(int q, const double* p, long long B, const double* r, long long N, double* o) {
    const dim3 g((unsigned)((B + 63) / 64)), blk(64);
    switch (q) {
        case 1: hipLaunchKernelGGL((k_garch_loglik_pq<P, 1>), g, blk, 0, 0, p, B, r, N, o); break;
        case 2: hipLaunchKernelGGL((k_garch_loglik_pq<P, 2>), g, blk, 0, 0, p, B, r, N, o); break;
        case 3: hipLaunchKernelGGL((k_garch_loglik_pq<P, 3>), g, blk, 0, 0, p, B, r, N, o); break;
        default: hipLaunchKernelGGL((k_garch_loglik_pq<P, 4>), g, blk, 0, 0, p, B, r, N, o); break;
    }
}

// ----------------------------------------------------------------------- UKF
struct UkfConst {
    double wm0, wm1, wc0, wc1, wm2_0, wm2_1, phi;
};

UkfConst ukf_const(double alpha = 1.6, double beta = 2.0, double kappa = 1.75) {
    const int L = 2;
    const double lam = (alpha * alpha) * (L + kappa) - L;        // estimate.py:234
    UkfConst c;
    c.wm1 = 1 / (2 * (L + lam));
    c.wm0 = lam / (L + lam);
    c.wc1 = c.wm1;
    c.wc0 = c.wm0 + (1 - alpha * alpha + beta);                  // :103-109
    c.wm2_0 = lam / (L + lam);
    c.wm2_1 = 1 / (2 * (L + lam));                               // :112-116
    c.phi = std::sqrt(L + lam);
    return c;
}

// Runs one UKF pass; returns false on the Z < 1e-10 failure (estimate.py:219-220) or a
// NaN mean / variance / Z (:270-271).  states != nullptr: the filtered means
// (state_estimation, :273) are written with stride `sstride`.
__device__ bool ukf_pass(const UkfConst& C, double a, double l, double q, const double* w, long long N,
                         double* xmean_last, double* LL, double* states = nullptr, long long sstride = 1) {
    double x = l, var = q;                                        // forecast.py:9: init (l, q)
    double xm = 0.0, ll = 0.0;
    for (long long t = 0; t < N; ++t) {
        const double dvar = (var <= 0) ? var + 1e-8 : var;        // custom_cholesky :72-74
        const double c0 = sqrt(dvar);
        const double X1a[5] = {x, x + C.phi * c0, x + C.phi * 0.0, x - C.phi * c0, x - C.phi * 0.0};
        const double X1b[5] = {0.0, 0.0 + C.phi * 0.0, 0.0 + C.phi * 1.0, 0.0 - C.phi * 0.0, 0.0 - C.phi * 1.0};
        double X[5];
        for (int i = 0; i < 5; ++i) X[i] = a * (X1a[i] - l) + l + q * X1b[i];   // f_vectorized :141
        xm = X[0] * C.wm0;
        for (int i = 1; i < 5; ++i) xm += X[i] * C.wm1;
        double P = 0.0;
        for (int i = 0; i < 5; ++i) {
            const double d = X[i] - xm;
            P += (d * (i == 0 ? C.wc0 : C.wc1)) * d;
        }
        const double sP = sqrt(P);
        const double X2[3] = {xm, xm + C.phi * sP, xm - C.phi * sP};             // generate_sp :145-169
        double h[3], Z = 0.0;
        for (int i = 0; i < 3; ++i) {
            const double eta = w[t] / exp(X2[i]);
            h[i] = (kInvSqrt2Pi * exp(-0.5 * (eta * eta))) * fabs(eta);
            Z += (i == 0 ? C.wm2_0 : C.wm2_1) * h[i];
        }
        if (Z <= 0 || Z < 1e-10) return false;
        double mean = 0.0;
        for (int i = 0; i < 3; ++i) mean += ((i == 0 ? C.wm2_0 : C.wm2_1) * X2[i] * h[i]) / Z;
        double v2 = 0.0;
        for (int i = 0; i < 3; ++i) {
            const double d = X2[i] - mean;
            v2 += (i == 0 ? C.wm2_0 : C.wm2_1) * ((h[i] / Z) * (d * d));
        }
        if (isnan(mean) || isnan(v2) || isnan(Z)) return false;
        if (states) states[t * sstride] = mean;
        ll += log(fabs(Z));
        x = mean;
        var = v2;
    }
    *xmean_last = xm;
    *LL = ll;
    return true;
}

// Forecast-only UKF pass (k_ukf_forecast, k_ukf_sigma): ukf_pass's recursion (estimate.py:230-281)
// with each step's dependent chain shortened, one window per thread (~150 waves on the chip, so
// the forecast is latency-bound):
//  * prediction in closed form: the five sigma points x + phi (0, +c0, 0, -c0, 0), noise
//    phi (0, 0, 1, 0, -1) through f = a (x - l) + l + q noise have the weighted mean
//    a (x - l) + l (wm0 + 4 wm1 = 1) and the covariance 2 wc1 phi^2 (a^2 dvar + q^2) -- no
//    square root of dvar on the chain;
//  * update about the predicted mean: with y = X2 - xm in {0, +phi sP, -phi sP}, the weighted
//    sums Z, Sy of (h, h y) are independent, mean = xm + Sy / Z; w / exp(X) as w * exp(-X) and
//    one reciprocal of Z (v_rcp_f64 + two Newton steps, ~1 ulp);
//  * the variance as the reference forms it, a sum of non-negative terms about the updated
//    mean, sum w_i h_i (y_i - mu)^2 / Z (estimate.py:226).  The shortcut Syy / Z - mu^2 cancels
//    when one sigma point carries nearly all the weight (a return far in the tail): it can round
//    below 0 and take custom_cholesky's var <= 0 -> +1e-8 branch (:72-74) where the reference's
//    variance is a tiny positive number (tests/test_ukf_variance_gpu.py pins that regime).
// The algebra is exact, the rounding differs from the sigma-point arithmetic by a few ulp per
// step; the filter contracts, and sigma stays within 1e-12 of the reference's goldens
// (tests/test_gpu_parity.py, tests/test_insample_gpu.py).  Same failure rule as ukf_pass
// (estimate.py:219-220, :270-271).
__device__ bool ukf_forecast_pass(const UkfConst& C, double a, double l, double q, const double* w, long long N,
                                  double* xmean_last) {
    double x = l, var = q;                                        // forecast.py:9: init (l, q)
    double xm = 0.0;
    const double kP = 2.0 * C.wc1 * (C.phi * C.phi), a2 = a * a, q2 = q * q;
    for (long long t = 0; t < N; ++t) {
        const double dvar = (var <= 0) ? var + 1e-8 : var;        // custom_cholesky :72-74
        xm = a * (x - l) + l;
        const double sP = sqrt(kP * fma(a2, dvar, q2));
        const double y[3] = {0.0, C.phi * sP, -(C.phi * sP)};
        const double wt = w[t];
        double Z = 0.0, Sy = 0.0, wv[3];
        for (int i = 0; i < 3; ++i) {
            const double eta = wt * exp(-(xm + y[i]));
            const double h = (kInvSqrt2Pi * exp(-0.5 * (eta * eta))) * fabs(eta);
            const double wi = (i == 0 ? C.wm2_0 : C.wm2_1) * h;
            wv[i] = wi;
            Z += wi;
            Sy = fma(wi, y[i], Sy);
        }
        if (Z <= 0 || Z < 1e-10) return false;
        const double rz = fast_rcp(Z);
        const double mu = Sy * rz;
        const double mean = xm + mu;
        const double d1 = y[1] - mu, d2 = y[2] - mu;
        const double v2 = fma(wv[0] * mu, mu, fma(wv[1] * d1, d1, (wv[2] * d2) * d2)) * rz;
        if (isnan(mean) || isnan(v2) || isnan(Z)) return false;
        x = mean;
        var = v2;
    }
    *xmean_last = xm;
    return true;
}

__global__ void k_ukf_forecast(UkfConst C, double a, double l, double q, const double* __restrict__ r, long long n_in,
                               long long T, double* __restrict__ out, int* err) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    double xm;
    if (!ukf_forecast_pass(C, a, l, q, r + t, n_in, &xm)) {
        atomicOr(err, 1);
        out[t] = __builtin_nan("");
        return;
    }
    out[t] = exp(xm);                                             // forecast.py:12 (Q19)
}

// cvq_sigma_tables' UKF leg: every asset in one launch (blockIdx.y = asset; its centred
// returns at r + d * rstride), sigma written as out[t * dim + d].
struct UkfPrmN {
    double a[3], l[3], q[3];
};

__global__ void k_ukf_sigma(UkfConst C, UkfPrmN U, const double* __restrict__ r, long long rstride, long long n_in,
                            long long T, double* __restrict__ out, int* err) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int d = blockIdx.y;
    double xm;
    if (!ukf_forecast_pass(C, U.a[d], U.l[d], U.q[d], r + d * rstride + t, n_in, &xm)) {
        atomicOr(err, 1);
        out[t * gridDim.y + d] = __builtin_nan("");
        return;
    }
    out[t * gridDim.y + d] = exp(xm);                             // forecast.py:12 (Q19)
}

__global__ void k_ukf_loglik(UkfConst C, const double* __restrict__ prm, long long B, const double* __restrict__ r,
                             long long N, double* __restrict__ out) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xm, ll;
    const bool ok = ukf_pass(C, prm[3 * b], prm[3 * b + 1], prm[3 * b + 2], r, N, &xm, &ll);
    out[b] = ok ? ll : -1e10;                                     // estimate.py:270-271
}

// KalmanFilterVolEstimation (estimate.py:7-51, init (l, q) as VolOptimizer.e_step,
// kalman_mean_reverting/optimize.py:28-32): LL and the filtered state path of each
// candidate.  Path layout [N][B] (time-major) so the B candidates' stores coalesce;
// a failed pass leaves LL = -1e10 and NaN in its column (state_estimation None).
__global__ void k_ukf_filter(UkfConst C, const double* __restrict__ prm, long long B, const double* __restrict__ r,
                             long long r_stride, long long N, double* __restrict__ ll_out,
                             double* __restrict__ states) {
    const long long b = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    double xm, ll;
    const bool ok = ukf_pass(C, prm[3 * b], prm[3 * b + 1], prm[3 * b + 2], r + b * r_stride, N, &xm, &ll,
                             states + b, B);
    ll_out[b] = ok ? ll : -1e10;
    if (!ok)
        for (long long t = 0; t < N; ++t) states[t * B + b] = __builtin_nan("");
}

// ------------------------------------------------------------------ KAT
__global__ void k_special(int fn, TConst tk, const double* __restrict__ x, long long n, double* __restrict__ out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    out[i] = fn == 0 ? stdtrit(tk, v) : fn == 1 ? ndtri(v) : fn == 2 ? erf(v) : stdtrit_tab_int<6>(tk, v);
}

// ------------------------------------------------------------ host helpers
struct DevBuf {
    double* p = nullptr;
    ~DevBuf() { if (p) (void)hipFree(p); }
};

int stage_in(const double* src, size_t n, int mem, DevBuf& tmp, const double** dptr) {
    if (mem == CVQ_MEM_DEVICE) { *dptr = src; return CVQ_OK; }
    CVQ_HIP_CHECK(hipMalloc((void**)&tmp.p, std::max<size_t>(n, 1) * sizeof(double)));
    CVQ_HIP_CHECK(hipMemcpy(tmp.p, src, n * sizeof(double), hipMemcpyHostToDevice));
    *dptr = tmp.p;
    return CVQ_OK;
}

int stage_out(double* dst, size_t n, int mem, DevBuf& tmp, double** dptr) {
    if (mem == CVQ_MEM_DEVICE) { *dptr = dst; return CVQ_OK; }
    CVQ_HIP_CHECK(hipMalloc((void**)&tmp.p, std::max<size_t>(n, 1) * sizeof(double)));
    *dptr = tmp.p;
    return CVQ_OK;
}

int finish_out(double* dst, size_t n, int mem, const DevBuf& tmp) {
    CVQ_HIP_CHECK(hipGetLastError());
    CVQ_HIP_CHECK(hipDeviceSynchronize());
    if (mem != CVQ_MEM_DEVICE) CVQ_HIP_CHECK(hipMemcpy(dst, tmp.p, n * sizeof(double), hipMemcpyDeviceToHost));
    return CVQ_OK;
}

struct DevInt {
    int* p = nullptr;
    ~DevInt() { if (p) (void)hipFree(p); }
};

template <int K>
void launch_filter(const MsmParamsN& P, int dim, const double* cond, long long N, long long n_in, long long T,
                   double* out, int* err, hipStream_t stream) {
    constexpr int L = Quad<K>::L;
    const long long threads = T * L;
    hipLaunchKernelGGL(k_msm_filter<K>, dim3((unsigned)((threads + 255) / 256), (unsigned)dim), dim3(256), 0, stream,
                       P, cond, N * (1LL << K), n_in, T, out, T * (1LL << K), err);
}

int launch_filter_k(int k, const MsmParamsN& P, int dim, const double* cond, long long N, long long n_in, long long T,
                    double* out, int* err, hipStream_t stream) {
    switch (k) {
        case 1: launch_filter<1>(P, dim, cond, N, n_in, T, out, err, stream); break;
        case 2: launch_filter<2>(P, dim, cond, N, n_in, T, out, err, stream); break;
        case 3: launch_filter<3>(P, dim, cond, N, n_in, T, out, err, stream); break;
        case 4: launch_filter<4>(P, dim, cond, N, n_in, T, out, err, stream); break;
        case 5: launch_filter<5>(P, dim, cond, N, n_in, T, out, err, stream); break;
        case 6: launch_filter<6>(P, dim, cond, N, n_in, T, out, err, stream); break;
        default: launch_filter<7>(P, dim, cond, N, n_in, T, out, err, stream); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

// Block length of the blocked filter for 2**k states and windows of n_in steps, or 0 for
// the step-by-step filter (k outside [2, 4], windows not longer than a block, or the
// full blocks a workgroup's windows cross would not fit kBlockLdsMax of LDS).
constexpr size_t kBlockLdsMax = 80 * 1024;
#ifndef CVQ_MSM_BLOCK
#define CVQ_MSM_BLOCK 32
#endif

size_t blocked_lds_bytes(int k, long long n_in, int B) {
    const long long S = 1LL << k;
    return (size_t)((kWinPerWG - 1 + n_in - 1) / B + 1) * S * S * sizeof(double);
}

int msm_block_len(int k, long long n_in) {
    if (k < 2 || k > 4 || CVQ_MSM_BLOCK <= 0) return 0;
    int B = CVQ_MSM_BLOCK;
    while (blocked_lds_bytes(k, n_in, B) > kBlockLdsMax) B *= 2;
    return n_in > B ? B : 0;
}

template <int K>
void launch_blocked(const MsmParamsN& P, int dim, const double* cond, long long N, long long n_in, long long T, int B,
                    double* G, double* out, int* err, hipStream_t stream) {
    constexpr int S = 1 << K;
    const long long nfull = N / B;
    hipLaunchKernelGGL(k_msm_gblocks<K>, dim3((unsigned)nfull, (unsigned)dim), dim3(4 * S), 0, stream, P, cond,
                       N * S, B, (int)nfull, G, nfull * S * S, err);
    hipLaunchKernelGGL(k_msm_windows<K>, dim3((unsigned)((T + kWinPerWG - 1) / kWinPerWG), (unsigned)dim),
                       dim3(4 * kWinPerWG), blocked_lds_bytes(K, n_in, B), stream, P, cond, N * S, G, nfull * S * S,
                       B, n_in, T, out, T * S, err);
}

int launch_blocked_k(int k, const MsmParamsN& P, int dim, const double* cond, long long N, long long n_in, long long T,
                     int B, double* G, double* out, int* err, hipStream_t stream) {
    switch (k) {
        case 2: launch_blocked<2>(P, dim, cond, N, n_in, T, B, G, out, err, stream); break;
        case 3: launch_blocked<3>(P, dim, cond, N, n_in, T, B, G, out, err, stream); break;
        default: launch_blocked<4>(P, dim, cond, N, n_in, T, B, G, out, err, stream); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

// Transfer-matrix scan filter (k_msm_blkscan -> k_msm_supscan -> k_msm_scanwin): 2 <= k <= 4
// (one wavefront per superblock scan); k = 5, 6 the wide variant (no stored prefixes, 256-thread
// superblock scans, one wavefront per window); windows longer than two blocks.
bool msm_scan_ok(int k, long long n_in) {
    return k >= 2 && k <= 6 && n_in > 2 * kScanB;
}

struct ScanLayout {                 // doubles of each scan buffer, per asset
    long long pre, suf, gf, sup, nfull, nsup;
};
ScanLayout scan_layout(int k, long long n_in, long long T) {
    const long long S = 1LL << k, N = n_in + T - 1;
    ScanLayout L;
    L.nfull = N / kScanB;
    L.nsup = (L.nfull + kScanC - 1) / kScanC;
    L.pre = k >= 5 ? 0 : T * S * S;                 // the wide scan stores no block prefixes
    L.suf = k >= 5 ? 0 : T * S;                     // (nor window-start suffixes)
    L.gf = L.nfull * S * S;
    L.sup = L.nsup * kScanC * S * S;
    return L;
}

// error flags of the scan filter: one per (asset, block) of k_msm_blkscan, after the error
// word's two doubles (0 when the scan filter does not run)
long long scan_flag_count(int k, long long n_in, long long T, int dim) {
    if (!msm_scan_ok(k, n_in)) return 0;
    const long long N = n_in + T - 1;
    return dim * ((N + kScanB - 1) / kScanB);
}

template <int K>
void launch_scan(const MsmParamsN& P, const StateMapQ& MQ, int dim, const double* r, long long N, long long n_in,
                 long long T, double* buf, double* fbs, int* err, hipStream_t stream) {
    constexpr int S = 1 << K;
    const ScanLayout L = scan_layout(K, n_in, T);
    double* Pre = buf;
    double* Suf1 = Pre + dim * L.pre;
    double* Gf = Suf1 + dim * L.suf;
    double* PG = Gf + dim * L.gf;
    double* SG = PG + dim * L.sup;
    const long long nblk = (N + kScanB - 1) / kScanB;
    hipLaunchKernelGGL(k_msm_blkscan<K>, dim3((unsigned)nblk, (unsigned)dim, 2), dim3(4 * S), 0, stream, P, r, N,
                       n_in, T, Pre, L.pre, Suf1, L.suf, Gf, L.gf, err);
    if (L.nsup > 0)
        hipLaunchKernelGGL(k_msm_supscan<K>, dim3((unsigned)L.nsup, (unsigned)dim, 2), dim3(4 * S), 0, stream, Gf,
                           L.gf, L.nfull, PG, SG, L.sup);
    hipLaunchKernelGGL(k_msm_scanwin<K>, dim3((unsigned)((T + 15) / 16), (unsigned)dim), dim3(256), 0, stream, Pre,
                       L.pre, Suf1, L.suf, Gf, L.gf, PG, SG, L.sup, L.nfull, n_in, T, MQ, dim, fbs);
}

template <int K>
void launch_scan_w(const MsmParamsN& P, const StateMap& M, int q, int dim, const double* r, long long N,
                   long long n_in, long long T, double* buf, double* fbs, int* err, hipStream_t stream) {
    constexpr int S = 1 << K;
    const ScanLayout L = scan_layout(K, n_in, T);
    double* Suf1 = buf;                                         // L.pre = 0: no prefixes
    double* Gf = Suf1 + dim * L.suf;
    double* PG = Gf + dim * L.gf;
    double* SG = PG + dim * L.sup;
    const long long nblk = (N + kScanB - 1) / kScanB;
    // block products only (z = 0): a window runs its first partial block as filter steps
    hipLaunchKernelGGL(k_msm_blkscan<K>, dim3((unsigned)nblk, (unsigned)dim, 1), dim3(4 * S), 0, stream, P, r, N,
                       n_in, T, nullptr, 0LL, Suf1, L.suf, Gf, L.gf, err);
    if (L.nsup > 0)
        hipLaunchKernelGGL(k_msm_supscan_w<K>, dim3((unsigned)L.nsup, (unsigned)dim, 2), dim3(256), 0, stream, Gf,
                           L.gf, L.nfull, PG, SG, L.sup);
    hipLaunchKernelGGL(k_msm_scanwin_w<K>, dim3((unsigned)((T + kWinGroup - 1) / kWinGroup), (unsigned)dim),
                       dim3(256), 0, stream, P, r, N, Gf, L.gf, PG, SG, L.sup, L.nfull, n_in, T, M, q, dim, fbs);
}

int launch_scan_k(int k, const MsmParamsN& P, const StateMapQ& MQ, int dim, const double* r, long long N,
                  long long n_in, long long T, double* buf, double* fbs, int* err, hipStream_t stream) {
    switch (k) {
        case 2: launch_scan<2>(P, MQ, dim, r, N, n_in, T, buf, fbs, err, stream); break;
        case 3: launch_scan<3>(P, MQ, dim, r, N, n_in, T, buf, fbs, err, stream); break;
        default: launch_scan<4>(P, MQ, dim, r, N, n_in, T, buf, fbs, err, stream); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

template <int K>
void launch_msm_ll(const MsmParams* P, long long B, const double* r, long long N, double* out) {
    constexpr int L = Quad<K>::L;
    const long long threads = B * L;
    hipLaunchKernelGGL(k_msm_loglik<K>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, 0, P, B, r, N, out);
}


}  // namespace

extern "C" {

int32_t cvq_msm_tables_scratch(int32_t dim, int32_t k, int64_t n_in, int64_t T, int64_t* doubles) {
    CVQ_REQUIRE(doubles != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(dim >= 1 && dim <= 3 && k >= 1 && k <= 7 && n_in >= 1 && T >= 1, CVQ_ERR_INVALID, "bad shape");
    const long long S = 1LL << k, N = n_in + T - 1;
    long long G;
    if (msm_scan_ok(k, n_in)) {                            // scan filter: prefixes, suffixes, block / superblock products
        const ScanLayout L = scan_layout(k, n_in, T);
        G = dim * (L.pre + L.suf + L.gf + 2 * L.sup);
    } else {
        const int B = msm_block_len(k, n_in);
        G = B ? dim * (N / B) * S * S : 0;                  // blocked filter: full-block products
    }
    // cond, filtered probabilities, [G], error word (2 doubles), scan filter: per-block error flags
    *doubles = dim * N * S + dim * T * S + G + 2 + (scan_flag_count(k, n_in, T, dim) + 1) / 2;
    return CVQ_OK;
}

int32_t cvq_msm_tables(int32_t device, void* stream, int32_t dim, int32_t k, const double* params,
                       const int32_t* state_map, int32_t q, const double* returns_c, int64_t n_in, int64_t T,
                       double* scratch, double* fbs_out, double* pi_out) {
    CVQ_REQUIRE(params && state_map && returns_c && scratch && fbs_out && pi_out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(dim >= 2 && dim <= 3, CVQ_ERR_UNSUPPORTED, "dim must be 2 or 3");
    CVQ_REQUIRE(k >= 1 && k <= 7, CVQ_ERR_UNSUPPORTED, "MSM k must be in [1, 7]");
    CVQ_REQUIRE(q >= 1 && q <= 8, CVQ_ERR_UNSUPPORTED, "q (unique vol states) must be in [1, 8]");
    CVQ_REQUIRE(n_in >= 1 && T >= 1, CVQ_ERR_INVALID, "n_in and T must be >= 1");
    const int S = 1 << k;
    MsmParamsN P{};
    StateMap M{};
    for (int d = 0; d < dim; ++d) {
        P.a[d] = msm_params(k, params[4 * d], params[4 * d + 1], params[4 * d + 2], params[4 * d + 3]);
        for (int s2 = 0; s2 < S; ++s2) {
            CVQ_REQUIRE(state_map[d * S + s2] >= 0 && state_map[d * S + s2] < q, CVQ_ERR_INVALID,
                        "state_map entries must be in [0, q)");
            M.u[d][s2] = (uint8_t)state_map[d * S + s2];
        }
    }
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    hipStream_t st = (hipStream_t)stream;
    const long long N = n_in + T - 1;
    const bool scan = msm_scan_ok(k, n_in);
    const int B = scan ? 0 : msm_block_len(k, n_in);
    double* cond = scratch;
    double* filt = cond + (long long)dim * N * S;
    double* G = filt + (long long)dim * T * S;
    long long gsz = B ? (long long)dim * (N / B) * S * S : 0;
    if (scan) {
        const ScanLayout L = scan_layout(k, n_in, T);
        gsz = dim * (L.pre + L.suf + L.gf + 2 * L.sup);
    }
    int* err = (int*)(G + gsz);
    // the scan filter's blocks overwrite their own error flags (err + 4 ...) on every run; the
    // step-by-step and blocked filters OR into the error word, reset here
    if (!scan) CVQ_HIP_CHECK(hipMemsetAsync(err, 0, sizeof(int), st));
    if (scan) {                        // densities computed per block inside; the collapse fused into the windows
        StateMapQ MQ{};                                  // k <= 4: <= 16 states
        MQ.q = q;
        for (int d = 0; d < dim && S <= 16; ++d)
            for (int s2 = 0; s2 < S; ++s2) MQ.u[d][s2] = M.u[d][s2];
        if (k >= 5) {
            if (k == 5) launch_scan_w<5>(P, M, q, dim, returns_c, N, n_in, T, G, fbs_out, err + 4, st);
            else launch_scan_w<6>(P, M, q, dim, returns_c, N, n_in, T, G, fbs_out, err + 4, st);
            CVQ_HIP_CHECK(hipGetLastError());
        } else {
            rc = launch_scan_k(k, P, MQ, dim, returns_c, N, n_in, T, G, fbs_out, err + 4, st);
        }
        if (rc) return rc;
    } else {
        hipLaunchKernelGGL(k_msm_cond, dim3((unsigned)((N * S + 255) / 256), (unsigned)dim), dim3(256), 0, st, P, S,
                           returns_c, N, cond);
        if (B) rc = launch_blocked_k(k, P, dim, cond, N, n_in, T, B, G, filt, err, st);
        else rc = launch_filter_k(k, P, dim, cond, N, n_in, T, filt, err, st);
        if (rc) return rc;
        hipLaunchKernelGGL(k_msm_fbs, dim3((unsigned)((T * dim + 255) / 256)), dim3(256), 0, st, M, dim, S, q, filt,
                           T, fbs_out);
    }
    const long long Q = dim == 2 ? (long long)q * q : (long long)q * q * q;
    hipLaunchKernelGGL(k_msm_pi, dim3((unsigned)((T * Q + 255) / 256)), dim3(256), 0, st, dim, q, fbs_out, T, pi_out);
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int32_t cvq_msm_tables_status(double* scratch, int32_t dim, int32_t k, int64_t n_in, int64_t T, void* stream) {
    CVQ_REQUIRE(scratch != nullptr, CVQ_ERR_INVALID, "NULL argument");
    const long long S = 1LL << k, N = n_in + T - 1;
    long long G;
    if (msm_scan_ok(k, n_in)) {
        const ScanLayout L = scan_layout(k, n_in, T);
        G = dim * (L.pre + L.suf + L.gf + 2 * L.sup);
    } else {
        const int B = msm_block_len(k, n_in);
        G = B ? dim * (N / B) * S * S : 0;
    }
    int e = 0;
    const int* err = (const int*)(scratch + dim * N * S + dim * T * S + G);
    if (msm_scan_ok(k, n_in)) {                            // the last run's per-block flags
        std::vector<int> fl((size_t)scan_flag_count(k, n_in, T, dim));
        CVQ_HIP_CHECK(hipMemcpyAsync(fl.data(), err + 4, fl.size() * sizeof(int), hipMemcpyDeviceToHost,
                                     (hipStream_t)stream));
        CVQ_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
        for (int f : fl) e |= f;
    } else {
        CVQ_HIP_CHECK(hipMemcpyAsync(&e, err, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
        CVQ_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    }
    CVQ_REQUIRE(e == 0, CVQ_ERR_NUMERIC, "MSM Bayes update normaliser is 0 (calc_prob.py:64-65)");
    return CVQ_OK;
}

int32_t cvq_sigma_tables(int32_t device, void* stream, int32_t model, int32_t dim, const int32_t* orders,
                         const double* params, const double* returns_c, int64_t n_in, int64_t T, int32_t* d_err,
                         double* sig_out) {
    CVQ_REQUIRE(params && returns_c && d_err && sig_out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(model == CVQ_GARCH || model == CVQ_UKF, CVQ_ERR_UNSUPPORTED, "model must be CVQ_GARCH or CVQ_UKF");
    CVQ_REQUIRE(dim >= 2 && dim <= 3, CVQ_ERR_UNSUPPORTED, "dim must be 2 or 3");
    CVQ_REQUIRE(n_in >= 1 && T >= 1, CVQ_ERR_INVALID, "n_in and T must be >= 1");
    GarchPrm G[3]{};
    int po[3] = {1, 1, 1}, qo[3] = {1, 1, 1};
    UkfPrmN U{};
    const double* pp = params;
    for (int d = 0; d < dim; ++d) {
        if (model == CVQ_GARCH) {
            if (orders) { po[d] = orders[2 * d]; qo[d] = orders[2 * d + 1]; }
            CVQ_REQUIRE(po[d] >= 1 && qo[d] >= 1 && po[d] <= kGarchMaxPQ && qo[d] <= kGarchMaxPQ, CVQ_ERR_UNSUPPORTED,
                        "GARCH orders must be 1 <= p, q <= 4");
            CVQ_REQUIRE(n_in >= po[d] && n_in >= qo[d], CVQ_ERR_INVALID, "window shorter than the GARCH order");
            double s = 0.0;
            bool pos = pp[0] > 0;
            for (int i = 0; i < 1 + po[d] + qo[d]; ++i) {
                G[d].v[i] = pp[i];
                if (i) { pos = pos && pp[i] > 0; s += pp[i]; }
            }
            CVQ_REQUIRE(pos && s < 1, CVQ_ERR_INVALID,
                        "GARCH parameters must be positive with sum(alpha) + sum(beta) < 1 (garch/estimation.py:22-38)");
            pp += 1 + po[d] + qo[d];
        } else {
            U.a[d] = pp[0];
            U.l[d] = pp[1];
            U.q[d] = pp[2];
            pp += 3;
        }
    }
    CVQ_DEVICE_SCOPE(device);
    hipStream_t st = (hipStream_t)stream;
    const long long N = n_in + T - 1;
    CVQ_HIP_CHECK(hipMemsetAsync(d_err, 0, sizeof(int32_t), st));
    if (model == CVQ_GARCH) {
        for (int d = 0; d < dim; ++d) {
            const double* r = returns_c + d * N;
            switch (po[d]) {
                case 1: launch_garch_sigma<1>(qo[d], G[d], r, n_in, T, sig_out + d, dim, st); break;
                case 2: launch_garch_sigma<2>(qo[d], G[d], r, n_in, T, sig_out + d, dim, st); break;
                case 3: launch_garch_sigma<3>(qo[d], G[d], r, n_in, T, sig_out + d, dim, st); break;
                default: launch_garch_sigma<4>(qo[d], G[d], r, n_in, T, sig_out + d, dim, st); break;
            }
        }
    } else {
        hipLaunchKernelGGL(k_ukf_sigma, dim3((unsigned)((T + 63) / 64), (unsigned)dim), dim3(64), 0, st, ukf_const(), U,
                           returns_c, N, n_in, T, sig_out, (int*)d_err);
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int32_t cvq_sigma_tables_status(const int32_t* d_err, void* stream) {
    CVQ_REQUIRE(d_err != nullptr, CVQ_ERR_INVALID, "NULL argument");
    int e = 0;
    CVQ_HIP_CHECK(hipMemcpyAsync(&e, d_err, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
    CVQ_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
    CVQ_REQUIRE(e == 0, CVQ_ERR_NUMERIC, "UKF normaliser Z < 1e-10 (estimate.py:219-220; reference returns None)");
    return CVQ_OK;
}

int32_t cvq_msm_filter(int32_t device, int32_t k, double m0, double sigma, double b, double gamma,
                       const double* returns_c, int64_t n_in, int64_t T, double* out, int32_t mem) {
    CVQ_REQUIRE(returns_c && out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(k >= 1 && k <= 7, CVQ_ERR_UNSUPPORTED, "MSM k must be in [1, 7]");
    CVQ_REQUIRE(n_in >= 1 && T >= 1, CVQ_ERR_INVALID, "n_in and T must be >= 1");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    MsmParamsN P{};
    P.a[0] = msm_params(k, m0, sigma, b, gamma);
    const int S = 1 << k;
    const long long N = n_in + T - 1;
    DevBuf rin, cond, dout;
    DevInt err;
    const double* d_r;
    double* d_out;
    if ((rc = stage_in(returns_c, N, mem, rin, &d_r))) return rc;
    if ((rc = stage_out(out, (size_t)T * S, mem, dout, &d_out))) return rc;
    CVQ_HIP_CHECK(hipMalloc((void**)&cond.p, (size_t)N * S * sizeof(double)));
    CVQ_HIP_CHECK(hipMalloc((void**)&err.p, sizeof(int)));
    CVQ_HIP_CHECK(hipMemset(err.p, 0, sizeof(int)));
    hipLaunchKernelGGL(k_msm_cond, dim3((unsigned)((N * S + 255) / 256), 1), dim3(256), 0, 0, P, S, d_r, N, cond.p);
    if ((rc = launch_filter_k(k, P, 1, cond.p, N, n_in, T, d_out, err.p, 0))) return rc;
    if ((rc = finish_out(out, (size_t)T * S, mem, dout))) return rc;
    int e = 0;
    CVQ_HIP_CHECK(hipMemcpy(&e, err.p, sizeof(int), hipMemcpyDeviceToHost));
    CVQ_REQUIRE(e == 0, CVQ_ERR_NUMERIC, "MSM Bayes update normaliser is 0 (calc_prob.py:64-65)");
    return CVQ_OK;
}

int32_t cvq_msm_marginals(int32_t device, int32_t k, double m0, double sigma, double b, double gamma,
                          const double* returns, int64_t N, double* marg_out, double* dens_out, int32_t mem) {
    CVQ_REQUIRE(returns && marg_out && dens_out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(k >= 1 && k <= 7, CVQ_ERR_UNSUPPORTED, "MSM k must be in [1, 7]");
    CVQ_REQUIRE(N >= 2, CVQ_ERR_INVALID, "N must be >= 2 (the marginals pair step i with return i - 1)");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    const MsmParams P = msm_params(k, m0, sigma, b, gamma);
    DevBuf rin, dm, dd;
    DevInt err;
    const double* d_r;
    double *d_m, *d_d;
    if ((rc = stage_in(returns, N, mem, rin, &d_r))) return rc;
    if ((rc = stage_out(marg_out, N - 1, mem, dm, &d_m))) return rc;
    if ((rc = stage_out(dens_out, N - 1, mem, dd, &d_d))) return rc;
    CVQ_HIP_CHECK(hipMalloc((void**)&err.p, sizeof(int)));
    CVQ_HIP_CHECK(hipMemset(err.p, 0, sizeof(int)));
    const int L = (1 << k) < 4 ? (1 << k) : 4;
    switch (k) {
        case 1: hipLaunchKernelGGL(k_msm_marginals<1>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        case 2: hipLaunchKernelGGL(k_msm_marginals<2>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        case 3: hipLaunchKernelGGL(k_msm_marginals<3>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        case 4: hipLaunchKernelGGL(k_msm_marginals<4>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        case 5: hipLaunchKernelGGL(k_msm_marginals<5>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        case 6: hipLaunchKernelGGL(k_msm_marginals<6>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
        default: hipLaunchKernelGGL(k_msm_marginals<7>, dim3(1), dim3(L), 0, 0, P, d_r, N, d_m, d_d, err.p); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    if ((rc = finish_out(marg_out, N - 1, mem, dm))) return rc;
    if ((rc = finish_out(dens_out, N - 1, mem, dd))) return rc;
    int e = 0;
    CVQ_HIP_CHECK(hipMemcpy(&e, err.p, sizeof(int), hipMemcpyDeviceToHost));
    CVQ_REQUIRE(e == 0, CVQ_ERR_NUMERIC, "MSM Bayes update normaliser is 0 (calc_prob.py:64-65)");
    return CVQ_OK;
}

int32_t cvq_garch_forecast(int32_t device, double omega, double alpha, double beta, const double* returns_c,
                           int64_t n_in, int64_t T, double* out, int32_t mem) {
    CVQ_REQUIRE(returns_c && out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(omega > 0 && alpha > 0 && beta > 0 && alpha + beta < 1, CVQ_ERR_INVALID,
                "GARCH parameters must be positive with alpha + beta < 1 (garch/estimation.py:22-38)");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf rin, dout;
    const double* d_r;
    double* d_out;
    if ((rc = stage_in(returns_c, n_in + T - 1, mem, rin, &d_r))) return rc;
    if ((rc = stage_out(out, T, mem, dout, &d_out))) return rc;
    hipLaunchKernelGGL(k_garch_forecast, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, 0, omega, alpha, beta, d_r,
                       n_in, T, d_out);
    return finish_out(out, T, mem, dout);
}

int32_t cvq_garch_forecast_pq(int32_t device, int32_t p, int32_t q, const double* params, const double* returns_c,
                              int64_t n_in, int64_t T, double* out, int32_t mem) {
    CVQ_REQUIRE(params && returns_c && out && n_in >= 1 && T >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_REQUIRE(p >= 1 && q >= 1 && p <= kGarchMaxPQ && q <= kGarchMaxPQ, CVQ_ERR_UNSUPPORTED,
                "GARCH orders must be 1 <= p, q <= 4");
    CVQ_REQUIRE(n_in >= p && n_in >= q, CVQ_ERR_INVALID, "window shorter than the GARCH order");
    double s = 0.0;
    bool pos = params[0] > 0;
    for (int i = 1; i <= p + q; ++i) { pos = pos && params[i] > 0; s += params[i]; }
    CVQ_REQUIRE(pos && s < 1, CVQ_ERR_INVALID,
                "GARCH parameters must be positive with sum(alpha) + sum(beta) < 1 (garch/estimation.py:22-38)");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf pin, rin, dout;
    const double *d_p, *d_r;
    double* d_out;
    // params always come from host memory (1 + p + q doubles)
    if ((rc = stage_in(params, 1 + p + q, CVQ_MEM_HOST, pin, &d_p)) ||
        (rc = stage_in(returns_c, n_in + T - 1, mem, rin, &d_r)) || (rc = stage_out(out, T, mem, dout, &d_out)))
        return rc;
    switch (p) {
        case 1: launch_garch_forecast_pq<1>(q, d_p, d_r, n_in, T, d_out); break;
        case 2: launch_garch_forecast_pq<2>(q, d_p, d_r, n_in, T, d_out); break;
        case 3: launch_garch_forecast_pq<3>(q, d_p, d_r, n_in, T, d_out); break;
        default: launch_garch_forecast_pq<4>(q, d_p, d_r, n_in, T, d_out); break;
    }
    return finish_out(out, T, mem, dout);
}

int32_t cvq_ukf_forecast(int32_t device, double a, double l, double q, const double* returns_c, int64_t n_in,
                         int64_t T, double* out, int32_t mem) {
    CVQ_REQUIRE(returns_c && out, CVQ_ERR_INVALID, "NULL argument");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf rin, dout;
    DevInt err;
    const double* d_r;
    double* d_out;
    if ((rc = stage_in(returns_c, n_in + T - 1, mem, rin, &d_r))) return rc;
    if ((rc = stage_out(out, T, mem, dout, &d_out))) return rc;
    CVQ_HIP_CHECK(hipMalloc((void**)&err.p, sizeof(int)));
    CVQ_HIP_CHECK(hipMemset(err.p, 0, sizeof(int)));
    hipLaunchKernelGGL(k_ukf_forecast, dim3((unsigned)((T + 63) / 64)), dim3(64), 0, 0, ukf_const(), a, l, q, d_r, n_in,
                       T, d_out, err.p);
    if ((rc = finish_out(out, T, mem, dout))) return rc;
    int e = 0;
    CVQ_HIP_CHECK(hipMemcpy(&e, err.p, sizeof(int), hipMemcpyDeviceToHost));
    CVQ_REQUIRE(e == 0, CVQ_ERR_NUMERIC, "UKF normaliser Z < 1e-10 (estimate.py:219-220; reference returns None)");
    return CVQ_OK;
}

int32_t cvq_msm_loglik(int32_t device, int32_t k, const double* params, int64_t B, const double* returns, int64_t N,
                       double* out, int32_t mem) {
    CVQ_REQUIRE(params && returns && out && B >= 1 && N >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_REQUIRE(k >= 1 && k <= 7, CVQ_ERR_UNSUPPORTED, "MSM k must be in [1, 7]");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    std::vector<double> hp((size_t)B * 4);
    if (mem == CVQ_MEM_DEVICE) CVQ_HIP_CHECK(hipMemcpy(hp.data(), params, hp.size() * sizeof(double), hipMemcpyDeviceToHost));
    else std::copy(params, params + hp.size(), hp.begin());
    std::vector<MsmParams> P((size_t)B);
    for (long long i = 0; i < B; ++i) P[i] = msm_params(k, hp[4 * i], hp[4 * i + 1], hp[4 * i + 2], hp[4 * i + 3]);
    MsmParams* dP = nullptr;
    CVQ_HIP_CHECK(hipMalloc((void**)&dP, P.size() * sizeof(MsmParams)));
    if (hipMemcpy(dP, P.data(), P.size() * sizeof(MsmParams), hipMemcpyHostToDevice) != hipSuccess) {
        (void)hipFree(dP);
        cvq::set_error("hipMemcpy of MSM parameters failed");
        return CVQ_ERR_HIP;
    }
    DevBuf rin, dout;
    const double* d_r;
    double* d_out;
    if ((rc = stage_in(returns, N, mem, rin, &d_r)) || (rc = stage_out(out, B, mem, dout, &d_out))) {
        (void)hipFree(dP);
        return rc;
    }
    switch (k) {
        case 1: launch_msm_ll<1>(dP, B, d_r, N, d_out); break;
        case 2: launch_msm_ll<2>(dP, B, d_r, N, d_out); break;
        case 3: launch_msm_ll<3>(dP, B, d_r, N, d_out); break;
        case 4: launch_msm_ll<4>(dP, B, d_r, N, d_out); break;
        case 5: launch_msm_ll<5>(dP, B, d_r, N, d_out); break;
        case 6: launch_msm_ll<6>(dP, B, d_r, N, d_out); break;
        default: launch_msm_ll<7>(dP, B, d_r, N, d_out); break;
    }
    rc = finish_out(out, B, mem, dout);
    (void)hipFree(dP);
    return rc;
}

int32_t cvq_garch_loglik(int32_t device, const double* params, int64_t B, const double* returns, int64_t N,
                         double* out, int32_t mem) {
    CVQ_REQUIRE(params && returns && out && B >= 1 && N >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf pin, rin, dout;
    const double *d_p, *d_r;
    double* d_out;
    if ((rc = stage_in(params, (size_t)B * 3, mem, pin, &d_p)) || (rc = stage_in(returns, N, mem, rin, &d_r)) ||
        (rc = stage_out(out, B, mem, dout, &d_out)))
        return rc;
    hipLaunchKernelGGL(k_garch_loglik, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, 0, d_p, B, d_r, N, d_out);
    return finish_out(out, B, mem, dout);
}

int32_t cvq_garch_loglik_pq(int32_t device, int32_t p, int32_t q, const double* params, int64_t B,
                            const double* returns, int64_t N, double* out, int32_t mem) {
    CVQ_REQUIRE(params && returns && out && B >= 1 && N >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_REQUIRE(p >= 1 && q >= 1 && p <= kGarchMaxPQ && q <= kGarchMaxPQ, CVQ_ERR_UNSUPPORTED,
                "GARCH orders must be 1 <= p, q <= 4");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf pin, rin, dout;
    const double *d_p, *d_r;
    double* d_out;
    if ((rc = stage_in(params, (size_t)B * (1 + p + q), mem, pin, &d_p)) || (rc = stage_in(returns, N, mem, rin, &d_r)) ||
        (rc = stage_out(out, B, mem, dout, &d_out)))
        return rc;
    switch (p) {
        case 1: launch_garch_pq<1>(q, d_p, B, d_r, N, d_out); break;
        case 2: launch_garch_pq<2>(q, d_p, B, d_r, N, d_out); break;
        case 3: launch_garch_pq<3>(q, d_p, B, d_r, N, d_out); break;
        default: launch_garch_pq<4>(q, d_p, B, d_r, N, d_out); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return finish_out(out, B, mem, dout);
}

int32_t cvq_ukf_loglik(int32_t device, const double* params, int64_t B, const double* returns, int64_t N, double* out,
                       int32_t mem) {
    CVQ_REQUIRE(params && returns && out && B >= 1 && N >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    DevBuf pin, rin, dout;
    const double *d_p, *d_r;
    double* d_out;
    if ((rc = stage_in(params, (size_t)B * 3, mem, pin, &d_p)) || (rc = stage_in(returns, N, mem, rin, &d_r)) ||
        (rc = stage_out(out, B, mem, dout, &d_out)))
        return rc;
    hipLaunchKernelGGL(k_ukf_loglik, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, 0, ukf_const(), d_p, B, d_r, N,
                       d_out);
    return finish_out(out, B, mem, dout);
}

int32_t cvq_ukf_filter(int32_t device, const double* params, int64_t B, const double* returns, int32_t per_candidate,
                       int64_t N, double* ll_out, double* states_out, int32_t mem) {
    CVQ_REQUIRE(params && returns && ll_out && states_out && B >= 1 && N >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    const long long r_stride = per_candidate ? N : 0;
    DevBuf pin, rin, dll, dst;
    const double *d_p, *d_r;
    double *d_ll, *d_st;
    if ((rc = stage_in(params, (size_t)B * 3, mem, pin, &d_p)) ||
        (rc = stage_in(returns, per_candidate ? (size_t)B * N : (size_t)N, mem, rin, &d_r)) ||
        (rc = stage_out(ll_out, B, mem, dll, &d_ll)) || (rc = stage_out(states_out, (size_t)B * N, mem, dst, &d_st)))
        return rc;
    hipLaunchKernelGGL(k_ukf_filter, dim3((unsigned)((B + 63) / 64)), dim3(64), 0, 0, ukf_const(), d_p, B, d_r,
                       r_stride, N, d_ll, d_st);
    if ((rc = finish_out(ll_out, B, mem, dll))) return rc;
    if (mem != CVQ_MEM_DEVICE)
        CVQ_HIP_CHECK(hipMemcpy(states_out, dst.p, (size_t)B * N * sizeof(double), hipMemcpyDeviceToHost));
    return CVQ_OK;
}

int32_t cvq_special(int32_t device, int32_t fn, double nu, const double* x, int64_t n, double* out, int32_t mem) {
    CVQ_REQUIRE(x && out && n >= 1, CVQ_ERR_INVALID, "bad argument");
    CVQ_REQUIRE(fn >= 0 && fn <= 3, CVQ_ERR_INVALID,
                "fn must be 0 (t.ppf), 1 (norm.ppf), 2 (erf) or 3 (t.ppf, the solve kernels' nu = 6 path)");
    CVQ_REQUIRE(fn != 3 || nu == 6.0, CVQ_ERR_INVALID, "fn 3 is the integer path for nu = 6");
    CVQ_DEVICE_SCOPE(device);
    int rc = CVQ_OK;
    TConst tk{};
    DevBuf cf;
    if (fn == 0 || fn == 3) {
        CVQ_REQUIRE(nu > 0, CVQ_ERR_INVALID, "nu must be > 0");
        if ((rc = make_tconst(nu, &tk, &cf.p))) return rc;
        CVQ_REQUIRE(fn != 3 || tk.q_c != nullptr, CVQ_ERR_UNSUPPORTED, "no direct t.ppf tables for this nu");
    }
    DevBuf xin, dout;
    const double* d_x;
    double* d_out;
    if ((rc = stage_in(x, n, mem, xin, &d_x)) || (rc = stage_out(out, n, mem, dout, &d_out))) return rc;
    hipLaunchKernelGGL(k_special, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, fn, tk, d_x, n, d_out);
    return finish_out(out, n, mem, dout);
}

}  // extern "C"
