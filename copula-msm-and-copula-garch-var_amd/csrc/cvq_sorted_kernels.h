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
// depth where every cell holds <= sorted_tail_cap nodes, so a level costs one
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

// Tail nodes per lane of the one-wave tail (bracket size that switches to it = 64x):
// measured best 4 for 2-D (LDS-bound occupancy at n = 256), 16 for 3-D.
#ifndef CVQ_SORT_TAIL2
#define CVQ_SORT_TAIL2 4
#endif
#ifndef CVQ_SORT_TAIL3
#define CVQ_SORT_TAIL3 16
#endif
__host__ __device__ constexpr int sorted_tail_per_lane(int dim) { return dim == 2 ? CVQ_SORT_TAIL2 : CVQ_SORT_TAIL3; }
__host__ __device__ constexpr int sorted_tail_cap(int dim) { return 64 * sorted_tail_per_lane(dim); }
constexpr int kSortMaxDepth = 16;                     // deepest tabulated bisection level
// Block tail (exact dyadic walks, after the first bisection level): once the cell holds at most
// NT * kSortBlk nodes the whole workgroup evaluates it once in v* order, kSortBlk consecutive
// positions per thread, and one block scan + two crossing searches decide every remaining level
// (COMPACT's block tail) -- instead of one range sum + one workgroup reduction per level.
#ifndef CVQ_SORT_BLK
#define CVQ_SORT_BLK 8
#endif
constexpr int kSortBlk = CVQ_SORT_BLK;
#ifndef CVQ_SORT_ILP
#define CVQ_SORT_ILP 4
#endif
#ifndef CVQ_SORT_SPLIT
#define CVQ_SORT_SPLIT 1           // 3-D: r0 split at sg0, the second slab (sg0, fg] from the same reduction
#endif
#ifndef CVQ_SORT_SPEC2
#define CVQ_SORT_SPEC2 1           // 2-D: (fg, sg1] reduced beside r0
#endif
#ifndef CVQ_SORT_SKIP
#define CVQ_SORT_SKIP 1            // range sums skip the partial rounds' slots past the range
#endif
// zero words after the node lists: a range sum's prefetch reads up to one round (kSortIlp x the
// widest workgroup) past its range
constexpr int kSortIdxPad = CVQ_SORT_ILP * 1024;
constexpr int kSortIlp = CVQ_SORT_ILP;                // nodes in flight per thread
#ifndef CVQ_SORT_FLAT2
#define CVQ_SORT_FLAT2 1           // 2-D table entries spread flat over 1024-thread workgroups too
#endif
#ifndef CVQ_SORT_ILP_GEN
#define CVQ_SORT_ILP_GEN 1
#endif
// nodes in flight per thread of a range sum: the Student nodes with a general power (PM = 0: a
// fitted nu, exp_node(ex log_node(b))) and the 3-D Student nodes take one at a time, so their
// temporaries fit the registers of 5 (2-D) / 4 (3-D) waves per SIMD: 4 in flight spilled 158-196
// / 68-83 VGPRs and ran the nu = 5.364 solves at a third of the speed (cfg 2 3.3 M vs 9.3 M
// VaR-dates/s), 2 spilled 8-11 and measured 1-3% slower than 1 (profiles/r04r)
// The 512 / 1024-thread 2-D Student instances (6 waves per SIMD, sorted_min_waves) take
// CVQ_SORT_ILP_WIDE_ST.
#ifndef CVQ_SORT_ILP_WIDE_ST
#define CVQ_SORT_ILP_WIDE_ST 1     // 2 spilled 2 VGPRs at 6 waves per SIMD
#endif
__host__ __device__ constexpr int sorted_ilp(int cop, int pm, int dim, int nt = 256) {
    return (cop == CVQ_STUDENT && (pm == 0 || dim == 3)) ? CVQ_SORT_ILP_GEN
         : (cop == CVQ_STUDENT && nt >= 512) ? CVQ_SORT_ILP_WIDE_ST : kSortIlp;
}

constexpr int kSortNT = 256;                          // threads per k_sorted workgroup

// SWEEP (2-D): the first bisection levels from ONE pass over each bracket group's
// nodes.  Pass A covers (lower, sg1] (r0, both second slabs, brackets 0, 1 and 3), pass B bracket
// 2's (sg1, vmax]; a pass records the prefix sum at every boundary of its list -- the fixed
// levels and the mids of the bracket trees' cells holding more than kPassCell nodes (host-pruned
// trees) -- and the levels below those cells run as SORTED's.  kPassMax bounds both lists.
constexpr int kPassCell = 1024;
constexpr int kPassMax = 512;
constexpr int kPassFix = 5;
#ifndef CVQ_PASS_ILP
#define CVQ_PASS_ILP 2                                // steps in flight per wave of a pass
#endif                           // pass A's boundaries of lower, vmin, sg0, fg, sg1

// Date-independent device tables of a SORTED plan.
struct SortedGeom {
    const uint32_t* idx;   // [G + pad] packed node indices, sorted by v* (2-D: i0 | j << 16;
                           //     3-D: a0 | i1 << 9 | j << 17, a0 = i0 + n [i1 == 0], the Q6 plane);
                           //     padded with zero words to a multiple of 4 (+ 4)
    const double* vs;      // [G] the sorted v*
    const int* tree;       // [4][1 << depth]: ub(mid) of heap node h (1 <= h < 2^depth) of each bracket's tree
    int G;
    int depth;
    int fix[6];            // ub() of lower, sg0, fg, sg1, vmin, vmax
    // SWEEP: pass A's then pass B's sorted boundary positions, and per boundary the packed
    // boundary indices of its two child cells' mids in the pruned trees ((left + 1) | (right + 1) << 16,
    // 0 = not subdivided); pass_root[b]: boundary index of bracket b's root mid (-1: none)
    const int* pass_bl;    // [pass_ma + pass_mb]
    const int* pass_ch;    // [pass_ma + pass_mb]
    int pass_ma, pass_mb;
    int pass_fix[kPassFix];
    int pass_root[4];
    int layout;            // node-word layout (sorted_pack)
    // the v*-sorted node words and v* (the solve order above is row-major inside each segment
    // between slab ends; the tail's prefix scan needs the tail cell's nodes in v* order)
    const uint32_t* tidx;
    const double* tvs;
};

// exp_node: cvq_special.h (the fast records clamp their logs at kLogFloor, within its domain)
constexpr double kLogFloor = -1.0e4;
// the Gaussian node's exp: the records carry the exponent's terms scaled by log2(e), so the node is
// 2^E' by exp2_node7 (4.0e-11 relative; no ln2 reduction: two FMAs and a multiply fewer than exp_node7,
// four FMAs fewer than the degree-9 exp_node).  CVQ_SORT_EXP2=0: unscaled records and exp_node7.
#ifndef CVQ_SORT_EXP2
#define CVQ_SORT_EXP2 1
#endif
constexpr double kGaussRecScale = CVQ_SORT_EXP2 ? 1.4426950408889634 : 1.0;   // log2(e)
__device__ __forceinline__ double exp_gauss(double x) { return CVQ_SORT_EXP2 ? exp2_node7(x) : exp_node7(x); }

// b^-(m/2) for the fast path's b = 1 + z^T R^-1 z / nu: the fast path requires finite
// |z| < 1e15 and R is positive definite, so 1 <= b < ~1e31 and b^(m/2) stays finite:
// pow_node_t's overflow guard is dropped (PM > 0: squarings, v_rcp_f64 + one Newton
// step, ~1e-15 relative).
// PM == 0 with m < 0 (a fitted, non-integer nu): b^ex = 2^(ex log2(e) log b), log_node_fast then exp2_node7
// (4.0e-11 relative; no ln2 reduction and no overflow guard: b < ~1e31 here), CVQ_SORT_EXP2=0: pow_node's
// log_node / exp_node (1.4e-14)
template <int PM>
__device__ __forceinline__ double pow_fast(double b, int m, double ex) {
    if constexpr (PM == 0) {
        if (CVQ_SORT_EXP2 && m < 0) return exp2_node7((ex * 1.4426950408889634) * log_node_fast(b));
        return pow_node(b, m, ex);
    } else {
        constexpr int k = PM >> 1;
        double r = 1.0, s2 = b;
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) {
            if ((k >> bit) & 1) r *= s2;
            if ((k >> (bit + 1)) == 0) break;
            s2 *= s2;
        }
        if constexpr (PM & 1) r *= sqrt(b);
        const double y = __builtin_amdgcn_rcp(r);
        return fma(y, fma(-r, y, 1.0), y);
    }
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

// Node words and LDS layouts.  The host packs LDS byte offsets of a node's records into
// its 32-bit word, so the node loop spends 1-2 integer ops per record address:
//   kLay2   (2-D): off0 | off2 << 16, absolute byte offsets (the kernel's LDS starts at 0)
//   kLay3F  (3-D, n <= 128, fixed layout): axis-0 record a0 in bits 4-11 (a0 * 16),
//           i1 in bits 12-18 (32-B axis-1 records), j in bits 25-31 (j * 16)
//   kLay3G  (3-D, n <= 255): a0 | i1 << 9 | j << 17, record indices
// with a0 = i0 + n on the plane i1 == 0 (Q6), whose axis-0 records are separate.
enum { kLay2 = 0, kLay3F = 1, kLay3G = 2 };
constexpr int kLay3FMaxN = 128;
constexpr int kLay3FAx1 = 4096, kLay3FAx2 = 8192, kLay3FBytes = 10240;   // byte offsets / size of its region
__host__ __device__ constexpr int sorted_layout(int dim, int n) {
    return dim == 2 ? kLay2 : (n <= kLay3FMaxN ? kLay3F : kLay3G);
}
inline uint32_t sorted_pack(int layout, int n, int i0, int i1, int j) {
    const int ns = (n + 1) & ~1;
    const int a0 = i0 + (layout != kLay2 && i1 == 0 ? n : 0);
    if (layout == kLay2) return (uint32_t)(16 * i0) | ((uint32_t)(16 * (ns + j)) << 16);
    if (layout == kLay3F) return ((uint32_t)a0 << 4) | ((uint32_t)i1 << 12) | ((uint32_t)j << 25);
    return (uint32_t)a0 | ((uint32_t)i1 << 9) | ((uint32_t)j << 17);
}
// LDS read at an absolute byte address (the packed offsets, valid because the kernel has no
// static LDS: its dynamic region starts at address 0 -- checked at kernel start).  Going
// through the extern array instead adds its (link-time, zero) address to every record.
typedef __attribute__((address_space(3))) const double lds_f64;
typedef double f64x2_t __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const f64x2_t lds_f64x2;
__device__ __forceinline__ const lds_f64* lds_at(uint32_t byte_off) { return (const lds_f64*)(size_t)byte_off; }
__device__ __forceinline__ uint32_t lds_base(const double* p) {
    return (uint32_t)(size_t)(__attribute__((address_space(3))) const double*)p;
}

// record indices (a0, i1, j) of a node word (the generic path's view)
template <int LAY>
__device__ __forceinline__ void unpack_node(uint32_t c, int ns, int* a0, int* i1, int* j) {
    if constexpr (LAY == kLay2) {
        *a0 = (int)(c & 0xFFFFu) >> 4;
        *i1 = 0;
        *j = ((int)(c >> 16) >> 4) - ns;
    } else if constexpr (LAY == kLay3F) {
        *a0 = (int)__builtin_amdgcn_ubfe(c, 4, 8);
        *i1 = (int)__builtin_amdgcn_ubfe(c, 12, 7);
        *j = (int)(c >> 25);
    } else {
        *a0 = (int)__builtin_amdgcn_ubfe(c, 0, 9);
        *i1 = (int)__builtin_amdgcn_ubfe(c, 9, 8);
        *j = (int)(c >> 17);
    }
}

// LDS doubles per grid point of the table region: the generic tables (3 DIM) or the
// fast records (16-B records per axis entry, 3-D: axis 0 twice + one extra axis-1
// value), whichever is larger; arrays are laid out with an even stride so every
// double2 is 16-B aligned.  16-B records keep a node at 32 B of LDS reads (2-D):
// the node loop is LDS-bandwidth bound, so wider records cost more than the VALU
// work they save (measured).
// largest n the kernel's register tables hold: 1024 in 2-D (the 16-bit LDS byte offsets of kLay2
// reach 16 (2 ns - 1) < 2^16), the 8-bit packing's 255 in 3-D.  Per width: the 256- to 512-thread
// 2-D instances hold n <= 512 (one or two grid indices per thread); n > 512 runs the 1024-thread
// instance (sorted_threads), so the others keep their register budget
__host__ __device__ constexpr int sorted_max_n(int dim) { return dim == 2 ? 1024 : 255; }
__host__ __device__ constexpr int sorted_max_n_nt(int dim, int nt) {
    return dim == 2 ? (nt >= 1024 ? 1024 : 512) : 255;
}
inline int sorted_stride(int n) { return (n + 1) & ~1; }
// doubles of the table region
__host__ __device__ inline int sorted_region_doubles(int layout, int n) {
    const int ns = (n + 1) & ~1;
    return layout == kLay2 ? 6 * ns : layout == kLay3F ? kLay3FBytes / 8 : 9 * ns;
}
constexpr int kSortScalars = 4;                // flags, arest, last (+ pad), after the reduction slots
inline size_t sorted_lds_bytes(int n, int nt, int dim, bool sweep = false, int layout = -1) {
    if (layout < 0) layout = sorted_layout(dim, n);
    // SWEEP: wave-total slots [NT / 64] + per boundary its prefix value, position and children
    const size_t sw = sweep ? sizeof(double) * ((size_t)nt / 64 + kPassMax) + sizeof(int) * 2 * kPassMax : 0;
    return sizeof(double) * ((size_t)sorted_region_doubles(layout, n) + 4 * (nt / 64) + kSortScalars) +
           sizeof(double2) * sorted_tail_cap(dim) + sw;
}

// mode 0: calc_var solve (snapshots + header, fused finalize when P.fin_var);
// mode 1: one slab per date (compute_integral): out[t] = I_t(bounds[2t], bounds[2t+1]].
// Minimum waves per SIMD asked of the register allocator: 5 for 2-D (measured
// +15% on config 5, neutral on 2), 4 for 3-D (<= 128 VGPRs; its exp chain sits at
// that boundary, and 5 measured slower).
#ifndef CVQ_SORT_MIN_WAVES2
#define CVQ_SORT_MIN_WAVES2 5
#endif
#ifndef CVQ_SORT_MIN_WAVES3
#define CVQ_SORT_MIN_WAVES3 4
#endif
#ifndef CVQ_SORT_MIN_WAVES2W
#define CVQ_SORT_MIN_WAVES2W 6     // 2-D, 512 / 1024 threads: three 512-thread dates per CU
#endif
// waves per SIMD the kernel is compiled for (its register budget).  The wide 2-D instances only
// run small date blocks (sorted_threads), where residency beats registers: at 6 waves a CU holds
// three 512-thread dates, so a 625-date block is resident at once (cfg 5: 103 -> 97 us); the
// 256-thread instances keep 5 (6 cost the full batch 5%, profiles/r04q)
// (the Student instances with a general power stay at 5: their quantile and node temporaries
// spill 13-15 VGPRs at 6).  cop / pm = -1: the width rule's generic value.
__host__ __device__ constexpr int sorted_min_waves(int dim, int nt = 256, int cop = -1, int pm = -1) {
    return dim == 2 ? ((nt >= 512 && !(cop == CVQ_STUDENT && pm == 0)) ? CVQ_SORT_MIN_WAVES2W : CVQ_SORT_MIN_WAVES2)
                    : CVQ_SORT_MIN_WAVES3;
}

// SWEEP (2-D): the fixed slabs and the first bisection levels come from one pass
// per bracket group instead of one strided range sum + one workgroup reduction per level: a
// pass evaluates every node of its range once, each wave a contiguous run of 64-position steps,
// recording the prefix sum at every boundary of its (host-pruned) list; every thread then walks
// those levels from LDS (slab = difference of two prefixes) with no further barrier, and the
// levels below the pruned trees run as SORTED's.  Pass A covers (lower, sg1], so r0, the second
// slab and brackets 0, 1, 3 need no other pass; bracket 2 (sg1, vmax] takes pass B.
template <int COP, bool MSM, int DIM, int NT, int PM, bool FUSED, int LAY, bool SWEEP = false>
__global__ __launch_bounds__(NT, sorted_min_waves(DIM, NT, COP, PM)) void k_sorted(StaticDev S, SolveConst P, SortedGeom G, const double* __restrict__ a,
                                               const double* __restrict__ tA, const double* __restrict__ tB,
                                               const double* __restrict__ pi, int mode,
                                               const double* __restrict__ bounds, double* __restrict__ out,
                                               double* __restrict__ snaps, Header* hdr, double* __restrict__ stamps_out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    constexpr int TPL = sorted_tail_per_lane(DIM), TCAP = sorted_tail_cap(DIM);
    const int n = S.n, tid = threadIdx.x, lane = tid & 63;
    const int ns = (n + 1) & ~1;                   // sorted_stride(n)
    const long long t = blockIdx.x;
    // One LDS region holds EITHER the generic tables (reference semantics: z, B, w per
    // axis; axis 0 of 3-D: w = the i1 == 0 weight) OR the fast records (16 B per axis
    // entry; 3-D axis 0 twice, [n, 2n) = the plane i1 == 0), chosen per date.
    // (no static __shared__ variables: the dynamic region starts at LDS address 0, so the
    // host-packed record offsets are addresses)
    double* zg = lds;                              // generic [DIM][n]
    double* Bg = zg + DIM * ns;                    // generic [DIM][n]
    double* wg = Bg + DIM * ns;                    // generic [DIM][n]
    double* fr0 = lds;                             // fast [ns (3-D: 2 ns)][2] axis 0
    // axis 1 (3-D): kLay3F 32-B records (c01 z1, c12 z1, g1 | z1, B'1); kLay3G [ns][2] + fg1 [ns]
    double* fr1 = LAY == kLay3F ? lds + kLay3FAx1 / 8 : fr0 + (DIM == 3 ? 4 : 2) * ns;
    double* fg1 = LAY == kLay3F ? fr1 + 2 : fr1 + (DIM == 3 ? 2 : 0) * ns;
    constexpr int R1 = LAY == kLay3F ? 4 : 2;      // doubles per axis-1 record
    constexpr int FG = LAY == kLay3F ? 4 : 1;      // fg1 stride
    double* fr2 = LAY == kLay3F ? lds + kLay3FAx2 / 8 : fg1 + (DIM == 3 ? 1 : 0) * ns;   // fast [ns][2] inner axis
    double2* tail = (double2*)(lds + sorted_region_doubles(LAY, n));   // [TCAP] (v*, value)
    double* red = (double*)(tail + TCAP);          // [2 parity][2 values][NT / 64] reduction slots
    int& flags = *(int*)(red + 4 * (NT / 64));     // bit 0: non-finite or zero table entry, bit 1: pi not rank 1
    double& s_arest = *(red + 4 * (NT / 64) + 1);  // 3-D: the axis-0 weight off the plane i1 == 0
    int& last = *(int*)(red + 4 * (NT / 64) + 2);  // fused finalize: this workgroup is the last
    double* sred = red + 4 * (NT / 64) + kSortScalars;   // SWEEP: [NT / 64] wave totals
    double* Pvs = sred + NT / 64;                  // SWEEP: [kPassMax] prefix values (pass A, then B)
    int* Bls = (int*)(Pvs + kPassMax);             // SWEEP: [kPassMax] boundary positions
    int* Chs = Bls + kPassMax;                     // SWEEP: [kPassMax] packed child boundaries

    // diagnostic phase stamps (CVQ_STAMPS=1, never in a timed run): COMPACT's slots --
    // 0 start, 1 tables, 2 first slab, 3 second slab, 4 bracket, 5 + level, 29 tail
    // build, 31 end, 25 / 26 realtime; 28 = nodes this date evaluated
    unsigned long long* stamps = stamps_out ? (unsigned long long*)stamps_out + t * 32 : nullptr;
    auto stamp = [&](int idx) {
        if (stamps && tid == 0 && idx < 32) stamps[idx] = __builtin_amdgcn_s_memtime();
    };
    long long nodes = 0;                           // nodes evaluated (thread 0, stamps only)
    stamp(0);
    if (stamps && tid == 0) {
        stamps[25] = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
        stamps[30] = blockIdx.x;                         // dispatch position (placement analysis)
        // placement: HW_ID (wave, SIMD, CU, SH, SE fields) and XCC_ID of this workgroup's first wave
        stamps[27] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                     ((unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32);
    }
    if (tid == 0) flags = 0;
    __syncthreads();
    // ---- tables: grid index i of every axis (table_entry; W factors of the rank-1 pi), the
    // axes unrolled so their latencies overlap; kept in registers until the path is chosen.
    // The DIM n entries are spread flat over the workgroup (entry e = tid + NT k is axis e / n,
    // index e mod n), so a wide workgroup's table phase is one entry deep (cfg 4 at 1024 threads:
    // 384 of them busy instead of 128; cfg 3's 512-point grid at 1024 threads: one entry per
    // thread instead of both axes on half of them; a lone date's table phase is on its latency
    // chain).  Otherwise (2-D below 1024 threads, or CVQ_SORT_FLAT2=0) thread tid holds indices
    // tid + NT k of both axes.
    constexpr int RPT = (sorted_max_n_nt(DIM, NT) + NT - 1) / NT;   // grid indices per thread
    constexpr bool FLAT = DIM == 3 || (CVQ_SORT_FLAT2 && NT >= 1024);   // 2-D at 512 threads: same depth, the division cost 1.5%
    constexpr int EPT = FLAT ? (DIM * sorted_max_n_nt(DIM, NT) + NT - 1) / NT : RPT * DIM;   // entries per thread
    constexpr int ILP = sorted_ilp(COP, PM, DIM, NT);              // range sums' nodes in flight
    const int q = MSM ? S.q : 1;
    const double* fb = MSM ? a + t * DIM * q : nullptr;     // forecasts_by_states[t] (DIM, q)
    double eA[EPT], eB[EPT], eW[EPT];
    auto slot = [&](int sl, int& ax, int& i) -> bool {      // entry sl of this thread: (axis, index)
        if constexpr (FLAT) {
            const int e = tid + sl * NT;
            ax = e / n;
            i = e - ax * n;
            return ax < DIM;
        } else {
            ax = sl % DIM;
            i = tid + (sl / DIM) * NT;
            return i < n;
        }
    };
    int bad = 0;
#pragma unroll
    for (int sl = 0; sl < EPT; ++sl) {
        int ax, i;
        if (!slot(sl, ax, i)) continue;
        {
            double A, B;
            if constexpr (FUSED) {
                table_entry<COP, MSM, COP == CVQ_STUDENT, (COP == CVQ_STUDENT && PM == 6 + DIM) ? 6 : 0>(
                    S, a, t * DIM + ax, ax, i, &A, &B);
            } else {
                A = tA[(t * DIM + ax) * n + i];
                B = tB[(t * DIM + ax) * n + i];
            }
            // 2-D: pi[a][b] = f0[a] f1[b]; 3-D: pi[L0][L1][L2] = f0[L1] f1[L2] f2[L0] (Q7)
            const int fax = DIM == 2 ? ax : (ax + 2) % 3;
            double w;
            if constexpr (MSM) {
                w = 0.0;
                for (int s2 = 0; s2 < q; ++s2) w = fma(fb[fax * q + s2], S.F[((size_t)ax * q + s2) * n + i], w);
            } else {
                w = S.F[(size_t)ax * n + i];
            }
            if (!(COP == CVQ_STUDENT && !MSM && !isfinite(A))) {   // dead entries: below
                if (!isfinite(A) || !isfinite(B)) bad |= 1;
                if (!(B * w > 0.0)) bad |= 1;              // fast records take logs of B w
                if (!(fabs(A) < 1.0e15)) bad |= 1;         // fast powers / exps need a bounded quadratic form
            }
            eA[sl] = A;
            eB[sl] = B;
            eW[sl] = w;
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
        double s0 = 1.0;
        if constexpr (MSM) {
            s0 = 0.0;
            for (int L = 0; L < q; ++L) s0 += fb[2 * q + L];
        }
        s_arest = s0;
    }
    if (tid == 0 && lds_base(lds) != 0) bad |= 4;          // packed offsets need the region at LDS 0
    if constexpr (SWEEP) {                                 // both passes' boundary lists -> LDS
        for (int k = tid; k < G.pass_ma + G.pass_mb; k += NT) {
            Bls[k] = G.pass_bl[k];
            Chs[k] = G.pass_ch[k];
        }
    }
    if (bad) atomicOr(&flags, bad);
    __syncthreads();
    const int fl = flags;
    const bool rank1 = !(fl & 2);
    const bool fast = rank1 && !(fl & 5);
    const double arest = DIM == 3 ? s_arest : 1.0;
    // Gaussian: -z^T R^-1 z / 2 = sum_c -Ri_cc z_c^2 / 2 + c01 z0 z1 + c02 z0 z2 + c12 z1 z2;
    // Student: 1 + z^T R^-1 z / nu = 1 + sum_c a_cc z_c^2 + a01 z0 z1 + a02 z0 z2 + a12 z1 z2
    const double kq = COP == CVQ_GAUSSIAN ? -0.5 : S.inv_nu;
    const double k01 = kq * (S.Ri[1] + S.Ri[DIM]);
    const double k02 = DIM == 2 ? k01 : kq * (S.Ri[2] + S.Ri[6]);
    const double k12 = DIM == 3 ? kq * (S.Ri[5] + S.Ri[7]) : 0.0;
    const double g02 = kGaussRecScale * k02;                // the Gaussian 3-D node's (0, 2) cross term, scaled
#pragma unroll
    for (int sl = 0; sl < EPT; ++sl) {
      int ax, i;
      if (!slot(sl, ax, i)) continue;
      {
        const double z = eA[sl], B = eB[sl], w = eW[sl];
        if (!fast) {
            zg[ax * n + i] = z;
            Bg[ax * n + i] = B;
            wg[ax * n + i] = w;
            continue;
        }
        const double kcc = kq * S.Ri[ax * (DIM + 1)] * (z * z);          // diagonal term of axis ax
        if constexpr (COP == CVQ_GAUSSIAN) {
            // log factors g = log(B w) - Ri_cc z^2 / 2, clamped at kLogFloor; E = sum g + cross; every
            // term that enters E scaled by kGaussRecScale (E' = E log2(e), the node 2^E')
            constexpr double L = kGaussRecScale;
            auto lg = [](double v) { return fmax(log(v), kLogFloor); };
            if (ax == 0) {
                fr0[2 * i] = DIM == 2 ? (L * k02) * z : z;
                fr0[2 * i + 1] = L * (lg(S.term1 * B * (DIM == 3 ? arest : w)) + kcc);
                if (DIM == 3) {                                              // plane i1 == 0 (Q6)
                    fr0[2 * (n + i)] = z;
                    fr0[2 * (n + i) + 1] = L * (lg(S.term1 * B * w) + kcc);
                }
            } else if (ax == DIM - 1) {
                fr2[2 * i] = z;
                fr2[2 * i + 1] = L * (lg(B * w) + kcc);
            } else {
                fr1[R1 * i] = (L * k01) * z;
                fr1[R1 * i + 1] = (L * k12) * z;
                fg1[FG * i] = L * (lg(B * w) + kcc);
            }
        } else if constexpr (COP == CVQ_PLACKETT) {       // rec0 = (-2 u, theta s), rec2 = ((theta - 1) v, s)
            double* r = ax == 0 ? fr0 + 2 * i : fr2 + 2 * i;
            r[0] = ax == 0 ? -2.0 * z : (S.theta - 1.0) * z;
            r[1] = (ax == 0 ? S.theta : 1.0) * (B * w);
        } else {                                           // Student: z and scale
            // GARCH / UKF: a dead entry (u in {0, 1}: z = +-inf, or NaN) zeroes every node through
            // it in the reference -- a non-finite z gives multivariate and univariate t pdfs of
            // 0 (student.py:130-131, :166-167), 0 / 0 = NaN, nan_to_num -> 0
            // (garch_integration_function.py:48) -- so its record is (0, 0): those nodes evaluate
            // to +0 on the fast path (scale 0 times a finite power) instead of sending the date to
            // the generic path (27% of cfg 5's dates hold such grid-edge entries)
            const bool dead = !MSM && !isfinite(z);
            const double sc = dead ? 0.0 : (ax == 0 ? S.term1 : 1.0) * B * (ax == 0 && DIM == 3 ? arest : w);
            const double zr = dead ? 0.0 : z;
            double* r = ax == 0 ? fr0 + 2 * i : ax == DIM - 1 ? fr2 + 2 * i : fr1 + R1 * i;
            r[0] = zr;
            r[1] = sc;
            if (DIM == 3 && ax == 0) {                                       // plane i1 == 0 (Q6)
                fr0[2 * (n + i)] = zr;
                fr0[2 * (n + i) + 1] = dead ? 0.0 : S.term1 * B * w;
            }
        }
      }
    }
    __syncthreads();

    stamp(1);
    // Student: b = 1 + z^T R^-1 z / nu = 1 + z0 (a00 z0 + k01 z1 + k02 z2) + z1 (a11 z1 + k12 z2) + a22 z2^2
    const double a00 = kq * S.Ri[0], a11 = kq * S.Ri[DIM + 1], a22 = kq * S.Ri[DIM * DIM - 1];
    // LDS records of a node word (host-packed offsets, see sorted_pack)
    auto rd2 = [](const lds_f64* r) {                  // one ds_read_b128
        const f64x2_t v = *(const lds_f64x2*)r;
        return make_double2(v.x, v.y);
    };
    auto rec0 = [&](uint32_t c) -> const lds_f64* {
        if constexpr (LAY == kLay2) return lds_at(c & 0xFFFFu);
        else if constexpr (LAY == kLay3F) return lds_at(c & 0xFF0u);
        else return lds_at(lds_base(fr0) + 16 * __builtin_amdgcn_ubfe(c, 0, 9));
    };
    auto rec1 = [&](uint32_t c) -> const lds_f64* {
        if constexpr (LAY == kLay3F) return lds_at(kLay3FAx1 + ((c >> 7) & 0xFE0u));
        else return lds_at(lds_base(fr1) + 16 * __builtin_amdgcn_ubfe(c, 9, 8));
    };
    auto rec2 = [&](uint32_t c) -> const lds_f64* {
        if constexpr (LAY == kLay2) return lds_at(c >> 16);
        else if constexpr (LAY == kLay3F) return lds_at(kLay3FAx2 + (c >> 21));
        else return lds_at(lds_base(fr2) + 16 * (c >> 17));
    };
    // Plackett node (plackett.py:66-69, Q11) from the records (-2 u, theta s0), (a1 v, s2),
    // a1 = theta - 1: P = 1 + a1 (u + v), num / theta = 1 + a1 (u + v - 2 u v) = P + (-2 u)(a1 v),
    // denominator (P (theta + 1 - P))^2 -- 12 FP64 operations and one reciprocal a node: v_rcp_f64
    // (2^-24.4) and one Newton step, 2.2e-15 relative (profiles/r04f/rcp_probe.txt), as pow_fast's
    // Student reciprocal (the VaR is unchanged by 1e-8 relative node noise)
    const double pl_h = -0.5 * (S.theta - 1.0), pl_k = S.theta + 1.0;
    auto plackett = [&](const double2 A, const double2 C) -> double {
        const double P = fma(pl_h, A.x, 1.0 + C.x);
        const double num = fma(A.x, C.x, P);
        const double d = P * (pl_k - P);
        const double den = d * d;
        double y = __builtin_amdgcn_rcp(den);
        y = fma(y, fma(-den, y, 1.0), y);
        y = den == 0.0 ? __builtin_inf() : y;             // num / 0 as IEEE division gives it (num * inf)
        return (num * y) * (A.y * C.y);
    };
    auto node_fast = [&](uint32_t c) -> double {
        const double2 A = rd2(rec0(c));
        const double2 C = rd2(rec2(c));
        if constexpr (COP == CVQ_GAUSSIAN) {
            if constexpr (DIM == 2) {
                return exp_gauss(fma(A.x, C.x, A.y + C.y));
            } else {
                const lds_f64* r1 = rec1(c);
                const double2 Bv = rd2(r1);
                const double g1 = LAY == kLay3F ? r1[2] : fg1[__builtin_amdgcn_ubfe(c, 9, 8)];
                return exp_gauss(fma(A.x, fma(g02, C.x, Bv.x), fma(Bv.y, C.x, (A.y + g1) + C.y)));
            }
        } else if constexpr (COP == CVQ_STUDENT) {
            double b, sc;
            if constexpr (DIM == 2) {
                b = fma(A.x, fma(a00, A.x, k02 * C.x), fma(a22 * C.x, C.x, 1.0));
                sc = A.y * C.y;
            } else {
                const double2 Bv = rd2(rec1(c));
                b = fma(A.x, fma(a00, A.x, fma(k01, Bv.x, k02 * C.x)), fma(Bv.x, fma(a11, Bv.x, k12 * C.x),
                                                                              fma(a22 * C.x, C.x, 1.0)));
                sc = (A.y * Bv.y) * C.y;
            }
            return sc * pow_fast<PM>(b, S.node_m, S.node_ex);
        } else {                                           // Plackett, 2-D
            return plackett(A, C);
        }
    };
    auto node_generic = [&](uint32_t c) -> double {
        int i0, i1, j;
        unpack_node<LAY>(c, ns, &i0, &i1, &j);
        if (DIM == 3 && i0 >= n) i0 -= n;                  // the plane's axis-0 record index
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
    // sum of the nodes at sorted positions [p0, p1), strided over the workgroup: the rounds start
    // at p0 rounded down to 64, so position q is always read by lane q mod 64; the first round
    // is predicated below p0, the last
    // (partial) one above p1, so their index loads are in flight together
    auto range_sum = [&](int p0, int p1) -> double {
        double acc[ILP];
#pragma unroll
        for (int u = 0; u < ILP; ++u) acc[u] = 0.0;
        int p = (p0 & ~63) + tid;
        if (fast && p0 < p1) {
            // the next round's node words are loaded before this round's nodes are evaluated (a
            // few dates per CU leave too few waves to cover the L2 latency of unpipelined loads).
            // Loads run up to a round past p1 (the lists carry kSortIdxPad zero words) and from
            // p0 rounded down to 64 (>= 0): unconditional, the first and last rounds select their
            // out-of-range nodes away
            uint32_t cn[ILP];
            const uint32_t* ip = G.idx + p;                // this thread's words of the next round
            {                                              // first round: positions below p0 masked
                uint32_t c[ILP];
#pragma unroll
                for (int u = 0; u < ILP; ++u) c[u] = ip[u * NT];
                ip += ILP * NT;
#pragma unroll
                for (int u = 0; u < ILP; ++u) cn[u] = ip[u * NT];
                // a slot whose wave starts at or past p1 holds no node of the range (short ranges):
                // skipped (the test is wave-uniform, lane 0 holds the wave's lowest position)
                const int wb = __builtin_amdgcn_readfirstlane(p);
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    if (CVQ_SORT_SKIP && wb + u * NT >= p1) continue;
                    const int q = p + u * NT;
                    const double v = node_fast(c[u]);
                    acc[u] += (q >= p0 && q < p1) ? v : 0.0;
                }
                p += ILP * NT;
            }
            uint32_t cm[ILP];
            // full rounds in pairs, the word buffers alternating (no register copies)
            for (; p + (2 * ILP - 1) * NT < p1; p += 2 * ILP * NT) {
                ip += ILP * NT;
#pragma unroll
                for (int u = 0; u < ILP; ++u) cm[u] = ip[u * NT];
#pragma unroll
                for (int u = 0; u < ILP; ++u) acc[u] += node_fast(cn[u]);
                ip += ILP * NT;
#pragma unroll
                for (int u = 0; u < ILP; ++u) cn[u] = ip[u * NT];
#pragma unroll
                for (int u = 0; u < ILP; ++u) acc[u] += node_fast(cm[u]);
            }
            if (p + (ILP - 1) * NT < p1) {            // an odd full round
                ip += ILP * NT;
#pragma unroll
                for (int u = 0; u < ILP; ++u) cm[u] = ip[u * NT];
#pragma unroll
                for (int u = 0; u < ILP; ++u) acc[u] += node_fast(cn[u]);
#pragma unroll
                for (int u = 0; u < ILP; ++u) cn[u] = cm[u];
                p += ILP * NT;
            }
            if (p < p1) {                                  // last round: positions from p1 on masked
                const int wb = __builtin_amdgcn_readfirstlane(p);
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    if (CVQ_SORT_SKIP && wb + u * NT >= p1) continue;
                    const double v = node_fast(cn[u]);
                    acc[u] += p + u * NT < p1 ? v : 0.0;
                }
            }
        } else {
            for (p = p0 + tid; p < p1; p += NT) acc[0] += node_generic(G.idx[p]);
        }
#pragma unroll
        for (int h = 1; h < ILP; h <<= 1)
#pragma unroll
            for (int u = 0; u + h < ILP; u += 2 * h) acc[u] += acc[u + h];
        return acc[0];
    };
    int parity = 0;
    auto team_sum = [&](double v) {                        // workgroup sum, identical in every thread; one barrier
        v = wave_sum(v);
        if constexpr (NT == 64) return v;
        double* rr = red + parity * (2 * (NT / 64));
        parity ^= 1;
        if (lane == 0) rr[tid >> 6] = v;
        __syncthreads();
        double s0 = rr[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) s0 += rr[w];
        return s0;
    };
    auto team_sum2 = [&](double v0, double v1, double& s0, double& s1) {   // two sums, one barrier
        v0 = wave_sum(v0);
        v1 = wave_sum(v1);
        double* rr = red + parity * (2 * (NT / 64));
        parity ^= 1;
        if (lane == 0) {
            rr[tid >> 6] = v0;
            rr[NT / 64 + (tid >> 6)] = v1;
        }
        __syncthreads();
        s0 = rr[0];
        s1 = rr[NT / 64];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) {
            s0 += rr[w];
            s1 += rr[NT / 64 + w];
        }
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
    // SWEEP pass: the nodes at sorted positions [ps, pe) summed once.  Wave w takes a contiguous
    // run of 64-position steps from ps rounded down to 64 (lane = position mod 64, the lanes of a
    // step reading consecutive positions as SORTED's range sums do), ILP steps per round with the
    // next round's node words in flight; each lane keeps a running sum.  At a step holding
    // boundaries (wave-uniform test) the wave reduces, per boundary, the running sums plus the
    // step's values below it: the wave's partial prefix.  The wave totals' exclusive scan then
    // turns partials into Pv[k] = sum of the nodes at [ps, Bl[k]) for every boundary k (ps <= Bl[k]
    // <= pe, sorted).  Returns the total; ends with a barrier.
    auto pass = [&](int ps, int pe, const int* Bl, double* Pv, int M) -> double {
        constexpr int W = NT / 64;
        constexpr int PILP = ILP < CVQ_PASS_ILP ? ILP : CVQ_PASS_ILP;
        const int wv = tid >> 6;
        const int a0 = ps & ~63;
        const int nsteps = (max(pe, a0) - a0 + 63) >> 6;
        const int spw = (nsteps + W - 1) / W;              // steps per wave
        const int rs = a0 + wv * spw * 64;                 // this wave's positions [rs, re)
        const int re = wv == W - 1 ? 0x7FFFFFFF : rs + spw * 64;
        const int nst = max(0, min(spw, nsteps - wv * spw));
        int i = 0;
        for (int hiI = M; i < hiI;) {                      // first boundary >= rs (wave-uniform)
            const int md = (i + hiI) >> 1;
            if (Bl[md] < rs) i = md + 1; else hiI = md;
        }
        const int i0 = i;
        int nb = i < M ? Bl[i] : 0x7FFFFFFF;
        double run = 0.0;
        auto sweep_steps = [&](auto nodef, auto ilp) {
            constexpr int PI = decltype(ilp)::value;
            const uint32_t* ip = G.idx + rs + lane;
            uint32_t cn[PI];
#pragma unroll
            for (int u = 0; u < PI; ++u) cn[u] = ip[u * 64];
            for (int st = 0; st < nst; st += PI) {
                uint32_t c[PI];
#pragma unroll
                for (int u = 0; u < PI; ++u) c[u] = cn[u];
                ip += PI * 64;                            // the lists carry kSortIdxPad zero words
#pragma unroll
                for (int u = 0; u < PI; ++u) cn[u] = ip[u * 64];
                double v[PI];
#pragma unroll
                for (int u = 0; u < PI; ++u) {
                    const int q = rs + (st + u) * 64 + lane;
                    const double x = nodef(c[u]);
                    v[u] = (q >= ps && q < pe) ? x : 0.0;
                }
#pragma unroll
                for (int u = 0; u < PI; ++u) {
                    if (st + u >= nst) break;
                    const int sb = rs + (st + u) * 64;
                    while (nb < sb + 64) {                 // boundaries inside this step (rare)
                        const double part = wave_sum(run + ((lane < nb - sb) ? v[u] : 0.0));
                        if (lane == 0) Pv[i] = part;
                        ++i;
                        nb = i < M ? Bl[i] : 0x7FFFFFFF;
                    }
                    run += v[u];
                }
            }
        };
        if (fast) sweep_steps(node_fast, std::integral_constant<int, PILP>());
        else sweep_steps(node_generic, std::integral_constant<int, 1>());   // reference-semantics nodes one at a time
        const double wt = wave_sum(run);
        while (nb < re) {                                  // boundaries past my last step (pe, or empty steps)
            if (lane == 0) Pv[i] = wt;
            ++i;
            nb = i < M ? Bl[i] : 0x7FFFFFFF;
        }
        if (lane == 0) sred[wv] = wt;
        __syncthreads();
        double base = 0.0, total = 0.0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const double sw = sred[w];
            if (w < wv) base += sw;
            total += sw;
        }
        for (int k = i0 + lane; k < i; k += 64) Pv[k] += base;
        __syncthreads();
        return total;
    };

    // solve state (calc_var_class.py:114-160 and the bisection's :250-309)
    double lo = __builtin_nan(""), hi = __builtin_nan("");
    int br = -1;                                           // bracket (tree) index; -1: NaN bracket (Q3)
    bool ustack = false;
    int plo = 0, phi = 0;                                  // the bracket's sorted positions [plo, phi)
    int h = 1;                                             // heap index of (lo, hi) in the bracket's tree
    const int* tr = G.tree;
    int tsz = 0;                                           // tabulated heap nodes [1, tsz)
    double prev = 0.0, prevU = 0.0;
    int nt = -1, it = 0;
    uint64_t mask = 0;
    double* sn = snaps + t * P.stride;
    // (i)-(iii) from r0 = I(lower, fg] and the second slab nr (Q1, Q3)
    auto bracket = [&](double r0, double nl, double nu, double nr) {
        const double F = (nl == P.fg) ? r0 + nr : r0 - nr;
        if (F > P.obj) { lo = P.vmin; hi = P.sg0; br = 0; }
        if (F < P.obj && nu == P.fg) { lo = P.sg0; hi = P.fg; br = 1; }
        if (F < P.obj && nu == P.sg1) { lo = P.sg1; hi = P.vmax; br = 2; }
        if (F > P.obj && nu == P.sg1) { lo = P.fg; hi = P.sg1; br = 3; }
        ustack = !(hi == P.sg0 || hi == P.sg1);
        plo = br >= 0 ? fixpos(lo) : 0;
        phi = br >= 0 ? max(fixpos(hi), plo) : 0;
        tr = G.tree + (max(br, 0) << G.depth);
        tsz = br >= 0 ? (1 << G.depth) : 0;
        prev = F;
        prevU = (nl == P.sg0) ? P.sg0 : P.fg;
        stamp(4);
    };
    // one bisection level from a slab value (adjust_integral :214-248, Q4 mask)
    auto level = [&](double mid, double val) {
        const double slab_lower = ustack ? lo : mid;
        const double Fn = (slab_lower == prevU) ? prev + val : prev - val;
        if (Fn != 0.0) mask |= (1ull << it);
        ustack = Fn < P.obj;
        prev = Fn;
        prevU = mid;
        return ustack;
    };
    bool passed = false;                                   // SWEEP: the passes gave the first levels
    if constexpr (SWEEP) {
      if (G.pass_ma > 0) {
        passed = true;
        // pass A over (lower, sg1]: r0 = I(lower, fg], both candidate second slabs and the pruned
        // trees of brackets 0, 1, 3 (its list holds lower, vmin, sg0, fg, sg1 at pass_fix[])
        const double totA = pass(G.fix[0], G.fix[3], Bls, Pvs, G.pass_ma);
        (void)totA;
        stamp(2);
        nodes += max(G.fix[3] - G.fix[0], 0);
        const double Pl = Pvs[G.pass_fix[0]], Ps0 = Pvs[G.pass_fix[2]], Pfg = Pvs[G.pass_fix[3]],
                     Ps1 = Pvs[G.pass_fix[4]];
        auto pfx = [&](double v) { return v == P.lower ? Pl : v == P.sg0 ? Ps0 : v == P.fg ? Pfg : Ps1; };
        const double r0 = Pfg - Pl;
        const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
        const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
        bracket(r0, nl, nu, pfx(nu) - pfx(nl));
        const int* Bl = Bls;
        const int* Ch = Chs;
        const double* Pv = Pvs;
        int ilo = 0, ihi = 0;                              // boundary indices of the cell's ends
        if (br == 0) { ilo = G.pass_fix[1]; ihi = G.pass_fix[2]; }
        if (br == 1) { ilo = G.pass_fix[2]; ihi = G.pass_fix[3]; }
        if (br == 3) { ilo = G.pass_fix[3]; ihi = G.pass_fix[4]; }
        if (br == 2) {                                     // pass B over the bracket's cell (sg1, vmax]
            Bl = Bls + G.pass_ma;
            Ch = Chs + G.pass_ma;
            Pv = Pvs + G.pass_ma;
            pass(plo, phi, Bl, Pvs + G.pass_ma, G.pass_mb);
            nodes += phi - plo;
            ilo = 0;
            ihi = G.pass_mb - 1;
        }
        stamp(3);
        // the pruned tree's levels from LDS, no barrier: slab = difference of two prefixes
        int im = br >= 0 ? G.pass_root[br] : -1;
        while (im >= 0 && it < P.K && phi - plo > TCAP) {
            const double mid = (lo + hi) / 2;
            if (tid == 0) sn[it] = mid;
            if (nt < 0 && !(hi - lo > P.tol)) nt = it;
            const double Pm = Pv[im];
            const int c = Ch[im];
            if (level(mid, ustack ? Pm - Pv[ilo] : Pv[ihi] - Pm)) { lo = mid; plo = Bl[im]; ilo = im; im = (c >> 16) - 1; }
            else                                                 { hi = mid; phi = Bl[im]; ihi = im; im = (c & 0xFFFF) - 1; }
            h = 2 * h + (ustack ? 1 : 0);
            ++it;
        }
      }
    }
    if (!passed) {
        // 3-D: r0 = I(lower, fg] as (lower, sg0] + (sg0, fg] when the positions are ordered -- the
        // second slab (sg0, fg] of the dates with r0 >= obj (cfg 4: 99.6% of its dates, VaR below -3.5)
        // then comes from the same pass and reduction instead of being evaluated a second time.  Not
        // in 2-D: the BASELINE 2-D workloads' dates have r0 < obj, and the extra live sum costs the
        // Plackett instances an occupancy step (75 -> 81 VGPRs)
        const bool split = CVQ_SORT_SPLIT && DIM == 3 && G.fix[0] <= G.fix[1] && G.fix[1] <= G.fix[2];
        // 2-D: the second slab's usual candidate (fg, sg1] (every BASELINE 2-D date has r0 < obj) is
        // summed beside r0 and reduced with it -- one phase and barrier fewer on the date's chain; the
        // same range sums and reduction order as alone, so the values are bit-identical
        const bool spec2 = CVQ_SORT_SPEC2 && DIM == 2 && G.fix[2] <= G.fix[3];
        double r0, n2 = 0.0;
        if (split) {
            const double p2 = range_sum(G.fix[1], G.fix[2]);
            team_sum2(range_sum(G.fix[0], G.fix[1]) + p2, p2, r0, n2);
        } else if (spec2) {
            const double p0 = range_sum(G.fix[0], G.fix[2]);
            team_sum2(p0, range_sum(G.fix[2], G.fix[3]), r0, n2);
        } else {
            r0 = team_sum(range_sum(G.fix[0], G.fix[2]));           // (lower, fg]
        }
        stamp(2);
        nodes += max(G.fix[2] - G.fix[0], 0) + (spec2 ? max(G.fix[3] - G.fix[2], 0) : 0);
        const double nl = (r0 >= P.obj) ? P.sg0 : P.fg;
        const double nu = (r0 < P.obj) ? P.sg1 : P.fg;
        double nr;
        if ((split && nl == P.sg0 && nu == P.fg) || (spec2 && nl == P.fg && nu == P.sg1)) {
            nr = n2;
        } else {
            nr = team_sum(range_sum(fixpos(nl), fixpos(nu)));
            nodes += max(fixpos(nu) - fixpos(nl), 0);
        }
        stamp(3);
        bracket(r0, nl, nu, nr);
    }
    // the remaining levels above the tails: one range sum + one workgroup reduction each
    const bool blk = P.exact_walk != 0;                    // block tail usable (after one level)
    constexpr int BCAP = NT * kSortBlk;
    {
        int pmt = h < tsz ? tr[h] : 0;                     // ub(mid) of heap node h, loaded a level ahead
        while (it < P.K && phi - plo > TCAP && !(blk && it >= 1 && phi - plo <= BCAP)) {
            const double mid = (lo + hi) / 2;
            if (tid == 0) sn[it] = mid;
            if (nt < 0 && !(hi - lo > P.tol)) nt = it;
            const bool tab = h < tsz;                      // tabulated; deeper: search (only if ties pile up)
            const int pm = tab ? pmt : sorted_ub(G.vs, plo, phi, mid);
            const bool ctab = 2 * h + 1 < tsz;             // both children tabulated: fetch them now,
            const int pl = ctab ? tr[2 * h] : 0;           // their latency hides behind this level's slab
            const int pr = ctab ? tr[2 * h + 1] : 0;
            const double val = team_sum(ustack ? range_sum(plo, pm) : range_sum(pm, phi));
            nodes += ustack ? pm - plo : phi - pm;
            if (level(mid, val)) { lo = mid; plo = pm; }
            else                 { hi = mid; phi = pm; }
            if (tab) h = 2 * h + (ustack ? 1 : 0);         // children: (lo, mid) = 2h, (mid, hi) = 2h + 1
            pmt = ustack ? pr : pl;
            if (it < 15) stamp(5 + it);
            ++it;
        }
    }

    // ---- block tail: the cell (lo, hi] = v*-sorted positions [plo, phi), TCAP < phi - plo <= BCAP.
    // Thread tid evaluates positions plo + tid * kSortBlk + m in order; a block scan turns the
    // values into F at every node threshold (F = prev + prefix when the last level moved lo, else
    // prev - (cell total - prefix): the reference's adjust_integral chain after its first level).
    // F is non-decreasing in v (node values >= 0; a NaN makes every later F NaN), so every
    // remaining decision "F(mid) < obj" is "mid < v_c", v_c the first tie-group end where
    // !(F < obj), and the zeros of F one interval (zero_interval): dyadic_walk writes them all.
    const bool blk_tail = it < P.K && blk && it >= 1 && phi - plo > TCAP;   // workgroup-uniform
    if (blk_tail) {
        constexpr int KB = kSortBlk;
        const int cnt = phi - plo;
        const int e0 = tid * KB;                           // my first cell entry
        uint32_t wd[KB];
        double vv[KB + 1];                                 // v* of my entries and of the next one
#pragma unroll
        for (int m = 0; m < KB; ++m) wd[m] = e0 + m < cnt ? G.tidx[plo + e0 + m] : 0u;
#pragma unroll
        for (int m = 0; m <= KB; ++m) vv[m] = e0 + m < cnt ? G.tvs[plo + e0 + m] : __builtin_inf();
        double pre[KB];                                    // my inclusive prefix
        double run = 0.0;
        auto eval_cell = [&](auto nodef) {
#pragma unroll
            for (int m = 0; m < KB; ++m) {
                const double v = e0 + m < cnt ? nodef(wd[m]) : 0.0;
                run += v;
                pre[m] = run;
            }
        };
        if (fast) eval_cell(node_fast);
        else eval_cell(node_generic);
        nodes += cnt;
        // block exclusive scan of the thread totals (one barrier); the tail buffer is free here
        double* wt = (double*)tail;                        // [NT / 64] wave totals
        int* ew = (int*)(wt + NT / 64);                    // [NT / 64][4] first crossing / zero / positive
        const double incl = wave_incl_scan_f64(run);
        if (lane == 63) wt[tid >> 6] = incl;
        __syncthreads();
        double base = incl - run, Stot = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) {
            const double x = wt[w];
            base += (w < (tid >> 6)) ? x : 0.0;
            Stot += x;
        }
        const double Flo = ustack ? prev : prev - Stot;   // F just above lo
        int mc = KB, ma = KB, mz = KB;
#pragma unroll
        for (int m = KB - 1; m >= 0; --m) {
            if (!(e0 + m < cnt && vv[m + 1] > vv[m])) continue;   // tie-group ends only (inf past the cell)
            const double pa = base + pre[m];
            const double Fv = ustack ? prev + pa : prev - (Stot - pa);
            if (!(Fv < P.obj)) mc = m;
            if (Fv == 0.0) ma = m;
            if (!(Fv <= 0.0)) mz = m;
        }
        const unsigned long long bc = __ballot(mc < KB), ba = __ballot(ma < KB), bz = __ballot(mz < KB);
        const int lc = bc ? (int)__builtin_ctzll(bc) : 0, la = ba ? (int)__builtin_ctzll(ba) : 0,
                  lz = bz ? (int)__builtin_ctzll(bz) : 0;
        const int mcl = __shfl(mc, lc, 64), mal = __shfl(ma, la, 64), mzl = __shfl(mz, lz, 64);
        if (lane == 0) {
            int* e = ew + 4 * (tid >> 6);
            e[0] = bc ? ((tid >> 6) * 64 + lc) * KB + mcl : kNoPos;
            e[1] = ba ? ((tid >> 6) * 64 + la) * KB + mal : kNoPos;
            e[2] = bz ? ((tid >> 6) * 64 + lz) * KB + mzl : kNoPos;
        }
        __syncthreads();
        stamp(29);
        if (tid < 64) {
            int ec = kNoPos, ea = kNoPos, ez = kNoPos;
#pragma unroll
            for (int w = 0; w < NT / 64; ++w) {                   // waves in position order: first wins
                const int* e = ew + 4 * w;
                if (ec == kNoPos && e[0] != kNoPos) ec = e[0];
                if (ea == kNoPos && e[1] != kNoPos) ea = e[1];
                if (ez == kNoPos && e[2] != kNoPos) ez = e[2];
            }
            const int kc = !(Flo < P.obj) ? 0 : (ec == kNoPos ? 1 : 2);
            const double vcs = kc == 2 ? G.tvs[plo + ec] : 0.0;
            const double inf = __builtin_inf();
            double vza, vzb;
            zero_interval(Flo, (Flo < 0.0 && ea != kNoPos) ? G.tvs[plo + ea] : inf,
                          (!(Flo > 0.0) && ez != kNoPos) ? G.tvs[plo + ez] : inf, vza, vzb);
            dyadic_walk(P, kc, vcs, vza, vzb, lo, hi, it, nt, mask, sn);
        }
    }
    // ---- tail: the bracket's <= TCAP nodes -> LDS, wave 0 finishes the levels
    if (!blk_tail && it < P.K) {
        const int tot = phi - plo;
        // exact walk: the cell's nodes in v* order (same node set: plo, phi are segment boundaries)
        const uint32_t* tix = P.exact_walk ? G.tidx : G.idx;
        const double* tv = P.exact_walk ? G.tvs : G.vs;
        for (int e = tid; e < tot; e += NT) {
            const uint32_t c = tix[plo + e];
            tail[e] = make_double2(tv[plo + e], fast ? node_fast(c) : node_generic(c));
        }
        __syncthreads();
        stamp(29);
        nodes += tot;
        if (tid < 64 && P.exact_walk) {
            // exact dyadic brackets: lane holds the tail's positions lane TPL + m (in order); one level by
            // masked sums if none ran yet (the reference's first level may subtract a slab it never
            // added, Q1), then F at every tie-group end from one prefix scan (F = prev + prefix when the
            // last level moved lo, else prev - (cell total - prefix): adjust_integral's chain), the two
            // crossing thresholds v_c (first end with !(F < obj)) and v_z (first with F != 0), and the
            // remaining levels in closed form (dyadic_walk) -- the COMPACT block tail's scheme
            double tx[TPL], ty[TPL];
#pragma unroll
            for (int m = 0; m < TPL; ++m) {
                const int e = lane * TPL + m;
                const double2 v = e < tot ? tail[e] : make_double2(__builtin_nan(""), 0.0);
                tx[m] = v.x;
                ty[m] = v.y;
            }
            if (it == 0) {
                const double mid = (lo + hi) / 2;
                if (tid == 0) sn[it] = mid;
                if (nt < 0 && !(hi - lo > P.tol)) nt = it;
                const double a0 = ustack ? lo : mid, b0 = ustack ? mid : hi;   // slab (a0, b0]
                double p = 0.0;
#pragma unroll
                for (int m = 0; m < TPL; ++m) p += (tx[m] > a0 && tx[m] <= b0) ? ty[m] : 0.0;
                const double val = wave_sum(p);
                const double slab_lower = ustack ? lo : mid;
                const double Fn = (slab_lower == prevU) ? prev + val : prev - val;
                if (Fn != 0.0) mask |= (1ull << it);
                ustack = Fn < P.obj;
                if (ustack) lo = mid; else hi = mid;
                prev = Fn;
                prevU = mid;
                ++it;
#pragma unroll
                for (int m = 0; m < TPL; ++m)                     // the cell's entries only
                    if (!(tx[m] > lo && tx[m] <= hi)) ty[m] = 0.0;
            }
            if (it < P.K) {
                double run = 0.0;
#pragma unroll
                for (int m = 0; m < TPL; ++m) run += (tx[m] > lo && tx[m] <= hi) ? ty[m] : 0.0;
                const double incl = wave_incl_scan_f64(run);
                const double Stot = readlane_f64(incl, 63);
                const double Flo = ustack ? prev : prev - Stot;   // F just above lo
                const double nx = __shfl(tx[0], (lane + 1) & 63, 64);
                double pa = incl - run;
                const double inf = __builtin_inf();
                double vc = inf, va = inf, vz = inf;        // first crossing / zero / positive-or-NaN end
#pragma unroll
                for (int m = 0; m < TPL; ++m) {
                    const bool in = tx[m] > lo && tx[m] <= hi;
                    pa += in ? ty[m] : 0.0;
                    const double tn = m + 1 < TPL ? tx[m + 1] : nx;
                    const bool gend = in && (lane * TPL + m == tot - 1 || !(tn <= tx[m]));   // last of its v*
                    const double Fv = ustack ? prev + pa : prev - (Stot - pa);
                    if (gend && vc == inf && !(Fv < P.obj)) vc = tx[m];
                    if (gend && va == inf && Fv == 0.0) va = tx[m];
                    if (gend && vz == inf && !(Fv <= 0.0)) vz = tx[m];
                }
                const unsigned long long bc = __ballot(vc != inf), ba = __ballot(va != inf), bz = __ballot(vz != inf);
                const int kc = !(Flo < P.obj) ? 0 : (bc ? 2 : 1);
                const double vcs = __shfl(vc, bc ? (int)__builtin_ctzll(bc) : 0, 64);
                const double vas = ba ? __shfl(va, (int)__builtin_ctzll(ba), 64) : inf;
                const double vzs = bz ? __shfl(vz, (int)__builtin_ctzll(bz), 64) : inf;
                double vza, vzb;
                zero_interval(Flo, vas, vzs, vza, vzb);
                dyadic_walk(P, kc, vcs, vza, vzb, lo, hi, it, nt, mask, sn);
            }
        } else if (tid < 64) {
            double tx[TPL], ty[TPL];
#pragma unroll
            for (int m = 0; m < TPL; ++m) {
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
                for (int m = 0; m < TPL; ++m) p += (tx[m] > a0 && tx[m] <= b0) ? ty[m] : 0.0;
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
    if (stamps && tid == 0) {
        stamps[26] = __builtin_amdgcn_s_memrealtime();
        stamps[28] = (unsigned long long)nodes;
    }
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
