// cvq_plan.hip -- plan lifecycle + C ABI of the quadrature / VaR solve (libcvq.so).
// See include/cvq.h for the contract and the reference interfaces replaced.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "cvq_common.h"
#include "cvq_quad_kernels.h"
#include "cvq_direct_kernels.h"
#include "cvq_compact_kernels.h"
#include "cvq_sorted_kernels.h"
#include "cvq_tppf_tables.h"

namespace cvq {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// Host image of one nu's Student-t data: CF coefficients, cubic guess tables and
// the direct (degree-5) tables, laid out as they are copied to the device.
struct TImage {
    TConst k{};                       // table pointers are offsets into `data` (as doubles)
    std::vector<double> data;
    long long off_tab = -1, off_q = -1;
};

static TImage build_timage(double nu) {
    TImage im;
    TConst& k = im.k;
    k.nu = nu;
    k.a = nu / 2;
    k.ln_nu = std::log(nu);
    k.lbeta = std::lgamma(nu / 2) + std::lgamma(0.5) - std::lgamma(nu / 2 + 0.5);
    k.ln_k = std::lgamma((nu + 1) / 2) - std::lgamma(nu / 2) - 0.5 * std::log(nu * M_PI);
    k.ln_tail = k.ln_k + (nu - 1) / 2 * k.ln_nu;
    k.split = (k.a + 1.0) / (k.a + 2.5);
    k.ln_a = std::log(k.a);
    k.inv_nu = 1.0 / nu;
    k.p_split = 0.05;
    k.cf_terms = kCfTerms;
    std::vector<double> c(2 * kCfTerms);
    ibeta_cf_coeffs(k.a, 0.5, c.data(), kCfTerms);
    ibeta_cf_coeffs(0.5, k.a, c.data() + kCfTerms, kCfTerms);
    TConst hk = k;                                    // host evaluation copy
    hk.cf_dir = c.data();
    hk.cf_cmp = c.data() + kCfTerms;
    std::vector<double> tab, quint;
    bool ok = false, qok = false;
    if (nu <= 1e5)
        for (int nc = 256, nv = 64; nc <= 4096 && !ok; nc *= 2, nv *= 2) ok = build_tppf_tables(hk, nc, nv, tab);
    if (ok)
        for (int nc = 256; nc <= 4096 && !qok; nc *= 2) qok = build_tppf_quintic(hk, nc, nc < 1024 ? 128 : nc / 4, quint);
    im.data = c;
    if (ok) {
        im.off_tab = (long long)im.data.size();
        im.data.insert(im.data.end(), tab.begin(), tab.end());
        k.n_c = hk.n_c;
        k.n_v = hk.n_v;
        k.inv_hc = hk.inv_hc;
        k.inv_hv = hk.inv_hv;
    }
    if (qok) {
        im.off_q = (long long)im.data.size();
        im.data.insert(im.data.end(), quint.begin(), quint.end());
        k.n_qc = hk.n_qc;
        k.n_qv = hk.n_qv;
        k.inv_qc = hk.inv_qc;
        k.inv_qv = hk.inv_qv;
    }
    return im;
}

// Student-t constants for nu with device copies of its tables in *d_cf (owned by
// the caller).  Table construction (~0.1 s for nu = 6) is cached per nu.
int make_tconst(double nu, TConst* tk, double** d_cf) {
    static std::mutex mu;
    static std::map<double, TImage> cache;
    const TImage* im;
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cache.find(nu);
        if (it == cache.end()) it = cache.emplace(nu, build_timage(nu)).first;
        im = &it->second;
    }
    CVQ_HIP_CHECK(hipMalloc((void**)d_cf, im->data.size() * sizeof(double)));
    CVQ_HIP_CHECK(hipMemcpy(*d_cf, im->data.data(), im->data.size() * sizeof(double), hipMemcpyHostToDevice));
    *tk = im->k;
    tk->cf_dir = *d_cf;
    tk->cf_cmp = *d_cf + kCfTerms;
    tk->tab_c = tk->tab_v = nullptr;
    tk->q_c = tk->q_v = nullptr;
    if (im->off_tab >= 0) {
        tk->tab_c = *d_cf + im->off_tab;
        tk->tab_v = tk->tab_c + 2 * (tk->n_c + 1);
    }
    if (im->off_q >= 0) {
        tk->q_c = *d_cf + im->off_q;
        tk->q_v = tk->q_c + 6 * tk->n_qc;
    }
    return CVQ_OK;
}

int compact_tail_cap();                      // cvq_compact.hip: the block tail's node capacity
int compact_nt();                            // cvq_compact.hip: threads per COMPACT workgroup
}  // namespace cvq

using namespace cvq;

struct cvq_plan {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    int strategy = CVQ_STRATEGY_PREFIX;
    double v_cap = 0.0;
    StaticDev S{};
    // static device buffers
    double* d_x = nullptr;
    double* d_F = nullptr;
    double* d_phi = nullptr;
    double* d_uvs = nullptr;
    double* d_cf = nullptr;      // Student-t CF coefficient tables
    int* d_kmax = nullptr;
    long long* d_off = nullptr;
    // per-date state
    long long T = 0, capT = 0;
    double* d_a = nullptr;       // fbs [T][dim][q] or sigma [T][dim]
    double* d_pi = nullptr;      // [T][Q]  (GARCH/UKF: ones)
    const double* in_a = nullptr;   // per-date inputs the kernels read: d_a / d_pi, or the
    const double* in_pi = nullptr;  // caller's device buffers (cvq_set_dates with CVQ_MEM_DEVICE)
    Header* zero_hdr = nullptr;     // header k_tables zeroes on its way (ensure_mass)
    double* d_tA = nullptr;      // [T][dim][n]
    double* d_tB = nullptr;
    double* d_C = nullptr;       // [T][G]
    bool tables_valid = false, mass_valid = false;
    // solve scratch
    long long capSnap = 0;
    double* d_snap = nullptr;
    Header* d_hdr = nullptr;
    int* d_err = nullptr;
    long long capIO = 0;
    double* d_io = nullptr;      // bounds (2T) + out (T) / var (T)
    unsigned long long* d_stamps = nullptr;   // diagnostic phase stamps (CVQ_STAMPS=1)
    bool count_nodes = false;    // cvq_plan_count_nodes: solves record their node counts (stamps)
    bool nodes_valid = false;    // the last solve recorded them
    // COMPACT: host grid copy, v* table, grid lookup buckets, fixed-level cuts for the
    // cached solve arguments
    std::vector<double> hx;
    double* d_vstar = nullptr;   // [n][n]
    int16_t* d_bucket = nullptr; // [nb]
    double bx0 = 0.0, binv = 0.0;
    int nb = 0;
    int16_t* d_cutfix = nullptr; // [n][kCutFixed]
    double cut_key[6] = {0, 0, 0, 0, 0, 0};
    bool cut_valid = false;
    std::vector<double> hvc;     // every v*(r, j >= 1), sorted (the bisection cells' node counts)
    int* d_ccount = nullptr;     // [4][2 << ccount_depth] cell node counts (nullptr: counted on device)
    int ccount_depth = -1;
    uint32_t* d_tlist = nullptr; // [n (n - 1)] nodes (r, j >= 1) in hvc's order: the block tail's list
    double* d_tvs = nullptr;     // [n (n - 1)] = hvc on the device
    int bstart[4] = {0, 0, 0, 0};   // ub(bracket lower) in hvc for the cached solve arguments
    int* d_defer = nullptr;      // [2 + T]: generic-path dates deferred by the fast kernel (count, ticket, list)
    int16_t* d_kcut = nullptr;   // [4][2^ccount_depth][n] per-row cuts of the bisection cells' mids
    int* d_fpair = nullptr;      // [3][NT RPT][2] COMPACT fixed slabs' half-row column ranges per thread slot
    bool kcut_ok = false;
    long long capDefer = 0;
    bool fast_hint = false;      // every date of the batch takes COMPACT's fast path (proven or asserted)
    // SORTED: reachable nodes sorted by v* (device: packed indices + v*; host: v*),
    // ub() of the fixed levels and the bisection trees for the cached solve arguments
    std::vector<double> hvs;
    uint32_t* d_sidx = nullptr;  // [G]
    double* d_svs = nullptr;     // [G]
    int* d_tree = nullptr;       // [4][1 << tree_depth]
    int tree_depth = 0;
    int* d_pass = nullptr;       // SWEEP: both passes' boundary positions, then their child links
    std::vector<uint32_t> hidx;  // SORTED node words (host copy, v*-sorted)
    uint32_t* d_pidx = nullptr;  // solve-order copies of the node words / v* (row-major inside
    double* d_pvs = nullptr;     // each segment between slab ends; ensure_sorted_tree)
    int pass_ma = 0, pass_mb = 0;   // SWEEP: boundaries of pass A / B (0: the SORTED levels instead)
    int pass_fix[kPassFix] = {0, 0, 0, 0, 0};
    int pass_root[4] = {-1, -1, -1, -1};
    int layout = 0;              // SORTED node-word layout (sorted_pack)
    int fixpos[6] = {0, 0, 0, 0, 0, 0};
    std::vector<int> hcuts;      // solve-order segment ends (ensure_sorted_tree; cvq_plan_debug_cuts)
    double tree_key[7] = {0, 0, 0, 0, 0, 0, 0};
    bool tree_valid = false;
    long long capStamps = 0;
    // optional per-kernel timing (HIP events on the plan's stream)
    int timing = 0;              // bitmask of kernel kinds timed with HIP events
    std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> events;
};

namespace {
enum TimedKernel { TK_TABLES = 0, TK_MASS = 1, TK_SOLVE = 2, TK_FINALIZE = 3, TK_SLAB = 4, TK_COUNT = 5 };

struct TimedScope {
    cvq_plan* p;
    int kind;
    hipEvent_t a = nullptr, b = nullptr;
    TimedScope(cvq_plan* p_, int kind_) : p(p_), kind(kind_) {
        if (!((p->timing >> kind) & 1)) return;
        if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) { a = b = nullptr; return; }
        (void)hipEventRecord(a, p->stream);
    }
    ~TimedScope() {
        if (!a) return;
        (void)hipEventRecord(b, p->stream);
        p->events.push_back({kind, {a, b}});
    }
};
}  // namespace

namespace {

template <typename T>
int dev_alloc(T** p, size_t count) {
    if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (count == 0) count = 1;
    CVQ_HIP_CHECK(hipMalloc((void**)p, count * sizeof(T)));
    return CVQ_OK;
}

int ensure_device(int device) {
    int n = 0;
    CVQ_HIP_CHECK(hipGetDeviceCount(&n));
    CVQ_REQUIRE(device >= 0 && device < n, CVQ_ERR_INVALID, "device index out of range");
    CVQ_HIP_CHECK(hipSetDevice(device));
    return CVQ_OK;
}

// --- bisection budget (calc_var_class.py:278: while any(upper - lower > tol))
int halvings(double w, double tol) {
    int k = 0;
    while (w > tol && k < 1000) { w = w / 2; ++k; }
    return k;
}

bool dyadic(double v, int* e) {
    for (int k = 0; k <= 40; ++k) {
        const double s = std::ldexp(v, k);
        if (s == std::floor(s) && std::fabs(s) < 9.0e15) { *e = k; return true; }
    }
    return false;
}

// K = iterations the reference needs for the widest bracket class; exact when
// every bisection point is exactly representable, else a margin is added and
// the device verifies convergence (header.error).
int bisect_budget(const cvq_solve_args& a, bool* exact) {
    const double br[4][2] = {{a.min_var, a.second_guess_lo}, {a.second_guess_lo, a.first_guess},
                             {a.second_guess_hi, a.max_var}, {a.first_guess, a.second_guess_hi}};
    int K = 0;
    bool ex = true;
    for (auto& b : br) {
        const int k = halvings(b[1] - b[0], a.tolerance);
        K = std::max(K, k);
        int e0, e1;
        if (!dyadic(b[0], &e0) || !dyadic(b[1], &e1)) { ex = false; continue; }
        const double mag = std::max(std::fabs(b[0]), std::fabs(b[1]));
        const int bits = std::max(e0, e1) + k + (int)std::ceil(std::log2(mag + 1.0)) + 1;
        if (bits > 52) ex = false;
    }
    *exact = ex;
    return K;
}

int pick_solve_shape(int nrows, int* tpd, int* rpt) {
    if (nrows <= 64) { *tpd = 64; *rpt = 1; }
    else if (nrows <= 128) { *tpd = 64; *rpt = 2; }
    else if (nrows <= 256) { *tpd = 64; *rpt = 4; }
    else if (nrows <= 512) { *tpd = 64; *rpt = 8; }
    else if (nrows <= 1024) { *tpd = 256; *rpt = 4; }
    else if (nrows <= 4096) { *tpd = 256; *rpt = 16; }
    else return CVQ_ERR_UNSUPPORTED;
    return CVQ_OK;
}

template <int TPD, int RPT>
void launch_solve_t(cvq_plan* p, const SolveConst& P, double* snaps, Header* hdr) {
    hipLaunchKernelGGL((k_solve_prefix<TPD, RPT>), dim3((unsigned)p->T), dim3(TPD), 0, p->stream, p->S, P, p->d_C,
                       snaps, hdr);
}
template <int TPD, int RPT>
void launch_slab_t(cvq_plan* p, const double* bounds, double* out) {
    hipLaunchKernelGGL((k_slab_prefix<TPD, RPT>), dim3((unsigned)p->T), dim3(TPD), 0, p->stream, p->S, p->d_C,
                       bounds, out);
}

// ---------------------------------------------------------------- DIRECT
// k_direct computes its own tables unless the plan is Student without direct
// t.ppf tables (then k_tables runs first and k_direct reads tA / tB).
bool direct_fused(const cvq_plan* p) { return p->S.copula != CVQ_STUDENT || p->S.tk.q_c != nullptr; }

template <int COP, bool MSM, int QT, int PM>
void launch_direct_qp(cvq_plan* p, const SolveConst& P, int mode, const double* bounds, double* out, double* snaps,
                      Header* hdr) {
    const int rpt = p->S.n <= 256 ? 1 : 2;
    constexpr bool fold = (COP == CVQ_STUDENT) && MSM;
    constexpr int cs = ((1 + QT + (fold ? 0 : 1)) + 1) & ~1;      // k_direct's column record
    const size_t lds = sizeof(double) * ((size_t)(cs + 1) * p->S.n + 8);
#define CVQ_DIRECT_LAUNCH(R, FU)                                                                                   \
    hipLaunchKernelGGL((k_direct<COP, MSM, QT, R, PM, FU>), dim3((unsigned)p->T), dim3(256), lds, p->stream, p->S, P, \
                       p->in_a, p->d_tA, p->d_tB, p->in_pi, mode, bounds, out, snaps, hdr)
    const bool fused = direct_fused(p);
    if (rpt == 1) { if (fused) CVQ_DIRECT_LAUNCH(1, true); else CVQ_DIRECT_LAUNCH(1, false); }
    else { if (fused) CVQ_DIRECT_LAUNCH(2, true); else CVQ_DIRECT_LAUNCH(2, false); }
#undef CVQ_DIRECT_LAUNCH
}

template <int COP, bool MSM, int QT>
void launch_direct_q(cvq_plan* p, const SolveConst& P, int mode, const double* bounds, double* out, double* snaps,
                     Header* hdr) {
    if constexpr (COP == CVQ_STUDENT) {
        if (p->S.node_m == 8) { launch_direct_qp<COP, MSM, QT, 8>(p, P, mode, bounds, out, snaps, hdr); return; }
        if (p->S.node_m == 9) { launch_direct_qp<COP, MSM, QT, 9>(p, P, mode, bounds, out, snaps, hdr); return; }
    }
    launch_direct_qp<COP, MSM, QT, 0>(p, P, mode, bounds, out, snaps, hdr);
}

template <int COP>
void launch_direct_c(cvq_plan* p, const SolveConst& P, int mode, const double* bounds, double* out, double* snaps,
                     Header* hdr) {
    if (p->S.model != CVQ_MSM) { launch_direct_q<COP, false, 1>(p, P, mode, bounds, out, snaps, hdr); return; }
    switch (p->S.q) {
        case 1: launch_direct_q<COP, true, 1>(p, P, mode, bounds, out, snaps, hdr); break;
        case 2: launch_direct_q<COP, true, 2>(p, P, mode, bounds, out, snaps, hdr); break;
        case 3: launch_direct_q<COP, true, 3>(p, P, mode, bounds, out, snaps, hdr); break;
        case 4: launch_direct_q<COP, true, 4>(p, P, mode, bounds, out, snaps, hdr); break;
        case 5: launch_direct_q<COP, true, 5>(p, P, mode, bounds, out, snaps, hdr); break;
        case 6: launch_direct_q<COP, true, 6>(p, P, mode, bounds, out, snaps, hdr); break;
        case 7: launch_direct_q<COP, true, 7>(p, P, mode, bounds, out, snaps, hdr); break;
        default: launch_direct_q<COP, true, 8>(p, P, mode, bounds, out, snaps, hdr); break;
    }
}

int launch_direct(cvq_plan* p, const SolveConst& P, int mode, const double* bounds, double* out, double* snaps,
                  Header* hdr) {
    switch (p->S.copula) {
        case CVQ_GAUSSIAN: launch_direct_c<CVQ_GAUSSIAN>(p, P, mode, bounds, out, snaps, hdr); break;
        case CVQ_STUDENT: launch_direct_c<CVQ_STUDENT>(p, P, mode, bounds, out, snaps, hdr); break;
        default: launch_direct_c<CVQ_PLACKETT>(p, P, mode, bounds, out, snaps, hdr); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int ensure_stamps(cvq_plan* p) {
    if (p->T > p->capStamps) {
        if (p->d_stamps) (void)hipFree(p->d_stamps);
        p->d_stamps = nullptr;
        p->capStamps = 0;
        CVQ_HIP_CHECK(hipMalloc((void**)&p->d_stamps, (size_t)p->T * 32 * 8));
        p->capStamps = p->T;
    }
    // slot 28 of each date accumulates its node count (COMPACT adds per wave)
    CVQ_HIP_CHECK(hipMemsetAsync(p->d_stamps, 0, (size_t)p->T * 32 * 8, p->stream));
    return CVQ_OK;
}

// ---------------------------------------------------------------- COMPACT
// Cut columns cnt_r(v) = largest j with x_j <= (v - x_r w1) / w0 (else 0), exactly
// as the device's count_le over [0, n-1] (create_grids.py:104-108, Q9/Q10).
int host_cnt(const std::vector<double>& x, double lev, double w0, double v) {
    if (!(v == v)) return 0;                                   // NaN level: count_le keeps klo
    const double g = (v - lev) / w0;
    int lo = 0, hi = (int)x.size() - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (x[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Ordered-integer view of doubles (monotone for all non-NaN values).
inline int64_t d2o(double d) {
    int64_t b;
    std::memcpy(&b, &d, 8);
    return b >= 0 ? b : ~(b & INT64_MAX);
}
inline double o2d(int64_t o) {
    const int64_t b = o >= 0 ? o : (~o) | INT64_MIN;
    double d;
    std::memcpy(&d, &b, 8);
    return d;
}

// v*(r, j): the smallest double v with x_j <= (v - lev_r) / w0, the exact FP64
// membership rule of the nested grid (Q10): node (r, j >= 1) lies in the slab
// (a, b] iff a < v* <= b, because (v - lev) / w0 is non-decreasing in v.
double vstar_exact(double xj, double lev, double w0) {
    auto pred = [&](double v) { return xj <= (v - lev) / w0; };
    double v = xj * w0 + lev;                                  // within a few ulps of v*
    int steps = 0;
    if (pred(v)) {
        for (double d; steps < 64 && pred(d = std::nextafter(v, -HUGE_VAL)); ++steps) v = d;
    } else {
        for (; steps < 64 && !pred(v); ++steps) v = std::nextafter(v, HUGE_VAL);
    }
    if (steps < 64) return v;
    // ordered-integer bisection (cancellation near 0: v* is ~ -ulp(lev) / 2, far below the
    // start's ulp); the span of the ordered range exceeds INT64_MAX, so distances are unsigned
    int64_t lo = d2o(-HUGE_VAL), hi = d2o(HUGE_VAL);           // pred(lo) false, pred(hi) true
    while ((uint64_t)hi - (uint64_t)lo > 1) {
        const int64_t m = (int64_t)((uint64_t)lo + ((uint64_t)hi - (uint64_t)lo) / 2);
        if (pred(o2d(m))) hi = m; else lo = m;
    }
    return o2d(hi);
}

void build_vstar(const std::vector<double>& x, double w0, double w1, std::vector<double>& out) {
    const int n = (int)x.size();
    out.assign((size_t)n * n, 0.0);
    for (int r = 0; r < n; ++r) {
        const double lev = x[r] * w1;                          // integration_algo.py:20 (2-D)
        for (int j = 0; j < n; ++j) out[(size_t)r * n + j] = vstar_exact(x[j], lev, w0);
    }
}

// SORTED: every reachable node (row r, inner j in [1, kmax_r]) with its v*, sorted
// by (v*, packed word); the word holds the LDS offsets of the node's records in the
// kernel's layout for (dim, n) (sorted_pack, cvq_sorted_kernels.h).
void build_sorted_nodes(const std::vector<double>& x, const StaticDev& S, const std::vector<int>& kmax, int lay,
                        std::vector<double>& vs, std::vector<uint32_t>& idx) {
    const int n = S.n;
    std::vector<std::pair<double, uint32_t>> nodes;
    nodes.reserve((size_t)S.G);
    for (int r = 0; r < S.nrows; ++r) {
        const int i0 = S.dim == 2 ? r : r / n, i1 = S.dim == 2 ? 0 : r % n;
        const double lev = S.dim == 2 ? x[i0] * S.w1 : x[i0] * S.w1 + x[i1] * S.w2;   // integration_algo.py:20
        for (int j = 1; j <= kmax[r]; ++j)
            nodes.emplace_back(vstar_exact(x[j], lev, S.w0), sorted_pack(lay, n, i0, i1, j));
    }
    std::sort(nodes.begin(), nodes.end());
    vs.resize(nodes.size());
    idx.resize(nodes.size());
    for (size_t k = 0; k < nodes.size(); ++k) {
        vs[k] = nodes[k].first;
        idx[k] = nodes[k].second;
    }
}

int host_ub(const std::vector<double>& vs, double v) {        // #{v* <= v}; NaN -> 0
    if (!(v == v)) return 0;
    return (int)(std::upper_bound(vs.begin(), vs.end(), v) - vs.begin());
}

// SWEEP's pass tables (k_sorted<SWEEP>): pass A over (lower, sg1] = positions [fix0, fix3), pass B
// over bracket 2's (sg1, vmax] = [fix3, fix5).  A pass's boundaries are its range ends, the fixed
// levels inside it and the mids of its brackets' trees pruned to the cells holding more than
// kPassCell nodes (a child is kept only under a kept parent, so a date's walk is a root path);
// per boundary the boundary indices of its two children's mids.  Needs lower <= vmin <= sg0 <= fg
// <= sg1 <= vmax (the solve's default levels); otherwise pass_ma = 0 and the solve runs SORTED's
// levels.  Pruning is coarsened until both lists fit kPassMax.
int build_pass_tables(cvq_plan* p, const SolveConst& P, const std::vector<int>& tree, int depth) {
    p->pass_ma = p->pass_mb = 0;
    for (int b = 0; b < 4; ++b) p->pass_root[b] = -1;
    const bool ordered = P.lower <= P.vmin && P.vmin <= P.sg0 && P.sg0 <= P.fg && P.fg <= P.sg1 && P.sg1 <= P.vmax;
    if (!ordered || p->S.dim != 2) return CVQ_OK;
    const int* fp = p->fixpos;                            // lower, sg0, fg, sg1, vmin, vmax
    const int bend[4][2] = {{fp[4], fp[1]}, {fp[1], fp[2]}, {fp[3], fp[5]}, {fp[2], fp[3]}};   // k_sorted's br
    for (int cell = kPassCell; cell < (1 << 30); cell *= 2) {
        // kept tree nodes per bracket: (heap node, position), pre-order
        std::vector<std::pair<int, int>> kept[4];
        for (int b = 0; b < 4; ++b) {
            std::vector<int> stack{1};
            std::vector<std::pair<int, int>> ends{{bend[b][0], std::max(bend[b][1], bend[b][0])}};
            while (!stack.empty()) {
                const int h = stack.back();
                const std::pair<int, int> e = ends.back();
                stack.pop_back();
                ends.pop_back();
                if (depth == 0 || h >= (1 << depth) || e.second - e.first <= cell) continue;
                const int pm = std::min(std::max(tree[((size_t)b << depth) + h], e.first), e.second);
                kept[b].emplace_back(h, pm);
                stack.push_back(2 * h + 1);
                ends.emplace_back(pm, e.second);
                stack.push_back(2 * h);
                ends.emplace_back(e.first, pm);
            }
        }
        // entries (position, tag): tag -1 - e = fixed level e, else (b << 24) | heap node; positions may
        // repeat (an empty slab), so every entry keeps its own index
        std::vector<std::pair<int, int>> ea, eb;
        const int fixv[kPassFix] = {fp[0], fp[4], fp[1], fp[2], fp[3]};
        for (int e = 0; e < kPassFix; ++e) ea.emplace_back(fixv[e], -1 - e);
        eb.emplace_back(fp[3], -1);
        eb.emplace_back(std::max(fp[5], fp[3]), -2);
        for (int b = 0; b < 4; ++b)
            for (auto& k : kept[b]) (b == 2 ? eb : ea).emplace_back(k.second, (b << 24) | k.first);
        if (ea.size() + eb.size() > (size_t)kPassMax) continue;
        std::stable_sort(ea.begin(), ea.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
            return x.first < y.first;
        });
        std::stable_sort(eb.begin(), eb.end(), [](const std::pair<int, int>& x, const std::pair<int, int>& y) {
            return x.first < y.first;
        });
        std::vector<int> la, lb, ca(ea.size(), 0), cb(eb.size(), 0);
        std::vector<std::vector<int>> where(4, std::vector<int>((size_t)1 << std::max(depth, 0), -1));
        for (size_t k = 0; k < ea.size(); ++k) {
            la.push_back(ea[k].first);
            if (ea[k].second < 0) p->pass_fix[-1 - ea[k].second] = (int)k;
            else where[(size_t)(ea[k].second >> 24)][(size_t)(ea[k].second & 0xFFFFFF)] = (int)k;
        }
        for (size_t k = 0; k < eb.size(); ++k) {
            lb.push_back(eb[k].first);
            if (eb[k].second >= 0) where[2][(size_t)(eb[k].second & 0xFFFFFF)] = (int)k;
        }
        const int hn = depth > 0 ? (1 << depth) : 0;
        for (int b = 0; b < 4; ++b) {
            std::vector<int>& ch = b == 2 ? cb : ca;
            const std::vector<int>& wb = where[(size_t)b];
            p->pass_root[b] = kept[b].empty() ? -1 : wb[1];
            for (auto& k : kept[b]) {
                const int hh = k.first;
                const int lft = 2 * hh < hn ? wb[(size_t)2 * hh] : -1;
                const int rgt = 2 * hh + 1 < hn ? wb[(size_t)2 * hh + 1] : -1;
                ch[(size_t)wb[(size_t)hh]] = (lft + 1) | ((rgt + 1) << 16);
            }
        }
        std::vector<int> h;
        h.insert(h.end(), la.begin(), la.end());
        h.insert(h.end(), lb.begin(), lb.end());
        h.insert(h.end(), ca.begin(), ca.end());
        h.insert(h.end(), cb.begin(), cb.end());
        if (int rc = dev_alloc(&p->d_pass, h.size())) return rc;
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_pass, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice, p->stream));
        CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));    // h is a local
        p->pass_ma = (int)la.size();
        p->pass_mb = (int)lb.size();
        return CVQ_OK;
    }
    return CVQ_OK;
}

// ub() of the fixed levels and, per bracket, of the bisection mids down to the depth
// where every cell holds <= sorted_tail_cap(dim) nodes (the device searches deeper levels).
int ensure_sorted_tree(cvq_plan* p, const SolveConst& P) {
    const double key[7] = {P.lower, P.sg0, P.fg, P.sg1, P.vmin, P.vmax, (double)P.K};
    if (p->tree_valid && std::memcmp(key, p->tree_key, sizeof key) == 0) return CVQ_OK;
    const std::vector<double>& vs = p->hvs;
    for (int e = 0; e < 6; ++e) p->fixpos[e] = host_ub(vs, key[e]);
    const double br[4][2] = {{P.vmin, P.sg0}, {P.sg0, P.fg}, {P.sg1, P.vmax}, {P.fg, P.sg1}};   // k_sorted's br
    const int dmax = std::max(0, std::min(kSortMaxDepth, P.K));
    std::vector<double> lo, hi;
    std::vector<int> tree;
    int depth = dmax;
    for (int d = 0; d <= dmax; ++d) {                          // cells of depth d: heap nodes [2^d, 2^(d+1))
        bool small = true;
        for (int b = 0; b < 4 && small; ++b) {
            double l = br[b][0], h = br[b][1];
            for (int h0 = 1 << d, k = 0; k < (1 << d) && small; ++k) {
                // walk from the root along the path bits of heap node h0 + k
                const int node = h0 + k;
                l = br[b][0];
                h = br[b][1];
                for (int bit = d - 1; bit >= 0; --bit) {
                    const double mid = (l + h) / 2;
                    if ((node >> bit) & 1) l = mid; else h = mid;
                }
                if (host_ub(vs, h) - host_ub(vs, l) > sorted_tail_cap(p->S.dim)) small = false;
            }
        }
        if (small) { depth = d; break; }
    }
    tree.assign((size_t)4 << depth, 0);
    for (int b = 0; b < 4; ++b) {
        lo.assign((size_t)1 << depth, 0.0);
        hi.assign((size_t)1 << depth, 0.0);
        if (depth > 0) { lo[1] = br[b][0]; hi[1] = br[b][1]; }
        for (int h = 1; h < (1 << depth); ++h) {
            const double mid = (lo[h] + hi[h]) / 2;            // the device's (lo + hi) / 2
            tree[((size_t)b << depth) + h] = host_ub(vs, mid);
            if (2 * h + 1 < (1 << depth)) {
                lo[2 * h] = lo[h]; hi[2 * h] = mid;
                lo[2 * h + 1] = mid; hi[2 * h + 1] = hi[h];
            }
        }
    }
    p->tree_valid = false;
    if (int rc = dev_alloc(&p->d_tree, tree.size())) return rc;
    CVQ_HIP_CHECK(hipMemcpyAsync(p->d_tree, tree.data(), tree.size() * sizeof(int), hipMemcpyHostToDevice, p->stream));
    // Solve order.  A solve only ever sums whole segments between consecutive slab ends (the
    // fixed levels and the tabulated mids) and its tail compares v*, so inside a segment the
    // node order is free: lay nodes out row-major there, so the lanes that read consecutive
    // positions read consecutive rows / columns -- distinct LDS bank slots -- instead of the
    // scattered records of the v* order.  A segment the device may search (it lies in a
    // bracket and is larger than the tail cap: the tree hit kSortMaxDepth) stays v*-sorted.
    const int G = (int)vs.size(), tcap = sorted_tail_cap(p->S.dim);
    std::vector<int> cuts(tree.begin(), tree.end());
    cuts.insert(cuts.end(), p->fixpos, p->fixpos + 6);
    cuts.push_back(0);
    cuts.push_back(G);
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    p->hcuts = cuts;
    const int bpos[4][2] = {{p->fixpos[4], p->fixpos[1]}, {p->fixpos[1], p->fixpos[2]},
                            {p->fixpos[3], p->fixpos[5]}, {p->fixpos[2], p->fixpos[3]}};
    std::vector<uint32_t> pidx(p->hidx);
    std::vector<double> pvs(vs);
    const int lay = p->layout, n = p->S.n, ns = (n + 1) & ~1;
    auto row_key = [&](uint32_t c) {                           // (i1, a0, j): rows of the inner axis
        int a0, i1, j;
        if (lay == kLay2) { a0 = (int)(c & 0xFFFFu) >> 4; i1 = 0; j = ((int)(c >> 16) >> 4) - ns; }
        else if (lay == kLay3F) { a0 = (int)((c >> 4) & 0xFFu); i1 = (int)((c >> 12) & 0x7Fu); j = (int)(c >> 25); }
        else { a0 = (int)(c & 0x1FFu); i1 = (int)((c >> 9) & 0xFFu); j = (int)(c >> 17); }
        return ((long long)i1 << 40) | ((long long)a0 << 20) | (long long)j;
    };
    for (size_t k = 0; k + 1 < cuts.size(); ++k) {
        const int c0 = cuts[k], c1 = std::min(cuts[k + 1], G);
        if (c1 - c0 < 2) continue;
        bool searchable = false;
        for (int b = 0; b < 4; ++b) searchable |= c1 - c0 > tcap && c0 >= bpos[b][0] && c1 <= bpos[b][1];
        if (searchable) continue;
        std::vector<std::pair<long long, int>> ord;
        ord.reserve((size_t)(c1 - c0));
        for (int q = c0; q < c1; ++q) ord.emplace_back(row_key(p->hidx[q]), q);
        std::sort(ord.begin(), ord.end());
        for (int q = c0; q < c1; ++q) {
            pidx[q] = p->hidx[ord[q - c0].second];
            pvs[q] = vs[ord[q - c0].second];
        }
    }
    pidx.resize(((pidx.size() + 3) & ~(size_t)3) + kSortIdxPad, 0u);
    if (int rc = dev_alloc(&p->d_pidx, pidx.size())) return rc;
    if (int rc = dev_alloc(&p->d_pvs, std::max<size_t>(pvs.size(), 1))) return rc;
    CVQ_HIP_CHECK(hipMemcpyAsync(p->d_pidx, pidx.data(), pidx.size() * sizeof(uint32_t), hipMemcpyHostToDevice,
                                 p->stream));
    CVQ_HIP_CHECK(hipMemcpyAsync(p->d_pvs, pvs.data(), pvs.size() * sizeof(double), hipMemcpyHostToDevice,
                                 p->stream));
    if (p->strategy == CVQ_STRATEGY_SWEEP) {
        int rc = build_pass_tables(p, P, tree, depth);
        if (rc) return rc;
    }
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    p->tree_depth = depth;
    std::memcpy(p->tree_key, key, sizeof key);
    p->tree_valid = true;
    return CVQ_OK;
}

// Grid lookup buckets: bucket b covers [x_0 + b h, x_0 + (b + 1) h); its entry is
// the largest j with x_j <= x_0 + b h (0 if none), a start for grid_count's probe.
void build_buckets(const std::vector<double>& x, std::vector<int16_t>& bk, double* bx0, double* binv) {
    const int n = (int)x.size(), nb = kBucketsPerPoint * n;
    const double h = (x[n - 1] - x[0]) / nb;
    *bx0 = x[0];
    *binv = h > 0.0 ? 1.0 / h : 0.0;
    bk.assign(nb, 0);
    int j = 0;
    for (int b = 0; b < nb; ++b) {
        const double edge = x[0] + b * h;
        while (j + 1 < n && x[j + 1] <= edge) ++j;
        bk[b] = (int16_t)j;
    }
}

// COMPACT: node counts of the bisection cells -- heap node h of bracket b's tree holds
// #{(r, j >= 1): lo_h < v*(r, j) <= hi_h}, with the device's mids (lo + hi) / 2 -- for
// every depth down to D, the first depth >= 1 whose cells all hold <= cap nodes (table
// [4][2 << D], heap nodes 1 .. 2^(D+1) - 1).  The kernel leaves its workgroup levels for
// the block tail from this table (a cell's sorted positions follow from the counts)
// instead of reducing bracket node counts at every level.  depth = -1: no such depth
// <= kCompactMaxDepth (the kernel counts and runs its one-wave tail).
constexpr int kCompactMaxDepth = 16;
void build_cell_counts(const std::vector<double>& vs, const SolveConst& P, int cap, std::vector<int>& cc,
                       int* depth) {
    const double br[4][2] = {{P.vmin, P.sg0}, {P.sg0, P.fg}, {P.sg1, P.vmax}, {P.fg, P.sg1}};   // k_compact's brackets
    std::vector<std::vector<int>> cnt;                      // cnt[d][(b << d) + k]: depth-d cell k of bracket b
    std::vector<double> lo(4), hi(4);
    for (int b = 0; b < 4; ++b) { lo[b] = br[b][0]; hi[b] = br[b][1]; }
    *depth = -1;
    for (int d = 0; d <= std::min(kCompactMaxDepth, std::max(P.K, 0)); ++d) {
        std::vector<int> c(lo.size());
        bool small = true;
        for (size_t e = 0; e < lo.size(); ++e) {
            c[e] = std::max(host_ub(vs, hi[e]) - host_ub(vs, lo[e]), 0);
            small = small && c[e] <= cap;
        }
        cnt.push_back(c);
        if (small && d >= 1) { *depth = d; break; }
        std::vector<double> l2(2 * lo.size()), h2(2 * lo.size());
        for (size_t e = 0; e < lo.size(); ++e) {            // children 2k (lower half), 2k + 1 (upper half)
            const double mid = (lo[e] + hi[e]) / 2;
            l2[2 * e] = lo[e]; h2[2 * e] = mid;
            l2[2 * e + 1] = mid; h2[2 * e + 1] = hi[e];
        }
        lo.swap(l2);
        hi.swap(h2);
    }
    cc.clear();
    if (*depth < 0) return;
    const int D = *depth;
    cc.assign((size_t)4 << (D + 1), 0);
    for (int d = 0; d <= D; ++d)
        for (int b = 0; b < 4; ++b)
            for (int k = 0; k < (1 << d); ++k)
                cc[((size_t)b << (D + 1)) + (1 << d) + k] = cnt[d][((size_t)b << d) + k];
}

// Fixed-level cut table (and the bisection cells' node counts) for the cached solve arguments.
int ensure_cutfix(cvq_plan* p, const SolveConst& P) {
    const double key[6] = {P.lower, P.sg0, P.fg, P.sg1, P.vmin, P.vmax};
    if (p->cut_valid && std::memcmp(key, p->cut_key, sizeof key) == 0) return CVQ_OK;
    const int n = p->S.n;
    int rc0 = CVQ_OK;
    std::vector<int16_t> h((size_t)n * kCutFixed, 0);
    for (int r = 0; r < n; ++r) {
        const double lev = p->hx[r] * p->S.w1;
        for (int e = 0; e < 6; ++e) h[(size_t)r * kCutFixed + e] = (int16_t)host_cnt(p->hx, lev, p->S.w0, key[e]);
    }
    p->cut_valid = false;
    if (!p->d_cutfix) CVQ_HIP_CHECK(hipMalloc((void**)&p->d_cutfix, h.size() * sizeof(int16_t)));
    CVQ_HIP_CHECK(hipMemcpyAsync(p->d_cutfix, h.data(), h.size() * sizeof(int16_t), hipMemcpyHostToDevice, p->stream));
    // COMPACT's fixed slabs (lower, fg], (sg0, fg], (fg, sg1]: each thread slot sums two half-rows
    // (the first or second half of a row's column range).  Sorted by length and paired longest with
    // shortest, a wave's lanes carry similar work (the fixed slabs are triangles and corner bands:
    // row lengths run from 0 to ~n, and the loops run to the wave's longest lane); any assignment
    // that takes every half-row once gives the same slab, so this is a schedule, not a semantics.
    // Each half-row goes to the kernel as its column range: row | j0 << 10 | len << 20 (len 0: none).
    {
        const int NT = compact_nt(), M = NT * ((n + NT - 1) / NT);
        std::vector<int> fp((size_t)3 * M * 2);
        const int cols[3][2] = {{kCutLower, kCutFg}, {kCutSg0, kCutFg}, {kCutFg, kCutSg1}};
        struct Half { int len, r, j0; };
        std::vector<Half> hl((size_t)2 * M);
        for (int sl = 0; sl < 3; ++sl) {
            for (int r = 0; r < n; ++r) {
                const int a = h[(size_t)r * kCutFixed + cols[sl][0]];
                const int b = std::max<int>(h[(size_t)r * kCutFixed + cols[sl][1]], a);
                const int m = a + (b - a + 1) / 2;
                hl[2 * r] = {m - a, r, a + 1};               // first half: columns (a, m]
                hl[2 * r + 1] = {b - m, r, m + 1};           // second half: (m, b]
            }
            for (int e = 2 * n; e < 2 * M; ++e) hl[e] = {0, 0, 0};
            std::stable_sort(hl.begin(), hl.end(), [](const Half& x, const Half& y) { return x.len > y.len; });
            auto word = [](const Half& x) {
                return x.len > 0 ? (int)((uint32_t)x.r | ((uint32_t)x.j0 << 10) | ((uint32_t)x.len << 20)) : 0;
            };
            for (int e = 0; e < M; ++e) {
                fp[((size_t)sl * M + e) * 2] = word(hl[e]);
                fp[((size_t)sl * M + e) * 2 + 1] = word(hl[2 * M - 1 - e]);
            }
        }
        if (!p->d_fpair && (rc0 = dev_alloc(&p->d_fpair, fp.size()))) return rc0;
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_fpair, fp.data(), fp.size() * sizeof(int), hipMemcpyHostToDevice, p->stream));
    }
    std::vector<int> cc;
    build_cell_counts(p->hvc, P, compact_tail_cap(), cc, &p->ccount_depth);
    const double blo[4] = {P.vmin, P.sg0, P.sg1, P.fg};      // k_compact's brackets' lower levels
    for (int b = 0; b < 4; ++b) p->bstart[b] = host_ub(p->hvc, blo[b]);
    if (p->ccount_depth >= 0) {
        CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));   // the previous table may still be read
        if (int rc = dev_alloc(&p->d_ccount, cc.size())) return rc;
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_ccount, cc.data(), cc.size() * sizeof(int), hipMemcpyHostToDevice, p->stream));
    }
    // per-row cuts of every tabulated bisection cell's mid (the levels' cnt_r(mid) without a grid
    // search): [4][2^D][n] int16, heap node h of bracket b at (b << D) + h; bounded to 4 MB
    const int D = p->ccount_depth;
    p->kcut_ok = D >= 1 && ((size_t)4 << D) * n * sizeof(int16_t) <= ((size_t)4 << 20);
    if (p->kcut_ok) {
        std::vector<int16_t> kc(((size_t)4 << D) * n, 0);
        const double br[4][2] = {{P.vmin, P.sg0}, {P.sg0, P.fg}, {P.sg1, P.vmax}, {P.fg, P.sg1}};
        for (int b = 0; b < 4; ++b) {
            std::vector<double> clo(1 << D), chi(1 << D);       // heap cell bounds, as the kernel halves them
            clo[1] = br[b][0];
            chi[1] = br[b][1];
            for (int h = 1; h < (1 << D); ++h) {
                const double mid = (clo[h] + chi[h]) / 2;
                if (2 * h + 1 < (1 << D)) {
                    clo[2 * h] = clo[h]; chi[2 * h] = mid;
                    clo[2 * h + 1] = mid; chi[2 * h + 1] = chi[h];
                }
                int16_t* dst = kc.data() + (((size_t)b << D) + h) * n;
                for (int r = 0; r < n; ++r) dst[r] = (int16_t)host_cnt(p->hx, p->hx[r] * p->S.w1, p->S.w0, mid);
            }
        }
        CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
        if (int rc = dev_alloc(&p->d_kcut, kc.size())) return rc;
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_kcut, kc.data(), kc.size() * sizeof(int16_t), hipMemcpyHostToDevice, p->stream));
    }
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    std::memcpy(p->cut_key, key, sizeof key);
    p->cut_valid = true;
    return CVQ_OK;
}

// COMPACT's fast node path needs, per date: MSM, pi_t = f0 (x) f1 bit for bit (the
// kernel's own test; compute_forecast_combinations builds it so); GARCH / UKF, finite
// marginal tables -- proven here when every sigma is finite and |x| / sigma <= 6: then
// u = Phi(x / sigma) lies in [Phi(-6), 1 - Phi(-6)] with Phi(-6) ~ 9.87e-10, i.e. strictly
// inside (0, 1), so t.ppf / norm.ppf and the densities are finite (Student: nu >= 1, the
// heaviest tail whose quantile at 9.87e-10 is still ~ -3.2e8; tests/test_fullsize_oracle_gpu.py
// runs sigma = xmax / 6 exactly at nu = 1).  Host inputs only.
bool fast_path_proven(const StaticDev& S, const std::vector<double>& hx, long long T, const double* a,
                      const double* b) {
    if (S.dim != 2 || hx.empty()) return false;
    if (S.model == CVQ_MSM) {
        const int q = S.q;
        for (long long t = 0; t < T; ++t) {
            const double* f = a + t * 2 * q;
            const double* pit = b + t * S.Q;
            for (int l = 0; l < S.Q; ++l)
                if (!(pit[l] == f[l / q] * f[q + l % q])) return false;
        }
        return true;
    }
    if (S.copula == CVQ_STUDENT && !(S.nu >= 1.0)) return false;
    if (S.copula == CVQ_STUDENT) {
        // Student (r05): an entry with u in {0, 1} is a dead record on the fast path (its nodes
        // are 0 in the reference, cvq_compact_kernels.h table phase), and a u strictly inside
        // is >= 2^-54 (1 + erf rounds to 0 or >= 2^-53), whose quantile at nu >= 1 is finite
        // (|z| <= ~6e15) with a finite density ratio: any finite sigma > 0 takes the fast path
        for (long long e = 0; e < 2 * T; ++e)
            if (!(std::isfinite(a[e]) && a[e] > 0.0)) return false;
        return true;
    }
    double xmax = 0.0;
    for (double x : hx) xmax = std::max(xmax, std::fabs(x));
    for (long long e = 0; e < 2 * T; ++e)
        if (!(std::isfinite(a[e]) && a[e] > 0.0 && xmax <= 6.0 * a[e])) return false;
    return true;
}

const char* solve_error_text(int err) {
    return (err & 4) ? "a date needs the generic node path (pi not rank 1 or a non-finite marginal table entry) "
                       "but the plan's fast-path hint said none would (cvq_set_fast_hint)"
         : (err & 2) ? "bisection needs more iterations than the snapshot budget (K)"
                     : "a date did not converge within the bisection budget (K)";
}

}  // namespace
namespace cvq {
int compact_max_n();                                                                  // cvq_compact.hip
int launch_compact(const StaticDev& S, const SolveConst& P, const CompactGeom& G, long long T, hipStream_t stream,
                   const double* a, const double* tA, const double* tB, const double* pi, bool fused, double* st,
                   double* snaps, Header* hdr, int* defer, bool generic, size_t abi);
int launch_sorted(const StaticDev& S, const SolveConst& P, const SortedGeom& G, long long T, hipStream_t stream,
                  const double* a, const double* tA, const double* tB, const double* pi, bool fused, int mode,
                  const double* bounds, double* out, double* snaps, Header* hdr, double* stamps,
                  bool sweep, size_t abi);                                            // cvq_sorted.hip
}
namespace {

bool sorted_family(const cvq_plan* p) {
    return p->strategy == CVQ_STRATEGY_SORTED || p->strategy == CVQ_STRATEGY_SWEEP;
}

// solve: the solve-order copies; slab (mode 1, any bounds): the v*-sorted arrays
SortedGeom sorted_geom(const cvq_plan* p, bool solve) {
    SortedGeom G{};
    G.idx = solve ? p->d_pidx : p->d_sidx;
    G.vs = solve ? p->d_pvs : p->d_svs;
    G.tree = p->d_tree;
    G.G = (int)p->S.G;
    G.depth = p->tree_depth;
    for (int e = 0; e < 6; ++e) G.fix[e] = p->fixpos[e];
    G.pass_bl = p->d_pass;
    G.pass_ch = p->d_pass ? p->d_pass + p->pass_ma + p->pass_mb : nullptr;
    G.pass_ma = solve ? p->pass_ma : 0;
    G.pass_mb = p->pass_mb;
    for (int e = 0; e < kPassFix; ++e) G.pass_fix[e] = p->pass_fix[e];
    for (int b = 0; b < 4; ++b) G.pass_root[b] = p->pass_root[b];
    G.layout = p->layout;
    G.tidx = p->d_sidx;
    G.tvs = p->d_svs;
    return G;
}

int launch_solve(cvq_plan* p, const SolveConst& P, double* snaps, Header* hdr) {
    TimedScope ts(p, TK_SOLVE);
    if (sorted_family(p)) {
        int rc = ensure_sorted_tree(p, P);
        if (rc) return rc;
        static const bool env_stamps = getenv("CVQ_STAMPS") != nullptr;   // diagnostic phase stamps
        const bool dbg_stamps = env_stamps || p->count_nodes;
        if (dbg_stamps && (rc = ensure_stamps(p))) return rc;
        p->nodes_valid = p->count_nodes;
        return launch_sorted(p->S, P, sorted_geom(p, true), p->T, p->stream, p->in_a, p->d_tA, p->d_tB, p->in_pi,
                             direct_fused(p), 0, nullptr, nullptr, snaps, hdr,
                             dbg_stamps ? (double*)p->d_stamps : nullptr,
                             p->strategy == CVQ_STRATEGY_SWEEP && p->pass_ma > 0, kernel_abi_key() ^ (sizeof(SortedGeom) << 40));
    }
    if (p->strategy == CVQ_STRATEGY_COMPACT && p->S.n <= compact_max_n()) {
        int rc = ensure_cutfix(p, P);
        if (rc) return rc;
        static const bool env_stamps = getenv("CVQ_STAMPS") != nullptr;
        const bool dbg_stamps = env_stamps || p->count_nodes;
        double* st = nullptr;
        if (dbg_stamps && (rc = ensure_stamps(p))) return rc;
        if (dbg_stamps) st = (double*)p->d_stamps;
        p->nodes_valid = p->count_nodes;
        if (p->capDefer < p->T + 2) {                      // zeroed once; the generic kernel resets it
            if ((rc = dev_alloc(&p->d_defer, (size_t)p->T + 2))) return rc;
            CVQ_HIP_CHECK(hipMemsetAsync(p->d_defer, 0, ((size_t)p->T + 2) * sizeof(int), p->stream));
            p->capDefer = p->T + 2;
        }
        const bool tab = p->ccount_depth >= 0;
        // CVQ_FPAIR=0: the fixed slabs' (r, n - 1 - r) half-row pairing instead of the host schedule (A/B)
        static const bool fpair_sched = !(getenv("CVQ_FPAIR") && atoi(getenv("CVQ_FPAIR")) == 0);
        const CompactGeom G{p->d_cutfix, p->d_vstar, p->d_bucket, p->bx0, p->binv, p->nb,
                            tab ? p->d_ccount : nullptr, p->ccount_depth, p->d_tlist, p->d_tvs,
                            {p->bstart[0], p->bstart[1], p->bstart[2], p->bstart[3]},
                            (tab && p->kcut_ok) ? p->d_kcut : nullptr, fpair_sched ? p->d_fpair : nullptr};
        return launch_compact(p->S, P, G, p->T, p->stream, p->in_a, p->d_tA, p->d_tB, p->in_pi, direct_fused(p), st,
                              snaps, hdr, p->d_defer, !p->fast_hint, kernel_abi_key() ^ (sizeof(CompactGeom) << 40));
    }
    if (p->strategy != CVQ_STRATEGY_PREFIX) {
        // profiling only: CVQ_STAMPS=1 (phase stamps)
        static const bool dbg_stamps = getenv("CVQ_STAMPS") != nullptr;
        double* st = nullptr;
        if (dbg_stamps) {
            if (int rc = ensure_stamps(p)) return rc;
            st = (double*)p->d_stamps;
        }
        return launch_direct(p, P, 0, nullptr, st, snaps, hdr);
    }
    int tpd, rpt;
    CVQ_REQUIRE(pick_solve_shape(p->S.nrows, &tpd, &rpt) == CVQ_OK, CVQ_ERR_UNSUPPORTED,
                "prefix solve supports at most 4096 rows (3-D n <= 64)");
    if (tpd == 64 && rpt == 1) launch_solve_t<64, 1>(p, P, snaps, hdr);
    else if (tpd == 64 && rpt == 2) launch_solve_t<64, 2>(p, P, snaps, hdr);
    else if (tpd == 64 && rpt == 4) launch_solve_t<64, 4>(p, P, snaps, hdr);
    else if (tpd == 64 && rpt == 8) launch_solve_t<64, 8>(p, P, snaps, hdr);
    else if (tpd == 256 && rpt == 4) launch_solve_t<256, 4>(p, P, snaps, hdr);
    else launch_solve_t<256, 16>(p, P, snaps, hdr);
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int launch_slab(cvq_plan* p, const double* bounds, double* out) {
    TimedScope ts(p, TK_SLAB);
    if (sorted_family(p)) {
        SolveConst P{};
        return launch_sorted(p->S, P, sorted_geom(p, false), p->T, p->stream, p->in_a, p->d_tA, p->d_tB, p->in_pi,
                             direct_fused(p), 1, bounds, out, nullptr, nullptr, nullptr, false,
                             kernel_abi_key() ^ (sizeof(SortedGeom) << 40));
    }
    if (p->strategy != CVQ_STRATEGY_PREFIX) {      // COMPACT: slabs of arbitrary bounds run k_direct
        SolveConst P{};
        return launch_direct(p, P, 1, bounds, out, nullptr, nullptr);
    }
    int tpd, rpt;
    CVQ_REQUIRE(pick_solve_shape(p->S.nrows, &tpd, &rpt) == CVQ_OK, CVQ_ERR_UNSUPPORTED,
                "prefix slab supports at most 4096 rows (3-D n <= 64)");
    if (tpd == 64 && rpt == 1) launch_slab_t<64, 1>(p, bounds, out);
    else if (tpd == 64 && rpt == 2) launch_slab_t<64, 2>(p, bounds, out);
    else if (tpd == 64 && rpt == 4) launch_slab_t<64, 4>(p, bounds, out);
    else if (tpd == 64 && rpt == 8) launch_slab_t<64, 8>(p, bounds, out);
    else if (tpd == 256 && rpt == 4) launch_slab_t<256, 4>(p, bounds, out);
    else launch_slab_t<256, 16>(p, bounds, out);
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

template <int COP, bool MSM>
void launch_tables_t(cvq_plan* p) {
    const long long total = p->T * p->S.dim * p->S.n;
    const unsigned blocks = (unsigned)((total + 255) / 256);
    hipLaunchKernelGGL((k_tables<COP, MSM>), dim3(blocks), dim3(256), 0, p->stream, p->S, p->T, p->in_a, p->d_tA,
                       p->d_tB, p->zero_hdr);
}

template <int COP, bool MSM, int DIM, int QT>
void launch_mass_q(cvq_plan* p) {
    const dim3 grid((unsigned)p->T, (unsigned)((p->S.nrows + 63) / 64));
    hipLaunchKernelGGL((k_mass<COP, MSM, DIM, QT>), grid, dim3(64), 0, p->stream, p->S, p->d_tA, p->d_tB, p->in_pi,
                       p->d_C);
}

template <int COP, bool MSM, int DIM>
void launch_mass_t(cvq_plan* p) {
    if constexpr (!MSM) {
        launch_mass_q<COP, false, DIM, 1>(p);
    } else {
        switch (p->S.q) {
            case 1: launch_mass_q<COP, true, DIM, 1>(p); break;
            case 2: launch_mass_q<COP, true, DIM, 2>(p); break;
            case 3: launch_mass_q<COP, true, DIM, 3>(p); break;
            case 4: launch_mass_q<COP, true, DIM, 4>(p); break;
            case 5: launch_mass_q<COP, true, DIM, 5>(p); break;
            case 6: launch_mass_q<COP, true, DIM, 6>(p); break;
            case 7: launch_mass_q<COP, true, DIM, 7>(p); break;
            default: launch_mass_q<COP, true, DIM, 8>(p); break;
        }
    }
}

template <int COP>
void launch_cop(cvq_plan* p, bool tables) {
    const bool msm = p->S.model == CVQ_MSM;
    if (tables) {
        if (msm) launch_tables_t<COP, true>(p); else launch_tables_t<COP, false>(p);
        return;
    }
    if (p->S.dim == 2) {
        if (msm) launch_mass_t<COP, true, 2>(p); else launch_mass_t<COP, false, 2>(p);
    } else if constexpr (COP != CVQ_PLACKETT) {
        if (msm) launch_mass_t<COP, true, 3>(p); else launch_mass_t<COP, false, 3>(p);
    }
}

int dispatch_cop(cvq_plan* p, bool tables) {
    switch (p->S.copula) {
        case CVQ_GAUSSIAN: launch_cop<CVQ_GAUSSIAN>(p, tables); break;
        case CVQ_STUDENT: launch_cop<CVQ_STUDENT>(p, tables); break;
        default: launch_cop<CVQ_PLACKETT>(p, tables); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

// Brings tables (and PREFIX prefixes) up to date.  hdr, if given, is a solve
// header to zero before the solve: folded into k_tables when that runs, else a
// memset.
int ensure_mass(cvq_plan* p, Header* hdr = nullptr) {
    CVQ_REQUIRE(p->T > 0, CVQ_ERR_STATE, "cvq_set_dates must be called first");
    CVQ_HIP_CHECK(hipSetDevice(p->device));
    if (p->strategy != CVQ_STRATEGY_PREFIX && direct_fused(p)) {   // k_direct / k_compact evaluate their tables
        if (hdr) CVQ_HIP_CHECK(hipMemsetAsync(hdr, 0, sizeof(Header), p->stream));
        return CVQ_OK;
    }
    if (!p->tables_valid) {
        TimedScope ts(p, TK_TABLES);
        p->zero_hdr = hdr;
        int rc = dispatch_cop(p, true);
        p->zero_hdr = nullptr;
        if (rc) return rc;
        p->tables_valid = true;
        p->mass_valid = false;
    } else if (hdr) {
        CVQ_HIP_CHECK(hipMemsetAsync(hdr, 0, sizeof(Header), p->stream));
    }
    if (!p->mass_valid && p->strategy == CVQ_STRATEGY_PREFIX) {
        TimedScope ts(p, TK_MASS);
        int rc = dispatch_cop(p, false);
        if (rc) return rc;
        p->mass_valid = true;
    }
    return CVQ_OK;
}

// PREFIX and SORTED hold only the nodes with level <= v_cap
bool materialised(const cvq_plan* p) {
    return p->strategy == CVQ_STRATEGY_PREFIX || sorted_family(p);
}

// The bisection of bracket (lo, hi] over K levels visits only exact dyadic points when the width
// W = hi - lo is a power of two and lo is an integer multiple N of q = W 2^-K with |N| + 2^K < 2^53:
// every cell end lo + k q (0 <= k <= 2^K) is then N' q with |N'| < 2^53, so (lo + hi) / 2 of the
// reference (calc_var_class.py:281) is exact at every level and the level-l bracket of a date is
// lo + c 2^(K-l) q with c read off the final cell (COMPACT's closed-form tail walk).
bool dyadic_bracket_ok(double lo, double hi, int K) {
    if (!(std::isfinite(lo) && std::isfinite(hi) && hi > lo) || K < 1 || K > 52) return false;
    const double W = hi - lo;
    if (W + lo != hi || hi - W != lo) return false;                // the width itself exact
    int e;
    if (std::frexp(W, &e) != 0.5) return false;                    // W = 2^(e-1)
    const double q = std::ldexp(W, -K);
    if (!(q > 0.0) || !std::isnormal(q)) return false;
    const double N = lo / q;                                       // exact: q is a power of two
    return N == std::floor(N) && std::fabs(N) + std::ldexp(1.0, K) < std::ldexp(1.0, 53);
}

bool dyadic_walk_ok(const cvq_solve_args& a, int K) {
    // k_compact's brackets (calc_var_class.py:137-149): (vmin, sg0], (sg0, fg], (sg1, vmax], (fg, sg1]
    return dyadic_bracket_ok(a.min_var, a.second_guess_lo, K) && dyadic_bracket_ok(a.second_guess_lo, a.first_guess, K) &&
           dyadic_bracket_ok(a.second_guess_hi, a.max_var, K) && dyadic_bracket_ok(a.first_guess, a.second_guess_hi, K);
}

SolveConst solve_const(const cvq_solve_args& a, int K) {
    SolveConst P;
    P.obj = a.obj_var;
    P.fg = a.first_guess;
    P.sg0 = a.second_guess_lo;
    P.sg1 = a.second_guess_hi;
    P.vmin = a.min_var;
    P.vmax = a.max_var;
    P.lower = a.lower;
    P.tol = a.tolerance;
    P.K = K;
    P.stride = K + 1;
    P.ptf_mean = a.ptf_mean;
    P.fin_var = nullptr;
    P.fin_err = nullptr;
    P.exact_walk = dyadic_walk_ok(a, K) ? 1 : 0;
    return P;
}

int check_args(const cvq_plan* p, const cvq_solve_args* a) {
    CVQ_REQUIRE(a != nullptr, CVQ_ERR_INVALID, "solve args is NULL");
    const double top = std::max({a->first_guess, a->second_guess_lo, a->second_guess_hi, a->max_var, a->min_var,
                                 a->lower});
    CVQ_REQUIRE(!materialised(p) || !(top > p->v_cap), CVQ_ERR_RANGE,
                "a VaR level in the solve arguments exceeds the plan's v_cap");
    CVQ_REQUIRE(a->tolerance > 0.0, CVQ_ERR_INVALID, "tolerance must be > 0");
    return CVQ_OK;
}

int ensure_snap(cvq_plan* p, long long need) {
    if (need > p->capSnap) {
        int rc = dev_alloc(&p->d_snap, (size_t)need);
        if (rc) return rc;
        p->capSnap = need;
    }
    return CVQ_OK;
}

int ensure_io(cvq_plan* p, long long need) {
    if (need > p->capIO) {
        int rc = dev_alloc(&p->d_io, (size_t)need);
        if (rc) return rc;
        p->capIO = need;
    }
    return CVQ_OK;
}

// Invert a symmetric dim x dim matrix (2 or 3) by cofactors; returns det.
double invert(const double* R, int d, double* Ri) {
    if (d == 2) {
        const double det = R[0] * R[3] - R[1] * R[2];
        Ri[0] = R[3] / det; Ri[1] = -R[1] / det; Ri[2] = -R[2] / det; Ri[3] = R[0] / det;
        return det;
    }
    const double a = R[0], b = R[1], c = R[2], d_ = R[3], e = R[4], f = R[5], g = R[6], h = R[7], i = R[8];
    const double A = e * i - f * h, B = -(d_ * i - f * g), C = d_ * h - e * g;
    const double det = a * A + b * B + c * C;
    Ri[0] = A / det; Ri[1] = -(b * i - c * h) / det; Ri[2] = (b * f - c * e) / det;
    Ri[3] = B / det; Ri[4] = (a * i - c * g) / det;  Ri[5] = -(a * f - c * d_) / det;
    Ri[6] = C / det; Ri[7] = -(a * h - b * g) / det; Ri[8] = (a * e - b * d_) / det;
    return det;
}

}  // namespace

// =================================================================== C ABI
extern "C" {

const char* cvq_last_error(void) { return g_err.c_str(); }
int32_t cvq_version(void) { return 10000; }

int32_t cvq_device_count(int32_t* count) {
    CVQ_REQUIRE(count != nullptr, CVQ_ERR_INVALID, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return CVQ_OK;
}

int32_t cvq_plan_create(const cvq_static* s, int32_t device, cvq_plan** out) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(s != nullptr && out != nullptr, CVQ_ERR_INVALID, "NULL argument");
    *out = nullptr;
    CVQ_REQUIRE(s->model >= CVQ_MSM && s->model <= CVQ_UKF, CVQ_ERR_INVALID, "unknown model kind");
    CVQ_REQUIRE(s->copula >= CVQ_GAUSSIAN && s->copula <= CVQ_PLACKETT, CVQ_ERR_INVALID, "unknown copula kind");
    CVQ_REQUIRE(s->dim == 2 || s->dim == 3, CVQ_ERR_UNSUPPORTED, "dim must be 2 or 3");
    CVQ_REQUIRE(!(s->copula == CVQ_PLACKETT && s->dim != 2), CVQ_ERR_UNSUPPORTED,
                "Plackett copula is only defined for 2-dimensional marginals (plackett.py:20-21)");
    CVQ_REQUIRE(s->n >= 2 && s->n <= 1024, CVQ_ERR_UNSUPPORTED, "num_points must be in [2, 1024]");
    CVQ_REQUIRE(s->n <= 512 || (s->strategy == CVQ_STRATEGY_SORTED && s->dim == 2), CVQ_ERR_UNSUPPORTED,
                "num_points > 512 needs the SORTED strategy in 2-D (every strategy takes n <= 512)");
    CVQ_REQUIRE(s->q >= 1 && s->q <= kMaxQ, CVQ_ERR_UNSUPPORTED, "q (unique vol states) must be in [1, 8]");
    int Q = 1;
    for (int d = 0; d < s->dim; ++d) Q *= s->q;
    CVQ_REQUIRE(s->n_combos == Q, CVQ_ERR_INVALID, "n_combos must equal q**dim");
    CVQ_REQUIRE(s->model == CVQ_MSM || s->q == 1, CVQ_ERR_INVALID, "GARCH/UKF plans have q == 1");
    CVQ_REQUIRE(s->x_values && s->step && s->densities && s->combos && s->weights && s->copula_params,
                CVQ_ERR_INVALID, "NULL static table");
    CVQ_REQUIRE(s->model != CVQ_MSM || s->vol_states != nullptr, CVQ_ERR_INVALID, "MSM needs vol_states");
    CVQ_REQUIRE(s->weights[0] > 0.0, CVQ_ERR_UNSUPPORTED, "weights[0] must be > 0");
    CVQ_REQUIRE(s->strategy >= CVQ_STRATEGY_PREFIX && s->strategy <= CVQ_STRATEGY_SWEEP, CVQ_ERR_INVALID,
                "unknown strategy");
    CVQ_REQUIRE(!(s->strategy == CVQ_STRATEGY_SWEEP && s->dim != 2), CVQ_ERR_UNSUPPORTED,
                "the SWEEP strategy is built for dim == 2");
    CVQ_REQUIRE(!((s->strategy == CVQ_STRATEGY_DIRECT || s->strategy == CVQ_STRATEGY_COMPACT) && s->dim != 2),
                CVQ_ERR_UNSUPPORTED, "the DIRECT and COMPACT strategies are built for dim == 2");
    CVQ_REQUIRE(!(s->strategy == CVQ_STRATEGY_SORTED && s->dim == 3 && s->n > 255), CVQ_ERR_UNSUPPORTED,
                "the SORTED strategy supports num_points <= 255 in 3-D");
    for (int l = 0; l < Q; ++l) {             // create_vol_combinations ij order (msm_estimation.py:384)
        int rem = l;
        for (int d = s->dim - 1; d >= 0; --d) {
            CVQ_REQUIRE(s->combos[l * s->dim + d] == rem % s->q, CVQ_ERR_INVALID,
                        "combos must be the ij-meshgrid index combinations");
            rem /= s->q;
        }
    }
    for (int i = 1; i < s->n; ++i)
        CVQ_REQUIRE(s->x_values[i] > s->x_values[i - 1], CVQ_ERR_INVALID, "x_values must be increasing");
    int rc = ensure_device(device);
    if (rc) return rc;

    cvq_plan* p = new cvq_plan();
    p->device = device;
    p->strategy = s->strategy;
    p->v_cap = s->v_cap;
    p->hx.assign(s->x_values, s->x_values + s->n);
    StaticDev& S = p->S;
    S.model = s->model;
    S.copula = s->copula;
    S.dim = s->dim;
    S.n = s->n;
    S.q = s->q;
    S.Q = Q;
    S.nrows = s->dim == 2 ? s->n : s->n * s->n;
    S.w0 = s->weights[0];
    {   // exact reciprocal: w0 = 2^e (frexp mantissa 1/2) and 1/w0 a normal double
        int e2 = 0;
        const double m2 = std::frexp(s->weights[0], &e2);
        S.w0_inv = (m2 == 0.5 && std::isnormal(1.0 / s->weights[0])) ? 1.0 / s->weights[0] : 0.0;
    }
    S.w1 = s->weights[1];
    S.w2 = s->dim == 3 ? s->weights[2] : 0.0;

    // copula constants, computed as the reference does on the host
    const int d = s->dim;
    const double* cp = s->copula_params;
    if (s->copula == CVQ_PLACKETT) {
        CVQ_REQUIRE(s->n_copula_params >= 1, CVQ_ERR_INVALID, "Plackett needs theta");
        S.theta = cp[0];
    } else {
        const int nrho = d * (d - 1) / 2;
        const int base = s->copula == CVQ_STUDENT ? 1 : 0;
        CVQ_REQUIRE(s->n_copula_params == base + nrho, CVQ_ERR_INVALID, "wrong copula parameter count");
        double R[9];
        int k = 0;
        for (int i = 0; i < d; ++i) R[i * d + i] = 1.0;
        for (int i = 0; i < d; ++i)                 // triu / tril fill (student_estimation.py:50-54)
            for (int j = i + 1; j < d; ++j) { R[i * d + j] = R[j * d + i] = cp[base + k]; ++k; }
        const double det = invert(R, d, S.Ri);
        if (s->copula == CVQ_STUDENT) {
            const double nu = cp[0];
            CVQ_REQUIRE(nu > 0.0, CVQ_ERR_INVALID, "nu must be > 0");
            S.nu = nu;
            S.inv_nu = 1.0 / nu;
            S.term1 = std::tgamma((nu + d) / 2) /
                      (std::tgamma(nu / 2) * std::pow(nu * M_PI, d / 2.0) * std::sqrt(det));   // student.py:138
            S.g_uni = std::tgamma((nu + 1) / 2) / (std::sqrt(nu * M_PI) * std::tgamma(nu / 2)); // :164
            S.inv_g_uni = 1.0 / S.g_uni;
            S.node_ex = -(nu + d) / 2;
            S.uni_ex = -(nu + 1) / 2;
            const double mu = nu + 1;
            S.uni_m = (mu == std::floor(mu) && mu <= 16.0) ? (int)mu : -1;
            const double m2 = -2.0 * S.node_ex;
            S.node_m = (m2 == std::floor(m2) && m2 <= 128.0) ? (int)m2 : -1;
            if (int rc2 = make_tconst(nu, &S.tk, &p->d_cf)) { cvq_plan_destroy(p); return rc2; }
        } else {
            S.term1 = 1 / (std::sqrt(std::pow(2 * M_PI, d) * det));                              // gaussian.py:107
        }
    }

    // static tables
    const int n = s->n, q = s->q;
    std::vector<double> F((size_t)d * q * n);
    for (int c = 0; c < d; ++c)                     // axis c uses densities[(c-1) mod dim] (Q5)
        for (int sidx = 0; sidx < q; ++sidx)
            for (int i = 0; i < n; ++i)
                F[((size_t)c * q + sidx) * n + i] =
                    s->densities[((size_t)((c - 1 + d) % d) * q + sidx) * n + i] * s->step[i];
    // geometry: reachable inner nodes per row at v_cap (create_grids.py:104-108)
    std::vector<int> kmax(S.nrows);
    std::vector<long long> off(S.nrows);
    long long G = 0;
    const double* x = s->x_values;
    for (int r = 0; r < S.nrows; ++r) {
        double lev;
        if (d == 2) lev = x[r] * S.w1;
        else lev = x[r / n] * S.w1 + x[r % n] * S.w2;
        const double g = (s->v_cap - lev) / S.w0;
        int k = 0;
        for (int j = 1; j < n; ++j) if (x[j] <= g) k = j;
        kmax[r] = k;
        off[r] = G;
        G += k;
    }
    S.G = G;
    rc = 0;
    do {
        if ((rc = dev_alloc(&p->d_x, n))) break;
        if ((rc = dev_alloc(&p->d_F, F.size()))) break;
        if ((rc = dev_alloc(&p->d_kmax, kmax.size()))) break;
        if ((rc = dev_alloc(&p->d_off, off.size()))) break;
        if ((rc = dev_alloc(&p->d_hdr, 1))) break;
        if ((rc = dev_alloc(&p->d_err, 4))) break;
    } while (0);
    if (rc) { cvq_plan_destroy(p); return rc; }
    hipError_t e = hipStreamCreateWithFlags(&p->own_stream, hipStreamNonBlocking);
    if (e != hipSuccess) { set_error("hipStreamCreate failed"); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
    p->stream = p->own_stream;
    e = hipMemset(p->d_err, 0, 4 * sizeof(int));         // error words + the fused-finalize ticket
    if (e == hipSuccess) e = hipMemset(p->d_hdr, 0, sizeof(Header));
    if (e == hipSuccess) e = hipMemcpy(p->d_x, x, n * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_F, F.data(), F.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_kmax, kmax.data(), kmax.size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_off, off.data(), off.size() * sizeof(long long), hipMemcpyHostToDevice);
    if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
    S.x = p->d_x;
    S.F = p->d_F;
    S.kmax = p->d_kmax;
    S.off = p->d_off;
    if (s->model == CVQ_MSM) {
        if ((rc = dev_alloc(&p->d_uvs, (size_t)d * q)) || (rc = dev_alloc(&p->d_phi, (size_t)d * q * n))) {
            cvq_plan_destroy(p);
            return rc;
        }
        e = hipMemcpy(p->d_uvs, s->vol_states, (size_t)d * q * sizeof(double), hipMemcpyHostToDevice);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
        const int total = d * q * n;
        hipLaunchKernelGGL(k_phi, dim3((total + 255) / 256), dim3(256), 0, p->stream, S, p->d_uvs, p->d_phi);
        e = hipStreamSynchronize(p->stream);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
        S.phi = p->d_phi;
    }
    if (sorted_family(p)) {                            // reachable nodes sorted by their exact threshold v*
        std::vector<uint32_t> idx;
        p->layout = sorted_layout(S.dim, n);
        build_sorted_nodes(p->hx, S, kmax, p->layout, p->hvs, idx);
        const size_t nv = idx.size();
        p->hidx = idx;
        idx.resize(((nv + 3) & ~(size_t)3) + kSortIdxPad, 0u);   // range sums' / passes' loads past the end
        if ((rc = dev_alloc(&p->d_sidx, idx.size())) || (rc = dev_alloc(&p->d_svs, nv))) {
            cvq_plan_destroy(p);
            return rc;
        }
        e = hipMemcpy(p->d_sidx, idx.data(), idx.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_svs, p->hvs.data(), nv * sizeof(double), hipMemcpyHostToDevice);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
    }
    // exact level thresholds + grid lookup buckets; only for grids k_compact runs (larger ones solve
    // on k_direct, and the tail list's 11-bit row / column fields would overflow)
    if (p->strategy == CVQ_STRATEGY_COMPACT && n <= compact_max_n()) {
        std::vector<double> vs;
        build_vstar(p->hx, S.w0, S.w1, vs);
        p->hvc.clear();
        p->hvc.reserve((size_t)n * (n - 1));
        // COMPACT's nodes: j >= 1 (Q9), sorted by v* (ties by (r, j)): hvc and the block tail's list
        std::vector<uint32_t> ord;
        ord.reserve((size_t)n * (n - 1));
        for (int r = 0; r < n; ++r)
            for (int j = 1; j < n; ++j) ord.push_back((uint32_t)(r * n + j));
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return vs[a] < vs[b]; });
        std::vector<uint32_t> tl(ord.size());
        for (size_t i = 0; i < ord.size(); ++i) {
            p->hvc.push_back(vs[ord[i]]);
            const uint32_t r = ord[i] / n, j = ord[i] % n;
            const bool gend = i + 1 == ord.size() || !(vs[ord[i + 1]] == vs[ord[i]]);
            tl[i] = r | (j << kTlColShift) | (gend ? kTlGroupEnd : 0u);
        }
        if ((rc = dev_alloc(&p->d_tlist, tl.size())) || (rc = dev_alloc(&p->d_tvs, p->hvc.size()))) {
            cvq_plan_destroy(p);
            return rc;
        }
        e = hipMemcpy(p->d_tlist, tl.data(), tl.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_tvs, p->hvc.data(), p->hvc.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
        std::vector<int16_t> bk;
        build_buckets(p->hx, bk, &p->bx0, &p->binv);
        p->nb = (int)bk.size();
        if ((rc = dev_alloc(&p->d_vstar, vs.size())) || (rc = dev_alloc(&p->d_bucket, bk.size()))) {
            cvq_plan_destroy(p);
            return rc;
        }
        e = hipMemcpy(p->d_vstar, vs.data(), vs.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(p->d_bucket, bk.data(), bk.size() * sizeof(int16_t), hipMemcpyHostToDevice);
        if (e != hipSuccess) { set_error(hipGetErrorString(e)); cvq_plan_destroy(p); return CVQ_ERR_HIP; }
    }
    *out = p;
    return CVQ_OK;
}

int32_t cvq_plan_destroy(cvq_plan* p) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    if (!p) return CVQ_OK;
    (void)hipSetDevice(p->device);
    if (p->own_stream) (void)hipStreamSynchronize(p->own_stream);
    if (p->stream != p->own_stream) (void)hipStreamSynchronize(p->stream);   // work still using our buffers
    for (auto& e : p->events) { (void)hipEventDestroy(e.second.first); (void)hipEventDestroy(e.second.second); }
    for (void* b : {(void*)p->d_x, (void*)p->d_F, (void*)p->d_phi, (void*)p->d_uvs, (void*)p->d_cf, (void*)p->d_kmax,
                    (void*)p->d_off, (void*)p->d_a, (void*)p->d_pi, (void*)p->d_tA, (void*)p->d_tB,
                    (void*)p->d_C, (void*)p->d_snap, (void*)p->d_hdr, (void*)p->d_err, (void*)p->d_io, (void*)p->d_stamps,
                    (void*)p->d_cutfix, (void*)p->d_kcut, (void*)p->d_fpair, (void*)p->d_ccount, (void*)p->d_tlist, (void*)p->d_tvs, (void*)p->d_defer, (void*)p->d_vstar, (void*)p->d_bucket, (void*)p->d_sidx, (void*)p->d_svs,
                    (void*)p->d_tree, (void*)p->d_pass,
                    (void*)p->d_pidx, (void*)p->d_pvs})
        if (b) (void)hipFree(b);
    if (p->own_stream) (void)hipStreamDestroy(p->own_stream);
    delete p;
    return CVQ_OK;
}

int32_t cvq_plan_set_stream(cvq_plan* p, void* s) {
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    p->stream = (hipStream_t)s;                       // NULL = the HIP null stream
    return CVQ_OK;
}

int32_t cvq_plan_info(const cvq_plan* p, int64_t* reach, int32_t* rows) {
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    if (reach) *reach = p->S.G;
    if (rows) *rows = p->S.nrows;
    return CVQ_OK;
}

int32_t cvq_plan_timing(cvq_plan* p, int32_t enable) {
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    for (auto& e : p->events) { (void)hipEventDestroy(e.second.first); (void)hipEventDestroy(e.second.second); }
    p->events.clear();
    p->timing = enable;
    return CVQ_OK;
}

int32_t cvq_plan_kernel_time(cvq_plan* p, int32_t kind, double* total_ms, int32_t* launches) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && total_ms != nullptr && launches != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_HIP_CHECK(hipSetDevice(p->device));          // the plan's device (its stream and buffers)
    CVQ_REQUIRE(kind >= 0 && kind < TK_COUNT, CVQ_ERR_INVALID, "unknown kernel kind");
    double tot = 0.0;
    int cnt = 0;
    for (auto& e : p->events) {
        if (e.first != kind) continue;
        CVQ_HIP_CHECK(hipEventSynchronize(e.second.second));
        float ms = 0.f;
        CVQ_HIP_CHECK(hipEventElapsedTime(&ms, e.second.first, e.second.second));
        tot += ms;
        ++cnt;
    }
    *total_ms = tot;
    *launches = cnt;
    return CVQ_OK;
}

int32_t cvq_plan_debug_stamps(cvq_plan* p, uint64_t* host, int64_t count) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && host != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_HIP_CHECK(hipSetDevice(p->device));          // the plan's device (its stream and buffers)
    CVQ_REQUIRE(p->d_stamps != nullptr, CVQ_ERR_STATE, "no stamps recorded (set CVQ_STAMPS=1; DIRECT, COMPACT or SORTED strategy)");
    CVQ_REQUIRE(count <= p->capStamps * 32, CVQ_ERR_INVALID, "count exceeds the stamp buffer");
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    CVQ_HIP_CHECK(hipMemcpy(host, p->d_stamps, count * 8, hipMemcpyDeviceToHost));
    return CVQ_OK;
}

int32_t cvq_plan_debug_nodes(cvq_plan* p, uint32_t* host, int64_t count, int32_t* fix) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && host != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_HIP_CHECK(hipSetDevice(p->device));          // the plan's device (its stream and buffers)
    CVQ_REQUIRE(p->d_pidx != nullptr && p->tree_valid, CVQ_ERR_STATE,
                "no solve-order node list (a SORTED plan builds it at its first solve)");
    CVQ_REQUIRE(count >= 0 && count <= (int64_t)p->S.G, CVQ_ERR_INVALID, "count must be in [0, reachable nodes]");
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    CVQ_HIP_CHECK(hipMemcpy(host, p->d_pidx, count * sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (fix) for (int e = 0; e < 6; ++e) fix[e] = p->fixpos[e];
    return CVQ_OK;
}

int32_t cvq_plan_debug_cuts(cvq_plan* p, int32_t* host, int64_t cap, int32_t* count) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && count != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(p->tree_valid, CVQ_ERR_STATE, "no solve-order node list (a SORTED plan builds it at its first solve)");
    *count = (int32_t)p->hcuts.size();
    if (host) for (int64_t k = 0; k < std::min<int64_t>(cap, (int64_t)p->hcuts.size()); ++k) host[k] = p->hcuts[k];
    return CVQ_OK;
}

int32_t cvq_plan_count_nodes(cvq_plan* p, int32_t enable) {
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    CVQ_REQUIRE(!enable || p->strategy == CVQ_STRATEGY_COMPACT || p->strategy == CVQ_STRATEGY_SORTED ||
                    p->strategy == CVQ_STRATEGY_SWEEP,
                CVQ_ERR_UNSUPPORTED, "node counts are recorded by the COMPACT, SORTED and SWEEP solves");
    p->count_nodes = enable != 0;
    p->nodes_valid = false;
    return CVQ_OK;
}

int32_t cvq_plan_nodes_evaluated(cvq_plan* p, int64_t* total) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && total != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_HIP_CHECK(hipSetDevice(p->device));          // the plan's device (its stream and buffers)
    CVQ_REQUIRE(p->nodes_valid && p->d_stamps != nullptr, CVQ_ERR_STATE,
                "no node counts recorded (cvq_plan_count_nodes(plan, 1), then cvq_solve)");
    std::vector<unsigned long long> h((size_t)p->T * 32);
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    CVQ_HIP_CHECK(hipMemcpy(h.data(), p->d_stamps, h.size() * 8, hipMemcpyDeviceToHost));
    long long s = 0;
    for (long long t = 0; t < p->T; ++t) s += (long long)h[(size_t)t * 32 + 28];
    *total = s;
    return CVQ_OK;
}

int32_t cvq_set_fast_hint(cvq_plan* p, int32_t on) {
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    p->fast_hint = on != 0;
    return CVQ_OK;
}

int32_t cvq_set_dates(cvq_plan* p, int64_t T, const double* a, const double* b, int32_t mem) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && a != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(T > 0, CVQ_ERR_INVALID, "T must be > 0");
    CVQ_REQUIRE(p->S.model != CVQ_MSM || b != nullptr, CVQ_ERR_INVALID, "MSM needs the forecast combinations");
    CVQ_HIP_CHECK(hipSetDevice(p->device));
    const StaticDev& S = p->S;
    const size_t na = (size_t)T * S.dim * (S.model == CVQ_MSM ? S.q : 1);
    const size_t npi = (size_t)T * S.Q;
    const bool realloc = T > p->capT;
    if (realloc) {
        int rc;
        if ((rc = dev_alloc(&p->d_a, na)) || (rc = dev_alloc(&p->d_pi, npi))) return rc;
        const bool tables = p->strategy == CVQ_STRATEGY_PREFIX || !direct_fused(p);
        if (tables && ((rc = dev_alloc(&p->d_tA, (size_t)T * S.dim * S.n)) ||
                       (rc = dev_alloc(&p->d_tB, (size_t)T * S.dim * S.n))))
            return rc;
        if (p->strategy == CVQ_STRATEGY_PREFIX && (rc = dev_alloc(&p->d_C, (size_t)T * S.G))) return rc;
        p->capT = T;
    }
    p->T = T;
    if (mem == CVQ_MEM_DEVICE) {
        // device-resident inputs are read in place by the next launches (no copy);
        // the caller keeps them alive and unchanged until the next cvq_set_dates
        p->in_a = a;
        p->in_pi = S.model == CVQ_MSM ? b : p->d_pi;
    } else {
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_a, a, na * sizeof(double), hipMemcpyHostToDevice, p->stream));
        if (S.model == CVQ_MSM)
            CVQ_HIP_CHECK(hipMemcpyAsync(p->d_pi, b, npi * sizeof(double), hipMemcpyHostToDevice, p->stream));
        p->in_a = p->d_a;
        p->in_pi = p->d_pi;
    }
    p->fast_hint = mem != CVQ_MEM_DEVICE && fast_path_proven(S, p->hx, T, a, b);
    if (S.model != CVQ_MSM && realloc) {          // GARCH/UKF: pi_t = [1.0] (Q = 1), set once
        std::vector<double> ones((size_t)p->capT * S.Q, 1.0);
        CVQ_HIP_CHECK(hipMemcpyAsync(p->d_pi, ones.data(), ones.size() * sizeof(double), hipMemcpyHostToDevice,
                                     p->stream));
        CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    }
    if (mem != CVQ_MEM_DEVICE) CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    p->tables_valid = false;
    p->mass_valid = false;
    return CVQ_OK;
}

int32_t cvq_slab(cvq_plan* p, const double* bounds, double* out, int32_t mem) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && bounds != nullptr && out != nullptr, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(p->T > 0, CVQ_ERR_STATE, "cvq_set_dates must be called first");
    if (mem != CVQ_MEM_DEVICE && materialised(p)) {
        for (long long t = 0; t < 2 * p->T; ++t)
            CVQ_REQUIRE(!(bounds[t] > p->v_cap), CVQ_ERR_RANGE, "a bound exceeds the plan's v_cap");
    }
    int rc = ensure_mass(p);
    if (rc) return rc;
    if (mem == CVQ_MEM_DEVICE) return launch_slab(p, bounds, out);
    if ((rc = ensure_io(p, 3 * p->T))) return rc;
    CVQ_HIP_CHECK(hipMemcpyAsync(p->d_io, bounds, 2 * p->T * sizeof(double), hipMemcpyHostToDevice, p->stream));
    if ((rc = launch_slab(p, p->d_io, p->d_io + 2 * p->T))) return rc;
    CVQ_HIP_CHECK(hipMemcpyAsync(out, p->d_io + 2 * p->T, p->T * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    return CVQ_OK;
}

int32_t cvq_snap_stride(const cvq_solve_args* a, int32_t* stride) {
    CVQ_REQUIRE(a != nullptr && stride != nullptr, CVQ_ERR_INVALID, "NULL argument");
    bool exact;
    int K = bisect_budget(*a, &exact);
    if (!exact) K += 2;
    CVQ_REQUIRE(K <= kMaxIters, CVQ_ERR_UNSUPPORTED, "bisection needs more than 62 iterations");
    *stride = K + 1;
    return CVQ_OK;
}

int32_t cvq_solve_local(cvq_plan* p, const cvq_solve_args* a, void* d_header, double* d_snaps) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && d_header != nullptr && d_snaps != nullptr, CVQ_ERR_INVALID, "NULL argument");
    int rc = check_args(p, a);
    if (rc) return rc;
    int32_t stride;
    if ((rc = cvq_snap_stride(a, &stride))) return rc;
    if ((rc = ensure_mass(p, (Header*)d_header))) return rc;
    return launch_solve(p, solve_const(*a, stride - 1), d_snaps, (Header*)d_header);
}

int32_t cvq_solve_finalize(cvq_plan* p, const cvq_solve_args* a, const void* d_headers, int32_t n_ranks,
                           const double* d_snaps, int64_t dates_per_rank, int64_t T_total, double* d_var) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && a != nullptr && d_headers && d_snaps && d_var, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(n_ranks >= 1 && T_total <= (int64_t)n_ranks * dates_per_rank, CVQ_ERR_INVALID,
                "T_total exceeds n_ranks * dates_per_rank");
    int32_t stride;
    int rc = cvq_snap_stride(a, &stride);
    if (rc) return rc;
    CVQ_HIP_CHECK(hipSetDevice(p->device));
    const unsigned blocks = (unsigned)std::max<long long>(1, (T_total + 255) / 256);
    TimedScope ts(p, TK_FINALIZE);
    hipLaunchKernelGGL(k_finalize, dim3(blocks), dim3(256), 0, p->stream, (const Header*)d_headers, n_ranks,
                       d_snaps, (long long)T_total, stride, stride - 1, a->ptf_mean, d_var, p->d_err);
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int32_t cvq_packed_block_len(const cvq_solve_args* a, int64_t dates_per_rank, int64_t* len, int64_t* header_offset) {
    CVQ_REQUIRE(a != nullptr && len != nullptr && dates_per_rank >= 1, CVQ_ERR_INVALID, "bad argument");
    int32_t stride;
    int rc = cvq_snap_stride(a, &stride);
    if (rc) return rc;
    const int64_t hoff = (dates_per_rank * stride + 1) & ~(int64_t)1;    // 16-B aligned header
    *len = hoff + 2;
    if (header_offset) *header_offset = hoff;
    return CVQ_OK;
}

int32_t cvq_solve_finalize_packed(cvq_plan* p, const cvq_solve_args* a, const double* d_blocks, int32_t n_ranks,
                                  int64_t dates_per_rank, int64_t T_total, double* d_var) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && a != nullptr && d_blocks && d_var, CVQ_ERR_INVALID, "NULL argument");
    CVQ_REQUIRE(n_ranks >= 1 && dates_per_rank >= 1 && T_total <= (int64_t)n_ranks * dates_per_rank, CVQ_ERR_INVALID,
                "T_total exceeds n_ranks * dates_per_rank");
    CVQ_REQUIRE(((uintptr_t)d_blocks & 15) == 0, CVQ_ERR_INVALID, "packed blocks must be 16-byte aligned");
    int32_t stride;
    int64_t len, hoff;
    int rc = cvq_snap_stride(a, &stride);
    if (rc || (rc = cvq_packed_block_len(a, dates_per_rank, &len, &hoff))) return rc;
    CVQ_HIP_CHECK(hipSetDevice(p->device));
    const unsigned blocks = (unsigned)std::max<long long>(1, (T_total + 255) / 256);
    TimedScope ts(p, TK_FINALIZE);
    hipLaunchKernelGGL(k_finalize_packed, dim3(blocks), dim3(256), 0, p->stream, d_blocks, n_ranks,
                       (long long)dates_per_rank, (long long)len, (long long)hoff, (long long)T_total, stride,
                       stride - 1, a->ptf_mean, d_var, p->d_err);
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

int32_t cvq_solve_status(cvq_plan* p, int32_t* iters_out) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr, CVQ_ERR_INVALID, "plan is NULL");
    CVQ_HIP_CHECK(hipSetDevice(p->device));
    int err[3] = {0, 0, 0};
    CVQ_HIP_CHECK(hipMemcpyAsync(err, p->d_err, 3 * sizeof(int), hipMemcpyDeviceToHost, p->stream));
    CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
    if (iters_out) *iters_out = err[1];
    CVQ_REQUIRE(err[0] == 0, CVQ_ERR_NUMERIC, solve_error_text(err[0]));
    return CVQ_OK;
}

int32_t cvq_solve(cvq_plan* p, const cvq_solve_args* a, double* var_out, int32_t* iters_out, int32_t mem) {
    cvq::DeviceScope device_scope;                 // the caller's current device, restored on return
    CVQ_REQUIRE(p != nullptr && var_out != nullptr, CVQ_ERR_INVALID, "NULL argument");
    int rc = check_args(p, a);
    if (rc) return rc;
    // DIRECT / COMPACT keep p->d_hdr zero themselves (zeroed at creation, reset by the fused finalize)
    if ((rc = ensure_mass(p, p->strategy != CVQ_STRATEGY_PREFIX ? nullptr : p->d_hdr))) return rc;
    bool exact;
    int K = bisect_budget(*a, &exact);
    if (!exact) K += 2;
    for (bool first = true;; first = false) {
        CVQ_REQUIRE(K <= kMaxIters, CVQ_ERR_NUMERIC, "bisection did not converge within 62 iterations");
        const int stride = K + 1;
        if ((rc = ensure_snap(p, p->T * stride))) return rc;
        double* d_var = var_out;
        if (mem != CVQ_MEM_DEVICE) {
            if ((rc = ensure_io(p, p->T))) return rc;
            d_var = p->d_io;
        }
        if (!first) CVQ_HIP_CHECK(hipMemsetAsync(p->d_hdr, 0, sizeof(Header), p->stream));
        SolveConst P = solve_const(*a, K);
        if (p->strategy != CVQ_STRATEGY_PREFIX) {       // finalize fused into the solve's last workgroup
            P.fin_var = d_var;
            P.fin_err = p->d_err;
        }
        if ((rc = launch_solve(p, P, p->d_snap, p->d_hdr))) return rc;
        if (p->strategy == CVQ_STRATEGY_PREFIX) {
            const unsigned blocks = (unsigned)((p->T + 255) / 256);
            TimedScope ts(p, TK_FINALIZE);
            hipLaunchKernelGGL(k_finalize, dim3(blocks), dim3(256), 0, p->stream, (const Header*)p->d_hdr, 1,
                               (const double*)p->d_snap, p->T, stride, K, a->ptf_mean, d_var, p->d_err);
            CVQ_HIP_CHECK(hipGetLastError());
        }
        if (mem == CVQ_MEM_DEVICE && iters_out == nullptr) return CVQ_OK;
        int err[4] = {0, 0, 0, 0};
        CVQ_HIP_CHECK(hipMemcpyAsync(err, p->d_err, 3 * sizeof(int), hipMemcpyDeviceToHost, p->stream));
        CVQ_HIP_CHECK(hipStreamSynchronize(p->stream));
        CVQ_REQUIRE(!(err[0] & 4), CVQ_ERR_NUMERIC, solve_error_text(err[0]));
        if (err[0]) { K += 4; continue; }          // a date needed more than K iterations: widen
        if (iters_out) *iters_out = err[1];
        if (mem != CVQ_MEM_DEVICE) {
            CVQ_HIP_CHECK(hipMemcpy(var_out, d_var, p->T * sizeof(double), hipMemcpyDeviceToHost));
        }
        return CVQ_OK;
    }
}

}  // extern "C"
