// cvq_common.h -- shared host/device definitions of libcvq (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/cvq.h"
#include "cvq_special.h"

namespace cvq {

constexpr int kMaxQ = 8;          // unique vol states per asset supported (MSM k <= 7)
constexpr int kMaxIters = 62;     // bisection snapshot budget (bits of the nonzero mask)

// Everything a quadrature kernel needs that is constant for a plan.  Passed by
// value as a kernel argument (fits the kernarg segment).
struct StaticDev {
    int model, copula, dim, n, q, Q;
    int nrows;                    // n^(dim-1) rows of the inner (last) axis
    int node_m;                   // pow fast-path code for -(nu+dim)/2 (see pow_node)
    double node_ex;               // -(nu+dim)/2
    double uni_ex;                // -(nu+1)/2
    int uni_m;                    // 2 * (nu+1)/2 when a half-integer <= 16, else -1
    double term1;                 // multivariate density constant (student.py:138 / gaussian.py:107)
    double g_uni;                 // univariate t constant (student.py:164)
    double inv_g_uni;             // 1 / g_uni (the integer-nu table path multiplies)
    double inv_nu, nu, theta;
    double Ri[9];                 // inverse correlation, row-major dim x dim
    double w0, w1, w2;            // portfolio weights
    double w0_inv;                // 1 / w0 when w0 is a power of two (then (v - lev) * w0_inv is the
                                  // reference's (v - lev) / w0 bit for bit), else 0: divide
    TConst tk;                    // Student-t quantile constants
    const double* x;              // [n] grid
    const double* F;              // [dim][q][n] static Delta factors dens[(c-1)%dim]*step (Q5)
    const double* phi;            // [dim][q][n] MSM: Phi(x_i / sigma_{d,s}), date independent
    const int* kmax;              // [nrows] inner nodes per row with level <= v_cap
    const long long* off;         // [nrows] row offset into a date's prefix block
    long long G;                  // reachable nodes per date (sum kmax)
};

// var_function's inner-axis coordinate g = (v - lev) / w0 (integration_algo.py:20, Q10), exact:
// a multiplication when 1 / w0 is exact (w0 a power of two, e.g. the 2-asset weights 1/2).
// (the division sits in a separate, non-inlined function: inlined, the compiler evaluates it
// next to the multiplication and selects, so the common case would still pay for it)
__host__ __device__ __attribute__((noinline)) inline double inner_coord_div(double d, double w0) { return d / w0; }
__host__ __device__ __forceinline__ double inner_coord(const StaticDev& S, double v, double lev) {
    if (S.w0_inv != 0.0) return (v - lev) * S.w0_inv;
    return inner_coord_div(v - lev, S.w0);
}

// Element idx of a global table through a 32-bit byte offset: the load takes the SGPR-base +
// VGPR-offset form (no 64-bit address arithmetic per load).  Tables below 4 GB only.
template <class T>
__device__ __forceinline__ T ld32(const T* __restrict__ base, unsigned idx) {
    return *(const T*)((const char*)base + idx * (unsigned)sizeof(T));
}

struct SolveConst {
    double obj, fg, sg0, sg1, vmin, vmax, lower, tol;
    int K;                        // bisection iterations executed (>= reference's count)
    int stride;                   // snapshot stride per date (K + 1)
    // fused finalize (single-rank DIRECT solve): the last workgroup to finish
    // resolves Q2/Q4 and writes fin_var[t] = snap[t][kstop] + ptf_mean.
    double ptf_mean;
    double* fin_var;              // nullptr: no fused finalize (sharded / PREFIX)
    int* fin_err;                 // [4]: error, kstop, N, workgroup ticket (0 between launches)
    int exact_walk;               // every bracket's bisection points are exact dyadics (dyadic_walk_ok):
                                  // COMPACT's tail walks its remaining levels in closed form, one per lane
};

struct alignas(16) Header {       // per-rank solve summary, all-gathered across ranks
    int32_t iters;                // max over dates of own convergence count (Q2)
    int32_t error;                // nonzero: a date did not converge within K
    uint64_t nonzero;             // bit k: some date had F != 0 at iteration k (Q4)
};

// Layout key of the structs passed between translation units (cvq_plan.hip launches the
// kernels compiled in cvq_compact.hip / cvq_sorted.hip): a stale object fails its launch
// with CVQ_ERR_STATE instead of reading misplaced pointers.
constexpr size_t kAbiVersion = 6;
__host__ __device__ constexpr size_t kernel_abi_key() {
    return kAbiVersion * 1000003u + sizeof(StaticDev) * 4099u + sizeof(SolveConst) * 67u + sizeof(Header);
}
}  // namespace cvq

// --------------------------------------------------------------- host errors
namespace cvq {
void set_error(const std::string& msg);

constexpr int kCfTerms = 400;     // continued-fraction coefficient table length

// Student-t constants for one nu + device copies of the two CF coefficient tables
// (written to *d_cf, 2 * kCfTerms doubles, owned by the caller).
int make_tconst(double nu, TConst* tk, double** d_cf);
}

#define CVQ_HIP_CHECK(expr)                                                        \
    do {                                                                           \
        hipError_t _e = (expr);                                                    \
        if (_e != hipSuccess) {                                                    \
            cvq::set_error(std::string("HIP error ") + hipGetErrorString(_e) +     \
                           " at " __FILE__ ":" + std::to_string(__LINE__) + ": " #expr); \
            return (_e == hipErrorOutOfMemory) ? CVQ_ERR_OOM : CVQ_ERR_HIP;        \
        }                                                                          \
    } while (0)

#define CVQ_REQUIRE(cond, code, msg)                                               \
    do {                                                                           \
        if (!(cond)) { cvq::set_error(msg); return (code); }                        \
    } while (0)

namespace cvq {
// The calling thread's current HIP device, restored when an entry point returns: the library
// switches to its plan's / argument's device for its own calls, and must not leave the caller
// (torch shares the process's current device) on another GPU.
struct DeviceScope {
    int prev = -1;
    DeviceScope() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceScope(const DeviceScope&) = delete;
    DeviceScope& operator=(const DeviceScope&) = delete;
};
}

// switch to device `dev` until the enclosing scope ends (range-checked; one per scope)
#define CVQ_DEVICE_SCOPE(dev)                                                      \
    cvq::DeviceScope _cvq_device_scope;                                            \
    do {                                                                           \
        int _nd = 0;                                                               \
        CVQ_HIP_CHECK(hipGetDeviceCount(&_nd));                                    \
        CVQ_REQUIRE((dev) >= 0 && (dev) < _nd, CVQ_ERR_INVALID, "device index out of range"); \
        CVQ_HIP_CHECK(hipSetDevice(dev));                                          \
    } while (0)
