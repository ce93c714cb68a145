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
    double inv_nu, nu, theta;
    double Ri[9];                 // inverse correlation, row-major dim x dim
    double w0, w1, w2;            // portfolio weights
    TConst tk;                    // Student-t quantile constants
    const double* x;              // [n] grid
    const double* F;              // [dim][q][n] static Delta factors dens[(c-1)%dim]*step (Q5)
    const double* phi;            // [dim][q][n] MSM: Phi(x_i / sigma_{d,s}), date independent
    const int* kmax;              // [nrows] inner nodes per row with level <= v_cap
    const long long* off;         // [nrows] row offset into a date's prefix block
    long long G;                  // reachable nodes per date (sum kmax)
};

struct SolveConst {
    double obj, fg, sg0, sg1, vmin, vmax, lower, tol;
    int K;                        // bisection iterations executed (>= reference's count)
    int stride;                   // snapshot stride per date (K + 1)
    // fused finalize (single-rank DIRECT solve): the last workgroup to finish
    // resolves Q2/Q4 and writes fin_var[t] = snap[t][kstop] + ptf_mean.
    double ptf_mean;
    double* fin_var;              // nullptr: no fused finalize (sharded / PREFIX)
    int* fin_err;                 // [4]: error, kstop, N, workgroup ticket (0 between launches)
};

struct alignas(16) Header {       // per-rank solve summary, all-gathered across ranks
    int32_t iters;                // max over dates of own convergence count (Q2)
    int32_t error;                // nonzero: a date did not converge within K
    uint64_t nonzero;             // bit k: some date had F != 0 at iteration k (Q4)
};

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
