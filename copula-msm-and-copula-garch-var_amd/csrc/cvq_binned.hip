// cvq_binned.hip -- launch side of the BINNED solve kernel (own translation unit:
// its template instances compile in parallel with cvq_plan.hip).
#include <hip/hip_runtime.h>

#define CVQ_NO_PLAN_KERNELS

#include "cvq_common.h"
#include "cvq_binned_kernels.h"

namespace cvq {
namespace {

struct BinLaunch {
    const StaticDev& S;
    const SolveConst& P;
    const BinGeom& BG;
    long long T;
    hipStream_t stream;
    const double *a, *pi;
    double *st, *snaps;
    Header* hdr;
};

template <int COP, bool MSM, int PM>
void launch_pm(const BinLaunch& L) {
    const size_t lds = sizeof(double) * ((size_t)5 * L.S.n + 5 * kRedW) +
                       sizeof(int16_t) * (L.S.n <= 256 ? 1 : 2) * 256 * (kE1 + 1);
    if (L.S.n <= 256)
        hipLaunchKernelGGL((k_binned<COP, MSM, 1, PM>), dim3((unsigned)L.T), dim3(256), lds, L.stream, L.S, L.P, L.BG,
                           L.a, L.pi, L.st, L.snaps, L.hdr);
    else
        hipLaunchKernelGGL((k_binned<COP, MSM, 2, PM>), dim3((unsigned)L.T), dim3(256), lds, L.stream, L.S, L.P, L.BG,
                           L.a, L.pi, L.st, L.snaps, L.hdr);
}

template <int COP, bool MSM>
void launch_m(const BinLaunch& L) {
    if constexpr (COP == CVQ_STUDENT) {
        if (L.S.node_m == 8) { launch_pm<COP, MSM, 8>(L); return; }      // nu = 6: b^-4, one rcp per node
    }
    launch_pm<COP, MSM, 0>(L);
}

template <int COP>
void launch_c(const BinLaunch& L) {
    if (L.S.model == CVQ_MSM) launch_m<COP, true>(L);
    else launch_m<COP, false>(L);
}

}  // namespace

int launch_binned(const StaticDev& S, const SolveConst& P, const BinGeom& BG, long long T, hipStream_t stream,
                  const double* a, const double* pi, double* st, double* snaps, Header* hdr) {
    const BinLaunch L{S, P, BG, T, stream, a, pi, st, snaps, hdr};
    switch (S.copula) {
        case CVQ_GAUSSIAN: launch_c<CVQ_GAUSSIAN>(L); break;
        case CVQ_STUDENT: launch_c<CVQ_STUDENT>(L); break;
        default: launch_c<CVQ_PLACKETT>(L); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

}  // namespace cvq
