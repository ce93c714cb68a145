// cvq_sorted.hip -- launch side of the SORTED solve kernel (own translation unit:
// its template instances compile in parallel with cvq_plan.hip).
#include <hip/hip_runtime.h>

#define CVQ_NO_PLAN_KERNELS

#include "cvq_common.h"
#include "cvq_sorted_kernels.h"

namespace cvq {
namespace {


struct SortedLaunch {
    const StaticDev& S;
    const SolveConst& P;
    const SortedGeom& G;
    long long T;
    hipStream_t stream;
    const double *a, *tA, *tB, *pi;
    int mode;
    const double* bounds;
    double *out, *snaps;
    Header* hdr;
    bool fused;
    double* stamps;
    bool sweep;
};

template <int COP, bool MSM, int DIM, int PM, bool FUSED, int LAY>
void launch_l(const SortedLaunch& L) {
    if constexpr (DIM == 2) {
        if (L.sweep && L.mode == 0) {                  // SWEEP: one pass per cell (2-D solves)
            hipLaunchKernelGGL((k_sorted<COP, MSM, DIM, kSortNT, PM, FUSED, LAY, true>), dim3((unsigned)L.T),
                               dim3(kSortNT), sorted_lds_bytes(L.S.n, kSortNT, DIM, true, LAY), L.stream, L.S, L.P,
                               L.G, L.a, L.tA, L.tB, L.pi, L.mode, L.bounds, L.out, L.snaps, L.hdr, L.stamps);
            return;
        }
    }
    hipLaunchKernelGGL((k_sorted<COP, MSM, DIM, kSortNT, PM, FUSED, LAY>), dim3((unsigned)L.T), dim3(kSortNT),
                       sorted_lds_bytes(L.S.n, kSortNT, DIM, false, LAY), L.stream, L.S, L.P, L.G, L.a, L.tA, L.tB,
                       L.pi, L.mode, L.bounds, L.out, L.snaps, L.hdr, L.stamps);
}

template <int COP, bool MSM, int DIM, int PM, bool FUSED>
void launch_f(const SortedLaunch& L) {
    if constexpr (DIM == 2) {
        if constexpr (COP == CVQ_STUDENT && PM > 0) {
            if (L.G.layout == kLay2W) { launch_l<COP, MSM, DIM, PM, FUSED, kLay2W>(L); return; }
        }
        launch_l<COP, MSM, DIM, PM, FUSED, kLay2>(L);
    } else {
        if (sorted_layout(DIM, L.S.n) == kLay3F) launch_l<COP, MSM, DIM, PM, FUSED, kLay3F>(L);
        else launch_l<COP, MSM, DIM, PM, FUSED, kLay3G>(L);
    }
}

template <int COP, bool MSM, int DIM, int PM>
void launch_pm(const SortedLaunch& L) {
    if (L.fused) launch_f<COP, MSM, DIM, PM, true>(L);
    else launch_f<COP, MSM, DIM, PM, false>(L);
}

template <int COP, bool MSM, int DIM>
void launch_d(const SortedLaunch& L) {
    if constexpr (COP == CVQ_STUDENT) {
        // integer nu + dim: b^-(nu+dim)/2 by squarings and one rcp (nu = 6: 8 in 2-D, 9 in 3-D)
        if (L.S.node_m == DIM + 6) { launch_pm<COP, MSM, DIM, DIM + 6>(L); return; }
    }
    launch_pm<COP, MSM, DIM, 0>(L);
}

template <int COP, bool MSM>
void launch_m(const SortedLaunch& L) {
    if (L.S.dim == 2) launch_d<COP, MSM, 2>(L);
    else if constexpr (COP != CVQ_PLACKETT) launch_d<COP, MSM, 3>(L);
}

template <int COP>
void launch_c(const SortedLaunch& L) {
    if (L.S.model == CVQ_MSM) launch_m<COP, true>(L);
    else launch_m<COP, false>(L);
}

}  // namespace

int launch_sorted(const StaticDev& S, const SolveConst& P, const SortedGeom& G, long long T, hipStream_t stream,
                  const double* a, const double* tA, const double* tB, const double* pi, bool fused, int mode,
                  const double* bounds, double* out, double* snaps, Header* hdr, double* stamps, bool sweep,
                  size_t abi) {
    CVQ_REQUIRE(abi == (kernel_abi_key() ^ (sizeof(SortedGeom) << 40)), CVQ_ERR_STATE,
                "libcvq objects built from different headers (rebuild all)");
    CVQ_REQUIRE(S.n <= sorted_max_n(S.dim), CVQ_ERR_UNSUPPORTED, "SORTED supports n <= 512 (2-D) / 255 (3-D)");
    const SortedLaunch L{S, P, G, T, stream, a, tA, tB, pi, mode, bounds, out, snaps, hdr, fused, stamps, sweep};
    switch (S.copula) {
        case CVQ_GAUSSIAN: launch_c<CVQ_GAUSSIAN>(L); break;
        case CVQ_STUDENT: launch_c<CVQ_STUDENT>(L); break;
        default: launch_c<CVQ_PLACKETT>(L); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

}  // namespace cvq
