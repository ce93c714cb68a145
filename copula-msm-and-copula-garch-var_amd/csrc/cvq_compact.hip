// cvq_compact.hip -- launch side of the COMPACT solve kernel (own translation
// unit: its template instances compile in parallel with cvq_plan.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#define CVQ_NO_PLAN_KERNELS

#include "cvq_common.h"
#include "cvq_compact_kernels.h"

#ifndef CVQ_COMPACT_NT
#define CVQ_COMPACT_NT 256
#endif

namespace cvq {
namespace {

struct CompactLaunch {
    const StaticDev& S;
    const SolveConst& P;
    const CompactGeom& G;
    long long T;
    hipStream_t stream;
    const double *a, *tA, *tB, *pi;
    double *st, *snaps;
    Header* hdr;
    int* defer;
    bool fused;
    bool generic;                // launch the deferred-date (generic path) kernel
};

// deferred (generic-path) dates: a small grid loops over them
constexpr long long kGenericGrid = 512;

template <int COP, bool MSM, int PM, bool FUSED, int RPT>
void launch_r(const CompactLaunch& L) {
    constexpr int NT = CVQ_COMPACT_NT;
    // experiment knob: extra dynamic LDS per workgroup (caps resident dates per CU)
    static const size_t lds_pad = getenv("CVQ_COMPACT_LDS_PAD") ? (size_t)atol(getenv("CVQ_COMPACT_LDS_PAD")) : 0;
    const size_t lds_fast = compact_lds_bytes<COP, false>(L.S.n, NT, L.G.nb) + lds_pad;
    const size_t lds_gen = compact_lds_bytes<COP, true>(L.S.n, NT, L.G.nb);
    hipLaunchKernelGGL((k_compact<COP, MSM, NT, RPT, PM, FUSED, false>), dim3((unsigned)L.T), dim3(NT), lds_fast, L.stream,
                       L.S, L.P, L.G, L.a, L.tA, L.tB, L.pi, L.st, L.snaps, L.hdr, L.generic ? L.defer : nullptr, L.T);
    if (!L.generic) return;
    hipLaunchKernelGGL((k_compact<COP, MSM, NT, RPT, PM, FUSED, true>), dim3((unsigned)std::min(L.T, kGenericGrid)),
                       dim3(NT), lds_gen, L.stream, L.S, L.P, L.G, L.a, L.tA, L.tB, L.pi, L.st, L.snaps, L.hdr, L.defer, L.T);
}

// rows per thread: ceil(n / NT) rounded up to 1, 2, 4 or 8 (n <= 8 NT)
template <int COP, bool MSM, int PM, bool FUSED>
void launch_f(const CompactLaunch& L) {
    constexpr int NT = CVQ_COMPACT_NT;
    const int rpt = (L.S.n + NT - 1) / NT;
#ifdef CVQ_DEV_CFG2            // experiment builds (tools/build_variant_compact.sh): cfg 2's instance only
    (void)rpt;
    launch_r<COP, MSM, PM, FUSED, 1>(L);
#else
    if (rpt <= 1) launch_r<COP, MSM, PM, FUSED, 1>(L);
    else if (rpt <= 2) launch_r<COP, MSM, PM, FUSED, 2>(L);
    else if (rpt <= 4) launch_r<COP, MSM, PM, FUSED, 4>(L);
    else launch_r<COP, MSM, PM, FUSED, 8>(L);
#endif
}

template <int COP, bool MSM, int PM>
void launch_pm(const CompactLaunch& L) {
#ifdef CVQ_DEV_CFG2
    launch_f<COP, MSM, PM, true>(L);
#else
    if (L.fused) launch_f<COP, MSM, PM, true>(L);
    else launch_f<COP, MSM, PM, false>(L);
#endif
}

template <int COP, bool MSM>
void launch_m(const CompactLaunch& L) {
    if constexpr (COP == CVQ_STUDENT) {
        if (L.S.node_m == 8) { launch_pm<COP, MSM, 8>(L); return; }      // nu = 6: b^-4, one rcp per node
    }
#ifndef CVQ_DEV_CFG2
    launch_pm<COP, MSM, 0>(L);
#endif
}

template <int COP>
void launch_c(const CompactLaunch& L) {
    if (L.S.model == CVQ_MSM) launch_m<COP, true>(L);
#ifndef CVQ_DEV_CFG2
    else launch_m<COP, false>(L);
#endif
}

}  // namespace

int compact_max_n() { return 8 * CVQ_COMPACT_NT; }
int compact_tail_cap() { return CVQ_COMPACT_NT * kBlkPerThread; }   // block tail: cell nodes per workgroup

int launch_compact(const StaticDev& S, const SolveConst& P, const CompactGeom& G, long long T, hipStream_t stream,
                   const double* a, const double* tA, const double* tB, const double* pi, bool fused, double* st,
                   double* snaps, Header* hdr, int* defer, bool generic, size_t abi) {
    // the kernel arguments are structs shared with cvq_plan.hip: refuse a stale object
    CVQ_REQUIRE(abi == (kernel_abi_key() ^ (sizeof(CompactGeom) << 40)), CVQ_ERR_STATE,
                "libcvq objects built from different headers (rebuild all)");
    const CompactLaunch L{S, P, G, T, stream, a, tA, tB, pi, st, snaps, hdr, defer, fused, generic};
#ifdef CVQ_DEV_CFG2
    launch_c<CVQ_STUDENT>(L);
#else
    switch (S.copula) {
        case CVQ_GAUSSIAN: launch_c<CVQ_GAUSSIAN>(L); break;
        case CVQ_STUDENT: launch_c<CVQ_STUDENT>(L); break;
        default: launch_c<CVQ_PLACKETT>(L); break;
    }
#endif
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

}  // namespace cvq
