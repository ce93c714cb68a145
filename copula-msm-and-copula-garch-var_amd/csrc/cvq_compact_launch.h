// cvq_compact_launch.h -- launch templates of the COMPACT solve kernel, shared by
// cvq_compact.hip (dispatch) and the instance slices of cvq_compact_inst.hip: each slice
// (copula x model x node power) is its own translation unit, so the kernel's template
// instances compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "cvq_common.h"
#include "cvq_compact_kernels.h"

#ifndef CVQ_COMPACT_NT
#define CVQ_COMPACT_NT 256
#endif
// the block tail's list words hold a row and a column < compact_max_n() = 2 NT in 11-bit fields
static_assert(2 * CVQ_COMPACT_NT - 1 <= (int)cvq::kTlRowMask, "tail list fields overflow");

namespace cvq {

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
    const size_t lds_fast = compact_lds_bytes<COP, false>(L.S.n, NT, L.G.nb);
    const size_t lds_gen = compact_lds_bytes<COP, true>(L.S.n, NT, L.G.nb);
    hipLaunchKernelGGL((k_compact<COP, MSM, NT, RPT, PM, FUSED, false>), dim3((unsigned)L.T), dim3(NT), lds_fast, L.stream,
                       L.S, L.P, L.G, L.a, L.tA, L.tB, L.pi, L.st, L.snaps, L.hdr, L.generic ? L.defer : nullptr, L.T);
    if (!L.generic) return;
    hipLaunchKernelGGL((k_compact<COP, MSM, NT, RPT, PM, FUSED, true>), dim3((unsigned)std::min(L.T, kGenericGrid)),
                       dim3(NT), lds_gen, L.stream, L.S, L.P, L.G, L.a, L.tA, L.tB, L.pi, L.st, L.snaps, L.hdr, L.defer, L.T);
}

// rows per thread: 1 or 2 (n <= compact_max_n() = 2 NT, the plan's num_points limit of 512)
template <int COP, bool MSM, int PM, bool FUSED>
void launch_f(const CompactLaunch& L) {
    constexpr int NT = CVQ_COMPACT_NT;
    const int rpt = (L.S.n + NT - 1) / NT;
    if (rpt <= 1) launch_r<COP, MSM, PM, FUSED, 1>(L);
    else launch_r<COP, MSM, PM, FUSED, 2>(L);
}

template <int COP, bool MSM, int PM>
void launch_pm(const CompactLaunch& L) {
    if (L.fused) launch_f<COP, MSM, PM, true>(L);
    else launch_f<COP, MSM, PM, false>(L);
}

// the instance slices (cvq_compact_inst.hip, one object per CVQ_INST_* in the Makefile)
void compact_slice_st_msm_8(const CompactLaunch& L);
void compact_slice_st_msm_0(const CompactLaunch& L);
void compact_slice_st_gar_8(const CompactLaunch& L);
void compact_slice_st_gar_0(const CompactLaunch& L);
void compact_slice_ga_msm(const CompactLaunch& L);
void compact_slice_ga_gar(const CompactLaunch& L);
void compact_slice_pl_msm(const CompactLaunch& L);
void compact_slice_pl_gar(const CompactLaunch& L);

}  // namespace cvq
