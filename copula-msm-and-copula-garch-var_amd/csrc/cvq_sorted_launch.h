// cvq_sorted_launch.h -- launch templates of the SORTED solve kernel, shared by
// cvq_sorted.hip (dispatch, the 256-thread instances and SWEEP) and the slices of
// cvq_sorted_inst.hip (the 512- and 1024-thread instances a small per-GPU date
// block uses), each its own translation unit so the instances compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include "cvq_common.h"
#include "cvq_sorted_kernels.h"

namespace cvq {

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

template <int NT, int COP, bool MSM, int DIM, int PM, bool FUSED, int LAY>
void sorted_launch_l(const SortedLaunch& L) {
    if constexpr (DIM == 2) {
        if (L.sweep && L.mode == 0) {                  // SWEEP: passes for the first levels (2-D solves)
            hipLaunchKernelGGL((k_sorted<COP, MSM, DIM, NT, PM, FUSED, LAY, true>), dim3((unsigned)L.T),
                               dim3(NT), sorted_lds_bytes(L.S.n, NT, DIM, true, LAY), L.stream, L.S, L.P,
                               L.G, L.a, L.tA, L.tB, L.pi, L.mode, L.bounds, L.out, L.snaps, L.hdr, L.stamps);
            return;
        }
    }
    hipLaunchKernelGGL((k_sorted<COP, MSM, DIM, NT, PM, FUSED, LAY>), dim3((unsigned)L.T), dim3(NT),
                       sorted_lds_bytes(L.S.n, NT, DIM, false, LAY), L.stream, L.S, L.P, L.G, L.a, L.tA, L.tB,
                       L.pi, L.mode, L.bounds, L.out, L.snaps, L.hdr, L.stamps);
}

template <int NT, int COP, bool MSM, int DIM, int PM, bool FUSED>
void sorted_launch_f(const SortedLaunch& L) {
    if constexpr (DIM == 2) {
        sorted_launch_l<NT, COP, MSM, DIM, PM, FUSED, kLay2>(L);
    } else {
        if (sorted_layout(DIM, L.S.n) == kLay3F) sorted_launch_l<NT, COP, MSM, DIM, PM, FUSED, kLay3F>(L);
        else sorted_launch_l<NT, COP, MSM, DIM, PM, FUSED, kLay3G>(L);
    }
}

template <int NT, int COP, bool MSM, int DIM, int PM>
void sorted_launch_pm(const SortedLaunch& L) {
    if (L.fused) sorted_launch_f<NT, COP, MSM, DIM, PM, true>(L);
    else sorted_launch_f<NT, COP, MSM, DIM, PM, false>(L);
}

template <int NT, int COP, bool MSM, int DIM>
void sorted_launch_d(const SortedLaunch& L) {
    if constexpr (COP == CVQ_STUDENT) {
        // integer nu + dim: b^-(nu+dim)/2 by squarings and one rcp (nu = 6: 8 in 2-D, 9 in 3-D)
        if (L.S.node_m == DIM + 6) { sorted_launch_pm<NT, COP, MSM, DIM, DIM + 6>(L); return; }
    }
    sorted_launch_pm<NT, COP, MSM, DIM, 0>(L);
}

template <int NT, int COP, bool MSM>
void sorted_launch_m(const SortedLaunch& L) {
    if (L.S.dim == 2) sorted_launch_d<NT, COP, MSM, 2>(L);
    else if constexpr (COP != CVQ_PLACKETT) sorted_launch_d<NT, COP, MSM, 3>(L);
}

template <int NT>
void sorted_launch_nt(const SortedLaunch& L) {
    switch (L.S.copula) {
        case CVQ_GAUSSIAN:
            if (L.S.model == CVQ_MSM) sorted_launch_m<NT, CVQ_GAUSSIAN, true>(L);
            else sorted_launch_m<NT, CVQ_GAUSSIAN, false>(L);
            break;
        case CVQ_STUDENT:
            if (L.S.model == CVQ_MSM) sorted_launch_m<NT, CVQ_STUDENT, true>(L);
            else sorted_launch_m<NT, CVQ_STUDENT, false>(L);
            break;
        default:
            if (L.S.model == CVQ_MSM) sorted_launch_m<NT, CVQ_PLACKETT, true>(L);
            else sorted_launch_m<NT, CVQ_PLACKETT, false>(L);
            break;
    }
}

// the wider instances (cvq_sorted_inst.hip)
void sorted_slice_384(const SortedLaunch& L);
void sorted_slice_512(const SortedLaunch& L);
void sorted_slice_1024(const SortedLaunch& L);

}  // namespace cvq
