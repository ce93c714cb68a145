// cvq_compact.hip -- launch side of the COMPACT solve kernel: dispatch to the instance
// slice of the plan's (copula, model, node power).  The slices are separate objects
// (cvq_compact_inst.hip), so their template instances compile in parallel with each
// other and with cvq_plan.hip.
#define CVQ_NO_PLAN_KERNELS
#include "cvq_compact_launch.h"

namespace cvq {

int compact_max_n() { return 2 * CVQ_COMPACT_NT; }      // 1 or 2 rows per thread (launch_f)
int compact_tail_cap() { return CVQ_COMPACT_NT * kBlkPerThread; }   // block tail: cell nodes per workgroup
int compact_nt() { return CVQ_COMPACT_NT; }

int launch_compact(const StaticDev& S, const SolveConst& P, const CompactGeom& G, long long T, hipStream_t stream,
                   const double* a, const double* tA, const double* tB, const double* pi, bool fused, double* st,
                   double* snaps, Header* hdr, int* defer, bool generic, size_t abi) {
    // the kernel arguments are structs shared with cvq_plan.hip: refuse a stale object
    CVQ_REQUIRE(abi == (kernel_abi_key() ^ (sizeof(CompactGeom) << 40)), CVQ_ERR_STATE,
                "libcvq objects built from different headers (rebuild all)");
    const CompactLaunch L{S, P, G, T, stream, a, tA, tB, pi, st, snaps, hdr, defer, fused, generic};
    const bool msm = S.model == CVQ_MSM;
    switch (S.copula) {
        case CVQ_STUDENT:
            if (S.node_m == 8) msm ? compact_slice_st_msm_8(L) : compact_slice_st_gar_8(L);
            else msm ? compact_slice_st_msm_0(L) : compact_slice_st_gar_0(L);
            break;
        case CVQ_GAUSSIAN: msm ? compact_slice_ga_msm(L) : compact_slice_ga_gar(L); break;
        default: msm ? compact_slice_pl_msm(L) : compact_slice_pl_gar(L); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

}  // namespace cvq
