// cvq_sorted.hip -- launch side of the SORTED solve kernel (own translation unit:
// its template instances compile in parallel with cvq_plan.hip).
#include <hip/hip_runtime.h>

#include <cstdlib>

#define CVQ_NO_PLAN_KERNELS

#include "cvq_sorted_launch.h"

namespace cvq {
namespace {

// Compute units of a device (cached; MI355X: 256).
int device_cus() {
    static int cus[64] = {0};
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return 256;
    if (!cus[d]) {
        int v = 0;
        cus[d] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0) ? v : 256;
    }
    return cus[d];
}

}  // namespace

// Threads per date (one workgroup each).  A date is a chain of dependent phases (tables, two
// fixed slabs, ~10 reduced levels, the tail), so a launch with few dates per CU is latency
// bound: wider workgroups split every range sum over more lanes and shorten the chain.  The
// widest width whose waves the chip holds at once (T NT / 64 <= CUs x 4 SIMDs x the kernel's
// waves per SIMD at that width, sorted_min_waves) -- i.e. a strong-scaling block of a few hundred dates per
// GPU runs 1024- or 512-thread dates, a full batch 256.  Counting whole workgroups per CU instead
// (625 dates: 384 threads, every workgroup resident) measured slower than 512 threads with the
// last ~100 dates starting late (cfg 3 133 vs 116 us, cfg 5 118 vs 103 us; profiles/r04o).
// CVQ_SORT_NT (256 / 384 / 512 / 1024) overrides (A/B).
// A 2-D grid with n > 512 needs the 1024-thread instance (sorted_max_n_nt).
int sorted_threads(long long T, int dim, int n) {
    const int nt_min = n > sorted_max_n_nt(dim, kSortNT) ? 1024 : kSortNT;
    const char* ev = getenv("CVQ_SORT_NT");            // read per launch: tests switch it per case
    const int env = ev ? atoi(ev) : 0;
    if ((env == 256 || env == 384 || env == 512 || env == 1024) && env >= nt_min) return env;
    for (int nt = 1024; nt > nt_min; nt >>= 1)
        if (T * (nt / 64) <= (long long)device_cus() * 4 * sorted_min_waves(dim, nt)) return nt;
    return nt_min;
}

int launch_sorted(const StaticDev& S, const SolveConst& P, const SortedGeom& G, long long T, hipStream_t stream,
                  const double* a, const double* tA, const double* tB, const double* pi, bool fused, int mode,
                  const double* bounds, double* out, double* snaps, Header* hdr, double* stamps, bool sweep,
                  size_t abi) {
    CVQ_REQUIRE(abi == (kernel_abi_key() ^ (sizeof(SortedGeom) << 40)), CVQ_ERR_STATE,
                "libcvq objects built from different headers (rebuild all)");
    CVQ_REQUIRE(S.n <= sorted_max_n(S.dim), CVQ_ERR_UNSUPPORTED, "SORTED supports n <= 1024 (2-D) / 255 (3-D)");
    CVQ_REQUIRE(!(sweep && S.n > sorted_max_n_nt(S.dim, kSortNT)), CVQ_ERR_UNSUPPORTED, "SWEEP supports n <= 512");
    const SortedLaunch L{S, P, G, T, stream, a, tA, tB, pi, mode, bounds, out, snaps, hdr, fused, stamps, sweep};
    const int nt = sorted_threads(T, S.dim, S.n);
    switch (nt) {
        case 1024: sorted_slice_1024(L); break;
        case 512: sorted_slice_512(L); break;
        case 384: sorted_slice_384(L); break;
        default: sorted_launch_nt<kSortNT>(L); break;
    }
    CVQ_HIP_CHECK(hipGetLastError());
    return CVQ_OK;
}

}  // namespace cvq
