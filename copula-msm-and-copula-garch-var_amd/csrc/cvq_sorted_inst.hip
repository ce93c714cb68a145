// cvq_sorted_inst.hip -- the 384-, 512- and 1024-thread k_sorted instances, compiled once per
// CVQ_SORT_SLICE (Makefile) so they build in parallel with the 256-thread ones.  The
// dispatch (which width a launch takes) is launch_sorted (cvq_sorted.hip).
#define CVQ_NO_PLAN_KERNELS
#include "cvq_sorted_launch.h"

namespace cvq {

#if defined(CVQ_SORT_SLICE_384)
void sorted_slice_384(const SortedLaunch& L) { sorted_launch_nt<384>(L); }
#elif defined(CVQ_SORT_SLICE_512)
void sorted_slice_512(const SortedLaunch& L) { sorted_launch_nt<512>(L); }
#elif defined(CVQ_SORT_SLICE_1024)
void sorted_slice_1024(const SortedLaunch& L) { sorted_launch_nt<1024>(L); }
#else
#error "cvq_sorted_inst.hip needs CVQ_SORT_SLICE_384, _512 or _1024"
#endif

}  // namespace cvq
