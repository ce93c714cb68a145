// cvq_compact_inst.hip -- one slice of the COMPACT kernel's template instances
// (copula x model x node power), compiled once per CVQ_INST_* (Makefile), so the
// slices build in parallel.  The dispatch is launch_compact (cvq_compact.hip).
#define CVQ_NO_PLAN_KERNELS
#include "cvq_compact_launch.h"

namespace cvq {

// Student node power: PM = 8 is nu = 6 (b^-4, one rcp per node), PM = 0 the general pow
#if defined(CVQ_INST_st_msm_8)
void compact_slice_st_msm_8(const CompactLaunch& L) { launch_pm<CVQ_STUDENT, true, 8>(L); }
#elif defined(CVQ_INST_st_msm_0)
void compact_slice_st_msm_0(const CompactLaunch& L) { launch_pm<CVQ_STUDENT, true, 0>(L); }
#elif defined(CVQ_INST_st_gar_8)
void compact_slice_st_gar_8(const CompactLaunch& L) { launch_pm<CVQ_STUDENT, false, 8>(L); }
#elif defined(CVQ_INST_st_gar_0)
void compact_slice_st_gar_0(const CompactLaunch& L) { launch_pm<CVQ_STUDENT, false, 0>(L); }
#elif defined(CVQ_INST_ga_msm)
void compact_slice_ga_msm(const CompactLaunch& L) { launch_pm<CVQ_GAUSSIAN, true, 0>(L); }
#elif defined(CVQ_INST_ga_gar)
void compact_slice_ga_gar(const CompactLaunch& L) { launch_pm<CVQ_GAUSSIAN, false, 0>(L); }
#elif defined(CVQ_INST_pl_msm)
void compact_slice_pl_msm(const CompactLaunch& L) { launch_pm<CVQ_PLACKETT, true, 0>(L); }
#elif defined(CVQ_INST_pl_gar)
void compact_slice_pl_gar(const CompactLaunch& L) { launch_pm<CVQ_PLACKETT, false, 0>(L); }
#else
#error "cvq_compact_inst.hip needs one CVQ_INST_* definition"
#endif

}  // namespace cvq
