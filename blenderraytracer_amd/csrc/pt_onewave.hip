// pt_onewave.hip — the one-wave pool kernel (trace_pool_kernel) and the lane-per-pixel kernel
// (trace_kernel) in a translation unit of their own, so that build.py can compile them with LLVM's
// AMDGPU register-pressure trackers (pt_trace.hip, launch_onewave_pool).
#define RT_ONEWAVE_TU 1
#include "pt_trace.hip"
