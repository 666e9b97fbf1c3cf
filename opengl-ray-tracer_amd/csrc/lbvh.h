// lbvh.h — opt-in device BVH build (lbvh.hip), called by rt_build_lbvh.
#pragma once

#include "../../include/rt_flat.h"

namespace rtl {

// Builds a linear BVH over the n device-resident shapes into nodes[2n-1]
// (root at 2n-2, one shape per leaf) and indices[n], on `stream` (a
// hipStream_t). Waits for completion; *ms = device time of the build.
// Returns 0, or a negative code on a HIP failure.
int lbvh_build(const FlatShape* shapes, int n, FlatNode* nodes, int* indices, void* stream, float* ms);

}  // namespace rtl
