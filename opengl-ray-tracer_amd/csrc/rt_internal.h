// rt_internal.h — entry points shared between the library's own translation units
// (rt_kernels.hip, rt_group.hip); not part of the C ABI (include/rt_api.h).
#pragma once

#include <hip/hip_runtime.h>

struct rt_ctx;

namespace rtx {

// rt_create, ordered on `stream` from the start when it is not null (the caller
// keeps it; as rt_set_stream). rt_create itself makes the context's own stream.
// Creating a context straight on its final stream matters on AMD: HIP deals
// streams to the GPU_MAX_HW_QUEUES hardware queues as they are created, and a
// throw-away stream per context (rt_create, then rt_set_stream) skews that
// deal, so that frame slots end up sharing a queue and running in order.
int create_ctx(rt_ctx** out, int device, hipStream_t stream);

}  // namespace rtx
