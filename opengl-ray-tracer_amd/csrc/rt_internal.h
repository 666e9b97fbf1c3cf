// rt_internal.h — entry points shared between the library's own translation units
// (rt_kernels.hip, rt_group.hip); not part of the C ABI (include/rt_api.h).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/rt_flat.h"

struct rt_ctx;

namespace rtx {

// rt_create, ordered on `stream` from the start when it is not null (the caller
// keeps it; as rt_set_stream). rt_create itself makes the context's own stream.
// Creating a context straight on its final stream matters on AMD: HIP deals
// streams to the GPU_MAX_HW_QUEUES hardware queues as they are created, and a
// throw-away stream per context (rt_create, then rt_set_stream) skews that
// deal, so that frame slots end up sharing a queue and running in order.
int create_ctx(rt_ctx** out, int device, hipStream_t stream);

// A non-blocking stream of the current device. own_queue: created with a full CU
// mask (hipExtStreamCreateWithCUMask), which HIP backs with a hardware queue of
// its own instead of dealing it onto one of the GPU_MAX_HW_QUEUES shared queues
// (falls back to a plain stream if that fails). rt_group's frame slots take it:
// with shared queues two of a 1-rank group's three slots landed on one queue and
// ran in order (1080p car 0.216 ms per frame against 0.184 with own queues and
// 0.183 in frames mode; profiles/r04c_strong1_queues.txt). Contexts made by
// rt_create take it when RT_STREAMS_CUMASK=1 is set.
hipError_t make_stream(hipStream_t* s, bool own_queue);

// Whether the context renders with camera `cam` and a root box equal to [lo, hi]:
// its camera as last set, and the root box its next render sees (the host's node
// records, whatever rt_update_nodes left pending included, grown by every rt_animate
// as k_refit grows it). rt_group computes the sky-row band from the group's own camera
// and root box on every rank; a member changed behind the group's back would get
// background rows where it draws geometry.
bool matches_view(const rt_ctx* c, const FlatCamera& cam, const float lo[3], const float hi[3]);

// The root box of matches_view (false without a scene or nodes). After rt_group's
// update calls every slot context holds the same one, computed on the host by the
// same operations on every rank.
bool view_root(const rt_ctx* c, float lo[3], float hi[3]);

// rt_animate without the device work: the animated shapes' records and this frame's
// growth (the union of every deferred frame's growToInclude boxes, per shape) stay on the
// host until the context's next device operation, whose one refit applies them all
// (k_refit AF_BOX). rt_group's frame slots take every frame this way: a slot renders
// every F-th frame, and its refit then runs once per frame it renders, not once per frame.
// The nodes grow exactly as by one rt_animate per frame (min / max of the same boxes).
int animate_deferred(rt_ctx* c, const FlatShape* shapes);

}  // namespace rtx
