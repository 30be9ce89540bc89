// pt_kernels_alt.h — host entry points of pt_kernels_alt.hip (the A/B traversal
// families) for the launchers of pt_kernels.hip.
#pragma once

#include "pt_kernels.h"
#include "pt_traverse.h"

namespace pupil {

// persistent grid of the traversal kernels: the resident capacity (pt_kernels.hip)
uint32_t trace4_blocks(const DeviceScene &sc, uint32_t ovf_threads);
// one persistent BVH8 launch (sc.bvh_width == 8); mode = tr::TraceMode, any = closest / any hit
void launch_trace8(int mode, bool any, const DeviceScene &sc, const PathState &ps, const Queues &q,
                   const tr::TraceJob &job, int *ovf, uint32_t ovf_threads, const TraceStats *stats, hipStream_t s);
// one-ray-per-lane grid-stride kernels (PUPIL_REFILL=0, or the BVH2 node format)
void launch_extend_lanes(const DeviceScene &sc, const PathState &ps, const Queues &q, const uint32_t *queue,
                         const uint32_t *queue_count, uint32_t static_count, int *ovf, uint32_t ovf_threads,
                         const TraceStats *stats, hipStream_t s);
void launch_shadow_lanes(const DeviceScene &sc, const PathState &ps, const Queues &q, int *ovf, uint32_t ovf_threads,
                         const TraceStats *stats, hipStream_t s);
void launch_trace_debug_lanes(const DeviceScene &sc, const float *rays, float *out, uint32_t n, int any, int *ovf,
                              uint32_t ovf_threads, hipStream_t s);

}  // namespace pupil
