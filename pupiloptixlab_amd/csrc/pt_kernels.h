// pt_kernels.h — host-visible declarations of the wavefront stages and the
// LBVH builder (implemented in pt_kernels.hip / bvh_build.hip).
#pragma once

#include <vector>

#include <hip/hip_runtime.h>

#include "pt_scene.h"

namespace pupil {

constexpr int kTraceBlock = 128;
// persistent BVH4 kernels: occupancy target (<= 72 VGPRs; 6 waves: 3 % slower, 8 waves at <= 64 VGPRs:
// 8-11 % slower, r03 / r05 A/B, profiles/r05_stack_ab.txt)
constexpr int kTraceWavesPerSimd = 7;
constexpr int kTraceWavesPerSimdTL = 5;  // two-level variant (<= 96 VGPRs; A/B r02 on config 5: 4 waves 688, 5: 743, 6: 716 Mrays/s)
constexpr int kStackOvf = 160;  // per-thread global overflow entries
constexpr int kRing = 16;       // persistent BVH4 kernels: per-lane LDS ring entries (spills to the overflow column)
// Wave-cooperative node fetch in k_trace4 (pt_traverse.h CoopFetch): 0 = each lane loads its own
// node (four 16-B loads per visit), 1 = the wave's distinct nodes are loaded a quarter per lane
// into a per-wave LDS image and read back from there
#ifndef PUPIL_COOP
#define PUPIL_COOP 0
#endif
constexpr bool kCoopFetch = PUPIL_COOP != 0;
// nodes one round of the cooperative fetch stages (16 per LDS-DMA wave-instruction)
#ifndef PUPIL_COOP_CHUNKS
#define PUPIL_COOP_CHUNKS 1
#endif
constexpr int kCoopChunks = PUPIL_COOP_CHUNKS;
// distance stack in k_trace4 (flat kernels): every LDS entry carries its entry distance and pops
// skip entries already beyond tmax (pt_traverse.h pop_live); the distances take a second LDS
// column, so it pairs with a smaller ring (PUPIL_TRACE_RING=8)
#ifndef PUPIL_DIST_STACK
#define PUPIL_DIST_STACK 0
#endif
constexpr bool kDistStack = PUPIL_DIST_STACK != 0;
// k_trace4's LDS ring: the cooperative fetch's staging (1 KiB + 256 B per wave and chunk) comes
// out of the ring so 14 blocks still fit a CU's 160 KiB
#ifndef PUPIL_TRACE_RING
#define PUPIL_TRACE_RING (PUPIL_COOP ? 13 : (PUPIL_DIST_STACK ? 8 : 16))
#endif
constexpr int kTraceRing = PUPIL_TRACE_RING;
static_assert(kTraceRing >= 8 && kTraceRing <= kRing, "trace ring");
// Stack entries a traversal may need: 3 per BVH4 level (4 children, one taken), plus
// 2 per instance entry in two-level mode.  Builds whose trees need more are rejected
// (or rebuilt with the depth-bounded Karras LBVH) at create time, so no kernel ever
// overwrites a live entry.
constexpr int kTraceStackEntries = kRing + kStackOvf;
// a smaller trace ring spills into a deeper overflow column: capacity >= kTraceStackEntries
constexpr int kTraceStackOvf = kStackOvf + (kRing - kTraceRing + 7) / 8 * 8;
constexpr int kShadeBlock = 256;
constexpr uint32_t kMaxDepth = 128;  // PTPass inspector range (pt_pass.cpp:225-237)
constexpr uint32_t kNumQueues = 9;  // 0 = miss, 1..7 = EMatType, 8 = unknown material
constexpr uint32_t kMissIndex = 0xFFFFFFFFu;

// Path state in HBM, structure of arrays indexed by path id
// p = sample * num_local_pixels + local_pixel.
struct PathState {
    float4 *ray_o;      // xyz origin of the current ray (and of its shadow ray: w = the shadow ray's tmax)
    float4 *ray_d;      // xyz direction
    float4 *hit;        // t, b1, b2, sorted primitive index (bits) or kMissIndex
    float4 *thr;        // xyz throughput, w = pdf of the BSDF sample that spawned the ray
    float4 *rad;        // xyz radiance
    uint4 *misc;        // x rng, y bounce (bits 0..23) | delta << 31, z/w texcoord (stale semantics, geometry.h:298-304)
    float4 *sh_d;       // shadow ray direction
    float4 *sh_c;       // pending NEE contribution
    uint8_t *mbin;      // extend -> material bin of the hit (0 miss, 1..7 EMatType, 8 unknown), 0xFF = not traced
    uint8_t *sflags;    // shade -> bit 0: extension ray spawned, bit 1: shadow ray spawned, bits 2..7: bounce tag
};

// Bounce tag of the shade flags byte: the flags partition after bounce b lists
// only bytes carrying tag(b), so the flags a path left when it died are never
// listed again and no per-bounce clear is needed.  Depths above 63 would alias
// the 6-bit tag: there the tag is 0 and the engine clears the bytes per bounce.
__host__ __device__ inline uint32_t sflag_tag(uint32_t max_depth, uint32_t bounce) {
    return max_depth <= 63u ? bounce % 63u + 1u : 0u;
}

// Queues are rebuilt by a stable partition (queue_partition.hip) after each
// stage, so every queue lists path ids in increasing order.
constexpr int kPartMaxBins = 9;
// counts[] slots
constexpr uint32_t kCntNext = 9, kCntShadow = 10;                      // queue lengths
// persistent-kernel work counters: per kind kWorkShards dequeue heads (one per
// XCD), one final exit counter and kWorkShards exit sub-counters, each on its
// own 128-B line.  Zero at allocation; the last wave of every persistent launch
// puts them back to zero.
constexpr uint32_t kWorkShards = 8, kWorkStride = 32, kWorkKind = (2 * kWorkShards + 1) * kWorkStride;
constexpr uint32_t kWorkExtend = 0, kWorkShadow = kWorkKind, kWorkRays = 2 * kWorkKind, kWorkFrame = 3 * kWorkKind;
constexpr uint32_t kWorkSlots = 4 * kWorkKind;
constexpr uint32_t kStartBins = 16;                                    // [16..24] material bin starts
constexpr uint32_t kStartNext = 25, kStartShadow = 26;                 // next / shadow regions of nxsh
constexpr uint32_t kScratch = 27;
constexpr uint32_t kCountSlots = 32;

struct Queues {
    uint32_t *bins;      // capacity: material bin b occupies [counts[kStartBins + b], + counts[b])
    uint32_t *nxsh;      // 2 * capacity: next ids from counts[kStartNext] (= 0), shadow ids from counts[kStartShadow]
    uint32_t *counts;    // kCountSlots entries, see above
    uint32_t *hist;      // partition scratch, partition_hist_entries(capacity)
    uint32_t *work;      // kWorkSlots persistent-kernel work heads (see kWorkExtend)
    uint32_t capacity;
};

// partition key modes (queue_partition.hip)
enum PartMode : int {
    kPartExclusive = 0,  // bin = key >> shift (0xFF = none)
    kPartFlags = 1,      // bin b <=> bit b of the key, if key >> 2 == tag (passed as `shift`)
};

struct FrameParams {
    uint32_t width, height;
    uint32_t num_local;    // local pixels
    uint32_t num_paths;    // num_local * spp
    uint32_t spp;
    uint32_t seed0;
    uint32_t cnt0;
    uint32_t accumulate;
    uint32_t max_depth;
    uint32_t compact;
    const uint32_t *pixel_map;  // local -> global pixel (null = identity)
    float4 *accum;
    float4 *frame;
    float *albedo;  // 3 floats per pixel
    float *normal;
    float *test;
    unsigned long long *nee_count;  // collect_stats: paths that reached the shadow test (main.cu:113-123)
    // shade: the AOV pointers above are indexed by the local pixel (compact output, or the
    // per-slot AOV scratch of a frame that completes in a later render); else by y*w+x
    uint32_t aov_local;
    // pipelined frame groups (engine.hip render_pipelined): a ring slot holds `group` frames of
    // spp samples; frame f of a slot writes its AOVs at + f * aov_frame_stride floats (0: one
    // frame per slot, or the render's own buffers)
    uint32_t group;
    uint32_t aov_frame_stride;
};

// Path-state records are streamed with non-temporal loads / stores (r03), so the GBs of path state a step moves do not push BVH nodes and primitive records out of
// the L2s and the Infinity Cache.
__device__ __forceinline__ float4 ld_ps(const float4 *a) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f v = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(a));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 ld_ps(const uint4 *a) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a));
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_ps(float4 *a, float4 v) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4f *>(a));
}
__device__ __forceinline__ void st_ps(uint4 *a, uint4 v) {
    typedef unsigned v4u __attribute__((ext_vector_type(4)));
    v4u w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(a));
}

// The instance holding global primitive `idx`: the last instance i in the guide's range with
// inst_first[i] <= idx (an instance without primitives shares its first id with the next one,
// which is the one that holds it), i.e. exactly prim_inst[idx].
#ifndef PUPIL_INST_GUIDE
#define PUPIL_INST_GUIDE 1
#endif
__device__ __forceinline__ uint32_t inst_of_prim(const DeviceScene &sc, uint32_t idx) {
    if (!PUPIL_INST_GUIDE) return sc.prim_inst[idx];
    const uint32_t k = idx >> sc.inst_guide_shift;
    uint32_t lo = sc.inst_guide[k], hi = sc.inst_guide[k + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (sc.inst_first[mid] <= idx) lo = mid;
        else hi = mid - 1u;
    }
    return lo;
}

struct TraceStats {
    unsigned long long *counters;  // [0..1] closest-hit nodes/prims, [14..15] shadow, [2..13] diagnostics,
                                   // [16] reference shadow rays, [18] distinct node fetches,
                                   // [20..23] queue accounting (handed, activated, retired, listed)
    // PUPIL_TRACE_TAIL diagnostics (STATS kernels only, else null): per wave of the
    // persistent launch, s_memrealtime (100 MHz) at start, when its dequeue found
    // the work list drained, at exit, and the rays it took
    unsigned long long *wave_times = nullptr;
};

// wavefront stages
// full = false: only the camera rays (the list shade then treats the batch as fresh paths)
void launch_generate(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, hipStream_t s, bool full);
// interleave_spp / num_local (primary extend, queue == null): dequeue the spp samples of
// a pixel on consecutive lanes (TraceJob::spp); 0 = path order
void launch_extend(const DeviceScene &sc, const PathState &ps, const Queues &q, const uint32_t *queue,
                   const uint32_t *queue_count, uint32_t static_count, int *ovf, uint32_t ovf_threads,
                   const TraceStats *stats, hipStream_t s, uint32_t interleave_spp = 0, uint32_t num_local = 0);
// which paths a shade launch walks: the material-bin partition (q.bins), a range of path
// ids (every path of a batch after its primary extend), the previous bounce's next list
// (q.nxsh), or that next list followed by a range (pipelined frames: the extension rays of
// the frames in flight, then the camera rays of the frame started in the same launch).
// Each path's bounce is read from its state (PathState::misc.y), so one launch may shade
// paths of several frames at different bounces; `tag` is the bounce tag the launch writes
// into the flags bytes (sflag_tag, or the pipeline's generation tag).
// fresh_range (list modes): the range is a batch whose k_generate stored only its camera rays
// (full = false), first frame seed fresh_seed0; its bounce-0 shade derives throughput 1,
// radiance 0 and the camera RNG instead of reading them.
enum ShadeList : int { kShadeBins = 0, kShadeAll = 1, kShadeNext = 2, kShadeNextRange = 3 };
void launch_shade(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, const Queues &q, uint32_t tag,
                  hipStream_t s, ShadeList list, uint32_t range_base, uint32_t range_n, uint32_t max_count,
                  bool fresh_range = false, uint32_t fresh_seed0 = 0);
// one persistent launch over the next + shadow lists of a bounce (BVH4 persistent path only)
// ahead_count > 0 (render-ahead, BVH4 kernels only): the launch also traces the camera
// rays of the next render.  `ps` is then the base of both buffer halves: this render's
// listed paths are at list_base + id, the next render's camera rays (generated there)
// at ahead_base + [0, ahead_count), dequeued pixel-major when ahead_spp > 1 (as the
// primary extend)
void launch_trace_mixed(const DeviceScene &sc, const PathState &ps, const Queues &q, int *ovf, uint32_t ovf_threads,
                        const TraceStats *stats, hipStream_t s, uint32_t ahead_count = 0, uint32_t list_base = 0,
                        uint32_t ahead_base = 0, uint32_t ahead_spp = 0, uint32_t ahead_local = 0);
// small frames (pt_frame.hip): every path of the frame -- camera ray, bounces, shadow rays --
// in one persistent launch (no partitions, one drain); the accumulate follows.  Flat BVH4 and
// two-level world mode only.  ray_cum: running totals of extension [0] and shadow [1] rays.
bool frame_kernel_supported(const DeviceScene &sc);
void launch_frame(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, uint32_t *work,
                  unsigned long long *ray_cum, int *ovf, uint32_t ovf_threads, uint32_t interleave_spp, hipStream_t s);
// running mean of the batch's frames into fp.accum / fp.frame; aov_src (or null): the
// frame's AOVs from the slot scratch (3n albedo, 3n normal, n test floats) copied to the
// outputs; clear_flags: zero the frame's flags bytes (its ring slot is free again)
// per axis max of |o| + 512 s over n BVH4 nodes into out[0..2] (float bits; clear: out is
// zeroed first, else the max also covers what it holds), the bound DeviceScene::node_bound holds
void launch_node_bound(const Bvh4Node *nodes, uint64_t n, uint32_t *out, hipStream_t s, bool clear = true);
void launch_accumulate(const FrameParams &fp, const PathState &ps, const float *aov_src, bool clear_flags,
                       hipStream_t s);
uint32_t trace_grid_blocks();
// stats (or null): the persistent kernels' counter variants (queue accounting, node visits)
void launch_trace_debug(const DeviceScene &sc, const float *rays, float *out, uint32_t n, int any, int *ovf,
                        uint32_t ovf_threads, uint32_t *work, hipStream_t s, const TraceStats *stats = nullptr);
void launch_debug_math(const float *x, const float *y2, float *out, uint32_t n, hipStream_t s);
// device emitter selection for n random numbers: area index, -1 env, -2 none
void launch_debug_select(const DeviceScene &sc, const float *p, int *out, uint32_t n, hipStream_t s);

// stable partition of path ids 0..n-1 by a key byte (queue_partition.hip)
uint32_t partition_hist_entries(uint32_t n);
// log_out (or null): the nbins counts; cum_out (or null): the counts are added to these
// nbins running 64-bit totals (rays traced since the engine was created); snap_out (or
// null): receives the totals as they were before this partition added to them; bin_mask (or 0 =
// every bin below nbins): the bins a key can name -- the others are reported empty without being
// ranked (the material partition of a scene with few materials)
void launch_partition(const uint8_t *keys, uint32_t n, uint32_t nbins, PartMode mode, uint32_t shift, uint32_t *out,
                      uint32_t *hist, uint32_t *counts_out, uint32_t *starts_out, uint32_t *total_out, uint32_t *log_out,
                      hipStream_t s, unsigned long long *cum_out = nullptr, unsigned long long *snap_out = nullptr,
                      uint32_t bin_mask = 0u);

// LBVH builder (bvh_build.hip)
struct BvhBuildInput {
    uint32_t num_prims;
    const uint32_t *prim_inst;      // device, global prim -> instance
    const DevInstance *instances;   // device
    const DevMaterial *materials;   // device
    uint32_t object_space;          // 1: BLAS build (vertices untransformed, shading records in primitive order)
};
struct BvhBuildOutput {
    Bvh4Node *nodes4;   // device, collapsed 4-wide quantized tree
    float4 *prims;      // device, kRecF4 * num_records (record slots, pt_scene.h)
    float4 *attrs;      // device, kAttrStride * n shading records (same order)
    uint32_t root_link4;      // link of the root (internal 0 or a leaf)
    uint32_t num_nodes4;
    uint32_t depth4;    // levels of the BVH4 (1 = root only); 0 = not measured (A/B collapse)
    uint32_t num_records = 0; // record slots (leaves on even slots; holes between)
    // first node of each BVH4 level (breadth-first collapse order) and the end; empty when
    // not measured.  Children always lie on a later level (bottom-up refits walk it backwards).
    std::vector<uint32_t> level_start;
};
int build_lbvh(const BvhBuildInput &in, BvhBuildOutput &out, uint32_t leaf_size, hipStream_t s, double *build_ms,
               bool force_lbvh = false);
// build_lbvh whose BVH4 fits the traversal stacks with `reserve` entries to spare:
// PLOC first, the Karras LBVH (depth bounded by the 30-bit Morton codes) when the
// PLOC tree is too deep.  Returns 0, -2 on a HIP error, -3 when no tree fits.
int build_bvh_bounded(const BvhBuildInput &in, BvhBuildOutput &out, uint32_t leaf_size, hipStream_t s,
                      double *build_ms, uint32_t reserve);
void free_lbvh(BvhBuildOutput &out);
// RenderInstanceUpdate without a rebuild: the records of the instances flagged in
// `moved` (device, one byte per instance) get their new world vertices and every BVH4 node
// box is refitted bottom up (topology kept, like the reference's IAS update); nbox: device
// scratch of 6 floats per node.  Needs the breadth-first level order; -1 when unavailable.
int refit_bvh4(const BvhBuildInput &in, BvhBuildOutput &out, const uint8_t *moved, float *nbox, hipStream_t s,
               double *ms);
// BVH4 over n >= 2 boxes (6 floats each: lo xyz, hi xyz) with the flattened build's PLOC +
// SAH collapse, one box per leaf: nodes (root 0, parents first) and, for leaf link
// make_leaf(p, 1), the box order[p]; depth = 4-wide levels
int build_bvh4_over_boxes(const float *h_boxes, uint32_t n, std::vector<Bvh4Node> &nodes,
                          std::vector<uint32_t> &order, uint32_t *depth, hipStream_t s);

}  // namespace pupil
