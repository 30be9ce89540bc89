// pt_kernels.hip — the wavefront path tracer on gfx950.
//
// One frame batch = `spp` consecutive frames of PTPass::OnRun
// (example/path_tracer/pt_pass.cpp:39-57) over the rank's pixels.  The
// reference's per-pixel megakernel (__raygen__main, main.cu:36-194) is cut at
// every optixTrace into stages that each run over a compacted queue:
//
//   generate  (main.cu:44-75)   camera ray + RNG init for every path
//   extend    (main.cu:77,158)  closest hit; bins the path by material type
//   shade<M>  (main.cu:84-183)  one kernel per EMatType: hit reconstruction,
//                               emission/MIS, RR, NEE sample + BSDF eval,
//                               BSDF sample -> shadow queue + next queue
//   shadow    (main.cu:119-140) any hit; adds the pending NEE contribution
//   accumulate(main.cu:185-193) running-mean over the batch's frames, in order
//
// Every float operation of the reference is reproduced in the same order, so
// a path gives bit-identical radiance to the reference-order CPU oracle.
#include "pt_kernels.h"
#include "pt_shade.h"
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

#include <cstdlib>
#include <algorithm>

namespace pupil {

namespace {

using namespace tr;

// full = 0 (list shading, PUPIL_FRESH_SHADE): only the camera ray is stored; the bounce-0
// shade of the fresh paths takes throughput 1, radiance 0 and the RNG from fresh_path
// instead of reading them (k_shade_all `fresh`).
__global__ __launch_bounds__(kShadeBlock) void k_generate(DeviceScene sc, FrameParams fp, PathState ps, uint32_t full) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= fp.num_paths) return;
    vec3 dir;
    const uint32_t rng = fresh_path(sc, fp, p, fp.seed0, dir);
    st_ps(ps.ray_d + p, make_float4(dir.x, dir.y, dir.z, 0.f));
    // a camera ray's origin is the camera's: the traversal and a fresh path's shade take it from
    // the scene (camera_origin), so only full records, read by stages that cannot tell, store it
    if (!full) return;
    st_ps(ps.ray_o + p, f4(camera_origin(sc.camera), 0.f));
    st_ps(ps.thr + p, make_float4(1.f, 1.f, 1.f, 0.f));
    st_ps(ps.rad + p, make_float4(0.f, 0.f, 0.f, 0.f));
    st_ps(ps.misc + p, make_uint4(rng, 0u, 0u, 0u));
}

// ------------------------------------------------------------------ shade
// All shading of a bounce in one launch (4 waves per SIMD: <= 128 VGPRs).  The material bins lie back to back in
// q.bins (bin 0 = miss, 1..7 = EMatType, 8 = unknown type), each in increasing
// path order, so a wave sees one material except at the 8 bin boundaries; the
// branch below is wave-uniform almost everywhere.  One launch instead of nine
// per bounce keeps empty-bin launches off the frame (they cost ~4 us each).
// SHADE_LIST (single-material scenes, ShadeList): no material partition; the launch
// walks the paths the last traversal traced -- a range of path ids after a primary
// extend, the previous bounce's next list, or both (pipelined frames) -- in increasing
// path order, and takes each path's bin from the hit (or the byte the traversal wrote).
// Only the miss / hit split diverges inside a wave, which costs less than the three
// partition launches.  Each path's bounce comes from its own state, so the paths of
// several frames in flight (pipelined renders, engine.hip) share one launch.
template <int LIST>
__global__ __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(4))) void k_shade_all(DeviceScene sc, FrameParams fp, PathState ps, Queues q,
                                                           uint32_t tag, uint32_t range_base, uint32_t range_n,
                                                           uint32_t fresh_range, uint32_t fresh_seed0) {
    const uint32_t n_list = LIST == kShadeNext || LIST == kShadeNextRange ? q.counts[kCntNext] : 0u;
    const uint32_t count = LIST == kShadeBins ? q.counts[kScratch]  // all traced paths (total of the bin partition)
                                              : n_list + (LIST == kShadeAll || LIST == kShadeNextRange ? range_n : 0u);
    uint32_t start[kPartMaxBins];
#pragma unroll
    for (int b = 0; b < kPartMaxBins; b++) start[b] = LIST == kShadeBins ? q.counts[kStartBins + b] : 0u;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const uint32_t p = LIST == kShadeBins ? q.bins[i] : (i < n_list ? q.nxsh[i] : range_base + (i - n_list));
        // bin of list position i: the last bin starting at or before i (an empty
        // bin starts where the next one does, so it is never the last such bin)
        uint32_t bin = 0;
        if (LIST == kShadeBins) {
#pragma unroll
            for (int b = 1; b < kPartMaxBins; b++) bin = i >= start[b] ? (uint32_t)b : bin;
        } else if (sc.single_bin) {  // the traversal wrote no bin byte (DeviceScene::single_bin)
            bin = __float_as_uint(ld_ps(ps.hit + p).w) == kMissIndex ? 0u : sc.single_bin;
        } else {
            bin = ps.mbin[p];
        }
        // the range part of a list launch is a fresh frame; with fresh_range its paths'
        // throughput, radiance and RNG were never stored (k_generate full = 0)
        const bool fresh = LIST != kShadeBins && fresh_range && i >= n_list;
        const uint32_t fresh_p = p - range_base;
        uint32_t flags = 0;
        switch (bin) {
        case 0: shade_miss(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        case PUPIL_MAT_DIFFUSE: flags = shade_hit<PUPIL_MAT_DIFFUSE>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        case PUPIL_MAT_DIELECTRIC: flags = shade_hit<PUPIL_MAT_DIELECTRIC>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        case PUPIL_MAT_ROUGH_DIELECTRIC:
            flags = shade_hit<PUPIL_MAT_ROUGH_DIELECTRIC>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0);
            break;
        case PUPIL_MAT_CONDUCTOR: flags = shade_hit<PUPIL_MAT_CONDUCTOR>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        case PUPIL_MAT_ROUGH_CONDUCTOR:
            flags = shade_hit<PUPIL_MAT_ROUGH_CONDUCTOR>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0);
            break;
        case PUPIL_MAT_PLASTIC: flags = shade_hit<PUPIL_MAT_PLASTIC>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        case PUPIL_MAT_ROUGH_PLASTIC: flags = shade_hit<PUPIL_MAT_ROUGH_PLASTIC>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        default: flags = shade_hit<0u>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0); break;
        }
        if (fp.nee_count) {  // collect_stats only: the reference's shadow-ray count, one atomic per wave
            const unsigned long long m = __ballot((flags & 4u) != 0u);
            if (m && __lane_id() == __ffsll((unsigned long long)__builtin_amdgcn_read_exec()) - 1)
                atomicAdd(fp.nee_count, (unsigned long long)__popcll(m));
        }
        ps.sflags[p] = (uint8_t)((flags & 3u) | tag << 2);
        if (LIST == kShadeBins) ps.mbin[p] = 0xFFu;  // listed again only if the next extend traces this path
    }
}

// Single-material scenes (DeviceScene::single_bin, list modes): the same launch with only the
// miss path and material MAT compiled, so the register budget is that material's, not the
// largest of the seven BSDFs' (126 VGPRs, 4 waves per SIMD): diffuse needs 101-105 and runs at
// 5 waves (96 VGPRs, 7-10 spills; config 4 -2.8 % per step, profiles/r04_shade_one_ab.txt);
// the other BSDFs spill 15-43 registers at 5 waves and stay at 4 (A/B: PUPIL_SHADE_ONE=0).
constexpr int shade_one_waves(uint32_t mat) { return mat == PUPIL_MAT_DIFFUSE ? 5 : 4; }
template <int LIST, uint32_t MAT>
__global__ __launch_bounds__(kShadeBlock) __attribute__((amdgpu_waves_per_eu(shade_one_waves(MAT)))) void k_shade_one(
    DeviceScene sc, FrameParams fp, PathState ps, Queues q, uint32_t tag, uint32_t range_base, uint32_t range_n,
    uint32_t fresh_range, uint32_t fresh_seed0) {
    static_assert(LIST != kShadeBins, "single-material shading walks a list");
    const uint32_t n_list = LIST == kShadeNext || LIST == kShadeNextRange ? q.counts[kCntNext] : 0u;
    const uint32_t count = n_list + (LIST == kShadeAll || LIST == kShadeNextRange ? range_n : 0u);
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        const uint32_t p = i < n_list ? q.nxsh[i] : range_base + (i - n_list);
        const bool miss = __float_as_uint(ld_ps(ps.hit + p).w) == kMissIndex;
        const bool fresh = fresh_range && i >= n_list;
        const uint32_t fresh_p = p - range_base;
        uint32_t flags = 0;
        if (miss) shade_miss(sc, fp, ps, p, fresh, fresh_p, fresh_seed0);
        else flags = shade_hit<MAT>(sc, fp, ps, p, fresh, fresh_p, fresh_seed0);
        if (fp.nee_count) {
            const unsigned long long m = __ballot((flags & 4u) != 0u);
            if (m && __lane_id() == __ffsll((unsigned long long)__builtin_amdgcn_read_exec()) - 1)
                atomicAdd(fp.nee_count, (unsigned long long)__popcll(m));
        }
        ps.sflags[p] = (uint8_t)((flags & 3u) | tag << 2);
    }
}

// ------------------------------------------------------------------ accumulate
__global__ __launch_bounds__(kShadeBlock) void k_accumulate(FrameParams fp, PathState ps, const float *aov_src,
                                                             uint32_t clear_flags) {
    const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
    if (l >= fp.num_local) return;
    const uint32_t out = fp.compact ? l : global_pixel(fp, l);
    if (aov_src) {  // the frame's AOVs, shaded in an earlier render (pipelined frames)
        const uint32_t n = fp.num_local;
        if (fp.albedo)
            for (int k = 0; k < 3; k++) fp.albedo[3 * out + k] = aov_src[3 * l + k];
        if (fp.normal)
            for (int k = 0; k < 3; k++) fp.normal[3 * out + k] = aov_src[3 * n + 3 * l + k];
        if (fp.test) fp.test[out] = aov_src[6 * n + l];
    }
    vec3 acc = f3(fp.accum[out]);
    // the samples' radiance 8 at a time: their loads issued together (one memory latency per
    // batch, not per sample); the lerps run in sample order as before
    constexpr uint32_t kBatch = 8;
    for (uint32_t s0 = 0; s0 < fp.spp; s0 += kBatch) {
        float4 rad[kBatch];
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++)
            if (s0 + j < fp.spp) rad[j] = ps.rad[(size_t)(s0 + j) * fp.num_local + l];
#pragma unroll
        for (uint32_t j = 0; j < kBatch; j++) {
            const uint32_t s = s0 + j;
            if (s >= fp.spp) break;
            if (clear_flags) ps.sflags[(size_t)s * fp.num_local + l] = 0u;
            vec3 L = f3(rad[j]);
            const uint32_t cnt = fp.cnt0 + (fp.accumulate ? s : 0u);
            if (fp.accumulate && cnt > 0) {  // main.cu:187-191
                const float t = 1.f / ((float)cnt + 1.f);
                L = lerp(acc, L, t);
            }
            acc = L;
        }
    }
    fp.accum[out] = f4(acc, 1.f);
    if (fp.frame) fp.frame[out] = f4(acc, 1.f);
}


__global__ void k_debug_math(const float *x, const float *y2, float *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float a = x[i], b = y2[i];
    float s, c;
    dm_sincos(a, s, c);
    out[6 * i + 0] = s;
    out[6 * i + 1] = c;
    out[6 * i + 2] = dm_acos(fminf(fmaxf(a, -1.f), 1.f));
    out[6 * i + 3] = dm_atan2(a, b);
    out[6 * i + 4] = sqrtf(fabs_(a));
    out[6 * i + 5] = 1.0f / a;
}

}  // namespace


__global__ void k_debug_select(DeviceScene sc, const float *p, int *out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float prob;
    const DevEmitter *e = select_emitter(sc, p[i], prob);
    out[i] = !e ? -2 : (e == sc.env && sc.has_env ? -1 : (int)(e - sc.areas));
}

void launch_debug_select(const DeviceScene &sc, const float *p, int *out, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_select, dim3((n + 255) / 256), dim3(256), 0, s, sc, p, out, n);
}

void launch_debug_math(const float *x, const float *y2, float *out, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_debug_math, dim3((n + 255) / 256), dim3(256), 0, s, x, y2, out, n);
}

// ------------------------------------------------------------------ launchers

void launch_generate(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, hipStream_t s, bool full) {
    const uint32_t blocks = (fp.num_paths + kShadeBlock - 1) / kShadeBlock;
    hipLaunchKernelGGL(k_generate, dim3(blocks), dim3(kShadeBlock), 0, s, sc, fp, ps, full ? 1u : 0u);
}


// Shade launch size: one thread per path of the batch (fp.num_paths bounds the
// traced count, which only the device knows), so the hardware dispatcher
// balances the waves instead of a grid-stride loop over a fixed grid (A/B at
// config 4: 3.75 vs 4.05 ms of shading per frame with 2048 blocks = twice the
// resident waves).  PUPIL_SHADE_BLOCKS overrides it (A/B knob).
static uint32_t shade_blocks(uint32_t num_paths) {
    static const int forced = [] {
        const char *e = std::getenv("PUPIL_SHADE_BLOCKS");
        return e ? std::min(1 << 20, std::max(64, std::atoi(e))) : 0;
    }();
    if (forced) return (uint32_t)forced;
    return std::max(64u, std::min(1u << 20, (num_paths + kShadeBlock - 1) / kShadeBlock));
}

// max_count: host bound on the paths the launch may list (the device knows the count)
void launch_shade(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, const Queues &q, uint32_t tag,
                  hipStream_t s, ShadeList list, uint32_t range_base, uint32_t range_n, uint32_t max_count,
                  bool fresh_range, uint32_t fresh_seed0) {
    const dim3 g(shade_blocks(max_count)), b(kShadeBlock);
    const uint32_t fr = fresh_range && list != kShadeBins ? 1u : 0u;
#define SHADE(L) \
    hipLaunchKernelGGL(k_shade_all<L>, g, b, 0, s, sc, fp, ps, q, tag, range_base, range_n, fr, fresh_seed0)
#define SHADE1(L, M) \
    hipLaunchKernelGGL((k_shade_one<L, M>), g, b, 0, s, sc, fp, ps, q, tag, range_base, range_n, fr, fresh_seed0)
#define SHADE1_ALL(L)                                                       \
    switch (sc.single_bin) {                                                \
    case PUPIL_MAT_DIFFUSE: SHADE1(L, PUPIL_MAT_DIFFUSE); break;             \
    case PUPIL_MAT_DIELECTRIC: SHADE1(L, PUPIL_MAT_DIELECTRIC); break;       \
    case PUPIL_MAT_ROUGH_DIELECTRIC: SHADE1(L, PUPIL_MAT_ROUGH_DIELECTRIC); break; \
    case PUPIL_MAT_CONDUCTOR: SHADE1(L, PUPIL_MAT_CONDUCTOR); break;         \
    case PUPIL_MAT_ROUGH_CONDUCTOR: SHADE1(L, PUPIL_MAT_ROUGH_CONDUCTOR); break; \
    case PUPIL_MAT_PLASTIC: SHADE1(L, PUPIL_MAT_PLASTIC); break;             \
    case PUPIL_MAT_ROUGH_PLASTIC: SHADE1(L, PUPIL_MAT_ROUGH_PLASTIC); break; \
    default: SHADE1(L, 0u); break;                                          \
    }
    static const bool one = [] {
        const char *e = std::getenv("PUPIL_SHADE_ONE");
        return !e || std::atoi(e) != 0;
    }();
    if (one && sc.single_bin && list != kShadeBins) {
        switch (list) {
        case kShadeAll: SHADE1_ALL(kShadeAll); break;
        case kShadeNext: SHADE1_ALL(kShadeNext); break;
        default: SHADE1_ALL(kShadeNextRange); break;
        }
        return;
    }
    switch (list) {
    case kShadeAll: SHADE(kShadeAll); break;
    case kShadeNext: SHADE(kShadeNext); break;
    case kShadeNextRange: SHADE(kShadeNextRange); break;
    default: SHADE(kShadeBins); break;
    }
#undef SHADE
#undef SHADE1
#undef SHADE1_ALL
}


void launch_accumulate(const FrameParams &fp, const PathState &ps, const float *aov_src, bool clear_flags,
                       hipStream_t s) {
    const uint32_t blocks = (fp.num_local + kShadeBlock - 1) / kShadeBlock;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(kShadeBlock), 0, s, fp, ps, aov_src, clear_flags ? 1u : 0u);
}

}  // namespace pupil
