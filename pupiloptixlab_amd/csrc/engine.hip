// engine.hip — host side of the HIP path tracer and the C ABI (include/pupil_pt.h).
//
// pupil_pt_create  = PTPass::SetScene + World::GetIASHandle + SBT build
//                    (example/path_tracer/pt_pass.cpp:107-209): scene arrays are
//                    copied to engine-owned HBM, materials get the host
//                    precompute of optix_material.cpp:87-119, the LBVH replaces
//                    the GAS/IAS.
// pupil_pt_render  = spp x PTPass::OnRun (pt_pass.cpp:39-57) as one wavefront batch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pupil_pt.h"
#include "accel_two_level.h"
#include "pt_kernels.h"

namespace {

thread_local std::string g_last_error;

// most event pairs pending at once: a PUPIL_STATS_TRACE_TIMING sequence that is never
// read folds its pairs into sums at this count, a deep timed render stops recording
constexpr uint32_t kMaxPairs = 4096;

int fail(int code, const std::string &msg) {
    g_last_error = msg;
    return code;
}

#define HIP_TRY(expr)                                                                                     \
    do {                                                                                                  \
        hipError_t _e = (expr);                                                                           \
        if (_e != hipSuccess)                                                                             \
            return fail(_e == hipErrorOutOfMemory ? PUPIL_ERR_OOM : PUPIL_ERR_HIP,                        \
                        std::string(#expr) + ": " + hipGetErrorString(_e));                               \
    } while (0)

using namespace pupil;

// fresnel::DiffuseReflectance (render/material/fresnel.h:67-94)
float diffuse_reflectance(float eta) {
    if (eta < 1) {
        return -1.4399f * (eta * eta) + 0.7099f * eta + 0.6681f + 0.0636f / eta;
    }
    const float inv_eta = 1.0f / eta;
    const float inv_eta2 = inv_eta * inv_eta;
    const float inv_eta3 = inv_eta2 * inv_eta;
    const float inv_eta4 = inv_eta3 * inv_eta;
    const float inv_eta5 = inv_eta4 * inv_eta;
    return 0.919317f - 3.4793f * inv_eta + 6.75335f * inv_eta2 - 7.80989f * inv_eta3 + 4.98554f * inv_eta4 -
           1.36881f * inv_eta5;
}

// GetPixelAverage (optix_material.cpp:15-42)
vec3 pixel_average(const pupil_texture &t) {
    if (t.type == PUPIL_TEX_RGB) return v3(t.c0[0], t.c0[1], t.c0[2]);
    if (t.type == PUPIL_TEX_CHECKERBOARD) {
        const float r = t.c0[0] + t.c1[0];
        const float g = t.c0[1] + t.c1[1];
        const float b = t.c0[2] + t.c1[2];
        return v3(r, g, b) * 0.5f;
    }
    if (t.type == PUPIL_TEX_BITMAP && t.rgba && t.width && t.height) {
        float r = 0.f, g = 0.f, b = 0.f;
        for (size_t i = 0, idx = 0; i < t.height; ++i)
            for (size_t j = 0; j < t.width; ++j) {
                r += t.rgba[idx++];
                g += t.rgba[idx++];
                b += t.rgba[idx++];
                idx++;
            }
        return v3(r, g, b) / (1.f * (float)t.height * (float)t.width);
    }
    return v3(0.f);
}

}  // namespace

namespace Pupil {
void set_last_error(const std::string &m) { g_last_error = m; }
}  // namespace Pupil

struct pupil_pt {
    int device = 0;
    hipStream_t own_stream = nullptr;
    DeviceScene sc{};
    std::vector<void *> allocs;
    BvhBuildOutput bvh{};
    bool two_level = false;  // TLAS + per-shape BLAS (accel_two_level.hip) instead of one flattened BVH
    bool primary_interleave = true;  // primary extend dequeues pixel-major (PUPIL_PRIMARY_ORDER)
    bool shade_list = false;  // shade walks the traced list instead of a material partition (PUPIL_SHADE_LIST)
    // list shading: a fresh batch's generate stores only its camera rays, and its bounce-0 shade
    // derives throughput, radiance and RNG (PUPIL_FRESH_SHADE=0: generate stores them all)
    bool fresh_shade = true;
    bool fresh() const { return fresh_shade && shade_list; }
    TwoLevelAccel tl{};
    uint32_t width = 0, height = 0, max_depth = 1;
    uint32_t num_prims = 0;
    uint32_t leaf_size = 2;  // primitives per BVH leaf (PUPIL_LEAF_SIZE)
    // Pipelined frames (render_pipelined, PUPIL_PIPE): the path state is a ring of K
    // slots of one batch each; consecutive renders that continue each other (OnRun
    // cadence, or PUPIL_HINT_CONTINUE) keep up to K frames in flight, each at its own
    // bounce, and every iteration of a render advances all of them by one bounce in ONE
    // persistent traversal launch and ONE shade launch.  A render returns with its own
    // frame complete; the frames ahead of it depend only on (seed, camera, scene) and
    // are dropped on any change.  ahead_mode: 1 = single-spp renders or the hint,
    // 2 = every render, 0 = off (PUPIL_AHEAD).
    int ahead_mode = 1;
    // a group of `frames` consecutive frames (seeds seed, seed + spp, ...) in one ring slot
    struct PipeFrame {
        uint32_t slot, seed, phases;  // phases = bounces traced + shaded so far (complete at max_depth)
        bool aov_scratch;             // AOVs wait in the slot's scratch until each frame's render
        uint32_t frames, consumed;    // frames in the group; accumulated (rendered) so far
    };
    std::vector<PipeFrame> pipe;      // in flight, oldest first
    // an iteration split over two renders (frame-group pacing, render_pipelined): the trace half
    // ran, the shade half is due at the start of the next render
    struct HalfIter {
        bool had, inject;
        PipeFrame nf;
        uint32_t nfp;
    };
    HalfIter half{};
    bool half_pending = false;
    bool pipe_split = true;           // PUPIL_PIPE_SPLIT=0: whole iterations only (A/B)
    // PUPIL_PIPE_GROUP_MAX: frames per group at most.  The latency bound is the group's paths
    // (PUPIL_PIPE_GROUP_PATHS, 4 M: two 1080p frames), so the heaviest OnRun carries the same
    // work at any tile share (profiles/r06_shard_probe_onrun.txt); 2 caps it at N = 1 sizes too
    uint32_t pipe_group_max = 64;
    uint32_t pipe_ramp = 1;           // PUPIL_PIPE_RAMP: groups one render may start ahead (0 = no limit)
    uint32_t pipe_slots = 0;          // K of the ring in use
    size_t pipe_np = 0;               // paths per slot
    uint32_t pipe_key[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // w, h, tile size, rank, world, spp, depth, local pixels, G
    size_t pipe_cap = 0;              // paths per ring slot (G frames)
    // PUPIL_PIPE_GROUP_PATHS: renders of fewer paths batch G = ceil(this / paths) frames per slot
    double pipe_group_paths = 4e6;
    // renders that start no frame ahead (a moving camera) with at most this many paths run as one
    // persistent launch per frame (pt_frame.hip); PUPIL_FRAME_PATHS, 0 = never.  Moving-camera
    // OnRuns at 1080p (r05 shard probe): one rank of 8 (260 k paths) 7.40 vs 8.47 ms per 8 OnRuns
    // in one launch vs the stage pipeline, one of 4 (518 k) 12.86 vs 10.56, one GPU 39.7 vs 22.8
    double frame_paths = 4e5;
    bool ring_fresh = true;           // the ring was (re)allocated: its flags bytes are not yet cleared
    uint32_t bin_mask = 0;            // material bins of the scene's instances + the miss bin (partition)
    uint32_t pipe_run = 0;            // consecutive renders that continued the previous one
    uint64_t frame_launches = 0;      // renders run as one persistent launch (pt_frame.hip)
    uint32_t pipe_next_seed = 0;      // random_seed of the render that would continue the last one
    uint32_t pipe_gen = 0;            // iterations so far (flags tags)
    uint32_t pipe_limit = 0;          // PUPIL_PIPE: most slots (0 = max_depth)
    // PUPIL_PIPE_GB: most HBM bytes for the ring's path state; default a quarter of the
    // device memory free when the engine was created (config 4 needs 9.5 GB, config 5 19 GB
    // of a 288 GB MI355X), so a drop-in pass leaves the rest of a shared device to others
    double pipe_budget = 0.0;
    uint64_t ring_bytes = 0;          // path state + queues + AOV scratch allocated now
    // PUPIL_PIPE_PATHS: a ring needs no more slots than it takes to put this many paths in
    // flight.  Frames ahead pay off by filling the launch tails of small launches; past
    // ~64 M paths per launch the tail is amortised and a larger ring only spreads the
    // traversal's path-state accesses (config 5, 133 M paths per frame: 2288 Mrays/s with
    // one slot, 2208 / 2195 / 2155 / 2093 with 2 / 3 / 4 / 6, profiles/r03_pipe_sweep_config5.txt)
    double pipe_paths = 64e6;
    bool pipe_valid = false;          // cleared by camera / instance / emitter updates
    float *aov_scratch = nullptr;     // K slots x 7 floats per local pixel
    size_t aov_cap = 0;
    hipStream_t last_stream = nullptr;  // of the last render (NULL = the default stream)
    bool rendered = false;
    double build_ms = 0.0;
    // path state / queues (grown on demand)
    size_t cap = 0;
    PathState ps{};
    Queues q{};
    int *ovf = nullptr;
    uint32_t ovf_threads = 0;
    // pixel map cache
    uint32_t *pixel_map = nullptr;
    uint32_t pm_key[5] = {0, 0, 0, 0, 0};
    uint32_t pm_count = 0;
    // stats
    unsigned long long *trace_counters = nullptr;  // [0] nodes [1] prims
    // device running totals of the extension and shadow rays listed by the flags partitions
    // ([0..1]); the first partition of a render copies them to [2..3] before adding, so the
    // render's own counts are [0..1] - [2..3] without a per-render clear (snap_taken)
    unsigned long long *ray_cum = nullptr;
    bool snap_taken = false;
    uint32_t *node_bound = nullptr;                // launch_node_bound's result (3 floats as bits)
    uint64_t primary_cum = 0;                      // host running total of camera rays
    uint32_t last_paths = 0, last_iters = 0;
    uint64_t last_primary = 0;
    bool last_stats = false;
    std::vector<hipEvent_t> trace_events;  // pairs
    std::vector<uint8_t> pair_kind;        // per pair: 0 extend, 1 shadow / mixed traversal, 2 shade, 3 one-launch frame
    // ev_begin / ev_end bracket renders that collect counters or stage times only (each event
    // leaves a few us of stream gap); ev_sync orders another stream after the last render
    hipEvent_t ev_begin = nullptr, ev_end = nullptr, ev_sync = nullptr;
    bool last_timed = false;  // the last render recorded ev_begin / ev_end
    uint32_t trace_pairs = 0;
    bool pairs_keep = false;  // the pairs of PUPIL_STATS_TRACE_TIMING renders accumulate until read
    // pairs of a PUPIL_STATS_TRACE_TIMING sequence folded into sums once kMaxPairs are pending
    double kept_ms[4] = {0.0, 0.0, 0.0, 0.0};
    uint64_t kept_n[4] = {0, 0, 0, 0};
    uint64_t refits = 0;  // acceleration structure refits / rebuilds after instance updates
    // PUPIL_TRACE_TAIL: per-wave start / drained / exit times of each traversal launch of a stats render
    unsigned long long *tail_buf = nullptr;
    uint32_t tail_waves = 0, tail_launches = 0;
    pupil_pt_counters totals{};
    // scene tables kept for dynamic updates (pupil_pt_update_instance / _update_emitters)
    std::vector<DevInstance> h_insts;
    DevInstance *d_insts = nullptr;
    DevMaterial *d_mats = nullptr;
    uint32_t *d_prim_inst = nullptr;
    DevEmitter *d_areas = nullptr, *d_env = nullptr;
    float *d_cdf = nullptr;
    uint32_t *d_guide = nullptr;
    pupil_emitter env_src{};  // the env emitter the tables were built from (same_env)
    bool env_src_valid = false;
    std::vector<DevEmitter> h_emit_areas;  // host sources of in-place emitter updates
    std::vector<float> h_emit_cdf;
    std::vector<uint32_t> h_emit_guide;
    // flattened-BVH refits: per-instance moved flags and the node-box scratch
    uint8_t *d_moved = nullptr;
    std::vector<uint8_t> h_moved;
    float *refit_box = nullptr;

    template <typename T>
    hipError_t alloc(T **p, size_t count) {
        hipError_t e = hipMalloc((void **)p, sizeof(T) * (count ? count : 1));
        if (e == hipSuccess) allocs.push_back(*p);
        return e;
    }
    template <typename T>
    hipError_t upload(T **p, const T *src, size_t count) {
        hipError_t e = alloc(p, count);
        if (e == hipSuccess && count) e = hipMemcpy(*p, src, sizeof(T) * count, hipMemcpyHostToDevice);
        return e;
    }
    void release(void *p) {
        if (!p) return;
        for (auto it = allocs.begin(); it != allocs.end(); ++it)
            if (*it == p) {
                allocs.erase(it);
                break;
            }
        (void)hipFree(p);
    }
    void release_state() {
        ring_bytes = 0;
        ring_fresh = true;
        void *bufs[] = {ps.ray_o, ps.ray_d, ps.hit,  ps.thr,  ps.rad,    ps.misc,
                        ps.sh_d, ps.sh_c, ps.mbin, ps.sflags, q.bins, q.nxsh, q.hist};
        for (void *b : bufs)
            if (b) (void)hipFree(b);
        ps = PathState{};
        q.bins = q.nxsh = q.hist = nullptr;
        cap = 0;
        pipe.clear();
        half_pending = false;
        pipe_valid = false;
    }
    ~pupil_pt() {
        (void)hipSetDevice(device);
        release_state();
        if (aov_scratch) (void)hipFree(aov_scratch);
        for (void *p : allocs) (void)hipFree(p);
        free_lbvh(bvh);
        free_two_level(tl);
        if (pixel_map) (void)hipFree(pixel_map);
        for (auto e : trace_events) (void)hipEventDestroy(e);
        if (ev_begin) (void)hipEventDestroy(ev_begin);
        if (ev_end) (void)hipEventDestroy(ev_end);
        if (ev_sync) (void)hipEventDestroy(ev_sync);
        if (own_stream) (void)hipStreamDestroy(own_stream);
    }
};

namespace {

int upload_texture(pupil_pt *pt, const pupil_texture &t, DevTexture &d) {
    std::memset(&d, 0, sizeof(d));
    d.type = t.type;
    d.width = t.width;
    d.height = t.height;
    d.filter = t.filter;
    for (int k = 0; k < 3; k++) {
        d.c0[k] = t.c0[k];
        d.c1[k] = t.c1[k];
    }
    for (int k = 0; k < 4; k++) {
        d.r0[k] = t.transform[k];
        d.r1[k] = t.transform[4 + k];
    }
    if (t.type == PUPIL_TEX_BITMAP) {
        if (!t.rgba || !t.width || !t.height) return fail(PUPIL_ERR_INVALID, "bitmap texture without texels");
        float4 *texels = nullptr;
        HIP_TRY(pt->upload(&texels, reinterpret_cast<const float4 *>(t.rgba), (size_t)t.width * t.height));
        d.data = texels;
    } else if (t.type > PUPIL_TEX_CHECKERBOARD) {
        return fail(PUPIL_ERR_INVALID, "unknown texture type");
    }
    return PUPIL_OK;
}

int convert_emitter(pupil_pt *pt, const pupil_emitter &e, DevEmitter &d) {
    std::memset(&d, 0, sizeof(d));
    d.type = e.type;
    d.select_probability = e.select_probability;
    d.area = e.area;
    d.radius = e.radius;
    int rc = upload_texture(pt, e.radiance, d.radiance);
    if (rc) return rc;
    for (int k = 0; k < 3; k++) {
        d.pos[k] = v3(e.pos[k][0], e.pos[k][1], e.pos[k][2]);
        d.nrm[k] = v3(e.nrm[k][0], e.nrm[k][1], e.nrm[k][2]);
        d.tex[k] = v2(e.tex[k][0], e.tex[k][1]);
    }
    d.center = v3(e.center[0], e.center[1], e.center[2]);
    d.color = v3(e.color[0], e.color[1], e.color[2]);
    d.scale = e.scale;
    for (int k = 0; k < 9; k++) {
        d.to_world[k] = e.to_world[k];
        d.to_local[k] = e.to_local[k];
    }
    if (e.type == PUPIL_EMITTER_ENV_MAP) {
        // BuildEnvMapCdfTable (world/emitter.cpp:107-149)
        const pupil_texture &t = e.radiance;
        if (t.type != PUPIL_TEX_BITMAP || !t.rgba) return fail(PUPIL_ERR_INVALID, "env map needs a bitmap");
        const size_t w = t.width, h = t.height;
        std::vector<float> col_cdf((w + 1) * h), row_cdf(h + 1), row_weight(h);
        size_t ci = 0, ri = 0;
        float row_sum = 0.f;
        row_cdf[ri++] = 0.f;
        for (size_t y = 0; y < h; ++y) {
            float col_sum = 0.f;
            col_cdf[ci++] = 0.f;
            for (size_t x = 0; x < w; ++x) {
                const size_t pix = y * w + x;
                col_sum += luminance(v3(t.rgba[pix * 4 + 0], t.rgba[pix * 4 + 1], t.rgba[pix * 4 + 2]));
                col_cdf[ci++] = col_sum;
            }
            for (size_t x = 1; x < w; ++x) col_cdf[ci - x - 1] /= col_sum;
            col_cdf[ci - 1] = 1.f;
            const float weight = std::sin((y + 0.5f) * kPi / h);
            row_weight[y] = weight;
            row_sum += col_sum * weight;
            row_cdf[ri++] = row_sum;
        }
        for (size_t y = 1; y < h; ++y) row_cdf[ri - y - 1] /= row_sum;
        row_cdf[ri - 1] = 1.f;
        d.normalization = 1.f / (row_sum * (2.f * kPi / w) * (kPi / h));
        d.map_w = (uint32_t)w;
        d.map_h = (uint32_t)h;
        float *a = nullptr, *b = nullptr, *c = nullptr;
        HIP_TRY(pt->upload(&a, row_cdf.data(), row_cdf.size()));
        HIP_TRY(pt->upload(&b, col_cdf.data(), col_cdf.size()));
        HIP_TRY(pt->upload(&c, row_weight.data(), row_weight.size()));
        d.row_cdf = a;
        d.col_cdf = b;
        d.row_weight = c;
    }
    return PUPIL_OK;
}

// EmitterGroup (render/emitter.h:110-135): the area emitters, their sequential selection
// CDF and its guide table (2^bits >= emitter count buckets, at most 2^20, guide[k] = first
// i with cdf[i] >= k / 2^bits; empty for PUPIL_EMITTER_SELECT=binary, the plain binary
// search A/B, or fewer than two emitters).  Bitmap radiance textures are uploaded here.
int emitter_tables(pupil_pt *pt, const pupil_scene_desc *scene, std::vector<DevEmitter> &areas, std::vector<float> &cdf,
                   std::vector<uint32_t> &guide, uint32_t &bits) {
    areas.assign(scene->num_area_emitters, DevEmitter{});
    cdf.assign(scene->num_area_emitters, 0.f);
    float sum_p = 0.f;
    for (uint32_t e = 0; e < scene->num_area_emitters; e++) {
        int rc = convert_emitter(pt, scene->area_emitters[e], areas[e]);
        if (rc) return rc;
        cdf[e] = sum_p + areas[e].select_probability;
        sum_p = cdf[e];
    }
    bits = 0;
    while ((1u << bits) < scene->num_area_emitters && bits < 20) bits++;
    const char *sel = std::getenv("PUPIL_EMITTER_SELECT");
    guide.clear();
    if (scene->num_area_emitters > 1 && !(sel && std::strcmp(sel, "binary") == 0)) {
        const uint32_t m = 1u << bits;
        guide.resize(m + 1);
        uint32_t i = 0;
        for (uint32_t k = 0; k <= m; k++) {
            const float t = (float)k / (float)m;
            while (i < cdf.size() && cdf[i] < t) i++;
            guide[k] = i;
        }
    }
    return PUPIL_OK;
}

// the scene's env emitter is the one the engine holds (an update may then keep its tables)
bool same_env(const pupil_pt *pt, const pupil_scene_desc *scene) {
    const bool has = scene->env && scene->env->type != PUPIL_EMITTER_NONE;
    if (has != pt->env_src_valid) return false;
    return !has || std::memcmp(&pt->env_src, scene->env, sizeof(pupil_emitter)) == 0;
}

// replaces the previous tables (creation, and updates that change their shapes)
int upload_emitters(pupil_pt *pt, const pupil_scene_desc *scene) {
    std::vector<DevEmitter> areas;
    std::vector<float> cdf;
    std::vector<uint32_t> g;
    uint32_t bits = 0;
    if (const int rc = emitter_tables(pt, scene, areas, cdf, g, bits)) return rc;
    DevEmitter *d_areas = nullptr, *d_env = nullptr;
    float *d_cdf = nullptr;
    uint32_t *d_guide = nullptr;
    if (pt->upload(&d_areas, areas.data(), areas.size()) || pt->upload(&d_cdf, cdf.data(), cdf.size()))
        return fail(PUPIL_ERR_OOM, "emitter upload failed");
    if (!g.empty() && pt->upload(&d_guide, g.data(), g.size())) return fail(PUPIL_ERR_OOM, "emitter guide upload failed");
    pt->env_src_valid = false;
    if (scene->env && scene->env->type != PUPIL_EMITTER_NONE) {
        pt->env_src = *scene->env;
        pt->env_src_valid = true;
        DevEmitter env;
        int rc = convert_emitter(pt, *scene->env, env);
        if (rc) return rc;
        if (pt->upload(&d_env, &env, 1)) return fail(PUPIL_ERR_OOM, "env upload failed");
    }
    pt->release(pt->d_areas);
    pt->release(pt->d_cdf);
    pt->release(pt->d_env);
    pt->release(pt->d_guide);
    pt->d_areas = d_areas;
    pt->d_cdf = d_cdf;
    pt->d_guide = d_guide;
    pt->sc.area_guide = d_guide;
    pt->sc.guide_bits = bits;
    pt->d_env = d_env;
    pt->sc.areas = d_areas;
    pt->sc.area_cdf = d_cdf;
    pt->sc.num_areas = scene->num_area_emitters;
    pt->sc.has_env = d_env ? 1u : 0u;
    pt->sc.env = d_env;
    return PUPIL_OK;
}

int ensure_state(pupil_pt *pt, size_t paths) {
    if (paths <= pt->cap) return PUPIL_OK;
    pt->release_state();
    const size_t n = paths;
    HIP_TRY(hipMalloc((void **)&pt->ps.ray_o, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.ray_d, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.hit, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.thr, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.rad, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.misc, sizeof(uint4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sh_d, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sh_c, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.mbin, n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sflags, n));
    HIP_TRY(hipMalloc((void **)&pt->q.bins, sizeof(uint32_t) * n));
    HIP_TRY(hipMalloc((void **)&pt->q.nxsh, sizeof(uint32_t) * 2 * n));
    HIP_TRY(hipMalloc((void **)&pt->q.hist, sizeof(uint32_t) * partition_hist_entries((uint32_t)n)));
    pt->q.capacity = (uint32_t)n;
    pt->cap = n;
    pt->ring_bytes = n * (8 * 16 + 2 + 4 + 8) + sizeof(uint32_t) * (size_t)partition_hist_entries((uint32_t)n);
    return PUPIL_OK;
}

// BVH4 node array the traversal walks (its size bounds the 32-bit node offsets, kMaxNodes4)
// the engine's own stream waits for everything enqueued so far on the stream of the last
// render (which itself waited for the renders before it on other streams)
hipError_t order_after_renders(pupil_pt *pt) {
    if (!pt->rendered || pt->last_stream == pt->own_stream) return hipSuccess;
    hipError_t e = hipEventRecord(pt->ev_sync, pt->last_stream);
    return e == hipSuccess ? hipStreamWaitEvent(pt->own_stream, pt->ev_sync, 0) : e;
}

uint64_t nodes4_count(const pupil_pt *pt) {
    return pt->two_level ? (pt->tl.world ? pt->tl.num_wnodes : pt->tl.num_nodes4) : pt->bvh.num_nodes4;
}

// DeviceScene::node_bound of the current BVH4 arrays (after every build and refit;
// one 12-B read back, the traversal kernels take it by value).  Live nodes only: in the
// two-level layouts the TLAS reserve [tlas_nodes, tlas_cap) is never written, and
// whatever an earlier allocation left there must not loosen the bound of every ray.
int refresh_node_bound(pupil_pt *pt) {
    pt->sc.node_bound[0] = pt->sc.node_bound[1] = pt->sc.node_bound[2] = 0.f;
    const uint64_t n = nodes4_count(pt);
    {  // LDS-resident top of the tree (pt_scene.h top_nodes) for the world-mode two-level structure, whose
       // braided TLAS every ray crosses first: -1.3 % per config-5 step; the flat trees of configs 3 / 4
       // pay 1.1 % per launch for the per-visit branch and run the kernel without it
       // (profiles/r05_top_nodes_bisect.txt; PUPIL_TOP_NODES=k forces k nodes, 0 off)
        const char *e = std::getenv("PUPIL_TOP_NODES");
        const uint32_t want = e ? (uint32_t)std::min<long>(kTopNodes, std::max(0L, std::atol(e)))
                                : (pt->two_level && pt->tl.world ? kTopNodes : 0u);
        uint64_t live = pt->sc.nodes4 ? n : 0;
        if (pt->two_level) live = std::min<uint64_t>(live, pt->tl.tlas_nodes);
        pt->sc.top_nodes = (uint32_t)std::min<uint64_t>(want, live);
    }
    if (!pt->sc.nodes4 || n == 0) return PUPIL_OK;
    if (pt->two_level) {
        const uint64_t tlas = std::min<uint64_t>(pt->tl.tlas_nodes, n), cap = std::min<uint64_t>(pt->tl.tlas_cap, n);
        launch_node_bound(pt->sc.nodes4, tlas, pt->node_bound, pt->own_stream, true);
        launch_node_bound(pt->sc.nodes4 + cap, n - cap, pt->node_bound, pt->own_stream, false);
    } else {
        launch_node_bound(pt->sc.nodes4, n, pt->node_bound, pt->own_stream, true);
    }
    uint32_t b[3];
    HIP_TRY(hipMemcpyAsync(b, pt->node_bound, sizeof(b), hipMemcpyDeviceToHost, pt->own_stream));
    HIP_TRY(hipStreamSynchronize(pt->own_stream));
    for (int a = 0; a < 3; a++) std::memcpy(&pt->sc.node_bound[a], &b[a], 4);
    return PUPIL_OK;
}

// Local pixel list of a rank: tiles t with t % world == rank, row-major tile
// order, row-major pixels inside a tile (clipped at the image border).

uint32_t local_pixels(uint32_t w, uint32_t h, uint32_t ts, uint32_t rank, uint32_t world, uint32_t *out) {
    if (world <= 1) {
        if (out)
            for (uint32_t i = 0; i < w * h; i++) out[i] = i;
        return w * h;
    }
    const uint32_t tx = (w + ts - 1) / ts, ty = (h + ts - 1) / ts;
    uint32_t n = 0;
    for (uint32_t t = rank; t < tx * ty; t += world) {
        const uint32_t bx = (t % tx) * ts, by = (t / tx) * ts;
        for (uint32_t y = by; y < by + ts && y < h; y++)
            for (uint32_t x = bx; x < bx + ts && x < w; x++) {
                if (out) out[n] = y * w + x;
                n++;
            }
    }
    return n;
}

// ------------------------------------------------------------------ frame schedules
// Shared state of one pupil_pt_render call.
struct RenderCtx {
    pupil_pt *pt;
    hipStream_t s;
    bool stats, timing;
    TraceStats ts_dev;
    const uint32_t *key;  // w, h, tile size, rank, world
    bool tail = false;
    bool trace_only = false;  // PUPIL_STATS_TRACE_TIMING: traversal launches only
    uint32_t pair = 0;
    bool open = false;
    const TraceStats *tsp() const { return stats ? &ts_dev : nullptr; }
    // stage events only on request: each hipEventRecord between two kernels costs
    // ~6 us of stream gap (9 per 1-spp render at D = 4)
    uint32_t pair_cap = 0;  // events created for this render
    void ev0(uint8_t kind) {
        open = timing && !(trace_only && kind == 2) && pair < pair_cap;
        if (!open) return;
        pt->pair_kind[pair] = kind;
        (void)hipEventRecord(pt->trace_events[2 * pair], s);
    }
    void ev1() {
        if (!open) return;
        (void)hipEventRecord(pt->trace_events[2 * pair + 1], s);
        pair++;
        open = false;
    }
    void tail_slot() {  // wave-time slice of the next traversal launch (PUPIL_TRACE_TAIL)
        if (tail && pt->tail_launches < kMaxDepth + 1)
            ts_dev.wave_times = pt->tail_buf + (size_t)pt->tail_launches++ * pt->tail_waves * 4;
        else
            ts_dev.wave_times = nullptr;
    }
    // path state of ring slot h: every array offset by h * paths
    PathState view(uint32_t h, size_t paths, size_t extra = 0) const {
        PathState v = pt->ps;
        const size_t o = (size_t)h * paths + extra;
        v.ray_o += o, v.ray_d += o, v.hit += o, v.thr += o, v.rad += o, v.misc += o;
        v.sh_d += o, v.sh_c += o, v.mbin += o, v.sflags += o;
        return v;
    }
};

// Pipelined frames.  The batch's path state is one slot of a ring of K slots.  A frame
// runs max_depth phases -- phase b: trace (b = 0: the camera rays, else the shadow +
// extension rays its bounce-(b-1) shade spawned) then the bounce-b shade -- and one
// iteration of the loop below advances every frame in flight by one phase with one
// flags partition over the ring, ONE persistent traversal launch (the listed shadow and
// extension rays of all frames, plus the camera rays of a frame started in that
// iteration) and ONE shade launch (each path at its own bounce).  A render runs the
// iterations its own frame still needs and then accumulates it, so the frame is
// complete when the call's work has run, as PTPass::OnRun requires
// (pt_pass.cpp:51-56); the other frames in flight belong to the renders that continue
// this one (random_seed + spp each, same camera, scene, tiling, spp and depth), and are
// dropped when the next render does not continue it.  Frames are started in the last
// run + 1 iterations of a render (run = renders in a row that continued the previous
// one), so a continued sequence reaches one iteration per render after K renders, and
// a render that is never continued (a moving camera) pays only for one frame's first
// phase ahead.  Per path, every operation and its order are those of the reference's
// per-pixel loop (main.cu:84-193): output is bit-identical to the oracle whatever the
// schedule.  Renders that collect counters, depths above 63 (the 6-bit flags tags) and
// PUPIL_AHEAD=0 run with K = 1: one frame at a time, D iterations.
int render_pipelined(RenderCtx &cx, const FrameParams &fp, const pupil_pt_launch *launch) {
    pupil_pt *pt = cx.pt;
    hipStream_t s = cx.s;
    const uint32_t D = fp.max_depth;
    const size_t np = fp.num_paths;
    const bool may_pipe = pt->ahead_mode != 0 &&
                          (pt->ahead_mode == 2 || launch->spp == 1 || (launch->hints & PUPIL_HINT_CONTINUE)) && !cx.stats &&
                          D >= 2 && D <= 63;  // the 6-bit flags tags of a slot stay unambiguous for 63 iterations
    // frames ahead are started only once a continuation is likely: the caller said so
    // (PUPIL_HINT_CONTINUE), or the last render was continued too.  A render after a change
    // (a camera moving every OnRun) then traces nothing it may discard.
    const bool cont_seed = pt->pipe_valid && pt->pipe_next_seed == launch->random_seed;
    const bool speculate = (launch->hints & PUPIL_HINT_CONTINUE) || pt->ahead_mode == 2 ||
                           (cont_seed && pt->pipe_run >= 1);
    uint32_t K = 1, G = 1;
    if (may_pipe) {
        // frame groups: 1-spp renders (the OnRun cadence) smaller than PUPIL_PIPE_GROUP_PATHS
        // (one rank's tiles, small films) batch G consecutive frames per ring slot, so each
        // traversal launch carries enough rays to amortise its tail; the renders whose frame an
        // earlier render already completed only accumulate it.  Batched renders (spp > 1, the
        // bench's progressive steps) keep one frame per slot (PUPIL_PIPE_GROUP_ALL=1: group them too)
        static const bool group_all = [] {
            const char *e = std::getenv("PUPIL_PIPE_GROUP_ALL");
            return e && std::atoi(e) != 0;
        }();
        if (launch->spp == 1 || group_all)
            G = (uint32_t)std::min((double)pt->pipe_group_max,
                                   std::max(1.0, std::ceil(pt->pipe_group_paths / (double)np)));
        K = pt->pipe_limit ? std::min(pt->pipe_limit, D) : D;
        constexpr double kPathBytes = 8 * 16 + 2 + 4 + 8 + 1;  // PathState + bins + nxsh + partition scratch
        K = std::min<uint32_t>(K, (uint32_t)std::max(1.0, std::floor(pt->pipe_budget / ((double)G * np * kPathBytes))));
        K = std::min<uint32_t>(K, (uint32_t)std::max(1.0, std::ceil(pt->pipe_paths / ((double)G * np))));
        while (K * G > 1 && (uint64_t)K * G * np >= (1ull << 31)) {
            if (G > 1) G--;
            else K--;
        }
    }
    uint32_t key[9] = {cx.key[0], cx.key[1], cx.key[2], cx.key[3], cx.key[4], fp.spp, D, fp.num_local, G};
    // this render continues the last one (OnRun cadence: the next seed, nothing changed);
    // frames in flight, if any, are then exactly the ones it and its successors need
    bool reset = !(cont_seed && K == pt->pipe_slots && np == pt->pipe_np &&
                   std::memcmp(key, pt->pipe_key, sizeof(key)) == 0 &&
                   (pt->pipe.empty() ||
                    pt->pipe.front().seed + pt->pipe.front().consumed * fp.spp == launch->random_seed));
    const uint32_t nl = fp.num_local;
    // a render that starts no frame ahead has none in flight either (speculation is off only
    // right after a reset) and works on slot 0, frame 0: the ring is allocated for frames ahead
    // only once a render speculates, so a camera moving every OnRun runs on the path-state
    // footprint of PUPIL_AHEAD=0.  K and G stay as computed: the pipeline key does not change
    // when speculation starts
    const auto ring_need = [&]() { return speculate ? (size_t)K * G * np : (size_t)np; };
    // a reset caused only by growing the ring (this render continues the last one) keeps the
    // run count, so the render after the first speculating one speculates as well
    const bool continued = !reset;
    if (ring_need() > pt->cap) {  // growing the ring loses its contents
        reset = true;
        pt->pipe.clear();
        int rc = ensure_state(pt, ring_need());
        while (rc == PUPIL_ERR_OOM && speculate && K * G > 1) {  // a smaller ring, down to no frames ahead
            if (K > 1) K = K > 2 ? K / 2 : 1;
            else G = G > 2 ? G / 2 : 1;
            rc = ensure_state(pt, ring_need());
        }
        if (rc) return rc;
        key[8] = G;
    }
    const size_t cap_paths = (size_t)G * np;  // paths per ring slot
    // AOV scratch holds the AOVs of frames shaded ahead of their render: needed only once a
    // render speculates (frames in flight imply an earlier speculating render allocated it), so a
    // moving camera keeps the footprint of PUPIL_AHEAD=0 here too
    if (speculate && K * G > 1 && (size_t)K * G * 7 * nl > pt->aov_cap) {
        reset = true;
        if (pt->aov_scratch) (void)hipFree(pt->aov_scratch);
        pt->aov_scratch = nullptr;
        pt->aov_cap = 0;
        HIP_TRY(hipMalloc((void **)&pt->aov_scratch, sizeof(float) * (size_t)K * G * 7 * nl));
        pt->aov_cap = (size_t)K * G * 7 * nl;
    }
    const PathState ring = pt->ps;
    if (reset) {
        // the dropped frames' flags / bins bytes are cleared (every other byte of the ring is
        // clear: a completed frame's accumulate clears its own)
        for (const auto &g : pt->pipe) {
            const size_t off = (size_t)g.slot * pt->pipe_cap, len = (size_t)g.frames * pt->pipe_np;
            if (off + len > pt->cap) continue;
            HIP_TRY(hipMemsetAsync(ring.sflags + off, 0, len, s));
            if (!pt->shade_list) HIP_TRY(hipMemsetAsync(ring.mbin + off, 0xFF, len, s));
        }
        if (pt->ring_fresh) {  // a new allocation: everything
            HIP_TRY(hipMemsetAsync(ring.sflags, 0, pt->cap, s));
            if (!pt->shade_list) HIP_TRY(hipMemsetAsync(ring.mbin, 0xFF, pt->cap, s));
            pt->ring_fresh = false;
        }
        pt->pipe.clear();
        pt->half_pending = false;  // an iteration split over the last render and this one is dropped
        pt->pipe_run = continued ? pt->pipe_run + 1 : 0;
        pt->pipe_slots = K;
        pt->pipe_np = np;
        pt->pipe_cap = cap_paths;
        std::memcpy(pt->pipe_key, key, sizeof(key));
    } else {
        pt->pipe_run++;
    }
    pt->pipe_valid = true;
    Queues &q = pt->q;
    // the flags partition scans the slots in use: [0, end of the last frame group)
    auto ring_end = [&]() {
        size_t e = 0;
        for (const auto &g : pt->pipe) e = std::max(e, (size_t)g.slot * cap_paths + (size_t)g.frames * np);
        return (uint32_t)e;
    };
    const uint32_t interleave0 = pt->primary_interleave;
    // a render that starts nothing ahead and needs no frame in flight, small enough (one rank's
    // tiles, small films): the whole frame in one persistent launch (pt_frame.hip), no
    // per-bounce traversal drain, shade launch or partition
    if (pt->frame_paths > 0.0 && !cx.stats && !speculate && pt->pipe.empty() && (double)np <= pt->frame_paths &&
        frame_kernel_supported(pt->sc)) {
        // this render's extension / shadow rays = the growth of the running totals from here
        HIP_TRY(hipMemcpyAsync(pt->ray_cum + 2, pt->ray_cum, 2 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, s));
        pt->snap_taken = true;
        FrameParams fs = fp;
        fs.group = 1;
        cx.ev0(3);  // traversal and shading in one kernel: timed apart from trace_ms (frame_ms)
        launch_frame(pt->sc, fs, ring, pt->q.work + kWorkFrame, pt->ray_cum, pt->ovf, pt->ovf_threads,
                     interleave0 && fp.spp > 1 ? fp.spp : 0u, s);
        cx.ev1();
        launch_accumulate(fp, ring, nullptr, true, s);
        pt->pipe_next_seed = launch->random_seed + fp.spp;
        pt->last_iters = D;
        pt->last_primary = np;
        pt->primary_cum += np;
        pt->frame_launches++;
        return PUPIL_OK;
    }
    // AOV scratch of ring slot `slot`, frame `f` of its group: 7 floats per local pixel
    auto scratch = [&](uint32_t slot, uint32_t f) { return pt->aov_scratch + ((size_t)slot * G + f) * 7 * nl; };
    uint64_t started = 0;
    // depths above 64: every 16 iterations the host reads the list lengths back and stops
    // once no path is left (all of them missed, were absorbed or were terminated by RR)
    const bool deep_exit = D > 64 && K == 1;
    pt->snap_taken = false;
    // One iteration in two halves: (a) start a frame group if due, list the rays the previous
    // shade spawned and trace them (with the new group's camera rays); (b) partition by
    // material, shade.  Frame-group pacing runs (a) at the end of the render before the one
    // that needs the iteration (below), (b) at that render's start.
    using Half = pupil_pt::HalfIter;
    // a render that starts on an empty pipeline (the first speculating render after a reset: it
    // traces its own frame from the camera rays) starts at most PUPIL_PIPE_RAMP groups ahead;
    // the renders after it fill the ring as before (one group more per iteration they run)
    uint32_t ahead_started = 0;
    bool fresh_start = false;
    auto trace_half = [&](uint32_t it, uint32_t L_it, uint32_t run) -> int {
        Half h{};
        h.had = !pt->pipe.empty();
        // start a frame group: this render's own on an empty pipeline (one frame unless
        // speculating), else the next one ahead in the last run + 1 iterations while a slot is free
        if (!h.had) fresh_start = true;
        h.inject = !h.had || (speculate && pt->pipe.size() < K && it + run + 1 >= L_it &&
                              (pt->pipe_ramp == 0 || !fresh_start || ahead_started < pt->pipe_ramp));
        if (h.inject && h.had) ahead_started++;
        // a group started on an empty pipeline (the render's own frame: after a reset, the first
        // speculating render) holds one frame when the ramp is limited, so that render traces
        // its own frame and at most PUPIL_PIPE_RAMP groups' first bounces, not G frames' worth
        // (r06 pacing: the heaviest OnRun after the camera stops)
        h.nf = pupil_pt::PipeFrame{0u, launch->random_seed, 0u, false,
                                   speculate && (h.had || pt->pipe_ramp == 0) ? G : 1u, 0u};
        if (h.inject && h.had) {
            h.nf.slot = (pt->pipe.back().slot + 1) % K;
            h.nf.seed = pt->pipe.back().seed + pt->pipe.back().frames * fp.spp;
        }
        h.nf.aov_scratch = h.had || h.nf.frames > 1;  // AOVs wait in the slot's scratch until the frame's render
        h.nfp = (uint32_t)(h.nf.frames * np);          // paths of the new group
        const uint32_t gspp = h.nf.frames * fp.spp;    // its samples per pixel
        const uint32_t interleave = interleave0 && gspp > 1 ? gspp : 0u;
        if (h.inject) {
            FrameParams fg = fp;
            fg.seed0 = h.nf.seed;
            fg.num_paths = h.nfp;
            launch_generate(pt->sc, fg, cx.view(h.nf.slot, cap_paths), s, !pt->fresh());
            started += h.nfp;
        }
        if (h.had) {
            // the rays the previous iteration's shade spawned, over the slots in use, in
            // increasing path id: next (bit 0) and shadow (bit 1) lists -> q.nxsh
            const uint32_t tag = pt->pipe_gen % 63u + 1u;
            launch_partition(ring.sflags, ring_end(), 2, kPartFlags, tag, q.nxsh, q.hist, q.counts + kCntNext,
                             q.counts + kStartNext, nullptr, nullptr, s, pt->ray_cum,
                             pt->snap_taken ? nullptr : pt->ray_cum + 2);
            pt->snap_taken = true;
            if (deep_exit && it % 16 == 0) {
                uint32_t c[2] = {1, 1};
                HIP_TRY(hipMemcpyAsync(c, q.counts + kCntNext, sizeof(c), hipMemcpyDeviceToHost, s));
                HIP_TRY(hipStreamSynchronize(s));
                if (c[0] == 0 && c[1] == 0) return 1;  // nothing left to trace or shade: the frame is complete
            }
            cx.ev0(1);
            cx.tail_slot();
            if (h.inject)  // + the new group's camera rays, dequeued first in every chunk (pixel-major)
                launch_trace_mixed(pt->sc, ring, q, pt->ovf, pt->ovf_threads, cx.tsp(), s, h.nfp, 0u,
                                   (uint32_t)(h.nf.slot * cap_paths), interleave, nl);
            else
                launch_trace_mixed(pt->sc, ring, q, pt->ovf, pt->ovf_threads, cx.tsp(), s);
            cx.ev1();
        } else {
            cx.ev0(0);
            cx.tail_slot();
            launch_extend(pt->sc, cx.view(h.nf.slot, cap_paths), q, nullptr, nullptr, h.nfp, pt->ovf, pt->ovf_threads,
                          cx.tsp(), s, interleave, nl);
            cx.ev1();
        }
        if (h.inject) {  // the group is in flight from here (ring_end covers it)
            h.nf.phases = 0;
            pt->pipe.push_back(h.nf);
        }
        pt->half = h;
        return 0;
    };
    auto shade_half = [&]() -> int {
        const Half h = pt->half;
        const uint32_t nring = ring_end();
        if (!pt->shade_list)  // material bins of every path traced in this iteration -> q.bins
            launch_partition(ring.mbin, nring, kPartMaxBins, kPartExclusive, 0u, q.bins, q.hist, q.counts,
                             q.counts + kStartBins, q.counts + kScratch, nullptr, s, nullptr, nullptr, pt->bin_mask);
        FrameParams fs = fp;
        fs.group = G;  // AOV frame of a sample: its group frame (samples per ring slot = G spp)
        if (h.inject && h.nf.aov_scratch) {  // AOVs of frames ahead wait in their slot's scratch
            fs.albedo = scratch(h.nf.slot, 0);
            fs.normal = fs.albedo + 3 * (size_t)nl;
            fs.test = fs.albedo + 6 * (size_t)nl;
            fs.aov_local = 1;
            fs.aov_frame_stride = (uint32_t)(7 * nl);
        }
        if (D > 63) HIP_TRY(hipMemsetAsync(ring.sflags, 0, nring, s));  // K = 1: tags would alias
        const uint32_t wtag = (pt->pipe_gen + 1u) % 63u + 1u;
        const ShadeList list =
            !pt->shade_list ? kShadeBins : (h.had ? (h.inject ? kShadeNextRange : kShadeNext) : kShadeAll);
        uint64_t live = 0;  // paths the launch may list
        for (const auto &g : pt->pipe) live += (uint64_t)g.frames * np;
        const uint32_t max_count = (uint32_t)std::min<uint64_t>(nring, live);
        cx.ev0(2);
        launch_shade(pt->sc, fs, ring, q, wtag, s, list, (uint32_t)(h.nf.slot * cap_paths), h.inject ? h.nfp : 0u,
                     max_count, pt->fresh(), h.nf.seed);
        cx.ev1();
        pt->pipe_gen++;
        for (auto &f : pt->pipe) f.phases++;
        return 0;
    };
    // the shade half of an iteration whose trace half the previous render ran (a reset above
    // dropped it with the frames it belonged to)
    if (pt->half_pending) {
        pt->half_pending = false;
        if (!reset)
            if (const int rc = shade_half()) return rc;
    }
    // iterations this render needs: none when an earlier render completed its frame
    const uint32_t L = pt->pipe.empty() ? D : D - pt->pipe.front().phases;
    for (uint32_t it = 0; it < L; it++) {
        const int rc = trace_half(it, L, pt->pipe_run);
        if (rc == 1) break;  // depth > 64: nothing left
        if (rc) return rc;
        if (const int rs = shade_half()) return rs;
    }
    // this render's frame is complete: accumulate it; the group's slot is free once all
    // its frames are accumulated
    pupil_pt::PipeFrame &g = pt->pipe.front();
    const uint32_t f = g.consumed;
    // (the accumulate clears the frame's flags bytes: no stale tag is ever listed again)
    launch_accumulate(fp, cx.view(g.slot, cap_paths, (size_t)f * np), g.aov_scratch ? scratch(g.slot, f) : nullptr,
                      true, s);
    if (++g.consumed == g.frames) pt->pipe.erase(pt->pipe.begin());
    // Frame-group pacing (r06): the render that displays a group's last frame, and would
    // otherwise do no traversal, runs the trace half of the iteration the next render needs;
    // that render starts with the shade half.  With G = 2 the traversal and the shade of every
    // iteration land in different OnRuns (~0.8 / 0.2 of an iteration) instead of one OnRun
    // doing all of it and the next none.  Speculative like the frames ahead: a reset drops it.
    if (pt->pipe_split && speculate && G > 1 && L == 0 && !pt->pipe.empty() && pt->pipe.front().phases < D) {
        const uint32_t L_next = D - pt->pipe.front().phases;
        const int rc = trace_half(0, L_next, pt->pipe_run + 1);
        if (rc < 0) return rc;
        pt->half_pending = rc == 0;
    }
    pt->pipe_next_seed = launch->random_seed + fp.spp;
    pt->last_iters = L;
    pt->last_primary = started;
    pt->primary_cum += started;
    return PUPIL_OK;
}

}  // namespace

extern "C" {

const char *pupil_last_error(void) { return g_last_error.c_str(); }
int pupil_abi_version(void) { return 6; }

int pupil_pt_local_pixels(uint32_t width, uint32_t height, uint32_t tile_size, uint32_t tile_rank, uint32_t tile_world,
                          uint32_t *out_pixels, uint32_t *inout_count) {
    if (!inout_count || width == 0 || height == 0) return fail(PUPIL_ERR_INVALID, "bad arguments");
    if (tile_world > 1 && (tile_size == 0 || tile_rank >= tile_world)) return fail(PUPIL_ERR_INVALID, "bad tiling");
    const uint32_t n = local_pixels(width, height, tile_size, tile_rank, tile_world, nullptr);
    if (out_pixels) {
        if (*inout_count < n) return fail(PUPIL_ERR_INVALID, "output too small");
        local_pixels(width, height, tile_size, tile_rank, tile_world, out_pixels);
    }
    *inout_count = n;
    return PUPIL_OK;
}

int pupil_pt_create(const pupil_scene_desc *scene, int device, pupil_pt **out) {
    if (!scene || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    *out = nullptr;
    if (scene->width == 0 || scene->height == 0) return fail(PUPIL_ERR_INVALID, "empty film");
    if (scene->num_instances == 0) return fail(PUPIL_ERR_INVALID, "scene has no instances");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PUPIL_ERR_HIP, "no HIP device");
    if (device < 0 || device >= ndev) return fail(PUPIL_ERR_INVALID, "bad device index");
    HIP_TRY(hipSetDevice(device));
    auto pt = new pupil_pt();
    pt->device = device;
    auto cleanup = [&](int rc) {
        delete pt;
        return rc;
    };
    if (hipStreamCreateWithFlags(&pt->own_stream, hipStreamNonBlocking) != hipSuccess)
        return cleanup(fail(PUPIL_ERR_HIP, "stream creation failed"));
    pt->width = scene->width;
    pt->height = scene->height;
    pt->max_depth = scene->max_depth ? scene->max_depth : 1;

    // shapes
    struct ShapeDev {
        float *pos = nullptr, *nrm = nullptr, *tex = nullptr;
        uint32_t *idx = nullptr;
    };
    std::vector<ShapeDev> shapes(scene->num_shapes);
    for (uint32_t s = 0; s < scene->num_shapes; s++) {
        const pupil_shape &sh = scene->shapes[s];
        if (sh.kind == PUPIL_SHAPE_MESH) {
            if (!sh.positions || !sh.indices || sh.num_faces == 0)
                return cleanup(fail(PUPIL_ERR_INVALID, "mesh without positions/indices"));
            for (size_t i = 0; i < 3 * (size_t)sh.num_faces; i++)
                if (sh.indices[i] >= sh.num_vertices) return cleanup(fail(PUPIL_ERR_INVALID, "index out of range"));
            if (pt->upload(&shapes[s].pos, sh.positions, 3 * (size_t)sh.num_vertices) ||
                (sh.normals && pt->upload(&shapes[s].nrm, sh.normals, 3 * (size_t)sh.num_vertices)) ||
                (sh.texcoords && pt->upload(&shapes[s].tex, sh.texcoords, 2 * (size_t)sh.num_vertices)) ||
                pt->upload(&shapes[s].idx, sh.indices, 3 * (size_t)sh.num_faces))
                return cleanup(fail(PUPIL_ERR_OOM, "mesh upload failed"));
        } else if (sh.kind != PUPIL_SHAPE_SPHERE) {
            return cleanup(fail(PUPIL_ERR_INVALID, "unknown shape kind"));
        }
    }
    // materials (optix_material.cpp:39-132 host precompute)
    std::vector<DevMaterial> mats(scene->num_materials);
    for (uint32_t m = 0; m < scene->num_materials; m++) {
        const pupil_material &src = scene->materials[m];
        DevMaterial &d = mats[m];
        std::memset(&d, 0, sizeof(d));
        d.type = src.type <= 7u ? src.type : 0u;
        d.twosided = src.twosided;
        d.nonlinear = src.nonlinear;
        if (d.type == PUPIL_MAT_DIELECTRIC || d.type == PUPIL_MAT_ROUGH_DIELECTRIC || d.type == PUPIL_MAT_PLASTIC ||
            d.type == PUPIL_MAT_ROUGH_PLASTIC)
            d.eta = src.int_ior / src.ext_ior;
        if (d.type == PUPIL_MAT_PLASTIC || d.type == PUPIL_MAT_ROUGH_PLASTIC) {
            const pupil_texture &dt = d.type == PUPIL_MAT_PLASTIC ? src.tex[0] : src.tex[1];
            const pupil_texture &stx = d.type == PUPIL_MAT_PLASTIC ? src.tex[1] : src.tex[2];
            const float diffuse_luminance = luminance(pixel_average(dt));
            const float specular_luminance = luminance(pixel_average(stx));
            d.specular_sampling_weight = specular_luminance / (specular_luminance + diffuse_luminance);
            d.int_fdr = diffuse_reflectance(1.f / d.eta);
        }
        for (int k = 0; k < 4; k++) {
            int rc = upload_texture(pt, src.tex[k], d.tex[k]);
            if (rc) return cleanup(rc);
        }
    }
    if (mats.empty()) {  // keep a valid pointer for instances without material
        DevMaterial d;
        std::memset(&d, 0, sizeof(d));
        mats.push_back(d);
    }
    // instances + primitive -> instance table
    std::vector<DevInstance> insts(scene->num_instances);
    std::vector<uint32_t> prim_inst;
    for (uint32_t i = 0; i < scene->num_instances; i++) {
        const pupil_instance &src = scene->instances[i];
        if (src.shape >= scene->num_shapes) return cleanup(fail(PUPIL_ERR_INVALID, "instance shape out of range"));
        if (src.material >= mats.size()) return cleanup(fail(PUPIL_ERR_INVALID, "instance material out of range"));
        const pupil_shape &sh = scene->shapes[src.shape];
        DevInstance &d = insts[i];
        std::memset(&d, 0, sizeof(d));
        std::memcpy(d.to_world, src.to_world, sizeof(d.to_world));
        std::memcpy(d.to_object, src.to_object, sizeof(d.to_object));
        d.kind = sh.kind;
        d.material = src.material;
        d.prim_offset = (uint32_t)prim_inst.size();
        d.emitter_offset = src.emitter_offset;
        d.flip_normals = src.flip_normals;
        d.flip_tex_coords = src.flip_tex_coords;
        d.bin = (mats[src.material].type >= 1u && mats[src.material].type <= 7u) ? mats[src.material].type : 8u;
        d.blas_root = kTraverseDone;
        d.positions = shapes[src.shape].pos;
        d.normals = shapes[src.shape].nrm;
        d.texcoords = shapes[src.shape].tex;
        d.indices = shapes[src.shape].idx;
        const uint32_t nprim = sh.kind == PUPIL_SHAPE_SPHERE ? 1u : sh.num_faces;
        if (src.emitter_offset >= 0 && (size_t)src.emitter_offset + nprim > scene->num_area_emitters)
            return cleanup(fail(PUPIL_ERR_INVALID, "emitter offset out of range"));
        prim_inst.insert(prim_inst.end(), nprim, i);
    }
    pt->num_prims = (uint32_t)prim_inst.size();
    if (prim_inst.size() >= (1ull << 31)) return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "more than 2^31 primitives"));
    DevInstance *d_insts = nullptr;
    DevMaterial *d_mats = nullptr;
    uint32_t *d_prim_inst = nullptr;
    // the shading's prim -> instance lookup (pt_kernels.h inst_of_prim): instance starts and a
    // guide table of at most ~8 K entries over the prim ids
    std::vector<uint32_t> inst_first(insts.size() + 1);
    for (size_t i = 0; i < insts.size(); i++) inst_first[i] = insts[i].prim_offset;
    inst_first[insts.size()] = (uint32_t)prim_inst.size();
    uint32_t guide_shift = 0;
    while ((prim_inst.size() >> guide_shift) > 8192u) guide_shift++;
    std::vector<uint32_t> inst_guide;
    if (!prim_inst.empty()) {
        const size_t nb = ((prim_inst.size() - 1) >> guide_shift) + 1;
        inst_guide.resize(nb + 1);
        for (size_t k = 0; k <= nb; k++)
            inst_guide[k] = prim_inst[std::min(k << guide_shift, prim_inst.size() - 1)];
    } else {
        inst_guide.assign(2, 0u);
    }
    uint32_t *d_inst_first = nullptr, *d_inst_guide = nullptr;
    if (pt->upload(&d_insts, insts.data(), insts.size()) || pt->upload(&d_mats, mats.data(), mats.size()) ||
        pt->upload(&d_prim_inst, prim_inst.data(), prim_inst.size()) ||
        pt->upload(&d_inst_first, inst_first.data(), inst_first.size()) ||
        pt->upload(&d_inst_guide, inst_guide.data(), inst_guide.size()))
        return cleanup(fail(PUPIL_ERR_OOM, "scene upload failed"));
    {
        int rc = upload_emitters(pt, scene);
        if (rc) return cleanup(rc);
    }
    pt->d_insts = d_insts;
    pt->d_mats = d_mats;
    pt->d_prim_inst = d_prim_inst;
    pt->leaf_size = 2u;  // with the 7-wave traversal: 2 beats 3 by 2 %, 1 and 4 are slower (config 4)
    if (const char *ls = std::getenv("PUPIL_LEAF_SIZE")) pt->leaf_size = (uint32_t)std::min(8, std::max(1, std::atoi(ls)));
    // Acceleration structure (replaces the GAS + IAS builds): one flattened BVH over
    // world-space primitives (default: on config 5 it traces 1.08x faster than the
    // two-level world mode), or a TLAS over per-instance BLASes (PUPIL_ACCEL=two_level,
    // which bench.py selects for config 5: cheaper instance updates; automatic when
    // the flattened primitive count would pass the flat build's 2^27 limit).  Both
    // give bit-identical hits.
    {
        std::vector<uint32_t> uses(scene->num_shapes, 0), inst_shape(scene->num_instances);
        uint64_t flat_prims = 0;
        for (uint32_t i = 0; i < scene->num_instances; i++) {
            inst_shape[i] = scene->instances[i].shape;
            uses[inst_shape[i]]++;
            const pupil_shape &sh = scene->shapes[inst_shape[i]];
            flat_prims += sh.kind == PUPIL_SHAPE_SPHERE ? 1u : sh.num_faces;
        }
        // leaf links hold 28-bit record slots, up to two per primitive (pt_scene.h kRecF4)
        pt->two_level = flat_prims >= (1ull << 27);
        if (const char *a = std::getenv("PUPIL_ACCEL")) {
            if (std::strcmp(a, "flat") == 0) pt->two_level = false;
            if (std::strcmp(a, "two_level") == 0) pt->two_level = true;
        }
        if (!pt->two_level && flat_prims >= (1ull << 27))
            return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "flattened BVH limited to 2^27 primitives"));
        if (pt->two_level) {
            std::vector<TwoLevelShape> tls(scene->num_shapes);
            for (uint32_t k = 0; k < scene->num_shapes; k++) {
                const pupil_shape &sh = scene->shapes[k];
                TwoLevelShape &t = tls[k];
                t = TwoLevelShape{};
                if (sh.kind != PUPIL_SHAPE_MESH || !uses[k]) continue;
                t.num_faces = sh.num_faces;
                t.num_vertices = sh.num_vertices;
                t.positions = shapes[k].pos;
                t.normals = shapes[k].nrm;
                t.texcoords = shapes[k].tex;
                t.indices = shapes[k].idx;
                float vmax = 0.f;
                for (size_t v = 0; v < 3 * (size_t)sh.num_vertices; v++) vmax = std::max(vmax, std::fabs(sh.positions[v]));
                t.vmax = vmax;
            }
            const int trc = build_two_level(tls, inst_shape, insts, d_insts, d_mats, pt->leaf_size, pt->own_stream, pt->tl);
            if (trc == -3) return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "TLAS + BLAS deeper than the traversal stacks hold"));
            if (trc == -4) return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "two-level record slots beyond the 28-bit leaf links"));
            if (trc != 0) return cleanup(fail(PUPIL_ERR_HIP, "two-level acceleration build failed"));
            pt->build_ms = pt->tl.build_ms;
        } else {
            BvhBuildInput bin{pt->num_prims, d_prim_inst, d_insts, d_mats};
            const int brc = build_bvh_bounded(bin, pt->bvh, pt->leaf_size, pt->own_stream, &pt->build_ms, 0);
            if (brc == -3) return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "BVH deeper than the traversal stacks hold"));
            if (brc != 0) return cleanup(fail(PUPIL_ERR_HIP, "LBVH build failed"));
        }
    }
    pt->h_insts = insts;
    DeviceScene &sc = pt->sc;
    sc.num_prims = pt->num_prims;
    if (pt->two_level) {
        sc.two_level = 1;
        sc.tl_world = pt->tl.world ? 1u : 0u;
        sc.nodes4 = pt->tl.world ? pt->tl.wnodes : pt->tl.nodes4;
        sc.prims = pt->tl.world ? pt->tl.wprims : pt->tl.prims;
        sc.wprims = pt->tl.wprims;
        sc.attrs = pt->tl.attrs;
        sc.root_link4 = pt->tl.root_link4;
    } else {
        sc.prims = pt->bvh.prims;
        sc.attrs = pt->bvh.attrs;
        sc.nodes4 = pt->bvh.nodes4;
        sc.root_link4 = pt->bvh.root_link4;
    }
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, pt->device);
    sc.num_cus = (uint32_t)std::max(1, cus);
    // persistent BVH4 kernels: refill once 16 lanes are idle (r02 re-tune on the SAH tree:
    // 16 / 12 beat 20 / 24 by ~0.7 % at N = 1 and the 8-way shard)
    sc.trace_refill = 16;
    if (const char *r = std::getenv("PUPIL_REFILL")) sc.trace_refill = (uint32_t)std::min(64, std::max(1, std::atoi(r)));
    if (const char *po = std::getenv("PUPIL_PRIMARY_ORDER")) pt->primary_interleave = std::strcmp(po, "path") != 0;
    {  // one material bin in the whole scene: the material partition orders nothing (auto; =bins / =list force)
        uint32_t bins = 0;
        for (const DevInstance &d : insts) bins |= 1u << d.bin;
        pt->shade_list = (bins & (bins - 1u)) == 0u;
        if (const char *sl = std::getenv("PUPIL_SHADE_LIST")) {
            if (std::strcmp(sl, "bins") == 0) pt->shade_list = false;
            if (std::strcmp(sl, "list") == 0) pt->shade_list = true;
        }
        sc.single_bin = pt->shade_list && bins && (bins & (bins - 1u)) == 0u ? (uint32_t)__builtin_ctz(bins) : 0u;
        pt->bin_mask = bins | 1u;  // the material bins a traced path can land in, and the miss bin
    }
    if (const char *fr = std::getenv("PUPIL_FRESH_SHADE")) pt->fresh_shade = std::atoi(fr) != 0;
    if (const char *a = std::getenv("PUPIL_AHEAD")) pt->ahead_mode = std::min(2, std::max(0, std::atoi(a)));
    if (const char *k = std::getenv("PUPIL_PIPE")) pt->pipe_limit = (uint32_t)std::min(63, std::max(0, std::atoi(k)));
    {  // ring budget: a quarter of the device memory free now (after the scene and its BVH)
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
        pt->pipe_budget = 0.25 * (double)free_b;
    }
    if (const char *g = std::getenv("PUPIL_PIPE_GB")) pt->pipe_budget = std::max(0.0, std::atof(g)) * 1e9;
    if (const char *g = std::getenv("PUPIL_PIPE_PATHS")) pt->pipe_paths = std::max(1.0, std::atof(g));
    if (const char *g = std::getenv("PUPIL_PIPE_GROUP_PATHS")) pt->pipe_group_paths = std::max(1.0, std::atof(g));
    if (const char *g = std::getenv("PUPIL_PIPE_GROUP_MAX")) pt->pipe_group_max = (uint32_t)std::min(64, std::max(1, std::atoi(g)));
    if (const char *g = std::getenv("PUPIL_PIPE_SPLIT")) pt->pipe_split = std::atoi(g) != 0;
    if (const char *g = std::getenv("PUPIL_PIPE_RAMP")) pt->pipe_ramp = (uint32_t)std::max(0, std::atoi(g));
    if (const char *g = std::getenv("PUPIL_FRAME_PATHS")) pt->frame_paths = std::max(0.0, std::atof(g));
    sc.trace_node_min = 8;  // node phase ends below 8 active lanes (7 waves: 8 and 12 beat 4 by 1.5 %; 2 is slower)
    if (const char *r = std::getenv("PUPIL_NODE_MIN")) sc.trace_node_min = (uint32_t)std::min(64, std::max(1, std::atoi(r)));
    if (nodes4_count(pt) > kMaxNodes4)
        return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "BVH4 larger than 2^26 nodes (32-bit node offsets)"));
    sc.prim_inst = d_prim_inst;
    sc.inst_first = d_inst_first;
    sc.inst_guide = d_inst_guide;
    sc.inst_guide_shift = guide_shift;
    sc.instances = d_insts;
    sc.materials = d_mats;
    std::memcpy(sc.camera.s2c, scene->sample_to_camera, sizeof(sc.camera.s2c));
    std::memcpy(sc.camera.c2w, scene->camera_to_world, sizeof(sc.camera.c2w));
    // traversal overflow stacks, counters, events
    pt->ovf_threads = trace_grid_blocks() * (uint32_t)kTraceBlock;
    if (pt->alloc(&pt->ovf, (size_t)pt->ovf_threads * std::max(kStackOvf, kTraceStackOvf)) || pt->alloc(&pt->trace_counters, 32) ||
        pt->alloc(&pt->ray_cum, 4) || pt->alloc(&pt->node_bound, 3) || pt->alloc(&pt->q.counts, kCountSlots) ||
        pt->alloc(&pt->q.work, kWorkSlots))
        return cleanup(fail(PUPIL_ERR_OOM, "workspace allocation failed"));
    if (hipMemset(pt->q.work, 0, kWorkSlots * sizeof(uint32_t)) != hipSuccess ||
        hipMemset(pt->ray_cum, 0, 4 * sizeof(unsigned long long)) != hipSuccess)
        return cleanup(fail(PUPIL_ERR_HIP, "workspace clear failed"));
    if (hipEventCreate(&pt->ev_begin) != hipSuccess || hipEventCreate(&pt->ev_end) != hipSuccess ||
        hipEventCreateWithFlags(&pt->ev_sync, hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(PUPIL_ERR_HIP, "event creation failed"));
    if (refresh_node_bound(pt) != PUPIL_OK) return cleanup(PUPIL_ERR_HIP);
    pt->totals.bvh_nodes = pt->two_level ? two_level_nodes(pt->tl) : pt->bvh.num_nodes4;
    pt->totals.two_level = pt->two_level ? 1u : 0u;
    pt->totals.bvh_depth = pt->two_level ? pt->tl.tlas_depth + pt->tl.blas_depth : pt->bvh.depth4;
    pt->totals.bvh_prims = pt->num_prims;
    pt->totals.build_ms = pt->build_ms;
    *out = pt;
    return PUPIL_OK;
}

int pupil_pt_set_camera(pupil_pt *pt, const float sample_to_camera[16], const float camera_to_world[16]) {
    if (!pt || !sample_to_camera || !camera_to_world) return fail(PUPIL_ERR_INVALID, "null argument");
    if (std::memcmp(pt->sc.camera.s2c, sample_to_camera, sizeof(pt->sc.camera.s2c)) != 0 ||
        std::memcmp(pt->sc.camera.c2w, camera_to_world, sizeof(pt->sc.camera.c2w)) != 0)
        pt->pipe_valid = false;  // frames in flight were started with the old view
    std::memcpy(pt->sc.camera.s2c, sample_to_camera, sizeof(pt->sc.camera.s2c));
    std::memcpy(pt->sc.camera.c2w, camera_to_world, sizeof(pt->sc.camera.c2w));
    return PUPIL_OK;
}

// RenderInstanceUpdate (ias_manager.cpp:116-151) for a set of instances: their new
// transforms, then ONE refit of the acceleration structure over all of them (the
// reference marks its IAS dirty per event and refits once in the next OnRun through
// GetIASHandle(2, true), pt_pass.cpp:46, ias_manager.cpp:199-211).  Flattened BVH: the
// moved instances' records get their new world vertices and every BVH4 node is refitted
// bottom up; two-level: their world records / BLAS copies and the TLAS boxes are
// refitted.  The render after it equals a render of a freshly created engine.  Ordered
// on the engine's stream after every render enqueued so far (no device-wide sync: other
// streams of the process keep running); returns once the structure is updated.
// Emitters follow with pupil_pt_update_emitters.
int pupil_pt_update_instances(pupil_pt *pt, uint32_t n, const uint32_t *ids, const float *to_world,
                              const float *to_object) {
    if (!pt || (n && (!ids || !to_world || !to_object))) return fail(PUPIL_ERR_INVALID, "null argument");
    for (uint32_t k = 0; k < n; k++)
        if (ids[k] >= pt->h_insts.size()) return fail(PUPIL_ERR_INVALID, "instance index out of range");
    if (n == 0) return PUPIL_OK;
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(order_after_renders(pt));  // no render may still read the old tables
    pt->pipe_valid = false;             // frames in flight were traced against the old geometry
    std::vector<uint32_t> changed;
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t id = ids[k];
        DevInstance &d = pt->h_insts[id];
        std::memcpy(d.to_world, to_world + 12 * (size_t)k, sizeof(d.to_world));
        std::memcpy(d.to_object, to_object + 12 * (size_t)k, sizeof(d.to_object));
        if (pt->two_level) refresh_instance_margins(d);  // they depend on the transform
        if (std::find(changed.begin(), changed.end(), id) == changed.end()) changed.push_back(id);
    }
    for (uint32_t id : changed)  // h_insts outlives the copies (the stream is synchronised below)
        HIP_TRY(hipMemcpyAsync(pt->d_insts + id, &pt->h_insts[id], sizeof(DevInstance), hipMemcpyHostToDevice,
                               pt->own_stream));
    pt->refits++;
    if (pt->two_level) {
        const auto t0 = std::chrono::steady_clock::now();
        // world mode refits the TLAS like the reference's IAS update (PUPIL_TL_UPDATE=rebuild: full build)
        const char *um = std::getenv("PUPIL_TL_UPDATE");
        const bool refit = !(um && std::strcmp(um, "rebuild") == 0);
        const int trc = rebuild_tlas(pt->tl, pt->h_insts, pt->d_insts, changed, pt->own_stream, refit);
        if (trc == -3) return fail(PUPIL_ERR_UNSUPPORTED, "TLAS + BLAS deeper than the traversal stacks hold");
        if (trc != 0) return fail(PUPIL_ERR_HIP, "TLAS rebuild failed");
        pt->sc.root_link4 = pt->tl.root_link4;
        if (const int rc = refresh_node_bound(pt)) return rc;
        pt->totals.bvh_nodes = two_level_nodes(pt->tl);
        pt->totals.bvh_depth = pt->tl.tlas_depth + pt->tl.blas_depth;
        pt->totals.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return PUPIL_OK;
    }
    BvhBuildInput bin{pt->num_prims, pt->d_prim_inst, pt->d_insts, pt->d_mats};
    // refit in place (PUPIL_FLAT_UPDATE=rebuild: full rebuild)
    const char *fu = std::getenv("PUPIL_FLAT_UPDATE");
    if (!(fu && std::strcmp(fu, "rebuild") == 0)) {
        if (!pt->d_moved) HIP_TRY(pt->alloc(&pt->d_moved, pt->h_insts.size()));
        if (!pt->refit_box) HIP_TRY(pt->alloc(&pt->refit_box, 6 * (size_t)std::max(1u, pt->bvh.num_nodes4)));
        pt->h_moved.assign(pt->h_insts.size(), 0);
        for (uint32_t id : changed) pt->h_moved[id] = 1;
        HIP_TRY(hipMemcpyAsync(pt->d_moved, pt->h_moved.data(), pt->h_moved.size(), hipMemcpyHostToDevice, pt->own_stream));
        double rms = 0.0;
        if (refit_bvh4(bin, pt->bvh, pt->d_moved, pt->refit_box, pt->own_stream, &rms) == 0) {
            pt->totals.build_ms = rms;
            return refresh_node_bound(pt);
        }
    }
    BvhBuildOutput nb{};
    double ms = 0.0;
    const int brc = build_bvh_bounded(bin, nb, pt->leaf_size, pt->own_stream, &ms, 0);
    if (brc != 0) {
        free_lbvh(nb);
        return fail(brc == -3 ? PUPIL_ERR_UNSUPPORTED : PUPIL_ERR_HIP,
                    brc == -3 ? "BVH deeper than the traversal stacks hold" : "LBVH rebuild failed");
    }
    free_lbvh(pt->bvh);
    pt->bvh = nb;
    if (pt->refit_box) {  // sized for the old tree
        pt->release(pt->refit_box);
        pt->refit_box = nullptr;
    }
    pt->sc.prims = nb.prims;
    pt->sc.attrs = nb.attrs;
    pt->sc.nodes4 = nb.nodes4;
    pt->sc.root_link4 = nb.root_link4;
    pt->totals.bvh_nodes = nb.num_nodes4;
    pt->totals.bvh_depth = nb.depth4;
    pt->totals.build_ms = ms;
    return refresh_node_bound(pt);
}

int pupil_pt_update_instance(pupil_pt *pt, uint32_t instance, const float to_world[12], const float to_object[12]) {
    if (!pt || !to_world || !to_object) return fail(PUPIL_ERR_INVALID, "null argument");
    return pupil_pt_update_instances(pt, 1, &instance, to_world, to_object);
}

// EmitterHelper reset after a transform change (world/world.cpp:45-54): the area
// emitter table, selection CDF and env emitter are replaced by the scene's.  When the
// tables keep their shapes (same emitter count, no bitmap radiance to upload, the same
// env) they are rewritten in place on the engine's stream after the renders enqueued so
// far; otherwise new tables are uploaded and the old ones freed.
int pupil_pt_update_emitters(pupil_pt *pt, const pupil_scene_desc *scene) {
    if (!pt || !scene) return fail(PUPIL_ERR_INVALID, "null argument");
    if (scene->num_area_emitters && !scene->area_emitters) return fail(PUPIL_ERR_INVALID, "missing emitter array");
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(order_after_renders(pt));
    pt->pipe_valid = false;
    bool in_place = pt->d_areas && scene->num_area_emitters == pt->sc.num_areas && same_env(pt, scene);
    for (uint32_t e = 0; in_place && e < scene->num_area_emitters; e++)
        in_place = scene->area_emitters[e].radiance.type != PUPIL_TEX_BITMAP;
    if (in_place) {
        std::vector<DevEmitter> areas;
        std::vector<float> cdf;
        std::vector<uint32_t> guide;
        uint32_t bits = 0;
        if (const int rc = emitter_tables(pt, scene, areas, cdf, guide, bits)) return rc;
        if (guide.empty() == (pt->d_guide != nullptr) || bits != pt->sc.guide_bits) in_place = false;
        if (in_place) {
            pt->h_emit_areas.swap(areas);  // kept alive until the copies have run (synchronised below)
            pt->h_emit_cdf.swap(cdf);
            pt->h_emit_guide.swap(guide);
            HIP_TRY(hipMemcpyAsync(pt->d_areas, pt->h_emit_areas.data(), sizeof(DevEmitter) * pt->h_emit_areas.size(),
                                   hipMemcpyHostToDevice, pt->own_stream));
            HIP_TRY(hipMemcpyAsync(pt->d_cdf, pt->h_emit_cdf.data(), sizeof(float) * pt->h_emit_cdf.size(),
                                   hipMemcpyHostToDevice, pt->own_stream));
            if (pt->d_guide)
                HIP_TRY(hipMemcpyAsync(pt->d_guide, pt->h_emit_guide.data(), sizeof(uint32_t) * pt->h_emit_guide.size(),
                                       hipMemcpyHostToDevice, pt->own_stream));
            HIP_TRY(hipStreamSynchronize(pt->own_stream));
            return PUPIL_OK;
        }
    }
    HIP_TRY(hipStreamSynchronize(pt->own_stream));  // the old tables are freed below
    return upload_emitters(pt, scene);
}

int pupil_pt_render(pupil_pt *pt, const pupil_pt_frame *out, const pupil_pt_launch *launch, void *hip_stream) {
    if (!pt || !out || !launch || !out->accum) return fail(PUPIL_ERR_INVALID, "null argument");
    if (launch->spp == 0) return PUPIL_OK;
    const uint32_t world = launch->tile_world ? launch->tile_world : 1u;
    const uint32_t ts = launch->tile_size ? launch->tile_size : 32u;
    if (launch->tile_rank >= world) return fail(PUPIL_ERR_INVALID, "tile_rank >= tile_world");
    HIP_TRY(hipSetDevice(pt->device));
    // NULL is HIP's default (null) stream, as everywhere in HIP: a caller that renders on
    // it and then reads the output on it (torch's default stream, for one) must see the
    // frame.  (Until r02 NULL selected the engine's own non-blocking stream, so e.g. a
    // gather issued on torch's default stream could read a frame still being rendered.)
    hipStream_t s = (hipStream_t)hip_stream;

    // local pixel map (cached per tiling)
    const uint32_t key[5] = {pt->width, pt->height, ts, launch->tile_rank, world};
    const uint32_t *map = nullptr;
    uint32_t num_local = pt->width * pt->height;
    if (world > 1) {
        if (!pt->pixel_map || std::memcmp(key, pt->pm_key, sizeof(key)) != 0) {
            num_local = local_pixels(pt->width, pt->height, ts, launch->tile_rank, world, nullptr);
            std::vector<uint32_t> host(num_local ? num_local : 1);
            local_pixels(pt->width, pt->height, ts, launch->tile_rank, world, host.data());
            if (pt->pixel_map) (void)hipFree(pt->pixel_map);
            pt->pixel_map = nullptr;
            HIP_TRY(hipMalloc((void **)&pt->pixel_map, sizeof(uint32_t) * host.size()));
            HIP_TRY(hipMemcpy(pt->pixel_map, host.data(), sizeof(uint32_t) * host.size(), hipMemcpyHostToDevice));
            std::memcpy(pt->pm_key, key, sizeof(key));
            pt->pm_count = num_local;
        }
        map = pt->pixel_map;
        num_local = pt->pm_count;
    }
    if (num_local == 0) return PUPIL_OK;
    const size_t paths = (size_t)num_local * launch->spp;
    if (paths >= (1ull << 31)) return fail(PUPIL_ERR_UNSUPPORTED, "too many paths in one batch");
    const bool stats = (launch->collect_stats & PUPIL_STATS_COUNTERS) != 0;
    const bool timing = (launch->collect_stats & PUPIL_STATS_TIMING) != 0;
    // The reference takes integrator.max_depth unclamped at SetScene (pt_pass.cpp:112-115;
    // only the inspector clamps to 1..128): any depth renders.  Diagnostics sized per
    // bounce (tail buffer) cover the first kMaxDepth launches.
    const uint32_t depth = std::max(1u, launch->max_depth ? launch->max_depth : pt->max_depth);
    if (pt->rendered && s != pt->last_stream) {  // another stream: after everything the last one holds
        HIP_TRY(hipEventRecord(pt->ev_sync, pt->last_stream));
        HIP_TRY(hipStreamWaitEvent(s, pt->ev_sync, 0));
    }

    FrameParams fp{};
    fp.width = pt->width;
    fp.height = pt->height;
    fp.num_local = num_local;
    fp.num_paths = (uint32_t)paths;
    fp.spp = launch->spp;
    fp.seed0 = launch->random_seed;
    fp.cnt0 = launch->sample_cnt;
    fp.accumulate = launch->accumulate;
    fp.max_depth = depth;
    fp.compact = out->compact;
    fp.aov_local = out->compact;
    fp.pixel_map = map;
    fp.accum = (float4 *)out->accum;
    fp.frame = (float4 *)out->frame;
    fp.albedo = (float *)out->albedo;
    fp.normal = (float *)out->normal;
    fp.test = (float *)out->test;
    fp.nee_count = stats ? pt->trace_counters + 16 : nullptr;

    // PUPIL_STATS_TRACE_TIMING: events around the traversal launches only, summed over
    // every render since pupil_pt_stats last read them (a timed sequence of renders)
    const bool trace_timing = (launch->collect_stats & PUPIL_STATS_TRACE_TIMING) != 0 && !timing;
    RenderCtx cx{pt, s, stats, timing || trace_timing, TraceStats{pt->trace_counters}, key};
    cx.trace_only = trace_timing;
    if (!(trace_timing && pt->pairs_keep)) {  // a new sum
        pt->trace_pairs = 0;
        for (int k = 0; k < 4; k++) pt->kept_ms[k] = 0.0, pt->kept_n[k] = 0;
    }
    if (trace_timing && pt->trace_pairs >= kMaxPairs) {  // a long unread sequence: fold the pending pairs
        HIP_TRY(hipEventSynchronize(pt->trace_events[2 * pt->trace_pairs - 1]));
        for (uint32_t i = 0; i < pt->trace_pairs; i++) {
            float m = 0.f;
            HIP_TRY(hipEventElapsedTime(&m, pt->trace_events[2 * i], pt->trace_events[2 * i + 1]));
            pt->kept_ms[pt->pair_kind[i]] += m;
            pt->kept_n[pt->pair_kind[i]]++;
        }
        pt->trace_pairs = 0;
    }
    cx.pair = trace_timing ? pt->trace_pairs : 0u;
    pt->pairs_keep = trace_timing;
    const bool tail = stats && std::getenv("PUPIL_TRACE_TAIL");
    if (tail && !pt->tail_buf) {
        pt->tail_waves = pt->ovf_threads / 64u;
        if (pt->alloc(&pt->tail_buf, (size_t)(kMaxDepth + 1) * pt->tail_waves * 4)) return fail(PUPIL_ERR_OOM, "tail buffer");
    }
    if (tail) HIP_TRY(hipMemsetAsync(pt->tail_buf, 0, sizeof(unsigned long long) * (kMaxDepth + 1) * pt->tail_waves * 4, s));
    cx.tail = tail;
    pt->tail_launches = 0;
    // events only when times are asked for: one pair per stage launch (kind 0 primary extend,
    // 1 bounce trace, 2 shade), at most two stage launches per iteration and kMaxPairs in all
    if (cx.timing) {
        const uint64_t pairs_needed = std::min<uint64_t>((uint64_t)cx.pair + 2ull * depth + 1ull, kMaxPairs + 2ull * 64);
        cx.pair_cap = (uint32_t)pairs_needed;
        while (pt->trace_events.size() < 2 * pairs_needed) {
            hipEvent_t e;
            HIP_TRY(hipEventCreate(&e));
            pt->trace_events.push_back(e);
        }
        if (pt->pair_kind.size() < pairs_needed) pt->pair_kind.resize(pairs_needed, 0);
    }
    pt->last_timed = stats || timing;
    if (pt->last_timed) HIP_TRY(hipEventRecord(pt->ev_begin, s));
    if (stats) HIP_TRY(hipMemsetAsync(pt->trace_counters, 0, 32 * sizeof(unsigned long long), s));
    const int rc = render_pipelined(cx, fp, launch);
    if (rc) return rc;
    if (pt->last_timed) HIP_TRY(hipEventRecord(pt->ev_end, s));
    HIP_TRY(hipGetLastError());
    pt->trace_pairs = cx.pair;
    pt->last_paths = fp.num_paths;
    pt->last_stats = stats;
    pt->last_stream = s;
    pt->rendered = true;
    return PUPIL_OK;
}

int pupil_pt_stats(pupil_pt *pt, pupil_pt_counters *out) {
    if (!pt || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(pt->device));
    if (pt->rendered) HIP_TRY(hipStreamSynchronize(pt->last_stream));
    pupil_pt_counters c = pt->totals;
    unsigned long long cum[4] = {0, 0, 0, 0};  // running totals, then their values before the last render
    HIP_TRY(hipMemcpy(cum, pt->ray_cum, sizeof(cum), hipMemcpyDeviceToHost));
    c.rays_traced_total = pt->primary_cum + cum[0] + cum[1];
    c.frames_in_flight = 0;  // frames started ahead of the next render (in groups: not yet accumulated)
    for (const auto &g : pt->pipe) c.frames_in_flight += g.frames - g.consumed;
    c.pipeline_slots = pt->pipe_slots;
    c.tlas_sah_splits = pt->two_level ? pt->tl.sah_splits : 0u;
    c.ring_bytes = pt->ring_bytes + sizeof(float) * (uint64_t)pt->aov_cap;
    c.ring_budget_bytes = (uint64_t)pt->pipe_budget;
    c.accel_refits = pt->refits;
    c.frame_launches = pt->frame_launches;
    for (int a = 0; a < 3; a++) c.node_bound[a] = pt->sc.node_bound[a];
    if (pt->last_paths) {
        // rays traced by the last render's launches (pipelined renders: of every frame in
        // flight; a render whose only iteration traced camera rays lists none)
        c.primary_rays = pt->last_primary;
        c.path_samples = pt->last_paths;
        c.extension_rays = pt->snap_taken ? cum[0] - cum[2] : 0u;
        c.shadow_rays = pt->snap_taken ? cum[1] - cum[3] : 0u;
        float ms = 0.f;
        if (pt->last_timed) HIP_TRY(hipEventElapsedTime(&ms, pt->ev_begin, pt->ev_end));
        c.last_render_ms = ms;
        double kind_ms[4] = {pt->kept_ms[0], pt->kept_ms[1], pt->kept_ms[2], pt->kept_ms[3]};
        uint64_t kind_n[4] = {pt->kept_n[0], pt->kept_n[1], pt->kept_n[2], pt->kept_n[3]};
        for (uint32_t i = 0; i < pt->trace_pairs; i++) {
            float m = 0.f;
            HIP_TRY(hipEventElapsedTime(&m, pt->trace_events[2 * i], pt->trace_events[2 * i + 1]));
            kind_ms[pt->pair_kind[i]] += m;
            kind_n[pt->pair_kind[i]]++;
        }
        pt->pairs_keep = false;  // read: the next PUPIL_STATS_TRACE_TIMING render starts a new sum
        c.trace_ms = kind_ms[0] + kind_ms[1];
        c.trace_launches = kind_n[0] + kind_n[1];
        c.extend_ms = kind_ms[0];
        c.extend_launches = kind_n[0];
        c.shade_ms = kind_ms[2];
        c.frame_ms = kind_ms[3];
        if (pt->last_stats && pt->tail_buf && pt->tail_launches) {  // PUPIL_TRACE_TAIL summary on stderr
            std::vector<unsigned long long> tb((size_t)pt->tail_launches * pt->tail_waves * 4);
            HIP_TRY(hipMemcpy(tb.data(), pt->tail_buf, sizeof(unsigned long long) * tb.size(), hipMemcpyDeviceToHost));
            for (uint32_t l = 0; l < pt->tail_launches; l++) {
                const unsigned long long *w = tb.data() + (size_t)l * pt->tail_waves * 4;
                std::vector<double> st, dr, ex;
                unsigned long long t0 = ~0ull, rays = 0;
                for (uint32_t k = 0; k < pt->tail_waves; k++)
                    if (w[4 * k + 2]) t0 = std::min(t0, w[4 * k]);
                for (uint32_t k = 0; k < pt->tail_waves; k++) {
                    if (!w[4 * k + 2]) continue;
                    st.push_back((double)(w[4 * k] - t0) * 0.01);  // 100 MHz -> us
                    dr.push_back(w[4 * k + 1] ? (double)(w[4 * k + 1] - t0) * 0.01 : -1.0);
                    ex.push_back((double)(w[4 * k + 2] - t0) * 0.01);
                    rays += w[4 * k + 3];
                }
                if (ex.empty()) continue;
                auto pct = [](std::vector<double> v, double q) {
                    std::sort(v.begin(), v.end());
                    return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
                };
                std::fprintf(stderr,
                             "[pupil tail] launch %u: %zu waves, %llu rays; start p50 %.1f max %.1f us; drained "
                             "first %.1f p50 %.1f us; exit p10 %.1f p50 %.1f p90 %.1f p99 %.1f max %.1f us\n",
                             l, ex.size(), rays, pct(st, 0.5), pct(st, 1.0), pct(dr, 0.0), pct(dr, 0.5), pct(ex, 0.1),
                             pct(ex, 0.5), pct(ex, 0.9), pct(ex, 0.99), pct(ex, 1.0));
            }
        }
        if (pt->last_stats) {
            unsigned long long tc[32];
            HIP_TRY(hipMemcpy(tc, pt->trace_counters, sizeof(tc), hipMemcpyDeviceToHost));
            if (std::getenv("PUPIL_TRACE_DIAG") && tc[2]) {  // SIMD efficiency, persistent kernels
                const unsigned long long *d = tc + 2;
                const double visits = (double)std::max(1ull, tc[0] + tc[14]);
                std::fprintf(stderr,
                             "[pupil] traversal: node loop %llu wave-iters, %.1f%% lanes active; leaf loop %llu wave-iters, "
                             "%.1f%% lanes active; %llu refills, %.1f lanes each; node visits %.0f, %.1f%% with no child "
                             "hit, %.1f%% of a popped node already beyond tmax\n",
                             d[0], 100.0 * (double)d[1] / (64.0 * (double)d[0]), d[2],
                             100.0 * (double)d[3] / (64.0 * (double)std::max(1ull, d[2])), d[4],
                             (double)d[5] / (double)std::max(1ull, d[4]), visits, 100.0 * (double)tc[9] / visits,
                             100.0 * (double)tc[8] / visits);
                if (tc[24])  // PUPIL_COOP builds: the cooperative node fetch
                    std::fprintf(stderr,
                                 "[pupil] coop fetch: %llu LDS-DMA wave-instructions (%.2f per node-loop iteration), "
                                 "%llu node slots (%.1f%% of the node visits, %.1f per DMA)\n",
                                 tc[24], (double)tc[24] / (double)std::max(1ull, d[0]), tc[25],
                                 100.0 * (double)tc[25] / visits, (double)tc[25] / (double)tc[24]);
            }
            c.node_loop_iters = tc[2];  // trace4_body dg[0..5]
            c.node_loop_lanes = tc[3];
            c.leaf_loop_iters = tc[4];
            c.leaf_loop_lanes = tc[5];
            c.refills = tc[6];
            c.refill_lanes = tc[7];
            c.node_visits = tc[0] + tc[14];
            c.prim_tests = tc[1] + tc[15];
            c.shadow_rays_reference = tc[16];
            c.unique_node_fetches = tc[18];
            c.coop_dma = tc[24];
            c.coop_slots = tc[25];
            c.queue_handed = tc[20];
            c.queue_activated = tc[21];
            c.queue_retired = tc[22];
            c.queue_listed = tc[23];
            c.extend_node_visits = tc[0];
            c.extend_prim_tests = tc[1];
            const double rays = (double)(c.primary_rays + c.extension_rays + c.shadow_rays);
            // 32 B ray read + 16 B hit write + 64 B per node + 48 B per primitive
            c.trace_bytes = rays * 48.0 + 64.0 * (double)c.node_visits + 48.0 * (double)c.prim_tests;
            c.extend_bytes = (double)(c.primary_rays + c.extension_rays) * 48.0 + 64.0 * (double)tc[0] +
                             48.0 * (double)tc[1];
        }
    }
    *out = c;
    return PUPIL_OK;
}

void pupil_pt_destroy(pupil_pt *pt) { delete pt; }

int pupil_pt_export_bvh4(pupil_pt *pt, uint32_t *num_nodes, void *nodes, uint32_t *num_records, float *records,
                         int32_t *root_link) {
    if (!pt || !num_nodes || !num_records || !root_link) return fail(PUPIL_ERR_INVALID, "null argument");
    if (pt->two_level) return fail(PUPIL_ERR_UNSUPPORTED, "only the flattened BVH4 is exported");
    HIP_TRY(hipSetDevice(pt->device));
    const uint32_t nn = pt->bvh.num_nodes4, nr = pt->bvh.num_records;
    if (nodes || records) {
        if (*num_nodes < nn || *num_records < nr) return fail(PUPIL_ERR_INVALID, "output too small");
        HIP_TRY(hipDeviceSynchronize());
        if (nodes && nn) HIP_TRY(hipMemcpy(nodes, pt->bvh.nodes4, sizeof(Bvh4Node) * nn, hipMemcpyDeviceToHost));
        if (records && nr) {  // record slots as 12 floats each (the 4th float4 of a slot is unused)
            std::vector<float4> h((size_t)kRecF4 * nr);
            HIP_TRY(hipMemcpy(h.data(), pt->bvh.prims, sizeof(float4) * h.size(), hipMemcpyDeviceToHost));
            for (size_t r = 0; r < nr; r++) std::memcpy(records + 12 * r, &h[kRecF4 * r], 3 * sizeof(float4));
        }
    }
    *num_nodes = nn;
    *num_records = nr;
    *root_link = (int32_t)pt->bvh.root_link4;
    return PUPIL_OK;
}

int pupil_pt_trace_rays(pupil_pt *pt, uint32_t n, const float *rays, float *out, int any_hit) {
    if (!pt || !rays || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    if (n == 0) return PUPIL_OK;
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(hipDeviceSynchronize());  // no render on another stream may still use the shared overflow stacks
    float *d_rays = nullptr, *d_out = nullptr;
    HIP_TRY(hipMalloc((void **)&d_rays, sizeof(float) * 8 * (size_t)n));
    hipError_t e = hipMalloc((void **)&d_out, sizeof(float) * 4 * (size_t)n);
    if (e == hipSuccess) e = hipMemcpy(d_rays, rays, sizeof(float) * 8 * (size_t)n, hipMemcpyHostToDevice);
    // PUPIL_TRACE_RAYS_STATS: the counter kernels (queue accounting, node visits), read back
    // by pupil_pt_stats like a collect_stats render's
    const bool stats = std::getenv("PUPIL_TRACE_RAYS_STATS") != nullptr;
    TraceStats ts{pt->trace_counters};
    if (e == hipSuccess) {
        e = hipMemsetAsync(pt->q.work + kWorkRays, 0, kWorkKind * sizeof(uint32_t), pt->own_stream);
        if (e == hipSuccess && stats) e = hipMemsetAsync(pt->trace_counters, 0, 32 * sizeof(unsigned long long), pt->own_stream);
        if (e == hipSuccess) e = hipEventRecord(pt->ev_begin, pt->own_stream);
        if (e == hipSuccess)
            launch_trace_debug(pt->sc, d_rays, d_out, n, any_hit, pt->ovf, pt->ovf_threads, pt->q.work + kWorkRays,
                               pt->own_stream, stats ? &ts : nullptr);
        if (e == hipSuccess) e = hipEventRecord(pt->ev_end, pt->own_stream);
        if (e == hipSuccess) e = hipStreamSynchronize(pt->own_stream);
    }
    if (e == hipSuccess && stats) {
        pt->last_paths = n;
        pt->last_iters = 0;
        pt->last_primary = n;
        pt->last_stats = true;
        pt->last_timed = true;
        pt->snap_taken = false;
        pt->trace_pairs = 0;
        for (int k = 0; k < 4; k++) pt->kept_ms[k] = 0.0, pt->kept_n[k] = 0;
        pt->rendered = true;
        pt->last_stream = pt->own_stream;
    }
    if (e == hipSuccess) e = hipMemcpy(out, d_out, sizeof(float) * 4 * (size_t)n, hipMemcpyDeviceToHost);
    (void)hipFree(d_rays);
    if (d_out) (void)hipFree(d_out);
    HIP_TRY(e);
    return PUPIL_OK;
}

int pupil_debug_select_emitter(pupil_pt *pt, uint32_t n, const float *p, int32_t *out) {
    if (!pt || !p || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    if (n == 0) return PUPIL_OK;
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(hipDeviceSynchronize());
    float *dp = nullptr;
    int *dout = nullptr;
    HIP_TRY(hipMalloc((void **)&dp, sizeof(float) * n));
    hipError_t err = hipMalloc((void **)&dout, sizeof(int) * n);
    if (err == hipSuccess) err = hipMemcpy(dp, p, sizeof(float) * n, hipMemcpyHostToDevice);
    if (err == hipSuccess) {
        launch_debug_select(pt->sc, dp, dout, n, pt->own_stream);
        err = hipStreamSynchronize(pt->own_stream);
    }
    if (err == hipSuccess) err = hipMemcpy(out, dout, sizeof(int) * n, hipMemcpyDeviceToHost);
    (void)hipFree(dp);
    if (dout) (void)hipFree(dout);
    HIP_TRY(err);
    return PUPIL_OK;
}

int pupil_debug_fill_tlas_reserve(pupil_pt *pt, float value) {
    if (!pt) return fail(PUPIL_ERR_INVALID, "null argument");
    if (!pt->two_level) return fail(PUPIL_ERR_UNSUPPORTED, "the flattened BVH has no TLAS reserve");
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(order_after_renders(pt));
    const uint64_t lo = pt->tl.tlas_nodes, hi = std::min<uint64_t>(pt->tl.tlas_cap, nodes4_count(pt));
    if (hi > lo) {
        std::vector<float> junk((hi - lo) * (sizeof(Bvh4Node) / sizeof(float)), value);
        HIP_TRY(hipMemcpyAsync((void *)(pt->sc.nodes4 + lo), junk.data(), sizeof(float) * junk.size(),
                               hipMemcpyHostToDevice, pt->own_stream));
        HIP_TRY(hipStreamSynchronize(pt->own_stream));
    }
    return refresh_node_bound(pt);
}

int pupil_debug_math(int device, uint32_t n, const float *x, const float *y2, float *out) {
    if (!x || !y2 || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(device));
    float *dx = nullptr, *dy = nullptr, *dout = nullptr;
    HIP_TRY(hipMalloc((void **)&dx, sizeof(float) * (n ? n : 1)));
    HIP_TRY(hipMalloc((void **)&dy, sizeof(float) * (n ? n : 1)));
    HIP_TRY(hipMalloc((void **)&dout, sizeof(float) * 6 * (n ? n : 1)));
    HIP_TRY(hipMemcpy(dx, x, sizeof(float) * n, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(dy, y2, sizeof(float) * n, hipMemcpyHostToDevice));
    launch_debug_math(dx, dy, dout, n, nullptr);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(out, dout, sizeof(float) * 6 * n, hipMemcpyDeviceToHost));
    (void)hipFree(dx);
    (void)hipFree(dy);
    (void)hipFree(dout);
    return PUPIL_OK;
}

}  // extern "C"
