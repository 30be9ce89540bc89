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
    uint32_t bvh_width = 4;  // flattened BVH node format (PUPIL_BVH_WIDTH)
    bool primary_interleave = true;  // primary extend dequeues pixel-major (PUPIL_PRIMARY_ORDER)
    bool shade_list = false;  // shade walks the traced list instead of a material partition (PUPIL_SHADE_LIST)
    TwoLevelAccel tl{};
    uint32_t width = 0, height = 0, max_depth = 1;
    uint32_t num_prims = 0;
    uint32_t leaf_size = 2;  // primitives per BVH leaf (PUPIL_LEAF_SIZE)
    bool mixed_trace = true;  // one persistent launch per bounce for shadow + extension rays (PUPIL_MIXED)
    // Render-ahead (PUPIL_AHEAD): the last mixed launch of a render also traces the
    // camera rays of the next render (seed + spp, same camera, tiling and batch), generated
    // into the other half of the path-state buffers, so the next render starts at its
    // first shade and the primary extend's launch tail is gone.  1 = single-spp renders
    // (the PTPass::OnRun cadence, pt_pass.cpp:39-57), 2 = every render, 0 = off.
    int ahead_mode = 1;
    bool ahead_valid = false;
    uint32_t ahead_seed = 0, ahead_spp = 0, ahead_local = 0, ahead_half = 0;
    uint32_t ahead_key[5] = {0, 0, 0, 0, 0};
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
    uint32_t *ray_log = nullptr;                   // per bounce: next, shadow
    uint32_t last_paths = 0, last_bounces = 0;
    bool last_stats = false;
    std::vector<hipEvent_t> trace_events;  // pairs
    std::vector<uint8_t> pair_kind;        // per pair: 0 extend, 1 shadow, 2 shade
    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    uint32_t trace_pairs = 0;
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
        void *bufs[] = {ps.ray_o, ps.ray_d, ps.hit,  ps.thr,  ps.rad,    ps.misc, ps.sh_o,
                        ps.sh_d, ps.sh_c, ps.mbin, ps.sflags, q.bins, q.nxsh, q.hist};
        for (void *b : bufs)
            if (b) (void)hipFree(b);
        ps = PathState{};
        q.bins = q.nxsh = q.hist = nullptr;
        cap = 0;
        ahead_valid = false;
    }
    ~pupil_pt() {
        (void)hipSetDevice(device);
        release_state();
        for (void *p : allocs) (void)hipFree(p);
        free_lbvh(bvh);
        free_two_level(tl);
        if (pixel_map) (void)hipFree(pixel_map);
        for (auto e : trace_events) (void)hipEventDestroy(e);
        if (ev_begin) (void)hipEventDestroy(ev_begin);
        if (ev_end) (void)hipEventDestroy(ev_end);
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

// EmitterGroup (render/emitter.h:110-135): area emitters, their sequential
// selection CDF and the env emitter; replaces the previous tables (updates).
int upload_emitters(pupil_pt *pt, const pupil_scene_desc *scene) {
    std::vector<DevEmitter> areas(scene->num_area_emitters);
    std::vector<float> cdf(scene->num_area_emitters);
    float sum_p = 0.f;
    for (uint32_t e = 0; e < scene->num_area_emitters; e++) {
        int rc = convert_emitter(pt, scene->area_emitters[e], areas[e]);
        if (rc) return rc;
        cdf[e] = sum_p + areas[e].select_probability;
        sum_p = cdf[e];
    }
    DevEmitter *d_areas = nullptr, *d_env = nullptr;
    float *d_cdf = nullptr;
    uint32_t *d_guide = nullptr;
    if (pt->upload(&d_areas, areas.data(), areas.size()) || pt->upload(&d_cdf, cdf.data(), cdf.size()))
        return fail(PUPIL_ERR_OOM, "emitter upload failed");
    // guide table: 2^bits >= emitter count buckets (at most 2^20), guide[k] = first i
    // with cdf[i] >= k / 2^bits (PUPIL_EMITTER_SELECT=binary: plain binary search, A/B)
    uint32_t bits = 0;
    while ((1u << bits) < scene->num_area_emitters && bits < 20) bits++;
    const char *sel = std::getenv("PUPIL_EMITTER_SELECT");
    const bool guide = scene->num_area_emitters > 1 && !(sel && std::strcmp(sel, "binary") == 0);
    if (guide) {
        const uint32_t m = 1u << bits;
        std::vector<uint32_t> g(m + 1);
        uint32_t i = 0;
        for (uint32_t k = 0; k <= m; k++) {
            const float t = (float)k / (float)m;
            while (i < cdf.size() && cdf[i] < t) i++;
            g[k] = i;
        }
        if (pt->upload(&d_guide, g.data(), g.size())) return fail(PUPIL_ERR_OOM, "emitter guide upload failed");
    }
    if (scene->env && scene->env->type != PUPIL_EMITTER_NONE) {
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
    HIP_TRY(hipMalloc((void **)&pt->ps.sh_o, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sh_d, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sh_c, sizeof(float4) * n));
    HIP_TRY(hipMalloc((void **)&pt->ps.mbin, n));
    HIP_TRY(hipMalloc((void **)&pt->ps.sflags, n));
    HIP_TRY(hipMalloc((void **)&pt->q.bins, sizeof(uint32_t) * n));
    HIP_TRY(hipMalloc((void **)&pt->q.nxsh, sizeof(uint32_t) * 2 * n));
    HIP_TRY(hipMalloc((void **)&pt->q.hist, sizeof(uint32_t) * partition_hist_entries((uint32_t)n)));
    pt->q.capacity = (uint32_t)n;
    pt->cap = n;
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

}  // namespace

extern "C" {

const char *pupil_last_error(void) { return g_last_error.c_str(); }
int pupil_abi_version(void) { return 2; }

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
    if (pt->upload(&d_insts, insts.data(), insts.size()) || pt->upload(&d_mats, mats.data(), mats.size()) ||
        pt->upload(&d_prim_inst, prim_inst.data(), prim_inst.size()))
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
    // the flattened primitive count would pass the flat build's 2^28 limit).  Both
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
        pt->two_level = flat_prims >= (1ull << 28);
        if (const char *a = std::getenv("PUPIL_ACCEL")) {
            if (std::strcmp(a, "flat") == 0) pt->two_level = false;
            if (std::strcmp(a, "two_level") == 0) pt->two_level = true;
        }
        if (!pt->two_level && flat_prims >= (1ull << 28))
            return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "flattened BVH limited to 2^28 primitives"));
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
            if (trc != 0) return cleanup(fail(PUPIL_ERR_HIP, "two-level acceleration build failed"));
            pt->build_ms = pt->tl.build_ms;
        } else {
            BvhBuildInput bin{pt->num_prims, d_prim_inst, d_insts, d_mats};
            if (const char *w = std::getenv("PUPIL_BVH_WIDTH"))  // node format: 4 (default), 8, or 2 (A/B)
                pt->bvh_width = (uint32_t)std::atoi(w) == 8 ? 8u : ((uint32_t)std::atoi(w) == 2 ? 2u : 4u);
            bin.wide8 = pt->bvh_width == 8 ? 1u : 0u;
            const int brc = build_bvh_bounded(bin, pt->bvh, pt->leaf_size, pt->own_stream, &pt->build_ms, 0);
            if (brc == -3) return cleanup(fail(PUPIL_ERR_UNSUPPORTED, "BVH deeper than the traversal stacks hold"));
            if (brc != 0) return cleanup(fail(PUPIL_ERR_HIP, "LBVH build failed"));
        }
    }
    pt->h_insts = insts;
    DeviceScene &sc = pt->sc;
    sc.num_prims = pt->num_prims;
    sc.bvh_width = 4;
    if (pt->two_level) {
        sc.two_level = 1;
        sc.nodes = nullptr;
        sc.root_link = (uint32_t)kTraverseDone;
        sc.tl_world = pt->tl.world ? 1u : 0u;
        sc.nodes4 = pt->tl.world ? pt->tl.wnodes : pt->tl.nodes4;
        sc.prims = pt->tl.world ? pt->tl.wprims : pt->tl.prims;
        sc.wprims = pt->tl.wprims;
        sc.attrs = pt->tl.attrs;
        sc.root_link4 = pt->tl.root_link4;
    } else {
        sc.nodes = pt->bvh.nodes;
        sc.prims = pt->bvh.prims;
        sc.attrs = pt->bvh.attrs;
        sc.root_link = pt->bvh.root_link;
        sc.nodes4 = pt->bvh.nodes4;
        sc.root_link4 = pt->bvh.root_link4;
        sc.nodes8 = pt->bvh.nodes8;
        sc.root_link8 = pt->bvh.root_link8;
        sc.bvh_width = pt->bvh_width;
    }
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, pt->device);
    sc.num_cus = (uint32_t)std::max(1, cus);
    // persistent BVH4 kernels: refill once 16 lanes are idle (r02 re-tune on the SAH tree:
    // 16 / 12 beat 20 / 24 by ~0.7 % at N = 1 and the 8-way shard; 0 = one-ray-per-lane A/B)
    sc.trace_refill = 16;
    if (const char *r = std::getenv("PUPIL_REFILL")) sc.trace_refill = (uint32_t)std::min(64, std::max(0, std::atoi(r)));
    if ((pt->two_level || sc.bvh_width == 8) && sc.trace_refill == 0) sc.trace_refill = 16;  // persistent kernels only
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
    }
    pt->mixed_trace = true;
    if (const char *m = std::getenv("PUPIL_MIXED")) pt->mixed_trace = std::atoi(m) != 0;
    if (const char *a = std::getenv("PUPIL_AHEAD")) pt->ahead_mode = std::min(2, std::max(0, std::atoi(a)));
    sc.trace_node_min = 8;  // node phase ends below 8 active lanes (7 waves: 8 and 12 beat 4 by 1.5 %; 2 is slower)
    if (const char *r = std::getenv("PUPIL_NODE_MIN")) sc.trace_node_min = (uint32_t)std::min(64, std::max(1, std::atoi(r)));
    sc.prim_inst = d_prim_inst;
    sc.instances = d_insts;
    sc.materials = d_mats;
    std::memcpy(sc.camera.s2c, scene->sample_to_camera, sizeof(sc.camera.s2c));
    std::memcpy(sc.camera.c2w, scene->camera_to_world, sizeof(sc.camera.c2w));
    // traversal overflow stacks, counters, events
    pt->ovf_threads = trace_grid_blocks() * (uint32_t)kTraceBlock;
    if (pt->alloc(&pt->ovf, (size_t)pt->ovf_threads * kStackOvf) || pt->alloc(&pt->trace_counters, 32) ||
        pt->alloc(&pt->ray_log, 2 * 130) || pt->alloc(&pt->q.counts, kCountSlots) ||
        pt->alloc(&pt->q.work, kWorkSlots))
        return cleanup(fail(PUPIL_ERR_OOM, "workspace allocation failed"));
    if (hipMemset(pt->q.work, 0, kWorkSlots * sizeof(uint32_t)) != hipSuccess)
        return cleanup(fail(PUPIL_ERR_HIP, "workspace clear failed"));
    if (hipEventCreate(&pt->ev_begin) != hipSuccess || hipEventCreate(&pt->ev_end) != hipSuccess)
        return cleanup(fail(PUPIL_ERR_HIP, "event creation failed"));
    pt->totals.bvh_nodes = pt->two_level ? two_level_nodes(pt->tl)
                           : (pt->sc.bvh_width == 8 ? pt->bvh.num_nodes8
                                                    : (pt->sc.bvh_width == 4 ? pt->bvh.num_nodes4 : pt->bvh.num_nodes));
    pt->totals.two_level = pt->two_level ? 1u : 0u;
    pt->totals.bvh_depth = pt->two_level ? pt->tl.tlas_depth + pt->tl.blas_depth
                                         : (pt->sc.bvh_width == 8 ? pt->bvh.depth8 : pt->bvh.depth4);
    pt->totals.bvh_prims = pt->num_prims;
    pt->totals.build_ms = pt->build_ms;
    *out = pt;
    return PUPIL_OK;
}

int pupil_pt_set_camera(pupil_pt *pt, const float sample_to_camera[16], const float camera_to_world[16]) {
    if (!pt || !sample_to_camera || !camera_to_world) return fail(PUPIL_ERR_INVALID, "null argument");
    if (std::memcmp(pt->sc.camera.s2c, sample_to_camera, sizeof(pt->sc.camera.s2c)) != 0 ||
        std::memcmp(pt->sc.camera.c2w, camera_to_world, sizeof(pt->sc.camera.c2w)) != 0)
        pt->ahead_valid = false;  // the render-ahead camera rays belong to the old view
    std::memcpy(pt->sc.camera.s2c, sample_to_camera, sizeof(pt->sc.camera.s2c));
    std::memcpy(pt->sc.camera.c2w, camera_to_world, sizeof(pt->sc.camera.c2w));
    return PUPIL_OK;
}

// RenderInstanceUpdate (ias_manager.cpp:116-151): new instance transform, then
// the acceleration structure is rebuilt over the updated world-space primitives
// (LBVH build, ~8 ms per 1M primitives); the render after it is identical to a
// render of a freshly created engine.  Emitters follow with pupil_pt_update_emitters.
int pupil_pt_update_instance(pupil_pt *pt, uint32_t instance, const float to_world[12], const float to_object[12]) {
    if (!pt || !to_world || !to_object) return fail(PUPIL_ERR_INVALID, "null argument");
    if (instance >= pt->h_insts.size()) return fail(PUPIL_ERR_INVALID, "instance index out of range");
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(hipDeviceSynchronize());  // no render may still read the old tables
    pt->ahead_valid = false;          // render-ahead hits were traced against the old geometry
    DevInstance &d = pt->h_insts[instance];
    std::memcpy(d.to_world, to_world, sizeof(d.to_world));
    std::memcpy(d.to_object, to_object, sizeof(d.to_object));
    if (pt->two_level) refresh_instance_margins(d);  // they depend on the transform
    HIP_TRY(hipMemcpy(pt->d_insts + instance, &d, sizeof(DevInstance), hipMemcpyHostToDevice));
    if (pt->two_level) {  // new world box for the instance, TLAS rebuilt over all instance boxes
        const auto t0 = std::chrono::steady_clock::now();
        // world mode refits the TLAS like the reference's IAS update (PUPIL_TL_UPDATE=rebuild: full build)
        const char *um = std::getenv("PUPIL_TL_UPDATE");
        const bool refit = !(um && std::strcmp(um, "rebuild") == 0);
        const int trc = rebuild_tlas(pt->tl, pt->h_insts, pt->d_insts, {instance}, pt->own_stream, refit);
        if (trc == -3) return fail(PUPIL_ERR_UNSUPPORTED, "TLAS + BLAS deeper than the traversal stacks hold");
        if (trc != 0) return fail(PUPIL_ERR_HIP, "TLAS rebuild failed");
        pt->sc.root_link4 = pt->tl.root_link4;
        pt->totals.bvh_nodes = two_level_nodes(pt->tl);
        pt->totals.bvh_depth = pt->tl.tlas_depth + pt->tl.blas_depth;
        pt->totals.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return PUPIL_OK;
    }
    BvhBuildInput bin{pt->num_prims, pt->d_prim_inst, pt->d_insts, pt->d_mats};
    bin.wide8 = pt->sc.bvh_width == 8 ? 1u : 0u;
    // refit in place (PUPIL_FLAT_UPDATE=rebuild, or the BVH2 / BVH8 node formats: full rebuild)
    const char *fu = std::getenv("PUPIL_FLAT_UPDATE");
    if (pt->sc.bvh_width == 4 && !(fu && std::strcmp(fu, "rebuild") == 0)) {
        double rms = 0.0;
        if (refit_bvh4(bin, pt->bvh, instance, pt->own_stream, &rms) == 0) {
            pt->totals.build_ms = rms;
            return PUPIL_OK;
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
    pt->sc.nodes = nb.nodes;
    pt->sc.prims = nb.prims;
    pt->sc.attrs = nb.attrs;
    pt->sc.root_link = nb.root_link;
    pt->sc.nodes4 = nb.nodes4;
    pt->sc.root_link4 = nb.root_link4;
    pt->sc.nodes8 = nb.nodes8;
    pt->sc.root_link8 = nb.root_link8;
    pt->totals.bvh_nodes = pt->sc.bvh_width == 8 ? nb.num_nodes8 : (pt->sc.bvh_width == 4 ? nb.num_nodes4 : nb.num_nodes);
    pt->totals.bvh_depth = pt->sc.bvh_width == 8 ? nb.depth8 : nb.depth4;
    pt->totals.build_ms = ms;
    return PUPIL_OK;
}

// EmitterHelper reset after a transform change (world/world.cpp:45-54): the area
// emitter table, selection CDF and env emitter are replaced by the scene's.
int pupil_pt_update_emitters(pupil_pt *pt, const pupil_scene_desc *scene) {
    if (!pt || !scene) return fail(PUPIL_ERR_INVALID, "null argument");
    if (scene->num_area_emitters && !scene->area_emitters) return fail(PUPIL_ERR_INVALID, "missing emitter array");
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(hipDeviceSynchronize());
    pt->ahead_valid = false;
    return upload_emitters(pt, scene);
}

int pupil_pt_render(pupil_pt *pt, const pupil_pt_frame *out, const pupil_pt_launch *launch, void *hip_stream) {
    if (!pt || !out || !launch || !out->accum) return fail(PUPIL_ERR_INVALID, "null argument");
    if (launch->spp == 0) return PUPIL_OK;
    // PTPass clamps the inspector's max_depth to 1..128 (pt_pass.cpp:225-237); the
    // per-bounce ray log and the stage-event list are sized for that range
    if ((launch->max_depth ? launch->max_depth : pt->max_depth) > kMaxDepth)
        return fail(PUPIL_ERR_INVALID, "max_depth above 128");
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
    const uint32_t depth = launch->max_depth ? launch->max_depth : pt->max_depth;
    // render-ahead: use the camera rays the previous render traced for this one, and
    // trace the next render's in this one's last mixed launch (BVH4 persistent kernels;
    // counter renders keep their own primary launch so the counters stay per render)
    const bool use_ahead = pt->ahead_valid && !stats && launch->random_seed == pt->ahead_seed && launch->spp == pt->ahead_spp &&
                           num_local == pt->ahead_local && std::memcmp(key, pt->ahead_key, sizeof(key)) == 0;
    const bool make_ahead = pt->ahead_mode != 0 &&
                            (pt->ahead_mode == 2 || launch->spp == 1 || (launch->hints & PUPIL_HINT_CONTINUE)) && !stats &&
                            depth >= 2 && pt->mixed_trace && pt->sc.bvh_width == 4 && pt->sc.trace_refill != 0 &&
                            paths < (1ull << 30);
    pt->ahead_valid = false;
    if (pt->rendered && s != pt->last_stream) HIP_TRY(hipStreamWaitEvent(s, pt->ev_end, 0));
    const size_t cap_before = pt->cap;
    int rc = ensure_state(pt, paths * (use_ahead || make_ahead ? 2 : 1));
    if (rc) return rc;
    const uint32_t half = use_ahead && pt->cap == cap_before ? pt->ahead_half : 0u;
    const bool ahead_in = use_ahead && pt->cap == cap_before;
    auto view = [&](uint32_t h) {  // path state of half h: every array offset by h * paths
        PathState v = pt->ps;
        const size_t o = (size_t)h * paths;
        v.ray_o += o, v.ray_d += o, v.hit += o, v.thr += o, v.rad += o, v.misc += o;
        v.sh_o += o, v.sh_d += o, v.sh_c += o, v.mbin += o, v.sflags += o;
        return v;
    };
    const PathState ps = view(half);

    FrameParams fp{};
    fp.width = pt->width;
    fp.height = pt->height;
    fp.num_local = num_local;
    fp.num_paths = (uint32_t)paths;
    fp.spp = launch->spp;
    fp.seed0 = launch->random_seed;
    fp.cnt0 = launch->sample_cnt;
    fp.accumulate = launch->accumulate;
    fp.max_depth = launch->max_depth ? launch->max_depth : pt->max_depth;
    fp.compact = out->compact;
    fp.pixel_map = map;
    fp.accum = (float4 *)out->accum;
    fp.frame = (float4 *)out->frame;
    fp.albedo = (float *)out->albedo;
    fp.normal = (float *)out->normal;
    fp.test = (float *)out->test;
    fp.nee_count = stats ? pt->trace_counters + 16 : nullptr;

    TraceStats ts_dev{pt->trace_counters};
    const TraceStats *tsp = stats ? &ts_dev : nullptr;
    const bool tail = stats && std::getenv("PUPIL_TRACE_TAIL");
    if (tail && !pt->tail_buf) {
        pt->tail_waves = pt->ovf_threads / 64u;
        if (pt->alloc(&pt->tail_buf, (size_t)(kMaxDepth + 1) * pt->tail_waves * 4)) return fail(PUPIL_ERR_OOM, "tail buffer");
    }
    if (tail) HIP_TRY(hipMemsetAsync(pt->tail_buf, 0, sizeof(unsigned long long) * (kMaxDepth + 1) * pt->tail_waves * 4, s));
    pt->tail_launches = 0;
    auto tail_slot = [&]() {  // wave-time slice of the next traversal launch
        if (tail) ts_dev.wave_times = pt->tail_buf + (size_t)pt->tail_launches++ * pt->tail_waves * 4;
    };
    const uint32_t bounces = fp.max_depth;
    // events: begin/end + one pair per stage launch (kind 0 extend, 1 shadow, 2 shade)
    const uint32_t pairs_needed = 3 * bounces + 1;
    while (pt->trace_events.size() < 2 * pairs_needed) {
        hipEvent_t e;
        HIP_TRY(hipEventCreate(&e));
        pt->trace_events.push_back(e);
    }
    pt->pair_kind.assign(pairs_needed, 0);
    uint32_t pair = 0;
    // stage events only on request: each hipEventRecord between two kernels costs
    // ~6 us of stream gap (9 per 1-spp render at D = 4)
    auto ev0 = [&](uint8_t kind) {
        if (!timing) return;
        pt->pair_kind[pair] = kind;
        (void)hipEventRecord(pt->trace_events[2 * pair], s);
    };
    auto ev1 = [&]() {
        if (!timing) return;
        (void)hipEventRecord(pt->trace_events[2 * pair + 1], s);
        pair++;
    };

    HIP_TRY(hipEventRecord(pt->ev_begin, s));
    if (stats) HIP_TRY(hipMemsetAsync(pt->trace_counters, 0, 32 * sizeof(unsigned long long), s));
    const uint32_t np = fp.num_paths;
    Queues &q = pt->q;
    // material bins of the traced paths -> q.bins (stable, increasing path id)
    auto bin_paths = [&]() {
        launch_partition(ps.mbin, np, kPartMaxBins, kPartExclusive, 0u, q.bins, q.hist, q.counts,
                         q.counts + kStartBins, q.counts + kScratch, nullptr, s);
    };
    // No per-stage clears: the primary extend writes every path's material bin,
    // each shade writes its paths' flags (with the bounce tag) and resets their
    // bin to 0xFF, the persistent kernels reset their own work heads, and the
    // flags partition logs the per-bounce ray counts.
    const uint32_t interleave = pt->primary_interleave && fp.spp > 1 ? fp.spp : 0u;
    if (!ahead_in) {  // else the previous render traced this one's camera rays (render-ahead)
        launch_generate(pt->sc, fp, ps, s);
        ev0(0);
        tail_slot();
        // camera rays: the spp samples of a pixel on consecutive lanes (PUPIL_PRIMARY_ORDER=path: path order)
        launch_extend(pt->sc, ps, q, nullptr, nullptr, np, pt->ovf, pt->ovf_threads, tsp, s, interleave, fp.num_local);
        ev1();
    }
    if (!pt->shade_list) bin_paths();
    for (uint32_t b = 0; b < bounces; b++) {
        const uint32_t tag = sflag_tag(fp.max_depth, b);
        if (tag == 0) HIP_TRY(hipMemsetAsync(ps.sflags, 0, np, s));
        ev0(2);
        launch_shade(pt->sc, fp, ps, q, b, s, !pt->shade_list ? kShadeBins : (b == 0 ? kShadeAll : kShadeNext));
        ev1();
        if (b + 1 < bounces) {  // the last shade never spawns shadow or extension rays
            // next (bit 0) and shadow (bit 1) lists -> q.nxsh, each in increasing path order
            // (grouping the next list by direction octant measured slower: 21.2 vs 20.8 ms extend)
            launch_partition(ps.sflags, np, 2, kPartFlags, tag, q.nxsh, q.hist, q.counts + kCntNext,
                             q.counts + kStartNext, nullptr, b < 128 ? pt->ray_log + 2 * b : nullptr, s);
            if (pt->mixed_trace && pt->sc.bvh_width >= 4 && pt->sc.trace_refill) {
                // render-ahead: the last mixed launch also traces the next render's camera rays,
                // generated into the other half of the buffers (seed + spp, this camera and tiling)
                const bool ahead_out = make_ahead && b + 2 == bounces;
                if (ahead_out) {
                    FrameParams fa = fp;
                    fa.seed0 = fp.seed0 + fp.spp;
                    launch_generate(pt->sc, fa, view(half ^ 1u), s);
                }
                ev0(1);
                tail_slot();
                if (ahead_out)  // addressed from the base of both halves (offsets stay non-negative)
                    launch_trace_mixed(pt->sc, pt->ps, q, pt->ovf, pt->ovf_threads, tsp, s, np, half * np,
                                       (half ^ 1u) * np, interleave, fp.num_local);
                else
                    launch_trace_mixed(pt->sc, ps, q, pt->ovf, pt->ovf_threads, tsp, s);
                ev1();
                if (ahead_out) {
                    pt->ahead_valid = true;
                    pt->ahead_seed = fp.seed0 + fp.spp;
                    pt->ahead_spp = fp.spp;
                    pt->ahead_local = num_local;
                    pt->ahead_half = half ^ 1u;
                    std::memcpy(pt->ahead_key, key, sizeof(key));
                }
            } else {
                ev0(1);
                launch_shadow(pt->sc, ps, q, pt->ovf, pt->ovf_threads, tsp, s);
                ev1();
                ev0(0);
                launch_extend(pt->sc, ps, q, q.nxsh, q.counts + kCntNext, 0u, pt->ovf, pt->ovf_threads, tsp, s);
                ev1();
            }
            if (!pt->shade_list) bin_paths();
        }
    }
    launch_accumulate(fp, ps, s);
    HIP_TRY(hipEventRecord(pt->ev_end, s));
    HIP_TRY(hipGetLastError());
    pt->trace_pairs = pair;
    pt->last_paths = fp.num_paths;
    pt->last_bounces = bounces < 129 ? bounces : 129;  // rays are logged for bounces 0..127
    pt->last_stats = stats;
    pt->last_stream = s;
    pt->rendered = true;
    return PUPIL_OK;
}

int pupil_pt_stats(pupil_pt *pt, pupil_pt_counters *out) {
    if (!pt || !out) return fail(PUPIL_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(pt->device));
    HIP_TRY(hipEventSynchronize(pt->ev_end));
    pupil_pt_counters c = pt->totals;
    if (pt->last_paths) {
        std::vector<uint32_t> log(2 * 130, 0);
        HIP_TRY(hipMemcpy(log.data(), pt->ray_log, sizeof(uint32_t) * log.size(), hipMemcpyDeviceToHost));
        c.primary_rays = pt->last_paths;
        c.path_samples = pt->last_paths;
        c.extension_rays = 0;
        c.shadow_rays = 0;
        for (uint32_t b = 0; b + 1 < pt->last_bounces; b++) {  // the last bounce spawns no rays
            c.extension_rays += log[2 * b];
            c.shadow_rays += log[2 * b + 1];
        }
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, pt->ev_begin, pt->ev_end));
        c.last_render_ms = ms;
        double kind_ms[3] = {0.0, 0.0, 0.0};
        uint64_t kind_n[3] = {0, 0, 0};
        for (uint32_t i = 0; i < pt->trace_pairs; i++) {
            float m = 0.f;
            HIP_TRY(hipEventElapsedTime(&m, pt->trace_events[2 * i], pt->trace_events[2 * i + 1]));
            kind_ms[pt->pair_kind[i]] += m;
            kind_n[pt->pair_kind[i]]++;
        }
        c.trace_ms = kind_ms[0] + kind_ms[1];
        c.trace_launches = kind_n[0] + kind_n[1];
        c.extend_ms = kind_ms[0];
        c.extend_launches = kind_n[0];
        c.shade_ms = kind_ms[2];
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
            for (int k = 0; k < 2 && std::getenv("PUPIL_TRACE_DIAG"); k++) {  // SIMD efficiency, persistent kernels
                const unsigned long long *d = tc + 2 + 6 * k;
                if (!d[0]) continue;
                std::fprintf(stderr,
                             "[pupil] %s: node loop %llu wave-iters, %.1f%% lanes active; leaf loop %llu wave-iters, "
                             "%.1f%% lanes active; %llu refills, %.1f lanes each\n",
                             k ? "shadow" : "extend", d[0], 100.0 * (double)d[1] / (64.0 * (double)d[0]), d[2],
                             100.0 * (double)d[3] / (64.0 * (double)std::max(1ull, d[2])), d[4],
                             (double)d[5] / (double)std::max(1ull, d[4]));
            }
            c.node_visits = tc[0] + tc[14];
            c.prim_tests = tc[1] + tc[15];
            c.shadow_rays_reference = tc[16];
            c.unique_node_fetches = tc[18];
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
    if (pt->two_level || pt->sc.bvh_width != 4) return fail(PUPIL_ERR_UNSUPPORTED, "only the flattened BVH4 is exported");
    HIP_TRY(hipSetDevice(pt->device));
    const uint32_t nn = pt->bvh.num_nodes4, nr = pt->bvh.num_records;
    if (nodes || records) {
        if (*num_nodes < nn || *num_records < nr) return fail(PUPIL_ERR_INVALID, "output too small");
        HIP_TRY(hipDeviceSynchronize());
        if (nodes && nn) HIP_TRY(hipMemcpy(nodes, pt->bvh.nodes4, sizeof(Bvh4Node) * nn, hipMemcpyDeviceToHost));
        if (records && nr) HIP_TRY(hipMemcpy(records, pt->bvh.prims, sizeof(float4) * 3 * (size_t)nr, hipMemcpyDeviceToHost));
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
    if (e == hipSuccess) {
        e = hipMemsetAsync(pt->q.work + kWorkRays, 0, kWorkKind * sizeof(uint32_t), pt->own_stream);
        if (e == hipSuccess)
            launch_trace_debug(pt->sc, d_rays, d_out, n, any_hit, pt->ovf, pt->ovf_threads, pt->q.work + kWorkRays,
                               pt->own_stream);
        e = hipStreamSynchronize(pt->own_stream);
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
