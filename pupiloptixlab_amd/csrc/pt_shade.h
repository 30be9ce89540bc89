// pt_shade.h — per-path device code of the wavefront shading stages (camera ray, hit
// reconstruction, emitter selection, the per-material shade and the miss shade), shared by the
// stage kernels (pt_kernels.hip) and the persistent small-frame kernel (pt_frame.hip).
#pragma once

#include "pt_kernels.h"
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

namespace pupil {
namespace {

using namespace tr;

// __raygen__main's camera ray (main.cu:53-75): path p of a batch whose first frame has
// seed seed0 (sample p / num_local, local pixel p % num_local); the RNG is initialised
// from (pixel, seed) and the film jitter drawn x first.  Returns the RNG after the two
// draws, the pixel, and the normalised world direction (the origin is the camera's).
__device__ __forceinline__ uint32_t camera_path(const Camera &cam, uint32_t width, uint32_t height,
                                                const uint32_t *pixel_map, uint32_t num_local, uint32_t seed0,
                                                uint32_t p, uint32_t &pixel, vec3 &dir) {
    const uint32_t s = p / num_local;
    const uint32_t l = p - s * num_local;
    pixel = pixel_map ? pixel_map[l] : l;
    uint32_t rng = rng_init(pixel, seed0 + s);  // main.cu:53
    const float jx = rng_next(rng);             // main.cu:55 (x drawn first)
    const float jy = rng_next(rng);
    const uint32_t y = pixel / width;
    const uint32_t x = pixel - y * width;
    const vec4 film = v4(((float)x + jx) / (float)width, ((float)y + jy) / (float)height, 0.f, 1.f);
    const float *m = cam.s2c;
    vec4 d = v4(dot(v4(m[0], m[1], m[2], m[3]), film), dot(v4(m[4], m[5], m[6], m[7]), film),
                dot(v4(m[8], m[9], m[10], m[11]), film), dot(v4(m[12], m[13], m[14], m[15]), film));
    const float inv_w = 1.0f / d.w;
    d = v4(d.x * inv_w, d.y * inv_w, d.z * inv_w, d.w * inv_w);
    d.w = 0.f;
    d = normalize(d);
    const float *c = cam.c2w;
    dir = normalize(v3(dot(v4(c[0], c[1], c[2], c[3]), d), dot(v4(c[4], c[5], c[6], c[7]), d),
                       dot(v4(c[8], c[9], c[10], c[11]), d)));
    return rng;
}


// ------------------------------------------------------------------ generate
__device__ __forceinline__ uint32_t global_pixel(const FrameParams &fp, uint32_t l) {
    return fp.pixel_map ? fp.pixel_map[l] : l;
}

// A fresh path's RNG after the camera ray's two draws (main.cu:53-55): path p of a batch whose
// first frame has seed seed0 (sample p / num_local, local pixel p % num_local)
// a fresh path's RNG after the camera draws and its camera ray direction (camera_path)
__device__ __forceinline__ uint32_t fresh_path(const DeviceScene &sc, const FrameParams &fp, uint32_t p, uint32_t seed0,
                                               vec3 &dir) {
    uint32_t pixel;
    return camera_path(sc.camera, fp.width, fp.height, fp.pixel_map, fp.num_local, seed0, p, pixel, dir);
}
// the RNG alone (main.cu:53-55: the two film draws follow the init)
__device__ __forceinline__ uint32_t fresh_rng_of(const FrameParams &fp, uint32_t p, uint32_t seed0) {
    const uint32_t s = p / fp.num_local;
    const uint32_t l = p - s * fp.num_local;
    uint32_t rng = rng_init(fp.pixel_map ? fp.pixel_map[l] : l, seed0 + s);
    (void)rng_next(rng);
    (void)rng_next(rng);
    return rng;
}

struct HitGeo {
    LocalGeo g;
    int emitter;
    uint32_t inst;
};

// __closesthit__default (main.cu:216-230) + Geometry::GetHitLocalGeometry
// (render/geometry.h:272-320), from the compact hit record and the primitive's
// shading record (bvh_build.hip k_attrs: object-space vertices, normals, uvs).
// ro_rec: the ray origin record, read only for a sphere hit (the triangle position is
// interpolated from the vertices)
__device__ __forceinline__ HitGeo reconstruct(const DeviceScene &sc, float4 h, const float4 *ro_rec, bool fresh,
                                             vec3 rd, vec2 stale_uv) {
    HitGeo out;
    const uint32_t idx = __float_as_uint(h.w);
    // flat: idx = record in traversal order, which names the instance; two-level:
    // idx = global primitive id -> instance -> the shape's record in primitive order
    uint32_t inst_id, gprim;
    bool sphere;
    const float4 *rec;
    float4 ra[7];  // the shading record (one 128-B line)
    if (sc.two_level) {
        gprim = idx;
        inst_id = inst_of_prim(sc, idx);
        const DevInstance &ti = sc.instances[inst_id];
        sphere = ti.kind == PUPIL_SHAPE_SPHERE;
        rec = sc.attrs + (size_t)kAttrStride * (sphere ? 0u : ti.attr_base + (idx - ti.prim_offset));
        for (int k = 0; k < 7; k++) ra[k] = rec[k];
    } else {
        rec = sc.attrs + (size_t)kAttrStride * idx;
        // the whole line in one round trip, with the instance: without the barrier the
        // compiler sinks the normal / texcoord loads below the instance's flags, a second
        // dependent fetch per hit
        for (int k = 0; k < 7; k++) ra[k] = rec[k];
        asm volatile("" ::"v"(ra[0].x), "v"(ra[0].y), "v"(ra[0].z), "v"(ra[0].w), "v"(ra[1].x), "v"(ra[1].y),
                     "v"(ra[1].z), "v"(ra[1].w), "v"(ra[2].x), "v"(ra[2].y), "v"(ra[2].z), "v"(ra[2].w), "v"(ra[3].x),
                     "v"(ra[3].y));
        asm volatile("" ::"v"(ra[3].z), "v"(ra[3].w), "v"(ra[4].x), "v"(ra[4].y), "v"(ra[4].z), "v"(ra[4].w),
                     "v"(ra[5].x), "v"(ra[5].y), "v"(ra[5].z), "v"(ra[5].w), "v"(ra[6].x), "v"(ra[6].y));
        const uint32_t ref = __float_as_uint(ra[0].w);
        gprim = ref & ~kPrimSphereBit;
        sphere = (ref & kPrimSphereBit) != 0u;
        inst_id = __float_as_uint(ra[1].w);
    }
    const DevInstance &in = sc.instances[inst_id];
    out.inst = inst_id;
    LocalGeo &g = out.g;
    g.texcoord = stale_uv;
    uint32_t local = 0;
    if (sphere) {
        // a fresh path's ray is a camera ray, whose origin k_generate does not store
        const vec3 ro = fresh ? camera_origin(sc.camera) : f3(ld_ps(ro_rec));
        g.position = ro + h.x * rd;
        const vec3 local_pos = xform_point(in.to_object, g.position);
        g.texcoord = sphere_texcoord(normalize(local_pos - v3(0.f)));
        g.normal = normalize(xform_normal(in.to_object, local_pos - v3(0.f)));
        if (in.flip_normals) g.normal = g.normal * -1.f;
    } else {
        local = gprim - in.prim_offset;
        const float4 a = ra[0];
        const float4 b = ra[1];
        const float4 c = ra[2];
        const vec3 p0 = v3(a.x, a.y, a.z);
        const vec3 p1 = v3(b.x, b.y, b.z);
        const vec3 p2 = v3(c.x, c.y, c.z);
        const float u = h.y, v = h.z;
        const float w = 1.f - u - v;
        g.position = w * p0 + u * p1 + v * p2;
        g.position = xform_point(in.to_world, g.position);
        vec3 n;
        if (in.normals) {
            const float4 d = ra[3], e = ra[4];
            const vec3 n0 = v3(c.w, d.x, d.y);
            const vec3 n1 = v3(d.z, d.w, e.x);
            const vec3 n2 = v3(e.y, e.z, e.w);
            n = w * n0 + u * n1 + v * n2;
        } else {
            n = cross(p1 - p0, p2 - p0);
        }
        g.normal = normalize(xform_normal(in.to_object, n));
        if (in.flip_normals) g.normal = g.normal * -1.f;
        if (in.texcoords) {
            const float4 t01 = ra[5], t2 = ra[6];
            const vec2 t0 = v2(t01.x, t01.y);
            const vec2 t1 = v2(t01.z, t01.w);
            const vec2 tt2 = v2(t2.x, t2.y);
            g.texcoord = w * t0 + u * t1 + v * tt2;
            if (in.flip_tex_coords) g.texcoord.y = 1.f - g.texcoord.y;
        }
    }
    out.emitter = in.emitter_offset >= 0 ? in.emitter_offset + (int)local : -1;
    return out;
}

// EmitterGroup::SelectOneEmiiter (render/emitter.h:110-135) as a binary search
// over the sequentially accumulated CDF: picks the same emitter as the scan.
// SelectOneEmiiter (render/emitter.h:110-135): the first area emitter i with
// p <= cdf[i] (the linear scan's sum_p + select_probability, accumulated in the same
// order), else the env emitter, else the last area emitter.  The guide table narrows
// the search to the bucket of p (expected O(1) for any emitter count); the binary
// search over that range returns exactly the linear scan's index.
__device__ __forceinline__ const DevEmitter *select_emitter(const DeviceScene &sc, float p, float &sel_prob) {
    uint32_t lo = 0, hi = sc.num_areas;
    if (sc.area_guide) {
        const uint32_t m = 1u << sc.guide_bits;
        const uint32_t k = min((uint32_t)(p * (float)m), m - 1u);  // exact: m is a power of two <= 2^24
        lo = sc.area_guide[k];
        hi = sc.area_guide[k + 1];
    }
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (p <= sc.area_cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    const DevEmitter *e = nullptr;
    if (lo < sc.num_areas) e = &sc.areas[lo];
    else if (sc.has_env) e = sc.env;
    else if (sc.num_areas > 0) e = &sc.areas[sc.num_areas - 1];
    sel_prob = e ? e->select_probability : 0.f;
    return e;
}

// One path that hit a surface of material MAT (0 = unknown type): emission and
// MIS at the hit, loop head, NEE sample, BSDF sample (main.cu:84-163).
// Returns the next/shadow flags byte (bit 0 extension ray, bit 1 shadow ray).
// p: path id (in a pipelined ring: slot * num_paths + sample * num_local + local pixel);
// its bounce is PathState::misc.y (loaded inside shade_hit / shade_miss: passing the
// record in from the launch kept it live across the whole shade, 137 instead of 123
// VGPRs, one wave less per SIMD).
// Last sample of its frame, and the local pixel (AOVs are written for the last sample);
// `frame_off`: the AOV offset of the sample's frame within a ring slot's frame group.
__device__ __forceinline__ bool last_sample(const FrameParams &fp, uint32_t p, uint32_t &l, uint32_t &frame_off) {
    const uint32_t q = p / fp.num_local;
    l = p - q * fp.num_local;
    const uint32_t s = q / fp.spp;  // frame (of the ring) the sample belongs to
    frame_off = fp.aov_frame_stride ? (s % fp.group) * fp.aov_frame_stride : 0u;
    return q - s * fp.spp + 1u == fp.spp;
}

// fresh: a path of the frame generated for this launch (bounce 0, throughput 1, radiance 0,
// RNG `fresh_rng`; k_generate stored only its camera ray)
template <uint32_t MAT>
__device__ __forceinline__ uint32_t shade_hit(const DeviceScene &sc, const FrameParams &fp, const PathState &ps,
                                              uint32_t p, bool fresh, uint32_t fresh_p, uint32_t fresh_seed0) {
    bool push_next = false, push_shadow = false;
    const float4 h = ld_ps(ps.hit + p);
    const vec3 ray_d = f3(ld_ps(ps.ray_d + p));
    // a fresh path's RNG after its camera draws, recomputed (k_generate stored only the ray)
    const uint32_t fresh_rng = fresh ? fresh_rng_of(fp, fresh_p, fresh_seed0) : 0u;
    const uint4 misc = fresh ? make_uint4(fresh_rng, 0u, 0u, 0u) : ld_ps(ps.misc + p);
    uint32_t rng = misc.x;
    const uint32_t flags = misc.y;
    const uint32_t bounce = flags & 0xFFFFFFu;
    float4 thr4 = fresh ? make_float4(1.f, 1.f, 1.f, 0.f) : ld_ps(ps.thr + p);
    vec3 T = f3(thr4);
    const float prev_pdf = thr4.w;
    // the radiance record is read only when this hit adds emission (at most one addition per
    // shade, so L + X is the same sum whenever it is formed): most shades never touch it
    vec3 L_add = v3(0.f);
    const vec2 stale_uv = v2(__uint_as_float(misc.z), __uint_as_float(misc.w));

    HitGeo hg = reconstruct(sc, h, ps.ray_o + p, fresh, ray_d, stale_uv);
    const DevInstance &in = sc.instances[hg.inst];
    const DevMaterial &mat = sc.materials[in.material];
    if (mat.twosided && dot(-ray_d, hg.g.normal) < 0.f) hg.g.normal = -hg.g.normal;  // geometry.h:316-320
    const LocalGeo &geo = hg.g;
    LocalBsdf bsdf = local_bsdf(mat, geo.texcoord);
    bsdf.type = MAT;

    bool alive = true;
    bool L_changed = fresh;  // rad is rewritten only when this hit adds emission (or was never stored)
    if (bounce == 0) {
        if (hg.emitter >= 0) {  // main.cu:88-92
            L_add = emitter_radiance(sc.areas[hg.emitter], geo.texcoord);
            L_changed = true;
        }
        const float test = rng_next(rng);                                                    // main.cu:101
        uint32_t l;
        uint32_t fo;
        if (last_sample(fp, p, l, fo)) {
            const uint32_t out = fp.aov_local ? l : global_pixel(fp, l);
            if (fp.albedo) {
                const vec3 al = bsdf_albedo(bsdf);
                fp.albedo[fo + 3 * out + 0] = al.x;
                fp.albedo[fo + 3 * out + 1] = al.y;
                fp.albedo[fo + 3 * out + 2] = al.z;
            }
            if (fp.normal) {
                fp.normal[fo + 3 * out + 0] = geo.normal.x;
                fp.normal[fo + 3 * out + 1] = geo.normal.y;
                fp.normal[fo + 3 * out + 2] = geo.normal.z;
            }
            if (fp.test) fp.test[fo + out] = test;
        }
    } else if (hg.emitter >= 0) {  // main.cu:171-182
        const DevEmitter &e = sc.areas[hg.emitter];
        vec3 Le;
        float pdf_e;
        emitter_eval_area(e, geo, f3(ld_ps(ps.ray_o + p)), Le, pdf_e);
        if (!is_zero(pdf_e)) {
            const float mis = (flags >> 31) ? 1.f : mis_weight(prev_pdf, pdf_e * e.select_probability);
            L_add = T * Le * mis;
            L_changed = true;
        }
    }

    // loop head (main.cu:103-111)
    const uint32_t depth = bounce + 1;
    if (depth >= fp.max_depth) alive = false;
    if (alive) {
        const float rr = depth > 2 ? 0.95f : 1.0f;
        if (rng_next(rng) > rr) alive = false;
        else T = T / rr;
    }
    float pdf_b = 0.f, sh_tmax = 0.f;
    uint32_t delta = 0;
    const bool nee = alive;  // the reference traces its shadow ray here unconditionally (main.cu:119-123)
    if (alive) {
        // direct light sampling (main.cu:114-141)
        float sel_prob;
        const DevEmitter *e = select_emitter(sc, rng_next(rng), sel_prob);
        const float x0 = rng_next(rng);
        const float x1 = rng_next(rng);
        const vec3 wo = to_local(-ray_d, geo.normal);
        if (e) {
            const EmitterSample es = emitter_sample_direct(*e, geo, v2(x0, x1));
            BsdfRec er;
            er.wi = to_local(es.wi, geo.normal);
            er.wo = wo;
            er.f = v3(0.f);
            er.pdf = 0.f;
            bsdf_eval_t<MAT>(bsdf, er);
            if (!is_zero(er.f * es.pdf)) {
                const float NoL = dot(geo.normal, es.wi);
                if (NoL > 0.f) {
                    const float mis = mis_weight(es.pdf, er.pdf);
                    const float pdf_l = es.pdf * sel_prob;
                    const vec3 C = T * es.radiance * er.f * NoL * mis / pdf_l;
                    sh_tmax = es.distance - 0.001f;
                    st_ps(ps.sh_d + p, f4(es.wi, 0.f));
                    st_ps(ps.sh_c + p, f4(C, 0.f));
                    push_shadow = true;
                }
            }
        }
        // BSDF sampling (main.cu:143-163)
        BsdfRec br;
        br.wo = wo;
        br.wi = v3(0.f);
        br.f = v3(0.f);
        br.pdf = 0.f;
        br.sampled_type = 0;
        bsdf_sample_t<MAT>(bsdf, br, rng);
        if (is_zero(br.f * fabs_(br.wi.z)) || is_zero(br.pdf)) {
            alive = false;
        } else {
            T = T * (br.f * fabs_(br.wi.z) / br.pdf);
            const vec3 nd = to_world(br.wi, geo.normal);
            st_ps(ps.ray_d + p, f4(nd, 0.f));
            pdf_b = br.pdf;
            delta = (br.sampled_type & kLobeDelta) ? 1u : 0u;
            push_next = true;
        }
    }
    // the shadow ray starts where the extension ray does (main.cu:119-123,158): one origin
    // record for both, w = the shadow ray's tmax (the extension ray's tmax is a constant)
    if (push_shadow || push_next) st_ps(ps.ray_o + p, f4(geo.position, sh_tmax));
    // A path that spawns no extension ray is never shaded again: its throughput and misc
    // records are dead (the shadow retire reads only sh_c and rad, the accumulate only
    // rad), and rad is rewritten only when this hit added emission.
    if (push_next) {
        st_ps(ps.thr + p, f4(T, pdf_b));
        st_ps(ps.misc + p, make_uint4(rng, (bounce + 1) | (delta << 31), __float_as_uint(geo.texcoord.x),
                                __float_as_uint(geo.texcoord.y)));
    }
    if (L_changed) {
        const vec3 L = f3(fresh ? make_float4(0.f, 0.f, 0.f, 0.f) : ld_ps(ps.rad + p)) + L_add;
        st_ps(ps.rad + p, f4(L, 0.f));
    }
    return (push_next ? 1u : 0u) | (push_shadow ? 2u : 0u) | (nee ? 4u : 0u);
}

// Paths whose ray left the scene (__miss__default, main.cu:196-212, and the
// env handling at main.cu:87-99 / 165-169).
__device__ __forceinline__ void shade_miss(const DeviceScene &sc, const FrameParams &fp, const PathState &ps,
                                           uint32_t p, bool fresh, uint32_t fresh_p, uint32_t fresh_seed0) {
    const uint32_t fresh_rng = fresh ? fresh_rng_of(fp, fresh_p, fresh_seed0) : 0u;
    const uint4 misc = fresh ? make_uint4(fresh_rng, 0u, 0u, 0u) : ld_ps(ps.misc + p);
    if ((misc.y & 0xFFFFFFu) == 0u) {
        float4 rad4 = fresh ? make_float4(0.f, 0.f, 0.f, 0.f) : ld_ps(ps.rad + p);
        vec3 L = f3(rad4);
        uint32_t rng = misc.x;
        if (sc.has_env) {
            vec3 Le;
            float pdf;
            const vec3 ro = fresh ? camera_origin(sc.camera) : f3(ld_ps(ps.ray_o + p));  // fresh: not stored
            env_eval(*sc.env, ro, f3(ld_ps(ps.ray_d + p)), Le, pdf);
            L = L + Le;  // main.cu:185, no MIS on the camera ray
        }
        const float test = rng_next(rng);
        uint32_t l;
        uint32_t fo;
        if (last_sample(fp, p, l, fo)) {
            const uint32_t out = fp.aov_local ? l : global_pixel(fp, l);
            if (fp.albedo) fp.albedo[fo + 3 * out] = fp.albedo[fo + 3 * out + 1] = fp.albedo[fo + 3 * out + 2] = 0.f;
            if (fp.normal) fp.normal[fo + 3 * out] = fp.normal[fo + 3 * out + 1] = fp.normal[fo + 3 * out + 2] = 0.f;
            if (fp.test) fp.test[fo + out] = test;
        }
        st_ps(ps.rad + p, f4(L, 0.f));
    } else if (sc.has_env) {
        const float4 thr4 = ld_ps(ps.thr + p);
        vec3 Le;
        float env_pdf;
        env_eval(*sc.env, f3(ld_ps(ps.ray_o + p)), f3(ld_ps(ps.ray_d + p)), Le, env_pdf);
        const float mis = mis_weight(thr4.w, env_pdf);  // main.cu:166-167
        const vec3 env_rad = Le * (f3(thr4) * mis);
        float4 rad4 = ld_ps(ps.rad + p);
        st_ps(ps.rad + p, f4(f3(rad4) + env_rad, 0.f));  // main.cu:185
    }
}

}  // namespace
}  // namespace pupil
