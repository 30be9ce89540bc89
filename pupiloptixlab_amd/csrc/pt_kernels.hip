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
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

#include <cstdlib>
#include <algorithm>

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
__device__ __forceinline__ vec3 camera_origin(const Camera &cam) { return v3(cam.c2w[3], cam.c2w[7], cam.c2w[11]); }

// Two-level: the object-space box ray of instance `in` (origin, reciprocal
// direction) and its slab-test bound (pt_traverse.h slab_error_pad), which adds the
// position margin at the exit of the instance's world box.
__device__ __forceinline__ void enter_instance(const DevInstance &in, const RayPre &r, vec3 rd, float tmax,
                                               const float bound[3], vec3 &bo, vec3 &bi, vec3 &be) {
    bo = xform_point(in.to_object, r.o);
    const vec3 d = xform_vector(in.to_object, rd);
    const float tiny = 1e-30f;
    bi = v3(1.f / (fabsf(d.x) < tiny ? copysignf(tiny, d.x) : d.x), 1.f / (fabsf(d.y) < tiny ? copysignf(tiny, d.y) : d.y),
            1.f / (fabsf(d.z) < tiny ? copysignf(tiny, d.z) : d.z));
    float te = tmax;
    te = fminf(te, fmaxf((in.wlo[0] - r.o.x) * r.idir.x, (in.whi[0] - r.o.x) * r.idir.x));
    te = fminf(te, fmaxf((in.wlo[1] - r.o.y) * r.idir.y, (in.whi[1] - r.o.y) * r.idir.y));
    te = fminf(te, fmaxf((in.wlo[2] - r.o.z) * r.idir.z, (in.whi[2] - r.o.z) * r.idir.z));
    te = fabsf(te) * 1.0001f;
    const float on = fmaxf(fmaxf(fabsf(r.o.x), fabsf(r.o.y)), fabsf(r.o.z));
    const float dn = fmaxf(fmaxf(fabsf(rd.x), fabsf(rd.y)), fabsf(rd.z));
    const float pad = __builtin_fmaf(in.margin[0], __builtin_fmaf(te, dn, on), in.margin[1]);
    be = v3(slab_error_pad(bo.x, bi.x, bound[0], pad), slab_error_pad(bo.y, bi.y, bound[1], pad),
            slab_error_pad(bo.z, bi.z, bound[2], pad));
}

// TL = two-level acceleration (DeviceScene::two_level): the TLAS leaves hold one
// instance each; entering one pushes the pending TLAS link and kReturnLink and
// switches the box tests to the instance's object-space ray; popping
// kReturnLink switches back.  Spheres are tested at their TLAS leaf.
template <int MODE, bool ANY, bool STATS, bool TL>
__device__ __forceinline__ void trace4_body(const DeviceScene &sc, const PathState &ps, const Queues &q,
                                            const TraceJob &job, int *ovf, uint32_t ovf_threads,
                                            const TraceStats &stats, int *s_ring, float *s_aux) {
    constexpr float kInf = __builtin_huge_valf();
    constexpr bool kMixed = MODE == kModeMixed || MODE == kModeMixedAhead;
    const uint32_t n_next = kMixed ? q.counts[kCntNext] : 0u;
    // mixed launches may carry the next render's camera rays (render-ahead, TraceJob::ahead_off)
    const uint32_t n_ahead = MODE == kModeMixedAhead ? job.static_count : 0u;
    const uint32_t count = kMixed ? n_next + q.counts[kCntShadow] : (job.count_ptr ? *job.count_ptr : job.static_count);
    RingStack st;
    st.lds = s_ring + threadIdx.x;
#if PUPIL_TRIM
    st.ovf_blk = ovf + blockIdx.x * blockDim.x;
    st.lds0 = s_ring;
#else
    st.ovf = ovf + blockIdx.x * blockDim.x + threadIdx.x;
#endif
    st.ovf_stride = ovf_threads;
    st.reset();
    uint32_t nv = 0, npt = 0, nv_sh = 0, npt_sh = 0;  // mixed: shadow-ray counts apart
    uint32_t n_unique = 0;  // STATS: distinct node fetches (per wave step)
    // STATS-only SIMD-efficiency diagnostics, each event counted by one lane:
    // node-loop wave iterations / active lanes, leaf-loop iterations / active
    // lanes, refills / lanes refilled
    unsigned long long dg[6] = {0, 0, 0, 0, 0, 0};
    bool active = false, drained = false;
    // XCD-sharded dequeue (one atomic head per XCD: a single head saturates at
    // ~88 dequeues/us, MI355X_MICROARCH.md 'dequeue', which is the refill rate
    // of this kernel).  The work list is cut into kWorkShards contiguous chunks;
    // workgroups start on chunk blockIdx % kWorkShards (the dispatcher deals
    // workgroups round-robin over the XCDs) and move on to the next chunk when
    // theirs is exhausted, so every item is taken exactly once.
    uint32_t shard = blockIdx.x % kWorkShards, tried = 0;
    unsigned long long t_start = 0, t_drained = 0, n_taken = 0;  // PUPIL_TRACE_TAIL
    // STATS: queue accounting of this wave (wave-uniform): list items the dequeue heads
    // handed it, lanes it activated, lanes it retired (counters[20..22]; every launch
    // must give handed = activated = retired = its list length, counters[23])
    uint32_t q_handed = 0, q_act = 0, q_ret = 0;
    if (STATS && stats.wave_times) t_start = __builtin_amdgcn_s_memrealtime();
    uint32_t best_key = 0;
    RayPre r{};
    float tmin = MODE == kModeRays ? 0.f : 0.001f, tmax = 0.f;  // tmin: a constant outside kModeRays
#if PUPIL_TRIM
    // state read only at a hit update or at the retire lives in LDS (s_aux), not in VGPRs:
    // the path id and the best hit's barycentrics
    float &b1 = s_aux[threadIdx.x];
    float &b2 = s_aux[kTraceBlock + threadIdx.x];
    uint32_t &p = reinterpret_cast<uint32_t *>(s_aux)[2 * kTraceBlock + threadIdx.x];
    uint32_t &best_idx = reinterpret_cast<uint32_t *>(s_aux)[3 * kTraceBlock + threadIdx.x];
    b1 = b2 = 0.f;
    p = 0;
    best_idx = kMissIndex;
#else
    uint32_t p = 0, best_idx = kMissIndex;
    float b1 = 0.f, b2 = 0.f;
#endif
    int node = kSentinel, leaf = 0;
    bool found = false;
    bool any = ANY;  // this lane's ray terminates on its first hit
    bool in_blas = false;  // TL: traversing an instance's BLAS
    uint32_t inst = 0;
    vec3 bo = v3(0.f), bi = v3(0.f);  // TL: box-test ray (object space inside a BLAS)
    vec3 be = v3(0.f);                // its slab-test bound (pt_traverse.h slab_error)
    // the ray direction: kept in r.d, or (PUPIL_TRIM) reloaded for the rare sphere test /
    // instance entry instead of being held across the loop
    auto ray_dir = [&]() -> vec3 {
#if PUPIL_TRIM
        if (MODE == kModeRays) {
            const float *r8 = job.rays + 8 * (size_t)p;
            return v3(r8[3], r8[4], r8[5]);
        }
        return f3(any ? ld_ps(ps.sh_d + p) : ld_ps(ps.ray_d + p));
#else
        return r.d;
#endif
    };
    for (;;) {
        // ---- refill idle lanes (one atomic per wave)
        const unsigned long long idle = __ballot(!active);
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        if (!drained && n_idle >= job.refill) {
            // chunk `shard`: list positions [lo, lo + len).  Mixed launches cut the
            // extension and the shadow list separately and give each chunk its
            // extension share first, so every chunk ends on (cheaper) shadow rays
            // and the launch tail is not made of closest-hit traversals.
            uint32_t lo, len, len_e = 0, lo_s = 0, lo_a = 0, len_a = 0;
            if (kMixed) {
                // chunk = its share of the render-ahead camera rays (kModeMixedAhead only:
                // coherent, traced first as in a primary launch, whose tail the bounce
                // rays then fill), of the extension list, then of the shadow list
                const uint32_t n_sh = count - n_next;
                lo = (uint32_t)((uint64_t)n_next * shard / kWorkShards);
                len_e = (uint32_t)((uint64_t)n_next * (shard + 1) / kWorkShards) - lo;
                lo_a = (uint32_t)((uint64_t)n_ahead * shard / kWorkShards);
                len_a = (uint32_t)((uint64_t)n_ahead * (shard + 1) / kWorkShards) - lo_a;
                lo_s = n_next + (uint32_t)((uint64_t)n_sh * shard / kWorkShards);
                len = len_e + len_a + (n_next + (uint32_t)((uint64_t)n_sh * (shard + 1) / kWorkShards) - lo_s);
            } else {
                lo = (uint32_t)((uint64_t)count * shard / kWorkShards);
                len = (uint32_t)((uint64_t)count * (shard + 1) / kWorkShards) - lo;
            }
            uint32_t base = 0;
            if (lane_id() == 0) base = atomicAdd(job.work + shard * kWorkStride, n_idle);
            base = __shfl(base, 0);
            if (STATS && lane_id() == 0) {
                dg[4]++;
                dg[5] += min(n_idle, base < len ? len - base : 0u);
            }
            if (STATS) n_taken += min(n_idle, base < len ? len - base : 0u);
            if (STATS) q_handed += min(n_idle, base < len ? len - base : 0u);
            const bool was_active = active;
            if (base + n_idle >= len) {  // chunk exhausted: continue on the next one
                shard = shard + 1 == kWorkShards ? 0u : shard + 1;
                if (++tried == kWorkShards) {
                    drained = true;
                    if (STATS && stats.wave_times) t_drained = __builtin_amdgcn_s_memrealtime();
                }
            }
            if (!active) {
                const uint32_t k = base + (uint32_t)__popcll(idle & lanemask_lt());
                const uint32_t ke = k - len_a;  // past the render-ahead share (len_a = 0 outside kModeMixedAhead)
                const uint32_t i = kMixed && ke >= len_e ? lo_s + (ke - len_e) : lo + ke;
                if (k < len) {
                    float4 o, d;
                    if (MODE == kModeExtend) {
                        p = job.queue ? job.queue[i] : (job.spp ? (i % job.spp) * job.num_local + i / job.spp : i);
                        o = ld_ps(ps.ray_o + p);
                        d = ld_ps(ps.ray_d + p);
                        tmin = 0.001f;
                        tmax = kMaxDistance;
                    } else if (MODE == kModeMixedAhead && k < len_a) {
                        // a camera ray of the next render (generated into the other half of the
                        // path state): the primary extend's pixel-major dequeue, then the offset
                        const uint32_t j = lo_a + k;
                        p = (job.spp ? (j % job.spp) * job.num_local + j / job.spp : j) + job.ahead_base;
                        any = false;
                        o = ld_ps(ps.ray_o + p);
                        d = ld_ps(ps.ray_d + p);
                        tmin = 0.001f;
                        tmax = kMaxDistance;
                    } else if (kMixed) {
                        p = q.nxsh[i] + (MODE == kModeMixedAhead ? job.list_base : 0u);
                        any = i >= n_next;
                        o = ld_ps(ps.ray_o + p);
                        d = any ? ld_ps(ps.sh_d + p) : ld_ps(ps.ray_d + p);
                        tmin = 0.001f;
                        tmax = any ? o.w : kMaxDistance;
                    } else {
                        p = i;
                        const float *r8 = job.rays + 8 * (size_t)i;
                        o = make_float4(r8[0], r8[1], r8[2], 0.f);
                        d = make_float4(r8[3], r8[4], r8[5], 0.f);
                        tmin = r8[6];
                        tmax = r8[7];
                    }
                    r = ray_pre(f3(o), f3(d));
                    best_key = 0xFFFFFFFFu;
                    best_idx = kMissIndex;
                    b1 = b2 = 0.f;
                    found = false;
                    st.reset();
                    node = (int)sc.root_link4;
                    leaf = 0;
                    be = slab_errors(r.o, r.idir, sc.node_bound);
                    if (TL) {
                        in_blas = false;
                        bo = r.o;
                        bi = r.idir;
                    }
                    if (node < 0) {
                        leaf = node;
                        node = kSentinel;
                    }
                    active = true;
                }
            }
            if (STATS) q_act += (uint32_t)__popcll(__ballot(active && !was_active));
        }
        if (!__any(active)) {
            if (drained) break;
            continue;
        }
        // ---- traverse until this lane's ray terminates or it needs a leaf while others do too
        if (active) {
            while ((uint32_t)node < (uint32_t)kSentinel) {
                const Bvh4Node n = load_node4(sc, node);
                if (STATS) {
                    if (kMixed && any) nv_sh++;
                    else nv++;
                    const unsigned long long m = __ballot(true);
                    if ((int)lane_id() == __ffsll((long long)m) - 1) {
                        dg[0]++;
                        dg[1] += (unsigned long long)__popcll(m);
                    }
                    // distinct nodes fetched by this wave step (lanes of a wave on the same node
                    // share one fetch): the gather rate the memory system actually serves
                    bool dup = false;
                    for (int j = 0; j < 64; j++) {
                        const int nj = __shfl(node, j);
                        if (j < (int)lane_id() && ((m >> j) & 1ull) && nj == node) dup = true;
                    }
                    n_unique += dup ? 0u : 1u;
                }
                float t[4];
                int l[4];
                if (TL) visit4(n, bo, bi, be, tmin, tmax, t, l);
                else visit4(n, r.o, r.idir, be, tmin, tmax, t, l);
                if (t[0] == kInf) {
                    node = st.pop();
                } else {
                    node = l[0];
                    st.reserve3();
                    st.push(l[3], t[3] != kInf);
                    st.push(l[2], t[2] != kInf);
                    st.push(l[1], t[1] != kInf);
                }
                if (node < 0 && leaf >= 0) {  // postpone the leaf, keep descending
                    leaf = node;
                    node = st.pop();
                }
                // leave for the leaf phase once fewer than node_min lanes still need a node
                if ((uint32_t)__popcll(__ballot(leaf >= 0)) < job.node_min) break;
            }
            while (leaf < 0) {
                if (STATS) {
                    const unsigned long long m = __ballot(true);
                    if ((int)lane_id() == __ffsll((long long)m) - 1) {
                        dg[2]++;
                        dg[3] += (unsigned long long)__popcll(m);
                    }
                }
                uint32_t &np_cnt = kMixed && any ? npt_sh : npt;
                if (TL && !in_blas) {  // a TLAS leaf: one instance
                    const uint32_t id = leaf_first(leaf);
                    const DevInstance &in = sc.instances[id];
                    if (in.kind == PUPIL_SHAPE_SPHERE) {
                        if (STATS) np_cnt++;
                        float ts;
                        if (intersect_unit_sphere(in.to_object, r.o, ray_dir(), tmin, tmax, ts)) {
                            if (any) {
                                found = true;
                                break;
                            }
                            if (ts < tmax || in.prim_offset < best_key) {
                                tmax = ts;
                                best_key = best_idx = in.prim_offset;
                                b1 = b2 = 0.f;
                                found = true;
                            }
                        }
                    } else {  // enter its BLAS; the pending TLAS link resumes after kReturnLink
                        st.reserve3();
                        st.push(node, true);
                        st.push(kReturnLink, true);
                        in_blas = true;
                        inst = id;
                        enter_instance(in, r, ray_dir(), tmax, sc.node_bound, bo, bi, be);
                        node = in.blas_root;
                        leaf = 0;
                        if (node < 0) {
                            leaf = node;
                            node = st.pop();
                        }
                        continue;
                    }
                } else if (TL) {
                    if (intersect_leaf_tl<STATS>(sc, r, leaf, inst, tmin, tmax, best_key, best_idx, b1, b2, np_cnt,
                                                 found, any))
                        break;
                } else if (intersect_leaf_dyn<STATS>(sc, r, leaf, tmin, tmax, best_key, best_idx, b1, b2, np_cnt,
                                                     found, any, ray_dir)) {
                    break;
                }
                leaf = node;
                if (node < 0) node = st.pop();
            }
            if (TL && node == kReturnLink && leaf >= 0 && !(any && found)) {  // BLAS exhausted: back to the TLAS
                in_blas = false;
                bo = r.o;
                bi = r.idir;
                be = slab_errors(r.o, r.idir, sc.node_bound);
                node = st.pop();
                if (node < 0) {
                    leaf = node;
                    node = st.pop();
                }
            }
        }
        const bool done = active && ((node == kSentinel && leaf >= 0) || (any && found));
        // ---- retire
        if (MODE == kModeExtend || kMixed) {
            uint32_t bin = 0;
            if (done && !any) {
                // hit index: the record (flat) or the global primitive id (two-level shading,
                // reconstruct(); the world-mode flat kernel keeps it in best_key)
                const uint32_t hidx = !TL && sc.two_level ? best_key : best_idx;
                st_ps(ps.hit + p, make_float4(found ? tmax : -1.f, b1, b2, __uint_as_float(found ? hidx : kMissIndex)));
                // single-material scenes: shading reads the bin off the hit (no dependent
                // record fetch here, which would stall the wave before its next refill)
                if (found && sc.single_bin == 0u) {
                    if (TL) {
                        bin = sc.instances[sc.prim_inst[best_idx]].bin;
                    } else {
                        const uint32_t mt = __float_as_uint(sc.prims[kRecF4 * best_idx + 2].w);
                        bin = (mt >= 1u && mt <= 7u) ? mt : 8u;
                    }
                }
                if (sc.single_bin == 0u) ps.mbin[p] = (uint8_t)bin;  // material bin for the partition
            }
        }
        if (kMixed) {
            if (done && any && !found) {  // main.cu:124-139 (shadow rays share the origin record, w = tmax)
                const float4 c = ld_ps(ps.sh_c + p);
                float4 L = ld_ps(ps.rad + p);
                L.x = L.x + c.x;
                L.y = L.y + c.y;
                L.z = L.z + c.z;
                st_ps(ps.rad + p, L);
            }
        } else if (MODE == kModeRays && done) {
            float *o = job.out + 4 * (size_t)p;
            o[0] = found ? (ANY ? 1.f : tmax) : -1.f;
            o[1] = b1;
            o[2] = b2;
            o[3] = __uint_as_float(found && !ANY ? best_key : 0xFFFFFFFFu);
        }
        if (STATS) q_ret += (uint32_t)__popcll(__ballot(done));
        if (done) active = false;
    }
    flush_stats<STATS>(&stats, nv, npt, 0);
    if (kMixed) flush_stats<STATS>(&stats, nv_sh, npt_sh, 14);
    flush_stats<STATS>(&stats, n_unique, 0u, 18);
    if (STATS && stats.wave_times && lane_id() == 0) {
        unsigned long long *w = stats.wave_times + 4ull * (blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u);
        w[0] = t_start;
        w[1] = t_drained;
        w[2] = __builtin_amdgcn_s_memrealtime();
        w[3] = n_taken;
    }
    // the last wave out resets the counters for the next launch (no memset per
    // launch).  Waves count out on kWorkShards sub-counters (blockIdx % shards),
    // the last of each sub-counter on the final one: the exit burst at the end
    // of a launch is spread over kWorkShards addresses instead of serialised
    // on one (~88 atomics/us per address).
    if (lane_id() == 0) {
        const uint32_t sub = blockIdx.x % kWorkShards;
        const uint32_t groups = min(gridDim.x, kWorkShards);
        const uint32_t sub_waves = (gridDim.x - sub + kWorkShards - 1u) / kWorkShards * (blockDim.x / 64u);
        if (STATS) {
            atomicAdd(&stats.counters[20], (unsigned long long)q_handed);
            atomicAdd(&stats.counters[21], (unsigned long long)q_act);
            atomicAdd(&stats.counters[22], (unsigned long long)q_ret);
        }
        if (atomicAdd(job.work + (kWorkShards + 1u + sub) * kWorkStride, 1u) == sub_waves - 1u &&
            atomicAdd(job.work + kWorkShards * kWorkStride, 1u) == groups - 1u) {
            for (uint32_t k = 0; k < 2u * kWorkShards + 1u; k++) atomicExch(job.work + k * kWorkStride, 0u);
            if (STATS) atomicAdd(&stats.counters[23], (unsigned long long)(count + n_ahead));  // once per launch
        }
    }
    if (STATS) {
        for (int k = 0; k < 6; k++) {
            unsigned long long v = dg[k];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            dg[k] = v;
        }
        if (lane_id() == 0)
            for (int k = 0; k < 6; k++) atomicAdd(&stats.counters[2 + k], dg[k]);
    }
}

template <int MODE, bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerSimd))) void k_trace4(
    DeviceScene sc, PathState ps, Queues q, TraceJob job, int *ovf, uint32_t ovf_threads, TraceStats stats) {
    __shared__ int s_ring[kRing * kTraceBlock];
    __shared__ float s_aux[PUPIL_TRIM ? 4 * kTraceBlock : 1];
    trace4_body<MODE, ANY, STATS, false>(sc, ps, q, job, ovf, ovf_threads, stats, s_ring, s_aux);
}

// two-level variant: 9 more live registers (object-space box ray, margin,
// instance) -> one wave less per SIMD so the loop does not spill
template <int MODE, bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerSimdTL))) void k_trace4tl(
    DeviceScene sc, PathState ps, Queues q, TraceJob job, int *ovf, uint32_t ovf_threads, TraceStats stats) {
    __shared__ int s_ring[kRing * kTraceBlock];
    __shared__ float s_aux[PUPIL_TRIM ? 4 * kTraceBlock : 1];
    trace4_body<MODE, ANY, STATS, true>(sc, ps, q, job, ovf, ovf_threads, stats, s_ring, s_aux);
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

// full = 0 (list shading, PUPIL_FRESH_SHADE): only the camera ray is stored; the bounce-0
// shade of the fresh paths takes throughput 1, radiance 0 and the RNG from fresh_path
// instead of reading them (k_shade_all `fresh`).
__global__ __launch_bounds__(kShadeBlock) void k_generate(DeviceScene sc, FrameParams fp, PathState ps, uint32_t full) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= fp.num_paths) return;
    vec3 dir;
    const uint32_t rng = fresh_path(sc, fp, p, fp.seed0, dir);
    st_ps(ps.ray_o + p, f4(camera_origin(sc.camera), 0.f));
    st_ps(ps.ray_d + p, make_float4(dir.x, dir.y, dir.z, 0.f));
    if (!full) return;
    st_ps(ps.thr + p, make_float4(1.f, 1.f, 1.f, 0.f));
    st_ps(ps.rad + p, make_float4(0.f, 0.f, 0.f, 0.f));
    st_ps(ps.misc + p, make_uint4(rng, 0u, 0u, 0u));
}

// ------------------------------------------------------------------ shade
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
__device__ __forceinline__ HitGeo reconstruct(const DeviceScene &sc, float4 h, const float4 *ro_rec, vec3 rd,
                                             vec2 stale_uv) {
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
        inst_id = sc.prim_inst[idx];
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
        const vec3 ro = f3(ld_ps(ro_rec));
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

    HitGeo hg = reconstruct(sc, h, ps.ray_o + p, ray_d, stale_uv);
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
#if PUPIL_SHADE_SKIP
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
#else
    {
        vec3 L = f3(fresh ? make_float4(0.f, 0.f, 0.f, 0.f) : ld_ps(ps.rad + p));
        if (L_changed) L = L + L_add;
        st_ps(ps.rad + p, f4(L, 0.f));
    }
    st_ps(ps.thr + p, f4(T, pdf_b));
    st_ps(ps.misc + p, make_uint4(rng, (bounce + 1) | (delta << 31), __float_as_uint(geo.texcoord.x),
                            __float_as_uint(geo.texcoord.y)));
#endif
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
            env_eval(*sc.env, f3(ld_ps(ps.ray_o + p)), f3(ld_ps(ps.ray_d + p)), Le, pdf);
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
// the other BSDFs spill 15-43 registers at 5 waves and stay at 4 (A/B: PUPIL_SHADE_ONE=0,
// -DPUPIL_SHADE_DIFFUSE_WAVES).
#ifndef PUPIL_SHADE_DIFFUSE_WAVES
#define PUPIL_SHADE_DIFFUSE_WAVES 5
#endif
constexpr int shade_one_waves(uint32_t mat) { return mat == PUPIL_MAT_DIFFUSE ? PUPIL_SHADE_DIFFUSE_WAVES : 4; }
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
    for (uint32_t s = 0; s < fp.spp; s++) {
        if (clear_flags) ps.sflags[(size_t)s * fp.num_local + l] = 0u;
        vec3 L = f3(ps.rad[(size_t)s * fp.num_local + l]);
        const uint32_t cnt = fp.cnt0 + (fp.accumulate ? s : 0u);
        if (fp.accumulate && cnt > 0) {  // main.cu:187-191
            const float t = 1.f / ((float)cnt + 1.f);
            L = lerp(acc, L, t);
        }
        acc = L;
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

// Persistent grid: exactly the resident capacity (CUs x 4 SIMDs x waves per SIMD).
// PUPIL_TRACE_GRID_WAVES (A/B knob): fewer waves per SIMD in the grid than the
// kernel's occupancy allows.
uint32_t trace4_blocks(const DeviceScene &sc, uint32_t ovf_threads) {
    static const int forced = [] {
        const char *e = std::getenv("PUPIL_TRACE_GRID_WAVES");
        return e ? std::max(1, std::atoi(e)) : 0;
    }();
    const uint32_t occ = sc.two_level && !sc.tl_world ? kTraceWavesPerSimdTL : kTraceWavesPerSimd;
    const uint32_t waves = forced ? std::min(occ, (uint32_t)forced) : occ;
    const uint32_t resident = sc.num_cus * 4u * waves / (kTraceBlock / 64u);
    return std::min(ovf_threads / kTraceBlock, std::max(1u, resident));
}

// persistent BVH4 traversal launch: flat or two-level variant, with or without counters
template <int MODE, bool ANY>
static void launch_trace4(const DeviceScene &sc, const PathState &ps, const Queues &q, const TraceJob &job, int *ovf,
                          uint32_t ovf_threads, const TraceStats *stats, hipStream_t s) {
    const TraceStats st = stats ? *stats : TraceStats{nullptr};
    const uint32_t blocks = trace4_blocks(sc, ovf_threads);
    if (sc.two_level && !sc.tl_world) {
        if (stats)
            hipLaunchKernelGGL((k_trace4tl<MODE, ANY, true>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                               ovf, ovf_threads, st);
        else
            hipLaunchKernelGGL((k_trace4tl<MODE, ANY, false>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                               ovf, ovf_threads, st);
    } else if (stats) {
        hipLaunchKernelGGL((k_trace4<MODE, ANY, true>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job, ovf,
                           ovf_threads, st);
    } else {
        hipLaunchKernelGGL((k_trace4<MODE, ANY, false>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job, ovf,
                           ovf_threads, st);
    }
}

void launch_trace_debug(const DeviceScene &sc, const float *rays, float *out, uint32_t n, int any, int *ovf,
                        uint32_t ovf_threads, uint32_t *work, hipStream_t s, const TraceStats *stats) {
    // the production kernel, fed from a ray array
    const TraceJob job{nullptr, nullptr, n, work, sc.trace_refill, sc.trace_node_min, rays, out, 0u, 0u};
    const Queues q{};
    if (any)
        launch_trace4<kModeRays, true>(sc, PathState{}, q, job, ovf, ovf_threads, stats, s);
    else
        launch_trace4<kModeRays, false>(sc, PathState{}, q, job, ovf, ovf_threads, stats, s);
}

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
uint32_t trace_grid_blocks() { return 256u * 16u; }

void launch_generate(const DeviceScene &sc, const FrameParams &fp, const PathState &ps, hipStream_t s, bool full) {
    const uint32_t blocks = (fp.num_paths + kShadeBlock - 1) / kShadeBlock;
    hipLaunchKernelGGL(k_generate, dim3(blocks), dim3(kShadeBlock), 0, s, sc, fp, ps, full ? 1u : 0u);
}

void launch_extend(const DeviceScene &sc, const PathState &ps, const Queues &q, const uint32_t *queue,
                   const uint32_t *queue_count, uint32_t static_count, int *ovf, uint32_t ovf_threads,
                   const TraceStats *stats, hipStream_t s, uint32_t interleave_spp, uint32_t num_local) {
    const TraceJob job{queue,   queue_count, static_count, q.work + kWorkExtend, sc.trace_refill, sc.trace_node_min,
                       nullptr, nullptr,     queue ? 0u : interleave_spp, num_local};
    launch_trace4<kModeExtend, false>(sc, ps, q, job, ovf, ovf_threads, stats, s);
}

void launch_trace_mixed(const DeviceScene &sc, const PathState &ps, const Queues &q, int *ovf, uint32_t ovf_threads,
                        const TraceStats *stats, hipStream_t s, uint32_t ahead_count, uint32_t list_base,
                        uint32_t ahead_base, uint32_t ahead_spp, uint32_t ahead_local) {
    const TraceJob job{nullptr,       nullptr,   ahead_count,          q.work + kWorkExtend,
                       sc.trace_refill, sc.trace_node_min, nullptr, nullptr,
                       ahead_count ? ahead_spp : 0u, ahead_local, list_base, ahead_base};
    if (ahead_count) launch_trace4<kModeMixedAhead, false>(sc, ps, q, job, ovf, ovf_threads, stats, s);
    else launch_trace4<kModeMixed, false>(sc, ps, q, job, ovf, ovf_threads, stats, s);
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
    if (one && PUPIL_SHADE_ONE_BUILD && sc.single_bin && list != kShadeBins) {
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

__global__ __launch_bounds__(256) void k_node_bound(const Bvh4Node *nodes, uint64_t n, uint32_t *out) {
    float m[3] = {0.f, 0.f, 0.f};
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256ull) {
        const Bvh4Node &b = nodes[i];
        m[0] = fmaxf(m[0], fabsf(b.ox) + 512.f * b.sx);  // upward rounding: slack of slab_error
        m[1] = fmaxf(m[1], fabsf(b.oy) + 512.f * b.sy);
        m[2] = fmaxf(m[2], fabsf(b.oz) + 512.f * b.sz);
    }
    for (int a = 0; a < 3; a++) {
        float v = m[a];
        for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
        if (lane_id() == 0) atomicMax(out + a, __float_as_uint(v));  // non-negative: uint order
    }
}

void launch_node_bound(const Bvh4Node *nodes, uint64_t n, uint32_t *out, hipStream_t s, bool clear) {
    if (clear) (void)hipMemsetAsync(out, 0, 3 * sizeof(uint32_t), s);
    if (n == 0) return;
    const uint64_t blocks = std::min<uint64_t>(2048, std::max<uint64_t>(1, (n + 255) / 256));
    hipLaunchKernelGGL(k_node_bound, dim3((uint32_t)blocks), dim3(256), 0, s, nodes, n, out);
}

void launch_accumulate(const FrameParams &fp, const PathState &ps, const float *aov_src, bool clear_flags,
                       hipStream_t s) {
    const uint32_t blocks = (fp.num_local + kShadeBlock - 1) / kShadeBlock;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(kShadeBlock), 0, s, fp, ps, aov_src, clear_flags ? 1u : 0u);
}

}  // namespace pupil
