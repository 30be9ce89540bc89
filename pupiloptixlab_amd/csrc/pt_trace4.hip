// pt_trace4.hip — the persistent BVH4 traversal kernels on gfx950 (the reference's
// optixTrace over IAS -> GAS: example/path_tracer/main.cu:77-82,158-163 closest hit,
// render/emitter.h:91-100 shadow any hit).  Split from pt_kernels.hip (the wavefront
// shading stages) so the traversal compiles, and is inspected (tools/isa_loop.py), on
// its own.
#include "pt_kernels.h"
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

#include <cstdlib>
#include <algorithm>

namespace pupil {

namespace {

using namespace tr;

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
// TOP: nodes [0, sc.top_nodes) are read from an LDS copy (DeviceScene::top_nodes; a separate
// instance, since the per-visit LDS-or-global branch costs 1.1 % where the copy does not pay)
// COOP: the wave-cooperative node fetch (pt_traverse.h CoopFetch; flat kernels only), staged in
// s_coop (per wave: 64 node offsets, then the 16 * kCoopChunks node image); the stack ring is
// RING entries (kTraceRing when COOP, leaving the LDS for the staging)
template <int MODE, bool ANY, bool STATS, bool TL, bool TOP = false, bool COOP = false, int RING = kRing>
__device__ __forceinline__ void trace4_body(const DeviceScene &sc, const PathState &ps, const Queues &q,
                                            const TraceJob &job, int *ovf, uint32_t ovf_threads,
                                            const TraceStats &stats, int *s_ring, float *s_aux, float *s_tst,
                                            Bvh4Node *s_top, float4 *s_coop = nullptr) {
    constexpr float kInf = __builtin_huge_valf();
    // the top of the tree (nodes [0, top), breadth first) into LDS: every ray starts there
    const uint32_t top = TOP ? sc.top_nodes : 0u;
    if (TOP) {
        for (uint32_t i = threadIdx.x; i < top * 4u; i += kTraceBlock)
            reinterpret_cast<float4 *>(s_top)[i] = reinterpret_cast<const float4 *>(sc.nodes4)[i];
        __syncthreads();
    }
    constexpr bool kMixed = MODE == kModeMixed || MODE == kModeMixedAhead;
    const uint32_t n_next = kMixed ? q.counts[kCntNext] : 0u;
    // mixed launches may carry the next render's camera rays (render-ahead, TraceJob::ahead_off)
    const uint32_t n_ahead = MODE == kModeMixedAhead ? job.static_count : 0u;
    const uint32_t count = kMixed ? n_next + q.counts[kCntShadow] : (job.count_ptr ? *job.count_ptr : job.static_count);
    LinStackT<RING, RING == kRing ? kStackOvf : kTraceStackOvf> st;
    st.lds = s_ring + threadIdx.x;
    st.ovf_blk = ovf + blockIdx.x * blockDim.x;
    st.lds0 = s_ring;
    st.ovf_stride = ovf_threads;
    constexpr bool kDist = kDistStack && !TL;
    if (STATS || kDist) st.tcol = s_tst + threadIdx.x;
    st.reset();
    CoopFetch<kCoopChunks> cf;
    if (COOP) {
        // this wave's staging: 256 B of node offsets, then the node image (wave-uniform base)
        const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        float4 *wbase = s_coop + w * (16u + 64u * kCoopChunks);
        cf.addr = reinterpret_cast<uint32_t *>(wbase);
        cf.stage = wbase + 16;
    }
    // STATS: visits of a popped node whose entry distance already exceeds the ray's tmax (a
    // stack holding distances could skip them without the fetch), visits where no child was hit
    uint32_t n_cullable = 0, n_nohit = 0;
    float t_node = 0.f;
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
    auto popn = [&]() { return kDist ? st.pop_live(tmax) : st.pop(); };
    // state read only at a hit update or at the retire lives in LDS (s_aux), not in VGPRs:
    // the path id and the best hit's barycentrics
    float &b1 = s_aux[threadIdx.x];
    float &b2 = s_aux[kTraceBlock + threadIdx.x];
    uint32_t &p = reinterpret_cast<uint32_t *>(s_aux)[2 * kTraceBlock + threadIdx.x];
    uint32_t &best_idx = reinterpret_cast<uint32_t *>(s_aux)[3 * kTraceBlock + threadIdx.x];
    b1 = b2 = 0.f;
    p = 0;
    best_idx = kMissIndex;
    int node = kSentinel, leaf = 0;
    bool found = false;
    bool any = ANY;  // this lane's ray terminates on its first hit
    bool in_blas = false;  // TL: traversing an instance's BLAS
    uint32_t inst = 0;
    vec3 bo = v3(0.f), bi = v3(0.f);  // TL: box-test ray (object space inside a BLAS)
    vec3 be = v3(0.f);                // its slab-test bound (pt_traverse.h slab_error)
    // the ray direction is reloaded for the rare sphere test / instance entry instead of
    // being held across the loop (r04: fewer live registers, profiles/r04_trim_state_ab.txt)
    auto ray_dir = [&]() -> vec3 {
        if (MODE == kModeRays) {
            const float *r8 = job.rays + 8 * (size_t)p;
            return v3(r8[3], r8[4], r8[5]);
        }
        return f3(any ? ld_ps(ps.sh_d + p) : ld_ps(ps.ray_d + p));
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
                        // no queue: the camera rays of a render (origin = the camera's, k_generate)
                        o = job.queue ? ld_ps(ps.ray_o + p) : f4(camera_origin(sc.camera), 0.f);
                        d = ld_ps(ps.ray_d + p);
                        tmin = 0.001f;
                        tmax = kMaxDistance;
                    } else if (MODE == kModeMixedAhead && k < len_a) {
                        // a camera ray of the next render (generated into the other half of the
                        // path state): the primary extend's pixel-major dequeue, then the offset
                        const uint32_t j = lo_a + k;
                        p = (job.spp ? (j % job.spp) * job.num_local + j / job.spp : j) + job.ahead_base;
                        any = false;
                        o = f4(camera_origin(sc.camera), 0.f);  // a camera ray (k_generate)
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
        // one node visit of this lane (node phase): box test, push / pop, postpone a leaf
        auto visit_node = [&](const Bvh4Node &n) {
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
        if (STATS) {
            n_cullable += t_node > tmax ? 1u : 0u;
            n_nohit += t[0] == kInf ? 1u : 0u;
        }
        if (t[0] == kInf) {
            node = popn();
            if (STATS) t_node = st.tpop;
        } else {
            node = l[0];
            if (STATS) t_node = t[0];
            st.reserve3();
            st.push3t(t[1], t[2], t[3], t[2] != kInf, t[3] != kInf);
            st.push3(l[1], l[2], l[3], t[1] != kInf, t[2] != kInf, t[3] != kInf);
            if (node == kEmptyLink) node = popn();  // degenerate child boxes only (LinStack)
        }
        if (node < 0 && leaf >= 0) {  // postpone the leaf, keep descending
            leaf = node;
            node = popn();
            if (STATS) t_node = st.tpop;
        }
        };
        if (COOP) {
            // wave-uniform node phase: every lane takes part in the fetch, lanes that need a
            // node visit it (the same visits in the same order per lane as the loop below)
            for (;;) {
                const bool want = active && (uint32_t)node < (uint32_t)kSentinel;
                if (!__any(want)) break;
                const Bvh4Node n = cf.template fetch<STATS>(sc.nodes4, node, want);
                if (want) visit_node(n);
                // leave for the leaf phase once fewer than node_min lanes still need a node
                if ((uint32_t)__popcll(__ballot(want && leaf >= 0)) < job.node_min) break;
            }
        }
        if (active) {
            if (!COOP) {
                while ((uint32_t)node < (uint32_t)kSentinel) {
                    Bvh4Node n;
                    if (TOP && (uint32_t)node < top) n = s_top[node];
                    else n = load_node4(sc, node);
                    visit_node(n);
                    // leave for the leaf phase once fewer than node_min lanes still need a node
                    if ((uint32_t)__popcll(__ballot(leaf >= 0)) < job.node_min) break;
                }
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
                        st.push(node);
                        st.push(kReturnLink);
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
                    if (intersect_leaf_tl<STATS>(sc, r, leaf, inst, tmin, tmax, best_key, best_idx, b1, b2,
                                                 np_cnt, found, any))
                        break;
                } else if (intersect_leaf_dyn<STATS>(sc, r, leaf, tmin, tmax, best_key, best_idx, b1, b2,
                                                     np_cnt, found, any, ray_dir)) {
                    break;
                }
                leaf = node;
                if (node < 0) node = popn();
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
                        bin = sc.instances[inst_of_prim(sc, best_idx)].bin;
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
    if (COOP) flush_stats<STATS>(&stats, cf.n_dma, cf.n_slots, 24);
    flush_stats<STATS>(&stats, n_cullable, n_nohit, 8);
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

template <int MODE, bool ANY, bool STATS, bool TOP>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerSimd))) void k_trace4(
    DeviceScene sc, PathState ps, Queues q, TraceJob job, int *ovf, uint32_t ovf_threads, TraceStats stats) {
    constexpr int ring = kCoopFetch || kDistStack ? kTraceRing : kRing;
    __shared__ int s_ring[ring * kTraceBlock];
    __shared__ float s_aux[4 * kTraceBlock];
    __shared__ float s_tst[STATS || kDistStack ? ring * kTraceBlock : 1];
    __shared__ Bvh4Node s_top[kCoopFetch || kDistStack ? 1 : kTopNodes];
    __shared__ float4 s_coop[kCoopFetch ? (kTraceBlock / 64) * (16 + 64 * kCoopChunks) : 1];
    // the cooperative fetch replaces the LDS top-of-tree copy (its hot nodes are one shared DMA)
    trace4_body<MODE, ANY, STATS, false, TOP && !kCoopFetch && !kDistStack, kCoopFetch, ring>(sc, ps, q, job, ovf, ovf_threads, stats,
                                                                              s_ring, s_aux, s_tst, s_top, s_coop);
}

// two-level variant: 9 more live registers (object-space box ray, margin,
// instance) -> one wave less per SIMD so the loop does not spill
template <int MODE, bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerSimdTL))) void k_trace4tl(
    DeviceScene sc, PathState ps, Queues q, TraceJob job, int *ovf, uint32_t ovf_threads, TraceStats stats) {
    __shared__ int s_ring[kRing * kTraceBlock];
    __shared__ float s_aux[4 * kTraceBlock];
    __shared__ float s_tst[STATS ? kRing * kTraceBlock : 1];
    trace4_body<MODE, ANY, STATS, true>(sc, ps, q, job, ovf, ovf_threads, stats, s_ring, s_aux, s_tst, nullptr);
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
    } else if (sc.top_nodes) {
        if (stats)
            hipLaunchKernelGGL((k_trace4<MODE, ANY, true, true>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                               ovf, ovf_threads, st);
        else
            hipLaunchKernelGGL((k_trace4<MODE, ANY, false, true>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                               ovf, ovf_threads, st);
    } else if (stats) {
        hipLaunchKernelGGL((k_trace4<MODE, ANY, true, false>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                           ovf, ovf_threads, st);
    } else {
        hipLaunchKernelGGL((k_trace4<MODE, ANY, false, false>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, job,
                           ovf, ovf_threads, st);
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

uint32_t trace_grid_blocks() { return 256u * 16u; }

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

}  // namespace pupil
