// pt_kernels_alt.hip — the A/B traversal families (PUPIL_BVH_WIDTH=2 / 8,
// PUPIL_REFILL=0) and the ray-query verification kernel, kept apart from the
// production persistent BVH4 kernels of pt_kernels.hip so that a change there
// recompiles and re-tests only those.  Every family is bit-exact against the oracle
// (tests/test_gpu_parity.py) and passes the queue accounting of the persistent
// kernels (test_persistent_queue_accounting).
#include "pt_kernels.h"
#include "pt_kernels_alt.h"
#include "pt_shading.h"
#include "pt_trace.h"
#include "pt_traverse.h"

#include <algorithm>
#include <cstdlib>

namespace pupil {

namespace {

using namespace tr;

// ------------------------------------------------------------------ extend
template <bool STATS, int W>
__global__ __launch_bounds__(kTraceBlock) void k_extend(DeviceScene sc, PathState ps, Queues q,
                                                        const uint32_t *queue, const uint32_t *queue_count,
                                                        uint32_t static_count, int *ovf, uint32_t ovf_threads,
                                                        TraceStats stats) {
    __shared__ int s_stack[kStackLds * kTraceBlock];
    const uint32_t count = queue_count ? *queue_count : static_count;
    Stack st;
    st.lds = s_stack + threadIdx.x;
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    st.ovf = ovf + gtid;
    st.ovf_stride = ovf_threads;
    uint32_t nv = 0, pt = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    const uint32_t wave_base = (blockIdx.x * blockDim.x) + (threadIdx.x & ~63u);
    for (uint32_t base = wave_base; base < count; base += stride) {
        const uint32_t i = base + lane_id();
        const bool valid = i < count;
        uint32_t p = 0;
        uint32_t bin = 0;
        if (valid) {
            p = queue ? queue[i] : i;
            const float4 o = ps.ray_o[p];
            const float4 d = ps.ray_d[p];
            const RayPre r = ray_pre(f3(o), f3(d));
            float tmax = kMaxDistance;
            uint32_t best_key = 0xFFFFFFFFu, best_idx = kMissIndex;
            float b1 = 0.f, b2 = 0.f;
            const bool hit = trace_ray<false, STATS, W>(sc, r, 0.001f, tmax, best_key, best_idx, b1, b2, st, nv, pt);
            ps.hit[p] = make_float4(hit ? tmax : -1.f, b1, b2, __uint_as_float(hit ? best_idx : kMissIndex));
            if (hit) {
                const uint32_t mt = __float_as_uint(sc.prims[3 * best_idx + 2].w);
                bin = (mt >= 1u && mt <= 7u) ? mt : 8u;
            }
            ps.mbin[p] = (uint8_t)bin;  // material bin for the partition
        }
    }
    flush_stats<STATS>(&stats, nv, pt);
}

// ------------------------------------------------------------------ shadow
template <bool STATS, int W>
__global__ __launch_bounds__(kTraceBlock) void k_shadow(DeviceScene sc, PathState ps, Queues q, int *ovf,
                                                        uint32_t ovf_threads, TraceStats stats) {
    __shared__ int s_stack[kStackLds * kTraceBlock];
    const uint32_t count = q.counts[kCntShadow];
    const uint32_t *shadow_q = q.nxsh + q.counts[kStartShadow];
    Stack st;
    st.lds = s_stack + threadIdx.x;
    const uint32_t gtid = blockIdx.x * blockDim.x + threadIdx.x;
    st.ovf = ovf + gtid;
    st.ovf_stride = ovf_threads;
    uint32_t nv = 0, pt = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = gtid; i < count; i += stride) {
        const uint32_t p = shadow_q[i];
        const float4 o = ps.ray_o[p];  // w = tmax
        const float4 d = ps.sh_d[p];
        const RayPre r = ray_pre(f3(o), f3(d));
        float tmax = o.w;
        uint32_t k = 0, idx = 0;
        float b1, b2;
        const bool occluded = trace_ray<true, STATS, W>(sc, r, 0.001f, tmax, k, idx, b1, b2, st, nv, pt);
        if (!occluded) {  // main.cu:124-139
            const float4 c = ps.sh_c[p];
            float4 L = ps.rad[p];
            L.x = L.x + c.x;
            L.y = L.y + c.y;
            L.z = L.z + c.z;
            ps.rad[p] = L;
        }
    }
    flush_stats<STATS>(&stats, nv, pt, 14);
}


// ------------------------------------------------------------------ persistent 8-wide traversal
// PUPIL_BVH_WIDTH=8 (flattened BVH): Bvh8Node trees traversed with node-group
// stack entries (Ylitie, Karras & Laine 2017, "Efficient incoherent ray traversal
// on GPUs through compressed wide BVHs"): a node visit tests its eight child boxes
// and leaves one group (child_base, hit slots, imask) instead of one entry per
// hit child, so there is no per-child sort or push; the next child is the hit slot
// with the lowest k ^ octant(ray), the build having placed each child in the slot
// of its centroid octant.  Leaf children add their record slots to a triangle
// group (node, 16 slot bits) that the leaf phase tests one record per step.
// Group words: node group = hit slots by priority << 24 | imask << 16 (>= 2^24),
// triangle group = record-slot bits (< 2^16).  Same persistent dequeue, refill
// and retire as trace4_body.
constexpr int kSpill8 = 4;
static_assert((kRing8 & (kRing8 - 1)) == 0, "ring size must be a power of two");

struct RingStack8 {
    uint2 *lds;  // this lane's column (stride kTraceBlock)
    int *ovf;    // this lane's overflow column (stride ovf_stride), 2 ints per entry
    uint32_t ovf_stride;
    int sp;
    int bot;

    __device__ __forceinline__ uint2 &slot(int i) { return lds[(i & (kRing8 - 1)) * kTraceBlock]; }
    __device__ __forceinline__ void reset() { sp = bot = 0; }
    // room for two pushes (create() bounds the tree: 2 entries per level fit)
    __device__ __forceinline__ void reserve2() {
        if (sp + 2 - bot > kRing8 && 2 * (bot + kSpill8) <= kStackOvf) {
#pragma unroll
            for (int k = 0; k < kSpill8; k++) {
                const uint2 e = slot(bot + k);
                ovf[(uint32_t)(2 * (bot + k)) * ovf_stride] = (int)e.x;
                ovf[(uint32_t)(2 * (bot + k) + 1) * ovf_stride] = (int)e.y;
            }
            bot += kSpill8;
        }
    }
    __device__ __forceinline__ void push(uint2 v, bool keep) {
        slot(sp) = v;  // harmless above the top when !keep
        sp += keep ? 1 : 0;
    }
    __device__ __forceinline__ uint2 pop() {
        sp--;
        if (sp < bot) {
            bot -= kSpill8;
#pragma unroll
            for (int k = 0; k < kSpill8; k++)
                slot(bot + k) = make_uint2((uint32_t)ovf[(uint32_t)(2 * (bot + k)) * ovf_stride],
                                           (uint32_t)ovf[(uint32_t)(2 * (bot + k) + 1) * ovf_stride]);
        }
        return slot(sp);
    }
};

// bits of an 8-bit mask moved from position k to k ^ oct (three conditional delta swaps)
__device__ __forceinline__ uint32_t xor_permute8(uint32_t m, uint32_t oct) {
    uint32_t t = ((m >> 1) ^ m) & ((oct & 1u) ? 0x55u : 0u);
    m ^= t | (t << 1);
    t = ((m >> 2) ^ m) & ((oct & 2u) ? 0x33u : 0u);
    m ^= t | (t << 2);
    t = ((m >> 4) ^ m) & ((oct & 4u) ? 0x0Fu : 0u);
    return m ^ (t | (t << 4));
}

// BVH8 (A/B family): the per-node rounding bound of r02 (pt_traverse.h visit4 takes
// one per ray from DeviceScene::node_bound, which the engine computes for BVH4 only):
// E = fma(512, s, |o_node - o_ray| + |o_node|) * |idir| 2^-21 for this node's o and s
struct AxisTerms {
    float b;       // s * idir (exact)
    float an, af;  // (o_node - o_ray) * idir - E, + E
};
__device__ __forceinline__ AxisTerms axis_terms8(float onode, float s, float oray, float idir) {
    AxisTerms t;
    const float A = onode - oray;
    const float a = A * idir;
    const float e = __builtin_fmaf(512.f, s, fabsf(A) + fabsf(onode)) * (fabsf(idir) * 0x1p-21f);
    t.b = s * idir;
    t.an = a - e;
    t.af = a + e;
    return t;
}

// The eight child boxes of a Bvh8Node with visit4's conservative slab test.
// Returns the node-group word of the hit internal children (priority order) and
// the record-slot bits of the hit leaf children.
__device__ __forceinline__ void visit8(const uint4 w0, const uint4 w2, const uint4 w3, const uint4 w4, uint32_t pvalid,
                                       vec3 ro, vec3 ridir, float tmin, float tmax, uint32_t oct, uint32_t &group,
                                       uint32_t &pbits) {
    const float ox = __uint_as_float(w0.x), oy = __uint_as_float(w0.y), oz = __uint_as_float(w0.z);
    const uint32_t exps = w0.w;
    const float sx = __uint_as_float((exps & 0xFFu) << 23);
    const float sy = __uint_as_float(((exps >> 8) & 0xFFu) << 23);
    const float sz = __uint_as_float(((exps >> 16) & 0xFFu) << 23);
    const bool px = ridir.x >= 0.f, py = ridir.y >= 0.f, pz = ridir.z >= 0.f;
    // w2 = qlo_x[2], qhi_x[2]; w3 = y; w4 = z
    const uint32_t nx0 = px ? w2.x : w2.z, nx1 = px ? w2.y : w2.w, fx0 = px ? w2.z : w2.x, fx1 = px ? w2.w : w2.y;
    const uint32_t ny0 = py ? w3.x : w3.z, ny1 = py ? w3.y : w3.w, fy0 = py ? w3.z : w3.x, fy1 = py ? w3.w : w3.y;
    const uint32_t nz0 = pz ? w4.x : w4.z, nz1 = pz ? w4.y : w4.w, fz0 = pz ? w4.z : w4.x, fz1 = pz ? w4.w : w4.y;
    const AxisTerms X = axis_terms8(ox, sx, ro.x, ridir.x);
    const AxisTerms Y = axis_terms8(oy, sy, ro.y, ridir.y);
    const AxisTerms Z = axis_terms8(oz, sz, ro.z, ridir.z);
    uint32_t acc = 0u;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint32_t nx = k < 4 ? nx0 : nx1, ny = k < 4 ? ny0 : ny1, nz = k < 4 ? nz0 : nz1;
        const uint32_t fx = k < 4 ? fx0 : fx1, fy = k < 4 ? fy0 : fy1, fz = k < 4 ? fz0 : fz1;
        const float tn = fmaxf(fmaxf(fmaxf(__builtin_fmaf(ubyte(nx, k & 3), X.b, X.an), __builtin_fmaf(ubyte(ny, k & 3), Y.b, Y.an)),
                                     __builtin_fmaf(ubyte(nz, k & 3), Z.b, Z.an)),
                               tmin);
        const float tf = fminf(fminf(fminf(__builtin_fmaf(ubyte(fx, k & 3), X.b, X.af), __builtin_fmaf(ubyte(fy, k & 3), Y.b, Y.af)),
                                     __builtin_fmaf(ubyte(fz, k & 3), Z.b, Z.af)),
                               tmax);
        acc |= tn <= tf ? ((1u << (24 + k)) | (3u << (2 * k))) : 0u;
    }
    const uint32_t imask = exps >> 24;
    pbits = acc & pvalid;
    group = (xor_permute8((acc >> 24) & imask, oct) << 24) | (imask << 16);
}

template <int MODE, bool ANY, bool STATS>
__device__ __forceinline__ void trace8_body(const DeviceScene &sc, const PathState &ps, const Queues &q,
                                            const TraceJob &job, int *ovf, uint32_t ovf_threads,
                                            const TraceStats &stats, uint2 *s_ring) {
    const uint32_t n_next = MODE == kModeMixed ? q.counts[kCntNext] : 0u;
    const uint32_t count =
        MODE == kModeShadow ? q.counts[kCntShadow]
                            : (MODE == kModeMixed ? n_next + q.counts[kCntShadow]
                                                  : (job.count_ptr ? *job.count_ptr : job.static_count));
    const uint32_t *shadow_q = MODE == kModeShadow ? q.nxsh + q.counts[kStartShadow] : nullptr;
    RingStack8 st;
    st.lds = s_ring + threadIdx.x;
    st.ovf = ovf + blockIdx.x * blockDim.x + threadIdx.x;
    st.ovf_stride = ovf_threads;
    st.reset();
    uint32_t nv = 0, npt = 0, nv_sh = 0, npt_sh = 0;
    uint32_t n_unique = 0;
    unsigned long long dg[6] = {0, 0, 0, 0, 0, 0};
    bool active = false, drained = false;
    uint32_t shard = blockIdx.x % kWorkShards, tried = 0;
    unsigned long long t_start = 0, t_drained = 0, n_taken = 0;
    uint32_t q_handed = 0, q_act = 0, q_ret = 0;  // STATS queue accounting, as trace4_body
    if (STATS && stats.wave_times) t_start = __builtin_amdgcn_s_memrealtime();
    uint32_t p = 0, best_key = 0, best_idx = kMissIndex;
    RayPre r{};
    float tmin = MODE == kModeRays ? 0.f : 0.001f, tmax = 0.f, b1 = 0.f, b2 = 0.f;  // tmin: a constant outside kModeRays
    uint32_t gbase = 0, gbits = 0, tbase = 0, tbits = 0, oct = 0;
    bool found = false;
    bool any = ANY;
    for (;;) {
        // ---- refill idle lanes (one atomic per wave), as trace4_body
        const unsigned long long idle = __ballot(!active);
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        if (!drained && n_idle >= job.refill) {
            uint32_t lo, len, len_e = 0, lo_s = 0;
            if (MODE == kModeMixed) {
                const uint32_t n_sh = count - n_next;
                lo = (uint32_t)((uint64_t)n_next * shard / kWorkShards);
                len_e = (uint32_t)((uint64_t)n_next * (shard + 1) / kWorkShards) - lo;
                lo_s = n_next + (uint32_t)((uint64_t)n_sh * shard / kWorkShards);
                len = len_e + (n_next + (uint32_t)((uint64_t)n_sh * (shard + 1) / kWorkShards) - lo_s);
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
            if (base + n_idle >= len) {
                shard = shard + 1 == kWorkShards ? 0u : shard + 1;
                if (++tried == kWorkShards) {
                    drained = true;
                    if (STATS && stats.wave_times) t_drained = __builtin_amdgcn_s_memrealtime();
                }
            }
            if (!active) {
                const uint32_t k = base + (uint32_t)__popcll(idle & lanemask_lt());
                const uint32_t i = MODE == kModeMixed && k >= len_e ? lo_s + (k - len_e) : lo + k;
                if (k < len) {
                    float4 o, d;
                    if (MODE == kModeExtend) {
                        p = job.queue ? job.queue[i] : (job.spp ? (i % job.spp) * job.num_local + i / job.spp : i);
                        o = ps.ray_o[p];
                        d = ps.ray_d[p];
                        tmin = 0.001f;
                        tmax = kMaxDistance;
                    } else if (MODE == kModeShadow) {
                        p = shadow_q[i];
                        o = ps.ray_o[p];
                        d = ps.sh_d[p];
                        tmin = 0.001f;
                        tmax = o.w;
                    } else if (MODE == kModeMixed) {
                        p = q.nxsh[i];
                        any = i >= n_next;
                        o = ps.ray_o[p];
                        d = any ? ps.sh_d[p] : ps.ray_d[p];
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
                    oct = (r.idir.x < 0.f ? 1u : 0u) | (r.idir.y < 0.f ? 2u : 0u) | (r.idir.z < 0.f ? 4u : 0u);
                    best_key = 0xFFFFFFFFu;
                    best_idx = kMissIndex;
                    b1 = b2 = 0.f;
                    found = false;
                    st.reset();
                    const int root = (int)sc.root_link8;
                    gbase = 0u;
                    tbase = 0u;
                    gbits = root == kSentinel || root < 0 ? 0u : (1u << (24 + oct)) | (1u << 16);  // node 0 in slot 0
                    tbits = root < 0 ? (1u << leaf_count(root)) - 1u : 0u;  // leaf root: records 0..n-1
                    active = true;
                }
            }
            if (STATS) q_act += (uint32_t)__popcll(__ballot(active && !was_active));
        }
        if (!__any(active)) {
            if (drained) break;
            continue;
        }
        if (active) {
            // ---- node phase: descend until this lane has leaf work and most of the wave does
            for (;;) {
                if (gbits < (1u << 24)) {  // no node group in hand
                    if (tbits != 0u || st.sp == 0) break;
                    const uint2 e = st.pop();
                    if (e.y < (1u << 16)) {  // triangle group
                        tbase = e.x;
                        tbits = e.y;
                        break;
                    }
                    gbase = e.x;
                    gbits = e.y;
                }
                const uint32_t j = (uint32_t)__builtin_ctz(gbits >> 24);
                gbits &= ~(1u << (24 + j));
                const uint32_t k = j ^ oct;
                const uint32_t child = gbase + (uint32_t)__builtin_popcount((gbits >> 16) & ((1u << k) - 1u));
                st.reserve2();
                st.push(make_uint2(gbase, gbits), gbits >= (1u << 24));
                const uint4 *np = reinterpret_cast<const uint4 *>(sc.nodes8 + child);
                const uint4 w0 = np[0], w1 = np[1], w2 = np[2], w3 = np[3], w4 = np[4];
                if (STATS) {
                    if (MODE == kModeMixed && any) nv_sh++;
                    else nv++;
                    const unsigned long long m = __ballot(true);
                    if ((int)lane_id() == __ffsll((long long)m) - 1) {
                        dg[0]++;
                        dg[1] += (unsigned long long)__popcll(m);
                    }
                    bool dup = false;
                    for (int jj = 0; jj < 64; jj++) {
                        const uint32_t cj = __shfl(child, jj);
                        if (jj < (int)lane_id() && ((m >> jj) & 1ull) && cj == child) dup = true;
                    }
                    n_unique += dup ? 0u : 1u;
                }
                uint32_t ng, nb;
                visit8(w0, w2, w3, w4, w1.y, r.o, r.idir, tmin, tmax, oct, ng, nb);
                if (nb) {
                    if (tbits == 0u) {
                        tbase = child;
                        tbits = nb;
                    } else {
                        st.push(make_uint2(child, nb), true);
                    }
                }
                gbase = w1.x;
                gbits = ng;
                // leave for the leaf phase once fewer than node_min lanes still have no leaf work
                if ((uint32_t)__popcll(__ballot(tbits == 0u)) < job.node_min) break;
            }
            // ---- leaf phase: one leaf child (its two record slots, loads issued together) per step
            while (tbits != 0u) {
                if (STATS) {
                    const unsigned long long m = __ballot(true);
                    if ((int)lane_id() == __ffsll((long long)m) - 1) {
                        dg[2]++;
                        dg[3] += (unsigned long long)__popcll(m);
                    }
                }
                const uint32_t j = (uint32_t)__builtin_ctz(tbits) & ~1u;
                const uint32_t pair = (tbits >> j) & 3u;
                tbits &= ~(3u << j);
                const uint32_t i0 = kLeafSlots * tbase + j;
                // both slots exist in the node's record block (holes are zero records)
                const float4 a0 = sc.prims[3 * i0 + 0], bb0 = sc.prims[3 * i0 + 1], c0 = sc.prims[3 * i0 + 2];
                const float4 a1 = sc.prims[3 * i0 + 3], bb1 = sc.prims[3 * i0 + 4], c1 = sc.prims[3 * i0 + 5];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    if (!((pair >> h) & 1u)) continue;
                    const float4 a = h ? a1 : a0, b = h ? bb1 : bb0, c = h ? c1 : c0;
                    if (STATS) {
                        if (MODE == kModeMixed && any) npt_sh++;
                        else npt++;
                    }
                    const uint32_t ref = __float_as_uint(a.w);
                    const uint32_t key = ref & ~kPrimSphereBit;
                    float t, hb1 = 0.f, hb2 = 0.f;
                    bool hit;
                    if (ref & kPrimSphereBit) {
                        const DevInstance &in = sc.instances[__float_as_uint(b.w)];
                        hit = intersect_unit_sphere(in.to_object, r.o, r.d, tmin, tmax, t);
                    } else {
                        hit = intersect_triangle(r, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z), tmin, tmax,
                                                 t, hb1, hb2);
                    }
                    if (hit) {
                        if (any) {
                            found = true;
                            break;
                        }
                        if (t < tmax || key < best_key) {
                            tmax = t;
                            best_key = key;
                            best_idx = i0 + (uint32_t)h;
                            b1 = hb1;
                            b2 = hb2;
                            found = true;
                        }
                    }
                }
                if (any && found) break;
            }
        }
        const bool done = active && ((gbits < (1u << 24) && tbits == 0u && st.sp == 0) || (any && found));
        // ---- retire
        if (MODE == kModeExtend || MODE == kModeMixed) {
            if (done && !any) {
                uint32_t bin = 0;
                ps.hit[p] = make_float4(found ? tmax : -1.f, b1, b2, __uint_as_float(found ? best_idx : kMissIndex));
                if (found) {
                    const uint32_t mt = __float_as_uint(sc.prims[3 * best_idx + 2].w);
                    bin = (mt >= 1u && mt <= 7u) ? mt : 8u;
                }
                ps.mbin[p] = (uint8_t)bin;
            }
        }
        if (MODE == kModeShadow || MODE == kModeMixed) {
            if (done && any && !found) {  // main.cu:124-139
                const float4 c = ps.sh_c[p];
                float4 L = ps.rad[p];
                L.x = L.x + c.x;
                L.y = L.y + c.y;
                L.z = L.z + c.z;
                ps.rad[p] = L;
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
    flush_stats<STATS>(&stats, nv, npt, MODE == kModeShadow ? 14 : 0);
    if (MODE == kModeMixed) flush_stats<STATS>(&stats, nv_sh, npt_sh, 14);
    flush_stats<STATS>(&stats, n_unique, 0u, 18);
    if (STATS && stats.wave_times && lane_id() == 0) {
        unsigned long long *w = stats.wave_times + 4ull * (blockIdx.x * (blockDim.x / 64u) + threadIdx.x / 64u);
        w[0] = t_start;
        w[1] = t_drained;
        w[2] = __builtin_amdgcn_s_memrealtime();
        w[3] = n_taken;
    }
    if (lane_id() == 0) {  // the last wave out resets the work counters (see trace4_body)
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
            if (STATS) atomicAdd(&stats.counters[23], (unsigned long long)count);  // once per launch
        }
    }
    if (STATS) {
        for (int k = 0; k < 6; k++) {
            unsigned long long v = dg[k];
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            dg[k] = v;
        }
        if (lane_id() == 0)
            for (int k = 0; k < 6; k++) atomicAdd(&stats.counters[(MODE == kModeShadow ? 8 : 2) + k], dg[k]);
    }
}

template <int MODE, bool ANY, bool STATS>
__global__ __launch_bounds__(kTraceBlock) __attribute__((amdgpu_waves_per_eu(kTraceWavesPerSimd8))) void k_trace8(
    DeviceScene sc, PathState ps, Queues q, TraceJob job, int *ovf, uint32_t ovf_threads, TraceStats stats) {
    __shared__ uint2 s_ring8[kRing8 * kTraceBlock];
    trace8_body<MODE, ANY, STATS>(sc, ps, q, job, ovf, ovf_threads, stats, s_ring8);
}


// ------------------------------------------------------------------ verification kernels
__global__ __launch_bounds__(kTraceBlock) void k_trace_debug(DeviceScene sc, const float *rays, float *out,
                                                             uint32_t n, int any, int *ovf, uint32_t ovf_threads) {
    __shared__ int s_stack[kStackLds * kTraceBlock];
    // grid-stride over at most ovf_threads threads: thread g owns overflow column g
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    Stack st;
    st.lds = s_stack + threadIdx.x;
    st.ovf = ovf + g;
    st.ovf_stride = ovf_threads;
    for (uint32_t i = g; i < n; i += gridDim.x * blockDim.x) {
    const float *r8 = rays + 8 * (size_t)i;
    const RayPre r = ray_pre(v3(r8[0], r8[1], r8[2]), v3(r8[3], r8[4], r8[5]));
    float tmax = r8[7];
    uint32_t key = 0xFFFFFFFFu, idx = kMissIndex, nv = 0, pt = 0;
    float b1 = 0.f, b2 = 0.f;
    bool hit;
    if (sc.bvh_width == 4) {
        if (any) hit = traverse4<true, false>(sc, r, r8[6], tmax, key, idx, b1, b2, st, nv, pt);
        else hit = traverse4<false, false>(sc, r, r8[6], tmax, key, idx, b1, b2, st, nv, pt);
    } else {
        if (any) hit = traverse<true, false>(sc, r, r8[6], tmax, key, idx, b1, b2, st, nv, pt);
        else hit = traverse<false, false>(sc, r, r8[6], tmax, key, idx, b1, b2, st, nv, pt);
    }
    float *o = out + 4 * (size_t)i;
    o[0] = hit ? (any ? 1.f : tmax) : -1.f;
    o[1] = b1;
    o[2] = b2;
    o[3] = __uint_as_float(hit && !any ? key : 0xFFFFFFFFu);
    }
}


}  // namespace

void launch_trace8(int mode, bool any, const DeviceScene &sc, const PathState &ps, const Queues &q,
                   const tr::TraceJob &job, int *ovf, uint32_t ovf_threads, const TraceStats *stats, hipStream_t s) {
    const TraceStats st = stats ? *stats : TraceStats{nullptr};
    const dim3 g(trace4_blocks(sc, ovf_threads)), b(kTraceBlock);
#define K8(M, A)                                                                                                   \
    do {                                                                                                           \
        if (stats) hipLaunchKernelGGL((k_trace8<M, A, true>), g, b, 0, s, sc, ps, q, job, ovf, ovf_threads, st);  \
        else hipLaunchKernelGGL((k_trace8<M, A, false>), g, b, 0, s, sc, ps, q, job, ovf, ovf_threads, st);       \
    } while (0)
    switch (mode) {  // the engine pipelines frames (kModeMixedAhead) on BVH4 trees only
    case kModeExtend: K8(kModeExtend, false); break;
    case kModeShadow: K8(kModeShadow, true); break;
    case kModeMixed: K8(kModeMixed, false); break;
    case kModeRays:
        if (any) K8(kModeRays, true);
        else K8(kModeRays, false);
        break;
    default: break;
    }
#undef K8
}

void launch_extend_lanes(const DeviceScene &sc, const PathState &ps, const Queues &q, const uint32_t *queue,
                         const uint32_t *queue_count, uint32_t static_count, int *ovf, uint32_t ovf_threads,
                         const TraceStats *stats, hipStream_t s) {
    const uint32_t blocks = ovf_threads / kTraceBlock;
    const TraceStats st = stats ? *stats : TraceStats{nullptr};
    const bool w4 = sc.bvh_width == 4;
#define EXTEND(S, W)                                                                                      \
    hipLaunchKernelGGL((k_extend<S, W>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, queue, queue_count, \
                       static_count, ovf, ovf_threads, st)
    if (stats) {
        if (w4) EXTEND(true, 4);
        else EXTEND(true, 2);
    } else {
        if (w4) EXTEND(false, 4);
        else EXTEND(false, 2);
    }
#undef EXTEND
}

void launch_shadow_lanes(const DeviceScene &sc, const PathState &ps, const Queues &q, int *ovf, uint32_t ovf_threads,
                         const TraceStats *stats, hipStream_t s) {
    const uint32_t blocks = ovf_threads / kTraceBlock;
    const TraceStats st = stats ? *stats : TraceStats{nullptr};
    const bool w4 = sc.bvh_width == 4;
#define SHADOW(S, W) \
    hipLaunchKernelGGL((k_shadow<S, W>), dim3(blocks), dim3(kTraceBlock), 0, s, sc, ps, q, ovf, ovf_threads, st)
    if (stats) {
        if (w4) SHADOW(true, 4);
        else SHADOW(true, 2);
    } else {
        if (w4) SHADOW(false, 4);
        else SHADOW(false, 2);
    }
#undef SHADOW
}

void launch_trace_debug_lanes(const DeviceScene &sc, const float *rays, float *out, uint32_t n, int any, int *ovf,
                              uint32_t ovf_threads, hipStream_t s) {
    const uint32_t blocks = std::min((n + kTraceBlock - 1) / kTraceBlock, std::max(1u, ovf_threads / kTraceBlock));
    hipLaunchKernelGGL(k_trace_debug, dim3(blocks), dim3(kTraceBlock), 0, s, sc, rays, out, n, any, ovf, ovf_threads);
}

}  // namespace pupil
