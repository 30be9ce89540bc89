// pt_traverse.h — device code of the persistent BVH4 traversal kernels
// (pt_kernels.hip: path tracing launches and the ray-query verification launch):
// leaf tests, the LDS ring stack, the persistent-kernel job descriptor and the
// quantized BVH4 box test.
#pragma once

#include "pt_kernels.h"
#include "pt_shading.h"
#include "pt_trace.h"

namespace pupil {
namespace tr {

constexpr int kSentinel = kTraverseDone;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ vec3 f3(float4 v) { return v3(v.x, v.y, v.z); }
__device__ __forceinline__ float4 f4(vec3 v, float w) { return make_float4(v.x, v.y, v.z, w); }
// every camera ray's origin (main.cu:53-75: the camera-to-world translation)
__device__ __forceinline__ vec3 camera_origin(const Camera &cam) { return v3(cam.c2w[3], cam.c2w[7], cam.c2w[11]); }

// Leaf intersection (flattened BVH4 and two-level world mode).  any = terminate on the first
// hit (shadow ray); a compile-time constant except in the mixed persistent kernel.
// dirf(): the ray direction, for sphere records only (the traversal may reload it instead of
// keeping it live)
template <bool STATS, typename DirF>
__device__ __forceinline__ bool intersect_leaf_dyn(const DeviceScene &sc, const RayPre &r, int leaf, float tmin,
                                                   float &tmax, uint32_t &best_key, uint32_t &best_idx, float &bb1,
                                                   float &bb2, uint32_t &prims_tested, bool &found, bool any,
                                                   DirF dirf) {
    const uint32_t first = leaf_first(leaf);
    const uint32_t count = leaf_count(leaf);
    for (uint32_t i = first; i < first + count; i++) {
        const float4 a = sc.prims[kRecF4 * i + 0];
        const float4 b = sc.prims[kRecF4 * i + 1];
        const float4 c = sc.prims[kRecF4 * i + 2];
        // the whole 48-B record in one round trip: without this the compiler sinks the
        // vertex loads below the sphere-bit branch, a second dependent fetch per record
        asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w), "v"(b.x), "v"(b.y), "v"(b.z), "v"(b.w), "v"(c.x),
                     "v"(c.y), "v"(c.z));
        const uint32_t ref = __float_as_uint(a.w);
        const uint32_t key = ref & ~kPrimSphereBit;
        if (STATS) prims_tested++;
        float t, b1 = 0.f, b2 = 0.f;
        bool hit;
        if (ref & kPrimSphereBit) {
            const DevInstance &in = sc.instances[__float_as_uint(b.w)];
            hit = intersect_unit_sphere(in.to_object, r.o, dirf(), tmin, tmax, t);
        } else {
            hit = intersect_triangle(r, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z), tmin, tmax, t, b1,
                                     b2);
        }
        if (hit) {
            if (any) {
                found = true;
                return true;
            }
            if (t < tmax || key < best_key) {
                tmax = t;
                best_key = key;
                best_idx = i;
                bb1 = b1;
                bb2 = b2;
                found = true;
            }
        }
    }
    return false;
}

// Two-level BLAS leaf: object-space triangle records of instance `inst`,
// tested in world space on fl(to_world * v) (the flattened build's and the
// oracle's world vertices), keyed by the global primitive id.
template <bool STATS>
__device__ __forceinline__ bool intersect_leaf_tl(const DeviceScene &sc, const RayPre &r, int leaf, uint32_t inst,
                                                  float tmin, float &tmax, uint32_t &best_key, uint32_t &best_idx,
                                                  float &bb1, float &bb2, uint32_t &prims_tested, bool &found,
                                                  bool any) {
    // the instance's world-space records (fl(to_world * v), precomputed per instance):
    // no per-triangle transform in the loop
    const float4 *rec = sc.wprims + kRecF4 * (int64_t)sc.instances[inst].wrec_delta;
    const uint32_t first = leaf_first(leaf);
    const uint32_t count = leaf_count(leaf);
    for (uint32_t i = first; i < first + count; i++) {
        const float4 a = rec[kRecF4 * i + 0];
        const float4 b = rec[kRecF4 * i + 1];
        const float4 c = rec[kRecF4 * i + 2];
        const uint32_t key = __float_as_uint(a.w);
        if (STATS) prims_tested++;
        float t, b1 = 0.f, b2 = 0.f;
        if (intersect_triangle(r, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), v3(c.x, c.y, c.z), tmin, tmax, t, b1, b2)) {
            if (any) {
                found = true;
                return true;
            }
            if (t < tmax || key < best_key) {
                tmax = t;
                best_key = key;
                best_idx = key;
                bb1 = b1;
                bb2 = b2;
                found = true;
            }
        }
    }
    return false;
}

// counters[0..1]: closest-hit (extend / ray queries), counters[14..15]: shadow
template <bool STATS>
__device__ __forceinline__ void flush_stats(const TraceStats *stats, uint32_t nv, uint32_t pt, int base = 0) {
    if (!STATS) return;
    // wave reduction then one atomic per wave
    unsigned long long a = nv, b = pt;
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        b += __shfl_xor(b, o);
    }
    if (lane_id() == 0) {
        atomicAdd(&stats->counters[base + 0], a);
        atomicAdd(&stats->counters[base + 1], b);
    }
}


// ------------------------------------------------------------------ persistent 4-wide traversal
// The production trace kernels for the quantized BVH4.  Waves are persistent
// and pull rays from the queue with one atomic per wave; a lane whose ray has
// terminated is refilled as soon as `refill` lanes of its wave are idle
// (Aila & Laine 2009, "dynamic fetch"), so a wave never idles on its longest
// ray.  The stack is a 16-entry LDS column per lane that spills its bottom 8
// entries to HBM when full, so push/pop are LDS-only in the common case.
constexpr int kSpill = 8;

// Entries [0, sp) of the LDS column in order, [0, nsp) in the overflow column (r05: replaces
// r01-r04's ring with a wrap mask and three conditional pushes, 141 -> 132 VALU per node visit
// with a hit, launch time unchanged: profiles/r05_stack_ab.txt).  A visit's pushes are three unconditional
// stores at sp, sp + 1, sp + 2 of the hit children's links in push order (far to near; the
// slots above the new top are harmless) and one add, instead of three conditional pushes;
// a full column spills its bottom 8 entries and moves the top ones down (rare: deep trees).
// Popping an empty child slot (kEmptyLink, possible only for degenerate child boxes whose
// empty planes the conservative slab bound lets through) pops again.
template <int RING, int OVF, int SPILL = (RING >= 11 ? kSpill : RING / 2)>
struct LinStackT {
    int *lds;  // this lane's column (stride kTraceBlock)
    int *ovf_blk;
    const int *lds0;
    __device__ __forceinline__ int *ovf_col() {
        uint32_t lane;
        asm volatile("v_mov_b32 %0, %1" : "=v"(lane) : "v"((uint32_t)(lds - lds0)));
        return ovf_blk + lane;
    }
    uint32_t ovf_stride;
    int sp;   // entries in the LDS column
    int nsp;  // entries in the overflow column (multiple of SPILL)
    // counter kernels only (null otherwise, compiled out): the entry distance of every LDS
    // entry in a parallel column, so a pop can tell whether the node lies beyond the ray's
    // current tmax (PUPIL_TRACE_DIAG "cullable visits"); entries reloaded from the overflow
    // column read 0 (unknown)
    float *tcol = nullptr;
    float tpop = 0.f;  // the last popped entry's distance

    __device__ __forceinline__ int &slot(int i) { return lds[i * kTraceBlock]; }
    __device__ __forceinline__ void reset() { sp = nsp = 0; }
    __device__ __forceinline__ void reserve3() {
        if (sp > RING - 3 && nsp + SPILL <= OVF) {
            int *ovf = ovf_col();
#pragma unroll
            for (int k = 0; k < SPILL; k++) ovf[(uint32_t)(nsp + k) * ovf_stride] = slot(k);
#pragma unroll
            for (int k = SPILL; k < RING; k++)
                if (k < sp) {
                    slot(k - SPILL) = slot(k);
                    if (tcol) tcol[(k - SPILL) * kTraceBlock] = tcol[k * kTraceBlock];
                }
            nsp += SPILL;
            sp -= SPILL;
        }
    }
    __device__ __forceinline__ void push(int v) {
        if (tcol) tcol[sp * kTraceBlock] = 0.f;
        slot(sp++) = v;
    }
    __device__ __forceinline__ void push3t(float t1, float t2, float t3, bool c2, bool c3) {
        if (!tcol) return;
        tcol[sp * kTraceBlock] = c3 ? t3 : (c2 ? t2 : t1);
        tcol[(sp + 1) * kTraceBlock] = c3 ? t2 : t1;
        tcol[(sp + 2) * kTraceBlock] = t1;
    }
    // the hit children of positions 1..3 of a sorted visit (c1 >= c2 >= c3: hits first)
    __device__ __forceinline__ void push3(int l1, int l2, int l3, bool c1, bool c2, bool c3) {
        slot(sp) = c3 ? l3 : (c2 ? l2 : l1);
        slot(sp + 1) = c3 ? l2 : l1;
        slot(sp + 2) = l1;
        sp += (c1 ? 1 : 0) + (c2 ? 1 : 0) + (c3 ? 1 : 0);
    }
    __device__ __forceinline__ int pop_raw() {
        if (sp == 0) {
            if (nsp == 0) return kSentinel;
            nsp -= SPILL;
            const int *ovf = ovf_col();
#pragma unroll
            for (int k = 0; k < SPILL; k++) {
                slot(k) = ovf[(uint32_t)(nsp + k) * ovf_stride];
                if (tcol) tcol[k * kTraceBlock] = 0.f;
            }
            sp = SPILL;
        }
        --sp;
        if (tcol) tpop = tcol[sp * kTraceBlock];
        return slot(sp);
    }
    __device__ __forceinline__ int pop() {
        int v = pop_raw();
        while (v == kEmptyLink) v = pop_raw();
        return v;
    }
    // distance stack (PUPIL_DIST_STACK builds, tcol set): also skips entries whose conservative
    // entry distance (the box test's lowered near plane, pushed with the link) already exceeds
    // the ray's current tmax -- no primitive inside can be hit at t <= tmax, so the visit the
    // pop would cause could only fail; entries reloaded from the overflow column read 0
    __device__ __forceinline__ int pop_live(float tmax) {
        int v = pop_raw();
        while (v != kSentinel && (v == kEmptyLink || tpop > tmax)) v = pop_raw();
        return v;
    }
};
using LinStack = LinStackT<kRing, kStackOvf>;

// Child order of a BVH4 visit: the nearest child is descended, the others pushed far to
// near (r03: partial sorts with 4 or 3 comparators were no faster).  Only the traversal
// order depends on it: hits are resolved by the (t, id) total order either way.

// Branch-free compare-exchange (selects, no divergent swap blocks).
__device__ __forceinline__ void csel(float &ta, int &la, float &tb, int &lb) {
    const bool c = tb < ta;
    const float t0 = c ? tb : ta, t1 = c ? ta : tb;
    const int l0 = c ? lb : la, l1 = c ? la : lb;
    ta = t0;
    tb = t1;
    la = l0;
    lb = l1;
}

// kModeMixed: one launch over the concatenated next + shadow lists of a bounce
// (q.nxsh[0, cnt_next) extension rays, then cnt_shadow shadow rays), so each
// bounce pays one persistent-kernel tail instead of two.
// kModeMixedAhead: kModeMixed plus the next render's camera rays (render-ahead,
// TraceJob::ahead_off); a separate instance so the plain mixed kernel keeps its registers
// (value 1, the separate any-hit launch of r01, is retired; the numbers name the kernel instances)
enum TraceMode : int { kModeExtend = 0, kModeRays = 2, kModeMixed = 3, kModeMixedAhead = 4 };

struct TraceJob {
    const uint32_t *queue;      // extend: path ids (null = identity)
    const uint32_t *count_ptr;  // device count (null = static_count)
    uint32_t static_count;
    uint32_t *work;             // kWorkKind counters: heads, final and sub exit counters (stride kWorkStride), zero at launch
    uint32_t refill;            // refill when at least this many lanes are idle (1..64)
    uint32_t node_min;          // node phase ends when fewer lanes than this still need a node (>= 1)
    const float *rays;          // kModeRays: 8 floats per ray (o, d, tmin, tmax)
    float *out;                 // kModeRays: 4 floats per ray
    // primary extend (queue == null): list position i -> path (i % spp) * num_local + i / spp,
    // so consecutive lanes take the spp samples of one pixel (coherent camera rays) while
    // path ids stay sample major; spp = 0: identity
    uint32_t spp;
    uint32_t num_local;
    // kModeMixedAhead (render-ahead, engine.hip): static_count camera rays of the next render
    // ride along; the path state passed is the base of both halves of the buffers, list path
    // ids are offset by list_base (this render's half), ahead position j -> path (pixel-major
    // as above) + ahead_base (the other half); both offsets are non-negative
    uint32_t list_base;
    uint32_t ahead_base;
};

__device__ __forceinline__ float ubyte(uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xFFu); }

// One node of the quantized BVH4.  Child plane k on an axis is
// P = o_node + q_k * s (s a power of two, so q_k * s is exact; the builder
// verified that fl(P) bounds the child box).  The slab distance is evaluated as
//     t = fma(q_k, s * idir, fma(o_node - o_ray, idir, -/+E))
// i.e. one fma per plane and three operations per axis and node shared by the four
// children.  E bounds every rounding against the exact (fl(P) - o_ray) / d
// (u = 2^-24; subtraction, both fmas, idir, fl(P) vs P):
//   u |idir| (5 |o_node| + 4 |o_ray| + 765 s) + 2u E
// and is taken per RAY, not per node: with M >= |o_node| + 512 s over every node
// (DeviceScene::node_bound, launch_node_bound)
//   E = (|o_ray| + M) |idir| 2^-21   (2^-21 = 8u)
// covers it with room for its own two roundings.  Near planes are lowered and far
// planes raised by E, so the test is conservative: a box containing a primitive the
// exact test would report is never culled, and closest hits stay independent of the
// BVH.  Overflow (huge idir) gives +-inf/NaN planes, which fmaxf/fminf ignore (IEEE
// maxNum), i.e. no culling on that axis.  (r02/r03 evaluated E per node from that
// node's o and s: 7 operations per axis instead of 3.)
__device__ __forceinline__ float slab_error(float oray, float idir, float bound) {
    return (fabsf(oray) + bound) * (fabsf(idir) * 0x1p-21f);
}
// two-level BLAS nodes: the object-space ray carries a position margin `pad`
// (DevInstance::margin), added to the bound before scaling by |idir|
__device__ __forceinline__ float slab_error_pad(float oray, float idir, float bound, float pad) {
    return __builtin_fmaf(fabsf(oray) + bound, 0x1p-21f, pad) * fabsf(idir);
}
__device__ __forceinline__ vec3 slab_errors(vec3 o, vec3 idir, const float bound[3]) {
    return v3(slab_error(o.x, idir.x, bound[0]), slab_error(o.y, idir.y, bound[1]), slab_error(o.z, idir.z, bound[2]));
}

__device__ __forceinline__ void visit4(const Bvh4Node &n, vec3 ro, vec3 ridir, vec3 e, float tmin, float tmax,
                                       float t[4], int l[4]) {
    constexpr float kInf = __builtin_huge_valf();
    const bool px = ridir.x >= 0.f, py = ridir.y >= 0.f, pz = ridir.z >= 0.f;
    const uint32_t nx = px ? n.qlo_x : n.qhi_x, fx = px ? n.qhi_x : n.qlo_x;
    const uint32_t ny = py ? n.qlo_y : n.qhi_y, fy = py ? n.qhi_y : n.qlo_y;
    const uint32_t nz = pz ? n.qlo_z : n.qhi_z, fz = pz ? n.qhi_z : n.qlo_z;
    const float ax = n.ox - ro.x, ay = n.oy - ro.y, az = n.oz - ro.z;
    const float bx = n.sx * ridir.x, by = n.sy * ridir.y, bz = n.sz * ridir.z;
    const float nearx = __builtin_fmaf(ax, ridir.x, -e.x), farx = __builtin_fmaf(ax, ridir.x, e.x);
    const float neary = __builtin_fmaf(ay, ridir.y, -e.y), fary = __builtin_fmaf(ay, ridir.y, e.y);
    const float nearz = __builtin_fmaf(az, ridir.z, -e.z), farz = __builtin_fmaf(az, ridir.z, e.z);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const float tn = fmaxf(fmaxf(fmaxf(__builtin_fmaf(ubyte(nx, k), bx, nearx), __builtin_fmaf(ubyte(ny, k), by, neary)),
                                     __builtin_fmaf(ubyte(nz, k), bz, nearz)),
                               tmin);
        const float tf = fminf(fminf(fminf(__builtin_fmaf(ubyte(fx, k), bx, farx), __builtin_fmaf(ubyte(fy, k), by, fary)),
                                     __builtin_fmaf(ubyte(fz, k), bz, farz)),
                               tmax);
        l[k] = n.child[k];
        t[k] = tn <= tf ? tn : kInf;  // an empty slot (planes 255 / 0) passes only for degenerate boxes: LinStack
    }
    csel(t[0], l[0], t[1], l[1]);
    csel(t[2], l[2], t[3], l[3]);
    csel(t[0], l[0], t[2], l[2]);
    csel(t[1], l[1], t[3], l[3]);
    csel(t[1], l[1], t[2], l[2]);
}

// Node fetch by a 32-bit byte offset from the uniform base (the engine keeps node
// arrays to at most 2^26 nodes = 4 GiB, kMaxNodes4), which the compiler turns into
// SGPR-base + VGPR-offset loads: one VALU op per visit instead of a 64-bit shift and add.
__device__ __forceinline__ Bvh4Node load_node4(const DeviceScene &sc, int node) {
    return *reinterpret_cast<const Bvh4Node *>(reinterpret_cast<const char *>(sc.nodes4) + ((uint32_t)node << 6));
}

// ------------------------------------------------------------------ wave-cooperative node fetch (r06)
// The per-lane fetch above issues four 16-B loads per visit, and the CU's texture path charges
// each wave-instruction for all 64 lane slots (~16 cycles) plus every distinct 128-B line its
// lanes touch (~22 per load at config 4, the same lines four times per visit).
// Here the wave fetches each distinct node once, a quarter per lane: lanes 4k..4k+3 load node
// k's four 16-B quarters with one LDS-DMA wave-instruction (16 nodes, 1 KiB, each line touched
// once), and every lane then reads its node's 64 B from the wave's LDS image (4 ds_read_b128).
// Distinct nodes: a lane whose lower neighbour wants the same node shares its slot (adjacent
// lanes hold consecutive work-list items, which agree near the root); that is exact for runs of
// equal nodes, so slot = leaders below the lane, minus one for a follower.
// The LDS image is swizzled so the 16 lanes of a ds_read_b128 group meet 16 distinct bank
// quads: quarter c of slot k sits at 16-B position 4k + ((c + (k >> 2)) & 3); the DMA writes
// lane-linearly, so lane 4k + q loads quarter (q - (k >> 2)) & 3 (the swizzle goes on the
// source address, MI355X_MICROARCH.md LDS / cdna_hip_programming.md rule 21).
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int CHUNKS>
struct CoopFetch {
    uint32_t *addr;  // this wave's 64 node byte offsets (LDS)
    float4 *stage;   // this wave's 16 * CHUNKS node image (LDS)
    // STATS: LDS-DMA wave-instructions issued, node slots fetched
    uint32_t n_dma = 0, n_slots = 0;

    // Every lane of the wave calls this (full EXEC); lanes with `want` get node `node`.
    template <bool STATS>
    __device__ __forceinline__ Bvh4Node fetch(const Bvh4Node *nodes, int node, bool want) {
        const uint32_t lane = lane_id();
        // the lower neighbour's wanted node (wave_shr:1; lane 0 sees -1, which no node equals)
        const int key = want ? node : -1;
        const int below = __builtin_amdgcn_update_dpp(-1, key, 0x138, 0xF, 0xF, false);
        const bool lead = want && below != node;
        const unsigned long long ml = __ballot(lead);
        const uint32_t n = (uint32_t)__popcll(ml);
        const uint32_t slot = mbcnt64(ml) - (lead ? 0u : 1u);
        if (lead) addr[slot] = (uint32_t)node << 6;
        if (STATS && lane == 0) n_slots += n;
        const char *base = reinterpret_cast<const char *>(nodes);
        const uint32_t k = lane >> 2;
        const uint32_t src_q = ((lane & 3u) - (k >> 2)) & 3u;
        Bvh4Node out;
        float4 *o4 = reinterpret_cast<float4 *>(&out);
        for (uint32_t b = 0; b < n; b += 16u * CHUNKS) {
#pragma unroll
            for (int c = 0; c < CHUNKS; c++) {
                const uint32_t s = b + 16u * c + k;
                if (s < n) {
                    const uint32_t off = addr[s] + (src_q << 4);
                    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void *)(base + off),
                                                     (__attribute__((address_space(3))) void *)(stage + 64 * c), 16, 0,
                                                     0);
                }
                if (STATS && lane == 0 && b + 16u * c < n) n_dma++;
            }
            __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA writes have landed
            asm volatile("" ::: "memory");
            const uint32_t r = slot - b;
            if (want && r < 16u * CHUNKS) {
                const uint32_t sw = (r >> 2) & 3u;
                const float4 *src = stage + 4u * r;
#pragma unroll
                for (uint32_t c = 0; c < 4; c++) o4[c] = src[(c + sw) & 3u];
            }
            if (b + 16u * CHUNKS < n) {
                __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): reads done before the next DMA
                asm volatile("" ::: "memory");
            }
        }
        return out;
    }
};


}  // namespace tr
}  // namespace pupil
