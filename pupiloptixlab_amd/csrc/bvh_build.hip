// bvh_build.hip — GPU LBVH builder (replaces optixAccelBuild for the GAS/IAS,
// framework/world/gas_manager.cpp:130-173, ias_manager.cpp:54-96).
//
// Pipeline (all on device, one stream):
//   1. k_prim_setup    object-space meshes -> world-space primitive records +
//                      AABBs (instances flattened; spheres keep their instance)
//   2. k_bounds        scene centroid bounds (wave reduce + ordered-int atomics)
//   3. k_morton        30-bit Morton code of each centroid
//   4. radix sort      hand-written stable LSD sort, 8-bit digits, wave-ballot
//                      multisplit ranking (k_sort_hist / k_sort_scan / k_sort_scatter)
//   5. k_karras        Karras 2012 hierarchy over the sorted codes (index-augmented)
//   6. k_refit         bottom-up AABBs, agent-scope release/acquire per arrival
//   7. collapse        4-wide quantized nodes (SAH-optimal slot distribution);
//                      subtrees of <= leaf_size primitives become one leaf
//   8. k_reorder       primitive records in Morton order (leaf ranges index them)
//   9. k_attrs         per-primitive shading records in the same order
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "bvh4_quant.h"
#include "pt_kernels.h"

namespace pupil {

namespace {

constexpr int kBlock = 256;

struct Aabb {
    float lo[3];
    float hi[3];
};

__device__ __forceinline__ uint32_t float_to_ordered(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ordered_to_float(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

__global__ void k_prim_setup(BvhBuildInput in, float4 *recs, Aabb *boxes) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= in.num_prims) return;
    const uint32_t inst_id = in.prim_inst[i];
    const DevInstance &inst = in.instances[inst_id];
    const uint32_t mtype = in.materials[inst.material].type;
    const uint32_t bin = (mtype >= 1u && mtype <= 7u) ? mtype : 8u;
    Aabb b;
    if (inst.kind == PUPIL_SHAPE_SPHERE) {
        const float *m = inst.to_world;
        const vec3 c = v3(m[3], m[7], m[11]);
        // exact extents of an affinely transformed unit sphere, padded
        const float ex = sqrtf(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]) * 1.001f;
        const float ey = sqrtf(m[4] * m[4] + m[5] * m[5] + m[6] * m[6]) * 1.001f;
        const float ez = sqrtf(m[8] * m[8] + m[9] * m[9] + m[10] * m[10]) * 1.001f;
        b.lo[0] = c.x - ex; b.lo[1] = c.y - ey; b.lo[2] = c.z - ez;
        b.hi[0] = c.x + ex; b.hi[1] = c.y + ey; b.hi[2] = c.z + ez;
        recs[3 * i + 0] = make_float4(c.x, c.y, c.z, __uint_as_float(i | kPrimSphereBit));
        recs[3 * i + 1] = make_float4(ex, ey, ez, __uint_as_float(inst_id));
        recs[3 * i + 2] = make_float4(0.f, 0.f, 0.f, __uint_as_float(bin));
    } else {
        const uint32_t local = i - inst.prim_offset;
        const uint32_t i0 = inst.indices[3 * local], i1 = inst.indices[3 * local + 1], i2 = inst.indices[3 * local + 2];
        const float *P = inst.positions;
        // world-space vertices: the CPU oracle applies the same row-major 3x4 product
        // (object_space: a BLAS keeps the input vertices untouched)
        vec3 w0 = v3(P[3 * i0], P[3 * i0 + 1], P[3 * i0 + 2]);
        vec3 w1 = v3(P[3 * i1], P[3 * i1 + 1], P[3 * i1 + 2]);
        vec3 w2 = v3(P[3 * i2], P[3 * i2 + 1], P[3 * i2 + 2]);
        if (!in.object_space) {
            w0 = xform_point(inst.to_world, w0);
            w1 = xform_point(inst.to_world, w1);
            w2 = xform_point(inst.to_world, w2);
        }
        b.lo[0] = fminf(fminf(w0.x, w1.x), w2.x);
        b.lo[1] = fminf(fminf(w0.y, w1.y), w2.y);
        b.lo[2] = fminf(fminf(w0.z, w1.z), w2.z);
        b.hi[0] = fmaxf(fmaxf(w0.x, w1.x), w2.x);
        b.hi[1] = fmaxf(fmaxf(w0.y, w1.y), w2.y);
        b.hi[2] = fmaxf(fmaxf(w0.z, w1.z), w2.z);
        recs[3 * i + 0] = make_float4(w0.x, w0.y, w0.z, __uint_as_float(i));
        recs[3 * i + 1] = make_float4(w1.x, w1.y, w1.z, __uint_as_float(inst_id));
        recs[3 * i + 2] = make_float4(w2.x, w2.y, w2.z, __uint_as_float(bin));
    }
    boxes[i] = b;
}

// centroid bounds -> 6 ordered uints (lo xyz as min, hi xyz as max)
__global__ void k_bounds(const Aabb *boxes, uint32_t n, uint32_t *out) {
    float lo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
    float hi[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const Aabb b = boxes[i];
        for (int k = 0; k < 3; k++) {
            const float c = 0.5f * (b.lo[k] + b.hi[k]);
            lo[k] = fminf(lo[k], c);
            hi[k] = fmaxf(hi[k], c);
        }
    }
    for (int k = 0; k < 3; k++) {
        for (int o = 32; o > 0; o >>= 1) {
            lo[k] = fminf(lo[k], __shfl_xor(lo[k], o));
            hi[k] = fmaxf(hi[k], __shfl_xor(hi[k], o));
        }
    }
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < 3; k++) {
            atomicMin(&out[k], float_to_ordered(lo[k]));
            atomicMax(&out[3 + k], float_to_ordered(hi[k]));
        }
    }
}

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__global__ void k_morton(const Aabb *boxes, uint32_t n, const uint32_t *bounds, uint32_t *keys, uint32_t *vals) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float lo[3], ext[3];
    for (int k = 0; k < 3; k++) {
        lo[k] = ordered_to_float(bounds[k]);
        const float h = ordered_to_float(bounds[3 + k]);
        ext[k] = h - lo[k];
    }
    const Aabb b = boxes[i];
    uint32_t q[3];
    for (int k = 0; k < 3; k++) {
        const float c = 0.5f * (b.lo[k] + b.hi[k]);
        float t = ext[k] > 0.f ? (c - lo[k]) / ext[k] : 0.5f;
        t = fminf(fmaxf(t * 1024.f, 0.f), 1023.f);
        q[k] = (uint32_t)t;
    }
    keys[i] = (expand_bits(q[0]) << 2) | (expand_bits(q[1]) << 1) | expand_bits(q[2]);
    vals[i] = i;
}

// ---------------------------------------------------------------- radix sort
constexpr int kSortItems = 16;
constexpr int kSortTile = kBlock * kSortItems;

__global__ __launch_bounds__(kBlock) void k_sort_hist(const uint32_t *keys, uint32_t n, int shift, uint32_t *hist,
                                                      uint32_t nblocks) {
    __shared__ uint32_t h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t base = blockIdx.x * kSortTile;
    for (int j = 0; j < kSortItems; j++) {
        const uint32_t i = base + j * kBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    hist[threadIdx.x * nblocks + blockIdx.x] = h[threadIdx.x];  // digit-major
}

// single-block exclusive scan of `count` entries (in place)
__global__ __launch_bounds__(1024) void k_sort_scan(uint32_t *data, uint32_t count) {
    __shared__ uint32_t partial[1024];
    const uint32_t per = (count + 1023) / 1024;
    const uint32_t begin = threadIdx.x * per;
    const uint32_t end = min(begin + per, count);
    uint32_t sum = 0;
    for (uint32_t i = begin; i < end; i++) sum += data[i];
    partial[threadIdx.x] = sum;
    __syncthreads();
    // Hillis-Steele inclusive scan over 1024 partial sums
    for (uint32_t off = 1; off < 1024; off <<= 1) {
        const uint32_t v = threadIdx.x >= off ? partial[threadIdx.x - off] : 0u;
        __syncthreads();
        partial[threadIdx.x] += v;
        __syncthreads();
    }
    uint32_t run = threadIdx.x > 0 ? partial[threadIdx.x - 1] : 0u;
    for (uint32_t i = begin; i < end; i++) {
        const uint32_t v = data[i];
        data[i] = run;
        run += v;
    }
}

__global__ __launch_bounds__(kBlock) void k_sort_scatter(const uint32_t *keys_in, const uint32_t *vals_in,
                                                         uint32_t *keys_out, uint32_t *vals_out, uint32_t n, int shift,
                                                         const uint32_t *offsets, uint32_t nblocks) {
    constexpr int kWaves = kBlock / 64;
    __shared__ uint32_t wave_count[kWaves][256];
    __shared__ uint32_t wave_off[kWaves][256];
    __shared__ uint32_t running[256];
    running[threadIdx.x] = offsets[threadIdx.x * nblocks + blockIdx.x];
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long lt = (1ull << lane) - 1ull;
    const uint32_t base = blockIdx.x * kSortTile;
    for (int j = 0; j < kSortItems; j++) {
        for (int w = 0; w < kWaves; w++) wave_count[w][threadIdx.x] = 0;
        __syncthreads();
        const uint32_t i = base + j * kBlock + threadIdx.x;
        const bool valid = i < n;
        uint32_t key = 0, val = 0, digit = 0;
        if (valid) {
            key = keys_in[i];
            val = vals_in[i];
            digit = (key >> shift) & 0xFFu;
        }
        unsigned long long peers = __ballot(valid);
        for (int b = 0; b < 8; b++) {
            const bool bit = (digit >> b) & 1u;
            const unsigned long long bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) wave_count[wave][digit] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            const uint32_t d = threadIdx.x;
            uint32_t r = running[d];
            for (int w = 0; w < kWaves; w++) {
                wave_off[w][d] = r;
                r += wave_count[w][d];
            }
            running[d] = r;
        }
        __syncthreads();
        if (valid) {
            const uint32_t pos = wave_off[wave][digit] + rank;
            keys_out[pos] = key;
            vals_out[pos] = val;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- Karras 2012
__device__ __forceinline__ int delta(const uint32_t *keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint32_t a = keys[i], b = keys[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

__global__ void k_karras(const uint32_t *keys, int n, int2 *children, int2 *ranges, int *parent_internal,
                         int *parent_leaf) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    int t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    const int gamma = i + s * d + min(d, 0);
    const int first = min(i, j), last = max(i, j);
    // child encoding here: >= 0 internal, < 0 -> leaf ~prim
    const int left = (first == gamma) ? ~gamma : gamma;
    const int right = (last == gamma + 1) ? ~(gamma + 1) : gamma + 1;
    children[i] = make_int2(left, right);
    ranges[i] = make_int2(first, last);
    if (left >= 0) parent_internal[left] = i;
    else parent_leaf[gamma] = i;
    if (right >= 0) parent_internal[right] = i;
    else parent_leaf[gamma + 1] = i;
}

__device__ __forceinline__ Aabb merge(const Aabb &a, const Aabb &b) {
    Aabb r;
    for (int k = 0; k < 3; k++) {
        r.lo[k] = fminf(a.lo[k], b.lo[k]);
        r.hi[k] = fmaxf(a.hi[k], b.hi[k]);
    }
    return r;
}

// Bottom-up refit.  The second thread to arrive at a node merges both
// children.  Bounds are published with an agent-scope release before the
// arrival atomic and read after an agent-scope acquire (L1s are per CU and the
// per-XCD L2s are not coherent, MI355X_MICROARCH.md "inter-workgroup visibility").
__global__ void k_refit(int n, const uint32_t *sorted_vals, const Aabb *prim_boxes, const int2 *children,
                        const int *parent_internal, const int *parent_leaf, Aabb *node_boxes, uint32_t *flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int node = parent_leaf[i];
    while (node >= 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t prev = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0u) return;  // first arrival: the sibling finishes the node
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const int2 c = children[node];
        const Aabb a = c.x >= 0 ? node_boxes[c.x] : prim_boxes[sorted_vals[~c.x]];
        const Aabb b = c.y >= 0 ? node_boxes[c.y] : prim_boxes[sorted_vals[~c.y]];
        node_boxes[node] = merge(a, b);
        node = node == 0 ? -1 : parent_internal[node];
    }
}

__device__ __forceinline__ int child_link(int c, const int2 *ranges, uint32_t leaf_size) {
    if (c < 0) return make_leaf((uint32_t)~c, 1u);
    const int2 r = ranges[c];
    const uint32_t cnt = (uint32_t)(r.y - r.x + 1);
    if (cnt <= leaf_size) return make_leaf((uint32_t)r.x, cnt);
    return c;
}

// ---------------------------------------------------------------- PLOC
// Parallel locally-ordered clustering (Meister & Bittner 2018) over the
// Morton-ordered primitives: each cluster finds its nearest neighbour (smallest
// union surface area, ties to the smaller index) within +-kPlocRadius (32: 2.5 % faster frames than 16 on config 4, 64 no better; profiles/r02_ploc_radius_ab.txt)
// positions, mutual pairs merge, the cluster list is compacted in order, and
// this repeats until one cluster is left.  It yields a tree of markedly lower
// SAH cost than the Karras hierarchy over the same order.  The result is
// converted to the LBVH arrays (children / ranges / parents / node boxes, root
// 0, subtrees contiguous in a new primitive order) so emit and the BVH4
// collapse are shared.  Refs: >= 0 internal node (creation id), < 0 leaf ~pos.
constexpr int kPlocRadius = 32;
constexpr int kScanBlock = 1024;
constexpr int kScanItems = 4;

__device__ __forceinline__ float half_area(const Aabb &b) {
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    return dx * dy + dy * dz + dz * dx;
}

__global__ void k_ploc_init(int n, const uint32_t *sorted_vals, const Aabb *prim_boxes, int *ref, Aabb *box) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ref[i] = ~i;
    box[i] = prim_boxes[sorted_vals[i]];
}

__global__ __launch_bounds__(kBlock) void k_ploc_nn(int m, const Aabb *box, int *nn) {
    __shared__ Aabb tile[kBlock + 2 * kPlocRadius];
    const int base = blockIdx.x * kBlock - kPlocRadius;
    for (int t = threadIdx.x; t < kBlock + 2 * kPlocRadius; t += kBlock) {
        const int j = base + t;
        if (j >= 0 && j < m) tile[t] = box[j];
    }
    __syncthreads();
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    const Aabb bi = tile[threadIdx.x + kPlocRadius];
    float best = __builtin_huge_valf();
    int bj = -1;
    const int j0 = max(0, i - kPlocRadius), j1 = min(m - 1, i + kPlocRadius);
    for (int j = j0; j <= j1; j++) {
        if (j == i) continue;
        const float a = half_area(merge(bi, tile[j - base]));
        if (a < best) {  // ascending j: ties keep the smaller index
            best = a;
            bj = j;
        }
    }
    nn[i] = bj;
}

// per cluster: low word = survives (1), high word = creates a node (1)
__global__ void k_ploc_flags(int m, const int *nn, unsigned long long *flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const int j = nn[i];
    const bool mutual = nn[j] == i;
    const unsigned long long keep = (mutual && i > j) ? 0ull : 1ull;
    const unsigned long long make = (mutual && i < j) ? 1ull : 0ull;
    flags[i] = keep | (make << 32);
}

// exclusive scan of 64-bit counts: block pass, block-sum pass, add pass
__global__ __launch_bounds__(kScanBlock) void k_scan64_blocks(unsigned long long *data, int n,
                                                            unsigned long long *sums) {
    __shared__ unsigned long long wsum[kScanBlock / 64];
    const int base = blockIdx.x * kScanBlock * kScanItems + threadIdx.x * kScanItems;
    unsigned long long v[kScanItems], tsum = 0;
    for (int k = 0; k < kScanItems; k++) {
        v[k] = base + k < n ? data[base + k] : 0ull;
        tsum += v[k];
    }
    unsigned long long inc = tsum;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long u = __shfl_up(inc, o);
        if ((int)__lane_id() >= o) inc += u;
    }
    if (__lane_id() == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const unsigned long long w = threadIdx.x < kScanBlock / 64 ? wsum[threadIdx.x] : 0ull;
        unsigned long long winc = w;
        for (int o = 1; o < kScanBlock / 64; o <<= 1) {
            const unsigned long long u = __shfl_up(winc, o);
            if ((int)threadIdx.x >= o) winc += u;
        }
        if (threadIdx.x < kScanBlock / 64) wsum[threadIdx.x] = winc - w;
        if (threadIdx.x == kScanBlock / 64 - 1) sums[blockIdx.x] = winc;
    }
    __syncthreads();
    unsigned long long run = wsum[threadIdx.x >> 6] + inc - tsum;
    for (int k = 0; k < kScanItems; k++) {
        if (base + k < n) data[base + k] = run;
        run += v[k];
    }
}

__global__ __launch_bounds__(kScanBlock) void k_scan64_sums(unsigned long long *sums, int nb,
                                                          unsigned long long *total) {
    // nb <= kScanBlock * kScanItems: reuse the block pass on a single block
    __shared__ unsigned long long wsum[kScanBlock / 64];
    const int base = threadIdx.x * kScanItems;
    unsigned long long v[kScanItems], tsum = 0;
    for (int k = 0; k < kScanItems; k++) {
        v[k] = base + k < nb ? sums[base + k] : 0ull;
        tsum += v[k];
    }
    unsigned long long inc = tsum;
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long u = __shfl_up(inc, o);
        if ((int)__lane_id() >= o) inc += u;
    }
    if (__lane_id() == 63) wsum[threadIdx.x >> 6] = inc;
    __syncthreads();
    if (threadIdx.x < 64) {
        const unsigned long long w = threadIdx.x < kScanBlock / 64 ? wsum[threadIdx.x] : 0ull;
        unsigned long long winc = w;
        for (int o = 1; o < kScanBlock / 64; o <<= 1) {
            const unsigned long long u = __shfl_up(winc, o);
            if ((int)threadIdx.x >= o) winc += u;
        }
        if (threadIdx.x < kScanBlock / 64) wsum[threadIdx.x] = winc - w;
        if (threadIdx.x == kScanBlock / 64 - 1) *total = winc;
    }
    __syncthreads();
    unsigned long long run = wsum[threadIdx.x >> 6] + inc - tsum;
    for (int k = 0; k < kScanItems; k++) {
        if (base + k < nb) sums[base + k] = run;
        run += v[k];
    }
}

__global__ void k_scan64_add(unsigned long long *data, int n, const unsigned long long *sums) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    data[i] += sums[i / (kScanBlock * kScanItems)];
}

__global__ void k_ploc_compact(int m, const int *ref, const Aabb *box, const int *nn,
                               const unsigned long long *flags, const unsigned long long *pos, int base_id,
                               int *ref_out, Aabb *box_out, int2 *node_child, Aabb *node_box, int *node_count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const unsigned long long f = flags[i];
    if (!(f & 1ull)) return;
    const unsigned long long p = pos[i];
    const int out = (int)(p & 0xFFFFFFFFull);
    if (f >> 32) {
        const int j = nn[i];
        const int id = base_id + (int)(p >> 32);
        const Aabb b = merge(box[i], box[j]);
        const int a = ref[i], c = ref[j];
        node_child[id] = make_int2(a, c);
        node_box[id] = b;
        node_count[id] = (a >= 0 ? node_count[a] : 1) + (c >= 0 ? node_count[c] : 1);
        ref_out[out] = id;
        box_out[out] = b;
    } else {
        ref_out[out] = ref[i];
        box_out[out] = box[i];
    }
}

// top-down: subtree [first, first + count) of the new primitive order
__global__ void k_ploc_place(int lo, int hi, const int2 *node_child, const int *node_count, int *first,
                             int *newpos) {
    const int id = lo + blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= hi) return;
    const int f = first[id];
    const int2 c = node_child[id];
    const int cl = c.x >= 0 ? node_count[c.x] : 1;
    if (c.x >= 0) first[c.x] = f;
    else newpos[~c.x] = f;
    if (c.y >= 0) first[c.y] = f + cl;
    else newpos[~c.y] = f + cl;
}

// creation id -> LBVH arrays (root 0), new primitive order
__global__ void k_ploc_export(int n, const int2 *node_child, const Aabb *node_box, const int *node_count,
                              const int *first, const int *newpos, int2 *children, int2 *ranges, Aabb *node_boxes,
                              int *parent_internal, int *parent_leaf) {
    const int id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= n - 1) return;
    const int fid = (n - 2) - id;
    const int2 c = node_child[id];
    const int a = c.x >= 0 ? (n - 2) - c.x : ~newpos[~c.x];
    const int b = c.y >= 0 ? (n - 2) - c.y : ~newpos[~c.y];
    children[fid] = make_int2(a, b);
    ranges[fid] = make_int2(first[id], first[id] + node_count[id] - 1);
    node_boxes[fid] = node_box[id];
    if (a >= 0) parent_internal[a] = fid;
    else parent_leaf[~a] = fid;
    if (b >= 0) parent_internal[b] = fid;
    else parent_leaf[~b] = fid;
}

__global__ void k_ploc_permute(int n, const int *newpos, const uint32_t *vals_in, uint32_t *vals_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    vals_out[newpos[i]] = vals_in[i];
}

// ---------------------------------------------------------------- BVH4 collapse
// Binary nodes at even depth become 4-wide nodes whose children are their
// grandchildren (or the child itself where the child is a leaf).
__global__ void k_depth(int n, const int *parent_internal, uint32_t *depth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    uint32_t d = 0;
    for (int p = i; p != 0; p = parent_internal[p]) d++;
    depth[i] = d;
}

__global__ void k_flag4(int n, const int2 *ranges, const uint32_t *depth, uint32_t leaf_size, uint32_t *flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    const int2 r = ranges[i];
    flags[i] = ((depth[i] & 1u) == 0u && (uint32_t)(r.y - r.x + 1) > leaf_size) ? 1u : 0u;
}

__global__ void k_emit4(int n, const uint32_t *sorted_vals, const Aabb *prim_boxes, const int2 *children,
                        const int2 *ranges, const Aabb *node_boxes, const uint32_t *flags, const uint32_t *idx4,
                        uint32_t leaf_size, Bvh4Node *nodes4) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1 || !flags[i]) return;
    int link[4];
    Aabb box[4];
    int nk = 0;
    auto add = [&](int c) {
        if (c < 0) {
            link[nk] = make_leaf((uint32_t)~c, 1u);
            box[nk] = prim_boxes[sorted_vals[~c]];
        } else {
            const int2 r = ranges[c];
            const uint32_t cnt = (uint32_t)(r.y - r.x + 1);
            link[nk] = cnt <= leaf_size ? make_leaf((uint32_t)r.x, cnt) : (int)idx4[c];
            box[nk] = node_boxes[c];
        }
        nk++;
    };
    const int2 c = children[i];
    for (int s = 0; s < 2; s++) {
        const int ch = s == 0 ? c.x : c.y;
        bool expand = false;
        if (ch >= 0) {
            const int2 r = ranges[ch];
            expand = (uint32_t)(r.y - r.x + 1) > leaf_size;  // odd-depth internal node: absorb it
        }
        if (expand) {
            const int2 g = children[ch];
            add(g.x);
            add(g.y);
        } else {
            add(ch);
        }
    }
    const Aabb nb = node_boxes[i];
    float clo[3][4], chi[3][4];
    for (int k = 0; k < 4; k++)
        for (int a = 0; a < 3; a++) {
            clo[a][k] = k < nk ? box[k].lo[a] : 0.f;
            chi[a][k] = k < nk ? box[k].hi[a] : 0.f;
        }
    Bvh4Node o;
    uint32_t ex, ey, ez;
    quantize_axis(nb.lo[0], nb.hi[0], clo[0], chi[0], nk, o.ox, ex, o.qlo_x, o.qhi_x);
    quantize_axis(nb.lo[1], nb.hi[1], clo[1], chi[1], nk, o.oy, ey, o.qlo_y, o.qhi_y);
    quantize_axis(nb.lo[2], nb.hi[2], clo[2], chi[2], nk, o.oz, ez, o.qlo_z, o.qhi_z);
    set_scales(o, ex, ey, ez);
    for (int k = 0; k < 4; k++) o.child[k] = k < nk ? link[k] : kEmptyLink;
    nodes4[idx4[i]] = o;
}

// ---------------------------------------------------------------- greedy BVH4 collapse
// Top-down, one level of 4-wide nodes per pass: a 4-wide node starts from its
// binary node's two children and repeatedly opens the child with the largest
// surface area (an internal binary node that is not a leaf-sized subtree) until
// it has four children (the wide-BVH collapse of Wald et al. 2008 / Ylitie et
// al. 2017).  Children that remain internal become the next level's 4-wide
// nodes, numbered breadth-first after a scan of their counts.
constexpr uint32_t kSahLeaf = 1u << 12;  // k_sah_dp decision: the subtree is one leaf
__device__ __forceinline__ bool opens(int c, const int2 *ranges, uint32_t leaf_size, const uint32_t *dec = nullptr) {
    if (c < 0) return false;
    if (dec) return (dec[c] & kSahLeaf) == 0u;
    const int2 r = ranges[c];
    return (uint32_t)(r.y - r.x + 1) > leaf_size;
}

__global__ void k_collapse_pick(int items, const int *item_node, const int2 *children, const int2 *ranges,
                                const Aabb *node_boxes, uint32_t leaf_size, int4 *clist,
                                unsigned long long *inner_count) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= items) return;
    const int b = item_node[t];
    int c[4];
    const int2 ch = children[b];
    c[0] = ch.x;
    c[1] = ch.y;
    int nk = 2;
    while (nk < 4) {
        int best = -1;
        float best_a = -1.f;
        for (int k = 0; k < nk; k++)
            if (opens(c[k], ranges, leaf_size)) {
                const float a = half_area(node_boxes[c[k]]);
                if (a > best_a) {
                    best_a = a;
                    best = k;
                }
            }
        if (best < 0) break;
        const int2 g = children[c[best]];
        c[best] = g.x;
        c[nk++] = g.y;
    }
    unsigned long long inner = 0;
    for (int k = 0; k < nk; k++) inner += opens(c[k], ranges, leaf_size) ? 1ull : 0ull;
    for (int k = nk; k < 4; k++) c[k] = kEmptyLink;
    clist[t] = make_int4(c[0], c[1], c[2], c[3]);
    inner_count[t] = inner;
}

__global__ void k_collapse_emit(int items, int base, int next_base, const int *item_node, const int4 *clist,
                                const unsigned long long *inner_pos, const uint32_t *sorted_vals,
                                const Aabb *prim_boxes, const int2 *ranges, const Aabb *node_boxes,
                                uint32_t leaf_size, int *next_items, Bvh4Node *nodes4, const uint32_t *dec) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= items) return;
    const int4 cl = clist[t];
    const int cc[4] = {cl.x, cl.y, cl.z, cl.w};
    int link[4];
    float clo[3][4], chi[3][4];
    int nk = 0;
    int pos = (int)inner_pos[t];
    for (int k = 0; k < 4; k++) {
        const int c = cc[k];
        if (c == kEmptyLink) break;
        Aabb b;
        if (c < 0) {
            link[nk] = make_leaf((uint32_t)~c, 1u);
            b = prim_boxes[sorted_vals[~c]];
        } else if (!opens(c, ranges, leaf_size, dec)) {
            const int2 r = ranges[c];
            link[nk] = make_leaf((uint32_t)r.x, (uint32_t)(r.y - r.x + 1));
            b = node_boxes[c];
        } else {
            next_items[pos] = c;
            link[nk] = next_base + pos;
            pos++;
            b = node_boxes[c];
        }
        for (int a = 0; a < 3; a++) {
            clo[a][nk] = b.lo[a];
            chi[a][nk] = b.hi[a];
        }
        nk++;
    }
    for (int k = nk; k < 4; k++)
        for (int a = 0; a < 3; a++) clo[a][k] = chi[a][k] = 0.f;
    const Aabb nb = node_boxes[item_node[t]];
    Bvh4Node o;
    uint32_t ex, ey, ez;
    quantize_axis(nb.lo[0], nb.hi[0], clo[0], chi[0], nk, o.ox, ex, o.qlo_x, o.qhi_x);
    quantize_axis(nb.lo[1], nb.hi[1], clo[1], chi[1], nk, o.oy, ey, o.qlo_y, o.qhi_y);
    quantize_axis(nb.lo[2], nb.hi[2], clo[2], chi[2], nk, o.oz, ez, o.qlo_z, o.qhi_z);
    set_scales(o, ex, ey, ez);
    for (int k = 0; k < 4; k++) o.child[k] = k < nk ? link[k] : kEmptyLink;
    nodes4[base + t] = o;
}

// ---------------------------------------------------------------- SAH-optimal BVH4 collapse
// (the default; PUPIL_BVH4_COLLAPSE=greedy keeps the greedy opening) The slot distribution of Ylitie, Karras & Laine 2017,
// section 4, for 4-wide nodes: bottom up over the binary tree, C(n, i) is the least
// cost of the subtree n when it may fill i slots of its parent, with
//   D(n, j)  = min over 0 < k < j of C(left, k) + C(right, j - k)
//   C(n, 1)  = A(n) + D(n, 4)            (n becomes a 4-wide node)
//   C(n, i)  = min(C(n, i - 1), D(n, i)) (n opened into up to i slots)
// Subtrees of at most leaf_size primitives are leaves, as in the greedy collapse, so
// their cost is the same in every distribution and only the surface area of the
// 4-wide nodes is minimised.  dec[n]: bits 0-1 / 2-3 / 4-5 the best k of D(n, 2/3/4),
// bits 8-10 "C(n, i) = C(n, i - 1)" for i = 2, 3, 4.
__global__ void k_sah_parents(int n, const int2 *children, int *parent, int *leaf_parent) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n - 1) return;
    const int2 c = children[b];
    if (c.x >= 0) parent[c.x] = b;
    else leaf_parent[~c.x] = b;
    if (c.y >= 0) parent[c.y] = b;
    else leaf_parent[~c.y] = b;
}

__device__ __forceinline__ float4 sah_cost(int c, const float4 *cost, const uint32_t *sorted_vals,
                                           const Aabb *prim_boxes) {
    if (c < 0) {  // one primitive: a leaf in every distribution
        const float a = half_area(prim_boxes[sorted_vals[~c]]);
        return make_float4(a, a, a, a);
    }
    const uint32_t *w = (const uint32_t *)(cost + c);  // written by another thread: device-coherent loads
    float4 v;
    v.x = __uint_as_float(__hip_atomic_load(w + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v.y = __uint_as_float(__hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v.z = __uint_as_float(__hip_atomic_load(w + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    v.w = __uint_as_float(__hip_atomic_load(w + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return v;
}

// one thread per primitive walks up; the second child to finish computes its parent
__global__ void k_sah_dp(int n, const int *parent, const int *leaf_parent, const int2 *children, const int2 *ranges,
                         const Aabb *node_boxes, const uint32_t *sorted_vals, const Aabb *prim_boxes,
                         uint32_t leaf_size, uint32_t sah_leaf, uint32_t *flags, float4 *cost, uint32_t *dec) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int b = leaf_parent[i];
    while (b >= 0) {
        __threadfence();
        if (atomicAdd(flags + b, 1u) == 0u) return;
        __threadfence();
        const int2 ch = children[b];
        const float4 l4 = sah_cost(ch.x, cost, sorted_vals, prim_boxes);
        const float4 r4 = sah_cost(ch.y, cost, sorted_vals, prim_boxes);
        const float cl[4] = {l4.x, l4.y, l4.z, l4.w}, cr[4] = {r4.x, r4.y, r4.z, r4.w};
        float d[5];
        uint32_t code = 0;
        for (int j = 2; j <= 4; j++) {
            float best = __builtin_huge_valf();
            uint32_t bk = 1;
            for (int k = 1; k < j; k++) {
                const float v = cl[k - 1] + cr[j - k - 1];
                if (v < best) {
                    best = v;
                    bk = (uint32_t)k;
                }
            }
            d[j] = best;
            code |= bk << (2 * (j - 2));
        }
        const int2 r = ranges[b];
        const float a = half_area(node_boxes[b]);
        float c4[4];
        const uint32_t cnt = (uint32_t)(r.y - r.x + 1);
        if (cnt <= leaf_size || (cnt <= sah_leaf && a * (float)cnt <= a + d[4])) {  // one leaf wherever it goes
            c4[0] = c4[1] = c4[2] = c4[3] = a * (float)cnt;
            code |= 7u << 8 | kSahLeaf;
        } else {
            c4[0] = a + d[4];
            for (int s = 2; s <= 4; s++) {
                if (c4[s - 2] <= d[s]) {
                    c4[s - 1] = c4[s - 2];
                    code |= 1u << (8 + s - 2);
                } else {
                    c4[s - 1] = d[s];
                }
            }
        }
        cost[b] = make_float4(c4[0], c4[1], c4[2], c4[3]);
        dec[b] = code;
        b = parent[b];
    }
}

// children of the 4-wide node made from binary node b: D(b, 4) distributed down the
// decisions, a subtree taking one slot (a leaf or the next level's 4-wide node) or
// being opened into the slots it was given
__global__ void k_collapse_pick_sah(int items, const int *item_node, const int2 *children, const int2 *ranges,
                                    const uint32_t *dec, uint32_t leaf_size, int4 *clist,
                                    unsigned long long *inner_count) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= items) return;
    const int b = item_node[t];
    const int2 ch = children[b];
    const uint32_t k4 = (dec[b] >> 4) & 3u;
    int wc[4], wi[4], nw = 0;  // work: (subtree, slots); slots add up to at most 4
    wc[nw] = ch.x, wi[nw++] = (int)k4;
    wc[nw] = ch.y, wi[nw++] = 4 - (int)k4;
    int c[4], nk = 0;
    while (nw > 0) {
        const int x = wc[--nw];
        int s = wi[nw];
        if (!opens(x, ranges, leaf_size, dec) || s <= 1) {
            c[nk++] = x;
            continue;
        }
        const uint32_t dx = dec[x];
        while (s > 1 && ((dx >> (8 + s - 2)) & 1u)) s--;  // C(x, s) = C(x, s - 1)
        if (s == 1) {
            c[nk++] = x;
            continue;
        }
        const int k = (int)((dx >> (2 * (s - 2))) & 3u);
        const int2 g = children[x];
        wc[nw] = g.x, wi[nw++] = k;
        wc[nw] = g.y, wi[nw++] = s - k;
    }
    unsigned long long inner = 0;
    for (int k = 0; k < nk; k++) inner += opens(c[k], ranges, leaf_size, dec) ? 1ull : 0ull;
    for (int k = nk; k < 4; k++) c[k] = kEmptyLink;
    clist[t] = make_int4(c[0], c[1], c[2], c[3]);
    inner_count[t] = inner;
}

// Shading record of each primitive in traversal (Morton) order, kAttrStride
// float4 per primitive: everything the hit reconstruction of
// Geometry::GetHitLocalGeometry (render/geometry.h:48-96) gathers from the
// object-space mesh, in one 128-B line instead of index + 3 x position / normal /
// uv gathers:  [0] p0 | global id (+ sphere bit)  [1] p1 | instance  [2] p2 | n0.x
// [3] n0.yz n1.xy  [4] n1.z n2.xyz  [5] t0 t1  [6] t2 | 0 0  [7] unused
__global__ void k_attrs(int n, const uint32_t *sorted_vals, const uint32_t *slot, BvhBuildInput in, float4 *attrs) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t prim = sorted_vals[i];
    const uint32_t inst_id = in.prim_inst[prim];
    const DevInstance &inst = in.instances[inst_id];
    // object_space (BLAS): records in the mesh's own primitive order, found by primitive id;
    // flattened: by record slot (the hit index)
    float4 *r = attrs + (size_t)kAttrStride * (in.object_space ? prim : slot[i]);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (inst.kind == PUPIL_SHAPE_SPHERE) {
        r[0] = make_float4(0.f, 0.f, 0.f, __uint_as_float(prim | kPrimSphereBit));
        r[1] = make_float4(0.f, 0.f, 0.f, __uint_as_float(inst_id));
        r[2] = r[3] = r[4] = r[5] = r[6] = r[7] = z;
        return;
    }
    const uint32_t local = prim - inst.prim_offset;
    const uint32_t i0 = inst.indices[3 * local], i1 = inst.indices[3 * local + 1], i2 = inst.indices[3 * local + 2];
    const float *P = inst.positions;
    r[0] = make_float4(P[3 * i0], P[3 * i0 + 1], P[3 * i0 + 2], __uint_as_float(prim));
    r[1] = make_float4(P[3 * i1], P[3 * i1 + 1], P[3 * i1 + 2], __uint_as_float(inst_id));
    float nn[9] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (inst.normals) {
        const float *N = inst.normals;
        const uint32_t id[3] = {i0, i1, i2};
        for (int v = 0; v < 3; v++)
            for (int c = 0; c < 3; c++) nn[3 * v + c] = N[3 * id[v] + c];
    }
    r[2] = make_float4(P[3 * i2], P[3 * i2 + 1], P[3 * i2 + 2], nn[0]);
    r[3] = make_float4(nn[1], nn[2], nn[3], nn[4]);
    r[4] = make_float4(nn[5], nn[6], nn[7], nn[8]);
    if (inst.texcoords) {
        const float *T = inst.texcoords;
        r[5] = make_float4(T[2 * i0], T[2 * i0 + 1], T[2 * i1], T[2 * i1 + 1]);
        r[6] = make_float4(T[2 * i2], T[2 * i2 + 1], 0.f, 0.f);
    } else {
        r[5] = r[6] = z;
    }
    r[7] = z;
}

__global__ void k_reorder(int n, const uint32_t *sorted_vals, const uint32_t *slot, const float4 *recs_in,
                          float4 *recs_out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t src = sorted_vals[i];
    float4 *o = recs_out + (size_t)kRecF4 * slot[i];
    o[0] = recs_in[3 * src + 0];
    o[1] = recs_in[3 * src + 1];
    o[2] = recs_in[3 * src + 2];
}

// Record slots (kRecF4): every leaf's slot count 2 ceil(c / 2) at its first primitive,
// scanned, gives each leaf a first slot on a 128-B line
__global__ void k_leaf_marks(const Bvh4Node *nodes, uint32_t m, unsigned long long *lsz) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    const Bvh4Node nd = nodes[j];
    for (int k = 0; k < 4; k++) {
        const int l = nd.child[k];
        if (l != kEmptyLink && l < 0) lsz[leaf_first(l)] = leaf_slots(leaf_count(l));
    }
}
// each leaf's primitives -> their slots; its link now names its first slot
__global__ void k_leaf_slots(Bvh4Node *nodes, uint32_t m, const unsigned long long *first_slot, uint32_t *slot) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= m) return;
    Bvh4Node nd = nodes[j];
    for (int k = 0; k < 4; k++) {
        const int l = nd.child[k];
        if (l == kEmptyLink || l >= 0) continue;
        const uint32_t f = leaf_first(l), c = leaf_count(l), fs = (uint32_t)first_slot[f];
        for (uint32_t q = 0; q < c; q++) slot[f + q] = fs + q;
        nd.child[k] = make_leaf(fs, c);
    }
    nodes[j] = nd;
}

template <typename T>
hipError_t dmalloc(T **p, size_t count) {
    return hipMalloc((void **)p, sizeof(T) * (count > 0 ? count : 1));
}

// Greedy breadth-first BVH4 collapse (k_collapse_pick / k_collapse_emit);
// nodes4 must hold n - 1 entries; returns the number of 4-wide nodes.
hipError_t collapse_bvh4(int n, const uint32_t *sorted_vals, const Aabb *prim_boxes, const int2 *children,
                         const int2 *ranges, const Aabb *node_boxes, uint32_t leaf_size, Bvh4Node *nodes4,
                         uint32_t *num_nodes4, uint32_t *depth4, std::vector<uint32_t> *level_start, hipStream_t s,
                         bool sah) {
    int *items_a = nullptr, *items_b = nullptr;
    // SAH-optimal slot distribution (k_sah_dp) instead of the greedy opening
    int *parent = nullptr, *leaf_parent = nullptr;
    uint32_t *sflags = nullptr, *dec = nullptr;
    float4 *cost = nullptr;
    sah = sah && n >= 2;
    int4 *clist = nullptr;
    unsigned long long *cnt = nullptr, *sums = nullptr, *total = nullptr;
    const int per = kScanBlock * kScanItems;
    const int cap = n;  // a level never has more 4-wide nodes than binary internal nodes
    hipError_t err = dmalloc(&items_a, cap);
    if (!err) err = dmalloc(&items_b, cap);
    if (!err) err = dmalloc(&clist, cap);
    if (!err) err = dmalloc(&cnt, cap);
    if (!err) err = dmalloc(&sums, (cap + per - 1) / per);
    if (!err) err = dmalloc(&total, 1);
    const auto grid = [](int m) { return dim3((unsigned)((m + kBlock - 1) / kBlock)); };
    if (!err && sah) {
        err = dmalloc(&parent, n);
        if (!err) err = dmalloc(&leaf_parent, n);
        if (!err) err = dmalloc(&sflags, n);
        if (!err) err = dmalloc(&cost, n);
        if (!err) err = dmalloc(&dec, n);
        if (!err) err = hipMemsetAsync(parent, 0xFF, sizeof(int) * n, s);  // root: -1
        if (!err) err = hipMemsetAsync(sflags, 0, sizeof(uint32_t) * n, s);
        if (!err) {
            hipLaunchKernelGGL(k_sah_parents, grid(n - 1), dim3(kBlock), 0, s, n, children, parent, leaf_parent);
            uint32_t sah_leaf = leaf_size;  // PUPIL_SAH_LEAF: larger leaves where the SAH prefers them (<= 8)
            if (const char *e = std::getenv("PUPIL_SAH_LEAF"))
                sah_leaf = (uint32_t)std::min(8, std::max((int)leaf_size, std::atoi(e)));
            hipLaunchKernelGGL(k_sah_dp, grid(n), dim3(kBlock), 0, s, n, parent, leaf_parent, children, ranges,
                               node_boxes, sorted_vals, prim_boxes, leaf_size, sah_leaf, sflags, cost, dec);
        }
    }
    int base = 0, items = 1;
    uint32_t levels = 0;  // breadth first: one iteration per BVH4 level
    if (level_start) level_start->clear();
    if (!err) err = hipMemsetAsync(items_a, 0, sizeof(int), s);  // binary root 0
    while (!err && items > 0) {
        if (level_start) level_start->push_back((uint32_t)base);
        if (sah)
            hipLaunchKernelGGL(k_collapse_pick_sah, grid(items), dim3(kBlock), 0, s, items, items_a, children, ranges,
                               dec, leaf_size, clist, cnt);
        else
            hipLaunchKernelGGL(k_collapse_pick, grid(items), dim3(kBlock), 0, s, items, items_a, children, ranges,
                               node_boxes, leaf_size, clist, cnt);
        const int nb = (items + per - 1) / per;
        hipLaunchKernelGGL(k_scan64_blocks, dim3(nb), dim3(kScanBlock), 0, s, cnt, items, sums);
        hipLaunchKernelGGL(k_scan64_sums, dim3(1), dim3(kScanBlock), 0, s, sums, nb, total);
        hipLaunchKernelGGL(k_scan64_add, grid(items), dim3(kBlock), 0, s, cnt, items, sums);
        hipLaunchKernelGGL(k_collapse_emit, grid(items), dim3(kBlock), 0, s, items, base, base + items, items_a, clist,
                           cnt, sorted_vals, prim_boxes, ranges, node_boxes, leaf_size, items_b, nodes4,
                           sah ? dec : nullptr);
        unsigned long long tot = 0;
        (void)hipMemcpyAsync(&tot, total, sizeof(tot), hipMemcpyDeviceToHost, s);
        err = hipStreamSynchronize(s);
        base += items;
        items = (int)tot;
        levels++;
        if (base + items > n - 1) err = hipErrorUnknown;  // cannot happen
        std::swap(items_a, items_b);
    }
    *num_nodes4 = (uint32_t)base;
    *depth4 = levels;
    if (level_start) level_start->push_back((uint32_t)base);
    void *bufs[] = {items_a, items_b, clist, cnt, sums, total, parent, leaf_parent, sflags, cost, dec};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    return err;
}

// PLOC topology (see the PLOC section) -> LBVH arrays and the new primitive order
hipError_t build_ploc(int n, const uint32_t *vals_in, uint32_t *vals_out, const Aabb *prim_boxes, int2 *children,
                      int2 *ranges, Aabb *node_boxes, int *parent_internal, int *parent_leaf, hipStream_t s) {
    int *ref_a = nullptr, *ref_b = nullptr, *nn = nullptr, *node_count = nullptr, *first = nullptr, *newpos = nullptr;
    Aabb *box_a = nullptr, *box_b = nullptr, *node_box = nullptr;
    int2 *node_child = nullptr;
    unsigned long long *flg = nullptr, *pos = nullptr, *sums = nullptr, *total = nullptr;
    const int per = kScanBlock * kScanItems;
    const int nsum = (n + per - 1) / per;
    hipError_t err = dmalloc(&ref_a, n);
    if (!err) err = dmalloc(&ref_b, n);
    if (!err) err = dmalloc(&nn, n);
    if (!err) err = dmalloc(&node_count, n);
    if (!err) err = dmalloc(&first, n);
    if (!err) err = dmalloc(&newpos, n);
    if (!err) err = dmalloc(&box_a, n);
    if (!err) err = dmalloc(&box_b, n);
    if (!err) err = dmalloc(&node_box, n);
    if (!err) err = dmalloc(&node_child, n);
    if (!err) err = dmalloc(&flg, n);
    if (!err) err = dmalloc(&pos, n);
    if (!err) err = dmalloc(&sums, nsum);
    if (!err) err = dmalloc(&total, 1);
    if (!err && nsum > per) err = hipErrorInvalidValue;  // > 16.7 G primitives
    std::vector<int2> iters;
    if (!err) {
        const auto grid = [](int m) { return dim3((unsigned)((m + kBlock - 1) / kBlock)); };
        hipLaunchKernelGGL(k_ploc_init, grid(n), dim3(kBlock), 0, s, n, vals_in, prim_boxes, ref_a, box_a);
        int m = n, base = 0;
        while (m > 1 && !err) {
            hipLaunchKernelGGL(k_ploc_nn, grid(m), dim3(kBlock), 0, s, m, box_a, nn);
            hipLaunchKernelGGL(k_ploc_flags, grid(m), dim3(kBlock), 0, s, m, nn, flg);
            (void)hipMemcpyAsync(pos, flg, sizeof(unsigned long long) * m, hipMemcpyDeviceToDevice, s);
            const int nb = (m + per - 1) / per;
            hipLaunchKernelGGL(k_scan64_blocks, dim3(nb), dim3(kScanBlock), 0, s, pos, m, sums);
            hipLaunchKernelGGL(k_scan64_sums, dim3(1), dim3(kScanBlock), 0, s, sums, nb, total);
            hipLaunchKernelGGL(k_scan64_add, grid(m), dim3(kBlock), 0, s, pos, m, sums);
            unsigned long long tot = 0;
            (void)hipMemcpyAsync(&tot, total, sizeof(tot), hipMemcpyDeviceToHost, s);
            err = hipStreamSynchronize(s);
            const int m_new = (int)(tot & 0xFFFFFFFFull), merges = (int)(tot >> 32);
            if (!err && (merges <= 0 || m_new != m - merges)) err = hipErrorUnknown;  // cannot happen
            if (err) break;
            hipLaunchKernelGGL(k_ploc_compact, grid(m), dim3(kBlock), 0, s, m, ref_a, box_a, nn, flg, pos, base,
                               ref_b, box_b, node_child, node_box, node_count);
            iters.push_back(make_int2(base, merges));
            base += merges;
            std::swap(ref_a, ref_b);
            std::swap(box_a, box_b);
            m = m_new;
        }
        if (!err) {
            (void)hipMemsetAsync(first + (n - 2), 0, sizeof(int), s);  // root = last node created
            for (size_t k = iters.size(); k-- > 0;) {
                const int lo = iters[k].x, hi = iters[k].x + iters[k].y;
                hipLaunchKernelGGL(k_ploc_place, grid(hi - lo), dim3(kBlock), 0, s, lo, hi, node_child, node_count,
                                   first, newpos);
            }
            hipLaunchKernelGGL(k_ploc_export, grid(n - 1), dim3(kBlock), 0, s, n, node_child, node_box, node_count,
                               first, newpos, children, ranges, node_boxes, parent_internal, parent_leaf);
            hipLaunchKernelGGL(k_ploc_permute, grid(n), dim3(kBlock), 0, s, n, newpos, vals_in, vals_out);
            err = hipStreamSynchronize(s);
        }
    }
    void *bufs[] = {ref_a, ref_b, nn, node_count, first, newpos, box_a, box_b, node_box, node_child, flg, pos,
                    sums, total};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    return err;
}

}  // namespace

void free_lbvh(BvhBuildOutput &out) {
    if (out.nodes4) (void)hipFree(out.nodes4);
    if (out.prims) (void)hipFree(out.prims);
    if (out.attrs) (void)hipFree(out.attrs);
    out.nodes4 = nullptr;
    out.prims = nullptr;
    out.attrs = nullptr;
}

int build_lbvh(const BvhBuildInput &in, BvhBuildOutput &out, uint32_t leaf_size, hipStream_t s, double *build_ms,
               bool force_lbvh) {
    const int n = (int)in.num_prims;
    if (n <= 0) {  // empty scene: every ray misses
        out = BvhBuildOutput{};
        out.root_link4 = (uint32_t)kTraverseDone;
        if (build_ms) *build_ms = 0.0;
        return 0;
    }
    if (leaf_size < 1) leaf_size = 1;
    if (leaf_size > (uint32_t)kLeafMax) leaf_size = kLeafMax;
    out.depth4 = 0;
    out.level_start.clear();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);

    float4 *recs = nullptr;
    Aabb *boxes = nullptr, *node_boxes = nullptr;
    uint32_t *bounds = nullptr, *keys = nullptr, *vals = nullptr, *keys2 = nullptr, *vals2 = nullptr, *hist = nullptr,
             *flags = nullptr;
    int2 *children = nullptr, *ranges = nullptr;
    int *parent_internal = nullptr, *parent_leaf = nullptr;
    const uint32_t nblocks = (uint32_t)((n + kSortTile - 1) / kSortTile);
    hipError_t err = hipSuccess;
    err = dmalloc(&recs, 3 * (size_t)n);
    if (!err) err = dmalloc(&boxes, n);
    if (!err) err = dmalloc(&node_boxes, n);
    if (!err) err = dmalloc(&bounds, 6);
    if (!err) err = dmalloc(&keys, n);
    if (!err) err = dmalloc(&vals, n);
    if (!err) err = dmalloc(&keys2, n);
    if (!err) err = dmalloc(&vals2, n);
    if (!err) err = dmalloc(&hist, 256 * (size_t)nblocks);
    if (!err) err = dmalloc(&flags, n);
    if (!err) err = dmalloc(&children, n);
    if (!err) err = dmalloc(&ranges, n);
    if (!err) err = dmalloc(&parent_internal, n);
    if (!err) err = dmalloc(&parent_leaf, n);
    if (err) {
        free_lbvh(out);
    } else {
        const uint32_t g = (uint32_t)((n + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_prim_setup, dim3(g), dim3(kBlock), 0, s, in, recs, boxes);
        const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
        (void)hipMemcpyAsync(bounds, init, sizeof(init), hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(k_bounds, dim3(min(g, 1024u)), dim3(kBlock), 0, s, boxes, (uint32_t)n, bounds);
        hipLaunchKernelGGL(k_morton, dim3(g), dim3(kBlock), 0, s, boxes, (uint32_t)n, bounds, keys, vals);
        uint32_t *ki = keys, *vi = vals, *ko = keys2, *vo = vals2;
        for (int shift = 0; shift < 30; shift += 8) {
            hipLaunchKernelGGL(k_sort_hist, dim3(nblocks), dim3(kBlock), 0, s, ki, (uint32_t)n, shift, hist, nblocks);
            hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, 256u * nblocks);
            hipLaunchKernelGGL(k_sort_scatter, dim3(nblocks), dim3(kBlock), 0, s, ki, vi, ko, vo, (uint32_t)n, shift,
                               hist, nblocks);
            uint32_t *t = ki; ki = ko; ko = t;
            t = vi; vi = vo; vo = t;
        }
        // ki/vi hold the sorted keys/values
        if (n > 1) {
            (void)hipMemsetAsync(parent_internal, 0xFF, sizeof(int) * n, s);
            (void)hipMemsetAsync(flags, 0, sizeof(uint32_t) * n, s);
            const uint32_t gi = (uint32_t)((n - 1 + kBlock - 1) / kBlock);
            const char *builder = std::getenv("PUPIL_BVH_BUILDER");
            const bool ploc = !force_lbvh && !(builder && std::strcmp(builder, "lbvh") == 0);
            if (ploc) {
                err = build_ploc(n, vi, vo, boxes, children, ranges, node_boxes, parent_internal, parent_leaf, s);
                uint32_t *t = vi;  // vo holds the PLOC primitive order
                vi = vo;
                vo = t;
            } else {
                hipLaunchKernelGGL(k_karras, dim3(gi), dim3(kBlock), 0, s, ki, n, children, ranges, parent_internal,
                                   parent_leaf);
                hipLaunchKernelGGL(k_refit, dim3(g), dim3(kBlock), 0, s, n, vi, boxes, children, parent_internal,
                                   parent_leaf, node_boxes, flags);
            }
            const char *collapse = std::getenv("PUPIL_BVH4_COLLAPSE");
            if (!err && !(collapse && std::strcmp(collapse, "parity") == 0)) {
                // 4-wide quantized tree: SAH-optimal slot distribution (PUPIL_BVH4_COLLAPSE=greedy:
                // greedy surface-area opening)
                err = dmalloc(&out.nodes4, (size_t)(n - 1));
                if (!err)
                    err = collapse_bvh4(n, vi, boxes, children, ranges, node_boxes, leaf_size, out.nodes4,
                                        &out.num_nodes4, &out.depth4, &out.level_start, s,
                                        !(collapse && std::strcmp(collapse, "greedy") == 0));
            } else if (!err) {
            // 4-wide quantized tree: depth parity -> flags -> compact indices -> nodes
            uint32_t *depth = ko, *flags4 = vo, *idx4 = nullptr;  // the sort's free ping-pong buffers
            err = dmalloc(&idx4, n);
            hipLaunchKernelGGL(k_depth, dim3(gi), dim3(kBlock), 0, s, n, parent_internal, depth);
            hipLaunchKernelGGL(k_flag4, dim3(gi), dim3(kBlock), 0, s, n, ranges, depth, leaf_size, flags4);
            uint32_t tail[2] = {0, 0};
            if (!err) {
                (void)hipMemcpyAsync(idx4, flags4, sizeof(uint32_t) * (n - 1), hipMemcpyDeviceToDevice, s);
                hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, idx4, (uint32_t)(n - 1));
                (void)hipMemcpyAsync(&tail[0], idx4 + (n - 2), sizeof(uint32_t), hipMemcpyDeviceToHost, s);
                (void)hipMemcpyAsync(&tail[1], flags4 + (n - 2), sizeof(uint32_t), hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                out.num_nodes4 = tail[0] + tail[1];
                err = dmalloc(&out.nodes4, out.num_nodes4 ? out.num_nodes4 : 1);
            }
            if (!err)
                hipLaunchKernelGGL(k_emit4, dim3(gi), dim3(kBlock), 0, s, n, vi, boxes, children, ranges, node_boxes,
                                   flags4, idx4, leaf_size, out.nodes4);
            (void)hipStreamSynchronize(s);
            if (idx4) (void)hipFree(idx4);
            }
        } else {
            err = dmalloc(&out.nodes4, 1);
            out.num_nodes4 = 0;
        }
        const bool leaf_root = (uint32_t)n <= leaf_size;
        const uint32_t *rec_vals = vi;
        const uint32_t nrec = (uint32_t)n;
        // record slots: each leaf on a 128-B line (kRecF4); the links are rewritten to slots
        uint32_t nslots = 0;
        uint32_t *slot = nullptr;
        unsigned long long *lsz = nullptr, *ssum = nullptr, *stot = nullptr;
        const int per = kScanBlock * kScanItems;
        const int nbs = (int)((nrec + per - 1) / per);
        if (!err) err = dmalloc(&slot, nrec);
        if (!err) err = dmalloc(&lsz, nrec);
        if (!err) err = dmalloc(&ssum, nbs);
        if (!err) err = dmalloc(&stot, 1);
        if (!err && nbs > per) err = hipErrorInvalidValue;
        if (!err) {
            const uint32_t m = leaf_root ? 0u : out.num_nodes4;
            err = hipMemsetAsync(lsz, 0, sizeof(unsigned long long) * nrec, s);
            if (leaf_root && !err) {
                const unsigned long long v = leaf_slots(nrec);
                err = hipMemcpyAsync(lsz, &v, sizeof(v), hipMemcpyHostToDevice, s);
            }
            if (m) hipLaunchKernelGGL(k_leaf_marks, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s, out.nodes4, m, lsz);
            hipLaunchKernelGGL(k_scan64_blocks, dim3(nbs), dim3(kScanBlock), 0, s, lsz, (int)nrec, ssum);
            hipLaunchKernelGGL(k_scan64_sums, dim3(1), dim3(kScanBlock), 0, s, ssum, nbs, stot);
            hipLaunchKernelGGL(k_scan64_add, dim3((nrec + kBlock - 1) / kBlock), dim3(kBlock), 0, s, lsz, (int)nrec, ssum);
            if (m) hipLaunchKernelGGL(k_leaf_slots, dim3((m + kBlock - 1) / kBlock), dim3(kBlock), 0, s, out.nodes4, m, lsz, slot);
            if (leaf_root) {  // the root leaf: slots 0 .. n-1
                std::vector<uint32_t> id(nrec);
                for (uint32_t q = 0; q < nrec; q++) id[q] = q;
                if (!err) err = hipMemcpyAsync(slot, id.data(), sizeof(uint32_t) * nrec, hipMemcpyHostToDevice, s);
                if (!err) err = hipStreamSynchronize(s);
            }
            unsigned long long tot = 0;
            if (!err) err = hipMemcpyAsync(&tot, stot, sizeof(tot), hipMemcpyDeviceToHost, s);
            if (!err) err = hipStreamSynchronize(s);
            nslots = (uint32_t)tot;
            if (!err && tot >= (1ull << 28)) err = hipErrorInvalidValue;  // leaf links hold 28-bit slots
        }
        if (!err) err = dmalloc(&out.prims, (size_t)kRecF4 * nslots);
        if (!err) err = hipMemsetAsync(out.prims, 0xFF, sizeof(float4) * kRecF4 * (size_t)std::max(1u, nslots), s);
        const size_t nattr = in.object_space ? (size_t)nrec : (size_t)nslots;
        if (!err) err = dmalloc(&out.attrs, (size_t)kAttrStride * nattr);
        if (!err) {
            const uint32_t gr = (nrec + kBlock - 1) / kBlock;
            hipLaunchKernelGGL(k_reorder, dim3(gr), dim3(kBlock), 0, s, (int)nrec, rec_vals, slot, recs, out.prims);
            hipLaunchKernelGGL(k_attrs, dim3(gr), dim3(kBlock), 0, s, (int)nrec, rec_vals, slot, in, out.attrs);
        }
        (void)hipStreamSynchronize(s);
        for (void *p : {(void *)slot, (void *)lsz, (void *)ssum, (void *)stot})
            if (p) (void)hipFree(p);
        if (err) free_lbvh(out);
        out.num_records = nslots;
        if (n == 1 || leaf_root) out.depth4 = 1;  // the root is a leaf
        out.root_link4 = leaf_root ? (uint32_t)make_leaf(0u, (uint32_t)n) : 0u;
        if (!err) err = hipGetLastError();
    }
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (build_ms) *build_ms = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(recs);
    (void)hipFree(boxes);
    (void)hipFree(node_boxes);
    (void)hipFree(bounds);
    (void)hipFree(keys);
    (void)hipFree(vals);
    (void)hipFree(keys2);
    (void)hipFree(vals2);
    (void)hipFree(hist);
    (void)hipFree(flags);
    (void)hipFree(children);
    (void)hipFree(ranges);
    (void)hipFree(parent_internal);
    (void)hipFree(parent_leaf);
    return err == hipSuccess ? 0 : -2;
}

// BVH4 over n boxes (lo xyz, hi xyz; the world-mode TLAS over braided entries,
// accel_two_level.hip): Morton order, PLOC and the SAH-optimal collapse of the flattened
// build with one box per leaf.  On return `nodes` holds the 4-wide nodes (root 0,
// breadth first: parents before children) whose leaf links make_leaf(p, 1) name the
// box order[p].  n >= 2.
int build_bvh4_over_boxes(const float *h_boxes, uint32_t n, std::vector<Bvh4Node> &nodes, std::vector<uint32_t> &order,
                          uint32_t *depth, hipStream_t s) {
    if (n < 2) return -1;
    const int m = (int)n;
    Aabb *boxes = nullptr, *node_boxes = nullptr;
    uint32_t *bounds = nullptr, *keys = nullptr, *vals = nullptr, *keys2 = nullptr, *vals2 = nullptr, *hist = nullptr;
    int2 *children = nullptr, *ranges = nullptr;
    int *parent_internal = nullptr, *parent_leaf = nullptr;
    Bvh4Node *nodes4 = nullptr;
    const uint32_t nblocks = (n + kSortTile - 1) / kSortTile;
    hipError_t err = dmalloc(&boxes, n);
    if (!err) err = dmalloc(&node_boxes, n);
    if (!err) err = dmalloc(&bounds, 6);
    if (!err) err = dmalloc(&keys, n);
    if (!err) err = dmalloc(&vals, n);
    if (!err) err = dmalloc(&keys2, n);
    if (!err) err = dmalloc(&vals2, n);
    if (!err) err = dmalloc(&hist, 256 * (size_t)nblocks);
    if (!err) err = dmalloc(&children, n);
    if (!err) err = dmalloc(&ranges, n);
    if (!err) err = dmalloc(&parent_internal, n);
    if (!err) err = dmalloc(&parent_leaf, n);
    if (!err) err = dmalloc(&nodes4, n - 1);
    uint32_t num4 = 0, d4 = 0;
    uint32_t *vi = vals, *vo = vals2;
    if (!err) err = hipMemcpyAsync(boxes, h_boxes, sizeof(Aabb) * n, hipMemcpyHostToDevice, s);
    if (!err) {
        const uint32_t g = (n + kBlock - 1) / kBlock;
        const uint32_t init[6] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u, 0u};
        (void)hipMemcpyAsync(bounds, init, sizeof(init), hipMemcpyHostToDevice, s);
        hipLaunchKernelGGL(k_bounds, dim3(min(g, 1024u)), dim3(kBlock), 0, s, boxes, n, bounds);
        hipLaunchKernelGGL(k_morton, dim3(g), dim3(kBlock), 0, s, boxes, n, bounds, keys, vals);
        uint32_t *ki = keys, *ko = keys2;
        for (int shift = 0; shift < 30; shift += 8) {
            hipLaunchKernelGGL(k_sort_hist, dim3(nblocks), dim3(kBlock), 0, s, ki, n, shift, hist, nblocks);
            hipLaunchKernelGGL(k_sort_scan, dim3(1), dim3(1024), 0, s, hist, 256u * nblocks);
            hipLaunchKernelGGL(k_sort_scatter, dim3(nblocks), dim3(kBlock), 0, s, ki, vi, ko, vo, n, shift, hist,
                               nblocks);
            std::swap(ki, ko);
            std::swap(vi, vo);
        }
        (void)hipMemsetAsync(parent_internal, 0xFF, sizeof(int) * n, s);
        err = build_ploc(m, vi, vo, boxes, children, ranges, node_boxes, parent_internal, parent_leaf, s);
        std::swap(vi, vo);  // vi: the PLOC box order
        std::vector<uint32_t> level_start;
        if (!err)
            err = collapse_bvh4(m, vi, boxes, children, ranges, node_boxes, 1u, nodes4, &num4, &d4, &level_start, s,
                                true);
    }
    if (!err) {
        nodes.resize(num4);
        order.resize(n);
        err = hipMemcpyAsync(nodes.data(), nodes4, sizeof(Bvh4Node) * num4, hipMemcpyDeviceToHost, s);
        if (!err) err = hipMemcpyAsync(order.data(), vi, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, s);
        if (!err) err = hipStreamSynchronize(s);
    }
    if (depth) *depth = d4;
    for (void *p : {(void *)boxes, (void *)node_boxes, (void *)bounds, (void *)keys, (void *)vals, (void *)keys2,
                    (void *)vals2, (void *)hist, (void *)children, (void *)ranges, (void *)parent_internal,
                    (void *)parent_leaf, (void *)nodes4})
        if (p) (void)hipFree(p);
    return err == hipSuccess ? 0 : -2;
}

int build_bvh_bounded(const BvhBuildInput &in, BvhBuildOutput &out, uint32_t leaf_size, hipStream_t s,
                      double *build_ms, uint32_t reserve) {
    const auto fits = [&](const BvhBuildOutput &o) {
        return o.depth4 == 0 || 3u * o.depth4 + reserve <= (uint32_t)kTraceStackEntries;
    };
    int rc = build_lbvh(in, out, leaf_size, s, build_ms);
    if (rc != 0 || fits(out)) return rc;
    // PLOC merges nearest neighbours bottom-up and can chain a skewed primitive
    // distribution into a deep tree; the Karras LBVH splits on Morton bits.
    free_lbvh(out);
    double ms2 = 0.0;
    rc = build_lbvh(in, out, leaf_size, s, &ms2, true);
    if (build_ms) *build_ms += ms2;
    if (rc != 0) return rc;
    if (!fits(out)) {
        free_lbvh(out);
        return -3;
    }
    return 0;
}

// ------------------------------------------------------------------ refit (RenderInstanceUpdate)
namespace {

// Records of the moved instance (b.w = instance) get its new world vertices, written
// exactly as k_prim_setup writes them (global id in a.w: sphere bit + id).
__global__ void k_refit_records(BvhBuildInput in, uint32_t n, float4 *recs_base, const uint8_t *moved) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    float4 *recs = recs_base + (size_t)kRecF4 * r;
    const uint32_t id = __float_as_uint(recs[1].w);
    if (id == kRecHole || !moved[id]) return;  // a hole slot, or an unmoved instance
    const uint32_t gid = __float_as_uint(recs[0].w) & ~kPrimSphereBit;
    const DevInstance &inst = in.instances[id];
    if (inst.kind == PUPIL_SHAPE_SPHERE) {
        const float *m = inst.to_world;
        const vec3 c = v3(m[3], m[7], m[11]);
        const float ex = sqrtf(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]) * 1.001f;
        const float ey = sqrtf(m[4] * m[4] + m[5] * m[5] + m[6] * m[6]) * 1.001f;
        const float ez = sqrtf(m[8] * m[8] + m[9] * m[9] + m[10] * m[10]) * 1.001f;
        recs[0] = make_float4(c.x, c.y, c.z, recs[0].w);
        recs[1] = make_float4(ex, ey, ez, recs[1].w);
        return;
    }
    const uint32_t local = gid - inst.prim_offset;
    const uint32_t i0 = inst.indices[3 * local], i1 = inst.indices[3 * local + 1], i2 = inst.indices[3 * local + 2];
    const float *P = inst.positions;
    const vec3 w0 = xform_point(inst.to_world, v3(P[3 * i0], P[3 * i0 + 1], P[3 * i0 + 2]));
    const vec3 w1 = xform_point(inst.to_world, v3(P[3 * i1], P[3 * i1 + 1], P[3 * i1 + 2]));
    const vec3 w2 = xform_point(inst.to_world, v3(P[3 * i2], P[3 * i2 + 1], P[3 * i2 + 2]));
    recs[0] = make_float4(w0.x, w0.y, w0.z, recs[0].w);
    recs[1] = make_float4(w1.x, w1.y, w1.z, recs[1].w);
    recs[2] = make_float4(w2.x, w2.y, w2.z, recs[2].w);
}

// One BVH4 level, bottom up: child boxes from the records under a leaf (exact; a
// sphere's padded box) or from the child's box of the previous launch; re-quantised.
__global__ void k_refit_level(Bvh4Node *nodes, uint32_t lo, uint32_t hi, const float4 *recs, float *nbox) {
    for (uint32_t j = lo + blockIdx.x * blockDim.x + threadIdx.x; j < hi; j += gridDim.x * blockDim.x) {
        const Bvh4Node n = nodes[j];
        float clo[3][4], chi[3][4];
        float nlo[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
        float nhi[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
        int link[4];
        int nk = 0;
        for (int k = 0; k < 4; k++) {
            const int l = n.child[k];
            if (l == kEmptyLink) continue;
            float bl[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
            float bh[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
            if (l >= 0) {
                for (int a = 0; a < 3; a++) {
                    bl[a] = nbox[6 * (size_t)l + a];
                    bh[a] = nbox[6 * (size_t)l + 3 + a];
                }
            } else {
                for (uint32_t r = leaf_first(l); r < leaf_first(l) + leaf_count(l); r++) {
                    const float4 a = recs[kRecF4 * r], b = recs[kRecF4 * r + 1], c = recs[kRecF4 * r + 2];
                    if (__float_as_uint(a.w) & kPrimSphereBit) {
                        bl[0] = fminf(bl[0], a.x - b.x);
                        bl[1] = fminf(bl[1], a.y - b.y);
                        bl[2] = fminf(bl[2], a.z - b.z);
                        bh[0] = fmaxf(bh[0], a.x + b.x);
                        bh[1] = fmaxf(bh[1], a.y + b.y);
                        bh[2] = fmaxf(bh[2], a.z + b.z);
                    } else {
                        bl[0] = fminf(bl[0], fminf(fminf(a.x, b.x), c.x));
                        bl[1] = fminf(bl[1], fminf(fminf(a.y, b.y), c.y));
                        bl[2] = fminf(bl[2], fminf(fminf(a.z, b.z), c.z));
                        bh[0] = fmaxf(bh[0], fmaxf(fmaxf(a.x, b.x), c.x));
                        bh[1] = fmaxf(bh[1], fmaxf(fmaxf(a.y, b.y), c.y));
                        bh[2] = fmaxf(bh[2], fmaxf(fmaxf(a.z, b.z), c.z));
                    }
                }
            }
            for (int a = 0; a < 3; a++) {
                clo[a][nk] = bl[a];
                chi[a][nk] = bh[a];
                nlo[a] = fminf(nlo[a], bl[a]);
                nhi[a] = fmaxf(nhi[a], bh[a]);
            }
            link[nk++] = l;
        }
        nodes[j] = encode_bvh4(nlo, nhi, clo, chi, link, nk);
        for (int a = 0; a < 3; a++) {
            nbox[6 * (size_t)j + a] = nlo[a];
            nbox[6 * (size_t)j + 3 + a] = nhi[a];
        }
    }
}

}  // namespace

int refit_bvh4(const BvhBuildInput &in, BvhBuildOutput &out, const uint8_t *moved, float *nbox, hipStream_t s,
               double *ms) {
    if (out.level_start.size() < 2 || !out.nodes4 || out.num_nodes4 == 0) return -1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0, s);
    hipError_t err = hipSuccess;
    {
        const uint32_t n = out.num_records;  // record slots (holes are skipped)
        hipLaunchKernelGGL(k_refit_records, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, in, n, out.prims, moved);
        for (size_t L = out.level_start.size() - 1; L-- > 0;) {
            const uint32_t lo = out.level_start[L], hi = out.level_start[L + 1];
            const uint32_t g = std::max(1u, std::min(4096u, (hi - lo + kBlock - 1) / kBlock));
            hipLaunchKernelGGL(k_refit_level, dim3(g), dim3(kBlock), 0, s, out.nodes4, lo, hi, out.prims, nbox);
        }
        err = hipGetLastError();
    }
    (void)hipEventRecord(e1, s);
    if (!err) err = hipEventSynchronize(e1);
    float t = 0.f;
    (void)hipEventElapsedTime(&t, e0, e1);
    if (ms) *ms = t;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return err == hipSuccess ? 0 : -2;
}

}  // namespace pupil
