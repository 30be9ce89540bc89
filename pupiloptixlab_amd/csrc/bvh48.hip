// bvh48.hip — the 48-B traversal layout of a BVH4 (r05): one array of 48-B slots that holds
// every node AND every leaf record, derived from the builder's 64-B nodes + 64-B record slots
// after each build and refit (engine.hip refresh_node_bound).
//
// Why: the persistent traversal is bound by vector-memory instruction processing -- every
// wave-wide 16-B-per-lane load costs the CU's one texture addresser ~24 cycles, 0.77 of it busy
// (profiles/r05_pmc_mempipe_config4.txt), and four more loads per node visit cost +30 % even
// from one lane (+19 %, profiles/r05_node_fetch_sensitivity.txt).  A 64-B node is four such
// loads; 16 B of it are the four 32-bit child links.  Here a node's children (internal nodes
// and the records of its leaves) form ONE contiguous block of slots, so a node needs one base
// index and a byte per leaf child instead of four links: 48 B, three loads per visit.
//
// Node slot (12 dwords):
//   0..2  origin x, y, z (floats, as the 64-B node)
//   3     exponent bytes of the x / y / z plane scales (scale bits = e << 23, the 64-B node's
//         float exactly)
//   4..9  quantized planes lo x, y, z, hi x, y, z, byte k = child position k
//   10    base: the block's first slot
//   11    byte k = (offset << 3) | code of child position k: its slot is base + offset, code 7 an
//         internal node, code c < 7 a leaf of c + 1 records -- so every child link
//         ~(((base + offset) << 3) | code) is ~(base << 3) - byte: one subtraction per child
//         (pt_scene.h kCode48Node)
// Record slot (12 dwords): the 64-B record's first 48 B (v0 | key, v1 | instance, v2 | material
// bin).  A hit names its 48-B slot; flat scenes get their shading records (attrs) scattered to the
// same slot numbers (attrs48), world-mode hits name the global primitive id as before.
#include "pt_kernels.h"
#include "../../include/pupil_pt.h"

#include <hipcub/device/device_scan.hpp>

#include <algorithm>
#include <vector>

namespace pupil {

namespace {

constexpr int kBlk = 256;

struct ChildInfo {
    int ni, nl, ne;
    uint32_t size;  // slots of the block: ni nodes + leaf records + one hole if any empty child
};

__device__ __forceinline__ int child_kind(int link) {  // 0 internal, 1 leaf, 2 empty
    if (link < 0) return 1;
    return link < kTraverseDone ? 0 : 2;
}

__device__ __forceinline__ ChildInfo child_info(const Bvh4Node &n) {
    ChildInfo c{0, 0, 0, 0u};
    uint32_t recs = 0;
    for (int k = 0; k < 4; k++) {
        const int l = n.child[k];
        const int kind = child_kind(l);
        if (kind == 0) c.ni++;
        else if (kind == 1) {
            c.nl++;
            recs += leaf_count(l);
        } else c.ne++;
    }
    c.size = (uint32_t)c.ni + recs + (c.ne ? 1u : 0u);
    return c;
}

// one frontier entry per node of the level: x = 64-B node index, y = its 48-B slot
__global__ void k48_size(const Bvh4Node *nodes, const int2 *front, uint32_t n, unsigned long long *sz) {
    const uint32_t i = blockIdx.x * kBlk + threadIdx.x;
    if (i >= n) return;
    const ChildInfo c = child_info(nodes[front[i].x]);
    sz[i] = ((unsigned long long)c.size << 32) | (unsigned long long)c.ni;  // packed: block slots | internal children
}

__device__ __forceinline__ uint32_t exp_byte(float s) { return (__float_as_uint(s) >> 23) & 0xFFu; }

__device__ __forceinline__ void put_slot(float4 *t48, uint64_t slot, float4 a, float4 b, float4 c) {
    float4 *o = t48 + (size_t)kSlot48F4 * slot;
    o[0] = a;
    o[1] = b;
    o[2] = c;
}

__global__ void k48_emit(const Bvh4Node *nodes, const float4 *prims, const int2 *front, uint32_t n,
                         const unsigned long long *off, uint32_t next_slot, uint32_t next_front, float4 *t48,
                         int2 *front_out, uint32_t *err, const float4 *attrs, float4 *attrs48) {
    const uint32_t i = blockIdx.x * kBlk + threadIdx.x;
    if (i >= n) return;
    const Bvh4Node nd = nodes[front[i].x];
    const ChildInfo ci = child_info(nd);
    const uint32_t base = next_slot + (uint32_t)(off[i] >> 32);
    uint32_t fo = next_front + (uint32_t)(off[i] & 0xFFFFFFFFull);
    // child positions: internal first, then leaves, then empties (stable within each kind)
    int order[4], m = 0;
    for (int kind = 0; kind < 3; kind++)
        for (int k = 0; k < 4; k++)
            if (child_kind(nd.child[k]) == kind) order[m++] = k;
    uint32_t q[6] = {0u, 0u, 0u, 0u, 0u, 0u};
    const uint32_t src[6] = {nd.qlo_x, nd.qlo_y, nd.qlo_z, nd.qhi_x, nd.qhi_y, nd.qhi_z};
    uint32_t bytes = 0;
    uint32_t rec = (uint32_t)ci.ni;                              // next record offset in the block
    const uint32_t hole = ci.size - 1u;                           // hole slot offset (when ci.ne > 0)
    for (int p = 0; p < 4; p++) {
        const int k = order[p];
        for (int a = 0; a < 6; a++) q[a] |= ((src[a] >> (8 * k)) & 0xFFu) << (8 * p);
        const int l = nd.child[k];
        const int kind = child_kind(l);
        if (kind == 0) {
            front_out[fo++] = make_int2(l, (int)(base + (uint32_t)p));
            bytes |= (((uint32_t)p << 3) | kCode48Node) << (8 * p);
        } else if (kind == 1) {
            const uint32_t first = leaf_first(l), cnt = leaf_count(l);
            if (cnt > kCode48Node) atomicOr(err, 1u);  // code 7 is the internal node
            bytes |= ((rec << 3) | (cnt - 1u)) << (8 * p);
            for (uint32_t j = 0; j < cnt; j++) {
                const float4 *r = prims + (size_t)kRecF4 * (first + j);
                put_slot(t48, base + rec + j, r[0], r[1], r[2]);
                if (attrs48)
                    for (uint32_t k = 0; k < kAttrStride; k++)
                        attrs48[(size_t)kAttrStride * (base + rec + j) + k] = attrs[(size_t)kAttrStride * (first + j) + k];
            }
            rec += cnt;
        } else {
            bytes |= (hole << 3) << (8 * p);  // a one-record leaf on the hole
        }
    }
    if (ci.ne) {
        const float4 z = make_float4(0.f, 0.f, 0.f, __uint_as_float(0x7FFFFFFFu));
        put_slot(t48, base + hole, z, make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f));
    }
    const uint32_t w3 = exp_byte(nd.sx) | (exp_byte(nd.sy) << 8) | (exp_byte(nd.sz) << 16);
    put_slot(t48, (uint32_t)front[i].y, make_float4(nd.ox, nd.oy, nd.oz, __uint_as_float(w3)),
             make_float4(__uint_as_float(q[0]), __uint_as_float(q[1]), __uint_as_float(q[2]), __uint_as_float(q[3])),
             make_float4(__uint_as_float(q[4]), __uint_as_float(q[5]), __uint_as_float(base), __uint_as_float(bytes)));
}

// a leaf root (tiny scenes): its records at slots 0 .. count-1
__global__ void k48_root_leaf(const float4 *prims, uint32_t first, uint32_t cnt, float4 *t48, const float4 *attrs,
                              float4 *attrs48) {
    const uint32_t j = threadIdx.x;
    if (j >= cnt) return;
    const float4 *r = prims + (size_t)kRecF4 * (first + j);
    put_slot(t48, j, r[0], r[1], r[2]);
    if (attrs48)
        for (uint32_t k = 0; k < kAttrStride; k++)
            attrs48[(size_t)kAttrStride * j + k] = attrs[(size_t)kAttrStride * (first + j) + k];
}

}  // namespace

void free_trav48(Trav48 &t) {
    if (t.slots) (void)hipFree(t.slots);
    if (t.attrs) (void)hipFree(t.attrs);
    t = Trav48{};
}

// Breadth first from the root, one level per step: block sizes, one exclusive scan (block
// slots and internal-child counts packed in 64 bits), then every node of the level writes its
// 48-B slot, its leaves' records and the next level's frontier.  Only nodes reachable from the
// root are read (the two-level layouts hold never-written TLAS reserve nodes).
int build_trav48(const Bvh4Node *nodes, uint64_t num_nodes, uint32_t root_link, const float4 *prims,
                 uint64_t num_slots64, const float4 *attrs, Trav48 &out, hipStream_t s) {
    const int root = (int)root_link;
    // capacity: every reachable node once, every record slot once, a hole per node
    const uint64_t need = 2 * num_nodes + num_slots64 + 1;
    if (need * 16ull * kSlot48F4 >= (1ull << 32)) return PUPIL_ERR_UNSUPPORTED;  // 32-bit byte offsets
    if (out.cap < need || (attrs && !out.attrs)) {
        free_trav48(out);
        if (hipMalloc((void **)&out.slots, sizeof(float4) * kSlot48F4 * need) != hipSuccess) return PUPIL_ERR_OOM;
        if (attrs && hipMalloc((void **)&out.attrs, sizeof(float4) * kAttrStride * need) != hipSuccess) {
            free_trav48(out);
            return PUPIL_ERR_OOM;
        }
        out.cap = need;
    }
    float4 *attrs48 = attrs ? out.attrs : nullptr;
    if (root == kTraverseDone || num_slots64 == 0) {
        out.root = (uint32_t)kTraverseDone;
        out.used = 0;
        return PUPIL_OK;
    }
    if (root < 0) {
        if (leaf_count(root) > kCode48Node) return PUPIL_ERR_UNSUPPORTED;
        hipLaunchKernelGGL(k48_root_leaf, dim3(1), dim3(64), 0, s, prims, leaf_first(root), leaf_count(root), out.slots,
                           attrs, attrs48);
        out.root = (uint32_t)make_leaf(0u, leaf_count(root));
        out.used = leaf_count(root);
        return hipGetLastError() == hipSuccess ? PUPIL_OK : PUPIL_ERR_HIP;
    }
    int2 *fa = nullptr, *fb = nullptr;
    unsigned long long *sz = nullptr, *off = nullptr;
    uint32_t *err = nullptr;
    void *tmp = nullptr;
    size_t tmp_bytes = 0;
    const size_t fcap = std::max<uint64_t>(1, num_nodes);
    hipError_t e = hipMalloc((void **)&fa, sizeof(int2) * fcap);
    if (e == hipSuccess) e = hipMalloc((void **)&fb, sizeof(int2) * fcap);
    if (e == hipSuccess) e = hipMalloc((void **)&sz, sizeof(unsigned long long) * fcap);
    if (e == hipSuccess) e = hipMalloc((void **)&off, sizeof(unsigned long long) * fcap);
    if (e == hipSuccess) e = hipMalloc((void **)&err, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(err, 0, sizeof(uint32_t), s);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, sz, off, (int)fcap, s);
    if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(1, tmp_bytes));
    const int2 r0 = make_int2(root, 0);
    if (e == hipSuccess) e = hipMemcpyAsync(fa, &r0, sizeof(int2), hipMemcpyHostToDevice, s);
    uint32_t level_n = 1, next_slot = 1;
    uint64_t visited = 0;
    while (e == hipSuccess && level_n > 0) {
        visited += level_n;
        if (visited > num_nodes) {  // not a tree (a cycle or a shared subtree): cannot happen for these builders
            e = hipErrorInvalidValue;
            break;
        }
        const dim3 g((level_n + kBlk - 1) / kBlk);
        hipLaunchKernelGGL(k48_size, g, dim3(kBlk), 0, s, nodes, fa, level_n, sz);
        size_t tb = tmp_bytes;
        e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, sz, off, (int)level_n, s);
        if (e != hipSuccess) break;
        unsigned long long last[2] = {0ull, 0ull};
        e = hipMemcpyAsync(&last[0], off + (level_n - 1), sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipMemcpyAsync(&last[1], sz + (level_n - 1), sizeof(unsigned long long), hipMemcpyDeviceToHost, s);
        hipLaunchKernelGGL(k48_emit, g, dim3(kBlk), 0, s, nodes, prims, fa, level_n, off, next_slot, 0u, out.slots, fb,
                           err, attrs, attrs48);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) break;
        const unsigned long long total = last[0] + last[1];
        const uint64_t slots = total >> 32, inner = total & 0xFFFFFFFFull;
        if (next_slot + slots > out.cap || inner > num_nodes) {
            e = hipErrorInvalidValue;
            break;
        }
        next_slot += (uint32_t)slots;
        level_n = (uint32_t)inner;
        std::swap(fa, fb);
    }
    uint32_t bad = 0;
    if (e == hipSuccess) e = hipMemcpy(&bad, err, sizeof(bad), hipMemcpyDeviceToHost);
    for (void *p : {(void *)fa, (void *)fb, (void *)sz, (void *)off, (void *)err, tmp})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return PUPIL_ERR_HIP;
    if (bad) return PUPIL_ERR_UNSUPPORTED;  // a leaf of 8 records (PUPIL_LEAF_SIZE / PUPIL_SAH_LEAF 8)
    out.root = (uint32_t)~(int)kCode48Node;  // slot 0, internal
    out.used = next_slot;
    return PUPIL_OK;
}

}  // namespace pupil
