// accel_two_level.hip — two-level acceleration structure (the reference's
// IAS -> GAS hierarchy, world/ias_manager.cpp:29-114 + world/gas_manager.cpp:61-185).
//
// One object-space BLAS per mesh shape, built by the GPU builder
// (bvh_build.hip, object_space mode: PLOC + greedy BVH4 collapse, 64 B
// quantized nodes), and one TLAS over the instances whose leaves hold one
// instance each.  All nodes live in one Bvh4Node array: the TLAS in
// [0, tlas_cap), the BLASes after it with their links rebased.
//
// Hits stay bit-identical to the flattened single-level BVH and to the CPU
// oracle: BLAS boxes are only used for culling (with a margin that covers the
// object-space ray's rounding, see instance_margin), and every triangle is
// tested in WORLD space on its world vertices fl(to_world * v), computed with
// the same xform_point the flattened build and the oracle use.
//
// The TLAS is rebuilt on the host from the instance world boxes (binned SAH
// over a few instances is microseconds); an instance update recomputes that
// instance's box on the GPU and rebuilds the TLAS, the BLASes never change
// (the reference refits its IAS, ias_manager.cpp:116-151).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <vector>

#include "accel_limits.h"
#include "accel_two_level.h"
#include "bvh4_quant.h"

namespace pupil {

namespace {

constexpr int kBlock = 256;

// World box of each listed instance: exact bounds of its world-space vertices
// fl(to_world * v) (a mesh: every vertex; a sphere: the padded box of
// bvh_build.hip k_prim_setup).  One block per instance.
__global__ __launch_bounds__(kBlock) void k_inst_bounds(const DevInstance *insts, const uint32_t *list,
                                                        const uint32_t *num_verts, float *out) {
    __shared__ float red[kBlock / 64][6];
    const uint32_t id = list[blockIdx.x];
    const DevInstance &in = insts[id];
    float *o = out + 6 * (size_t)id;
    if (in.kind == PUPIL_SHAPE_SPHERE) {
        if (threadIdx.x == 0) {
            const float *m = in.to_world;
            const float ex = sqrtf(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]) * 1.001f;
            const float ey = sqrtf(m[4] * m[4] + m[5] * m[5] + m[6] * m[6]) * 1.001f;
            const float ez = sqrtf(m[8] * m[8] + m[9] * m[9] + m[10] * m[10]) * 1.001f;
            o[0] = m[3] - ex;
            o[1] = m[7] - ey;
            o[2] = m[11] - ez;
            o[3] = m[3] + ex;
            o[4] = m[7] + ey;
            o[5] = m[11] + ez;
        }
        return;
    }
    float v[6] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf(),
                  -__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
    const uint32_t nv = num_verts[id];
    for (uint32_t i = threadIdx.x; i < nv; i += blockDim.x) {
        const float *P = in.positions + 3 * (size_t)i;
        const vec3 w = xform_point(in.to_world, v3(P[0], P[1], P[2]));
        v[0] = fminf(v[0], w.x);
        v[1] = fminf(v[1], w.y);
        v[2] = fminf(v[2], w.z);
        v[3] = fmaxf(v[3], w.x);
        v[4] = fmaxf(v[4], w.y);
        v[5] = fmaxf(v[5], w.z);
    }
    for (int s = 32; s > 0; s >>= 1)
        for (int k = 0; k < 6; k++) {
            const float x = __shfl_xor(v[k], s);
            v[k] = k < 3 ? fminf(v[k], x) : fmaxf(v[k], x);
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 6; k++) red[threadIdx.x >> 6][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0)
        for (int k = 0; k < 6; k++) {
            float x = red[0][k];
            for (int w = 1; w < kBlock / 64; w++) x = k < 3 ? fminf(x, red[w][k]) : fmaxf(x, red[w][k]);
            o[k] = x;
        }
}

// World-space triangle records of each listed mesh instance: its BLAS records'
// vertices through fl(to_world * v) (the product the flattened build and the
// oracle test), so the two-level leaf test needs no per-triangle transform.
// Grid: x over the instance's primitives, y over the list.
__global__ __launch_bounds__(kBlock) void k_world_records(const DevInstance *insts, const uint32_t *list,
                                                          const uint32_t *num_prims, const float4 *obj, float4 *wrec) {
    const uint32_t id = list[blockIdx.y];
    const DevInstance &in = insts[id];
    if (in.kind == PUPIL_SHAPE_SPHERE) return;
    const uint32_t n = num_prims[id];  // the shape's BLAS record slots
    const uint32_t base = in.rec_base;  // the shape's first BLAS record slot
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const float4 a = obj[kRecF4 * (size_t)(base + j) + 0];
        const float4 b = obj[kRecF4 * (size_t)(base + j) + 1];
        const float4 c = obj[kRecF4 * (size_t)(base + j) + 2];
        float4 *o = wrec + kRecF4 * (size_t)((int64_t)base + j + in.wrec_delta);
        if (__float_as_uint(a.w) == kRecHole) {  // a hole slot stays a hole
            o[0] = a;
            o[1] = b;
            continue;
        }
        const vec3 w0 = xform_point(in.to_world, v3(a.x, a.y, a.z));
        const vec3 w1 = xform_point(in.to_world, v3(b.x, b.y, b.z));
        const vec3 w2 = xform_point(in.to_world, v3(c.x, c.y, c.z));
        // flat record format (bvh_build.hip k_prim_setup): a.w = global id, b.w = instance, c.w = material bin
        o[0] = make_float4(w0.x, w0.y, w0.z, __uint_as_float(in.prim_offset + __float_as_uint(a.w)));
        o[1] = make_float4(w1.x, w1.y, w1.z, __uint_as_float(id));
        o[2] = make_float4(w2.x, w2.y, w2.z, __uint_as_float(in.bin));
    }
}

// World-space copy of a mesh instance's BLAS (world mode), one BVH4 level per
// launch from the deepest up: the node keeps the shared BLAS topology, and each
// child box is refitted to the world geometry under it -- a leaf child's box is
// the exact bounds of its world records fl(to_world * v), an inner child's box is
// the world box its own copy got one launch earlier -- then quantised
// conservatively.  Links move to the copy: inner links to wnode_base, leaf links
// to the instance's world records (+ wrec_delta).  Records bounded exactly keep
// the leaf test's hits; the boxes are as tight as a fresh world-space build of the
// same topology (transforming object boxes would inflate every box it rotates).
__global__ __launch_bounds__(kBlock) void k_world_refit(const DevInstance *insts, const uint32_t *inst,
                                                        uint32_t lo, uint32_t hi, const Bvh4Node *obj,
                                                        const float4 *wrec, Bvh4Node *wn, float *wbox) {
    const DevInstance &in = insts[*inst];
    for (uint32_t j = lo + blockIdx.x * blockDim.x + threadIdx.x; j < hi; j += gridDim.x * blockDim.x) {
        const Bvh4Node n = obj[in.obj_nbase + j];
        float clo[3][4], chi[3][4], nlo[3], nhi[3];
        int link[4];
        int nk = 0;
        for (int a = 0; a < 3; a++) {
            nlo[a] = __builtin_huge_valf();
            nhi[a] = -__builtin_huge_valf();
        }
        for (int k = 0; k < 4; k++) {
            const int l = n.child[k];
            if (l == kEmptyLink) continue;
            float bl[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
            float bh[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
            if (l >= 0) {
                const int w = (int)(l - (int)in.obj_nbase + (int)in.wnode_base);
                for (int a = 0; a < 3; a++) {
                    bl[a] = wbox[6 * (size_t)w + a];
                    bh[a] = wbox[6 * (size_t)w + 3 + a];
                }
                link[nk] = w;
            } else {
                const uint32_t first = (uint32_t)((int64_t)leaf_first(l) + in.wrec_delta), cnt = leaf_count(l);
                for (uint32_t r = first; r < first + cnt; r++)
                    for (int v = 0; v < 3; v++) {
                        const float4 p = wrec[kRecF4 * (size_t)r + v];
                        bl[0] = fminf(bl[0], p.x);
                        bl[1] = fminf(bl[1], p.y);
                        bl[2] = fminf(bl[2], p.z);
                        bh[0] = fmaxf(bh[0], p.x);
                        bh[1] = fmaxf(bh[1], p.y);
                        bh[2] = fmaxf(bh[2], p.z);
                    }
                link[nk] = make_leaf(first, cnt);
            }
            for (int a = 0; a < 3; a++) {
                clo[a][nk] = bl[a];
                chi[a][nk] = bh[a];
                nlo[a] = fminf(nlo[a], bl[a]);
                nhi[a] = fmaxf(nhi[a], bh[a]);
            }
            nk++;
        }
        wn[in.wnode_base + j] = encode_bvh4(nlo, nhi, clo, chi, link, nk);
        float *b = wbox + 6 * (size_t)(in.wnode_base + j);
        for (int a = 0; a < 3; a++) {
            b[a] = nlo[a];
            b[3 + a] = nhi[a];
        }
    }
}

// World-mode TLAS refit (RenderInstanceUpdate; the reference refits its IAS,
// ias_manager.cpp:116-151): the TLAS keeps its topology and every node over the
// TLAS level [lo, hi) of `order` gets its child boxes anew -- a TLAS or world BLAS
// node child: the exact world box its refit left in wbox (TLAS levels run deepest
// first); a record leaf: the exact bounds of its world records; a sphere record: its
// instance's world box -- then is quantised conservatively, like k_world_refit.
__global__ __launch_bounds__(kBlock) void k_tlas_refit(const uint32_t *order, uint32_t lo, uint32_t hi,
                                                       const float4 *wrec, const float *inst_box, Bvh4Node *wn,
                                                       float *wbox) {
    for (uint32_t j = lo + blockIdx.x * blockDim.x + threadIdx.x; j < hi; j += gridDim.x * blockDim.x) {
        const uint32_t v = order[j];
        const Bvh4Node n = wn[v];
        float clo[3][4], chi[3][4], nlo[3], nhi[3];
        int link[4];
        int nk = 0;
        for (int a = 0; a < 3; a++) {
            nlo[a] = __builtin_huge_valf();
            nhi[a] = -__builtin_huge_valf();
        }
        for (int k = 0; k < 4; k++) {
            const int l = n.child[k];
            if (l == kEmptyLink) continue;
            float bl[3] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf()};
            float bh[3] = {-__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
            if (l >= 0) {
                for (int a = 0; a < 3; a++) {
                    bl[a] = wbox[6 * (size_t)l + a];
                    bh[a] = wbox[6 * (size_t)l + 3 + a];
                }
            } else {
                const uint32_t first = leaf_first(l), cnt = leaf_count(l);
                if (__float_as_uint(wrec[kRecF4 * (size_t)first].w) & kPrimSphereBit) {
                    const uint32_t i = __float_as_uint(wrec[kRecF4 * (size_t)first + 1].w);
                    for (int a = 0; a < 3; a++) {
                        bl[a] = inst_box[6 * (size_t)i + a];
                        bh[a] = inst_box[6 * (size_t)i + 3 + a];
                    }
                } else {
                    for (uint32_t r = first; r < first + cnt; r++)
                        for (int c = 0; c < 3; c++) {
                            const float4 q = wrec[kRecF4 * (size_t)r + c];
                            bl[0] = fminf(bl[0], q.x);
                            bl[1] = fminf(bl[1], q.y);
                            bl[2] = fminf(bl[2], q.z);
                            bh[0] = fmaxf(bh[0], q.x);
                            bh[1] = fmaxf(bh[1], q.y);
                            bh[2] = fmaxf(bh[2], q.z);
                        }
                }
            }
            link[nk] = l;
            for (int a = 0; a < 3; a++) {
                clo[a][nk] = bl[a];
                chi[a][nk] = bh[a];
                nlo[a] = fminf(nlo[a], bl[a]);
                nhi[a] = fmaxf(nhi[a], bh[a]);
            }
            nk++;
        }
        wn[v] = encode_bvh4(nlo, nhi, clo, chi, link, nk);
        for (int a = 0; a < 3; a++) {
            wbox[6 * (size_t)v + a] = nlo[a];
            wbox[6 * (size_t)v + 3 + a] = nhi[a];
        }
    }
}

// Rebase the links of one BLAS copied into the combined node array.
__global__ void k_relink(Bvh4Node *nodes, uint32_t count, uint32_t node_base, uint32_t prim_base) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    Bvh4Node &n = nodes[node_base + i];
    for (int k = 0; k < 4; k++) n.child[k] = rebase_link(n.child[k], node_base, prim_base);
}

struct HostBox {
    float lo[3], hi[3];
    void grow(const HostBox &b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const {
        const float dx = std::max(0.f, hi[0] - lo[0]), dy = std::max(0.f, hi[1] - lo[1]),
                    dz = std::max(0.f, hi[2] - lo[2]);
        return dx * dy + dy * dz + dz * dx;
    }
    static HostBox empty() {
        const float inf = __builtin_huge_valf();
        return HostBox{{inf, inf, inf}, {-inf, -inf, -inf}};
    }
};

// Top-down SAH split of ids[b, e) over all three axes (r02 tried the widest centroid
// axis only): ranges above 1024 entries (world-mode braided entries) by 64-bin binned
// SAH per axis, O(n) per split; smaller ones by a full sweep over the centroid order
// of each axis.  binned (or null): counts the splits the binned SAH chose.
uint32_t sah_split(std::vector<uint32_t> &ids, uint32_t b, uint32_t e, const std::vector<HostBox> &boxes,
                   uint32_t *binned) {
    HostBox cb = HostBox::empty();
    for (uint32_t i = b; i < e; i++) {
        const HostBox &x = boxes[ids[i]];
        for (int k = 0; k < 3; k++) {
            const float c = 0.5f * (x.lo[k] + x.hi[k]);
            cb.lo[k] = std::min(cb.lo[k], c);
            cb.hi[k] = std::max(cb.hi[k], c);
        }
    }
    const uint32_t n = e - b;
    if (n > 1024) {
        constexpr int kBins = 64;
        float best = __builtin_huge_valf();
        int best_axis = -1, best_cut = 0;
        for (int axis = 0; axis < 3; axis++) {
            const float lo = cb.lo[axis], ext = cb.hi[axis] - cb.lo[axis];
            if (!(ext > 0.f)) continue;
            HostBox bb[kBins];
            uint32_t cnt[kBins] = {};
            for (auto &x : bb) x = HostBox::empty();
            for (uint32_t i = b; i < e; i++) {
                const HostBox &x = boxes[ids[i]];
                const float c = 0.5f * (x.lo[axis] + x.hi[axis]);
                const int k = std::min(kBins - 1, std::max(0, (int)((c - lo) / ext * kBins)));
                bb[k].grow(x);
                cnt[k]++;
            }
            float right[kBins];
            HostBox acc = HostBox::empty();
            uint32_t rn = 0;
            for (int k = kBins - 1; k > 0; k--) {
                acc.grow(bb[k]);
                rn += cnt[k];
                right[k] = acc.area() * (float)rn;
            }
            acc = HostBox::empty();
            uint32_t ln = 0;
            for (int k = 1; k < kBins; k++) {
                acc.grow(bb[k - 1]);
                ln += cnt[k - 1];
                if (ln == 0 || ln == n) continue;
                const float cost = acc.area() * (float)ln + right[k];
                if (cost < best) {
                    best = cost;
                    best_axis = axis;
                    best_cut = k;
                }
            }
        }
        if (best_axis >= 0) {
            const float lo = cb.lo[best_axis], ext = cb.hi[best_axis] - cb.lo[best_axis];
            const auto mid = std::stable_partition(ids.begin() + b, ids.begin() + e, [&](uint32_t id) {
                const float c = 0.5f * (boxes[id].lo[best_axis] + boxes[id].hi[best_axis]);
                return std::min(kBins - 1, std::max(0, (int)((c - lo) / ext * kBins))) < best_cut;
            });
            const uint32_t m = (uint32_t)(mid - ids.begin());
            if (m > b && m < e) {
                if (binned) (*binned)++;
                return m;
            }
        }
    }
    // full sweep per axis over the centroid order; the best axis's order is kept
    float best = __builtin_huge_valf();
    int best_axis = 0;
    uint32_t best_split = b + n / 2;
    std::vector<float> right(n + 1, 0.f);
    for (int axis = 0; axis < 3; axis++) {
        if (!(cb.hi[axis] - cb.lo[axis] > 0.f) && axis != 2) continue;
        std::stable_sort(ids.begin() + b, ids.begin() + e, [&](uint32_t x, uint32_t y) {
            return boxes[x].lo[axis] + boxes[x].hi[axis] < boxes[y].lo[axis] + boxes[y].hi[axis];
        });
        HostBox acc = HostBox::empty();
        for (uint32_t i = n; i-- > 1;) {
            acc.grow(boxes[ids[b + i]]);
            right[i] = acc.area() * (float)(n - i);
        }
        acc = HostBox::empty();
        for (uint32_t i = 1; i < n; i++) {
            acc.grow(boxes[ids[b + i - 1]]);
            const float cost = acc.area() * (float)i + right[i];
            if (cost < best) {
                best = cost;
                best_axis = axis;
                best_split = b + i;
            }
        }
    }
    std::stable_sort(ids.begin() + b, ids.begin() + e, [&](uint32_t x, uint32_t y) {
        return boxes[x].lo[best_axis] + boxes[x].hi[best_axis] < boxes[y].lo[best_axis] + boxes[y].hi[best_axis];
    });
    return best_split;
}

// 4-wide TLAS node over ids[b, e) (two levels of binary SAH splits); returns its link.
// links == nullptr: leaves are instances (object mode); else leaves are the entry
// links themselves (world mode: nodes of the world BLAS copies, or records)
int build_tlas_node(std::vector<uint32_t> &ids, uint32_t b, uint32_t e, const std::vector<HostBox> &boxes,
                    std::vector<Bvh4Node> &nodes, uint32_t level, uint32_t &depth, const std::vector<int> *links = nullptr,
                    uint32_t *binned = nullptr) {
    if (e - b == 1) return links ? (*links)[ids[b]] : make_leaf(ids[b], 1u);
    depth = std::max(depth, level + 1);
    uint32_t ranges[4][2];
    int nk = 0;
    const uint32_t m = sah_split(ids, b, e, boxes, binned);
    const uint32_t half[2][2] = {{b, m}, {m, e}};
    for (auto &h : half) {
        if (h[1] - h[0] > 1) {
            const uint32_t mm = sah_split(ids, h[0], h[1], boxes, binned);
            ranges[nk][0] = h[0];
            ranges[nk++][1] = mm;
            ranges[nk][0] = mm;
            ranges[nk++][1] = h[1];
        } else {
            ranges[nk][0] = h[0];
            ranges[nk++][1] = h[1];
        }
    }
    const uint32_t self = (uint32_t)nodes.size();
    nodes.emplace_back();
    int link[4];
    float clo[3][4] = {}, chi[3][4] = {};
    HostBox nb = HostBox::empty();
    for (int k = 0; k < nk; k++) {
        HostBox cb = HostBox::empty();
        for (uint32_t i = ranges[k][0]; i < ranges[k][1]; i++) cb.grow(boxes[ids[i]]);
        nb.grow(cb);
        for (int a = 0; a < 3; a++) {
            clo[a][k] = cb.lo[a];
            chi[a][k] = cb.hi[a];
        }
        link[k] = build_tlas_node(ids, ranges[k][0], ranges[k][1], boxes, nodes, level + 1, depth, links, binned);
    }
    nodes[self] = encode_bvh4(nb.lo, nb.hi, clo, chi, link, nk);
    return (int)self;
}

// Object-space box margin of an instance (see accel_two_level.h).  A world hit
// X = o + t d on the triangle fl(M v_k) maps through the float inverse A to
// within c u |A| (|M| |v| + |m_t|) of the object triangle, and the computed
// object ray fl(A o) + t fl(A d) differs from A X by c u (|A| (|o| + t |d|) + |a_t|),
// c <= 8.  The margin uses 2^-18 = 32 u (a factor 4 of headroom) with infinity
// norms, so an object-space BLAS box never culls a triangle the world-space
// test reports.
void instance_margin(DevInstance &d, float vmax) {
    d.vmax = vmax;
    float anorm = 0.f, at = 0.f, mnorm = 0.f, mt = 0.f;
    for (int r = 0; r < 3; r++) {
        anorm = std::max(anorm, std::fabs(d.to_object[4 * r]) + std::fabs(d.to_object[4 * r + 1]) +
                                    std::fabs(d.to_object[4 * r + 2]));
        mnorm = std::max(mnorm, std::fabs(d.to_world[4 * r]) + std::fabs(d.to_world[4 * r + 1]) +
                                    std::fabs(d.to_world[4 * r + 2]));
        at = std::max(at, std::fabs(d.to_object[4 * r + 3]));
        mt = std::max(mt, std::fabs(d.to_world[4 * r + 3]));
    }
    const float c = 0x1p-18f;
    d.margin[0] = c * anorm;
    d.margin[1] = c * (anorm * (mnorm * vmax + mt) + at);
}

// World mode: the TLAS entries of instance `id` -- its world BLAS root expanded
// `braid` levels down (partial re-braiding, Benthin et al. 2017), each with its
// world box decoded from the quantised parent (or the instance box at the root).
// The copy's top nodes come first in breadth-first order, so one download covers them.
bool world_entries(TwoLevelAccel &acc, const DevInstance &d, uint32_t id, uint32_t sphere_rec, hipStream_t s) {
    auto &out = acc.entries[id];
    out.clear();
    const std::array<float, 6> ibox = {d.wlo[0], d.wlo[1], d.wlo[2], d.whi[0], d.whi[1], d.whi[2]};
    if (d.kind == PUPIL_SHAPE_SPHERE) {
        out.push_back({make_leaf(sphere_rec, 1u), ibox});
        return true;
    }
    if (d.blas_root == kTraverseDone) return true;
    const int root = d.blas_root >= 0 ? (int)(d.blas_root - (int)d.obj_nbase + (int)d.wnode_base)
                                      : make_leaf((uint32_t)((int64_t)leaf_first(d.blas_root) + d.wrec_delta),
                                                  leaf_count(d.blas_root));
    out.push_back({root, ibox});
    uint32_t levels_nodes = 0, width = 1;
    for (uint32_t l = 0; l < acc.braid; l++, width *= 4) levels_nodes += width;
    const uint32_t ntop = std::min(d.obj_ncount, levels_nodes);
    std::vector<Bvh4Node> top(ntop);
    if (ntop && (hipMemcpyAsync(top.data(), acc.wnodes + d.wnode_base, sizeof(Bvh4Node) * ntop, hipMemcpyDeviceToHost,
                                s) != hipSuccess ||
                 hipStreamSynchronize(s) != hipSuccess))
        return false;
    for (uint32_t l = 0; l < acc.braid; l++) {
        std::vector<std::pair<int, std::array<float, 6>>> next;
        for (const auto &e : out) {
            const int j = e.first - (int)d.wnode_base;
            if (e.first < 0 || j < 0 || j >= (int)ntop) {
                next.push_back(e);
                continue;
            }
            const Bvh4Node &n = top[(size_t)j];
            const float sc3[3] = {n.sx, n.sy, n.sz};
            const float org[3] = {n.ox, n.oy, n.oz};
            const uint32_t qlo[3] = {n.qlo_x, n.qlo_y, n.qlo_z}, qhi[3] = {n.qhi_x, n.qhi_y, n.qhi_z};
            for (int k = 0; k < 4; k++) {
                if (n.child[k] == kEmptyLink) continue;
                std::array<float, 6> b;
                for (int a = 0; a < 3; a++) {
                    b[a] = qdecode(org[a], (qlo[a] >> (8 * k)) & 0xFFu, sc3[a]);
                    b[3 + a] = qdecode(org[a], (qhi[a] >> (8 * k)) & 0xFFu, sc3[a]);
                }
                next.push_back({n.child[k], b});
            }
        }
        out.swap(next);
    }
    return true;
}

}  // namespace

void refresh_instance_margins(DevInstance &d) {
    if (d.kind != PUPIL_SHAPE_SPHERE) instance_margin(d, d.vmax);
}

// World mode, RenderInstanceUpdate: the TLAS keeps its topology and its boxes are
// refitted bottom up on the GPU, one launch per TLAS level from the deepest (r03; the
// host refit it replaces re-encoded every node on the CPU: 26 ms at braid 6, 0.8 s at
// braid 8).  false: no level order (no TLAS nodes, or a failed build) -- rebuild.
bool refit_world_tlas(TwoLevelAccel &acc, hipStream_t s) {
    if (acc.tlas_nodes == 0 || acc.tlas_level_start.size() < 2 || !acc.d_tlas_order) return false;
    for (size_t L = 0; L + 1 < acc.tlas_level_start.size(); L++) {
        const uint32_t lo = acc.tlas_level_start[L], hi = acc.tlas_level_start[L + 1];
        if (hi <= lo) continue;
        const uint32_t g = std::min(1024u, (hi - lo + kBlock - 1) / kBlock);
        hipLaunchKernelGGL(k_tlas_refit, dim3(std::max(1u, g)), dim3(kBlock), 0, s, acc.d_tlas_order, lo, hi,
                           acc.wprims, acc.d_boxes, acc.wnodes, acc.d_wbox);
    }
    return hipGetLastError() == hipSuccess && hipStreamSynchronize(s) == hipSuccess;
}

int rebuild_tlas(TwoLevelAccel &acc, std::vector<DevInstance> &insts, DevInstance *d_insts,
                 const std::vector<uint32_t> &changed, hipStream_t s, bool refit) {
    const uint32_t n = (uint32_t)insts.size();
    if (!changed.empty()) {
        if (hipMemcpyAsync(acc.d_list, changed.data(), sizeof(uint32_t) * changed.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess)
            return -1;
        hipLaunchKernelGGL(k_inst_bounds, dim3((uint32_t)changed.size()), dim3(kBlock), 0, s, d_insts, acc.d_list,
                           acc.d_verts, acc.d_boxes);
        if (acc.wprims)  // the changed instances' world-space triangle records
            hipLaunchKernelGGL(k_world_records, dim3(256, (uint32_t)changed.size()), dim3(kBlock), 0, s, d_insts,
                               acc.d_list, acc.d_faces, acc.prims, acc.wprims);
        if (acc.world)  // ... and their world BLAS copies, refitted level by level from the deepest
            for (size_t c = 0; c < changed.size(); c++) {
                const uint32_t id = changed[c];
                if (insts[id].kind == PUPIL_SHAPE_SPHERE || insts[id].obj_ncount == 0) continue;
                const std::vector<uint32_t> &ls = acc.shape_levels[acc.inst_shape[id]];
                for (size_t L = ls.size() - 1; L-- > 0;) {
                    const uint32_t lo = ls[L], hi = ls[L + 1];
                    const uint32_t g = std::min(1024u, (hi - lo + kBlock - 1) / kBlock);
                    hipLaunchKernelGGL(k_world_refit, dim3(std::max(1u, g)), dim3(kBlock), 0, s, d_insts,
                                       acc.d_list + c, lo, hi, acc.nodes4, acc.wprims, acc.wnodes, acc.d_wbox);
                }
            }
        std::vector<float> h(6 * (size_t)n);
        if (hipMemcpyAsync(h.data(), acc.d_boxes, sizeof(float) * h.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return -1;
        for (uint32_t id : changed) {
            for (int k = 0; k < 3; k++) {
                insts[id].wlo[k] = h[6 * (size_t)id + k];
                insts[id].whi[k] = h[6 * (size_t)id + 3 + k];
            }
            if (hipMemcpyAsync(d_insts + id, &insts[id], sizeof(DevInstance), hipMemcpyHostToDevice, s) != hipSuccess)
                return -1;
        }
    }
    if (acc.world) {  // TLAS over the braided entries of every instance
        // sphere records follow the mesh records, in instance order, one leaf (2 slots) each
        uint32_t srec = acc.num_wprims;
        std::vector<uint32_t> sphere_rec(n, 0);
        for (uint32_t i = 0; i < n; i++)
            if (insts[i].kind == PUPIL_SHAPE_SPHERE) {
                sphere_rec[i] = srec;
                srec += leaf_slots(1u);
            }
        for (uint32_t id : changed)
            if (!world_entries(acc, insts[id], id, sphere_rec[id], s)) return -1;
        if (refit && refit_world_tlas(acc, s)) return 0;
        std::vector<HostBox> eb;
        std::vector<int> links;
        for (uint32_t i = 0; i < n; i++)
            for (const auto &e : acc.entries[i]) {
                HostBox b;
                for (int a = 0; a < 3; a++) {
                    b.lo[a] = e.second[a];
                    b.hi[a] = e.second[3 + a];
                }
                eb.push_back(b);
                links.push_back(e.first);
            }
        std::vector<uint32_t> ids(eb.size());
        std::iota(ids.begin(), ids.end(), 0u);
        std::vector<Bvh4Node> nodes;
        uint32_t depth = 0;
        int root = kTraverseDone;
        uint32_t binned = 0;
        // above 64 entries the TLAS is built like the flattened BVH (GPU Morton order, PLOC,
        // SAH-optimal 4-wide collapse, one entry per leaf) and its leaf links are replaced by
        // the entries' links; PUPIL_TL_BUILDER=host keeps the host's top-down binned SAH
        const char *tb = std::getenv("PUPIL_TL_BUILDER");
        const bool gpu_tlas = ids.size() > 64 && !(tb && std::strcmp(tb, "host") == 0);
        if (ids.size() == 1) {
            root = links[0];
        } else if (gpu_tlas) {
            std::vector<uint32_t> order;
            if (build_bvh4_over_boxes(&eb[0].lo[0], (uint32_t)eb.size(), nodes, order, &depth, s) != 0) return -1;
            for (Bvh4Node &nd : nodes)
                for (int k = 0; k < 4; k++)
                    if (nd.child[k] < 0) nd.child[k] = links[order[leaf_first(nd.child[k])]];
            root = 0;
            binned = (uint32_t)nodes.size();  // every TLAS node placed by the SAH collapse
        } else if (!ids.empty()) {
            root = build_tlas_node(ids, 0, (uint32_t)ids.size(), eb, nodes, 0u, depth, &links, &binned);
        }
        if (nodes.size() > acc.tlas_cap) return -1;
        if (3u * depth + 3u * acc.blas_depth > (uint32_t)kTraceStackEntries) return -3;
        acc.tlas_depth = depth;
        if (!nodes.empty() &&
            hipMemcpyAsync(acc.wnodes, nodes.data(), sizeof(Bvh4Node) * nodes.size(), hipMemcpyHostToDevice, s) !=
                hipSuccess)
            return -1;
        acc.tlas_nodes = (uint32_t)nodes.size();
        acc.sah_splits = binned;
        {  // TLAS levels for the GPU refits: node ids by level, deepest first
            std::vector<uint32_t> level(nodes.size(), 0u), bfs;
            if (!nodes.empty()) bfs.push_back(0u);
            for (size_t h = 0; h < bfs.size(); h++)
                for (int k = 0; k < 4; k++) {
                    const int l = nodes[bfs[h]].child[k];
                    if (l == kEmptyLink || l < 0 || (size_t)l >= nodes.size()) continue;
                    level[l] = level[bfs[h]] + 1u;
                    bfs.push_back((uint32_t)l);
                }
            acc.tlas_level_start.assign(1, 0u);
            std::vector<uint32_t> order;
            if (bfs.size() == nodes.size()) {  // every node reached from the root (node 0)
                // breadth-first order has non-decreasing levels: reversed, deepest level first
                order.assign(bfs.rbegin(), bfs.rend());
                for (uint32_t j = 1; j <= (uint32_t)order.size(); j++)
                    if (j == (uint32_t)order.size() || level[order[j]] != level[order[j - 1]])
                        acc.tlas_level_start.push_back(j);
            } else {
                acc.tlas_level_start.clear();  // not a tree rooted at node 0: refits rebuild
            }
            if (!order.empty() && (hipMemcpyAsync(acc.d_tlas_order, order.data(), sizeof(uint32_t) * order.size(),
                                                  hipMemcpyHostToDevice, s) != hipSuccess ||
                                   hipStreamSynchronize(s) != hipSuccess))  // `order` dies with this block
                return -1;
        }
        acc.root_link4 = (uint32_t)root;
        return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
    }
    std::vector<HostBox> boxes(n);
    for (uint32_t i = 0; i < n; i++)
        for (int k = 0; k < 3; k++) {
            boxes[i].lo[k] = insts[i].wlo[k];
            boxes[i].hi[k] = insts[i].whi[k];
        }
    std::vector<uint32_t> ids;  // instances with geometry (an empty mesh has no BLAS)
    for (uint32_t i = 0; i < n; i++)
        if (insts[i].kind == PUPIL_SHAPE_SPHERE || insts[i].blas_root != kTraverseDone) ids.push_back(i);
    std::vector<Bvh4Node> nodes;
    uint32_t depth = 0, binned = 0;
    const int root = ids.empty() ? kTraverseDone
                                 : build_tlas_node(ids, 0, (uint32_t)ids.size(), boxes, nodes, 0u, depth, nullptr, &binned);
    if (nodes.size() > acc.tlas_cap) return -1;
    // a lane inside a BLAS holds the TLAS entries, the pending link + kReturnLink and the BLAS entries
    if (3u * depth + 2u + 3u * acc.blas_depth > (uint32_t)kTraceStackEntries) return -3;
    acc.tlas_depth = depth;
    if (!nodes.empty() &&
        hipMemcpyAsync(acc.nodes4, nodes.data(), sizeof(Bvh4Node) * nodes.size(), hipMemcpyHostToDevice, s) !=
            hipSuccess)
        return -1;
    acc.tlas_nodes = (uint32_t)nodes.size();
    acc.sah_splits = binned;
    acc.root_link4 = (uint32_t)root;
    return hipStreamSynchronize(s) == hipSuccess ? 0 : -1;
}

int build_two_level(const std::vector<TwoLevelShape> &shapes, const std::vector<uint32_t> &inst_shape,
                    std::vector<DevInstance> &insts, DevInstance *d_insts, const DevMaterial *d_mats,
                    uint32_t leaf_size, hipStream_t s, TwoLevelAccel &acc) {
    const auto t0 = std::chrono::steady_clock::now();
    acc = TwoLevelAccel{};
    const uint32_t n = (uint32_t)insts.size();
    const char *mode = std::getenv("PUPIL_TL_MODE");  // world (default) | object (A/B)
    acc.world = !(mode && std::strcmp(mode, "object") == 0);
    // braid 8 = TLAS over the nodes 8 levels below each instance root.  Config 5 with the GPU-built
    // TLAS and GPU refits (r03, profiles/r03_tlas_braid_ab.txt): braid 6 / 7 / 8 -> 434 / 445 / 415 ms
    // per step, instance update 1.4 / 1.5 / 1.9 ms, build 37 / 61 / 131-148 ms.  r04 (two alternating
    // rounds, profiles/r04_config5_braid_ab.txt): braid 8 / 10 / 11 / 12 -> 402 / 392-395 / 398-400 /
    // 397-398 ms per step, 37.1 / 35.6 / 36.5 / 36.5 node visits per ray, update 2.0 / 3.0 / 3.1 / 3.4 ms,
    // build 138 / 277-290 / 311-321 / 333-336 ms: braid 10 is the default
    if (const char *b = std::getenv("PUPIL_TL_BRAID")) acc.braid = (uint32_t)std::min(12, std::max(0, std::atoi(b)));
    // BLAS per mesh shape that some instance uses
    std::vector<uint8_t> used(shapes.size(), 0);
    std::vector<uint32_t> shape_of(n);
    for (uint32_t i = 0; i < n; i++) {
        shape_of[i] = insts[i].kind == PUPIL_SHAPE_SPHERE ? 0xFFFFFFFFu : inst_shape[i];
        if (shape_of[i] != 0xFFFFFFFFu) used[shape_of[i]] = 1;
    }
    std::vector<BvhBuildOutput> blas(shapes.size());
    // prim_base: a shape's first primitive (shading records, one per primitive); rec_base: its
    // first BLAS record slot (pt_scene.h kRecF4: leaves on even slots, holes between)
    std::vector<uint32_t> node_base(shapes.size(), 0), prim_base(shapes.size(), 0), rec_base(shapes.size(), 0);
    acc.tlas_cap = std::max(1u, n);
    uint32_t total_nodes = acc.tlas_cap, total_prims = 0, total_slots = 0, max_faces = 1;
    uint64_t nodes64 = acc.tlas_cap, slots64 = 0;  // the same sums without wrap-around
    for (size_t k = 0; k < shapes.size(); k++)
        if (used[k]) max_faces = std::max(max_faces, shapes[k].num_faces);
    uint32_t *zeros = nullptr;
    DevInstance *d_ident = nullptr;
    int rc = 0;
    if (hipMalloc((void **)&zeros, sizeof(uint32_t) * max_faces) != hipSuccess ||
        hipMemset(zeros, 0, sizeof(uint32_t) * max_faces) != hipSuccess ||
        hipMalloc((void **)&d_ident, sizeof(DevInstance)) != hipSuccess)
        rc = -1;
    for (size_t k = 0; k < shapes.size() && !rc; k++) {
        if (!used[k]) continue;
        const TwoLevelShape &sh = shapes[k];
        DevInstance id{};
        const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        std::memcpy(id.to_world, I, sizeof(I));
        std::memcpy(id.to_object, I, sizeof(I));
        id.kind = PUPIL_SHAPE_MESH;
        id.emitter_offset = -1;
        id.positions = sh.positions;
        id.normals = sh.normals;
        id.texcoords = sh.texcoords;
        id.indices = sh.indices;
        if (hipMemcpy(d_ident, &id, sizeof(id), hipMemcpyHostToDevice) != hipSuccess) {
            rc = -1;
            break;
        }
        BvhBuildInput bin{sh.num_faces, zeros, d_ident, d_mats, 1u};
        double ms = 0.0;
        if (sh.num_faces) {
            const int brc = build_bvh_bounded(bin, blas[k], leaf_size, s, &ms, 2u);
            if (brc != 0) {
                rc = brc == -3 ? -3 : -1;
                break;
            }
            acc.blas_depth = std::max(acc.blas_depth, blas[k].depth4);
        }
        node_base[k] = total_nodes;
        prim_base[k] = total_prims;
        rec_base[k] = total_slots;
        if (blas[k].level_start.size() < 2) acc.world = false;  // no level order (A/B node layouts): object mode
        total_nodes += blas[k].num_nodes4;
        total_prims += sh.num_faces;
        total_slots += sh.num_faces ? blas[k].num_records : 0u;
        nodes64 += blas[k].num_nodes4;
        slots64 += sh.num_faces ? blas[k].num_records : 0u;
    }
    // object-space BLAS leaf links name record slots in 28 bits, object-mode TLAS leaves an
    // instance id (accel_limits.h); both structures need the object BLASes
    if (!rc && (nodes64 > kMaxNodes4 || two_level_fit(slots64, 0, 0, n, false) == TwoLevelFit::None)) {
        std::fprintf(stderr, "[pupil] two-level: %llu BLAS record slots / %llu nodes / %u instances exceed the link limits\n",
                     (unsigned long long)slots64, (unsigned long long)nodes64, n);
        rc = -4;
    }
    if (!rc && (hipMalloc((void **)&acc.nodes4, sizeof(Bvh4Node) * total_nodes) != hipSuccess ||
                hipMalloc((void **)&acc.prims, sizeof(float4) * kRecF4 * (size_t)std::max(1u, total_slots)) != hipSuccess ||
                hipMalloc((void **)&acc.attrs, sizeof(float4) * kAttrStride * (size_t)std::max(1u, total_prims)) !=
                    hipSuccess ||
                hipMalloc((void **)&acc.d_boxes, sizeof(uint32_t) * 6 * (size_t)n) != hipSuccess ||
                hipMalloc((void **)&acc.d_list, sizeof(uint32_t) * n) != hipSuccess ||
                hipMalloc((void **)&acc.d_verts, sizeof(uint32_t) * n) != hipSuccess))
        rc = -1;
    for (size_t k = 0; k < shapes.size() && !rc; k++) {
        if (!used[k]) continue;
        const BvhBuildOutput &b = blas[k];
        const uint32_t nf = shapes[k].num_faces;
        if (nf == 0) continue;
        if ((b.num_nodes4 && hipMemcpyAsync(acc.nodes4 + node_base[k], b.nodes4, sizeof(Bvh4Node) * b.num_nodes4,
                                            hipMemcpyDeviceToDevice, s) != hipSuccess) ||
            hipMemcpyAsync(acc.prims + kRecF4 * (size_t)rec_base[k], b.prims, sizeof(float4) * kRecF4 * (size_t)b.num_records,
                           hipMemcpyDeviceToDevice, s) != hipSuccess ||
            hipMemcpyAsync(acc.attrs + kAttrStride * (size_t)prim_base[k], b.attrs, sizeof(float4) * kAttrStride * nf,
                           hipMemcpyDeviceToDevice, s) != hipSuccess) {
            rc = -1;
            break;
        }
        if (b.num_nodes4)
            hipLaunchKernelGGL(k_relink, dim3((b.num_nodes4 + kBlock - 1) / kBlock), dim3(kBlock), 0, s, acc.nodes4,
                               b.num_nodes4, node_base[k], rec_base[k]);
    }
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = -1;
    for (auto &b : blas) free_lbvh(b);
    if (zeros) (void)hipFree(zeros);
    if (d_ident) (void)hipFree(d_ident);
    if (rc) {
        free_two_level(acc);
        return rc;
    }
    acc.num_nodes4 = total_nodes;
    acc.num_prims = total_prims;
    // per instance: BLAS root / record base / margin / world-record base, then the
    // world records, the world boxes and the TLAS
    std::vector<uint32_t> verts(n, 0), faces(n, 0), all(n);
    uint64_t wbase = 0, spheres = 0;
    for (uint32_t i = 0; i < n; i++) spheres += insts[i].kind == PUPIL_SHAPE_SPHERE ? 1u : 0u;
    // world mode: the TLAS first, at most one node per entry; an instance contributes at
    // most min(4^braid, 4 x its BLAS nodes + 1) entries (the links `braid` levels below its
    // root), a sphere one (64-bit sum: many instances must not wrap the reserve)
    if (acc.world) {
        uint64_t width = 1;
        for (uint32_t l = 0; l < acc.braid; l++) width *= 4;
        uint64_t cap = 0;
        for (uint32_t i = 0; i < n; i++)
            cap += shape_of[i] == 0xFFFFFFFFu ? 1u : std::min<uint64_t>(width, 4ull * blas[shape_of[i]].num_nodes4 + 1u);
        if (cap > kMaxNodes4) {
            std::fprintf(stderr, "[pupil] two-level: %llu braided TLAS entries exceed the node limit, object mode\n",
                         (unsigned long long)cap);
            acc.world = false;
        } else {
            acc.tlas_cap = (uint32_t)std::max<uint64_t>(1u, cap);
        }
    }
    uint64_t wnodes = acc.tlas_cap;
    for (uint32_t i = 0; i < n; i++) {
        all[i] = i;
        DevInstance &d = insts[i];
        if (shape_of[i] == 0xFFFFFFFFu) {
            d.blas_root = kTraverseDone;
            d.attr_base = 0;
            d.margin[0] = d.margin[1] = 0.f;
            continue;
        }
        const uint32_t k = shape_of[i];
        d.blas_root = shapes[k].num_faces ? rebase_link((int)blas[k].root_link4, node_base[k], rec_base[k])
                                          : kTraverseDone;
        d.attr_base = prim_base[k];
        d.rec_base = rec_base[k];
        d.wrec_delta = (int32_t)((int64_t)wbase - (int64_t)rec_base[k]);
        const uint32_t slots = shapes[k].num_faces ? blas[k].num_records : 0u;
        wbase += slots;
        d.obj_nbase = node_base[k];
        d.obj_ncount = blas[k].num_nodes4;
        d.wnode_base = (uint32_t)wnodes;
        wnodes += blas[k].num_nodes4;
        verts[i] = shapes[k].num_vertices;
        faces[i] = slots;  // the BLAS record slots k_world_records copies
        instance_margin(d, shapes[k].vmax);
    }
    // world-mode leaf links name world record slots (the meshes' copies, then one 2-slot leaf
    // per sphere) in 28 bits: beyond that the object-space structure serves the scene
    // PUPIL_DEBUG_TL_FALLBACK (tests only): force the fallback below (1) or the node-limit one (2)
    const int force_fallback = [] {
        const char *e = std::getenv("PUPIL_DEBUG_TL_FALLBACK");
        return e ? std::atoi(e) : 0;
    }();
    // object mode keeps only the per-instance TLAS slots [0, max(1, n)) before its BLASes
    // (node_base): the braided reserve sized above must go with world mode
    auto to_object_mode = [&]() {
        acc.world = false;
        acc.tlas_cap = std::max(1u, n);
    };
    if (acc.world && (force_fallback == 1 || two_level_fit(slots64, wbase, spheres, n, true) != TwoLevelFit::World)) {
        std::fprintf(stderr, "[pupil] two-level: %llu world record slots + %llu spheres exceed the 28-bit leaf links, object mode\n",
                     (unsigned long long)wbase, (unsigned long long)spheres);
        to_object_mode();
    }
    int trc = 0;
    if (wbase >= (1ull << 31) ||
        hipMalloc((void **)&acc.wprims, sizeof(float4) * kRecF4 * (size_t)std::max<uint64_t>(1, wbase)) != hipSuccess ||
        hipMalloc((void **)&acc.d_faces, sizeof(uint32_t) * n) != hipSuccess ||
        hipMemcpy(acc.d_faces, faces.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess) {
        free_two_level(acc);
        return -1;
    }
    acc.num_wprims = (uint32_t)wbase;
    // the traversal addresses nodes by 32-bit offsets (kMaxNodes4): instance copies beyond
    // that take the object-space structure, whose BLASes are shared
    if (acc.world && (force_fallback == 2 || wnodes > kMaxNodes4)) {
        std::fprintf(stderr, "[pupil] two-level: %llu world BLAS copy nodes exceed the node limit, object mode\n",
                     (unsigned long long)wnodes);
        to_object_mode();
    }
    if (acc.world) {  // world BLAS copies + sphere records appended to the world records
        acc.entries.assign(n, {});
        acc.inst_shape = shape_of;
        acc.shape_levels.assign(shapes.size(), {});
        for (size_t k = 0; k < shapes.size(); k++) acc.shape_levels[k] = blas[k].level_start;
        // one leaf (2 slots: the record, then a hole) per sphere
        const float4 hole = make_float4(qfloat(kRecHole), qfloat(kRecHole), qfloat(kRecHole), qfloat(kRecHole));
        std::vector<float4> sph(2 * kRecF4 * spheres, hole);
        uint32_t si = 0;
        for (uint32_t i = 0; i < n; i++) {
            if (insts[i].kind != PUPIL_SHAPE_SPHERE) continue;
            float4 *r = sph.data() + 2 * kRecF4 * si;
            r[0] = make_float4(0.f, 0.f, 0.f, qfloat(insts[i].prim_offset | kPrimSphereBit));
            r[1] = make_float4(0.f, 0.f, 0.f, qfloat(i));
            r[2] = make_float4(0.f, 0.f, 0.f, qfloat(insts[i].bin));
            si++;
        }
        float4 *grown = nullptr;
        if (wnodes >= (1ull << 31) ||
            hipMalloc((void **)&acc.wnodes, sizeof(Bvh4Node) * (size_t)wnodes) != hipSuccess ||
            hipMalloc((void **)&acc.d_wbox, sizeof(float) * 6 * (size_t)wnodes) != hipSuccess ||
            hipMalloc((void **)&acc.d_tlas_order, sizeof(uint32_t) * (size_t)std::max(1u, acc.tlas_cap)) != hipSuccess ||
            hipMalloc((void **)&grown, sizeof(float4) * kRecF4 * (size_t)std::max<uint64_t>(1, wbase + 2 * spheres)) !=
                hipSuccess ||
            (spheres && hipMemcpy(grown + kRecF4 * wbase, sph.data(), sizeof(float4) * sph.size(), hipMemcpyHostToDevice) !=
                            hipSuccess)) {
            if (grown) (void)hipFree(grown);
            free_two_level(acc);
            return -1;
        }
        (void)hipFree(acc.wprims);
        acc.wprims = grown;
        acc.num_wnodes = (uint32_t)wnodes;
    }
    if (hipMemcpy(acc.d_verts, verts.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_insts, insts.data(), sizeof(DevInstance) * n, hipMemcpyHostToDevice) != hipSuccess ||
        (trc = rebuild_tlas(acc, insts, d_insts, all, s)) != 0) {
        free_two_level(acc);
        return trc == -3 ? -3 : -1;
    }
    acc.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return 0;
}

void free_two_level(TwoLevelAccel &acc) {
    void *p[] = {acc.nodes4, acc.prims, acc.attrs, acc.d_boxes, acc.d_list, acc.d_verts, acc.wprims, acc.d_faces,
                 acc.wnodes, acc.d_wbox, acc.d_tlas_order};
    for (void *x : p)
        if (x) (void)hipFree(x);
    acc = TwoLevelAccel{};
}

}  // namespace pupil
