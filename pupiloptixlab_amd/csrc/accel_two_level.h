// accel_two_level.h — two-level acceleration structure (TLAS over instances,
// one object-space BLAS per mesh shape); see accel_two_level.hip.
#pragma once

#include <array>
#include <utility>
#include <vector>

#include "pt_kernels.h"

namespace pupil {

struct TwoLevelShape {  // one mesh shape (device arrays, object space)
    uint32_t num_faces, num_vertices;
    const float *positions, *normals, *texcoords;
    const uint32_t *indices;
    float vmax;  // largest |coordinate| of its vertices (host-computed; for the box margin)
};

struct TwoLevelAccel {
    Bvh4Node *nodes4 = nullptr;  // [0, tlas_cap) TLAS, then the rebased BLASes
    float4 *prims = nullptr;     // 3 float4 per BLAS primitive, object space, BLAS leaf order; w of [0] = local id
    float4 *attrs = nullptr;     // kAttrStride float4 per BLAS primitive, the mesh's own primitive order
    float4 *wprims = nullptr;    // 3 float4 per (mesh instance, BLAS primitive): world vertices fl(to_world * v),
                                 // instance-major, BLAS leaf order; w of [0] = global primitive id
    uint32_t num_wprims = 0;
    float *d_boxes = nullptr;    // 6 floats per instance: world box
    uint32_t *d_list = nullptr, *d_verts = nullptr;  // scratch: instance list, vertices per instance
    uint32_t *d_faces = nullptr;                     // BLAS primitives per instance (world records)
    uint32_t tlas_cap = 0, tlas_nodes = 0, num_nodes4 = 0, num_prims = 0;
    uint32_t tlas_depth = 0, blas_depth = 0;  // BVH4 levels (deepest BLAS); see kTraceStackEntries
    uint32_t sah_splits = 0;  // TLAS nodes of the last build placed by an SAH (GPU collapse, or host binned splits)
    // "world" mode (PUPIL_TL_MODE, default): every mesh instance gets a world-space copy of
    // its shape's BLAS (child boxes transformed and re-quantised conservatively) and the
    // TLAS is built over the nodes `braid` levels below each instance root, so the whole
    // structure is one BVH4 the flat traversal kernels walk (no ray transform, no
    // return markers, the flat kernel's occupancy).  HBM pays one BLAS copy per instance.
    bool world = false;
    uint32_t braid = 10;  // PUPIL_TL_BRAID
    Bvh4Node *wnodes = nullptr;  // [0, tlas_cap) TLAS, then the per-instance world BLAS copies
    float *d_wbox = nullptr;     // world box of every copied node (6 floats)
    uint32_t num_wnodes = 0;
    std::vector<std::vector<std::pair<int, std::array<float, 6>>>> entries;  // per instance: TLAS entries
    std::vector<uint32_t> inst_shape;                  // shape of each instance (0xFFFFFFFF: sphere)
    // world-mode TLAS refits (GPU, one launch per level, deepest first): the TLAS node ids
    // ordered by level from the deepest (d_tlas_order) and where each level starts in it
    uint32_t *d_tlas_order = nullptr;
    std::vector<uint32_t> tlas_level_start;
    std::vector<std::vector<uint32_t>> shape_levels;   // per shape: BVH4 level starts of its BLAS (+ end)
    uint32_t root_link4 = (uint32_t)kTraverseDone;
    double build_ms = 0.0;
};

// Link of a node or leaf of one BLAS after it is copied to node_base / prim_base.
PT_HD int rebase_link(int link, uint32_t node_base, uint32_t prim_base) {
    if (link == kEmptyLink || link == kTraverseDone) return link;
    if (link >= 0) return link + (int)node_base;
    return make_leaf(leaf_first(link) + prim_base, leaf_count(link));
}

// Builds the BLASes, fills the two-level fields of every instance (host copy
// `insts`, uploaded to d_insts), their world boxes and the TLAS.
// inst_shape[i] = shape index of instance i (ignored for spheres).  Returns 0, -1 on a HIP
// error, -3 when the TLAS + BLAS depth exceeds the traversal stacks, -4 when the BLAS record
// slots or instances exceed the 28-bit leaf links (accel_limits.h; past the world-mode limit
// alone the build falls back to object mode instead).
int build_two_level(const std::vector<TwoLevelShape> &shapes, const std::vector<uint32_t> &inst_shape,
                    std::vector<DevInstance> &insts, DevInstance *d_insts, const DevMaterial *d_mats,
                    uint32_t leaf_size, hipStream_t s, TwoLevelAccel &acc);
// Recomputes the world boxes of the `changed` instances (transforms already in
// insts / d_insts) and rebuilds the TLAS.  -3: the TLAS + BLAS depth exceeds the
// traversal stacks (kTraceStackEntries).
// refit (world mode): keep the TLAS topology and refit its boxes instead of rebuilding.
int rebuild_tlas(TwoLevelAccel &acc, std::vector<DevInstance> &insts, DevInstance *d_insts,
                 const std::vector<uint32_t> &changed, hipStream_t s, bool refit = false);
void free_two_level(TwoLevelAccel &acc);
// BLAS box margins of an instance after its transform changed (uses its stored vmax)
void refresh_instance_margins(DevInstance &d);
// nodes of the traversed structure (object mode: TLAS + shared BLASes; world mode: TLAS + copies)
inline uint64_t two_level_nodes(const TwoLevelAccel &a) {
    return a.tlas_nodes + ((a.world ? a.num_wnodes : a.num_nodes4) - a.tlas_cap);
}

}  // namespace pupil
