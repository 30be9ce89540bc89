// pt_scene.h — device-resident scene layout of the MI355X path tracer.
//
// Everything the wavefront kernels read lives in one POD struct (DeviceScene)
// passed by value as a kernel argument.  Layout choices (HBM-first):
//   * BVH nodes: 64 B quantized 4-wide nodes (Bvh4Node), 64 B aligned so one
//     node = one half L2 line; leaves index a Morton-ordered array of 48 B
//     primitive records (3 x float4: world-space triangle vertices; the first w
//     carries the global primitive id).
//   * Shading data stays in object space and is gathered only on hits
//     (reference: geometry.h:48-96 interpolates object-space attributes then
//     transforms), so the traversal working set is nodes + prim records only.
#pragma once

#include "../../include/pupil_pt.h"
#include "accel_limits.h"
#include "pt_math.h"

namespace pupil {

// cuda::Texture (framework/cuda/texture.h:10-57)
struct DevTexture {
    uint32_t type;  // PUPIL_TEX_*
    uint32_t width, height;
    uint32_t filter;  // bitmap: 0 point, 1 linear
    float c0[3];
    float c1[3];
    float r0[4];  // transform row 0
    float r1[4];  // transform row 1
    const float4 *data;  // bitmap texels (device)
};

// Flattened optix::material::Material (render/material/optix_material.h:87-98)
// with the host precompute of optix_material.cpp:87-119 already applied.
struct DevMaterial {
    uint32_t type;
    uint32_t twosided;
    uint32_t nonlinear;
    float eta;                       // int_ior / ext_ior
    float int_fdr;                   // plastic: DiffuseReflectance(1/eta)
    float specular_sampling_weight;  // plastic
    float pad[2];
    DevTexture tex[4];
};

// optix::Emitter (render/emitter.h:13-24)
struct DevEmitter {
    uint32_t type;
    float select_probability;
    float area;
    float radius;
    DevTexture radiance;
    vec3 pos[3];
    vec3 nrm[3];
    vec2 tex[3];
    vec3 center;
    vec3 color;
    // env map
    float scale;
    float normalization;
    uint32_t map_w, map_h;
    float to_world[9];
    float to_local[9];
    const float *row_cdf;     // map_h + 1
    const float *col_cdf;     // (map_w + 1) * map_h
    const float *row_weight;  // map_h
};

struct DevInstance {
    float to_world[12];
    float to_object[12];
    uint32_t kind;  // PUPIL_SHAPE_*
    uint32_t material;
    uint32_t prim_offset;  // first global primitive id
    int32_t emitter_offset;
    uint32_t flip_normals;
    uint32_t flip_tex_coords;
    // object-space mesh attributes (null for spheres / missing)
    const float *positions;
    const float *normals;
    const float *texcoords;
    const uint32_t *indices;
    // two-level acceleration (DeviceScene::two_level; see accel_two_level.hip)
    int32_t blas_root;    // link of the shape's BLAS root in the combined BVH4 node array
    uint32_t attr_base;   // first shading record of the shape's BLAS primitives (local order)
    uint32_t bin;         // material bin of the instance's hits (0 miss, 1..7 EMatType, 8 unknown)
    float margin[2];      // object-space box margin: margin[0] * (|o| + t |d|) + margin[1]
    float wlo[3], whi[3];  // world box of the instance's world-space primitives
    int32_t wrec_delta;    // world-space record of BLAS record slot i: wprims[kRecF4 * (i + wrec_delta)]
    uint32_t rec_base;     // the shape's first BLAS record slot (two-level; attr_base counts primitives)
    // world-space copy of the shape's BLAS (two-level "world" mode): object nodes
    // [obj_nbase, obj_nbase + obj_ncount) -> world nodes from wnode_base
    uint32_t obj_nbase, obj_ncount, wnode_base;
    float vmax;  // largest |object-space vertex coordinate| of the shape (margins)
};

// 4-wide node with 8-bit quantized child boxes: 64 B = one half L2 line holds
// what four 64 B BVH2 nodes spread over two levels.  Child k's box is
// origin + q * s per axis, s a power of two stored as a float (r03: the traversal
// reads it directly instead of decoding an exponent byte, 6 VALU per node visit);
// the builder rounds q outward and verifies the decoded float box contains the
// exact child box (conservative culling).
struct alignas(64) Bvh4Node {
    float ox, oy, oz;
    float sx;           // scale of the x planes (2^(e-127))
    int32_t child[4];   // links (see below); kEmptyLink for unused slots
    uint32_t qlo_x, qlo_y, qlo_z;  // byte k = child k
    uint32_t qhi_x, qhi_y, qhi_z;
    float sy, sz;       // scales of the y and z planes
};
constexpr int kEmptyLink = 0x7FFFFFFF;
// BVH4 nodes the flat traversal keeps in LDS: the root, its 4 children and the first 11 of
// the third level of the breadth-first layout; 1 KB per 128-lane block keeps 14 blocks (7
// waves per SIMD) within the CU's 160 KB of LDS in 512-B allocation granules
constexpr uint32_t kTopNodes = 16;
// Largest BVH4 node array: the traversal addresses nodes by 32-bit byte offsets.
constexpr uint64_t kMaxNodes4 = 1ull << 26;
// Traversal terminator (stack bottom); also the root link of an empty scene.
// Inner-node links are < kTraverseDone, leaf links are negative.
constexpr int kTraverseDone = 0x76543210;
// Two-level traversal: stack marker below a BLAS's entries; popping it returns
// the lane to the TLAS (a positive link above kTraverseDone, never a node index).
constexpr int kReturnLink = 0x7654321F;

// Child link encoding (make_leaf / leaf_first / leaf_count) and its 28-bit limit: accel_limits.h.

constexpr uint32_t kPrimSphereBit = 0x80000000u;
// Primitive records: 4 float4 = 64 B per record slot (v0 | global id + sphere bit, v1 |
// instance, v2 | material bin, unused), and every leaf starts on an even slot, i.e. on a
// 128-B L2 line: a two-primitive leaf is one line instead of 96 B straddling up to two.  A
// leaf of c primitives takes 2 ceil(c / 2) slots; unused slots are holes (all bits set).
constexpr uint32_t kRecF4 = 4;
constexpr uint32_t kRecHole = 0xFFFFFFFFu;  // a.w and b.w of a hole slot
PT_HD uint32_t leaf_slots(uint32_t count) { return (count + 1u) & ~1u; }
constexpr uint32_t kAttrStride = 8;  // float4 per shading record (one 128-B line)

struct Camera {
    float s2c[16];  // sample_to_camera, row-major (mat4x4 r0..r3)
    float c2w[16];  // camera_to_world
};

struct DeviceScene {
    const Bvh4Node *nodes4;
    const float4 *prims;  // kRecF4 float4 per record slot, leaf order (holes between leaves)
    const float4 *attrs;  // kAttrStride float4 per primitive, same order (hit reconstruction)
    uint32_t num_prims;
    uint32_t root_link4;  // link of the root (internal 0 or a leaf), kTraverseDone = empty
    uint32_t trace_refill;  // BVH4 kernels: refill a wave's idle lanes once this many are idle
    uint32_t num_cus;       // compute units of the device (persistent grid size)
    uint32_t trace_node_min;  // BVH4 kernels: node phase ends when fewer lanes need a node
    // nodes [0, top_nodes) are copied into each traversal block's LDS at launch and read from
    // there (the collapse emits the BVH4 breadth first: the root and the levels below it,
    // which every ray visits); <= kTopNodes, 0 = off (refresh_node_bound)
    uint32_t top_nodes;
    // per axis, max over every BVH4 node of |o| + 512 s (launch_node_bound after each build
    // and refit): the slab test's rounding bound is then one value per ray (pt_traverse.h
    // slab_error) instead of one per node visit
    float node_bound[3];
    // every instance has this material bin (1..8; 0 = several): shading then derives a
    // path's bin from its hit record and the persistent traversal writes no bin byte
    uint32_t single_bin;
    uint32_t tl_world;        // two-level "world" mode: nodes4 = braided TLAS + world-space BLAS copies,
                              // prims = flat-format world records; traversed by the flat kernels
    uint32_t two_level;       // 1: nodes4 = TLAS over instances + object-space BLAS per shape;
                              //    prims/attrs = BLAS records, hit index = global primitive id
    const float4 *wprims;       // two-level: per-instance world-space triangle records (see accel_two_level.hip)
    const uint32_t *prim_inst;  // global prim id -> instance (the builders; 4 B per primitive)
    // global prim id -> instance for the shading (inst_of_prim): inst_first[i] = instance i's
    // first global primitive id (num_instances + 1 entries, the last = num_prims), and a guide
    // table over prim ids, inst_guide[k] = the instance holding prim min(k << inst_guide_shift,
    // num_prims - 1): a few kB that stay in the L1 / L2, where prim_inst is 40 MB at config 5
    const uint32_t *inst_first;
    const uint32_t *inst_guide;
    uint32_t inst_guide_shift;
    const DevInstance *instances;
    const DevMaterial *materials;
    const DevEmitter *areas;
    const float *area_cdf;  // sequential CDF of select_probability (emitter.h:110-120)
    // guide table over area_cdf (Chen & Asau's indexed search): area_guide[k] = first i
    // with area_cdf[i] >= k / 2^guide_bits, k = 0..2^guide_bits, so the pick for p lies in
    // [guide[k], guide[k+1]] with k = floor(p 2^guide_bits); null = plain binary search
    const uint32_t *area_guide;
    uint32_t guide_bits;
    uint32_t num_areas;
    uint32_t has_env;
    const DevEmitter *env;
    Camera camera;
};

}  // namespace pupil
