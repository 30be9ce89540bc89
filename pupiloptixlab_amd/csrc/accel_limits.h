// accel_limits.h — index limits of the BVH4 leaf-link encoding (pt_scene.h make_leaf:
// ~((first << 3) | (count - 1)), negative only while first < 2^28), as plain host code
// with no HIP dependency so a CPU test checks them (tests/test_limits.py).
#pragma once

#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define PL_HD __host__ __device__ __forceinline__
#else
#define PL_HD inline
#endif

namespace pupil {

// Child link encoding of a BVH4 node: link >= 0 -> internal node index; link < 0 -> leaf,
// ~link = (first << 3) | (count - 1), count in [1, 8] (first = record slot, or the instance
// of a two-level TLAS leaf).
constexpr int kLeafMax = 8;
PL_HD int make_leaf(uint32_t first, uint32_t count) { return ~(int)((first << 3) | (count - 1)); }
PL_HD uint32_t leaf_first(int link) { return ((uint32_t)~link) >> 3; }
PL_HD uint32_t leaf_count(int link) { return (((uint32_t)~link) & 7u) + 1u; }

// first record slot (or TLAS instance id) a leaf link can name
constexpr uint64_t kMaxLeafFirst = 1ull << 28;

// Which two-level structure (accel_two_level.hip) a scene fits:
//   object_slots  record slots of all object-space BLASes (object-mode BLAS leaf links)
//   world_slots   world-space record slots of every mesh instance (world-mode BLAS copies)
//   spheres       built-in sphere instances (world mode: one 2-slot leaf each after the meshes)
//   instances     instances (object-mode TLAS leaves name an instance id)
// The object-space BLASes exist in both modes (the world copies take their topology), so
// past their limit the scene is unsupported; past the world limit it falls back to object mode.
enum class TwoLevelFit { World, Object, None };
inline TwoLevelFit two_level_fit(uint64_t object_slots, uint64_t world_slots, uint64_t spheres, uint64_t instances,
                                 bool want_world) {
    if (object_slots >= kMaxLeafFirst || instances >= kMaxLeafFirst) return TwoLevelFit::None;
    if (want_world && world_slots + 2 * spheres < kMaxLeafFirst) return TwoLevelFit::World;
    return TwoLevelFit::Object;
}

}  // namespace pupil
