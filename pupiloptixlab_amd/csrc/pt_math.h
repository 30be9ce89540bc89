// pt_math.h — small vector algebra shared by the HIP kernels and the host side
// of the engine.  Operation order follows the reference's vec_math.h exactly
// (framework/cuda/vec_math.h: operator/ = multiply by reciprocal :425-436,
// normalize = v * (1/sqrt(dot)) :477-479, lerp = a + t*(b-a) :439-441), so the
// engine's float results are reproducible by the CPU oracle.  Build with
// -ffp-contract=off (see Makefile): no FMA contraction anywhere.
#pragma once

#include <stdint.h>

#include "../../include/pupil_detmath.h"

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define PT_HD __host__ __device__ __forceinline__
#define PT_D __device__ __forceinline__
#else
#include <math.h>
#define PT_HD inline
#define PT_D inline
#endif

namespace pupil {

constexpr float kEps = 0.000001f;       // optix/util.h:8
constexpr float kMaxDistance = 1e16f;   // optix/util.h:9
constexpr float kPi = 3.14159265358979323846f;
constexpr float k1OverPi = 0.318309886183790671538f;

struct vec2 {
    float x, y;
};
struct vec3 {
    float x, y, z;
};
struct vec4 {
    float x, y, z, w;
};

PT_HD vec2 v2(float x, float y) { return vec2{x, y}; }
PT_HD vec3 v3(float x, float y, float z) { return vec3{x, y, z}; }
PT_HD vec3 v3(float s) { return vec3{s, s, s}; }
PT_HD vec4 v4(float x, float y, float z, float w) { return vec4{x, y, z, w}; }

PT_HD vec3 operator+(vec3 a, vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD vec3 operator-(vec3 a, vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD vec3 operator-(vec3 a) { return v3(-a.x, -a.y, -a.z); }
PT_HD vec3 operator*(vec3 a, vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD vec3 operator*(vec3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
PT_HD vec3 operator*(float s, vec3 a) { return v3(s * a.x, s * a.y, s * a.z); }
PT_HD vec3 operator/(vec3 a, float s) {
    float inv = 1.0f / s;
    return a * inv;
}
PT_HD vec3 operator/(vec3 a, vec3 b) { return v3(a.x / b.x, a.y / b.y, a.z / b.z); }
PT_HD vec3 operator-(float s, vec3 a) { return v3(s - a.x, s - a.y, s - a.z); }
PT_HD vec2 operator+(vec2 a, vec2 b) { return v2(a.x + b.x, a.y + b.y); }
PT_HD vec2 operator*(vec2 a, float s) { return v2(a.x * s, a.y * s); }
PT_HD vec2 operator*(float s, vec2 a) { return v2(s * a.x, s * a.y); }

PT_HD float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD float dot(vec4 a, vec4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
PT_HD vec3 cross(vec3 a, vec3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
PT_HD float length(vec3 v) { return sqrtf(dot(v, v)); }
PT_HD vec3 normalize(vec3 v) {
    float inv_len = 1.0f / sqrtf(dot(v, v));
    return v * inv_len;
}
PT_HD vec4 normalize(vec4 v) {
    float inv_len = 1.0f / sqrtf(dot(v, v));
    return v4(v.x * inv_len, v.y * inv_len, v.z * inv_len, v.w * inv_len);
}
PT_HD vec3 lerp(vec3 a, vec3 b, float t) { return a + t * (b - a); }
PT_HD float fabs_(float v) { return __builtin_fabsf(v); }  // IEEE abs (clears the sign of -0 too)
PT_HD float fmax_(float a, float b) { return a > b ? a : b; }
PT_HD float fmin_(float a, float b) { return a < b ? a : b; }

// optix/util.h:169-179
PT_HD bool is_zero(float v) { return fabs_(v) < kEps; }
PT_HD bool is_zero(vec3 v) { return fabs_(v.x) < kEps && fabs_(v.y) < kEps && fabs_(v.z) < kEps; }
// optix/util.h:165-167
PT_HD float mis_weight(float x, float y) { return x / (x + y); }
// optix/util.h:161-163
PT_HD float luminance(vec3 c) { return 0.2126f * c.x + 0.7152f * c.y + 0.0722f * c.z; }

// Row-major 3x4 affine transform (the OptixInstance transform layout).
struct xform34 {
    float m[12];
};
PT_HD vec3 xform_point(const float *m, vec3 p) {
    return v3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
              m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
PT_HD vec3 xform_vector(const float *m, vec3 v) {
    return v3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
              m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
// optixTransformNormalFromObjectToWorldSpace: n_w = (M^-1)^T n, with M^-1 = to_object
PT_HD vec3 xform_normal(const float *inv, vec3 n) {
    return v3(inv[0] * n.x + inv[4] * n.y + inv[8] * n.z, inv[1] * n.x + inv[5] * n.y + inv[9] * n.z,
              inv[2] * n.x + inv[6] * n.y + inv[10] * n.z);
}

}  // namespace pupil
