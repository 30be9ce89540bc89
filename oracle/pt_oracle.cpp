// pt_oracle.cpp — CPU ORACLE (test infrastructure only).
//
// A scalar C++ restatement of the reference path tracer, used by tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker and
// CPU baseline.  Nothing in pupiloptixlab_amd/ links, loads or calls it.
//
// PARITY STATUS: unpinned against the reference's own outputs.  The
// reference (OptiX 7.5 + CUDA + Windows/D3D12, empty submodules) cannot be
// built or run in this image and ships no tests, golden images or known-answer
// vectors.  This restatement is pinned instead by
// independent known-answer tests (tests/test_oracle_kat.py: a pure-Python
// restatement of cuda::Random, Fresnel/GGX identities, white-furnace and
// energy checks, brute-force vs BVH hits) and by committed fixtures it
// generated (tests/golden/, tests/golden/make_golden.py).
//
// It follows, line by line:
//   __raygen__main / __miss__* / __closesthit__*   example/path_tracer/main.cu:36-233
//   cuda::Random                                   framework/cuda/random.h:14-40
//   optix util (sampling, ONB, MIS, IsZero)        framework/optix/util.h:8-183
//   Geometry::GetHitLocalGeometry                  framework/render/geometry.h:48-96
//   cuda::Texture::Sample                          framework/cuda/texture.h:33-57
//   fresnel / ggx                                  framework/render/material/{fresnel,ggx}.h
//   the seven BSDFs                                framework/render/material/bsdf/*.h
//   Material::LoadMaterial host precompute         framework/render/material/optix_material.cpp:39-132
//   Emitter / EmitterGroup / Tri/Sphere/Env        framework/render/emitter.h, emitter/*.h
// The transcendental functions come from include/pupil_detmath.h (the same
// deterministic libm the engine uses), and every expression keeps the
// reference's evaluation order, so a path's radiance is reproducible bit for
// bit.  Ray queries use this file's own SAH BVH; closest hits are resolved by
// (t, primitive id) so the result does not depend on the BVH.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/pupil_detmath.h"
#ifdef ORACLE_SYSTEM_LIBM
// Test build only (tests/test_detmath.py): the host's libm instead of the shared
// deterministic one, to show the choice of libm does not bias the image.
namespace oracle_syslibm {
inline float dm_sin(float x) { return std::sin(x); }
inline float dm_cos(float x) { return std::cos(x); }
inline float dm_acos(float x) { return std::acos(x); }
inline float dm_atan2(float y, float x) { return std::atan2(y, x); }
}  // namespace oracle_syslibm
#define pupil_dm oracle_syslibm
#endif
#include "../include/pupil_pt.h"

namespace oracle {

// ------------------------------------------------------------------ vec_math.h
struct float2 {
    float x, y;
};
struct float3 {
    float x, y, z;
};
struct float4 {
    float x, y, z, w;
};
inline float2 make_float2(float x, float y) { return {x, y}; }
inline float3 make_float3(float x, float y, float z) { return {x, y, z}; }
inline float3 make_float3(float s) { return {s, s, s}; }
inline float4 make_float4(float x, float y, float z, float w) { return {x, y, z, w}; }
inline float3 operator+(const float3 &a, const float3 &b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float3 operator-(const float3 &a, const float3 &b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float3 operator-(const float3 &a) { return {-a.x, -a.y, -a.z}; }
inline float3 operator*(const float3 &a, const float3 &b) { return {a.x * b.x, a.y * b.y, a.z * b.z}; }
inline float3 operator*(const float3 &a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float3 operator*(float s, const float3 &a) { return {a.x * s, a.y * s, a.z * s}; }
inline float3 operator/(const float3 &a, float s) {
    float inv = 1.0f / s;
    return a * inv;
}
inline float3 operator/(const float3 &a, const float3 &b) { return {a.x / b.x, a.y / b.y, a.z / b.z}; }
inline float3 operator-(float s, const float3 &a) { return {s - a.x, s - a.y, s - a.z}; }
inline void operator+=(float3 &a, const float3 &b) { a = a + b; }
inline void operator*=(float3 &a, const float3 &b) { a = a * b; }
inline void operator*=(float3 &a, float s) { a = a * s; }
inline void operator/=(float3 &a, float s) {
    float inv = 1.0f / s;
    a *= inv;
}
inline float2 operator+(const float2 &a, const float2 &b) { return {a.x + b.x, a.y + b.y}; }
inline float2 operator*(const float2 &a, float s) { return {a.x * s, a.y * s}; }
inline float4 operator*(const float4 &a, float s) { return {a.x * s, a.y * s, a.z * s, a.w * s}; }
inline void operator/=(float4 &a, float s) {
    float inv = 1.0f / s;
    a = a * inv;
}
inline float dot(const float3 &a, const float3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float dot(const float4 &a, const float4 &b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
inline float3 cross(const float3 &a, const float3 &b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float length(const float3 &v) { return sqrtf(dot(v, v)); }
inline float3 normalize(const float3 &v) {
    float invLen = 1.0f / sqrtf(dot(v, v));
    return v * invLen;
}
inline float4 normalize(const float4 &v) {
    float invLen = 1.0f / sqrtf(dot(v, v));
    return v * invLen;
}
inline float3 lerp(const float3 &a, const float3 &b, float t) { return a + t * (b - a); }
inline float absf(float v) { return std::fabs(v); }

struct mat4x4 {
    float4 r0, r1, r2, r3;
};
inline float4 operator*(const mat4x4 &m, const float4 &v) {
    return make_float4(dot(m.r0, v), dot(m.r1, v), dot(m.r2, v), dot(m.r3, v));
}

const float M_PIf_ = 3.14159265358979323846f;
const float M_1_PIf_ = 0.318309886183790671538f;

// ------------------------------------------------------------------ cuda::Random
class Random {
    unsigned int m_seed = 0;

public:
    void Init(unsigned int N, unsigned int val0, unsigned int val1) {
        unsigned int v0 = val0;
        unsigned int v1 = val1;
        unsigned int s0 = 0;
        for (unsigned int n = 0; n < N; n++) {
            s0 += 0x9e3779b9;
            v0 += ((v1 << 4) + 0xa341316c) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4);
            v1 += ((v0 << 4) + 0xad90777d) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761e);
        }
        m_seed = v0;
    }
    unsigned int GetSeed() const { return m_seed; }
    float Next() {
        const unsigned int LCG_A = 1664525u;
        const unsigned int LCG_C = 1013904223u;
        m_seed = (LCG_A * m_seed + LCG_C);
        return static_cast<float>(m_seed & 0x00FFFFFF) / 0x01000000;
    }
    // make_float2(Next(), Next()) evaluated x first (nvcc order)
    float2 Next2() {
        const float x = Next();
        const float y = Next();
        return make_float2(x, y);
    }
};

// ------------------------------------------------------------------ optix/util.h
constexpr float EPS = 0.000001f;
constexpr float MAX_DISTANCE = 1e16f;
inline float3 UniformSampleTriangle(float u1, float u2) {
    const float sqrt_u1 = sqrtf(u1);
    return make_float3(1.f - sqrt_u1, sqrt_u1 * (1.f - u2), u2 * sqrt_u1);
}
inline float3 UniformSampleSphere(float u1, float u2) {
    const float z = 1.f - 2.f * u1;
    const float sin_theta = sqrtf(std::fmax(0.f, 1.f - z * z));
    const float phi = 2.f * M_PIf_ * u2;
    return make_float3(sin_theta * pupil_dm::dm_cos(phi), sin_theta * pupil_dm::dm_sin(phi), z);
}
inline float3 CosineSampleHemisphere(float u1, float u2) {
    float3 p{0.f, 0.f, 0.f};
    const float sin_theta = sqrtf(u1);
    const float phi = 2.0f * M_PIf_ * u2;
    p.x = sin_theta * pupil_dm::dm_cos(phi);
    p.y = sin_theta * pupil_dm::dm_sin(phi);
    p.z = sqrtf(std::fmax(0.f, 1.f - sin_theta * sin_theta));
    return p;
}
inline float CosineSampleHemispherePdf(float3 v) { return v.z > 0.f ? M_1_PIf_ * v.z : 0.f; }
inline float3 UniformSampleHemisphere(float u1, float u2) {
    float3 p{0.f, 0.f, 0.f};
    const float z = 1.f - 2.f * u1;
    const float sin_theta = sqrtf(std::fmax(0.f, 1.f - z * z));
    const float phi = 2.0f * M_PIf_ * u2;
    p.x = sin_theta * pupil_dm::dm_cos(phi);
    p.y = sin_theta * pupil_dm::dm_sin(phi);
    p.z = absf(z);
    return p;
}
inline float UniformSampleHemispherePdf(float3 v) { return v.z > 0.f ? M_1_PIf_ * 0.5f : 0.f; }
inline float3 Reflect(float3 v) {
    v.x = -v.x;
    v.y = -v.y;
    return v;
}
inline float3 Reflect(float3 v, float3 normal) { return -v + 2 * dot(v, normal) * normal; }
inline float3 Refract(float3 v, float cos_theta_t, float eta) {
    float scale = -(cos_theta_t < 0.f ? 1.f / eta : eta);
    return normalize(make_float3(scale * v.x, scale * v.y, cos_theta_t));
}
inline float3 Refract(float3 v, float3 normal, float cos_theta_t, float eta) {
    if (cos_theta_t < 0) eta = 1 / eta;
    return normal * (dot(v, normal) * eta + cos_theta_t) - v * eta;
}
inline void BuildONB(float3 N, float3 &b1, float3 &b2) {
    float sign = copysignf(1.f, N.z);
    float a = -1.f / (sign + N.z);
    float b = N.x * N.y * a;
    b1 = make_float3(1.f + sign * N.x * N.x * a, sign * b, -sign * N.x);
    b2 = make_float3(b, sign + N.y * N.y * a, -N.y);
}
inline float3 ToLocal(float3 v, float3 N) {
    float3 b1, b2;
    BuildONB(N, b1, b2);
    return make_float3(dot(v, b1), dot(v, b2), dot(v, N));
}
inline float3 ToWorld(float3 v, float3 N) {
    float3 b1, b2;
    BuildONB(N, b1, b2);
    return b1 * v.x + b2 * v.y + N * v.z;
}
inline float2 GetSphereTexcoord(float3 local_p) {
    float phi = pupil_dm::dm_atan2(local_p.y, local_p.x);
    phi = phi < 0.f ? phi + M_PIf_ * 2.f : phi;
    float theta = pupil_dm::dm_acos(local_p.z);
    return make_float2(phi * M_1_PIf_ * 0.5f, theta * M_1_PIf_);
}
inline float GetLuminance(float3 c) { return 0.2126f * c.x + 0.7152f * c.y + 0.0722f * c.z; }
inline float MISWeight(float x, float y) { return x / (x + y); }
inline bool IsZero(float v) { return absf(v) < EPS; }
inline bool IsZero(float3 v) { return absf(v.x) < EPS && absf(v.y) < EPS && absf(v.z) < EPS; }
inline float Lerp(float a, float b, float t) { return a + t * (b - a); }

// ------------------------------------------------------------------ cuda::Texture
struct Texture {
    unsigned int type = PUPIL_TEX_RGB;
    float3 rgb{0, 0, 0}, patch1{0, 0, 0}, patch2{0, 0, 0};
    float4 r0{1, 0, 0, 0}, r1{0, 1, 0, 0};
    unsigned int w = 0, h = 0, filter = 0;
    const float *texels = nullptr;  // rgba

    float3 Sample(float2 texcoord) const {
        const float4 tex = make_float4(texcoord.x, texcoord.y, 0.f, 1.f);
        float tex_x = dot(r0, tex);
        float tex_y = dot(r1, tex);
        float3 color{0, 0, 0};
        switch (type) {
            case PUPIL_TEX_RGB: color = rgb; break;
            case PUPIL_TEX_CHECKERBOARD: {
                tex_x = tex_x - (tex_x > 0.f ? floorf(tex_x) : ceilf(tex_x));
                tex_y = tex_y - (tex_y > 0.f ? floorf(tex_y) : ceilf(tex_y));
                if (tex_x < 0.f) tex_x += 1.f;
                if (tex_y < 0.f) tex_y += 1.f;
                if (tex_x > 0.5f)
                    color = tex_y > 0.5f ? patch1 : patch2;
                else
                    color = tex_y > 0.5f ? patch2 : patch1;
            } break;
            case PUPIL_TEX_BITMAP: color = Bitmap(tex_x, tex_y); break;
        }
        return color;
    }
    // tex2D(normalized coords, wrap) emulation: point, or bilinear with 8-bit weights
    float3 Bitmap(float x, float y) const {
        if (!texels || !w || !h) return make_float3(0.f);
        const int W = (int)w, H = (int)h;
        auto wrap = [](int i, int n) {
            int r = i % n;
            return r < 0 ? r + n : r;
        };
        auto fetch = [&](int ix, int iy) {
            const float *c = texels + 4 * ((size_t)wrap(iy, H) * W + wrap(ix, W));
            return make_float3(c[0], c[1], c[2]);
        };
        if (filter == 0) return fetch((int)floorf(x * (float)W), (int)floorf(y * (float)H));
        const float fx = x * (float)W - 0.5f, fy = y * (float)H - 0.5f;
        const float x0 = floorf(fx), y0 = floorf(fy);
        const float ax = floorf((fx - x0) * 256.f + 0.5f) / 256.f;
        const float ay = floorf((fy - y0) * 256.f + 0.5f) / 256.f;
        const float3 a = fetch((int)x0, (int)y0) * (1.f - ax) + fetch((int)x0 + 1, (int)y0) * ax;
        const float3 b = fetch((int)x0, (int)y0 + 1) * (1.f - ax) + fetch((int)x0 + 1, (int)y0 + 1) * ax;
        return a * (1.f - ay) + b * ay;
    }
};

Texture MakeTexture(const pupil_texture &t) {
    Texture r;
    r.type = t.type;
    r.rgb = make_float3(t.c0[0], t.c0[1], t.c0[2]);
    r.patch1 = r.rgb;
    r.patch2 = make_float3(t.c1[0], t.c1[1], t.c1[2]);
    r.r0 = make_float4(t.transform[0], t.transform[1], t.transform[2], t.transform[3]);
    r.r1 = make_float4(t.transform[4], t.transform[5], t.transform[6], t.transform[7]);
    r.w = t.width;
    r.h = t.height;
    r.filter = t.filter;
    r.texels = t.rgba;
    return r;
}

// ------------------------------------------------------------------ fresnel.h
namespace fresnel {
inline float DielectricReflectance(float eta, float cos_theta_i, float &cos_theta_t) {
    float scale = cos_theta_i > 0.f ? 1.f / eta : eta;
    float cos_theta_t2 = 1.f - (1.f - cos_theta_i * cos_theta_i) * (scale * scale);
    if (cos_theta_t2 <= 0.0f) {
        cos_theta_t = 0.0f;
        return 1.0f;
    }
    float o_cos_theta_i = cos_theta_i;
    cos_theta_i = absf(cos_theta_i);
    cos_theta_t = sqrtf(std::fmax(0.f, cos_theta_t2));
    float rs = (cos_theta_i - eta * cos_theta_t) / (cos_theta_i + eta * cos_theta_t);
    float rp = (eta * cos_theta_i - cos_theta_t) / (eta * cos_theta_i + cos_theta_t);
    cos_theta_t = o_cos_theta_i > 0.f ? -cos_theta_t : cos_theta_t;
    return 0.5f * (rs * rs + rp * rp);
}
inline float DielectricReflectance(float eta, float cos_theta_i) {
    float cos_theta_t;
    return DielectricReflectance(eta, cos_theta_i, cos_theta_t);
}
inline float ConductorReflectance(float eta, float k, float cos_theta_i) {
    float cos_theta_i2 = cos_theta_i * cos_theta_i;
    float sin_theta_i2 = 1.f - cos_theta_i2;
    float sin_theta_i4 = sin_theta_i2 * sin_theta_i2;
    float t1 = eta * eta - k * k - sin_theta_i2;
    float a2pb2 = sqrtf(std::fmax(0.f, t1 * t1 + 4.f * k * k * eta * eta));
    float a = sqrtf(std::fmax(0.f, 0.5f * (a2pb2 + t1)));
    float term1 = a2pb2 + cos_theta_i2;
    float term2 = 2.f * a * cos_theta_i;
    float rs2 = (term1 - term2) / (term1 + term2);
    float term3 = a2pb2 * cos_theta_i2 + sin_theta_i4;
    float term4 = term2 * sin_theta_i2;
    float rp2 = rs2 * (term3 - term4) / (term3 + term4);
    return 0.5f * (rp2 + rs2);
}
inline float3 ConductorReflectance(const float3 eta, const float3 k, float cos_theta_i) {
    return make_float3(ConductorReflectance(eta.x, k.x, cos_theta_i), ConductorReflectance(eta.y, k.y, cos_theta_i),
                       ConductorReflectance(eta.z, k.z, cos_theta_i));
}
inline float DiffuseReflectance(float eta) {
    if (eta < 1) {
        return -1.4399f * (eta * eta) + 0.7099f * eta + 0.6681f + 0.0636f / eta;
    } else {
        float inv_eta = 1.0f / eta;
        float inv_eta2 = inv_eta * inv_eta;
        float inv_eta3 = inv_eta2 * inv_eta;
        float inv_eta4 = inv_eta3 * inv_eta;
        float inv_eta5 = inv_eta4 * inv_eta;
        return 0.919317f - 3.4793f * inv_eta + 6.75335f * inv_eta2 - 7.80989f * inv_eta3 + 4.98554f * inv_eta4 -
               1.36881f * inv_eta5;
    }
}
}  // namespace fresnel

// ------------------------------------------------------------------ ggx.h (GGX_Sample_Visible_Area)
namespace ggx {
inline float Lambda(float3 w, float alpha) {
    float a2 = alpha * alpha;
    float3 v2 = w * w;
    return (-1.f + sqrtf(1.f + (v2.x + v2.y) * a2 / v2.z)) / 2.f;
}
inline float G1(float3 w, float alpha) { return 1.f / (1.f + Lambda(w, alpha)); }
inline float G(float3 wi, float3 wo, float alpha) { return G1(wi, alpha) * G1(wo, alpha); }
inline float D(float3 wh, float alpha) {
    float a2 = alpha * alpha;
    float3 v2 = wh * wh;
    float t = (v2.x + v2.y) / a2 + v2.z;
    return 1.f / (M_PIf_ * a2 * t * t);
}
inline float Pdf(float3 wo, float3 wh, float alpha) { return D(wh, alpha) * G1(wo, alpha) * dot(wo, wh) / absf(wo.z); }
inline float3 Sample(float3 wo, float alpha, float2 xi) {
    float3 vh = normalize(make_float3(alpha * wo.x, alpha * wo.y, wo.z));
    float3 T1 = wo.z < 0.9999f ? normalize(cross(make_float3(0.f, 0.f, 1.f), vh)) : make_float3(1.f, 0.f, 0.f);
    float3 T2 = cross(vh, T1);
    float r = sqrtf(xi.x);
    float phi = 2.f * M_PIf_ * xi.y;
    float t1 = r * pupil_dm::dm_cos(phi);
    float t2 = r * pupil_dm::dm_sin(phi);
    float s = 0.5f * (1.f + vh.z);
    t2 = (1.f - s) * sqrtf(1.f - t1 * t1) + s * t2;
    float3 nh = t1 * T1 + t2 * T2 + sqrtf(std::fmax(0.f, 1.f - t1 * t1 - t2 * t2)) * vh;
    float3 ne = make_float3(alpha * nh.x, alpha * nh.y, std::fmax(0.f, nh.z));
    return normalize(ne);
}
}  // namespace ggx

// ------------------------------------------------------------------ bsdf/*.h
enum Lobe : unsigned int {
    Unknown = 0,
    DiffuseReflection = 1 << 1,
    GlossyReflection = 1 << 3,
    GlossyTransmission = 1 << 4,
    DeltaReflection = 1 << 5,
    DeltaTransmission = 1 << 6,
    Delta = DeltaReflection | DeltaTransmission
};

struct BsdfSamplingRecord {
    float3 wi{0, 0, 0};
    float3 wo{0, 0, 0};
    float3 f = make_float3(0.f);
    float pdf = 0.f;
    Random *sampler = nullptr;
    unsigned int sampled_type = Unknown;
};

struct DiffuseL {
    float3 reflectance;
    void GetBsdf(BsdfSamplingRecord &record) const {
        float3 f = make_float3(0.f);
        if (record.wi.z > 0.f && record.wo.z > 0.f) f = reflectance * M_1_PIf_;
        record.f = f;
    }
    void GetPdf(BsdfSamplingRecord &record) const {
        float pdf = 0.f;
        if (record.wi.z > 0.f && record.wo.z > 0.f) pdf = CosineSampleHemispherePdf(record.wi);
        record.pdf = pdf;
    }
    void Sample(BsdfSamplingRecord &record) const {
        float2 xi = record.sampler->Next2();
        record.wi = CosineSampleHemisphere(xi.x, xi.y);
        GetPdf(record);
        GetBsdf(record);
        record.sampled_type = DiffuseReflection;
    }
};

struct DielectricL {
    float eta;
    float3 specular_reflectance, specular_transmittance;
    void GetBsdf(BsdfSamplingRecord &record) const { record.f = make_float3(0.f); }
    void GetPdf(BsdfSamplingRecord &record) const { record.pdf = 0.f; }
    void Sample(BsdfSamplingRecord &record) const {
        float cos_theta_t;
        float fr = fresnel::DielectricReflectance(eta, record.wo.z, cos_theta_t);
        if (record.sampler->Next() < fr) {
            record.wi = Reflect(record.wo);
            record.pdf = fr;
            record.f = specular_reflectance * fr / absf(record.wi.z);
            record.sampled_type = DeltaReflection;
        } else {
            record.wi = Refract(record.wo, cos_theta_t, eta);
            record.pdf = 1.f - fr;
            float factor = cos_theta_t < 0.f ? 1.f / eta : eta;
            record.f = specular_transmittance * (1.f - fr) * factor * factor / absf(record.wi.z);
            record.sampled_type = DeltaTransmission;
        }
    }
};

struct RoughDielectricL {
    float alpha, eta;
    float3 specular_reflectance, specular_transmittance;
    void GetBsdf(BsdfSamplingRecord &record) const {
        record.f = make_float3(0.f);
        if (IsZero(record.wo.z)) return;
        float3 wh;
        bool sample_reflect = record.wo.z * record.wi.z > 0.f;
        if (sample_reflect)
            wh = normalize(record.wo + record.wi);
        else
            wh = normalize(record.wo + record.wi * (record.wo.z > 0.f ? eta : 1.f / eta));
        wh = wh * (wh.z > 0.f ? 1.f : -1.f);
        float F = fresnel::DielectricReflectance(eta, dot(record.wo, wh));
        float G = ggx::G(record.wi, record.wo, alpha);
        float D = ggx::D(wh, alpha);
        if (sample_reflect) {
            record.f = specular_reflectance * F * G * D / (4.f * absf(record.wi.z) * absf(record.wo.z));
        } else {
            float _eta = record.wo.z > 0.f ? eta : 1.f / eta;
            float sqrt_denom = dot(record.wo, wh) + _eta * dot(record.wi, wh);
            record.f = specular_transmittance * absf((1.f - F) * D * G * dot(record.wi, wh) * dot(record.wo, wh) /
                                                     (sqrt_denom * sqrt_denom * record.wi.z * record.wo.z));
        }
    }
    void GetPdf(BsdfSamplingRecord &record) const {
        record.pdf = 0.f;
        bool sample_reflect = record.wo.z * record.wi.z > 0.f;
        float3 wh;
        float dwh_dwo;
        if (sample_reflect) {
            wh = normalize(record.wo + record.wi);
            dwh_dwo = 1.f / (4.f * dot(record.wi, wh));
        } else {
            float _eta = record.wo.z > 0.f ? eta : 1.f / eta;
            wh = normalize(record.wo + record.wi * _eta);
            float sqrt_denom = dot(record.wo, wh) + _eta * dot(record.wi, wh);
            dwh_dwo = (_eta * _eta * dot(record.wi, wh)) / (sqrt_denom * sqrt_denom);
        }
        wh = wh * (wh.z > 0.f ? 1.f : -1.f);
        float3 wo = record.wo * (record.wo.z > 0.f ? 1.f : -1.f);
        float F = fresnel::DielectricReflectance(eta, dot(record.wo, wh));
        record.pdf = absf(ggx::Pdf(wo, wh, alpha) * (sample_reflect ? F : 1.f - F) * dwh_dwo);
    }
    void Sample(BsdfSamplingRecord &record) const {
        float2 xi = record.sampler->Next2();
        float3 wo = record.wo * (record.wo.z > 0.f ? 1.f : -1.f);
        float3 wh = ggx::Sample(wo, alpha, xi);
        float cos_theta_t = 0.f;
        float F = fresnel::DielectricReflectance(eta, dot(record.wo, wh), cos_theta_t);
        if (record.sampler->Next() < F) {
            record.wi = Reflect(record.wo, wh);
            record.sampled_type = GlossyReflection;
        } else {
            if (IsZero(cos_theta_t)) return;
            record.wi = Refract(record.wo, wh, cos_theta_t, eta);
            record.sampled_type = GlossyTransmission;
            if (record.wi.z * record.wo.z >= 0.f) return;
        }
        GetPdf(record);
        GetBsdf(record);
    }
};

struct ConductorL {
    float3 eta, k, specular_reflectance;
    void GetBsdf(BsdfSamplingRecord &record) const { record.f = make_float3(0.f); }
    void GetPdf(BsdfSamplingRecord &record) const { record.pdf = 0.f; }
    void Sample(BsdfSamplingRecord &record) const {
        record.wi = Reflect(record.wo);
        record.pdf = 1.f;
        float3 fr = fresnel::ConductorReflectance(eta, k, record.wo.z);
        record.f = specular_reflectance * fr / absf(record.wi.z);
        record.sampled_type = DeltaReflection;
    }
};

struct RoughConductorL {
    float alpha;
    float3 eta, k, specular_reflectance;
    void GetBsdf(BsdfSamplingRecord &record) const {
        record.f = make_float3(0.f);
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float3 wh = normalize(record.wi + record.wo);
        float3 fresnel_o = fresnel::ConductorReflectance(eta, k, dot(record.wo, wh));
        record.f = specular_reflectance * ggx::D(wh, alpha) * fresnel_o * ggx::G(record.wi, record.wo, alpha) /
                   (4.f * record.wi.z * record.wo.z);
    }
    void GetPdf(BsdfSamplingRecord &record) const {
        record.pdf = 0.f;
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float3 wh = normalize(record.wi + record.wo);
        wh = normalize(wh);
        record.pdf = ggx::Pdf(record.wo, wh, alpha) / (4.f * dot(record.wo, wh));
    }
    void Sample(BsdfSamplingRecord &record) const {
        float2 xi = record.sampler->Next2();
        record.wi = Reflect(record.wo, ggx::Sample(record.wo, alpha, xi));
        GetPdf(record);
        GetBsdf(record);
        record.sampled_type = DiffuseReflection;  // as in rough_conductor.h:45
    }
};

struct PlasticL {
    float eta, int_fdr, specular_sampling_weight;
    bool nonlinear;
    float3 diffuse_reflectance, specular_reflectance;
    float3 Diff() const {
        return diffuse_reflectance /
               (1.f - (nonlinear ? diffuse_reflectance * int_fdr : make_float3(int_fdr)));
    }
    float SpecProb(float fresnel_o) const {
        return (fresnel_o * specular_sampling_weight) /
               (fresnel_o * specular_sampling_weight + (1 - fresnel_o) * (1.f - specular_sampling_weight));
    }
    void GetBsdf(BsdfSamplingRecord &record) const {
        record.f = make_float3(0.f);
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float fresnel_i = fresnel::DielectricReflectance(eta, record.wi.z);
        float3 diff = Diff();
        record.f = diff * (1.f - fresnel_i) * (1.f - fresnel_o) * CosineSampleHemispherePdf(record.wi) /
                   (eta * eta * record.wi.z);
    }
    void GetPdf(BsdfSamplingRecord &record) const {
        record.pdf = 0.f;
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float specular_prob = SpecProb(fresnel_o);
        record.pdf = CosineSampleHemispherePdf(record.wi) * (1.f - specular_prob);
    }
    void Sample(BsdfSamplingRecord &record) const {
        if (record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float2 xi = record.sampler->Next2();
        float specular_prob = SpecProb(fresnel_o);
        if (xi.x < specular_prob) {
            record.sampled_type = DeltaReflection;
            record.wi = Reflect(record.wo);
            record.f = specular_reflectance * fresnel_o / record.wi.z;
            record.pdf = specular_prob;
        } else {
            record.sampled_type = DiffuseReflection;
            record.wi = CosineSampleHemisphere((xi.x - specular_prob) / (1.f - specular_prob), xi.y);
            float fresnel_i = fresnel::DielectricReflectance(eta, record.wi.z);
            float3 diff = Diff();
            record.f = diff * (1.f - fresnel_i) * (1.f - fresnel_o) * CosineSampleHemispherePdf(record.wi) /
                       (eta * eta * record.wi.z);
            record.pdf = CosineSampleHemispherePdf(record.wi) * (1.f - specular_prob);
        }
    }
};

struct RoughPlasticL {
    float eta, int_fdr, specular_sampling_weight, alpha;
    bool nonlinear;
    float3 diffuse_reflectance, specular_reflectance;
    float3 Diff() const {
        return diffuse_reflectance /
               (1.f - (nonlinear ? diffuse_reflectance * int_fdr : make_float3(int_fdr)));
    }
    float SpecProb(float fresnel_o) const {
        return (fresnel_o * specular_sampling_weight) /
               (fresnel_o * specular_sampling_weight + (1 - fresnel_o) * (1.f - specular_sampling_weight));
    }
    void GetBsdf(BsdfSamplingRecord &record) const {
        record.f = make_float3(0.f);
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float3 wh = normalize(record.wi + record.wo);
        record.f = specular_reflectance * fresnel::DielectricReflectance(eta, dot(wh, record.wo)) * ggx::D(wh, alpha) *
                   ggx::G(record.wi, record.wo, alpha) / (4.f * record.wo.z * record.wi.z);
        float fresnel_i = fresnel::DielectricReflectance(eta, record.wi.z);
        float3 diff = Diff();
        record.f += diff * (1.f - fresnel_i) * (1.f - fresnel_o) * M_1_PIf_ / (eta * eta);
    }
    void GetPdf(BsdfSamplingRecord &record) const {
        record.pdf = 0.f;
        if (record.wi.z <= 0.f || record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float specular_prob = SpecProb(fresnel_o);
        float diffuse_prob = 1.f - specular_prob;
        float3 wh = normalize(record.wi + record.wo);
        record.pdf = specular_prob * ggx::Pdf(record.wo, wh, alpha) / (4.f * dot(record.wi, wh));
        record.pdf += diffuse_prob * CosineSampleHemispherePdf(record.wi);
    }
    void Sample(BsdfSamplingRecord &record) const {
        record.wi = make_float3(0.f);
        if (record.wo.z <= 0.f) return;
        float fresnel_o = fresnel::DielectricReflectance(eta, record.wo.z);
        float specular_prob = SpecProb(fresnel_o);
        float2 xi = record.sampler->Next2();
        if (xi.y < specular_prob) {
            xi.y /= specular_prob;
            float3 wh = ggx::Sample(record.wo, alpha, xi);
            record.wi = Reflect(record.wo, wh);
            record.sampled_type = GlossyReflection;
        } else {
            xi.y = (xi.y - specular_prob) / (1.f - specular_prob);
            record.wi = CosineSampleHemisphere(xi.x, xi.y);
            record.sampled_type = DiffuseReflection;
        }
        GetPdf(record);
        GetBsdf(record);
    }
};

// optix::material::Material (host-precomputed) and Material::LocalBsdf
struct Material {
    unsigned int type = PUPIL_MAT_UNKNOWN;
    bool twosided = false, nonlinear = false;
    float int_ior = 1.f, ext_ior = 1.f, eta = 1.f;
    float m_int_fdr = 0.f, m_specular_sampling_weight = 0.f;
    Texture tex[4];
};

struct LocalBsdf {
    unsigned int type = PUPIL_MAT_UNKNOWN;
    DiffuseL diffuse{};
    DielectricL dielectric{};
    RoughDielectricL rough_dielectric{};
    ConductorL conductor{};
    RoughConductorL rough_conductor{};
    PlasticL plastic{};
    RoughPlasticL rough_plastic{};

    void Sample(BsdfSamplingRecord &r) const {
        switch (type) {
            case PUPIL_MAT_DIFFUSE: diffuse.Sample(r); break;
            case PUPIL_MAT_DIELECTRIC: dielectric.Sample(r); break;
            case PUPIL_MAT_ROUGH_DIELECTRIC: rough_dielectric.Sample(r); break;
            case PUPIL_MAT_CONDUCTOR: conductor.Sample(r); break;
            case PUPIL_MAT_ROUGH_CONDUCTOR: rough_conductor.Sample(r); break;
            case PUPIL_MAT_PLASTIC: plastic.Sample(r); break;
            case PUPIL_MAT_ROUGH_PLASTIC: rough_plastic.Sample(r); break;
            default: break;  // no bsdf: the path ends (f = 0)
        }
    }
    void Eval(BsdfSamplingRecord &r) const {
#define EVAL(x)      \
    x.GetBsdf(r);    \
    x.GetPdf(r);     \
    break;
        switch (type) {
            case PUPIL_MAT_DIFFUSE: EVAL(diffuse)
            case PUPIL_MAT_DIELECTRIC: EVAL(dielectric)
            case PUPIL_MAT_ROUGH_DIELECTRIC: EVAL(rough_dielectric)
            case PUPIL_MAT_CONDUCTOR: EVAL(conductor)
            case PUPIL_MAT_ROUGH_CONDUCTOR: EVAL(rough_conductor)
            case PUPIL_MAT_PLASTIC: EVAL(plastic)
            case PUPIL_MAT_ROUGH_PLASTIC: EVAL(rough_plastic)
            default: break;
        }
#undef EVAL
    }
    float3 GetAlbedo() const {
        switch (type) {
            case PUPIL_MAT_DIFFUSE: return diffuse.reflectance;
            case PUPIL_MAT_DIELECTRIC: return dielectric.specular_reflectance;
            case PUPIL_MAT_ROUGH_DIELECTRIC: return rough_dielectric.specular_reflectance;
            case PUPIL_MAT_CONDUCTOR: return conductor.specular_reflectance;
            case PUPIL_MAT_ROUGH_CONDUCTOR: return rough_conductor.specular_reflectance;
            case PUPIL_MAT_PLASTIC: return plastic.diffuse_reflectance;
            case PUPIL_MAT_ROUGH_PLASTIC: return rough_plastic.diffuse_reflectance;
        }
        return make_float3(0.f);
    }
};

LocalBsdf GetLocalBsdf(const Material &m, float2 uv) {
    LocalBsdf l;
    l.type = m.type;
    switch (m.type) {
        case PUPIL_MAT_DIFFUSE: l.diffuse.reflectance = m.tex[0].Sample(uv); break;
        case PUPIL_MAT_DIELECTRIC:
            l.dielectric.eta = m.int_ior / m.ext_ior;
            l.dielectric.specular_reflectance = m.tex[0].Sample(uv);
            l.dielectric.specular_transmittance = m.tex[1].Sample(uv);
            break;
        case PUPIL_MAT_ROUGH_DIELECTRIC:
            l.rough_dielectric.alpha = m.tex[0].Sample(uv).x;
            l.rough_dielectric.eta = m.eta;
            l.rough_dielectric.specular_reflectance = m.tex[1].Sample(uv);
            l.rough_dielectric.specular_transmittance = m.tex[2].Sample(uv);
            break;
        case PUPIL_MAT_CONDUCTOR:
            l.conductor.eta = m.tex[0].Sample(uv);
            l.conductor.k = m.tex[1].Sample(uv);
            l.conductor.specular_reflectance = m.tex[2].Sample(uv);
            break;
        case PUPIL_MAT_ROUGH_CONDUCTOR:
            l.rough_conductor.alpha = m.tex[0].Sample(uv).x;
            l.rough_conductor.eta = m.tex[1].Sample(uv);
            l.rough_conductor.k = m.tex[2].Sample(uv);
            l.rough_conductor.specular_reflectance = m.tex[3].Sample(uv);
            break;
        case PUPIL_MAT_PLASTIC:
            l.plastic.eta = m.eta;
            l.plastic.nonlinear = m.nonlinear;
            l.plastic.int_fdr = m.m_int_fdr;
            l.plastic.diffuse_reflectance = m.tex[0].Sample(uv);
            l.plastic.specular_reflectance = m.tex[1].Sample(uv);
            l.plastic.specular_sampling_weight = m.m_specular_sampling_weight;
            break;
        case PUPIL_MAT_ROUGH_PLASTIC:
            l.rough_plastic.eta = m.eta;
            l.rough_plastic.nonlinear = m.nonlinear;
            l.rough_plastic.int_fdr = m.m_int_fdr;
            l.rough_plastic.alpha = m.tex[0].Sample(uv).x;
            l.rough_plastic.diffuse_reflectance = m.tex[1].Sample(uv);
            l.rough_plastic.specular_reflectance = m.tex[2].Sample(uv);
            l.rough_plastic.specular_sampling_weight = m.m_specular_sampling_weight;
            break;
        default: break;
    }
    return l;
}

float3 GetPixelAverage(const pupil_texture &t) {  // optix_material.cpp:15-42
    switch (t.type) {
        case PUPIL_TEX_RGB: return make_float3(t.c0[0], t.c0[1], t.c0[2]);
        case PUPIL_TEX_CHECKERBOARD: {
            float r = t.c0[0] + t.c1[0];
            float g = t.c0[1] + t.c1[1];
            float b = t.c0[2] + t.c1[2];
            return make_float3(r, g, b) * 0.5f;
        }
        case PUPIL_TEX_BITMAP: {
            float r = 0.f, g = 0.f, b = 0.f;
            if (!t.rgba) return make_float3(0.f);
            for (size_t i = 0, idx = 0; i < t.height; ++i)
                for (size_t j = 0; j < t.width; ++j) {
                    r += t.rgba[idx++];
                    g += t.rgba[idx++];
                    b += t.rgba[idx++];
                    idx++;
                }
            return make_float3(r, g, b) / (1.f * (float)t.height * (float)t.width);
        }
    }
    return make_float3(0.f);
}

Material LoadMaterial(const pupil_material &src) {  // optix_material.cpp:39-132
    Material m;
    m.type = src.type <= 7u ? src.type : PUPIL_MAT_UNKNOWN;
    m.twosided = src.twosided != 0;
    m.nonlinear = src.nonlinear != 0;
    m.int_ior = src.int_ior;
    m.ext_ior = src.ext_ior;
    for (int k = 0; k < 4; k++) m.tex[k] = MakeTexture(src.tex[k]);
    if (m.type == PUPIL_MAT_ROUGH_DIELECTRIC || m.type == PUPIL_MAT_PLASTIC || m.type == PUPIL_MAT_ROUGH_PLASTIC)
        m.eta = src.int_ior / src.ext_ior;
    if (m.type == PUPIL_MAT_PLASTIC || m.type == PUPIL_MAT_ROUGH_PLASTIC) {
        const int di = m.type == PUPIL_MAT_PLASTIC ? 0 : 1;
        float diffuse_luminance = GetLuminance(GetPixelAverage(src.tex[di]));
        float specular_luminance = GetLuminance(GetPixelAverage(src.tex[di + 1]));
        m.m_specular_sampling_weight = specular_luminance / (specular_luminance + diffuse_luminance);
        m.m_int_fdr = fresnel::DiffuseReflectance(1.f / m.eta);
    }
    return m;
}

// ------------------------------------------------------------------ emitters
struct LocalGeometry {
    float3 position{0, 0, 0};
    float3 normal{0, 0, 0};
    float2 texcoord{0, 0};
};
struct EmitterSampleRecord {
    float3 radiance{0, 0, 0};
    float3 wi{0, 0, 0};
    float distance = 0.f;  // uninitialised in the reference when pdf stays 0
    float pdf = 0.f;
    bool is_delta = false;  // never set for area emitters in the reference
};
struct EmitEvalRecord {
    float3 radiance{0, 0, 0};
    float pdf = 0.f;  // the reference leaves it uninitialised when LNoL <= 0
};

struct Emitter {
    unsigned int type = PUPIL_EMITTER_NONE;
    float select_probability = 0.f;
    Texture radiance;
    float area = 0.f;
    float3 v_pos[3], v_nrm[3];
    float2 v_tex[3];
    float3 center{0, 0, 0};
    float sphere_radius = 0.f;
    float3 color{0, 0, 0};
    // env map
    unsigned int map_w = 0, map_h = 0;
    std::vector<float> row_cdf, col_cdf, row_weight;
    float3 to_world[3], to_local[3];
    float normalization = 0.f, scale = 1.f;

    float3 GetRadiance(float2 tex) const {
        if (type == PUPIL_EMITTER_CONST_ENV) return color;
        return radiance.Sample(tex);
    }
    void SampleDirect(EmitterSampleRecord &ret, const LocalGeometry &hit_geo, float2 xi) const {
        switch (type) {
            case PUPIL_EMITTER_TRI_AREA: {  // area.h:17-34
                float3 t = UniformSampleTriangle(xi.x, xi.y);
                float3 position = v_pos[0] * t.x + v_pos[1] * t.y + v_pos[2] * t.z;
                float3 normal = normalize(v_nrm[0] * t.x + v_nrm[1] * t.y + v_nrm[2] * t.z);
                float2 tex = v_tex[0] * t.x + v_tex[1] * t.y + v_tex[2] * t.z;
                ret.radiance = radiance.Sample(tex);
                ret.wi = normalize(position - hit_geo.position);
                float NoL = dot(hit_geo.normal, ret.wi);
                float LNoL = dot(normal, -ret.wi);
                if (NoL > 0.f && LNoL > 0.f) {
                    float distance = length(position - hit_geo.position);
                    ret.pdf = distance * distance / (LNoL * area);
                    ret.distance = distance;
                }
            } break;
            case PUPIL_EMITTER_SPHERE: {  // sphere.h:14-31
                float3 t = UniformSampleSphere(xi.x, xi.y);
                float3 position = t * sphere_radius + center;
                float3 normal = normalize(t);
                float2 tex = GetSphereTexcoord(t);
                ret.radiance = radiance.Sample(tex);
                ret.wi = normalize(position - hit_geo.position);
                float NoL = dot(hit_geo.normal, ret.wi);
                float LNoL = dot(normal, -ret.wi);
                if (NoL > 0.f && LNoL > 0.f) {
                    float distance = length(position - hit_geo.position);
                    ret.pdf = distance * distance / (LNoL * area);
                    ret.distance = distance;
                }
            } break;
            case PUPIL_EMITTER_CONST_ENV: {  // env.h:70-79
                float3 local_wi = UniformSampleHemisphere(xi.x, xi.y);
                ret.wi = ToWorld(local_wi, hit_geo.normal);
                ret.pdf = UniformSampleHemispherePdf(local_wi);
                ret.distance = MAX_DISTANCE;
                ret.radiance = color;
                ret.is_delta = false;
            } break;
            case PUPIL_EMITTER_ENV_MAP: {  // env.h:23-49
                unsigned int row_index = 0;
                for (; row_index < row_cdf.size() - 1; ++row_index)
                    if (xi.x <= row_cdf[row_index]) break;
                unsigned int col_index = 0;
                for (int i = row_index * (map_w + 1); col_index < map_w - 1; ++i, ++col_index)
                    if (xi.y <= col_cdf[i]) break;
                const float phi = col_index * M_PIf_ * 2.f / map_w;
                const float theta = row_index * M_PIf_ / map_h;
                const float st = pupil_dm::dm_sin(theta);
                const auto local_wi = make_float3(st * pupil_dm::dm_sin(M_PIf_ - phi), pupil_dm::dm_cos(theta),
                                                  st * pupil_dm::dm_cos(M_PIf_ - phi));
                ret.wi = make_float3(dot(to_world[0], local_wi), dot(to_world[1], local_wi), dot(to_world[2], local_wi));
                ret.distance = MAX_DISTANCE;
                const float2 tex = make_float2(phi * 0.5f * M_1_PIf_, theta * M_1_PIf_);
                ret.radiance = radiance.Sample(tex) * scale;
                ret.is_delta = false;
                ret.pdf = GetLuminance(ret.radiance) * row_weight[row_index] * normalization /
                          std::fmax(1e-4f, absf(st));
                if (ret.pdf < 0.f) ret.pdf = 0.f;
            } break;
        }
    }
    void Eval(EmitEvalRecord &ret, const LocalGeometry &g, float3 scatter_pos) const {
        switch (type) {
            case PUPIL_EMITTER_TRI_AREA:
            case PUPIL_EMITTER_SPHERE: {  // area.h:36-45 / sphere.h:33-43
                float3 dir = normalize(scatter_pos - g.position);
                float LNoL = dot(g.normal, dir);
                if (LNoL > 0.f) {
                    float distance = length(scatter_pos - g.position);
                    ret.pdf = distance * distance / (LNoL * area);
                    ret.radiance = radiance.Sample(g.texcoord);
                }
            } break;
            case PUPIL_EMITTER_CONST_ENV:
                ret.pdf = 0.25f * M_1_PIf_;
                ret.radiance = color;
                break;
            case PUPIL_EMITTER_ENV_MAP: {  // env.h:51-64
                float3 dir = normalize(g.position - scatter_pos);
                dir = make_float3(dot(to_local[0], dir), dot(to_local[1], dir), dot(to_local[2], dir));
                const float phi = M_PIf_ - pupil_dm::dm_atan2(dir.x, dir.z);
                const float theta = pupil_dm::dm_acos(dir.y);
                const float2 tex = make_float2(phi * 0.5f * M_1_PIf_, theta * M_1_PIf_);
                unsigned int row_index = static_cast<unsigned int>(tex.y * map_h);
                row_index = std::min(row_index, map_h - 2u);
                ret.radiance = radiance.Sample(tex) * scale;
                ret.pdf = GetLuminance(ret.radiance) *
                          Lerp(row_weight[row_index], row_weight[row_index + 1], tex.y * map_h - 1.f * row_index) *
                          normalization / std::fmax(1e-4f, absf(pupil_dm::dm_sin(theta)));
            } break;
        }
    }
};

Emitter LoadEmitter(const pupil_emitter &e) {
    Emitter r;
    r.type = e.type;
    r.select_probability = e.select_probability;
    r.radiance = MakeTexture(e.radiance);
    r.area = e.area;
    for (int k = 0; k < 3; k++) {
        r.v_pos[k] = make_float3(e.pos[k][0], e.pos[k][1], e.pos[k][2]);
        r.v_nrm[k] = make_float3(e.nrm[k][0], e.nrm[k][1], e.nrm[k][2]);
        r.v_tex[k] = make_float2(e.tex[k][0], e.tex[k][1]);
        r.to_world[k] = make_float3(e.to_world[3 * k], e.to_world[3 * k + 1], e.to_world[3 * k + 2]);
        r.to_local[k] = make_float3(e.to_local[3 * k], e.to_local[3 * k + 1], e.to_local[3 * k + 2]);
    }
    r.center = make_float3(e.center[0], e.center[1], e.center[2]);
    r.sphere_radius = e.radius;
    r.color = make_float3(e.color[0], e.color[1], e.color[2]);
    r.scale = e.scale;
    if (e.type == PUPIL_EMITTER_ENV_MAP && e.radiance.rgba) {  // BuildEnvMapCdfTable, emitter.cpp:107-149
        const size_t w = e.radiance.width, h = e.radiance.height;
        const float *data = e.radiance.rgba;
        r.col_cdf.resize((w + 1) * h);
        r.row_cdf.resize(h + 1);
        r.row_weight.resize(h);
        size_t col_index = 0, row_index = 0;
        float row_sum = 0.f;
        r.row_cdf[row_index++] = 0.f;
        for (auto y = 0u; y < h; ++y) {
            float col_sum = 0.f;
            r.col_cdf[col_index++] = 0.f;
            for (auto x = 0u; x < w; ++x) {
                auto pixel_index = y * w + x;
                col_sum += GetLuminance(make_float3(data[pixel_index * 4], data[pixel_index * 4 + 1],
                                                    data[pixel_index * 4 + 2]));
                r.col_cdf[col_index++] = col_sum;
            }
            for (auto x = 1u; x < w; ++x) r.col_cdf[col_index - x - 1] /= col_sum;
            r.col_cdf[col_index - 1] = 1.f;
            float weight = std::sin((y + 0.5f) * M_PIf_ / h);
            r.row_weight[y] = weight;
            row_sum += col_sum * weight;
            r.row_cdf[row_index++] = row_sum;
        }
        for (auto y = 1u; y < h; ++y) r.row_cdf[row_index - y - 1] /= row_sum;
        r.row_cdf[row_index - 1] = 1.f;
        r.normalization = 1.f / (row_sum * (2.f * M_PIf_ / w) * (M_PIf_ / h));
        r.map_w = (unsigned int)w;
        r.map_h = (unsigned int)h;
    }
    return r;
}

struct EmitterGroup {  // emitter.h:104-136 (points / directionals are always empty)
    std::vector<Emitter> areas;
    const Emitter *env = nullptr;
    const Emitter *SelectOneEmiiter(float p) const {
        unsigned int i = 0;
        float sum_p = 0.f;
        const Emitter *emitter_cb = nullptr;
        for (; i < areas.size(); ++i) {
            if (p <= sum_p + areas[i].select_probability) return &areas[i];
            sum_p += areas[i].select_probability;
            emitter_cb = &areas[i];
        }
        return env ? env : emitter_cb;
    }
};

// ------------------------------------------------------------------ geometry + acceleration
struct Instance {
    float to_world[12], to_object[12];
    unsigned int kind, material, flip_normals, flip_tex_coords;
    int emitter_index_offset;
    const pupil_shape *shape;
    unsigned int prim_offset;
};

inline float3 XformPoint(const float *m, float3 p) {
    return make_float3(m[0] * p.x + m[1] * p.y + m[2] * p.z + m[3], m[4] * p.x + m[5] * p.y + m[6] * p.z + m[7],
                       m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11]);
}
inline float3 XformVector(const float *m, float3 v) {
    return make_float3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[4] * v.x + m[5] * v.y + m[6] * v.z,
                       m[8] * v.x + m[9] * v.y + m[10] * v.z);
}
inline float3 XformNormal(const float *inv, float3 n) {  // (M^-1)^T n
    return make_float3(inv[0] * n.x + inv[4] * n.y + inv[8] * n.z, inv[1] * n.x + inv[5] * n.y + inv[9] * n.z,
                       inv[2] * n.x + inv[6] * n.y + inv[10] * n.z);
}

struct Prim {
    float3 v0, v1, v2;  // world-space triangle (unused for spheres)
    unsigned int id;    // global primitive id
    unsigned int inst;
    bool sphere;
};

struct Ray {
    float3 o, d;
    float3 idir;
    int kx, ky, kz;
    float Sx, Sy, Sz;
};

inline float Comp(const float3 &v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

Ray MakeRay(float3 o, float3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    const float tiny = 1e-30f;
    r.idir = make_float3(1.f / (absf(d.x) < tiny ? copysignf(tiny, d.x) : d.x),
                         1.f / (absf(d.y) < tiny ? copysignf(tiny, d.y) : d.y),
                         1.f / (absf(d.z) < tiny ? copysignf(tiny, d.z) : d.z));
    // watertight set-up (Woop et al. 2013): kz = largest |d| component
    const float ax = absf(d.x), ay = absf(d.y), az = absf(d.z);
    int kz = 0;
    if (ay > ax) kz = 1;
    if (az > (kz == 0 ? ax : ay)) kz = 2;
    int kx = (kz + 1) % 3, ky = (kx + 1) % 3;
    if (Comp(d, kz) < 0.f) std::swap(kx, ky);
    r.kx = kx;
    r.ky = ky;
    r.kz = kz;
    r.Sx = Comp(d, kx) / Comp(d, kz);
    r.Sy = Comp(d, ky) / Comp(d, kz);
    r.Sz = 1.0f / Comp(d, kz);
    return r;
}

bool HitTriangle(const Ray &r, const Prim &p, float tmin, float tmax, float &t, float &b1, float &b2) {
    const float3 A = p.v0 - r.o, B = p.v1 - r.o, C = p.v2 - r.o;
    const float Ax = Comp(A, r.kx) - r.Sx * Comp(A, r.kz);
    const float Ay = Comp(A, r.ky) - r.Sy * Comp(A, r.kz);
    const float Bx = Comp(B, r.kx) - r.Sx * Comp(B, r.kz);
    const float By = Comp(B, r.ky) - r.Sy * Comp(B, r.kz);
    const float Cx = Comp(C, r.kx) - r.Sx * Comp(C, r.kz);
    const float Cy = Comp(C, r.ky) - r.Sy * Comp(C, r.kz);
    float U = Cx * By - Cy * Bx, V = Ax * Cy - Ay * Cx, W = Bx * Ay - By * Ax;
    if (U == 0.f || V == 0.f || W == 0.f) {
        U = (float)((double)Cx * (double)By - (double)Cy * (double)Bx);
        V = (float)((double)Ax * (double)Cy - (double)Ay * (double)Cx);
        W = (float)((double)Bx * (double)Ay - (double)By * (double)Ax);
    }
    if ((U < 0.f || V < 0.f || W < 0.f) && (U > 0.f || V > 0.f || W > 0.f)) return false;
    const float det = U + V + W;
    if (det == 0.f) return false;
    const float Az = r.Sz * Comp(A, r.kz), Bz = r.Sz * Comp(B, r.kz), Cz = r.Sz * Comp(C, r.kz);
    const float T = U * Az + V * Bz + W * Cz;
    const float rcp = 1.0f / det;
    const float tt = T * rcp;
    if (!(tt >= tmin && tt <= tmax)) return false;
    t = tt;
    b1 = V * rcp;
    b2 = W * rcp;
    return true;
}

// Unit sphere in object space, closest-approach discriminant (Ray Tracing Gems
// ch. 7), the same arithmetic as csrc/pt_trace.h intersect_unit_sphere.
bool HitSphere(const Instance &in, const Ray &r, float tmin, float tmax, float &t) {
    const float3 f = XformPoint(in.to_object, r.o);
    const float3 od = XformVector(in.to_object, r.d);
    const float a = dot(od, od);
    const float bp = -dot(f, od);
    const float3 l = f + od * (bp / a);
    const float disc = a * (1.f - dot(l, l));
    if (disc < 0.f) return false;
    const float c = dot(f, f) - 1.f;
    const float q = bp + std::copysign(sqrtf(disc), bp);
    const float r0 = c / q, r1 = q / a;
    const float t0 = std::fmin(r0, r1), t1 = std::fmax(r0, r1);
    if (t0 >= tmin && t0 <= tmax) {
        t = t0;
        return true;
    }
    if (t1 >= tmin && t1 <= tmax) {
        t = t1;
        return true;
    }
    return false;
}

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box &b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(float3 p) {
        const float v[3] = {p.x, p.y, p.z};
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], v[k]);
            hi[k] = std::max(hi[k], v[k]);
        }
    }
    float area() const {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        if (dx < 0.f) return 0.f;
        return 2.f * (dx * dy + dy * dz + dz * dx);
    }
};

struct Node {
    Box box;
    int left = -1, right = -1;  // children, or -1
    unsigned int first = 0, count = 0;
};

// The engine's quantized BVH4 node (pupiloptixlab_amd/csrc/pt_scene.h Bvh4Node,
// 64 B), for CPU traversal of the GPU's own arrays (oracle_set_bvh4): child k's
// plane on an axis is o + q_k * s (s a power of two, one float per axis); link >= 0
// inner node, < 0 leaf with ~link = first_record << 3 | (count - 1), kQEmpty unused.
struct QNode {
    float ox, oy, oz;
    float sx;
    int32_t child[4];
    uint32_t qlo[3], qhi[3];
    float sy, sz;
};
static_assert(sizeof(QNode) == 64, "Bvh4Node layout");
constexpr int32_t kQEmpty = 0x7FFFFFFF, kQDone = 0x76543210;

struct Scene {
    unsigned int width = 0, height = 0, max_depth = 1;
    // engine BVH4 arrays (oracle_set_bvh4); empty = this file's own SAH BVH
    std::vector<QNode> q4;
    std::vector<uint32_t> q4_rec_prim;  // record -> primitive id (the record's a.w)
    int32_t q4_root = kQDone;
    float q4_bound[3] = {0.f, 0.f, 0.f};  // per axis max |o| + 512 s over q4 (engine node_bound)
    mat4x4 sample_to_camera{}, camera_to_world{};
    std::vector<Material> materials;
    std::vector<Instance> instances;
    EmitterGroup emitters;
    Emitter env_storage;
    std::vector<Prim> prims;
    std::vector<Box> prim_boxes;
    std::vector<unsigned int> order;
    std::vector<Node> nodes;

    int Build(unsigned int lo, unsigned int hi) {  // binned SAH (16 bins)
        Node n;
        Box cb;
        for (unsigned int i = lo; i < hi; i++) {
            n.box.grow(prim_boxes[order[i]]);
            const Box &b = prim_boxes[order[i]];
            cb.grow(make_float3(0.5f * (b.lo[0] + b.hi[0]), 0.5f * (b.lo[1] + b.hi[1]), 0.5f * (b.lo[2] + b.hi[2])));
        }
        const int idx = (int)nodes.size();
        nodes.push_back(n);
        const unsigned int count = hi - lo;
        if (count <= 2) {
            nodes[idx].first = lo;
            nodes[idx].count = count;
            return idx;
        }
        int best_axis = -1;
        float best_cost = INFINITY, best_split = 0.f;
        constexpr int kBins = 16;
        for (int axis = 0; axis < 3; axis++) {
            const float a0 = cb.lo[axis], a1 = cb.hi[axis];
            if (!(a1 > a0)) continue;
            Box bins[kBins];
            unsigned int cnt[kBins] = {};
            for (unsigned int i = lo; i < hi; i++) {
                const Box &b = prim_boxes[order[i]];
                const float c = 0.5f * (b.lo[axis] + b.hi[axis]);
                int bi = (int)((c - a0) / (a1 - a0) * kBins);
                bi = std::min(std::max(bi, 0), kBins - 1);
                bins[bi].grow(b);
                cnt[bi]++;
            }
            Box left_acc;
            unsigned int left_cnt = 0;
            float left_area[kBins];
            unsigned int left_n[kBins];
            for (int b = 0; b < kBins - 1; b++) {
                left_acc.grow(bins[b]);
                left_cnt += cnt[b];
                left_area[b] = left_acc.area();
                left_n[b] = left_cnt;
            }
            Box right_acc;
            unsigned int right_cnt = 0;
            for (int b = kBins - 1; b > 0; b--) {
                right_acc.grow(bins[b]);
                right_cnt += cnt[b];
                if (left_n[b - 1] == 0 || right_cnt == 0) continue;
                const float cost = left_area[b - 1] * left_n[b - 1] + right_acc.area() * right_cnt;
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = a0 + (a1 - a0) * (float)b / kBins;
                }
            }
        }
        unsigned int mid;
        if (best_axis < 0) {
            mid = lo + count / 2;
        } else {
            auto *beg = order.data() + lo, *end = order.data() + hi;
            auto *m = std::partition(beg, end, [&](unsigned int p) {
                const Box &b = prim_boxes[p];
                return 0.5f * (b.lo[best_axis] + b.hi[best_axis]) < best_split;
            });
            mid = (unsigned int)(m - order.data());
            if (mid == lo || mid == hi) mid = lo + count / 2;
        }
        const int l = Build(lo, mid);
        const int r = Build(mid, hi);
        nodes[idx].left = l;
        nodes[idx].right = r;
        return idx;
    }

    static bool BoxHit(const Box &b, const Ray &r, float tmin, float tmax) {
        float tn = tmin, tf = tmax;
        const float o[3] = {r.o.x, r.o.y, r.o.z}, id[3] = {r.idir.x, r.idir.y, r.idir.z};
        for (int k = 0; k < 3; k++) {
            float t0 = (b.lo[k] - o[k]) * id[k], t1 = (b.hi[k] - o[k]) * id[k];
            if (t0 > t1) std::swap(t0, t1);
            tn = std::max(tn, t0);
            tf = std::min(tf, t1);
        }
        return tn <= tf * 1.0000004f;  // conservative (Ize 2013)
    }

    // Child entry distances of an engine BVH4 node: the GPU's conservative
    // quantized slab test restated (pt_traverse.h visit4 / slab_error): per axis
    // t = fma(q, s * idir, fma(o_node - o_ray, idir, -/+E)),
    // E = (|o_ray| + M) * (|idir| * 2^-21), M = q4_bound (max |o| + 512 s over the nodes).
    void QVisit(const QNode &n, const Ray &r, float tmin, float tmax, float t[4]) const {
        const float o[3] = {n.ox, n.oy, n.oz}, ro[3] = {r.o.x, r.o.y, r.o.z}, id[3] = {r.idir.x, r.idir.y, r.idir.z};
        float bn[3], an[3], af[3];
        uint32_t qn[3], qf[3];
        for (int a = 0; a < 3; a++) {
            const float sc = a == 0 ? n.sx : (a == 1 ? n.sy : n.sz);
            const float A = o[a] - ro[a];
            const float e = (std::fabs(ro[a]) + q4_bound[a]) * (std::fabs(id[a]) * 0x1p-21f);
            bn[a] = sc * id[a];
            an[a] = std::fma(A, id[a], -e);
            af[a] = std::fma(A, id[a], e);
            const bool pos = id[a] >= 0.f;
            qn[a] = pos ? n.qlo[a] : n.qhi[a];
            qf[a] = pos ? n.qhi[a] : n.qlo[a];
        }
        for (int k = 0; k < 4; k++) {
            float tn = tmin, tf = tmax;
            for (int a = 0; a < 3; a++) {
                tn = std::fmax(std::fma((float)((qn[a] >> (8 * k)) & 0xFFu), bn[a], an[a]), tn);
                tf = std::fmin(std::fma((float)((qf[a] >> (8 * k)) & 0xFFu), bn[a], af[a]), tf);
            }
            t[k] = (tn <= tf && n.child[k] != kQEmpty) ? tn : INFINITY;
        }
    }
    // closest hit / any hit over the engine's BVH4: children visited near to far
    bool QTrace(const Ray &r, float tmin, float tmax, bool any, unsigned int &prim, float &t, float &b1, float &b2,
                uint64_t *nodes_visited) const {
        if (q4_root == kQDone) return false;
        bool found = false;
        unsigned int best = 0xFFFFFFFFu;
        int32_t stack[512];
        int sp = 0;
        stack[sp++] = q4_root;
        while (sp) {
            const int32_t link = stack[--sp];
            if (link < 0) {
                const uint32_t first = ((uint32_t)~link) >> 3, count = (((uint32_t)~link) & 7u) + 1u;
                for (uint32_t i = first; i < first + count; i++) {
                    const Prim &p = prims[q4_rec_prim[i]];
                    float tt, u = 0.f, v = 0.f;
                    const bool hit = p.sphere ? HitSphere(instances[p.inst], r, tmin, tmax, tt)
                                              : HitTriangle(r, p, tmin, tmax, tt, u, v);
                    if (hit && any) return true;
                    if (hit && (tt < tmax || p.id < best)) {
                        tmax = tt;
                        best = p.id;
                        t = tt;
                        b1 = u;
                        b2 = v;
                        found = true;
                    }
                }
                continue;
            }
            if (nodes_visited) (*nodes_visited)++;
            const QNode &n = q4[(size_t)link];
            float tk[4];
            QVisit(n, r, tmin, tmax, tk);
            int order[4] = {0, 1, 2, 3};  // insertion sort, far to near
            for (int a = 1; a < 4; a++)
                for (int b = a; b > 0 && tk[order[b]] > tk[order[b - 1]]; b--) std::swap(order[b], order[b - 1]);
            for (int j = 0; j < 4; j++)  // farthest first, the nearest ends on top
                if (tk[order[j]] != INFINITY && sp < 512) stack[sp++] = n.child[order[j]];
        }
        prim = best;
        return found;
    }

    // optixTrace closest hit; ties broken by the smaller primitive id
    bool Closest(const Ray &r, float tmin, float tmax, unsigned int &prim, float &t, float &b1, float &b2,
                 uint64_t *nodes_visited = nullptr) const {
        if (!q4_rec_prim.empty()) return QTrace(r, tmin, tmax, false, prim, t, b1, b2, nodes_visited);
        bool found = false;
        unsigned int best = 0xFFFFFFFFu;
        int stack[128];
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            const Node &n = nodes[stack[--sp]];
            if (nodes_visited) (*nodes_visited)++;
            if (!BoxHit(n.box, r, tmin, tmax)) continue;
            if (n.left < 0) {
                for (unsigned int i = n.first; i < n.first + n.count; i++) {
                    const Prim &p = prims[order[i]];
                    float tt, u = 0.f, v = 0.f;
                    const bool hit = p.sphere ? HitSphere(instances[p.inst], r, tmin, tmax, tt)
                                              : HitTriangle(r, p, tmin, tmax, tt, u, v);
                    if (hit && (tt < tmax || p.id < best)) {
                        tmax = tt;
                        best = p.id;
                        t = tt;
                        b1 = u;
                        b2 = v;
                        found = true;
                    }
                }
            } else {
                stack[sp++] = n.right;
                stack[sp++] = n.left;
            }
        }
        prim = best;
        return found;
    }
    // shadow rays: TERMINATE_ON_FIRST_HIT
    bool Occluded(const Ray &r, float tmin, float tmax) const {
        if (!q4_rec_prim.empty()) {
            unsigned int prim;
            float t, b1, b2;
            return QTrace(r, tmin, tmax, true, prim, t, b1, b2, nullptr);
        }
        int stack[128];
        int sp = 0;
        stack[sp++] = 0;
        while (sp) {
            const Node &n = nodes[stack[--sp]];
            if (!BoxHit(n.box, r, tmin, tmax)) continue;
            if (n.left < 0) {
                for (unsigned int i = n.first; i < n.first + n.count; i++) {
                    const Prim &p = prims[order[i]];
                    float tt, u, v;
                    if (p.sphere ? HitSphere(instances[p.inst], r, tmin, tmax, tt) : HitTriangle(r, p, tmin, tmax, tt, u, v))
                        return true;
                }
            } else {
                stack[sp++] = n.right;
                stack[sp++] = n.left;
            }
        }
        return false;
    }

    // __closesthit__default + Geometry::GetHitLocalGeometry (geometry.h:272-320)
    void HitGeometry(unsigned int prim_id, float t, float b1, float b2, float3 ray_o, float3 ray_d,
                     LocalGeometry &ret, int &emitter_index, unsigned int &material) const {
        const Prim &p = prims[prim_id];
        const Instance &in = instances[p.inst];
        const unsigned int local = p.id - in.prim_offset;
        if (p.sphere) {
            ret.position = ray_o + t * ray_d;
            const float3 local_pos = XformPoint(in.to_object, ret.position);
            ret.texcoord = GetSphereTexcoord(normalize(local_pos - make_float3(0.f)));
            ret.normal = normalize(XformNormal(in.to_object, local_pos - make_float3(0.f)));
            if (in.flip_normals) ret.normal *= -1.f;
        } else {
            const pupil_shape &s = *in.shape;
            const unsigned int v0 = s.indices[3 * local], v1 = s.indices[3 * local + 1], v2 = s.indices[3 * local + 2];
            auto P = [&](unsigned int v) {
                return make_float3(s.positions[3 * v], s.positions[3 * v + 1], s.positions[3 * v + 2]);
            };
            const float3 p0 = P(v0), p1 = P(v1), p2 = P(v2);
            ret.position = (1.f - b1 - b2) * p0 + b1 * p1 + b2 * p2;
            ret.position = XformPoint(in.to_world, ret.position);
            if (s.normals) {
                auto N = [&](unsigned int v) {
                    return make_float3(s.normals[3 * v], s.normals[3 * v + 1], s.normals[3 * v + 2]);
                };
                ret.normal = (1.f - b1 - b2) * N(v0) + b1 * N(v1) + b2 * N(v2);
            } else {
                ret.normal = cross(p1 - p0, p2 - p0);
            }
            ret.normal = normalize(XformNormal(in.to_object, ret.normal));
            if (in.flip_normals) ret.normal *= -1.f;
            if (s.texcoords) {
                auto T = [&](unsigned int v) { return make_float2(s.texcoords[2 * v], s.texcoords[2 * v + 1]); };
                ret.texcoord = T(v0) * (1.f - b1 - b2) + T(v1) * b1 + T(v2) * b2;
                if (in.flip_tex_coords) ret.texcoord.y = 1.f - ret.texcoord.y;
            }
        }
        const Material &m = materials[in.material];
        if (dot(-ray_d, ret.normal) < 0.f && m.twosided) ret.normal = -ret.normal;
        emitter_index = in.emitter_index_offset >= 0 ? in.emitter_index_offset + (int)local : -1;
        material = in.material;
    }
};

bool LoadScene(const pupil_scene_desc &d, Scene &sc) {
    sc.width = d.width;
    sc.height = d.height;
    sc.max_depth = d.max_depth ? d.max_depth : 1;
    auto row = [](const float *m, int r) { return make_float4(m[4 * r], m[4 * r + 1], m[4 * r + 2], m[4 * r + 3]); };
    sc.sample_to_camera = {row(d.sample_to_camera, 0), row(d.sample_to_camera, 1), row(d.sample_to_camera, 2),
                           row(d.sample_to_camera, 3)};
    sc.camera_to_world = {row(d.camera_to_world, 0), row(d.camera_to_world, 1), row(d.camera_to_world, 2),
                          row(d.camera_to_world, 3)};
    for (unsigned int i = 0; i < d.num_materials; i++) sc.materials.push_back(LoadMaterial(d.materials[i]));
    if (sc.materials.empty()) sc.materials.push_back(Material{});
    unsigned int prim_offset = 0;
    for (unsigned int i = 0; i < d.num_instances; i++) {
        const pupil_instance &src = d.instances[i];
        Instance in;
        std::memcpy(in.to_world, src.to_world, sizeof(in.to_world));
        std::memcpy(in.to_object, src.to_object, sizeof(in.to_object));
        in.shape = &d.shapes[src.shape];
        in.kind = in.shape->kind;
        in.material = src.material;
        in.flip_normals = src.flip_normals;
        in.flip_tex_coords = src.flip_tex_coords;
        in.emitter_index_offset = src.emitter_offset;
        in.prim_offset = prim_offset;
        sc.instances.push_back(in);
        const unsigned int n = in.kind == PUPIL_SHAPE_SPHERE ? 1u : in.shape->num_faces;
        for (unsigned int f = 0; f < n; f++) {
            Prim p;
            p.id = prim_offset + f;
            p.inst = i;
            p.sphere = in.kind == PUPIL_SHAPE_SPHERE;
            Box b;
            if (p.sphere) {
                const float *m = in.to_world;
                const float ex = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]) * 1.001f;
                const float ey = std::sqrt(m[4] * m[4] + m[5] * m[5] + m[6] * m[6]) * 1.001f;
                const float ez = std::sqrt(m[8] * m[8] + m[9] * m[9] + m[10] * m[10]) * 1.001f;
                b.grow(make_float3(m[3] - ex, m[7] - ey, m[11] - ez));
                b.grow(make_float3(m[3] + ex, m[7] + ey, m[11] + ez));
                p.v0 = p.v1 = p.v2 = make_float3(m[3], m[7], m[11]);
            } else {
                const pupil_shape &s = *in.shape;
                auto W = [&](unsigned int v) {
                    return XformPoint(in.to_world,
                                      make_float3(s.positions[3 * v], s.positions[3 * v + 1], s.positions[3 * v + 2]));
                };
                p.v0 = W(s.indices[3 * f]);
                p.v1 = W(s.indices[3 * f + 1]);
                p.v2 = W(s.indices[3 * f + 2]);
                b.grow(p.v0);
                b.grow(p.v1);
                b.grow(p.v2);
            }
            sc.prims.push_back(p);
            sc.prim_boxes.push_back(b);
        }
        prim_offset += n;
    }
    sc.order.resize(sc.prims.size());
    for (size_t i = 0; i < sc.order.size(); i++) sc.order[i] = (unsigned int)i;
    sc.nodes.reserve(2 * sc.prims.size());
    if (!sc.prims.empty()) sc.Build(0, (unsigned int)sc.prims.size());
    for (unsigned int i = 0; i < d.num_area_emitters; i++) sc.emitters.areas.push_back(LoadEmitter(d.area_emitters[i]));
    if (d.env && d.env->type != PUPIL_EMITTER_NONE) {
        sc.env_storage = LoadEmitter(*d.env);
        sc.emitters.env = &sc.env_storage;
    }
    return true;
}

struct Stats {
    std::atomic<uint64_t> primary{0}, extension{0}, shadow{0};
};

// ------------------------------------------------------------------ __raygen__main (main.cu:36-194)
struct FrameOut {
    float *accum;  // float4 per output pixel
    float *albedo, *normal, *test;
};

void RenderPixel(const Scene &sc, unsigned int pixel_index, unsigned int out_index, unsigned int random_seed,
                 unsigned int sample_cnt, bool accumulated_flag, unsigned int max_depth, bool write_aov,
                 const FrameOut &out, uint64_t counts[4]) {
    const unsigned int w = sc.width, h = sc.height;
    const unsigned int ix = pixel_index % w, iy = pixel_index / w;
    float3 radiance = make_float3(0.f), env_radiance = make_float3(0.f), throughput = make_float3(1.f);
    float env_pdf = 0.f;
    Random random;
    random.Init(4, pixel_index, random_seed);
    const float jx = random.Next();
    const float jy = random.Next();
    const float2 subpixel = make_float2((static_cast<float>(ix) + jx) / static_cast<float>(w),
                                        (static_cast<float>(iy) + jy) / static_cast<float>(h));
    const float4 point_on_film = make_float4(subpixel.x, subpixel.y, 0.f, 1.f);
    float4 d = sc.sample_to_camera * point_on_film;
    d /= d.w;
    d.w = 0.f;
    d = normalize(d);
    const float4 dw = sc.camera_to_world * d;
    float3 ray_direction = normalize(make_float3(dw.x, dw.y, dw.z));
    float3 ray_origin = make_float3(sc.camera_to_world.r0.w, sc.camera_to_world.r1.w, sc.camera_to_world.r2.w);

    // hit record persists across traces (stale texcoord semantics)
    LocalGeometry geo;
    LocalBsdf bsdf;
    int emitter_index = -1;
    bool done = false;
    auto trace = [&](float3 o, float3 dir) {
        const Ray r = MakeRay(o, dir);
        unsigned int prim;
        float t, b1, b2;
        if (!sc.Closest(r, 0.001f, 1e16f, prim, t, b1, b2)) {
            if (sc.emitters.env) {  // __miss__default
                const float3 nd = normalize(dir);
                LocalGeometry env_local;
                env_local.position = o + nd;
                EmitEvalRecord er;
                sc.emitters.env->Eval(er, env_local, o);
                env_radiance = er.radiance;
                env_pdf = er.pdf;
            }
            done = true;
            return;
        }
        // prim is the global id; prims are stored in id order
        unsigned int mat;
        sc.HitGeometry(prim, t, b1, b2, o, dir, geo, emitter_index, mat);
        bsdf = GetLocalBsdf(sc.materials[mat], geo.texcoord);
    };
    trace(ray_origin, ray_direction);
    counts[0]++;

    if (!done) {
        if (emitter_index >= 0) radiance += sc.emitters.areas[emitter_index].GetRadiance(geo.texcoord);
        if (write_aov) {
            const float3 al = bsdf.GetAlbedo();
            out.albedo[3 * out_index] = al.x, out.albedo[3 * out_index + 1] = al.y, out.albedo[3 * out_index + 2] = al.z;
            out.normal[3 * out_index] = geo.normal.x, out.normal[3 * out_index + 1] = geo.normal.y,
            out.normal[3 * out_index + 2] = geo.normal.z;
        }
    } else if (write_aov) {
        for (int k = 0; k < 3; k++) out.albedo[3 * out_index + k] = out.normal[3 * out_index + k] = 0.f;
    }
    const float test = random.Next();
    if (write_aov) out.test[out_index] = test;

    unsigned int depth = 0;
    while (!done) {
        ++depth;
        if (depth >= max_depth) break;
        float rr = depth > 2 ? 0.95 : 1.0;
        if (random.Next() > rr) break;
        throughput /= rr;
        counts[3]++;  // the reference traces its shadow ray here unconditionally (main.cu:119-123)
        {
            const Emitter *emitter = sc.emitters.SelectOneEmiiter(random.Next());
            EmitterSampleRecord esr;
            const float2 xi = random.Next2();
            if (emitter) {
                emitter->SampleDirect(esr, geo, xi);
                BsdfSamplingRecord eval_record;
                eval_record.wi = ToLocal(esr.wi, geo.normal);
                eval_record.wo = ToLocal(-ray_direction, geo.normal);
                eval_record.sampler = &random;
                bsdf.Eval(eval_record);
                const float3 f = eval_record.f;
                const float pdf = eval_record.pdf;
                // Reordered from main.cu:119-141, radiance-equivalent: the reference traces the
                // shadow ray first and calls Eval only when unoccluded, but Eval (GetBsdf +
                // GetPdf) draws no random numbers (optix_material.h:57-62; only Sample does,
                // bsdf/*.h), so testing occlusion only for a non-zero contribution changes no
                // pixel and no later RNG draw.  counts[2] = shadow rays traced here, counts[3] =
                // the reference's unconditional count.
                if (!IsZero(f * esr.pdf)) {
                    const float NoL = dot(geo.normal, esr.wi);
                    if (NoL > 0.f) {
                        counts[2]++;
                        const bool occluded = sc.Occluded(MakeRay(geo.position, esr.wi), 0.001f, esr.distance - 0.001f);
                        if (!occluded) {
                            float mis = esr.is_delta ? 1.f : MISWeight(esr.pdf, pdf);
                            esr.pdf *= emitter->select_probability;
                            radiance += throughput * esr.radiance * f * NoL * mis / esr.pdf;
                        }
                    }
                }
            }
        }
        {
            BsdfSamplingRecord bsdf_sample_record;
            bsdf_sample_record.wo = ToLocal(-ray_direction, geo.normal);
            bsdf_sample_record.sampler = &random;
            bsdf.Sample(bsdf_sample_record);
            if (IsZero(bsdf_sample_record.f * absf(bsdf_sample_record.wi.z)) || IsZero(bsdf_sample_record.pdf)) break;
            throughput *= bsdf_sample_record.f * absf(bsdf_sample_record.wi.z) / bsdf_sample_record.pdf;
            ray_origin = geo.position;
            ray_direction = ToWorld(bsdf_sample_record.wi, geo.normal);
            const LocalGeometry prev_geo = geo;
            (void)prev_geo;
            trace(ray_origin, ray_direction);
            counts[1]++;
            if (done) {
                float mis = MISWeight(bsdf_sample_record.pdf, env_pdf);
                env_radiance *= throughput * mis;
                break;
            }
            if (emitter_index >= 0) {
                const Emitter &emitter = sc.emitters.areas[emitter_index];
                EmitEvalRecord emit_record;
                emitter.Eval(emit_record, geo, ray_origin);
                if (!IsZero(emit_record.pdf)) {
                    float mis = (bsdf_sample_record.sampled_type & Delta)
                                    ? 1.f
                                    : MISWeight(bsdf_sample_record.pdf, emit_record.pdf * emitter.select_probability);
                    radiance += throughput * emit_record.radiance * mis;
                }
            }
        }
    }
    radiance += env_radiance;
    float *acc = out.accum + 4 * out_index;
    if (accumulated_flag && sample_cnt > 0) {
        const float t = 1.f / (sample_cnt + 1.f);
        const float3 pre = make_float3(acc[0], acc[1], acc[2]);
        radiance = lerp(pre, radiance, t);
    }
    acc[0] = radiance.x, acc[1] = radiance.y, acc[2] = radiance.z, acc[3] = 1.f;
}

}  // namespace oracle

extern "C" {

struct oracle_stats {
    uint64_t primary_rays, extension_rays, shadow_rays;
    double seconds;
    uint32_t threads;
    uint64_t shadow_rays_reference;  // loop iterations reaching main.cu:119-123
};

typedef struct oracle_scene oracle_scene;

oracle_scene *oracle_scene_create(const pupil_scene_desc *d) {
    auto *sc = new oracle::Scene();
    oracle::LoadScene(*d, *sc);
    return reinterpret_cast<oracle_scene *>(sc);
}

void oracle_scene_destroy(oracle_scene *s) { delete reinterpret_cast<oracle::Scene *>(s); }

// Traverse the engine's own BVH4 (pupil_pt_export_bvh4: 64-B nodes, 12-float world
// records whose a.w holds the primitive id | sphere bit) instead of this file's BVH;
// the primitives are still tested on this file's data.  num_records = 0 restores it.
int oracle_set_bvh4(oracle_scene *s, uint32_t num_nodes, const void *nodes, uint32_t num_records,
                    const float *records, int32_t root_link) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    sc.q4.assign(reinterpret_cast<const oracle::QNode *>(nodes), reinterpret_cast<const oracle::QNode *>(nodes) + num_nodes);
    sc.q4_rec_prim.resize(num_records);
    for (uint32_t i = 0; i < num_records; i++) {
        uint32_t bits;
        std::memcpy(&bits, &records[12 * i + 3], 4);
        if (bits == 0xFFFFFFFFu) {  // a hole slot between leaves (no leaf names it)
            sc.q4_rec_prim[i] = 0xFFFFFFFFu;
            continue;
        }
        bits &= 0x7FFFFFFFu;  // sphere bit
        if (bits >= sc.prims.size()) return -1;
        sc.q4_rec_prim[i] = bits;
    }
    sc.q4_root = root_link;
    sc.q4_bound[0] = sc.q4_bound[1] = sc.q4_bound[2] = 0.f;
    for (const auto &n : sc.q4) {
        sc.q4_bound[0] = std::fmax(sc.q4_bound[0], std::fabs(n.ox) + 512.f * n.sx);
        sc.q4_bound[1] = std::fmax(sc.q4_bound[1], std::fabs(n.oy) + 512.f * n.sy);
        sc.q4_bound[2] = std::fmax(sc.q4_bound[2], std::fabs(n.oz) + 512.f * n.sz);
    }
    for (const auto &n : sc.q4)
        for (int k = 0; k < 4; k++)
            if (n.child[k] >= 0 && n.child[k] != oracle::kQEmpty && (uint32_t)n.child[k] >= num_nodes) return -1;
    return 0;
}

// spp consecutive OnRun frames (pt_pass.cpp:51-56) over the given pixels.
// pixels == NULL renders the whole image (out index = pixel index).
int oracle_render(oracle_scene *s, uint32_t random_seed, uint32_t sample_cnt, uint32_t spp, uint32_t max_depth,
                  uint32_t accumulate, const uint32_t *pixels, uint32_t num_pixels, float *accum, float *albedo,
                  float *normal, float *test, int threads, oracle_stats *stats) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    if (!pixels) num_pixels = sc.width * sc.height;
    if (max_depth == 0) max_depth = sc.max_depth;
    if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
    std::vector<float> scratch_aov;
    if (!albedo || !normal || !test) {
        scratch_aov.resize((size_t)num_pixels * 7);
        albedo = scratch_aov.data();
        normal = albedo + 3 * (size_t)num_pixels;
        test = normal + 3 * (size_t)num_pixels;
    }
    oracle::FrameOut out{accum, albedo, normal, test};
    std::atomic<uint32_t> next{0};
    std::atomic<uint64_t> c0{0}, c1{0}, c2{0}, c3{0};
    const auto t0 = std::chrono::steady_clock::now();
    auto worker = [&]() {
        uint64_t counts[4] = {0, 0, 0, 0};
        const uint32_t chunk = 64;
        while (true) {
            const uint32_t b = next.fetch_add(chunk);
            if (b >= num_pixels) break;
            for (uint32_t i = b; i < std::min(num_pixels, b + chunk); i++) {
                const uint32_t pix = pixels ? pixels[i] : i;
                for (uint32_t f = 0; f < spp; f++)
                    oracle::RenderPixel(sc, pix, i, random_seed + f, sample_cnt + (accumulate ? f : 0), accumulate != 0,
                                        max_depth, f + 1 == spp, out, counts);
            }
        }
        c0 += counts[0];
        c1 += counts[1];
        c2 += counts[2];
        c3 += counts[3];
    };
    std::vector<std::thread> pool;
#if defined(PUPIL_FASTMATH_EMULATION)
    // -ftz=true of -use_fast_math: denormal results flush to zero, denormal inputs read as zero
    auto ftz_worker = [&]() {
        unsigned csr;
        __asm__ volatile("stmxcsr %0" : "=m"(csr));
        csr |= 0x8040u;  // FTZ | DAZ
        __asm__ volatile("ldmxcsr %0" : : "m"(csr));
        worker();
    };
    for (int t = 0; t < threads; t++) pool.emplace_back(ftz_worker);
#else
    for (int t = 0; t < threads; t++) pool.emplace_back(worker);
#endif
    for (auto &t : pool) t.join();
    const auto t1 = std::chrono::steady_clock::now();
    if (stats) {
        stats->primary_rays = c0;
        stats->extension_rays = c1;
        stats->shadow_rays = c2;
        stats->seconds = std::chrono::duration<double>(t1 - t0).count();
        stats->threads = (uint32_t)threads;
        stats->shadow_rays_reference = c3;
    }
    return 0;
}

// ---- known-answer helpers for tests
void oracle_rng_sequence(uint32_t pixel, uint32_t seed, uint32_t n, float *out, uint32_t *states) {
    oracle::Random r;
    r.Init(4, pixel, seed);
    for (uint32_t i = 0; i < n; i++) {
        out[i] = r.Next();
        if (states) states[i] = r.GetSeed();
    }
}

// camera ray of (pixel, seed): origin xyz, dir xyz
void oracle_camera_ray(oracle_scene *s, uint32_t pixel, uint32_t seed, float *o6) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    using namespace oracle;
    Random random;
    random.Init(4, pixel, seed);
    const float jx = random.Next(), jy = random.Next();
    const unsigned int ix = pixel % sc.width, iy = pixel / sc.width;
    const float4 pf = make_float4((static_cast<float>(ix) + jx) / static_cast<float>(sc.width),
                                  (static_cast<float>(iy) + jy) / static_cast<float>(sc.height), 0.f, 1.f);
    float4 d = sc.sample_to_camera * pf;
    d /= d.w;
    d.w = 0.f;
    d = normalize(d);
    const float4 dw = sc.camera_to_world * d;
    const float3 dir = normalize(make_float3(dw.x, dw.y, dw.z));
    o6[0] = sc.camera_to_world.r0.w, o6[1] = sc.camera_to_world.r1.w, o6[2] = sc.camera_to_world.r2.w;
    o6[3] = dir.x, o6[4] = dir.y, o6[5] = dir.z;
}

// closest hits for n rays (o,d packed 6 floats); out: t, b1, b2, prim id bits (0xFFFFFFFF miss)
void oracle_closest(oracle_scene *s, uint32_t n, const float *rays, float *out, int brute_force) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    using namespace oracle;
    for (uint32_t i = 0; i < n; i++) {
        const Ray r = MakeRay(make_float3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]),
                              make_float3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]));
        unsigned int prim = 0xFFFFFFFFu;
        float t = -1.f, b1 = 0.f, b2 = 0.f;
        bool hit = false;
        if (brute_force) {
            float tmax = 1e16f;
            for (const Prim &p : sc.prims) {
                float tt, u = 0.f, v = 0.f;
                const bool h = p.sphere ? HitSphere(sc.instances[p.inst], r, 0.001f, tmax, tt)
                                        : HitTriangle(r, p, 0.001f, tmax, tt, u, v);
                if (h && (tt < tmax || p.id < prim)) {
                    tmax = tt;
                    prim = p.id;
                    t = tt;
                    b1 = u;
                    b2 = v;
                    hit = true;
                }
            }
        } else {
            hit = sc.Closest(r, 0.001f, 1e16f, prim, t, b1, b2);
        }
        uint32_t bits = hit ? prim : 0xFFFFFFFFu;
        out[4 * i] = hit ? t : -1.f;
        out[4 * i + 1] = b1;
        out[4 * i + 2] = b2;
        std::memcpy(&out[4 * i + 3], &bits, 4);
    }
}

// one BSDF Sample + Eval on a material of the scene: out = wi(3), f(3), pdf, type, eval f(3), eval pdf
void oracle_bsdf(oracle_scene *s, uint32_t material, float u, float v, const float *wo, const float *wi_eval,
                 uint32_t rng_seed, float *out) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    using namespace oracle;
    LocalBsdf l = GetLocalBsdf(sc.materials[material], make_float2(u, v));
    Random r;
    r.Init(4, rng_seed, 0);
    BsdfSamplingRecord rec;
    rec.wo = make_float3(wo[0], wo[1], wo[2]);
    rec.sampler = &r;
    l.Sample(rec);
    out[0] = rec.wi.x, out[1] = rec.wi.y, out[2] = rec.wi.z;
    out[3] = rec.f.x, out[4] = rec.f.y, out[5] = rec.f.z;
    out[6] = rec.pdf;
    out[7] = (float)rec.sampled_type;
    BsdfSamplingRecord ev;
    ev.wo = rec.wo;
    ev.wi = make_float3(wi_eval[0], wi_eval[1], wi_eval[2]);
    ev.sampler = &r;
    l.Eval(ev);
    out[8] = ev.f.x, out[9] = ev.f.y, out[10] = ev.f.z;
    out[11] = ev.pdf;
}

// one SampleDirect of area emitter `emitter` (env when emitter == num areas) from a shading point
// (emitter.h / area.h / sphere.h / env.h): out = wi(3), pdf, distance, radiance(3)
int oracle_emitter_sample(oracle_scene *s, uint32_t emitter, const float *pos, const float *nrm, float x0, float x1,
                          float *out) {
    auto &sc = *reinterpret_cast<oracle::Scene *>(s);
    using namespace oracle;
    const Emitter *e = emitter < sc.emitters.areas.size() ? &sc.emitters.areas[emitter] : sc.emitters.env;
    if (!e) return -1;
    LocalGeometry g;
    g.position = make_float3(pos[0], pos[1], pos[2]);
    g.normal = make_float3(nrm[0], nrm[1], nrm[2]);
    EmitterSampleRecord r;
    e->SampleDirect(r, g, make_float2(x0, x1));
    out[0] = r.wi.x, out[1] = r.wi.y, out[2] = r.wi.z;
    out[3] = r.pdf;
    out[4] = r.distance;
    out[5] = r.radiance.x, out[6] = r.radiance.y, out[7] = r.radiance.z;
    return 0;
}

// host evaluation of the probe pupil_debug_math runs on the device
void oracle_math(uint32_t n, const float *x, const float *y2, float *out) {
    for (uint32_t i = 0; i < n; i++) {
        const float a = x[i], b = y2[i];
        out[6 * i + 0] = pupil_dm::dm_sin(a);
        out[6 * i + 1] = pupil_dm::dm_cos(a);
        out[6 * i + 2] = pupil_dm::dm_acos(std::fmin(std::fmax(a, -1.f), 1.f));
        out[6 * i + 3] = pupil_dm::dm_atan2(a, b);
        out[6 * i + 4] = sqrtf(std::fabs(a));
        out[6 * i + 5] = 1.0f / a;
    }
}

uint32_t oracle_num_prims(oracle_scene *s) { return (uint32_t) reinterpret_cast<oracle::Scene *>(s)->prims.size(); }

}  // extern "C"
