// pt_shading.h — the per-hit mathematics of the path tracer, written
// branch-flattened for the wavefront shade kernels: RNG, texture lookup,
// sampling helpers, Fresnel/GGX, the seven BSDFs and the emitters.
//
// Every function states the reference lines it reproduces; expression
// evaluation order is kept identical to the reference so the CPU oracle
// (oracle/, an independent restatement) agrees bit for bit.
#pragma once

#include "pt_scene.h"

namespace pupil {

using pupil_dm::dm_acos;
using pupil_dm::dm_atan2;
using pupil_dm::dm_cos;
using pupil_dm::dm_sin;
using pupil_dm::dm_sincos;

// ----------------------------------------------------------------- RNG
// cuda::Random (framework/cuda/random.h:14-40): TEA-4 seeding, LCG stepping.
PT_HD uint32_t rng_init(uint32_t val0, uint32_t val1) {
    uint32_t v0 = val0, v1 = val1, s0 = 0;
    for (uint32_t n = 0; n < 4; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
PT_HD float rng_next(uint32_t &s) {
    s = 1664525u * s + 1013904223u;
    return (float)(s & 0x00FFFFFFu) / 16777216.0f;
}

// ----------------------------------------------------------------- textures
// cuda::Texture::Sample (framework/cuda/texture.h:33-57)
PT_D vec3 tex_sample(const DevTexture &t, vec2 uv) {
    if (t.type == 0u) return v3(t.c0[0], t.c0[1], t.c0[2]);
    const vec4 tc = v4(uv.x, uv.y, 0.f, 1.f);
    float tx = dot(v4(t.r0[0], t.r0[1], t.r0[2], t.r0[3]), tc);
    float ty = dot(v4(t.r1[0], t.r1[1], t.r1[2], t.r1[3]), tc);
    if (t.type == 2u) {
        tx = tx - (tx > 0.f ? floorf(tx) : ceilf(tx));
        ty = ty - (ty > 0.f ? floorf(ty) : ceilf(ty));
        if (tx < 0.f) tx += 1.f;
        if (ty < 0.f) ty += 1.f;
        bool p1;
        if (tx > 0.5f)
            p1 = ty > 0.5f;
        else
            p1 = !(ty > 0.5f);
        return p1 ? v3(t.c0[0], t.c0[1], t.c0[2]) : v3(t.c1[0], t.c1[1], t.c1[2]);
    }
    // bitmap: normalized coords, wrap addressing (CudaTextureManager defaults,
    // cuda/texture.cpp:82-88); point or bilinear with 8-bit weights like tex2D.
    if (t.data == nullptr || t.width == 0 || t.height == 0) return v3(0.f);
    const int W = (int)t.width, H = (int)t.height;
    auto wrapi = [](int i, int n) { int r = i % n; return r < 0 ? r + n : r; };
    if (t.filter == 0u) {
        int ix = (int)floorf(tx * (float)W);
        int iy = (int)floorf(ty * (float)H);
        float4 c = t.data[wrapi(iy, H) * W + wrapi(ix, W)];
        return v3(c.x, c.y, c.z);
    }
    float fx = tx * (float)W - 0.5f;
    float fy = ty * (float)H - 0.5f;
    float x0f = floorf(fx), y0f = floorf(fy);
    // tex2D linear filtering keeps 8 fractional bits of the weights
    float ax = floorf((fx - x0f) * 256.f + 0.5f) / 256.f;
    float ay = floorf((fy - y0f) * 256.f + 0.5f) / 256.f;
    int x0 = wrapi((int)x0f, W), y0 = wrapi((int)y0f, H);
    int x1 = wrapi((int)x0f + 1, W), y1 = wrapi((int)y0f + 1, H);
    float4 c00 = t.data[y0 * W + x0], c10 = t.data[y0 * W + x1];
    float4 c01 = t.data[y1 * W + x0], c11 = t.data[y1 * W + x1];
    vec3 a = v3(c00.x, c00.y, c00.z) * (1.f - ax) + v3(c10.x, c10.y, c10.z) * ax;
    vec3 b = v3(c01.x, c01.y, c01.z) * (1.f - ax) + v3(c11.x, c11.y, c11.z) * ax;
    return a * (1.f - ay) + b * ay;
}

// ----------------------------------------------------------------- sampling helpers
// optix/util.h:33-36
PT_HD vec3 uniform_sample_triangle(float u1, float u2) {
    const float s = sqrtf(u1);
    return v3(1.f - s, s * (1.f - u2), u2 * s);
}
// optix/util.h:38-43
PT_HD vec3 uniform_sample_sphere(float u1, float u2) {
    const float z = 1.f - 2.f * u1;
    const float sin_theta = sqrtf(fmaxf(0.f, 1.f - z * z));
    const float phi = 2.f * kPi * u2;
    float s, c;
    dm_sincos(phi, s, c);
    return v3(sin_theta * c, sin_theta * s, z);
}
// optix/util.h:45-54
PT_HD vec3 cosine_sample_hemisphere(float u1, float u2) {
    const float sin_theta = sqrtf(u1);
    const float phi = 2.0f * kPi * u2;
    float s, c;
    dm_sincos(phi, s, c);
    return v3(sin_theta * c, sin_theta * s, sqrtf(fmaxf(0.f, 1.f - sin_theta * sin_theta)));
}
// optix/util.h:55-57
PT_HD float cosine_hemisphere_pdf(vec3 v) { return v.z > 0.f ? k1OverPi * v.z : 0.f; }
// optix/util.h:59-72
PT_HD vec3 uniform_sample_hemisphere(float u1, float u2) {
    const float z = 1.f - 2.f * u1;
    const float sin_theta = sqrtf(fmaxf(0.f, 1.f - z * z));
    const float phi = 2.0f * kPi * u2;
    float s, c;
    dm_sincos(phi, s, c);
    return v3(sin_theta * c, sin_theta * s, fabs_(z));
}
PT_HD float uniform_hemisphere_pdf(vec3 v) { return v.z > 0.f ? k1OverPi * 0.5f : 0.f; }
// optix/util.h:74-92
PT_HD vec3 reflect_local(vec3 v) { return v3(-v.x, -v.y, v.z); }
PT_HD vec3 reflect_n(vec3 v, vec3 n) { return -v + 2.f * dot(v, n) * n; }
PT_HD vec3 refract_local(vec3 v, float cos_theta_t, float eta) {
    const float scale = -(cos_theta_t < 0.f ? 1.f / eta : eta);
    return normalize(v3(scale * v.x, scale * v.y, cos_theta_t));
}
PT_HD vec3 refract_n(vec3 v, vec3 n, float cos_theta_t, float eta) {
    if (cos_theta_t < 0.f) eta = 1.f / eta;
    return n * (dot(v, n) * eta + cos_theta_t) - v * eta;
}
// optix/util.h:95-115 (Duff et al. ONB)
PT_HD void build_onb(vec3 n, vec3 &b1, vec3 &b2) {
    const float sign = copysignf(1.f, n.z);
    const float a = -1.f / (sign + n.z);
    const float b = n.x * n.y * a;
    b1 = v3(1.f + sign * n.x * n.x * a, sign * b, -sign * n.x);
    b2 = v3(b, sign + n.y * n.y * a, -n.y);
}
PT_HD vec3 to_local(vec3 v, vec3 n) {
    vec3 b1, b2;
    build_onb(n, b1, b2);
    return v3(dot(v, b1), dot(v, b2), dot(v, n));
}
PT_HD vec3 to_world(vec3 v, vec3 n) {
    vec3 b1, b2;
    build_onb(n, b1, b2);
    return b1 * v.x + b2 * v.y + n * v.z;
}
// optix/util.h:117-128
PT_HD vec2 sphere_texcoord(vec3 p) {
    float phi = dm_atan2(p.y, p.x);
    phi = phi < 0.f ? phi + kPi * 2.f : phi;
    const float theta = dm_acos(p.z);
    return v2(phi * k1OverPi * 0.5f, theta * k1OverPi);
}

// ----------------------------------------------------------------- Fresnel (material/fresnel.h)
PT_HD float fresnel_dielectric(float eta, float cos_theta_i, float &cos_theta_t) {
    const float scale = cos_theta_i > 0.f ? 1.f / eta : eta;
    const float cos_theta_t2 = 1.f - (1.f - cos_theta_i * cos_theta_i) * (scale * scale);
    if (cos_theta_t2 <= 0.0f) {
        cos_theta_t = 0.0f;
        return 1.0f;
    }
    const float o_cos_theta_i = cos_theta_i;
    cos_theta_i = fabs_(cos_theta_i);
    cos_theta_t = sqrtf(fmaxf(0.f, cos_theta_t2));
    const float rs = (cos_theta_i - eta * cos_theta_t) / (cos_theta_i + eta * cos_theta_t);
    const float rp = (eta * cos_theta_i - cos_theta_t) / (eta * cos_theta_i + cos_theta_t);
    cos_theta_t = o_cos_theta_i > 0.f ? -cos_theta_t : cos_theta_t;
    return 0.5f * (rs * rs + rp * rp);
}
PT_HD float fresnel_dielectric(float eta, float cos_theta_i) {
    float c;
    return fresnel_dielectric(eta, cos_theta_i, c);
}
PT_HD float fresnel_conductor1(float eta, float k, float cos_theta_i) {
    const float cos_theta_i2 = cos_theta_i * cos_theta_i;
    const float sin_theta_i2 = 1.f - cos_theta_i2;
    const float sin_theta_i4 = sin_theta_i2 * sin_theta_i2;
    const float t1 = eta * eta - k * k - sin_theta_i2;
    const float a2pb2 = sqrtf(fmaxf(0.f, t1 * t1 + 4.f * k * k * eta * eta));
    const float a = sqrtf(fmaxf(0.f, 0.5f * (a2pb2 + t1)));
    const float term1 = a2pb2 + cos_theta_i2;
    const float term2 = 2.f * a * cos_theta_i;
    const float rs2 = (term1 - term2) / (term1 + term2);
    const float term3 = a2pb2 * cos_theta_i2 + sin_theta_i4;
    const float term4 = term2 * sin_theta_i2;
    const float rp2 = rs2 * (term3 - term4) / (term3 + term4);
    return 0.5f * (rp2 + rs2);
}
PT_HD vec3 fresnel_conductor(vec3 eta, vec3 k, float cos_theta_i) {
    return v3(fresnel_conductor1(eta.x, k.x, cos_theta_i), fresnel_conductor1(eta.y, k.y, cos_theta_i),
              fresnel_conductor1(eta.z, k.z, cos_theta_i));
}

// ----------------------------------------------------------------- GGX (material/ggx.h, VNDF variant)
PT_HD float ggx_lambda(vec3 w, float alpha) {
    const float a2 = alpha * alpha;
    const vec3 v2 = w * w;
    return (-1.f + sqrtf(1.f + (v2.x + v2.y) * a2 / v2.z)) / 2.f;
}
PT_HD float ggx_g1(vec3 w, float alpha) { return 1.f / (1.f + ggx_lambda(w, alpha)); }
PT_HD float ggx_g(vec3 wi, vec3 wo, float alpha) { return ggx_g1(wi, alpha) * ggx_g1(wo, alpha); }
PT_HD float ggx_d(vec3 wh, float alpha) {
    const float a2 = alpha * alpha;
    const vec3 v2 = wh * wh;
    const float t = (v2.x + v2.y) / a2 + v2.z;
    return 1.f / (kPi * a2 * t * t);
}
PT_HD float ggx_pdf(vec3 wo, vec3 wh, float alpha) {
    return ggx_d(wh, alpha) * ggx_g1(wo, alpha) * dot(wo, wh) / fabs_(wo.z);
}
PT_HD vec3 ggx_sample(vec3 wo, float alpha, vec2 xi) {
    const vec3 vh = normalize(v3(alpha * wo.x, alpha * wo.y, wo.z));
    const vec3 T1 = wo.z < 0.9999f ? normalize(cross(v3(0.f, 0.f, 1.f), vh)) : v3(1.f, 0.f, 0.f);
    const vec3 T2 = cross(vh, T1);
    const float r = sqrtf(xi.x);
    const float phi = 2.f * kPi * xi.y;
    float sp, cp;
    dm_sincos(phi, sp, cp);
    const float t1 = r * cp;
    float t2 = r * sp;
    const float s = 0.5f * (1.f + vh.z);
    t2 = (1.f - s) * sqrtf(1.f - t1 * t1) + s * t2;
    const vec3 nh = t1 * T1 + t2 * T2 + sqrtf(fmaxf(0.f, 1.f - t1 * t1 - t2 * t2)) * vh;
    const vec3 ne = v3(alpha * nh.x, alpha * nh.y, fmaxf(0.f, nh.z));
    return normalize(ne);
}

// ----------------------------------------------------------------- BSDFs
// EBsdfLobeType (bsdf/bsdf.h:7-24)
constexpr uint32_t kLobeDiffuseReflection = 1u << 1;
constexpr uint32_t kLobeGlossyReflection = 1u << 3;
constexpr uint32_t kLobeGlossyTransmission = 1u << 4;
constexpr uint32_t kLobeDeltaReflection = 1u << 5;
constexpr uint32_t kLobeDeltaTransmission = 1u << 6;
constexpr uint32_t kLobeDelta = kLobeDeltaReflection | kLobeDeltaTransmission;

// Material::LocalBsdf (optix_material.h:100-110) in one flat record.
// a/b/c hold the per-type colours in the order GetLocal fills them.
struct LocalBsdf {
    uint32_t type;
    uint32_t nonlinear;
    float alpha, eta, int_fdr, ssw;
    vec3 a, b, c;
};

// BsdfSamplingRecord (bsdf/bsdf.h:26-36)
struct BsdfRec {
    vec3 wi, wo;
    vec3 f;
    float pdf;
    uint32_t sampled_type;
};

// Material::GetLocalBsdf (optix_material.h:172-184) + each type's GetLocal
PT_D LocalBsdf local_bsdf(const DevMaterial &m, vec2 uv) {
    LocalBsdf l;
    l.type = m.type;
    l.nonlinear = m.nonlinear;
    l.eta = m.eta;
    l.int_fdr = m.int_fdr;
    l.ssw = m.specular_sampling_weight;
    l.alpha = 0.f;
    l.a = l.b = l.c = v3(0.f);
    switch (m.type) {
        case PUPIL_MAT_DIFFUSE: l.a = tex_sample(m.tex[0], uv); break;
        case PUPIL_MAT_DIELECTRIC:
            l.a = tex_sample(m.tex[0], uv);
            l.b = tex_sample(m.tex[1], uv);
            break;
        case PUPIL_MAT_ROUGH_DIELECTRIC:
            l.alpha = tex_sample(m.tex[0], uv).x;
            l.a = tex_sample(m.tex[1], uv);
            l.b = tex_sample(m.tex[2], uv);
            break;
        case PUPIL_MAT_CONDUCTOR:
            l.a = tex_sample(m.tex[0], uv);  // eta
            l.b = tex_sample(m.tex[1], uv);  // k
            l.c = tex_sample(m.tex[2], uv);  // specular_reflectance
            break;
        case PUPIL_MAT_ROUGH_CONDUCTOR:
            l.alpha = tex_sample(m.tex[0], uv).x;
            l.a = tex_sample(m.tex[1], uv);
            l.b = tex_sample(m.tex[2], uv);
            l.c = tex_sample(m.tex[3], uv);
            break;
        case PUPIL_MAT_PLASTIC:
            l.a = tex_sample(m.tex[0], uv);  // diffuse
            l.b = tex_sample(m.tex[1], uv);  // specular
            break;
        case PUPIL_MAT_ROUGH_PLASTIC:
            l.alpha = tex_sample(m.tex[0], uv).x;
            l.a = tex_sample(m.tex[1], uv);
            l.b = tex_sample(m.tex[2], uv);
            break;
        default: break;
    }
    return l;
}

// LocalBsdf::GetAlbedo (optix_material.h:146-164)
PT_HD vec3 bsdf_albedo(const LocalBsdf &l) {
    switch (l.type) {
        case PUPIL_MAT_DIFFUSE:
        case PUPIL_MAT_DIELECTRIC:
        case PUPIL_MAT_ROUGH_DIELECTRIC:
        case PUPIL_MAT_PLASTIC:
        case PUPIL_MAT_ROUGH_PLASTIC: return l.a;
        case PUPIL_MAT_CONDUCTOR:
        case PUPIL_MAT_ROUGH_CONDUCTOR: return l.c;
        default: return v3(0.f);
    }
}

// --- diffuse (bsdf/diffuse.h:14-34)
PT_HD void diffuse_eval(const LocalBsdf &l, BsdfRec &r) {
    vec3 f = v3(0.f);
    if (r.wi.z > 0.f && r.wo.z > 0.f) f = l.a * k1OverPi;
    r.f = f;
    float pdf = 0.f;
    if (r.wi.z > 0.f && r.wo.z > 0.f) pdf = cosine_hemisphere_pdf(r.wi);
    r.pdf = pdf;
}
PT_HD void diffuse_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    const float x0 = rng_next(rng);
    const float x1 = rng_next(rng);
    r.wi = cosine_sample_hemisphere(x0, x1);
    diffuse_eval(l, r);
    r.sampled_type = kLobeDiffuseReflection;
}

// --- dielectric (bsdf/dielectric.h:20-45): delta lobes, Eval is zero
PT_HD void dielectric_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    float cos_theta_t;
    const float fr = fresnel_dielectric(l.eta, r.wo.z, cos_theta_t);
    if (rng_next(rng) < fr) {
        r.wi = reflect_local(r.wo);
        r.pdf = fr;
        r.f = l.a * fr / fabs_(r.wi.z);
        r.sampled_type = kLobeDeltaReflection;
    } else {
        r.wi = refract_local(r.wo, cos_theta_t, l.eta);
        r.pdf = 1.f - fr;
        const float factor = cos_theta_t < 0.f ? 1.f / l.eta : l.eta;
        r.f = l.b * (1.f - fr) * factor * factor / fabs_(r.wi.z);
        r.sampled_type = kLobeDeltaTransmission;
    }
}

// --- rough dielectric (bsdf/rough_dielectric.h:21-96)
PT_HD void rough_dielectric_f(const LocalBsdf &l, BsdfRec &r) {
    r.f = v3(0.f);
    if (is_zero(r.wo.z)) return;
    vec3 wh;
    const bool sample_reflect = r.wo.z * r.wi.z > 0.f;
    if (sample_reflect)
        wh = normalize(r.wo + r.wi);
    else
        wh = normalize(r.wo + r.wi * (r.wo.z > 0.f ? l.eta : 1.f / l.eta));
    wh = wh * (wh.z > 0.f ? 1.f : -1.f);
    const float F = fresnel_dielectric(l.eta, dot(r.wo, wh));
    const float G = ggx_g(r.wi, r.wo, l.alpha);
    const float D = ggx_d(wh, l.alpha);
    if (sample_reflect) {
        r.f = l.a * F * G * D / (4.f * fabs_(r.wi.z) * fabs_(r.wo.z));
    } else {
        const float eta_ = r.wo.z > 0.f ? l.eta : 1.f / l.eta;
        const float sqrt_denom = dot(r.wo, wh) + eta_ * dot(r.wi, wh);
        r.f = l.b * fabs_((1.f - F) * D * G * dot(r.wi, wh) * dot(r.wo, wh) /
                          (sqrt_denom * sqrt_denom * r.wi.z * r.wo.z));
    }
}
PT_HD void rough_dielectric_pdf(const LocalBsdf &l, BsdfRec &r) {
    r.pdf = 0.f;
    const bool sample_reflect = r.wo.z * r.wi.z > 0.f;
    vec3 wh;
    float dwh_dwo;
    if (sample_reflect) {
        wh = normalize(r.wo + r.wi);
        dwh_dwo = 1.f / (4.f * dot(r.wi, wh));
    } else {
        const float eta_ = r.wo.z > 0.f ? l.eta : 1.f / l.eta;
        wh = normalize(r.wo + r.wi * eta_);
        const float sqrt_denom = dot(r.wo, wh) + eta_ * dot(r.wi, wh);
        dwh_dwo = (eta_ * eta_ * dot(r.wi, wh)) / (sqrt_denom * sqrt_denom);
    }
    wh = wh * (wh.z > 0.f ? 1.f : -1.f);
    const vec3 wo = r.wo * (r.wo.z > 0.f ? 1.f : -1.f);
    const float F = fresnel_dielectric(l.eta, dot(r.wo, wh));
    r.pdf = fabs_(ggx_pdf(wo, wh, l.alpha) * (sample_reflect ? F : 1.f - F) * dwh_dwo);
}
PT_HD void rough_dielectric_eval(const LocalBsdf &l, BsdfRec &r) {
    rough_dielectric_f(l, r);
    rough_dielectric_pdf(l, r);
}
PT_HD void rough_dielectric_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    const float x0 = rng_next(rng);
    const float x1 = rng_next(rng);
    const vec3 wo = r.wo * (r.wo.z > 0.f ? 1.f : -1.f);
    const vec3 wh = ggx_sample(wo, l.alpha, v2(x0, x1));
    float cos_theta_t = 0.f;
    const float F = fresnel_dielectric(l.eta, dot(r.wo, wh), cos_theta_t);
    if (rng_next(rng) < F) {
        r.wi = reflect_n(r.wo, wh);
        r.sampled_type = kLobeGlossyReflection;
    } else {
        if (is_zero(cos_theta_t)) return;
        r.wi = refract_n(r.wo, wh, cos_theta_t, l.eta);
        r.sampled_type = kLobeGlossyTransmission;
        if (r.wi.z * r.wo.z >= 0.f) return;
    }
    rough_dielectric_pdf(l, r);
    rough_dielectric_f(l, r);
}

// --- conductor (bsdf/conductor.h:19-35)
PT_HD void conductor_sample(const LocalBsdf &l, BsdfRec &r) {
    r.wi = reflect_local(r.wo);
    r.pdf = 1.f;
    const vec3 fr = fresnel_conductor(l.a, l.b, r.wo.z);
    r.f = l.c * fr / fabs_(r.wi.z);
    r.sampled_type = kLobeDeltaReflection;
}

// --- rough conductor (bsdf/rough_conductor.h:21-47)
PT_HD void rough_conductor_f(const LocalBsdf &l, BsdfRec &r) {
    r.f = v3(0.f);
    if (r.wi.z <= 0.f || r.wo.z <= 0.f) return;
    const vec3 wh = normalize(r.wi + r.wo);
    const vec3 fresnel_o = fresnel_conductor(l.a, l.b, dot(r.wo, wh));
    r.f = l.c * ggx_d(wh, l.alpha) * fresnel_o * ggx_g(r.wi, r.wo, l.alpha) / (4.f * r.wi.z * r.wo.z);
}
PT_HD void rough_conductor_pdf(const LocalBsdf &l, BsdfRec &r) {
    r.pdf = 0.f;
    if (r.wi.z <= 0.f || r.wo.z <= 0.f) return;
    vec3 wh = normalize(r.wi + r.wo);
    wh = normalize(wh);
    r.pdf = ggx_pdf(r.wo, wh, l.alpha) / (4.f * dot(r.wo, wh));
}
PT_HD void rough_conductor_eval(const LocalBsdf &l, BsdfRec &r) {
    rough_conductor_f(l, r);
    rough_conductor_pdf(l, r);
}
PT_HD void rough_conductor_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    const float x0 = rng_next(rng);
    const float x1 = rng_next(rng);
    r.wi = reflect_n(r.wo, ggx_sample(r.wo, l.alpha, v2(x0, x1)));
    rough_conductor_pdf(l, r);
    rough_conductor_f(l, r);
    r.sampled_type = kLobeDiffuseReflection;  // sic: rough_conductor.h:45
}

// --- plastic (bsdf/plastic.h:32-81)
PT_HD vec3 plastic_diff(const LocalBsdf &l) {
    return l.a / (1.f - (l.nonlinear ? l.a * l.int_fdr : v3(l.int_fdr)));
}
PT_HD float plastic_specular_prob(const LocalBsdf &l, float fresnel_o) {
    return (fresnel_o * l.ssw) / (fresnel_o * l.ssw + (1.f - fresnel_o) * (1.f - l.ssw));
}
PT_HD void plastic_eval(const LocalBsdf &l, BsdfRec &r) {
    r.f = v3(0.f);
    if (!(r.wi.z <= 0.f || r.wo.z <= 0.f)) {
        const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
        const float fresnel_i = fresnel_dielectric(l.eta, r.wi.z);
        const vec3 diff = plastic_diff(l);
        r.f = diff * (1.f - fresnel_i) * (1.f - fresnel_o) * cosine_hemisphere_pdf(r.wi) / (l.eta * l.eta * r.wi.z);
    }
    r.pdf = 0.f;
    if (r.wi.z <= 0.f || r.wo.z <= 0.f) return;
    const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
    const float specular_prob = plastic_specular_prob(l, fresnel_o);
    r.pdf = cosine_hemisphere_pdf(r.wi) * (1.f - specular_prob);
}
PT_HD void plastic_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    if (r.wo.z <= 0.f) return;
    const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
    const float x0 = rng_next(rng);
    const float x1 = rng_next(rng);
    const float specular_prob = plastic_specular_prob(l, fresnel_o);
    if (x0 < specular_prob) {
        r.sampled_type = kLobeDeltaReflection;
        r.wi = reflect_local(r.wo);
        r.f = l.b * fresnel_o / r.wi.z;
        r.pdf = specular_prob;
    } else {
        r.sampled_type = kLobeDiffuseReflection;
        r.wi = cosine_sample_hemisphere((x0 - specular_prob) / (1.f - specular_prob), x1);
        const float fresnel_i = fresnel_dielectric(l.eta, r.wi.z);
        const vec3 diff = plastic_diff(l);
        r.f = diff * (1.f - fresnel_i) * (1.f - fresnel_o) * cosine_hemisphere_pdf(r.wi) / (l.eta * l.eta * r.wi.z);
        r.pdf = cosine_hemisphere_pdf(r.wi) * (1.f - specular_prob);
    }
}

// --- rough plastic (bsdf/rough_plastic.h:31-86)
PT_HD void rough_plastic_f(const LocalBsdf &l, BsdfRec &r) {
    r.f = v3(0.f);
    if (r.wi.z <= 0.f || r.wo.z <= 0.f) return;
    const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
    const vec3 wh = normalize(r.wi + r.wo);
    r.f = l.b * fresnel_dielectric(l.eta, dot(wh, r.wo)) * ggx_d(wh, l.alpha) * ggx_g(r.wi, r.wo, l.alpha) /
          (4.f * r.wo.z * r.wi.z);
    const float fresnel_i = fresnel_dielectric(l.eta, r.wi.z);
    const vec3 diff = plastic_diff(l);
    r.f = r.f + diff * (1.f - fresnel_i) * (1.f - fresnel_o) * k1OverPi / (l.eta * l.eta);
}
PT_HD void rough_plastic_pdf(const LocalBsdf &l, BsdfRec &r) {
    r.pdf = 0.f;
    if (r.wi.z <= 0.f || r.wo.z <= 0.f) return;
    const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
    const float specular_prob = plastic_specular_prob(l, fresnel_o);
    const float diffuse_prob = 1.f - specular_prob;
    const vec3 wh = normalize(r.wi + r.wo);
    r.pdf = specular_prob * ggx_pdf(r.wo, wh, l.alpha) / (4.f * dot(r.wi, wh));
    r.pdf = r.pdf + diffuse_prob * cosine_hemisphere_pdf(r.wi);
}
PT_HD void rough_plastic_eval(const LocalBsdf &l, BsdfRec &r) {
    rough_plastic_f(l, r);
    rough_plastic_pdf(l, r);
}
PT_HD void rough_plastic_sample(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    r.wi = v3(0.f);
    if (r.wo.z <= 0.f) return;
    const float fresnel_o = fresnel_dielectric(l.eta, r.wo.z);
    const float specular_prob = plastic_specular_prob(l, fresnel_o);
    float x0 = rng_next(rng);
    float x1 = rng_next(rng);
    if (x1 < specular_prob) {
        x1 = x1 / specular_prob;
        const vec3 wh = ggx_sample(r.wo, l.alpha, v2(x0, x1));
        r.wi = reflect_n(r.wo, wh);
        r.sampled_type = kLobeGlossyReflection;
    } else {
        x1 = (x1 - specular_prob) / (1.f - specular_prob);
        r.wi = cosine_sample_hemisphere(x0, x1);
        r.sampled_type = kLobeDiffuseReflection;
    }
    rough_plastic_pdf(l, r);
    rough_plastic_f(l, r);
}

// Material::LocalBsdf::Eval / Sample dispatch.  The wavefront shade kernels
// instantiate this with a compile-time material type, so each kernel is
// branch-free over materials (the reference dispatches through
// optixDirectCall, optix_material.h:113-121).
template <uint32_t MAT>
PT_HD void bsdf_eval_t(const LocalBsdf &l, BsdfRec &r) {
    if constexpr (MAT == PUPIL_MAT_DIFFUSE) diffuse_eval(l, r);
    else if constexpr (MAT == PUPIL_MAT_DIELECTRIC || MAT == PUPIL_MAT_CONDUCTOR) { r.f = v3(0.f); r.pdf = 0.f; }
    else if constexpr (MAT == PUPIL_MAT_ROUGH_DIELECTRIC) rough_dielectric_eval(l, r);
    else if constexpr (MAT == PUPIL_MAT_ROUGH_CONDUCTOR) rough_conductor_eval(l, r);
    else if constexpr (MAT == PUPIL_MAT_PLASTIC) plastic_eval(l, r);
    else if constexpr (MAT == PUPIL_MAT_ROUGH_PLASTIC) rough_plastic_eval(l, r);
}
template <uint32_t MAT>
PT_HD void bsdf_sample_t(const LocalBsdf &l, BsdfRec &r, uint32_t &rng) {
    if constexpr (MAT == PUPIL_MAT_DIFFUSE) diffuse_sample(l, r, rng);
    else if constexpr (MAT == PUPIL_MAT_DIELECTRIC) dielectric_sample(l, r, rng);
    else if constexpr (MAT == PUPIL_MAT_ROUGH_DIELECTRIC) rough_dielectric_sample(l, r, rng);
    else if constexpr (MAT == PUPIL_MAT_CONDUCTOR) conductor_sample(l, r);
    else if constexpr (MAT == PUPIL_MAT_ROUGH_CONDUCTOR) rough_conductor_sample(l, r, rng);
    else if constexpr (MAT == PUPIL_MAT_PLASTIC) plastic_sample(l, r, rng);
    else if constexpr (MAT == PUPIL_MAT_ROUGH_PLASTIC) rough_plastic_sample(l, r, rng);
}

// ----------------------------------------------------------------- emitters
// LocalGeometry (render/geometry.h:252-256)
struct LocalGeo {
    vec3 position;
    vec3 normal;
    vec2 texcoord;
};

// EmitterSampleRecord (render/emitter/types.h:17-26); is_delta is never set
// for area / sphere emitters in the reference (uninitialised) -> false here.
struct EmitterSample {
    vec3 radiance;
    vec3 wi;
    float distance;
    float pdf;
};

PT_D vec3 emitter_radiance(const DevEmitter &e, vec2 tex) {  // Emitter::GetRadiance (emitter.h:54-71)
    if (e.type == PUPIL_EMITTER_CONST_ENV) return e.color;
    return tex_sample(e.radiance, tex);
}

PT_D void env_map_eval(const DevEmitter &e, vec3 dir_world, vec3 &radiance, float &pdf);

// Emitter::SampleDirect (emitter.h:73-88, emitter/{area,sphere,env}.h)
PT_D EmitterSample emitter_sample_direct(const DevEmitter &e, const LocalGeo &hit, vec2 xi) {
    EmitterSample s;
    s.pdf = 0.f;
    s.distance = 0.f;
    s.radiance = v3(0.f);
    s.wi = v3(0.f, 0.f, 1.f);
    if (e.type == PUPIL_EMITTER_TRI_AREA) {  // area.h:17-34
        const vec3 t = uniform_sample_triangle(xi.x, xi.y);
        const vec3 position = e.pos[0] * t.x + e.pos[1] * t.y + e.pos[2] * t.z;
        const vec3 normal = normalize(e.nrm[0] * t.x + e.nrm[1] * t.y + e.nrm[2] * t.z);
        const vec2 tex = e.tex[0] * t.x + e.tex[1] * t.y + e.tex[2] * t.z;
        s.radiance = tex_sample(e.radiance, tex);
        s.wi = normalize(position - hit.position);
        const float NoL = dot(hit.normal, s.wi);
        const float LNoL = dot(normal, -s.wi);
        if (NoL > 0.f && LNoL > 0.f) {
            const float distance = length(position - hit.position);
            s.pdf = distance * distance / (LNoL * e.area);
            s.distance = distance;
        }
    } else if (e.type == PUPIL_EMITTER_SPHERE) {  // sphere.h:14-31
        const vec3 t = uniform_sample_sphere(xi.x, xi.y);
        const vec3 position = t * e.radius + e.center;
        const vec3 normal = normalize(t);
        const vec2 tex = sphere_texcoord(t);
        s.radiance = tex_sample(e.radiance, tex);
        s.wi = normalize(position - hit.position);
        const float NoL = dot(hit.normal, s.wi);
        const float LNoL = dot(normal, -s.wi);
        if (NoL > 0.f && LNoL > 0.f) {
            const float distance = length(position - hit.position);
            s.pdf = distance * distance / (LNoL * e.area);
            s.distance = distance;
        }
    } else if (e.type == PUPIL_EMITTER_CONST_ENV) {  // env.h:70-79
        const vec3 local_wi = uniform_sample_hemisphere(xi.x, xi.y);
        s.wi = to_world(local_wi, hit.normal);
        s.pdf = uniform_hemisphere_pdf(local_wi);
        s.distance = kMaxDistance;
        s.radiance = e.color;
    } else if (e.type == PUPIL_EMITTER_ENV_MAP) {  // env.h:23-49
        uint32_t row = 0;
        for (; row < e.map_h; ++row)  // row_cdf has map_h + 1 entries
            if (xi.x <= e.row_cdf[row]) break;
        uint32_t col = 0;
        for (uint32_t i = row * (e.map_w + 1); col < e.map_w - 1; ++i, ++col)
            if (xi.y <= e.col_cdf[i]) break;
        const float phi = col * kPi * 2.f / e.map_w;
        const float theta = row * kPi / e.map_h;
        float st, ct, sp, cp;
        dm_sincos(theta, st, ct);
        dm_sincos(kPi - phi, sp, cp);
        const vec3 local_wi = v3(st * sp, ct, st * cp);
        s.wi = v3(dot(v3(e.to_world[0], e.to_world[1], e.to_world[2]), local_wi),
                  dot(v3(e.to_world[3], e.to_world[4], e.to_world[5]), local_wi),
                  dot(v3(e.to_world[6], e.to_world[7], e.to_world[8]), local_wi));
        s.distance = kMaxDistance;
        const vec2 tex = v2(phi * 0.5f * k1OverPi, theta * k1OverPi);
        s.radiance = tex_sample(e.radiance, tex) * e.scale;
        s.pdf = luminance(s.radiance) * e.row_weight[row] * e.normalization / fmaxf(1e-4f, fabs_(st));
        if (s.pdf < 0.f) s.pdf = 0.f;
    }
    return s;
}

// Emitter::Eval for the area emitters hit by an extension ray (area.h:36-45,
// sphere.h:33-43).  Returns pdf 0 when the reference leaves the record
// uninitialised (LNoL <= 0).
PT_D void emitter_eval_area(const DevEmitter &e, const LocalGeo &g, vec3 scatter_pos, vec3 &radiance, float &pdf) {
    pdf = 0.f;
    radiance = v3(0.f);
    const vec3 dir = normalize(scatter_pos - g.position);
    const float LNoL = dot(g.normal, dir);
    if (LNoL > 0.f) {
        const float distance = length(scatter_pos - g.position);
        pdf = distance * distance / (LNoL * e.area);
        radiance = tex_sample(e.radiance, g.texcoord);
    }
}

// env.h:51-64 (EnvMap::Eval) on a world direction
PT_D void env_map_eval(const DevEmitter &e, vec3 dir_world, vec3 &radiance, float &pdf) {
    const vec3 dir = v3(dot(v3(e.to_local[0], e.to_local[1], e.to_local[2]), dir_world),
                        dot(v3(e.to_local[3], e.to_local[4], e.to_local[5]), dir_world),
                        dot(v3(e.to_local[6], e.to_local[7], e.to_local[8]), dir_world));
    const float phi = kPi - dm_atan2(dir.x, dir.z);
    const float theta = dm_acos(dir.y);
    const vec2 tex = v2(phi * 0.5f * k1OverPi, theta * k1OverPi);
    uint32_t row = (uint32_t)(tex.y * e.map_h);
    if (row > e.map_h - 2u) row = e.map_h - 2u;
    radiance = tex_sample(e.radiance, tex) * e.scale;
    const float w0 = e.row_weight[row], w1 = e.row_weight[row + 1];
    const float lw = w0 + (tex.y * e.map_h - 1.f * row) * (w1 - w0);
    pdf = luminance(radiance) * lw * e.normalization / fmaxf(1e-4f, fabs_(dm_sin(theta)));
}

// __miss__default env evaluation (main.cu:196-212): position = o + normalize(d)
PT_D void env_eval(const DevEmitter &e, vec3 ray_o, vec3 ray_d, vec3 &radiance, float &pdf) {
    if (e.type == PUPIL_EMITTER_CONST_ENV) {  // env.h:81-84
        pdf = 0.25f * k1OverPi;
        radiance = e.color;
        return;
    }
    const vec3 nd = normalize(ray_d);
    const vec3 position = ray_o + nd;
    const vec3 dir = normalize(position - ray_o);
    env_map_eval(e, dir, radiance, pdf);
}

}  // namespace pupil
