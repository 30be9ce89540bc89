/*
 * pupil_detmath.h — deterministic single-precision transcendental functions.
 *
 * Why this exists: the reference path tracer calls sinf/cosf/acos/atan2 inside
 * the BSDF/emitter math (framework/optix/util.h:38-54,117-128,
 * framework/render/material/ggx.h:213-216, framework/render/emitter/env.h:217-247).
 * The HIP device libm (ocml) and the host libm (glibc) round those functions
 * differently, so a GPU render and a CPU render of the same path would drift by
 * an ulp and diverge at silhouettes.  Both the HIP engine and the CPU oracle
 * therefore call these functions, which are written with +,-,*,/,sqrt and exact
 * rounding ops only.  Compiled with -ffp-contract=off on both sides, every
 * result is bit-identical on gfx950 and x86-64 (sqrt and divide are correctly
 * rounded on both; see tests/test_gpu_parity.py::test_detmath_bit_exact).
 *
 * The polynomials are the classic Cody-Waite / Cephes single-precision
 * approximations (max error ~2 ulp over the ranges the tracer uses); accuracy
 * against float64 is pinned in tests/test_detmath.py.
 */
#pragma once

#if defined(__HIPCC__) || defined(__HIP__)
#define PUPIL_DM_HD __host__ __device__ __forceinline__
#else
#define PUPIL_DM_HD inline
#endif

namespace pupil_dm {

/* PUPIL_FASTMATH_EMULATION (host only; oracle/Makefile liboracle_fastmath.so, test
 * infrastructure for tools/fastmath_sensitivity.py -- never the engine): the error
 * model of CUDA -use_fast_math, which the reference is compiled with
 * (CMakeLists.txt:45).  Each result is displaced deterministically (a hash of the
 * input) by up to the documented maximum error: __sinf / __cosf 2^-21.41 absolute,
 * acosf 2 ulp, atan2f 3 ulp (CUDA C Programming Guide, Mathematical Functions). */
#if defined(PUPIL_FASTMATH_EMULATION) && !defined(__HIP_DEVICE_COMPILE__)
inline float dm_fm_noise(float x, unsigned salt) {
    unsigned u;
    __builtin_memcpy(&u, &x, 4);
    u = (u ^ (salt * 0x9e3779b9u)) * 0x85ebca6bu;
    u ^= u >> 13;
    u *= 0xc2b2ae35u;
    u ^= u >> 16;
    return (float)(int)u * (1.0f / 2147483648.0f); /* [-1, 1) */
}
#define PUPIL_DM_FM_ABS(v, x, salt, err) ((v) + (err) * pupil_dm::dm_fm_noise((x), (salt)))
#define PUPIL_DM_FM_ULP(v, x, salt, ulps) ((v) * (1.0f + (ulps) * 5.9604645e-8f * pupil_dm::dm_fm_noise((x), (salt))))
#else
#define PUPIL_DM_FM_ABS(v, x, salt, err) (v)
#define PUPIL_DM_FM_ULP(v, x, salt, ulps) (v)
#endif

constexpr float kPi = 3.14159265358979323846f;
constexpr float kPiOver2 = 1.57079632679489661923f;
constexpr float kPiOver4 = 0.785398163397448309616f;

PUPIL_DM_HD float dm_abs(float x) { return x < 0.f ? -x : x; }

/* round-to-nearest-even: an exact IEEE operation on both targets
 * (v_rndne_f32 on gfx950, roundss/nearbyint on x86-64) */
PUPIL_DM_HD float dm_rint(float x) { return __builtin_rintf(x); }

/* sin/cos of x for |x| < ~8192 (the tracer only feeds [−4π, 4π]).
 * Cody-Waite reduction by pi/2 with a 3-part constant, then minimax
 * polynomials on [-pi/4, pi/4]. */
PUPIL_DM_HD void dm_sincos(float x, float &s, float &c) {
    const float two_over_pi = 0.636619772367581343076f;
    const float dp1 = 1.5703125f;                 /* 8 significant bits: j*dp1 exact */
    const float dp2 = 4.837512969970703125e-4f;
    const float dp3 = 7.54978995489188216e-8f;
    float j = dm_rint(x * two_over_pi);
    float r = x - j * dp1;
    r = r - j * dp2;
    r = r - j * dp3;
    int q = (int)j;
    float z = r * r;
    float ps = ((-1.9515295891e-4f * z + 8.3321608736e-3f) * z - 1.6666654611e-1f);
    ps = ps * z;
    ps = ps * r;
    ps = ps + r;
    float pc = ((2.443315711809948e-5f * z - 1.388731625493765e-3f) * z + 4.166664568298827e-2f);
    pc = pc * z;
    pc = pc * z;
    pc = pc - 0.5f * z;
    pc = pc + 1.0f;
    switch (q & 3) {
        case 0: s = ps; c = pc; break;
        case 1: s = pc; c = -ps; break;
        case 2: s = -ps; c = -pc; break;
        default: s = -pc; c = ps; break;
    }
    s = PUPIL_DM_FM_ABS(s, x, 1u, 3.6e-7f);
    c = PUPIL_DM_FM_ABS(c, x, 2u, 3.6e-7f);
}

PUPIL_DM_HD float dm_sin(float x) { float s, c; dm_sincos(x, s, c); return s; }
PUPIL_DM_HD float dm_cos(float x) { float s, c; dm_sincos(x, s, c); return c; }

/* asin core for |x| <= 1 (Cephes asinf structure) */
PUPIL_DM_HD float dm_asin(float x) {
    float sign = 1.f;
    float a = x;
    if (a < 0.f) { sign = -1.f; a = -a; }
    if (a > 1.f) a = 1.f;
    bool flag = false;
    float z, v;
    if (a > 0.5f) {
        z = 0.5f * (1.0f - a);
        v = sqrtf(z);
        flag = true;
    } else {
        z = a * a;
        v = a;
    }
    float p = ((((4.2163199048e-2f * z + 2.4181311049e-2f) * z + 4.5470025998e-2f) * z + 7.4953002686e-2f) * z + 1.6666752422e-1f);
    p = p * z;
    p = p * v;
    p = p + v;
    if (flag) {
        p = p + p;
        p = kPiOver2 - p;
    }
    return sign * p;
}

PUPIL_DM_HD float dm_acos_exact(float x) {
    if (x < -0.5f) {
        float h = 0.5f * (1.0f + x);
        return kPi - 2.0f * dm_asin(sqrtf(h));
    }
    if (x > 0.5f) {
        float h = 0.5f * (1.0f - x);
        return 2.0f * dm_asin(sqrtf(h));
    }
    return kPiOver2 - dm_asin(x);
}

PUPIL_DM_HD float dm_acos(float x) { return PUPIL_DM_FM_ULP(dm_acos_exact(x), x, 3u, 2.0f); }

/* atan for any finite x (Cephes atanf structure) */
PUPIL_DM_HD float dm_atan(float x) {
    float sign = 1.f;
    if (x < 0.f) { sign = -1.f; x = -x; }
    float y;
    if (x > 2.414213562373095f) {
        y = kPiOver2;
        x = -1.0f / x;
    } else if (x > 0.4142135623730950f) {
        y = kPiOver4;
        x = (x - 1.0f) / (x + 1.0f);
    } else {
        y = 0.0f;
    }
    float z = x * x;
    float p = (((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f);
    p = p * z;
    p = p * x;
    p = p + x;
    y = y + p;
    return sign * y;
}

/* atan2 with the libm quadrant conventions (atan2(±0, +0) = ±0, atan2(±0, -0) = ±pi) */
PUPIL_DM_HD float dm_atan2_exact(float y, float x) {
    if (x == 0.f) {
        if (y > 0.f) return kPiOver2;
        if (y < 0.f) return -kPiOver2;
        return 0.f;
    }
    float z = dm_atan(y / x);
    if (x < 0.f) {
        if (y < 0.f) z = z - kPi;
        else z = z + kPi;
    }
    return z;
}

PUPIL_DM_HD float dm_atan2(float y, float x) { return PUPIL_DM_FM_ULP(dm_atan2_exact(y, x), y + x, 4u, 3.0f); }

}  // namespace pupil_dm
