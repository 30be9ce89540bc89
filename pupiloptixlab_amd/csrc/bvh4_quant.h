// bvh4_quant.h — conservative 8-bit quantisation of BVH4 child boxes, shared by
// the GPU builder (bvh_build.hip) and the host TLAS builder (accel_two_level.hip).
// Child k's plane on an axis decodes as origin + q * scale with scale a power of
// two (q * scale exact, one rounding in the add); the encoder checks the decoded
// planes enclose the child interval and doubles the scale until they do.
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

#include "pt_scene.h"

namespace pupil {

PT_HD uint32_t qbits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
#endif
}
PT_HD float qfloat(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f;
    std::memcpy(&f, &u, 4);
    return f;
#endif
}

// decode used by the traversal: origin + (float)q * scale (q*scale is exact)
PT_HD float qdecode(float origin, uint32_t q, float scale) { return origin + (float)q * scale; }

// Up to N (4 or 8) child intervals [clo[k], chi[k]] (k < nk) inside [lo, hi] on
// one axis; byte k % 4 of word k / 4 of qlo / qhi holds child k's plane.
template <int N>
PT_HD void quantize_axis_n(float lo, float hi, const float *clo, const float *chi, int nk, float &origin,
                           uint32_t &ebyte, uint32_t *qlo, uint32_t *qhi) {
    origin = lo;
    const float ext = hi - lo;
    float scale;
    if (!(ext > 0.f)) {
        scale = qfloat(1u << 23);  // 2^-126
    } else {
        scale = exp2f(ceilf(log2f(ext / 254.f)));
        if (!(scale > 0.f)) scale = qfloat(1u << 23);
    }
    for (int attempt = 0; attempt < 8; attempt++) {
        bool ok = true;
        for (int w = 0; w < N / 4; w++) qlo[w] = qhi[w] = 0u;
        for (int k = 0; k < N; k++) {
            uint32_t a = 255u, b = 0u;  // empty slot: lo > hi
            if (k < nk) {
                float fa = floorf((clo[k] - origin) / scale);
                float fb = ceilf((chi[k] - origin) / scale);
                fa = fminf(fmaxf(fa, 0.f), 255.f);
                fb = fminf(fmaxf(fb, 0.f), 255.f);
                a = (uint32_t)fa;
                b = (uint32_t)fb;
                while (a > 0u && qdecode(origin, a, scale) > clo[k]) a--;
                while (b < 255u && qdecode(origin, b, scale) < chi[k]) b++;
                if (qdecode(origin, a, scale) > clo[k] || qdecode(origin, b, scale) < chi[k]) ok = false;
            }
            qlo[k >> 2] |= a << (8 * (k & 3));
            qhi[k >> 2] |= b << (8 * (k & 3));
        }
        if (ok) break;
        scale = scale * 2.f;
    }
    ebyte = (qbits(scale) >> 23) & 0xFFu;
}

PT_HD void quantize_axis(float lo, float hi, const float *clo, const float *chi, int nk, float &origin,
                         uint32_t &ebyte, uint32_t &qlo, uint32_t &qhi) {
    quantize_axis_n<4>(lo, hi, clo, chi, nk, origin, ebyte, &qlo, &qhi);
}

// The per-axis plane scales of a node from their biased exponents.
PT_HD void set_scales(Bvh4Node &o, uint32_t ex, uint32_t ey, uint32_t ez) {
    o.sx = qfloat(ex << 23);
    o.sy = qfloat(ey << 23);
    o.sz = qfloat(ez << 23);
}

// One BVH4 node from its box, nk <= 4 child boxes and links.
PT_HD Bvh4Node encode_bvh4(const float nlo[3], const float nhi[3], const float clo[3][4], const float chi[3][4],
                           const int link[4], int nk) {
    Bvh4Node o;
    uint32_t ex, ey, ez;
    quantize_axis(nlo[0], nhi[0], clo[0], chi[0], nk, o.ox, ex, o.qlo_x, o.qhi_x);
    quantize_axis(nlo[1], nhi[1], clo[1], chi[1], nk, o.oy, ey, o.qlo_y, o.qhi_y);
    quantize_axis(nlo[2], nhi[2], clo[2], chi[2], nk, o.oz, ez, o.qlo_z, o.qhi_z);
    set_scales(o, ex, ey, ez);
    for (int k = 0; k < 4; k++) o.child[k] = k < nk ? link[k] : kEmptyLink;
    return o;
}

}  // namespace pupil
