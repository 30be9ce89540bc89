// pt_trace.h — ray/primitive intersection and BVH traversal for gfx950.
//
// Replaces optixTrace over the reference's IAS->GAS hierarchy
// (example/path_tracer/main.cu:77-82,158-163; render/emitter.h:91-100).
//  * Triangles: watertight test (Woop, Benthin, Wald 2013) — OptiX's built-in
//    triangle test is watertight too; barycentrics follow OptiX (b1 weights v1,
//    b2 weights v2).  Both faces are hit (OPTIX_INSTANCE_FLAG_NONE).
//  * Spheres: unit sphere in object space (OptiX built-in sphere module, the
//    radius/centre folded into the instance transform, shape.cpp:106-125).
//  * Closest hit uses a total order on (t, primitive id), so the result is the
//    same for any BVH and any traversal order (the CPU oracle builds its own
//    BVH and must agree bit for bit).
//  * Box tests are conservative (Ize 2013: t_far scaled by 1+2*gamma(3)), so
//    culling never drops a primitive the exact test would report.
#pragma once

#include "pt_scene.h"

namespace pupil {

struct RayPre {
    vec3 o, d;
    vec3 idir;  // for slab tests
    int kx, ky, kz;
    float Sx, Sy, Sz;
};

PT_HD float comp(vec3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

PT_HD RayPre ray_pre(vec3 o, vec3 d) {
    RayPre r;
    r.o = o;
    r.d = d;
    const float tiny = 1e-30f;
    r.idir = v3(1.f / (fabs_(d.x) < tiny ? copysignf(tiny, d.x) : d.x),
                1.f / (fabs_(d.y) < tiny ? copysignf(tiny, d.y) : d.y),
                1.f / (fabs_(d.z) < tiny ? copysignf(tiny, d.z) : d.z));
    const float ax = fabs_(d.x), ay = fabs_(d.y), az = fabs_(d.z);
    int kz = 0;
    if (ay > ax) kz = 1;
    if (az > (kz == 0 ? ax : ay)) kz = 2;
    int kx = kz + 1;
    if (kx == 3) kx = 0;
    int ky = kx + 1;
    if (ky == 3) ky = 0;
    if (comp(d, kz) < 0.f) {
        int t = kx;
        kx = ky;
        ky = t;
    }
    r.kx = kx;
    r.ky = ky;
    r.kz = kz;
    const float dz = comp(d, kz);
    r.Sx = comp(d, kx) / dz;
    r.Sy = comp(d, ky) / dz;
    r.Sz = 1.0f / dz;
    return r;
}

// Watertight ray/triangle; returns true and (t, b1, b2) if tmin <= t <= tmax.
PT_HD bool intersect_triangle(const RayPre &r, vec3 v0, vec3 v1, vec3 v2, float tmin, float tmax, float &t_out,
                              float &b1, float &b2) {
    const vec3 A = v0 - r.o, B = v1 - r.o, C = v2 - r.o;
    const float Akz = comp(A, r.kz), Bkz = comp(B, r.kz), Ckz = comp(C, r.kz);
    const float Ax = comp(A, r.kx) - r.Sx * Akz;
    const float Ay = comp(A, r.ky) - r.Sy * Akz;
    const float Bx = comp(B, r.kx) - r.Sx * Bkz;
    const float By = comp(B, r.ky) - r.Sy * Bkz;
    const float Cx = comp(C, r.kx) - r.Sx * Ckz;
    const float Cy = comp(C, r.ky) - r.Sy * Ckz;
    float U = Cx * By - Cy * Bx;
    float V = Ax * Cy - Ay * Cx;
    float W = Bx * Ay - By * Ax;
    if (U == 0.f || V == 0.f || W == 0.f) {  // edge hit: recompute exactly-rounded in double
        U = (float)((double)Cx * (double)By - (double)Cy * (double)Bx);
        V = (float)((double)Ax * (double)Cy - (double)Ay * (double)Cx);
        W = (float)((double)Bx * (double)Ay - (double)By * (double)Ax);
    }
    if ((U < 0.f || V < 0.f || W < 0.f) && (U > 0.f || V > 0.f || W > 0.f)) return false;
    const float det = U + V + W;
    if (det == 0.f) return false;
    const float Az = r.Sz * Akz, Bz = r.Sz * Bkz, Cz = r.Sz * Ckz;
    const float T = U * Az + V * Bz + W * Cz;
    const float rcp = 1.0f / det;
    const float t = T * rcp;
    if (!(t >= tmin && t <= tmax)) return false;
    t_out = t;
    b1 = V * rcp;
    b2 = W * rcp;
    return true;
}

// Unit sphere at the origin in object space; inv = row-major 3x4 world->object.
// Discriminant from the closest-approach vector l = f - (f.d / d.d) d
// (Haines et al., Ray Tracing Gems ch. 7): its rounding error grows like
// u |f| instead of the u |f|^2 of b^2 - a c, so a reported hit lies within
// r (1 + 2^-10) of the centre for ray origins up to ~10^4 radii away and the
// 1.001-padded sphere boxes of every BVH (GPU and oracle) contain it: grazing
// hits do not depend on the tree.  Roots: q = b' + sign(b') sqrt(disc),
// t = c / q and q / a.
PT_HD bool intersect_unit_sphere(const float *inv, vec3 o, vec3 d, float tmin, float tmax, float &t_out) {
    const vec3 f = xform_point(inv, o);
    const vec3 od = xform_vector(inv, d);
    const float a = dot(od, od);
    const float bp = -dot(f, od);
    const vec3 l = f + od * (bp / a);
    const float disc = a * (1.f - dot(l, l));
    if (disc < 0.f) return false;
    const float c = dot(f, f) - 1.f;
    const float q = bp + copysignf(sqrtf(disc), bp);
    const float r0 = c / q, r1 = q / a;
    const float t0 = fminf(r0, r1), t1 = fmaxf(r0, r1);
    if (t0 >= tmin && t0 <= tmax) {
        t_out = t0;
        return true;
    }
    if (t1 >= tmin && t1 <= tmax) {
        t_out = t1;
        return true;
    }
    return false;
}

constexpr float kBoxConservative = 1.0000004f;  // 1 + 2*gamma(3)

// Slab test of one box; returns entry distance or +inf when missed.
PT_HD float box_entry(const RayPre &r, vec3 lo, vec3 hi, float tmin, float tmax) {
    const float tx0 = (lo.x - r.o.x) * r.idir.x, tx1 = (hi.x - r.o.x) * r.idir.x;
    const float ty0 = (lo.y - r.o.y) * r.idir.y, ty1 = (hi.y - r.o.y) * r.idir.y;
    const float tz0 = (lo.z - r.o.z) * r.idir.z, tz1 = (hi.z - r.o.z) * r.idir.z;
    const float tn = fmaxf(fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fminf(tz0, tz1)), tmin);
    float tf = fminf(fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fmaxf(tz0, tz1)), tmax);
    tf = tf * kBoxConservative;
    return tn <= tf ? tn : __builtin_huge_valf();
}

}  // namespace pupil
