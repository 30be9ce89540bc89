// hmath.h — host-side transform / camera algebra.
//
// util::Mat4 (framework/util/type.h:73-112) is a row-major float[16] whose
// operator* is XMMatrixMultiply (plain A*B on the stored rows); the reference
// uses it column-vector style (TransformPoint, transform.cpp:123-130).  The
// DirectXMath functions the reference calls (XMMatrixPerspectiveFovRH,
// XMMatrixLookAtRH, XMMatrixInverse, XMMatrixTranspose) are restated here from
// their documented definitions; the camera matrices they produce are handed
// to both the engine and the CPU oracle, so they need not be bit-identical to
// DirectXMath (which cannot run here).
#pragma once

#include <cmath>
#include <cstring>

namespace Pupil::util {

struct Float3 {
    float x = 0.f, y = 0.f, z = 0.f;
};

struct Mat4 {
    float e[16];
    static Mat4 Identity() {
        Mat4 m;
        std::memset(m.e, 0, sizeof(m.e));
        m.e[0] = m.e[5] = m.e[10] = m.e[15] = 1.f;
        return m;
    }
    static Mat4 Rows(float a0, float a1, float a2, float a3, float b0, float b1, float b2, float b3, float c0,
                     float c1, float c2, float c3, float d0, float d1, float d2, float d3) {
        Mat4 m;
        const float v[16] = {a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3, d0, d1, d2, d3};
        std::memcpy(m.e, v, sizeof(v));
        return m;
    }
    float &at(int r, int c) { return e[4 * r + c]; }
    float at(int r, int c) const { return e[4 * r + c]; }
    Mat4 operator*(const Mat4 &b) const {  // XMMatrixMultiply
        Mat4 m;
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++)
                m.e[4 * r + c] = at(r, 0) * b.at(0, c) + at(r, 1) * b.at(1, c) + at(r, 2) * b.at(2, c) + at(r, 3) * b.at(3, c);
        return m;
    }
    Mat4 Transpose() const {
        Mat4 m;
        for (int r = 0; r < 4; r++)
            for (int c = 0; c < 4; c++) m.e[4 * r + c] = at(c, r);
        return m;
    }
    // general 4x4 inverse (cofactor expansion in double, rounded to float)
    Mat4 Inverse() const {
        double a[16];
        for (int k = 0; k < 16; k++) a[k] = e[k];
        double inv[16];
        inv[0] = a[5] * a[10] * a[15] - a[5] * a[11] * a[14] - a[9] * a[6] * a[15] + a[9] * a[7] * a[14] +
                 a[13] * a[6] * a[11] - a[13] * a[7] * a[10];
        inv[4] = -a[4] * a[10] * a[15] + a[4] * a[11] * a[14] + a[8] * a[6] * a[15] - a[8] * a[7] * a[14] -
                 a[12] * a[6] * a[11] + a[12] * a[7] * a[10];
        inv[8] = a[4] * a[9] * a[15] - a[4] * a[11] * a[13] - a[8] * a[5] * a[15] + a[8] * a[7] * a[13] +
                 a[12] * a[5] * a[11] - a[12] * a[7] * a[9];
        inv[12] = -a[4] * a[9] * a[14] + a[4] * a[10] * a[13] + a[8] * a[5] * a[14] - a[8] * a[6] * a[13] -
                  a[12] * a[5] * a[10] + a[12] * a[6] * a[9];
        inv[1] = -a[1] * a[10] * a[15] + a[1] * a[11] * a[14] + a[9] * a[2] * a[15] - a[9] * a[3] * a[14] -
                 a[13] * a[2] * a[11] + a[13] * a[3] * a[10];
        inv[5] = a[0] * a[10] * a[15] - a[0] * a[11] * a[14] - a[8] * a[2] * a[15] + a[8] * a[3] * a[14] +
                 a[12] * a[2] * a[11] - a[12] * a[3] * a[10];
        inv[9] = -a[0] * a[9] * a[15] + a[0] * a[11] * a[13] + a[8] * a[1] * a[15] - a[8] * a[3] * a[13] -
                 a[12] * a[1] * a[11] + a[12] * a[3] * a[9];
        inv[13] = a[0] * a[9] * a[14] - a[0] * a[10] * a[13] - a[8] * a[1] * a[14] + a[8] * a[2] * a[13] +
                  a[12] * a[1] * a[10] - a[12] * a[2] * a[9];
        inv[2] = a[1] * a[6] * a[15] - a[1] * a[7] * a[14] - a[5] * a[2] * a[15] + a[5] * a[3] * a[14] +
                 a[13] * a[2] * a[7] - a[13] * a[3] * a[6];
        inv[6] = -a[0] * a[6] * a[15] + a[0] * a[7] * a[14] + a[4] * a[2] * a[15] - a[4] * a[3] * a[14] -
                 a[12] * a[2] * a[7] + a[12] * a[3] * a[6];
        inv[10] = a[0] * a[5] * a[15] - a[0] * a[7] * a[13] - a[4] * a[1] * a[15] + a[4] * a[3] * a[13] +
                  a[12] * a[1] * a[7] - a[12] * a[3] * a[5];
        inv[14] = -a[0] * a[5] * a[14] + a[0] * a[6] * a[13] + a[4] * a[1] * a[14] - a[4] * a[2] * a[13] -
                  a[12] * a[1] * a[6] + a[12] * a[2] * a[5];
        inv[3] = -a[1] * a[6] * a[11] + a[1] * a[7] * a[10] + a[5] * a[2] * a[11] - a[5] * a[3] * a[10] -
                 a[9] * a[2] * a[7] + a[9] * a[3] * a[6];
        inv[7] = a[0] * a[6] * a[11] - a[0] * a[7] * a[10] - a[4] * a[2] * a[11] + a[4] * a[3] * a[10] +
                 a[8] * a[2] * a[7] - a[8] * a[3] * a[6];
        inv[11] = -a[0] * a[5] * a[11] + a[0] * a[7] * a[9] + a[4] * a[1] * a[11] - a[4] * a[3] * a[9] -
                  a[8] * a[1] * a[7] + a[8] * a[3] * a[5];
        inv[15] = a[0] * a[5] * a[10] - a[0] * a[6] * a[9] - a[4] * a[1] * a[10] + a[4] * a[2] * a[9] +
                  a[8] * a[1] * a[6] - a[8] * a[2] * a[5];
        double det = a[0] * inv[0] + a[1] * inv[4] + a[2] * inv[8] + a[3] * inv[12];
        Mat4 m;
        if (det == 0.0) {
            std::memset(m.e, 0, sizeof(m.e));
            return m;
        }
        det = 1.0 / det;
        for (int k = 0; k < 16; k++) m.e[k] = (float)(inv[k] * det);
        return m;
    }
};

// util::Transform (framework/util/transform.h/.cpp): every builder
// left-multiplies (matrix = op * matrix).
struct Transform {
    Mat4 matrix = Mat4::Identity();

    void Translate(float x, float y, float z) {
        matrix = Mat4::Rows(1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1) * matrix;
    }
    void Scale(float x, float y, float z) {
        matrix = Mat4::Rows(x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1) * matrix;
    }
    // transform.cpp:7-56 (quaternion rotation about a unit axis, degrees)
    void Rotate(float ux, float uy, float uz, float angle) {
        const float u_len = std::sqrt(ux * ux + uy * uy + uz * uz);
        ux /= u_len, uy /= u_len, uz /= u_len;
        const float theta = angle / 180.f * 3.14159265358979323846f;
        const float a = std::cos(0.5f * theta);
        const float b = std::sin(0.5f * theta) * ux;
        const float c = std::sin(0.5f * theta) * uy;
        const float d = std::sin(0.5f * theta) * uz;
        const Mat4 r = Mat4::Rows(1.f - 2.f * c * c - 2.f * d * d, 2.f * b * c - 2.f * a * d, 2.f * a * c + 2.f * b * d,
                                  0.f, 2.f * b * c + 2.f * a * d, 1.f - 2.f * b * b - 2.f * d * d,
                                  2.f * c * d - 2.f * a * b, 0.f, 2.f * b * d - 2.f * a * c, 2.f * a * b + 2.f * c * d,
                                  1.f - 2.f * b * b - 2.f * c * c, 0.f, 0.f, 0.f, 0.f, 1.f);
        matrix = r * matrix;
    }
    // transform.cpp:58-69: camera_to_world = transpose(inverse(XMMatrixLookAtRH))
    void LookAt(const Float3 &eye, const Float3 &target, const Float3 &up) {
        auto sub = [](Float3 a, Float3 b) { return Float3{a.x - b.x, a.y - b.y, a.z - b.z}; };
        auto norm = [](Float3 v) {
            const float l = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
            return Float3{v.x / l, v.y / l, v.z / l};
        };
        auto crs = [](Float3 a, Float3 b) {
            return Float3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
        };
        auto dt = [](Float3 a, Float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
        const Float3 r2 = norm(sub(eye, target));  // LookToLH(eye, -(target-eye))
        const Float3 r0 = norm(crs(up, r2));
        const Float3 r1 = crs(r2, r0);
        const Float3 neg{-eye.x, -eye.y, -eye.z};
        // XMMatrixLookToLH builds rows (R, D) then transposes: row-vector view matrix
        Mat4 view_rows = Mat4::Rows(r0.x, r0.y, r0.z, dt(r0, neg), r1.x, r1.y, r1.z, dt(r1, neg), r2.x, r2.y, r2.z,
                                    dt(r2, neg), 0, 0, 0, 1);
        const Mat4 world_to_camera = view_rows.Transpose();
        matrix = world_to_camera.Inverse().Transpose();
    }
};

// util::Camera::GetSampleToCameraMatrix (framework/util/camera.cpp:7-20)
inline Mat4 SampleToCamera(float fov_y_deg, float aspect, float near_clip, float far_clip) {
    const double half = 0.5 * (double)(fov_y_deg / 180.f * 3.14159265358979323846f);
    const float height = (float)(std::cos(half) / std::sin(half));
    const float width = height / aspect;
    const float range = far_clip / (near_clip - far_clip);
    // XMMatrixPerspectiveFovRH (row-vector convention)
    const Mat4 proj = Mat4::Rows(width, 0, 0, 0, 0, height, 0, 0, 0, 0, range, -1.f, 0, 0, range * near_clip, 0);
    const Mat4 tr = Mat4::Rows(1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 1.f, 1.f, 0, 1);   // XMMatrixTranslation(1,1,0)
    const Mat4 sc = Mat4::Rows(0.5f, 0, 0, 0, 0, 0.5f, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1);  // XMMatrixScaling(.5,.5,1)
    return (proj * tr * sc).Inverse().Transpose();
}

}  // namespace Pupil::util
