// gs_math.h — small column-major vector/matrix types that replace Apple
// <simd/simd.h> on the splat path (SURVEY §8b "Other drop-ins").  Layout is
// identical to simd_float4x4: four float4 columns, m.columns[c][r].
// The simd_* aliases let host code written against the reference's camera /
// renderer headers compile unchanged.
#pragma once

#include <cmath>
#include <cstdint>

namespace gs {

struct float2 { float x, y; };
struct float3 { float x, y, z; };
struct float4 {
    float x, y, z, w;
    float& operator[](int i) { return (&x)[i]; }
    float operator[](int i) const { return (&x)[i]; }
};
struct float4x4 {
    float4 columns[4];
    const float* data() const { return &columns[0].x; }
    float* data() { return &columns[0].x; }
};
struct quatf { float4 vector; };  // (x, y, z, w) like simd_quatf

inline float2 make_float2(float x, float y) { return {x, y}; }
inline float3 make_float3(float x, float y, float z) { return {x, y, z}; }
inline float4 make_float4(float x, float y, float z, float w) { return {x, y, z, w}; }
inline float3 operator+(float3 a, float3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline float3 operator-(float3 a, float3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float3 operator*(float3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
inline float3& operator+=(float3& a, float3 b) { a = a + b; return a; }
inline float2 operator-(float2 a, float2 b) { return {a.x - b.x, a.y - b.y}; }
inline float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(float3 a) { return std::sqrt(dot(a, a)); }
inline float3 normalize(float3 a) { float l = length(a); return {a.x / l, a.y / l, a.z / l}; }
inline float3 cross(float3 a, float3 b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline float clamp(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

inline float4x4 identity4x4() {
    float4x4 m{};
    for (int i = 0; i < 4; ++i) m.columns[i][i] = 1.0f;
    return m;
}
inline float4x4 matrix4x4(float4 c0, float4 c1, float4 c2, float4 c3) { return {{c0, c1, c2, c3}}; }

// a·b with the fixed summation order used everywhere on the path.
inline float4x4 mul(const float4x4& a, const float4x4& b) {
    float4x4 o{};
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            o.columns[c][r] = ((a.columns[0][r] * b.columns[c][0] + a.columns[1][r] * b.columns[c][1]) +
                               a.columns[2][r] * b.columns[c][2]) + a.columns[3][r] * b.columns[c][3];
    return o;
}

// Unit quaternion for a rotation of `angle` radians about `axis` (simd_quaternion).
inline quatf quaternion(float angle, float3 axis) {
    float3 n = normalize(axis);
    float s = std::sin(angle * 0.5f);
    return {{n.x * s, n.y * s, n.z * s, std::cos(angle * 0.5f)}};
}
inline quatf quaternion(float ix, float iy, float iz, float r) { return {{ix, iy, iz, r}}; }
inline quatf mul(quatf p, quatf q) {  // Hamilton product p*q
    const float4 a = p.vector, b = q.vector;
    return {{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
             a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z}};
}
inline float3 act(quatf q, float3 v) {  // rotate v by unit quaternion q (simd_act)
    const float3 u = {q.vector.x, q.vector.y, q.vector.z};
    const float s = q.vector.w;
    float3 t = cross(u, v) * 2.0f;
    return v + t * s + cross(u, t);
}

}  // namespace gs

// Apple-simd spellings used by the reference's host API (trackball_camera.h,
// instanced_splat_renderer.h, renderable.h).
using simd_float2 = gs::float2;
using simd_float3 = gs::float3;
using simd_float4 = gs::float4;
using simd_float4x4 = gs::float4x4;
using simd_quatf = gs::quatf;
inline simd_float2 simd_make_float2(float x, float y) { return gs::make_float2(x, y); }
inline simd_float3 simd_make_float3(float x, float y, float z) { return gs::make_float3(x, y, z); }
inline simd_float4 simd_make_float4(float x, float y, float z, float w) { return gs::make_float4(x, y, z, w); }
inline float simd_dot(simd_float3 a, simd_float3 b) { return gs::dot(a, b); }
inline float simd_length(simd_float3 a) { return gs::length(a); }
inline simd_float3 simd_normalize(simd_float3 a) { return gs::normalize(a); }
inline simd_float3 simd_cross(simd_float3 a, simd_float3 b) { return gs::cross(a, b); }
inline float simd_clamp(float v, float lo, float hi) { return gs::clamp(v, lo, hi); }
inline simd_float4x4 simd_matrix(simd_float4 a, simd_float4 b, simd_float4 c, simd_float4 d) {
    return gs::matrix4x4(a, b, c, d);
}
inline simd_float4x4 simd_mul(const simd_float4x4& a, const simd_float4x4& b) { return gs::mul(a, b); }
inline simd_quatf simd_mul(simd_quatf a, simd_quatf b) { return gs::mul(a, b); }
inline simd_quatf simd_quaternion(float angle, simd_float3 axis) { return gs::quaternion(angle, axis); }
inline simd_quatf simd_quaternion(float ix, float iy, float iz, float r) { return gs::quaternion(ix, iy, iz, r); }
inline simd_float3 simd_act(simd_quatf q, simd_float3 v) { return gs::act(q, v); }
static const simd_float4x4 matrix_identity_float4x4 = gs::identity4x4();
