// camera.cpp — TrackballCamera drop-in and the C-ABI
// camera helpers.  Matrices follow trackball_camera.mm:136-163; the
// normalize/dot forms are the contract's, since Apple simd's
// exact float sequence is not available here (parity unpinned, §3).
#include <cmath>
#include <cstring>

#include "gsplat.h"
#include "gsplat/trackball_camera.h"

namespace {

void look_at(const float* eye, const float* center, const float* up, float* m) {
    gs::float3 e{eye[0], eye[1], eye[2]}, c{center[0], center[1], center[2]}, u0{up[0], up[1], up[2]};
    gs::float3 f = gs::normalize(c - e);
    gs::float3 s = gs::normalize(gs::cross(f, u0));
    gs::float3 u = gs::cross(s, f);
    const float cols[16] = {s.x, u.x, -f.x, 0.0f, s.y, u.y, -f.y, 0.0f, s.z, u.z, -f.z, 0.0f,
                            -gs::dot(s, e), -gs::dot(u, e), gs::dot(f, e), 1.0f};
    std::memcpy(m, cols, sizeof cols);
}

void perspective_rad(float fov_rad, float aspect, float zn, float zf, float* m) {
    float ys = 1.0f / std::tan(fov_rad * 0.5f);
    float xs = ys / aspect;
    float zr = zf - zn;
    float zs = -(zf + zn) / zr;
    float wz = -2.0f * zf * zn / zr;
    std::memset(m, 0, 64);
    m[0] = xs;
    m[5] = ys;
    m[10] = zs;
    m[11] = -1.0f;
    m[14] = wz;
}

float deg_to_rad(float deg) { return (float)((double)deg * M_PI / 180.0); }  // .mm:133

}  // namespace

extern "C" void gs_look_at(const float eye[3], const float center[3], const float up[3], float out[16]) {
    look_at(eye, center, up, out);
}

extern "C" void gs_perspective(float fov_degrees, float aspect, float zn, float zf, float out[16]) {
    perspective_rad(deg_to_rad(fov_degrees), aspect, zn, zf, out);
}

// ---- TrackballCamera (trackball_camera.mm) ----------------------------------

TrackballCamera::TrackballCamera()
    : position(simd_make_float3(0, 0, 5)), target(simd_make_float3(0, 0, 0)), up(simd_make_float3(0, -1, 0)),
      distance(5.0f), viewportWidth(800), viewportHeight(600), isRotating(false), isPanning(false),
      lastMousePos(simd_make_float2(0, 0)), mouseDownPos(simd_make_float2(0, 0)) {}

void TrackballCamera::setViewportSize(int w, int h) {
    viewportWidth = w;
    viewportHeight = h;
}

void TrackballCamera::setTarget(simd_float3 t) { target = t; }

void TrackballCamera::setPosition(simd_float3 p) {
    position = p;
    distance = simd_length(position - target);
}

void TrackballCamera::setDistance(float d) {
    distance = simd_clamp(d, minDistance, maxDistance);
    simd_float3 dir = simd_normalize(position - target);
    position = target + dir * distance;
}

void TrackballCamera::handleMouseDown(float x, float y, int button) {
    lastMousePos = simd_make_float2(x, y);
    mouseDownPos = simd_make_float2(x, y);
    if (button == 0) isRotating = true;
    else if (button == 1 || button == 2) isPanning = true;
}

void TrackballCamera::handleMouseUp() {
    isRotating = false;
    isPanning = false;
}

void TrackballCamera::handleMouseMove(float x, float y) {
    simd_float2 cur = simd_make_float2(x, y);
    simd_float2 d = lastMousePos - cur;
    if (isRotating) {
        // world-up yaw then camera-right pitch about the target (.mm:55-83)
        float dx = d.x * rotateSpeed * 0.01f;
        float dy = d.y * rotateSpeed * 0.01f;
        simd_float3 viewDir = simd_normalize(target - position);
        simd_float3 right = simd_normalize(simd_cross(viewDir, simd_make_float3(0, 1, 0)));
        simd_quatf rx = simd_quaternion(-dy, right);
        simd_quatf ry = simd_quaternion(-dx, simd_make_float3(0, 1, 0));
        simd_quatf rot = simd_mul(ry, rx);
        simd_float3 off = simd_act(rot, position - target);
        position = target + off;
        up = simd_normalize(simd_act(rot, up));
    } else if (isPanning) {
        simd_float3 right = simd_normalize(simd_cross(target - position, up));
        simd_float3 upv = simd_normalize(simd_cross(right, target - position));
        float px = d.x * panSpeed * distance / viewportHeight;
        float py = -d.y * panSpeed * distance / viewportHeight;
        simd_float3 off = right * px + upv * py;
        position += off;
        target += off;
    }
    lastMousePos = cur;
}

void TrackballCamera::handleScroll(float delta) {
    float zoom = std::pow(0.95f, delta * zoomSpeed);
    setDistance(distance * zoom);
}

simd_float3 TrackballCamera::projectToSphere(float x, float y) {
    float nx = (2.0f * x / viewportWidth) - 1.0f;
    float ny = 1.0f - (2.0f * y / viewportHeight);
    float l = nx * nx + ny * ny;
    float z = l <= 0.5f ? std::sqrt(1.0f - l) : 0.5f / std::sqrt(l);
    return simd_normalize(simd_make_float3(nx, ny, z));
}

simd_float4x4 TrackballCamera::getViewMatrix() const { return makeLookAt(position, target, up); }

simd_float4x4 TrackballCamera::getProjectionMatrix() const {
    float aspect = (float)viewportWidth / (float)viewportHeight;
    return makePerspective(deg_to_rad(fov), aspect, nearPlane, farPlane);
}

simd_float4x4 TrackballCamera::makeLookAt(simd_float3 eye, simd_float3 center, simd_float3 u) const {
    simd_float4x4 m;
    const float e[3] = {eye.x, eye.y, eye.z}, c[3] = {center.x, center.y, center.z}, up3[3] = {u.x, u.y, u.z};
    look_at(e, c, up3, m.data());
    return m;
}

simd_float4x4 TrackballCamera::makePerspective(float fovRadians, float aspect, float zn, float zf) const {
    simd_float4x4 m;
    perspective_rad(fovRadians, aspect, zn, zf, m.data());
    return m;
}

simd_quatf TrackballCamera::rotationBetweenVectors(simd_float3 start, simd_float3 dest) {
    start = simd_normalize(start);
    dest = simd_normalize(dest);
    float cosT = simd_dot(start, dest);
    if (cosT < -0.999999f) {
        simd_float3 axis = simd_cross(simd_make_float3(0, 0, 1), start);
        if (simd_length(axis) < 0.01f) axis = simd_cross(simd_make_float3(1, 0, 0), start);
        return simd_quaternion((float)M_PI, simd_normalize(axis));
    }
    simd_float3 axis = simd_cross(start, dest);
    float s = std::sqrt((1.0f + cosT) * 2.0f);
    float inv = 1.0f / s;
    // Argument order as the reference passes it (trackball_camera.mm:187):
    // simd_quaternion(ix, iy, iz, r) receives (s/2, axis/s), so the real part
    // lands in ix.  Kept for behaviour-identical drags (drop-in contract).
    return simd_quaternion(s * 0.5f, axis.x * inv, axis.y * inv, axis.z * inv);
}
