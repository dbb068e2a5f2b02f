// trackball_camera.h — drop-in for src/trackball_camera.h:1-64 with the Apple
// simd types replaced by gsplat/gs_math.h (same names via simd_* aliases,
// same column-major layout).  Defaults and matrices match the reference
// (trackball_camera.mm:5-17, 127-163).
#pragma once

#include "gsplat/gs_math.h"

class TrackballCamera {
public:
    TrackballCamera();

    void setViewportSize(int width, int height);
    void setTarget(simd_float3 target);
    void setPosition(simd_float3 position);
    void setDistance(float distance);

    void handleMouseDown(float x, float y, int button);
    void handleMouseMove(float x, float y);
    void handleMouseUp();
    void handleScroll(float delta);

    simd_float4x4 getViewMatrix() const;
    simd_float4x4 getProjectionMatrix() const;
    simd_float3 getPosition() const { return position; }
    simd_float3 getTarget() const { return target; }
    simd_float3 getUp() const { return up; }

    float rotateSpeed = 1.0f;
    float zoomSpeed = 1.2f;
    float panSpeed = 0.3f;
    float minDistance = 0.1f;
    float maxDistance = 100.0f;

    float fov = 45.0f;
    float nearPlane = 0.1f;
    float farPlane = 1000.0f;

private:
    simd_float3 position;
    simd_float3 target;
    simd_float3 up;
    float distance;
    int viewportWidth;
    int viewportHeight;
    bool isRotating;
    bool isPanning;
    simd_float2 lastMousePos;
    simd_float2 mouseDownPos;

    simd_float3 projectToSphere(float x, float y);
    simd_float4x4 makeLookAt(simd_float3 eye, simd_float3 center, simd_float3 up) const;
    simd_float4x4 makePerspective(float fovRadians, float aspect, float near, float far) const;
    simd_quatf rotationBetweenVectors(simd_float3 start, simd_float3 dest);
};
