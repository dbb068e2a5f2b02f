// instanced_splat_renderer.h — drop-in for src/instanced_splat_renderer.h:1-34.
//
// Same class name and methods.  The Metal handles become HIP ones:
//   initialize(void* device)  -> `device` points to an int HIP device ordinal
//                                (nullptr = device 0)
//   render(void* commandBuffer, void* drawableTexture, ...)
//                             -> commandBuffer = hipStream_t (nullptr = default
//                                stream), drawableTexture = float* device
//                                framebuffer, width*height*4 fp32 RGBA
// Everything is forwarded to the C-ABI in gsplat.h.
#pragma once

#include <string>
#include <vector>

#include "gsplat.h"
#include "gsplat/gs_math.h"

struct SplatInstance {  // instanced_splat_renderer.h:6-11 (56-B AoS record)
    float rotation[4];
    float scale[3];
    float position[3];
    float color[4];
};

class InstancedSplatRenderer {
public:
    explicit InstancedSplatRenderer(std::string filepath, const gs_options* opt = nullptr);
    ~InstancedSplatRenderer();
    InstancedSplatRenderer(const InstancedSplatRenderer&) = delete;
    InstancedSplatRenderer& operator=(const InstancedSplatRenderer&) = delete;

    bool initialize(void* device);

    void render(void* commandBuffer, void* drawableTexture, const simd_float4x4& viewMatrix,
                const simd_float4x4& projectionMatrix, float viewportWidth, float viewportHeight);

    int getPointCount() const;

    // Same, into a BGRA8Unorm drawable-format device buffer (width*height*4 B),
    // the reference's drawable pixel format (metal_renderer.mm:58).
    void renderBGRA8(void* commandBuffer, void* drawableTexture, const simd_float4x4& viewMatrix,
                     const simd_float4x4& projectionMatrix, float viewportWidth, float viewportHeight);

    // Additions (not in the reference): status of the last call, frame stats.
    gs_status lastStatus() const { return status_; }
    gs_stats lastStats() const;
    gs_handle* handle() const { return handle_; }

private:
    gs_handle* handle_ = nullptr;
    gs_status status_ = GS_OK;
};
