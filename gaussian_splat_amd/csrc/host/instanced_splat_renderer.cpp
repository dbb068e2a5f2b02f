// instanced_splat_renderer.cpp — C++ drop-in over the C-ABI
// (src/instanced_splat_renderer.h:13-34 semantics: the ctor never throws and
// leaves an empty scene on load failure (.mm:346-349); render() returns
// silently when there is nothing to draw (.mm:434-440)).
#include "gsplat/instanced_splat_renderer.h"

#include <cstdio>

InstancedSplatRenderer::InstancedSplatRenderer(std::string filepath, const gs_options* opt) {
    status_ = gs_create(filepath.c_str(), opt, &handle_);
    if (status_ != GS_OK) {
        std::fprintf(stderr, "InstancedSplatRenderer: %s\n", gs_last_error());
        handle_ = nullptr;
    }
}

InstancedSplatRenderer::~InstancedSplatRenderer() { gs_destroy(handle_); }

bool InstancedSplatRenderer::initialize(void* device) {
    if (!handle_) return false;
    int ordinal = device ? *static_cast<int*>(device) : 0;
    status_ = gs_initialize(handle_, ordinal);
    if (status_ != GS_OK) std::fprintf(stderr, "InstancedSplatRenderer::initialize: %s\n", gs_last_error());
    return status_ == GS_OK;
}

void InstancedSplatRenderer::render(void* commandBuffer, void* drawableTexture, const simd_float4x4& viewMatrix,
                                    const simd_float4x4& projectionMatrix, float viewportWidth,
                                    float viewportHeight) {
    if (!handle_ || gs_point_count(handle_) == 0 || !drawableTexture) return;
    status_ = gs_render(handle_, viewMatrix.data(), projectionMatrix.data(), (int32_t)viewportWidth,
                        (int32_t)viewportHeight, static_cast<float*>(drawableTexture), 1, commandBuffer);
}

void InstancedSplatRenderer::renderBGRA8(void* commandBuffer, void* drawableTexture, const simd_float4x4& viewMatrix,
                                         const simd_float4x4& projectionMatrix, float viewportWidth,
                                         float viewportHeight) {
    if (!handle_ || gs_point_count(handle_) == 0 || !drawableTexture) return;
    status_ = gs_render_bgra8(handle_, viewMatrix.data(), projectionMatrix.data(), (int32_t)viewportWidth,
                              (int32_t)viewportHeight, static_cast<uint8_t*>(drawableTexture), 1, commandBuffer);
}

int InstancedSplatRenderer::getPointCount() const { return (int)gs_point_count(handle_); }

gs_stats InstancedSplatRenderer::lastStats() const {
    gs_stats s{};
    if (handle_) gs_last_stats(handle_, &s);
    return s;
}
