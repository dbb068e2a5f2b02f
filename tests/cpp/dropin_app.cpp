// dropin_app.cpp — the reference's call sites (src/main.mm:55-58, 69-72, 179,
// 192-198) compiled against the drop-in headers (include/gsplat/*.h) and
// libgsplat.so, with no Python in the loop.
//
//   dropin_app <scene.ply> <width> <height> <out.bin> [frames] [bgra8]
//
// Writes to <out.bin>: the view and projection matrices the camera produced
// (2 x 16 float32, column-major), then the last frame's framebuffer (fp32
// RGBA, width*height*4 floats, or BGRA8 bytes with `bgra8`).  Prints
// "points N" (getPointCount) and exits nonzero on any failure.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "gsplat/instanced_splat_renderer.h"
#include "gsplat/trackball_camera.h"

static int die(const char* what) {
    std::fprintf(stderr, "dropin_app: %s (%s)\n", what, gs_last_error());
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s scene.ply width height out.bin [frames] [bgra8]\n", argv[0]);
        return 2;
    }
    const std::string plyPath = argv[1];
    const int drawableWidth = std::atoi(argv[2]), drawableHeight = std::atoi(argv[3]);
    const int frames = argc > 5 ? std::atoi(argv[5]) : 1;
    const bool bgra8 = argc > 6 && std::string(argv[6]) == "bgra8";

    // main.mm:55-58
    TrackballCamera camera;
    camera.setViewportSize(drawableWidth, drawableHeight);
    camera.setPosition(simd_make_float3(0, 2, 5));
    camera.setTarget(simd_make_float3(0, 0, 0));

    // main.mm:69-72: the ctor loads and crops, initialize uploads (device: an ordinal)
    InstancedSplatRenderer splatRenderer(plyPath);
    int device = 0;
    if (!splatRenderer.initialize(&device)) return die("initialize");
    std::printf("points %d\n", splatRenderer.getPointCount());  // main.mm:179

    // the drawable: a device framebuffer; the command buffer: a HIP stream
    const size_t npix = (size_t)drawableWidth * drawableHeight;
    const size_t bytes = npix * (bgra8 ? 4 : 16);
    void* drawable = nullptr;
    hipStream_t commandBuffer = nullptr;
    if (hipMalloc(&drawable, bytes) != hipSuccess) return die("hipMalloc");
    if (hipStreamCreate(&commandBuffer) != hipSuccess) return die("hipStreamCreate");

    // main.mm:192-198, once per frame
    for (int f = 0; f < frames; ++f) {
        if (bgra8)
            splatRenderer.renderBGRA8(commandBuffer, drawable, camera.getViewMatrix(), camera.getProjectionMatrix(),
                                      drawableWidth, drawableHeight);
        else
            splatRenderer.render(commandBuffer, drawable, camera.getViewMatrix(), camera.getProjectionMatrix(),
                                 drawableWidth, drawableHeight);
        if (splatRenderer.lastStatus() != GS_OK) return die("render");
    }
    std::vector<unsigned char> host(bytes);
    if (hipMemcpyAsync(host.data(), drawable, bytes, hipMemcpyDeviceToHost, commandBuffer) != hipSuccess ||
        hipStreamSynchronize(commandBuffer) != hipSuccess)
        return die("readback");

    const simd_float4x4 V = camera.getViewMatrix(), P = camera.getProjectionMatrix();
    FILE* out = std::fopen(argv[4], "wb");
    if (!out) return die("open output");
    const bool ok = std::fwrite(V.data(), 4, 16, out) == 16 && std::fwrite(P.data(), 4, 16, out) == 16 &&
                    std::fwrite(host.data(), 1, bytes, out) == bytes;
    std::fclose(out);
    hipFree(drawable);
    hipStreamDestroy(commandBuffer);
    return ok ? 0 : die("write output");
}
