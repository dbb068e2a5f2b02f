// scene_io.h — host-side scene ingest into the device layout (SURVEY §8f
// rank 1: parallel / mmap PLY ingest + direct SoA upload).
//
// A handle keeps its scene on the host as the HBM planes themselves
// (DESIGN.md §4): p0 (x, y, z, opacity), p1 (qw, qx, qy, qz), p2 (sx, sy, sz,
// c0), p3 (c1, c2), SH coefficient planes sh4[m][n] (k-major, r,g,b
// interleaved) and the trailing coefficient sh1[n].  gs_initialize is then
// one copy per plane.  Every builder crops (instanced_splat_renderer.mm:
// 382-386) and converts on all host cores into uninitialised buffers (no
// zero-fill pass), and yields exactly the floats of the reference path
// PLYLoader::load -> PointData -> SplatInstance.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>

#include "gsplat.h"
#include "gsplat/ply_loader.h"

namespace gsio {

// Planes are written once by their builder and read-only afterwards, so
// handles may share them: a full-range gs_create_subset (every rank of a
// replicated group) keeps one host copy of the scene, not one per rank.
struct FloatBuf {
    std::shared_ptr<float[]> p;
    size_t n = 0;
    void alloc(size_t count) {
        p.reset(count ? new float[count] : nullptr);  // uninitialised
        n = count;
    }
    float* data() const { return p.get(); }
};

int sh_coeffs(int deg);  // coefficients per channel: 0, 3, 8, 15

struct HostPlanes {
    int64_t n = 0;
    int sh_degree = 0;
    FloatBuf p0, p1, p2, p3, sh4, sh1;
    int np4() const { return 3 * sh_coeffs(sh_degree) / 4; }   // float4 SH planes
    bool tail() const { return (3 * sh_coeffs(sh_degree)) % 4 != 0; }  // + sh1
    void alloc(int64_t count, int deg);
};

// Worker threads for host conversion (GS_LOAD_THREADS, else OMP_NUM_THREADS,
// else the hardware threads; at most 64).
int load_threads();

// Crop + pack a host SoA scene (gs_scene_soa) / PointData array (+ raw f_dc
// triples for SH > 0, else the converted colour).
gs_status planes_from_soa(const gs_scene_soa& sc, float crop_radius, bool crop, int sh_degree, HostPlanes* out);
gs_status planes_from_points(const PointData* pts, int64_t n, const float* raw_dc, float crop_radius, bool crop,
                             int sh_degree, HostPlanes* out);
// Binary PLY straight into planes: mmap, header as PLYLoader::load reads it,
// vertices converted in parallel chunks.  *handled = false (and GS_OK) for
// files this path leaves to PLYLoader: ASCII, truncated payloads, unreadable
// headers.
gs_status planes_from_ply(const char* path, float crop_radius, bool crop, int sh_degree, HostPlanes* out,
                          bool* handled);
// Splats [b, e) of src (the whole range shares src's buffers).
void planes_subset(const HostPlanes& src, int64_t b, int64_t e, HostPlanes* out);

}  // namespace gsio
