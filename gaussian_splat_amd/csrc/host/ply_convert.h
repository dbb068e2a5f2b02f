// ply_convert.h — per-property conversion shared by the PLYLoader drop-in
// (ply_loader.cpp) and the direct PLY -> device-plane ingest (scene_io.cpp),
// so both produce the same floats: property -> PointData slot by name
// (src/ply_loader.cpp:56-82), sigmoid(opacity) (:116), exp(scale) (:117-119),
// DC -> RGB with the clamp and the all-zero skip (:9,11-20,133).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "gsplat/ply_loader.h"

namespace gsply {

constexpr float kShC0 = 0.28209479177387814f;  // ply_loader.cpp:9

enum Slot {
    S_X, S_Y, S_Z, S_NX, S_NY, S_NZ, S_R, S_G, S_B, S_OP, S_SX, S_SY, S_SZ, S_R0, S_R1, S_R2, S_R3, S_REST
};

// PointData float index of a property name, -1 if the loader ignores it.
inline int slot_of(const std::string& n) {
    static const char* names[] = {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2",
                                  "opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1",
                                  "rot_2", "rot_3"};
    for (int i = 0; i < 17; ++i)
        if (n == names[i]) return i;
    if (n.compare(0, 7, "f_rest_") == 0) {
        const char* s = n.c_str() + 7;
        char* end = nullptr;
        long v = std::strtol(s, &end, 10);
        if (end != s && v >= 0 && v < 45) return S_REST + (int)v;
    }
    return -1;
}

inline void store(PointData& p, int slot, float v) {
    float* f = &p.x;
    if (slot < 0) return;
    if (slot == S_OP) f[S_OP] = 1.0f / (1.0f + std::exp(-v));
    else if (slot >= S_SX && slot <= S_SZ) f[slot] = std::exp(v);
    else f[slot] = v;
}

inline void dc_to_rgb(PointData& p) {
    if (p.r != 0 || p.g != 0 || p.b != 0) {
        float* c = &p.r;
        for (int k = 0; k < 3; ++k) {
            float v = 0.5f + kShC0 * c[k];
            c[k] = std::max(0.0f, std::min(1.0f, v));
        }
    }
}

}  // namespace gsply
