// oracle/_ref driver: exposes the reference's OWN src/ply_loader.cpp (compiled
// unchanged from /root/reference by oracle/Makefile) through a tiny C ABI so
// tests can pin the oracle's I1 restatement and the product loader against it.
// Test infrastructure only.  This file is ours; no reference source is copied.
#include "ply_loader.h"

#include <cstring>
#include <vector>

static_assert(sizeof(PointData) == 62 * sizeof(float), "PointData is 62 packed floats");

extern "C" long long ref_ply_load(const char* path, float* out, long long max_points) {
    std::vector<PointData> pts;
    bool ok = PLYLoader::load(path, pts);
    long long n = static_cast<long long>(pts.size());
    if (out && max_points > 0) {
        long long m = n < max_points ? n : max_points;
        std::memcpy(out, pts.data(), static_cast<size_t>(m) * sizeof(PointData));
    }
    return ok ? n : -1 - n;  // -1-n: loader returned false (n points still reported)
}
