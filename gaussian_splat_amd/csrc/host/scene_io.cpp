// scene_io.cpp — host scene ingest into the HBM plane layout (scene_io.h).
//
// Reference path replaced: PLYLoader::load
// converts one vertex at a time on one thread into a 248-B PointData vector
// (src/ply_loader.cpp:88-146), the renderer copies that into 56-B SplatInstance
// AoS with the crop (instanced_splat_renderer.mm:359-388) and uploads it.
// Here a binary file is mapped, its vertices are converted on all host cores
// straight into the device planes, and the crop is a parallel count + scan +
// compacting write.  The per-property arithmetic is ply_convert.h, shared
// with the PLYLoader drop-in, so the floats are the same.
#include "scene_io.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ply_convert.h"

namespace gsio {

int sh_coeffs(int deg) { return deg <= 0 ? 0 : (deg == 1 ? 3 : (deg == 2 ? 8 : 15)); }

void HostPlanes::alloc(int64_t count, int deg) {
    n = count;
    sh_degree = deg;
    const size_t m = (size_t)std::max<int64_t>(count, 0);
    p0.alloc(m * 4);
    p1.alloc(m * 4);
    p2.alloc(m * 4);
    p3.alloc(m * 2);
    sh4.alloc((size_t)np4() * m * 4);
    sh1.alloc(tail() ? m : 0);
}

int load_threads() {
    const char* e = std::getenv("GS_LOAD_THREADS");
    if (!e) e = std::getenv("OMP_NUM_THREADS");
    int t = e ? std::atoi(e) : 0;
    if (t <= 0) t = (int)std::max(1u, std::thread::hardware_concurrency());
    return std::min(t, 64);
}

namespace {

// f(chunk, begin, end) over [0, n) in `chunks` contiguous chunks, one thread each.
template <typename F>
void parallel_chunks(int64_t n, int chunks, F&& f) {
    if (chunks <= 1 || n < 2) {
        f(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> pool;
    pool.reserve((size_t)chunks);
    for (int c = 0; c < chunks; ++c) {
        const int64_t b = n * c / chunks, e = n * (c + 1) / chunks;
        pool.emplace_back([&f, c, b, e] { f(c, b, e); });
    }
    for (auto& t : pool) t.join();
}

int chunks_for(int64_t n) { return n < 65536 ? 1 : load_threads(); }

// One splat in the reference's SplatInstance terms (+ the SH coefficients).
struct Splat {
    float pos[3], opacity, rot[4], scale[3], color[3];
    const float* rest;  // 45 f_rest in file (channel-major) order, or null
};

inline void put(const HostPlanes& P, int64_t k, const Splat& s) {
    float* a = P.p0.data() + 4 * k;
    a[0] = s.pos[0], a[1] = s.pos[1], a[2] = s.pos[2], a[3] = s.opacity;
    std::memcpy(P.p1.data() + 4 * k, s.rot, 16);
    float* c = P.p2.data() + 4 * k;
    c[0] = s.scale[0], c[1] = s.scale[1], c[2] = s.scale[2], c[3] = s.color[0];
    float* d = P.p3.data() + 2 * k;
    d[0] = s.color[1], d[1] = s.color[2];
    const int K = sh_coeffs(P.sh_degree);
    if (!K) return;
    // k-major, rgb-interleaved coefficient stream: flat j = 3k + ch <- f_rest[ch*15 + k]
    float flat[48];
    for (int kk = 0; kk < K; ++kk)
        for (int ch = 0; ch < 3; ++ch) flat[3 * kk + ch] = s.rest ? s.rest[ch * 15 + kk] : 0.0f;
    const int NF = 3 * K, NP4 = NF / 4;
    const size_t n = (size_t)P.n;
    for (int m = 0; m < NP4; ++m) std::memcpy(P.sh4.data() + ((size_t)m * n + (size_t)k) * 4, &flat[4 * m], 16);
    if (NF % 4) P.sh1.data()[k] = flat[NF - 1];
}

inline bool kept(const float* p, bool crop, float r) {
    return !crop || (std::fabs(p[0]) < r && std::fabs(p[1]) < r && std::fabs(p[2]) < r);
}

// Crop + pack: pos(i, float[3]) gives the position the crop tests, splat(i,
// Splat&) the whole splat.  Two parallel passes when cropping (count kept per
// chunk, then write at the chunk's scanned offset), one otherwise.
template <typename PosF, typename SplatF>
gs_status build(int64_t n, bool crop, float r, int deg, PosF&& pos, SplatF&& splat, HostPlanes* out) {
    const int chunks = chunks_for(n);
    std::vector<int64_t> base((size_t)chunks + 1, 0);
    if (crop) {
        parallel_chunks(n, chunks, [&](int c, int64_t b, int64_t e) {
            int64_t k = 0;
            float p[3];
            for (int64_t i = b; i < e; ++i) {
                pos(i, p);
                k += kept(p, true, r) ? 1 : 0;
            }
            base[(size_t)c + 1] = k;
        });
        for (int c = 0; c < chunks; ++c) base[(size_t)c + 1] += base[(size_t)c];
    } else {
        for (int c = 0; c <= chunks; ++c) base[(size_t)c] = n * c / chunks;
    }
    try {
        out->alloc(crop ? base[(size_t)chunks] : n, deg);
    } catch (const std::bad_alloc&) {
        return GS_ERR_OOM;
    }
    parallel_chunks(n, chunks, [&](int c, int64_t b, int64_t e) {
        int64_t k = base[(size_t)c];
        Splat s;
        float p[3];
        for (int64_t i = b; i < e; ++i) {
            if (crop) {
                pos(i, p);
                if (!kept(p, true, r)) continue;
            }
            splat(i, s);
            put(*out, k++, s);
        }
    });
    return GS_OK;
}

}  // namespace

gs_status planes_from_soa(const gs_scene_soa& sc, float crop_radius, bool crop, int sh_degree, HostPlanes* out) {
    auto pos = [&](int64_t i, float* p) { std::memcpy(p, sc.pos + 3 * i, 12); };
    auto splat = [&](int64_t i, Splat& s) {
        std::memcpy(s.pos, sc.pos + 3 * i, 12);
        s.opacity = sc.opacity[i];
        std::memcpy(s.rot, sc.rot + 4 * i, 16);
        std::memcpy(s.scale, sc.scale + 3 * i, 12);
        std::memcpy(s.color, sc.color + 3 * i, 12);
        s.rest = sc.sh_rest ? sc.sh_rest + 45 * i : nullptr;
    };
    return build(sc.n, crop, crop_radius, sh_degree, pos, splat, out);
}

gs_status planes_from_points(const PointData* pts, int64_t n, const float* raw_dc, float crop_radius, bool crop,
                             int sh_degree, HostPlanes* out) {
    auto pos = [&](int64_t i, float* p) { p[0] = pts[i].x, p[1] = pts[i].y, p[2] = pts[i].z; };
    auto splat = [&](int64_t i, Splat& s) {
        const PointData& q = pts[i];
        s.pos[0] = q.x, s.pos[1] = q.y, s.pos[2] = q.z;
        s.opacity = q.opacity;
        s.rot[0] = q.rot_0, s.rot[1] = q.rot_1, s.rot[2] = q.rot_2, s.rot[3] = q.rot_3;
        s.scale[0] = q.scale_x, s.scale[1] = q.scale_y, s.scale[2] = q.scale_z;
        if (sh_degree > 0 && raw_dc) std::memcpy(s.color, raw_dc + 3 * i, 12);
        else s.color[0] = q.r, s.color[1] = q.g, s.color[2] = q.b;
        s.rest = q.sh_rest;
    };
    return build(n, crop, crop_radius, sh_degree, pos, splat, out);
}

namespace {

struct Mapping {
    void* base = MAP_FAILED;
    size_t bytes = 0;
    ~Mapping() {
        if (base != MAP_FAILED) munmap(base, bytes);
    }
};

}  // namespace

gs_status planes_from_ply(const char* path, float crop_radius, bool crop, int sh_degree, HostPlanes* out,
                          bool* handled) {
    using namespace gsply;
    *handled = false;
    int vcount = 0;
    std::vector<std::string> names;
    long long off = 0;
    if (!PLYLoader::scanBinary(path, vcount, names, off)) return GS_OK;  // ASCII / bad header: PLYLoader
    const size_t np = names.size(), stride = np * 4;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return GS_OK;
    struct stat st {};
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < (size_t)off + (size_t)vcount * stride) {
        close(fd);  // truncated payload: PLYLoader replays the reference's chunk-buffer reuse
        return GS_OK;
    }
    Mapping map;
    map.bytes = (size_t)st.st_size;
    map.base = mmap(nullptr, map.bytes, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (map.base == MAP_FAILED) return GS_OK;
    (void)madvise(map.base, map.bytes, MADV_WILLNEED);
    const char* data = static_cast<const char*>(map.base) + off;

    std::vector<int> slot(np);
    int col[S_REST] = {};  // last property index of each named slot (load() overwrites in file order)
    std::fill(std::begin(col), std::end(col), -1);
    for (size_t j = 0; j < np; ++j) {
        slot[j] = slot_of(names[j]);
        if (slot[j] >= 0 && slot[j] < S_REST) col[slot[j]] = (int)j;
    }
    auto val = [&](int64_t i, int j) {
        float v;
        std::memcpy(&v, data + (size_t)i * stride + (size_t)j * 4, 4);  // 4 B per property, as load() reads
        return v;
    };
    auto pos = [&](int64_t i, float* p) {
        for (int c = 0; c < 3; ++c) p[c] = col[S_X + c] >= 0 ? val(i, col[S_X + c]) : 0.0f;
    };
    auto splat = [&](int64_t i, Splat& s) {
        // the reference's per-vertex conversion into a PointData (defaults for
        // absent properties), then its SplatInstance fields
        thread_local PointData q;
        q = PointData();
        const char* v = data + (size_t)i * stride;
        for (size_t j = 0; j < np; ++j) {
            float x;
            std::memcpy(&x, v + j * 4, 4);
            store(q, slot[j], x);
        }
        float dc[3];
        for (int c = 0; c < 3; ++c) dc[c] = col[S_R + c] >= 0 ? val(i, col[S_R + c]) : 0.0f;
        dc_to_rgb(q);
        s.pos[0] = q.x, s.pos[1] = q.y, s.pos[2] = q.z;
        s.opacity = q.opacity;
        s.rot[0] = q.rot_0, s.rot[1] = q.rot_1, s.rot[2] = q.rot_2, s.rot[3] = q.rot_3;
        s.scale[0] = q.scale_x, s.scale[1] = q.scale_y, s.scale[2] = q.scale_z;
        if (sh_degree > 0) std::memcpy(s.color, dc, 12);
        else s.color[0] = q.r, s.color[1] = q.g, s.color[2] = q.b;
        s.rest = q.sh_rest;
    };
    gs_status st2 = build(vcount, crop, crop_radius, sh_degree, pos, splat, out);
    if (st2 == GS_OK) *handled = true;
    return st2;
}

void planes_subset(const HostPlanes& src, int64_t b, int64_t e, HostPlanes* out) {
    const int64_t m = std::max<int64_t>(e - b, 0);
    if (b == 0 && m == src.n) {  // read-only planes: share them
        *out = src;
        return;
    }
    out->alloc(m, src.sh_degree);
    if (!m) return;
    std::memcpy(out->p0.data(), src.p0.data() + 4 * b, (size_t)m * 16);
    std::memcpy(out->p1.data(), src.p1.data() + 4 * b, (size_t)m * 16);
    std::memcpy(out->p2.data(), src.p2.data() + 4 * b, (size_t)m * 16);
    std::memcpy(out->p3.data(), src.p3.data() + 2 * b, (size_t)m * 8);
    for (int k = 0; k < src.np4(); ++k)
        std::memcpy(out->sh4.data() + (size_t)k * m * 4, src.sh4.data() + ((size_t)k * src.n + b) * 4, (size_t)m * 16);
    if (src.tail()) std::memcpy(out->sh1.data(), src.sh1.data() + b, (size_t)m * 4);
}

}  // namespace gsio
