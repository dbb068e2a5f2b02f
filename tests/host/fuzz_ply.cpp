// Host-only robustness harness for the PLY ingest (PLYLoader::load and the
// direct mmap path gsio::planes_from_ply), built with -fsanitize=address,
// undefined by tests/test_ply_fuzz.py.  Loads every given file, then seeded
// mutants of each: truncations (inside the header and the payload), flipped
// header bytes, and edited vertex counts / property lines.  Any memory error
// or undefined behaviour aborts under the sanitizers; a loader may reject a
// file, but must not crash.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "gsplat/ply_loader.h"
#include "scene_io.h"

static std::string read_file(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static void write_file(const std::string& p, const std::string& s) {
    std::ofstream f(p, std::ios::binary | std::ios::trunc);
    f.write(s.data(), (std::streamsize)s.size());
}

static int load_all(const std::string& p) {
    int ok = 0;
    std::vector<PointData> pts;
    std::vector<float> raw;
    try {
        ok += PLYLoader::load(p, pts) ? 1 : 0;
        ok += PLYLoader::load(p, pts, &raw, 3) ? 1 : 0;
    } catch (const std::bad_alloc&) {
        std::printf("bad_alloc (PLYLoader): %s\n", p.c_str());
    }
    for (int deg = 0; deg <= 3; ++deg)
        for (int crop = 0; crop < 2; ++crop) {
            gsio::HostPlanes hp;
            bool handled = false;
            try {
                if (gsio::planes_from_ply(p.c_str(), 5.0f, crop != 0, deg, &hp, &handled) == GS_OK && handled) ++ok;
            } catch (const std::bad_alloc&) {
                std::printf("bad_alloc (planes_from_ply): %s\n", p.c_str());
            }
        }
    return ok;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: fuzz_ply TMPDIR MUTANTS_PER_FILE FILE...\n");
        return 2;
    }
    const std::string tmp = argv[1];
    const int nmut = std::atoi(argv[2]);
    std::mt19937 rng(12345);
    long loads = 0, accepted = 0;
    for (int a = 3; a < argc; ++a) {
        const std::string src = read_file(argv[a]);
        accepted += load_all(argv[a]);
        ++loads;
        const size_t hdr = src.find("end_header");
        for (int m = 0; m < nmut; ++m) {
            std::string s = src;
            const int kind = m % 5;
            if (kind == 0 && !s.empty()) {  // truncate anywhere
                s.resize(rng() % s.size());
            } else if (kind == 1 && hdr != std::string::npos && hdr + 11 < s.size()) {  // truncate the payload
                s.resize(hdr + 11 + rng() % (s.size() - hdr - 11));
            } else if (kind == 2 && hdr != std::string::npos) {  // flip header bytes
                for (int k = 0; k < 3; ++k) s[rng() % (hdr + 10)] = (char)(rng() & 0xFF);
            } else if (kind == 3) {  // edit the vertex count
                const size_t v = s.find("element vertex ");
                if (v != std::string::npos) {
                    const size_t e = s.find('\n', v);
                    static const char* counts[] = {"0", "1", "-5", "2147483647", "4294967296", "99999999999", "abc",
                                                   "7"};
                    s = s.substr(0, v) + "element vertex " + counts[rng() % 8] + s.substr(e);
                }
            } else if (kind == 4) {  // drop or duplicate a property line
                const size_t p = s.find("property float", rng() % (hdr == std::string::npos ? 1 : hdr + 1));
                if (p != std::string::npos) {
                    const size_t e = s.find('\n', p);
                    if (e != std::string::npos)
                        s = (rng() & 1) ? s.substr(0, p) + s.substr(e + 1) : s.substr(0, e + 1) + s.substr(p);
                }
            }
            const std::string path = tmp + "/mut_" + std::to_string(a) + "_" + std::to_string(m) + ".ply";
            write_file(path, s);
            accepted += load_all(path);
            ++loads;
            std::remove(path.c_str());
        }
    }
    std::printf("fuzz_ply: %ld files, %ld accepted loads\n", loads, accepted);
    return 0;
}
