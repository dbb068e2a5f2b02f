// ply_loader.h — drop-in for the reference's src/ply_loader.h:1-44.
// Same struct, same class, same static entry point and bool contract; the
// implementation (gaussian_splat_amd/csrc/host/ply_loader.cpp) reads the
// file with one bulk read and converts binary vertices on all host cores.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

// 62 floats, 248 bytes — identical layout to src/ply_loader.h:7-28.
struct PointData {
    float x, y, z;
    float nx, ny, nz;
    float r, g, b;                     // loader-converted DC colour (shToRGB)
    float opacity;                     // sigmoid(opacity)
    float scale_x, scale_y, scale_z;   // exp(scale_i)
    float rot_0, rot_1, rot_2, rot_3;  // w, x, y, z (raw)
    float sh_rest[45];                 // f_rest_0..44 in file order

    PointData()
        : x(0), y(0), z(0), nx(0), ny(0), nz(0), r(0), g(0), b(0), opacity(1.0f), scale_x(0.01f),
          scale_y(0.01f), scale_z(0.01f), rot_0(1), rot_1(0), rot_2(0), rot_3(0) {
        for (int i = 0; i < 45; i++) sh_rest[i] = 0.0f;
    }
};

class PLYLoader {
public:
    // src/ply_loader.h:33 — reproduces the reference's results, quirks included.
    static bool load(const std::string& filepath, std::vector<PointData>& points);

    // Extended entry point: also returns the raw f_dc triples (needed for SH
    // degree > 0 colour, which the reference discards at load time).
    static bool load(const std::string& filepath, std::vector<PointData>& points, std::vector<float>* raw_dc,
                     bool compat = true);

    // Header of a binary PLY as load() reads it (properties of every element,
    // 4 bytes each): vertex count, property names and the payload offset.
    // False for ASCII files and headers load() rejects.
    static bool scanBinary(const std::string& filepath, int& vertexCount, std::vector<std::string>& names,
                           long long& dataOffset);

private:
    struct PropertyInfo {
        std::string name;
        std::string type;
    };
    static bool parseHeader(std::istream& file, int& vertexCount, std::vector<PropertyInfo>& properties,
                            bool& isBinary);
};
