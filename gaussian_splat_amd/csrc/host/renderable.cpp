// renderable.cpp — Renderable value types (src/renderable.cpp:1-78 behaviour:
// grid/axes line lists, PLY -> uint8 point vertices).
#include "gsplat/renderable.h"

#include <algorithm>
#include <cmath>

#include "gsplat/ply_loader.h"

Grid::Grid(int size, float spacing) {
    const float half = size * spacing * 0.5f;
    const uint8_t c[4] = {255, 255, 255, 230};
    auto line = [&](float x0, float z0, float x1, float z1) {
        vertices.push_back({{x0, 0.0f, z0}, {c[0], c[1], c[2], c[3]}});
        vertices.push_back({{x1, 0.0f, z1}, {c[0], c[1], c[2], c[3]}});
    };
    for (int i = 0; i <= size; i++) line(-half, -half + i * spacing, half, -half + i * spacing);
    for (int i = 0; i <= size; i++) line(-half + i * spacing, -half, -half + i * spacing, half);
}

Axes::Axes(float length) {
    const uint8_t rgb[3][4] = {{255, 0, 0, 255}, {0, 255, 0, 255}, {0, 0, 255, 255}};
    for (int a = 0; a < 3; ++a) {
        Vertex o{{0.0f, 0.0f, 0.0f}, {rgb[a][0], rgb[a][1], rgb[a][2], rgb[a][3]}};
        Vertex e = o;
        e.position[a] = length;
        vertices.push_back(o);
        vertices.push_back(e);
    }
}

TriangleMesh::TriangleMesh(const std::vector<Vertex>& verts) : vertices(verts), modelMatrix(matrix_identity_float4x4) {}

PointCloud::PointCloud(int numPoints, float radius) {
    // Fibonacci sphere: deterministic, evenly spread.
    const float golden = 2.39996322972865332f;
    for (int i = 0; i < numPoints; ++i) {
        float y = numPoints > 1 ? 1.0f - 2.0f * (i + 0.5f) / numPoints : 0.0f;
        float r = std::sqrt(std::max(0.0f, 1.0f - y * y));
        float th = golden * i;
        vertices.push_back({{radius * r * std::cos(th), radius * y, radius * r * std::sin(th)}, {255, 255, 255, 255}});
    }
}

GaussianSplat::GaussianSplat(const std::string& filepath) : loaded(false) {
    std::vector<PointData> pts;
    if (!PLYLoader::load(filepath, pts)) return;
    vertices.reserve(pts.size());
    for (const auto& p : pts) {
        Vertex v;
        v.position[0] = p.x;
        v.position[1] = p.y;
        v.position[2] = p.z;
        v.color[0] = static_cast<uint8_t>(p.r * 255.0f);
        v.color[1] = static_cast<uint8_t>(p.g * 255.0f);
        v.color[2] = static_cast<uint8_t>(p.b * 255.0f);
        v.color[3] = static_cast<uint8_t>(p.opacity * 255.0f);
        vertices.push_back(v);
    }
    loaded = true;
}
