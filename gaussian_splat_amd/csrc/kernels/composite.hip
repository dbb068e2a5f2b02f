// composite.hip — per-tile front-to-back alpha composite.
//
// One 256-lane workgroup per 16x16 tile, one pixel per lane.  The tile's
// depth-sorted splat list is streamed through LDS in batches of 256 records
// (each lane gathers one 48-B record by splat id), then every lane walks the
// batch: coverage (K6 closed form), gaussian + 0.01 cutoff (F1,
// tile.metal:191-197), composite (A1: tile.metal:251-266, or A1': live
// 50-layer rule, 50layer.metal:208-222).  Per-splat pixel rects give a
// wave-uniform skip (the 64 lanes of a wave are 4 pixel rows of the tile),
// and the workgroup stops fetching once every lane has saturated.
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

template <int MODE>
__global__ __launch_bounds__(256) void composite_kernel(CompositeArgs a) {
    __shared__ float4 s0[kTileThreads], s1[kTileThreads], s2[kTileThreads];
    // Grid covers only the owned tile rows: ty = row_rem + k * row_mod.
    const int owned_row = blockIdx.x / a.tiles_x;
    const int tx = blockIdx.x - owned_row * a.tiles_x;
    const int ty = a.row_rem + owned_row * a.row_mod;
    const int tile = ty * a.tiles_x + tx;
    const int width = a.width, height = a.height;
    const uint32_t* __restrict__ sorted_vals = a.vals;
    const float4* __restrict__ rec = a.rec;
    const int tid = threadIdx.x;
    const int px = tx * kTile + (tid & 15);
    const int py = ty * kTile + (tid >> 4);
    const bool inside = px < width && py < height;
    const float fx = (float)px + 0.5f;
    const float fy = (float)py + 0.5f;
    // pixel rows covered by this wave, tile columns
    const uint32_t wy0 = (uint32_t)(ty * kTile + (tid >> 6) * 4), wy1 = wy0 + 3;
    const uint32_t wx0 = (uint32_t)(tx * kTile), wx1 = wx0 + 15;

    const uint2 rg = a.ranges[tile];
    float A = 0.0f;  // tile: accumulated alpha; live50: transmittance stored as T
    float T = 1.0f;
    float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    bool done = !inside;
    bool any = false;

    for (uint32_t b = rg.x; b < rg.y; b += kTileThreads) {
        if (__syncthreads_count(!done) == 0) break;
        const uint32_t j = b + tid;
        if (j < rg.y) {
            const uint32_t id = sorted_vals[j];
            const float4* r = rec + (size_t)a.rec_stride * id;
            s0[tid] = r[0];
            s1[tid] = r[1];
            s2[tid] = r[2];
        }
        __syncthreads();
        const uint32_t cnt = rg.y - b < (uint32_t)kTileThreads ? rg.y - b : (uint32_t)kTileThreads;
        for (uint32_t k = 0; k < cnt; ++k) {
            if (__builtin_amdgcn_readfirstlane((int)__all(done))) break;
            const float4 c = s2[k];
            const uint32_t lo = __builtin_amdgcn_readfirstlane(__float_as_uint(c.z));
            const uint32_t hi = __builtin_amdgcn_readfirstlane(__float_as_uint(c.w));
            // wave-uniform rect skip (rect is conservative)
            if ((hi >> 16) < wy0 || (lo >> 16) > wy1 || (hi & 0xFFFFu) < wx0 || (lo & 0xFFFFu) > wx1) continue;
            const float4 aa = s0[k];
            const float4 bb = s1[k];
            const float dx = fx - aa.x;
            const float dy = aa.y - fy;
            const float u = __builtin_fmaf(dy, aa.w, dx * aa.z);
            const float v = __builtin_fmaf(dy, bb.y, dx * bb.x);
            const float q = __builtin_fmaf(v, v, u * u);
            if (!done && fabsf(u) <= 3.0f && fabsf(v) <= 3.0f && q <= kQMax) {
                const float alpha = bb.z * gs_exp(-0.5f * q);
                any = true;
                if constexpr (MODE == 0) {
                    const float sa = alpha * (1.0f - A);
                    C0 = __builtin_fmaf(bb.w, sa, C0);
                    C1 = __builtin_fmaf(c.x, sa, C1);
                    C2 = __builtin_fmaf(c.y, sa, C2);
                    A = A + sa;
                    if (A >= kSat) done = true;
                } else {
                    C0 = __builtin_fmaf(bb.w, T, C0);
                    C1 = __builtin_fmaf(c.x, T, C1);
                    C2 = __builtin_fmaf(c.y, T, C2);
                    T = T * (1.0f - alpha);
                    if (T < kTMin) done = true;
                }
            }
        }
    }
    if (inside) {
        float4 o;
        if constexpr (MODE == 0) {
            o = make_float4(C0, C1, C2, A);
        } else {
            o = make_float4(C0, C1, C2, any ? 1.0f - T : 0.0f);
        }
        // compact = owned tile rows stacked (multi-GPU band buffer)
        const int orow = a.compact ? owned_row * kTile + (py - ty * kTile) : py;
        a.out[(size_t)orow * width + px] = o;
    }
}

hipError_t launch_composite(const CompositeArgs& a, int mode, hipStream_t st) {
    if (a.row_mod < 1 || a.row_rem < 0 || a.row_rem >= a.row_mod) return hipErrorInvalidValue;
    const int owned_rows = a.tiles_y > a.row_rem ? (a.tiles_y - a.row_rem + a.row_mod - 1) / a.row_mod : 0;
    dim3 grid(a.tiles_x * owned_rows);
    if (grid.x == 0) return hipSuccess;
    if (mode == 0)
        composite_kernel<0><<<grid, 256, 0, st>>>(a);
    else
        composite_kernel<1><<<grid, 256, 0, st>>>(a);
    return hipGetLastError();
}

}  // namespace gs
