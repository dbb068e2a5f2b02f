// binning.hip — tile binning.
//
// duplicate: every visible splat writes one (key, value) pair per tile of its
//   conservative pixel rect: key = tile_id << 15 | dkey, value = splat index.
//   Pairs are written in splat-index order, so a stable sort keeps the
//   reference's tie rule (equal half depth -> arrival order = index order,
//   shaders/gaussian_splat_tile.metal:244).
// tile_ranges: boundary detection on the sorted keys -> [start, end) per tile.
#include "gs_kernels.h"

namespace gs {

__global__ __launch_bounds__(256) void duplicate_kernel(const float4* __restrict__ rec,
                                                        const uint32_t* __restrict__ dkey,
                                                        const uint32_t* __restrict__ ntiles,
                                                        const uint32_t* __restrict__ offsets, uint32_t n,
                                                        uint32_t tiles_x, uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals) {
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n || ntiles[i] == 0) return;
    float4 c = rec[3 * (size_t)i + 2];
    uint32_t lo = __float_as_uint(c.z), hi = __float_as_uint(c.w);
    uint32_t tx0 = (lo & 0xFFFFu) >> 4, ty0 = (lo >> 16) >> 4;
    uint32_t tx1 = (hi & 0xFFFFu) >> 4, ty1 = (hi >> 16) >> 4;
    uint32_t off = offsets[i];
    uint32_t dk = dkey[i];
    for (uint32_t ty = ty0; ty <= ty1; ++ty) {
        for (uint32_t tx = tx0; tx <= tx1; ++tx) {
            keys[off] = ((ty * tiles_x + tx) << kDepthBits) | dk;
            vals[off] = i;
            ++off;
        }
    }
}

__global__ __launch_bounds__(256) void tile_ranges_kernel(const uint32_t* __restrict__ keys, uint32_t npairs,
                                                          uint2* __restrict__ ranges) {
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= npairs) return;
    uint32_t t = keys[i] >> kDepthBits;
    if (i == 0) {
        ranges[t].x = 0;
    } else {
        uint32_t p = keys[i - 1] >> kDepthBits;
        if (p != t) {
            ranges[p].y = i;
            ranges[t].x = i;
        }
    }
    if (i == npairs - 1) ranges[t].y = npairs;
}

hipError_t launch_duplicate(const float4* rec, const uint32_t* dkey, const uint32_t* ntiles,
                            const uint32_t* offsets, uint32_t n, uint32_t tiles_x, uint32_t* keys,
                            uint32_t* vals, hipStream_t st) {
    if (n == 0) return hipSuccess;
    duplicate_kernel<<<(n + 255) / 256, 256, 0, st>>>(rec, dkey, ntiles, offsets, n, tiles_x, keys, vals);
    return hipGetLastError();
}

hipError_t launch_tile_ranges(const uint32_t* keys, uint32_t npairs, uint2* ranges, uint32_t ntiles_total,
                              hipStream_t st) {
    hipError_t e = hipMemsetAsync(ranges, 0, sizeof(uint2) * ntiles_total, st);
    if (e != hipSuccess || npairs == 0) return e;
    tile_ranges_kernel<<<(npairs + 255) / 256, 256, 0, st>>>(keys, npairs, ranges);
    return hipGetLastError();
}

}  // namespace gs
