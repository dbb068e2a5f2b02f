// binning.hip — tile binning.
//
// Depth-first binning: splats are first sorted by their 15-bit depth key
// (stable, so equal half depths keep index = arrival order,
// shaders/gaussian_splat_tile.metal:244), then every splat, visited in that
// order, emits one (bin, splat index) pair per 32x32 bin of its conservative
// pixel rect.  A stable sort of the pairs by bin id alone then yields each
// bin's list in S1 order: 2 digit passes over P (11 bin bits at 1080p)
// instead of 4 over a 28-bit (tile, depth) key, and ~half the pairs of
// 16x16 binning.
// The bin ranges [start, end) come out of the last sort pass (radix_sort.hip).
//
// Bin-first order (the default): the same pairs are emitted in
// splat index order with the splat's depth key carried above the bin id
// (key = dkey << bin_bits | bin), sorted by bin id alone, and each bin's list
// is then put in depth order by a stable per-bin sort (bin_depth_sort.hip).
#include "gs_kernels.h"

namespace gs {

__global__ __launch_bounds__(256) void duplicate_kernel(const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ rect_lo,
                                                        const uint32_t* __restrict__ rect_hi,
                                                        const uint32_t* __restrict__ offsets, uint32_t n,
                                                        uint32_t tiles_x, RowOwnership own, bool masked,
                                                        const uint32_t* __restrict__ dkey, int bin_bits,
                                                        uint32_t* __restrict__ keys,
                                                        uint32_t* __restrict__ vals) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n) return;
    const BinRect r = bin_rect(rect_lo[j], rect_hi[j], masked);
    if (r.empty) return;  // culled
    const uint32_t i = order ? order[j] : j;
    const uint32_t hi = dkey ? dkey[j] << bin_bits : 0u;  // depth key above the bin id
    uint32_t off = offsets[j];
    for (uint32_t by = r.by0; by <= r.by1; ++by) {
        if (!owns_bin_row(by, own)) continue;
        for (uint32_t bx = r.bx0; bx <= r.bx1; ++bx) {
            if (bin_excluded(r, by, bx)) continue;  // the ellipse misses this bin
            keys[off] = hi | (by * tiles_x + bx);
            vals[off] = i;
            ++off;
        }
    }
}

hipError_t launch_duplicate(const uint32_t* order, const uint32_t* rect_lo, const uint32_t* rect_hi,
                            const uint32_t* offsets, uint32_t n, uint32_t tiles_x, RowOwnership own, bool masked,
                            const uint32_t* dkey, int bin_bits, uint32_t* keys, uint32_t* vals, hipStream_t st) {
    if (n == 0) return hipSuccess;
    if (dkey && (order || bin_bits + kDepthBits > 32)) return hipErrorInvalidValue;
    duplicate_kernel<<<(n + 255) / 256, 256, 0, st>>>(order, rect_lo, rect_hi, offsets, n, tiles_x, own, masked,
                                                      dkey, bin_bits, keys, vals);
    return hipGetLastError();
}

}  // namespace gs
