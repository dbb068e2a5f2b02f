// scan.hip — exclusive prefix sum of per-splat tile counts (reduce-then-scan);
// the counts are derived from the depth-sorted packed rects on the fly.
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kScanIpt = kScanItems / 256;  // 16 consecutive items per lane

struct CountSrc {
    const uint32_t* lo;
    const uint32_t* hi;
    uint32_t world, rank;
};

__device__ __forceinline__ uint32_t count_at(const CountSrc& c, uint32_t i) {
    return rect_tile_count(c.lo[i], c.hi[i], c.world, c.rank);
}

__global__ __launch_bounds__(256) void scan_reduce_kernel(CountSrc src, uint32_t n,
                                                          uint64_t* __restrict__ partials) {
    __shared__ uint64_t tmp[4];
    const uint32_t base = blockIdx.x * kScanItems;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) s += count_at(src, i);
    }
    uint64_t total;
    block256_exclusive_scan<uint64_t>(s, tmp, &total);
    if (threadIdx.x == 0) partials[blockIdx.x] = total;
}

// One workgroup scans all partials (<= a few thousand) exclusively in place.
__global__ __launch_bounds__(256) void scan_partials_kernel(uint64_t* __restrict__ partials, uint32_t nb,
                                                            uint64_t* __restrict__ total) {
    __shared__ uint64_t tmp[4];
    uint64_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
        uint32_t i = b0 + threadIdx.x;
        uint64_t v = i < nb ? partials[i] : 0;
        uint64_t t;
        uint64_t ex = block256_exclusive_scan<uint64_t>(v, tmp, &t);
        if (i < nb) partials[i] = carry + ex;
        carry += t;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void scan_down_kernel(CountSrc src, uint32_t n,
                                                        const uint64_t* __restrict__ partials,
                                                        uint32_t* __restrict__ offsets) {
    __shared__ uint32_t tmp[4];
    const uint32_t base = blockIdx.x * kScanItems + threadIdx.x * kScanIpt;
    uint32_t v[kScanIpt];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        uint32_t idx = base + k;
        v[k] = idx < n ? count_at(src, idx) : 0u;
        s += v[k];
    }
    uint32_t t;
    uint32_t ex = block256_exclusive_scan<uint32_t>(s, tmp, &t);
    uint32_t run = (uint32_t)partials[blockIdx.x] + ex;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        uint32_t idx = base + k;
        if (idx < n) offsets[idx] = run;
        run += v[k];
    }
}

hipError_t launch_tile_count_scan(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, int world,
                                  int rank, uint32_t* offsets, uint64_t* partials, uint64_t* total, hipStream_t st) {
    const CountSrc src{rect_lo, rect_hi, (uint32_t)world, (uint32_t)rank};
    uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) {
        return hipMemsetAsync(total, 0, sizeof(uint64_t), st);
    }
    scan_reduce_kernel<<<nb, 256, 0, st>>>(src, n, partials);
    scan_partials_kernel<<<1, 256, 0, st>>>(partials, nb, total);
    scan_down_kernel<<<nb, 256, 0, st>>>(src, n, partials, offsets);
    return hipGetLastError();
}

}  // namespace gs
