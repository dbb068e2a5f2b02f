// scan.hip — exclusive prefix sum of per-splat tile counts (reduce-then-scan);
// the counts are derived from the depth-sorted packed rects on the fly.
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kScanIpt = kScanItems / 256;  // 16 consecutive items per lane

struct CountSrc {
    const uint32_t* lo;
    const uint32_t* hi;
    RowOwnership own;
    bool masked;  // rect words carry the bin-exclusion mask
};

__device__ __forceinline__ uint32_t count_at(const CountSrc& c, uint32_t i) {
    return rect_tile_count(c.lo[i], c.hi[i], c.own, c.masked);
}

// Per block: pair count -> partials[b], contributing splats -> partials[nb + b].
__global__ __launch_bounds__(256) void scan_reduce_kernel(CountSrc src, uint32_t n,
                                                          uint64_t* __restrict__ partials) {
    __shared__ uint64_t tmp[4];
    const uint32_t base = blockIdx.x * kScanItems;
    uint64_t s = 0, vis = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) {
            const uint32_t c = count_at(src, i);
            s += c;
            vis += c > 0;
        }
    }
    uint64_t total, vtotal;
    block256_exclusive_scan<uint64_t>(s, tmp, &total);
    block256_exclusive_scan<uint64_t>(vis, tmp, &vtotal);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = total;
        partials[gridDim.x + blockIdx.x] = vtotal;
    }
}

// One workgroup scans all partials (<= a few thousand) exclusively in place.
// seg_sample (may be null): the per-bin depth sort's sample since the last
// scan (bin_depth_sort.hip) is moved into total[2..3] and reset, so it comes
// back to the host with the pair count.
__global__ __launch_bounds__(256) void scan_partials_kernel(uint64_t* __restrict__ partials, uint32_t nb,
                                                            uint64_t* __restrict__ total,
                                                            uint32_t* __restrict__ seg_sample) {
    if (seg_sample && threadIdx.x == 0) {
        total[2] = seg_sample[0];
        total[3] = seg_sample[1];
        seg_sample[0] = 0u;
        seg_sample[1] = 0u;
    }
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
    uint64_t vis = 0;
    for (uint32_t b = threadIdx.x; b < nb; b += 256) vis += partials[nb + b];
    uint64_t vt;
    block256_exclusive_scan<uint64_t>(vis, tmp, &vt);
    if (threadIdx.x == 0) {
        total[0] = carry;
        total[1] = vt;
    }
}

// Down-sweep: counts are loaded striped (coalesced), transposed through LDS
// so each lane scans kScanIpt consecutive items, and stored striped again
// (lane-consecutive stores would be 64 partial-line writes per instruction).
__device__ __forceinline__ uint32_t pad32(uint32_t i) { return i + (i >> 5); }  // LDS bank spread

__global__ __launch_bounds__(256) void scan_down_kernel(CountSrc src, uint32_t n,
                                                        const uint64_t* __restrict__ partials,
                                                        uint32_t* __restrict__ offsets) {
    __shared__ uint32_t tmp[4];
    __shared__ uint32_t st[kScanItems + kScanItems / 32];
    const uint32_t blk = blockIdx.x * kScanItems, tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const uint32_t i = k * 256 + tid;
        st[pad32(i)] = blk + i < n ? count_at(src, blk + i) : 0u;
    }
    __syncthreads();
    uint32_t v[kScanIpt];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        v[k] = st[pad32(tid * kScanIpt + k)];
        s += v[k];
    }
    uint32_t t;
    const uint32_t ex = block256_exclusive_scan<uint32_t>(s, tmp, &t);  // (ends with a barrier)
    uint32_t run = (uint32_t)partials[blockIdx.x] + ex;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        st[pad32(tid * kScanIpt + k)] = run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const uint32_t i = k * 256 + tid;
        if (blk + i < n) offsets[blk + i] = st[pad32(i)];
    }
}

hipError_t launch_tile_count_scan(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, RowOwnership own,
                                  bool masked, uint32_t* offsets, uint64_t* partials, uint64_t* total,
                                  uint32_t* seg_sample, hipStream_t st) {
    const CountSrc src{rect_lo, rect_hi, own, masked};
    uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) {
        return hipMemsetAsync(total, 0, 4 * sizeof(uint64_t), st);
    }
    scan_reduce_kernel<<<nb, 256, 0, st>>>(src, n, partials);
    scan_partials_kernel<<<1, 256, 0, st>>>(partials, nb, total, seg_sample);
    scan_down_kernel<<<nb, 256, 0, st>>>(src, n, partials, offsets);
    return hipGetLastError();
}

}  // namespace gs
