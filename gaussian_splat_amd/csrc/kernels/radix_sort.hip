// radix_sort.hip — stable LSD radix sort of (uint32 key, uint32 value) pairs.
//
// The per-view depth sort + tile binning of the north star:
// keys are tile_id << 15 | dkey, and only the significant bits are sorted
// (tile bits + 15), 8 bits per pass.  Each pass is three launches:
//   hist    : per-block digit histogram            (reads 4 B/pair)
//   rowscan : per-digit exclusive scan over blocks  (tiny)
//   scatter : stable block-local rank + coalesced write-out through LDS
//             (reads 8 B/pair, writes 8 B/pair)
// Stability inside a block: wave w owns the contiguous sub-range
// [w*1024, (w+1)*1024) of the block's 4096 items and ranks it in order with a
// ballot match over the 8 digit bits and a wave-private LDS counter — no
// workgroup barrier inside the ranking loop (64-lane waves, v_mbcnt).
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kRsThreads = 256;
constexpr int kRsWaves = kRsThreads / 64;
constexpr int kRsIpt = kSortTile / kRsThreads;  // 16 items per lane
constexpr int kRsWaveItems = 64 * kRsIpt;       // 1024 contiguous items per wave
constexpr int kRsBits = 8;

static_assert(kSortBins == 1 << kRsBits, "bins");

__global__ __launch_bounds__(256) void rs_hist_kernel(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                      uint32_t mask, uint32_t* __restrict__ hist,
                                                      uint32_t nblocks) {
    __shared__ uint32_t h[kRsWaves][kSortBins];
    for (int i = threadIdx.x; i < kRsWaves * kSortBins; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t base = blockIdx.x * kSortTile + wave * kRsWaveItems;
#pragma unroll 4
    for (int k = 0; k < kRsIpt; ++k) {
        uint32_t idx = base + k * 64 + lane;
        if (idx < n) atomicAdd(&h[wave][(keys[idx] >> shift) & mask], 1u);
    }
    __syncthreads();
    uint32_t d = threadIdx.x;
    hist[(size_t)d * nblocks + blockIdx.x] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// One workgroup per digit: exclusive scan of its row (one entry per block).
__global__ __launch_bounds__(256) void rs_rowscan_kernel(uint32_t* __restrict__ hist, uint32_t nblocks,
                                                         uint32_t* __restrict__ digit_total) {
    __shared__ uint32_t tmp[4];
    uint32_t* row = hist + (size_t)blockIdx.x * nblocks;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += kRsThreads) {
        uint32_t i = b0 + threadIdx.x;
        uint32_t v = i < nblocks ? row[i] : 0u;
        uint32_t t;
        uint32_t ex = block256_exclusive_scan<uint32_t>(v, tmp, &t);
        if (i < nblocks) row[i] = carry + ex;
        carry += t;
    }
    if (threadIdx.x == 0) digit_total[blockIdx.x] = carry;
}

__global__ __launch_bounds__(256) void rs_scatter_kernel(const uint32_t* __restrict__ kin,
                                                         const uint32_t* __restrict__ vin,
                                                         uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         uint32_t n, int shift, uint32_t mask,
                                                         const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ digit_total,
                                                         uint32_t nblocks) {
    __shared__ uint32_t wh[kRsWaves][kSortBins];  // wave-private running counts
    __shared__ uint32_t blk_start[kSortBins];     // block-local digit start
    __shared__ uint32_t gbase[kSortBins];         // global start of this block's digit run
    __shared__ uint32_t sk[kSortTile];
    __shared__ uint32_t sv[kSortTile];
    __shared__ uint32_t tmp[4];

    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (int i = tid; i < kRsWaves * kSortBins; i += kRsThreads) (&wh[0][0])[i] = 0;
    // Global exclusive digit prefix (every block recomputes the 256-entry scan).
    uint32_t tot;
    uint32_t dpre = block256_exclusive_scan<uint32_t>(digit_total[tid], tmp, &tot);
    gbase[tid] = dpre + hist[(size_t)tid * nblocks + blockIdx.x];
    __syncthreads();

    const uint32_t base = blockIdx.x * kSortTile + wave * kRsWaveItems;
    uint32_t key[kRsIpt], val[kRsIpt], rank[kRsIpt];
#pragma unroll
    for (int k = 0; k < kRsIpt; ++k) {
        uint32_t idx = base + k * 64 + lane;
        bool valid = idx < n;
        key[k] = valid ? kin[idx] : 0u;
        val[k] = valid ? vin[idx] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kRsIpt; ++k) {
        uint32_t idx = base + k * 64 + lane;
        bool valid = idx < n;
        uint32_t d = (key[k] >> shift) & mask;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kRsBits; ++b) {
            bool bit = (d >> b) & 1u;
            uint64_t bal = __ballot(bit);
            peers &= bit ? bal : ~bal;
        }
        uint32_t below = mbcnt(peers);
        uint32_t old = wh[wave][d];
        rank[k] = old + below;
        if (valid && below == 0) wh[wave][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {
        // digit tid: exclusive offsets across waves (wave order = item order)
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < kRsWaves; ++w) {
            uint32_t c = wh[w][tid];
            wh[w][tid] = s;
            s += c;
        }
        uint32_t t2;
        blk_start[tid] = block256_exclusive_scan<uint32_t>(s, tmp, &t2);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRsIpt; ++k) {
        uint32_t idx = base + k * 64 + lane;
        if (idx < n) {
            uint32_t d = (key[k] >> shift) & mask;
            uint32_t pos = blk_start[d] + wh[wave][d] + rank[k];
            sk[pos] = key[k];
            sv[pos] = val[k];
        }
    }
    __syncthreads();
    const uint32_t blk0 = blockIdx.x * kSortTile;
    const uint32_t cnt = n - blk0 < (uint32_t)kSortTile ? n - blk0 : (uint32_t)kSortTile;
    for (uint32_t j = tid; j < cnt; j += kRsThreads) {
        uint32_t k = sk[j];
        uint32_t d = (k >> shift) & mask;
        uint32_t g = gbase[d] + (j - blk_start[d]);
        kout[g] = k;
        vout[g] = sv[j];
    }
}

size_t radix_sort_scratch_words(uint32_t n) {
    size_t nb = (n + kSortTile - 1) / kSortTile;
    return (size_t)kSortBins * (nb > 0 ? nb : 1) + kSortBins;
}

hipError_t launch_radix_sort(uint32_t* keys, uint32_t* vals, uint32_t* tmp_keys, uint32_t* tmp_vals, uint32_t n,
                             int bits, uint32_t* scratch, bool* result_in_tmp, hipStream_t st) {
    *result_in_tmp = false;
    if (n <= 1 || bits <= 0) return hipSuccess;
    uint32_t nb = (n + kSortTile - 1) / kSortTile;
    uint32_t* hist = scratch;
    uint32_t* dtot = scratch + (size_t)kSortBins * nb;
    uint32_t *ki = keys, *vi = vals, *ko = tmp_keys, *vo = tmp_vals;
    for (int shift = 0; shift < bits; shift += kRsBits) {
        int w = bits - shift < kRsBits ? bits - shift : kRsBits;
        uint32_t mask = (1u << w) - 1u;
        rs_hist_kernel<<<nb, kRsThreads, 0, st>>>(ki, n, shift, mask, hist, nb);
        rs_rowscan_kernel<<<kSortBins, kRsThreads, 0, st>>>(hist, nb, dtot);
        rs_scatter_kernel<<<nb, kRsThreads, 0, st>>>(ki, vi, ko, vo, n, shift, mask, hist, dtot, nb);
        uint32_t* t;
        t = ki; ki = ko; ko = t;
        t = vi; vi = vo; vo = t;
        *result_in_tmp = !*result_in_tmp;
    }
    return hipGetLastError();
}

}  // namespace gs
