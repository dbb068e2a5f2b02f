// shard.hip — multi-GPU exchange kernels.
//
// Scenes are sharded by splat index (rank r holds a contiguous index range).
// Row scheme: every 32-px bin row has an owning rank
// (owner[by]); each rank projects its shard, then sends each visible splat's
// 48-B exchange record to the ranks owning a bin row its rect touches.
// Slab scheme (§6b): each visible splat goes to the rank whose depth-key slab
// holds its key.  Either way received records arrive in source-rank order,
// i.e. in global index order, so the receiving rank's stable sort reproduces
// the single-GPU order of its bins (rows) or of its depth range (slabs).
#include <algorithm>

#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

// Exchange buffers (gsplat.h, gs_exchange_regions): n records as four
// regions, each grouped by destination on the send side: the 48-B records as
// the projection wrote them (cell masks included), then the binning rect
// words lo, hi (bin masks included) and the depth keys, 4 B each.  An
// all-to-all per region leaves the receiver its records and three SoA arrays
// in source-rank order: the rank bins and sorts straight from them.
// kShardItems splats per 256-lane workgroup: 4 rounds of 64 per wave, so a
// rank's shard spreads over many workgroups (750k splats: 733; blocks of
// 4096 left 183 workgroups on 256 CUs, pack 75 us)
constexpr int kShWaves = 4;
constexpr int kShIpt = kShardItems / 256;
constexpr int kShWaveItems = 64 * kShIpt;
static_assert(kShIpt * 256 == kShardItems, "shard block");


// Depth slab of a key: the d with bounds[d] <= key < bounds[d + 1].
__device__ __forceinline__ uint32_t slab_of(uint32_t key, const DestRule& r, int world) {
    uint32_t d = 0;
    while ((int)d + 1 < world && key >= r.bounds[d + 1]) ++d;
    return d;
}

__global__ __launch_bounds__(256) void shard_count_kernel(const uint32_t* __restrict__ rect_lo,
                                                          const uint32_t* __restrict__ rect_hi, uint32_t n,
                                                          int world, const DestRule rule, bool masked,
                                                          uint32_t* __restrict__ dest_mask,
                                                          uint32_t* __restrict__ counts, uint32_t nblocks) {
    __shared__ uint32_t wc[kShWaves][kMaxWorld];
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t base = blockIdx.x * kShardItems + wave * kShWaveItems;
    uint32_t cnt = 0;  // lane d holds this wave's count for destination d
    for (int k = 0; k < kShIpt; ++k) {
        uint32_t i = base + k * 64 + lane;
        uint32_t m = 0;
        if (i < n) {
            const BinRect r = bin_rect(rect_lo[i], rect_hi[i], masked);
            if (!r.empty) m = rule.slabs ? 1u << slab_of(rule.dkey[i], rule, world) : row_mask(r.by0, r.by1, rule.owner);
        }
        if (i < n) dest_mask[i] = m;
        for (int d = 0; d < world; ++d) {
            uint64_t b = __ballot((m >> d) & 1u);
            if (lane == (uint32_t)d) cnt += (uint32_t)__popcll(b);
        }
    }
    if (lane < (uint32_t)kMaxWorld) wc[wave][lane] = cnt;
    __syncthreads();
    if (threadIdx.x < (uint32_t)world) {
        uint32_t d = threadIdx.x;
        counts[(size_t)d * nblocks + blockIdx.x] = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
    }
}

// One 1024-lane workgroup per destination row; each lane scans kRowIpt
// consecutive block counts in registers, one block-wide scan joins them (one
// round for up to 8192 blocks = 8.4M splats; the 256-lane loop it replaces
// took 24 dependent rounds, 16 us, at a 6.25M-splat shard).
constexpr int kRowThreads = 1024, kRowIpt = 8;
__global__ __launch_bounds__(kRowThreads) void rows_scan_kernel(uint32_t* __restrict__ counts, uint32_t nblocks,
                                                                uint32_t* __restrict__ row_total) {
    constexpr int W = kRowThreads / 64;
    constexpr uint32_t CH = kRowThreads * kRowIpt;
    __shared__ uint32_t tmp[W];
    uint32_t* row = counts + (size_t)blockIdx.x * nblocks;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += CH) {
        const uint32_t i0 = b0 + threadIdx.x * kRowIpt;
        uint32_t v[kRowIpt], s = 0;
#pragma unroll
        for (int k = 0; k < kRowIpt; ++k) {
            v[k] = i0 + k < nblocks ? row[i0 + k] : 0u;
            s += v[k];
        }
        const uint32_t inc = wave_scan_dpp<false>(s);
        if (lane == 63) tmp[wave] = inc;
        __syncthreads();
        uint32_t base = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t x = tmp[w];
            base += (uint32_t)w < wave ? x : 0u;
            tot += x;
        }
        __syncthreads();
        uint32_t run = carry + base + inc - s;
#pragma unroll
        for (int k = 0; k < kRowIpt; ++k) {
            if (i0 + k < nblocks) row[i0 + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) row_total[blockIdx.x] = carry;
}

__global__ __launch_bounds__(256) void shard_pack_kernel(const float4* __restrict__ rec,
                                                         const uint32_t* __restrict__ rlo,
                                                         const uint32_t* __restrict__ rhi,
                                                         const uint32_t* __restrict__ dkey,
                                                         const uint32_t* __restrict__ dest_mask, uint32_t n,
                                                         int world, const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ dest_total,
                                                         uint32_t nblocks, float4* __restrict__ send) {
    __shared__ uint32_t wc[kShWaves][kMaxWorld];   // per-wave counts -> per-wave offsets
    __shared__ uint32_t base_d[kMaxWorld];         // this block's start in destination d
    __shared__ float4 stg[kShWaves][3 * 64];       // per wave: one destination's run of a round
    __shared__ uint32_t sside[kShWaves][3][kShWaveItems];  // per wave: its side words for one destination
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t base = blockIdx.x * kShardItems + wave * kShWaveItems;
    // Every round's records are loaded up front, before the block's offsets
    // (one memory round trip per wave, not one per round and destination).
    // The records go through a per-wave LDS stage: a destination's run of a
    // round (consecutive in the send buffer) is written by consecutive lanes,
    // 16 B each, so every store instruction covers whole cache lines (lane-
    // per-record stores at a 48-B stride left each a third of every line:
    // 257 -> 165 us for a 6.25M-splat shard at 8 ranks).
    float4 r0[kShIpt], r1[kShIpt], r2[kShIpt];
    uint32_t mk[kShIpt], lo[kShIpt], hi[kShIpt], dk[kShIpt];
#pragma unroll
    for (int k = 0; k < kShIpt; ++k) {
        const uint32_t i = base + k * 64 + lane;
        mk[k] = i < n ? dest_mask[i] : 0u;
        r0[k] = r1[k] = r2[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        lo[k] = hi[k] = dk[k] = 0u;
        if (mk[k]) {
            const float4* src = rec + kRecFloat4 * (size_t)i;
            r0[k] = src[0];
            r1[k] = src[1];
            r2[k] = src[2];
            lo[k] = rlo[i];
            hi[k] = rhi[i];
            dk[k] = dkey[i];
        }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < kShIpt; ++k) {
        for (int d = 0; d < world; ++d) {
            uint64_t b = __ballot((mk[k] >> d) & 1u);
            if (lane == (uint32_t)d) cnt += (uint32_t)__popcll(b);
        }
    }
    if (lane < (uint32_t)kMaxWorld) wc[wave][lane] = cnt;
    __syncthreads();
    if (threadIdx.x < (uint32_t)world) {
        uint32_t d = threadIdx.x, s = 0;
        for (int w = 0; w < kShWaves; ++w) {
            uint32_t c = wc[w][d];
            wc[w][d] = s;
            s += c;
        }
        uint32_t pre = 0;
        for (uint32_t e = 0; e < d; ++e) pre += dest_total[e];
        base_d[d] = pre + counts[(size_t)d * nblocks + blockIdx.x];
    }
    __syncthreads();
    // the side regions follow all T records (T = every destination's total)
    uint32_t T = 0;
    for (int e = 0; e < world; ++e) T += dest_total[e];
    uint32_t* const side_lo = reinterpret_cast<uint32_t*>(send + (size_t)kXRecFloat4 * T);
    uint32_t* const side_hi = side_lo + T;
    uint32_t* const side_key = side_hi + T;
    // Destination by destination: this wave's records for d (every round's,
    // consecutive in d's region from the wave's offset) leave run by run
    // through the record stage; their side words gather in LDS and leave
    // together, one coalesced run per region.
    float4* const stage = stg[wave];
    for (int d = 0; d < world; ++d) {
        const uint32_t pos0 = base_d[d] + wc[wave][d];
        uint32_t acc = 0;  // this wave's records for d so far
#pragma unroll
        for (int k = 0; k < kShIpt; ++k) {
            const bool bit = (mk[k] >> d) & 1u;
            const uint64_t b = __ballot(bit);
            if (b == 0) continue;
            const uint32_t c = (uint32_t)__popcll(b), j = mbcnt(b);
            if (bit) {
                stage[3u * j] = r0[k];
                stage[3u * j + 1u] = r1[k];
                stage[3u * j + 2u] = r2[k];
                sside[wave][0][acc + j] = lo[k];
                sside[wave][1][acc + j] = hi[k];
                sside[wave][2][acc + j] = dk[k];
            }
            wave_lds_sync();
            float4* dst = send + (size_t)kXRecFloat4 * (pos0 + acc);
            for (uint32_t q = lane; q < 3u * c; q += 64) dst[q] = stage[q];
            wave_lds_sync();  // (the stage is refilled by the next run)
            acc += c;
        }
        for (uint32_t q = lane; q < acc; q += 64) {
            side_lo[pos0 + q] = sside[wave][0][q];
            side_hi[pos0 + q] = sside[wave][1][q];
            side_key[pos0 + q] = sside[wave][2][q];
        }
        wave_lds_sync();  // (the side stage is refilled by the next destination)
    }
}

hipError_t launch_shard_count(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, int world,
                              const DestRule& rule, bool masked,
                              uint32_t* dest_mask, uint32_t* counts, uint32_t nblocks, hipStream_t st) {
    if (world < 1 || world > kMaxWorld) return hipErrorInvalidValue;
    if (nblocks == 0) return hipSuccess;
    if (rule.slabs ? !rule.dkey : !rule.owner) return hipErrorInvalidValue;
    shard_count_kernel<<<nblocks, 256, 0, st>>>(rect_lo, rect_hi, n, world, rule, masked, dest_mask, counts,
                                                nblocks);
    return hipGetLastError();
}

// Depth-slab boundaries are placed on pair counts (the composite's work), so
// the histogram weighs each visible splat by its (splat, bin) pairs.  2048
// bins of 16 depth keys, accumulated in LDS per block (keys concentrate in a
// few hundred bins: global atomics per splat would serialise on them).
__global__ __launch_bounds__(256) void slab_histogram_kernel(const uint32_t* __restrict__ dkey,
                                                             const uint32_t* __restrict__ rect_lo,
                                                             const uint32_t* __restrict__ rect_hi, uint32_t n,
                                                             bool masked, unsigned long long* __restrict__ hist) {
    __shared__ uint32_t h[kSlabBins];
    for (uint32_t k = threadIdx.x; k < (uint32_t)kSlabBins; k += 256) h[k] = 0;
    __syncthreads();
    const uint32_t end = min(n, (blockIdx.x + 1) * (uint32_t)kScanItems);
    for (uint32_t i = blockIdx.x * kScanItems + threadIdx.x; i < end; i += 256) {
        const uint32_t c = rect_tile_count(rect_lo[i], rect_hi[i], RowOwnership{nullptr, 0}, masked);
        if (c) atomicAdd(&h[(dkey[i] & (kSlabKeys - 1)) >> kSlabBinShift], c);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < (uint32_t)kSlabBins; k += 256)
        if (h[k]) atomicAdd(&hist[k], (unsigned long long)h[k]);
}

hipError_t launch_slab_histogram(const uint32_t* dkey, const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n,
                                 bool masked, unsigned long long* hist, hipStream_t st) {
    if (n == 0) return hipSuccess;
    slab_histogram_kernel<<<(n + kScanItems - 1) / kScanItems, 256, 0, st>>>(dkey, rect_lo, rect_hi, n, masked, hist);
    return hipGetLastError();
}

hipError_t launch_rows_scan(uint32_t* counts, uint32_t nblocks, int rows, uint32_t* row_total, hipStream_t st) {
    if (rows <= 0) return hipSuccess;
    rows_scan_kernel<<<rows, kRowThreads, 0, st>>>(counts, nblocks, row_total);
    return hipGetLastError();
}

hipError_t launch_shard_pack(const float4* rec, const uint32_t* rlo, const uint32_t* rhi, const uint32_t* dkey,
                             const uint32_t* dest_mask, uint32_t n, int world, const uint32_t* counts,
                             const uint32_t* dest_total, uint32_t nblocks, float4* send, hipStream_t st) {
    if (nblocks == 0) return hipSuccess;
    shard_pack_kernel<<<nblocks, 256, 0, st>>>(rec, rlo, rhi, dkey, dest_mask, n, world, counts, dest_total, nblocks,
                                               send);
    return hipGetLastError();
}

// dst[i] += src[i] over float4s (the depth-slab RGBA reduce of a transport
// without collectives: contributions summed on one device in rank order).
__global__ __launch_bounds__(256) void accumulate_kernel(float4* __restrict__ dst, const float4* __restrict__ src,
                                                         size_t n4) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
        const float4 a = dst[i], b = src[i];
        dst[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}

hipError_t launch_accumulate(float4* dst, const float4* src, size_t n4, hipStream_t st) {
    if (n4 == 0) return hipSuccess;
    const size_t blocks = std::min<size_t>((n4 + 255) / 256, 8192);
    accumulate_kernel<<<(unsigned)blocks, 256, 0, st>>>(dst, src, n4);
    return hipGetLastError();
}


}  // namespace gs
