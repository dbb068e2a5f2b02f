// radix_sort.hip — stable LSD radix sort of uint32 keys with NV uint32 value
// arrays, onesweep style: one kernel per 8-bit digit pass.
//
// Used twice per frame by the binning stage: splats by
// 15-bit depth key carrying (index, rect_lo, rect_hi) — 2 passes over N — then
// (tile, splat) pairs by tile id — 2 passes over P at 1080p.
//
//   os_hist    one read of the keys -> per-block digit histograms of EVERY
//              pass (LDS atomics), os_reduce sums them per digit (no global
//              atomics), os_offsets scans each pass's 256 bins
//   os_pass    per tile of 512 x IPT items: stable tile-local ranks (wave-private
//              ballot match, no barrier in the ranking loop), publish the tile's
//              digit counts, decoupled look-back for the exclusive prefix over
//              earlier tiles, then coalesced write-out of each array staged
//              through LDS.  (1 + NV) x 4 B read and written per item per pass.
//
// Inter-workgroup protocol (MI355X_MICROARCH.md §Workgroup dispatch, "R2"):
// every look-back word is a self-describing 64-bit granule {flag:2 | count:62}
// written by ONE agent-scope atomic store and read by agent-scope relaxed
// atomic loads (sc1, never L1-cached); the data is the flag, so no fences are
// needed.  Tiles are numbered by an atomic ticket (not blockIdx), so a tile
// only ever waits on tiles already held by running workgroups; spins are
// bounded (an error word is set instead of hanging).  All words are zeroed
// by one hipMemsetAsync per sort.
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kOsThreads = 512;
constexpr int kOsWaves = kOsThreads / 64;
constexpr int kOsHistItems = 16384;
constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint64_t kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 24;

static_assert(kSortBins == 256, "8-bit digits");

template <int NV>
struct SortIO {
    const uint32_t* kin;
    const uint32_t* vin[NV];  // vin[0] may be null: value = item index
    uint32_t* kout;
    uint32_t* vout[NV];
};

constexpr int ipt_for(int nv) { return nv == 1 ? 16 : 8; }
constexpr uint32_t tile_items(int nv) { return (uint32_t)kOsThreads * ipt_for(nv); }

template <typename T, int NW>
__device__ __forceinline__ T block_exclusive_scan(T v, T* tmp, T* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    T inc = wave_inclusive_scan(v);
    if (lane == 63) tmp[wave] = inc;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
        T x = tmp[w];
        base += (uint32_t)w < wave ? x : T(0);
        tot += x;
    }
    *total = tot;
    __syncthreads();
    return base + inc - v;
}

// Lanes of one wave holding the same digit: mask of peers (digit_bits ballots).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int digit_bits) {
    uint64_t peers = __ballot(valid);
    for (int b = 0; b < digit_bits; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// Per-block digit histograms of every pass (plain LDS atomics, wave-private
// copies), written as partials [block][pass*256 + digit]; os_offsets reduces
// them.  No global atomics.
__global__ __launch_bounds__(256) void os_hist_kernel(const uint32_t* __restrict__ keys, uint32_t n, SortPlan plan,
                                                      uint32_t* __restrict__ partial) {
    __shared__ uint32_t h[4][kMaxSortPasses * kSortBins];
    for (int i = threadIdx.x; i < 4 * kMaxSortPasses * kSortBins; i += 256) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t base = blockIdx.x * (uint32_t)kOsHistItems;
#pragma unroll 4
    for (uint32_t k = 0; k < (uint32_t)kOsHistItems / 256; ++k) {
        const uint32_t i = base + k * 256 + threadIdx.x;
        if (i < n) {
            const uint32_t key = keys[i];
            for (int p = 0; p < plan.passes; ++p)
                atomicAdd(&h[wave][p * kSortBins + ((key >> plan.shift[p]) & plan.mask[p])], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < plan.passes * kSortBins; i += 256)
        partial[(size_t)i * gridDim.x + blockIdx.x] = h[0][i] + h[1][i] + h[2][i] + h[3][i];
}

// One workgroup per (pass, digit): sum its row of block partials.
__global__ __launch_bounds__(256) void os_reduce_kernel(const uint32_t* __restrict__ partial, uint32_t nblocks,
                                                        uint32_t* __restrict__ hist) {
    __shared__ uint32_t tmp[4];
    const uint32_t* row = partial + (size_t)blockIdx.x * nblocks;
    uint32_t c = 0;
    for (uint32_t b = threadIdx.x; b < nblocks; b += 256) c += row[b];
    uint32_t t;
    block256_exclusive_scan<uint32_t>(c, tmp, &t);
    if (threadIdx.x == 0) hist[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void os_offsets_kernel(const uint32_t* __restrict__ hist, int passes,
                                                         uint32_t* __restrict__ offs) {
    __shared__ uint32_t tmp[4];
    for (int p = 0; p < passes; ++p) {
        uint32_t t;
        offs[p * kSortBins + threadIdx.x] = block256_exclusive_scan<uint32_t>(hist[p * kSortBins + threadIdx.x], tmp, &t);
    }
}

template <int NV>
__global__ __launch_bounds__(512) void os_pass_kernel(SortIO<NV> io, uint32_t n, int shift, uint32_t mask,
                                                      int digit_bits, const uint32_t* __restrict__ offs,
                                                      uint64_t* status, uint32_t* ctr, uint32_t* err) {
    constexpr int IPT = ipt_for(NV);
    constexpr uint32_t TILE = tile_items(NV);
    constexpr uint32_t WAVE_ITEMS = 64u * IPT;
    __shared__ uint32_t wh[kOsWaves][kSortBins];  // wave-private running counts -> wave offsets
    __shared__ uint32_t blk_start[kSortBins];     // tile-local start of each digit
    __shared__ uint32_t gbase[kSortBins];         // global start of this tile's digit run
    __shared__ uint32_t stage[TILE];
    __shared__ uint8_t sdig[TILE];                // digit of each staged slot
    __shared__ uint32_t tmp[kOsWaves];
    __shared__ uint32_t s_tile;

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < kOsWaves * kSortBins; i += kOsThreads) (&wh[0][0])[i] = 0;
    if (tid == 0) s_tile = atomicAdd(ctr, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint32_t base = tile * TILE + wave * WAVE_ITEMS;

    uint32_t key[IPT], pos[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t idx = base + k * 64 + lane;
        key[k] = idx < n ? io.kin[idx] : 0u;
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t idx = base + k * 64 + lane;
        const bool valid = idx < n;
        const uint32_t d = (key[k] >> shift) & mask;
        const uint64_t peers = match_digit(d, valid, digit_bits);
        const uint32_t below = mbcnt(peers);
        const uint32_t old = wh[wave][d];
        pos[k] = old + below;
        if (valid && below == 0) wh[wave][d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    uint32_t c = 0;
    if (tid < kSortBins) {
#pragma unroll
        for (int w = 0; w < kOsWaves; ++w) {
            const uint32_t x = wh[w][tid];
            wh[w][tid] = c;
            c += x;
        }
        // publish this tile's count of digit tid as early as possible
        __hip_atomic_store(&status[(size_t)tile * kSortBins + tid], (tile == 0 ? kFlagPre : kFlagAgg) | c,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<uint32_t, kOsWaves>(tid < kSortBins ? c : 0u, tmp, &tot);
    if (tid < kSortBins) {
        blk_start[tid] = ex;
        uint64_t excl = 0;
        if (tile > 0) {
            int64_t t = (int64_t)tile - 1;
            uint32_t spins = 0;
            while (true) {
                const uint64_t v = __hip_atomic_load(&status[(size_t)t * kSortBins + tid], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t f = v & ~kValMask;
                if (f == 0) {
                    if (++spins > kSpinLimit) {
                        atomicOr(err, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += v & kValMask;
                if (f == kFlagPre || t == 0) break;
                --t;
            }
            __hip_atomic_store(&status[(size_t)tile * kSortBins + tid], kFlagPre | (excl + c), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        gbase[tid] = offs[tid] + (uint32_t)excl;
    }
    __syncthreads();
    const uint32_t t0 = tile * TILE;
    const uint32_t cnt = n - t0 < TILE ? n - t0 : TILE;
    // keys: stage in tile-local sorted order, remember digits, write out
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t idx = base + k * 64 + lane;
        if (idx < n) {
            const uint32_t d = (key[k] >> shift) & mask;
            pos[k] += blk_start[d] + wh[wave][d];
            stage[pos[k]] = key[k];
            sdig[pos[k]] = (uint8_t)d;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t j = tid + k * kOsThreads;
        if (j < cnt) {
            const uint32_t d = sdig[j];
            io.kout[gbase[d] + (j - blk_start[d])] = stage[j];
        }
    }
    // values: same permutation
#pragma unroll
    for (int a = 0; a < NV; ++a) {
        uint32_t v[IPT];
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t idx = base + k * 64 + lane;
            v[k] = idx < n ? (io.vin[a] ? io.vin[a][idx] : idx) : 0u;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t idx = base + k * 64 + lane;
            if (idx < n) stage[pos[k]] = v[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t j = tid + k * kOsThreads;
            if (j < cnt) {
                const uint32_t d = sdig[j];
                io.vout[a][gbase[d] + (j - blk_start[d])] = stage[j];
            }
        }
    }
}

SortPlan make_sort_plan(int bits) {
    SortPlan p{};
    if (bits <= 0) return p;
    p.passes = (bits + 7) / 8;
    // balanced digit widths (e.g. 13 -> 7+6, 15 -> 8+7)
    int left = bits;
    for (int i = 0; i < p.passes; ++i) {
        const int w = (left + (p.passes - i) - 1) / (p.passes - i);
        p.shift[i] = bits - left;
        p.width[i] = w;
        p.mask[i] = (1u << w) - 1u;
        left -= w;
    }
    return p;
}

namespace {
constexpr size_t kHeadWords = (size_t)kMaxSortPasses * (2 * kSortBins + 2) + 8;  // hist, offs, ctr, err
}

size_t radix_sort_scratch_words(uint32_t n) {
    const size_t tiles = (n + tile_items(3) - 1) / tile_items(3);  // the smaller tile bounds both
    const size_t hblocks = (n + kOsHistItems - 1) / kOsHistItems;
    return kHeadWords + 2 * (size_t)kMaxSortPasses * (tiles ? tiles : 1) * kSortBins +
           (hblocks ? hblocks : 1) * kMaxSortPasses * kSortBins + 64;
}

template <int NV>
static hipError_t radix_sort_impl(const uint32_t* keys_in, const uint32_t* const* vals_in, uint32_t* keys,
                                  uint32_t* const* vals, uint32_t* tmp_keys, uint32_t* const* tmp_vals, uint32_t n,
                                  int bits, uint32_t* scratch, bool* result_in_tmp, hipStream_t st) {
    *result_in_tmp = false;
    const SortPlan plan = make_sort_plan(bits);
    if (n == 0 || plan.passes == 0) return hipSuccess;
    const uint32_t tiles = (n + tile_items(NV) - 1) / tile_items(NV);
    uint32_t* hist = scratch;                            // [passes][256]
    uint32_t* offs = hist + kMaxSortPasses * kSortBins;  // [passes][256]
    uint32_t* ctr = offs + kMaxSortPasses * kSortBins;   // [passes]
    uint32_t* err = ctr + kMaxSortPasses;
    uint64_t* status = reinterpret_cast<uint64_t*>(scratch + kHeadWords);
    const size_t status_words = (size_t)plan.passes * tiles * kSortBins;
    hipError_t e = hipMemsetAsync(scratch, 0, kHeadWords * 4 + status_words * 8, st);
    if (e != hipSuccess) return e;
    const uint32_t hblocks = (n + kOsHistItems - 1) / kOsHistItems;
    uint32_t* partial = reinterpret_cast<uint32_t*>(status + (size_t)kMaxSortPasses * tiles * kSortBins);
    os_hist_kernel<<<hblocks, 256, 0, st>>>(keys_in, n, plan, partial);
    os_reduce_kernel<<<plan.passes * kSortBins, 256, 0, st>>>(partial, hblocks, hist);
    os_offsets_kernel<<<1, 256, 0, st>>>(hist, plan.passes, offs);
    // Pass 0 reads the caller's arrays; later passes ping-pong between
    // (keys, vals) and (tmp_keys, tmp_vals), arranged so the last pass lands
    // in (keys, vals) unless that would make pass 0 write what it reads.
    bool alias = keys_in == keys;
    for (int a = 0; a < NV; ++a) alias = alias || (vals_in[a] && vals_in[a] == vals[a]);
    const bool start_final = (plan.passes % 2) == 1 && !alias;
    *result_in_tmp = (plan.passes % 2) == 1 && alias;
    SortIO<NV> io;
    io.kin = keys_in;
    for (int a = 0; a < NV; ++a) io.vin[a] = vals_in[a];
    bool to_final = start_final;
    for (int p = 0; p < plan.passes; ++p) {
        io.kout = to_final ? keys : tmp_keys;
        for (int a = 0; a < NV; ++a) io.vout[a] = to_final ? vals[a] : tmp_vals[a];
        os_pass_kernel<NV><<<tiles, kOsThreads, 0, st>>>(io, n, plan.shift[p], plan.mask[p], plan.width[p],
                                                         offs + p * kSortBins, status + (size_t)p * tiles * kSortBins,
                                                         ctr + p, err);
        io.kin = io.kout;
        for (int a = 0; a < NV; ++a) io.vin[a] = io.vout[a];
        to_final = !to_final;
    }
    return hipGetLastError();
}

hipError_t launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys, uint32_t* vals,
                             uint32_t* tmp_keys, uint32_t* tmp_vals, uint32_t n, int bits, uint32_t* scratch,
                             bool* result_in_tmp, hipStream_t st) {
    const uint32_t* vi[1] = {vals_in};
    uint32_t* vo[1] = {vals};
    uint32_t* vt[1] = {tmp_vals};
    return radix_sort_impl<1>(keys_in, vi, keys, vo, tmp_keys, vt, n, bits, scratch, result_in_tmp, st);
}

hipError_t launch_radix_sort3(const uint32_t* keys_in, const uint32_t* const* vals_in, uint32_t* keys,
                              uint32_t* const* vals, uint32_t* tmp_keys, uint32_t* const* tmp_vals, uint32_t n,
                              int bits, uint32_t* scratch, bool* result_in_tmp, hipStream_t st) {
    return radix_sort_impl<3>(keys_in, vals_in, keys, vals, tmp_keys, tmp_vals, n, bits, scratch, result_in_tmp, st);
}

}  // namespace gs
