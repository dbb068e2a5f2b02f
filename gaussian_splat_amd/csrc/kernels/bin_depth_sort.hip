// bin_depth_sort.hip — per-bin stable depth sort of the (splat, bin) lists
// (bin-first binning order).
//
// The pairs are emitted in splat index (arrival) order with each splat's
// 15-bit depth key carried above the bin id, and sorted stably by bin id
// alone (radix_sort.hip, ranges from its last pass).  Each bin's list is then
// in index order, and a stable sort of the list by depth key leaves it in
// (depth key, index) order: exactly the per-pixel insertion sort of
// gaussian_splat_tile.metal:239-249 with arrival = index, and the same lists
// the depth-first order (global depth sort of all splats, then binning)
// produces, without its two passes over every splat.
//
// One workgroup per bin.  A list of up to kSegLdsMax pairs is sorted inside
// the workgroup: every lane holds up to IPT items ((dkey - kmin) << 17 |
// list position) in registers; items are unique, so "stable by depth key" is
// plain ascending item order.  Only the bits of the list's own key range
// [kmin, kmax] are sorted (a bin's keys span ~12 of the 15 bits: 2 LSD
// passes of 6; a range of <= 256 keys takes 1 pass, a single key none),
// ranked with wave-ballot digit matching and wave-private LDS counters (the
// ranking of rts_pass_kernel) and exchanged through one LDS array.  The vals
// are finally gathered by list position and written back in place.
// (A counting order — LDS histogram over the key range, then a rank inside
// each key's bucket — was measured slower: 110 vs 96 us at the bench config,
// its bucket-rank loop costs the largest bucket of the wave.)
// Longer lists (a hot bin of a dense scene) take a chunked LSD over global
// memory, one workgroup per bin, through the bin sort's spare buffers.
#include <hip/hip_ext.h>

#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kSegPosBits = 17;  // list position field of an item (lists <= 2^17 in LDS)
static_assert(kDepthBits + kSegPosBits == 32, "item = dkey << 17 | position");

template <int NT>
struct SegRankLds {
    uint32_t wh[NT / 64][256];  // wave-private digit counts -> wave offsets
    uint32_t start[256];        // tile-local start of each digit
    uint32_t tmp[2 * (NT / 64)];
};

template <int NT>
__device__ __forceinline__ uint32_t seg_block_exclusive_scan(uint32_t v, uint32_t* tmp, uint32_t* total) {
    constexpr int W = NT / 64;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_scan_dpp<false>(v);
    if (lane == 63) tmp[wave] = inc;
    block_lds_sync();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t x = tmp[w];
        base += (uint32_t)w < wave ? x : 0u;
        tot += x;
    }
    *total = tot;
    block_lds_sync();
    return base + inc - v;
}

template <int WIDTH>
__device__ __forceinline__ uint64_t seg_match_digit(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < WIDTH; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// Stable rank of the items of one tile by digit (it[k] >> shift) & (2^WIDTH
// - 1), WIDTH <= 8.  Items are laid out wave-blocked: slot k of lane l of
// wave w is tile position w * kmax * 64 + k * 64 + l (< m valid).  On return
// pos[k] is the item's position in the tile's stable digit order, L.start[]
// the tile-local start of every digit and, for thread t < 2^WIDTH, *count the
// tile's count of digit t.
template <int NT, int IPT, int WIDTH>
__device__ __forceinline__ void seg_rank(const uint32_t (&it)[IPT], uint32_t (&pos)[IPT], int kmax, uint32_t m,
                                         int shift, SegRankLds<NT>& L, uint32_t* count) {
    static_assert(NT >= 256 && WIDTH <= 8, "one lane per digit");
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t base = wave * (uint32_t)kmax * 64u;
    constexpr uint32_t nd = 1u << WIDTH, mask = nd - 1u;
    for (uint32_t i = lane; i < nd; i += 64u) L.wh[wave][i] = 0u;
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        if (k < kmax) {
            const bool valid = base + (uint32_t)k * 64u + lane < m;
            const uint32_t d = (it[k] >> shift) & mask;
            const uint64_t peers = seg_match_digit<WIDTH>(d, valid);
            const uint32_t below = mbcnt(peers);
            const uint32_t old = L.wh[wave][d];
            pos[k] = old + below;
            if (valid && below == 0) L.wh[wave][d] = old + (uint32_t)__popcll(peers);
        }
    }
    block_lds_sync();
    uint32_t c = 0;
    if (tid < nd) {
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) {
            const uint32_t x = L.wh[w][tid];
            L.wh[w][tid] = c;
            c += x;
        }
    }
    uint32_t tot;
    const uint32_t ex = seg_block_exclusive_scan<NT>(tid < nd ? c : 0u, L.tmp, &tot);
    if (tid < nd) L.start[tid] = ex;
    *count = c;
    block_lds_sync();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        if (k < kmax && base + (uint32_t)k * 64u + lane < m) {
            const uint32_t d = (it[k] >> shift) & mask;
            pos[k] += L.start[d] + L.wh[wave][d];
        }
    }
}

// Workgroup-uniform (min lo, max hi); tmp >= 2 * NT / 64 words of LDS.
template <int NT>
__device__ __forceinline__ uint2 seg_block_minmax(uint32_t lo, uint32_t hi, uint32_t* tmp) {
    constexpr int W = NT / 64;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t a = wave_scan_dpp<true>(~lo), b = wave_scan_dpp<true>(hi);  // lane 63: the wave's
    if (lane == 63) {
        tmp[wave] = a;
        tmp[W + wave] = b;
    }
    block_lds_sync();
    uint32_t ra = 0, rb = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        ra = max(ra, tmp[w]);
        rb = max(rb, tmp[W + w]);
    }
    block_lds_sync();
    return make_uint2(~ra, rb);
}

// One LSD pass of the in-LDS sort over digit (it >> shift) & (2^WIDTH - 1).
template <int NT, int IPT, int WIDTH>
__device__ __forceinline__ void seg_pass(uint32_t (&it)[IPT], uint32_t (&pos)[IPT], int kmax, uint32_t m,
                                         int shift, SegRankLds<NT>& L, uint32_t* stage) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t base = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (uint32_t)kmax * 64u;
    uint32_t cnt;
    seg_rank<NT, IPT, WIDTH>(it, pos, kmax, m, shift, L, &cnt);
#pragma unroll
    for (int k = 0; k < IPT; ++k)
        if (k < kmax && base + (uint32_t)k * 64u + lane < m) stage[pos[k]] = it[k];
    block_lds_sync();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t p = base + (uint32_t)k * 64u + lane;
        if (k < kmax && p < m) it[k] = stage[p];
    }
    // the next pass rewrites stage / L only after seg_rank's barriers
}

// A list longer than the workgroup holds: LSD over global memory, chunks of
// NT * IPT pairs in list order; (keys, vals) -> (tmp_keys, tmp_vals) ->
// (keys, vals) at the list's own offsets [s, s + m).  run: 256 words of LDS.
template <int NT, int IPT>
__device__ __forceinline__ void sort_list_global(uint32_t s, uint32_t m, uint32_t* keys, uint32_t* vals, uint32_t* tmp_keys,
                                 uint32_t* tmp_vals, int bin_bits, SegRankLds<NT>& L, uint32_t* run) {
    constexpr uint32_t CH = (uint32_t)NT * IPT;
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int pass = 0; pass < 2; ++pass) {
        const uint32_t* sk = (pass == 0 ? keys : tmp_keys) + s;
        const uint32_t* sv = (pass == 0 ? vals : tmp_vals) + s;
        uint32_t* dk = (pass == 0 ? tmp_keys : keys) + s;
        uint32_t* dv = (pass == 0 ? tmp_vals : vals) + s;
        const int shift = bin_bits + 8 * pass, width = pass == 0 ? 8 : kDepthBits - 8;
        const uint32_t mask = (1u << width) - 1u;
        // digit histogram of the whole list -> running digit starts
        for (uint32_t i = lane; i < 256u; i += 64u) L.wh[wave][i] = 0u;
        wave_lds_sync();
        for (uint32_t p = tid; p < m; p += NT) atomicAdd(&L.wh[wave][(sk[p] >> shift) & mask], 1u);
        block_lds_sync();
        uint32_t c = 0;
        if (tid < 256u)
            for (int w = 0; w < NT / 64; ++w) c += L.wh[w][tid];
        uint32_t tot;
        const uint32_t ex = seg_block_exclusive_scan<NT>(tid < 256u ? c : 0u, L.tmp, &tot);
        if (tid < 256u) run[tid] = ex;
        block_lds_sync();
        for (uint32_t c0 = 0; c0 < m; c0 += CH) {
            const uint32_t cm = m - c0 < CH ? m - c0 : CH;
            const int kmax = (int)((cm + NT - 1) / NT);
            const uint32_t base = wave * (uint32_t)kmax * 64u;
            uint32_t kk[IPT], vv[IPT], pos[IPT];
#pragma unroll
            for (int k = 0; k < IPT; ++k) {
                const uint32_t p = base + (uint32_t)k * 64u + lane;
                const bool ok = k < kmax && p < cm;
                kk[k] = ok ? sk[c0 + p] : 0u;
                vv[k] = ok ? sv[c0 + p] : 0u;
            }
            uint32_t cnt;
            if (pass == 0) seg_rank<NT, IPT, 8>(kk, pos, kmax, cm, shift, L, &cnt);
            else seg_rank<NT, IPT, kDepthBits - 8>(kk, pos, kmax, cm, shift, L, &cnt);
#pragma unroll
            for (int k = 0; k < IPT; ++k) {
                const uint32_t p = base + (uint32_t)k * 64u + lane;
                if (k < kmax && p < cm) {
                    const uint32_t d = (kk[k] >> shift) & mask;
                    const uint32_t g = run[d] + (pos[k] - L.start[d]);
                    dk[g] = kk[k];
                    dv[g] = vv[k];
                }
            }
            block_lds_sync();  // every lane has read run[] / start[]
            if (tid < 256u) run[tid] += cnt;
            block_lds_sync();
        }
        __syncthreads();  // this pass's global writes are visible to the next pass's reads
    }
}

#ifndef GS_SEG_MINW  // min waves per SIMD (launch bounds: caps the VGPRs)
#define GS_SEG_MINW 6
#endif
#ifndef GS_SEG_SMALL_MINW
#define GS_SEG_SMALL_MINW 6
#endif

// CLS (GS_SEG_CLASSES): 0 every list; 1 the lists of at most kSegSmallMax
// pairs only; 2 the longer ones only (two launches over every bin, so that
// short lists run in narrow workgroups, more bins at a time, and long ones
// keep the wide workgroup's LDS capacity).
template <int NT, int IPT, int MINW = 1, int CLS = 0>
__global__ __launch_bounds__(NT, MINW) void bin_depth_sort_kernel(const uint2* __restrict__ ranges,
                                                                  uint32_t* __restrict__ keys,
                                                                  uint32_t* __restrict__ vals,
                                                                  uint32_t* __restrict__ tmp_keys,
                                                                  uint32_t* __restrict__ tmp_vals, int bin_bits,
                                                                  uint32_t* __restrict__ sample,
                                                                  const unsigned long long* __restrict__ guard) {
    static_assert((uint32_t)NT * IPT <= (1u << kSegPosBits), "position field");
    __shared__ SegRankLds<NT> L;
    __shared__ uint32_t stage[NT * IPT];
    if (guard && *guard == 0ull) return;  // (whole grid: the fallback lists of a frame with no open tile)
    const uint2 rg = decode_range(ranges[blockIdx.x]);
    const uint32_t m = rg.y > rg.x ? rg.y - rg.x : 0u;
    if (sample && threadIdx.x == 0) {  // for the host's choice of binning order
        if (blockIdx.x == 0) atomicOr(&sample[1], kSegSampleValid);
        if (m > (uint32_t)NT * IPT) atomicAdd(&sample[0], m);
    }
    if (m < 2u) return;  // nothing to order
    if constexpr (CLS == 1)
        if (m > kSegSmallMax) return;
    if constexpr (CLS == 2)
        if (m <= kSegSmallMax) return;
    const uint32_t s = rg.x;
    if (m > (uint32_t)NT * IPT) {  // a hot bin: chunked LSD over global memory
        sort_list_global<NT, 8>(s, m, keys, vals, tmp_keys, tmp_vals, bin_bits, L, stage);
        return;
    }
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kmax = (int)((m + NT - 1) / NT);  // slots per lane (<= IPT)
    const uint32_t base = wave * (uint32_t)kmax * 64u;
    uint32_t it[IPT], pos[IPT];
    // every key loaded before the first use (positions clamped into the list,
    // branch-free): one memory round trip, not one per slot
#pragma unroll
    for (int k = 0; k < IPT; ++k) it[k] = keys[s + min(base + (uint32_t)k * 64u + lane, m - 1u)];
    uint32_t lo = 0xFFFFFFFFu, hi = 0u;
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t p = base + (uint32_t)k * 64u + lane;
        const bool ok = k < kmax && p < m;
        const uint32_t dk = it[k] >> bin_bits;
        it[k] = ok ? (dk << kSegPosBits) | p : 0xFFFFFFFFu;
        lo = ok ? min(lo, dk) : lo;
        hi = ok ? max(hi, dk) : hi;
    }
    // the list's key range: sort only its bits (none if every key is equal,
    // and the list is already in order)
    const uint2 ext = seg_block_minmax<NT>(lo, hi, L.tmp);
    const uint32_t kmin = ext.x, span = ext.y - ext.x;
    if (span == 0) return;
#pragma unroll
    for (int k = 0; k < IPT; ++k)
        if (k < kmax && base + (uint32_t)k * 64u + lane < m) it[k] -= kmin << kSegPosBits;
    if (span < (1u << 8)) {
        seg_pass<NT, IPT, 8>(it, pos, kmax, m, kSegPosBits, L, stage);
    } else if (span < (1u << 12)) {
        seg_pass<NT, IPT, 6>(it, pos, kmax, m, kSegPosBits, L, stage);
        seg_pass<NT, IPT, 6>(it, pos, kmax, m, kSegPosBits + 6, L, stage);
    } else {
        seg_pass<NT, IPT, 8>(it, pos, kmax, m, kSegPosBits, L, stage);
        seg_pass<NT, IPT, kDepthBits - 8>(it, pos, kmax, m, kSegPosBits + 8, L, stage);
    }
    // gather by list position, then write back in place once every lane's
    // gathers have landed
    uint32_t v[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t p = base + (uint32_t)k * 64u + lane;
#ifdef GS_SEG_ABL_NOGATHER  // ablation (timing only): coalesced read of the own slot (ids stay valid)
        v[k] = (k < kmax && p < m) ? vals[s + p] : 0u;
#else
        v[k] = vals[s + ((k < kmax && p < m) ? (it[k] & ((1u << kSegPosBits) - 1u)) : 0u)];
#endif
    }
#pragma unroll
    for (int k = 0; k < IPT; ++k) asm volatile("" ::"v"(v[k]));  // loads complete before the barrier
    __syncthreads();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t p = base + (uint32_t)k * 64u + lane;
        if (k < kmax && p < m) vals[s + p] = v[k];
    }
}

hipError_t launch_bin_depth_sort(const uint2* ranges, uint32_t nbins, uint32_t* keys, uint32_t* vals,
                                 uint32_t* tmp_keys, uint32_t* tmp_vals, int bin_bits, uint32_t* sample,
                                 hipStream_t st, hipEvent_t done, const unsigned long long* guard, bool short_lists) {
    if (nbins == 0) return done ? hipEventRecord(done, st) : hipSuccess;
    if (bin_bits < 0 || bin_bits + kDepthBits > 32) return hipErrorInvalidValue;
    // one workgroup per bin
    static_assert(GS_SEG_NT * GS_SEG_IPT == kSegLdsMax, "gs_kernels.h");
    // Frames of many bins (4K: 8160; their lists are short) sort in two size
    // classes: the long lists first (that launch samples every list), then the
    // short ones in 256-lane workgroups, twice the bins at a time; the second
    // launch's packet carries `done`.  Frames of few bins (1080p: 2040, lists
    // of ~2-3k pairs, more of them past the short class) keep one launch: the
    // long class alone then leaves the part idle (profiles/r06/ab_seg_classes.txt).
    static_assert(GS_SEG_SMALL_NT * GS_SEG_SMALL_IPT == kSegSmallMax && kSegSmallMax < kSegLdsMax, "gs_kernels.h");
    if (GS_SEG_CLASSES && nbins >= (uint32_t)GS_SEG_CLASS_MIN_BINS) {
        hipExtLaunchKernelGGL((bin_depth_sort_kernel<GS_SEG_NT, GS_SEG_IPT, GS_SEG_MINW, 2>), dim3(nbins),
                              dim3(GS_SEG_NT), 0, st, nullptr, nullptr, 0, ranges, keys, vals, tmp_keys, tmp_vals,
                              bin_bits, sample, guard);
        hipExtLaunchKernelGGL((bin_depth_sort_kernel<GS_SEG_SMALL_NT, GS_SEG_SMALL_IPT, GS_SEG_SMALL_MINW, 1>),
                              dim3(nbins), dim3(GS_SEG_SMALL_NT), 0, st, nullptr, done, 0, ranges, keys, vals, tmp_keys,
                              tmp_vals, bin_bits, nullptr, guard);
        return hipGetLastError();
    }
    if (GS_SEG_SHORT && short_lists) {  // (a still camera's front lists: every list in 256-lane workgroups)
        hipExtLaunchKernelGGL((bin_depth_sort_kernel<GS_SEG_SMALL_NT, GS_SEG_SMALL_IPT, GS_SEG_SMALL_MINW>), dim3(nbins),
                              dim3(GS_SEG_SMALL_NT), 0, st, nullptr, done, 0, ranges, keys, vals, tmp_keys, tmp_vals,
                              bin_bits, sample, guard);
        return hipGetLastError();
    }
    hipExtLaunchKernelGGL((bin_depth_sort_kernel<GS_SEG_NT, GS_SEG_IPT, GS_SEG_MINW>), dim3(nbins), dim3(GS_SEG_NT), 0,
                          st, nullptr, done, 0, ranges, keys, vals, tmp_keys, tmp_vals, bin_bits, sample, guard);
    return hipGetLastError();
}

}  // namespace gs
