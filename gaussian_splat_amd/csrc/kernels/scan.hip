// scan.hip — binning: exclusive prefix sum of per-splat
// bin counts (reduce-then-scan; the counts come from the packed rects on the
// fly) and the duplicate step that emits the (bin, splat) pairs.
//
// Depth-first order: splats sorted by their 15-bit depth key (stable, so
// equal half depths keep index = arrival order,
// shaders/gaussian_splat_tile.metal:244) are visited in that order and each
// emits one (bin, splat index) pair per 32x32 bin of its conservative pixel
// rect; a stable sort of the pairs by bin id alone (radix_sort.hip, 2 digit
// passes over P at 1080p, ranges from the last pass) yields each bin's list
// in S1 order.  Bin-first order: the same pairs in splat index
// order with the depth key carried above the bin id (key = dkey << bin_bits
// | bin); after the bin sort each list is put in depth order by a stable
// per-bin sort (bin_depth_sort.hip).
#include <hip/hip_ext.h>

#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kScanIpt = kScanItems / 256;  // 16 consecutive items per lane
#ifndef GS_BUF_LOADS  // A/B knob: 1 = the count and duplicate kernels read through raw buffer resources (BufU32)
#define GS_BUF_LOADS 0
#endif

struct CountSrc {
    const uint32_t* lo;
    const uint32_t* hi;
    RowOwnership own;
    bool masked;  // rect words carry the bin-exclusion mask
};

// Per block: pair count -> partials[b], contributing splats -> partials[nb + b].
__global__ __launch_bounds__(256) void scan_reduce_kernel(CountSrc src, uint32_t n,
                                                          uint64_t* __restrict__ partials,
                                                          uint2* __restrict__ fill, uint32_t nfill,
                                                          uint32_t* __restrict__ zero, uint32_t nzero) {
    __shared__ uint2 tmp[4];
    const uint32_t base = blockIdx.x * kScanItems;
    // every rect loaded before the first use (clamped, branch-free): one
    // memory round trip instead of one per item (a conditional load is waited
    // for inside its branch)
    uint32_t lo[kScanIpt], hi[kScanIpt];
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const uint32_t i = min(base + k * 256 + threadIdx.x, n - 1u);
        lo[k] = src.lo[i];
        hi[k] = src.hi[i];
    }
    // 32-bit sums: a block's pairs are at most 4096 splats x 16384 bins (4096^2 frames)
    uint32_t s = 0, vis = 0;
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const bool in = base + k * 256 + threadIdx.x < n;
        const uint32_t c = in ? rect_tile_count(lo[k], hi[k], src.own, src.masked) : 0u;
        s += c;
        vis += c > 0;
    }
    // the frame's bin ranges start empty and the first sort pass's digit
    // counts at zero (saves two fill dispatches; stored after the loads, which
    // a store would otherwise delay: vmcnt counts both)
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nfill; i += gridDim.x * 256u)
        fill[i] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < nzero; i += gridDim.x * 256u) zero[i] = 0u;
    // block sums: wave reductions (DPP), then one barrier
    s = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(s), 63);
    vis = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(vis), 63);
    const uint32_t wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63u) == 0) tmp[wave] = make_uint2(s, vis);
    __syncthreads();
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = (uint64_t)tmp[0].x + tmp[1].x + tmp[2].x + tmp[3].x;
        partials[gridDim.x + blockIdx.x] = (uint64_t)tmp[0].y + tmp[1].y + tmp[2].y + tmp[3].y;
    }
}

// One workgroup scans all partials (<= a few thousand) exclusively in place.
// seg_sample (may be null): the per-bin depth sort's sample since the last
// scan (bin_depth_sort.hip) is moved into total[2..3] and reset, so it comes
// back to the host with the pair count.
// One 1024-lane workgroup: each lane scans kPartIpt consecutive block sums in
// registers, one block-wide scan joins them (a single pass for nb <= 4096;
// larger grids loop).
constexpr int kPartThreads = 1024;
constexpr uint32_t kPartLookback = 4;  // (scan_partials_kernel prow)
constexpr int kPartIpt = 4;

template <typename T>
__device__ __forceinline__ T block1024_exclusive_scan(T v, T* tmp, T* total) {
    constexpr int W = kPartThreads / 64;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const T inc = wave_inclusive_scan(v);
    if (lane == 63) tmp[wave] = inc;
    __syncthreads();
    T base = T(0), tot = T(0);
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const T x = tmp[w];
        base += (uint32_t)w < wave ? x : T(0);
        tot += x;
    }
    *total = tot;
    __syncthreads();
    return base + inc - v;
}

// src (may be null): the block sums come from there instead (the fused
// preprocess's, PreFuse: 3 x nb words) and are cleared after reading; the
// third row's sum (the duplicate's wave-max work) goes to total[4].
// prow (src only): the row whose sums are scanned into the offsets, 0 (every
// pair) or 3 (the front pairs a depth-cut frame emits, launch_front_count);
// kPartLookback: none (the front duplicate finds its blocks' offsets by
// look-back): partials[0..nb] are cleared for it and total[0] is 0;
// row 0's sum is total[8] either way (the frame's every pair: the pair buffers
// must hold them all, so npairs is 0 when they do not).  guard (may be null):
// nothing is done while *guard == 0 (the fallback lists' regeneration).
// kept (may be null): also receives the pair count.
__global__ __launch_bounds__(kPartThreads) void scan_partials_kernel(uint64_t* __restrict__ partials, uint32_t nb,
                                                                     uint64_t* __restrict__ total,
                                                                     uint32_t* __restrict__ seg_sample,
                                                                     uint32_t* __restrict__ npairs, uint64_t cap,
                                                                     unsigned long long* __restrict__ src,
                                                                     unsigned long long seq, uint32_t prow,
                                                                     const unsigned long long* __restrict__ guard,
                                                                     uint32_t* __restrict__ kept) {
    if (guard && *guard == 0ull) return;
    if (seg_sample && threadIdx.x == 0) {
        total[2] = seg_sample[0];
        total[3] = seg_sample[1];
        seg_sample[0] = 0u;
        seg_sample[1] = 0u;
    }
    __shared__ uint64_t tmp[kPartThreads / 64];
    constexpr uint32_t CH = kPartThreads * kPartIpt;
    uint64_t carry = 0, vis = 0, wmax = 0, all = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += CH) {
        const uint32_t i0 = b0 + threadIdx.x * kPartIpt;
        uint64_t v[kPartIpt], s = 0;
#pragma unroll
        for (int k = 0; k < kPartIpt; ++k) {
            if (src) {
                v[k] = i0 + k < nb && prow != kPartLookback ? (uint64_t)src[(size_t)prow * nb + i0 + k] : 0u;
                all += i0 + k < nb ? (uint64_t)src[i0 + k] : 0u;
                vis += i0 + k < nb ? (uint64_t)src[nb + i0 + k] : 0u;
                wmax += i0 + k < nb ? (uint64_t)src[2u * nb + i0 + k] : 0u;
                // (rows 0-2 are atomic sums: cleared for the next frame; row 3 is stored whole by every front frame)
                if (i0 + k < nb) src[i0 + k] = src[nb + i0 + k] = src[2u * nb + i0 + k] = 0ull;  // (read by this lane only)
            } else {
                v[k] = i0 + k < nb ? partials[i0 + k] : 0u;
                vis += i0 + k < nb ? partials[nb + i0 + k] : 0u;
            }
            s += v[k];
        }
        uint64_t t;
        uint64_t run = carry + block1024_exclusive_scan<uint64_t>(s, tmp, &t);
#pragma unroll
        for (int k = 0; k < kPartIpt; ++k) {
            if (i0 + k < nb && partials) partials[i0 + k] = run;  // (look-back: 0, every block's status cleared)
            run += v[k];
        }
        carry += t;
    }
    if (prow == kPartLookback && partials && threadIdx.x == 0) partials[nb] = 0u;  // (the duplicate's block ticket)
    uint64_t vt, wt = 0, at = carry;
    block1024_exclusive_scan<uint64_t>(vis, tmp, &vt);
    if (src) block1024_exclusive_scan<uint64_t>(wmax, tmp, &wt);
    if (src && prow) block1024_exclusive_scan<uint64_t>(all, tmp, &at);
    if (threadIdx.x == 0) {
        if (!seg_sample && !partials) total[2] = total[3] = 0u;  // (totals only: no sample this frame)
        total[0] = carry;
        total[1] = vt;
        total[4] = wt;
        total[8] = at;
        // (0: the pair buffers are too small; look-back: the duplicate's last
        // block stores the front pairs' count over the 1 that lets it run)
        if (npairs) *npairs = at <= cap ? (prow == kPartLookback ? (at > 0u ? 1u : 0u) : (uint32_t)carry) : 0u;
        if (kept) *kept = (uint32_t)carry;
        // (seq: the host polls total[5]; the totals are visible before it)
        if (seq) __hip_atomic_store(reinterpret_cast<unsigned long long*>(total) + 5, seq, __ATOMIC_RELEASE,
                                    __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// a / b for the small quotients of the emission (a < 2^32, b < 2^16): float
// reciprocal, then one correction step (the estimate is off by at most one)
__device__ __forceinline__ uint32_t udiv_est(uint32_t a, uint32_t b) {
    uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
    const int64_t r = (int64_t)a - (int64_t)q * b;
    if (r < 0) --q;
    else if (r >= (int64_t)b) ++q;
    return q;
}

// Position (0..15) of the i-th set bit of a 16-bit mask (i < popcount).
__device__ __forceinline__ uint32_t nth_bit16(uint32_t m, uint32_t i) {
    uint32_t b = 0;
    uint32_t c = (uint32_t)__builtin_popcount(m & 0xFFu);
    if (i >= c) { i -= c; m >>= 8; b += 8; }
    c = (uint32_t)__builtin_popcount(m & 0xFu);
    if (i >= c) { i -= c; m >>= 4; b += 4; }
    c = (uint32_t)__builtin_popcount(m & 0x3u);
    if (i >= c) { i -= c; m >>= 2; b += 2; }
    return b + (i >= (m & 1u) ? 1u : 0u);
}

// ---- filtered emission (depth-cut frames) ---------------------
// A 16-bit table in LDS (a cut table, min(cut, 0xFFFF); depth keys are < 2^15)
// decides per (splat, bin) whether a pair is emitted: front (FM 2), dk <=
// tab[bin], the pairs a depth-cut frame's front lists hold; behind (FM 3), dk
// > tab[bin], the fallback lists' pairs of the bins whose table entry is the
// cut of a bin with an open quadrant (0xFFFF elsewhere: none).
enum : int { kDupPlain = 0, kDupMark = 1, kDupFront = 2, kDupBehind = 3 };

// A rect within 4x4 bins (the only ones with excluded bins).
__device__ __forceinline__ bool small_rect(const BinRect& r) { return r.bx1 - r.bx0 < 4u && r.by1 - r.by0 < 4u; }

// Its bins as a 16-bit mask (bit dy * 4 + dx), minus the excluded ones.
__device__ __forceinline__ uint32_t rect_inc16(const BinRect& r) {
    const uint32_t cols = r.bx1 - r.bx0 + 1u, rows = r.by1 - r.by0 + 1u, rm = (1u << cols) - 1u;
    uint32_t inc = 0u;
#pragma unroll
    for (uint32_t dy = 0; dy < 4u; ++dy)
        if (dy < rows) inc |= rm << (4u * dy);
    return inc & ~r.excl;
}

template <bool BEHIND>
__device__ __forceinline__ bool tab_keep(const uint16_t* tab, uint32_t bin, uint32_t dk) {
    const uint32_t t = tab[bin];
    return BEHIND ? dk > t : dk <= t;
}

// The bins of inc16 (a small rect's) that the table keeps.  The first four
// bins' table words are read together (independent LDS reads, one wait:
// nearly every rect has at most four bins; an unused slot reads the rect's
// first bin, in the frame), the rest one by one.  (Measured and not kept, the
// count at 50M: a 2x2 fast path with a loop for every other rect, 0.34 ->
// 0.41 ms, since a wave pays the loop's serial reads whenever any of its
// rects is three bins wide or tall; row bases selected instead of multiplied,
// 0.34 -> 0.39 ms.)
template <bool BEHIND>
__device__ __forceinline__ uint32_t filter_inc16(uint32_t inc, const BinRect& r, uint32_t tiles_x, const uint16_t* tab,
                                                 uint32_t dk) {
    const uint32_t b00 = r.by0 * tiles_x + r.bx0;
    auto bin_of = [&](uint32_t b) { return b00 + (b >> 2) * tiles_x + (b & 3u); };
    uint32_t m = inc, bit[4], t[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t b = m ? (uint32_t)__builtin_ctz(m) : 0u;
        bit[j] = m ? 1u << b : 0u;
        m &= m - 1u;
        t[j] = tab[bin_of(b)];
    }
    uint32_t out = 0u;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool keep = BEHIND ? dk > t[j] : dk <= t[j];
        out |= keep ? bit[j] : 0u;
    }
    while (m) {  // (rects of more than four bins)
        const uint32_t b = (uint32_t)__builtin_ctz(m);
        m &= m - 1u;
        if (tab_keep<BEHIND>(tab, bin_of(b), dk)) out |= 1u << b;
    }
    return out;
}

// Pairs an item emits under filter mode FM (every bin row owned).  Front: a
// small rect its kept bins; a larger one every bin (they are emitted whole
// and marked, kBehindFlag, so the sort's first pass still drops their behind
// pairs; such splats are few).  Behind: every kept bin (a loop: the fallback
// runs only when quadrants are open).
template <int FM>
__device__ __forceinline__ uint32_t filtered_count(uint32_t lo, uint32_t hi, bool masked, uint32_t dk, uint32_t tiles_x,
                                                   uint32_t nbins, const uint16_t* tab) {
    const BinRect r = bin_rect(lo, hi, masked);
    if (r.empty) return 0u;
    if constexpr (FM == kDupFront) {
        if (small_rect(r))
            return (uint32_t)__builtin_popcount(filter_inc16<false>(rect_inc16(r), r, tiles_x, tab, dk));
        return (r.bx1 - r.bx0 + 1u) * (r.by1 - r.by0 + 1u);  // (a larger rect has no excluded bins)
    } else {
        uint32_t c = 0u;
        for (uint32_t by = r.by0; by <= r.by1; ++by)
            for (uint32_t bx = r.bx0; bx <= r.bx1; ++bx)
                c += !bin_excluded(r, by, bx) && tab_keep<true>(tab, by * tiles_x + bx, dk) ? 1u : 0u;
        return c;
    }
}

// Stages the table (nbins words, min(t, 0xFFFF)) in LDS: four loads per lane
// issued together (clamped, so none waits inside a branch), then the stores.
__device__ __forceinline__ void stage_tab16(const uint32_t* __restrict__ t, uint32_t nbins, uint16_t* tab) {
    for (uint32_t i0 = threadIdx.x; i0 < nbins; i0 += 4u * blockDim.x) {
        uint32_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = t[min(i0 + k * blockDim.x, nbins - 1u)];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (i0 + k * blockDim.x < nbins) tab[i0 + k * blockDim.x] = (uint16_t)min(v[k], 0xFFFFu);
    }
}

// Per 4096-item block (the scan's and the duplicate's blocking): the pairs the
// block's items emit under FM into out[b] and, when vis is set, the items
// that emit any into vis[b] (plain stores).  Persistent: a workgroup stages
// the table in LDS once and then walks blocks blockIdx.x, + gridDim.x, ...,
// loading the next block's rects and keys while it counts the current one
// (one table copy per workgroup instead of per block: at 50M splats @4K,
// 12k blocks would read 16 KB each).  guard (may be null): nothing while
// *guard == 0.
constexpr int kCountGrid = 512;  // 2 workgroups of 1024 lanes per CU
template <int FM>
__global__ __launch_bounds__(1024) void filtered_count_kernel(const uint32_t* __restrict__ rect_lo,
                                                              const uint32_t* __restrict__ rect_hi,
                                                              const uint32_t* __restrict__ dkey, uint32_t n, bool masked,
                                                              uint32_t tiles_x, const uint32_t* __restrict__ table,
                                                              uint32_t nbins, unsigned long long* __restrict__ out,
                                                              unsigned long long* __restrict__ vis,
                                                              const unsigned long long* __restrict__ guard) {
    if (guard && *guard == 0ull) return;
    extern __shared__ uint16_t tab[];
    __shared__ uint2 wsum[2][16];  // (double-buffered: one barrier per block)
    constexpr int IPT = kScanItems / 1024;
    const uint32_t tid = threadIdx.x, nblocks = (n + kScanItems - 1) / kScanItems;
    uint32_t lo[IPT], hi[IPT], dk[IPT];
    auto load = [&](uint32_t b, uint32_t* l, uint32_t* h, uint32_t* d) {
#if GS_BUF_LOADS  // (A/B: raw buffer loads, reads past n return 0)
        const uint32_t base = b < nblocks ? b * kScanItems : n;
        const BufU32 blo(rect_lo, base, n, kScanItems), bhi(rect_hi, base, n, kScanItems), bdk(dkey, base, n, kScanItems);
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            l[k] = blo[k * 1024 + tid];
            h[k] = bhi[k * 1024 + tid];
            d[k] = bdk[k * 1024 + tid];
        }
#else  // (clamped: none waits in a branch; past n counted as nothing below)
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t j = min(b * kScanItems + k * 1024 + tid, n - 1u);
            l[k] = rect_lo[j];
            h[k] = rect_hi[j];
            d[k] = dkey[j];
        }
#endif
    };
    uint32_t b = blockIdx.x;
    load(b, lo, hi, dk);
    stage_tab16(table, nbins, tab);
    __syncthreads();
    for (int par = 0; b < nblocks; b += gridDim.x, par ^= 1) {
        uint32_t nlo[IPT], nhi[IPT], ndk[IPT];
        load(b + gridDim.x, nlo, nhi, ndk);  // (the next block's, in flight while this one counts)
        uint32_t c = 0u, v = 0u;
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t x =
                b * kScanItems + k * 1024 + tid < n ? filtered_count<FM>(lo[k], hi[k], masked, dk[k], tiles_x, nbins, tab) : 0u;
            c += x;
            v += x > 0u;
        }
        c = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(c), 63);
        v = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(v), 63);
        if ((tid & 63u) == 0) wsum[par][tid >> 6] = make_uint2(c, v);
        block_lds_sync();
        if (tid == 0) {
            uint64_t sc = 0, sv = 0;
#pragma unroll
            for (int w = 0; w < 16; ++w) {
                sc += wsum[par][w].x;
                sv += wsum[par][w].y;
            }
            out[b] = sc;
            if (vis) vis[b] = sv;
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            lo[k] = nlo[k];
            hi[k] = nhi[k];
            dk[k] = ndk[k];
        }
    }
}

// Wave-cooperative emission of 64 consecutive items' pairs (every bin row
// owned): the items own the contiguous pair range [off0, off0 + T); lane q of
// a 64-pair chunk writes pair off0 + q0 + q (coalesced).  Its item: the last
// lane whose range starts at or before it (start marks in mk, this wave's 64
// LDS words, an inclusive max-scan); its bin: the (q - start)-th bin of that
// item's rect in row-major order, minus the excluded bins -- exactly what
// emit_bin_pairs writes there.  c: the item's pair count (0: none), start:
// its first pair - off0.  on_pair(g, bin, key) runs for every pair written
// (g absolute) and returns the key stored.
// gen: the wave's chunk counter (GS_DUP_TAG: a mark carries its chunk's
// number, so stale marks are ignored instead of cleared; mk starts at ~0).
#ifndef GS_DUP_TAG  // A/B knob
#define GS_DUP_TAG 0
#endif
// inc: the item's emitted bins of a rect within 4x4 bins (bit dy*4 + dx; the
// included ones with excluded bins, or the kept ones of a filtered emission),
// or 0: every bin of the rect in row-major order (minus none).
template <typename F>
__device__ __forceinline__ void coop_emit(uint32_t* mk, uint32_t lane, const BinRect& r, uint32_t inc, uint32_t c,
                                          uint32_t start, uint32_t off0, uint32_t val, uint32_t khi, uint32_t tiles_x,
                                          uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, uint32_t& gen,
                                          F&& on_pair) {
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<true>(c > 0u ? start + c : 0u), 63);
    const uint32_t cols = r.bx1 - r.bx0 + 1u;
    const uint32_t pa = r.bx0 | (r.by0 << 16), pb = (cols & 0xFFFFu) | (inc << 16);
    uint32_t carry = 0;
    for (uint32_t q0 = 0; q0 < T; q0 += 64u) {
#if GS_DUP_TAG
        ++gen;
        wave_lds_sync();  // the last chunk's mark reads are done
        if (c > 0u && start >= q0 && start - q0 < 64u) mk[start - q0] = gen << 7 | (lane + 1u);
        wave_lds_sync();
        const uint32_t mv = mk[lane];
        uint32_t own1 = wave_scan_dpp<true>(mv >> 7 == gen ? mv & 127u : 0u);
#else
        wave_lds_sync();  // the last chunk's mark reads are done
        mk[lane] = 0u;
        wave_lds_sync();
        if (c > 0u && start >= q0 && start - q0 < 64u) mk[start - q0] = lane + 1u;
        wave_lds_sync();
        uint32_t own1 = wave_scan_dpp<true>(mk[lane]);
#endif
        own1 = own1 > carry ? own1 : carry;
        carry = (uint32_t)__builtin_amdgcn_readlane((int)own1, 63);
        const int ol = (int)(own1 > 0u ? own1 - 1u : 0u);
        const uint32_t o_start = (uint32_t)__shfl((int)start, ol, 64);
        const uint32_t o_pa = (uint32_t)__shfl((int)pa, ol, 64);
        const uint32_t o_pb = (uint32_t)__shfl((int)pb, ol, 64);
        const uint32_t o_val = (uint32_t)__shfl((int)val, ol, 64);
        const uint32_t o_khi = (uint32_t)__shfl((int)khi, ol, 64);
        const uint32_t q = q0 + lane;
        if (q < T) {
            const uint32_t li = q - o_start, oinc = o_pb >> 16, ocols = o_pb & 0xFFFFu;
            uint32_t dy, dx;
            if (oinc) {
                const uint32_t b = nth_bit16(oinc, li);
                dy = b >> 2;
                dx = b & 3u;
            } else {
                dy = udiv_est(li, ocols);
                dx = li - dy * ocols;
            }
            const uint32_t bin = ((o_pa >> 16) + dy) * tiles_x + (o_pa & 0xFFFFu) + dx;
            keys[off0 + q] = on_pair(off0 + q, bin, o_khi | bin);
            vals[off0 + q] = o_val;
        }
    }
}

__device__ __forceinline__ uint32_t pad32(uint32_t i) { return i + (i >> 5); }  // LDS bank spread

// Down-sweep fused with the duplicate: the block's pair offsets are scanned
// in LDS (counts loaded striped, transposed so each lane scans kScanIpt
// consecutive items, read back striped), then every splat emits its pairs
// straight from its rect in registers (striped, one splat per lane per
// round: neighbouring lanes write neighbouring pair runs).  The rects are
// read once here and the offsets never leave LDS.
#ifndef GS_DUP_THREADS  // A/B knob
#define GS_DUP_THREADS 1024
#endif
constexpr int kDupThreads = GS_DUP_THREADS;          // 16 waves: many waves to hide the pair stores
#ifndef GS_DUP_COOP  // A/B knob: 1 = wave-cooperative emission when every bin row is owned
#define GS_DUP_COOP 1
#endif
constexpr int kDupIpt = kScanItems / kDupThreads;    // 4 items per lane

// Exclusive scan over a kDupThreads-lane workgroup (LDS-only barriers).
__device__ __forceinline__ uint32_t block_dup_exclusive_scan(uint32_t v, uint32_t* tmp, uint32_t* total) {
    constexpr int W = kDupThreads / 64;
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

// Decoupled look-back (the front duplicate, GS_DUP_LOOKBACK): block b's
// status word lb[b] is 0 (not yet), kLbAgg | its pair count, or kLbIncl | the
// pairs of blocks 0..b.  Called by wave 0 with the block's count; returns the
// pairs of blocks 0..b-1 in every lane.  Each step reads the 64 statuses below
// a window at once (per-lane addresses: vector loads at agent scope, which
// see other XCDs' stores); it is complete when every status up to the
// nearest inclusive one is published.  Blocks are numbered by a ticket
// (lb[nb]) taken at start, so every predecessor a block waits for is already
// running.  The spin is bounded (kLbSpinMax sleeps): a block that gives up
// sums what it saw, and its pair run is then dropped by the capacity test,
// never written out of bounds.
constexpr uint64_t kLbAgg = 1ull << 62, kLbIncl = 2ull << 62;
constexpr uint32_t kLbSpinMax = 1u << 20;
__device__ __forceinline__ uint32_t lookback_prefix(uint64_t* lb, uint32_t b, uint32_t count) {
    const uint32_t lane = threadIdx.x & 63u;
    if (lane == 0)
        __hip_atomic_store(lb + b, (b ? kLbAgg : kLbIncl) | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (b == 0) return 0u;
    uint32_t excl = 0;
    for (int64_t w = b;; w -= 64) {
        const int64_t idx = w - 1 - (int64_t)lane;
        uint64_t v = kLbIncl, incl, below;
        uint32_t first;
        for (uint32_t spin = 0;; ++spin) {
            v = idx >= 0 ? __hip_atomic_load(lb + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kLbIncl;
            incl = __ballot((v >> 62) == 2u);
            first = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;
            below = first >= 63u ? ~0ull : (2ull << first) - 1ull;  // (lanes 0..first)
            if ((__ballot((v >> 62) == 0u) & below) == 0ull || spin >= kLbSpinMax) break;
            __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t mine = lane <= first ? (uint32_t)v : 0u;
        excl += (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(mine), 63);
        if (first < 64u) break;
    }
    if (lane == 0)
        __hip_atomic_store(lb + b, kLbIncl | (uint64_t)(excl + count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return excl;
}

// FM (filter mode): kDupPlain every pair; kDupMark every pair, those behind
// their bin's cut (ftab, the cut table) marked with kBehindFlag; kDupFront the
// front pairs (filtered_count; the block's offsets are then scanned from
// launch_front_count's sums); kDupBehind the fallback lists' pairs (ftab: the
// open bins' cuts, one splat per lane).
// LB (kDupFront): the block's offset by look-back (lookback_prefix; lb: nb
// status words and the ticket), no scan of counts before; the block numbered
// last stores the front pairs' count into np_out; a block whose pairs would
// pass cap writes none.
template <int FM, bool LB = false>
__global__ __launch_bounds__(kDupThreads) void scan_duplicate_kernel(CountSrc src, uint32_t n,
                                                                     const uint64_t* __restrict__ partials,
                                                                     const uint32_t* __restrict__ order,
                                                                     const uint32_t* __restrict__ dkey, int bin_bits,
                                                                     uint32_t tiles_x, uint32_t* __restrict__ keys,
                                                                     uint32_t* __restrict__ vals,
                                                                     const uint32_t* __restrict__ npairs,
                                                                     PassCounts pc, const uint32_t* __restrict__ fcut,
                                                                     uint32_t nbins, uint64_t* __restrict__ lb = nullptr,
                                                                     uint32_t* np_out = nullptr,  // (may be npairs)
                                                                     uint32_t cap = 0u) {
    // no pairs, or more than the buffers hold (the host re-runs); (LB: no
    // guard, the capacity test below keeps every store in the buffers)
    if (!LB && *npairs == 0u) return;
    __shared__ uint32_t tmp[kDupThreads / 64];
    __shared__ uint32_t lbs[2];  // (LB) the block's ticket, then its offset
    __shared__ uint32_t st[kScanItems + kScanItems / 32];
    __shared__ uint32_t lh[kDupCountTiles][kSortBins];  // digit counts of the block's first sort tiles
    __shared__ uint32_t mk[kDupThreads / 64][64];        // coop_emit's start marks, per wave
    extern __shared__ uint16_t scut[];                   // (fcut, dynamic: nbins words) the table, min(t, 0xFFFF)
    static_assert(sizeof tmp + sizeof st + sizeof lh + sizeof mk + kDupCutBins * 2 <= kLdsBytes,
                  "scan_duplicate_kernel's LDS (static + the largest cut table) exceeds a gfx950 workgroup's");
    const uint32_t nblocks = (n + kScanItems - 1) / kScanItems;
    uint32_t bid = blockIdx.x;
    if constexpr (LB) {
        if (threadIdx.x == 0)
            lbs[0] = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(lb + nblocks), 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        block_lds_sync();
        bid = lbs[0];
    }
    const uint32_t blk = bid * kScanItems, tid = threadIdx.x;
    // every global load of the block up front (clamped, branch-free), before
    // the first pair store: vmcnt counts loads and stores together, so a load
    // issued between stores would wait for them
    // (absent arrays read a stand-in, so no load sits in a branch, where its
    // value would be waited for at once)
    uint64_t part = LB ? 0ull : partials[bid];
    uint32_t rlo[kDupIpt], rhi[kDupIpt], dk[kDupIpt], ord[kDupIpt];
#if GS_BUF_LOADS  // (A/B: raw buffer loads, reads past n return 0; those items get the empty rect below)
    const BufU32 blo(src.lo, blk, n, kScanItems), bhi(src.hi, blk, n, kScanItems),
        bdk(dkey ? dkey : src.lo, blk, n, kScanItems), bord(order ? order : src.lo, blk, n, kScanItems);
#pragma unroll
    for (int k = 0; k < kDupIpt; ++k) {
        const uint32_t i = k * kDupThreads + tid;
        rlo[k] = blo[i];
        rhi[k] = bhi[i];
        dk[k] = bdk[i];
        ord[k] = bord[i];
    }
#else
    const uint32_t* dsrc = dkey ? dkey : src.lo;
    const uint32_t* osrc = order ? order : src.lo;
#pragma unroll
    for (int k = 0; k < kDupIpt; ++k) {
        const uint32_t j = min(blk + k * kDupThreads + tid, n - 1u);
        rlo[k] = src.lo[j];
        rhi[k] = src.hi[j];
        dk[k] = dsrc[j];
        ord[k] = osrc[j];
    }
#endif
    if (FM != kDupPlain) stage_tab16(fcut, nbins, scut);  // (a depth key is < 2^15: min(t, 0xFFFF) keeps every comparison)
    if (pc.C)
        for (uint32_t i = tid; i < kDupCountTiles * kSortBins; i += kDupThreads) (&lh[0][0])[i] = 0u;
    if (FM >= kDupFront) block_lds_sync();  // (the counts below read the table)
    uint32_t finc[kDupIpt];  // (kDupFront) a small rect's kept bins, reused by the emission
#pragma unroll
    for (int k = 0; k < kDupIpt; ++k) {
        const uint32_t i = k * kDupThreads + tid;
        if (blk + i >= n) {
            rlo[k] = kEmptyRectLo;
            rhi[k] = 0u;
        }
        finc[k] = 0u;
        uint32_t c;
        if constexpr (FM == kDupFront) {
            const BinRect r = bin_rect(rlo[k], rhi[k], src.masked);
            if (r.empty) {
                c = 0u;
            } else if (small_rect(r)) {
                finc[k] = filter_inc16<false>(rect_inc16(r), r, tiles_x, scut, dk[k]);
                c = (uint32_t)__builtin_popcount(finc[k]);
            } else {
                c = (r.bx1 - r.bx0 + 1u) * (r.by1 - r.by0 + 1u);  // (no excluded bins)
            }
        } else if constexpr (FM == kDupBehind) {
            c = filtered_count<FM>(rlo[k], rhi[k], src.masked, dk[k], tiles_x, nbins, scut);
        } else {
            c = rect_tile_count(rlo[k], rhi[k], src.own, src.masked);
        }
        st[pad32(i)] = c;
    }
    block_lds_sync();
    uint32_t v[kDupIpt];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kDupIpt; ++k) {
        v[k] = st[pad32(tid * kDupIpt + k)];
        s += v[k];
    }
    uint32_t t;
    const uint32_t ex = block_dup_exclusive_scan(s, tmp, &t);  // (ends with a barrier)
    if constexpr (LB) {
        if (tid < 64u) {
            const uint32_t e = lookback_prefix(lb, bid, t);
            if (tid == 0) {
                lbs[1] = e;
                if (bid == nblocks - 1u) *np_out = e + t <= cap ? e + t : 0u;  // (the sort's count)
            }
        }
        block_lds_sync();
        part = lbs[1];
        if (part + t > cap) return;  // (only after a spin gave up: the frame's count then differs from P)
    }
    {
        uint32_t run = (uint32_t)part + ex;
#pragma unroll
        for (int k = 0; k < kDupIpt; ++k) {
            st[pad32(tid * kDupIpt + k)] = run;
            run += v[k];
        }
    }
    block_lds_sync();
    // the first sort pass's digit counts per tile of pc.tile pairs (rts_count
    // without its key re-read): the block's pairs are contiguous from its
    // partial, so its first kDupCountTiles tiles count in LDS
    const uint32_t t_lo = pc.C ? (uint32_t)(part / pc.tile) : 0u;
    // (kDupMark, kDupFront) the behind-the-cut mark, from the LDS table
    auto mark = [&](uint32_t bin, uint32_t key) -> uint32_t {
        return (key >> bin_bits) > (uint32_t)scut[bin] ? key | kBehindFlag : key;
    };
    auto count = [&](uint32_t g, uint32_t bin, uint32_t key) -> uint32_t {  // (pc.C) the pair's digit into its tile's counts
        if (FM == kDupMark || FM == kDupFront) {
            key = mark(bin, key);
            if (key & kBehindFlag) return key;  // (the filter drops it)
        } else if (pc.cut && (key >> bin_bits) > pc.cut[bin]) {
            return key;  // (behind its bin's cut: the filter drops it)
        }
        const uint32_t t = udiv_est(g, pc.tile), d = bin & pc.mask;
        if (t - t_lo < kDupCountTiles) atomicAdd(&lh[t - t_lo][d], 1u);
        else atomicAdd(&pc.C[(size_t)d * pc.ntiles + t], 1u);
        return key;
    };
    if (FM != kDupBehind && GS_DUP_COOP && !src.own.owner) {
        // wave-cooperative emission (every bin row owned): each wave's 64
        // consecutive items of a round own one contiguous pair run, written
        // 64 pairs per step by all lanes, so a large splat does not hold its
        // wave's other lanes idle (coop_emit; the same pairs at the same
        // offsets as the per-lane loop below)
        const uint32_t lane = tid & 63u, wave = tid >> 6;
        uint32_t gen = 0;
        mk[wave][lane] = ~0u;  // (no chunk's tag)
#pragma unroll
        for (int k = 0; k < kDupIpt; ++k) {
            const uint32_t i = k * kDupThreads + tid, j = blk + i;
            const BinRect r = bin_rect(rlo[k], rhi[k], src.masked);  // (items past n: the empty rect)
            uint32_t inc, c;
            if (FM == kDupFront && small_rect(r)) {  // (its kept bins; a larger rect emits every bin, marked)
                inc = finc[k];
                c = (uint32_t)__builtin_popcount(inc);
            } else {
                inc = r.excl ? rect_inc16(r) : 0u;
                c = j < n && !r.empty ? rect_tile_count(rlo[k], rhi[k], src.own, src.masked) : 0u;
            }
            const uint32_t off = st[pad32(i)];
            const uint32_t off0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)off);
            const uint32_t khi = dkey ? dk[k] << bin_bits : 0u;
            const uint32_t val = order ? ord[k] : j;
            if (pc.C) coop_emit(mk[wave], lane, r, inc, c, off - off0, off0, val, khi, tiles_x, keys, vals, gen, count);
            else if (FM == kDupMark || FM == kDupFront)
                coop_emit(mk[wave], lane, r, inc, c, off - off0, off0, val, khi, tiles_x, keys, vals, gen,
                          [&](uint32_t, uint32_t bin, uint32_t key) { return mark(bin, key); });
            else coop_emit(mk[wave], lane, r, inc, c, off - off0, off0, val, khi, tiles_x, keys, vals, gen,
                           [](uint32_t, uint32_t, uint32_t key) { return key; });
        }
    } else
#pragma unroll
    for (int k = 0; k < kDupIpt; ++k) {
        const uint32_t i = k * kDupThreads + tid, j = blk + i;
        const BinRect r = bin_rect(rlo[k], rhi[k], src.masked);
        if (j >= n || r.empty) continue;
        const uint32_t off = st[pad32(i)];
        const uint32_t key_hi = dkey ? dk[k] << bin_bits : 0u;  // depth key above the bin id
        const uint32_t val = order ? ord[k] : j;
        if constexpr (FM == kDupBehind) {  // (the fallback lists: the kept bins, filtered_count's)
            const uint32_t d = dk[k];
            emit_bin_pairs_if(r, tiles_x, src.own, key_hi, val, off, keys, vals,
                              [&](uint32_t bin) { return tab_keep<true>(scut, bin, d); }, [](uint32_t, uint32_t) {});
            continue;
        }
        auto keep = [](uint32_t) { return true; };
        if (pc.C) {
            uint32_t t = off / pc.tile, next = (t + 1u) * pc.tile;  // pair offsets rise by one
            emit_bin_pairs_if(r, tiles_x, src.own, key_hi, val, off, keys, vals, keep, [&](uint32_t g, uint32_t bin) {
                if (g == next) {
                    ++t;
                    next += pc.tile;
                }
                if (pc.cut && key_hi >> bin_bits > pc.cut[bin]) return;  // (dropped by the filtered pass)
                const uint32_t d = bin & pc.mask;
                if (t - t_lo < kDupCountTiles) atomicAdd(&lh[t - t_lo][d], 1u);
                else atomicAdd(&pc.C[(size_t)d * pc.ntiles + t], 1u);
            });
        } else {
            emit_bin_pairs_if(r, tiles_x, src.own, key_hi, val, off, keys, vals, keep, [](uint32_t, uint32_t) {});
        }
    }
    if (pc.C) {
        block_lds_sync();
        for (uint32_t i = tid; i < kDupCountTiles * kSortBins; i += kDupThreads) {
            const uint32_t t = i / kSortBins, d = i % kSortBins, v = (&lh[0][0])[i];
            if (v && t_lo + t < pc.ntiles) atomicAdd(&pc.C[(size_t)d * pc.ntiles + t_lo + t], v);
        }
    }
}

// Depth-ordered items: the down-sweep writes every item's pair offset and a
// second kernel emits one splat per lane.  In depth order the splats' sizes
// follow their depth (near splats are large), so 4096-item blocks of the fused
// kernel are badly unbalanced (the last blocks emit many times the pairs):
// 245 us against 123 + 16 us for these two kernels at 6M splats / 4K.
__global__ __launch_bounds__(256) void scan_down_kernel(CountSrc src, uint32_t n,
                                                        const uint64_t* __restrict__ partials,
                                                        uint32_t* __restrict__ offsets) {
    __shared__ uint32_t tmp[4];
    __shared__ uint32_t st[kScanItems + kScanItems / 32];
    const uint32_t blk = blockIdx.x * kScanItems, tid = threadIdx.x;
    uint32_t lo[kScanIpt], hi[kScanIpt];  // (all loads first, as in scan_reduce)
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const uint32_t j = min(blk + k * 256 + tid, n - 1u);
        lo[k] = src.lo[j];
        hi[k] = src.hi[j];
    }
#pragma unroll
    for (int k = 0; k < kScanIpt; ++k) {
        const uint32_t i = k * 256 + tid;
        st[pad32(i)] = blk + i < n ? rect_tile_count(lo[k], hi[k], src.own, src.masked) : 0u;
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

// dks (optional, depth-cut frames): the items' depth keys in the same order,
// carried above the bin id (key = dkey << bin_bits | bin) for the first sort
// pass's cut filter.
__global__ __launch_bounds__(256) void duplicate_kernel(CountSrc src, uint32_t n, const uint32_t* __restrict__ order,
                                                        const uint32_t* __restrict__ offsets, uint32_t tiles_x,
                                                        uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                        const uint32_t* __restrict__ npairs,
                                                        const uint32_t* __restrict__ dks, int bin_bits) {
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= n || *npairs == 0u) return;
    const BinRect r = bin_rect(src.lo[j], src.hi[j], src.masked);
    if (r.empty) return;  // culled
    emit_bin_pairs(r, tiles_x, src.own, dks ? dks[j] << bin_bits : 0u, order ? order[j] : j, offsets[j], keys, vals);
}

// Depth-ordered duplicate, wave-cooperative (every bin row owned): in depth
// order the splats' sizes follow their depth, so one splat per lane leaves
// most lanes idle behind a few large near splats.  A wave's 64 splats own the
// contiguous pair range [off0, off0 + T); lane q of a 64-pair chunk writes
// pair off0 + q0 + q (coalesced).  Its splat: the last lane whose range
// starts at or before it (start marks in LDS, an inclusive max-scan); its
// bin: the (q - start)-th bin of that splat's rect in row-major order, minus
// the excluded bins -- exactly what duplicate_kernel's loop writes there.
__global__ __launch_bounds__(256) void duplicate_coop_kernel(CountSrc src, uint32_t n,
                                                             const uint32_t* __restrict__ order,
                                                             const uint32_t* __restrict__ offsets, uint32_t tiles_x,
                                                             uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                             const uint32_t* __restrict__ npairs,
                                                             const uint32_t* __restrict__ dks, int bin_bits) {
    __shared__ uint32_t mk[4][64];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t w0 = blockIdx.x * 256u + wave * 64u;
    if (w0 >= n || *npairs == 0u) return;  // (whole wave; no workgroup barrier below)
    const uint32_t j = w0 + lane, jc = j < n ? j : n - 1u;
    uint32_t lo = src.lo[jc], hi = src.hi[jc];
    const uint32_t off = offsets[jc];
    const uint32_t val = order ? order[jc] : jc;
    const uint32_t khi = dks ? dks[jc] << bin_bits : 0u;  // (depth-cut frames: the depth key above the bin id)
    if (j >= n) {
        lo = kEmptyRectLo;
        hi = 0u;
    }
    const BinRect r = bin_rect(lo, hi, src.masked);
    const uint32_t c = rect_tile_count(lo, hi, src.own, src.masked);
    const uint32_t off0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)off);  // lane 0 is valid
    uint32_t gen = 0;
    mk[wave][lane] = ~0u;  // (no chunk's tag)
    coop_emit(mk[wave], lane, r, r.excl ? rect_inc16(r) : 0u, c, off - off0, off0, val, khi, tiles_x, keys, vals, gen,
              [](uint32_t, uint32_t, uint32_t key) { return key; });
}

hipError_t launch_tile_count_totals(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, RowOwnership own,
                                    bool masked, uint64_t* partials, uint64_t* total, uint32_t* seg_sample,
                                    uint2* ranges, uint32_t nranges, uint32_t* npairs, uint64_t cap,
                                    uint32_t* zero, uint32_t nzero, hipStream_t st, hipEvent_t done,
                                    unsigned long long seq) {
    const CountSrc src{rect_lo, rect_hi, own, masked};
    const uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) {
        if (nranges) {
            const hipError_t e = hipMemsetAsync(ranges, 0xFF, (size_t)nranges * sizeof(uint2), st);
            if (e != hipSuccess) return e;
        }
        if (nzero) {
            const hipError_t e = hipMemsetAsync(zero, 0, (size_t)nzero * 4, st);
            if (e != hipSuccess) return e;
        }
    } else {
        scan_reduce_kernel<<<nb, 256, 0, st>>>(src, n, partials, ranges, nranges, zero, nzero);
    }
    hipExtLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kPartThreads), 0, st, nullptr, done, 0, partials, nb,
                          total, seg_sample, npairs, cap, nullptr, seq, 0u, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_scan_partials_fused(unsigned long long* part, uint32_t nb, uint64_t* partials, uint64_t* total,
                                      uint32_t* seg_sample, uint32_t* npairs, uint64_t cap, hipStream_t st,
                                      hipEvent_t done, unsigned long long seq, bool front, bool lookback) {
    if (!part) return hipErrorInvalidValue;
    hipExtLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(kPartThreads), 0, st, nullptr, done, 0, partials, nb,
                          total, seg_sample, npairs, cap, part, seq, lookback ? kPartLookback : front ? 3u : 0u,
                          nullptr, nullptr);
    return hipGetLastError();
}

// (dynamic LDS of a staged table of nbins 16-bit words)
static size_t tab_lds(uint32_t nbins) { return ((size_t)nbins * 2 + 15) & ~(size_t)15; }

hipError_t launch_front_count(const uint32_t* rect_lo, const uint32_t* rect_hi, const uint32_t* dkey, uint32_t n,
                              bool masked, uint32_t tiles_x, const uint32_t* cut, uint32_t nbins,
                              unsigned long long* out, hipStream_t st) {
    const uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) return hipSuccess;
    if (!cut || !out || nbins > kDupCutBins) return hipErrorInvalidValue;
    filtered_count_kernel<kDupFront><<<min(nb, (uint32_t)kCountGrid), 1024, tab_lds(nbins), st>>>(
        rect_lo, rect_hi, dkey, n, masked, tiles_x, cut, nbins, out, nullptr, nullptr);
    return hipGetLastError();
}

hipError_t launch_fallback_pairs(const uint32_t* rect_lo, const uint32_t* rect_hi, const uint32_t* dkey, uint32_t n,
                                 bool masked, uint32_t tiles_x, int bin_bits, const uint32_t* table, uint32_t nbins,
                                 const unsigned long long* open, uint64_t* part, uint64_t* total, uint32_t* npairs,
                                 uint32_t* kept, uint64_t cap, uint32_t* keys, uint32_t* vals, hipStream_t st) {
    const uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) return hipSuccess;
    if (!table || !open || !part || !total || !npairs || nbins > kDupCutBins || bin_bits + kDepthBits > 31)
        return hipErrorInvalidValue;
    // per-block pair counts and items with pairs (the scan's two rows), their
    // scan into npairs / kept (only with an open quadrant), then the pairs
    filtered_count_kernel<kDupBehind><<<min(nb, (uint32_t)kCountGrid), 1024, tab_lds(nbins), st>>>(
        rect_lo, rect_hi, dkey, n, masked, tiles_x, table, nbins, reinterpret_cast<unsigned long long*>(part),
        reinterpret_cast<unsigned long long*>(part) + nb, open);
    scan_partials_kernel<<<1, kPartThreads, 0, st>>>(part, nb, total, nullptr, npairs, cap, nullptr, 0ull, 0u, open,
                                                     kept);
    const CountSrc src{rect_lo, rect_hi, RowOwnership{nullptr, 0u}, masked};
    scan_duplicate_kernel<kDupBehind><<<nb, kDupThreads, tab_lds(nbins), st>>>(
        src, n, part, nullptr, dkey, bin_bits, tiles_x, keys, vals, npairs, PassCounts{}, table, nbins);
    return hipGetLastError();
}

hipError_t launch_scan_duplicate(const uint32_t* order, const uint32_t* rect_lo, const uint32_t* rect_hi,
                                 const uint64_t* partials, uint32_t n, uint32_t tiles_x, RowOwnership own, bool masked,
                                 const uint32_t* dkey, int bin_bits, uint32_t* keys, uint32_t* vals,
                                 const uint32_t* npairs, hipStream_t st, uint32_t* offsets, PassCounts pc,
                                 const uint32_t* fcut, uint32_t nbins, bool front, uint32_t* np_out, uint32_t cap) {
    const uint32_t nb = (n + kScanItems - 1) / kScanItems;
    if (nb == 0) return hipSuccess;
    // (order: dkey holds the items' depth keys in that order)
    if (dkey && bin_bits + kDepthBits > 32) return hipErrorInvalidValue;
    const CountSrc src{rect_lo, rect_hi, own, masked};
    // (the marks: index order, the cooperative emission, the flag above the depth key)
    if (np_out && (order || own.owner)) return hipErrorInvalidValue;  // (look-back: index order, every row owned)
    if ((fcut || front) &&
        (!fcut || order || own.owner || !GS_DUP_COOP || !dkey || nbins > kDupCutBins || bin_bits + kDepthBits > 31))
        return hipErrorInvalidValue;
    if (order) {  // depth order: per-item offsets, then one splat per lane
        if (!offsets) return hipErrorInvalidValue;
        scan_down_kernel<<<nb, 256, 0, st>>>(src, n, partials, offsets);
#ifndef GS_AB_DUP_LANE
        if (!own.owner)
            duplicate_coop_kernel<<<(n + 255) / 256, 256, 0, st>>>(src, n, order, offsets, tiles_x, keys, vals, npairs,
                                                                   dkey, bin_bits);
        else
#endif
            duplicate_kernel<<<(n + 255) / 256, 256, 0, st>>>(src, n, order, offsets, tiles_x, keys, vals, npairs, dkey,
                                                              bin_bits);
        return hipGetLastError();
    }
    // (the cut table sized to the frame: a block that fits beside the previous
    // composite's workgroups starts sooner)
    const size_t lds = fcut ? tab_lds(nbins) : 0;
    if (np_out) {  // (offsets by look-back: partials holds nb + 1 cleared words)
        uint64_t* lb = const_cast<uint64_t*>(partials);
        if (front)
            scan_duplicate_kernel<kDupFront, true><<<nb, kDupThreads, lds, st>>>(
                src, n, partials, order, dkey, bin_bits, tiles_x, keys, vals, npairs, pc, fcut, nbins, lb, np_out, cap);
        else if (fcut)
            scan_duplicate_kernel<kDupMark, true><<<nb, kDupThreads, lds, st>>>(
                src, n, partials, order, dkey, bin_bits, tiles_x, keys, vals, npairs, pc, fcut, nbins, lb, np_out, cap);
        else
            scan_duplicate_kernel<kDupPlain, true><<<nb, kDupThreads, lds, st>>>(
                src, n, partials, order, dkey, bin_bits, tiles_x, keys, vals, npairs, pc, fcut, nbins, lb, np_out, cap);
    } else if (front)
        scan_duplicate_kernel<kDupFront><<<nb, kDupThreads, lds, st>>>(src, n, partials, order, dkey, bin_bits, tiles_x,
                                                                       keys, vals, npairs, pc, fcut, nbins);
    else if (fcut)
        scan_duplicate_kernel<kDupMark><<<nb, kDupThreads, lds, st>>>(src, n, partials, order, dkey, bin_bits, tiles_x,
                                                                      keys, vals, npairs, pc, fcut, nbins);
    else
        scan_duplicate_kernel<kDupPlain><<<nb, kDupThreads, lds, st>>>(src, n, partials, order, dkey, bin_bits, tiles_x,
                                                                       keys, vals, npairs, pc, fcut, nbins);
    return hipGetLastError();
}

}  // namespace gs
