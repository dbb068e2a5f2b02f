// radix_sort.hip — stable LSD radix sort of uint32 keys with NV uint32 value
// arrays, reduce-then-scan per digit pass (no inter-workgroup waiting).
//
// Used twice per frame by the binning stage: splats by
// 15-bit depth key carrying (index, rect_lo, rect_hi) — 2 passes over N — then
// (bin, splat) pairs by bin id — 2 passes over P at 1080p.
//
// Per pass (digit width <= 8 bits, D = 2^width digits):
//   rts_count  per tile of 512 x IPT items: LDS digit histogram (wave-private
//              copies) -> C[digit][tile]
//   rts_scan   one workgroup per digit: exclusive scan of its row of C over the
//              tiles (in place) + the digit's total
//   rts_pass   per tile: digit starts = block scan of the D totals; stable
//              tile-local ranks (wave-private ballot match); each array staged
//              through LDS in tile-sorted order and written out as coalesced
//              digit runs at start[d] + C[d][tile] + rank
//
// Why not onesweep: a decoupled look-back reads status words written by
// workgroups on other XCDs (agent-scope loads that miss the per-XCD L2), so
// every look-back hop costs a trip to the fabric; measured on MI355X the
// onesweep pass took 85-90 us where this pass takes 57-64 us plus ~20 us of
// count+scan.  The count kernel re-reads the keys once per
// pass (4 B/item), which is the price of having no cross-workgroup wait.
#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

constexpr int kRsThreads = 512;
constexpr int kRsWaves = kRsThreads / 64;

static_assert(kSortBins == 256, "8-bit digits");

template <int NV>
struct SortIO {
    const uint32_t* kin;
    const uint32_t* vin[NV];  // vin[0] may be null: value = item index
    uint32_t* kout;
    uint32_t* vout[NV];
};

#ifndef GS_RS_IPT1  // A/B knobs (tools/build_variant.py)
#define GS_RS_IPT1 8  // 4096-pair tiles: sort stage 115.7 vs 119.6 us for 6144 (16: 129) after the run-end merge skip (profiles/r03/ab_sort_tile_ipt.txt)
#endif
#ifndef GS_RS_PASS_WAVES  // min waves per SIMD of the pass kernel (HIP launch bounds)
#define GS_RS_PASS_WAVES 1
#endif
constexpr int ipt_for(int nv) { return nv == 1 ? GS_RS_IPT1 : 8; }
#ifndef GS_RS_PAIR_STAGE  // A/B knob: 1 = one-array passes stage (key, value) pairs through LDS together
#define GS_RS_PAIR_STAGE 0
#endif
constexpr uint32_t tile_items(int nv) { return (uint32_t)kRsThreads * ipt_for(nv); }

// Exclusive scan over the kRsThreads-lane workgroup (LDS-only barriers).
__device__ __forceinline__ uint32_t block512_exclusive_scan(uint32_t v, uint32_t* tmp, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t inc = wave_scan_dpp<false>(v);
    if (lane == 63) tmp[wave] = inc;
    block_lds_sync();
    uint32_t base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) {
        const uint32_t x = tmp[w];
        base += (uint32_t)w < wave ? x : 0u;
        tot += x;
    }
    *total = tot;
    block_lds_sync();
    return base + inc - v;
}

// Lanes of one wave holding the same digit: mask of peers (BITS ballots).
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        peers &= bit ? bal : ~bal;
    }
    return peers;
}

// SortFilter::keep against the LDS copy of the cut table (SortFilter::lds_bins)
__device__ __forceinline__ bool keep_lds(const SortFilter& f, const uint16_t* tab, uint32_t key) {
    return (((key & f.kmask) >> f.dshift) <= (uint32_t)tab[key & f.bmask]) != (f.behind != 0u);
}
// Copies the cut table into LDS (min(cut, 0xFFFF): depth keys are < 2^15).
__device__ __forceinline__ void stage_filter_table(const SortFilter& f, uint16_t* tab) {
    for (uint32_t i = threadIdx.x; i < f.lds_bins; i += blockDim.x) tab[i] = (uint16_t)min(f.cut[i], 0xFFFFu);
    __syncthreads();
}

// FILT (the first pass of a depth-cut frame's bin sort, SortFilter): only
// the items at or ahead of their bin's cut are counted and sorted.  Compiled
// in only where it is used, so the other kernels keep their registers.
template <int NV, bool FILT, bool STRIDE = false>
__global__ __launch_bounds__(512) void rts_count_kernel(const uint32_t* __restrict__ keys, uint32_t n, int shift,
                                                        uint32_t mask, uint32_t* __restrict__ C, uint32_t ntiles,
                                                        const uint32_t* __restrict__ n_dev, const SortFilter flt) {
    constexpr uint32_t TILE = tile_items(NV);
    if (n_dev) n = *n_dev;  // tiles past it count zeros
    if (n == 0u) return;    // (nothing to sort: the scan and the pass return at once)
    __shared__ uint32_t h[kRsWaves][kSortBins];
    extern __shared__ uint16_t ftab[];  // (FILT, flt.lds_bins words)
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    if (FILT && flt.lds_bins) stage_filter_table(flt, ftab);
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    for (int i = tid; i < kRsWaves * kSortBins; i += kRsThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint32_t t0 = tile * TILE;
    constexpr int K = TILE / kRsThreads;
    if (t0 >= n) {  // (n read on the device: tiles past it count zeros)
    } else {
        // all keys loaded first (clamped): one memory round trip
        uint32_t kk[K];
#pragma unroll
        for (int k = 0; k < K; ++k) kk[k] = keys[min(t0 + k * kRsThreads + tid, n - 1u)];
        bool keep[K];
#pragma unroll
        for (int k = 0; k < K; ++k) keep[k] = !FILT || (flt.lds_bins ? keep_lds(flt, ftab, kk[k]) : flt.keep(kk[k]));
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (t0 + k * kRsThreads + tid < n && keep[k])
                atomicAdd(&h[wave][(kk[k] >> shift) & mask], 1u);
    }
    __syncthreads();
    if (tid <= mask) {
        uint32_t c = 0;
#pragma unroll
        for (int w = 0; w < kRsWaves; ++w) c += h[w][tid];
        C[(size_t)tid * ntiles + tile] = c;
    }
    if constexpr (!STRIDE) break;
    __syncthreads();  // (the next tile clears h)
    }
}

// One 1024-lane workgroup per digit: each lane scans kRsScanIpt consecutive
// tile counts in registers, one block-wide scan joins them (one pass for up
// to 4096 tiles; larger grids loop).
constexpr int kRsScanThreads = 1024;
constexpr int kRsScanIpt = 4;

__global__ __launch_bounds__(kRsScanThreads) void rts_scan_kernel(uint32_t* __restrict__ C, uint32_t ntiles,
                                                                  uint32_t* __restrict__ totals,
                                                                  const uint32_t* __restrict__ n_dev) {
    constexpr int W = kRsScanThreads / 64;
    if (n_dev && *n_dev == 0u) {  // nothing to sort (the passes return at once too)
        if (threadIdx.x == 0) totals[blockIdx.x] = 0u;
        return;
    }
    constexpr uint32_t CH = kRsScanThreads * kRsScanIpt;
    __shared__ uint32_t tmp[W];
    uint32_t* row = C + (size_t)blockIdx.x * ntiles;
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < ntiles; b0 += CH) {
        const uint32_t i0 = b0 + threadIdx.x * kRsScanIpt;
        uint32_t v[kRsScanIpt], s = 0;
#pragma unroll
        for (int k = 0; k < kRsScanIpt; ++k) {
            v[k] = i0 + k < ntiles ? row[i0 + k] : 0u;
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
        for (int k = 0; k < kRsScanIpt; ++k) {
            if (i0 + k < ntiles) row[i0 + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// ranges (last pass only, may be null): per key value k = key & rmask, the
// global extent [x, ~y) of k's run in the sorted output, stored as {x, ~end}
// and merged with atomicMin over tiles (order-independent, so deterministic);
// the caller fills the array with 0xFF first (empty = {~0, ~0} = [~0, 0)).
// Bits above rmask ride along unsorted (the bin-first binning carries each
// pair's depth key there, bin_depth_sort.hip).
// STRIDE: a fixed grid loops over the tiles (the depth-cut fallback lists'
// sort, whose input is usually empty: a small grid then costs little).
template <int NV, int BITS, bool FILT, bool STRIDE = false>
#ifdef GS_RS_PASS_W8  // A/B knob: every pass at 8 waves per SIMD (the filtered ones spill)
#define GS_RS_PASS_ATTR __attribute__((amdgpu_waves_per_eu(8, 8)))
#else
#define GS_RS_PASS_ATTR
#endif
__global__ __launch_bounds__(512, GS_RS_PASS_WAVES) GS_RS_PASS_ATTR void rts_pass_kernel(SortIO<NV> io, uint32_t n, int shift, uint32_t mask,
                                                       const uint32_t* __restrict__ C,
                                                       const uint32_t* __restrict__ totals, uint32_t ntiles,
                                                       uint2* __restrict__ ranges, uint32_t rmask,
                                                       const uint32_t* __restrict__ n_dev, const SortFilter flt) {
    constexpr int IPT = ipt_for(NV);
    constexpr uint32_t TILE = tile_items(NV);
    if (n_dev) n = *n_dev;
    if (blockIdx.x * TILE >= n) return;  // (whole workgroup: before any barrier)
    constexpr uint32_t WAVE_ITEMS = 64u * IPT;
    constexpr uint32_t ND = 1u << BITS;
    __shared__ uint32_t wh[kRsWaves][ND];  // wave-private running counts -> wave offsets
    __shared__ uint32_t blk_start[ND];     // tile-local start of each digit
    __shared__ uint32_t gbase[ND];         // global start of this tile's digit run
    // (one array: keys and values staged together as (key, value) pairs, one
    // scatter and one gather through LDS instead of one per array)
    constexpr bool kPair = NV == 1 && GS_RS_PAIR_STAGE;
    __shared__ uint32_t stage[kPair ? 2 * TILE : TILE];
    __shared__ uint32_t tmp[kRsWaves];
    __shared__ uint32_t rflag[ND];         // (ranges, shift > 0: run-end merges this tile skips)

    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    extern __shared__ uint16_t ftab[];  // (FILT, flt.lds_bins words)
    if (FILT && flt.lds_bins) stage_filter_table(flt, ftab);
    for (uint32_t tile = blockIdx.x; tile * TILE < n; tile += gridDim.x) {
    for (uint32_t i = tid; i < kRsWaves * ND; i += kRsThreads) (&wh[0][0])[i] = 0;
    // Keys and all value arrays are loaded up front so their latency hides
    // behind the ranking.  Barriers here order LDS only: they never wait for
    // this tile's outstanding global stores.
    const uint32_t base = tile * TILE + wave * WAVE_ITEMS;
    uint32_t key[IPT], pos[IPT], val[NV][IPT];
    if constexpr (NV == 1) {
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t idx = base + k * 64 + lane;
            key[k] = idx < n ? io.kin[idx] : 0u;
        }
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t idx = base + k * 64 + lane;
            val[0][k] = idx < n ? (io.vin[0] ? io.vin[0][idx] : idx) : 0u;
        }
    } else {
        // several value arrays, the first possibly absent (value = index):
        // unconditional loads, positions clamped into the input (a per-item
        // select waits for each load where it is made), an absent array not
        // read at all (a uniform branch) and its index substituted when
        // staged.  (For one array the conditional loads keep fewer registers
        // live: measured faster there.)
#pragma unroll
        for (int k = 0; k < IPT; ++k) key[k] = io.kin[min(base + k * 64 + lane, n - 1u)];
#pragma unroll
        for (int a = 0; a < NV; ++a) {
            if (io.vin[a]) {
#pragma unroll
                for (int k = 0; k < IPT; ++k) val[a][k] = io.vin[a][min(base + k * 64 + lane, n - 1u)];
            } else {
#pragma unroll
                for (int k = 0; k < IPT; ++k) val[a][k] = 0u;
            }
        }
    }
    // global start of every digit of this tile (independent of the ranking)
    uint32_t all;
    const uint32_t dstart = block512_exclusive_scan(tid <= mask ? totals[tid] : 0u, tmp, &all);
    if (tid <= mask) gbase[tid] = dstart + C[(size_t)tid * ntiles + tile];
    // Run-end merges (ranges, a last pass above lower digits).  The input is
    // sorted by its low `shift` bits (LSD), so a key's run starts in the first
    // tile that holds the key's low value with its digit.  When the previous
    // tile lies wholly inside this tile's first low value and holds digit d,
    // no run of (d, that low value) starts here: bit 0 of rflag[d] skips the
    // start merge; bit 1 the end merge, mirrored with the next tile.  Any
    // other run end still merges with atomicMin (an extra merge is harmless),
    // so only tiles at a low value's edges merge: each merge is a memory-side
    // atomic on a few contended lines (measured 14 us per frame unskipped).
    const bool rskip = ranges && shift > 0;
    const uint32_t lm = (1u << shift) - 1u;
    uint32_t lo_first = 0, lo_last = 0;
    if (rskip) {
        const uint32_t t0 = tile * TILE, t1 = min(t0 + TILE, n);
        lo_first = io.kin[t0] & lm;
        lo_last = io.kin[t1 - 1] & lm;
        if (tid <= mask) {
            const uint32_t* Cd = C + (size_t)tid * ntiles;
            uint32_t f = 0;
            if (tile > 0 && (io.kin[t0 - TILE] & lm) == lo_first && (io.kin[t0 - 1] & lm) == lo_first &&
                Cd[tile] != Cd[tile - 1])
                f |= 1u;
            if (t1 < n) {  // (tile + 1 < ntiles)
                const uint32_t t2 = min(t1 + TILE, n);
                const uint32_t after = tile + 2 < ntiles ? Cd[tile + 2] : totals[tid];
                if ((io.kin[t1] & lm) == lo_last && (io.kin[t2 - 1] & lm) == lo_last && after != Cd[tile + 1])
                    f |= 2u;
            }
            rflag[tid] = f;
        }
    }
    uint32_t keep = 0;  // (filtered: bit k = slot k is kept)
    if constexpr (FILT) {
        if (tile == 0 && tid == 0) *flt.kept = all;  // (the items every tile keeps)
#pragma unroll
        for (int k = 0; k < IPT; ++k)
            keep |= (base + k * 64 + lane < n && (flt.lds_bins ? keep_lds(flt, ftab, key[k]) : flt.keep(key[k])))
                        ? 1u << k : 0u;
    }
    // slot k of this lane holds an item to sort
    auto kept = [&](int k) -> bool {
        if constexpr (FILT) return (keep >> k) & 1u;
        else return base + k * 64 + lane < n;
    };
    // Stable ranks: slot k of every lane in order, a wave's lanes matched by
    // digit (ballots), the wave's running count per digit in LDS.  (A second,
    // independent counting chain over half the slots was measured: the per-bin
    // sort unchanged, this pass slower.)
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const bool valid = kept(k);
        const uint32_t d = (key[k] >> shift) & mask;
        const uint64_t peers = match_digit<BITS>(d, valid);
        const uint32_t below = mbcnt(peers);
        const uint32_t old = wh[wave][d];
        pos[k] = old + below;
        if (valid && below == 0) wh[wave][d] = old + (uint32_t)__popcll(peers);
    }
    block_lds_sync();
    uint32_t c = 0;
    if (tid < ND) {
#pragma unroll
        for (int w = 0; w < kRsWaves; ++w) {
            const uint32_t x = wh[w][tid];
            wh[w][tid] = c;
            c += x;
        }
    }
    uint32_t tot;
    const uint32_t ex = block512_exclusive_scan(tid < ND ? c : 0u, tmp, &tot);
    if (tid < ND) blk_start[tid] = ex;
    block_lds_sync();
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        if (kept(k)) {
            const uint32_t d = (key[k] >> shift) & mask;
            pos[k] += blk_start[d] + wh[wave][d];
        }
    }
    const uint32_t t0 = tile * TILE;
    const uint32_t cnt = FILT ? tot : (n - t0 < TILE ? n - t0 : TILE);  // (the tile's kept items)
    // keys: stage in tile-local sorted order, write out; each slot's global
    // destination (from its staged key's digit) stays in registers for the
    // value arrays
    uint2* const stage2 = reinterpret_cast<uint2*>(stage);
#pragma unroll
    for (int k = 0; k < IPT; ++k)
        if (kept(k)) {
            const uint32_t sk = FILT ? key[k] & flt.kmask : key[k];
            if constexpr (kPair) stage2[pos[k]] = make_uint2(sk, io.vin[0] ? val[0][k] : base + k * 64 + lane);
            else stage[pos[k]] = sk;
        }
    block_lds_sync();
    uint32_t gdst[IPT];
#pragma unroll
    for (int k = 0; k < IPT; ++k) {
        const uint32_t j = tid + k * kRsThreads;
        if (j < cnt) {
            uint32_t key, v = 0u;
            if constexpr (kPair) {
                const uint2 kv = stage2[j];
                key = kv.x;
                v = kv.y;
            } else {
                key = stage[j];
            }
            const uint32_t d = (key >> shift) & mask;
            const uint32_t g = gbase[d] + (j - blk_start[d]);
            gdst[k] = g;
            io.kout[g] = key;
            if constexpr (kPair) io.vout[0][g] = v;
#ifdef GS_RS_ABL_NORANGES  // ablation (timing only): no run ends
            if (false) {
#else
            if (ranges) {
#endif
                // run ends of this key inside the tile (the tile's output is a
                // contiguous, fully sorted slice of the final order per digit)
                const uint32_t rk = key & rmask;
                const uint32_t kprev = j == 0 ? 0u : (kPair ? stage2[j - 1].x : stage[j - 1]);
                const uint32_t knext = j + 1 == cnt ? 0u : (kPair ? stage2[j + 1].x : stage[j + 1]);
                const bool s0 = j == 0 || (kprev & rmask) != rk;
                const bool s1 = j + 1 == cnt || (knext & rmask) != rk;
                if (s0 || s1) {
                    const uint32_t lo = key & lm;
                    const uint32_t fl = rskip ? rflag[d] : 0u;
                    if (s0 && !(lo == lo_first && (fl & 1u))) atomicMin(&ranges[rk].x, g);
                    if (s1 && !(lo == lo_last && (fl & 2u))) atomicMin(&ranges[rk].y, ~(g + 1u));
                }
            }
        }
    }
    // values: same permutation (already written with the keys when staged as pairs)
#pragma unroll
    for (int a = 0; a < (kPair ? 0 : NV); ++a) {
        block_lds_sync();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t idx = base + k * 64 + lane;
            if (kept(k)) stage[pos[k]] = (NV == 1 || io.vin[a]) ? val[a][k] : idx;
        }
        block_lds_sync();
#pragma unroll
        for (int k = 0; k < IPT; ++k) {
            const uint32_t j = tid + k * kRsThreads;
            if (j < cnt) io.vout[a][gdst[k]] = stage[j];
        }
    }
    if constexpr (!STRIDE) break;
    __syncthreads();  // (the next tile reuses the LDS arrays)
    }
}

SortPlan make_sort_plan(int bits, bool narrow_first) {
    SortPlan p{};
    if (bits <= 0) return p;
    p.passes = (bits + 7) / 8;
    // balanced digit widths, the wider first (13 -> 7+6, 15 -> 8+7) or, with
    // narrow_first, the narrower (15 -> 7+8).  Measured: the one-array bin
    // sort is faster wide-first (1080p 128 vs 135 us), the three-array depth
    // sort narrow-first (6M splats 145 vs 132 us): its low 8-bit digits split
    // a 4096-item tile into 256 runs of ~16 items, partial lines per array.
    int left = bits;
    for (int i = 0; i < p.passes; ++i) {
        const int w = narrow_first ? left / (p.passes - i) : (left + (p.passes - i) - 1) / (p.passes - i);
        p.shift[i] = bits - left;
        p.width[i] = w;
        p.mask[i] = (1u << w) - 1u;
        left -= w;
    }
    return p;
}

uint32_t radix_sort_tile_items() { return tile_items(1); }

size_t radix_sort_scratch_words(uint32_t n) {
    const uint32_t t = tile_items(1) < tile_items(3) ? tile_items(1) : tile_items(3);  // the smaller tile bounds both
    const size_t tiles = (n + t - 1) / t;
    return (size_t)(tiles ? tiles : 1) * kSortBins + kSortBins;
}

// rts_pass_kernel for a digit width (the ballot match unrolled per width);
// STRIDE: `tiles` workgroups loop over all the tiles
template <int NV, bool FILT, bool STRIDE = false, typename... A>
static hipError_t launch_pass(int width, uint32_t tiles, hipStream_t st, size_t lds, A... args) {
    switch (width) {
    case 1: rts_pass_kernel<NV, 1, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 2: rts_pass_kernel<NV, 2, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 3: rts_pass_kernel<NV, 3, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 4: rts_pass_kernel<NV, 4, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 5: rts_pass_kernel<NV, 5, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 6: rts_pass_kernel<NV, 6, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 7: rts_pass_kernel<NV, 7, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    case 8: rts_pass_kernel<NV, 8, FILT, STRIDE><<<tiles, kRsThreads, lds, st>>>(args...); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int NV>
static hipError_t radix_sort_impl(const uint32_t* keys_in, const uint32_t* const* vals_in, uint32_t* keys,
                                  uint32_t* const* vals, uint32_t* tmp_keys, uint32_t* const* tmp_vals, uint32_t n,
                                  int bits, uint32_t* scratch, bool* result_in_tmp, uint2* ranges, hipStream_t st,
                                  const uint32_t* n_dev, bool first_counted, const SortFilter& flt = SortFilter{}) {
    // (first_counted with a filter: the producer counted only the kept items,
    // PassCounts::cut; not with the strided fallback grids)
    if (flt.cut && (NV != 1 || !flt.kept || (first_counted && flt.stride_grid))) return hipErrorInvalidValue;
    if (flt.lds_bins > kDupCutBins || (flt.lds_bins && flt.flag)) return hipErrorInvalidValue;
    const size_t flds = flt.lds_bins ? ((size_t)flt.lds_bins * 2 + 15) & ~(size_t)15 : 0;  // (dynamic LDS of the filtered kernels)
    *result_in_tmp = false;
    const SortPlan plan = make_sort_plan(bits, NV > 1);
    if (n == 0 || plan.passes == 0) return hipSuccess;
    const uint32_t tiles = (n + tile_items(NV) - 1) / tile_items(NV);
    uint32_t* C = scratch;                                   // [digit][tile]
    uint32_t* totals = scratch + (size_t)tiles * kSortBins;  // [digit]
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
        uint2* const rg = p + 1 == plan.passes ? ranges : nullptr;
        const uint32_t rmask = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
        // (the filter drops items in pass 0; the later passes sort what it kept)
        const bool filt = p == 0 && flt.cut != nullptr;
        hipError_t e = hipSuccess;
        if constexpr (NV == 1) {
            if (flt.cut && flt.stride_grid) {  // (every pass on a fixed grid looping over the tiles)
                const uint32_t g = tiles < flt.stride_grid ? tiles : flt.stride_grid;
                if (filt)
                    rts_count_kernel<NV, true, true><<<g, kRsThreads, flds, st>>>(io.kin, n, plan.shift[p], plan.mask[p], C,
                                                                             tiles, n_dev, flt);
                else
                    rts_count_kernel<NV, false, true><<<g, kRsThreads, 0, st>>>(io.kin, n, plan.shift[p], plan.mask[p],
                                                                              C, tiles, n_dev, SortFilter{});
                rts_scan_kernel<<<plan.mask[p] + 1, kRsScanThreads, 0, st>>>(C, tiles, totals, n_dev);
                e = filt ? launch_pass<NV, true, true>(plan.width[p], g, st, flds, io, n, plan.shift[p], plan.mask[p], C,
                                                       totals, tiles, rg, rmask, n_dev, flt)
                         : launch_pass<NV, false, true>(plan.width[p], g, st, 0, io, n, plan.shift[p], plan.mask[p], C,
                                                        totals, tiles, rg, rmask, n_dev, SortFilter{});
                if (e != hipSuccess) return e;
                if (filt) n_dev = flt.kept;
                io.kin = io.kout;
                for (int a = 0; a < NV; ++a) io.vin[a] = io.vout[a];
                to_final = !to_final;
                continue;
            }
            if (filt) {
                if (!first_counted)
                    rts_count_kernel<NV, true><<<tiles, kRsThreads, flds, st>>>(io.kin, n, plan.shift[p], plan.mask[p], C,
                                                                            tiles, n_dev, flt);
                rts_scan_kernel<<<plan.mask[p] + 1, kRsScanThreads, 0, st>>>(C, tiles, totals, n_dev);
                e = launch_pass<NV, true>(plan.width[p], tiles, st, flds, io, n, plan.shift[p], plan.mask[p], C, totals,
                                          tiles, rg, rmask, n_dev, flt);
            }
        }
        if (!filt) {
            if (p > 0 || !first_counted)  // (pass 0's counts may come from the producer)
                rts_count_kernel<NV, false><<<tiles, kRsThreads, 0, st>>>(io.kin, n, plan.shift[p], plan.mask[p], C,
                                                                         tiles, n_dev, SortFilter{});
            rts_scan_kernel<<<plan.mask[p] + 1, kRsScanThreads, 0, st>>>(C, tiles, totals, n_dev);
            e = launch_pass<NV, false>(plan.width[p], tiles, st, 0, io, n, plan.shift[p], plan.mask[p], C, totals,
                                       tiles, rg, rmask, n_dev, SortFilter{});
        }
        if (e != hipSuccess) return e;
        if (filt) n_dev = flt.kept;
        io.kin = io.kout;
        for (int a = 0; a < NV; ++a) io.vin[a] = io.vout[a];
        to_final = !to_final;
    }
    return hipGetLastError();
}

hipError_t launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys, uint32_t* vals,
                             uint32_t* tmp_keys, uint32_t* tmp_vals, uint32_t n, int bits, uint32_t* scratch,
                             bool* result_in_tmp, hipStream_t st, uint2* ranges, const uint32_t* n_dev,
                             bool first_counted, const SortFilter& flt) {
    const uint32_t* vi[1] = {vals_in};
    uint32_t* vo[1] = {vals};
    uint32_t* vt[1] = {tmp_vals};
    return radix_sort_impl<1>(keys_in, vi, keys, vo, tmp_keys, vt, n, bits, scratch, result_in_tmp, ranges, st,
                              n_dev, first_counted, flt);
}

hipError_t launch_radix_sort3(const uint32_t* keys_in, const uint32_t* const* vals_in, uint32_t* keys,
                              uint32_t* const* vals, uint32_t* tmp_keys, uint32_t* const* tmp_vals, uint32_t n,
                              int bits, uint32_t* scratch, bool* result_in_tmp, hipStream_t st) {
    return radix_sort_impl<3>(keys_in, vals_in, keys, vals, tmp_keys, tmp_vals, n, bits, scratch, result_in_tmp,
                              nullptr, st, nullptr, false);
}

}  // namespace gs
