// gs_kernels.h — host-side launchers of the HIP kernels (one translation unit
// per stage).  All launches are asynchronous on the given stream.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_device.h"

namespace gs {

// ---- preprocess.hip ------------------------------------------------------
// Writes the 48-B record (visible splats), the 15-bit depth key and the packed
// pixel rect (empty rect for culled splats).
// t0/t1: optional events recorded by the kernel's own dispatch (timing
// without extra packets).
// zero8 (optional): two 64-bit words the kernel clears (the frame's
// composite fetch counter and open tile count, CompositeArgs::fetched /
// open_tiles), so no memset dispatch is needed.
// Bin-first single-GPU frames: the preprocess also does the
// reduce half of the scan.  Every workgroup adds its splats' pair counts and
// visible count into part[b] / part[nb + b] of its scan block b (kScanItems
// splats; integer atomics, so the sums are exact), and into part[2 nb + b]
// the sum over its waves of the largest per-splat pair count (the
// duplicate's wave-serial emission work in index order, for the binning-order
// model: gs_handle OrderModel::wmax), and the grid fills the
// frame's empty bin ranges and zeroes the first sort pass's digit counts
// (what scan_reduce_kernel does otherwise).  part (3 nb words) starts at zero
// and is consumed and cleared again by launch_scan_partials_fused, which
// reports the wave-max sum in total[4].
struct PreFuse {
    unsigned long long* part = nullptr;  // null: off
    uint32_t nb = 0;                     // scan blocks
    uint2* fill = nullptr;
    uint32_t nfill = 0;
    uint32_t* zero = nullptr;
    uint32_t nzero = 0;
    unsigned long long* zero64 = nullptr;  // (look-back statuses, launch_scan_duplicate np_out)
    uint32_t nzero64 = 0;
};
// Row-scheme projections (gs_shard_project): the preprocess also writes each
// splat's destination mask (the ranks owning a bin row its rect touches) and
// adds each block's per-destination counts into counts[d * nblocks + b]
// (kShardItems splats per block; counts zeroed first): what
// launch_shard_count does otherwise.
struct ShardFuse {
    const uint8_t* owner = nullptr;  // null: off
    int world = 0;
    uint32_t* dest_mask = nullptr;
    uint32_t* counts = nullptr;
    uint32_t nblocks = 0;
};
hipError_t launch_preprocess(const SceneDev& s, int sh_degree, const FrameUniforms& U, float4* rec,
                             uint32_t* dkey, uint32_t* rect_lo, uint32_t* rect_hi, hipStream_t st,
                             hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr,
                             unsigned long long* zero8 = nullptr, const PreFuse& fuse = PreFuse{},
                             const ShardFuse& shard = ShardFuse{});

// ---- scan.hip --------------------------------------------------------------
constexpr int kScanItems = 4096;  // per block
// Per-block sums of rect_tile_count(rect_lo[i], rect_hi[i], own) and their
// exclusive scan into partials (2 * ceil(n / kScanItems) u64); total[0] = P,
// total[1] = items with a nonzero count, total[2..3] = the per-bin depth sort
// sample (seg_sample, 2 words, may be null; reset), see launch_bin_depth_sort.
// total may be host-mapped (the host reads it after a stream sync, no copy).
// ranges[0..nranges) are set to the empty range (~0, ~0) on the way.
// npairs (device u32) = P when P <= cap (the pair buffers' capacity), else 0:
// the kernels after it read the pair count from there, so they can be queued
// before the host has seen P (an overflowing frame makes them no-ops and the
// host re-queues them with larger buffers).  Then launch_scan_duplicate.
// zero[0..nzero) is cleared on the way (the first sort pass's digit counts,
// PassCounts).
hipError_t launch_tile_count_totals(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, RowOwnership own,
                                    bool masked, uint64_t* partials, uint64_t* total, uint32_t* seg_sample,
                                    uint2* ranges, uint32_t nranges, uint32_t* npairs, uint64_t cap,
                                    uint32_t* zero, uint32_t nzero, hipStream_t st, hipEvent_t done = nullptr,
                                    unsigned long long seq = 0);
// (done: recorded by the totals kernel's own dispatch packet, not a separate
// marker packet, which would leave a ~6 us bubble in the stream.)
// The scan half alone, after a preprocess with PreFuse: the block sums in
// part (2 x nb words: pairs, visible splats) are scanned into partials (as
// launch_tile_count_totals leaves them) and part is cleared for the next
// frame.
// front (a depth-cut frame's front-only emission, launch_front_count): the
// offsets are scanned from the front pairs' block sums (part row 3, nb words
// after the three atomic rows), total[0] = the front pairs; total[8] = every
// pair of the frame (row 0) either way, and npairs is 0 when the pair buffers
// cannot hold them all (the fallback lists may need them).
// lookback (front-only or not): no offsets; partials[0..nb] (nb + 1 words) are
// cleared for the duplicate's look-back, total[0] = 0 and npairs = 1 (the
// duplicate stores the front pairs' count there), or 0 as above.  partials
// and npairs may then be null (the totals alone, on a stream of their own
// beside the duplicate: the preprocess cleared the statuses, PreFuse::zero64;
// seg_sample null too: total[2..3] = 0, no sample).
hipError_t launch_scan_partials_fused(unsigned long long* part, uint32_t nb, uint64_t* partials, uint64_t* total,
                                      uint32_t* seg_sample, uint32_t* npairs, uint64_t cap, hipStream_t st,
                                      hipEvent_t done = nullptr, unsigned long long seq = 0, bool front = false,
                                      bool lookback = false);
// Front-only emission of a depth-cut frame (index order, every
// bin row owned): per 4096-splat block, the pairs the front duplicate emits
// (launch_scan_duplicate front): a splat whose rect lies within 4x4 bins
// emits the bins with dkey <= cut[bin]; a larger one every bin (marked behind
// its cut, kBehindFlag, as kDupMark frames mark every pair).  out[b] = the
// block's sum (plain stores; nbins <= kDupCutBins, the table staged in LDS).
hipError_t launch_front_count(const uint32_t* rect_lo, const uint32_t* rect_hi, const uint32_t* dkey, uint32_t n,
                              bool masked, uint32_t tiles_x, const uint32_t* cut, uint32_t nbins,
                              unsigned long long* out, hipStream_t st);
// The fallback lists' pairs of a front-only frame (which never wrote the
// pairs behind the cuts): with *open != 0, every (splat, bin) pair with
// dkey > table[bin] (the open bins' cuts, ~0 elsewhere), in index order,
// key = dkey << bin_bits | bin, into keys/vals; *npairs = *kept = their
// number (<= cap).  part (2 * nblocks words) and total (>= 9 words): scratch.
// Nothing runs while *open == 0 (npairs keeps cut_finalize's 0).
hipError_t launch_fallback_pairs(const uint32_t* rect_lo, const uint32_t* rect_hi, const uint32_t* dkey, uint32_t n,
                                 bool masked, uint32_t tiles_x, int bin_bits, const uint32_t* table, uint32_t nbins,
                                 const unsigned long long* open, uint64_t* part, uint64_t* total, uint32_t* npairs,
                                 uint32_t* kept, uint64_t cap, uint32_t* keys, uint32_t* vals, hipStream_t st);
// (seq > 0: after total[0..4] the totals kernel stores seq into total[5] with
// a system-scope release, for a host that polls host-mapped `total` instead
// of waiting for `done`.)
// The first LSD pass's digit counts of the pairs, C[digit][tile] with
// `ntiles` columns, tiles of `tile` pairs, digit = bin & mask: the index-order
// duplicate adds them up as it writes (C zeroed before), so the sort skips
// that pass's count kernel (launch_radix_sort first_counted).  C null: off.
struct PassCounts {
    uint32_t* C = nullptr;
    uint32_t tile = 0, mask = 0, ntiles = 0;
    // (depth-cut frames) count only the pairs the sort's filtered first pass
    // keeps, dkey <= cut[bin] (SortFilter::keep), so that pass needs no count
    // kernel of its own (launch_radix_sort first_counted with the filter)
    const uint32_t* cut = nullptr;
};
constexpr uint32_t kDupCountTiles = 8;  // sort tiles a duplicate block counts in LDS (the rest: global atomics)
// Down-sweep fused with the duplicate: for j < n, item j (splat order[j], or j
// when order is null) with rect (rect_lo[j], rect_hi[j]) emits (bin, splat)
// for each bin of its rect whose row this rank owns, minus the excluded bins,
// at its pair offset.  dkey (may be null): key = dkey[j] << bin_bits | bin,
// the depth key riding above the bin id (index order: for the per-bin sort;
// depth order, dkey in that order: for a depth-cut frame's sort filter).
// Index order runs one fused kernel; depth order (order set) a down-sweep
// into offsets (n words of scratch) and a one-splat-per-lane duplicate.
// Nothing is written when *npairs == 0 (see launch_tile_count_totals).
// fcut (optional; index order, every bin row owned, nbins <= kDupCutBins,
// bin_bits + kDepthBits <= 31): the depth-cut frame's cut table.  Each block
// stages it in LDS and sets bit 31 (kBehindFlag) of every pair key behind its
// bin's cut, so the sort's filtered first pass tests one bit (SortFilter::flag)
// instead of gathering cut[bin] per pair.
constexpr uint32_t kDupCutBins = 16384;
constexpr uint32_t kBehindFlag = 0x80000000u;
// front (with fcut): only the pairs launch_front_count counted, at offsets
// scanned from its sums (launch_scan_partials_fused front).  np_out (with
// front): each block counts its own front pairs and finds its offset by a
// decoupled look-back over partials (nb + 1 words cleared by
// launch_scan_partials_fused lookback; launch_front_count is not needed); the
// front pairs' count goes to *np_out; pairs past cap are never written.
hipError_t launch_scan_duplicate(const uint32_t* order, const uint32_t* rect_lo, const uint32_t* rect_hi,
                                 const uint64_t* partials, uint32_t n, uint32_t tiles_x, RowOwnership own, bool masked,
                                 const uint32_t* dkey, int bin_bits, uint32_t* keys, uint32_t* vals,
                                 const uint32_t* npairs, hipStream_t st,
                                 uint32_t* offsets = nullptr, PassCounts pc = PassCounts{},
                                 const uint32_t* fcut = nullptr, uint32_t nbins = 0, bool front = false,
                                 uint32_t* np_out = nullptr, uint32_t cap = 0);

// ---- bin_depth_sort.hip ------------------------------------------------------
// Per bin b with list [start, end) = decode_range(ranges[b]) of (key, val)
// pairs, key = dkey << bin_bits | b: stable sort of the list by dkey
// (ties keep list order).  vals are permuted in place; keys of lists longer
// than kSegLdsMax are permuted too (they go through tmp_keys / tmp_vals, at
// the same offsets), shorter ones keep their keys unsorted.  Afterwards each
// bin's vals are in (dkey, list position) order.
// sample (2 words, zeroed by the next scan): [0] += pairs of the lists longer
// than kSegLdsMax (sorted through global memory, ~3x the cost per pair),
// [1] |= kSegSampleValid once the sort ran.
#ifndef GS_SEG_NT  // A/B knobs (tools/build_variant.py): the per-bin sort's common size class
#define GS_SEG_NT 512
#endif
#ifndef GS_SEG_IPT
#define GS_SEG_IPT 16
#endif
constexpr uint32_t kSegLdsMax = GS_SEG_NT * GS_SEG_IPT;  // lists sorted inside one workgroup (bin_depth_sort.hip)
#ifndef GS_SEG_CLASSES  // 1: frames of >= GS_SEG_CLASS_MIN_BINS bins sort short lists (<= kSegSmallMax) in a launch of narrower workgroups
#define GS_SEG_CLASSES 1
#endif
#ifndef GS_SEG_CLASS_MIN_BINS
#define GS_SEG_CLASS_MIN_BINS 4096
#endif
#ifndef GS_SEG_SHORT  // A/B knob: 1 = frames of fewer bins whose lists are front lists (short_lists) sort in 256-lane workgroups
#define GS_SEG_SHORT 1
#endif
#ifndef GS_SEG_SMALL_NT
#define GS_SEG_SMALL_NT 256
#endif
#ifndef GS_SEG_SMALL_IPT
#define GS_SEG_SMALL_IPT 16
#endif
constexpr uint32_t kSegSmallMax = GS_SEG_SMALL_NT * GS_SEG_SMALL_IPT;
constexpr uint32_t kSegSampleValid = 0x80000000u;
// guard (optional): nothing is done while *guard == 0 (the fallback lists).
hipError_t launch_bin_depth_sort(const uint2* ranges, uint32_t nbins, uint32_t* keys, uint32_t* vals,
                                 uint32_t* tmp_keys, uint32_t* tmp_vals, int bin_bits, uint32_t* sample,
                                 hipStream_t st, hipEvent_t done = nullptr,
                                 const unsigned long long* guard = nullptr, bool short_lists = false);

// ---- radix_sort.hip --------------------------------------------------------
constexpr int kSortBins = 256;   // 8-bit digits
constexpr int kMaxSortPasses = 4;
struct SortPlan {
    int passes;
    int shift[kMaxSortPasses];
    int width[kMaxSortPasses];
    uint32_t mask[kMaxSortPasses];
};
SortPlan make_sort_plan(int bits, bool narrow_first = false);  // narrow_first: the depth sort (radix_sort.hip)
// Scratch words (uint32) needed by launch_radix_sort for n items.
size_t radix_sort_scratch_words(uint32_t n);
// Items per tile of launch_radix_sort (its C matrix has ceil(n / tile) columns
// at the start of the scratch).
uint32_t radix_sort_tile_items();
// Stable LSD sort on key bits [0, bits).  Reads (keys_in, vals_in) — vals_in
// may be null (value = index) — and leaves the result in (keys, vals), or in
// (tmp_keys, tmp_vals) when *result_in_tmp (only if the inputs alias the
// outputs and the pass count is odd).
// ranges (optional): key-value extents of the sorted output, stored as
// {start, ~end} (fill with 0xFF before; empty key = {~0, ~0}); see
// decode_range.
// n_dev (optional): the item count is read on the device from *n_dev (<= n;
// n sizes the grids and the scratch), so the sort can be queued before the
// host knows it.
// Filter (the bin sorts of a depth-cut frame): only items whose
// depth key (key >> dshift) lies at or ahead of their bin's cut (<=
// cut[key & bmask]; behind it, > cut[...], with `behind`: the fallback lists)
// are counted and sorted; the first pass drops the others and stores the
// number kept in *kept (the later passes read it, as n_dev); the result holds
// the kept items.
struct SortFilter {
    const uint32_t* cut = nullptr;  // null: every item
    uint32_t bmask = 0;
    int dshift = 0;
    uint32_t* kept = nullptr;
    uint32_t behind = 0;
    uint32_t stride_grid = 0;  // > 0: every pass on at most this many workgroups, looping over the tiles
    // flag: the duplicate marked the pairs behind their cut (kBehindFlag), the
    // front lists keep the unmarked ones (cut is then only the "filter on"
    // sign); kmask: the key bits below the flag (the depth test of a marked
    // frame's fallback lists; the pass stores kept keys masked with it)
    uint32_t flag = 0;
    uint32_t kmask = ~0u;
    // lds_bins > 0 (<= kDupCutBins): the count and pass kernels copy the cut
    // table into LDS as 16-bit words first and test against that copy (the
    // fallback lists' filter: a few open bins, every pair of the frame tested)
    uint32_t lds_bins = 0;
    __device__ __forceinline__ bool keep(uint32_t key) const {
        if (flag) return (key & kBehindFlag) == 0u;
        return (((key & kmask) >> dshift) <= cut[key & bmask]) != (behind != 0u);
    }
};
hipError_t launch_radix_sort(const uint32_t* keys_in, const uint32_t* vals_in, uint32_t* keys, uint32_t* vals,
                             uint32_t* tmp_keys, uint32_t* tmp_vals, uint32_t n, int bits, uint32_t* scratch,
                             bool* result_in_tmp, hipStream_t st, uint2* ranges = nullptr,
                             const uint32_t* n_dev = nullptr, bool first_counted = false,
                             const SortFilter& flt = SortFilter{});
// Same with three value arrays (vals_in[0] may be null: value = index).
hipError_t launch_radix_sort3(const uint32_t* keys_in, const uint32_t* const* vals_in, uint32_t* keys,
                              uint32_t* const* vals, uint32_t* tmp_keys, uint32_t* const* tmp_vals, uint32_t n,
                              int bits, uint32_t* scratch, bool* result_in_tmp, hipStream_t st);

// ---- composite.hip ---------------------------------------------------------
struct CompositeArgs {
    const uint32_t* vals;   // sorted splat ids (index into rec)
    const uint2* ranges;    // [bins] -> [start, end) into vals
    const float4* rec;      // records, rec_stride float4 apart (3 local, 4 exchange)
    const uint32_t* dkey;   // depth keys parallel to rec (MLAB reads half(zF) from them)
    int rec_stride;
    int width, height, tiles_x, tiles_y;  // frame and 32x32 bin grid
    const uint16_t* rows;   // owned bin rows, ascending (nullptr: every row)
    int nrows;              // number of owned bin rows
    int compact;            // 1: write the owned bin rows stacked (band buffer)
    int cell_mask;          // 1: record rect words carry the cell-exclusion mask (FrameUniforms)
    float4* out;            // fp32 RGBA, or (when out_bgra8 is set) unused
    uint32_t* out_bgra8;    // packed BGRA8Unorm (metal_renderer.mm:58), converted in-kernel
    // per-pixel fragment cap (0 = none): thr[py * width + px] = splat id of the
    // cap-th covering fragment in index (arrival) order, UINT32_MAX if fewer
    int cap;
    const uint32_t* thr;    // read by the capped composite
    uint32_t* thr_out;      // written by launch_cap_threshold
    // Depth-slab multi-GPU.  slab 1: transmittance pass,
    // t_out[pixel] = the slab's own transmittance (1 - A for the tile rule).
    // slab 2: colour pass starting from the ordered product of the earlier
    // slabs' transmittance, t_all[j * W * H + pixel] for j < slab_rank;
    // writes (C, delta A) contributions that sum over slabs to the frame.
    int slab;
    int slab_rank;
    float* t_out;
    const float* t_all;
    // optional: += the records the workgroups fetched (staged batches and the
    // prefetched one; each of a bin's four tiles fetches its list itself),
    // the early-out-aware basis of the composite's algorithmic bytes
    unsigned long long* fetched;
    // Depth-cut frames (gs_options.depth_split; modes 0/1, no cap, DESIGN.md
    // §4), per 8x8 quadrant (wave), with plain stores to its own words of its
    // bin's 128-B record qrec[bin * kQrecWords ...] (no workgroup barrier, no
    // contended atomic, and a cache line written only by the bin's four tiles,
    // which run on one XCD).  pass 1, the front lists: every quadrant q (tile
    // of the bin * 4 + wave) writes its cut position to word q (the end of the
    // last batch it walked with an open pixel, ~0 while one stays open;
    // launch_cut_finalize turns them into the next cuts) and its open flag to
    // word 16 + q: 1 if a pixel stays open at the end of a list that was cut
    // (cut_in[bin] < kDepthInf); an open quadrant writes its pixels' state
    // (C, T) into `state` and adds one to open_q_count.  pass 2: the open
    // quadrants only, resumed from their state with the fallback lists.
    int pass;
    uint32_t* qrec;
    unsigned long long* open_q_count;
    float4* state;
    const uint32_t* cut_in;   // may be null: no list was cut
    // Dispatch order of the bins (tile / live50 strip composite, single-GPU
    // frames; null: row-major): order[p] is the bin of the p-th pair of
    // workgroups, a permutation of [0, tiles_x * tiles_y) written by
    // launch_order_bins from an earlier frame's quadrant records, costliest
    // bins first, so the launch's last workgroups are short ones.  Which
    // workgroup renders which bin does not change any pixel.
    const uint32_t* order;
    // (optional, strip composite pass 1) wcost[2 bin + half] = the records the
    // bin's top / bottom half workgroup fetched: launch_order_bins' costs
    uint32_t* wcost;
};
// One 256-lane workgroup per owned 16x16 tile.  mode 0 = tile rule (A >= 0.99
// break), 1 = live50 rule (T < 0.01 break), 2 = MLAB k-buffer (a.vals
// index-ordered, a.dkey set, no cap); with a.cap > 0 only fragments with
// id <= thr[pixel] are composited.
hipError_t launch_composite(const CompositeArgs& a, int mode, hipStream_t st, hipEvent_t t0 = nullptr,
                            hipEvent_t t1 = nullptr);
// Tile and live-50 frames of more than kStripMinBins composited bins run the
// strip kernel (two 16x16 tiles per workgroup, two pixels per lane, the
// longest-first bin order: CompositeArgs::order / wcost); fewer bins (a rank's
// band at 8 ranks, small frames) run one workgroup per tile: with less than a
// round of workgroups the slowest one bounds the launch, and a tile walks its
// bin's list one pixel per lane.  Same pixels either way.
#ifndef GS_STRIP_MIN_BINS  // A/B knob
#define GS_STRIP_MIN_BINS 512
#endif
constexpr uint32_t kStripMinBins = GS_STRIP_MIN_BINS;
bool composite_strip(uint32_t bins);
// Depth cuts: the next cut of every bin from the largest of its 16 quadrants'
// cut positions (CompositeArgs::qrec): ~0 -> 0xFFFF (every pair), 0 -> 0,
// else the depth key of the list record before it plus `margin`, at most
// 0xFFFF.  vals and dkey: the composited lists and depth keys.
// With fb.cut_in (the frame's lists were cut), the same kernel prepares the
// fallback lists' sort: fb.table[bin] = cut_in[bin] for a bin with an open
// quadrant (its pairs behind the cut are sorted again), else ~0 (none);
// *fb.n = *fb.npairs when a quadrant is open, else 0, and *fb.kept = 0 (so
// every fallback kernel returns at once when none is); the bin ranges are
// cleared for the fallback sort when one is open.  Bins in rows another
// rank owns (own.owner, rows of tiles_x bins) get cut 0 and no fallback:
// their quadrant records were never written by this rank's composite.
struct CutFallback {
    const uint32_t* cut_in = nullptr;  // null: no fallback (the lists were whole)
    const unsigned long long* open = nullptr;
    const uint32_t* npairs = nullptr;
    uint32_t* table = nullptr;
    uint32_t* n = nullptr;
    uint32_t* kept = nullptr;
    uint2* ranges = nullptr;
    // (optional) host-mapped word: the frame's open-quadrant count, written by
    // the kernel's first lane, read by the host's dilation controller later
    // without a sync (a stale value only delays its reaction)
    unsigned long long* host_open = nullptr;
};
hipError_t launch_cut_finalize(const uint32_t* qrec, const uint32_t* vals, const uint32_t* dkey, uint32_t* cut_out,
                               uint32_t nbins, uint32_t tiles_x, const RowOwnership& own, uint32_t margin,
                               hipStream_t st, const CutFallback& fb);
// Per-pixel cap thresholds from INDEX-ordered bin lists (a.vals / a.ranges):
// walks each pixel's covering fragments in arrival order and records the id
// of the a.cap-th one in a.thr_out (tile.metal:7,199-202; 50layer.metal:8,170).
hipError_t launch_cap_threshold(const CompositeArgs& a, hipStream_t st);
// Spatially dilated cuts (a moving camera): out[bin] = the
// largest cut over the bins within r rows / columns of it (clamped to the
// grid).  A deeper cut only moves pairs from the fallback lists into the front
// lists, so any r gives the same image.
hipError_t launch_cut_dilate(const uint32_t* cut, uint32_t* out, uint32_t tiles_x, uint32_t tiles_y, int r,
                             hipStream_t st);
// Longest-first bin order for the next composite on this buffer set (one
// workgroup): a bin's cost is the records its two half-bin workgroups
// fetched in the front lists' composite (CompositeArgs::wcost); order = the
// bins by cost, descending, in 128 log-spaced buckets (ties in any order).
// nbins <= kOrderMaxBins.
constexpr uint32_t kOrderMaxBins = 1u << 16;
hipError_t launch_order_bins(const uint32_t* wcost, uint32_t nbins, uint32_t* order, hipStream_t st);

// ---- shard.hip (multi-GPU tile-row ownership / depth slabs) ---------------
constexpr int kXRecFloat4 = 3;  // 48-B exchange record: the projection's record (its first 48 B)
constexpr int kXSideWords = 3;  // + binning rect lo, hi and depth key per record (gs_exchange_regions)
constexpr int kMaxWorld = 32;
constexpr int kSlabKeys = 1 << kDepthBits;  // 15-bit depth keys
constexpr int kSlabBinShift = 4;            // slab histogram: 2048 bins of 16 keys
constexpr int kSlabBins = kSlabKeys >> kSlabBinShift;
// Destination rule of a multi-GPU frame: bin-row owners (owner[by]) or, with
// slabs, depth-key slabs (rank d receives keys in [bounds[d], bounds[d+1])).
struct DestRule {
    const uint8_t* owner;
    const uint32_t* dkey;
    uint32_t bounds[kMaxWorld + 1];
    int slabs;
};
// dest_mask[i]: bit r set iff splat i goes to rank r (a bin row of its rect
// owned by r, or its depth key in r's slab).
// counts: [world][nblocks] per-block destination counts (kShardItems splats per block).
constexpr int kShardItems = 1024;
hipError_t launch_shard_count(const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n, int world,
                              const DestRule& rule, bool masked,
                              uint32_t* dest_mask, uint32_t* counts, uint32_t nblocks, hipStream_t st);
// hist[key >> kSlabBinShift] += (splat, bin) pairs of every visible splat
// (hist: kSlabBins u64, zeroed by the caller).
hipError_t launch_slab_histogram(const uint32_t* dkey, const uint32_t* rect_lo, const uint32_t* rect_hi, uint32_t n,
                                 bool masked, unsigned long long* hist, hipStream_t st);
// Exclusive scan of each destination row; dest_total[world].
hipError_t launch_rows_scan(uint32_t* counts, uint32_t nblocks, int rows, uint32_t* dest_total, hipStream_t st);
// Pack the exchange regions (records, then rect lo / hi and depth-key words
// of all T = sum(dest_total) records) grouped by destination, splat-index
// order inside.
hipError_t launch_shard_pack(const float4* rec, const uint32_t* rlo, const uint32_t* rhi, const uint32_t* dkey,
                             const uint32_t* dest_mask, uint32_t n, int world, const uint32_t* counts,
                             const uint32_t* dest_total, uint32_t nblocks, float4* send, hipStream_t st);
// dst[i] += src[i] for n4 float4s.
hipError_t launch_accumulate(float4* dst, const float4* src, size_t n4, hipStream_t st);
}  // namespace gs
