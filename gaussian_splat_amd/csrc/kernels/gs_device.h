// gs_device.h — device-side building blocks of the splat pipeline (gfx950).
//
// Arithmetic follows DESIGN.md §2 op for op (explicit __builtin_fmaf where
// the contract fuses, plain ops elsewhere; the whole library is compiled with
// -ffp-contract=off), so records and framebuffers agree bit for bit with the
// CPU oracle.  Reference lines are cited on each step.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// The kernels size their LDS for gfx950 (160 KB per CU, up to 160 KB per
// workgroup: order_bins_kernel and the duplicate's cut table use more than
// the 64 KB of earlier CDNA parts), so the device code builds for gfx950 only.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "libgsplat's kernels are written for gfx950 (MI355X): build with --offload-arch=gfx950"
#endif

namespace gs {

constexpr int kLdsBytes = 160 * 1024;     // LDS per CU (and per workgroup) on gfx950
constexpr int kTile = 16;                 // 16x16-pixel tiles (gaussian_splat_types.h:9 budget)
constexpr int kTileThreads = kTile * kTile;
// Binning granularity: 32x32-pixel bins of 2x2 tiles.  Splats are binned per
// bin (P/N ~2.3 instead of ~4.4 per 16x16 tile); the composite still works
// per 16x16 tile, the 4 tiles of a bin sharing one workgroup and one list.
constexpr int kBin = 32;
constexpr int kBinShift = 5;
constexpr int kBinThreads = 1024;
constexpr int kDepthBits = 15;            // positive half bit patterns are < 0x7C01
constexpr uint32_t kDepthInf = 0x7C00u;

constexpr float kQMax = 9.21034037197618f;  // 2 ln 100: exp(-q/2) >= 0.01 (tile.metal:193)
constexpr float kTMin = 0.01f;            // 50layer.metal:219
// Composite contract.  The conic is scaled by
// kConicScale = sqrt(log2(e)/2) when a record is staged for a tile, so that
// q' = u'^2 + v'^2 = q log2(e)/2 and the gaussian is 2^-q' with no scale op:
//   box test |u| <= 3 (the quad, tile.metal:142-156)  ->  |u'| <= kBoxS,
//   cutoff exp(-q/2) >= 0.01 (tile.metal:191-195)      ->  q' <= log2(100).
// The tile rule (tile.metal:251-266) tracks T = 1 - A: sa = a*T, C += rgb*sa,
// T -= sa, break once T <= kTSat (A >= 0.99, :261); alpha out = 1 - T.
constexpr float kConicScale = 0.8493217825889587f;
constexpr float kBoxS = 2.5479652881622314f;   // float(3 * sqrt(log2(e)/2))
constexpr float kQMaxS = 6.643856048583984f;   // float(log2(100))
constexpr float kTSat = 0.01f;

// Uniforms of one frame (tile.metal:16-21 plus derived values).
struct FrameUniforms {
    float V[16];      // view, column-major
    float P[16];      // projection
    float VP[16];     // P·V (instanced_splat_renderer.mm:453), host-computed
    float campos[4];  // eye position for SH view directions
    int32_t width, height;
    int32_t tiles_x, tiles_y;  // 32x32 bins (see kBin)
    int32_t cell_mask;         // 1: records carry the 8x8-cell exclusion mask (frames <= 4096 px)
    // pixel rows [band_y0, band_y1] the rects are clipped to: the frame
    // (0, height - 1), or one rank's band in the replicated-scene scheme
    // (gs_band_render), where splats outside it are culled before their colour
    int32_t band_y0, band_y1;
};

// Record rect words (record float4 #2 .zw).  With cell masks (frames up to
// kCellMaskDim px) each word is x (12 bits) | 4 mask bits | y (12 bits) | 4
// mask bits; the 16-bit mask marks the 8x8 pixel cells (global 8-px grid,
// first 4x4 cells of the rect, row-major) that the splat's q <= 2 ln 100
// ellipse provably misses.  A zero mask excludes nothing (always safe).
constexpr int kCellMaskDim = 4096;
__device__ __forceinline__ uint32_t rect_coords(uint32_t w, bool masked) { return masked ? w & 0x0FFF0FFFu : w; }
__device__ __forceinline__ uint32_t rect_cell_mask(uint32_t lo, uint32_t hi) {
    return ((lo >> 12) & 0xFu) | ((lo >> 28) << 4) | (((hi >> 12) & 0xFu) << 8) | ((hi >> 28) << 12);
}
__device__ __forceinline__ uint32_t rect_with_mask(uint32_t w, uint32_t m4lo, uint32_t m4hi) {
    return w | (m4lo << 12) | (m4hi << 28);
}

// A window [base, base + span) of a u32 array of n items, read through a raw
// buffer resource (uniform: scalar registers): one 32-bit offset per load
// instead of a 64-bit address, and reads past n return 0 (no clamping, so no
// load waits inside a branch).  Dword 3 of a gfx9 raw buffer descriptor.
struct BufU32 {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ BufU32(const uint32_t* p, uint32_t base, uint32_t n, uint32_t span)
        : r(__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(p) + base, (short)0,
                                              (int)((base < n ? min(n - base, span) : 0u) * 4u), 0x00020000)) {}
    __device__ __forceinline__ uint32_t operator[](uint32_t i) const {  // (i: within the window)
        return __builtin_amdgcn_raw_buffer_load_b32(r, (int)(i * 4u), 0, 0);
    }
};

// Scene SoA resident in HBM: coalesced 16-B loads per lane.
struct SceneDev {
    const float4* p0;   // x, y, z, opacity
    const float4* p1;   // qw, qx, qy, qz
    const float4* p2;   // sx, sy, sz, c0   (c = rgb for SH0, raw f_dc otherwise)
    const float2* p3;   // c1, c2
    const float4* sh4;  // [plane][n] coefficient planes, k-major (r,g,b interleaved)
    const float* sh1;   // [n] trailing coefficient (deg 1 and 3)
    uint32_t n;
};

// 48-byte record = 3 float4: (cx, cy, ax, ay) (bx, by, op, r) (g, b, rect_lo, rect_hi)
struct Record3 {
    float4 a, b, c;
};
// float4 slots per record in the frame's record array: 3, or 4 (64-B aligned
// slots, the 4th zero: a record then lies in one half of a 128-B line;
// A/B knob GS_REC_F4)
#ifndef GS_REC_F4
#define GS_REC_F4 3
#endif
constexpr int kRecFloat4 = GS_REC_F4;
static_assert(kRecFloat4 == 3 || kRecFloat4 == 4, "record slot");

__device__ __forceinline__ float xform_row(const float* m, int r, float x, float y, float z) {
    return __builtin_fmaf(m[8 + r], z, __builtin_fmaf(m[4 + r], y, __builtin_fmaf(m[0 + r], x, m[12 + r])));
}

__device__ __forceinline__ float dot3(float a0, float a1, float a2, float b0, float b1, float b2) {
    return __builtin_fmaf(a2, b2, __builtin_fmaf(a1, b1, a0 * b0));
}

// 2^t by rint + degree-6 fma chain + ldexp (oracle ora_exp2_poly, op for op).
__device__ __forceinline__ float gs_exp2_poly(float t) {
    float n = __builtin_rintf(t);
    float f = t - n;
    float p = 1.5403530393381606e-4f;
    p = __builtin_fmaf(p, f, 1.3333558146428443e-3f);
    p = __builtin_fmaf(p, f, 9.6181291076284772e-3f);
    p = __builtin_fmaf(p, f, 5.5504108664821580e-2f);
    p = __builtin_fmaf(p, f, 2.4022650695910071e-1f);
    p = __builtin_fmaf(p, f, 6.9314718055994531e-1f);
    p = __builtin_fmaf(p, f, 1.0f);
    return __builtin_ldexpf(p, (int)n);
}

// F1 gaussian on the scaled conic: exp(-q/2) = 2^-q' (oracle ora_gauss2, op
// for op): n = rint(-q'), f = -q' - n (exact), a degree-5 minimax polynomial
// of 2^f on [-1/2, 1/2] (relative error 1.7e-7 in f32), scaled by 2^n.
__device__ __forceinline__ float gs_gauss2(float qs) {
    const float t = -qs;
    const float n = __builtin_rintf(t);
    const float f = t - n;
    float p = 1.3267117319628596e-3f;
    p = __builtin_fmaf(p, f, 9.6715930849313736e-3f);
    p = __builtin_fmaf(p, f, 5.5507261306047440e-2f);
    p = __builtin_fmaf(p, f, 2.4022240936756134e-1f);
    p = __builtin_fmaf(p, f, 6.9314700365066528e-1f);
    p = __builtin_fmaf(p, f, 1.0f);
    return __builtin_ldexpf(p, (int)n);
}

// IEEE half bits, round to nearest even (v_cvt_f16_f32).
__device__ __forceinline__ uint32_t half_bits(float f) {
    _Float16 h = (_Float16)f;
    return (uint32_t)__builtin_bit_cast(unsigned short, h);
}

// Packed inclusive pixel rect: lo = x0 | y0 << 16, hi = x1 | y1 << 16.  A culled
// splat carries the empty rect (lo = 0xFFFFFFFF, hi = 0).
constexpr uint32_t kEmptyRectLo = 0xFFFFFFFFu;

// Bin ranges as written by the last bin-sort pass: {start, ~end}.
__device__ __forceinline__ uint2 decode_range(uint2 r) { return make_uint2(r.x, ~r.y); }

// Multi-GPU ownership: every 32-px bin row has one owning
// rank, owner[by].  The default table gives each rank a contiguous, balanced
// range of bin rows (few splats straddle a boundary, so the record exchange
// stays small); callers may install their own (gs_shard_set_rows).  A null
// table means a single GPU: the rank owns every row.
struct RowOwnership {
    const uint8_t* owner;
    uint32_t rank;
};

__device__ __forceinline__ bool owns_bin_row(uint32_t by, const RowOwnership& o) {
    return !o.owner || o.owner[by] == o.rank;
}

// Ranks owning any of the bin rows ty0..ty1 (the row scheme's destinations).
__device__ __forceinline__ uint32_t row_mask(uint32_t ty0, uint32_t ty1, const uint8_t* __restrict__ owner) {
    uint32_t m = 0;
    for (uint32_t by = ty0; by <= ty1; ++by) m |= 1u << owner[by];
    return m;
}

// Bin rect of a splat from its packed pixel rect words.  With `masked`
// (frames up to kCellMaskDim px, FrameUniforms::cell_mask) the words also
// carry a 16-bit bin-exclusion mask over the first 4x4 bins of the rect
// (same packing as the record's cell mask): bins the splat's ellipse
// provably misses, which get no (splat, bin) pair.
struct BinRect {
    uint32_t bx0, by0, bx1, by1;
    uint32_t excl;  // bit (by - by0) * 4 + (bx - bx0)
    bool empty;
};
__device__ __forceinline__ BinRect bin_rect(uint32_t lo, uint32_t hi, bool masked) {
    const uint32_t l = rect_coords(lo, masked), h = rect_coords(hi, masked);
    const uint32_t x0 = l & 0xFFFFu, x1 = h & 0xFFFFu;
    BinRect r;
    r.empty = x1 < x0;  // culled (the empty rect survives masking: x0 = 0xFFF > x1 = 0)
    r.bx0 = x0 >> kBinShift;
    r.bx1 = x1 >> kBinShift;
    r.by0 = (l >> 16) >> kBinShift;
    r.by1 = (h >> 16) >> kBinShift;
    r.excl = masked ? rect_cell_mask(lo, hi) : 0u;
    return r;
}
__device__ __forceinline__ bool bin_excluded(const BinRect& r, uint32_t by, uint32_t bx) {
    const uint32_t dy = by - r.by0, dx = bx - r.bx0;
    return dy < 4u && dx < 4u && ((r.excl >> (dy * 4u + dx)) & 1u);
}

// (splat, bin) pairs of the rect: owned bin rows, minus excluded bins.
__device__ __forceinline__ uint32_t rect_tile_count(uint32_t lo, uint32_t hi, const RowOwnership& o, bool masked) {
    const BinRect r = bin_rect(lo, hi, masked);
    if (r.empty) return 0u;
    const uint32_t cols = r.bx1 - r.bx0 + 1u;
    if (!o.owner && !r.excl) return (r.by1 - r.by0 + 1u) * cols;
    uint32_t n = 0;
    for (uint32_t by = r.by0; by <= r.by1; ++by) {
        if (o.owner && o.owner[by] != o.rank) continue;
        const uint32_t dy = by - r.by0;
        n += cols - (dy < 4u ? (uint32_t)__builtin_popcount((r.excl >> (dy * 4u)) & 0xFu) : 0u);
    }
    return n;
}

// Per-bin depth cuts (gs_options.depth_split).  A depth-cut
// frame's bin lists (the front lists) hold the pairs whose depth key lies at
// or ahead of their bin's cut in S1 order, dkey <= cut[bin]: every pair is
// emitted, and the bin sort's first pass drops the others (SortFilter).  The
// fallback lists for the quadrants those lists leave open are the same
// frame's pairs of the bins with an open quadrant behind the cut, picked by
// the first pass of their own bin sort.  S1 composites ascending dkey, so each
// bin's front list precedes all its other pairs.
constexpr uint32_t kQrecWords = 32;  // per bin: 16 quadrant cut positions, 16 open flags (CompositeArgs)

// The (bin, splat) pairs of one splat, from pair offset `off` on: one per bin
// of its rect in an owned bin row, minus the bins its ellipse provably misses
// (row-major bin order), for which keep(bin) holds.  key = key_hi | bin id.
// on_pair(offset, bin) is called for every pair written.
template <typename Keep, typename F>
__device__ __forceinline__ void emit_bin_pairs_if(const BinRect& r, uint32_t tiles_x, const RowOwnership& own,
                                                  uint32_t key_hi, uint32_t val, uint32_t off,
                                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals, Keep&& keep,
                                                  F&& on_pair) {
    for (uint32_t by = r.by0; by <= r.by1; ++by) {
        if (!owns_bin_row(by, own)) continue;
        for (uint32_t bx = r.bx0; bx <= r.bx1; ++bx) {
            if (bin_excluded(r, by, bx)) continue;  // the ellipse misses this bin
            const uint32_t bin = by * tiles_x + bx;
            if (!keep(bin)) continue;
            keys[off] = key_hi | bin;
            vals[off] = val;
            on_pair(off, bin);
            ++off;
        }
    }
}
__device__ __forceinline__ void emit_bin_pairs(const BinRect& r, uint32_t tiles_x, const RowOwnership& own,
                                               uint32_t key_hi, uint32_t val, uint32_t off,
                                               uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    emit_bin_pairs_if(r, tiles_x, own, key_hi, val, off, keys, vals, [](uint32_t) { return true; },
                      [](uint32_t, uint32_t) {});
}

// fp32 RGBA -> BGRA8Unorm texel: clamp to [0, 1], scale by 255, round to
// nearest even (the Metal/Vulkan unorm conversion rule; parity unpinned: no
// Metal runtime here), bytes B, G, R, A from low to high address.
__host__ __device__ inline uint32_t unorm8(float x) {
    x = x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f;  // NaN -> 0
    return (uint32_t)__builtin_rintf(x * 255.0f);
}
__host__ __device__ inline uint32_t pack_bgra8(float r, float g, float b, float a) {
    return unorm8(b) | (unorm8(g) << 8) | (unorm8(r) << 16) | (unorm8(a) << 24);
}

}  // namespace gs
