// gs_masks.h — the exclusion masks of a visible splat's rect,
// computed once, by the preprocess, from its record.  The row scheme's
// receiving ranks do not recompute them: the 8x8-cell mask travels in the
// exchanged 48-B record's rect words and the 32x32-bin mask in the exchanged
// binning rect lo / hi words (gs_exchange_regions).
#pragma once

#include "gs_device.h"

namespace gs {

// Cell-exclusion masks (gs_device.h): which cells of the rect's first 4x4
// the q <= 2 ln 100 ellipse provably misses.  In pixel offsets
// X = px + 0.5 - cx, Y = cy - (py + 0.5) the record gives u = X ax + Y ay,
// v = X bx + Y by, so q = aX^2 + 2bXY + cY^2 with a = ax^2 + bx^2,
// b = ax ay + bx by, c = ay^2 + by^2, det = ac - b^2.  For each row band of
// pixel centres [Ya, Yb] the ellipse's X extent is closed form: X(Y) =
// (-bY +- sqrt(Qa - det Y^2)) / a, extremal at the band ends or at the
// ellipse's own x-extreme points Y = -+b sqrt(Q/(c det)).  Q and the X range
// carry a margin, so a cell is excluded only when no pixel centre of it can
// be covered (the composite then skips a record that would add exact zeros).
// The ellipse terms are shared by the 8x8-cell and 32x32-bin masks; a band's
// X range becomes the row's candidate cells [ql, qh] in integers.
struct EllipseX {
    float b, ia, det, Qa, ymax, xs, ys, pad;
    bool ok;
};
__device__ __forceinline__ EllipseX ellipse_x(float ax, float ay, float bx, float by) {
    EllipseX e;
    const float a = ax * ax + bx * bx, c = ay * ay + by * by;
    e.b = ax * ay + bx * by;
    // det = ac - b^2 = (ax by - ay bx)^2: the record's axes are orthogonal, so
    // the cross product does not cancel (ac - b^2 would, for thin ellipses)
    const float cr = ax * by - ay * bx;
    e.det = cr * cr;
    e.ok = e.det > 0.0f && a > 0.0f && c > 0.0f && e.det < 3.0e38f;  // degenerate: no claim
    // hardware approximations (v_rcp_f32, v_sqrt_f32: ~1 ulp) are well inside
    // the 0.2 % margin on Q and the padding on X
    const float Q = kQMax * 1.002f + 1e-3f;
    e.Qa = Q * a;
    e.ia = __builtin_amdgcn_rcpf(a);
    const float idet = __builtin_amdgcn_rcpf(e.det);
    e.ymax = __builtin_amdgcn_sqrtf(e.Qa * idet);               // |Y| reach of the ellipse
    e.xs = __builtin_amdgcn_sqrtf(Q * c * idet);                // X of the x-extreme points
    e.ys = e.b * e.xs * __builtin_amdgcn_rcpf(c);               // max-X point at Y = -ys, min-X at +ys
    e.pad = 0.01f + 1e-3f * fabsf(e.xs);
    return e;
}
// The exclusion mask of the rect's first 4x4 cells of 1 << shift px (3: the
// composite's 8x8 cells, 5: 32x32 bins); 0 (no claim) for a rect of one cell
// or wider than 4 cells.  shift is per lane: one loop serves the lanes that
// need cells and those that need bins.
__device__ __forceinline__ uint32_t cell_exclusion_mask(const EllipseX& e, float cx, float cy, uint32_t x0, uint32_t y0,
                                                        uint32_t x1, uint32_t y1, uint32_t shift) {
    const uint32_t CS = 1u << shift;
    const float fcs = (float)CS, ICS = shift == 3u ? 0.125f : 0.03125f;
    const uint32_t cx0 = x0 >> shift, cy0 = y0 >> shift, cx1 = x1 >> shift, cy1 = y1 >> shift;
    if (cx1 - cx0 >= 4u || cy1 - cy0 >= 4u) return 0u;
    if (cx1 == cx0 && cy1 == cy0) return 0u;  // one cell: the rect itself decides
    if (!e.ok) return 0u;
    const uint32_t all = (1u << (cx1 - cx0 + 1u)) - 1u;  // the rect's cells in a row
    const float fcx0 = (float)cx0;
    uint32_t excl = 0;
    for (uint32_t r = 0; r <= cy1 - cy0; ++r) {
        const float pyA = (float)((cy0 + r) * CS);  // band's pixel rows pyA .. pyA+CS-1
        float yl = cy - (pyA + (fcs - 0.5f)), yh = cy - (pyA + 0.5f);
        yl = fmaxf(yl, -e.ymax);
        yh = fminf(yh, e.ymax);
        uint32_t keep = 0u;  // (none unless the band meets the ellipse)
        if (yl <= yh) {
            auto root = [&](float y) { return __builtin_amdgcn_sqrtf(fmaxf(e.Qa - e.det * y * y, 0.0f)); };
            const float rl = root(yl), rh = root(yh);
            const float xmax = ((-e.ys >= yl && -e.ys <= yh) ? e.xs : fmaxf(-e.b * yl + rl, -e.b * yh + rh) * e.ia) + e.pad;
            const float xmin = ((e.ys >= yl && e.ys <= yh) ? -e.xs : fminf(-e.b * yl - rl, -e.b * yh - rh) * e.ia) - e.pad;
            // cell q (pixel centres X = (cx0+q) CS + 0.5 - cx .. + CS - 1) is a
            // candidate iff its first centre <= xmax and its last >= xmin
            const float qh = fminf(fmaxf(floorf((xmax + cx - 0.5f) * ICS) - fcx0, -1.0f), 4.0f);
            const float ql = fminf(fmaxf(ceilf((xmin + cx + 0.5f) * ICS - 1.0f) - fcx0, 0.0f), 5.0f);
            keep = ((1u << ((uint32_t)(int)qh + 1u)) - 1u) & ~((1u << (uint32_t)(int)ql) - 1u);
        }
        excl |= (all & ~keep) << (r * 4u);
    }
    return excl;
}

// A bin mask that excludes every bin of the rect keeps its first one (see
// bins_from_cells).
__device__ __forceinline__ uint32_t keep_one_bin(uint32_t b, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    const uint32_t cols = (x1 >> 5) - (x0 >> 5) + 1u, rows = (y1 >> 5) - (y0 >> 5) + 1u;
    if (cols > 4u || rows > 4u) return b;
    const uint32_t row = (1u << cols) - 1u;
    uint32_t all = 0u;
#pragma unroll
    for (uint32_t r = 0; r < 4u; ++r) all |= r < rows ? row << (4u * r) : 0u;
    return b == all ? b & ~1u : b;
}

// The bin-exclusion mask of a rect within 4x4 8-px cells (so within 2x2
// bins) from its cell mask: a bin is excluded when every cell of the rect in
// it is.  Bit br*4 + bq: bin (bx0 + bq, by0 + br), bx0 = x0 >> 5.
__device__ __forceinline__ uint32_t bins_from_cells(uint32_t cexcl, uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    const uint32_t cx0 = x0 >> 3, cy0 = y0 >> 3, cx1 = x1 >> 3, cy1 = y1 >> 3;
    const uint32_t ncol = cx1 - cx0 + 1u, nrow = cy1 - cy0 + 1u;
    // cells of the rect in bin column 0 / row 0: those before the next 4-cell boundary
    const uint32_t split_x = min(4u - (cx0 & 3u), ncol), split_y = min(4u - (cy0 & 3u), nrow);
    const uint32_t col0 = (1u << split_x) - 1u, col1 = ((1u << ncol) - 1u) & ~col0;
    uint32_t row0 = 0u, row1 = 0u;  // the rect's cell bits (4 per cell row) of bin row 0 / 1
#pragma unroll
    for (uint32_t r = 0; r < 4u; ++r) {
        const uint32_t m = r < nrow ? 0xFu << (4u * r) : 0u;
        if (r < split_y) row0 |= m;
        else row1 |= m;
    }
    uint32_t b = 0u;
    const uint32_t inc = ~cexcl;  // (cells not excluded)
    auto colm = [](uint32_t c) { return c | c << 4 | c << 8 | c << 12; };
    if ((inc & row0 & colm(col0)) == 0u) b |= 1u;
    if (col1 && (inc & row0 & colm(col1)) == 0u) b |= 2u;
    if (row1 && (inc & row1 & colm(col0)) == 0u) b |= 16u;
    if (col1 && row1 && (inc & row1 & colm(col1)) == 0u) b |= 32u;
    // a splat whose ellipse reaches no pixel centre of its rect keeps its
    // first bin: every non-empty rect emits a pair (gs_stats.visible counts
    // the oracle's visible splats; the pair adds exact zeros)
    const uint32_t allb = (col1 ? 3u : 1u) * (row1 ? 17u : 1u);
    if (b == allb) b &= ~1u;
    return b;
}

// Both masks of a visible splat: the record's 8x8-cell mask (rect within 4x4
// cells, else 0) and the binning rect's 32x32-bin mask, from the record's
// centre (cx, cy), axes (ax, ay), (bx, by) and pixel rect.
struct RectMasks {
    uint32_t cell, bin;
};
__device__ __forceinline__ RectMasks rect_masks(float cx, float cy, float ax, float ay, float bx, float by, uint32_t x0,
                                                uint32_t y0, uint32_t x1, uint32_t y1) {
    const EllipseX ex = ellipse_x(ax, ay, bx, by);
    const bool small = (x1 >> 3) - (x0 >> 3) < 4u && (y1 >> 3) - (y0 >> 3) < 4u;
    const uint32_t m = cell_exclusion_mask(ex, cx, cy, x0, y0, x1, y1, small ? 3u : 5u);
    return RectMasks{small ? m : 0u, small ? bins_from_cells(m, x0, y0, x1, y1) : keep_one_bin(m, x0, y0, x1, y1)};
}

}  // namespace gs
