// composite.hip — per-tile front-to-back alpha composite.
//
// One 256-lane workgroup per 16x16 tile, one pixel per lane, each wave an
// 8x8 quadrant.  Lists are binned per 32x32 bin (2x2 tiles: 2.35 instead of
// 4.38 pairs per splat, so sorting is cheaper); the four tiles of a bin are
// consecutive workgroups on one XCD and share the bin list through its L2.
// The list is streamed through LDS in batches of 256 records (one 48-B record
// gathered per lane), software-pipelined: the next batch is in flight into
// registers while the current one is composited.  Per batch every wave
// compacts the records whose pixel rect overlaps its quadrant (64 per
// ballot) and walks only those, two at a time with both records' LDS reads
// issued first: coverage (K6 closed form), gaussian + 0.01 cutoff (F1,
// tile.metal:191-197) and the composite (A1, tile.metal:251-266; or the live
// 50-layer rule, 50layer.metal:208-222).  A finer per-quadrant ellipse test
// was measured and removed: it cost more VALU than the bodies it skipped.
// The per-pixel body is branch-free (a non-covering splat contributes an
// exact zero), a wave leaves the batch once all 64 of its pixels are
// saturated, and the workgroup stops fetching once all 256 are.
// Bins are dealt to workgroups XCD-aware: the four tiles of a bin run on
// one XCD and share the bin's list through its L2.
#include <hip/hip_ext.h>


#include "gs_kernels.h"
#include "gs_wave.h"

namespace gs {

#ifdef GS_COMPOSITE_TRACE
// Debug build only (tools/composite_trace.py): per strip workgroup, its start
// and end (s_memrealtime, 100 MHz), its bin pair slot and the fetched record
// count, written with vector stores by lane 0; read by
// gs_debug_composite_trace, which no product path calls.
__device__ unsigned long long g_comp_trace[4 * 65536];
#endif

// MLAB k-buffer (gaussian_splat.metal:201-361): six premultiplied half
// layers + half depths per pixel in registers, updated per covering fragment
// in arrival order with the reference's insertion and under-merge, resolved
// front to back.  Every op is a correctly rounded half op (oracle: mlab_*).
namespace mlab {
using h16 = _Float16;
__device__ __forceinline__ h16 mul(h16 a, h16 b) { return (h16)((float)a * (float)b); }  // exact in f32, one rounding
__device__ __forceinline__ h16 add(h16 a, h16 b) { return (h16)((float)a + (float)b); }  // no double-rounding tie
__device__ __forceinline__ h16 sub(h16 a, h16 b) { return (h16)((float)a - (float)b); }
constexpr int kLayers = 6;  // NUM_OIT_LAYERS (gaussian_splat.metal:11)
struct KBuf {
    h16 L[kLayers][4];
    h16 D[kLayers];
    __device__ __forceinline__ void clear() {  // all attachments (0,0,0,1) (instanced_splat_renderer.mm:540)
#pragma unroll
        for (int i = 0; i < kLayers; ++i) {
            L[i][0] = L[i][1] = L[i][2] = (h16)0.0f;
            L[i][3] = (h16)1.0f;
            D[i] = (h16)0.0f;
        }
        D[3] = (h16)1.0f;  // depths01.a
    }
    __device__ __forceinline__ void insert(float r, float g, float b, float alpha, h16 nd) {  // :206-294
        // alpha is rounded to f32 first (float alpha = g * opacity, :200), then
        // to half: keep the compiler from fusing the product and the
        // conversion into one v_fma_mix rounding
        asm volatile("" : "+v"(alpha));
        const h16 ha = (h16)alpha;
        h16 nl[4] = {mul((h16)r, ha), mul((h16)g, ha), mul((h16)b, ha), sub((h16)1.0f, ha)};
#pragma unroll
        for (int i = 0; i < kLayers; ++i) {
            const bool ins = nd >= D[i];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const h16 t = L[i][c];
                L[i][c] = ins ? nl[c] : t;
                nl[c] = ins ? t : nl[c];
            }
            const h16 t = D[i];
            D[i] = ins ? nd : t;
            nd = ins ? t : nd;
        }
        const int l = kLayers - 1;
        const bool closer = nd >= D[l];
        h16 m[4];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const h16 fr = closer ? nl[c] : L[l][c], bk = closer ? L[l][c] : nl[c];
            const h16 ba = closer ? L[l][3] : nl[3];
            m[c] = add(bk, mul(fr, ba));
        }
        m[3] = mul(nl[3], L[l][3]);  // front.a * back.a (commutative)
#pragma unroll
        for (int c = 0; c < 4; ++c) L[l][c] = m[c];
        D[l] = closer ? nd : D[l];
    }
    __device__ __forceinline__ float4 resolve() const {  // :330-361
        h16 C0 = (h16)0.0f, C1 = C0, C2 = C0, at = (h16)1.0f;
#pragma unroll
        for (int i = 0; i < kLayers; ++i) {
            C0 = add(C0, mul(L[i][0], at));
            C1 = add(C1, mul(L[i][1], at));
            C2 = add(C2, mul(L[i][2], at));
            at = mul(at, L[i][3]);
        }
        return make_float4((float)C0, (float)C1, (float)C2, (float)sub((h16)1.0f, at));
    }
};
}  // namespace mlab

// MODE 0: tile rule, 1: live50 rule, 2: cap threshold pass (index-ordered
// lists; per pixel the id of the a.cap-th covering fragment), 3: MLAB
// k-buffer (index-ordered lists, no early out).  CAP: composite
// only fragments with id <= thr[pixel] (the first a.cap in arrival order).
// SLAB (depth-slab multi-GPU): 1 = transmittance pass, 2 =
// colour pass from the earlier slabs' transmittance product.
//
// Staged record (per tile): the conic scaled by kConicScale
// and its offset at the tile origin, so a lane's coverage is four fmas on
// its tile-local pixel centre (lx, ly) = (px - tx0 + 1/2, py - ty0 + 1/2):
//   u' = fma(Ax', lx, fma(-Ay', ly, U0)),  U0 = fma(Ax', tx0 - cx, Ay' (cy - ty0))
// and likewise v' from (Bx', By', V0).
// One 48-B LDS slot per staged record (first the raw gathered record):
//   a = (U0, V0, Ax', -Ay')   b = (Bx', -By', opacity, r)   c = (g, b, id, half(zF))
// (id: the splat id, cap modes; half(zF) bits: MLAB), and the wave lists hold
// slot byte offsets (u16), so a record's reads take one address VGPR.
struct StagedRec {
    float4 a, b, c;
};
static_assert(sizeof(StagedRec) == 48, "staged record slot");
__device__ __forceinline__ const StagedRec& staged_at(const StagedRec* base, uint32_t off) {
    return *reinterpret_cast<const StagedRec*>(reinterpret_cast<const char*>(base) + off);
}

// PASS (depth-cut frames, gs_options.depth_split; modes 0/1,
// no cap, no slabs): 1 = the front lists (CompositeArgs: a tile left open
// with a cut list keeps its per-pixel state, every tile raises its bin's next
// cut); 2 = the fallback lists, resuming the open tiles only.
//
// SGPR budget: at most 62 (TotalSGPRs <= 64, tests/test_kernel_resources.py).
// gfx950 allocates a wave's SGPRs in blocks of 16 (plus 16), from 800 per
// SIMD, and the composite shares its SIMDs with the preprocess kernel
// (96-SGPR class) in the pipelined frame.  Left alone the pass-1 kernel takes
// 68-76 SGPRs (the 96 class, against 80 for pass 0): standalone no slower,
// but in the co-run with the preprocess its span grew 0.445 -> 0.527 ms and
// the frame 0.687 -> 0.738 ms (profiles/r04/ab_composite_sgpr.txt).  The cap
// costs pass 1 one spilled dword (stored at entry, reloaded at the end).
#define GS_COMPOSITE_SGPRS 62
template <int MODE, bool CAP, int SLAB = 0, int PASS = 0>
__global__ __launch_bounds__(256, MODE == 3 ? 4 : 8) __attribute__((amdgpu_num_sgpr(GS_COMPOSITE_SGPRS))) void composite_kernel(CompositeArgs a, uint32_t nwg) {
    constexpr bool kIds = CAP || MODE == 2;  // the body needs the splat id
    static_assert(PASS == 0 || ((MODE == 0 || MODE == 1) && !CAP && SLAB == 0), "depth-cut passes: tile/live50 rules");
    __shared__ StagedRec srec[kTileThreads];
    __shared__ uint16_t wlist[4][kTileThreads];  // per wave: slot byte offsets
    __shared__ uint8_t sqm[kTileThreads];  // per staged record: the quadrants it may reach
    __shared__ uint32_t sopen[4];          // per wave: pixels still open after its last walk

    // XCD-aware bijective remap (blocks b and b+8 share an XCD,
    // cdna_hip_programming.md §5, T1): bins dealt round-robin over the XCDs,
    // a bin's 4 tiles on one XCD (they share its list through that L2).
    // Measured against giving each XCD a contiguous band of bin rows: -2 %
    // composite, since the bands' costs differ and the launch ends with the
    // slowest XCD.
    const uint32_t orig = blockIdx.x;
    const uint32_t full = nwg & ~31u;
    const uint32_t kk = orig >> 3;
    const uint32_t wg = orig < full ? 32u * (kk >> 2) + 4u * (orig & 7u) + (kk & 3u) : orig;

    // Grid covers only the owned bin rows.  The four 16x16
    // tiles of a bin are consecutive workgroups (same XCD / L2).
    const uint32_t per_row = 4u * (uint32_t)a.tiles_x;
    const int owned_row = (int)(wg / per_row);
    const uint32_t k4 = wg - (uint32_t)owned_row * per_row;
    const int bx = (int)(k4 >> 2);
    const int by = a.rows ? (int)a.rows[owned_row] : owned_row;
    const int tx = 2 * bx + (int)(k4 & 1u), ty = 2 * by + (int)((k4 >> 1) & 1u);
    const int width = a.width, height = a.height;
    const uint32_t bin = (uint32_t)(by * a.tiles_x + bx);
    // (depth cuts: the bin's 128-B quadrant record, CompositeArgs::qrec; this
    // tile's quadrants are [4 (k4 & 3), +4))
    uint32_t* const qr = a.qrec ? a.qrec + (size_t)bin * kQrecWords : nullptr;
    const uint32_t tq = (k4 & 3u) * 4u;
    uint4 oq = make_uint4(0u, 0u, 0u, 0u);  // (PASS 2) the tile's open quadrants
    if constexpr (PASS == 2) {
        oq = *reinterpret_cast<const uint4*>(qr + 16u + tq);
        if ((oq.x | oq.y | oq.z | oq.w) == 0u) return;  // (whole workgroup) the front list finished the tile
    }
    const int tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
    // PASS 1: the bin's list was cut (a quadrant left open keeps its state)
    const bool trunc = PASS == 1 && a.cut_in && a.cut_in[bin] < kDepthInf;
    // this wave's quadrant: pixels [tx0 + ox, +7] x [ty0 + oy, +7]
    const uint32_t tx0 = (uint32_t)(tx * kTile), ty0 = (uint32_t)(ty * kTile);
    const uint32_t lxi = (wave & 1u) * 8u + (lane & 7u), lyi = (wave >> 1) * 8u + (lane >> 3);
    const int px = (int)(tx0 + lxi);
    const int py = (int)(ty0 + lyi);
    const bool inside = px < width && py < height;
    const float lx = (float)lxi + 0.5f;  // tile-local pixel centre (exact)
    const float ly = (float)lyi + 0.5f;
    const float ftx0 = (float)tx0, fty0 = (float)ty0;

    // (a tile wholly outside the frame, the last bin row's lower half, has
    // nothing to composite)
    uint2 rg = decode_range(a.ranges[bin]);
    if (tx0 >= (uint32_t)width || ty0 >= (uint32_t)height) rg.y = rg.x;
    // Pixels outside the frame start finished (T = 0): for the tile and live50
    // rules "finished" is then just the break test on T itself, so no
    // separate per-lane flag is carried through the loop.
    float T = inside ? 1.0f : 0.0f;  // transmittance (tile rule: T = 1 - A)
    float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    // compact = owned bin rows stacked (multi-GPU band buffer)
    const int orow = a.compact ? owned_row * kBin + (py - by * kBin) : py;
    const size_t pix = (size_t)py * width + px;
    // PASS 2: this quadrant was left open by the front list (else its pixels
    // start finished, and were written already)
    const bool resumed = PASS == 2 && (wave == 0 ? oq.x : wave == 1 ? oq.y : wave == 2 ? oq.z : oq.w) != 0u;
    if constexpr (PASS == 2) {
        T = 0.0f;
        if (inside && resumed) {  // the state the front list left: the same registers, resumed
            const float4 st = a.state[pix];
            C0 = st.x;
            C1 = st.y;
            C2 = st.z;
            T = st.w;
        }
    }
    bool done = !inside;  // MODE 2 / 3
    uint32_t thr = 0xFFFFFFFFu;  // CAP: last admitted id; MODE 2: result
    int cnt = 0;                 // MODE 2: covering fragments seen
    if constexpr (CAP) {
        if (inside) thr = a.thr[pix];
    }
    // slab colour pass: the state the earlier (farther) slabs leave, exactly
    // the ordered product of their transmittance, rank order = depth order
    float T0 = 1.0f;
    mlab::KBuf kb;
    if constexpr (MODE == 3) kb.clear();
    if constexpr (SLAB == 2) {
        float ts = 1.0f;
        if (inside)
            for (int j = 0; j < a.slab_rank; ++j) ts *= a.t_all[((size_t)j * height + py) * width + px];
        // saturated before this slab (T <= 0.01 / T < 0.01): the loop broke earlier
        if (inside) T = ts;
        T0 = T;
    }
    auto finished = [&]() -> bool {
        if constexpr (MODE == 0) return T <= kTSat;
        else if constexpr (MODE == 1) return T < kTMin;
        else return done;
    };

    // One record at this lane's pixel: coverage (K6 closed form: the quad box
    // |uv| <= 3 and the 0.01 cutoff, tile.metal:142-156,191-195), then the
    // gaussian alpha (:197) and the composite update (A1).  Skipping a lane is
    // bit-identical to adding its exact zero, so the update sits in the
    // gaussian's exec-masked block.
    auto body_v = [&](const float4 aa, const float4 bb, const float2 cc, uint32_t id, _Float16 hd) {
        const float u = __builtin_fmaf(aa.z, lx, __builtin_fmaf(aa.w, ly, aa.x));
        const float v = __builtin_fmaf(bb.x, lx, __builtin_fmaf(bb.y, ly, aa.y));
        const float qq = __builtin_fmaf(v, v, u * u);
        const bool covered = fmaxf(fabsf(u), fabsf(v)) <= kBoxS && qq <= kQMaxS;
        if constexpr (MODE == 2) {
            // arrival order: the a.cap-th covering fragment fixes the threshold
            const bool in = !done && covered;
            cnt += in ? 1 : 0;
            if (in && cnt == a.cap) {
                thr = id;
                done = true;
            }
        } else if constexpr (MODE == 3) {
            if (!done && covered) kb.insert(bb.w, cc.x, cc.y, bb.z * gs_gauss2(qq), hd);
        } else {
            bool in = !finished() && covered;
            if constexpr (CAP) in = in && id <= thr;
            if (in) {
                const float alpha = bb.z * gs_gauss2(qq);
                if constexpr (MODE == 0) {
                    const float sa = alpha * T;
                    C0 = __builtin_fmaf(bb.w, sa, C0);
                    C1 = __builtin_fmaf(cc.x, sa, C1);
                    C2 = __builtin_fmaf(cc.y, sa, C2);
                    T = T - sa;
                } else {
                    C0 = __builtin_fmaf(bb.w, T, C0);
                    C1 = __builtin_fmaf(cc.x, T, C1);
                    C2 = __builtin_fmaf(cc.y, T, C2);
                    T = T * (1.0f - alpha);
                }
            }
        }
    };
    auto body = [&](uint32_t off) {
        const StagedRec& r = staged_at(srec, off);
        body_v(r.a, r.b, make_float2(r.c.x, r.c.y), kIds ? __float_as_uint(r.c.z) : 0u,
               MODE == 3 ? __builtin_bit_cast(_Float16, (uint16_t)__float_as_uint(r.c.w)) : (_Float16)0.0f);
    };

    // Software pipeline: while batch b is composited, batch b+1's records are
    // in flight into registers and batch b+2's ids are being loaded.
    // Coalesced gathers: wave w stages records 64w..64w+63 of a batch, and
    // their 192 16-B chunks are loaded by its 64 lanes three apiece (chunk
    // c = lane + 64i is part c % 3 of record c / 3), so adjacent lanes read
    // adjacent bytes of one record; the owner lane of each record collects
    // its chunks through LDS.  Every lane loads, its list position clamped to
    // the last entry: a conditional load joins the old and the loaded
    // registers, and the copy the compiler then emits waits for the load it
    // was meant to overlap.
    const uint32_t last = rg.y > rg.x ? rg.y - 1u : rg.x;
    uint32_t ck[3], cp[3];  // this lane's chunks: record (in the wave's 64) and part
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const uint32_t c = lane + 64u * (uint32_t)i;
        ck[i] = c / 3u;
        cp[i] = c - 3u * ck[i];
    }
    float4 rc[3] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f),
                    make_float4(0.f, 0.f, 0.f, 0.f)};
    uint32_t id_cur = 0, id_next = 0;
    auto gather = [&](uint32_t own_id) {
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t idk = (uint32_t)__shfl((int)own_id, (int)ck[i], 64);
            rc[i] = a.rec[(size_t)a.rec_stride * idk + cp[i]];
        }
    };
    if (rg.y > rg.x) {
        const uint32_t j = rg.x + tid;
        id_cur = a.vals[j < last ? j : last];
        gather(id_cur);
        id_next = a.vals[j + kTileThreads < last ? j + kTileThreads : last];
    }
    // records this workgroup fetched: the first batch, then one prefetched
    // batch per batch it composites (the early-out stops both)
    const uint32_t len = rg.y > rg.x ? rg.y - rg.x : 0u;  // (empty bins: {~0, 0})
    uint32_t fetched = len < (uint32_t)kTileThreads ? len : (uint32_t)kTileThreads;
    uint32_t wend = 0u;  // (PASS 1) end of the last batch this wave walked with an open pixel
    for (uint32_t b = rg.x; b < rg.y; b += kTileThreads) {
        // every wave publishes whether it still has open pixels; one LDS
        // barrier both orders that and frees the slots of the last batch
        // (__syncthreads_count takes three)
        if (b != rg.x) {
            const bool open = __ballot(!finished()) != 0;
            if (lane == 0) sopen[wave] = open ? 1u : 0u;
            block_lds_sync();
            const uint4 o = *reinterpret_cast<const uint4*>(sopen);
            if ((o.x | o.y | o.z | o.w) == 0u) break;
        }
        if (rg.y - b > (uint32_t)kTileThreads) {
            const uint32_t left = rg.y - b - (uint32_t)kTileThreads;
            fetched += left < (uint32_t)kTileThreads ? left : (uint32_t)kTileThreads;
        }
        // the wave's gathered chunks into their records' slots (raw layout):
        // chunk c of the wave is float4 192 w + c of the slot array
#pragma unroll
        for (int i = 0; i < 3; ++i) reinterpret_cast<float4*>(srec)[192u * wave + lane + 64u * (uint32_t)i] = rc[i];
        wave_lds_sync();  // the wave's 64 slots are only touched by this wave until the barrier
        if (b + tid < rg.y) {
            // record (cx, cy, ax, ay) (bx, by, op, r) (g, b, rect_lo, rect_hi)
            // staged for this tile (scaled conic, offsets at the tile origin)
            StagedRec& st = srec[tid];
            const float4 r0 = st.a, r1 = st.b, r2 = st.c;
            const float ax = r0.z * kConicScale, ay = r0.w * kConicScale;
            const float bxs = r1.x * kConicScale, bys = r1.y * kConicScale;
            const float ex = ftx0 - r0.x, ey = r0.y - fty0;
            st.a = make_float4(__builtin_fmaf(ax, ex, ay * ey), __builtin_fmaf(bxs, ex, bys * ey), ax, -ay);
            st.b = make_float4(bxs, -bys, r1.z, r1.w);
            uint32_t sid = 0, shd = 0;
            if constexpr (kIds) sid = id_cur;
            if constexpr (MODE == 3) shd = kDepthInf - a.dkey[id_cur];  // half(zF) (dkey = 0x7C00 - half bits)
            st.c = make_float4(r2.x, r2.y, __uint_as_float(sid), __uint_as_float(shd));
            // which of the tile's 8x8 quadrants (wave w: column w & 1, row
            // w >> 1) the record's rect reaches and its cell mask does not
            // rule out: computed once here instead of by every wave
            const uint32_t wlo = __float_as_uint(r2.z), whi = __float_as_uint(r2.w);
            const uint32_t lo = rect_coords(wlo, a.cell_mask), hi = rect_coords(whi, a.cell_mask);
            const uint32_t x0 = lo & 0xFFFFu, y0 = lo >> 16, x1 = hi & 0xFFFFu, y1 = hi >> 16;
            const bool c0 = !(x1 < tx0 || x0 > tx0 + 7u), c1 = !(x1 < tx0 + 8u || x0 > tx0 + 15u);
            const bool w0 = !(y1 < ty0 || y0 > ty0 + 7u), w1 = !(y1 < ty0 + 8u || y0 > ty0 + 15u);
            uint32_t qm = (uint32_t)(c0 && w0) | (uint32_t)(c1 && w0) << 1 | (uint32_t)(c0 && w1) << 2 |
                          (uint32_t)(c1 && w1) << 3;
            if (a.cell_mask && qm) {
                const uint32_t cm = rect_cell_mask(wlo, whi);
#pragma unroll
                for (uint32_t w = 0; w < 4; ++w) {
                    const uint32_t dcx = (tx0 >> 3) + (w & 1u) - (x0 >> 3), dcy = (ty0 >> 3) + (w >> 1) - (y0 >> 3);
                    if (dcx < 4u && dcy < 4u && ((cm >> (dcy * 4u + dcx)) & 1u)) qm &= ~(1u << w);
                }
            }
            sqm[tid] = (uint8_t)qm;
        }
        __syncthreads();
        {
            const uint32_t j = b + 2u * kTileThreads + tid;
            id_cur = id_next;
            gather(id_cur);
            id_next = a.vals[j < last ? j : last];
        }
        const uint32_t cnt_b = rg.y - b < (uint32_t)kTileThreads ? rg.y - b : (uint32_t)kTileThreads;
        // wave-level compaction of the splats reaching this quadrant (index order kept)
        uint32_t nl = 0;
        if (__ballot(!finished()) != 0) {
            wend = b + cnt_b;
            for (uint32_t k0 = 0; k0 < cnt_b; k0 += 64) {
                const uint32_t k = k0 + lane;
                const bool hit = k < cnt_b && ((sqm[k] >> wave) & 1u);
                const uint64_t m = __ballot(hit);
                if (hit) wlist[wave][nl + mbcnt(m)] = (uint16_t)(k * sizeof(StagedRec));
                nl += (uint32_t)__popcll(m);
            }
        }
        wave_lds_sync();  // wlist[wave] is only touched by this wave
        uint32_t i = 0;
        if constexpr (MODE == 2 || MODE == 3) {
            for (; i < nl; ++i) {
                if (__ballot(!done) == 0) break;
                body(wlist[wave][i]);
            }
        } else {
            // two records per step, both records' LDS reads issued before
            // either body; the next pair's slot offsets are read one step ahead
            const uint32_t* wl2 = reinterpret_cast<const uint32_t*>(wlist[wave]);
            uint32_t w2 = nl >= 2 ? wl2[0] : 0u;
            for (; i + 1 < nl; i += 2) {
                if (__ballot(!finished()) == 0) break;
                const StagedRec& p0 = staged_at(srec, w2 & 0xFFFFu);
                const StagedRec& p1 = staged_at(srec, w2 >> 16);
                const float4 a0 = p0.a, b0 = p0.b;
                const float2 c0 = make_float2(p0.c.x, p0.c.y);
                const float4 a1 = p1.a, b1 = p1.b;
                const float2 c1 = make_float2(p1.c.x, p1.c.y);
                const uint32_t i0 = kIds ? __float_as_uint(p0.c.z) : 0u, i1 = kIds ? __float_as_uint(p1.c.z) : 0u;
                if (i + 3 < nl) w2 = wl2[(i >> 1) + 1];
                body_v(a0, b0, c0, i0, (_Float16)0.0f);
                body_v(a1, b1, c1, i1, (_Float16)0.0f);
            }
            if (i < nl && __ballot(!finished()) != 0) body(wlist[wave][i++]);
        }
    }
    if (tid == 0 && a.fetched) (void)atomicAdd(a.fetched, (unsigned long long)fetched);
    // PASS 1, per quadrant (no workgroup barrier, no contended atomic): a
    // pixel still open at the end of a list that was cut keeps its state for
    // the fallback lists instead of its final value
    bool open_w = false, keep = false;
    if constexpr (PASS == 1) {
        open_w = __ballot(!finished()) != 0;
        keep = open_w && trunc;
    }
    const bool write = inside && (PASS != 2 || resumed);  // (PASS 2: the rest was written by pass 1)
    if (write) {
        if (keep) {
            a.state[pix] = make_float4(C0, C1, C2, T);  // (C, T)
        } else if constexpr (SLAB == 1) {
            a.t_out[pix] = T;
        } else if constexpr (SLAB == 2) {
            // contributions: colour and the alpha this slab adds (sum over slabs)
            a.out[pix] = make_float4(C0, C1, C2, T0 - T);
        } else if constexpr (MODE == 2) {
            a.thr_out[pix] = thr;
        } else {
            const float4 o = MODE == 3 ? kb.resolve() : make_float4(C0, C1, C2, 1.0f - T);
            if (a.out_bgra8)
                a.out_bgra8[(size_t)orow * width + px] = pack_bgra8(o.x, o.y, o.z, o.w);
            else
                a.out[(size_t)orow * width + px] = o;
        }
    }
    // the quadrant's record words, after its pixels (a store queued before
    // them would hold the pixel stores' wait, vmcnt counting stores too): its
    // cut position (the end of the last batch it walked with an open pixel,
    // ~0 while one stays open) and its open flag
    if constexpr (PASS == 1) {
        if (lane == 0) {
            qr[tq + wave] = open_w ? 0xFFFFFFFFu : wend;
            qr[16u + tq + wave] = keep ? 1u : 0u;
            if (keep) (void)atomicAdd(a.open_q_count, 1ull);
        }
    }
}

// Strip composite: the tile and live50 rules (MODE 0/1; no cap, no depth
// slabs; depth-cut PASS 0/1/2), the bench frame's kernel.  The same contract
// as composite_kernel, op for op, with more pixels per record read:
//  - one 256-lane workgroup per half bin (two 16x16 tiles side by side, the
//    bin's top or bottom row of tiles), so each bin record is gathered and
//    staged twice per bin instead of four times;
//  - each wave a 16x8 strip of one tile, two pixels per lane (tile-local
//    (lx, ly) and (lx + 8, ly): the two 8x8 quadrants of the strip), so one
//    broadcast read of a staged record (40 B) serves both quadrants and the
//    inner fma(-A'y, ly, U0) of the coverage test is shared by them;
//  - per record and wave a 2-bit quadrant selector (from the record's rect
//    and 8x8 cell mask, as composite_kernel's per-quadrant filter), tested in
//    scalar registers: a pixel whose quadrant the record cannot reach skips
//    its coverage test.
// Staged slot (48 B): a = (Ax', -Ay', Bx', -By'), b = (opacity, r, g, b),
// c = (U0, V0) at the left tile's origin, then at the right tile's.
#ifndef GS_COMPOSITE_LPT  // A/B knob: 0 = row-major bin order even when CompositeArgs::order is set
#define GS_COMPOSITE_LPT 1
#endif
#ifndef GS_STRIP_PRIO_TOP  // the first batches' issue priority (then one lower every two batches)
#define GS_STRIP_PRIO_TOP 3
#endif
#ifndef GS_STRIP_PRIO  // A/B knob: 1 = issue priority falls with the batches a workgroup has walked
#define GS_STRIP_PRIO 1
#endif
#ifndef GS_STRIP_PIPE  // A/B knob: 1 = the walk reads one record ahead (rolling), 0 = two records per step
#define GS_STRIP_PIPE 1
#endif
#ifndef GS_STRIP_WAVES  // A/B knob: waves per SIMD the strip composite is built for
#define GS_STRIP_WAVES 8
#endif
#ifndef GS_STRIP_PAD
#define GS_STRIP_PAD 0
#endif
template <int MODE, int PASS>
__global__ __launch_bounds__(256, GS_STRIP_WAVES) __attribute__((amdgpu_num_sgpr(GS_COMPOSITE_SGPRS))) void composite_strip_kernel(
    CompositeArgs a, uint32_t nwg) {
    static_assert(MODE == 0 || MODE == 1, "strip composite: tile / live50 rules");
    __shared__ float4 srec[3 * kTileThreads];    // 256 slots of 48 B (raw record, then staged)
    __shared__ uint16_t wlist[4][kTileThreads + 4];  // per wave: slot byte offset | selector << 14
    __shared__ uint8_t sqm[kTileThreads];        // per staged record: the 8 quadrants it may reach
    __shared__ uint32_t sopen[4];
#if GS_STRIP_PAD  // A/B knob: LDS padding (bytes) that caps the workgroups per CU
    __shared__ uint32_t lds_pad[GS_STRIP_PAD / 4];
    if (a.width < 0) lds_pad[blockIdx.x % (GS_STRIP_PAD / 4)] = 0;  // (never: keeps the array)
#endif

    // XCD-aware remap (as composite_kernel): blocks b and b + 8 share an XCD,
    // so a bin's two halves (consecutive wg) run on one XCD and share its list
    // through that L2; bins dealt round-robin over the XCDs.
    const uint32_t orig = blockIdx.x;
    const uint32_t full = nwg & ~15u;
    const uint32_t kk = orig >> 3;
    const uint32_t wg = orig < full ? 16u * (kk >> 1) + 2u * (orig & 7u) + (kk & 1u) : orig;
    const uint32_t per_row = 2u * (uint32_t)a.tiles_x;
    int owned_row, bx, by;
    const uint32_t half = wg & 1u;  // the bin's top (0) or bottom (1) row of tiles
    if (GS_COMPOSITE_LPT && a.order && !a.rows) {  // (single-GPU frames: every row owned)
        const uint32_t ob = a.order[wg >> 1];
        owned_row = by = (int)(ob / (uint32_t)a.tiles_x);
        bx = (int)(ob - (uint32_t)by * (uint32_t)a.tiles_x);
    } else {
        owned_row = (int)(wg / per_row);
        bx = (int)((wg - (uint32_t)owned_row * per_row) >> 1);
        by = a.rows ? (int)a.rows[owned_row] : owned_row;
    }
    const int width = a.width, height = a.height;
    const uint32_t bin = (uint32_t)(by * a.tiles_x + bx);
    const uint32_t tx0 = (uint32_t)(bx * kBin), ty0 = (uint32_t)(by * kBin) + 16u * half;  // left tile's origin
    const int tid = threadIdx.x;
#ifdef GS_COMPOSITE_TRACE
    const unsigned long long trace_t0 = __builtin_amdgcn_s_memrealtime();
#endif
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
    const uint32_t wt = wave >> 1, ws = wave & 1u;  // the wave's tile (left / right) and strip (top / bottom)
    // quadrant records of depth-cut frames: tile k4 = 2 half + wt of the bin,
    // quadrants (x half, y half) = (0, ws) and (1, ws): words 4 k4 + 2 ws + {0, 1}
    uint32_t* const qr = a.qrec ? a.qrec + (size_t)bin * kQrecWords : nullptr;
    const uint32_t qA = 4u * (2u * half + wt) + 2u * ws;
    bool resA = false, resB = false;  // (PASS 2) the quadrants left open by the front list
    if constexpr (PASS == 2) {
        const uint4 f0 = *reinterpret_cast<const uint4*>(qr + 16u + 8u * half);
        const uint4 f1 = *reinterpret_cast<const uint4*>(qr + 20u + 8u * half);
        if ((f0.x | f0.y | f0.z | f0.w | f1.x | f1.y | f1.z | f1.w) == 0u) return;  // (whole workgroup)
        resA = qr[16u + qA] != 0u;
        resB = qr[17u + qA] != 0u;
    }
    const bool trunc = PASS == 1 && a.cut_in && a.cut_in[bin] < kDepthInf;
    // this lane's pixels: A = (ttx0 + lxi, py), B = A + (8, 0), ttx0 = tx0 + 16 wt
    const uint32_t lxi = lane & 7u, lyi = 8u * ws + (lane >> 3);
    const float lxA = (float)lxi + 0.5f, lxB = (float)lxi + 8.5f, ly = (float)lyi + 0.5f;  // tile-local (exact)
    const int pxA = (int)(tx0 + 16u * wt + lxi), pxB = pxA + 8, py = (int)(ty0 + lyi);
    const bool inA = pxA < width && py < height, inB = pxB < width && py < height;
    const float ftx0 = (float)tx0, ftx1 = (float)(tx0 + 16u), fty0 = (float)ty0;

    uint2 rg = decode_range(a.ranges[bin]);
    if (tx0 >= (uint32_t)width || ty0 >= (uint32_t)height) rg.y = rg.x;  // both tiles outside the frame
    // pixels outside the frame start finished (T = 0), see composite_kernel
    float TA = inA ? 1.0f : 0.0f, TB = inB ? 1.0f : 0.0f;
    float A0 = 0.0f, A1 = 0.0f, A2 = 0.0f, B0 = 0.0f, B1 = 0.0f, B2 = 0.0f;
    const size_t pixA = (size_t)py * width + pxA, pixB = pixA + 8;
    if constexpr (PASS == 2) {
        TA = 0.0f;
        TB = 0.0f;
        if (inA && resA) {
            const float4 st = a.state[pixA];
            A0 = st.x, A1 = st.y, A2 = st.z, TA = st.w;
        }
        if (inB && resB) {
            const float4 st = a.state[pixB];
            B0 = st.x, B1 = st.y, B2 = st.z, TB = st.w;
        }
    }
    auto fin = [](float T) -> bool {
        if constexpr (MODE == 0) return T <= kTSat;
        else return T < kTMin;
    };
    // One pixel and one record (composite_kernel's body_v): coverage, the
    // gaussian alpha and the update, the update exec-masked (an uncovered or
    // finished pixel adds an exact zero).
    auto pixel = [&](float lx, float tu, float tv, const float4& aa, const float4& bb, float& T, float& C0, float& C1,
                     float& C2) {
        const float u = __builtin_fmaf(aa.x, lx, tu);
        const float v = __builtin_fmaf(aa.z, lx, tv);
        const float qq = __builtin_fmaf(v, v, u * u);
        const bool covered = fmaxf(fabsf(u), fabsf(v)) <= kBoxS && qq <= kQMaxS;
        if (!fin(T) && covered) {
            const float alpha = bb.x * gs_gauss2(qq);
            if constexpr (MODE == 0) {
                const float sa = alpha * T;
                C0 = __builtin_fmaf(bb.y, sa, C0);
                C1 = __builtin_fmaf(bb.z, sa, C1);
                C2 = __builtin_fmaf(bb.w, sa, C2);
                T = T - sa;
            } else {
                C0 = __builtin_fmaf(bb.y, T, C0);
                C1 = __builtin_fmaf(bb.z, T, C1);
                C2 = __builtin_fmaf(bb.w, T, C2);
                T = T * (1.0f - alpha);
            }
        }
    };
    // a record for both of the wave's quadrants; sel (scalar): bit 0 quadrant
    // A may be reached, bit 1 quadrant B
    auto body = [&](const float4& aa, const float4& bb, const float2& cc, uint32_t sel) {
        const float tu = __builtin_fmaf(aa.y, ly, cc.x);  // fma(-A'y, ly, U0)
        const float tv = __builtin_fmaf(aa.w, ly, cc.y);  // fma(-B'y, ly, V0)
        if (sel & 1u) pixel(lxA, tu, tv, aa, bb, TA, A0, A1, A2);
        if (sel & 2u) pixel(lxB, tu, tv, aa, bb, TB, B0, B1, B2);
    };

    // Gathers as composite_kernel: wave w loads records 64w..64w+63 of a
    // batch as 192 adjacent 16-B chunks (lane + 64 i), the next batch in
    // flight while the current one is composited.
    const uint32_t last = rg.y > rg.x ? rg.y - 1u : rg.x;
    float4 rc[3] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f),
                    make_float4(0.f, 0.f, 0.f, 0.f)};
    uint32_t id_next = 0;
    // (the chunk's record and part are recomputed per gather from a lane id
    // the compiler cannot hoist: kept live across the walk they spilled)
    auto gather = [&](uint32_t own_id) {
        uint32_t ln;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(ln));
        ln = __builtin_amdgcn_mbcnt_hi(~0u, ln);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const uint32_t c = ln + 64u * (uint32_t)i;
            const uint32_t ck = (c * 43691u) >> 17;  // c / 3 for c < 2^15
            const uint32_t idk = (uint32_t)__shfl((int)own_id, (int)ck, 64);
            rc[i] = a.rec[idk * (uint32_t)a.rec_stride + (c - 3u * ck)];
        }
    };
    if (rg.y > rg.x) {
        const uint32_t j = rg.x + tid;
        gather(a.vals[j < last ? j : last]);
        id_next = a.vals[j + kTileThreads < last ? j + kTileThreads : last];
    }
    const uint32_t len = rg.y > rg.x ? rg.y - rg.x : 0u;
    uint32_t fetched = len < (uint32_t)kTileThreads ? len : (uint32_t)kTileThreads;
    uint32_t wendA = 0u, wendB = 0u;  // (PASS 1) end of the last batch each quadrant walked with an open pixel
    const uint32_t* const wl2 = reinterpret_cast<const uint32_t*>(wlist[wave]);
    for (uint32_t b = rg.x; b < rg.y; b += kTileThreads) {
#if GS_STRIP_PRIO
        // (A/B) progress-ordered issue priority: a workgroup's waves drop
        // priority as they walk batches, so late-started workgroups are not
        // starved behind older ones (age arbitration) into a long drain
        {
            const uint32_t nb = (b - rg.x) / kTileThreads;
            if (nb == 0) __builtin_amdgcn_s_setprio(GS_STRIP_PRIO_TOP);
            else if (nb == 2) __builtin_amdgcn_s_setprio(GS_STRIP_PRIO_TOP > 1 ? GS_STRIP_PRIO_TOP - 1 : 0);
            else if (nb == 4) __builtin_amdgcn_s_setprio(GS_STRIP_PRIO_TOP > 2 ? GS_STRIP_PRIO_TOP - 2 : 0);
            else if (nb == 6) __builtin_amdgcn_s_setprio(0);
        }
#endif
        if (b != rg.x) {  // early out (one LDS barrier, as composite_kernel)
            const bool open = __ballot(!fin(TA) || !fin(TB)) != 0;
            if (lane == 0) sopen[wave] = open ? 1u : 0u;
            block_lds_sync();
            const uint4 o = *reinterpret_cast<const uint4*>(sopen);
            if ((o.x | o.y | o.z | o.w) == 0u) break;
        }
        if (rg.y - b > (uint32_t)kTileThreads) {
            const uint32_t left = rg.y - b - (uint32_t)kTileThreads;
            fetched += left < (uint32_t)kTileThreads ? left : (uint32_t)kTileThreads;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) srec[192u * wave + lane + 64u * (uint32_t)i] = rc[i];
        wave_lds_sync();  // the wave's 64 slots are only touched by this wave until the barrier
        if (b + tid < rg.y) {
            // raw (cx, cy, ax, ay) (bx, by, op, r) (g, b, rect_lo, rect_hi),
            // staged for both tiles (scaled conic, offsets at each tile's origin)
            float4* st = &srec[3u * tid];
            const float4 r0 = st[0], r1 = st[1], r2 = st[2];
            const float ax = r0.z * kConicScale, ay = r0.w * kConicScale;
            const float bxs = r1.x * kConicScale, bys = r1.y * kConicScale;
            const float exl = ftx0 - r0.x, exr = ftx1 - r0.x, ey = r0.y - fty0;
            const float aye = ay * ey, bye = bys * ey;
            st[0] = make_float4(ax, -ay, bxs, -bys);
            st[1] = make_float4(r1.z, r1.w, r2.x, r2.y);
            st[2] = make_float4(__builtin_fmaf(ax, exl, aye), __builtin_fmaf(bxs, exl, bye), __builtin_fmaf(ax, exr, aye),
                                __builtin_fmaf(bxs, exr, bye));
            // the 8 quadrants (columns c = 0..3 of 8 px from tx0, rows r = 0..1
            // from ty0) the rect reaches and the cell mask does not rule out;
            // bit 4 (c >> 1) + 2 r + (c & 1): wave w's selector is bits 2w, 2w+1
            const uint32_t wlo = __float_as_uint(r2.z), whi = __float_as_uint(r2.w);
            const uint32_t lo = rect_coords(wlo, a.cell_mask), hi = rect_coords(whi, a.cell_mask);
            const int rx0 = (int)(lo & 0xFFFFu) - (int)tx0, rx1 = (int)(hi & 0xFFFFu) - (int)tx0;
            const int ry0 = (int)(lo >> 16) - (int)ty0, ry1 = (int)(hi >> 16) - (int)ty0;
            const int cl = max(rx0, 0) >> 3, ch = min(rx1, 31) >> 3;
            const int rl = max(ry0, 0) >> 3, rh = min(ry1, 15) >> 3;
            uint32_t cols = rx1 >= 0 && cl <= ch ? (2u << ch) - (1u << cl) : 0u;
            const uint32_t rows = ry1 >= 0 && rl <= rh ? (2u << rh) - (1u << rl) : 0u;
            uint32_t ex0 = 0u, ex1 = 0u;  // excluded columns in rows 0 / 1
            if (a.cell_mask) {
                const uint32_t cm = rect_cell_mask(wlo, whi);
                // the rect's cell grid starts at (x0 >> 3, y0 >> 3); column c is
                // rect cell dx + c, row r rect cell dy + r
                const int dx = (int)(tx0 >> 3) - (int)((lo & 0xFFFFu) >> 3);
                const int dy = (int)(ty0 >> 3) - (int)(lo >> 19);
                auto row_excl = [&](int dcy) -> uint32_t {
                    if (dcy < 0 || dcy > 3) return 0u;
                    const uint32_t rb = (cm >> (4 * dcy)) & 0xFu;  // rect cells 0..3 of that row
                    if (dx >= 4 || dx <= -4) return 0u;
                    return (dx >= 0 ? rb >> dx : rb << (-dx)) & 0xFu;
                };
                ex0 = row_excl(dy);
                ex1 = row_excl(dy + 1);
            }
            auto spread = [](uint32_t c4) { return (c4 & 3u) | ((c4 & 0xCu) << 2); };  // columns -> bits 0,1,4,5
            const uint32_t qm = ((rows & 1u) ? spread(cols & ~ex0) : 0u) | ((rows & 2u) ? spread(cols & ~ex1) << 2 : 0u);
            sqm[tid] = (uint8_t)qm;
        }
        __syncthreads();
        {
            const uint32_t j = b + 2u * kTileThreads + tid;
            gather(id_next);
            id_next = a.vals[j < last ? j : last];
        }
        const uint32_t cnt_b = rg.y - b < (uint32_t)kTileThreads ? rg.y - b : (uint32_t)kTileThreads;
        // wave-level compaction of the records reaching an open quadrant of
        // this strip (index order kept), with their selectors
        const uint32_t open2 = (__ballot(!fin(TA)) != 0 ? 1u : 0u) | (__ballot(!fin(TB)) != 0 ? 2u : 0u);
        if constexpr (PASS == 1) {
            if (open2 & 1u) wendA = b + cnt_b;
            if (open2 & 2u) wendB = b + cnt_b;
        }
        uint32_t nl = 0;
        if (open2) {
            for (uint32_t k0 = 0; k0 < cnt_b; k0 += 64) {
                const uint32_t k = k0 + lane;
                const uint32_t sel = k < cnt_b ? (sqm[k] >> (2u * wave)) & open2 : 0u;
                const uint64_t m = __ballot(sel != 0u);
                if (sel) wlist[wave][nl + mbcnt(m)] = (uint16_t)(k * 48u | sel << 14);
                nl += (uint32_t)__popcll(m);
            }
            // three empty entries (selector 0) after the list: the half pair of an
            // odd list and the walk's unconditional read-ahead of the next pair
            if (lane < 3u) wlist[wave][nl + lane] = 0;
        }
        wave_lds_sync();  // wlist[wave] is only touched by this wave
        // two records per step, both records' LDS reads issued before either
        // body; the next pair of entries is read one step ahead.  The c half
        // read depends on the wave's tile, so the walk is instantiated per tile.
        auto walk = [&](auto tile) {
            constexpr uint32_t kC = 32u + 8u * decltype(tile)::value;
            const char* base = reinterpret_cast<const char*>(srec);
            if (nl == 0u) return;
            auto ld4 = [&](uint32_t o) { return *reinterpret_cast<const float4*>(base + o); };
            auto ld2 = [&](uint32_t o) { return *reinterpret_cast<const float2*>(base + o); };
#if GS_STRIP_PIPE
            // Rolling read-ahead, one record deep: while record i is
            // composited, record i + 1's reads are in flight (two register
            // sets, A and B, alternate), so every LDS read has a record's
            // bodies to hide behind.
            uint32_t w2 = wl2[0];
            uint32_t o = w2 & 0x3FFFu;
            float4 aA = ld4(o), bA = ld4(o + 16u);
            float2 cA = ld2(o + kC);
            for (uint32_t i = 0; i < nl; i += 2) {
                if (__ballot(!fin(TA) || !fin(TB)) == 0) break;
                const uint32_t e = __builtin_amdgcn_readfirstlane(w2);
                o = (w2 >> 16) & 0x3FFFu;
                const float4 aB = ld4(o), bB = ld4(o + 16u);
                const float2 cB = ld2(o + kC);
                w2 = wl2[(i >> 1) + 1];  // (past the list: empty entries)
                body(aA, bA, cA, (e >> 14) & 3u);
                o = w2 & 0x3FFFu;
                aA = ld4(o);
                bA = ld4(o + 16u);
                cA = ld2(o + kC);
                body(aB, bB, cB, e >> 30);
            }
#else
            uint32_t w2 = wl2[0];
            for (uint32_t i = 0; i < nl; i += 2) {
                if (__ballot(!fin(TA) || !fin(TB)) == 0) break;
                const uint32_t e = __builtin_amdgcn_readfirstlane(w2);
                const uint32_t o0 = w2 & 0x3FFFu, o1 = (w2 >> 16) & 0x3FFFu;
                const float4 a0 = ld4(o0), b0 = ld4(o0 + 16u);
                const float2 c0 = ld2(o0 + kC);
                const float4 a1 = ld4(o1), b1 = ld4(o1 + 16u);
                const float2 c1 = ld2(o1 + kC);
                if (i + 2 < nl) w2 = wl2[(i >> 1) + 1];
                body(a0, b0, c0, (e >> 14) & 3u);
                body(a1, b1, c1, e >> 30);
            }
#endif
        };
        if (wt) walk(std::integral_constant<uint32_t, 1>{});
        else walk(std::integral_constant<uint32_t, 0>{});
    }
    if (tid == 0 && a.fetched) (void)atomicAdd(a.fetched, (unsigned long long)fetched);
    if (PASS == 1 && tid == 0 && a.wcost) a.wcost[2u * bin + half] = fetched;  // (the next bin order's cost)
#ifdef GS_COMPOSITE_TRACE
    __syncthreads();
    if (tid == 0 && blockIdx.x < 65536u) {
        g_comp_trace[4u * blockIdx.x + 0] = trace_t0;
        g_comp_trace[4u * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        g_comp_trace[4u * blockIdx.x + 2] = wg;
        g_comp_trace[4u * blockIdx.x + 3] = fetched;
    }
#endif
    // PASS 1, per quadrant: a pixel still open at the end of a cut list keeps
    // its state for the fallback lists instead of its final value
    bool openA = false, openB = false, keepA = false, keepB = false;
    if constexpr (PASS == 1) {
        openA = __ballot(!fin(TA)) != 0;
        openB = __ballot(!fin(TB)) != 0;
        keepA = openA && trunc;
        keepB = openB && trunc;
    }
    // (pixel positions recomputed from a fresh lane id: kept live across the
    // loop they cost registers the walk needs)
    uint32_t ln;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0" : "=v"(ln));
    ln = __builtin_amdgcn_mbcnt_hi(~0u, ln);
    const int qx = (int)(tx0 + 16u * wt + (ln & 7u)), qy = (int)(ty0 + 8u * ws + (ln >> 3));
    const int orow = a.compact ? owned_row * kBin + (qy - by * kBin) : qy;
    auto store = [&](bool res, bool keep, int px, float C0, float C1, float C2, float T) {
        if (px >= width || qy >= height || (PASS == 2 && !res)) return;  // (PASS 2: the rest was written by pass 1)
        const size_t pix = (size_t)qy * width + px;
        if (keep) {
            a.state[pix] = make_float4(C0, C1, C2, T);
        } else if (a.out_bgra8) {
            a.out_bgra8[(size_t)orow * width + px] = pack_bgra8(C0, C1, C2, 1.0f - T);
        } else {
            a.out[(size_t)orow * width + px] = make_float4(C0, C1, C2, 1.0f - T);
        }
    };
    store(resA, keepA, qx, A0, A1, A2, TA);
    store(resB, keepB, qx + 8, B0, B1, B2, TB);
    if constexpr (PASS == 1) {
        if (lane == 0) {
            qr[qA] = openA ? 0xFFFFFFFFu : wendA;
            qr[qA + 1u] = openB ? 0xFFFFFFFFu : wendB;
            qr[16u + qA] = keepA ? 1u : 0u;
            qr[17u + qA] = keepB ? 1u : 0u;
            const uint32_t nk = (keepA ? 1u : 0u) + (keepB ? 1u : 0u);
            if (nk) (void)atomicAdd(a.open_q_count, (unsigned long long)nk);
        }
    }
}

#ifndef GS_COMPOSITE_STRIP  // A/B knob: 0 = the tile/live50 frames on composite_kernel
#define GS_COMPOSITE_STRIP 1
#endif

bool composite_strip(uint32_t bins) { return GS_COMPOSITE_STRIP && bins > kStripMinBins; }

template <int MODE, bool CAP, int SLAB = 0, int PASS = 0>
static hipError_t launch_mode(const CompositeArgs& a, hipStream_t st, hipEvent_t t0 = nullptr,
                              hipEvent_t t1 = nullptr) {
    if (a.nrows < 0 || a.nrows > a.tiles_y || (!a.rows && a.nrows != a.tiles_y)) return hipErrorInvalidValue;
    // (the strip kernel for launches of many bins; a small one -- a rank's band
    // at 8 ranks, a small frame -- on the tile kernel: there the slowest
    // workgroup bounds the launch, and a tile's walks one pixel per lane)
    constexpr bool kStripOk = (MODE == 0 || MODE == 1) && !CAP && SLAB == 0;
    const bool kStrip = kStripOk && composite_strip((uint32_t)(a.tiles_x * a.nrows));
    const uint32_t nwg = (uint32_t)((kStrip ? 2 : 4) * a.tiles_x * a.nrows);
    if (nwg == 0) {  // no owned tiles: the timing events still mark the (empty) stage
        if (t0 && hipEventRecord(t0, st) != hipSuccess) return hipGetLastError();
        if (t1 && hipEventRecord(t1, st) != hipSuccess) return hipGetLastError();
        return hipSuccess;
    }
    // t0/t1 (optional) are recorded by the dispatch packet itself
    if constexpr (kStripOk) {
        if (kStrip) {
            hipExtLaunchKernelGGL(composite_strip_kernel<MODE < 2 ? MODE : 0, PASS>, dim3(nwg), dim3(kTileThreads), 0, st,
                                  t0, t1, 0, a, nwg);
            return hipGetLastError();
        }
    }
    hipExtLaunchKernelGGL(composite_kernel<MODE, CAP, SLAB, PASS>, dim3(nwg), dim3(kTileThreads), 0, st, t0, t1, 0, a,
                          nwg);
    return hipGetLastError();
}

hipError_t launch_composite(const CompositeArgs& a, int mode, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
    const bool cap = a.cap > 0;
    if (cap && !a.thr) return hipErrorInvalidValue;
    if (a.order && (a.rows || a.compact || a.nrows != a.tiles_y)) return hipErrorInvalidValue;  // (whole frames only)
    if (a.pass) {  // depth-cut frames: tile / live50 rules, no cap, no depth slabs (owned rows allowed)
        if (cap || a.slab || (!a.out && !a.out_bgra8) || !a.qrec || !a.state ||
            (mode != 0 && mode != 1) || a.pass > 2 || (a.pass == 1 && !a.open_q_count))
            return hipErrorInvalidValue;
        if (a.pass == 1)
            return mode == 0 ? launch_mode<0, false, 0, 1>(a, st, t0, t1) : launch_mode<1, false, 0, 1>(a, st, t0, t1);
        return mode == 0 ? launch_mode<0, false, 0, 2>(a, st, t0, t1) : launch_mode<1, false, 0, 2>(a, st, t0, t1);
    }
    if (a.slab) {  // full frame, no cap
        if (cap || a.rows || a.compact || a.out_bgra8 || (a.slab == 1 ? !a.t_out : (!a.out || (a.slab_rank && !a.t_all))))
            return hipErrorInvalidValue;
        if (a.slab == 1) return mode == 0 ? launch_mode<0, false, 1>(a, st, t0, t1) : launch_mode<1, false, 1>(a, st, t0, t1);
        if (a.slab == 2) return mode == 0 ? launch_mode<0, false, 2>(a, st, t0, t1) : launch_mode<1, false, 2>(a, st, t0, t1);
        return hipErrorInvalidValue;
    }
    if (mode == 2) return cap || !a.dkey ? hipErrorInvalidValue : launch_mode<3, false>(a, st, t0, t1);  // MLAB
    if (mode == 0) return cap ? launch_mode<0, true>(a, st, t0, t1) : launch_mode<0, false>(a, st, t0, t1);
    return cap ? launch_mode<1, true>(a, st, t0, t1) : launch_mode<1, false>(a, st, t0, t1);
}

__global__ __launch_bounds__(256) void cut_finalize_kernel(const uint32_t* __restrict__ qrec,
                                                           const uint32_t* __restrict__ vals,
                                                           const uint32_t* __restrict__ dkey, uint32_t* __restrict__ cut,
                                                           uint32_t nbins, uint32_t tiles_x, const RowOwnership own,
                                                           uint32_t margin, const CutFallback fb) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    const bool any_open = fb.cut_in && *fb.open != 0ull;
    if (fb.cut_in && b == 0) {
        *fb.n = any_open ? *fb.npairs : 0u;
        *fb.kept = 0u;
        if (fb.host_open) *fb.host_open = *fb.open;
    }
    if (b >= nbins) return;
    if (!owns_bin_row(b / tiles_x, own)) {  // (another rank's bin: no record, no pairs)
        cut[b] = 0u;
        if (fb.cut_in) {
            fb.table[b] = 0xFFFFFFFFu;
            if (any_open) fb.ranges[b] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        }
        return;
    }
    const uint4* q = reinterpret_cast<const uint4*>(qrec + (size_t)b * kQrecWords);  // (the bin's 16 positions, 16 flags)
    uint32_t p = 0u, open = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint4 v = q[i];
        p = max(p, max(max(v.x, v.y), max(v.z, v.w)));
        const uint4 f = q[4 + i];
        open |= f.x | f.y | f.z | f.w;
    }
    uint32_t c = 0u;
    if (p == 0xFFFFFFFFu) c = 0xFFFFu;
    else if (p > 0u) c = min(dkey[vals[p - 1u]] + margin, 0xFFFFu);
    cut[b] = c;
    if (fb.cut_in) {
        fb.table[b] = open ? fb.cut_in[b] : 0xFFFFFFFFu;
        if (any_open) fb.ranges[b] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
    }
}

hipError_t launch_cut_finalize(const uint32_t* qrec, const uint32_t* vals, const uint32_t* dkey, uint32_t* cut_out,
                               uint32_t nbins, uint32_t tiles_x, const RowOwnership& own, uint32_t margin,
                               hipStream_t st, const CutFallback& fb) {
    if (nbins == 0) return hipSuccess;
    if (tiles_x == 0) return hipErrorInvalidValue;
    if (fb.cut_in && (!fb.open || !fb.npairs || !fb.table || !fb.n || !fb.kept || !fb.ranges))
        return hipErrorInvalidValue;
    cut_finalize_kernel<<<(nbins + 255) / 256, 256, 0, st>>>(qrec, vals, dkey, cut_out, nbins, tiles_x, own, margin,
                                                             fb);
    return hipGetLastError();
}

// Longest-first bin order (launch_order_bins): one 1024-lane workgroup, a
// counting sort of the bins into 128 cost buckets (log2 with two mantissa
// bits), costliest first.
__global__ __launch_bounds__(1024) void order_bins_kernel(const uint32_t* __restrict__ wcost, uint32_t nbins,
                                                          uint32_t* __restrict__ order) {
    constexpr int kB = 128;
    __shared__ uint32_t cnt[kB];
    __shared__ uint8_t bk[kOrderMaxBins];  // each bin's bucket, between the two phases
    static_assert(kOrderMaxBins + kB * 4 <= kLdsBytes, "order_bins_kernel's LDS exceeds a gfx950 workgroup's");
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    if (tid < kB) cnt[tid] = 0u;
    __syncthreads();
    for (uint32_t b = tid; b < nbins; b += 1024u) {
        const uint2 c2 = reinterpret_cast<const uint2*>(wcost)[b];  // (the bin's two halves)
        const uint32_t cost = c2.x + c2.y;
        uint32_t k = 0u;
        if (cost) {
            const uint32_t e = 31u - (uint32_t)__builtin_clz(cost);  // <= 31
            const uint32_t m = e >= 2u ? (cost >> (e - 2u)) & 3u : (cost << (2u - e)) & 3u;
            k = min(1u + e * 4u + m, (uint32_t)kB - 1u);
        }
        bk[b] = (uint8_t)k;
        atomicAdd(&cnt[k], 1u);
    }
    __syncthreads();
    if (tid < 64u) {  // exclusive offsets, costliest bucket first: one wave, two buckets a lane
        const uint32_t hi = cnt[kB - 1 - 2 * lane], lo = cnt[kB - 2 - 2 * lane];
        const uint32_t inc = wave_scan_dpp<false>(hi + lo);
        cnt[kB - 1 - 2 * lane] = inc - hi - lo;
        cnt[kB - 2 - 2 * lane] = inc - lo;
    }
    __syncthreads();
    for (uint32_t b = tid; b < nbins; b += 1024u) order[atomicAdd(&cnt[bk[b]], 1u)] = b;
}

__global__ __launch_bounds__(256) void cut_dilate_kernel(const uint32_t* __restrict__ cut, uint32_t* __restrict__ out,
                                                         uint32_t tiles_x, uint32_t tiles_y, int r) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= tiles_x * tiles_y) return;
    const int by = (int)(b / tiles_x), bx = (int)(b - (uint32_t)by * tiles_x);
    const int y0 = max(by - r, 0), y1 = min(by + r, (int)tiles_y - 1);
    const int x0 = max(bx - r, 0), x1 = min(bx + r, (int)tiles_x - 1);
    uint32_t m = 0u;
    for (int y = y0; y <= y1; ++y)
        for (int x = x0; x <= x1; ++x) m = max(m, cut[(uint32_t)y * tiles_x + (uint32_t)x]);
    out[b] = m;
}

hipError_t launch_cut_dilate(const uint32_t* cut, uint32_t* out, uint32_t tiles_x, uint32_t tiles_y, int r,
                             hipStream_t st) {
    const uint32_t n = tiles_x * tiles_y;
    if (n == 0) return hipSuccess;
    if (!cut || !out || r < 0) return hipErrorInvalidValue;
    cut_dilate_kernel<<<(n + 255) / 256, 256, 0, st>>>(cut, out, tiles_x, tiles_y, r);
    return hipGetLastError();
}

hipError_t launch_order_bins(const uint32_t* wcost, uint32_t nbins, uint32_t* order, hipStream_t st) {
    if (nbins == 0) return hipSuccess;
    if (!wcost || !order || nbins > kOrderMaxBins) return hipErrorInvalidValue;
    order_bins_kernel<<<1, 1024, 0, st>>>(wcost, nbins, order);
    return hipGetLastError();
}

#ifdef GS_COMPOSITE_TRACE
extern "C" int gs_debug_composite_trace(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_comp_trace), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_cap_threshold(const CompositeArgs& a, hipStream_t st) {
    if (a.cap <= 0 || !a.thr_out) return hipErrorInvalidValue;
    return launch_mode<2, false>(a, st);
}

}  // namespace gs
