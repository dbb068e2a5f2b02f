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

#ifdef GS_COMPOSITE_COUNTERS
// Debug build only (-DGS_COMPOSITE_COUNTERS): per-wave work counters.
__device__ unsigned long long g_cc[20];
__device__ uint32_t g_tile_fetch[1u << 16];  // per tile (bin * 4 + tile of the bin): records fetched
#define GS_CC(i, v) (void)atomicAdd(&g_cc[i], (unsigned long long)(v))
#else
#define GS_CC(i, v) (void)0
#endif
#ifdef GS_COMPOSITE_TIMERS
// Debug build only (-DGS_COMPOSITE_TIMERS): shader-clock cycles per wave
// spent in each phase of the batch loop, summed over waves (tools/composite_counters.py).
__device__ unsigned long long g_ct[8];
#define GS_CT_DECL unsigned long long ct_acc[6] = {0, 0, 0, 0, 0, 0}, ct_t = clock64(), ct_t0 = ct_t
#define GS_CT(i)                                   \
    do {                                           \
        const unsigned long long ct_n = clock64(); \
        ct_acc[i] += ct_n - ct_t;                  \
        ct_t = ct_n;                               \
    } while (0)
#define GS_CT_FLUSH()                                                                            \
    do {                                                                                         \
        if (lane == 0) {                                                                         \
            for (int ci = 0; ci < 6; ++ci) (void)atomicAdd(&g_ct[ci], ct_acc[ci]);               \
            (void)atomicAdd(&g_ct[6], clock64() - ct_t0);                                        \
            (void)atomicAdd(&g_ct[7], 1ull);                                                     \
        }                                                                                        \
    } while (0)
#else
#define GS_CT_DECL (void)0
#define GS_CT(i) (void)0
#define GS_CT_FLUSH() (void)0
#endif
#ifdef GS_COMPOSITE_TRACE
// Debug build only (-DGS_COMPOSITE_TRACE): per wave {start, end} realtime
// (100 MHz), HW_ID and XCC_ID, for the occupancy / tail analysis of
// tools/composite_trace.py.
constexpr uint32_t kTraceMax = 1u << 18;
__device__ uint4 g_trace[kTraceMax];
#define GS_TR_DECL const uint32_t tr_t0 = (uint32_t)__builtin_amdgcn_s_memrealtime()
#define GS_TR_FLUSH()                                                                                    \
    do {                                                                                                 \
        const uint32_t tr_t1 = (uint32_t)__builtin_amdgcn_s_memrealtime();                              \
        const uint32_t slot = blockIdx.x * 4u + (threadIdx.x >> 6);                                      \
        if ((threadIdx.x & 63u) == 0 && slot < kTraceMax)                                                \
            g_trace[slot] = make_uint4(tr_t0, tr_t1, __builtin_amdgcn_s_getreg((31 << 11) | 4),          \
                                       __builtin_amdgcn_s_getreg((31 << 11) | 20));                      \
    } while (0)
#else
#define GS_TR_DECL (void)0
#define GS_TR_FLUSH() (void)0
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

// PASS (two-slab frames; modes 0/1, no cap, fp32 output):
// 1 = the first slab, leaving the state (C, T) of every tile with an open
// pixel; 2 = the second slab, resuming those tiles only.
template <int MODE, bool CAP, int SLAB = 0, int PASS = 0>
__global__ __launch_bounds__(256, MODE == 3 ? 4 : 8) void composite_kernel(CompositeArgs a, uint32_t nwg) {
    constexpr bool kIds = CAP || MODE == 2;  // the body needs the splat id
    static_assert(PASS == 0 || ((MODE == 0 || MODE == 1) && !CAP && SLAB == 0), "two-slab passes: tile/live50 rules");
    __shared__ StagedRec srec[kTileThreads];
    __shared__ uint16_t wlist[4][kTileThreads];  // per wave: slot byte offsets
    __shared__ uint8_t sqm[kTileThreads];  // per staged record: the quadrants it may reach
    __shared__ uint32_t sopen[4];          // per wave: pixels still open after its last walk
    __shared__ uint32_t sopen_end[4];      // (PASS 1) the same at the end of the list

    // XCD-aware bijective remap (blocks b and b+8 share an XCD,
    // cdna_hip_programming.md §5, T1).
    GS_TR_DECL;
    const uint32_t orig = blockIdx.x;
#if defined(GS_XCD_MAP) && GS_XCD_MAP == 0
    // A/B: each XCD a contiguous run of tiles (a band of bin rows)
    const uint32_t xcd = orig & 7u, q8 = nwg >> 3, r8 = nwg & 7u;
    const uint32_t wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
#else
    // Bins dealt round-robin over the XCDs, a bin's 4 tiles on one XCD (they
    // share its list through that L2).  Measured against giving each XCD a
    // contiguous band of bin rows: -2 % composite, since the bands' costs
    // differ and the launch ends with the slowest XCD.
    const uint32_t full = nwg & ~31u;
    const uint32_t kk = orig >> 3;
    const uint32_t wg = orig < full ? 32u * (kk >> 2) + 4u * (orig & 7u) + (kk & 3u) : orig;
#endif

    // Grid covers only the owned bin rows.  The four 16x16
    // tiles of a bin are consecutive workgroups (same XCD / L2).
    const uint32_t per_row = 4u * (uint32_t)a.tiles_x;
    const int owned_row = (int)(wg / per_row);
    const uint32_t k4 = wg - (uint32_t)owned_row * per_row;
    const int bx = (int)(k4 >> 2);
    const int by = a.rows ? (int)a.rows[owned_row] : owned_row;
    const int tx = 2 * bx + (int)(k4 & 1u), ty = 2 * by + (int)((k4 >> 1) & 1u);
    const int width = a.width, height = a.height;
    const uint32_t tile_flag = (uint32_t)(by * a.tiles_x + bx) * 4u + (k4 & 3u);  // (two-slab open4 slot)
    if constexpr (PASS == 2) {
        if (a.open4[tile_flag] == 0) return;  // (whole workgroup) every pixel finished in the first slab
    }
    const int tid = threadIdx.x;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t lane = tid & 63;
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
    uint2 rg = decode_range(a.ranges[by * a.tiles_x + bx]);
    if (tx0 >= (uint32_t)width || ty0 >= (uint32_t)height) rg.y = rg.x;
    // Pixels outside the frame start finished (T = 0): for the tile and live50
    // rules "finished" is then just the break test on T itself, so no
    // separate per-lane flag is carried through the loop.
    float T = inside ? 1.0f : 0.0f;  // transmittance (tile rule: T = 1 - A)
    float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
    // compact = owned bin rows stacked (multi-GPU band buffer)
    const int orow = a.compact ? owned_row * kBin + (py - by * kBin) : py;
    if constexpr (PASS == 2) {
        if (inside) {  // the state the first slab left: the same registers, resumed
            const float4 st = a.out[(size_t)orow * width + px];
            C0 = st.x;
            C1 = st.y;
            C2 = st.z;
            T = st.w;
        }
    }
    bool done = !inside;  // MODE 2 / 3
#ifdef GS_COMPOSITE_COUNTERS
    uint32_t cc_n4 = 0, cc_n2 = 0, cc_nl = 0;
    uint32_t cc_b4 = 0, cc_bl = 0, cc_br = 0, cc_be = 0;  // per batch
    __shared__ uint16_t cc_bmr[kTileThreads], cc_bme[kTileThreads];
    // this lane's 4x4 block of the tile (bit row * 4 + column) and its lane group
    const uint32_t cc_blk = ((wave >> 1) * 2u + (lane >> 5)) * 4u + (wave & 1u) * 2u + ((lane >> 2) & 1u);
    const uint64_t cc_g4 = ((lane >> 5) ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull) &
                           ((lane & 4u) ? 0xF0F0F0F0F0F0F0F0ull : 0x0F0F0F0F0F0F0F0Full);
#endif
    uint32_t thr = 0xFFFFFFFFu;  // CAP: last admitted id; MODE 2: result
    int cnt = 0;                 // MODE 2: covering fragments seen
    if constexpr (CAP) {
        if (inside) thr = a.thr[(size_t)py * width + px];
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
#ifdef GS_COMPOSITE_COUNTERS
    auto cc_rec = [&](uint32_t off) {
        const uint32_t k = off / (uint32_t)sizeof(StagedRec);
        const bool gopen = (__ballot(!finished()) & cc_g4) != 0;
        cc_br += (gopen && ((cc_bmr[k] >> cc_blk) & 1u)) ? 1u : 0u;
        cc_be += (gopen && ((cc_bme[k] >> cc_blk) & 1u)) ? 1u : 0u;
    };
    auto cc_batch = [&]() {
        if constexpr (MODE == 0) {
            uint32_t x[4] = {cc_b4, cc_bl, cc_br, cc_be};
            for (int o = 32; o > 0; o >>= 1)
                for (int q = 0; q < 4; ++q) x[q] = max(x[q], (uint32_t)__shfl_xor((int)x[q], o, 64));
            if (lane == 0) {
                GS_CC(1, x[0]);
                GS_CC(2, x[1]);
                GS_CC(14, x[2]);
                GS_CC(15, x[3]);
            }
        }
        cc_b4 = cc_bl = cc_br = cc_be = 0;
    };
#endif

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
#ifdef GS_COMPOSITE_COUNTERS
            {
                const uint64_t m = __ballot(in);
                if (lane == 0 && m) GS_CC(4, 1);
                if (lane == 0) GS_CC(7, __popcll(m));
                // footprint estimates: open / covered lanes per body, and per
                // 4x4 / 8x4 lane group the bodies it would walk (covered lane
                // and an open lane in the group), per lane its own walk
                const uint64_t mo = __ballot(!finished()), mc = __ballot(covered);
                if (lane == 0) GS_CC(8, __popcll(mo));
                if (lane == 0) GS_CC(9, __popcll(mc));
                const uint64_t g4 = ((lane >> 5) ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull) &
                                    ((lane & 4u) ? 0xF0F0F0F0F0F0F0F0ull : 0x0F0F0F0F0F0F0F0Full);
                const uint64_t g2 = (lane >> 5) ? 0xFFFFFFFF00000000ull : 0xFFFFFFFFull;
                cc_n4 += ((mo & g4) && (mc & g4)) ? 1u : 0u;
                cc_n2 += ((mo & g2) && (mc & g2)) ? 1u : 0u;
                cc_nl += in ? 1u : 0u;
                cc_b4 += ((mo & g4) && (mc & g4)) ? 1u : 0u;
                cc_bl += in ? 1u : 0u;
            }
#endif
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
    if (lane == 0) GS_CC(0, 1);
    if (tid == 0) GS_CC(6, rg.y - rg.x);
    // records this workgroup fetched: the first batch, then one prefetched
    // batch per batch it composites (the early-out stops both)
    const uint32_t len = rg.y > rg.x ? rg.y - rg.x : 0u;  // (empty bins: {~0, 0})
    uint32_t fetched = len < (uint32_t)kTileThreads ? len : (uint32_t)kTileThreads;
    GS_CT_DECL;
    for (uint32_t b = rg.x; b < rg.y; b += kTileThreads) {
        GS_CT(5);
#ifdef GS_AB_SYNC_COUNT
        if (__syncthreads_count(!finished()) == 0) break;
#else
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
#endif
        GS_CT(0);
        if (rg.y - b > (uint32_t)kTileThreads) {
            const uint32_t left = rg.y - b - (uint32_t)kTileThreads;
            fetched += left < (uint32_t)kTileThreads ? left : (uint32_t)kTileThreads;
        }
        if (tid == 0) GS_CC(5, 1);
        // the wave's gathered chunks into their records' slots (raw layout)
#pragma unroll
        for (int i = 0; i < 3; ++i)
            (cp[i] == 0 ? srec[64u * wave + ck[i]].a : cp[i] == 1 ? srec[64u * wave + ck[i]].b
                                                                   : srec[64u * wave + ck[i]].c) = rc[i];
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
            {
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
#ifdef GS_COMPOSITE_COUNTERS
                {
                    const uint32_t cm = a.cell_mask ? rect_cell_mask(wlo, whi) : 0u;
                    const float eu = 1.5f * (fabsf(st.a.z) + fabsf(st.a.w)), ev = 1.5f * (fabsf(st.b.x) + fabsf(st.b.y));
                    uint32_t bmr = 0, bme = 0;
                    for (uint32_t j = 0; j < 4; ++j)
                        for (uint32_t i = 0; i < 4; ++i) {
                            const uint32_t bx0 = tx0 + 4u * i, by0 = ty0 + 4u * j;
                            bool hit = !(x1 < bx0 || x0 > bx0 + 3u) && !(y1 < by0 || y0 > by0 + 3u);
                            const uint32_t dcx = (bx0 >> 3) - (x0 >> 3), dcy = (by0 >> 3) - (y0 >> 3);
                            if (dcx < 4u && dcy < 4u && ((cm >> (dcy * 4u + dcx)) & 1u)) hit = false;
                            const float cxl = 4.0f * (float)i + 2.0f, cyl = 4.0f * (float)j + 2.0f;
                            const float uc = st.a.x + st.a.z * cxl + st.a.w * cyl;
                            const float vc = st.a.y + st.b.x * cxl + st.b.y * cyl;
                            const float tu = fmaxf(fabsf(uc) - eu, 0.0f), tv = fmaxf(fabsf(vc) - ev, 0.0f);
                            const bool he = fmaxf(tu, tv) <= kBoxS * 1.001f && tu * tu + tv * tv <= kQMaxS * 1.001f;
                            bmr |= hit ? 1u << (4u * j + i) : 0u;
                            bme |= (hit && he) ? 1u << (4u * j + i) : 0u;
                        }
                    cc_bmr[tid] = (uint16_t)bmr;
                    cc_bme[tid] = (uint16_t)bme;
                    // staged records, and those whose rect reaches the tile at all
                    GS_CC(16, 1);
                    if (qm) GS_CC(17, 1);
                }
#endif
            }
        }
        GS_CT(1);
        __syncthreads();
        GS_CT(2);
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
            for (uint32_t k0 = 0; k0 < cnt_b; k0 += 64) {
                const uint32_t k = k0 + lane;
                const bool hit = k < cnt_b && ((sqm[k] >> wave) & 1u);
                const uint64_t m = __ballot(hit);
                if (hit) wlist[wave][nl + mbcnt(m)] = (uint16_t)(k * sizeof(StagedRec));
                nl += (uint32_t)__popcll(m);
            }
        }
        wave_lds_sync();  // wlist[wave] is only touched by this wave
        GS_CT(3);
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
#ifdef GS_COMPOSITE_COUNTERS
                cc_rec(wlist[wave][i]);
#endif
                body_v(a0, b0, c0, i0, (_Float16)0.0f);
#ifdef GS_COMPOSITE_COUNTERS
                cc_rec(wlist[wave][i + 1]);
#endif
                body_v(a1, b1, c1, i1, (_Float16)0.0f);
            }
            if (i < nl && __ballot(!finished()) != 0) {
#ifdef GS_COMPOSITE_COUNTERS
                cc_rec(wlist[wave][i]);
#endif
                body(wlist[wave][i++]);
            }
        }
        if (lane == 0) GS_CC(3, i);
#ifdef GS_COMPOSITE_COUNTERS
        cc_batch();
#endif
        GS_CT(4);
    }
    GS_CT_FLUSH();
    GS_TR_FLUSH();
#ifdef GS_COMPOSITE_COUNTERS
    if constexpr (MODE == 0) {
        uint32_t x4 = cc_n4, x2 = cc_n2, xl = cc_nl, sl = cc_nl;
        for (int o = 32; o > 0; o >>= 1) {
            x4 = max(x4, (uint32_t)__shfl_xor((int)x4, o, 64));
            x2 = max(x2, (uint32_t)__shfl_xor((int)x2, o, 64));
            xl = max(xl, (uint32_t)__shfl_xor((int)xl, o, 64));
            sl += (uint32_t)__shfl_xor((int)sl, o, 64);
        }
        if (lane == 0) {
            GS_CC(10, x4);
            GS_CC(11, x2);
            GS_CC(12, xl);
            GS_CC(13, sl);
        }
    }
#endif
    if (tid == 0 && a.fetched) (void)atomicAdd(a.fetched, (unsigned long long)fetched);
#ifdef GS_COMPOSITE_COUNTERS
    if (tid == 0 && MODE == 0 && tile_flag < (1u << 16)) g_tile_fetch[tile_flag] = fetched;
#endif
    bool keep_state = false;
    if constexpr (PASS == 1) {
        // does any pixel of the tile remain open for the second slab?
        const bool open_w = __ballot(!finished()) != 0;
        if (lane == 0) sopen_end[wave] = open_w ? 1u : 0u;
        __syncthreads();
        const uint4 o = *reinterpret_cast<const uint4*>(sopen_end);
        keep_state = (o.x | o.y | o.z | o.w) != 0u;
        if (tid == 0) {
            a.open4[tile_flag] = keep_state ? 1 : 0;
            if (keep_state && a.open_tiles) (void)atomicAdd(a.open_tiles, 1ull);
        }
    }
    if (!inside) return;
    if constexpr (PASS == 1) {
        if (keep_state) {  // (C, T) for the second slab; final pixels otherwise
            a.out[(size_t)orow * width + px] = make_float4(C0, C1, C2, T);
            return;
        }
    }
    if constexpr (SLAB == 1) {
        a.t_out[(size_t)py * width + px] = T;
    } else if constexpr (SLAB == 2) {
        // contributions: colour and the alpha this slab adds (sum over slabs)
        a.out[(size_t)py * width + px] = make_float4(C0, C1, C2, T0 - T);
    } else if constexpr (MODE == 2) {
        a.thr_out[(size_t)py * width + px] = thr;
    } else {
        const float4 o = MODE == 3 ? kb.resolve() : make_float4(C0, C1, C2, 1.0f - T);
        if (a.out_bgra8)
            a.out_bgra8[(size_t)orow * width + px] = pack_bgra8(o.x, o.y, o.z, o.w);
        else
            a.out[(size_t)orow * width + px] = o;
    }
}

template <int MODE, bool CAP, int SLAB = 0, int PASS = 0>
static hipError_t launch_mode(const CompositeArgs& a, hipStream_t st, hipEvent_t t0 = nullptr,
                              hipEvent_t t1 = nullptr) {
    if (a.nrows < 0 || a.nrows > a.tiles_y || (!a.rows && a.nrows != a.tiles_y)) return hipErrorInvalidValue;
    const uint32_t nwg = (uint32_t)(4 * a.tiles_x * a.nrows);
    if (nwg == 0) {  // no owned tiles: the timing events still mark the (empty) stage
        if (t0 && hipEventRecord(t0, st) != hipSuccess) return hipGetLastError();
        if (t1 && hipEventRecord(t1, st) != hipSuccess) return hipGetLastError();
        return hipSuccess;
    }
    // t0/t1 (optional) are recorded by the dispatch packet itself
    hipExtLaunchKernelGGL(composite_kernel<MODE, CAP, SLAB, PASS>, dim3(nwg), dim3(kTileThreads), 0, st, t0, t1, 0, a,
                          nwg);
    return hipGetLastError();
}

hipError_t launch_composite(const CompositeArgs& a, int mode, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
    const bool cap = a.cap > 0;
    if (cap && !a.thr) return hipErrorInvalidValue;
    if (a.pass) {  // two-slab frames: tile / live50 rules, fp32 output, no cap, no depth slabs
        if (cap || a.slab || a.out_bgra8 || !a.out || !a.open4 || (mode != 0 && mode != 1) || a.pass > 2)
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

hipError_t launch_cap_threshold(const CompositeArgs& a, hipStream_t st) {
    if (a.cap <= 0 || !a.thr_out) return hipErrorInvalidValue;
    return launch_mode<2, false>(a, st);
}

}  // namespace gs

#ifdef GS_COMPOSITE_TIMERS
extern "C" int gs_debug_composite_timers(unsigned long long* out) {
    unsigned long long zero[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_ct), sizeof zero) != hipSuccess) return 1;
    return hipMemcpyToSymbol(HIP_SYMBOL(gs::g_ct), zero, sizeof zero) != hipSuccess;
}
#endif
#ifdef GS_COMPOSITE_TRACE
extern "C" int gs_debug_composite_trace(void* out, unsigned n) {  // n uint4 entries
    if (n > gs::kTraceMax) n = gs::kTraceMax;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_trace), (size_t)n * 16) != hipSuccess;
}
#endif
#ifdef GS_COMPOSITE_COUNTERS
extern "C" int gs_debug_composite_tile_fetch(uint32_t* out, unsigned n) {
    if (n > (1u << 16)) n = 1u << 16;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_tile_fetch), (size_t)n * 4) != hipSuccess;
}
extern "C" int gs_debug_composite_counters(unsigned long long* out) {
    unsigned long long zero[20] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gs::g_cc), sizeof zero) != hipSuccess) return 1;
    return hipMemcpyToSymbol(HIP_SYMBOL(gs::g_cc), zero, sizeof zero) != hipSuccess;
}
#endif
