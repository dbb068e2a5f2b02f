// renderer.cpp — libgsplat C-ABI: scene ownership, HBM layout, frame pipeline.
//
// Replaces InstancedSplatRenderer's host side (src/instanced_splat_renderer.mm):
//   ctor (:339-393)        -> gs_create*: PLY load, crop, host SoA
//   initialize (:399-422)  -> gs_initialize: HBM SoA upload (no shader compile,
//                             no hot-reload watcher: kernels are AOT for gfx950)
//   render (:424-578)      -> gs_render: preprocess -> scan -> duplicate ->
//                             radix sort -> tile ranges -> composite, all on
//                             the caller's stream, into a caller-owned fp32
//                             RGBA framebuffer (no 504 B/pixel list buffer,
//                             no per-frame ~1 GB clear).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <functional>
#include <vector>

#include "../kernels/gs_kernels.h"
#include "gsplat.h"
#include "gsplat/ply_loader.h"
#include "gs_internal.h"
#include "scene_io.h"

namespace {

thread_local std::string g_last_error;

gs_status fail(gs_status s, const std::string& msg) {
    g_last_error = msg;
    return s;
}

#define GS_HIP(expr)                                                                               \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            return fail(e_ == hipErrorOutOfMemory ? GS_ERR_OOM : GS_ERR_DEVICE,                    \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                        \
    } while (0)

#ifndef GS_DUP_FILTER_COUNT  // A/B knob: 1 = a depth-cut frame's duplicate counts the filtered pass's digits
#define GS_DUP_FILTER_COUNT 0
#endif
#ifndef GS_DUP_FLAG  // A/B knob: 1 = the bin-first duplicate marks the pairs behind their cut (kBehindFlag)
#define GS_DUP_FLAG 1
#endif
#ifndef GS_CUT_DILATE_AHEAD  // A/B knob: 1 = the next frame's dilated cuts are made by this frame's tail
#define GS_CUT_DILATE_AHEAD 1
#endif
#ifndef GS_FB_LDS  // A/B knob: 1 = the fallback lists' filter tests an LDS copy of its table
#define GS_FB_LDS 1
#endif
#ifndef GS_HOST_POLL  // A/B knob: 1 = the host polls the pair count's sequence word instead of an event
#define GS_HOST_POLL 0
#endif
#ifndef GS_HOST_SET_WAIT  // A/B knob: 1 = the host waits for a buffer set's last reader (no GPU wait packet)
#define GS_HOST_SET_WAIT 1
#endif
#ifndef GS_BAND_LOCAL  // A/B knob: 1 = contiguous band frames bin without an owner table (gs_handle::band_local)
#define GS_BAND_LOCAL 1
#endif
#ifndef GS_DUP_FRONT  // A/B knob: 1 = a bin-first depth-cut frame emits only its front pairs (launch_front_count)
#define GS_DUP_FRONT 1
#endif
#ifndef GS_DUP_FRONT_DILATED  // A/B knob: 1 = front-only emission also while the set's cuts are dilated (moving camera)
#define GS_DUP_FRONT_DILATED 0
#endif
#ifndef GS_AUX_TOTALS  // A/B knob: 1 = a look-back frame's totals kernel runs on a stream of its own, beside the duplicate
#define GS_AUX_TOTALS 1
#endif
#ifndef GS_AUX_ALL  // A/B knob: 1 = every depth-cut frame (not only front-only ones) gets look-back + aux totals
#define GS_AUX_ALL 0
#endif
#ifndef GS_DUP_LOOKBACK  // A/B knob: 1 = the front-only duplicate finds its offsets by look-back (no count kernel)
#define GS_DUP_LOOKBACK 1
#endif
#ifndef GS_DUP_FRONT_COUNT  // A/B knob: 1 = the front-only duplicate counts the first sort pass's digits
#define GS_DUP_FRONT_COUNT 1
#endif

struct DevBuf {
    void* ptr = nullptr;
    size_t bytes = 0;
    void release() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        bytes = 0;
    }
    // Grows monotonically (never shrinks; reused across frames).
    hipError_t reserve(size_t want) {
        if (want <= bytes) return hipSuccess;
        release();
        size_t b = std::max<size_t>(want + want / 8, 256);
        b = (b + 255) & ~size_t(255);
        hipError_t e = hipMalloc(&ptr, b);
        if (e == hipSuccess) bytes = b;
        return e;
    }
    template <typename T>
    T* as() const { return static_cast<T*>(ptr); }
};

using gsio::sh_coeffs;

}  // namespace

// (gs_internal.h) the calling thread's gs_last_error() text
void gs_set_last_error(const std::string& msg) { g_last_error = msg; }



struct gs_handle {
    gs_options opt{};
    // host copy of the scene (post-crop) in the HBM plane layout (scene_io.h)
    int64_t n = 0;
    gsio::HostPlanes hp;
    // device
    int device = -1;
    bool initialized = false;
    DevBuf p0, p1, p2, p3, sh4, sh1;
    // per-frame scratch
    DevBuf rec, dkey, rlo, rhi, offsets, partials, keys, vals, tkeys, tvals, sort_scratch, ranges, fb, thr;
    DevBuf dsk, dso, dsl, dsh, dtk, dto, dtl, dth;  // depth sort: keys, order, rect lo/hi (+ ping-pong)
    DevBuf xmask, xcounts, xtotal;  // multi-GPU exchange
    // depth-slab frames: full-frame ownership; the colour pass
    // (gs_slab_composite) reuses the bin lists of the transmittance pass
    bool slab_frame = false;
    bool slab_lists = false;
    int32_t slab_w = 0, slab_h = 0;  // frame of the last gs_slab_project
    uint32_t* host_xtotal = nullptr;                                    // pinned, kMaxWorld
    uint64_t* host_total = nullptr;  // pinned, mapped: the scan writes P here directly
    uint64_t* dev_total = nullptr;   // its device-side address
    hipEvent_t ev[14] = {};  // stage boundaries 0..7; 8 = exchange done (shard frames); 9..13 second slab
    // stage_timing 2: packet events (preprocess start/stop, composite start/stop)
    // in a ring of per-frame slots, read without stalling the frames
    static constexpr int kKevRing = 64;
    // [0, 1] preprocess start/stop, [2, 3] composite start/stop
    hipEvent_t kev[kKevRing][4] = {};
    int64_t kev_frames = 0;    // frames recorded since stage timing was (re)set
    int kev_slot = 0;          // slot of the frame being enqueued
    bool kev_pending = false;  // last frame's kernel times not yet copied into stats
    bool shard_frame = false;
    // a band frame whose owned rows are contiguous: the projection clips the
    // rects to the band, so the binning needs no owner table (every pair it
    // emits lies in an owned row) and runs the single-GPU chain (fused scan,
    // cooperative duplicate, depth cuts); the composite keeps the table
    bool band_local = false;
    bool events = false;
    uint32_t* last_keys = nullptr;  // sorted pair arrays of the last frame
    uint32_t* last_vals = nullptr;
    uint32_t* last_tmp_keys = nullptr;  // the bin sort's other buffers (free once it is done)
    uint32_t* last_tmp_vals = nullptr;
    int last_key_bits = 0;              // bin id bits of the pair keys (depth key above, bin-first)
    bool bin_first_frame = false;       // the last frame used the bin-first order
    DevBuf seg_sample;                  // per-bin depth sort sample (launch_bin_depth_sort)
    DevBuf npairs;                      // P on the device (0 when it overflows the pair buffers)
    DevBuf fetch;                       // per buffer set: [2 set] records the composite fetched, [2 set + 1] open tiles (u64)
    int stats_set = -1;                 // buffer set of the frame in `stats` (its fetch counter)
    int64_t stats_fixed_bytes = 0;      // composite bytes besides the records: range words + output
    hipEvent_t totals_ev = nullptr;     // P is in host_total
    hipStream_t aux = nullptr;          // (GS_AUX_TOTALS) a look-back frame's totals kernel
    // gs_shard_render_split: the rank render's composite on a stream of its
    // own; comp_done follows its tail, the next rank render's lists wait for
    // it; the projection then leaves the fetch counters to the render
    hipEvent_t comp_done = nullptr;
    bool split_render = false;
    hipEvent_t xcount_ev = nullptr;  // (pack_exchange) the destination counts are in host_xtotal
    hipEvent_t pre_ev = nullptr;        // recorded by that frame's preprocess dispatch
    unsigned long long totals_seq = 0;  // (GS_HOST_POLL) the last totals kernel's sequence number, host_total[5]
    struct OrderModel {                 // inputs of the binning-order choice (bin_first_order)
        int32_t w = 0, h = 0;
        int64_t n = -1;
        uint64_t frame_pairs = 0;       // P of the last scanned frame
        uint64_t sample_pairs = 0;      // P of the last bin-first frame (the sample's frame)
        double long_share = 0.0;        // share of its pairs in lists longer than kSegLdsMax
        uint64_t wmax = 0, wmax_pairs = 0;  // a bin-first frame's wave-max emission work and its P
    } order;
    gs_stats stats{};
    // Bin-first single-GPU frames: the preprocess sums each scan block's
    // pairs into ppart (PreFuse), prepared by render_frame (prepare_lists)
    struct ListPrep {
        bool ok = false;
        bool front = false;  // the frame emits only its front pairs (launch_front_count; depth cuts)
        bool aux = false;    // (look-back) its totals kernel on the aux stream, after the preprocess's pre_ev
        uint32_t cap = 0;
        gs::PassCounts pc;
    } fused_prep;
    bool front_last = false;   // the frame in `stats` emitted only its front pairs (its fallback regenerates)
    uint64_t pairs_emitted = 0;  // pairs the frame's duplicate wrote (= stats.pairs unless front_last)
    static constexpr uint64_t kEmittedOnDevice = ~0ull;  // (look-back: in npairs[set], read by gs_last_stats)
    DevBuf fbpart, fbtot;      // front_last frames' fallback pair scan (2 rows per block; totals)
    DevBuf ppart;
    size_t ppart_words = 0;
    bool ppart_dirty = false;  // a fused preprocess ran without its scan (error path): clear first
    bool fused_last = false;   // the frame in `stats` scanned fused block sums
    int order_pick = -1;       // binning order decided before the preprocess (-1: not yet)
    // multi-GPU shard config
    int32_t rank = 0, world = 1;
    std::vector<uint8_t> custom_owner;  // gs_shard_set_rows (empty: default ranges)
    std::vector<uint8_t> owner_host;    // table currently on the device
    std::vector<uint16_t> rows_host;    // this rank's owned bin rows
    DevBuf owner_dev, rows_dev;
    gs::CompositeArgs slab_ca{};
    // frames_in_flight 2: projection/sort stream, and the second set of the
    // buffers a frame's composite reads (swapped into the members above)
    hipStream_t side = nullptr;
    hipEvent_t sorted_ev = nullptr;        // side stream -> composite stream hand-off
    hipEvent_t set_free[2] = {};           // last use of each buffer set on a composite stream
    int set = 0;
    bool last_pipe = false;  // the last frame ran pipelined (a switch into pipelining waits for the caller's stream)
    DevBuf alt_rec, alt_dkey, alt_keys, alt_vals, alt_tkeys, alt_tvals, alt_ranges, alt_thr, alt_rlo, alt_rhi,
        alt_qrec, alt_fkeys, alt_fvals;
    // Depth cuts (gs_options.depth_split).  cutbuf, per buffer
    // set, two per-bin cut tables: a frame's front lists keep the pairs at or
    // ahead of the cuts its set's previous frame (two frames back) left in
    // one; its composite writes the quadrant records (qrec: cut positions and
    // open flags, one set each, swapped) and launch_cut_finalize turns them
    // into the other table; then the roles swap.  fkeys/fvals (per set): the
    // front lists, sorted out of keys/vals, which keep every pair of the frame
    // for the fallback lists (its bins with an open quadrant, behind their
    // cuts: fbtab, fbn, sorted with scratch2; composite stream only).
    // cstate: the open quadrants' pixel states.  kept: per set, the front
    // lists' pairs [set] and the fallback lists' [2 + set] (gs_last_stats).
    // cutord: per buffer set, two bin-order tables beside the cut tables
    // (the same roles and phase): the composite's longest-first dispatch
    // order (CompositeArgs::order), single-GPU frames only.
    // cutdil: per set, the dilated copy of the cut table a moving camera's
    // frame reads (cut_r[set] > 0); cut_r: the set's dilation radius in bins,
    // raised while its frames leave quadrants open (the counts come back in
    // host_total[6 + set], written by cut_finalize) and lowered again after
    // kCutCalm frames with none.  dil_r: the radius of the set's table in
    // cutdil dilated ahead, by the tail of the frame that wrote the cuts (on
    // the composite stream, off the next frame's critical path); 0 = none.
    DevBuf qrec, cutbuf, cutord, cutdil, wcost, cstate, fkeys, fvals, fbtab, fbn, scratch2, kept;
    int cut_r[2] = {0, 0};
    int cut_calm[2] = {0, 0};
    int dil_r[2] = {0, 0};
    int dil_slot[2] = {0, 0};    // per set: cutdil slot the set's next frame reads
    int dil_wslot[2] = {1, 1};   // per set: slot the current frame's tail dilates ahead into
    uint32_t cut_bins = 0;       // bins per table in cutbuf
    int32_t cut_w = 0, cut_h = 0, cut_mode = -1;
    int cut_phase[2] = {0, 0};   // per set: which table the next frame reads
    bool cut_valid[2] = {false, false};
    bool cut_frame = false;      // the frame in `stats` used depth cuts
    bool cut_pending = false;    // the frame being enqueued is a depth-cut frame (render_frame)
    const uint32_t* cut_in = nullptr;  // (its cuts; null: none yet, every pair in its lists)
    uint32_t* cut_out = nullptr;
    const uint32_t* ord_in = nullptr;  // (its bin order, valid with cut_in)
    uint32_t* ord_out = nullptr;
    bool cut_lists = false;      // the frame in `stats` filtered its lists at the cuts (front pairs: kept[set])
    uint32_t pair_cap = 0;       // pair capacity of the set of the last build_bin_lists
    uint32_t* cut_table(int set, int role) const {
        return cutbuf.as<uint32_t>() + (size_t)(2 * set + ((cut_phase[set] + role) & 1)) * cut_bins;
    }
    uint32_t* order_table(int set, int role) const {
        return cutord.as<uint32_t>() + (size_t)(2 * set + ((cut_phase[set] + role) & 1)) * cut_bins;
    }
    void swap_sets() {
        std::swap(rec, alt_rec);
        std::swap(dkey, alt_dkey);
        std::swap(keys, alt_keys);
        std::swap(vals, alt_vals);
        std::swap(tkeys, alt_tkeys);
        std::swap(tvals, alt_tvals);
        std::swap(ranges, alt_ranges);
        std::swap(thr, alt_thr);
        std::swap(rlo, alt_rlo);
        std::swap(rhi, alt_rhi);
        std::swap(qrec, alt_qrec);
        std::swap(fkeys, alt_fkeys);
        std::swap(fvals, alt_fvals);
        set ^= 1;
    }
    int64_t index_base = 0;

    ~gs_handle() {
        for (DevBuf* b : {&p0, &p1, &p2, &p3, &sh4, &sh1, &rec, &dkey, &rlo, &rhi, &offsets, &partials, &keys,
                          &vals, &tkeys, &tvals, &sort_scratch, &ranges, &fb, &thr, &dsk, &dso, &dsl, &dsh, &dtk, &dto,
                          &dtl, &dth, &xmask, &xcounts, &xtotal, &owner_dev, &rows_dev, &alt_rec,
                          &alt_dkey, &alt_keys, &alt_vals, &alt_tkeys, &alt_tvals, &alt_ranges, &alt_thr, &alt_rlo,
                          &alt_rhi, &alt_qrec, &alt_fkeys, &alt_fvals, &seg_sample, &npairs, &fetch, &qrec, &cutbuf,
                          &cstate, &fkeys, &fvals, &fbtab, &fbn, &scratch2, &kept, &ppart, &cutord, &cutdil, &wcost,
                          &fbpart, &fbtot})
            b->release();
        if (side) (void)hipStreamDestroy(side);
        if (sorted_ev) (void)hipEventDestroy(sorted_ev);
        if (totals_ev) (void)hipEventDestroy(totals_ev);
        if (pre_ev) (void)hipEventDestroy(pre_ev);
        if (comp_done) (void)hipEventDestroy(comp_done);
        if (xcount_ev) (void)hipEventDestroy(xcount_ev);
        if (aux) (void)hipStreamDestroy(aux);
        for (auto& e : set_free)
            if (e) (void)hipEventDestroy(e);
        if (host_total) (void)hipHostFree(host_total);
        if (host_xtotal) (void)hipHostFree(host_xtotal);
        if (events) {
            for (auto& e : ev) (void)hipEventDestroy(e);
            for (auto& slot : kev)
                for (auto& e : slot) (void)hipEventDestroy(e);
        }
    }

    gs::SceneDev scene_dev() const {
        gs::SceneDev s;
        s.p0 = p0.as<const float4>();
        s.p1 = p1.as<const float4>();
        s.p2 = p2.as<const float4>();
        s.p3 = p3.as<const float2>();
        s.sh4 = sh4.as<const float4>();
        s.sh1 = sh1.as<const float>();
        s.n = (uint32_t)n;
        return s;
    }
};

namespace {

gs_status check_options(const gs_options& opt) {
    if (opt.sh_degree < 0 || opt.sh_degree > 3) return fail(GS_ERR_INVALID_ARG, "sh_degree must be 0..3");
    if (opt.cap < 0) return fail(GS_ERR_INVALID_ARG, "cap must be >= 0");
    if (opt.mode != GS_MODE_TILE && opt.mode != GS_MODE_LIVE50 && opt.mode != GS_MODE_MLAB)
        return fail(GS_ERR_INVALID_ARG, "bad mode");
    if (opt.frames_in_flight < 0 || opt.frames_in_flight > 2)
        return fail(GS_ERR_INVALID_ARG, "frames_in_flight must be 1 or 2");
    if (opt.binning < 0 || opt.binning > 2) return fail(GS_ERR_INVALID_ARG, "binning must be 0, 1 or 2");
    if (opt.depth_split < 0 || opt.depth_split > 1) return fail(GS_ERR_INVALID_ARG, "depth_split must be 0 or 1");
    return GS_OK;
}

gs_status adopt_planes(gs_handle* h, gs_status built, const gs_options& opt) {
    if (built == GS_ERR_OOM) return fail(GS_ERR_OOM, "host scene planes");
    if (built != GS_OK) return built;
    if (h->hp.n >= (int64_t)UINT32_MAX) return fail(GS_ERR_UNSUPPORTED, "more than 2^32-1 splats");
    h->opt = opt;
    h->n = h->hp.n;
    return GS_OK;
}

// Crop (instanced_splat_renderer.mm:382-386) into the host planes.
gs_status build_scene(gs_handle* h, const gs_scene_soa* sc, const gs_options& opt) {
    if (!sc || sc->n < 0 || (sc->n > 0 && (!sc->pos || !sc->rot || !sc->scale || !sc->opacity || !sc->color)))
        return fail(GS_ERR_INVALID_ARG, "gs_scene_soa: null array");
    gs_status s = check_options(opt);
    if (s != GS_OK) return s;
    if (opt.sh_degree > 0 && !sc->sh_rest) return fail(GS_ERR_INVALID_ARG, "sh_degree > 0 needs sh_rest");
    if (sc->n >= (int64_t)UINT32_MAX && !opt.crop) return fail(GS_ERR_UNSUPPORTED, "more than 2^32-1 splats");
    return adopt_planes(h, gsio::planes_from_soa(*sc, opt.crop_radius, opt.crop != 0, opt.sh_degree, &h->hp), opt);
}

gs_status scene_from_points(const PointData* pts, int64_t n, const std::vector<float>* raw_dc,
                            const gs_options& opt, gs_handle* h) {
    gs_status s = check_options(opt);
    if (s != GS_OK) return s;
    return adopt_planes(h, gsio::planes_from_points(pts, n, raw_dc ? raw_dc->data() : nullptr, opt.crop_radius,
                                                    opt.crop != 0, opt.sh_degree, &h->hp),
                        opt);
}

// Host-side frame uniforms; VP = P·V with the contract's summation order.
gs::FrameUniforms make_uniforms(const float* V, const float* P, int W, int H) {
    gs::FrameUniforms u{};
    std::memcpy(u.V, V, 64);
    std::memcpy(u.P, P, 64);
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            u.VP[c * 4 + r] = ((P[0 * 4 + r] * V[c * 4 + 0] + P[1 * 4 + r] * V[c * 4 + 1]) +
                               P[2 * 4 + r] * V[c * 4 + 2]) + P[3 * 4 + r] * V[c * 4 + 3];
    for (int j = 0; j < 3; ++j)
        u.campos[j] = -((V[j * 4 + 0] * V[12] + V[j * 4 + 1] * V[13]) + V[j * 4 + 2] * V[14]);
    u.campos[3] = 0.0f;
    u.width = W;
    u.height = H;
    u.tiles_x = (W + gs::kBin - 1) / gs::kBin;  // binning granularity (32x32 bins)
    u.tiles_y = (H + gs::kBin - 1) / gs::kBin;
    u.cell_mask = (W <= gs::kCellMaskDim && H <= gs::kCellMaskDim) ? 1 : 0;
    u.band_y0 = 0;
    u.band_y1 = H - 1;
    return u;
}

// Depth cuts: a tile's cut is the depth key of the last
// record it staged before its pixels finished, plus this margin (dkey units:
// one is 2^-10 of relative depth), so that the next frames' views, which move,
// still find their tiles' saturation inside the front lists.
constexpr uint32_t kCutMargin = 64;
uint32_t cut_margin() {  // GS_CUT_MARGIN overrides (A/B, tests)
    static const char* env = std::getenv("GS_CUT_MARGIN");
    static const uint32_t m = env ? (uint32_t)std::strtoul(env, nullptr, 10) : kCutMargin;
    return m;
}

// Depth cuts on (gs_options.depth_split; GS_DEPTH_SPLIT=0|1 overrides, A/B).
bool depth_cuts_on(const gs_handle* h) {
    static const char* env = std::getenv("GS_DEPTH_SPLIT");
    return env ? env[0] == '1' : h->opt.depth_split == 1;
}

int bits_for(uint32_t v) {  // bits needed to represent values < v
    int b = 0;
    while (b < 32 && (1ull << b) < v) ++b;
    return b;
}

// Binning order of a frame (gs_options.binning).  Both orders
// build the same lists; the default picks the cheaper chain with a cost model
// measured on MI355X (1080p uniform / heavy-tailed,
// 4K, 50M @ 4K, with and without depth cuts):
//   depth-first: global depth sort ~21 ps per splat, depth-order duplicate
//                (wave-cooperative) ~4.7 ps per pair;
//   bin-first:   index-order duplicate ~75 ps per unit of wave-max work W
//                (the sum over waves of 64 splats of the largest pair count:
//                the duplicate emits a wave's splats in lockstep, so a few
//                huge splats dominate a heavy-tailed scene), plus the per-bin
//                depth sort of the pairs that reach it, ~6 ps per pair in
//                lists that fit LDS, ~20 ps in longer ones, ~4.9 ns per bin.
// With depth cuts the per-bin sort sees the front lists only (about 0.3 P,
// lists that fit LDS).  W comes from the last bin-first frame (the fused
// preprocess measures it, PreFuse), scaled with P; before any, 0.07 P (the
// uniform scenes' measured ratio).  P (scaled by the item count: multi-GPU
// frames receive a varying number of records) and the long-list share come
// from the previous frames at the same resolution; with no history the frame
// goes depth-first.
// Bin-first needs the depth key to fit above the bin id in a 32-bit pair key.
// GS_BINNING=depth|bin overrides the option (A/B timing).
// nrows: the bin rows this frame composites (multi-GPU ranks own a band of
// them; the per-bin sort's fixed cost is paid for those only; -1: all).
bool bin_first_order(gs_handle* h, const gs::FrameUniforms& U, uint32_t m, int nrows = -1, bool cuts = false) {
    static const char* env = std::getenv("GS_BINNING");
    int b = h->opt.binning;
    if (env && std::strcmp(env, "depth") == 0) b = GS_BINNING_DEPTH_FIRST;
    if (env && std::strcmp(env, "bin") == 0) b = GS_BINNING_BIN_FIRST;
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    if (b == GS_BINNING_DEPTH_FIRST || std::max(bits_for(T), 1) + gs::kDepthBits > 32) return false;
    if (b == GS_BINNING_BIN_FIRST) return true;
    auto& o = h->order;
    if (o.w != U.width || o.h != U.height) {  // new history
        o = gs_handle::OrderModel{};
        o.w = U.width;
        o.h = U.height;
    }
    const bool known = o.frame_pairs > 0 && o.n > 0;
    const double P = known ? (double)o.frame_pairs * (double)m / (double)o.n : 0.0;  // pairs scale with items
    o.n = (int64_t)m;  // items of this frame (the scan that follows reads its P)
    if (!known) return false;
    const double Ps = cuts ? 0.3 * P : P;             // pairs through the per-bin sort
    const double f = cuts ? 0.0 : o.long_share;      // (front lists fit LDS)
    const double bins = nrows >= 0 ? (double)nrows * U.tiles_x : (double)T;
    // The index-order duplicate: every bin row owned (nrows < 0), it emits
    // wave-cooperatively (scan.hip coop_emit), so its cost follows the pairs
    // and the splats (round 5: 68 / 83 / 658 us at 1080p / heavy-tailed
    // 1080p / 50M @4K, 12.6 / 18.1 / 188M pairs); with an owner table, one
    // splat per lane, its cost follows the wave-max work W the fused
    // preprocess measures (round 4: 67 / 354 / 1003 us against W = 0.73M /
    // 3.53M / 15.9M).
    double dup_ps;
    if (nrows < 0 || h->band_local) {  // (a clipped band bins without its owner table)
        dup_ps = 2.6 * P + 3.0 * (double)m;
    } else {
        const double W = o.wmax_pairs > 0 ? (double)o.wmax * P / (double)o.wmax_pairs : 0.07 * P;
        dup_ps = 75.0 * W;
    }
    const double bin_ps = dup_ps + 6.0 * Ps * (1.0 - f) + 20.0 * Ps * f + 4900.0 * bins;
    const double depth_ps = 21.0 * (double)m + 4.7 * P;
    return bin_ps < depth_ps;
}

gs_status check_ready(gs_handle* h) {
    if (!h) return fail(GS_ERR_INVALID_ARG, "null handle");
    if (!h->initialized) return fail(GS_ERR_STATE, "gs_initialize not called");
    GS_HIP(hipSetDevice(h->device));
    return GS_OK;
}

gs_status ensure_frame_scratch(gs_handle* h) {
    const size_t n = (size_t)std::max<int64_t>(h->n, 1);
    GS_HIP(h->rec.reserve(n * gs::kRecFloat4 * 16));
    GS_HIP(h->dkey.reserve(n * 4));
    GS_HIP(h->rlo.reserve(n * 4));
    GS_HIP(h->rhi.reserve(n * 4));
    GS_HIP(h->partials.reserve(((n + gs::kScanItems - 1) / gs::kScanItems + 1) * 24));  // (3 rows: depth-cut front lists)
    if (!h->host_total) {  // written by the scan kernel itself, read after the stream sync
        GS_HIP(hipHostMalloc((void**)&h->host_total, 128, hipHostMallocMapped | hipHostMallocCoherent));
        GS_HIP(hipHostGetDevicePointer((void**)&h->dev_total, h->host_total, 0));
        h->host_total[6] = h->host_total[7] = ~0ull;  // (the sets' open-quadrant counts: none yet)
    }
    if (!h->seg_sample.ptr) {
        GS_HIP(h->seg_sample.reserve(16));
        GS_HIP(hipMemset(h->seg_sample.ptr, 0, 16));
    }
    GS_HIP(h->npairs.reserve(8));  // (per buffer set: a set's depth-cut fallback reads its own)
    GS_HIP(h->fetch.reserve(32));  // per buffer set: [2 set] records fetched, [2 set + 1] open tiles (depth cuts)
    if (!h->totals_ev) GS_HIP(hipEventCreateWithFlags(&h->totals_ev, hipEventDisableTiming));
    if (h->opt.stage_timing && !h->events) {
        for (auto& e : h->ev) GS_HIP(hipEventCreate(&e));
        for (auto& slot : h->kev)
            for (auto& e : slot) GS_HIP(hipEventCreate(&e));
        h->events = true;
    }
    return GS_OK;
}

// Stage timing (gs_options.stage_timing): 1 = an event between every stage
// (complete breakdown; each event packet costs a few us of gap), 2 = events
// carried by the preprocess and composite dispatch packets only (no gaps).
void mark(gs_handle* h, int k, hipStream_t st) {
    if (h->opt.stage_timing == 1 && h->events) (void)hipEventRecord(h->ev[k], st);
    // debugging aid: GS_DEBUG_SYNC=<bitmask of stages> finishes and reports them
    static const long dbg = std::getenv("GS_DEBUG_SYNC") ? std::strtol(std::getenv("GS_DEBUG_SYNC"), nullptr, 0) : 0;
    if (dbg & (1L << k)) {
        const hipError_t e = hipStreamSynchronize(st);
        std::fprintf(stderr, "[gsplat] stage %d done: %s\n", k, hipGetErrorString(e));
    }
}

float elapsed(gs_handle* h, int a, int b) {
    float ms = 0.0f;
    // (an event this frame did not record, e.g. a shard render without its
    // project: 0, and the error is not left for the next launch's check)
    if (h->opt.stage_timing == 1 && h->events && hipEventElapsedTime(&ms, h->ev[a], h->ev[b]) != hipSuccess) {
        (void)hipGetLastError();
        ms = 0.0f;
    }
    return ms;
}

// The frame's composite fetch counter (one per buffer set; the preprocess of
// the frame clears it).
unsigned long long* fetch_counter(gs_handle* h) { return h->fetch.as<unsigned long long>() + 2 * h->set; }
// Its open tile count (depth cuts), cleared with it.
unsigned long long* open_counter(gs_handle* h) { return h->fetch.as<unsigned long long>() + 2 * h->set + 1; }

hipEvent_t kernel_event(gs_handle* h, int k) {
    return h->opt.stage_timing == 2 && h->events ? h->kev[h->kev_slot][k] : nullptr;
}

// First launch of a frame: pick its packet-event slot.
void begin_frame(gs_handle* h, hipStream_t st) {
    h->kev_slot = (int)(h->kev_frames % gs_handle::kKevRing);
    h->kev_pending = false;
    mark(h, 0, st);
}

// Kernel times of packet-event slot `k` (waits for that frame's composite).
gs_status slot_times(gs_handle* h, int k, float* pre, float* comp, float* total) {
    GS_HIP(hipEventSynchronize(h->kev[k][3]));
    GS_HIP(hipEventElapsedTime(pre, h->kev[k][0], h->kev[k][1]));
    GS_HIP(hipEventElapsedTime(comp, h->kev[k][2], h->kev[k][3]));
    if (total) GS_HIP(hipEventElapsedTime(total, h->kev[k][0], h->kev[k][3]));
    return GS_OK;
}

// Bin-row ownership of the frame as the kernels see it.
struct Ownership {
    gs::RowOwnership dev{nullptr, 0};  // owner table (nullptr: single GPU)
    const uint16_t* rows = nullptr;    // owned bin rows (nullptr: all)
    int nrows = 0;
};

// Default table: rank r owns the contiguous bin rows [r*R/world, (r+1)*R/world).
std::vector<uint8_t> default_row_owner(int R, int world) {
    std::vector<uint8_t> o((size_t)R);
    for (int r = 0; r < world; ++r)
        for (int by = (int)((int64_t)r * R / world); by < (int)((int64_t)(r + 1) * R / world); ++by) o[by] = (uint8_t)r;
    return o;
}

gs_status frame_ownership(gs_handle* h, int tiles_y, hipStream_t st, Ownership* out) {
    *out = Ownership{};
    if (h->world == 1 || h->slab_frame) {  // every bin row
        out->nrows = tiles_y;
        return GS_OK;
    }
    std::vector<uint8_t> o = (int)h->custom_owner.size() == tiles_y ? h->custom_owner
                                                                    : default_row_owner(tiles_y, h->world);
    if (!h->custom_owner.empty() && (int)h->custom_owner.size() != tiles_y)
        return fail(GS_ERR_INVALID_ARG, "gs_shard_set_rows: table has " + std::to_string(h->custom_owner.size()) +
                                            " rows, the frame has " + std::to_string(tiles_y));
    if (o != h->owner_host) {
        std::vector<uint16_t> rows;
        for (int by = 0; by < tiles_y; ++by)
            if (o[by] == h->rank) rows.push_back((uint16_t)by);
        GS_HIP(h->owner_dev.reserve(o.size()));
        GS_HIP(h->rows_dev.reserve(std::max<size_t>(rows.size(), 1) * 2));
        GS_HIP(hipMemcpyAsync(h->owner_dev.ptr, o.data(), o.size(), hipMemcpyHostToDevice, st));
        if (!rows.empty())
            GS_HIP(hipMemcpyAsync(h->rows_dev.ptr, rows.data(), rows.size() * 2, hipMemcpyHostToDevice, st));
        GS_HIP(hipStreamSynchronize(st));  // the host vectors are the staging copies
        h->owner_host = std::move(o);
        h->cut_valid[0] = h->cut_valid[1] = false;  // (cuts of other bins)
        h->rows_host = std::move(rows);
    }
    out->dev = gs::RowOwnership{h->owner_dev.as<uint8_t>(), (uint32_t)h->rank};
    out->rows = h->rows_dev.as<uint16_t>();
    out->nrows = (int)h->rows_host.size();
    return GS_OK;
}

// Pair-key bits of a frame's bin ids: at least one, since the bin ranges are
// written by the last sort pass (a single-bin frame still needs one pass).
int list_key_bits(const gs::FrameUniforms& U) { return std::max(bits_for((uint32_t)(U.tiles_x * U.tiles_y)), 1); }

// Pair capacity of the current buffer set: at least `want` (0 on failure).
uint32_t reserve_pairs(gs_handle* h, uint64_t want) {
    const size_t p = (size_t)std::max<uint64_t>(want, 1) * 4;
    // (depth-cut frames: the front lists in their own pair buffers)
    const bool cut = h->cut_pending;
    auto smallest = [&]() {
        size_t m = std::min({h->keys.bytes, h->vals.bytes, h->tkeys.bytes, h->tvals.bytes});
        return cut ? std::min({m, h->fkeys.bytes, h->fvals.bytes}) : m;
    };
    // growing frees the set's buffers: its last composite must be done
    if (p > smallest() && hipEventSynchronize(h->set_free[h->set]) != hipSuccess) return 0;
    for (DevBuf* b : {&h->keys, &h->vals, &h->tkeys, &h->tvals})
        if (b->reserve(p) != hipSuccess) return 0;
    if (cut)
        for (DevBuf* b : {&h->fkeys, &h->fvals})
            if (b->reserve(p) != hipSuccess) return 0;
    const size_t c = smallest() / 4;
    const uint32_t cap = (uint32_t)std::min<size_t>(c, UINT32_MAX - 1);
    if (h->sort_scratch.reserve(gs::radix_sort_scratch_words(cap) * 4) != hipSuccess) return 0;
    return cap;
}

// Index order: the duplicate counts the first sort pass's digits itself when
// a duplicate block's pairs (estimated from p_est) fit its LDS count tiles;
// beyond them counts would go to contended global atomics (none then).
gs::PassCounts pass_counts(gs_handle* h, uint32_t m, bool index_order, const gs::SortPlan& plan, uint32_t cap,
                           uint64_t p_est) {
    gs::PassCounts pc;
    const double per_block = (double)p_est * gs::kScanItems / (double)std::max<uint32_t>(m, 1);
    if (index_order && plan.passes > 0 && per_block <= (double)(gs::kDupCountTiles - 1) * gs::radix_sort_tile_items()) {
        pc.C = h->sort_scratch.as<uint32_t>();
        pc.tile = gs::radix_sort_tile_items();
        pc.mask = plan.mask[0];
        pc.ntiles = (cap + pc.tile - 1) / pc.tile;
    }
    return pc;
}

// Buffers of a frame's lists over m items: bin ranges, offsets (depth
// order), the pair capacity (>= the last frame's P) and the first pass's
// digit counting.
gs_status prepare_lists(gs_handle* h, uint32_t m, bool index_order, const gs::FrameUniforms& U,
                        gs_handle::ListPrep* lp) {
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    GS_HIP(h->ranges.reserve((size_t)std::max<uint32_t>(T, 1) * sizeof(uint2)));
    if (!index_order) GS_HIP(h->offsets.reserve((size_t)std::max<uint32_t>(m, 1) * 4));
    lp->cap = reserve_pairs(h, h->order.frame_pairs);
    if (!lp->cap) return fail(GS_ERR_OOM, "pair buffers");
    // the sort scratch holds the first pass's digit counts (pc.C, taken just
    // below) and the depth sort's over m items: sized for both here, so no
    // later reserve of this frame can move it
    GS_HIP(h->sort_scratch.reserve(gs::radix_sort_scratch_words(std::max<uint32_t>(std::max<uint32_t>(m, 1), lp->cap)) * 4));
    lp->pc = pass_counts(h, m, index_order, gs::make_sort_plan(list_key_bits(U)), lp->cap, h->order.frame_pairs);
    return GS_OK;
}

// Binning order of this frame: decided once, before its preprocess when
// that fuses the scan (render_frame), else here.
bool pick_bin_first(gs_handle* h, const gs::FrameUniforms& U, uint32_t m, int nrows) {
    const int p = h->order_pick;
    h->order_pick = -1;
    return p >= 0 ? p == 1 : bin_first_order(h, U, m, nrows);
}

// Bin lists from m splats visited in `order` (nullptr = index order) with
// rects (rect_lo, rect_hi) in that order: per-block pair totals and their
// scan (P and the visible count to host) -> down-sweep fused with the
// duplicate -> stable sort by bin id -> ranges.  Marks 3..6 when `timed`.
// The duplicate and the sort are queued before the host waits for P: they
// read the pair count on the device and are sized by the pair buffers'
// capacity (grown to the last frame's P); a frame whose P exceeds it runs
// them as no-ops, and they are queued again once the buffers have grown.
// Depth-cut frames with cuts (h->cut_pending, h->cut_in): every pair is
// emitted and the bin sort's first pass keeps the front lists' (dkey <=
// cut[bin], SortFilter), their count left on the device (h->kept, read by
// gs_last_stats); *pairs and h->stats.pairs are every pair of the frame.
// tail (optional): queues what reads the lists (per-bin sort, composite ...)
// right behind them, before the host waits for P, so that the GPU never waits
// for the host; called again, with the lists, if they are queued again.
// Waits until the totals kernel has published sequence number `seq` in
// host_total[5] (its release store follows total[0..4]).  The kernel is a few
// microseconds behind the projection, so the host spins; past a second it
// falls back to a stream sync (an error if the word still differs).
hipError_t wait_totals(gs_handle* h, unsigned long long seq, hipStream_t st) {
    volatile unsigned long long* w = reinterpret_cast<volatile unsigned long long*>(h->host_total) + 5;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if (__atomic_load_n(reinterpret_cast<const unsigned long long*>(h->host_total) + 5, __ATOMIC_ACQUIRE) == seq)
            return hipSuccess;
        if ((spin & 1023u) == 1023u && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
    }
    const hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    return *w == seq ? hipSuccess : hipErrorUnknown;
}

using ListTail = std::function<gs_status(const uint32_t* sorted_vals)>;
gs_status build_bin_lists(gs_handle* h, uint32_t m, const uint32_t* order, const uint32_t* rect_lo,
                          const uint32_t* rect_hi, const gs::FrameUniforms& U, const Ownership& own, bool timed,
                          hipStream_t st, const uint32_t** vals_out, uint64_t* pairs,
                          const uint32_t* carry_dkey = nullptr, const ListTail* tail = nullptr,
                          hipStream_t tail_st = nullptr) {
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    const int bits = list_key_bits(U);
    const gs::SortPlan plan = gs::make_sort_plan(bits);
    // the preprocess already summed the scan blocks (render_frame, PreFuse)
    const bool fused = h->fused_prep.ok && !order && own.dev.owner == nullptr;
    gs_handle::ListPrep lp = h->fused_prep;
    h->fused_prep.ok = false;
    h->fused_last = fused;
    if (!fused) {
        gs_status ps = prepare_lists(h, m, order == nullptr, U, &lp);
        if (ps != GS_OK) return ps;
    }
    uint32_t cap = lp.cap;
    gs::PassCounts pc = lp.pc;
    uint32_t* const np = h->npairs.as<uint32_t>() + h->set;  // P on the device (this set's)
    const bool cut_frame = h->cut_pending && h->cut_in && carry_dkey;
    // (front-only emission: decided with the fused preprocess, render_frame)
    const bool front = fused && lp.front && cut_frame;
    gs::SortFilter flt;  // front lists: the pairs at or ahead of their bin's cut
    if (cut_frame) {
        GS_HIP(h->kept.reserve(16));
        flt.cut = h->cut_in;
        flt.bmask = (1u << bits) - 1u;
        flt.dshift = bits;
        flt.kept = h->kept.as<uint32_t>() + h->set;
        pc.cut = h->cut_in;  // (the duplicate counts only the pairs the filtered first pass keeps)
#if !GS_DUP_FILTER_COUNT
        pc = gs::PassCounts{};
#endif
        // the duplicate marks the pairs behind the cut from an LDS copy of the
        // table, so the filtered pass and its count test a bit instead of
        // gathering cut[bin] per pair (index order, every bin row owned)
        flt.flag = GS_DUP_FLAG && !order && !own.dev.owner && T <= gs::kDupCutBins &&
                   bits + gs::kDepthBits <= 31 ? 1u : 0u;
        // (front-only frames count the first pass's digits in the duplicate:
        // its pairs are few and nearly all kept)
        if (front) flt.flag = 1u;
        if (front && GS_DUP_FRONT_COUNT) pc = lp.pc;
    }
    h->front_last = front;
    // (front-only, GS_DUP_LOOKBACK: no count kernel; the duplicate's blocks
    // count their front pairs and find their offsets by look-back)
    // (and every depth-cut frame whose totals run beside the duplicate, lp.aux)
    const bool lookb = fused && GS_DUP_LOOKBACK && (front || lp.aux);
    // the host learns P by polling the totals kernel's sequence word in
    // host-mapped memory (GS_HOST_POLL) or by an event in its dispatch packet
    const unsigned long long seq = GS_HOST_POLL ? ++h->totals_seq : 0ull;
    hipEvent_t tev = GS_HOST_POLL ? nullptr : h->totals_ev;
    if (fused) {
        const uint32_t nb = (m + gs::kScanItems - 1) / gs::kScanItems;
        if (front && !lookb)  // the front pairs' block sums into ppart's fourth row
            GS_HIP(gs::launch_front_count(rect_lo, rect_hi, carry_dkey, m, U.cell_mask != 0, (uint32_t)U.tiles_x,
                                          h->cut_in, T, h->ppart.as<unsigned long long>() + (size_t)3 * nb, st));
        if (lookb && lp.aux) {
            // the totals alone, for the host, on the aux stream beside the
            // duplicate (which needs none of them: the preprocess cleared its
            // statuses); the host waits for them before the next frame's
            // preprocess is queued, which adds into ppart again
            GS_HIP(hipStreamWaitEvent(h->aux, h->pre_ev, 0));
            GS_HIP(gs::launch_scan_partials_fused(h->ppart.as<unsigned long long>(), nb, nullptr, h->dev_total,
                                                  nullptr, nullptr, cap, h->aux, tev, seq, front, lookb));
        } else {
            GS_HIP(gs::launch_scan_partials_fused(h->ppart.as<unsigned long long>(), nb, h->partials.as<uint64_t>(),
                                                  h->dev_total, h->seg_sample.as<uint32_t>() + 2 * h->set, np, cap,
                                                  st, tev, seq, front, lookb));
        }
        h->ppart_dirty = false;
    } else {
        GS_HIP(gs::launch_tile_count_totals(rect_lo, rect_hi, m, own.dev, U.cell_mask != 0, h->partials.as<uint64_t>(),
                                            h->dev_total, h->seg_sample.as<uint32_t>() + 2 * h->set,
                                            h->ranges.as<uint2>(), T, np, cap, pc.C,
                                            pc.C ? (pc.mask + 1) * pc.ntiles : 0u, st, tev, seq));
    }
    if (timed) mark(h, 3, st);
    // pairs (bin, splat) in visiting order (bin-first: the depth key above the
    // bin id), then a stable sort by bin id only; the last pass also writes
    // the bin ranges
    bool in_tmp = false;
    auto enqueue_lists = [&]() -> hipError_t {
        hipError_t e = gs::launch_scan_duplicate(order, rect_lo, rect_hi, h->partials.as<uint64_t>(), m,
                                                 (uint32_t)U.tiles_x, own.dev, U.cell_mask != 0, carry_dkey, bits,
                                                 h->keys.as<uint32_t>(), h->vals.as<uint32_t>(),
                                                 np, st, h->offsets.as<uint32_t>(), pc,
                                                 flt.flag ? h->cut_in : nullptr, flt.flag ? T : 0u, front,
                                                 lookb ? np : nullptr, cap);
        if (e != hipSuccess) return e;
        if (timed) mark(h, 4, st);
        // (depth-cut frames: sorted into fkeys/fvals, so keys/vals keep every
        // pair for the fallback lists)
        return gs::launch_radix_sort(h->keys.as<uint32_t>(), h->vals.as<uint32_t>(),
                                     cut_frame ? h->fkeys.as<uint32_t>() : h->keys.as<uint32_t>(),
                                     cut_frame ? h->fvals.as<uint32_t>() : h->vals.as<uint32_t>(),
                                     h->tkeys.as<uint32_t>(), h->tvals.as<uint32_t>(), cap, bits,
                                     h->sort_scratch.as<uint32_t>(), &in_tmp, st, h->ranges.as<uint2>(), np,
                                     pc.C != nullptr, flt);
    };
    auto lists_done = [&]() -> gs_status {
        uint32_t* fk = cut_frame ? h->fkeys.as<uint32_t>() : h->keys.as<uint32_t>();
        uint32_t* fv = cut_frame ? h->fvals.as<uint32_t>() : h->vals.as<uint32_t>();
        uint32_t* sk = in_tmp ? h->tkeys.as<uint32_t>() : fk;
        uint32_t* sv = in_tmp ? h->tvals.as<uint32_t>() : fv;
        h->last_keys = sk;
        h->last_vals = sv;
        h->last_tmp_keys = in_tmp ? fk : h->tkeys.as<uint32_t>();
        h->last_tmp_vals = in_tmp ? fv : h->tvals.as<uint32_t>();
        h->last_key_bits = bits;
        h->pair_cap = cap;
        if (timed) mark(h, 5, st);
        if (timed && !carry_dkey) mark(h, 6, st);  // (ranges come out of the last sort pass)
        *vals_out = sv;
        return tail ? (*tail)(sv) : GS_OK;
    };
    GS_HIP(enqueue_lists());
    gs_status ts = lists_done();
    if (ts != GS_OK) return ts;
    if (seq) {  // (the GPU goes on with the lists meanwhile)
        GS_HIP(wait_totals(h, seq, st));
    } else {
        GS_HIP(hipEventSynchronize(h->totals_ev));
    }
    // P: the pairs the duplicate writes; P_all: every pair of the frame (the
    // same unless front-only; the pair buffers hold P_all, so that the
    // fallback lists always fit)
    // (look-back: total[0] is not scanned; a frame that is not front-only
    // writes every pair)
    const uint64_t P_all = h->host_total[8], P = lookb && !front ? P_all : h->host_total[0];
    h->stats.visible = (int64_t)h->host_total[1];
    if (fused && P_all > 0) {  // the duplicate's wave-max work (PreFuse), for the binning-order model
        h->order.wmax = h->host_total[4];
        h->order.wmax_pairs = P_all;
    }
    h->stats.pairs = (int64_t)P_all;
    // the last per-bin depth sort's share of pairs in lists too long for LDS
    if ((h->host_total[3] & gs::kSegSampleValid) && h->order.sample_pairs)
        h->order.long_share = (double)h->host_total[2] / (double)h->order.sample_pairs;
    h->order.frame_pairs = P_all;
    if (P_all >= (uint64_t)UINT32_MAX) return fail(GS_ERR_UNSUPPORTED, "more than 2^32-1 (splat,bin) pairs");
    if (P_all > cap) {
        // the queued lists were no-ops (ranges still empty): grow, queue again.
        // The no-op tail (composite, next cuts, fallback lists) may sit on its
        // own stream: it reads the pair buffers reserve_pairs frees and counts
        // into the counters cleared below, so it drains first too.
        GS_HIP(hipStreamSynchronize(st));
        if (tail && tail_st && tail_st != st) GS_HIP(hipStreamSynchronize(tail_st));
        if (lp.aux) GS_HIP(hipStreamSynchronize(h->aux));
        // (the no-op tail's cut_finalize published an open-quadrant count of
        // a composite that never ran: discard it, the re-queued tail writes
        // the real one for the dilation controller)
        if (tail && h->host_total) h->host_total[6 + h->set] = ~0ull;
        if (!(cap = reserve_pairs(h, P_all))) return fail(GS_ERR_OOM, "pair buffers");
        // (look-back: 1 lets the duplicate run, its last block stores the
        // count; the statuses and the ticket cleared again)
        const uint32_t p32 = lookb ? 1u : (uint32_t)P;
        GS_HIP(hipMemcpy(np, &p32, 4, hipMemcpyHostToDevice));
        if (lookb)
            GS_HIP(hipMemsetAsync(h->partials.as<uint64_t>(), 0,
                                  ((size_t)(m + gs::kScanItems - 1) / gs::kScanItems + 1) * 8, st));
        pc = pass_counts(h, m, order == nullptr, plan, cap, lookb ? P_all : P);
        if (cut_frame) pc.cut = h->cut_in;
#if !GS_DUP_FILTER_COUNT
        if (cut_frame && !(front && GS_DUP_FRONT_COUNT)) pc = gs::PassCounts{};
#endif
        if (pc.C) GS_HIP(hipMemsetAsync(pc.C, 0, (size_t)(pc.mask + 1) * pc.ntiles * 4, st));
        if (tail) GS_HIP(hipMemsetAsync(fetch_counter(h), 0, 16, st));  // (the no-op frame's composite counted into these)
        // the bin ranges empty again: the no-op frame's tail may have written
        // some (a front-only frame's fallback lists are regenerated from the
        // rects, not from the empty pair arrays), and the re-queued sort's
        // last pass writes only the bins its lists hold
        GS_HIP(hipMemsetAsync(h->ranges.ptr, 0xFF, (size_t)T * sizeof(uint2), st));
        GS_HIP(enqueue_lists());
        if ((ts = lists_done()) != GS_OK) return ts;
    }
    h->stats.sort_bits = bits;
    h->stats.sort_passes = gs::make_sort_plan(bits).passes;
    h->pairs_emitted = lookb && front ? gs_handle::kEmittedOnDevice : P;
    *pairs = P_all;
    return GS_OK;
}

// Grows a buffer that kernels queued on `st` may still use: waits for them
// first (growth frees the old allocation).  Rare: the buffers only grow.
hipError_t reserve_after(DevBuf& b, size_t bytes, hipStream_t st) {
    if (bytes <= b.bytes) return hipSuccess;
    const hipError_t e = hipStreamSynchronize(st);
    return e != hipSuccess ? e : b.reserve(bytes);
}

// Depth cuts apply to this frame's composite rule and size:
// tile / live50 rules, no fragment cap, the depth key above the bin id.
#ifndef GS_CUT_DILATE_MAX  // A/B knobs of the dilation controller
#define GS_CUT_DILATE_MAX 3
#endif
#ifndef GS_CUT_OPEN_TOL
#define GS_CUT_OPEN_TOL 0
#endif
constexpr int kCutDilateMax = GS_CUT_DILATE_MAX;  // bins (3: a 7x7 neighbourhood)
constexpr int kCutCalm = 8;       // frames with no open quadrant before the radius drops by one
// open quadrants a frame may leave without widening the radius: a few cost the
// fallback lists little (they run on the composite stream, off the next
// frame's chain), a wider radius costs every bin's front list
// (profiles/r05/ab_dilate_radius.txt)
constexpr uint64_t kCutOpenTolerated = GS_CUT_OPEN_TOL;

bool cut_rule(const gs_handle* h, const gs::FrameUniforms& U) {
    return h->opt.cap == 0 && (h->opt.mode == GS_MODE_TILE || h->opt.mode == GS_MODE_LIVE50) &&
           list_key_bits(U) + gs::kDepthBits <= 32;
}

// Depth-cut state of the frame being enqueued on the current set
// (h->cut_pending, cut_in, cut_out): the set's two cut tables (cutbuf), the
// quadrant records, the open tiles' pixel states.  A set's tables hold cuts
// only from a depth-cut frame at this frame size, composite rule and bin-row
// ownership (frame_ownership drops them); any other frame on the set
// invalidates them.  st, sp: the streams that may still use the buffers.
gs_status setup_cuts(gs_handle* h, const gs::FrameUniforms& U, bool cut_frame, hipStream_t st, hipStream_t sp) {
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    if (h->cut_w != U.width || h->cut_h != U.height || h->cut_mode != h->opt.mode) {
        h->cut_valid[0] = h->cut_valid[1] = false;
        h->cut_w = U.width;
        h->cut_h = U.height;
        h->cut_mode = h->opt.mode;
    }
    h->cut_pending = false;
    h->cut_in = h->cut_out = nullptr;
    h->ord_in = h->ord_out = nullptr;
    if (!cut_frame) {
        h->cut_valid[h->set] = false;
        return GS_OK;
    }
    if (h->cut_bins < T) {
        GS_HIP(hipStreamSynchronize(st));
        GS_HIP(hipStreamSynchronize(sp));
        GS_HIP(h->cutbuf.reserve((size_t)T * 4 * 4));
        GS_HIP(h->cutord.reserve((size_t)T * 4 * 4));
        GS_HIP(h->wcost.reserve((size_t)T * 2 * 4));
        GS_HIP(h->cutdil.reserve((size_t)4 * T * 4));  // (two slots per set, see dil_slot)
        h->dil_r[0] = h->dil_r[1] = 0;
        h->cut_bins = T;
        h->cut_valid[0] = h->cut_valid[1] = false;
    }
    GS_HIP(h->qrec.reserve((size_t)T * gs::kQrecWords * 4));
    GS_HIP(reserve_after(h->cstate, (size_t)U.width * U.height * 16, st));
    h->cut_in = h->cut_valid[h->set] ? h->cut_table(h->set, 0) : nullptr;
    h->cut_out = h->cut_table(h->set, 1);
    // Dilation (a moving camera): a bin's content moves between the frame that
    // left its cut and this one, so a quadrant whose new content saturates
    // deeper is left open and finishes from the fallback lists, whose first
    // sort pass reads every pair of the frame.  While the set's frames leave
    // quadrants open, its cuts are dilated: each bin reads the deepest cut
    // within cut_r bins of it (a still camera leaves none open: r stays 0).
    {
        const int S = h->set;
        const uint64_t opened = h->host_total ? h->host_total[6 + S] : ~0ull;
        if (h->host_total) h->host_total[6 + S] = ~0ull;  // (consumed; ~0: no new count since)
        if (opened != ~0ull) {
            if (opened > kCutOpenTolerated) {
                h->cut_r[S] = std::min(h->cut_r[S] + 1, kCutDilateMax);
                h->cut_calm[S] = 0;
            } else if (opened > 0) {
                h->cut_calm[S] = 0;
            } else if (h->cut_r[S] > 0 && ++h->cut_calm[S] >= kCutCalm) {
                --h->cut_r[S];
                h->cut_calm[S] = 0;
            }
        }
        static const char* fixed_r = std::getenv("GS_CUT_DILATE");  // (A/B: a fixed radius)
        if (fixed_r) h->cut_r[S] = std::max(0, std::atoi(fixed_r));
        // two dilated tables per set: the one this frame reads (dil_slot[S],
        // made ahead by the tail of the frame that wrote its cuts, or here)
        // and the one this frame's tail dilates ahead into, which therefore
        // never is this frame's input, even when the tail is queued twice
        // (build_bin_lists' pair-buffer regrowth)
        uint32_t* d = h->cutdil.as<uint32_t>() + (size_t)(2 * S + h->dil_slot[S]) * T;
        h->dil_wslot[S] = h->dil_slot[S] ^ 1;
        if (h->cut_in && h->cut_r[S] > 0 && GS_CUT_DILATE_AHEAD && h->dil_r[S] >= h->cut_r[S]) {
            // dilated ahead by the tail of the frame that wrote these cuts
            // (a wider radius than the controller's now only moves pairs from
            // the fallback lists to the front lists: the same image)
            h->cut_in = d;
            h->stats.cut_dilate = (uint32_t)h->dil_r[S];
        } else if (h->cut_in && h->cut_r[S] > 0) {  // (the radius just grew: on the side stream, ahead of the lists)
            GS_HIP(gs::launch_cut_dilate(h->cut_in, d, (uint32_t)U.tiles_x, (uint32_t)U.tiles_y, h->cut_r[S], sp));
            h->cut_in = d;
            h->stats.cut_dilate = (uint32_t)h->cut_r[S];
        }
        h->dil_r[S] = 0;  // (cutdil[S] is this frame's input now; the tail may dilate the next one)
    }
    // (the order tables are written by single-GPU frames only, and a change
    // of ownership invalidates the cuts, so a valid cut table has its order)
    h->ord_in = h->cut_in && T <= gs::kOrderMaxBins ? h->order_table(h->set, 0) : nullptr;
    h->ord_out = T <= gs::kOrderMaxBins ? h->order_table(h->set, 1) : nullptr;
    h->cut_valid[h->set] = false;  // (true again once this frame's composite is queued)
    h->cut_pending = true;
    return GS_OK;
}

// Depth-cut frames, after the front lists' composite on sc:
// the next cuts of this set (from the quadrant records), and the fallback
// lists of the quadrants it left open: the frame's pairs (keys/vals, every
// pair, still there) of the bins with an open quadrant that lie behind the
// cut, picked by the first pass of their own bin sort (SortFilter `behind`,
// against the table cut_finalize writes), put in depth order per bin and
// composited from the saved states.  Nothing waits for the host: with no
// quadrant open, cut_finalize leaves a pair count of 0 and every kernel here
// returns at once (the usual case).  The front lists' buffers are free by
// then (same stream).
// Front-only frames (h->front_last) wrote no pair behind a cut: their
// fallback lists' pairs are emitted here from the splats' rects (m items,
// rect_lo / rect_hi / dkey), the bins with an open quadrant only.
gs_status cut_tail(gs_handle* h, const gs::FrameUniforms& U, gs::CompositeArgs ca, const uint32_t* dkey,
                   const gs::RowOwnership& own, hipStream_t sc, uint32_t m, const uint32_t* rect_lo,
                   const uint32_t* rect_hi) {
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    gs::CutFallback fb;
    if (h->cut_in) {
        GS_HIP(reserve_after(h->fbtab, (size_t)T * 4, sc));
        GS_HIP(reserve_after(h->fbn, 4, sc));
        fb.cut_in = h->cut_in;
        fb.open = open_counter(h);
        fb.npairs = h->npairs.as<uint32_t>() + h->set;
        fb.table = h->fbtab.as<uint32_t>();
        fb.n = h->fbn.as<uint32_t>();
        fb.kept = h->kept.as<uint32_t>() + 2 + h->set;
        fb.ranges = h->ranges.as<uint2>();
        if (h->dev_total) fb.host_open = reinterpret_cast<unsigned long long*>(h->dev_total) + 6 + h->set;
    }
    GS_HIP(gs::launch_cut_finalize(ca.qrec, ca.vals, dkey, h->cut_out, T, (uint32_t)U.tiles_x, own, cut_margin(), sc,
                                   fb));
    // the set's next composite's longest-first bin order (single-GPU frames),
    // from what this frame's workgroups fetched
    if (ca.wcost && h->ord_out) GS_HIP(gs::launch_order_bins(ca.wcost, T, h->ord_out, sc));
    // the set's next cuts, dilated here at the set's current radius while a
    // moving camera keeps them dilated (setup_cuts then reads them without a
    // kernel ahead of the projection), into the set's other dilated table
    // (dil_wslot: never this frame's input, so a tail queued twice, as after a
    // pair-buffer regrowth, cannot change what the frame's lists read).  On
    // the composite stream, which has slack while the side stream's
    // projection and chain bound the frame (1080p); a stream of its own
    // measured no better (profiles/r05/ab_dilate_radius.txt).
    if (GS_CUT_DILATE_AHEAD && h->cut_out && h->cut_r[h->set] > 0 && h->cutdil.bytes >= (size_t)4 * T * 4) {
        const int S = h->set;
        uint32_t* d = h->cutdil.as<uint32_t>() + (size_t)(2 * S + h->dil_wslot[S]) * T;
        GS_HIP(gs::launch_cut_dilate(h->cut_out, d, (uint32_t)U.tiles_x, (uint32_t)U.tiles_y, h->cut_r[S], sc));
        h->dil_r[S] = h->cut_r[S];
        h->dil_slot[S] = h->dil_wslot[S];  // (the set's next frame reads it; idempotent when queued twice)
    }
    if (!h->cut_in) return GS_OK;  // (whole lists: no quadrant can be left open)
#ifdef GS_AB_NO_FALLBACK  // timing ablation build only: exact only while no quadrant is left open
    return GS_OK;
#endif
    const int bits = h->last_key_bits;
    const uint32_t cap = h->pair_cap;
    GS_HIP(reserve_after(h->scratch2, gs::radix_sort_scratch_words(cap) * 4, sc));
    gs::SortFilter flt;
    flt.cut = fb.table;
    flt.bmask = (1u << bits) - 1u;
    flt.dshift = bits;
    flt.kept = fb.kept;
    flt.behind = 1;
    // (a marked frame's pairs carry kBehindFlag above the depth key: the test
    // and the kept keys go without it)
    if (bits + gs::kDepthBits <= 31) flt.kmask = ~gs::kBehindFlag;
    // (the table tested in LDS: every pair of the frame is tested against a
    // few open bins; GS_FB_LDS=0: the global gather, A/B)
    if (GS_FB_LDS && T <= gs::kDupCutBins) flt.lds_bins = T;
    if (h->front_last) {
        // the fallback pairs regenerated into keys/vals (free: the front lists
        // were sorted out of them on the side stream before this composite
        // ran), counted and scanned on the device; the sort keeps them all
        // (no pair carries the behind mark) on the same looping grid
        const uint32_t nb = (m + gs::kScanItems - 1) / gs::kScanItems;
        GS_HIP(reserve_after(h->fbpart, (size_t)std::max<uint32_t>(nb, 1) * 16, sc));
        GS_HIP(reserve_after(h->fbtot, 16 * 8, sc));
        GS_HIP(gs::launch_fallback_pairs(rect_lo, rect_hi, dkey, m, U.cell_mask != 0, (uint32_t)U.tiles_x, bits, fb.table,
                                         T, fb.open, h->fbpart.as<uint64_t>(), h->fbtot.as<uint64_t>(), fb.n, fb.kept,
                                         cap, h->keys.as<uint32_t>(), h->vals.as<uint32_t>(), sc));
        flt.behind = 0;
        flt.flag = 1u;
        flt.kmask = ~0u;
        flt.lds_bins = 0;
    }
    // (usually no quadrant is open and the sort's input is empty: a fixed
    // grid that loops over the tiles then costs a few workgroups, not one
    // per tile of the frame's pairs)
    flt.stride_grid = 512;
    bool in_tmp = false;
    uint32_t* fk = h->fkeys.as<uint32_t>();
    uint32_t* fv = h->fvals.as<uint32_t>();
    GS_HIP(gs::launch_radix_sort(h->keys.as<uint32_t>(), h->vals.as<uint32_t>(), fk, fv, h->tkeys.as<uint32_t>(),
                                 h->tvals.as<uint32_t>(), cap, bits, h->scratch2.as<uint32_t>(), &in_tmp, sc,
                                 h->ranges.as<uint2>(), fb.n, false, flt));
    uint32_t* sk = in_tmp ? h->tkeys.as<uint32_t>() : fk;
    uint32_t* sv = in_tmp ? h->tvals.as<uint32_t>() : fv;
    uint32_t* tk = in_tmp ? fk : h->tkeys.as<uint32_t>();
    uint32_t* tv = in_tmp ? fv : h->tvals.as<uint32_t>();
    GS_HIP(gs::launch_bin_depth_sort(h->ranges.as<uint2>(), T, sk, sv, tk, tv, bits, nullptr, sc, nullptr,
                                     open_counter(h)));
    ca.vals = sv;
    ca.ranges = h->ranges.as<uint2>();
    ca.pass = 2;
    ca.fetched = nullptr;
    GS_HIP(gs::launch_composite(ca, h->opt.mode, sc));
    return GS_OK;
}

// Binning + sort + composite over m items (local splats, or received
// exchange records): depth sort -> bin lists in depth order -> composite.
// With a fragment cap, per-pixel thresholds come first from index-ordered
// bin lists (counted in the depth-sort stage time).
gs_status bin_sort_composite(gs_handle* h, uint32_t m, const uint32_t* dkey, const uint32_t* rect_lo,
                             const uint32_t* rect_hi, const float4* rec, int rec_stride, const gs::FrameUniforms& U,
                             int compact, float4* out, uint32_t* out_bgra8, hipStream_t st, float* slab_t = nullptr,
                             const hipStream_t* composite_stream = nullptr) {
    // the composite runs on *composite_stream when given (frames_in_flight 2:
    // the caller's stream, while st is the handle's side stream) once the
    // lists are ready on st.  A pointer, since the caller's stream may be the
    // null stream.
    const hipStream_t sc = composite_stream ? *composite_stream : st;
    // (recorded = the last list kernel's dispatch packet carried sorted_ev)
    auto handoff = [&](bool recorded = false) -> hipError_t {
        if (sc == st) return hipSuccess;
        hipError_t e = recorded ? hipSuccess : hipEventRecord(h->sorted_ev, st);
        return e != hipSuccess ? e : hipStreamWaitEvent(sc, h->sorted_ev, 0);
    };
    Ownership own;
    gs_status so = frame_ownership(h, U.tiles_y, st, &own);
    if (so != GS_OK) return so;
    // the binning's ownership: none for a clipped band (h->band_local)
    Ownership bown = own;
    if (h->band_local && !slab_t) bown.dev = gs::RowOwnership{nullptr, 0};
    const size_t mm = (size_t)std::max<uint32_t>(m, 1);
    for (DevBuf* b : {&h->dsk, &h->dso, &h->dsl, &h->dsh, &h->dtk, &h->dto, &h->dtl, &h->dth})
        GS_HIP(b->reserve(mm * 4));
    GS_HIP(h->partials.reserve(((mm + gs::kScanItems - 1) / gs::kScanItems + 1) * 24));
    GS_HIP(h->sort_scratch.reserve(gs::radix_sort_scratch_words((uint32_t)mm) * 4));
    gs::CompositeArgs ca{};
    ca.rec = rec;
    ca.rec_stride = rec_stride;
    ca.width = U.width;
    ca.height = U.height;
    ca.tiles_x = U.tiles_x;
    ca.tiles_y = U.tiles_y;
    ca.rows = own.rows;
    ca.nrows = own.nrows;
    ca.compact = compact;
    ca.cell_mask = U.cell_mask;
    ca.out = out;
    ca.out_bgra8 = out_bgra8;
    ca.cap = h->opt.cap;
    ca.dkey = dkey;
    const uint32_t* vals = nullptr;
    uint64_t P = 0;
    const bool mlab = h->opt.mode == GS_MODE_MLAB;
    // depth cuts: decided before the lists (render_frame, render_received)
    const bool cut_ok = h->cut_pending && !slab_t;
    h->cut_frame = false;
    if (mlab && (ca.cap > 0 || slab_t))
        return fail(GS_ERR_UNSUPPORTED, "MLAB mode has no fragment cap and no depth slabs");
    if (mlab) {
        // MLAB k-buffer: arrival (index) order per pixel, no depth sort
        mark(h, 2, st);
        gs_status s = build_bin_lists(h, m, nullptr, rect_lo, rect_hi, U, bown, true, st, &vals, &P);
        if (s != GS_OK) return s;
        ca.vals = vals;
        ca.ranges = h->ranges.as<uint2>();
        GS_HIP(handoff());
        ca.fetched = fetch_counter(h);
        GS_HIP(gs::launch_composite(ca, h->opt.mode, sc, kernel_event(h, 2), kernel_event(h, 3)));
        mark(h, 7, sc);
        h->stats.pairs = (int64_t)P;
        return GS_OK;
    }
    if (!mlab && pick_bin_first(h, U, m, own.dev.owner ? own.nrows : -1)) {
        // Bin-first: bin lists in arrival (index) order with
        // the depth key carried in the pair keys, then each list stably
        // sorted by depth key -> (depth, index) order, the same lists as the
        // depth-first order below.
        h->bin_first_frame = true;
        // Depth cuts: the lists hold the pairs at or in front
        // of their bin's cut; the composite keeps the state of each tile they
        // leave open and raises the bins' cuts for the frame after next, and
        // the fallback lists finish the open tiles.  The per-pixel operation
        // sequence is the full lists' (same image, bit for bit).
        const bool cutf = cut_ok && (h->opt.mode == GS_MODE_TILE || h->opt.mode == GS_MODE_LIVE50) && ca.cap == 0;
        h->cut_frame = cutf;
        mark(h, 2, st);
        // (the per-bin sort stays on the side stream: on the composite stream,
        // beside the next frame's projection, it was starved)
        const hipStream_t sd = st;
        if (slab_t) {
            ca.slab = 1;
            ca.t_out = slab_t;
        }
        ca.fetched = fetch_counter(h);
        if (cutf) {
            ca.pass = 1;
            ca.qrec = h->qrec.as<uint32_t>();
            ca.open_q_count = open_counter(h);
            ca.state = h->cstate.as<float4>();
            ca.cut_in = h->cut_in;
            // (the longest-first order: whole frames on the strip kernel)
            const bool ordered = !own.dev.owner && gs::composite_strip((uint32_t)(U.tiles_x * U.tiles_y));
            ca.order = ordered ? h->ord_in : nullptr;
            ca.wcost = ordered ? h->wcost.as<uint32_t>() : nullptr;
        }
        // everything that reads the lists, queued before the host waits for P
        const ListTail tail = [&](const uint32_t* sv) -> gs_status {
            gs::CompositeArgs c = ca;
            c.vals = sv;
            c.ranges = h->ranges.as<uint2>();
            if (c.cap > 0) {  // per-pixel cap thresholds from the lists in arrival order
                GS_HIP(h->thr.reserve((size_t)U.width * U.height * 4));
                c.thr_out = h->thr.as<uint32_t>();
                GS_HIP(gs::launch_cap_threshold(c, sd));
                c.thr = h->thr.as<uint32_t>();
            }
            // (one sample word pair per buffer set, for the binning-order
            // model; not from cut lists, whose short lists would understate
            // the per-bin sort of whole ones)
            GS_HIP(gs::launch_bin_depth_sort(h->ranges.as<uint2>(), (uint32_t)(U.tiles_x * U.tiles_y), h->last_keys,
                                             h->last_vals, h->last_tmp_keys, h->last_tmp_vals, h->last_key_bits,
                                             cutf && h->cut_in ? nullptr : h->seg_sample.as<uint32_t>() + 2 * h->set,
                                             sd, sc != st ? h->sorted_ev : nullptr, nullptr,
                                             cutf && h->front_last));  // (front lists: short)
            mark(h, 6, sd);
            GS_HIP(handoff(true));
            GS_HIP(gs::launch_composite(c, h->opt.mode, sc, kernel_event(h, 2), kernel_event(h, 3)));
            if (slab_t) {
                h->slab_ca = c;
                h->slab_lists = true;
            }
            // the next cuts of this set, then the fallback lists
            if (cutf) {
                gs_status fs_ = cut_tail(h, U, c, dkey, own.dev, sc, m, rect_lo, rect_hi);
                if (fs_ != GS_OK) return fs_;
            }
            mark(h, 7, sc);
            return GS_OK;
        };
        gs_status s = build_bin_lists(h, m, nullptr, rect_lo, rect_hi, U, bown, true, st, &vals, &P, dkey, &tail, sc);
        if (s != GS_OK) return s;
        h->order.sample_pairs = P;
        if (cutf) {  // this frame's cuts are read by its set's next frame
            h->cut_phase[h->set] ^= 1;
            h->cut_valid[h->set] = true;
        }
        return GS_OK;
    }
    h->bin_first_frame = false;
    if (ca.cap > 0) {
        // 0. per-pixel cap thresholds from the lists in arrival (index) order
        GS_HIP(h->thr.reserve((size_t)U.width * U.height * 4));
        gs_status s = build_bin_lists(h, m, nullptr, rect_lo, rect_hi, U, bown, false, st, &vals, &P);
        if (s != GS_OK) return s;
        ca.vals = vals;
        ca.ranges = h->ranges.as<uint2>();
        ca.thr_out = h->thr.as<uint32_t>();
        GS_HIP(gs::launch_cap_threshold(ca, st));
        ca.thr = h->thr.as<uint32_t>();
    }
    // 1. splats by depth (descending zF == ascending dkey), ties by index,
    //    carrying (index, rect) so everything downstream reads sequentially
    bool in_tmp = false;
    const uint32_t* vin[3] = {nullptr, rect_lo, rect_hi};
    uint32_t* vout[3] = {h->dso.as<uint32_t>(), h->dsl.as<uint32_t>(), h->dsh.as<uint32_t>()};
    uint32_t* vtmp[3] = {h->dto.as<uint32_t>(), h->dtl.as<uint32_t>(), h->dth.as<uint32_t>()};
    GS_HIP(gs::launch_radix_sort3(dkey, vin, h->dsk.as<uint32_t>(), vout, h->dtk.as<uint32_t>(), vtmp, m,
                                  gs::kDepthBits, h->sort_scratch.as<uint32_t>(), &in_tmp, st));
    const uint32_t* order = in_tmp ? vtmp[0] : vout[0];
    const uint32_t* slo = in_tmp ? vtmp[1] : vout[1];
    const uint32_t* shi = in_tmp ? vtmp[2] : vout[2];
    mark(h, 2, st);
    // Depth cuts in depth order: the pair keys carry the sorted
    // depth keys above the bin ids, so the bin sort's first pass filters at
    // the cuts exactly as in bin-first frames; the composite, the next cuts
    // and the fallback lists are queued behind the lists (ListTail).
    const bool cutf = cut_ok && (h->opt.mode == GS_MODE_TILE || h->opt.mode == GS_MODE_LIVE50) && ca.cap == 0 &&
                      list_key_bits(U) + gs::kDepthBits <= 32;
    h->cut_frame = cutf;
    if (cutf) {
        const uint32_t* sdk = in_tmp ? h->dtk.as<uint32_t>() : h->dsk.as<uint32_t>();  // (dkeys in depth order)
        ca.fetched = fetch_counter(h);
        ca.pass = 1;
        ca.qrec = h->qrec.as<uint32_t>();
        ca.open_q_count = open_counter(h);
        ca.state = h->cstate.as<float4>();
        ca.cut_in = h->cut_in;
        const bool ordered = !own.dev.owner && gs::composite_strip((uint32_t)(U.tiles_x * U.tiles_y));
        ca.order = ordered ? h->ord_in : nullptr;
        ca.wcost = ordered ? h->wcost.as<uint32_t>() : nullptr;
        const ListTail tail = [&](const uint32_t* sv) -> gs_status {
            gs::CompositeArgs c = ca;
            c.vals = sv;
            c.ranges = h->ranges.as<uint2>();
            mark(h, 6, st);
            GS_HIP(handoff());
            GS_HIP(gs::launch_composite(c, h->opt.mode, sc, kernel_event(h, 2), kernel_event(h, 3)));
            gs_status fs_ = cut_tail(h, U, c, dkey, own.dev, sc, m, slo, shi);
            if (fs_ != GS_OK) return fs_;
            mark(h, 7, sc);
            return GS_OK;
        };
        gs_status s = build_bin_lists(h, m, order, slo, shi, U, bown, true, st, &vals, &P, sdk, &tail, sc);
        if (s != GS_OK) return s;
        h->cut_phase[h->set] ^= 1;  // this frame's cuts are read by its set's next frame
        h->cut_valid[h->set] = true;
        h->stats.pairs = (int64_t)P;
        return GS_OK;
    }
    // 2. bin lists in depth order
    gs_status s = build_bin_lists(h, m, order, slo, shi, U, bown, true, st, &vals, &P);
    if (s != GS_OK) return s;
    ca.vals = vals;
    ca.ranges = h->ranges.as<uint2>();
    if (slab_t) {  // depth-slab transmittance pass; the colour pass reuses the lists
        ca.slab = 1;
        ca.t_out = slab_t;
    }
    GS_HIP(handoff());
    ca.fetched = fetch_counter(h);
    GS_HIP(gs::launch_composite(ca, h->opt.mode, sc, kernel_event(h, 2), kernel_event(h, 3)));
    if (slab_t) {
        h->slab_ca = ca;
        h->slab_lists = true;
    }
    mark(h, 7, sc);
    h->stats.pairs = (int64_t)P;
    return GS_OK;
}

void fill_stats(gs_handle* h, uint64_t P, const gs::FrameUniforms& U) {
    gs_stats& s = h->stats;
    s.splats = h->n;
    s.pairs = (int64_t)P;
    s.tiles = (int64_t)U.tiles_x * U.tiles_y;
    s.width = U.width;
    s.height = U.height;
    const int64_t N = h->n, T = s.tiles;
    const int64_t bin = 56 + (h->opt.sh_degree > 0 ? 4 * 3 * sh_coeffs(h->opt.sh_degree) : 0);
    // Algorithmic bytes: what each stage must move at minimum.
    const int64_t Pi = (int64_t)P, dpass = gs::make_sort_plan(gs::kDepthBits).passes;
    s.bytes_preprocess = N * (bin + 48 + 12);  // record, depth key, rect lo/hi
    // reduce-then-scan LSD: per pass the count kernel reads the keys (4 B)
    // and the scatter moves key + values (read + write); the depth sort's
    // first pass generates the index values instead of reading them
    s.bytes_depth_sort = dpass > 0 ? N * (4 * dpass + 28 + 32 * (dpass - 1)) : 0;
    // scan: per-block totals from the rects (8 B).  Duplicate, bin-first:
    // one fused kernel reads the rects again and the depth keys (12 B);
    // depth-first: down-sweep (rects + offsets written, 12 B) and duplicate
    // (rects, order, offsets, 16 B).  Both write the pairs (8 B each).
    s.bytes_scan = N * 8 + T * 8;  // (+ the empty bin ranges, filled on the way)
    if (h->fused_last)  // the block sums came from the preprocess: the scan reads them
        s.bytes_scan = (N + gs::kScanItems - 1) / gs::kScanItems * 16 + T * 8;
    // (front-only frames write only their front pairs, counted first by
    // launch_front_count: another read of the rects and depth keys)
    // (look-back: the emitted count is on the device; P until gs_last_stats
    // reads it, and no separate count kernel)
    const bool pe_dev = h->front_last && h->pairs_emitted == gs_handle::kEmittedOnDevice;
    const int64_t Pe = h->front_last && !pe_dev ? (int64_t)h->pairs_emitted : Pi;
    if (h->front_last && !pe_dev) s.bytes_scan += N * 12;
    s.bytes_duplicate = (h->bin_first_frame ? N * 12 : N * 28) + Pe * 8;
    s.binning = h->bin_first_frame ? GS_BINNING_BIN_FIRST : GS_BINNING_DEPTH_FIRST;
    if (h->bin_first_frame) {
        // per-bin depth sort: keys read, vals gathered and written back (12 B
        // per pair)
        s.bytes_depth_sort = Pi * 12;
    }
    s.bytes_sort = Pi * 20 * (int64_t)s.sort_passes;
    s.bytes_ranges = 0;  // ranges come out of the last sort pass
    // upper bound until the fetch counter is read (gs_last_stats): every tile
    // of a bin reads the whole list; the early-out stops that short
    h->stats_fixed_bytes = 4 * T * 8 + (int64_t)U.width * U.height * 16;
    h->stats_set = h->set;
    s.bytes_composite = h->stats_fixed_bytes + 4 * Pi * (4 + 48);
    s.records_fetched = -1;
    s.pairs_sorted = Pi;
    s.cut_frame = h->cut_frame ? 1 : 0;
    s.front_only = h->front_last ? 1 : 0;
    h->cut_lists = h->cut_frame && h->cut_in;
    // (depth-cut frames with cuts: the first sort pass reads every pair, keeps
    // the front lists' P1; the rest runs on P1 -- set by gs_last_stats)
    // stage_timing 2: read lazily (gs_last_stats / gs_kernel_times), so a
    // frame never waits for itself
    if (h->opt.stage_timing == 2 && h->events) {
        h->kev_pending = true;
        ++h->kev_frames;
    }
    if (h->opt.stage_timing == 1 && h->events) {
        (void)hipEventSynchronize(h->ev[7]);
        s.ms_preprocess = elapsed(h, 0, 1);
        s.ms_exchange = h->shard_frame ? elapsed(h, 1, 8) : 0.0f;
        s.ms_depth_sort = elapsed(h, h->shard_frame ? 8 : 1, 2);
        s.ms_scan = elapsed(h, 2, 3);
        s.ms_duplicate = elapsed(h, 3, 4);
        s.ms_sort = elapsed(h, 4, 5);
        s.ms_ranges = elapsed(h, 5, 6);
        if (h->bin_first_frame) {  // the per-bin depth sort runs between marks 5 and 6
            s.ms_depth_sort = s.ms_ranges;
            s.ms_ranges = 0.0f;
        }
        s.ms_composite = elapsed(h, 6, 7);
        s.ms_total = elapsed(h, 0, 7);
    }
}

}  // namespace

extern "C" {

int32_t gs_abi_version(void) { return GSPLAT_ABI_VERSION; }

const char* gs_last_error(void) { return g_last_error.c_str(); }

void gs_default_options(gs_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof *o);
    o->mode = GS_MODE_TILE;
    o->sh_degree = 0;
    o->crop = 1;
    o->crop_radius = 5.0f;
    o->stage_timing = 0;
    o->frames_in_flight = 1;
    o->depth_split = 1;  // per-bin depth cuts: same image, fewer pairs sorted
}

gs_status gs_create_from_soa(const gs_scene_soa* scene, const gs_options* opt, gs_handle** out) {
    if (!out) return fail(GS_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    gs_options o;
    gs_default_options(&o);
    if (opt) o = *opt;
    gs_handle* h = new gs_handle();
    gs_status s = build_scene(h, scene, o);
    if (s != GS_OK) {
        delete h;
        return s;
    }
    *out = h;
    return GS_OK;
}

gs_status gs_create_from_points(const float* points, int64_t n, const gs_options* opt, gs_handle** out) {
    if (!out || (!points && n > 0) || n < 0) return fail(GS_ERR_INVALID_ARG, "bad points");
    *out = nullptr;
    gs_options o;
    gs_default_options(&o);
    if (opt) o = *opt;
    if (o.sh_degree != 0) return fail(GS_ERR_INVALID_ARG, "PointData carries converted colour only: sh_degree 0");
    gs_handle* h = new gs_handle();
    gs_status s = scene_from_points(reinterpret_cast<const PointData*>(points), n, nullptr, o, h);
    if (s != GS_OK) {
        delete h;
        return s;
    }
    *out = h;
    return GS_OK;
}

gs_status gs_create(const char* ply_path, const gs_options* opt, gs_handle** out) {
    if (!out || !ply_path) return fail(GS_ERR_INVALID_ARG, "null argument");
    *out = nullptr;
    gs_options o;
    gs_default_options(&o);
    if (opt) o = *opt;
    gs_status s = check_options(o);
    if (s != GS_OK) return s;
    gs_handle* h = new gs_handle();
    // binary files: mapped and converted in parallel straight into the HBM
    // plane layout (scene_io.h); anything else through the PLYLoader drop-in.
    // GS_PLY_DIRECT=0 takes the PLYLoader path for every file (A/B).
    static const char* direct_env = std::getenv("GS_PLY_DIRECT");
    bool handled = false;
    if (!(direct_env && direct_env[0] == '0')) {
        s = adopt_planes(h, gsio::planes_from_ply(ply_path, o.crop_radius, o.crop != 0, o.sh_degree, &h->hp, &handled),
                         o);
        if (s != GS_OK) {
            delete h;
            return s;
        }
    }
    if (!handled) {
        std::vector<PointData> pts;
        std::vector<float> dc;
        if (!PLYLoader::load(ply_path, pts, &dc, true)) {
            delete h;
            return fail(GS_ERR_IO, std::string("failed to load PLY: ") + ply_path);
        }
        s = scene_from_points(pts.data(), (int64_t)pts.size(), &dc, o, h);
    }
    if (s != GS_OK) {
        delete h;
        return s;
    }
    *out = h;
    return GS_OK;
}

gs_status gs_create_subset(const gs_handle* src, int64_t begin, int64_t end, gs_handle** out) {
    if (!out) return fail(GS_ERR_INVALID_ARG, "out is null");
    *out = nullptr;
    if (!src || begin < 0 || end < begin || end > src->n) return fail(GS_ERR_INVALID_ARG, "gs_create_subset: bad range");
    gs_handle* h = new gs_handle();
    try {
        gsio::planes_subset(src->hp, begin, end, &h->hp);
    } catch (const std::bad_alloc&) {
        delete h;
        return fail(GS_ERR_OOM, "gs_create_subset: host planes");
    }
    h->opt = src->opt;
    h->n = h->hp.n;
    *out = h;
    return GS_OK;
}

gs_status gs_get_scene(const gs_handle* h, float* pos, float* rot, float* scale, float* opacity, float* color,
                       float* sh_rest) {
    if (!h) return fail(GS_ERR_INVALID_ARG, "null handle");
    const gsio::HostPlanes& hp = h->hp;
    const int K = sh_coeffs(hp.sh_degree), NF = 3 * K, NP4 = hp.np4();
    const size_t n = (size_t)hp.n;
    for (size_t i = 0; i < n; ++i) {
        const float *a = hp.p0.data() + 4 * i, *b = hp.p1.data() + 4 * i, *c = hp.p2.data() + 4 * i,
                    *d = hp.p3.data() + 2 * i;
        if (pos) std::memcpy(pos + 3 * i, a, 12);
        if (opacity) opacity[i] = a[3];
        if (rot) std::memcpy(rot + 4 * i, b, 16);
        if (scale) std::memcpy(scale + 3 * i, c, 12);
        if (color) color[3 * i] = c[3], color[3 * i + 1] = d[0], color[3 * i + 2] = d[1];
        if (sh_rest) {
            float* r = sh_rest + 45 * i;
            std::memset(r, 0, 45 * 4);
            for (int j = 0; j < NF; ++j) {  // flat j = 3k + ch <- f_rest[ch*15 + k]
                const float v = j / 4 < NP4 ? hp.sh4.data()[((size_t)(j / 4) * n + i) * 4 + j % 4] : hp.sh1.data()[i];
                r[(j % 3) * 15 + j / 3] = v;
            }
        }
    }
    return GS_OK;
}

gs_status gs_initialize(gs_handle* h, int32_t device) {
    if (!h) return fail(GS_ERR_INVALID_ARG, "null handle");
    if (h->initialized)  // idempotent: a retried group initialize reuses the upload, streams and events
        return h->device == device ? GS_OK : fail(GS_ERR_STATE, "handle already initialized on another device");
    int count = 0;
    GS_HIP(hipGetDeviceCount(&count));
    if (device < 0 || device >= count) return fail(GS_ERR_DEVICE, "no such HIP device");
    GS_HIP(hipSetDevice(device));
    h->device = device;
    // HBM layout: the host planes are already in it, one copy each
    const size_t n = (size_t)std::max<int64_t>(h->n, 1), m = (size_t)h->n;
    const gsio::HostPlanes& hp = h->hp;
    GS_HIP(h->p0.reserve(n * 16));
    GS_HIP(h->p1.reserve(n * 16));
    GS_HIP(h->p2.reserve(n * 16));
    GS_HIP(h->p3.reserve(n * 8));
    if (m) {
        GS_HIP(hipMemcpy(h->p0.ptr, hp.p0.data(), m * 16, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(h->p1.ptr, hp.p1.data(), m * 16, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(h->p2.ptr, hp.p2.data(), m * 16, hipMemcpyHostToDevice));
        GS_HIP(hipMemcpy(h->p3.ptr, hp.p3.data(), m * 8, hipMemcpyHostToDevice));
    }
    if (h->opt.sh_degree > 0) {
        GS_HIP(h->sh4.reserve((size_t)std::max(hp.np4(), 1) * n * 16));
        GS_HIP(h->sh1.reserve(n * 4));
        if (m && hp.np4()) GS_HIP(hipMemcpy(h->sh4.ptr, hp.sh4.data(), (size_t)hp.np4() * m * 16, hipMemcpyHostToDevice));
        if (m && hp.tail()) GS_HIP(hipMemcpy(h->sh1.ptr, hp.sh1.data(), m * 4, hipMemcpyHostToDevice));
    }
    // frames_in_flight 2: the side stream (projection .. per-bin sort, the
    // frame's critical path, HBM- and latency-bound) runs at the highest queue
    // priority, so the dispatcher prefers its workgroups and the overlapping
    // composite (VALU-bound) fills the remaining slots.  GS_SIDE_PRIORITY=0:
    // default priority (A/B).
    int least = 0, greatest = 0;
    GS_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    const char* sp_env = std::getenv("GS_SIDE_PRIORITY");
    const bool high = !(sp_env && sp_env[0] == '0');
    GS_HIP(hipStreamCreateWithPriority(&h->side, hipStreamNonBlocking, high ? greatest : 0));
    GS_HIP(hipStreamCreateWithPriority(&h->aux, hipStreamNonBlocking, high ? greatest : 0));
    GS_HIP(hipEventCreateWithFlags(&h->pre_ev, hipEventDisableTiming));
    GS_HIP(hipEventCreateWithFlags(&h->comp_done, hipEventDisableTiming));
    GS_HIP(hipEventCreateWithFlags(&h->xcount_ev, hipEventDisableTiming));
    GS_HIP(hipEventCreateWithFlags(&h->sorted_ev, hipEventDisableTiming));
    for (auto& e : h->set_free) GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    h->initialized = true;
    return GS_OK;
}

int64_t gs_point_count(const gs_handle* h) { return h ? h->n : 0; }

void gs_destroy(gs_handle* h) {
    if (!h) return;
    if (h->device >= 0) (void)hipSetDevice(h->device);
    delete h;
}

gs_status gs_set_mode(gs_handle* h, int32_t mode) {
    if (!h || (mode != GS_MODE_TILE && mode != GS_MODE_LIVE50 && mode != GS_MODE_MLAB))
        return fail(GS_ERR_INVALID_ARG, "bad mode");
    h->opt.mode = mode;
    return GS_OK;
}

gs_status gs_set_stage_timing(gs_handle* h, int32_t mode) {
    if (!h || mode < 0 || mode > 2) return fail(GS_ERR_INVALID_ARG, "stage_timing must be 0, 1 or 2");
    h->opt.stage_timing = mode;
    h->kev_frames = 0;
    h->kev_pending = false;
    return GS_OK;
}

gs_status gs_set_frames_in_flight(gs_handle* h, int32_t n) {
    if (!h || n < 1 || n > 2) return fail(GS_ERR_INVALID_ARG, "frames_in_flight must be 1 or 2");
    h->opt.frames_in_flight = n;
    return GS_OK;
}

gs_status gs_set_depth_split(gs_handle* h, int32_t depth_split) {
    if (!h || depth_split < 0 || depth_split > 1) return fail(GS_ERR_INVALID_ARG, "depth_split must be 0 or 1");
    // (the next frame's ensure_frame_scratch allocates the two-slab buffers)
    h->opt.depth_split = depth_split;
    return GS_OK;
}

gs_status gs_set_cap(gs_handle* h, int32_t cap) {
    if (!h || cap < 0) return fail(GS_ERR_INVALID_ARG, "bad cap");
    h->opt.cap = cap;
    return GS_OK;
}

// One frame into a caller-owned framebuffer: fp32 RGBA (16 B/pixel) or, with
// bgra8, packed BGRA8Unorm (4 B/pixel, converted inside the composite).
static gs_status render_frame(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H,
                              void* out_user, int32_t out_is_device, bool bgra8, void* stream, bool band = false) {
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if (!view || !proj || !out_user || W <= 0 || H <= 0 || W > 65535 || H > 65535)
        return fail(GS_ERR_INVALID_ARG, "gs_render: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    gs::FrameUniforms U = make_uniforms(view, proj, W, H);
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    if (T == 0 || bits_for(T) > 32) return fail(GS_ERR_UNSUPPORTED, "bad tile count");
    if ((s = ensure_frame_scratch(h)) != GS_OK) return s;
    int compact = 0, band_nrows = -1;
    h->band_local = false;
    if (band) {
        // this rank's owned bin rows into a compact band; with contiguous
        // ownership the rects are clipped to the band's pixel rows (splats
        // off it are culled before their colour is read)
        h->slab_frame = false;
        h->slab_lists = false;
        Ownership own;
        if ((s = frame_ownership(h, U.tiles_y, st, &own)) != GS_OK) return s;
        if (own.nrows == 0) {  // no owned rows: an empty band
            std::memset(&h->stats, 0, sizeof h->stats);
            return GS_OK;
        }
        const std::vector<uint16_t>& rows = h->rows_host;
        if (own.dev.owner && (int)rows.back() - (int)rows.front() + 1 == (int)rows.size()) {
            U.band_y0 = (int32_t)rows.front() * gs::kBin;
            U.band_y1 = std::min(H, ((int32_t)rows.back() + 1) * gs::kBin) - 1;
            h->band_local = GS_BAND_LOCAL != 0;
        } else if (!own.dev.owner) {
            h->band_local = GS_BAND_LOCAL != 0;  // (world 1: the band is the frame)
        }
        compact = own.dev.owner ? 1 : 0;
        band_nrows = own.nrows;
    }
    const size_t bytes = (size_t)W * H * (bgra8 ? 4 : 16);
    void* out = out_user;
    if (!out_is_device) {
        GS_HIP(h->fb.reserve(bytes));
        out = h->fb.ptr;
    }
    std::memset(&h->stats, 0, sizeof h->stats);
    h->shard_frame = false;
    // frames_in_flight 2: projection .. binning on the side stream, into the
    // other buffer set, once the composite that last read that set is done
    const bool pipe = h->opt.frames_in_flight >= 2 && out_is_device && h->opt.stage_timing != 1;
    hipStream_t sp = pipe ? h->side : st;
    if (pipe) {
        h->swap_sets();
        if ((s = ensure_frame_scratch(h)) != GS_OK) return s;
    }
    // (a wait packet only when that composite may still run: each costs a
    // few us of stream bubble)
    if (hipEventQuery(h->set_free[h->set]) != hipSuccess) {
        // (GS_HOST_SET_WAIT, A/B) the host waits instead of a wait packet in
        // the side stream: the set's last composite ends with the co-run, long
        // before the side stream finishes the previous frame's chain, so the
        // projection is still queued in time and its stream has no barrier
        if (GS_HOST_SET_WAIT && pipe) GS_HIP(hipEventSynchronize(h->set_free[h->set]));
        else GS_HIP(hipStreamWaitEvent(sp, h->set_free[h->set], 0));
    }
    if (h->split_render) {  // (a split rank render's composite may still count into this set's counters)
        if (hipEventQuery(h->comp_done) != hipSuccess) GS_HIP(hipStreamWaitEvent(sp, h->comp_done, 0));
        h->split_render = false;
    }
    if (pipe && !h->last_pipe) {  // the side stream starts after everything the caller's stream holds
        GS_HIP(hipEventRecord(h->sorted_ev, st));
        GS_HIP(hipStreamWaitEvent(sp, h->sorted_ev, 0));
    }
    h->last_pipe = pipe;
    begin_frame(h, sp);
    // Bin-first frames of one GPU: the preprocess also sums every scan
    // block's pairs, fills the empty bin ranges and zeroes the first sort
    // pass's counts (PreFuse), so the chain starts at the scan of the block
    // sums.  The binning order and the list buffers are settled first.
    // GS_FUSED_SCAN=0: the separate reduce pass (A/B).
    static const char* fs_env = std::getenv("GS_FUSED_SCAN");
    gs::PreFuse fuse;
    h->fused_prep = gs_handle::ListPrep{};
    h->order_pick = -1;
    const bool whole = band ? h->band_local : h->world == 1;  // (the binning owns every row it sees)
    const bool cut_on = depth_cuts_on(h) && whole && cut_rule(h, U);
    bool cut_frame = false;
    if (whole && h->n > 0 && h->opt.mode != GS_MODE_MLAB && !(fs_env && fs_env[0] == '0')) {
        const bool bf = bin_first_order(h, U, (uint32_t)h->n, h->band_local ? band_nrows : -1, cut_on);
        h->order_pick = bf ? 1 : 0;
        cut_frame = cut_on;
        if ((s = setup_cuts(h, U, cut_frame, st, sp)) != GS_OK) return s;
        if (bf) {
            if ((s = prepare_lists(h, (uint32_t)h->n, true, U, &h->fused_prep)) != GS_OK) return s;
            const uint32_t nb = (uint32_t)((h->n + gs::kScanItems - 1) / gs::kScanItems);
            // (four rows: the three atomic sums of PreFuse, and the front
            // pairs' block sums a front-only frame stores, launch_front_count)
            GS_HIP(h->ppart.reserve((size_t)nb * 32));
            if (h->ppart_words != (size_t)nb * 4 || h->ppart_dirty) {
                GS_HIP(hipMemsetAsync(h->ppart.ptr, 0, (size_t)nb * 32, sp));  // (then kept clear by the scan)
                h->ppart_words = (size_t)nb * 4;
            }
            fuse.part = h->ppart.as<unsigned long long>();
            fuse.nb = nb;
            fuse.fill = h->ranges.as<uint2>();
            fuse.nfill = T;
            // Front-only emission (a frame with cuts, the duplicate's table in
            // LDS, the behind mark above the depth key): the duplicate writes
            // the front lists' pairs alone, so neither it nor the sort's first
            // pass moves the pairs behind the cuts (most of a frame's: 86 % at
            // 50M @4K); the fallback lists regenerate theirs when a quadrant
            // is left open (cut_tail).
            // (not while the set's cuts are dilated: a moving camera leaves
            // quadrants open, and regenerating their fallback pairs from every
            // splat's rect costs more than the whole pairs' sort pass it saves)
            h->fused_prep.front = GS_DUP_FRONT && h->cut_in && (GS_DUP_FRONT_DILATED || h->cut_r[h->set] == 0) &&
                                  T <= gs::kDupCutBins &&
                                  list_key_bits(U) + gs::kDepthBits <= 31;
            h->fused_prep.pc.cut = h->cut_in;  // (with cuts: the duplicate counts only the pairs the filter keeps)
#if !GS_DUP_FILTER_COUNT
            if (h->cut_in && !(h->fused_prep.front && GS_DUP_FRONT_COUNT)) h->fused_prep.pc = gs::PassCounts{};
#endif
            fuse.zero = h->fused_prep.pc.C;
            fuse.nzero = h->fused_prep.pc.C ? (h->fused_prep.pc.mask + 1) * h->fused_prep.pc.ntiles : 0u;
            // (look-back frames: the preprocess clears the duplicate's statuses
            // and ticket, so its totals kernel can run beside the duplicate;
            // not while the preprocess's dispatch carries timing events)
            // (depth-cut frames only: the aux totals carry no per-bin sort
            // sample, which only frames without cuts use)
            h->fused_prep.aux = GS_AUX_TOTALS && GS_DUP_LOOKBACK && cut_frame && h->cut_in && !kernel_event(h, 1) &&
                                (h->fused_prep.front || (GS_AUX_ALL && T <= gs::kDupCutBins &&
                                                         list_key_bits(U) + gs::kDepthBits <= 31));
            if (h->fused_prep.aux) {
                fuse.zero64 = reinterpret_cast<unsigned long long*>(h->partials.as<uint64_t>());
                fuse.nzero64 = nb + 1;
            }
            h->fused_prep.ok = true;
            h->ppart_dirty = true;  // (until its scan is queued)
        }
    }
    if (!cut_frame && (s = setup_cuts(h, U, false, st, sp)) != GS_OK) return s;
    GS_HIP(gs::launch_preprocess(h->scene_dev(), h->opt.sh_degree, U, h->rec.as<float4>(), h->dkey.as<uint32_t>(),
                                 h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(), sp, kernel_event(h, 0),
                                 h->fused_prep.aux ? h->pre_ev : kernel_event(h, 1), fetch_counter(h), fuse));
    mark(h, 1, sp);
    if ((s = bin_sort_composite(h, (uint32_t)h->n, h->dkey.as<uint32_t>(), h->rlo.as<uint32_t>(),
                                h->rhi.as<uint32_t>(), h->rec.as<float4>(), gs::kRecFloat4, U, compact,
                                bgra8 ? nullptr : static_cast<float4*>(out),
                                bgra8 ? static_cast<uint32_t*>(out) : nullptr, sp, nullptr, &st)) != GS_OK)
        return s;
    GS_HIP(hipEventRecord(h->set_free[h->set], st));  // this set's last reader
    const uint64_t P = (uint64_t)h->stats.pairs;
    if (!out_is_device) {
        GS_HIP(hipMemcpyAsync(out_user, out, bytes, hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));
    }
    fill_stats(h, P, U);
    if (bgra8) {
        h->stats.bytes_composite -= (int64_t)W * H * 12;
        h->stats_fixed_bytes -= (int64_t)W * H * 12;
    }
    return GS_OK;
}

gs_status gs_render(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H, float* out_rgba,
                    int32_t out_is_device, void* stream) {
    return render_frame(h, view, proj, W, H, out_rgba, out_is_device, false, stream);
}

gs_status gs_render_bgra8(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H,
                          uint8_t* out_bgra, int32_t out_is_device, void* stream) {
    return render_frame(h, view, proj, W, H, out_bgra, out_is_device, true, stream);
}

gs_status gs_last_stats(gs_handle* h, gs_stats* out) {
    if (!h || !out) return fail(GS_ERR_INVALID_ARG, "null argument");
    if (h->kev_pending) {  // stage_timing 2: kernel times of the last frame
        gs_status s = slot_times(h, h->kev_slot, &h->stats.ms_preprocess, &h->stats.ms_composite,
                                 &h->stats.ms_total);
        if (s != GS_OK) return s;
        h->kev_pending = false;
    }
    if (h->stats_set >= 0 && h->stats.records_fetched < 0) {  // the last frame's composite fetch counter
        unsigned long long v = 0;
        GS_HIP(hipSetDevice(h->device));
        GS_HIP(hipEventSynchronize(h->set_free[h->stats_set]));
        if (h->split_render) GS_HIP(hipEventSynchronize(h->comp_done));  // (its composite counts on its own stream)
        GS_HIP(hipMemcpy(&v, h->fetch.as<unsigned long long>() + 2 * h->stats_set, 8, hipMemcpyDeviceToHost));
        h->stats.records_fetched = (int64_t)v;
        h->stats.bytes_composite = h->stats_fixed_bytes + (int64_t)v * (4 + 48);
        if (h->stats.cut_frame) {
            // depth cuts: the front lists' pairs (the first sort pass reads all
            // P, counting and scattering, and writes the kept P1; the second
            // pass and the per-bin sort run on P1); the tiles those lists left
            // open and the pairs of their fallback lists (emitted, sorted,
            // per-bin sorted; each open tile's 256 pixel states written and
            // read back)
            gs_stats& s = h->stats;
            if (h->front_last && h->pairs_emitted == gs_handle::kEmittedOnDevice) {
                uint32_t pe = 0;  // (look-back: the duplicate's last block stored it)
                GS_HIP(hipMemcpy(&pe, h->npairs.as<uint32_t>() + h->stats_set, 4, hipMemcpyDeviceToHost));
                s.bytes_duplicate += ((int64_t)pe - s.pairs) * 8;
                h->pairs_emitted = pe;
            }
            if (h->cut_lists) {
                uint32_t k1 = 0;
                GS_HIP(hipMemcpy(&k1, h->kept.as<uint32_t>() + h->stats_set, 4, hipMemcpyDeviceToHost));
                // (the first pass reads the emitted pairs: every pair, or the
                // front pairs of a front-only frame)
                const int64_t P = h->front_last ? (int64_t)h->pairs_emitted : s.pairs, P1 = (int64_t)k1;
                s.pairs_sorted = P1;
                s.bytes_sort = P * 12 + P1 * 8 + P1 * 20 * (int64_t)(s.sort_passes - 1);
                if (h->bin_first_frame) s.bytes_depth_sort = P1 * 12;  // (depth-first: the global depth sort, unchanged)
            }
            unsigned long long open = 0;
            uint32_t P2 = 0;
            GS_HIP(hipMemcpy(&open, h->fetch.as<unsigned long long>() + 2 * h->stats_set + 1, 8,
                             hipMemcpyDeviceToHost));
            if (open) GS_HIP(hipMemcpy(&P2, h->kept.as<uint32_t>() + 2 + h->stats_set, 4, hipMemcpyDeviceToHost));
            s.open_tiles = (int64_t)open;
            s.pairs_sorted += (int64_t)P2;
            if (open && h->front_last) {  // the fallback pairs regenerated from the rects, then sorted
                s.bytes_duplicate += s.splats * 24 + (int64_t)P2 * 8;
                s.bytes_sort += (int64_t)P2 * 20 * (int64_t)s.sort_passes;
                s.bytes_depth_sort += (int64_t)P2 * 12;
                s.bytes_composite += (int64_t)open * 64 * 32;
            } else if (open) {  // the fallback sort's first pass reads every pair again
                s.bytes_sort += s.pairs * 12 + (int64_t)P2 * 8 + (int64_t)P2 * 20 * (int64_t)(s.sort_passes - 1);
                s.bytes_depth_sort += (int64_t)P2 * 12;
                s.bytes_composite += (int64_t)open * 64 * 32;  // (8x8 quadrants)
            }
        }
    }
    *out = h->stats;
    return GS_OK;
}

gs_status gs_kernel_times(gs_handle* h, int32_t max_frames, float* ms_preprocess, float* ms_composite,
                          int32_t* count) {
    if (!h || !count || max_frames < 0 || (max_frames > 0 && (!ms_preprocess || !ms_composite)))
        return fail(GS_ERR_INVALID_ARG, "gs_kernel_times: bad arguments");
    *count = 0;
    if (h->opt.stage_timing != 2 || !h->events) return GS_OK;
    const int64_t n = std::min<int64_t>({(int64_t)max_frames, h->kev_frames, (int64_t)gs_handle::kKevRing});
    for (int64_t j = 0; j < n; ++j) {  // oldest first
        const int k = (int)((h->kev_frames - n + j) % gs_handle::kKevRing);
        gs_status s = slot_times(h, k, &ms_preprocess[j], &ms_composite[j], nullptr);
        if (s != GS_OK) return s;
    }
    *count = (int32_t)n;
    return GS_OK;
}

gs_status gs_project_host(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H,
                          void* records, uint32_t* dkeys, uint32_t* ntiles) {
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if (!view || !proj || W <= 0 || H <= 0) return fail(GS_ERR_INVALID_ARG, "bad arguments");
    if ((s = ensure_frame_scratch(h)) != GS_OK) return s;
    const gs::FrameUniforms U = make_uniforms(view, proj, W, H);
    hipStream_t st = nullptr;
    GS_HIP(hipEventSynchronize(h->set_free[h->set]));  // a pipelined composite may still read the set
    GS_HIP(gs::launch_preprocess(h->scene_dev(), h->opt.sh_degree, U, h->rec.as<float4>(), h->dkey.as<uint32_t>(),
                                 h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(), st));
    GS_HIP(hipStreamSynchronize(st));
    const size_t n = (size_t)h->n;
    if (records) {
        GS_HIP(hipMemcpy2D(records, sizeof(gs::Record3), h->rec.ptr, (size_t)gs::kRecFloat4 * 16, sizeof(gs::Record3),
                           n, hipMemcpyDeviceToHost));
        if (U.cell_mask) {  // the cell-exclusion mask is internal: export the reference record
            uint32_t* w = static_cast<uint32_t*>(records);
            for (size_t i = 0; i < n; ++i) {
                w[12 * i + 10] &= 0x0FFF0FFFu;
                w[12 * i + 11] &= 0x0FFF0FFFu;
            }
        }
    }
    if (dkeys) GS_HIP(hipMemcpy(dkeys, h->dkey.ptr, n * 4, hipMemcpyDeviceToHost));
    if (ntiles) {
        std::vector<uint32_t> lo(n), hi(n);
        GS_HIP(hipMemcpy(lo.data(), h->rlo.ptr, n * 4, hipMemcpyDeviceToHost));
        GS_HIP(hipMemcpy(hi.data(), h->rhi.ptr, n * 4, hipMemcpyDeviceToHost));
        const uint32_t cm = U.cell_mask ? 0x0FFF0FFFu : 0xFFFFFFFFu;  // strip the bin-exclusion mask
        for (size_t i = 0; i < n; ++i) {
            const uint32_t l = lo[i] & cm, u = hi[i] & cm;
            const uint32_t x0 = l & 0xFFFF, x1 = u & 0xFFFF, y0 = l >> 16, y1 = u >> 16;
            ntiles[i] = x1 < x0 ? 0u : ((x1 >> 4) - (x0 >> 4) + 1) * ((y1 >> 4) - (y0 >> 4) + 1);
        }
    }
    return GS_OK;
}

gs_status gs_sorted_pairs_host(gs_handle* h, uint32_t* keys, uint32_t* vals, int64_t cap, int64_t* count) {
    if (!h || !count) return fail(GS_ERR_INVALID_ARG, "null argument");
    if (h->cut_lists)  // (a depth-cut frame without cuts yet has whole lists)
        return fail(GS_ERR_UNSUPPORTED, "the last frame's lists were cut at per-bin depths (depth_split = 0 keeps them whole)");
    int64_t P = h->stats.pairs;
    *count = P;
    if (!h->last_keys || P == 0) return GS_OK;
    int64_t m = std::min(P, cap);
    GS_HIP(hipSetDevice(h->device));
    GS_HIP(hipDeviceSynchronize());
    if (keys) {
        GS_HIP(hipMemcpy(keys, h->last_keys, (size_t)m * 4, hipMemcpyDeviceToHost));
        // bin-first pair keys carry the depth key above the bin id
        const uint32_t mask = h->last_key_bits >= 32 ? 0xFFFFFFFFu : (1u << h->last_key_bits) - 1u;
        for (int64_t i = 0; i < m; ++i) keys[i] &= mask;
    }
    if (vals) GS_HIP(hipMemcpy(vals, h->last_vals, (size_t)m * 4, hipMemcpyDeviceToHost));
    return GS_OK;
}

gs_status gs_radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* tmp_keys, uint32_t* tmp_vals, int64_t n,
                              int32_t bits, void* stream) {
    if (n < 0 || n >= (int64_t)UINT32_MAX || bits < 0 || bits > 32 || (n > 0 && (!keys || !vals || !tmp_keys || !tmp_vals)))
        return fail(GS_ERR_INVALID_ARG, "gs_radix_sort_pairs: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    uint32_t* scratch = nullptr;
    GS_HIP(hipMalloc(&scratch, gs::radix_sort_scratch_words((uint32_t)n) * 4));
    bool in_tmp = false;
    hipError_t e = gs::launch_radix_sort(keys, vals, keys, vals, tmp_keys, tmp_vals, (uint32_t)n, bits, scratch,
                                         &in_tmp, st);
    if (e == hipSuccess && in_tmp) {
        e = hipMemcpyAsync(keys, tmp_keys, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(vals, tmp_vals, (size_t)n * 4, hipMemcpyDeviceToDevice, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(scratch);
    GS_HIP(e);
    return GS_OK;
}

// ---- multi-GPU: tile-row ownership ---------------------------
int32_t gs_exchange_record_bytes(void) { return gs::kXRecFloat4 * 16 + gs::kXSideWords * 4; }

int32_t gs_exchange_regions(int32_t* bytes_per_record) {
    static_assert(GS_XREGIONS == 1 + gs::kXSideWords, "gsplat.h");
    if (bytes_per_record) {
        bytes_per_record[0] = gs::kXRecFloat4 * 16;
        for (int k = 1; k <= gs::kXSideWords; ++k) bytes_per_record[k] = 4;
    }
    return GS_XREGIONS;
}

gs_status gs_shard_configure(gs_handle* h, int32_t rank, int32_t world, int64_t index_base) {
    if (!h || world < 1 || world > gs::kMaxWorld || rank < 0 || rank >= world || index_base < 0 ||
        index_base + h->n >= (int64_t)UINT32_MAX)
        return fail(GS_ERR_INVALID_ARG, "gs_shard_configure: bad rank/world/index_base");
    h->rank = rank;
    h->world = world;
    h->index_base = index_base;
    h->custom_owner.clear();
    h->owner_host.clear();
    return GS_OK;
}

gs_status gs_shard_set_rows(gs_handle* h, const uint8_t* owner, int32_t nrows) {
    if (!h || nrows < 0 || (nrows > 0 && !owner)) return fail(GS_ERR_INVALID_ARG, "gs_shard_set_rows: bad arguments");
    for (int32_t i = 0; i < nrows; ++i)
        if (owner[i] >= h->world) return fail(GS_ERR_INVALID_ARG, "gs_shard_set_rows: owner >= world");
    h->custom_owner.assign(owner, owner + nrows);
    return GS_OK;
}

}  // extern "C"

namespace {

// The row scheme's destination buffers: masks, per-block counts, totals.
gs_status reserve_exchange(gs_handle* h) {
    const uint32_t n = (uint32_t)h->n;
    const uint32_t nb = (n + gs::kShardItems - 1) / gs::kShardItems;
    GS_HIP(h->xmask.reserve((size_t)std::max<uint32_t>(n, 1) * 4));
    GS_HIP(h->xcounts.reserve((size_t)std::max<uint32_t>(nb, 1) * h->world * 4));
    GS_HIP(h->xtotal.reserve(gs::kMaxWorld * 4));
    if (!h->host_xtotal) GS_HIP(hipHostMalloc((void**)&h->host_xtotal, gs::kMaxWorld * 4, hipHostMallocDefault));
    return GS_OK;
}

// Preprocess of a shard frame (both multi-GPU schemes).  owner (row scheme):
// the projection also writes the destination masks and per-block counts
// (ShardFuse), so pack_exchange skips its count kernel.
gs_status shard_preprocess(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H,
                           hipStream_t st, gs::FrameUniforms* U, const uint8_t* owner = nullptr) {
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if (!view || !proj || W <= 0 || H <= 0) return fail(GS_ERR_INVALID_ARG, "shard frame: bad arguments");
    if ((s = ensure_frame_scratch(h)) != GS_OK) return s;
    *U = make_uniforms(view, proj, W, H);
    // a pipelined composite may still read the set (a wait packet only then)
    if (hipEventQuery(h->set_free[h->set]) != hipSuccess) GS_HIP(hipStreamWaitEvent(st, h->set_free[h->set], 0));
    std::memset(&h->stats, 0, sizeof h->stats);
    h->shard_frame = true;
    h->slab_lists = false;
    h->band_local = false;  // (a shard frame bins with its owner table; an earlier band frame may have set it)
    begin_frame(h, st);
    gs::ShardFuse sf;
    // (a split rank render's composite may still count into the fetch
    // counters: that render clears them itself)
    unsigned long long* const zero8 = h->split_render ? nullptr : fetch_counter(h);
    if (owner) {
        if ((s = reserve_exchange(h)) != GS_OK) return s;
        sf.owner = owner;
        sf.world = h->world;
        sf.dest_mask = h->xmask.as<uint32_t>();
        sf.counts = h->xcounts.as<uint32_t>();
        sf.nblocks = (uint32_t)((h->n + gs::kShardItems - 1) / gs::kShardItems);
        if (sf.nblocks) GS_HIP(hipMemsetAsync(sf.counts, 0, (size_t)sf.nblocks * h->world * 4, st));
    }
    GS_HIP(gs::launch_preprocess(h->scene_dev(), h->opt.sh_degree, *U, h->rec.as<float4>(), h->dkey.as<uint32_t>(),
                                 h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(), st, kernel_event(h, 0),
                                 kernel_event(h, 1), zero8, gs::PreFuse{}, sf));
    mark(h, 1, st);
    return GS_OK;
}

// Destination masks by `rule`, per-destination counts (to host), then the
// exchange records grouped by destination, index order inside.
gs_status pack_exchange(gs_handle* h, const gs::DestRule& rule, bool masked, void* send, int64_t send_cap_bytes,
                        int64_t* send_counts, hipStream_t st, bool counted = false) {
    const uint32_t n = (uint32_t)h->n;
    const uint32_t nb = (n + gs::kShardItems - 1) / gs::kShardItems;
    gs_status rs = reserve_exchange(h);
    if (rs != GS_OK) return rs;
    // (the scan writes every destination's total; with no splats it does not run)
    if (nb == 0) GS_HIP(hipMemsetAsync(h->xtotal.ptr, 0, gs::kMaxWorld * 4, st));
    if (!counted)  // (counted: the projection wrote the masks and counts, ShardFuse)
        GS_HIP(gs::launch_shard_count(h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(), n, h->world, rule, masked,
                                      h->xmask.as<uint32_t>(), h->xcounts.as<uint32_t>(), nb, st));
    GS_HIP(gs::launch_rows_scan(h->xcounts.as<uint32_t>(), nb, nb ? h->world : 0, h->xtotal.as<uint32_t>(), st));
    GS_HIP(hipMemcpyAsync(h->host_xtotal, h->xtotal.ptr, h->world * 4, hipMemcpyDeviceToHost, st));
    GS_HIP(hipEventRecord(h->xcount_ev, st));
    auto pack = [&]() -> hipError_t {
        return gs::launch_shard_pack(h->rec.as<float4>(), h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(),
                                     h->dkey.as<uint32_t>(), h->xmask.as<uint32_t>(), n, h->world,
                                     h->xcounts.as<uint32_t>(), h->xtotal.as<uint32_t>(), nb,
                                     static_cast<float4*>(send), st);
    };
    // A send buffer that holds every splat once per rank cannot overflow: the
    // pack is queued before the host waits for the counts (one round trip,
    // under the pack); a smaller one is checked against them first.
    // (the host waits for the counts alone, not for the pack behind them: the
    // caller queues its next work, a render, while the pack runs)
    const bool roomy = send && send_cap_bytes >= (int64_t)n * h->world * gs_exchange_record_bytes();
    if (roomy) GS_HIP(pack());
    GS_HIP(hipEventSynchronize(h->xcount_ev));
    int64_t total = 0;
    for (int d = 0; d < h->world; ++d) {
        send_counts[d] = h->host_xtotal[d];
        total += h->host_xtotal[d];
    }
    if (roomy) return GS_OK;
    if (total * gs_exchange_record_bytes() > send_cap_bytes)
        return fail(GS_ERR_OOM, "exchange: send buffer too small (" +
                                    std::to_string(total * gs_exchange_record_bytes()) + " bytes needed)");
    if (total > 0 && !send) return fail(GS_ERR_INVALID_ARG, "exchange: null send buffer");
    GS_HIP(pack());
    return GS_OK;
}

// Received records -> depth sort -> bin lists -> composite (rows: owned rows
// into a compact band; slabs: transmittance pass over the full frame).
gs_status render_received(gs_handle* h, void* recv, int64_t m, int32_t W, int32_t H, float* out_rgba, float* slab_t,
                          hipStream_t st, const hipStream_t* sc = nullptr) {
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if ((m > 0 && !recv) || m < 0 || m >= (int64_t)UINT32_MAX || !(out_rgba || slab_t) || W <= 0 || H <= 0)
        return fail(GS_ERR_INVALID_ARG, "shard render: bad arguments");
    if ((s = ensure_frame_scratch(h)) != GS_OK) return s;
    // received records bin with the owner table (band_local is a gs_band_render
    // frame's, whose rects were clipped to the band: not these)
    h->band_local = false;
    const float I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const gs::FrameUniforms U = make_uniforms(I, I, W, H);
    const uint32_t T = (uint32_t)(U.tiles_x * U.tiles_y);
    // the exchange regions (gs_exchange_regions): m records, then their
    // binning rect lo / hi words and depth keys (SoA, source-rank order)
    float4* rv = static_cast<float4*>(recv);
    const uint32_t* rlo = reinterpret_cast<const uint32_t*>(rv + (size_t)gs::kXRecFloat4 * m);
    const uint32_t* rhi = rlo + m;
    const uint32_t* rkey = rhi + m;
    h->fused_prep.ok = false;
    // (a composite on its own stream, gs_shard_render_split: this render's
    // lists overwrite what the last one's composite and tail read, and its
    // cut setup reads the cuts that tail wrote; its fetch counters, which the
    // projection clears otherwise, are cleared here, behind that composite)
    // (also the first plain render after a split one: its projection left
    // the counters alone too)
    const bool was_split = h->split_render;
    h->split_render = sc != nullptr;
    if (sc || was_split) {
        if (hipEventQuery(h->comp_done) != hipSuccess) GS_HIP(hipStreamWaitEvent(st, h->comp_done, 0));
        GS_HIP(hipMemsetAsync(fetch_counter(h), 0, 16, st));
    }
    // depth cuts of the owned bins: the cuts and the quadrant
    // records are indexed by global bin, the pixel states by global pixel;
    // the binning order is picked for them
    Ownership own;
    if ((s = frame_ownership(h, U.tiles_y, st, &own)) != GS_OK) return s;
    const bool cut_on = !slab_t && m > 0 && depth_cuts_on(h) && cut_rule(h, U);
    if ((s = setup_cuts(h, U, cut_on, st, st)) != GS_OK) return s;
    h->order_pick = h->opt.mode == GS_MODE_MLAB ? -1 : bin_first_order(h, U, (uint32_t)m, own.nrows, cut_on) ? 1 : 0;
    mark(h, 8, st);
    if ((s = bin_sort_composite(h, (uint32_t)m, rkey, rlo, rhi, rv, gs::kXRecFloat4, U, slab_t ? 0 : 1,
                                reinterpret_cast<float4*>(out_rgba), nullptr, st, slab_t, sc)) != GS_OK)
        return s;
    // stage times span both calls: preprocess (project) ... composite; the
    // exchange between them falls inside the depth-sort interval
    fill_stats(h, (uint64_t)h->stats.pairs, U);
    h->stats.tiles = T;
    GS_HIP(hipEventRecord(h->set_free[h->set], st));
    if (sc) GS_HIP(hipEventRecord(h->comp_done, *sc));
    return GS_OK;
}

}  // namespace

extern "C" {

gs_status gs_shard_project(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H, void* send,
                           int64_t send_cap_bytes, int64_t* send_counts, void* stream) {
    if (!send_counts) return fail(GS_ERR_INVALID_ARG, "gs_shard_project: bad arguments");
    hipStream_t st = static_cast<hipStream_t>(stream);
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if (!view || !proj || W <= 0 || H <= 0) return fail(GS_ERR_INVALID_ARG, "gs_shard_project: bad arguments");
    h->slab_frame = false;
    // the owner table first: the projection counts the destinations itself
    Ownership own;
    if ((s = frame_ownership(h, (H + gs::kBin - 1) / gs::kBin, st, &own)) != GS_OK) return s;
    if (!own.dev.owner) return fail(GS_ERR_STATE, "gs_shard_project: world size 1");
    gs::FrameUniforms U;
    if ((s = shard_preprocess(h, view, proj, W, H, st, &U, own.dev.owner)) != GS_OK) return s;
    gs::DestRule rule{};
    rule.owner = own.dev.owner;
    return pack_exchange(h, rule, U.cell_mask != 0, send, send_cap_bytes, send_counts, st, true);
}

// Replicated-scene bands (SURVEY §8(e) fallback): the handle
// holds the whole scene; the rank renders its owned bin rows into a compact
// band (the gs_shard_render layout) with no exchange.  With contiguous
// ownership the rects are clipped to the band's pixel rows, so splats off
// the band are culled before their colour is read.
gs_status gs_band_render(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H, float* out_band,
                         void* stream) {
    if (!out_band) return fail(GS_ERR_INVALID_ARG, "gs_band_render: null output");
    // (two frames in flight like gs_render when the options ask for them)
    return render_frame(h, view, proj, W, H, out_band, 1, false, stream, true);
}

gs_status gs_shard_render_split(gs_handle* h, void* recv, int64_t m, int32_t W, int32_t H, float* out_rgba,
                                void* stream, void* composite_stream) {
    if (!out_rgba) return fail(GS_ERR_INVALID_ARG, "gs_shard_render_split: null output");
    const hipStream_t sc = static_cast<hipStream_t>(composite_stream);
    return render_received(h, recv, m, W, H, out_rgba, nullptr, static_cast<hipStream_t>(stream), &sc);
}

gs_status gs_shard_render(gs_handle* h, void* recv, int64_t m, int32_t W, int32_t H, float* out_rgba,
                          void* stream) {
    if (!out_rgba) return fail(GS_ERR_INVALID_ARG, "gs_shard_render: null output");
    if (h) h->slab_frame = false;
    return render_received(h, recv, m, W, H, out_rgba, nullptr, static_cast<hipStream_t>(stream));
}

// ---- depth slabs ---------------------------------------------
gs_status gs_slab_project(gs_handle* h, const float* view, const float* proj, int32_t W, int32_t H, uint64_t* hist,
                          void* stream) {
    if (!hist) return fail(GS_ERR_INVALID_ARG, "gs_slab_project: null histogram");
    if (h && h->opt.cap > 0) return fail(GS_ERR_UNSUPPORTED, "depth slabs: no fragment cap (it spans all slabs)");
    if (h && h->opt.mode == GS_MODE_MLAB) return fail(GS_ERR_UNSUPPORTED, "depth slabs: no MLAB mode");
    hipStream_t st = static_cast<hipStream_t>(stream);
    if (h) h->slab_frame = true;
    gs::FrameUniforms U;
    gs_status s = shard_preprocess(h, view, proj, W, H, st, &U);
    if (s != GS_OK) return s;
    GS_HIP(hipMemsetAsync(hist, 0, (size_t)gs::kSlabBins * 8, st));
    GS_HIP(gs::launch_slab_histogram(h->dkey.as<uint32_t>(), h->rlo.as<uint32_t>(), h->rhi.as<uint32_t>(),
                                     (uint32_t)h->n, U.cell_mask != 0,
                                     reinterpret_cast<unsigned long long*>(hist), st));
    h->slab_w = W;
    h->slab_h = H;
    return GS_OK;
}

gs_status gs_slab_bounds(const uint64_t* hist, int32_t world, uint32_t* bounds) {
    static_assert(GS_SLAB_BINS == gs::kSlabBins && GS_SLAB_BIN_KEYS == (1 << gs::kSlabBinShift), "gsplat.h");
    if (!hist || !bounds || world < 1 || world > gs::kMaxWorld)
        return fail(GS_ERR_INVALID_ARG, "gs_slab_bounds: bad arguments");
    uint64_t total = 0;
    for (int k = 0; k < gs::kSlabBins; ++k) total += hist[k];
    // bounds[d] = first key of the first bin whose preceding pairs reach d/world of the total
    bounds[0] = 0;
    uint64_t cum = 0;
    int k = 0;
    for (int d = 1; d < world; ++d) {
        const unsigned __int128 target = (unsigned __int128)total * (unsigned)d;
        while (k < gs::kSlabBins && (unsigned __int128)cum * (unsigned)world < target) cum += hist[k++];
        bounds[d] = (uint32_t)k << gs::kSlabBinShift;
    }
    bounds[world] = gs::kSlabKeys;
    return GS_OK;
}

gs_status gs_slab_pack(gs_handle* h, const uint32_t* bounds, void* send, int64_t send_cap_bytes, int64_t* send_counts,
                       void* stream) {
    if (!h || !bounds || !send_counts) return fail(GS_ERR_INVALID_ARG, "gs_slab_pack: bad arguments");
    if (!h->slab_frame || !h->shard_frame) return fail(GS_ERR_STATE, "gs_slab_pack: call gs_slab_project first");
    gs::DestRule rule{};
    rule.dkey = h->dkey.as<uint32_t>();
    rule.slabs = 1;
    for (int d = 0; d <= h->world; ++d) {
        if (d > 0 && bounds[d] < bounds[d - 1]) return fail(GS_ERR_INVALID_ARG, "gs_slab_pack: bounds not ascending");
        rule.bounds[d] = bounds[d];
    }
    const bool masked = h->slab_w <= gs::kCellMaskDim && h->slab_h <= gs::kCellMaskDim;
    return pack_exchange(h, rule, masked, send, send_cap_bytes, send_counts, static_cast<hipStream_t>(stream));
}

gs_status gs_slab_render(gs_handle* h, void* recv, int64_t m, int32_t W, int32_t H, float* t_local, void* stream) {
    if (!t_local) return fail(GS_ERR_INVALID_ARG, "gs_slab_render: null transmittance buffer");
    if (!h || !h->slab_frame) return fail(GS_ERR_STATE, "gs_slab_render: not a slab frame (gs_slab_project)");
    return render_received(h, recv, m, W, H, nullptr, t_local, static_cast<hipStream_t>(stream));
}

gs_status gs_slab_composite(gs_handle* h, const float* t_all, float* out_rgba, void* stream) {
    gs_status s = check_ready(h);
    if (s != GS_OK) return s;
    if (!out_rgba || (h->rank > 0 && !t_all)) return fail(GS_ERR_INVALID_ARG, "gs_slab_composite: bad arguments");
    if (!h->slab_lists) return fail(GS_ERR_STATE, "gs_slab_composite: no transmittance pass (gs_slab_render)");
    gs::CompositeArgs ca = h->slab_ca;
    ca.slab = 2;
    ca.slab_rank = h->rank;
    ca.t_all = t_all;
    ca.t_out = nullptr;
    ca.fetched = nullptr;  // (records_fetched counts the transmittance pass)
    ca.out = reinterpret_cast<float4*>(out_rgba);
    GS_HIP(gs::launch_composite(ca, h->opt.mode, static_cast<hipStream_t>(stream)));
    GS_HIP(hipEventRecord(h->set_free[h->set], static_cast<hipStream_t>(stream)));
    return GS_OK;
}

// ---- PLY / camera -----------------------------------------------------------
gs_status gs_ply_load(const char* path, int32_t compat, float** points, int64_t* n) {
    if (!path || !points || !n) return fail(GS_ERR_INVALID_ARG, "null argument");
    *points = nullptr;
    *n = 0;
    std::vector<PointData> pts;
    bool ok = PLYLoader::load(path, pts, nullptr, compat != 0);
    if (!pts.empty()) {
        float* buf = static_cast<float*>(std::malloc(pts.size() * sizeof(PointData)));
        if (!buf) return fail(GS_ERR_OOM, "malloc");
        std::memcpy(buf, pts.data(), pts.size() * sizeof(PointData));
        *points = buf;
        *n = (int64_t)pts.size();
    }
    return ok ? GS_OK : fail(GS_ERR_IO, std::string("PLY load failed: ") + path);
}

void gs_ply_free(float* points) { std::free(points); }

}  // extern "C"
