/*
 * gsplat.h — C-ABI of libgsplat.so, the MI355X-native Gaussian-splat tile
 * rasterizer.  Plain pointers and sizes only; no C++ or torch types cross it.
 *
 * It replaces the reference's splat renderer host class and its Metal passes
 * (nshelton/gaussian_splat):
 *
 *   reference                                             here
 *   ----------------------------------------------------- -----------------------------
 *   InstancedSplatRenderer(std::string)                   gs_create()
 *     src/instanced_splat_renderer.h:15, .mm:339-393       (PLY load + crop + upload prep)
 *   bool initialize(void* device)                         gs_initialize()
 *     src/instanced_splat_renderer.h:18, .mm:399-422
 *   void render(cmdBuf, drawable, view, proj, w, h)       gs_render()
 *     src/instanced_splat_renderer.h:21-26, .mm:424-578    (offscreen fp32 RGBA in HBM)
 *   int getPointCount() const                             gs_point_count()
 *     src/instanced_splat_renderer.h:28
 *   PLYLoader::load(path, vector<PointData>&)             gs_ply_load() / gs_ply_free()
 *     src/ply_loader.h:33, src/ply_loader.cpp:22-205
 *   (Metal GPU time, src/metal_renderer.mm:123-126)       gs_last_stats()
 *   (stderr + bool returns)                               gs_status + gs_last_error()
 *
 * Matrices are column-major float[16] exactly like simd_float4x4 (m[col*4+row]).
 * All GPU work of one call is enqueued on the caller's HIP stream; gs_render is
 * asynchronous when `out_rgba` is device memory.
 */
#ifndef GSPLAT_H
#define GSPLAT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSPLAT_ABI_VERSION 10

typedef enum {
    GS_OK = 0,
    GS_ERR_INVALID_ARG = 1,
    GS_ERR_IO = 2,
    GS_ERR_PARSE = 3,
    GS_ERR_DEVICE = 4,
    GS_ERR_OOM = 5,
    GS_ERR_COMM = 6,
    GS_ERR_UNSUPPORTED = 7,
    GS_ERR_STATE = 8
} gs_status;

/* Composite rule.  TILE = gaussian_splat_tile.metal:251-266 (contract
 * default); LIVE50 = gaussian_splat_50layer.metal:208-222; MLAB = the
 * 6-layer k-buffer of gaussian_splat.metal:201-361 (arrival order, half
 * arithmetic, resolve output before the drawable blend; no cap, no slabs). */
typedef enum { GS_MODE_TILE = 0, GS_MODE_LIVE50 = 1, GS_MODE_MLAB = 2 } gs_mode;
typedef enum { GS_BINNING_DEFAULT = 0, GS_BINNING_DEPTH_FIRST = 1, GS_BINNING_BIN_FIRST = 2 } gs_binning;

typedef struct gs_options {
    int32_t mode;          /* gs_mode */
    int32_t sh_degree;     /* 0..3; 0 = loader-converted DC colour (reference behaviour) */
    int32_t crop;          /* 1 = keep |x|,|y|,|z| < crop_radius (instanced_splat_renderer.mm:382-386) */
    float crop_radius;     /* 5.0 in the reference */
    int32_t stage_timing;  /* gs_last_stats timing: 0 off; 1 = an event between every stage (full
                              breakdown; each event adds a few us of gap); 2 = events carried by
                              the preprocess and composite dispatches only (no gaps) */
    int32_t cap;           /* per-pixel fragment cap by arrival order, 0 = none (contract default);
                              32 = gaussian_splat_tile.metal:7, 50 = gaussian_splat_50layer.metal:8 */
    int32_t frames_in_flight; /* 1 (default): a gs_render runs entirely on the caller's stream.
                              2: projection, sorting and binning of a frame run on an internal
                              stream of the handle and overlap the previous frame's composite
                              (double-buffered scratch); the composite, and so the output, stays
                              on the caller's stream in call order.  Device outputs only;
                              stage_timing 1 renders with 1. */
    int32_t binning;       /* order in which the bin lists are built (same lists, same image):
                              0 = default: chosen per frame by a cost model fed with the pair
                              count of the previous frame at the same resolution (the first frame
                              at a resolution goes depth-first), 1 = depth-first (global depth
                              sort of the splats, then binning), 2 = bin-first (bin lists in
                              arrival order, then a stable per-bin depth sort).  DESIGN.md §1 */
    int32_t depth_split;   /* per-bin depth cuts (modes tile/live50, no cap;
                              single-GPU frames, the row scheme's rank renders
                              (gs_shard_render) and band renders of contiguous rows
                              (gs_band_render) alike): 1 (gs_default_options) = a frame's bin lists
                              hold only the pairs at or in front of their bin's cut, the depth at
                              which the bin's tiles saturated in the previous frame on the same
                              buffer set, plus a margin; a tile those lists leave open finishes
                              from its saved state with the rest of its bin's pairs (fallback
                              lists).  Same image, bit for bit, for any camera path; 0 = whole
                              lists */
    int32_t reserved[3];
} gs_options;

/* Scene as SoA host arrays (all float32, n splats).  Used by
 * gs_create_from_soa; gs_create fills the same fields from a .ply. */
typedef struct gs_scene_soa {
    int64_t n;
    const float *pos;      /* n*3 x,y,z */
    const float *rot;      /* n*4 w,x,y,z (raw; normalised on device, tile.metal:41) */
    const float *scale;    /* n*3 activated: exp(scale_i) (ply_loader.cpp:117-119) */
    const float *opacity;  /* n activated: sigmoid (ply_loader.cpp:116) */
    const float *color;    /* n*3: rgb (sh_degree 0) or raw f_dc (sh_degree > 0) */
    const float *sh_rest;  /* n*45 f_rest in PLY (channel-major) order, or NULL */
} gs_scene_soa;

/* Per-frame statistics of the last gs_render on a handle. */
typedef struct gs_stats {
    int64_t splats;        /* N on the device (post-crop) */
    int64_t visible;       /* splats that touch >= 1 tile */
    int64_t pairs;         /* P = (splat, tile) pairs */
    int64_t tiles;         /* T */
    int32_t width, height;
    int32_t sort_bits;     /* significant key bits sorted */
    int32_t sort_passes;
    /* stage times in ms (all with stage_timing = 1; preprocess, composite and
       total with stage_timing = 2) */
    float ms_preprocess, ms_scan, ms_duplicate, ms_sort, ms_ranges, ms_composite, ms_total;
    int64_t bytes_preprocess, bytes_scan, bytes_duplicate, bytes_sort, bytes_ranges, bytes_composite;
    float ms_depth_sort;   /* splats by depth key (ms_sort = pairs by tile) */
    float ms_exchange;     /* multi-GPU: destination count + pack + exchange (between the shard calls) */
    int64_t bytes_depth_sort;
    int32_t binning;       /* order the last frame's bin lists were built in: GS_BINNING_DEPTH_FIRST
                              (ms_depth_sort = global depth sort) or GS_BINNING_BIN_FIRST
                              (ms_depth_sort = per-bin depth sort after the bin sort) */
    int32_t front_only;    /* 1: a depth-cut frame whose duplicate wrote only its front pairs (the
                              pairs at or ahead of their bin's cut; the fallback lists' pairs were
                              regenerated from the splats when a quadrant stayed open), DESIGN.md §4 */
    /* records the composite's workgroups fetched (each of a 32-px bin's four
       16x16 tiles reads the bin's list itself; a tile stops fetching once its
       pixels saturate): the basis of bytes_composite = 8 B per workgroup +
       52 B per fetched record + the framebuffer.  gs_last_stats waits for the
       last frame's composite to read it. */
    int64_t records_fetched;
    /* pairs the frame actually emitted and sorted (= pairs, except in
       depth-cut frames, gs_options.depth_split: the front lists' pairs plus
       the fallback lists'), the 8x8-pixel quadrants the front lists left
       open (open_tiles), and
       cut_frame = 1 for a depth-cut frame.  Read with records_fetched.
       cut_dilate: the radius in 32-px bins over which the frame's cuts were
       dilated (0 unless the buffer set's recent frames left quadrants open:
       a moving camera).
       Renamed in ABI 10 (same offsets and types): cut_frame was two_slab and
       cut_dilate was depth_cut; the old names stay as deprecated aliases of
       the same storage for one release (README "Changes"). */
    int64_t pairs_sorted;
    int64_t open_tiles;
    union {
        int32_t cut_frame;
        int32_t two_slab; /* deprecated alias of cut_frame */
    };
    union {
        uint32_t cut_dilate;
        uint32_t depth_cut; /* deprecated alias of cut_dilate */
    };
} gs_stats;

typedef struct gs_handle gs_handle;

/* ---- library ---------------------------------------------------------- */
int32_t gs_abi_version(void);
const char *gs_last_error(void);          /* thread-local; valid until next call on this thread */
void gs_default_options(gs_options *opt); /* tile mode, sh 0, crop on (r = 5) */

/* ---- scene / handle (InstancedSplatRenderer) -------------------------- */
gs_status gs_create(const char *ply_path, const gs_options *opt, gs_handle **out);
gs_status gs_create_from_soa(const gs_scene_soa *scene, const gs_options *opt, gs_handle **out);
/* PointData array (62 floats per point, src/ply_loader.h:7-28), sh_degree 0. */
gs_status gs_create_from_points(const float *points, int64_t n, const gs_options *opt, gs_handle **out);
/* A handle over splats [begin, end) of a loaded (cropped) scene, same options:
 * a shard without re-reading the file (no reference counterpart). */
gs_status gs_create_subset(const gs_handle *scene, int64_t begin, int64_t end, gs_handle **out);
/* The loaded (post-crop) scene back as host SoA arrays in gs_scene_soa layout
 * (n = gs_point_count; any pointer may be NULL; sh_rest: n*45 in PLY order,
 * zero beyond the handle's SH degree). */
gs_status gs_get_scene(const gs_handle *h, float *pos, float *rot, float *scale, float *opacity, float *color,
                       float *sh_rest);
gs_status gs_initialize(gs_handle *h, int32_t device_ordinal); /* uploads the scene to HBM */
int64_t gs_point_count(const gs_handle *h);
void gs_destroy(gs_handle *h);
gs_status gs_set_mode(gs_handle *h, int32_t mode);
/* Per-pixel fragment cap (0 = none): keep the first `cap` covering fragments
 * of each pixel in arrival (= splat index) order, as the reference's
 * fixed-size per-pixel lists do (tile.metal:199-202, 50layer.metal:170). */
gs_status gs_set_cap(gs_handle *h, int32_t cap);
gs_status gs_set_depth_split(gs_handle *h, int32_t depth_split); /* gs_options.depth_split, between frames */
/* Switch gs_options.stage_timing (0, 1 or 2) on a live handle. */
gs_status gs_set_stage_timing(gs_handle *h, int32_t mode);
/* Switch gs_options.frames_in_flight (1 or 2) on a live handle. */
gs_status gs_set_frames_in_flight(gs_handle *h, int32_t n);

/* ---- frame (InstancedSplatRenderer::render) --------------------------- */
/* out_rgba: width*height*4 float32, row-major, y down.  out_is_device = 1:
 * HBM pointer, async on `hip_stream`; 0: host pointer, the call syncs. */
gs_status gs_render(gs_handle *h, const float view[16], const float proj[16], int32_t width,
                    int32_t height, float *out_rgba, int32_t out_is_device, void *hip_stream);
/* Same frame, written as packed BGRA8Unorm (4 B/pixel, bytes B,G,R,A): the
 * drawable format of metal_renderer.mm:58 / instanced_splat_renderer.mm:269-271,
 * converted inside the composite (clamp [0,1], x255, round to nearest even). */
gs_status gs_render_bgra8(gs_handle *h, const float view[16], const float proj[16], int32_t width,
                          int32_t height, uint8_t *out_bgra, int32_t out_is_device, void *hip_stream);
gs_status gs_last_stats(gs_handle *h, gs_stats *out);
/* stage_timing 2: preprocess and composite kernel times (ms, from the events
 * in their dispatch packets) of the last min(max_frames, 64) frames rendered
 * since stage timing was set, oldest first; waits for those frames.  *count
 * = frames written (0 when stage_timing != 2). */
gs_status gs_kernel_times(gs_handle *h, int32_t max_frames, float *ms_preprocess, float *ms_composite,
                          int32_t *count);

/* ---- stage-level entry points (tests, multi-GPU orchestration) --------- */
/* Project all splats; copies the 48-byte records (gs_record layout below),
 * depth keys and tile counts to HOST arrays of length gs_point_count(). */
gs_status gs_project_host(gs_handle *h, const float view[16], const float proj[16], int32_t width,
                          int32_t height, void *records, uint32_t *dkeys, uint32_t *ntiles);
/* Sorted (key, value) pairs of the last frame copied to host; returns count. */
gs_status gs_sorted_pairs_host(gs_handle *h, uint32_t *keys, uint32_t *vals, int64_t cap, int64_t *count);
/* Stand-alone LSD radix sort of device arrays (stable, key bits [0, bits)).
 * tmp_keys/tmp_vals: n elements each; result ends in keys/vals. */
gs_status gs_radix_sort_pairs(uint32_t *keys, uint32_t *vals, uint32_t *tmp_keys, uint32_t *tmp_vals,
                              int64_t n, int32_t bits, void *hip_stream);

/* ---- multi-GPU: bin-row ownership across ranks ----- */
/* No reference counterpart (the reference is single-GPU Metal).
 * Shard = contiguous splat-index range [index_base, index_base + n) of the
 * global scene.  Every 32-px bin row of the frame has one owning rank. */
gs_status gs_shard_configure(gs_handle *h, int32_t rank, int32_t world, int64_t index_base);
/* Bin-row ownership: owner[by] = rank owning 32-px bin row by, for every
 * bin row of the frame (ceil(height/32) entries).  Default (no table, or
 * nrows = 0): rank r owns the contiguous rows [r*R/world, (r+1)*R/world).
 * Every rank must install the same table (e.g. rebalanced from the last
 * frame's per-row cost). */
gs_status gs_shard_set_rows(gs_handle *h, const uint8_t *owner, int32_t nrows);
/* Exchange buffers (send and receive alike) hold n records as GS_XREGIONS
 * regions one after another: the n 48-B records (the projection's record,
 * exclusion masks included), then n binning-rect lo words, n hi words and n
 * 15-bit depth keys (4 B each).  On the send side every region is grouped by
 * destination (the same counts); an all-to-all moves each region separately
 * (per-peer sizes = records x that region's bytes per record, listed by
 * gs_exchange_regions), which leaves the receiver the same layout in
 * source-rank order. */
#define GS_XREGIONS 4
/* Project the local shard and pack, for every visible splat and every rank
 * owning a bin row its rect touches, one exchange record into `send`
 * (device memory, capacity `send_cap_bytes`), grouped by destination, index
 * order inside.  Writes world send counts (in records) to host `send_counts`.
 * Bytes per record over all regions: gs_exchange_record_bytes(). */
gs_status gs_shard_project(gs_handle *h, const float view[16], const float proj[16], int32_t width,
                           int32_t height, void *send, int64_t send_cap_bytes, int64_t *send_counts,
                           void *hip_stream);
/* Bin, sort and composite the received records (recv_count of them, in the
 * exchange layout above, concatenated in source-rank order, i.e. global
 * index order) into this rank's band buffer `out_rgba` (device): the owned
 * bin rows stacked in ascending order, 32 pixel rows each, width pixels
 * wide, fp32 RGBA.  `recv` (device) is read only. */
gs_status gs_shard_render(gs_handle *h, void *recv, int64_t recv_count, int32_t width, int32_t height,
                          float *out_rgba, void *hip_stream);
/* The same render with its composite on a second stream: the lists (scan,
 * duplicate, sorts) run on hip_stream, the composite and the depth-cut tail
 * on composite_stream once the lists are ready, so work the caller queues on
 * hip_stream next (the next frame's gs_shard_project) runs beside this
 * composite.  out_rgba is complete on composite_stream; recv must stay valid
 * until then.  The next render's lists wait for this composite on the device.
 * (Two frames in flight per rank: DESIGN.md §6e.) */
gs_status gs_shard_render_split(gs_handle *h, void *recv, int64_t recv_count, int32_t width, int32_t height,
                                float *out_rgba, void *hip_stream, void *composite_stream);

/* Replicated-scene bands (SURVEY §8(e) fallback).  The handle
 * holds the WHOLE scene (gs_create / gs_create_subset over all splats) and is
 * configured with gs_shard_configure(h, rank, world, 0) (+ gs_shard_set_rows).
 * Renders this rank's owned 32-px bin rows of the frame into out_band (device,
 * fp32 RGBA, the gs_shard_render band layout: owned rows stacked in ascending
 * order, rows x 32 x width); no exchange.  Bit-identical to those rows of
 * gs_render.  With world 1 the band is the whole frame. */
gs_status gs_band_render(gs_handle *h, const float view[16], const float proj[16], int32_t width, int32_t height,
                         float *out_band, void *stream);
int32_t gs_exchange_record_bytes(void); /* 60: every region's bytes per record */
/* Bytes per record of each exchange region into bytes_per_record[GS_XREGIONS]
 * (may be null); returns GS_XREGIONS. */
int32_t gs_exchange_regions(int32_t *bytes_per_record);

/* ---- multi-GPU: depth slabs + RGBA reduce --------- */
/* The north star's scheme: splat-index shards, each rank composites one
 * depth slab of the whole frame, and the per-pixel RGBA+weight contributions
 * are sum-reduced (RCCL) into the frame.  Per frame, on every rank:
 *   gs_slab_project   preprocess the shard; hist (device, GS_SLAB_BINS u64) =
 *                     its (splat, bin) pairs per GS_SLAB_BIN_KEYS 15-bit depth keys
 *   (all-reduce SUM of hist; gs_slab_bounds on the host, same on every rank)
 *   gs_slab_pack      one exchange record per visible splat, to the rank whose
 *                     slab [bounds[d], bounds[d+1]) holds its key
 *   (all-to-all of counts and records)
 *   gs_slab_render    sort/bin/composite the slab over the full frame; t_local
 *                     (device, W*H f32) = the slab's own transmittance
 *   (all-gather of t_local into t_all, rank-major [world][H][W])
 *   gs_slab_composite colour pass starting from the product of the earlier
 *                     ranks' (farther slabs') transmittance; out_rgba (device,
 *                     W*H*4 f32) = (C, delta alpha) contributions
 *   (reduce SUM of out_rgba = the frame)
 * Rank order is composite (far-to-near) order.  APPROXIMATE: the frame equals
 * the 1-GPU frame up to fp32 reassociation of the transmittance product, and a
 * pixel within rounding of the 0.99 / 0.01 break may stop one fragment
 * earlier or later; the row scheme above is the bit-identical
 * one.  No fragment cap.  `recv` must stay alive until gs_slab_composite
 * returns. */
#define GS_SLAB_BINS 2048   /* histogram bins ... */
#define GS_SLAB_BIN_KEYS 16 /* ... of 16 depth keys: slab bounds are multiples of 16 */
gs_status gs_slab_project(gs_handle *h, const float view[16], const float proj[16], int32_t width, int32_t height,
                          uint64_t *hist, void *hip_stream);
/* bounds[world + 1] (depth keys) from the summed histogram (host): slabs of
 * equal pair counts, to one histogram bin. */
gs_status gs_slab_bounds(const uint64_t *hist, int32_t world, uint32_t *bounds);
gs_status gs_slab_pack(gs_handle *h, const uint32_t *bounds, void *send, int64_t send_cap_bytes, int64_t *send_counts,
                       void *hip_stream);
gs_status gs_slab_render(gs_handle *h, void *recv, int64_t recv_count, int32_t width, int32_t height, float *t_local,
                         void *hip_stream);
gs_status gs_slab_composite(gs_handle *h, const float *t_all, float *out_rgba, void *hip_stream);

/* ---- multi-GPU from one process (gs_create_sharded) ------ */
/* A group splits the (cropped) scene into num_gpus contiguous splat-index
 * shards, one per device, and renders whole frames into devices[0] with the
 * bin-row scheme (bit-identical to one GPU) or the depth-slab
 * scheme.  One worker thread per rank drives the gs_shard_* /
 * gs_slab_* steps above; collectives run over RCCL (xGMI) when every rank has
 * its own device (GS_TRANSPORT_AUTO), or as peer copies (GS_TRANSPORT_COPY,
 * required when ranks share a device).  Drop-in use: replace
 * gs_create/gs_initialize/gs_render by their gs_group counterparts. */
typedef struct gs_group gs_group;
typedef enum { GS_SCHEME_ROWS = 0, GS_SCHEME_SLABS = 1, GS_SCHEME_BANDS = 2 } gs_scheme;
typedef enum { GS_TRANSPORT_AUTO = 0, GS_TRANSPORT_RCCL = 1, GS_TRANSPORT_COPY = 2 } gs_transport;
gs_status gs_create_sharded(const char *ply_path, const gs_options *opt, int32_t num_gpus, gs_group **out);
gs_status gs_create_sharded_from_handle(const gs_handle *scene, int32_t num_gpus, gs_group **out);
/* Replicated-scene group: every rank holds the WHOLE
 * (cropped) scene and renders its owned bin rows (GS_SCHEME_BANDS, the only
 * scheme of such a group); the bands are gathered into the frame on
 * devices[0].  Bit-identical to one GPU's frame. */
gs_status gs_create_replicated(const char *ply_path, const gs_options *opt, int32_t num_gpus, gs_group **out);
gs_status gs_create_replicated_from_handle(const gs_handle *scene, int32_t num_gpus, gs_group **out);
/* devices: num_gpus ordinals (NULL = 0 .. num_gpus-1; repeats allowed with
 * GS_TRANSPORT_COPY); transport: gs_transport. */
gs_status gs_group_initialize(gs_group *g, const int32_t *devices, int32_t transport);
gs_status gs_group_set_scheme(gs_group *g, int32_t scheme);
/* Bound of every host wait of the group (default 60 s, or GS_COMM_TIMEOUT_MS).
 * A wait that expires, or an RCCL communicator reporting an asynchronous
 * error (ncclCommGetAsyncError, polled during the waits), aborts every
 * communicator and fails the call with GS_ERR_COMM; the group is then
 * unusable.  (No reference counterpart: instanced_splat_renderer.mm:319-336
 * is the reference's only failure path.) */
gs_status gs_group_set_timeout(gs_group *g, int32_t timeout_ms);
/* The frame (fp32 RGBA, W*H*16 B) on devices[0]: out_is_device = 1 async on
 * hip_stream (a stream of devices[0]); 0 = host memory, the call syncs. */
gs_status gs_group_render(gs_group *g, const float view[16], const float proj[16], int32_t width, int32_t height,
                          float *out_rgba, int32_t out_is_device, void *hip_stream);
/* Two frames in flight, rows scheme: n = 2 lets
 * gs_group_render_pipelined overlap one frame's record all-to-all (on a
 * communicator set of its own) with the previous frame's render and gather.
 * n = 1 (default): gs_group_render only.  Not while a frame is in flight. */
gs_status gs_group_set_frames_in_flight(gs_group *g, int32_t n);
/* Projects this view's frame and starts its all-to-all, then renders and
 * gathers the PREVIOUS call's frame into out_rgba (same conventions as
 * gs_group_render; out_rgba must hold that frame: the previous call's width
 * x height): *produced = 1 when out_rgba holds that frame (0 on the first
 * call).  Every frame is bit-identical to gs_group_render's of the same
 * view.  gs_group_flush finishes the frame still in flight (*produced = 0 when
 * none); gs_group_render fails with GS_ERR_STATE while one is. */
gs_status gs_group_render_pipelined(gs_group *g, const float view[16], const float proj[16], int32_t width,
                                    int32_t height, float *out_rgba, int32_t out_is_device, void *hip_stream,
                                    int32_t *produced);
gs_status gs_group_flush(gs_group *g, float *out_rgba, int32_t out_is_device, void *hip_stream, int32_t *produced);
int64_t gs_group_point_count(const gs_group *g);
int32_t gs_group_size(const gs_group *g);
int32_t gs_group_transport(const gs_group *g); /* the transport in use, -1 before initialize */
gs_status gs_group_last_stats(gs_group *g, int32_t rank, gs_stats *out);
void gs_group_destroy(gs_group *g);

/* ---- PLY loader (PLYLoader::load drop-in) ----------------------------- */
/* Loads into a malloc'd PointData array (62 floats/point).  compat = 1
 * reproduces every reference quirk (ASCII 2N points). */
gs_status gs_ply_load(const char *path, int32_t compat, float **points, int64_t *n);
void gs_ply_free(float *points);

/* ---- camera math (TrackballCamera::makeLookAt / makePerspective) ------ */
void gs_look_at(const float eye[3], const float center[3], const float up[3], float out[16]);
void gs_perspective(float fov_degrees, float aspect, float znear, float zfar, float out[16]);

/* 48-byte per-splat record (preprocess output, composite input). */
typedef struct gs_record {
    float cx, cy, ax, ay;
    float bx, by, opacity, r;
    float g, b;
    uint32_t rect_lo, rect_hi;
} gs_record;

#ifdef __cplusplus
}
#endif
#endif /* GSPLAT_H */
