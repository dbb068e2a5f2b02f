/*
 * gs_oracle.h — CPU ORACLE for the Gaussian-splat tile rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) — never as the product path.  The product
 * (gaussian_splat_amd/libgsplat.so) never links or loads it.
 *
 * What it is: a plain-C restatement of the reference's per-frame algorithm
 * (nshelton/gaussian_splat), following SURVEY.md §8(a) row by row:
 *   I1  PLYLoader::load / parseHeader / shToRGB   src/ply_loader.cpp:22-205,207-248,11-20
 *   I2  crop |x|,|y|,|z| < 5                      src/instanced_splat_renderer.mm:382-386
 *   C1  makeLookAt / makePerspective / P·V        src/trackball_camera.mm:136-163,
 *                                                 src/instanced_splat_renderer.mm:453
 *   K1  quaternionToMatrix                        shaders/gaussian_splat_tile.metal:40-49
 *   K2  computeCovariance3D                       shaders/gaussian_splat_tile.metal:51-60
 *   K3  vertex_main projection                    shaders/gaussian_splat_tile.metal:85-131
 *   K4  eigenSym2x2 + 3-sigma radii               shaders/gaussian_splat_tile.metal:62-83,136-140
 *   K5  quad emit                                 shaders/gaussian_splat_tile.metal:142-156
 *   K6  fixed-function raster (closed form)       pipeline, instanced_splat_renderer.mm:136-156
 *   F1  fragment_main: gaussian, alpha            shaders/gaussian_splat_tile.metal:184-197
 *   S1  insertion sort, descending half depth     shaders/gaussian_splat_tile.metal:239-249
 *   A1  front-to-back composite, A>=0.99 break    shaders/gaussian_splat_tile.metal:251-266
 *   A1' live-50 composite, T<0.01 break           shaders/gaussian_splat_50layer.metal:208-222
 *   N2  SH degree 1..3 colour (no reference counterpart; standard 3DGS basis)
 *
 * Parity status:
 *   - I1 is PINNED: tests compare this restatement with the reference's own
 *     src/ply_loader.cpp compiled unchanged into oracle/_ref/ (oracle/Makefile).
 *   - C1, K1-K6, F1, S1 and A1 are "parity unpinned" by execution: the Metal shaders
 *     and the Apple-simd camera cannot be built in this image (no Metal
 *     toolchain, no metal_stdlib, no <simd/simd.h>), and the reference ships
 *     no tests or golden vectors.  They are checked against hand-derived
 *     known-answer vectors (tests/golden/known_answers.json), each computed
 *     by hand from the cited reference lines.
 *
 * Arithmetic contract: every expression is evaluated in the order written in
 * DESIGN.md §2 (explicit fmaf where a fused op is specified, none elsewhere;
 * compile with -ffp-contract=off).  The HIP kernels follow the same order, so
 * per-splat records and framebuffers are expected to agree bit for bit.
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* PointData layout of src/ply_loader.h:7-28 — 62 floats, 248 bytes. */
#define ORA_POINT_FLOATS 62

/* I1: restatement of PLYLoader::load.  On success *out is malloc'd with
 * (*n) * 62 floats in PointData order.  Returns 1 on success (non-empty),
 * 0 on failure (mirrors the reference's bool). */
int ora_ply_load(const char *path, float **out, int64_t *n);
void ora_free(void *p);

/* I2: crop, returns number kept; keep[] receives kept indices (crop order). */
int64_t ora_crop(const float *points, int64_t n, float radius, int64_t *keep);

/* C1 camera math (column-major float4x4, m[col*4+row]). */
void ora_look_at(const float eye[3], const float center[3], const float up[3], float out[16]);
void ora_perspective(float fov_degrees, float aspect, float znear, float zfar, float out[16]);
void ora_mat4_mul(const float a[16], const float b[16], float out[16]); /* out = a·b */
void ora_camera_position(const float view[16], float out[3]);

typedef struct {
    int64_t n;
    const float *pos;      /* n*3 */
    const float *rot;      /* n*4, w x y z, raw (normalised in K1) */
    const float *scale;    /* n*3, activated (exp) */
    const float *opacity;  /* n, activated (sigmoid) */
    const float *color;    /* n*3: rgb (sh_degree==0) or raw f_dc (sh_degree>0) */
    const float *sh_rest;  /* n*45, PLY order (channel-major), or NULL */
    int sh_degree;         /* 0..3 */
} ora_scene;

/* Per-splat projection record: exactly the 48-byte record the HIP
 * preprocess kernel writes (gaussian_splat_amd/csrc/kernels/gs_common.h). */
typedef struct {
    float cx, cy, ax, ay;       /* centre (window px, y down); A = e1 * 3/r1 */
    float bx, by, opacity, r;   /* B = e2 * 3/r2; opacity; red */
    float g, b;                 /* green, blue */
    uint32_t rect_lo, rect_hi;  /* inclusive pixel rect: x0|y0<<16, x1|y1<<16 */
} ora_record;

typedef struct {
    float zf;          /* -view.z */
    float a, b, c;     /* 2D covariance (+1e-4 on a, c) */
    float r1, r2;      /* 3-sigma radii */
    float e1x, e1y;    /* major eigenvector */
    uint32_t dkey;     /* 0x7C00 - half_bits(zf): ascending = descending depth */
    uint32_t ntiles;   /* tiles touched by rect (0 = culled) */
    int visible;
} ora_debug;

/* MLAB = the 6-layer k-buffer of gaussian_splat.metal:201-361 (half
 * arithmetic, arrival order, resolve front to back); no cap, no slabs. */
enum { ORA_MODE_TILE = 0, ORA_MODE_LIVE50 = 1, ORA_MODE_MLAB = 2 };

typedef struct {
    int mode;          /* ORA_MODE_TILE (default contract) or ORA_MODE_LIVE50 */
    int cap;           /* 0 = no cap; else keep first `cap` fragments in arrival (= index) order */
    int nthreads;      /* OpenMP threads, <=0 = default */
} ora_options;

typedef struct {
    int64_t visible;   /* splats with at least one tile */
    int64_t pairs;     /* (splat, tile) pairs P */
    int64_t tiles;     /* T */
} ora_stats;

/* K1..K5 + tile rect for splat i. */
void ora_project(const ora_scene *s, int64_t i, const float view[16], const float proj[16],
                 const float vp[16], const float campos[3], int width, int height,
                 ora_record *rec, ora_debug *dbg);

/* Whole-scene projection (OpenMP). Arrays are length n. */
void ora_project_all(const ora_scene *s, const float view[16], const float proj[16],
                     int width, int height, ora_record *rec, uint32_t *dkey, uint32_t *ntiles,
                     int nthreads);

/* Full frame: out_rgba is width*height*4 floats, row-major, y down. */
int ora_render(const ora_scene *s, const float view[16], const float proj[16], int width,
               int height, const ora_options *opt, float *out_rgba, ora_stats *stats);

/* Bin, sort (S1) and composite an explicit record list (index = arrival
 * order) into the 32-px pixel rows r (r = py / 32) with owner[r] == rank
 * (owner == NULL: every row); compact = 1 writes the owned rows stacked in
 * ascending order (the multi-GPU band layout).  Culled records are all-zero
 * (dkey 0, rect_hi 0, opacity 0). */
int ora_composite_records(const ora_record *rec, const uint32_t *dkey, int64_t n, int width, int height,
                          const ora_options *opt, const uint8_t *owner, int rank, int compact, float *out,
                          ora_stats *stats);

/* Depth-slab multi-GPU decomposition:
 * pass 1 writes W*H floats, the slab's own transmittance (tile rule: 1 - A,
 * with the A >= 0.99 break; live50: T with the T < 0.01 break); pass 2 starts
 * from the product of t_all[j] (j < slab_rank, [world][H][W]) and writes the
 * (C, delta alpha) contributions, W*H*4 floats, whose sum over slabs is the
 * frame.  No cap.  Returns 0 on bad arguments. */
int ora_composite_slab(const ora_record *rec, const uint32_t *dkey, int64_t n, int width, int height,
                       const ora_options *opt, int pass, int slab_rank, const float *t_all, float *out);

/* Composite a single synthetic fragment list (depth, rgb, alpha) with the S1
 * sort and A1 / A1' rule — the unit the reference's tile_sort_composite and
 * compute_sort_composite operate on.  frags: n*5 floats (depth, r, g, b, a),
 * in arrival order.  out: rgba. */
void ora_composite_list(const float *frags, int n, int mode, int cap, float out[4]);

/* Helpers exposed for tests. */
uint16_t ora_f32_to_f16_bits(float f);
float ora_expf(float x);
float ora_gauss(float q); /* exp(-q/2) (round-1 form, test helper) */
float ora_gauss2(float qs); /* 2^-qs: the composite gaussian on the scaled conic (F1) */
/* fp32 RGBA -> BGRA8Unorm (metal_renderer.mm:58, instanced_splat_renderer.mm:269-271):
 * per channel clamp to [0,1], x255, round half to even; bytes B,G,R,A.
 * Parity unpinned (Metal's conversion cannot run here). */
void ora_to_bgra8(const float *rgba, int64_t npix, uint8_t *bgra);

#ifdef __cplusplus
}
#endif
#endif
