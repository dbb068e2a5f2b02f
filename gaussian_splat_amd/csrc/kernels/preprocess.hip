// preprocess.hip — per-splat projection.
//
// One lane per splat, SoA float4 loads (fully coalesced 16 B/lane), output the
// 48-byte composite record, the 15-bit depth key and the tile count.  This is
// the reference's vertex_main (shaders/gaussian_splat_tile.metal:85-157) run
// ONCE per splat instead of six times per instance, plus the closed form of
// Metal's fixed-function quad raster (K6) reduced to a conservative pixel
// rectangle.  Memory-bound: N·(B_in + 56) bytes per frame.
#include "gs_device.h"
#include <hip/hip_ext.h>

#include "gs_kernels.h"
#include "gs_masks.h"
#include "gs_wave.h"

namespace gs {

#ifndef GS_PRE_NT  // A/B knob: scene loads with the non-temporal hint (read once per frame)
#define GS_PRE_NT 1
#endif
typedef float gs_f4 __attribute__((ext_vector_type(4)));
typedef float gs_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float4 scene_load(const float4* p) {
#if GS_PRE_NT
    const gs_f4 v = __builtin_nontemporal_load(reinterpret_cast<const gs_f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
#else
    return *p;
#endif
}
__device__ __forceinline__ float2 scene_load(const float2* p) {
#if GS_PRE_NT
    const gs_f2 v = __builtin_nontemporal_load(reinterpret_cast<const gs_f2*>(p));
    return make_float2(v.x, v.y);
#else
    return *p;
#endif
}
__device__ __forceinline__ float scene_load(const float* p) {
#if GS_PRE_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

// A splat's SH rest coefficients, k-major with r,g,b interleaved: flat j =
// 3k + ch, in float4 planes (coalesced across lanes) plus one scalar plane.
template <int DEG>
struct ShCoef {
    static constexpr int K = DEG == 0 ? 0 : (DEG == 1 ? 3 : (DEG == 2 ? 8 : 15));
    static constexpr int NF = 3 * K;
    float c[NF > 0 ? NF : 1];
};
template <int DEG>
__device__ __forceinline__ void sh_load(const SceneDev& s, uint32_t i, ShCoef<DEG>& k) {
    constexpr int NF = ShCoef<DEG>::NF, NP4 = NF / 4;
#pragma unroll
    for (int m = 0; m < NP4; ++m) {
        const float4 v = scene_load(&s.sh4[(size_t)m * s.n + i]);
        k.c[4 * m + 0] = v.x;
        k.c[4 * m + 1] = v.y;
        k.c[4 * m + 2] = v.z;
        k.c[4 * m + 3] = v.w;
    }
    if constexpr (NF % 4 != 0) k.c[NF - 1] = scene_load(&s.sh1[i]);
}

template <int DEG>
__device__ __forceinline__ void sh_color(const ShCoef<DEG>& coef, float px, float py, float pz,
                                         const float* campos, float c0, float c1, float c2,
                                         float& r, float& g, float& b) {
    if constexpr (DEG == 0) {
        r = c0; g = c1; b = c2;  // colour converted at load (ply_loader.cpp:132-139)
    } else {
        if (c0 == 0.0f && c1 == 0.0f && c2 == 0.0f) {  // all-zero f_dc quirk (ply_loader.cpp:133)
            r = g = b = 0.0f;
            return;
        }
        const float SH_C0 = 0.28209479177387814f;
        const float C1 = 0.4886025119029199f;
        float dx = px - campos[0], dy = py - campos[1], dz = pz - campos[2];
        float l2 = __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx));
        float inv = 1.0f / sqrtf(l2);
        float x = dx * inv, y = dy * inv, z = dz * inv;
        constexpr int K = DEG == 1 ? 3 : (DEG == 2 ? 8 : 15);
        float bas[K];
        bas[0] = (-C1) * y;
        bas[1] = C1 * z;
        bas[2] = (-C1) * x;
        if constexpr (DEG >= 2) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            bas[3] = 1.0925484305920792f * xy;
            bas[4] = -1.0925484305920792f * yz;
            bas[5] = 0.31539156525252005f * ((2.0f * zz - xx) - yy);
            bas[6] = -1.0925484305920792f * xz;
            bas[7] = 0.5462742152960396f * (xx - yy);
            if constexpr (DEG >= 3) {
                bas[8] = (-0.5900435899266435f * y) * (3.0f * xx - yy);
                bas[9] = (2.890611442640554f * xy) * z;
                bas[10] = (-0.4570457994644658f * y) * ((4.0f * zz - xx) - yy);
                bas[11] = (0.3731763325901154f * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
                bas[12] = (-0.4570457994644658f * x) * ((4.0f * zz - xx) - yy);
                bas[13] = (1.445305721320277f * z) * (xx - yy);
                bas[14] = (-0.5900435899266435f * x) * (xx - 3.0f * yy);
            }
        }
        float acc0 = SH_C0 * c0, acc1 = SH_C0 * c1, acc2 = SH_C0 * c2;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc0 = __builtin_fmaf(bas[k], coef.c[3 * k + 0], acc0);
            acc1 = __builtin_fmaf(bas[k], coef.c[3 * k + 1], acc1);
            acc2 = __builtin_fmaf(bas[k], coef.c[3 * k + 2], acc2);
        }
        acc0 = acc0 + 0.5f;
        acc1 = acc1 + 0.5f;
        acc2 = acc2 + 0.5f;
        r = fminf(fmaxf(acc0, 0.0f), 1.0f);
        g = fminf(fmaxf(acc1, 0.0f), 1.0f);
        b = fminf(fmaxf(acc2, 0.0f), 1.0f);
    }
}


#ifndef GS_PRE_EARLY  // A/B knob: 1 = rotation, scale (and the SH0 colour) loaded with the position
#define GS_PRE_EARLY 0     // (one dependent round trip fewer, bytes for culled splats too)
#endif

#ifndef GS_PRE_PRIO  // A/B knob: issue priority (0..3) of the projection's waves
#define GS_PRE_PRIO 0
#endif

#ifndef GS_PRE_FULLREC  // A/B knob: 1 = culled splats of a full frame write a zero record (whole-line record stores)
#define GS_PRE_FULLREC 1
#endif

#ifndef GS_PRE_BAND_CULL  // A/B knob: 1 = band frames cull splats off the band before their covariance
#define GS_PRE_BAND_CULL 1
#endif

#ifndef GS_PRE_WAVES  // A/B knob: min waves per SIMD (caps the VGPRs)
#define GS_PRE_WAVES 8
#endif

// EPI: what follows the per-splat work.  0: nothing (each lane returns on its
// own); 1: the scan's reduce half and fills (PreFuse).  The epilogue is
// compiled only into its own instance, so the plain kernel keeps its
// registers (63 VGPRs, no scratch).
// Band frames (U.band_y0 > 0 or U.band_y1 < H - 1): true when
// the splat's rect provably misses the band's pixel rows, from its centre row
// and a bound on its half-height that needs no covariance: the 2D
// covariance's largest eigenvalue is at most 1.5 ||A||_F^2 s_max^2 + 1e-4
// (A = J W, Gershgorin over A Sigma A^T with lambda_max(Sigma) = s_max^2),
// so hy <= 1.0117 * 3 sqrt(l1) * 1.0001 + 1 (the rect code below); slack
// factors and a pixel of margin each side cover the rounding.  A splat this
// culls gets exactly what the full path gives it (an empty rect).
__device__ __forceinline__ bool band_culled(const FrameUniforms& U, const float* V, float vx, float vy, float zf,
                                            float ndcy, const float4& a2) {
    const float fx = U.P[0] * ((float)U.width * 0.5f), fy = U.P[5] * ((float)U.height * 0.5f);
    const float iz = 1.0f / zf, iz2 = iz * iz;
    const float j00 = fx * iz, j02 = ((-fx) * vx) * iz2, j11 = fy * iz, j12 = ((-fy) * vy) * iz2;
    const float a00 = __builtin_fmaf(j02, V[2], j00 * V[0]), a01 = __builtin_fmaf(j02, V[6], j00 * V[4]);
    const float a02 = __builtin_fmaf(j02, V[10], j00 * V[8]), a10 = __builtin_fmaf(j12, V[2], j11 * V[1]);
    const float a11 = __builtin_fmaf(j12, V[6], j11 * V[5]), a12 = __builtin_fmaf(j12, V[10], j11 * V[9]);
    const float n2 = a00 * a00 + a01 * a01 + a02 * a02 + a10 * a10 + a11 * a11 + a12 * a12;
    const float smax = fmaxf(fmaxf(fabsf(a2.x), fabsf(a2.y)), fabsf(a2.z));
    const float l1 = (1.5f * n2) * (smax * smax) * 1.001f + 3e-4f;
    const float hy = (1.0117f * 3.0f) * sqrtf(l1) * 1.0002f + 2.0f;
    const float cy = (1.0f - ndcy) * ((float)U.height * 0.5f);
    // (NaN anywhere: both false, not culled, the full path decides)
    return cy - hy - 0.5f > (float)U.band_y1 + 1.0f || cy + hy - 0.5f < (float)U.band_y0 - 1.0f;
}

template <int DEG, int EPI, bool BAND = false>
__global__ __launch_bounds__(256, (EPI == 2 && DEG == 3) ? 7 : GS_PRE_WAVES) void preprocess_kernel(SceneDev s, const FrameUniforms U,
                                                         float4* __restrict__ rec, uint32_t* __restrict__ dkey,
                                                         uint32_t* __restrict__ rect_lo,
                                                         uint32_t* __restrict__ rect_hi,
                                                         unsigned long long* __restrict__ zero8,
                                                         const PreFuse fuse, const ShardFuse shard) {
    uint32_t i = blockIdx.x * 256u + threadIdx.x;
#if GS_PRE_PRIO
    // (A/B) the projection bounds the pipelined frame (projection + chain):
    // its waves ahead of the co-running composite's in issue arbitration
    __builtin_amdgcn_s_setprio(GS_PRE_PRIO);
#endif
    if (i < 2 && zero8) zero8[i] = 0ull;
    if constexpr (EPI == 0)
        if (i >= s.n) return;
    uint32_t rlo = kEmptyRectLo, rhi = 0u;
    uint32_t key = 0;
    if (i < s.n) {
    const float* V = U.V;
    const float* VP = U.VP;

    float4 a0 = scene_load(&s.p0[i]);
#if GS_PRE_EARLY
    float4 q_e = scene_load(&s.p1[i]);
    float4 a2_e = scene_load(&s.p2[i]);
    [[maybe_unused]] float2 a3_e;
    if constexpr (DEG == 0) a3_e = scene_load(&s.p3[i]);
#endif
    float px = a0.x, py = a0.y, pz = a0.z;
    // K3: view position, zFront (tile.metal:94-105)
    float vx = xform_row(V, 0, px, py, pz);
    float vy = xform_row(V, 1, px, py, pz);
    float vz = xform_row(V, 2, px, py, pz);
    float zf = -vz;
#if GS_PRE_EARLY
    // (an empty asm consuming the early loads: the compiler otherwise sinks
    // them back into the branch that uses them)
    asm volatile("" : "+v"(q_e.x), "+v"(q_e.y), "+v"(q_e.z), "+v"(q_e.w), "+v"(a2_e.x), "+v"(a2_e.y), "+v"(a2_e.z),
                 "+v"(a2_e.w));
    if constexpr (DEG == 0) asm volatile("" : "+v"(a3_e.x), "+v"(a3_e.y));
#endif
    if (zf >= 1e-4f) {
        // K6 z-clip on NDC z in [0,1] (tile.metal:145-152)
        float clx = xform_row(VP, 0, px, py, pz);
        float cly = xform_row(VP, 1, px, py, pz);
        float clz = xform_row(VP, 2, px, py, pz);
        float clw = xform_row(VP, 3, px, py, pz);
        float invw = 1.0f / clw;
        float ndcz = clz * invw;
        if (ndcz >= 0.0f && ndcz <= 1.0f && zf >= 0.001f) {
#if GS_PRE_EARLY
            const float4 q = q_e, a2 = a2_e;
#else
            float4 a2 = scene_load(&s.p2[i]);
            // (BAND: a splat whose rect provably misses the band's rows is
            // culled before its rotation is read and its covariance formed)
            if (!BAND || !band_culled(U, V, vx, vy, zf, cly * invw, a2)) {
            float4 q = scene_load(&s.p1[i]);
#endif
            // K1 (tile.metal:40-49)
            float qs = q.x * q.x;
            qs = __builtin_fmaf(q.y, q.y, qs);
            qs = __builtin_fmaf(q.z, q.z, qs);
            qs = __builtin_fmaf(q.w, q.w, qs);
            float qi = 1.0f / sqrtf(qs);
            float w = q.x * qi, x = q.y * qi, y = q.z * qi, z = q.w * qi;
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
            float wx = w * x, wy = w * y, wz = w * z;
            float R00 = 1.0f - 2.0f * (yy + zz), R10 = 2.0f * (xy + wz), R20 = 2.0f * (xz - wy);
            float R01 = 2.0f * (xy - wz), R11 = 1.0f - 2.0f * (xx + zz), R21 = 2.0f * (yz + wx);
            float R02 = 2.0f * (xz + wy), R12 = 2.0f * (yz - wx), R22 = 1.0f - 2.0f * (xx + yy);
            // K2: M = R S, Sigma = M M^T (tile.metal:51-60)
            float M00 = R00 * a2.x, M01 = R01 * a2.y, M02 = R02 * a2.z;
            float M10 = R10 * a2.x, M11 = R11 * a2.y, M12 = R12 * a2.z;
            float M20 = R20 * a2.x, M21 = R21 * a2.y, M22 = R22 * a2.z;
            float S00 = dot3(M00, M01, M02, M00, M01, M02);
            float S01 = dot3(M00, M01, M02, M10, M11, M12);
            float S02 = dot3(M00, M01, M02, M20, M21, M22);
            float S11 = dot3(M10, M11, M12, M10, M11, M12);
            float S12 = dot3(M10, M11, M12, M20, M21, M22);
            float S22 = dot3(M20, M21, M22, M20, M21, M22);
            // K3 + Jacobian (tile.metal:109-127): cov = J (W Sigma W^T) J^T,
            // evaluated as A Sigma A^T with A = J W (2x3; the contract's order,
            // Sigma symmetric, J's zero entries skipped).
            // W(r,c) = V[c*4+r]; J with the reference's z-column sign (:117-123).
            float fx = U.P[0] * ((float)U.width * 0.5f);
            float fy = U.P[5] * ((float)U.height * 0.5f);
            float iz = 1.0f / zf;
            float iz2 = iz * iz;
            float J00 = fx * iz, J02 = ((-fx) * vx) * iz2;
            float J11 = fy * iz, J12 = ((-fy) * vy) * iz2;
            float A00 = __builtin_fmaf(J02, V[2], J00 * V[0]);
            float A01 = __builtin_fmaf(J02, V[6], J00 * V[4]);
            float A02 = __builtin_fmaf(J02, V[10], J00 * V[8]);
            float A10 = __builtin_fmaf(J12, V[2], J11 * V[1]);
            float A11 = __builtin_fmaf(J12, V[6], J11 * V[5]);
            float A12 = __builtin_fmaf(J12, V[10], J11 * V[9]);
            float B00 = dot3(A00, A01, A02, S00, S01, S02);
            float B01 = dot3(A00, A01, A02, S01, S11, S12);
            float B02 = dot3(A00, A01, A02, S02, S12, S22);
            float B10 = dot3(A10, A11, A12, S00, S01, S02);
            float B11 = dot3(A10, A11, A12, S01, S11, S12);
            float B12 = dot3(A10, A11, A12, S02, S12, S22);
            float ca = dot3(B00, B01, B02, A00, A01, A02);
            float cb = dot3(B00, B01, B02, A10, A11, A12);
            float cc = dot3(B10, B11, B12, A10, A11, A12);
            ca = ca + 1e-4f;  // tile.metal:129-131
            cc = cc + 1e-4f;
            // K4 eigenSym2x2 (tile.metal:62-83) and radii (:136-140)
            float tr = ca + cc;
            float det = ca * cc - cb * cb;
            float disc = fmaxf(0.0f, (0.25f * tr) * tr - det);
            float sq = sqrtf(disc);
            float l1 = 0.5f * tr + sq;
            float l2 = 0.5f * tr - sq;
            float e1x, e1y;
            if (fabsf(cb) > 1e-8f) {
                float ux = l1 - cc, uy = cb;
                float il = 1.0f / sqrtf(__builtin_fmaf(uy, uy, ux * ux));
                e1x = ux * il;
                e1y = uy * il;
            } else if (ca >= cc) {
                e1x = 1.0f;
                e1y = 0.0f;
            } else {
                e1x = 0.0f;
                e1y = 1.0f;
            }
            float e2x = -e1y, e2y = e1x;
            l1 = fmaxf(l1, 0.0f);
            l2 = fmaxf(l2, 0.0f);
            float r1 = 3.0f * sqrtf(l1);
            float r2 = 3.0f * sqrtf(l2);
            if (r1 > 0.0f && r2 > 0.0f) {
                float W_ = (float)U.width, H_ = (float)U.height;
                float ndcx = clx * invw, ndcy = cly * invw;
                float cx = (ndcx + 1.0f) * (W_ * 0.5f);
                float cy = (1.0f - ndcy) * (H_ * 0.5f);
                float k1 = 3.0f / r1, k2 = 3.0f / r2;
                float hbx = r1 * fabsf(e1x) + r2 * fabsf(e2x);
                float hby = r1 * fabsf(e1y) + r2 * fabsf(e2y);
                float hex = 1.0117f * sqrtf((r1 * e1x) * (r1 * e1x) + (r2 * e2x) * (r2 * e2x));
                float hey = 1.0117f * sqrtf((r1 * e1y) * (r1 * e1y) + (r2 * e2y) * (r2 * e2y));
                float hx = fminf(hbx, hex) * 1.0001f + 1.0f;
                float hy = fminf(hby, hey) * 1.0001f + 1.0f;
                float x0f = ceilf(cx - hx - 0.5f), x1f = floorf(cx + hx - 0.5f);
                float y0f = ceilf(cy - hy - 0.5f), y1f = floorf(cy + hy - 0.5f);
                x0f = fmaxf(x0f, 0.0f);
                y0f = fmaxf(y0f, (float)U.band_y0);  // (0 unless a band frame)
                x1f = fminf(x1f, W_ - 1.0f);
                y1f = fminf(y1f, (float)U.band_y1);  // (H - 1 unless a band frame)
                if (x0f <= x1f && y0f <= y1f) {
                    uint32_t x0 = (uint32_t)x0f, x1 = (uint32_t)x1f, y0 = (uint32_t)y0f, y1 = (uint32_t)y1f;
                    float cr, cg, cbl;
                    // (colour inputs loaded only for splats on screen; loading
                    // them with the shape, a round trip earlier, was measured
                    // slower: 0.30-0.33 vs 0.29 ms, 45 more live registers)
#if GS_PRE_EARLY
                    float2 a3;
                    if constexpr (DEG == 0) a3 = a3_e;
                    else a3 = scene_load(&s.p3[i]);
#else
                    const float2 a3 = scene_load(&s.p3[i]);
#endif
                    ShCoef<DEG> coef;
                    if constexpr (DEG > 0) sh_load<DEG>(s, i, coef);
                    sh_color<DEG>(coef, px, py, pz, U.campos, a2.w, a3.x, a3.y, cr, cg, cbl);
                    float4* o = rec + kRecFloat4 * (size_t)i;
                    const float4 ra = make_float4(cx, cy, e1x * k1, e1y * k1);
                    const float4 rb = make_float4(e2x * k2, e2y * k2, a0.w, cr);
                    // 8x8 cells of the rect the ellipse provably misses (the
                    // composite skips them; frames up to kCellMaskDim px)
#ifdef GS_AB_NO_MASKS  // A/B build: masks off (cost of the masks in this kernel)
                    const uint32_t excl = 0u, bexcl = 0u;
#else
                    uint32_t excl = 0u, bexcl = 0u;
                    if (U.cell_mask) {
                        // a rect within 4x4 cells: its cell mask, and the bin
                        // mask from it; a wider one: no cell claim, its bin mask
                        const RectMasks rm = rect_masks(cx, cy, ra.z, ra.w, rb.x, rb.y, x0, y0, x1, y1);
                        excl = rm.cell;
                        bexcl = rm.bin;
                    }
#endif
                    o[0] = ra;
                    o[1] = rb;
                    if constexpr (kRecFloat4 == 4) o[3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // (whole 64-B slot)
                    o[2] = make_float4(cg, cbl,
                                       __uint_as_float(rect_with_mask(x0 | (y0 << 16), excl & 0xFu, (excl >> 4) & 0xFu)),
                                       __uint_as_float(rect_with_mask(x1 | (y1 << 16), (excl >> 8) & 0xFu, excl >> 12)));
                    key = kDepthInf - half_bits(zf);
                    // binning rect: the same words plus the bin-exclusion mask
                    rlo = rect_with_mask(x0 | (y0 << 16), bexcl & 0xFu, (bexcl >> 4) & 0xFu);
                    rhi = rect_with_mask(x1 | (y1 << 16), (bexcl >> 8) & 0xFu, bexcl >> 12);
                }
            }
#if !GS_PRE_EARLY
            }  // (the band cull)
#endif
        }
    }
#if GS_PRE_FULLREC
    // a culled splat writes a zero record too, so a wave's record stores
    // cover whole lines instead of leaving holes (partially written lines);
    // no list ever holds a culled splat, so its record is never read.  Not in
    // band frames, whose clipped rects cull most splats: there the zeros
    // would outweigh the records.
    if (rlo == kEmptyRectLo && U.band_y0 == 0 && U.band_y1 == U.height - 1) {  // (a visible splat's x0 < 0xFFFF)
        float4* o = rec + kRecFloat4 * (size_t)i;
#pragma unroll
        for (int k = 0; k < kRecFloat4; ++k) o[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#endif
    dkey[i] = key;
    rect_lo[i] = rlo;
    rect_hi[i] = rhi;
    }
    if constexpr (EPI == 2) {
        // the row scheme's destination count (ShardFuse): each splat's
        // destination mask, and this workgroup's per-destination counts into
        // its shard block's (lane d of every wave counts destination d)
        __shared__ uint32_t wc[4][kMaxWorld];
        uint32_t m = 0u;
        if (i < s.n) {
            const BinRect r = bin_rect(rlo, rhi, U.cell_mask != 0);
            if (!r.empty) m = row_mask(r.by0, r.by1, shard.owner);
            shard.dest_mask[i] = m;
        }
        const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
        uint32_t cnt = 0u;
        for (int d = 0; d < shard.world; ++d) {
            const uint64_t bal = __ballot((m >> d) & 1u);
            if (lane == (uint32_t)d) cnt = (uint32_t)__popcll(bal);
        }
        if (lane < (uint32_t)kMaxWorld) wc[wave][lane] = cnt;
        __syncthreads();
        if (threadIdx.x < (uint32_t)shard.world) {
            const uint32_t d = threadIdx.x, c = wc[0][d] + wc[1][d] + wc[2][d] + wc[3][d];
            if (c) atomicAdd(&shard.counts[(size_t)d * shard.nblocks + blockIdx.x / (uint32_t)(kShardItems / 256)], c);
        }
    }
    if constexpr (EPI == 1) {
        // the scan's reduce half: this workgroup's pairs and visible splats
        // into its scan block's sums (the counts scan_duplicate recomputes)
        __shared__ uint3 wsum[4];
        const uint32_t c = rect_tile_count(rlo, rhi, RowOwnership{nullptr, 0u}, U.cell_mask != 0);
        const uint32_t ws = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(c), 63);
        const uint32_t wv = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<false>(c > 0u ? 1u : 0u), 63);
        const uint32_t wm = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp<true>(c), 63);  // (largest count)
        if ((threadIdx.x & 63u) == 0) wsum[threadIdx.x >> 6] = make_uint3(ws, wv, wm);
        // the frame's empty bin ranges and zeroed digit counts
        const uint32_t g = blockIdx.x * 256u + threadIdx.x;
        for (uint32_t z = g; z < fuse.nfill; z += gridDim.x * 256u) fuse.fill[z] = make_uint2(0xFFFFFFFFu, 0xFFFFFFFFu);
        for (uint32_t z = g; z < fuse.nzero; z += gridDim.x * 256u) fuse.zero[z] = 0u;
        for (uint32_t z = g; z < fuse.nzero64; z += gridDim.x * 256u) fuse.zero64[z] = 0ull;
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t b = blockIdx.x / (uint32_t)(kScanItems / 256);
            const uint32_t ps = wsum[0].x + wsum[1].x + wsum[2].x + wsum[3].x;
            const uint32_t pv = wsum[0].y + wsum[1].y + wsum[2].y + wsum[3].y;
            const uint32_t pm = wsum[0].z + wsum[1].z + wsum[2].z + wsum[3].z;
            if (ps) atomicAdd(&fuse.part[b], (unsigned long long)ps);
            if (pv) atomicAdd(&fuse.part[fuse.nb + b], (unsigned long long)pv);
            if (pm) atomicAdd(&fuse.part[2u * fuse.nb + b], (unsigned long long)pm);
        }
    }
}

hipError_t launch_preprocess(const SceneDev& s, int sh_degree, const FrameUniforms& U, float4* rec,
                             uint32_t* dkey, uint32_t* rect_lo, uint32_t* rect_hi, hipStream_t st, hipEvent_t t0,
                             hipEvent_t t1, unsigned long long* zero8, const PreFuse& fuse, const ShardFuse& shard) {
    if (fuse.part && fuse.nb != (s.n + kScanItems - 1) / kScanItems) return hipErrorInvalidValue;
    if (s.n == 0 && fuse.part) {  // no grid: the fills as copies
        if (fuse.nfill && hipMemsetAsync(fuse.fill, 0xFF, (size_t)fuse.nfill * sizeof(uint2), st) != hipSuccess)
            return hipGetLastError();
        if (fuse.nzero && hipMemsetAsync(fuse.zero, 0, (size_t)fuse.nzero * 4, st) != hipSuccess)
            return hipGetLastError();
        if (fuse.nzero64 && hipMemsetAsync(fuse.zero64, 0, (size_t)fuse.nzero64 * 8, st) != hipSuccess)
            return hipGetLastError();
    }
    if (s.n == 0) {
        // no dispatch: the timing events still mark the (empty) stage
        if (zero8 && hipMemsetAsync(zero8, 0, 16, st) != hipSuccess) return hipGetLastError();
        if (t0 && hipEventRecord(t0, st) != hipSuccess) return hipGetLastError();
        if (t1 && hipEventRecord(t1, st) != hipSuccess) return hipGetLastError();
        return hipSuccess;
    }
    dim3 grid((s.n + 255) / 256), block(256);
    // t0/t1 (optional) are recorded by the dispatch packet itself: no extra
    // barrier packets around the kernel
    if (fuse.part && shard.owner) return hipErrorInvalidValue;
    if (shard.owner && (!shard.dest_mask || !shard.counts || shard.world < 1 || shard.world > kMaxWorld ||
                        shard.nblocks != (s.n + kShardItems - 1) / kShardItems))
        return hipErrorInvalidValue;
    const int epi = fuse.part ? 1 : shard.owner ? 2 : 0;
    // (band frames: the band cull, its own instances, so the full frame's
    // kernels keep their code; not with GS_PRE_EARLY, which loads before it)
    const bool band = GS_PRE_BAND_CULL && !GS_PRE_EARLY && epi != 2 && (U.band_y0 > 0 || U.band_y1 < U.height - 1);
    switch (sh_degree * 3 + epi) {
#define GS_PRE_CASE(D, E)                                                                                          \
    case D * 3 + E:                                                                                                \
        if (band && E != 2)                                                                                        \
            hipExtLaunchKernelGGL((preprocess_kernel<D, E, (E != 2)>), grid, block, 0, st, t0, t1, 0, s, U, rec,  \
                                  dkey, rect_lo, rect_hi, zero8, fuse, shard);                                     \
        else                                                                                                       \
            hipExtLaunchKernelGGL((preprocess_kernel<D, E>), grid, block, 0, st, t0, t1, 0, s, U, rec, dkey,       \
                                  rect_lo, rect_hi, zero8, fuse, shard);                                           \
        break;
        GS_PRE_CASE(0, 0) GS_PRE_CASE(0, 1) GS_PRE_CASE(0, 2)
        GS_PRE_CASE(1, 0) GS_PRE_CASE(1, 1) GS_PRE_CASE(1, 2)
        GS_PRE_CASE(2, 0) GS_PRE_CASE(2, 1) GS_PRE_CASE(2, 2)
        GS_PRE_CASE(3, 0) GS_PRE_CASE(3, 1) GS_PRE_CASE(3, 2)
#undef GS_PRE_CASE
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace gs
