/*
 * gs_oracle.c — CPU ORACLE (test infrastructure only; see gs_oracle.h header
 * for who may use it and for its parity status).
 *
 * Every function cites the reference lines it restates.  Floating-point
 * evaluation order follows DESIGN.md §2 exactly; build with -ffp-contract=off.
 */
#include "gs_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TILE 16
#define OWN_ROW 32 /* multi-GPU ownership unit: 32-px bin rows, owner[by] */
/* 2*ln(100): exp(-q/2) < 0.01 <=> q > 2 ln 100 (tile.metal:191-195). */
#define ORA_QMAX 9.21034037197618f
/* 0.01 transmittance (50layer.metal:219). */
#define ORA_TMIN 0.01f
/* Composite contract: the record's conic is scaled by
 * sqrt(log2(e)/2) per tile, so q' = q log2(e)/2 and the gaussian is 2^-q';
 * box |u| <= 3 -> |u'| <= ORA_BOXS, cutoff exp(-q/2) >= 0.01 -> q' <= log2 100.
 * The tile rule tracks T = 1 - A and breaks at T <= 0.01 (A >= 0.99,
 * tile.metal:261). */
#define ORA_CONIC_S 0.8493217825889587f
#define ORA_BOXS 2.5479652881622314f
#define ORA_QMAXS 6.643856048583984f
#define ORA_TSAT 0.01f

static const float SH_C0 = 0.28209479177387814f; /* ply_loader.cpp:9 */
static const float SH_C1 = 0.4886025119029199f;
static const float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
static const float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

void ora_free(void *p) { free(p); }

/* ------------------------------------------------------------------------ */
/* Numeric helpers                                                          */
/* ------------------------------------------------------------------------ */

/* IEEE binary16 round-to-nearest-even of a float (F1 stores half(depth),
 * tile.metal:203; 50layer.metal:175). */
uint16_t ora_f32_to_f16_bits(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t ax = x & 0x7FFFFFFFu;
    if (ax > 0x7F800000u) return (uint16_t)(sign | 0x7E00u);  /* NaN */
    if (ax >= 0x47800000u) return (uint16_t)(sign | 0x7C00u); /* >= 65536 -> inf */
    int e = (int)(ax >> 23);
    if (e < 113) {                                            /* < 2^-14: subnormal half */
        if (e < 102) return (uint16_t)sign;
        uint32_t mant = (ax & 0x7FFFFFu) | 0x800000u;
        int shift = 126 - e;
        uint32_t m = mant >> shift;
        uint32_t rem = mant & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (m & 1u))) m++;
        return (uint16_t)(sign | m);
    }
    uint32_t h = ((uint32_t)(e - 112) << 10) | ((ax & 0x7FFFFFu) >> 13);
    uint32_t rem = ax & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t)(sign | h);
}

/* 2^t for t in [-7, 0]: rint + degree-6 polynomial + ldexp.  Defined by op
 * sequence (rint, fmaf chain, ldexp) so the GPU reproduces it bit for bit. */
static float ora_exp2_poly(float t) {
    float n = rintf(t);
    float f = t - n;
    float p = 1.5403530393381606e-4f;
    p = fmaf(p, f, 1.3333558146428443e-3f);
    p = fmaf(p, f, 9.6181291076284772e-3f);
    p = fmaf(p, f, 5.5504108664821580e-2f);
    p = fmaf(p, f, 2.4022650695910071e-1f);
    p = fmaf(p, f, 6.9314718055994531e-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)n);
}

/* exp(x) = 2^(x log2 e); |rel err| < 5e-7 on [-4.7, 0]. */
float ora_expf(float x) { return ora_exp2_poly(x * 1.44269504088896341f); }

/* The F1 gaussian exp(-q/2) (tile.metal:191) as 2^(q * (-log2(e)/2)): one
 * rounding before the polynomial.  |rel err| < 5e-7 for q in [0, 9.22];
 * tile.metal evaluates exp in relaxed math and stores alpha as half, so this
 * is far inside the reference's own precision. */
float ora_gauss(float q) { return ora_exp2_poly(q * -0.72134752044448170f); }

/* The composite's gaussian on the scaled conic: 2^-qs = exp(-q/2) with
 * n = rint(-qs), f = -qs - n (exact), a degree-5 minimax polynomial of 2^f
 * on [-1/2, 1/2] (relative error 1.7e-7 in f32) and ldexp; op for op the
 * kernel's gs_gauss2. */
float ora_gauss2(float qs) {
    float t = -qs;
    float n = rintf(t);
    float f = t - n;
    float p = 1.3267117319628596e-3f;
    p = fmaf(p, f, 9.6715930849313736e-3f);
    p = fmaf(p, f, 5.5507261306047440e-2f);
    p = fmaf(p, f, 2.4022240936756134e-1f);
    p = fmaf(p, f, 6.9314700365066528e-1f);
    p = fmaf(p, f, 1.0f);
    return ldexpf(p, (int)n);
}

static uint8_t ora_unorm8(float x) {
    if (!(x > 0.0f)) return 0; /* also NaN */
    if (x >= 1.0f) return 255;
    float y = x * 255.0f;
    float f = floorf(y), d = y - f; /* round half to even, explicitly */
    if (d > 0.5f || (d == 0.5f && fmodf(f, 2.0f) != 0.0f)) f += 1.0f;
    return (uint8_t)f;
}

void ora_to_bgra8(const float *rgba, int64_t npix, uint8_t *bgra) {
    for (int64_t i = 0; i < npix; ++i) {
        bgra[4 * i + 0] = ora_unorm8(rgba[4 * i + 2]);
        bgra[4 * i + 1] = ora_unorm8(rgba[4 * i + 1]);
        bgra[4 * i + 2] = ora_unorm8(rgba[4 * i + 0]);
        bgra[4 * i + 3] = ora_unorm8(rgba[4 * i + 3]);
    }
}

/* ------------------------------------------------------------------------ */
/* I1: PLY loader restatement (src/ply_loader.cpp)                           */
/* ------------------------------------------------------------------------ */

enum { P_X, P_Y, P_Z, P_NX, P_NY, P_NZ, P_R, P_G, P_B, P_OP, P_SX, P_SY, P_SZ, P_R0, P_R1, P_R2, P_R3, P_SH };

static void point_default(float *p) { /* PointData() ctor, ply_loader.h:18-27 */
    memset(p, 0, ORA_POINT_FLOATS * sizeof(float));
    p[P_OP] = 1.0f;
    p[P_SX] = p[P_SY] = p[P_SZ] = 0.01f;
    p[P_R0] = 1.0f;
}

/* shToRGB, ply_loader.cpp:11-20, applied only when any f_dc != 0 (:133). */
static void point_dc_to_rgb(float *p) {
    if (p[P_R] != 0.0f || p[P_G] != 0.0f || p[P_B] != 0.0f) {
        for (int c = 0; c < 3; ++c) {
            float v = 0.5f + SH_C0 * p[P_R + c];
            v = fmaxf(0.0f, fminf(1.0f, v));
            p[P_R + c] = v;
        }
    }
}

typedef struct {
    char type[64];
    char name[64];
} ora_prop;

static int read_line(FILE *f, char *buf, size_t cap) {
    /* std::getline: up to '\n', newline dropped, '\r' kept. */
    size_t k = 0;
    int c;
    int any = 0;
    while ((c = fgetc(f)) != EOF) {
        any = 1;
        if (c == '\n') break;
        if (k + 1 < cap) buf[k++] = (char)c;
    }
    buf[k] = 0;
    return any;
}

/* Property name -> PointData slot; f_rest_<i> -> P_SH + i (ply_loader.cpp:56-82). */
static int prop_slot(const char *name) {
    static const char *names[] = {"x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2",
                                  "opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1",
                                  "rot_2", "rot_3"};
    for (int i = 0; i < 17; ++i)
        if (strcmp(name, names[i]) == 0) return i;
    if (strncmp(name, "f_rest_", 7) == 0) {
        const char *s = name + 7;
        char *end = NULL;
        long v = strtol(s, &end, 10);
        if (end != s && v >= 0 && v < 45) return P_SH + (int)v;
    }
    return -1;
}

/* Store one property value with the loader's activations (:116-119). */
static void point_set(float *p, int slot, float v) {
    if (slot < 0) return;
    switch (slot) {
    case P_OP: p[P_OP] = 1.0f / (1.0f + expf(-v)); break;
    case P_SX: case P_SY: case P_SZ: p[slot] = expf(v); break;
    default: p[slot] = v; break;
    }
}

/* parseHeader, ply_loader.cpp:207-248. */
static int parse_header(FILE *f, int *vcount, ora_prop **props, int *nprops, int *binary) {
    char line[4096];
    if (!read_line(f, line, sizeof line) || strcmp(line, "ply") != 0) return 0;
    int cap = 64, np = 0;
    ora_prop *pp = (ora_prop *)malloc(sizeof(ora_prop) * cap);
    *vcount = 0;
    *binary = 0;
    while (read_line(f, line, sizeof line)) {
        char tok[64] = {0}, a[64] = {0}, b[64] = {0};
        int k = sscanf(line, "%63s %63s %63s", tok, a, b);
        if (k < 1) continue;
        if (strcmp(tok, "format") == 0) {
            *binary = (strcmp(a, "binary_little_endian") == 0 || strcmp(a, "binary_big_endian") == 0);
        } else if (strcmp(tok, "element") == 0) {
            if (strcmp(a, "vertex") == 0) *vcount = (int)strtol(b, NULL, 10);
        } else if (strcmp(tok, "property") == 0) {
            if (np == cap) { cap *= 2; pp = (ora_prop *)realloc(pp, sizeof(ora_prop) * cap); }
            snprintf(pp[np].type, 64, "%s", a);
            snprintf(pp[np].name, 64, "%s", b);
            np++;
        } else if (strcmp(tok, "end_header") == 0) {
            break;
        }
    }
    *props = pp;
    *nprops = np;
    return *vcount > 0 && np > 0;
}

/* One ASCII token as `iss >> value` would read it; returns 0 on failure. */
static int ascii_float(const char **cur, float *out) {
    const char *s = *cur;
    while (*s && isspace((unsigned char)*s)) s++;
    if (!*s) return 0;
    const char *t = s;
    if (*t == '+' || *t == '-') t++;
    if (!(isdigit((unsigned char)*t) || (*t == '.' && isdigit((unsigned char)t[1])))) return 0;
    char *end = NULL;
    float v = strtof(s, &end);
    if (end == s) return 0;
    *out = v;
    *cur = end;
    return 1;
}

int ora_ply_load(const char *path, float **out, int64_t *n) {
    *out = NULL;
    *n = 0;
    FILE *f = fopen(path, "rb");
    if (!f) return 0;
    int vcount = 0, nprops = 0, binary = 0;
    ora_prop *props = NULL;
    if (!parse_header(f, &vcount, &props, &nprops, &binary)) {
        free(props);
        fclose(f);
        return 0;
    }
    int *slot = (int *)malloc(sizeof(int) * nprops);
    for (int j = 0; j < nprops; ++j) slot[j] = prop_slot(props[j].name);

    /* points.resize(vertexCount) (:52): vcount default points first. */
    int64_t total = vcount;
    int64_t capn = binary ? (int64_t)vcount : 2 * (int64_t)vcount;
    float *pts = (float *)malloc(sizeof(float) * ORA_POINT_FLOATS * (size_t)(capn > 0 ? capn : 1));
    for (int64_t i = 0; i < vcount; ++i) point_default(pts + i * ORA_POINT_FLOATS);

    if (binary) {
        /* Every property read as 4 LE bytes regardless of declared type (:85);
         * endianness ignored; a short read keeps stale chunk bytes (:95). */
        const int CHUNK = 10000;
        size_t stride = (size_t)nprops;
        float *buf = (float *)calloc((size_t)CHUNK * stride, sizeof(float));
        for (int c0 = 0; c0 < vcount; c0 += CHUNK) {
            int cn = vcount - c0 < CHUNK ? vcount - c0 : CHUNK;
            size_t got = fread(buf, 1, (size_t)cn * stride * 4, f);
            (void)got;
            for (int i = 0; i < cn; ++i) {
                float *p = pts + (int64_t)(c0 + i) * ORA_POINT_FLOATS;
                const float *v = buf + (size_t)i * stride;
                for (int j = 0; j < nprops; ++j) point_set(p, slot[j], v[j]);
                point_dc_to_rgb(p);
            }
        }
        free(buf);
    } else {
        /* ASCII path: resize() then push_back() -> 2N points, defaults first
         * (:52,155-199). */
        char *line = (char *)malloc(1 << 20);
        for (int i = 0; i < vcount; ++i) {
            if (!read_line(f, line, 1 << 20)) break;
            float *p = pts + total * ORA_POINT_FLOATS;
            point_default(p);
            const char *cur = line;
            int ok = 1;
            for (int j = 0; j < nprops; ++j) {
                float v = 0.0f;
                if (ok) ok = ascii_float(&cur, &v);
                if (!ok) v = 0.0f;
                point_set(p, slot[j], v);
            }
            point_dc_to_rgb(p);
            total++;
        }
        free(line);
    }
    free(slot);
    free(props);
    fclose(f);
    *out = pts;
    *n = total;
    return total > 0;
}

/* ------------------------------------------------------------------------ */
/* I2: crop (instanced_splat_renderer.mm:382-386)                            */
/* ------------------------------------------------------------------------ */
int64_t ora_crop(const float *pts, int64_t n, float r, int64_t *keep) {
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const float *p = pts + i * ORA_POINT_FLOATS;
        if (fabsf(p[P_X]) < r && fabsf(p[P_Y]) < r && fabsf(p[P_Z]) < r) keep[k++] = i;
    }
    return k;
}

/* ------------------------------------------------------------------------ */
/* C1: camera (trackball_camera.mm:136-163), VP = P·V (.mm:453)              */
/* ------------------------------------------------------------------------ */
static void v3_normalize(const float v[3], float o[3]) {
    float len = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    o[0] = v[0] / len;
    o[1] = v[1] / len;
    o[2] = v[2] / len;
}
static void v3_cross(const float a[3], const float b[3], float o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
static float v3_dot(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

void ora_look_at(const float eye[3], const float center[3], const float up[3], float m[16]) {
    float d[3] = {center[0] - eye[0], center[1] - eye[1], center[2] - eye[2]};
    float f[3], s0[3], s[3], u[3];
    v3_normalize(d, f);
    v3_cross(f, up, s0);
    v3_normalize(s0, s);
    v3_cross(s, f, u);
    /* columns (.mm:142-145) */
    m[0] = s[0]; m[1] = u[0]; m[2] = -f[0]; m[3] = 0.0f;
    m[4] = s[1]; m[5] = u[1]; m[6] = -f[1]; m[7] = 0.0f;
    m[8] = s[2]; m[9] = u[2]; m[10] = -f[2]; m[11] = 0.0f;
    m[12] = -v3_dot(s, eye); m[13] = -v3_dot(u, eye); m[14] = v3_dot(f, eye); m[15] = 1.0f;
}

void ora_perspective(float fov_degrees, float aspect, float zn, float zf, float m[16]) {
    /* getProjectionMatrix: fov * M_PI / 180.0f in double, passed as float (.mm:131-134). */
    float fov = (float)((double)fov_degrees * 3.14159265358979323846 / 180.0);
    float ys = 1.0f / tanf(fov * 0.5f);
    float xs = ys / aspect;
    float zr = zf - zn;
    float zs = -(zf + zn) / zr;
    float wz = -2.0f * zf * zn / zr;
    memset(m, 0, 16 * sizeof(float));
    m[0] = xs;
    m[5] = ys;
    m[10] = zs;
    m[11] = -1.0f;
    m[14] = wz;
}

void ora_mat4_mul(const float a[16], const float b[16], float o[16]) {
    float t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = ((a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1]) +
                            a[2 * 4 + r] * b[c * 4 + 2]) + a[3 * 4 + r] * b[c * 4 + 3];
    memcpy(o, t, sizeof t);
}

/* Eye position of a rigid view matrix: -(R^T t). */
void ora_camera_position(const float v[16], float o[3]) {
    for (int j = 0; j < 3; ++j)
        o[j] = -((v[j * 4 + 0] * v[12] + v[j * 4 + 1] * v[13]) + v[j * 4 + 2] * v[14]);
}

/* ------------------------------------------------------------------------ */
/* K1..K5 projection                                                        */
/* ------------------------------------------------------------------------ */

/* row r of M·(x,y,z,1), M column-major: fma(c2,z, fma(c1,y, fma(c0,x,c3))) */
static float xform_row(const float *m, int r, float x, float y, float z) {
    return fmaf(m[8 + r], z, fmaf(m[4 + r], y, fmaf(m[0 + r], x, m[12 + r])));
}

static float dot3f(float a0, float a1, float a2, float b0, float b1, float b2) {
    return fmaf(a2, b2, fmaf(a1, b1, a0 * b0));
}

/* N2: SH colour (standard 3DGS real basis).  Degree 0 reproduces shToRGB
 * (ply_loader.cpp:11-20) including the all-zero quirk (:133). */
static void sh_color(const ora_scene *s, int64_t i, const float campos[3], float rgb[3]) {
    const float *dc = s->color + i * 3;
    if (s->sh_degree <= 0) {
        rgb[0] = dc[0]; rgb[1] = dc[1]; rgb[2] = dc[2];
        return;
    }
    if (dc[0] == 0.0f && dc[1] == 0.0f && dc[2] == 0.0f) {
        rgb[0] = rgb[1] = rgb[2] = 0.0f;
        return;
    }
    const float *p = s->pos + i * 3;
    float dx = p[0] - campos[0], dy = p[1] - campos[1], dz = p[2] - campos[2];
    float l2 = fmaf(dz, dz, fmaf(dy, dy, dx * dx));
    float inv = 1.0f / sqrtf(l2);
    float x = dx * inv, y = dy * inv, z = dz * inv;
    float bas[16];
    int K = 0;
    if (s->sh_degree >= 1) {
        bas[1] = (-SH_C1) * y;
        bas[2] = SH_C1 * z;
        bas[3] = (-SH_C1) * x;
        K = 3;
    }
    if (s->sh_degree >= 2) {
        float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        bas[4] = SH_C2[0] * xy;
        bas[5] = SH_C2[1] * yz;
        bas[6] = SH_C2[2] * ((2.0f * zz - xx) - yy);
        bas[7] = SH_C2[3] * xz;
        bas[8] = SH_C2[4] * (xx - yy);
        K = 8;
        if (s->sh_degree >= 3) {
            bas[9] = (SH_C3[0] * y) * (3.0f * xx - yy);
            bas[10] = (SH_C3[1] * xy) * z;
            bas[11] = (SH_C3[2] * y) * ((4.0f * zz - xx) - yy);
            bas[12] = (SH_C3[3] * z) * ((2.0f * zz - 3.0f * xx) - 3.0f * yy);
            bas[13] = (SH_C3[4] * x) * ((4.0f * zz - xx) - yy);
            bas[14] = (SH_C3[5] * z) * (xx - yy);
            bas[15] = (SH_C3[6] * x) * (xx - 3.0f * yy);
            K = 15;
        }
    }
    const float *rest = s->sh_rest + i * 45;
    for (int c = 0; c < 3; ++c) {
        float acc = SH_C0 * dc[c];
        for (int k = 1; k <= K; ++k) acc = fmaf(bas[k], rest[c * 15 + (k - 1)], acc);
        acc = acc + 0.5f;
        rgb[c] = fminf(fmaxf(acc, 0.0f), 1.0f);
    }
}

void ora_project(const ora_scene *s, int64_t i, const float V[16], const float P[16],
                 const float VP[16], const float campos[3], int W, int H, ora_record *rec,
                 ora_debug *dbg) {
    memset(rec, 0, sizeof *rec);
    memset(dbg, 0, sizeof *dbg);
    const float *p = s->pos + i * 3;
    float px = p[0], py = p[1], pz = p[2];

    /* K3: view position, zFront = -view.z, cull zF < 1e-4 (tile.metal:94-105). */
    float vx = xform_row(V, 0, px, py, pz);
    float vy = xform_row(V, 1, px, py, pz);
    float vz = xform_row(V, 2, px, py, pz);
    float zf = -vz;
    dbg->zf = zf;
    if (!(zf >= 1e-4f)) return;

    /* K6 z-clip: Metal keeps 0 <= clip.z/clip.w <= 1 (tile.metal:145-152). */
    float clx = xform_row(VP, 0, px, py, pz);
    float cly = xform_row(VP, 1, px, py, pz);
    float clz = xform_row(VP, 2, px, py, pz);
    float clw = xform_row(VP, 3, px, py, pz);
    float invw = 1.0f / clw;
    float ndcz = clz * invw;
    if (!(ndcz >= 0.0f && ndcz <= 1.0f)) return;
    if (!(zf >= 0.001f)) return; /* fragment discard depth < 0.001 (tile.metal:187) */

    /* K1: normalise quaternion (w,x,y,z) and build R (tile.metal:40-49). */
    const float *q = s->rot + i * 4;
    float qs = q[0] * q[0];
    qs = fmaf(q[1], q[1], qs);
    qs = fmaf(q[2], q[2], qs);
    qs = fmaf(q[3], q[3], qs);
    float qi = 1.0f / sqrtf(qs);
    float w = q[0] * qi, x = q[1] * qi, y = q[2] * qi, z = q[3] * qi;
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, xz = x * z, yz = y * z;
    float wx = w * x, wy = w * y, wz = w * z;
    float R[3][3]; /* R[row][col] */
    R[0][0] = 1.0f - 2.0f * (yy + zz); R[1][0] = 2.0f * (xy + wz); R[2][0] = 2.0f * (xz - wy);
    R[0][1] = 2.0f * (xy - wz); R[1][1] = 1.0f - 2.0f * (xx + zz); R[2][1] = 2.0f * (yz + wx);
    R[0][2] = 2.0f * (xz + wy); R[1][2] = 2.0f * (yz - wx); R[2][2] = 1.0f - 2.0f * (xx + yy);

    /* K2: M = R S, Sigma = M M^T (tile.metal:51-60). */
    const float *sc = s->scale + i * 3;
    float M[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) M[r][c] = R[r][c] * sc[c];
    float S[3][3];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) S[r][c] = dot3f(M[r][0], M[r][1], M[r][2], M[c][0], M[c][1], M[c][2]);
    /* (S is symmetric bit for bit: dot3f's products commute) */

    /* K3 + Jacobian (tile.metal:109-127): cov2d = J (W Sigma W^T) J^T,
     * evaluated as A Sigma A^T with A = J W, W(i,j) =
     * V[col j][row i], J with the reference's z-column sign (:117-123) and
     * its zero entries skipped. */
    float fx = P[0] * ((float)W * 0.5f);
    float fy = P[5] * ((float)H * 0.5f);
    float iz = 1.0f / zf;
    float iz2 = iz * iz;
    float J00 = fx * iz, J02 = ((-fx) * vx) * iz2;
    float J11 = fy * iz, J12 = ((-fy) * vy) * iz2;
    float A[2][3];
    for (int c = 0; c < 3; ++c) {
        A[0][c] = fmaf(J02, V[c * 4 + 2], J00 * V[c * 4 + 0]);
        A[1][c] = fmaf(J12, V[c * 4 + 2], J11 * V[c * 4 + 1]);
    }
    float B[2][3];
    for (int r = 0; r < 2; ++r)
        for (int c = 0; c < 3; ++c) B[r][c] = dot3f(A[r][0], A[r][1], A[r][2], S[0][c], S[1][c], S[2][c]);
    float a = dot3f(B[0][0], B[0][1], B[0][2], A[0][0], A[0][1], A[0][2]);
    float b = dot3f(B[0][0], B[0][1], B[0][2], A[1][0], A[1][1], A[1][2]);
    float c = dot3f(B[1][0], B[1][1], B[1][2], A[1][0], A[1][1], A[1][2]);
    a = a + 1e-4f; /* tile.metal:129-131 */
    c = c + 1e-4f;

    /* K4: eigenSym2x2 (tile.metal:62-83), radii (:136-140). */
    float tr = a + c;
    float det = a * c - b * b;
    float disc = fmaxf(0.0f, (0.25f * tr) * tr - det);
    float sq = sqrtf(disc);
    float l1 = 0.5f * tr + sq;
    float l2 = 0.5f * tr - sq;
    float e1x, e1y;
    if (fabsf(b) > 1e-8f) {
        float ux = l1 - c, uy = b;
        float il = 1.0f / sqrtf(fmaf(uy, uy, ux * ux));
        e1x = ux * il;
        e1y = uy * il;
    } else if (a >= c) {
        e1x = 1.0f; e1y = 0.0f;
    } else {
        e1x = 0.0f; e1y = 1.0f;
    }
    float e2x = -e1y, e2y = e1x;
    l1 = fmaxf(l1, 0.0f);
    l2 = fmaxf(l2, 0.0f);
    float r1 = 3.0f * sqrtf(l1);
    float r2 = 3.0f * sqrtf(l2);
    dbg->a = a; dbg->b = b; dbg->c = c;
    dbg->r1 = r1; dbg->r2 = r2;
    dbg->e1x = e1x; dbg->e1y = e1y;
    if (!(r1 > 0.0f && r2 > 0.0f)) return; /* zero-area quad covers no pixel */

    /* K5/K6 closed form: centre in window px, uv scales. */
    float ndcx = clx * invw, ndcy = cly * invw;
    float cx = (ndcx + 1.0f) * ((float)W * 0.5f);
    float cy = (1.0f - ndcy) * ((float)H * 0.5f);
    float k1 = 3.0f / r1, k2 = 3.0f / r2;

    /* Conservative pixel rect: min(box AABB, ellipse AABB) * (1+1e-4) + 1px. */
    float hbx = r1 * fabsf(e1x) + r2 * fabsf(e2x);
    float hby = r1 * fabsf(e1y) + r2 * fabsf(e2y);
    float hex = 1.0117f * sqrtf((r1 * e1x) * (r1 * e1x) + (r2 * e2x) * (r2 * e2x));
    float hey = 1.0117f * sqrtf((r1 * e1y) * (r1 * e1y) + (r2 * e2y) * (r2 * e2y));
    float hx = fminf(hbx, hex) * 1.0001f + 1.0f;
    float hy = fminf(hby, hey) * 1.0001f + 1.0f;
    float x0f = ceilf(cx - hx - 0.5f), x1f = floorf(cx + hx - 0.5f);
    float y0f = ceilf(cy - hy - 0.5f), y1f = floorf(cy + hy - 0.5f);
    x0f = fmaxf(x0f, 0.0f);
    y0f = fmaxf(y0f, 0.0f);
    x1f = fminf(x1f, (float)(W - 1));
    y1f = fminf(y1f, (float)(H - 1));
    if (!(x0f <= x1f && y0f <= y1f)) return;
    uint32_t x0 = (uint32_t)x0f, x1 = (uint32_t)x1f, y0 = (uint32_t)y0f, y1 = (uint32_t)y1f;

    float rgb[3];
    sh_color(s, i, campos, rgb);

    rec->cx = cx;
    rec->cy = cy;
    rec->ax = e1x * k1;
    rec->ay = e1y * k1;
    rec->bx = e2x * k2;
    rec->by = e2y * k2;
    rec->opacity = s->opacity[i];
    rec->r = rgb[0];
    rec->g = rgb[1];
    rec->b = rgb[2];
    rec->rect_lo = x0 | (y0 << 16);
    rec->rect_hi = x1 | (y1 << 16);
    dbg->dkey = 0x7C00u - ora_f32_to_f16_bits(zf);
    dbg->ntiles = ((x1 / TILE) - (x0 / TILE) + 1) * ((y1 / TILE) - (y0 / TILE) + 1);
    dbg->visible = 1;
}

void ora_project_all(const ora_scene *s, const float V[16], const float P[16], int W, int H,
                     ora_record *rec, uint32_t *dkey, uint32_t *ntiles, int nthreads) {
    float VP[16], cam[3];
    ora_mat4_mul(P, V, VP);
    ora_camera_position(V, cam);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < s->n; ++i) {
        ora_debug d;
        ora_project(s, i, V, P, VP, cam, W, H, &rec[i], &d);
        dkey[i] = d.dkey;
        ntiles[i] = d.visible ? d.ntiles : 0;
    }
}

/* ------------------------------------------------------------------------ */
/* F1 + S1 + A1: per-pixel composite                                        */
/* ------------------------------------------------------------------------ */

/* Coverage + gaussian of record j at pixel (px,py): returns alpha or -1.
 * The conic is staged per 16x16 tile (the composite kernel's workgroup):
 * scaled by sqrt(log2(e)/2), offset at the tile origin (tx0, ty0); the pixel
 * centre enters tile-local, (lx, ly) = (px - tx0 + 1/2, py - ty0 + 1/2). */
static float frag_alpha(const ora_record *r, int px, int py) {
    int tx0 = px & ~(TILE - 1), ty0 = py & ~(TILE - 1);
    float ax = r->ax * ORA_CONIC_S, ay = r->ay * ORA_CONIC_S;
    float bx = r->bx * ORA_CONIC_S, by = r->by * ORA_CONIC_S;
    float ex = (float)tx0 - r->cx, ey = r->cy - (float)ty0;
    float u0 = fmaf(ax, ex, ay * ey), v0 = fmaf(bx, ex, by * ey);
    float lx = (float)(px - tx0) + 0.5f, ly = (float)(py - ty0) + 0.5f;
    float u = fmaf(ax, lx, fmaf(-ay, ly, u0));
    float v = fmaf(bx, lx, fmaf(-by, ly, v0));
    if (!(fmaxf(fabsf(u), fabsf(v)) <= ORA_BOXS)) return -1.0f; /* K6 quad coverage |uv| <= 3 */
    float q = fmaf(v, v, u * u);
    if (!(q <= ORA_QMAXS)) return -1.0f; /* g < 0.01 discard, tile.metal:193 */
    return r->opacity * ora_gauss2(q); /* tile.metal:197 */
}

typedef struct {
    uint32_t key; /* dkey */
    uint32_t idx;
} kv;

static int kv_cmp(const void *a, const void *b) {
    const kv *x = (const kv *)a, *y = (const kv *)b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);
}

/* ---- MLAB k-buffer (gaussian_splat.metal:201-361) ------------------------
 * Metal half arithmetic is emulated op by op: each half op is computed
 * exactly in double (sums and products of two halves are exact there) and
 * rounded once to the nearest half, ties to even, i.e. a correctly rounded
 * half op, as gfx950's v_*_f16 are.  Halves are carried as floats. */
static float hr(double x) {
    if (x != x) return (float)x;
    double ax = fabs(x);
    if (ax >= 65520.0) return x > 0 ? INFINITY : -INFINITY; /* RNE past 65504 */
    if (ax == 0.0) return (float)x;
    int E;
    frexp(ax, &E);   /* ax in [2^(E-1), 2^E) */
    int e = E - 1;
    if (e < -14) e = -14; /* subnormal quantum 2^-24 */
    double q = ldexp(1.0, e - 10);
    double v = rint(ax / q) * q;
    return (float)(x < 0 ? -v : v);
}

static float half_from_bits(uint32_t b) {
    uint32_t e = (b >> 10) & 0x1Fu, m = b & 0x3FFu;
    float v = e ? ldexpf((float)(m | 0x400u), (int)e - 25) : ldexpf((float)m, -24);
    return (b & 0x8000u) ? -v : v;
}

#define MLAB_LAYERS 6 /* NUM_OIT_LAYERS, gaussian_splat.metal:11 */
typedef struct {
    float L[MLAB_LAYERS][4]; /* premultiplied rgb + visibility (half values) */
    float D[MLAB_LAYERS];    /* half depths */
} mlab_kbuf;

/* Clear to (0,0,0,1) on all 8 attachments (instanced_splat_renderer.mm:540):
 * layers (0,0,0,1); depths01 = (0,0,0,1) -> depth[3] starts at 1. */
static void mlab_clear(mlab_kbuf *k) {
    for (int i = 0; i < MLAB_LAYERS; ++i) {
        k->L[i][0] = k->L[i][1] = k->L[i][2] = 0.0f;
        k->L[i][3] = 1.0f;
        k->D[i] = 0.0f;
    }
    k->D[3] = 1.0f;
}

/* fragment_main (gaussian_splat.metal:206-294), one covering fragment. */
static void mlab_insert(mlab_kbuf *k, float r, float g, float b, float alpha, float depth_h) {
    float ha = hr(alpha);
    float nl[4] = {hr((double)hr(r) * ha), hr((double)hr(g) * ha), hr((double)hr(b) * ha), hr(1.0 - (double)ha)};
    float nd = depth_h;
    for (int i = 0; i < MLAB_LAYERS; ++i) { /* :245-259 */
        if (nd >= k->D[i]) {
            for (int c = 0; c < 4; ++c) {
                float t = k->L[i][c];
                k->L[i][c] = nl[c];
                nl[c] = t;
            }
            float t = k->D[i];
            k->D[i] = nd;
            nd = t;
        }
    }
    const int last = MLAB_LAYERS - 1; /* :261-271 merge under */
    int closer = nd >= k->D[last];
    const float *front = closer ? nl : k->L[last];
    const float *back = closer ? k->L[last] : nl;
    float m[4];
    for (int c = 0; c < 3; ++c) m[c] = hr((double)back[c] + hr((double)front[c] * back[3]));
    m[3] = hr((double)front[3] * back[3]);
    for (int c = 0; c < 4; ++c) k->L[last][c] = m[c];
    if (closer) k->D[last] = nd;
}

/* resolve_main (gaussian_splat.metal:330-361): layers front to back. */
static void mlab_resolve(const mlab_kbuf *k, float out[4]) {
    float C[3] = {0.0f, 0.0f, 0.0f}, at = 1.0f;
    for (int i = 0; i < MLAB_LAYERS; ++i) {
        for (int c = 0; c < 3; ++c) C[c] = hr((double)C[c] + hr((double)k->L[i][c] * at));
        at = hr((double)at * k->L[i][3]);
    }
    out[0] = C[0]; out[1] = C[1]; out[2] = C[2];
    out[3] = hr(1.0 - (double)at);
}

/* Composite `cnt` fragments given in S1 order (dkey asc, index asc). */
static void composite(int mode, const float *frag_rgb_a, int cnt, float out[4]) {
    if (mode == ORA_MODE_TILE) { /* tile.metal:251-266 */
        float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f; /* T = 1 - A */
        for (int k = 0; k < cnt; ++k) {
            const float *f = frag_rgb_a + k * 4;
            float sa = f[3] * T;
            C0 = fmaf(f[0], sa, C0);
            C1 = fmaf(f[1], sa, C1);
            C2 = fmaf(f[2], sa, C2);
            T = T - sa;
            if (T <= ORA_TSAT) break; /* A >= 0.99 */
        }
        out[0] = C0; out[1] = C1; out[2] = C2; out[3] = 1.0f - T;
    } else { /* 50layer.metal:208-222 */
        float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
        for (int k = 0; k < cnt; ++k) {
            const float *f = frag_rgb_a + k * 4;
            C0 = fmaf(f[0], T, C0);
            C1 = fmaf(f[1], T, C1);
            C2 = fmaf(f[2], T, C2);
            T = T * (1.0f - f[3]);
            if (T < ORA_TMIN) break;
        }
        out[0] = C0; out[1] = C1; out[2] = C2; out[3] = cnt > 0 ? 1.0f - T : 0.0f;
    }
}

void ora_composite_list(const float *frags, int n, int mode, int cap, float out[4]) {
    if (mode == ORA_MODE_MLAB) { /* arrival order through the k-buffer; no cap */
        mlab_kbuf kb;
        mlab_clear(&kb);
        for (int k = 0; k < n; ++k) {
            const float *f = frags + k * 5;
            mlab_insert(&kb, f[1], f[2], f[3], f[4], hr(f[0]));
        }
        mlab_resolve(&kb, out);
        return;
    }
    int cnt = (cap > 0 && n > cap) ? cap : n; /* overflow dropped by arrival (tile.metal:202) */
    kv *ord = (kv *)malloc(sizeof(kv) * (cnt > 0 ? cnt : 1));
    for (int k = 0; k < cnt; ++k) {
        ord[k].key = 0x7C00u - ora_f32_to_f16_bits(frags[k * 5]);
        ord[k].idx = (uint32_t)k;
    }
    qsort(ord, (size_t)cnt, sizeof(kv), kv_cmp); /* stable S1 by index tiebreak */
    float *f = (float *)malloc(sizeof(float) * 4 * (cnt > 0 ? cnt : 1));
    for (int k = 0; k < cnt; ++k) {
        const float *s = frags + ord[k].idx * 5;
        f[k * 4 + 0] = s[1]; f[k * 4 + 1] = s[2]; f[k * 4 + 2] = s[3]; f[k * 4 + 3] = s[4];
    }
    out[0] = out[1] = out[2] = out[3] = 0.0f;
    if (cnt > 0) composite(mode, f, cnt, out);
    free(f);
    free(ord);
}

/* slab: 0 = plain composite; 1 = depth-slab transmittance pass (out = W*H
 * floats, the slab's own transmittance); 2 = colour pass from the ordered
 * product of the earlier slabs' transmittance t_all[j][py][px], j < slab_rank
 * (out = (C, delta alpha) contributions).  DESIGN.md §6b. */
static int composite_records_impl(const ora_record *rec, const uint32_t *dkey, int64_t n, int W, int H,
                                  const ora_options *opt, const uint8_t *owner, int rank, int compact, float *out,
                                  ora_stats *st, int slab, int slab_rank, const float *t_all) {
    int mode = opt ? opt->mode : ORA_MODE_TILE;
    int cap = opt ? opt->cap : 0;
    int nth = opt ? opt->nthreads : 0;
#ifdef _OPENMP
    if (nth > 0) omp_set_num_threads(nth);
#endif
    int TW = (W + TILE - 1) / TILE, TH = (H + TILE - 1) / TILE, T = TW * TH;
    /* ownership of 32-px rows; slot[r] = position of owned row r in the band buffer */
    int NR = (H + OWN_ROW - 1) / OWN_ROW;
    int *slot = (int *)malloc(sizeof(int) * (size_t)(NR > 0 ? NR : 1));
    for (int r = 0, k = 0; r < NR; ++r) slot[r] = (!owner || owner[r] == rank) ? k++ : -1;
#define ORA_OWNED(ty) (slot[((ty) * TILE) / OWN_ROW] >= 0)
    /* Oracle binning uses the record rect widened by 2 px, so a too-tight
     * product rect shows up as a framebuffer mismatch.  Records with a zero
     * rect (rect_hi == 0 && rect_lo == 0 && opacity == 0) are culled. */
    int64_t *cnt = (int64_t *)calloc((size_t)T + 1, sizeof(int64_t));
    int64_t visible = 0, pairs = 0;
#define ORA_RECT(i, X0, Y0, X1, Y1)                                                            \
    int X0 = (int)(rec[i].rect_lo & 0xFFFF) - 2, Y0 = (int)(rec[i].rect_lo >> 16) - 2;          \
    int X1 = (int)(rec[i].rect_hi & 0xFFFF) + 2, Y1 = (int)(rec[i].rect_hi >> 16) + 2;          \
    if (X0 < 0) X0 = 0;                                                                        \
    if (Y0 < 0) Y0 = 0;                                                                        \
    if (X1 > W - 1) X1 = W - 1;                                                                \
    if (Y1 > H - 1) Y1 = H - 1;
    for (int64_t i = 0; i < n; ++i) {
        if (!dkey[i] && !rec[i].rect_hi && !rec[i].opacity) continue;
        visible++;
        pairs += (int64_t)((rec[i].rect_hi & 0xFFFF) / TILE - (rec[i].rect_lo & 0xFFFF) / TILE + 1) *
                 ((rec[i].rect_hi >> 16) / TILE - (rec[i].rect_lo >> 16) / TILE + 1);
        ORA_RECT(i, x0, y0, x1, y1)
        for (int ty = y0 / TILE; ty <= y1 / TILE; ++ty) {
            if (!ORA_OWNED(ty)) continue;
            for (int tx = x0 / TILE; tx <= x1 / TILE; ++tx) cnt[ty * TW + tx + 1]++;
        }
    }
    for (int t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
    int64_t total = cnt[T];
    uint32_t *list = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(total > 0 ? total : 1));
    int64_t *cur = (int64_t *)malloc(sizeof(int64_t) * (size_t)T);
    memcpy(cur, cnt, sizeof(int64_t) * (size_t)T);
    for (int64_t i = 0; i < n; ++i) { /* index order = arrival order */
        if (!dkey[i] && !rec[i].rect_hi && !rec[i].opacity) continue;
        ORA_RECT(i, x0, y0, x1, y1)
        for (int ty = y0 / TILE; ty <= y1 / TILE; ++ty) {
            if (!ORA_OWNED(ty)) continue;
            for (int tx = x0 / TILE; tx <= x1 / TILE; ++tx) list[cur[ty * TW + tx]++] = (uint32_t)i;
        }
    }
#undef ORA_RECT
    free(cur);

#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        size_t kcap = 1024;
        kv *ord = (kv *)malloc(sizeof(kv) * kcap);
        float *fr = (float *)malloc(sizeof(float) * 4 * kcap);
        kv *sel = (kv *)malloc(sizeof(kv) * kcap);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4)
#endif
        for (int t = 0; t < T; ++t) {
            int tx = t % TW, ty = t / TW;
            if (!ORA_OWNED(ty)) continue;
            int64_t b = cnt[t], e = cnt[t + 1], m = e - b;
            if ((size_t)m > kcap) {
                kcap = (size_t)m;
                ord = (kv *)realloc(ord, sizeof(kv) * kcap);
                sel = (kv *)realloc(sel, sizeof(kv) * kcap);
                fr = (float *)realloc(fr, sizeof(float) * 4 * kcap);
            }
            for (int64_t k = 0; k < m; ++k) {
                ord[k].key = dkey[list[b + k]];
                ord[k].idx = list[b + k];
            }
            /* S1 order: descending half depth == ascending dkey; ties keep
             * arrival (index) order. */
            if (cap == 0 && mode != ORA_MODE_MLAB) qsort(ord, (size_t)m, sizeof(kv), kv_cmp);
            for (int py = ty * TILE; py < ty * TILE + TILE && py < H; ++py) {
                int orow = compact ? slot[py / OWN_ROW] * OWN_ROW + py % OWN_ROW : py;
                for (int px = tx * TILE; px < tx * TILE + TILE && px < W; ++px) {
                    float *o = out + ((size_t)orow * W + px) * (slab == 1 ? 1 : 4);
                    int c = 0;
                    if (mode == ORA_MODE_MLAB) { /* arrival order, k-buffer, resolve */
                        mlab_kbuf kb;
                        mlab_clear(&kb);
                        for (int64_t k = 0; k < m; ++k) {
                            const ora_record *r = &rec[ord[k].idx];
                            float al = frag_alpha(r, px, py);
                            if (al < 0.0f) continue;
                            mlab_insert(&kb, r->r, r->g, r->b, al, half_from_bits(0x7C00u - ord[k].key));
                        }
                        mlab_resolve(&kb, o);
                        continue;
                    }
                    if (slab) { /* depth slab: same walk, from the slab's start state */
                        float ts = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f;
                        if (slab == 2)
                            for (int j = 0; j < slab_rank; ++j) ts *= t_all[((size_t)j * H + py) * W + px];
                        float T = slab == 2 ? ts : 1.0f, T0 = T;
                        if (mode == ORA_MODE_TILE) {
                            if (!(T <= ORA_TSAT))
                                for (int64_t k = 0; k < m; ++k) {
                                    const ora_record *r = &rec[ord[k].idx];
                                    float al = frag_alpha(r, px, py);
                                    if (al < 0.0f) continue;
                                    float sa = al * T;
                                    C0 = fmaf(r->r, sa, C0);
                                    C1 = fmaf(r->g, sa, C1);
                                    C2 = fmaf(r->b, sa, C2);
                                    T = T - sa;
                                    if (T <= ORA_TSAT) break;
                                }
                        } else {
                            if (!(T < ORA_TMIN))
                                for (int64_t k = 0; k < m; ++k) {
                                    const ora_record *r = &rec[ord[k].idx];
                                    float al = frag_alpha(r, px, py);
                                    if (al < 0.0f) continue;
                                    C0 = fmaf(r->r, T, C0);
                                    C1 = fmaf(r->g, T, C1);
                                    C2 = fmaf(r->b, T, C2);
                                    T = T * (1.0f - al);
                                    if (T < ORA_TMIN) break;
                                }
                        }
                        if (slab == 1) {
                            o[0] = T;
                        } else {
                            o[0] = C0; o[1] = C1; o[2] = C2; o[3] = T0 - T;
                        }
                        continue;
                    }
                    if (cap == 0) {
                        if (mode == ORA_MODE_TILE) { /* fused early-break walk */
                            float T = 1.0f, C0 = 0.0f, C1 = 0.0f, C2 = 0.0f; /* T = 1 - A */
                            for (int64_t k = 0; k < m; ++k) {
                                const ora_record *r = &rec[ord[k].idx];
                                float al = frag_alpha(r, px, py);
                                if (al < 0.0f) continue;
                                float sa = al * T;
                                C0 = fmaf(r->r, sa, C0);
                                C1 = fmaf(r->g, sa, C1);
                                C2 = fmaf(r->b, sa, C2);
                                T = T - sa;
                                if (T <= ORA_TSAT) break;
                            }
                            o[0] = C0; o[1] = C1; o[2] = C2; o[3] = 1.0f - T;
                            continue;
                        }
                        for (int64_t k = 0; k < m; ++k) {
                            const ora_record *r = &rec[ord[k].idx];
                            float al = frag_alpha(r, px, py);
                            if (al < 0.0f) continue;
                            fr[c * 4 + 0] = r->r; fr[c * 4 + 1] = r->g; fr[c * 4 + 2] = r->b;
                            fr[c * 4 + 3] = al;
                            c++;
                        }
                    } else {
                        /* cap: first `cap` covering fragments in arrival order,
                         * then S1 sort (50layer.metal:170-176,197-206). */
                        int ns = 0;
                        for (int64_t k = 0; k < m && ns < cap; ++k) {
                            const ora_record *r = &rec[ord[k].idx];
                            if (frag_alpha(r, px, py) < 0.0f) continue;
                            sel[ns++] = ord[k];
                        }
                        qsort(sel, (size_t)ns, sizeof(kv), kv_cmp);
                        for (int k = 0; k < ns; ++k) {
                            const ora_record *r = &rec[sel[k].idx];
                            fr[c * 4 + 0] = r->r; fr[c * 4 + 1] = r->g; fr[c * 4 + 2] = r->b;
                            fr[c * 4 + 3] = frag_alpha(r, px, py);
                            c++;
                        }
                    }
                    o[0] = o[1] = o[2] = o[3] = 0.0f; /* empty pixel (tile.metal:227-230) */
                    if (c > 0) composite(mode, fr, c, o);
                }
            }
        }
        free(ord);
        free(sel);
        free(fr);
    }
    if (st) {
        st->visible = visible;
        st->pairs = pairs;
        st->tiles = T;
    }
#undef ORA_OWNED
    free(slot);
    free(list);
    free(cnt);
    return 1;
}

int ora_composite_records(const ora_record *rec, const uint32_t *dkey, int64_t n, int W, int H,
                          const ora_options *opt, const uint8_t *owner, int rank, int compact, float *out,
                          ora_stats *st) {
    if (opt && opt->mode == ORA_MODE_MLAB && opt->cap > 0) return 0;
    return composite_records_impl(rec, dkey, n, W, H, opt, owner, rank, compact, out, st, 0, 0, NULL);
}

int ora_composite_slab(const ora_record *rec, const uint32_t *dkey, int64_t n, int W, int H, const ora_options *opt,
                       int pass, int slab_rank, const float *t_all, float *out) {
    if ((pass != 1 && pass != 2) || (opt && (opt->cap > 0 || opt->mode == ORA_MODE_MLAB)) ||
        (pass == 2 && slab_rank > 0 && !t_all))
        return 0;
    return composite_records_impl(rec, dkey, n, W, H, opt, NULL, 0, 0, out, NULL, pass, slab_rank, t_all);
}

int ora_render(const ora_scene *s, const float V[16], const float P[16], int W, int H,
               const ora_options *opt, float *out, ora_stats *st) {
    int64_t n = s->n;
    ora_record *rec = (ora_record *)malloc(sizeof(ora_record) * (size_t)(n > 0 ? n : 1));
    uint32_t *dkey = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    uint32_t *nt = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(n > 0 ? n : 1));
    ora_project_all(s, V, P, W, H, rec, dkey, nt, opt ? opt->nthreads : 0);
    int ok = ora_composite_records(rec, dkey, n, W, H, opt, NULL, 0, 0, out, st);
    free(rec);
    free(dkey);
    free(nt);
    return ok;
}
