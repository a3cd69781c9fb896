/*
 * insitu_oracle.c -- CPU ORACLE (test infrastructure only; see insitu_oracle.h).
 *
 * A line-by-line C99 restatement of the scenery-insitu GLSL compute shaders that make up
 * the distributed VDI hot path.  Reference files (read-only, /root/reference):
 *   src/test/resources/graphics/scenery/insitu/VDIGenerator.comp        (VG:)
 *   src/test/resources/graphics/scenery/insitu/AccumulateVDI.comp       (AV:)
 *   src/test/resources/graphics/scenery/insitu/VolumeRaycaster.comp     (VR:)
 *   src/test/resources/graphics/scenery/insitu/AccumulatePlainImage.comp(AP:)
 *   src/test/resources/graphics/scenery/insitu/PlainImageCompositor.comp(PC:)
 *   src/test/resources/graphics/scenery/insitu/VDICompositor.comp       (VC:)
 * Line citations below use those prefixes.
 *
 * Build: see oracle/Makefile (gcc -O3 -march=x86-64-v3 -ffp-contract=off -fopenmp).  NEVER build with
 * -ffast-math: the contract is IEEE binary32 with the explicit fmaf() calls below.
 */
#include "insitu_oracle.h"
#include <math.h>
#include <string.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------
 * Robustness variants (built as separate libraries by the oracle/Makefile `variants` target;
 * tests/test_parity_robustness.py and tools/parity_robustness.py).  Each
 * replaces one part of the numerical contract with another plausible implementation of the same
 * GLSL, to measure how far outputs move:
 *   ORC_NOFMA          the shader expressions without contraction (every * and + rounded apart)
 *   ORC_LIBM_POW       pow() from the C library instead of exp2(y*log2(x)) with fixed polynomials
 *   ORC_FIXED_WEIGHTS  texture-unit filtering: trilinear and LUT weights rounded to 8 fraction bits
 *   ORC_LUT_EDGE       LUT lookups without the texel-centre shift (s*n instead of s*n - 0.5)
 * Default build: none of them (the contract).
 * ---------------------------------------------------------------------------------- */
#ifdef ORC_NOFMA
#define SFMA(a, b, c) ((a) * (b) + (c))
#else
#define SFMA(a, b, c) fmaf(a, b, c)
#endif
#ifdef ORC_FIXED_WEIGHTS
#define QW(f) (floorf((f) * 256.0f + 0.5f) * (1.0f / 256.0f))
#else
#define QW(f) (f)
#endif
#ifdef ORC_LUT_EDGE
#define LUT_SHIFT 0.0f
#else
#define LUT_SHIFT -0.5f
#endif

/* ------------------------------------------------------------------------------------
 * GLSL helpers with the documented evaluation order
 * ---------------------------------------------------------------------------------- */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* GLSL min/max: min(x,y) = y < x ? y : x ; max(x,y) = x < y ? y : x (spec definitions) */
static inline float gmin(float x, float y) { return (y < x) ? y : x; }
static inline float gmax(float x, float y) { return (x < y) ? y : x; }
/* GLSL mix(x,y,a) = x*(1-a) + y*a, contracted: fma(y, a, x*(1-a)) */
static inline float gmix(float x, float y, float a) { return SFMA(y, a, x * (1.0f - a)); }

typedef struct { float x, y, z, w; } v4;

static inline v4 mat_vec(const float* m, v4 v) {
    /* column-major mat4 * vec4: ((c0*x + c1*y) + c2*z) + c3*w, contracted */
    v4 r;
    r.x = SFMA(m[12], v.w, SFMA(m[8], v.z, SFMA(m[4], v.y, m[0] * v.x)));
    r.y = SFMA(m[13], v.w, SFMA(m[9], v.z, SFMA(m[5], v.y, m[1] * v.x)));
    r.z = SFMA(m[14], v.w, SFMA(m[10], v.z, SFMA(m[6], v.y, m[2] * v.x)));
    r.w = SFMA(m[15], v.w, SFMA(m[11], v.z, SFMA(m[7], v.y, m[3] * v.x)));
    return r;
}
static inline v4 v4mix(v4 a, v4 b, float t) {
    v4 r = { gmix(a.x, b.x, t), gmix(a.y, b.y, t), gmix(a.z, b.z, t), gmix(a.w, b.w, t) };
    return r;
}
static inline float len4(float x, float y, float z, float w) {
    return sqrtf(SFMA(w, w, SFMA(z, z, SFMA(y, y, x * x))));
}
static inline float len3(float x, float y, float z) {
    return sqrtf(SFMA(z, z, SFMA(y, y, x * x)));
}
/* v *= 1/v.w  (VG:318, VG:320, AV:144, AV:215, AV:247) */
static inline v4 persp_div(v4 v) {
    float r = 1.0f / v.w;
    v4 o = { v.x * r, v.y * r, v.z * r, v.w * r };
    return o;
}

void orc_mat4_mul(const float* a, const float* b, float* out) {
    /* (A*B) column c = A * B[c]  (GLSL mat4 product) */
    float t[16];
    for (int c = 0; c < 4; ++c) {
        v4 col = { b[c * 4 + 0], b[c * 4 + 1], b[c * 4 + 2], b[c * 4 + 3] };
        v4 r = mat_vec(a, col);
        t[c * 4 + 0] = r.x; t[c * 4 + 1] = r.y; t[c * 4 + 2] = r.z; t[c * 4 + 3] = r.w;
    }
    memcpy(out, t, sizeof t);
}

/* ------------------------------------------------------------------------------------
 * Deterministic log2 / exp2 / pow (GLSL: pow(x,y) := exp2(y*log2(x)); precision is
 * implementation-defined there, so the contract fixes one algorithm).
 * ---------------------------------------------------------------------------------- */
float orc_log2(float x) {
    if (x != x || x < 0.0f) return NAN;
    if (x == 0.0f) return -INFINITY;
    if (x == INFINITY) return INFINITY;
    int eadj = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; eadj = -23; }   /* subnormal: *2^23 */
    uint32_t u = f2u(x);
    int e = (int)((u >> 23) & 0xffu) - 127 + eadj;
    float m = u2f((u & 0x007fffffu) | 0x3f800000u);                 /* [1,2) */
    if (m > 1.41421354f) { m = m * 0.5f; e += 1; }                  /* [0.7071,1.4142] */
    float f = m - 1.0f;                                              /* exact */
    float s = f / (2.0f + f);
    float z = s * s;
    /* ln(1+f) = 2s + 2s*z*(1/3 + z/5 + z^2/7 + z^3/9 + z^4/11) */
    float p = fmaf(z, 0.0909090936f, 0.111111112f);
    p = fmaf(z, p, 0.142857149f);
    p = fmaf(z, p, 0.200000003f);
    p = fmaf(z, p, 0.333333343f);
    float s2 = s + s;
    float ln = fmaf(s2 * z, p, s2);
    return fmaf(ln, 1.44269502f, (float)e);
}

float orc_exp2(float y) {
    if (y != y) return y;
    if (y >= 128.0f) return INFINITY;
    if (y < -150.0f) return 0.0f;
    float n = rintf(y);                                              /* nearest, ties even */
    float f = y - n;                                                 /* exact, |f| <= 0.5 */
    float p = 1.52527336e-05f;                                       /* ln2^k/k!, k = 7..1 */
    p = fmaf(p, f, 1.54035297e-04f);
    p = fmaf(p, f, 1.33335581e-03f);
    p = fmaf(p, f, 9.61812911e-03f);
    p = fmaf(p, f, 5.55041087e-02f);
    p = fmaf(p, f, 2.40226507e-01f);
    p = fmaf(p, f, 6.93147182e-01f);
    p = fmaf(p, f, 1.0f);
    int ni = (int)n;
    if (ni > 127) return (p * u2f(0x7f000000u)) * 2.0f;             /* 2^127 * 2 */
    if (ni >= -126) return p * u2f((uint32_t)(ni + 127) << 23);
    return (p * u2f((uint32_t)(ni + 127 + 64) << 23)) * u2f((uint32_t)(127 - 64) << 23);
}

float orc_pow(float x, float y) {
#ifdef ORC_LIBM_POW
    return powf(x, y);
#else
    return orc_exp2(y * orc_log2(x));
#endif
}
static inline float orc_ln(float x) { return orc_log2(x) * 0.693147182f; }

/* VG:80-82 adjustOpacity */
static inline float adjust_opacity(float a, float modified_step_length) {
    return 1.0f - orc_pow(1.0f - a, modified_step_length);
}

/* rgba8 UNORM store: round(clamp(x,0,1)*255) */
static inline uint8_t unorm8(float x) {
    float q = (x > 0.0f) ? ((x < 1.0f) ? x : 1.0f) : 0.0f;
    return (uint8_t)(int)floorf(fmaf(q, 255.0f, 0.5f));
}

/* ------------------------------------------------------------------------------------
 * scenery sampleVolume / convert / intersectBoundingBox  (EXTERNAL in the reference;
 * called at AV:4, VG:337, VR:117, AP:3).  Contract:
 *   p = im * wpos (voxel space, voxel centres at integer coordinates; this is
 *       texture(volume, (p+0.5)/dims) of scenery's SampleSimpleVolume, evaluated directly)
 *   val = trilinear(p), clamp-to-edge, on raw voxel values
 *   raw = val * conv_scale + conv_offset        (convert, unorm folded into conv_scale)
 *   a   = TF(raw + 0.001), rgb = colormap(raw + 0.001), linear LUTs, texel centres,
 *         clamp-to-edge
 *   bbox: intersectBox(im*wfront, im*wback - im*wfront, 0, dims)  (VG:64-78)
 * ---------------------------------------------------------------------------------- */
static inline float voxel(const orc_brick* b, int x, int y, int z) {
    size_t idx = ((size_t)z * (size_t)b->dims[1] + (size_t)y) * (size_t)b->dims[0] + (size_t)x;
    switch (b->dtype) {
    case ORC_U8: return (float)((const uint8_t*)b->data)[idx];
    case ORC_U16: return (float)((const uint16_t*)b->data)[idx];
    default: return ((const float*)b->data)[idx];
    }
}

/* floor + clamp to valid texel pair, shared by trilinear and LUT lookups */
static inline void texel_pair(float t, int n, int* i0, int* i1, float* frac) {
    float fl = floorf(t);
    *frac = t - fl;
    if (!(fl >= -1.0f)) fl = -1.0f;            /* also catches NaN */
    if (fl > (float)n) fl = (float)n;
    int i = (int)fl;
    int a = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    int c = i + 1 < 0 ? 0 : (i + 1 > n - 1 ? n - 1 : i + 1);
    *i0 = a; *i1 = c;
}

static inline float trilinear(const orc_brick* b, float u, float v, float w) {
    int x0, x1, y0, y1, z0, z1;
    float fx, fy, fz;
    texel_pair(u, b->dims[0], &x0, &x1, &fx);
    texel_pair(v, b->dims[1], &y0, &y1, &fy);
    texel_pair(w, b->dims[2], &z0, &z1, &fz);
    fx = QW(fx);
    fy = QW(fy);
    fz = QW(fz);
    float c00 = gmix(voxel(b, x0, y0, z0), voxel(b, x1, y0, z0), fx);
    float c10 = gmix(voxel(b, x0, y1, z0), voxel(b, x1, y1, z0), fx);
    float c01 = gmix(voxel(b, x0, y0, z1), voxel(b, x1, y0, z1), fx);
    float c11 = gmix(voxel(b, x0, y1, z1), voxel(b, x1, y1, z1), fx);
    float c0 = gmix(c00, c10, fy);
    float c1 = gmix(c01, c11, fy);
    return gmix(c0, c1, fz);
}

static inline v4 sample_volume(const orc_brick* b, const orc_transfer* tf, v4 wpos) {
    v4 p = mat_vec(b->im, wpos);
    float val = trilinear(b, p.x, p.y, p.z);
    float raw = SFMA(val, tf->conv_scale, tf->conv_offset);
    float s = raw + 0.001f;
    int i0, i1;
    float fr;
    texel_pair(SFMA(s, (float)tf->n_tf, LUT_SHIFT), tf->n_tf, &i0, &i1, &fr);
    fr = QW(fr);
    float a = gmix(tf->tf[i0], tf->tf[i1], fr);
    texel_pair(SFMA(s, (float)tf->n_cm, LUT_SHIFT), tf->n_cm, &i0, &i1, &fr);
    fr = QW(fr);
    const float* c0 = tf->cmap + 4 * i0;
    const float* c1 = tf->cmap + 4 * i1;
    v4 r = { gmix(c0[0], c1[0], fr), gmix(c0[1], c1[1], fr), gmix(c0[2], c1[2], fr), a };
    return r;
}

/* VG:64-78 intersectBox on (im*wfront, im*wback - im*wfront, 0, sourcemax) */
static inline void intersect_bbox(const orc_brick* b, v4 wfront, v4 wback, float* tnear, float* tfar) {
    v4 mf = mat_vec(b->im, wfront);
    v4 mb = mat_vec(b->im, wback);
    float ro[3] = { mf.x, mf.y, mf.z };
    float rd[3] = { mb.x - mf.x, mb.y - mf.y, mb.z - mf.z };
    float tmn[3], tmx[3];
    for (int k = 0; k < 3; ++k) {
        float invR = 1.0f / rd[k];
        float tbot = invR * (0.0f - ro[k]);
        float ttop = invR * ((float)b->dims[k] - ro[k]);
        tmn[k] = gmin(ttop, tbot);
        tmx[k] = gmax(ttop, tbot);
    }
    *tnear = gmax(gmax(tmn[0], tmn[1]), gmax(tmn[0], tmn[2]));
    *tfar = gmin(gmin(tmx[0], tmx[1]), gmin(tmx[0], tmx[2]));
}

/* ------------------------------------------------------------------------------------
 * VDI generation, one pixel.  VG:263-600 with AV:1-352 spliced at VG:476.
 * ---------------------------------------------------------------------------------- */
#define ORC_MAX_VOLUMES 8

typedef struct {
    const orc_brick* b[ORC_MAX_VOLUMES];   /* the volumes of one VDI ($repeat, VG:333-347), in order */
    int nb;
    const orc_transfer* tf;
    const orc_camera* cam;
    float ipv[16], pv[16];
    int W, H, S;
    float* color;
    float* depth;
    uint32_t* octree;
    int32_t* passes;
    int ncx, ncy, ncz;
    float interval_size;
    int x_base;        /* column of colour/depth row 0 (band outputs); 0 for whole-frame outputs */
    int pass_stride;   /* row stride of passes (W, or the band width) */
} vdi_job;

/* VG:244-254 findZInterval_view */
static inline int find_z_interval_view(const vdi_job* J, float z_view) {
    float dist_from_front = fabsf(z_view - (-1.0f * 0.1f));
    float q = floorf(dist_from_front / J->interval_size);
    /* int(floor(q)); values >= ncz are out of the image and their atomics are dropped */
    if (!(q < (float)J->ncz)) return J->ncz;
    return (int)q;
}

/* AV:143-177 / AV:315-331: octree cell counts of one written supersegment */
static void octree_update(const vdi_job* J, float uvx, float uvy, float start, float end, int cx, int cy) {
    v4 s = { uvx, uvy, start, 1.0f };
    v4 e = { uvx, uvy, end, 1.0f };
    v4 sw = persp_div(mat_vec(J->ipv, s));
    v4 ew = persp_div(mat_vec(J->ipv, e));
    v4 sv = mat_vec(J->cam->view, sw);
    v4 ev = mat_vec(J->cam->view, ew);
    int sc = find_z_interval_view(J, sv.z);
    int ec = find_z_interval_view(J, ev.z);
    if (cx < 0 || cx >= J->ncx || cy < 0 || cy >= J->ncy) return;
    for (int j = sc; j <= ec && j < J->ncz; ++j) {
        size_t idx = ((size_t)j * (size_t)J->ncy + (size_t)cy) * (size_t)J->ncx + (size_t)cx;
        __atomic_fetch_add(&J->octree[idx], 1u, __ATOMIC_RELAXED);   /* imageAtomicAdd */
    }
}

static void write_supersegment(const vdi_job* J, int gx, int gy, int index, float start, float end, v4 c) {
    /* VG:204-225; no index<S guard in the shader: out-of-image stores are discarded */
    if (index < 0 || index >= J->S) return;
    size_t px = (size_t)(gx - J->x_base) * (size_t)J->H + (size_t)gy;
    float* col = J->color + (px * (size_t)J->S + (size_t)index) * 4;
    col[0] = c.x; col[1] = c.y; col[2] = c.z; col[3] = c.w;
    float* dep = J->depth + px * (size_t)(2 * J->S) + (size_t)(2 * index);
    dep[0] = start;
    dep[1] = end;
}

static void vdi_pixel(const vdi_job* J, int gx, int gy) {
    const int W = J->W, H = J->H;
    const float nw = J->cam->nw;
    /* VG:286-287 grid cell of this pixel */
    int cx = (int)floorf(((float)gx / (float)W) * (float)J->ncx);
    int cy = (int)floorf(((float)gy / (float)H) * (float)J->ncy);
    /* VG:305-320 */
    float tcx = (float)gx / (float)W, tcy = (float)gy / (float)H;
    float uvx = SFMA(tcx, 2.0f, -1.0f), uvy = SFMA(tcy, 2.0f, -1.0f);
    v4 front = { uvx, uvy, -1.0f, 1.0f }, back = { uvx, uvy, 1.0f, 1.0f };
    v4 wfront = persp_div(mat_vec(J->ipv, front));
    v4 wback = persp_div(mat_vec(J->ipv, back));
    /* VG:330-347; the $repeat block once per volume, in order (one volume: the single brick case) */
    float tnear = 1.0f, tfar = 0.0f, tmax = J->cam->tmax;
    float n, f;
    int vis[ORC_MAX_VOLUMES];
    float localNear[ORC_MAX_VOLUMES], localFar[ORC_MAX_VOLUMES];
    for (int v = 0; v < J->nb; ++v) {
        vis[v] = 0;
        localNear[v] = 0.0f;
        localFar[v] = 0.0f;
        intersect_bbox(J->b[v], wfront, wback, &n, &f);
        f = gmin(tmax, f);
        if (n < f) {
            localNear[v] = n; localFar[v] = f;
            tnear = gmin(tnear, gmax(0.0f, n));
            tfar = gmax(tfar, f);
            vis[v] = 1;
        }
    }
    const int maxSupersegments = J->S;       /* VG:352 */
    int supersegmentNum = 0;
    int iter = 0;
    if (tnear < tfar) {
        float dsteps = truncf((tfar - tnear) / nw);            /* VG:372 */
        int numSteps = (dsteps > 2.0e9f) ? 2000000000 : (int)dsteps;
        float low_thresh = 0.0f, high_thresh = 1.732f;       /* VG:380-381 */
        int supsegs_written = 0, thresh_found = 0;
        int desired_supsegs = maxSupersegments;
        int delta = (int)floorf(0.15f * (float)maxSupersegments);   /* VG:388 */
        float mid_thresh = 0.0001f;                          /* VG:393 */
        int first_iteration = 1;
        while (!thresh_found || !supsegs_written) {         /* VG:404 */
            iter++;
            if (iter > 64) break;  /* never reached: the search ends in <= 24 passes */
            if (thresh_found) supsegs_written = 1;
            float newSupSegThresh = mid_thresh;
            int num_terminations = 0;
            int supersegmentIsOpen = 0;
            float supSegStartPoint = 0.0f, supSegEndPoint = 0.0f;
            int lastSample = 0, transparentSample = 0;
            v4 supersegmentAdjusted = { 0, 0, 0, 0 };
            float step = tnear;
            float step_prev = step - nw;
            v4 wprev = v4mix(wfront, wback, step_prev);
            float ndc_step = 0.0f;
            int steps_in_supseg = 0, steps_trunc_trans = 0;
            v4 curV = { 0, 0, 0, 0 };
            for (int i = 0; i < numSteps; ++i, step += nw) {  /* VG:447 */
                if (i == numSteps - 1) lastSample = 1;
                v4 wpos = v4mix(wfront, wback, step);
                /* ---- AccumulateVDI.comp, spliced once per volume (VG:476, $insert{Accumulate}) ---- */
                for (int v = 0; v < J->nb; ++v) {
                if (vis[v] && step > localNear[v] && step < localFar[v]) {    /* AV:1 */
                    transparentSample = 0;
                    v4 x = sample_volume(J->b[v], J->tf, wpos);            /* AV:4 */
                    if (x.x > -0.5f || lastSample) {                        /* AV:12 */
                        float newAlpha = x.w;
                        float w = adjust_opacity(newAlpha,
                            len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w)); /* AV:20 */
                        if (w <= 0.0f) transparentSample = 1;              /* AV:24 */
                        if (supersegmentIsOpen) {                           /* AV:34 */
                            v4 jump_pos = v4mix(wfront, wback, nw * (float)steps_in_supseg);       /* AV:50 */
                            float segLen = len4(jump_pos.x - wfront.x, jump_pos.y - wfront.y,
                                                jump_pos.z - wfront.z, jump_pos.w - wfront.w);     /* AV:52 */
                            float inva = 1.0f / curV.w;                                             /* AV:53 */
                            supersegmentAdjusted.x = curV.x * inva;
                            supersegmentAdjusted.y = curV.y * inva;
                            supersegmentAdjusted.z = curV.z * inva;
                            supersegmentAdjusted.w = adjust_opacity(curV.w, 1.0f / segLen);        /* AV:54 */
                            /* AV:69 diffPremultiplied(supersegmentAdjusted, x) (VG:84-89) */
                            float ax = supersegmentAdjusted.x * supersegmentAdjusted.w;
                            float ay = supersegmentAdjusted.y * supersegmentAdjusted.w;
                            float az = supersegmentAdjusted.z * supersegmentAdjusted.w;
                            float bx = x.x * x.w, by = x.y * x.w, bz = x.z * x.w;
                            float diff = len3(ax - bx, ay - by, az - bz);
                            if (diff >= newSupSegThresh) {                  /* AV:74, AV:91 */
                                num_terminations++;
                                supersegmentIsOpen = 0;
                                /* AV:103-106: segLen_trunc == segLen, so the adjusted colour is
                                 * recomputed from identical operands (same value) */
                                supSegEndPoint = ndc_step;                  /* AV:126 */
                                steps_in_supseg = 0;
                                steps_trunc_trans = 0;
                                if (thresh_found) {                         /* AV:132-180 */
                                    write_supersegment(J, gx, gy, supersegmentNum, supSegStartPoint,
                                                       supSegEndPoint, supersegmentAdjusted);
                                    octree_update(J, uvx, uvy, supSegStartPoint, supSegEndPoint, cx, cy);
                                    supersegmentNum++;
                                }
                            }
                        }
                        if (!supersegmentIsOpen && !transparentSample) {    /* AV:185 */
                            supersegmentIsOpen = 1;
                            v4 ndcStart = persp_div(mat_vec(J->pv, wpos)); /* AV:214-217 */
                            supSegStartPoint = ndcStart.z;
                            curV.x = curV.y = curV.z = curV.w = 0.0f;      /* AV:221 */
                        }
                        if (supersegmentIsOpen) {                           /* AV:225 */
                            float t = 1.0f - curV.w;                        /* AV:228-229 */
                            curV.x = SFMA(t * x.x, w, curV.x);
                            curV.y = SFMA(t * x.y, w, curV.y);
                            curV.z = SFMA(t * x.z, w, curV.z);
                            curV.w = SFMA(t, w, curV.w);
                            steps_in_supseg++;
                            if (!transparentSample) {                       /* AV:239-249 */
                                steps_trunc_trans = steps_in_supseg;
                                float step_next = step + nw;
                                v4 wnext = v4mix(wfront, wback, step_next);
                                v4 ndcPos = persp_div(mat_vec(J->pv, wnext));
                                ndc_step = ndcPos.z;
                            }
                        }
                        if (lastSample && supersegmentIsOpen) {             /* AV:257 */
                            v4 jump_pos = v4mix(wfront, wback, nw * (float)steps_trunc_trans);   /* AV:265 */
                            float segLen = len4(jump_pos.x - wfront.x, jump_pos.y - wfront.y,
                                                jump_pos.z - wfront.z, jump_pos.w - wfront.w);
                            float inva = 1.0f / curV.w;
                            supersegmentAdjusted.x = curV.x * inva;
                            supersegmentAdjusted.y = curV.y * inva;
                            supersegmentAdjusted.z = curV.z * inva;
                            supersegmentAdjusted.w = adjust_opacity(curV.w, 1.0f / segLen);
                            num_terminations++;
                            supersegmentIsOpen = 0;
                            supSegEndPoint = ndc_step;                      /* AV:299 */
                            steps_in_supseg = 0;
                            if (thresh_found) {                             /* AV:304-334 */
                                write_supersegment(J, gx, gy, supersegmentNum, supSegStartPoint,
                                                   supSegEndPoint, supersegmentAdjusted);
                                octree_update(J, uvx, uvy, supSegStartPoint, supSegEndPoint, cx, cy);
                                supersegmentNum++;
                            }
                        }
                    }
                }
                }
                /* ---- end AccumulateVDI ---- */
                wprev = wpos;                                               /* VG:487 */
            }
            if (!supsegs_written) {                                         /* VG:497-529 */
                if (fabsf(high_thresh - low_thresh) < 0.000001f) {
                    thresh_found = 1;
                    mid_thresh = (num_terminations == 0) ? low_thresh : high_thresh;
                    continue;
                } else if (num_terminations > desired_supsegs) {
                    low_thresh = mid_thresh;
                } else if (num_terminations < (desired_supsegs - delta)) {
                    high_thresh = mid_thresh;
                } else {
                    thresh_found = 1;
                    continue;
                }
                if (first_iteration) {
                    first_iteration = 0;
                    if (num_terminations < desired_supsegs) {
                        thresh_found = 1;
                        continue;
                    }
                }
                mid_thresh = (low_thresh + high_thresh) / 2.0f;
            }
        }
    }
    /* VG:553-590 zero-fill the unused slots */
    for (int i = supersegmentNum; i < maxSupersegments; ++i) {
        v4 z = { 0, 0, 0, 0 };
        write_supersegment(J, gx, gy, i, 0.0f, 0.0f, z);
    }
    if (J->passes) J->passes[(size_t)gy * (size_t)J->pass_stride + (size_t)(gx - J->x_base)] = iter;
}

static int vdi_job_init(vdi_job* J, const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam,
                        int W, int H, int S, float* color, float* depth, uint32_t* octree, int32_t* passes) {
    if (!brick || !tf || !cam || !color || !depth || !octree) return -1;
    if (W <= 0 || H <= 0 || S <= 0 || tf->n_tf <= 0 || tf->n_cm <= 0) return -2;
    J->b[0] = brick; J->nb = 1; J->tf = tf; J->cam = cam;
    orc_mat4_mul(cam->inv_view, cam->inv_proj, J->ipv);   /* VG:289 */
    orc_mat4_mul(cam->proj, cam->view, J->pv);            /* VG:290 */
    J->W = W; J->H = H; J->S = S;
    J->color = color; J->depth = depth; J->octree = octree; J->passes = passes;
    J->ncx = W / 8; J->ncy = H / 8; J->ncz = S;            /* DistributedVolumes.kt:342 */
    J->interval_size = (20.0f - 0.1f) / (float)S;          /* VG:241-247 */
    J->x_base = 0;
    J->pass_stride = W;
    return 0;
}

int orc_vdi_generate(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam,
                     int W, int H, int S, float* color, float* depth, uint32_t* octree,
                     int32_t* passes, int x0, int x1) {
    vdi_job J;
    int rc = vdi_job_init(&J, brick, tf, cam, W, H, S, color, depth, octree, passes);
    if (rc) return rc;
    if (x0 < 0) x0 = 0;
    if (x1 > W) x1 = W;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int gx = x0; gx < x1; ++gx)
        for (int gy = 0; gy < H; ++gy) vdi_pixel(&J, gx, gy);
    return 0;
}

int orc_vdi_generate_mt(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam,
                        int W, int H, int S, float* color, float* depth, uint32_t* octree,
                        int32_t* passes, int nthreads) {
    vdi_job J;
    int rc = vdi_job_init(&J, brick, tf, cam, W, H, S, color, depth, octree, passes);
    if (rc) return rc;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int gx = 0; gx < W; ++gx)
        for (int gy = 0; gy < H; ++gy) vdi_pixel(&J, gx, gy);
    (void)nthreads;
    return 0;
}

int orc_vdi_generate_cols(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam,
                          int W, int H, int S, int x0, int x1, float* color, float* depth, uint32_t* octree,
                          int32_t* passes, int nthreads) {
    vdi_job J;
    if (x0 < 0 || x1 > W || x0 >= x1) return -3;
    int rc = vdi_job_init(&J, brick, tf, cam, W, H, S, color, depth, octree, passes);
    if (rc) return rc;
    J.x_base = x0;
    J.pass_stride = x1 - x0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int gx = x0; gx < x1; ++gx)
        for (int gy = 0; gy < H; ++gy) vdi_pixel(&J, gx, gy);
    (void)nthreads;
    return 0;
}

int orc_vdi_generate_multi(const orc_brick* const* bricks, int nb, const orc_transfer* tf, const orc_camera* cam,
                           int W, int H, int S, int x0, int x1, float* color, float* depth, uint32_t* octree,
                           int32_t* passes, int nthreads) {
    vdi_job J;
    if (!bricks || nb < 1 || nb > ORC_MAX_VOLUMES || x0 < 0 || x1 > W || x0 >= x1) return -3;
    int rc = vdi_job_init(&J, bricks[0], tf, cam, W, H, S, color, depth, octree, passes);
    if (rc) return rc;
    for (int v = 0; v < nb; ++v) {
        if (!bricks[v]) return -1;
        J.b[v] = bricks[v];
    }
    J.nb = nb;
    J.x_base = x0;
    J.pass_stride = x1 - x0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int gx = x0; gx < x1; ++gx)
        for (int gy = 0; gy < H; ++gy) vdi_pixel(&J, gx, gy);
    (void)nthreads;
    return 0;
}

/* ------------------------------------------------------------------------------------
 * Plain mode.  VR:76-163 with AP:1-14 spliced at VR:143.
 * ---------------------------------------------------------------------------------- */
/* VR:63-69 EncodeFloatRGBA */
static inline void encode_float_rgba(float v, float enc[4]) {
    enc[0] = 1.0f * v;
    enc[1] = 255.0f * v;
    enc[2] = 65025.0f * v;
    enc[3] = 16581375.0f * v;
    for (int k = 0; k < 4; ++k) enc[k] = enc[k] - floorf(enc[k]);   /* fract */
    const float c = 1.0f / 255.0f;
    float e0 = SFMA(-enc[1], c, enc[0]);
    float e1 = SFMA(-enc[2], c, enc[1]);
    float e2 = SFMA(-enc[3], c, enc[2]);
    float e3 = SFMA(-enc[3], 0.0f, enc[3]);
    enc[0] = e0; enc[1] = e1; enc[2] = e2; enc[3] = e3;
}

void orc_encode_depth_rgba8(float v, uint8_t out[4]) {
    float enc[4];
    encode_float_rgba(v, enc);
    for (int k = 0; k < 4; ++k) out[k] = unorm8(enc[k]);
}

/* PC:25-29 DecodeFloatRGBA on an rgba8 texel (imageLoad of rgba8 = c/255) */
float orc_decode_depth_rgba8(const uint8_t in[4]) {
    const float d0 = 1.0f / 1.0f, d1 = 1.0f / 255.0f, d2 = 1.0f / 65025.0f, d3 = 1.0f / 16581375.0f;
    float v0 = (float)in[0] / 255.0f, v1 = (float)in[1] / 255.0f;
    float v2 = (float)in[2] / 255.0f, v3 = (float)in[3] / 255.0f;
    return SFMA(v3, d3, SFMA(v2, d2, SFMA(v1, d1, v0 * d0)));
}

int orc_plain_raycast(const orc_brick* brick, const orc_transfer* tf, const orc_camera* cam,
                      int dim0, int dim1, uint8_t* color, uint8_t* depth, int gy0, int gy1) {
    if (!brick || !tf || !cam || !color || !depth || dim0 <= 0 || dim1 <= 0) return -1;
    float ipv[16];
    orc_mat4_mul(cam->inv_view, cam->inv_proj, ipv);      /* VR:88 */
    const float nw = cam->nw, fwnw = cam->fwnw;
    if (gy0 < 0) gy0 = 0;
    if (gy1 > dim1) gy1 = dim1;
    for (int gy = gy0; gy < gy1; ++gy) {
        for (int gx = 0; gx < dim0; ++gx) {
            float tcx = (float)gx / (float)dim0, tcy = (float)gy / (float)dim1;   /* VR:96 */
            float uvx = SFMA(tcx, 2.0f, -1.0f), uvy = SFMA(tcy, 2.0f, -1.0f);
            v4 front = { uvx, uvy, -1.0f, 1.0f }, back = { uvx, uvy, 1.0f, 1.0f };
            v4 wfront = persp_div(mat_vec(ipv, front));
            v4 wback = persp_div(mat_vec(ipv, back));
            float tnear = 1.0f, tfar = 0.0f, tmax = cam->tmax, n, f;   /* VR:112-125 */
            int vis = 0;
            intersect_bbox(brick, wfront, wback, &n, &f);
            f = gmin(tmax, f);
            if (n < f) {
                tnear = gmin(tnear, gmax(0.0f, n));
                tfar = gmax(tfar, f);
                vis = 1;
            }
            size_t o = ((size_t)gy * (size_t)dim0 + (size_t)gx) * 4;
            if (tnear < tfar) {                                         /* VR:129 */
                int numSteps;
                if (fwnw > 0.00001f) {                                  /* VR:132-135 */
                    float q = orc_ln(SFMA(tfar, fwnw, nw) / SFMA(tnear, fwnw, nw)) / orc_ln(1.0f + fwnw);
                    numSteps = (q > 2.0e9f) ? 2000000000 : (int)q;
                } else {
                    float q = truncf((tfar - tnear) / nw + 1.0f);
                    numSteps = (q > 2.0e9f) ? 2000000000 : (int)q;
                }
                float step = tnear;
                v4 v = { 0, 0, 0, 0 };
                for (int i = 0; i < numSteps; ++i, step = step + SFMA(step, fwnw, nw)) {   /* VR:139 */
                    v4 wpos = v4mix(wfront, wback, step);
                    if (vis) {                                           /* AP:1-14 */
                        v4 x = sample_volume(brick, tf, wpos);
                        float t = 1.0f - v.w;
                        v.x = SFMA(t * x.x, x.w, v.x);
                        v.y = SFMA(t * x.y, x.w, v.y);
                        v.z = SFMA(t * x.z, x.w, v.z);
                        v.w = SFMA(t, x.w, v.w);
                        if (v.w >= 1.0f) break;
                    }
                }
                color[o + 0] = unorm8(v.x); color[o + 1] = unorm8(v.y);
                color[o + 2] = unorm8(v.z); color[o + 3] = unorm8(v.w);
                orc_encode_depth_rgba8(tnear, depth + o);               /* VR:155-157 */
            } else {
                memset(color + o, 0, 4);                                 /* VR:159-160 */
                memset(depth + o, 0, 4);
            }
        }
    }
    return 0;
}

/* PC:35-92 */
int orc_plain_composite(const uint8_t* vdis_color, const uint8_t* vdis_depth, int dim0,
                        int rows, int nprocs, uint8_t* out) {
    if (!vdis_color || !vdis_depth || !out || dim0 <= 0 || rows <= 0 || nprocs <= 0 || nprocs > 50) return -1;
    for (int gy = 0; gy < rows; ++gy) {
        for (int gx = 0; gx < dim0; ++gx) {
            int frontSupersegment[50];
            for (int i = 0; i < nprocs; ++i) frontSupersegment[i] = 0;
            float C[4] = { 0, 0, 0, 0 };
            for (int i = 0; i < nprocs; ++i) {
                float colour[4] = { 0, 0, 0, 0 };
                float lowDepth = 200.0f;
                int lowIndex = -1;
                for (int j = 0; j < nprocs; ++j) {
                    if (frontSupersegment[j] >= 1) continue;         /* numInputSupersegments = 1 */
                    size_t o = (((size_t)j * (size_t)rows + (size_t)gy) * (size_t)dim0 + (size_t)gx) * 4;
                    float d = orc_decode_depth_rgba8(vdis_depth + o);
                    if (d < lowDepth && d != 0.0f) {                 /* PC:73 */
                        lowDepth = d;
                        lowIndex = j;
                        for (int k = 0; k < 4; ++k) colour[k] = (float)vdis_color[o + k] / 255.0f;
                    }
                }
                float t = 1.0f - C[3];                               /* PC:81-82 */
                C[0] = SFMA(t * colour[0], colour[3], C[0]);
                C[1] = SFMA(t * colour[1], colour[3], C[1]);
                C[2] = SFMA(t * colour[2], colour[3], C[2]);
                C[3] = SFMA(t, colour[3], C[3]);
                if (lowIndex != -1) frontSupersegment[lowIndex]++;
            }
            size_t o = ((size_t)gy * (size_t)dim0 + (size_t)gx) * 4;
            for (int k = 0; k < 4; ++k) out[o + k] = unorm8(C[k]);
        }
    }
    return 0;
}

/* VDI flatten: determineNextSupseg order (VC:58-91) + accumulateSupseg (VG:147-185) */
int orc_vdi_flatten(const float* const* colors, const float* const* depths, int V, int S,
                    int H, int W, int strip_w, int x_offset, const float* ipv, uint8_t* out) {
    if (!colors || !depths || !ipv || !out || V <= 0 || V > 64 || S <= 0 || H <= 0 || strip_w <= 0) return -1;
    for (int xl = 0; xl < strip_w; ++xl) {
        for (int gy = 0; gy < H; ++gy) {
            int gx = x_offset + xl;
            float ndc_x = SFMA((float)gx / (float)W, 2.0f, -1.0f);      /* VG:152-153 */
            float ndc_y = SFMA((float)gy / (float)H, 2.0f, -1.0f);
            size_t px = (size_t)xl * (size_t)H + (size_t)gy;
            int front[64];
            for (int j = 0; j < V; ++j) front[j] = 0;
            float C[4] = { 0, 0, 0, 0 };
            for (;;) {
                float lowDepth = 100000.0f, startDepth = 0.0f, endDepth = 0.0f;   /* VC:60-64 */
                float colour[4] = { 0, 0, 0, 0 };
                int lowIndex = -1;
                for (int j = 0; j < V; ++j) {
                    if (front[j] >= S) continue;
                    const float* dj = depths[j] + px * (size_t)(2 * S) + (size_t)(2 * front[j]);
                    float cur = dj[0];
                    if (cur < lowDepth && cur != 0.0f) {                 /* VC:81 */
                        lowDepth = cur;
                        lowIndex = j;
                        startDepth = cur;
                        endDepth = dj[1];
                        const float* cj = colors[j] + (px * (size_t)S + (size_t)front[j]) * 4;
                        colour[0] = cj[0]; colour[1] = cj[1]; colour[2] = cj[2]; colour[3] = cj[3];
                    }
                }
                if (lowIndex < 0) break;
                /* accumulateSupseg(colour, startDepth, endDepth) VG:147-185 */
                v4 s = { ndc_x, ndc_y, startDepth, 1.0f };
                v4 e = { ndc_x, ndc_y, endDepth, 1.0f };
                v4 sw = persp_div(mat_vec(ipv, s));
                v4 ew = persp_div(mat_vec(ipv, e));
                float length_in_supseg = len4(sw.x - ew.x, sw.y - ew.y, sw.z - ew.z, sw.w - ew.w);
                float adj_alpha = adjust_opacity(colour[3], length_in_supseg);
                float t = 1.0f - C[3];
                C[0] = SFMA(t * colour[0], adj_alpha, C[0]);
                C[1] = SFMA(t * colour[1], adj_alpha, C[1]);
                C[2] = SFMA(t * colour[2], adj_alpha, C[2]);
                C[3] = SFMA(t, adj_alpha, C[3]);
                front[lowIndex]++;
            }
            size_t o = ((size_t)gy * (size_t)strip_w + (size_t)xl) * 4;
            for (int k = 0; k < 4; ++k) out[o + k] = unorm8(C[k]);
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------
 * VDICompositor.comp (VC) -- the re-supersegmenting compositor of VDI mode.
 * Per pixel of the strip: the V input lists are merged front to back by determineNextSupseg
 * (VC:58-91); gaps between consecutive inputs become transparent samples (VC:299-315); a
 * supersegment state machine with the same diffPremultiplied test as the generator (VC:317-392)
 * and its own threshold binary search (VC:209-223, 427-458; mid starts at 0.866, delta 3, no
 * first-iteration shortcut) writes at most S_out output supersegments (VC:102-150), the rest
 * are zeroed (VC:461-468).  The unused accumulated_adjusted (VC:332-335) is dead code and
 * skipped.  ndc_x uses the pixel's global x (VC:204 uses the strip-local x with the full window
 * width; DESIGN.md lists this as a deliberate deviation).
 * ---------------------------------------------------------------------------------- */
static void vc_write(float* oc, float* od, int S_out, size_t px, int index, float start, float end, v4 c) {
    if (index < 0 || index >= S_out) return;   /* VC:146-148 out-of-image imageStore: discarded */
    float* col = oc + (px * (size_t)S_out + (size_t)index) * 4;
    col[0] = c.x; col[1] = c.y; col[2] = c.z; col[3] = c.w;
    float* dep = od + px * (size_t)(2 * S_out) + (size_t)(2 * index);
    dep[0] = start;
    dep[1] = end;
}

static inline v4 vc_world(const float* ipv, float ndc_x, float ndc_y, float z) {
    v4 p = { ndc_x, ndc_y, z, 1.0f };
    return persp_div(mat_vec(ipv, p));
}

int orc_vdi_composite(const float* const* colors, const float* const* depths, int V, int S, int S_out,
                      int H, int W, int strip_w, int x_offset, const float* ipv,
                      float* out_color, float* out_depth, int32_t* passes, int ndc_x_strip_local) {
    if (!colors || !depths || !ipv || !out_color || !out_depth || V <= 0 || V > 64 || S <= 0 || S_out <= 0 ||
        H <= 0 || W <= 0 || strip_w <= 0)
        return -1;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int xl = 0; xl < strip_w; ++xl) {
        for (int gy = 0; gy < H; ++gy) {
            const int gx = x_offset + xl;
            const size_t px = (size_t)xl * (size_t)H + (size_t)gy;
            /* VC:204-205: the shader takes gl_GlobalInvocationID.x, i.e. the strip-local column, over the
             * full window width (ndc_x_strip_local, the reference-faithful mode); the default uses the
             * pixel's global column, which is what the formula means on every rank */
            const float ndc_x = SFMA((float)(ndc_x_strip_local ? xl : gx) / (float)W, 2.0f, -1.0f);
            const float ndc_y = SFMA((float)gy / (float)H, 2.0f, -1.0f);
            int supersegmentNum = 0;                                             /* VC:207 */
            float low_thresh = 0.0f, high_thresh = 1.732f;                       /* VC:209-211 */
            float mid_thresh = (high_thresh + low_thresh) / 2.0f;
            int thresh_found = 0, supsegs_written = 0;
            const int desired_supsegs = S_out, delta = 3;                        /* VC:219-220 */
            int iter = 0;
            int front[64];
            while (!thresh_found || !supsegs_written) {                          /* VC:225 */
                iter++;
                if (iter > 64) break;  /* safety only: the search ends in <= 23 passes */
                if (thresh_found) supsegs_written = 1;
                const float newSupSegThresh = mid_thresh;
                int num_terminations = 0;
                int open = 0;
                float ssStart = 0.0f, ssEnd = 0.0f, ssEndTT = 0.0f;
                v4 adj = { 0, 0, 0, 0 }, curV = { 0, 0, 0, 0 };
                for (int j = 0; j < V; ++j) front[j] = 0;
                int complete = 0;
                while (!complete) {                                              /* VC:256 */
                    int transparent = 0;
                    /* determineNextSupseg VC:58-91 */
                    float startDepth = 0.0f, endDepth = 0.0f, lowDepth = 100000.0f;
                    v4 colour = { 0, 0, 0, 0 };
                    int processId = -1;
                    for (int j = 0; j < V; ++j) {
                        if (front[j] >= S) continue;
                        const float* dj = depths[j] + px * (size_t)(2 * S) + (size_t)(2 * front[j]);
                        const float cur = dj[0];
                        if (cur < lowDepth && cur != 0.0f) {
                            lowDepth = cur;
                            processId = j;
                            startDepth = cur;
                            endDepth = dj[1];
                            const float* cj = colors[j] + (px * (size_t)S + (size_t)front[j]) * 4;
                            colour.x = cj[0]; colour.y = cj[1]; colour.z = cj[2]; colour.w = cj[3];
                        }
                    }
                    if (endDepth == 0.0f) complete = 1;                          /* VC:277-284 */
                    const v4 ssw0 = vc_world(ipv, ndc_x, ndc_y, startDepth);     /* VC:286-291 */
                    const v4 sew0 = vc_world(ipv, ndc_x, ndc_y, endDepth);
                    const float length_in_sample = len4(ssw0.x - sew0.x, ssw0.y - sew0.y, ssw0.z - sew0.z,
                                                        ssw0.w - sew0.w);
                    float adj_alpha = adjust_opacity(colour.w, length_in_sample); /* VC:293 */
                    adj_alpha = gmax(adj_alpha, 0.000001f);                      /* VC:295 */
                    if (open) {                                                  /* VC:297 */
                        if (startDepth > ssEnd) {                                /* VC:299-315 */
                            transparent = 1;
                            colour.x = colour.y = colour.z = colour.w = 0.0f;
                            adj_alpha = 0.0f;
                            endDepth = startDepth;
                            startDepth = ssEnd;
                        }
                        const v4 sw = vc_world(ipv, ndc_x, ndc_y, ssStart);      /* VC:317-322 */
                        const v4 ew = vc_world(ipv, ndc_x, ndc_y, ssEnd);
                        const float segLen = len4(sw.x - ew.x, sw.y - ew.y, sw.z - ew.z, sw.w - ew.w);
                        const float inva = 1.0f / curV.w;                        /* VC:325-326 */
                        adj.x = curV.x * inva;
                        adj.y = curV.y * inva;
                        adj.z = curV.z * inva;
                        adj.w = adjust_opacity(curV.w, 1.0f / segLen);
                        const float t = 1.0f - curV.w;                           /* VC:328-330 */
                        v4 acc;
                        acc.x = SFMA(t * colour.x, adj_alpha, curV.x);
                        acc.y = SFMA(t * colour.y, adj_alpha, curV.y);
                        acc.z = SFMA(t * colour.z, adj_alpha, curV.z);
                        acc.w = SFMA(t, adj_alpha, curV.w);
                        /* VC:338 diffPremultiplied(supersegmentAdjusted, colour) (VC:93-98) */
                        const float diff = len3(adj.x * adj.w - colour.x * colour.w,
                                                adj.y * adj.w - colour.y * colour.w,
                                                adj.z * adj.w - colour.z * colour.w);
                        if (diff >= newSupSegThresh || complete) {               /* VC:350-384 */
                            num_terminations++;
                            open = 0;
                            if (thresh_found) {
                                const v4 tw = vc_world(ipv, ndc_x, ndc_y, ssEndTT);
                                const float seglen_tt = len4(sw.x - tw.x, sw.y - tw.y, sw.z - tw.z, sw.w - tw.w);
                                adj.w = adjust_opacity(curV.w, 1.0f / seglen_tt);
                                vc_write(out_color, out_depth, S_out, px, supersegmentNum, ssStart, ssEndTT, adj);
                                supersegmentNum++;
                            }
                        } else {                                                 /* VC:385-392 */
                            curV = acc;
                            ssEnd = endDepth;
                            if (!transparent) ssEndTT = endDepth;
                        }
                    }
                    if (!open && !transparent) {                                 /* VC:395-408 */
                        ssStart = startDepth;
                        ssEnd = endDepth;
                        ssEndTT = endDepth;
                        curV.x = colour.x * adj_alpha;
                        curV.y = colour.y * adj_alpha;
                        curV.z = colour.z * adj_alpha;
                        curV.w = adj_alpha;
                        open = 1;
                    }
                    if (processId != -1 && !transparent) front[processId]++;    /* VC:410-417 */
                }
                if (!supsegs_written) {                                          /* VC:427-458 */
                    if (fabsf(high_thresh - low_thresh) < 0.000001f) {
                        thresh_found = 1;
                        mid_thresh = (num_terminations == 0) ? low_thresh : high_thresh;
                        continue;
                    } else if (num_terminations > desired_supsegs) {
                        low_thresh = mid_thresh;
                    } else if (num_terminations < (desired_supsegs - delta)) {
                        high_thresh = mid_thresh;
                    } else {
                        thresh_found = 1;
                        continue;
                    }
                    mid_thresh = (low_thresh + high_thresh) / 2.0f;
                }
            }
            for (int i = supersegmentNum; i < S_out; ++i) {                       /* VC:461-468 */
                v4 z = { 0, 0, 0, 0 };
                vc_write(out_color, out_depth, S_out, px, i, 0.0f, 0.0f, z);
            }
            if (passes) passes[(size_t)gy * (size_t)strip_w + (size_t)xl] = iter;
        }
    }
    return 0;
}
