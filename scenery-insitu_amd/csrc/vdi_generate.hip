// vdi_generate.hip -- VDI generation for gfx950: VDIGenerator.comp + AccumulateVDI.comp.
//
// Two kernels per frame, each covering all local bricks (after vdi_tile_len_kernel and a radix
// sort have ordered the tiles longest-first):
//
//  vdi_sample_kernel  one lane = one ray, one wave = one 8x8 pixel tile, tiles in the sorted
//      order.  Ray setup (VDIGenerator.comp:278-372) and the FIRST raymarch pass of the threshold
//      search (threshold 1e-4, :393) plus the counts of the next four levels of the search tree's
//      spine, with the brick sampled coherently by the tile.  Every in-brick sample's {LUT
//      coordinate, adjusted opacity} goes to the per-sample cache (8 bytes, lane-interleaved per
//      wave; positions are recomputed from the running ray parameter only where a written
//      supersegment needs its NDC depth).  A ray whose first pass closes
//      <= S supersegments is final right there -- the search accepts that threshold and the
//      write pass would replay the identical pass (:497-529) -- so the pass stores its
//      supersegments as it goes and the octree cells are counted from them afterwards.  The
//      other rays are appended to a queue (one atomic per wave).
//
//  vdi_search_kernel  persistent lanes pull queued rays from the queue and run the rest of the
//      binary search (:404-539) and the write pass by replaying the cache: no brick access, so
//      a ray needs no spatial coherence with its neighbours and a lane that finishes a ray
//      takes the next one.  Rays need 1..24 passes, so per-lane work differs by more than an
//      order of magnitude inside a tile; the queue keeps the lanes busy instead of idling
//      until the slowest ray of their tile is done.  Late search passes (INSITU_SPEC_FROM on)
//      store their supersegments as they go, so a pass the search accepts at its own threshold
//      is its own write pass.
//
// Rays the cache cannot hold run the whole search in vdi_sample_kernel and re-sample the brick
// every pass (vdi_march).  All paths evaluate the same float operations in the same order, so
// their results are bit-identical (tests/test_gpu_parity.py).
#include "insitu_sampling.h"
#include "insitu_filter.h"

#pragma clang fp contract(off)

namespace insitu {

#ifdef INSITU_DIAG
// diagnostics build only (tools/diag_build.sh): per-frame decision statistics printed to stderr
__device__ unsigned long long g_diag[16];
__device__ __forceinline__ void diag_count(int i, bool c) {
    const unsigned long long act = __ballot(1), b = __ballot(c);
    if ((int)(__lane_id()) == __builtin_ctzll(act)) {
        atomicAdd(&g_diag[(i & 3) + 8 * (i >> 2)], (unsigned long long)__popcll(b));
        atomicAdd(&g_diag[(i & 3) + 8 * (i >> 2) + 4], b ? 1ull : 0ull);
    }
}
#define INSITU_DIAG_COUNT(i, c) diag_count((i), (c))
#else
#define INSITU_DIAG_COUNT(i, c) ((void)0)
#endif
// diagnostics build (-DINSITU_DIAG_TIME): per wave, the shader-clock cycles of the search loop's sections
// (pops, regroup, replay, the round-end checks, the round-end code), summed over the waves
#ifdef INSITU_DIAG_TIME
__device__ unsigned long long g_dtime[8];
#define INSITU_T_DECL                                   \
    unsigned long long dt_acc[8] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull, 0ull}; \
    unsigned long long dt_mark = __builtin_readcyclecounter();
#define INSITU_T_MARK(i)                                          \
    {                                                             \
        const unsigned long long t_ = __builtin_readcyclecounter(); \
        dt_acc[i] += t_ - dt_mark;                                \
        dt_mark = t_;                                             \
    }
#define INSITU_T_FLUSH()                                                               \
    if (lane == 0)                                                                     \
        for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_dtime[i_], dt_acc[i_]);
#else
#define INSITU_T_DECL
#define INSITU_T_MARK(i)
#define INSITU_T_FLUSH()
#endif
#if defined(INSITU_ABL_CLASSIFY2) || defined(INSITU_ABL_EST2) || defined(INSITU_ABL_LEN2) || defined(INSITU_ABL_LOGEXP2)
// sensitivity experiments only (tools/variant_build.sh): redundant work whose result is multiplied by
// a runtime zero, to measure what extra VALU per sample costs
__device__ float g_abl_zero = 0.0f;
#endif

// VDIGenerator.comp:244-254
__device__ __forceinline__ int find_z_interval_view(float z_view, float interval_size, int ncz) {
    float dist_from_front = __builtin_fabsf(z_view - (-1.0f * 0.1f));
    float q = __builtin_floorf(dist_from_front / interval_size);
    if (!(q < (float)ncz)) return ncz;
    return (int)q;
}

#ifndef INSITU_SAMPLE_XCD_CHUNK
#define INSITU_SAMPLE_XCD_CHUNK 4    // consecutive blocks one XCD runs back to back (xcd_block; round 5 at 4 waves per SIMD: 4 / 8 against 16 -0.1 / -0.05 ms, 32 +0.3)
#endif
#ifndef INSITU_MERGE_MIN_BLOCKS
#define INSITU_MERGE_MIN_BLOCKS 3   // vdi_merge_kernel: waves per SIMD (A/B switch)
#endif
#ifndef INSITU_FINISH_MIN_BLOCKS
#define INSITU_FINISH_MIN_BLOCKS 1  // vdi_finish_kernel: waves per SIMD asked of the compiler (A/B switch)
#endif
#ifndef INSITU_SAMPLE_MIN_BLOCKS
#define INSITU_SAMPLE_MIN_BLOCKS 3   // 3 waves per SIMD (<= 168 VGPRs): measured 10.3 vs 11.4 ms at 2 waves
#endif
// offset (in chunks) of chunk c of a ray from its first chunk: the cache is lane-interleaved per sampling wave,
// chunk c of lane l at base + 64 c + l, so the 64 lanes storing their chunk c write 2 KiB in one piece
// (measured against one run per ray, -0.8 ms, and against groups of 2 or 4 chunks per lane: equal / +0.9 ms
// at N=1, pairs +0.23 ms on the 8-GPU share; the variants are in the history up to
// round 5's last commit)
__host__ __device__ __forceinline__ size_t chunk_off(uint32_t c) { return (size_t)c * 64u; }

// offset (in 64-byte slots) of slot c of a merged ray from its first slot: a lane's consecutive slots in pairs,
// one 128-byte line per pair, the pairs lane-interleaved (round 5: -0.4 ms of merged search against single slots)
__host__ __device__ __forceinline__ size_t mslot_off(uint32_t c) { return (size_t)(c / 2u) * 128u + (c % 2u); }

struct RayOut {
    float4* color;   // entry 0 of this pixel's block; slot i at + i*slot_stride
    float2* depth;
    uint32_t slot_stride;
};

// AccumulateVDI.comp:143-177 / :315-331 -- the z intervals [sc, ec] of one written supersegment
__device__ __forceinline__ void octree_range(const VdiGenParams& P, float uvx, float uvy, float start, float end,
                                             int& sc, int& ec) {
    f4 sw = persp_div(mat_vec(P.ipv, f4{uvx, uvy, start, 1.0f}));
    f4 ew = persp_div(mat_vec(P.ipv, f4{uvx, uvy, end, 1.0f}));
    float sz = mat_row(P.view, 2, sw);
    float ez = mat_row(P.view, 2, ew);
    sc = find_z_interval_view(sz, P.interval_size, P.S);
    ec = find_z_interval_view(ez, P.interval_size, P.S);
}

// ... and its octree cell counts
__device__ __forceinline__ void octree_update(const VdiGenParams& P, uint32_t* octree, float uvx, float uvy,
                                              float start, float end, int cx, int cy) {
    int sc, ec;
    octree_range(P, uvx, uvy, start, end, sc, ec);
    if (cx < 0 || cx >= P.ncx || cy < 0 || cy >= P.ncy) return;
    for (int j = sc; j <= ec && j < P.S; ++j)
        atomicAdd(&octree[((uint32_t)j * (uint32_t)P.ncy + (uint32_t)cy) * (uint32_t)P.ncx + (uint32_t)cx], 1u);
}

struct Ray {
    f4 wfront, wback;
    float uvx, uvy, localNear, localFar, tnear, tfar;
    int cx, cy, numSteps;
    bool hit;
};

// VDIGenerator.comp:282-320: grid cell, NDC and the world-space ray of pixel (gx, gy)
__device__ __forceinline__ void ray_dirs(const VdiGenParams& P, int gx, int gy, Ray& r) {
    r.cx = (int)__builtin_floorf(((float)gx / (float)P.W) * (float)P.ncx);   // :286-287
    r.cy = (int)__builtin_floorf(((float)gy / (float)P.H) * (float)P.ncy);
    const float tcx = (float)gx / (float)P.W, tcy = (float)gy / (float)P.H;
    r.uvx = __builtin_fmaf(tcx, 2.0f, -1.0f);
    r.uvy = __builtin_fmaf(tcy, 2.0f, -1.0f);
    r.wfront = persp_div(mat_vec(P.ipv, f4{r.uvx, r.uvy, -1.0f, 1.0f}));
    r.wback = persp_div(mat_vec(P.ipv, f4{r.uvx, r.uvy, 1.0f, 1.0f}));
}

// VDIGenerator.comp:278-372 for one brick (a1)
__device__ __forceinline__ Ray ray_setup(const VdiGenParams& P, const BrickDesc& brick, int gx, int gy) {
    Ray r;
    ray_dirs(P, gx, gy, r);
    float n, f;
    r.tnear = 1.0f;
    r.tfar = 0.0f;
    r.localNear = 0.0f;
    r.localFar = 0.0f;
    intersect_bbox(brick, r.wfront, r.wback, n, f);
    f = gmin(P.tmax, f);
    if (n < f) {
        r.localNear = n;
        r.localFar = f;
        r.tnear = gmin(r.tnear, gmax(0.0f, n));
        r.tfar = gmax(r.tfar, f);
    }
    r.hit = r.tnear < r.tfar;
    r.numSteps = 0;
    if (r.hit) {
        const float dsteps = __builtin_truncf((r.tfar - r.tnear) / P.nw);   // VDIGenerator.comp:372
        r.numSteps = (dsteps > 2.0e9f) ? 2000000000 : (int)dsteps;
    }
    return r;
}

// output entries of pixel (gx, gy) of brick b in the [d][b][xt][i][y][xx] send layout
__device__ __forceinline__ RayOut ray_out(const VdiGenParams& P, int gx, int gy, int b) {
    const int d = gx / P.strip_w, xl = gx - d * P.strip_w;
    const size_t blockE = (size_t)P.strip_tiles * (size_t)P.S * (size_t)P.H * 8;
    const size_t e0 = ((size_t)d * (size_t)P.B + (size_t)b) * blockE +
                      (((size_t)(xl >> 3) * (size_t)P.S) * (size_t)P.H + (size_t)gy) * 8 + (size_t)(xl & 7);
    return RayOut{P.color + e0, P.depth + e0, (uint32_t)P.H * 8u};
}

// AccumulateVDI.comp:225-251 front-to-back accumulation of a sample into the open supersegment:
// curV.rgb = fma(t * x.rgb, w, curV.rgb), curV.a = fma(t, w, curV.a) with t = 1 - curV.a, in pairs
__device__ __forceinline__ f4 accumulate(const f4& curV, const f4& xv, float wv) {
    const float t = 1.0f - curV.w;
    const f2v w2{wv, wv};
    return join2(pk_fma(lo2(xv) * t, w2, lo2(curV)), pk_fma(f2v{t * xv.z, t}, w2, hi2(curV)));
}

// The per-ray variables of one raymarch pass (AccumulateVDI.comp).
//
// Segmentation interval of a pass.  The threshold enters a pass only through the decisions
// `diff^2 >= thresh_sq`; every decision that closed bounds thresh_sq from above by its diff^2,
// every one that did not, from below.  So the pass makes exactly the same decisions -- the same
// supersegments, the same count -- for every squared threshold in (lo, hi], lo = the largest
// non-closing diff^2, hi = the smallest closing one (bounds on them when a filtered decision was
// certain without the exact value: see seg_lo_bound / seg_hi_bound).  A search pass whose squared
// threshold falls in the interval
// of the pass at `low` or at `high` has that pass's outcome: it is skipped (free_walk), which
// removes a third of the replays of the longest rays.  Results are identical by construction.
struct SegState {
    int nterm;
    bool open, transparent;
    float startPt, endPt;
    float tt_step;   // ray parameter of the last non-transparent sample (its next position's NDC z is
                     // the supersegment end, AccumulateVDI.comp:243-248, evaluated at the close)
    int steps_in, steps_tt;
    f4 adj, curV;
    float lo, hi;       // segmentation interval (TRACK == 1): bounds from margins and exact values
    float lo_a, hi_a;   // ... and the extreme estimates of precomputed-threshold decisions (PRE)
    __device__ __forceinline__ void reset() {
        nterm = 0;
        open = transparent = false;
        tt_step = 0.0f;
        startPt = 0.0f;             // with TRACK == 2 the interval's lo in search passes (thresholds > 0)
        endPt = __builtin_inff();   // with TRACK == 2 the interval's hi in search passes
        steps_in = steps_tt = 0;
        adj = f4{0.0f, 0.0f, 0.0f, 0.0f};
        curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
        lo = 0.0f;                  // diff^2 >= 0: 0 is as good as -inf for thresholds > 0
        lo_a = -1.0f;               // no estimate recorded (seg_lo_bound keeps it)
        hi = hi_a = __builtin_inff();
    }
};

// det_log2 with its one division replaced by a hardware reciprocal (estimate only), x in [0, 1]
__device__ __forceinline__ float approx_log2(float x) {
    const uint32_t u = __float_as_uint(x);
    int e = (int)((u >> 23) & 0xffu) - 127;
    float m = __uint_as_float((u & 0x007fffffu) | 0x3f800000u);
    const bool big = m > 1.41421354f;
    m = big ? m * 0.5f : m;
    e += big ? 1 : 0;
    const float f = m - 1.0f;
    const float sv = f * __builtin_amdgcn_rcpf(2.0f + f);
    const float z = sv * sv;
    float p = __builtin_fmaf(z, 0.0909090936f, 0.111111112f);
    p = __builtin_fmaf(z, p, 0.142857149f);
    p = __builtin_fmaf(z, p, 0.200000003f);
    p = __builtin_fmaf(z, p, 0.333333343f);
    const float s2 = sv + sv;
    const float r = __builtin_fmaf(__builtin_fmaf(s2 * z, p, s2), 1.44269502f, (float)e);
    return (x == 0.0f) ? -__builtin_inff() : r;   // x >= 2^-24 or 0 here (x = 1 - opacity)
}

// estimate of the squared supersegment difference (AccumulateVDI.comp:50-69).  The adjusted colour
// times the adjusted opacity is formed as curV.rgb * (rcp(curV.a) * aw): the same three rounded
// factors as (curV.rgb * rcp(curV.a)) * aw, so the same relative error budget.
__device__ __forceinline__ float approx_diff_sq(const f4& curV, int steps, const f4& xv, const f4& wfront,
                                                const f4& wback, float nw) {
    const f4 jp = v4mix(wfront, wback, nw * (float)steps);
    const float dx = jp.x - wfront.x, dy = jp.y - wfront.y, dz = jp.z - wfront.z, dw = jp.w - wfront.w;
#ifdef INSITU_ABL_LEN2
    // timing ablation: the segment length a second time, folded in with weight 0
    const float zz = g_abl_zero;
    const f4 jq = v4mix(wfront, wback, nw * (float)steps + zz);
    const float ex = jq.x - wfront.x, ey = jq.y - wfront.y, ez = jq.z - wfront.z, ew = jq.w - wfront.w;
    const float il2 = __builtin_amdgcn_rsqf(__builtin_fmaf(ew, ew, __builtin_fmaf(ez, ez, __builtin_fmaf(ey, ey, ex * ex))));
    const float inv_len = __builtin_fmaf(il2, zz, __builtin_amdgcn_rsqf(__builtin_fmaf(dw, dw, __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx)))));
#else
    const float inv_len = __builtin_amdgcn_rsqf(__builtin_fmaf(dw, dw, __builtin_fmaf(dz, dz, __builtin_fmaf(dy, dy, dx * dx))));
#endif
#if defined(INSITU_ABL_LOGEXP2)
    const float zz2 = g_abl_zero;
    const float aw2 = 1.0f - __builtin_amdgcn_exp2f(inv_len * __builtin_amdgcn_logf(1.0f - curV.w + zz2));
    const float aw = __builtin_fmaf(aw2, zz2, 1.0f - __builtin_amdgcn_exp2f(inv_len * __builtin_amdgcn_logf(1.0f - curV.w)));
#elif INSITU_HW_TRANSCENDENTALS
    // v_log_f32 / v_exp_f32: measured exhaustively on gfx950 (tools/hw_transcendental_error.hip) at
    // < 1 ulp over the arguments they get here -- inside the error budget of filter_margin
    const float aw = 1.0f - __builtin_amdgcn_exp2f(inv_len * __builtin_amdgcn_logf(1.0f - curV.w));
#else
    const float aw = 1.0f - det_exp2(inv_len * approx_log2(1.0f - curV.w));
#endif
    const float k = __builtin_amdgcn_rcpf(curV.w) * aw;
    // (ax, ay) - (bx, by) in pairs, az - bz alone: the same roundings as the scalar form
    const f2v exy = lo2(curV) * k - lo2(xv) * xv.w;
    const float ez = curV.z * k - xv.z * xv.w;
    return sumsq3(exy.x, exy.y, ez);
}

// exact adjusted colour of the open supersegment after `steps` samples (AccumulateVDI.comp:50-54)
__device__ __forceinline__ f4 exact_adjusted(const f4& curV, int steps, const f4& wfront, const f4& wback, float nw) {
    const f4 jp = v4mix(wfront, wback, nw * (float)steps);
    const float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);
    const float inva = 1.0f / curV.w;
    return f4{curV.x * inva, curV.y * inva, curV.z * inva, adjust_opacity(curV.w, 1.0f / segLen)};
}

__device__ __forceinline__ float exact_diff_sq(const f4& adj, const f4& xv) {
    const float ax = adj.x * adj.w, ay = adj.y * adj.w, az = adj.z * adj.w;
    const float bx = xv.x * xv.w, by = xv.y * xv.w, bz = xv.z * xv.w;
    return sumsq3(ax - bx, ay - by, az - bz);                                          // :69 (squared)
}

// the decision `diff >= threshold` (:74), filtered or exact; sets adj when it computed it exactly.
// bnd: the exact diff^2, or -- when the filtered estimate decided -- a bound on it in the direction
// that matters for the segmentation interval (a lower bound for a close, an upper one otherwise);
// with PRE the estimate itself (est = true), which seg_lo_bound / seg_hi_bound turn into bounds
// PRE: the decision thresholds th.hi / th.lo of make_thr (uniform thresholds: scalar registers);
// otherwise the margin is evaluated per sample (per-lane thresholds: two fewer live registers)
template <bool FILTERED, bool PRE>
__device__ __forceinline__ bool close_decision(const f4& curV, int steps, const f4& xv, const f4& wfront,
                                               const f4& wback, float nw, const Thr& th, float cmag, f4& adj,
                                               bool& have_adj, float& bnd, bool& est) {
    if constexpr (FILTERED) {
#ifdef INSITU_ABL_EST2
        const float zz = g_abl_zero;
        const float a2 = approx_diff_sq(curV, steps + (int)zz, xv, wfront, wback, nw + zz);
        const float a = __builtin_fmaf(a2, zz, approx_diff_sq(curV, steps, xv, wfront, wback, nw));
#else
        const float a = approx_diff_sq(curV, steps, xv, wfront, wback, nw);
#endif
        if constexpr (PRE) {   // NaN fails both tests; inf and huge estimates go to the exact path
            const bool yes = a >= th.hi && a < 1.0e30f, no = a < th.lo;
            INSITU_DIAG_COUNT(0, true);            // [0] decisions, [4] wave-level calls
            INSITU_DIAG_COUNT(1, !yes && !no);     // [1] exact fallbacks, [5] calls with any
            if (yes || no) {
                bnd = a;
                est = true;
                return yes;
            }
        } else {               // NaN / inf / huge estimates fail both tests (m is NaN)
            const float g = a - th.sq;
            const float m = (a < 1.0e30f) ? filter_margin(a, cmag) : __builtin_nanf("");
            INSITU_DIAG_COUNT(0, true);
            INSITU_DIAG_COUNT(1, !(g >= m) && !(g < -m));
            if (g >= m) {
                bnd = a - m;
                return true;
            }
            if (g < -m) {
                bnd = a + m;
                return false;
            }
        }
    }
    adj = exact_adjusted(curV, steps, wfront, wback, nw);
    have_adj = true;
    bnd = exact_diff_sq(adj, xv);
    return bnd >= th.sq;
}

// AccumulateVDI.comp:12-335 for one in-brick sample given its colour x, adjusted opacity w and
// its ray parameter stp (the running `step` of VDIGenerator.comp:447).  Positions are needed
// only for supersegment boundaries: ndc_of(t) = NDC z of mix(wfront, wback, t), evaluated when
// a supersegment opens (at stp, AccumulateVDI.comp:214-217) and when it closes (at the step after
// its last non-transparent sample, AccumulateVDI.comp:243-248 -- the same `step + nw` the loop
// increment computes, so the same bits as evaluating it at every sample).
// emit(start, end, adjusted colour, steps) runs for every supersegment that closes; with FILTERED
// the adjusted colour handed to emit is exact only when want_adj is set (the write pass).  With
// DEFER the colour handed over is the raw accumulated curV and steps its step count, from which
// vdi_finish_kernel computes the adjusted colour (AccumulateVDI.comp:50-54) afterwards.
// th.sq = sq_threshold(threshold): `diff >= threshold` is tested as `diff^2 >= th.sq` (th: make_thr).
// TRACK: 0 no segmentation interval, 1 in s.lo / s.hi, 2 in s.startPt / s.endPt while !want_adj
// (a search pass of vdi_search_kernel needs no supersegment positions: no extra registers).
template <bool FILTERED = false, int TRACK = 0, bool DEFER = false, bool PRE = false, class NdcOf, class Emit>
__device__ __forceinline__ void seg_sample(SegState& s, const f4 xv, const float wv, const float stp, NdcOf ndc_of,
                                           const bool last, const Thr& th, const f4& wfront,
                                           const f4& wback, const float nw, const float cmag, Emit emit,
                                           const bool want_adj = true) {
    s.transparent = false;
    if (!(xv.x > -0.5f || last)) return;                                             // :12
    if (wv <= 0.0f) s.transparent = true;                                            // :24-26
    const bool positions = TRACK != 2 || want_adj;
    if (s.open) {                                                                    // :34-91
        bool have_adj = false;
        float bnd;
        bool est = false;
        const bool close = close_decision<FILTERED, PRE>(s.curV, s.steps_in, xv, wfront, wback, nw, th, cmag, s.adj,
                                                         have_adj, bnd, est);
        if constexpr (TRACK == 1) {
            if (PRE && est) {
                if (close) s.hi_a = __builtin_fminf(s.hi_a, bnd);
                else s.lo_a = __builtin_fmaxf(s.lo_a, bnd);
            } else {
                if (close) s.hi = __builtin_fminf(s.hi, bnd);
                else s.lo = __builtin_fmaxf(s.lo, bnd);
            }
        }
        if constexpr (TRACK == 2) {
            if (!want_adj) {
                if (PRE && est) {
                    if (close) s.hi_a = __builtin_fminf(s.hi_a, bnd);
                    else s.lo_a = __builtin_fmaxf(s.lo_a, bnd);
                } else {
                    if (close) s.endPt = __builtin_fminf(s.endPt, bnd);
                    else s.startPt = __builtin_fmaxf(s.startPt, bnd);
                }
            }
        }
        if (close) {
            if (!DEFER && FILTERED && want_adj && !have_adj) s.adj = exact_adjusted(s.curV, s.steps_in, wfront, wback, nw);
            const int steps = s.steps_in;
            s.nterm++;
            s.open = false;
            if (positions) s.endPt = ndc_of(s.tt_step + nw);                        // :126 (ndc_step)
            s.steps_in = 0;
            s.steps_tt = 0;
            emit(s.startPt, s.endPt, DEFER ? s.curV : s.adj, steps);                // :132-180
        }
    }
    if (!s.open && !s.transparent) {                                                 // :185-221
        s.open = true;
        if (positions) s.startPt = ndc_of(stp);
        s.curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if (s.open) {                                                                    // :225-251
        s.curV = accumulate(s.curV, xv, wv);
        s.steps_in++;
        if (!s.transparent) {
            s.steps_tt = s.steps_in;
            if (positions) s.tt_step = stp;                                          // ndc_step at :243-248
        }
    }
    if (last && s.open) {                                                            // :257-335
        if (!DEFER && (!FILTERED || want_adj)) s.adj = exact_adjusted(s.curV, s.steps_tt, wfront, wback, nw);
        s.nterm++;
        s.open = false;
        if (positions) s.endPt = ndc_of(s.tt_step + nw);                            // :299
        s.steps_in = 0;
        emit(s.startPt, s.endPt, DEFER ? s.curV : s.adj, s.steps_tt);
    }
}

// seg_sample<true, 1, true, PRE> (the search kernel's replay: filtered decisions, segmentation interval in
// s.lo / s.hi, deferred colours, supersegment boundaries as ray parameters) with the state updates written as
// selects: the same float operations on the same operands, so the same states and the same stores.  Only the
// rare paths branch -- the exact decision (0.01 % of the decisions) and the stores of storing lanes -- and the
// estimate is computed for every lane of the wave (in the branching form some lane of the wave needs it at
// almost every sample).  `on` gates the whole sample (a lane past the end of its pass: no state change).
template <bool PRE, class Emit>
__device__ __forceinline__ void seg_sample_sel(SegState& s, const f4 xv, const float wv, const float stp, const bool on,
                                               const bool last, const Thr& th, const f4& wfront, const f4& wback,
                                               const float nw, const float cmag, Emit emit, const bool store) {
    const bool v = on && (xv.x > -0.5f || last);                                    // :12
    const bool tr = wv <= 0.0f;                                                      // :24-26
    const bool o = v && s.open;                                                      // :34-91
    const float a = approx_diff_sq(s.curV, s.steps_in, xv, wfront, wback, nw);
    bool close, est;
    if constexpr (PRE) {   // NaN fails both tests; inf and huge estimates go to the exact path
        const bool yes = a >= th.hi && a < 1.0e30f, no = a < th.lo;
        close = yes;
        est = yes || no;
    } else {
        const float g = a - th.sq;
        const float m = (a < 1.0e30f) ? filter_margin(a, cmag) : __builtin_nanf("");
        close = g >= m;
        est = close || g < -m;
    }
    INSITU_DIAG_COUNT(0, o);
    INSITU_DIAG_COUNT(1, o && !est);
    float bnd = a;
    if (o && !est) {   // exact decision (close_decision's fallback)
        const f4 adj = exact_adjusted(s.curV, s.steps_in, wfront, wback, nw);
        bnd = exact_diff_sq(adj, xv);
        close = bnd >= th.sq;
        if (close) s.hi = __builtin_fminf(s.hi, bnd);
        else s.lo = __builtin_fmaxf(s.lo, bnd);
    }
    close = close && o;
    if constexpr (PRE) {   // TRACK == 1 bounds of the estimate-decided samples
        const bool eu = o && est;
        s.hi_a = __builtin_fminf(s.hi_a, (eu && close) ? a : __builtin_inff());
        s.lo_a = __builtin_fmaxf(s.lo_a, (eu && !close) ? a : -1.0f);   // (lo_a >= -1 always)
    } else {
        const bool eu = o && est;
        const float m = filter_margin(a, cmag);
        s.hi = __builtin_fminf(s.hi, (eu && close) ? a - m : __builtin_inff());
        s.lo = __builtin_fmaxf(s.lo, (eu && !close) ? a + m : 0.0f);   // (lo >= 0 always)
    }
    if (close && store) emit(s.startPt, s.tt_step + nw, s.curV, s.steps_in);       // :126, :132-180
    s.nterm += close ? 1 : 0;
    const bool open1 = s.open && !close;
    s.steps_in = close ? 0 : s.steps_in;
    s.steps_tt = close ? 0 : s.steps_tt;
    const bool opening = v && !open1 && !tr;                                         // :185-221
    s.startPt = opening ? stp : s.startPt;
    const f4 base{opening ? 0.0f : s.curV.x, opening ? 0.0f : s.curV.y, opening ? 0.0f : s.curV.z,
                  opening ? 0.0f : s.curV.w};
    const bool open2 = open1 || opening;
    const bool acc = v && open2;                                                     // :225-251
    const f4 nv = accumulate(base, xv, wv);
    s.curV = f4{acc ? nv.x : base.x, acc ? nv.y : base.y, acc ? nv.z : base.z, acc ? nv.w : base.w};
    s.steps_in += acc ? 1 : 0;
    const bool tt = acc && !tr;
    s.steps_tt = tt ? s.steps_in : s.steps_tt;
    s.tt_step = tt ? stp : s.tt_step;
    const bool lc = v && last && open2;                                              // :257-335
    if (lc && store) emit(s.startPt, s.tt_step + nw, s.curV, s.steps_tt);           // :299
    s.nterm += lc ? 1 : 0;
    s.open = open2 && !lc;
    s.steps_in = lc ? 0 : s.steps_in;
}

// The supersegment counter of one raymarch pass without the supersegments themselves: the
// decisions of seg_sample (same float operations, same order) but only `nterm` is kept -- what a
// search pass needs (VDIGenerator.comp:497-529 reads num_terminations only).
struct CountState {
    f4 curV;
    int steps_in, nterm;
    bool open;
    float lo, hi, lo_a, hi_a;   // segmentation interval (see SegState)
    __device__ __forceinline__ void reset() {
        curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
        steps_in = nterm = 0;
        open = false;
        lo = 0.0f;
        lo_a = -1.0f;
        hi = hi_a = __builtin_inff();
    }
};

template <bool FILTERED, bool PRE>
__device__ __forceinline__ void count_sample(CountState& s, const f4 xv, const float wv, const bool last,
                                             const Thr& th, const f4& wfront, const f4& wback,
                                             const float nw, const float cmag) {
    if (!(xv.x > -0.5f || last)) return;
    const bool transparent = wv <= 0.0f;
    if (s.open) {
        f4 adj;
        bool have_adj = false;
        float bnd;
        bool est = false;
        if (close_decision<FILTERED, PRE>(s.curV, s.steps_in, xv, wfront, wback, nw, th, cmag, adj, have_adj, bnd, est)) {
            if (est) s.hi_a = __builtin_fminf(s.hi_a, bnd);
            else s.hi = __builtin_fminf(s.hi, bnd);
            s.nterm++;
            s.open = false;
            s.steps_in = 0;
        } else {
            if (est) s.lo_a = __builtin_fmaxf(s.lo_a, bnd);
            else s.lo = __builtin_fmaxf(s.lo, bnd);
        }
    }
    if (!s.open && !transparent) {
        s.open = true;
        s.curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if (s.open) {
        s.curV = accumulate(s.curV, xv, wv);
        s.steps_in++;
    }
    if (last && s.open) {
        s.nterm++;
        s.open = false;
    }
}

// Pass 1 and the spine counts of vdi_sample_kernel / vdi_merge_kernel: count_sample's state with the bounds of
// the exact decisions (lo, hi: changed by 0.01 % of the decisions) kept in LDS -- bnd[0] = lo, bnd[256] = hi,
// the lane's slots -- instead of two VGPRs per threshold (the kernel then fits 4 waves per SIMD).  The same
// decisions and values as count_sample.  (Pass 1 needs only its count and segmentation interval: count_sample
// makes the same decisions and counts as seg_sample with deferred colours.)
struct CountStateL {
    f4 curV;
    int steps_in, nterm;
    bool open;
    float lo_a, hi_a;
    __device__ __forceinline__ void reset() {
        curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
        steps_in = nterm = 0;
        open = false;
        lo_a = -1.0f;
        hi_a = __builtin_inff();
    }
};

template <bool FILTERED, bool PRE>
__device__ __forceinline__ void count_sample_l(CountStateL& s, float* bnd, const f4 xv, const float wv, const bool last,
                                               const Thr& th, const f4& wfront, const f4& wback, const float nw,
                                               const float cmag) {
    if (!(xv.x > -0.5f || last)) return;
    const bool transparent = wv <= 0.0f;
    if (s.open) {
        f4 adj;
        bool have_adj = false;
        float b;
        bool est = false;
        if (close_decision<FILTERED, PRE>(s.curV, s.steps_in, xv, wfront, wback, nw, th, cmag, adj, have_adj, b, est)) {
            if (est) s.hi_a = __builtin_fminf(s.hi_a, b);
            else bnd[256] = __builtin_fminf(bnd[256], b);
            s.nterm++;
            s.open = false;
            s.steps_in = 0;
        } else {
            if (est) s.lo_a = __builtin_fmaxf(s.lo_a, b);
            else bnd[0] = __builtin_fmaxf(bnd[0], b);
        }
    }
    if (!s.open && !transparent) {
        s.open = true;
        s.curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
    }
    if (s.open) {
        s.curV = accumulate(s.curV, xv, wv);
        s.steps_in++;
    }
    if (last && s.open) {
        s.nterm++;
        s.open = false;
    }
}

// Thresholds of the search tree below a node: child 2i+1 follows "n > S" (low = mid), child
// 2i+2 follows "n < S - delta" (high = mid), each with mid = (low + high) / 2 exactly as
// VDIGenerator.comp:519-527 computes it.  Node 0 is (low, high, mid) itself.
__device__ __forceinline__ float tree_threshold(float low, float high, float mid, int node) {
    const uint32_t m = (uint32_t)node + 1u;
    const int depth = 31 - __builtin_clz(m);
    for (int bit = depth - 1; bit >= 0; --bit) {
        if (((m >> bit) & 1u) == 0u) low = mid;
        else high = mid;
        mid = (low + high) / 2.0f;
    }
    return mid;
}

// Threshold search state (VDIGenerator.comp:380-393)
struct Search {
    float low, high, mid;
    int iter;
    bool found, written, first;
};

// VDIGenerator.comp:497-529, after a pass that did not write
__device__ __forceinline__ void search_update(Search& q, int n, int S, int delta) {
    if (__builtin_fabsf(q.high - q.low) < 0.000001f) {
        q.found = true;
        q.mid = (n == 0) ? q.low : q.high;
        return;
    } else if (n > S) {
        q.low = q.mid;
    } else if (n < S - delta) {
        q.high = q.mid;
    } else {
        q.found = true;
        return;
    }
    if (q.first) {
        q.first = false;
        if (n < S) {
            q.found = true;
            return;
        }
    }
    q.mid = (q.low + q.high) / 2.0f;
}

// One step of the search walk with the count n of the pass at q.mid and that pass's segmentation
// interval (lo, hi]: the bound the step moves inherits the interval.  iv = (seg_low, seg_high).
__device__ __forceinline__ void search_step(Search& q, int n, int S, int delta, float lo, float hi, float4& iv,
                                            int& n_high) {
    if (!(__builtin_fabsf(q.high - q.low) < 0.000001f)) {   // search_update's first test
        if (n > S) {
            iv.x = lo;
            iv.y = hi;
        } else if (n < S - delta) {
            iv.z = lo;
            iv.w = hi;
            n_high = n;
        }
    }
    search_update(q, n, S, delta);
}

// Passes whose squared threshold lies in the segmentation interval of the pass at `low` or at
// `high` are decided without replaying the ray: same decisions, same count (the bound they move
// keeps its interval).  Stops at the first threshold neither interval covers.
__device__ __forceinline__ void free_walk(Search& q, const float4 iv, int n_high, int S, int delta) {
    while (!q.found && q.iter < 63) {
        const float t = sq_threshold(q.mid);
        int n;
        if (t > iv.x && t <= iv.y) n = S + 1;   // the pass at `low` closed more than S
        else if (t > iv.z && t <= iv.w) n = n_high;
        else break;
        q.iter++;
        search_update(q, n, S, delta);
    }
}

__device__ __forceinline__ void store_slot(const RayOut& o, int i, float start, float end, const f4& c) {
    const uint32_t off = (uint32_t)i * o.slot_stride;
    o.color[off] = make_float4(c.x, c.y, c.z, c.w);
    o.depth[off] = make_float2(start, end);
}

// The slots past a ray's supersegments are not zero-filled (VDIGenerator.comp:553-590 does): the
// per-pixel count (seg_pending) bounds every reader, and the reference-layout readback
// (insitu_read) writes the zeros.  At 1920x1080 x 8 bricks that is ~8 GB of HBM writes per frame.
__device__ __forceinline__ void finish_ray(const RayOut& o, int nseg, int S, uint8_t* passes, int iter) {
    (void)o;
    (void)nseg;
    (void)S;
    if (passes) *passes = (uint8_t)iter;
}

// NDC z of the ray position at parameter t (VDIGenerator.comp:290, AccumulateVDI.comp:214-217, 247)
__device__ __forceinline__ float ndc_at(const VdiGenParams& P, const f4& wfront, const f4& wback, float t) {
    return persp_div(mat_vec(P.pv, v4mix(wfront, wback, t))).z;
}
// the same from rows 2 and 3 of pv kept in LDS ({m2, m6, m10, m14}, {m3, m7, m11, m15}): the search
// kernel evaluates it only at supersegment boundaries of write passes, and 16 matrix entries held
// in scalar registers through its replay loop would spill them (same operations, same bits)
__device__ __forceinline__ float ndc_at_rows(const float4* rows, const f4& wfront, const f4& wback, float t) {
    const f4 v = v4mix(wfront, wback, t);
    const float4 a = rows[0], b = rows[1];
    const float z = __builtin_fmaf(a.w, v.w, __builtin_fmaf(a.z, v.z, __builtin_fmaf(a.y, v.y, a.x * v.x)));
    const float w = __builtin_fmaf(b.w, v.w, __builtin_fmaf(b.z, v.z, __builtin_fmaf(b.y, v.y, b.x * v.x)));
    return z * (1.0f / w);
}

// One raymarch pass over the brick (VDIGenerator.comp:447-488 with AccumulateVDI.comp spliced in),
// software-pipelined: the voxel loads of sample i+1 are issued before sample i is computed and
// interpolated after it, so only a computed float (the LUT coordinate) is carried to the next step.
// Carrying the loaded voxels instead made the compiler copy registers with loads still pending at
// the loop latch, i.e. wait for vmcnt(0) there -- for every outstanding load and store of the wave.
// The loads are issued for every step (texel_pair clamps each address into the brick), so every
// path has the same memory operations.
// sample_fn(i, coord, colour, w, step, last) runs for every in-brick sample and returns false to
// end the pass early; flush_fn() runs after the next sample's voxels arrived (stores placed there
// are younger than the loads the next step waits for).
template <int DT, class SampleFn, class FlushFn>
__device__ __forceinline__ void march_pass(const VdiGenParams& P, const BrickDesc& brick, const float* s_tf,
                                           const float4* s_cm, const Ray& R, SampleFn sample_fn, FlushFn flush_fn) {
    const float nw = P.nw;
    float step = R.tnear;
    f4 wprev = v4mix(R.wfront, R.wback, step - nw);
    f4 wpos = v4mix(R.wfront, R.wback, step);
    bool in_cur = R.numSteps > 0 && step > R.localNear && step < R.localFar;   // AccumulateVDI.comp:1
    float sc_cur;
    {
        VoxelFetch f;
        fetch_voxels<DT>(brick, wpos, f);
        sc_cur = voxel_coord(brick, f);
    }
    for (int i = 0; i < R.numSteps; ++i) {
        const bool last = (i == R.numSteps - 1);
        const float step_n = step + nw;                        // the loop increment of :447
        const f4 wnext = v4mix(R.wfront, R.wback, step_n);     // next position
        const bool in_nxt = !last && step_n > R.localNear && step_n < R.localFar;
        VoxelFetch nxt;
        fetch_voxels<DT>(brick, wnext, nxt);
        if (in_cur) {
            const f4 x = classify_sample(sc_cur, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
            float w = 0.0f;
            if (x.x > -0.5f || last)
                w = adjust_opacity(x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
            if (!sample_fn(i, sc_cur, x, w, step, last)) break;
        }
        sc_cur = voxel_coord(brick, nxt);
        flush_fn();
        wprev = wpos;
        wpos = wnext;
        step = step_n;
        in_cur = in_nxt;
    }
}
template <int DT, class SampleFn>
__device__ __forceinline__ void march_pass(const VdiGenParams& P, const BrickDesc& brick, const float* s_tf,
                                           const float4* s_cm, const Ray& R, SampleFn sample_fn) {
    march_pass<DT>(P, brick, s_tf, s_cm, R, sample_fn, [] {});
}

// The whole search in place, re-sampling the brick every pass (rays without cache space).
template <int DT>
__device__ void vdi_march(const VdiGenParams& P, const BrickDesc& brick, uint32_t* octree, uint8_t* passes,
                          uint16_t* pending, const float* s_tf, const float4* s_cm, const Ray& R, const RayOut& o) {
    const float nw = P.nw;
    const int S = P.S;
    const int delta = (int)__builtin_floorf(0.15f * (float)S);                      // :386-388
    int nseg = 0;
    Search q{0.0f, 1.732f, 0.0001f, 0, false, false, true};                          // :380-393
    if (R.hit) {
        SegState st;
        auto ndc_of = [&](float t) { return ndc_at(P, R.wfront, R.wback, t); };
        while (!q.found || !q.written) {                                             // :404
            q.iter++;
            if (q.iter > 64) break;
            if (q.found) q.written = true;
            const Thr th{sq_threshold(q.mid), 0.0f, 0.0f};   // exact decisions only
            const bool write = q.found;
            st.reset();
            auto emit = [&](float s0, float e0, const f4& a, int) {
                if (write) {
                    if (nseg < S) store_slot(o, nseg, s0, e0, a);
                    octree_update(P, octree, R.uvx, R.uvy, s0, e0, R.cx, R.cy);
                    nseg++;
                }
            };
            march_pass<DT>(P, brick, s_tf, s_cm, R, [&](int, float, const f4& x, float w, float stp, bool last) {
                seg_sample(st, x, w, stp, ndc_of, last, th, R.wfront, R.wback, nw, P.xfer.cmag, emit);
                // a search pass that has closed more than S supersegments is decided
                // (:511-514 only asks n > S, or n == 0): skip its remaining samples
                return write || st.nterm <= S;
            });
            if (!q.written) search_update(q, st.nterm, S, delta);
        }
    }
    // stored supersegments, octree cells counted inline here
    *pending = (uint16_t)((nseg < S ? nseg : S) | kPendingCounted);
    finish_ray(o, nseg, S, passes, q.iter);
}

// ---- several volumes in one VDI (merge_bricks) --------------------------------------------------
// VDIGenerator.comp renders all the volumes of a rank into ONE sub-VDI: its $repeat block intersects
// every volume (tnear/tfar span all of them, :333-347) and $insert{Accumulate} splices AccumulateVDI
// once per volume into the step loop, so at each step every volume whose (localNear, localFar) holds
// the step feeds its sample, in volume order, into the one supersegment state machine (AV:1).
// These rays run the whole search here, re-sampling the volumes every pass (no sample cache).
struct MultiRay {
    f4 wfront, wback;
    float uvx, uvy, tnear, tfar;
    float ln[kMaxBricks], lf[kMaxBricks];
    uint32_t vis;   // bit v: volume v is hit
    int cx, cy, numSteps;
};

__device__ __forceinline__ MultiRay multi_ray_setup(const VdiGenParams& P, int gx, int gy) {
    MultiRay r;
    Ray d;
    ray_dirs(P, gx, gy, d);
    r.wfront = d.wfront;
    r.wback = d.wback;
    r.uvx = d.uvx;
    r.uvy = d.uvy;
    r.cx = d.cx;
    r.cy = d.cy;
    r.tnear = 1.0f;
    r.tfar = 0.0f;
    r.vis = 0u;
#pragma unroll
    for (int v = 0; v < kMaxBricks; ++v) {
        r.ln[v] = 0.0f;
        r.lf[v] = 0.0f;
        if (v >= P.nvolumes) continue;
        float n, f;
        intersect_bbox(P.bricks[v], r.wfront, r.wback, n, f);
        f = gmin(P.tmax, f);
        if (n < f) {
            r.ln[v] = n;
            r.lf[v] = f;
            r.tnear = gmin(r.tnear, gmax(0.0f, n));
            r.tfar = gmax(r.tfar, f);
            r.vis |= 1u << v;
        }
    }
    r.numSteps = 0;
    if (r.tnear < r.tfar) {
        const float dsteps = __builtin_truncf((r.tfar - r.tnear) / P.nw);   // VDIGenerator.comp:372
        r.numSteps = (dsteps > 2.0e9f) ? 2000000000 : (int)dsteps;
    }
    return r;
}

// The whole search of one merged-volume ray in place, re-sampling the volumes every pass (rays
// without cache space).
template <int DT>
__device__ void merge_search_in_place(const VdiGenParams& P, const float* s_tf, const float4* s_cm, const MultiRay& R,
                                      const RayOut& o, int gx, int gy) {
    const float nw = P.nw;
    const int S = P.S;
    const int delta = (int)__builtin_floorf(0.15f * (float)S);                      // :386-388
    int nseg = 0;
    Search q{0.0f, 1.732f, 0.0001f, 0, false, false, true};                          // :380-393
    auto ndc_of = [&](float t) { return ndc_at(P, R.wfront, R.wback, t); };
    if (R.tnear < R.tfar) {
        SegState st;
        while (!q.found || !q.written) {                                             // :404
            q.iter++;
            if (q.iter > 64) break;
            if (q.found) q.written = true;
            const Thr th{sq_threshold(q.mid), 0.0f, 0.0f};   // exact decisions only
            const bool write = q.found;
            st.reset();
            auto emit = [&](float s0, float e0, const f4& a, int) {
                if (write) {
                    if (nseg < S) store_slot(o, nseg, s0, e0, a);
                    octree_update(P, P.octree, R.uvx, R.uvy, s0, e0, R.cx, R.cy);
                    nseg++;
                }
            };
            float step = R.tnear;
            f4 wprev = v4mix(R.wfront, R.wback, step - nw);
            bool decided = false;
            for (int i = 0; i < R.numSteps && !decided; ++i) {                      // :447
                const bool last = (i == R.numSteps - 1);
                const f4 wpos = v4mix(R.wfront, R.wback, step);
                for (int v = 0; v < P.nvolumes; ++v) {                               // $insert{Accumulate} per volume
                    if (!((R.vis >> v) & 1u) || !(step > R.ln[v] && step < R.lf[v])) continue;   // AV:1
                    const BrickDesc& bk = P.bricks[v];
                    VoxelFetch f;
                    fetch_voxels<DT>(bk, wpos, f);
                    const float sc = voxel_coord(bk, f);
                    const f4 x = classify_sample(sc, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
                    float w = 0.0f;
                    if (x.x > -0.5f || last)
                        w = adjust_opacity(x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
                    seg_sample(st, x, w, step, ndc_of, last, th, R.wfront, R.wback, nw, P.xfer.cmag, emit);
                    // a search pass that has closed more than S supersegments is decided (:511-514)
                    if (!write && st.nterm > S) {
                        decided = true;
                        break;
                    }
                }
                wprev = wpos;                                                        // :487
                step = step + nw;
            }
            if (!q.written) search_update(q, st.nterm, S, delta);
        }
    }
    P.seg_pending[(size_t)gy * (size_t)P.W + (size_t)gx] = (uint16_t)((nseg < S ? nseg : S) | kPendingCounted);
    finish_ray(o, nseg, S, P.passes ? P.passes + (size_t)gy * (size_t)P.W + (size_t)gx : nullptr, q.iter);
}

// One raymarch pass over the merged volumes (VDIGenerator.comp:447-488 with $insert{Accumulate} per
// volume): at every step each volume whose (localNear, localFar) holds the step feeds its sample, in
// volume order (AccumulateVDI.comp:1).  sample_fn(i, coord, colour, w, step, last) runs per sample
// (i = step index) and returns false to end the pass; flush_fn() after each.
template <int DT, class SampleFn, class FlushFn>
__device__ __forceinline__ void march_multi(const VdiGenParams& P, const float* s_tf, const float4* s_cm,
                                            const MultiRay& R, SampleFn sample_fn, FlushFn flush_fn) {
    const float nw = P.nw;
    float step = R.tnear;
    f4 wprev = v4mix(R.wfront, R.wback, step - nw);
    // The volumes holding the step (step > localNear && step < localFar, AccumulateVDI.comp:1) change only
    // where the step passes an interval end: each lane keeps its mask `in` and the next end `bnext`, and
    // re-evaluates both when the step reaches it; the wave walks only the volumes some lane is in (wm),
    // in volume order -- not all of them with a per-volume test at every step.
    uint32_t in = 0u, wm = 0u;
    float bnext = -__builtin_inff();
    for (int i = 0; i < R.numSteps; ++i) {
        const bool last = (i == R.numSteps - 1);
        const f4 wpos = v4mix(R.wfront, R.wback, step);
        if (__ballot(step >= bnext) != 0ull) {   // (wave-uniform) some lane reached an interval end
            if (step >= bnext) {
                in = 0u;
                bnext = __builtin_inff();
#pragma unroll
                for (int v = 0; v < kMaxBricks; ++v) {
                    if (v >= P.nvolumes || !((R.vis >> v) & 1u)) continue;
                    if (step > R.ln[v] && step < R.lf[v]) in |= 1u << v;
                    if (step <= R.ln[v]) bnext = gmin(bnext, R.ln[v]);   // flips at the first step > ln
                    if (step < R.lf[v]) bnext = gmin(bnext, R.lf[v]);    // flips at the first step >= lf
                }
            }
            wm = 0u;
#pragma unroll
            for (int v = 0; v < kMaxBricks; ++v)
                if (__ballot((in >> v) & 1u) != 0ull) wm |= 1u << v;
        }
        for (uint32_t m = wm; m != 0u; m &= m - 1u) {
            const int v = __builtin_ctz(m);   // (wave-uniform)
            if (!((in >> v) & 1u)) continue;
            const BrickDesc& bk = P.bricks[v];
            VoxelFetch f;
            fetch_voxels<DT>(bk, wpos, f);
            const float sc = voxel_coord(bk, f);
            const f4 x = classify_sample(sc, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
            float w = 0.0f;
            if (x.x > -0.5f || last)
                w = adjust_opacity(x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
            const bool go = sample_fn(i, sc, x, w, step, last);
            flush_fn();
            if (!go) return;
        }
        wprev = wpos;
        step = step + nw;
    }
}
#ifndef INSITU_PASS1_PRE
#define INSITU_PASS1_PRE 1    // pass 1 and the spine counts decide with make_thr's thresholds (A/B switch)
#endif
#ifndef INSITU_PASS1_STOP
#define INSITU_PASS1_STOP 1   // pass 1 and the spine counts stop at S + 1 closes (A/B switch)
#endif
#ifndef INSITU_SPEC_LEVELS
#define INSITU_SPEC_LEVELS 4   // search levels pass 1 counts along the "fewer than S - delta" spine (0..5)
#endif
// Stores of chunk c (counted from the ray's first chunk) of one ray: 32 bytes {LUT coordinate x4,
// adjusted opacity x4}.  at(c) is the chunk's address (merged volumes' step indices go beside it).
struct PlainChunkStore {   // the two-kernel generator: the search kernel reads the cache after this launch
    float4* first;         // the ray's first chunk
    __device__ __forceinline__ float4* at(uint32_t c) const { return first + 2 * chunk_off(c); }
    __device__ __forceinline__ void operator()(uint32_t c, const float4& cv, const float4& wv) const {
        float4* e = at(c);
        e[0] = cv;
        e[1] = wv;
    }
};
// Merged volumes: 64-byte chunk slots {coord x4, opacity x4, step indices 4 x u16, 8 B unused}, so the
// search kernel's replay of a chunk reads ONE 128-byte line (with the step indices in a separate array it
// read two: a line for the chunk and one for its 8 bytes of indices).  Slot c of a ray at first + 4*mslot_off(c).
struct MergedChunkStore {
    float4* first;
    __device__ __forceinline__ float4* at(uint32_t c) const { return first + 4 * mslot_off(c); }
    // slots 2 c2 and 2 c2 + 1 of a lane, one 128-byte line, written in one piece (the slots' 24 padding bytes are
    // not written: -0.2 ms of merge kernel against whole-slot stores, round 5)
    __device__ __forceinline__ void pair(uint32_t c2, const float4& ca, const float4& wa, const float4& cb, const float4& wb,
                                         const uint4& s) const {
        float4* e = at(2 * c2);
        e[0] = ca;
        e[1] = wa;
        *reinterpret_cast<uint2*>(e + 2) = make_uint2(s.x, s.y);
        e[4] = cb;
        e[5] = wb;
        *reinterpret_cast<uint2*>(e + 6) = make_uint2(s.z, s.w);
    }
};

// Pass 1 (threshold 1e-4) of a ray with cache space, and the queue record of the rest of its search
// (VDIGenerator.comp:380-539).  march(sample_fn, flush_fn) runs the raymarch pass: march_pass over a
// brick, or march_multi over the volumes of a merged VDI (MERGED: each sample's step index is cached
// too, and a ray with more samples than its cache space (cap_samples) stops: returns false and is
// searched in place).  Returns true with pr filled in.
// p1: the block's pass-1 LDS area (p1_lds_floats): per lane the bounds of the exact decisions of pass 1 and of
// the spine levels (count_sample_l) and the chunk being filled
template <int DT, bool FILTERED, bool MERGED, class March, class Store>
__device__ bool first_pass_impl(const VdiGenParams& P, const f4& wfront, const f4& wback, uint32_t cap_samples,
                                PendingRay& pr, float* p1, March march, Store store_fn) {
    const float nw = P.nw;
    const int S = P.S;
    const Thr th1 = uniform_thr(make_thr(sq_threshold(0.0001f), P.xfer.cmag));        // :393
    const int tid = threadIdx.x;
    float* const bl = p1 + tid;                  // bounds of level l at bl[512 l] (lo), bl[512 l + 256] (hi)
    // the chunk being filled {coord x4, opacity x4}; merged volumes (paired slots, MergedChunkStore): the pair
    // being filled {coord x4, opacity x4} x 2 and its 8 step indices (u16), stored as one 128-byte line
    constexpr bool PAIRS = MERGED;
    float* const chk = p1 + 512 * (INSITU_SPEC_LEVELS + 1) + (PAIRS ? 20 : 8) * tid;
    CountStateL st;   // pass 1 (level 0)
    st.reset();
    // The same pass also counts the supersegments at the thresholds the search tries next: the
    // sampling, classification and opacity of a sample are shared, so the counts cost only the
    // state machines.  They follow the tree's "n < S - delta" spine (high = mid at every level:
    // 0.866, 0.433, 0.217, 0.108 ...), the path every searched ray takes for its first three levels
    // and 84 % of them for four (tools/checkpoint_study.py, brick 7 of the bench): a searching ray
    // enters the search kernel INSITU_SPEC_LEVELS passes further on.
    const float root_mid = (0.0001f + 1.732f) / 2.0f;                                // :519-527
    constexpr int K = INSITU_SPEC_LEVELS;
    CountStateL cs[K > 0 ? K : 1];
    Thr tk[K > 0 ? K : 1];
#pragma unroll
    for (int l = 0, node = 0; l < K; ++l, node = 2 * node + 2) {
        cs[l].reset();
        tk[l] = uniform_thr(make_thr(sq_threshold(tree_threshold(0.0001f, 1.732f, root_mid, node)), P.xfer.cmag));
    }
#pragma unroll
    for (int l = 0; l <= K; ++l) {
        bl[512 * l] = 0.0f;                     // lo (diff^2 >= 0)
        bl[512 * l + 256] = __builtin_inff();   // hi
    }
    // Pass 1 stores nothing: 97 % of the config-2 rays close more than S supersegments at 1e-4 and go
    // on searching (their S speculative stores were 0.8 GB of wasted writes per frame, in the kernel
    // whose memory pipeline is its limit: -1.3 ms); the rest are queued with the threshold found, and
    // the search kernel's write pass replays this pass from the cache (same decisions, same bits)
    bool overflow = false;
    (void)cap_samples;
    int k = 0;
    float step_first = 0.0f;
    bool last_final = false;
    bool store_chunk = false;   // the chunk (in LDS, chk) is stored whole (2 x 16 B) once complete
    march([&](int i, float sc, const f4& x, float w, float stp, bool last) {
        // cache chunk layout: 4 samples per 32 B = {coord x4, opacity x4}
        const int j = k & 3;
        if constexpr (MERGED) {
            if ((uint32_t)k >= cap_samples) {
                overflow = true;
                return false;
            }
        } else {
            (void)i;
        }
        if constexpr (PAIRS) {
            const int pp = k & 7, h = pp >> 2;
            chk[8 * h + j] = sc;
            chk[8 * h + 4 + j] = w;
            reinterpret_cast<uint16_t*>(chk + 16)[pp] = (uint16_t)i;
            store_chunk = pp == 7 || last;
        } else {
            chk[j] = sc;
            chk[4 + j] = w;
            store_chunk = j == 3 || last;   // stored by the flush hook, after the next sample's loads
        }
        if (k == 0) step_first = stp;
        k++;
        last_final = last;
        // decisions filtered like the search passes' (exact only near the threshold); the closing
        // supersegments' colours are deferred (emit).  A pass that has closed more than S
        // supersegments is decided ("n > S", VDIGenerator.comp:511-514): it stops there, as the
        // search kernel's passes do.  Its segmentation interval then bounds the decisions of the
        // samples seen so far, which is all the "n > S" conclusion rests on (every threshold in it
        // closes the same S + 1 supersegments over that prefix).
#ifdef INSITU_ABL_NOPASS1
        if (false)   // ablation (timing only, wrong results): sampling and cache fill without pass 1
#else
        if (!INSITU_PASS1_STOP || st.nterm <= S)
#endif
            count_sample_l<FILTERED, INSITU_PASS1_PRE>(st, bl, x, w, last, th1, wfront, wback, nw, P.xfer.cmag);
#pragma unroll
        for (int l = 0; l < K; ++l)
            if (!INSITU_PASS1_STOP || cs[l].nterm <= S)
                count_sample_l<FILTERED, INSITU_PASS1_PRE>(cs[l], bl + 512 * (l + 1), x, w, last, tk[l], wfront, wback, nw,
                                                          P.xfer.cmag);
        return true;   // the cache needs every sample
    }, [&] {
#ifndef INSITU_ABL_NOSTORE
        if (store_chunk) {
            const float4 bc = *reinterpret_cast<const float4*>(chk), bw = *reinterpret_cast<const float4*>(chk + 4);
            if constexpr (PAIRS) {
                store_fn.pair((uint32_t)(k - 1) >> 3, bc, bw, *reinterpret_cast<const float4*>(chk + 8),
                              *reinterpret_cast<const float4*>(chk + 12), *reinterpret_cast<const uint4*>(chk + 16));
            } else {
                store_fn((uint32_t)(k - 1) >> 2, bc, bw);
            }
        }
#endif
        store_chunk = false;
    });
    if constexpr (MERGED) {
        if (overflow) return false;
    }
    if ((k & (PAIRS ? 7 : 3)) != 0 && !last_final) {   // flush a partial chunk (the ray left the brick early)
        const float4 bc = *reinterpret_cast<const float4*>(chk), bw = *reinterpret_cast<const float4*>(chk + 4);
        if constexpr (PAIRS) {
            store_fn.pair((uint32_t)k >> 3, bc, bw, *reinterpret_cast<const float4*>(chk + 8),
                          *reinterpret_cast<const float4*>(chk + 12), *reinterpret_cast<const uint4*>(chk + 16));
        } else {
            store_fn((uint32_t)k >> 2, bc, bw);
        }
    }
    if (st.nterm <= S) {
        // accepted at 1e-4 (VDIGenerator.comp:497-529 first iteration): queued with the search found
        // after one pass, so only the write pass is left -- a replay of this pass
        pr.seg_low[0] = pr.seg_high[0] = __builtin_inff();
        pr.seg_low[1] = pr.seg_high[1] = -__builtin_inff();
        pr.n_high = 0u;
        pr.n = (uint32_t)k;
        pr.step_first = step_first;
        pr.last_final = last_final ? 1u : 0u;
        pr.low = 0.0f;
        pr.high = 1.732f;
        pr.mid = 0.0001f;
        pr.iter_found = 1u | 0x100u;
        return true;
    }
    // walk the speculated levels while the search stays on the spine (VDIGenerator.comp:497-529;
    // pass 1 closed more than S, so low = 1e-4 with pass 1's segmentation interval): level l+1's
    // threshold is the tree's, i.e. the mid search_update computes after level l went "fewer",
    // then the passes the intervals decide
    const int delta = (int)__builtin_floorf(0.15f * (float)S);
    Search q{0.0001f, 1.732f, root_mid, 1, false, false, false};
    // the segmentation intervals recorded estimates where the filter decided: bounds from them
    float lo[K + 1], hi[K + 1];   // level 0: pass 1
#pragma unroll
    for (int l = 0; l <= K; ++l) {
        lo[l] = bl[512 * l];
        hi[l] = bl[512 * l + 256];
        if constexpr (FILTERED) {
            const CountStateL& c = l == 0 ? st : cs[l > 0 ? l - 1 : 0];
            lo[l] = __builtin_fmaxf(lo[l], seg_lo_bound(c.lo_a, P.xfer.cmag));
            hi[l] = __builtin_fminf(hi[l], seg_hi_bound(c.hi_a, P.xfer.cmag));
        }
    }
    float4 iv{lo[0], hi[0], __builtin_inff(), -__builtin_inff()};
    int n_high = 0;
    bool on_spine = true;
#pragma unroll
    for (int l = 0; l < K; ++l) {
        if (!on_spine || q.found) break;
        q.iter++;
        on_spine = cs[l].nterm < S - delta && !(__builtin_fabsf(q.high - q.low) < 0.000001f);
        search_step(q, cs[l].nterm, S, delta, lo[l + 1], hi[l + 1], iv, n_high);
    }
    free_walk(q, iv, n_high, S, delta);
    pr.seg_low[0] = iv.x;
    pr.seg_low[1] = iv.y;
    pr.seg_high[0] = iv.z;
    pr.seg_high[1] = iv.w;
    pr.n_high = (uint32_t)n_high;
    pr.n = (uint32_t)k;
    pr.step_first = step_first;
    pr.last_final = last_final ? 1u : 0u;
    pr.low = q.low;
    pr.high = q.high;
    pr.mid = q.mid;
    pr.iter_found = (uint32_t)q.iter | (q.found ? 0x100u : 0u);
    return true;
}

// pass 1 of a brick ray (march_pass: software-pipelined voxel loads)
template <int DT, bool FILTERED, class Store>
__device__ __forceinline__ bool vdi_first_pass(const VdiGenParams& P, const BrickDesc& brick, const float* s_tf,
                                               const float4* s_cm, const Ray& R, PendingRay& pr, float* p1, Store store_fn) {
    return first_pass_impl<DT, FILTERED, false>(P, R.wfront, R.wback, 0u, pr, p1, [&](auto sample_fn, auto flush_fn) {
        march_pass<DT>(P, brick, s_tf, s_cm, R, sample_fn, flush_fn);
    }, store_fn);
}

// Merged volumes (merge_bricks): the first pass of every ray over all of the rank's volumes, its
// samples and their step indices cached, the ray queued for vdi_search_kernel<., true> -- the
// sampling/search split of the brick rays.  A ray whose samples outgrow its cache space (estimated
// from its volume intervals) is searched in place by re-sampling, as are rays without cache space.
template <int DT, bool FILTERED>
__global__ __launch_bounds__(256, INSITU_MERGE_MIN_BLOCKS) void vdi_merge_kernel(const VdiGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm));
    stage_luts(P.xfer, s_cm, s_tf);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int tile = xcd_block((int)blockIdx.x, (int)gridDim.x) * 4 + wave;
    if (P.tile_ids) {   // longest tiles first (vdi_tile_len_kernel + sort), as the brick sampling kernel
        const int ntiles = P.ytiles * P.nstrips * P.strip_tiles;
        const int j = xcd_block((int)blockIdx.x, (int)gridDim.x, INSITU_SAMPLE_XCD_CHUNK) * 4 + wave;
        tile = j < ntiles ? (int)P.tile_ids[ntiles + j] : 4 * ntiles;   // sorted half (past the end: invalid)
    }
    const int yt = tile % P.ytiles, ct = tile / P.ytiles;
    const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
    const int xl = xt * 8 + (lane & 7), gy = yt * 8 + (lane >> 3);
    const bool valid = d < P.nstrips && xl < P.strip_w && gy < P.H;
    const int gx = d * P.strip_w + xl;
    MultiRay R{};
    if (valid) R = multi_ray_setup(P, gx, gy);
    const bool hit = valid && R.tnear < R.tfar && R.numSteps > 0;
    // cache space: the samples the volume intervals hold (+2 per volume for rounding at the ends)
    uint32_t cap = 0;
    if (hit && R.numSteps < 65536) {
        for (int v = 0; v < P.nvolumes; ++v) {
            if (!((R.vis >> v) & 1u)) continue;
            const float span = (R.lf[v] - gmax(R.ln[v], R.tnear)) / P.nw;
            cap += (span > 0.0f ? (uint32_t)__builtin_fminf(span, 65536.0f) : 0u) + 2u;
        }
        cap = cap < (uint32_t)R.numSteps * (uint32_t)P.nvolumes ? cap : (uint32_t)R.numSteps * (uint32_t)P.nvolumes;
    }
    float* cache = nullptr;
    uint32_t chunk = 0;
    if (P.cache) {
        // 64-byte slots (MergedChunkStore), i.e. two 32-byte cache units each, lane-interleaved
        const uint32_t need = (cap + 3u) >> 2;
        uint32_t mx = need;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        constexpr uint32_t G = 2;   // (slots in pairs, mslot_off)
        const uint32_t total = (mx + G - 1) / G * G * 128u;   // cache units of the wave's 64 x mx slots
        unsigned long long base = 0;
        if (lane == 63 && total) base = atomicAdd(&P.ctr->cache_cursor, (unsigned long long)total);
        base = __shfl(base, 63);
        if (need && base + total <= (unsigned long long)P.cache_chunks) {
            chunk = (uint32_t)(base + 2ull * G * (unsigned long long)lane);
            cache = P.cache + 8 * (size_t)chunk;
        }
    }
    bool pend = false;
    PendingRay pr{};
    if (valid) {
        const RayOut o = ray_out(P, gx, gy, 0);
        if (cache) {
            pend = first_pass_impl<DT, FILTERED, true>(P, R.wfront, R.wback, cap, pr,
                                                       reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm) +
                                                                                lut_tf_slots(P.xfer.n_tf)),
                                                       [&](auto sample_fn, auto flush_fn) {
                                                           march_multi<DT>(P, s_tf, s_cm, R, sample_fn, flush_fn);
                                                       }, MergedChunkStore{reinterpret_cast<float4*>(cache)});
            pr.pix = (uint32_t)gy * (uint32_t)P.W + (uint32_t)gx;
            pr.b = 0u;
            pr.chunk = chunk;
            pr.nsteps = (uint32_t)R.numSteps;
        }
        if (!pend) {
            if (hit && cache) atomicAdd(&P.ctr->cap_overflow, 1u);   // outgrew its space: (rare) in place
            merge_search_in_place<DT>(P, s_tf, s_cm, R, o, gx, gy);
        }
    }
    {   // rays that hit a volume but got no cache space (a reported statistic)
        const unsigned long long mr = __ballot(hit && !cache);
        if (mr && lane == __builtin_ctzll(mr)) atomicAdd(&P.ctr->march_rays, (uint32_t)__popcll(mr));
    }
    const unsigned long long mp = __ballot(pend);
    uint32_t q0 = 0;
    if (mp && lane == __builtin_ctzll(mp)) q0 = atomicAdd(&P.ctr->queue_count, (uint32_t)__popcll(mp));
    if (mp) q0 = __shfl(q0, __builtin_ctzll(mp));
    if (pend) P.queue[q0 + (uint32_t)__popcll(mp & ((1ull << lane) - 1ull))] = pr;
}

#ifndef INSITU_TILE_CLASS_SHIFT
#define INSITU_TILE_CLASS_SHIFT 4   // length classes of 2^4 = 16 samples (measured 2..8: 3-4 best)
#endif
// The sort key of every (brick, tile) for the longest-tiles-first order: the longest ray of the tile's
// SUPER-TILE (P.super_tile^2 tiles, 1 = the tile itself) in 16-sample classes (high byte), then the
// super-tile's position and the tile's place in it (so a class keeps the spatial order, and the tiles of a
// super-tile stay consecutive in the sorted list: the sampling kernel's XCD chunks hand them to one XCD at
// nearly the same time, so the brick blocks their rays share are read into its L2 once) -- the ray setup of
// vdi_sample_kernel, nothing else.  One wave per tile; a block holds max(4, sup^2) waves, whole super-tiles.
__global__ __launch_bounds__(1024) void vdi_tile_len_kernel(const VdiGenParams P) {
    __shared__ int s_max[4];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int sup = P.super_tile, sup2 = sup * sup;
    const int spb = (int)(blockDim.x >> 6) / sup2;   // super-tiles per block
    const int b = (int)blockIdx.y;
    const int nct = P.nstrips * P.strip_tiles;       // global column tiles
    const int ntiles = P.ytiles * nct;
    const int nsx = (nct + sup - 1) / sup, nsy = (P.ytiles + sup - 1) / sup;
    const int sl = wave / sup2, sub = wave - sl * sup2;
    const int si = (int)blockIdx.x * spb + sl;
    const int sx = si / nsy, sy = si - sx * nsy;
    const int ct = sx * sup + sub / sup, yt = sy * sup + sub % sup;
    const bool tile_ok = si < nsx * nsy && ct < nct && yt < P.ytiles;   // (wave-uniform)
    if (threadIdx.x < 4) s_max[threadIdx.x] = 0;
    __syncthreads();
    int steps = 0;
    if (tile_ok) {
        const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
        const int xl = xt * 8 + (lane & 7), gy = yt * 8 + (lane >> 3);
        if (d < P.nstrips && xl < P.strip_w && gy < P.H) {
            if (P.nvolumes > 0) {   // merged volumes: the ray through all of them (one sub-VDI, b = 0)
                const MultiRay M = multi_ray_setup(P, d * P.strip_w + xl, gy);
                steps = M.tnear < M.tfar ? M.numSteps : 0;
            } else {
                const Ray R = ray_setup(P, P.bricks[b], d * P.strip_w + xl, gy);
                steps = R.hit ? R.numSteps : 0;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) steps = max(steps, __shfl_xor(steps, o));
    if (lane == 0 && steps > 0) atomicMax(&s_max[sl], steps);
    __syncthreads();
    if (lane == 0 && tile_ok) {
        const int tile = ct * P.ytiles + yt;
        // the sampling wave of this tile takes 64 x its longest ray's chunks (vdi_sample_kernel)
        const uint32_t mx = (steps > 0 && steps < 65536) ? ((uint32_t)steps + 3u) >> 2 : 0u;
        if (P.measure_cache && mx) atomicAdd(&P.ctr->cache_need, (unsigned long long)mx * 64ull);
        const uint32_t pos = (uint32_t)b * (uint32_t)ntiles + (uint32_t)tile;
        // < 2^24 (host-checked for sup <= 4); sup = 1: spos = pos
        const uint32_t spos = (((uint32_t)b * (uint32_t)nsx + (uint32_t)sx) * (uint32_t)nsy + (uint32_t)sy) * (uint32_t)sup2 +
                              (uint32_t)sub;
        const uint32_t cls = (uint32_t)min(s_max[sl] >> INSITU_TILE_CLASS_SHIFT, 255);
        P.tile_keys[pos] = (cls << 24) | (0xffffffu - spos);
        P.tile_ids[pos] = pos;
    }
}

// The same keys from 16 of a tile's 64 rays (pixels {0, 2, 5, 7}^2 of the 8x8 tile: the corners and an
// inner grid), 16 tiles per block: a quarter of the ray setups and of the waves.  The key only orders the
// sampling tiles (the results do not depend on it); frames that measure the cache demand use the exact
// kernel above.  Super-tiles of 1 tile only.
__global__ __launch_bounds__(256) void vdi_tile_len_sub_kernel(const VdiGenParams P) {
    const int b = (int)blockIdx.y;
    const int nct = P.nstrips * P.strip_tiles;
    const int ntiles = P.ytiles * nct;
    const int lane = threadIdx.x & 63;
    const int tile = (int)blockIdx.x * 16 + (int)(threadIdx.x >> 4);   // tile = ct * ytiles + yt
    const int s = lane & 15;
    const int pxy[4] = {0, 2, 5, 7};
    int steps = 0;
    if (tile < ntiles) {
        const int yt = tile % P.ytiles, ct = tile / P.ytiles;
        const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
        const int xl = xt * 8 + pxy[s & 3], gy = yt * 8 + pxy[s >> 2];
        if (d < P.nstrips && xl < P.strip_w && gy < P.H) {
            if (P.nvolumes > 0) {
                const MultiRay M = multi_ray_setup(P, d * P.strip_w + xl, gy);
                steps = M.tnear < M.tfar ? M.numSteps : 0;
            } else {
                const Ray R = ray_setup(P, P.bricks[b], d * P.strip_w + xl, gy);
                steps = R.hit ? R.numSteps : 0;
            }
        }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) steps = max(steps, __shfl_xor(steps, o));
    if (s == 0 && tile < ntiles) {
        const uint32_t pos = (uint32_t)b * (uint32_t)ntiles + (uint32_t)tile;
        const uint32_t cls = (uint32_t)min(steps >> INSITU_TILE_CLASS_SHIFT, 255);
        P.tile_keys[pos] = (cls << 24) | (0xffffffu - pos);
        P.tile_ids[pos] = pos;
    }
}

// One 8x8 pixel tile of brick b, one lane per ray: ray setup, cache space, pass 1 + the spine counts
// (vdi_first_pass) or the in-place search of rays without cache space (vdi_march), and the queue
// records of the rays still searching.
template <int DT, bool FILTERED>
__device__ __forceinline__ void sample_tile(const VdiGenParams& P, const float* s_tf, const float4* s_cm, float* p1, int lane,
                                            int b, int tile) {
    const int yt = tile % P.ytiles;
    const int ct = tile / P.ytiles;                   // global column tile
    const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
    const int xx = lane & 7, yy = lane >> 3;
    const int xl = xt * 8 + xx, gy = yt * 8 + yy;
    const bool valid = d < P.nstrips && xl < P.strip_w && gy < P.H;
    const int gx = d * P.strip_w + xl;
    const BrickDesc& brick = P.bricks[b];
    Ray R{};
    if (valid) R = ray_setup(P, brick, gx, gy);

    // cache space for the whole wave: prefix scan of the lanes' chunk counts, one 64-bit
    // atomic per wave (all 64 lanes are active here)
    float* cache = nullptr;
    uint32_t chunk = 0;
    unsigned long long base = 0;
    uint32_t total = 0;
    if (P.cache) {
        // (a cached ray's supersegment step counts fit the 16-bit seg_steps entries)
        const uint32_t need = (valid && R.hit && R.numSteps < 65536) ? ((uint32_t)R.numSteps + 3u) >> 2 : 0u;
        // lane-interleaved (chunk_off): chunk c of lane l at base + c*64 + l, so the 64 lanes storing their chunk c
        // write 2 KiB in one piece (the wave takes 64 x its longest ray's chunks)
        uint32_t mx = need;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        total = mx * 64u;
        if (lane == 63 && total) base = atomicAdd(&P.ctr->cache_cursor, (unsigned long long)total);
        base = __shfl(base, 63);
        if (need && base + total <= (unsigned long long)P.cache_chunks) {
            chunk = (uint32_t)(base + (unsigned long long)lane);
            cache = P.cache + 8 * (size_t)chunk;
        }
    }
    {   // rays that hit the brick but got no cache space: searched by re-sampling (a reported statistic)
        const unsigned long long mr = __ballot(valid && R.hit && R.numSteps > 0 && !cache);
        if (mr && lane == __builtin_ctzll(mr)) atomicAdd(&P.ctr->march_rays, (uint32_t)__popcll(mr));
    }
    bool pend = false;
    PendingRay pr{};
    if (valid) {
        const RayOut o = ray_out(P, gx, gy, b);
        uint32_t* oct = P.octree + (size_t)b * P.octree_stride;
        uint8_t* pas = P.passes ? P.passes + (size_t)b * P.passes_stride + (size_t)gy * (size_t)P.W + (size_t)gx
                                : nullptr;
        uint16_t* pnd = P.seg_pending + (size_t)b * P.passes_stride + (size_t)gy * (size_t)P.W + (size_t)gx;
        if (cache) {
            pend = vdi_first_pass<DT, FILTERED>(P, brick, s_tf, s_cm, R, pr, p1,
                                                PlainChunkStore{reinterpret_cast<float4*>(cache)});
            pr.pix = (uint32_t)gy * (uint32_t)P.W + (uint32_t)gx;
            pr.b = (uint32_t)b;
            pr.chunk = chunk;
        } else {
#ifndef INSITU_ABL_NOMARCH
            vdi_march<DT>(P, brick, oct, pas, pnd, s_tf, s_cm, R, o);
#endif
        }
    }
    // append the unfinished rays to the search queue (one atomic per wave and class): long rays
    // from the front, short ones from the back
    const bool lng = pend && pr.n >= P.long_samples;
    const unsigned long long ml = __ballot(lng), ms = __ballot(pend && !lng);
    uint32_t ql = 0, qs = 0;
    if (ml && lane == __builtin_ctzll(ml)) ql = atomicAdd(&P.ctr->queue_count, (uint32_t)__popcll(ml));
    if (ms && lane == __builtin_ctzll(ms)) qs = atomicAdd(&P.ctr->queue_short, (uint32_t)__popcll(ms));
    if (ml) ql = __shfl(ql, __builtin_ctzll(ml));
    if (ms) qs = __shfl(qs, __builtin_ctzll(ms));
    uint32_t slot = 0;
    if (pend) {
        const unsigned long long below = (1ull << lane) - 1ull;
        slot = lng ? ql + (uint32_t)__popcll(ml & below) : P.queue_cap - 1u - (qs + (uint32_t)__popcll(ms & below));
        P.queue[slot] = pr;
    }
}

template <int DT, bool FILTERED>
__global__ __launch_bounds__(256, INSITU_SAMPLE_MIN_BLOCKS) void vdi_sample_kernel(const VdiGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm));
    stage_luts(P.xfer, s_cm, s_tf);

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // XCD-aware order over all (brick, tile-block) pairs: each XCD walks a contiguous range, i.e.
    // mostly one brick and neighbouring tiles, so its L2 holds the brick region its rays sample
    const int lin = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int logical = xcd_block(lin, (int)(gridDim.x * gridDim.y), INSITU_SAMPLE_XCD_CHUNK);
    int b, tile;
    if (P.tile_ids) {
        // longest tiles first (vdi_tile_len_kernel + sort): the launch ends with short tiles, not
        // with a long one started late.  Within a length class the order is the XCD order above.
        const int ntiles = P.ytiles * P.nstrips * P.strip_tiles;
        const int j = logical * 4 + wave;
        const int total = P.B * ntiles;
        const uint32_t id = P.tile_ids[total + (j < total ? j : total - 1)];   // sorted half
        b = (int)(id / (uint32_t)ntiles);
        tile = j < total ? (int)(id - (uint32_t)b * (uint32_t)ntiles) : 4 * ntiles;   // (past the end: invalid)
    } else {
        b = logical / (int)gridDim.x;
        tile = (logical - b * (int)gridDim.x) * 4 + wave;
    }
    // (wave-uniform: the brick descriptor is then read into scalar registers, not into ~25 VGPRs)
    b = __builtin_amdgcn_readfirstlane(b);
    tile = __builtin_amdgcn_readfirstlane(tile);
    sample_tile<DT, FILTERED>(P, s_tf, s_cm, reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm) + lut_tf_slots(P.xfer.n_tf)),
                              lane, b, tile);
}

// Persistent lanes over the queue: the rest of the threshold search and the write pass, replayed
// from the cache 4 samples (one 32-byte chunk) per loop trip.
//
// When the queue is short (few rays per GPU: the per-GPU work of a multi-GPU run) the frame time is
// the latency of the rays with the most passes, and most of the GPU idles.  Then a GROUP of G lanes
// (G = 2^d - 1) takes one ray and, in one replay round, evaluates the pass counts of all G
// thresholds of the next d levels of the binary search tree; walking the tree with those counts
// lands exactly where d sequential passes would (same thresholds, same decisions), so a ray needs
// ceil(levels / d) rounds instead of one pass per level.  G = 1 is the plain sequential search.
#ifndef INSITU_SPEC_WRITE
#define INSITU_SPEC_WRITE 1   // search passes of a group's root store their supersegments: an accepted pass needs no write pass
#endif
#ifndef INSITU_SPEC_FROM
#define INSITU_SPEC_FROM 8    // ... from this pass number on: later passes are accepted more often (measured 7..9)
#endif
#ifndef INSITU_SPEC_FROM_GROUP
#define INSITU_SPEC_FROM_GROUP 7   // ... with tree groups (short queues: the per-GPU share of many GPUs)
#endif
#ifndef INSITU_SEARCH_MIN_WAVES
#define INSITU_SEARCH_MIN_WAVES 3    // 3 waves per SIMD: <= 168 VGPRs (hang guard)
#endif
constexpr int kMaxSearchDepth = 6;
#ifndef INSITU_REGROUP_MAX_DEPTH
#define INSITU_REGROUP_MAX_DEPTH 4   // deepest tree a regroup forms (15 lanes per ray)
#endif
constexpr int kMaxRegroupDepth = INSITU_REGROUP_MAX_DEPTH;

// the sampling kernels' LDS: the LUTs, then the pass-1 area of first_pass_impl (per lane the exact-decision bounds
// of pass 1 and the spine levels, and the chunk being filled)
constexpr int kP1LdsFloats = 512 * (INSITU_SPEC_LEVELS + 1) + 8 * 256;
__host__ __device__ __forceinline__ size_t sample_lds_bytes(int n_tf, int n_cm) {
    return lut_lds_bytes(n_tf, n_cm) + (size_t)kP1LdsFloats * 4;
}
// vdi_merge_kernel: the same with the pair staging of paired merged slots (20 words per lane)
__host__ __device__ __forceinline__ size_t merge_lds_bytes(int n_tf, int n_cm) {
    return lut_lds_bytes(n_tf, n_cm) + (size_t)(512 * (INSITU_SPEC_LEVELS + 1) + 20 * 256) * 4;
}

__host__ __device__ __forceinline__ size_t search_lds_bytes(int n_tf, int n_cm) {
    // LUTs, then per lane: chunk 0 (2 x float4), pass result, search intervals (float4 each), count;
    // then rows 2 and 3 of pv; then per lane the diagnostics' queue slot (u32) and pop time (u64), and
    // (merged volumes) chunk 0's step indices (uint2)
    return lut_lds_bytes(n_tf, n_cm) + 4 * 256 * 16 + 256 * 4 + 2 * 16 + 256 * 4 + 256 * 8 + 256 * 8;
}

#ifndef INSITU_GROUP_BATCH
#define INSITU_GROUP_BATCH 6   // tree-group mode: lanes that must have ended a round before the round-end code runs (one brick per GPU: 6.71 -> 6.49 ms)
#endif
#ifndef INSITU_SEL_REPLAY
#define INSITU_SEL_REPLAY 1   // the search replay's state updates as selects (seg_sample_sel; A/B switch)
#endif
#ifndef INSITU_SEARCH_PRE
#define INSITU_SEARCH_PRE 1   // search passes decide with make_thr's thresholds (A/B switch)
#endif
#ifndef INSITU_DEEP_WINDOW
#define INSITU_DEEP_WINDOW 3e-3f   // search range (high - low) below which the exact window spans it (measured: 1e-4..1e-1)
#endif
// The decision thresholds of a search pass.  Deep in the search (high - low below
// INSITU_DEEP_WINDOW) every threshold still to come lies in (low, high), a few ulps to a few 1e-4
// apart, while the filtered decisions' bounds are loose by the margin (~1e-5 relative): the
// segmentation interval of a pass then cannot cover the next threshold and free_walk replays passes
// that make the same decisions.  There the exact window spans the whole remaining range: samples
// whose estimate could lie on either side of ANY remaining threshold take the exact path, the
// others are certain for all of them, so the pass's interval is exact across the range.
__device__ __forceinline__ Thr search_thr(float t_sq, float c, const Search& q) {
    if (!INSITU_SEARCH_PRE) return Thr{t_sq, 0.0f, 0.0f};
    Thr r = make_thr(t_sq, c);
    if (!q.found && q.high - q.low < INSITU_DEEP_WINDOW) {
        r.hi = __builtin_fmaxf(r.hi, make_thr(sq_threshold(q.high), c).hi);
        r.lo = __builtin_fminf(r.lo, make_thr(sq_threshold(q.low), c).lo);
    }
    return r;
}

// MERGED: the rays of merged volumes (vdi_merge_kernel), whose samples are the in-interval (step,
// volume) pairs of VDIGenerator.comp's $repeat -- several, one or none per step: each sample's step
// index comes from its chunk's slot (4 per chunk, MergedChunkStore), `last` is its step being the ray's last, and a write
// pass advances the ray parameter step by step to it (the same running sum, the same bits)
template <bool FILTERED, bool MERGED>
__device__ __forceinline__ void search_loop(const VdiGenParams& P, float4* smem) {
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm));
    // chunk 0 of every lane's ray, kept in LDS (structure of arrays: conflict-free 16-byte
    // accesses) so a pass can restart without waiting for memory
    float4* s_c0 = smem + lut_cm_slots(P.xfer.n_cm) + lut_tf_slots(P.xfer.n_tf);   // 16-byte aligned after the TF
    float4* s_w0 = s_c0 + 256;
    // per lane: the result of its last pass {count, segmentation interval lo, hi} (read by its
    // group), and the ray's segmentation intervals (seg_low, seg_high) and count at `high`
    float4* s_res = s_c0 + 512;
    float4* s_iv = s_c0 + 768;
    int* s_nh = reinterpret_cast<int*>(s_c0 + 1024);
    float4* s_pv = s_c0 + 1024 + 64;   // after the 256 ints (rows 2 and 3 of pv, staged by the kernel)
    // diagnostics (P.debug_rays): per lane the ray's queue slot and pop time, kept out of registers
    uint32_t* s_dbg_slot = reinterpret_cast<uint32_t*>(s_c0 + 1024 + 66);
    unsigned long long* s_dbg_t0 = reinterpret_cast<unsigned long long*>(s_c0 + 1024 + 66 + 64);
    // MERGED: the step indices of every lane's chunk 0 (beside s_c0 / s_w0)
    uint2* s_s0 = reinterpret_cast<uint2*>(s_c0 + 1024 + 66 + 64 + 128);
    const int tid = threadIdx.x;
    const int lane = threadIdx.x & 63;
    GenCounters* const ctr = P.ctr;
    // the sampling kernel's queue: long rays from the front, short ones from the back
    const uint32_t qlong = ctr->queue_count;
    const uint32_t qlen = qlong + ctr->queue_short;
    if (qlen == 0u) return;   // block-uniform
    // pipelined frames: as many searching blocks as the queue needs (between one and two per CU); the others
    // leave their wave slots to the next frame's first pass, which runs beside this search (block-uniform)
    unsigned long long lanes = (unsigned long long)P.search_lanes;
    if (P.search_block_rays > 0) {
        uint32_t active = (qlen + (uint32_t)P.search_block_rays - 1u) / (uint32_t)P.search_block_rays;
        active = active < (uint32_t)P.search_min_blocks ? (uint32_t)P.search_min_blocks : active;
        if (blockIdx.x >= active) return;
        const unsigned long long al = (unsigned long long)active * 256ull;
        lanes = al < lanes ? al : lanes;
    }
    // group size from the queue length against the lanes the search grid keeps resident
    int d = 1;
    const unsigned long long cap = lanes * (unsigned long long)P.search_oversub;
    if ((unsigned long long)qlen * 15ull <= cap) d = 4;
    else if ((unsigned long long)qlen * 7ull <= cap) d = 3;
    else if ((unsigned long long)qlen * 3ull <= cap) d = 2;
    if (P.search_depth > 0) d = P.search_depth;   // fixed by the caller (tests), 1..kMaxSearchDepth
    // the group layout: G = 2^d - 1 consecutive lanes per ray; re-formed with deeper trees once the queue
    // is drained (regroup below), so these are wave-uniform variables
    int G = (1 << d) - 1;
    int node = lane % G, gbase = lane - node;
    bool member = lane < (64 / G) * G;
    bool leader_lane = member && node == 0;
    int spec_from = G == 1 ? INSITU_SPEC_FROM : INSITU_SPEC_FROM_GROUP;   // INSITU_SPEC_WRITE
    // the LDS slots of the lane's ray (chunk 0, search intervals, diagnostics): its group leader's at the pop,
    // kept when a regroup moves the ray to other lanes
    int home = tid;

    const int S = P.S;
    const int delta = (int)__builtin_floorf(0.15f * (float)S);
    // the step in a vector register: the kernel's scalar registers are oversubscribed (spilled to VGPR lanes),
    // and a spilled nw cost a v_readlane per replayed sample
    float nw = P.nw;
    asm volatile("" : "+v"(nw));
    bool active = false, drained = false;
    // the ray of the lane: its record is consumed at the pop, only what the replay needs stays live
    uint32_t pix = 0, bslot = 0;     // pixel gy * W + gx, local brick slot
    uint32_t chunk = 0;              // first cache chunk (2 float4 each)
    uint32_t nsteps = 0;             // MERGED: the ray's numSteps
    float step_first = 0.0f;         // ray parameter of the first cached sample
    bool last_final = false;         // the last cached sample is the ray's last sample
    f4 wfront{}, wback{};            // world-space ray (VDIGenerator.comp:289-290)
    size_t e0 = 0;                   // entry of slot 0 of the pixel's output block (ray_out)
    const size_t slot_stride = (size_t)P.H * 8;
    Search q{};                      // root of the group's current round (identical in all its lanes)
    Thr th{};                        // this lane's tree node threshold (or the final one); margin per sample
    SegState st;
    st.reset();
    int nseg = 0, k = 0, n = 0, nchunks = 1, pre_chunk = 0;
    uint32_t cur_step = 0;           // MERGED: the step index stp belongs to
    uint2 s4{}, ps4{};               // MERGED: step indices of the chunk being replayed / the next one
    float stp = 0.0f;                // ray parameter of the sample being replayed (write pass positions)
#ifdef INSITU_DEBUG_REPLAYS
    uint32_t dbg_rounds = 0;         // diagnostics build: rounds (replays) of the ray, recorded with P.debug_rays
#endif
    float4 c4{}, w4{};               // chunk being replayed
    float4 pc4{}, pw4{};             // next chunk, loaded one loop trip ahead
    auto ndc_of = [](float t) { return t; };   // write passes store ray parameters (vdi_finish_kernel)
    // a popped ray: its record, search state and chunk 0 (slot r of the queue)
    auto take = [&](uint32_t r, uint32_t slot) {
        const PendingRay pr = P.queue[slot];
        home = (tid - lane) + gbase;   // (every lane of the group writes the same values there)
        pix = pr.pix;
        bslot = pr.b;
        chunk = pr.chunk;
        nsteps = pr.nsteps;
        step_first = pr.step_first;
        last_final = pr.last_final != 0u;
        const int gy = (int)(pix / (uint32_t)P.W), gx = (int)(pix - (uint32_t)gy * (uint32_t)P.W);
        {
            Ray R;
            ray_dirs(P, gx, gy, R);
            wfront = R.wfront;
            wback = R.wback;
        }
        e0 = (size_t)(ray_out(P, gx, gy, (int)bslot).color - P.color);
        const float4* cbase = reinterpret_cast<const float4*>(P.cache) + 2 * (size_t)chunk;
        n = (int)pr.n;
        nchunks = (n + 3) >> 2;
        // search state after the passes done so far (VDIGenerator.comp:497-529); q.iter
        // counts them
        q = Search{pr.low, pr.high, pr.mid, (int)(pr.iter_found & 0xffu), (pr.iter_found & 0x100u) != 0,
                   false, false};
        q.written = q.found;   // found already: only the write pass is left
        s_iv[home] = make_float4(pr.seg_low[0], pr.seg_low[1], pr.seg_high[0], pr.seg_high[1]);
        s_nh[home] = (int)pr.n_high;
        th = search_thr(sq_threshold(q.found ? q.mid : tree_threshold(q.low, q.high, q.mid, node)), P.xfer.cmag, q);
        st.reset();
        k = 0;
        nseg = 0;
        stp = step_first;
        s_c0[home] = cbase[0];
        s_w0[home] = cbase[1];
        if constexpr (MERGED) s_s0[home] = *reinterpret_cast<const uint2*>(cbase + 2);
        active = true;
        if (P.debug_rays) {
            s_dbg_slot[home] = r;
            s_dbg_t0[home] = wall_clock64();
#ifdef INSITU_DEBUG_REPLAYS
            dbg_rounds = 1;
#endif
        }
    };
    // every wave leaves the loop: when the queue is drained and its lanes are idle, or -- never
    // expected; a guard against a logic error hanging the GPU -- at a wall-clock bound
    // (s_memrealtime, 100 MHz): a frame's search takes tens of ms, so 10 s means a logic error;
    // the wave raises the fault flag and leaves instead of hanging the GPU.  A clock
    // compare rather than a trip counter: the counter's extra live register made the loop spill.
    // (the clock is read every 256 trips, counted in a scalar register: s_memrealtime and its lgkmcnt(0)
    // wait at the top of every trip cost ~40 cycles each)
    const unsigned long long t_end = wall_clock64() + 1000000000ull;
    uint32_t trips = 0u;
    INSITU_T_DECL
    for (;;) {
        INSITU_T_MARK(4)   // (the round-end code, and the checks of trips that continued after the replay)
        if ((++trips & 255u) == 0u && wall_clock64() > t_end) {
            if (lane == 0) atomicOr(&ctr->fault, 1u);
            break;
        }
        const unsigned long long idle = __ballot(!active && leader_lane);
        if (idle != 0ull && !drained) {   // wave-uniform: give every idle group the next ray
            const int first = __builtin_ctzll(idle);
            const uint32_t cnt = (uint32_t)__popcll(idle);
            uint32_t base = 0;
            if (lane == first) base = atomicAdd(&ctr->queue_head, cnt);
            base = __shfl(base, first);
            INSITU_T_MARK(5)   // (the claim: ballot, atomic, broadcast)
            if (base + cnt >= qlen) {
                // pipelined frames: the claim that drains the queue (one wave's) starts the next frame's first pass
                // (the flag's address and value come from the counters, read here only: no live registers)
                if (base < qlen && lane == first) {
                    unsigned long long* const flag = ctr->pipe_flag;
                    if (flag) __hip_atomic_store(flag, ctr->pipe_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                drained = true;
            }
            uint32_t r = base + (uint32_t)__popcll(idle & ((1ull << lane) - 1ull));
            r = __shfl(r, gbase);   // the group's leader holds the group's slot
            if (!active && member && r < qlen) take(r, r < qlong ? r : P.queue_cap - 1u - (r - qlong));   // long rays first
        }
        INSITU_T_MARK(0)
        if (__ballot(active) == 0ull) {
            if (drained) break;
            continue;
        }
        // Regroup: once the queue is drained a wave holds fewer and fewer rays -- the ones that need the
        // most passes -- and its other lanes idle.  When the rays left in the wave fit deeper search trees,
        // every ray waits at the start of its next round until all of them are there, and then the wave's
        // 64 lanes are dealt out again: R rays in groups of 2^d' - 1 consecutive lanes, each ray's state
        // broadcast from its old leader (its LDS slots stay where they are: `home`).  A group of 2^d' - 1
        // lanes evaluates d' levels of the search tree per round (the same thresholds, the same walk), so
        // the rays left take fewer rounds.  wave-uniform: drained, d and G.
        bool hold = false;
        if (P.regroup && drained) {
            const unsigned long long lead = __ballot(active && leader_lane);
            const int R = __popcll(lead);
            int dn = d;
            while (dn < kMaxRegroupDepth && R * ((1 << (dn + 1)) - 1) <= 64) dn++;
            if (dn > d) {
                if (__ballot(active && k != 0) == 0ull) {
                    const int Gn = (1 << dn) - 1;
                    const int g = lane / Gn, nd = lane - g * Gn;
                    unsigned long long m = lead;   // the g-th ray's old leader lane
                    for (int i = 0; i < g && m != 0ull; ++i) m &= m - 1ull;
                    const int src = m != 0ull ? __builtin_ctzll(m) : 0;
                    pix = (uint32_t)__shfl((int)pix, src);
                    bslot = (uint32_t)__shfl((int)bslot, src);
                    chunk = (uint32_t)__shfl((int)chunk, src);
                    nsteps = (uint32_t)__shfl((int)nsteps, src);
                    step_first = __shfl(step_first, src);
                    last_final = __shfl((int)last_final, src) != 0;
                    n = __shfl(n, src);
                    q.low = __shfl(q.low, src);
                    q.high = __shfl(q.high, src);
                    q.mid = __shfl(q.mid, src);
                    q.iter = __shfl(q.iter, src);
                    q.found = __shfl((int)q.found, src) != 0;
                    q.written = __shfl((int)q.written, src) != 0;
                    home = __shfl(home, src);
                    wfront = f4{__shfl(wfront.x, src), __shfl(wfront.y, src), __shfl(wfront.z, src), __shfl(wfront.w, src)};
                    wback = f4{__shfl(wback.x, src), __shfl(wback.y, src), __shfl(wback.z, src), __shfl(wback.w, src)};
                    e0 = (size_t)(uint32_t)__shfl((int)(uint32_t)e0, src) |
                         ((size_t)(uint32_t)__shfl((int)(uint32_t)(e0 >> 32), src) << 32);
#ifdef INSITU_DEBUG_REPLAYS
                    dbg_rounds = (uint32_t)__shfl((int)dbg_rounds, src);
#endif
                    if (lane == 0) atomicAdd(&ctr->regroups, 1u);
                    d = dn;
                    G = Gn;
                    node = nd;
                    gbase = g * Gn;
                    member = g < R;
                    leader_lane = member && nd == 0;
                    spec_from = INSITU_SPEC_FROM_GROUP;
                    active = member;
                    nchunks = (n + 3) >> 2;
                    if (active) {   // the ray's next round (k = 0, as at the round end that led here)
                        th = search_thr(sq_threshold(q.found ? q.mid : tree_threshold(q.low, q.high, q.mid, node)),
                                        P.xfer.cmag, q);
                        st.reset();
                        k = 0;
                        nseg = 0;
                        stp = step_first;
                    }
                } else {
                    hold = active && k == 0;   // (wait at the round start for the others)
                }
            }
        }
        INSITU_T_MARK(1)
        INSITU_DIAG_COUNT(2, active && k < n && !hold);   // [2] replaying lanes, [6] wave trips
        if (active && k < n && !hold) {
            // chunk 0 comes from LDS when a pass starts, every later chunk was loaded one trip ahead
            if (k == 0) {
                c4 = s_c0[home];
                w4 = s_w0[home];
                pre_chunk = 0;
                if constexpr (MERGED) {
                    s4 = s_s0[home];
                    cur_step = s4.x & 0xffffu;   // the first sample's step: stp = step_first there
                }
            } else {
                c4 = pc4;
                w4 = pw4;
                if constexpr (MERGED) s4 = ps4;
            }
            pre_chunk++;
            if (pre_chunk < nchunks) {
                // (merged volumes: 64-byte slots, MergedChunkStore)
                const float4* nx = reinterpret_cast<const float4*>(P.cache) + 2 * (size_t)chunk +
                                   (MERGED ? 4 * mslot_off((uint32_t)pre_chunk) : 2 * chunk_off((uint32_t)pre_chunk));
                pc4 = nx[0];
                pw4 = nx[1];
                if constexpr (MERGED) ps4 = *reinterpret_cast<const uint2*>(nx + 2);
            }
            // transfer function + colour map of the 4 samples: independent of the segment state, so
            // evaluated up front (samples past the ray's end classify junk that is never used)
            const f4 x0 = classify_sample(c4.x, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
            const f4 x1 = classify_sample(c4.y, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
            const f4 x2 = classify_sample(c4.z, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
#ifdef INSITU_ABL_CLASSIFY2
            // timing ablation: a second classification of the 4 samples folded in with weight 0.
            // 1: the same coordinates (bank conflicts as the real lookups); 2: one coordinate for
            // the whole wave (broadcast reads: no conflicts); 3: the VALU work only (no LDS reads)
            f4 x3 = classify_sample(c4.w, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
            {
                const float zz = g_abl_zero;
#if INSITU_ABL_CLASSIFY2 == 2
                const float u = zz + 0.3f;
#define INSITU_ABL_C(v) classify_sample(u + (v) * zz, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm)
#elif INSITU_ABL_CLASSIFY2 == 3
#define INSITU_ABL_C(v) classify_fake((v) + zz, P.xfer.n_tf, P.xfer.n_cm)
#else
#define INSITU_ABL_C(v) classify_sample((v) + zz, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm)
#endif
                const f4 y0 = INSITU_ABL_C(c4.x);
                const f4 y1 = INSITU_ABL_C(c4.y);
                const f4 y2 = INSITU_ABL_C(c4.z);
                const f4 y3 = INSITU_ABL_C(c4.w);
#undef INSITU_ABL_C
                x3.x = __builtin_fmaf((y0.x + y0.y) + (y0.z + y0.w) + (y1.x + y1.y) + (y1.z + y1.w) + (y2.x + y2.y) +
                                          (y2.z + y2.w) + (y3.x + y3.y) + (y3.z + y3.w), zz, x3.x);
            }
#else
            const f4 x3 = classify_sample(c4.w, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
#endif
            const bool write = q.written && node == 0;
            // INSITU_SPEC_WRITE: the root's search passes store too (into the ray's own slots, which the
            // accepted pass or the write pass overwrites; readers stop at the final count)
            const bool store = (q.written || (INSITU_SPEC_WRITE && q.iter + 1 >= spec_from)) && node == 0;
            auto emit = [&](float s0, float e1, const f4& cv, int steps) {
                INSITU_DIAG_COUNT(4, store);   // [8] storing lanes per closing block, [12] such blocks
                if (store) {
                    // stored supersegments: raw curV + step count, adjusted colour and octree cells
                    // done afterwards (vdi_finish_kernel); the ones past S are not stored, their
                    // cells are counted here (:132-180)
                    if (nseg < S) {
                        const size_t e = e0 + (size_t)nseg * slot_stride;
                        P.color[e] = make_float4(cv.x, cv.y, cv.z, cv.w);
                        P.depth[e] = make_float2(s0, e1);
                        P.seg_steps[e] = (uint16_t)steps;
                    } else if (write) {   // (s0, e1: ray parameters, as stored)
                        const int gy = (int)(pix / (uint32_t)P.W), gx = (int)(pix - (uint32_t)gy * (uint32_t)P.W);
                        Ray R;
                        ray_dirs(P, gx, gy, R);
                        octree_update(P, P.octree + (size_t)bslot * P.octree_stride, R.uvx, R.uvy,
                                      ndc_at_rows(s_pv, wfront, wback, s0), ndc_at_rows(s_pv, wfront, wback, e1), R.cx,
                                      R.cy);
                    }
                    nseg++;
                }
            };
            // a search pass that has closed more than S supersegments is decided (the walk only asks
            // n > S, n < S - delta or n == 0): the lane skips the rest of it (k = n)
#if INSITU_SEL_REPLAY
            if constexpr (FILTERED && INSITU_SPEC_WRITE) {
                // the select form: no branch per sample (seg_sample_sel); a lane past its pass's end changes nothing
                // (merged volumes: a storing lane advances the ray parameter to the sample's step first)
#define INSITU_REPLAY_SEL(XV, WV, SI)                                                                          \
    {                                                                                                          \
        const bool on = k < n;                                                                                 \
        bool last;                                                                                             \
        if constexpr (MERGED) {                                                                                \
            const uint32_t si = (SI);                                                                          \
            last = si + 1u == nsteps;                                                                          \
            if (store && on)                                                                                   \
                while (cur_step < si) {   /* VDIGenerator.comp:447's running sum, step by step */              \
                    stp = stp + nw;                                                                            \
                    cur_step++;                                                                                \
                }                                                                                              \
        } else {                                                                                               \
            last = last_final && k == n - 1;                                                                   \
        }                                                                                                      \
        seg_sample_sel<INSITU_SEARCH_PRE>(st, (XV), (WV), stp, on, last, th, wfront, wback, nw, P.xfer.cmag, emit, store); \
        if constexpr (!MERGED) stp = stp + nw;                                                                 \
        k = on ? ((!q.written && st.nterm > S) ? n : k + 1) : k;                                               \
    }
                INSITU_REPLAY_SEL(x0, w4.x, s4.x & 0xffffu)
                INSITU_REPLAY_SEL(x1, w4.y, s4.x >> 16)
                INSITU_REPLAY_SEL(x2, w4.z, s4.y & 0xffffu)
                INSITU_REPLAY_SEL(x3, w4.w, s4.y >> 16)
#undef INSITU_REPLAY_SEL
            } else
#endif
            {
#define INSITU_REPLAY(XV, WV, SI)                                                                              \
    if (k < n) {                                                                                               \
        bool last;                                                                                             \
        if constexpr (MERGED) {                                                                                \
            const uint32_t si = (SI);                                                                          \
            last = si + 1u == nsteps;                                                                       \
            if (store)                                                                                         \
                while (cur_step < si) {   /* VDIGenerator.comp:447's running sum, step by step */              \
                    stp = stp + nw;                                                                            \
                    cur_step++;                                                                                \
                }                                                                                              \
        } else {                                                                                               \
            last = last_final && k == n - 1;                                                                \
        }                                                                                                      \
        seg_sample<FILTERED, INSITU_SPEC_WRITE ? 1 : 2, true, INSITU_SEARCH_PRE>(st, (XV), (WV), stp, ndc_of, last, th, wfront, \
                                      wback, nw, P.xfer.cmag, emit, store);                                    \
        if constexpr (!MERGED) stp = stp + nw;                                                                 \
        k = (!q.written && st.nterm > S) ? n : k + 1;                                                          \
    }
            INSITU_REPLAY(x0, w4.x, s4.x & 0xffffu)
            INSITU_REPLAY(x1, w4.y, s4.x >> 16)
            INSITU_REPLAY(x2, w4.z, s4.y & 0xffffu)
            INSITU_REPLAY(x3, w4.w, s4.y >> 16)
#undef INSITU_REPLAY
            }
        }
        INSITU_T_MARK(2)
        // end of a round once every lane of the group has finished its pass
        const unsigned long long fin = __ballot(active && k >= n);
        const unsigned long long gmask = ((1ull << G) - 1ull) << gbase;   // G <= 63
        const bool round_end = active && (fin & gmask) == gmask;
        const unsigned long long re = __ballot(round_end);
        if (re == 0ull) continue;
        // the end-of-round code runs with only the finishing lanes active: batch it
        if (__popcll(re) < (G == 1 ? P.round_batch : INSITU_GROUP_BATCH) && __ballot(active && k < n && !hold) != 0ull) continue;
        INSITU_T_MARK(3)
        INSITU_DIAG_COUNT(3, round_end);         // [3] lanes ending a round, [7] wave round-end blocks
        // publish the pass results of the group's tree nodes (lanes gbase .. gbase+G-1); the lanes
        // of one wave read each other's entries in order, no block barrier needed
        if (round_end) {
            float lo = INSITU_SPEC_WRITE ? st.lo : st.startPt, hi = INSITU_SPEC_WRITE ? st.hi : st.endPt;
            if constexpr (FILTERED && INSITU_SEARCH_PRE) {   // bounds from the recorded extreme estimates
                lo = __builtin_fmaxf(lo, seg_lo_bound(st.lo_a, P.xfer.cmag));
                hi = __builtin_fminf(hi, seg_hi_bound(st.hi_a, P.xfer.cmag));
            }
            s_res[tid] = make_float4(__int_as_float(st.nterm), lo, hi, 0.0f);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        INSITU_T_MARK(3)   // (the round-end checks and the publication of the pass results)
        if (round_end) {
            bool done = q.written;
            if (done) {
                q.iter++;   // the write pass
            } else {
                // walk the tree: the decisions of up to d sequential passes (VDIGenerator.comp:497-529),
                // then the passes the segmentation intervals decide (every lane of the group walks)
                float4 iv = s_iv[home];
                int n_high = s_nh[home];
                int at = 0;
                bool stored = false;   // INSITU_SPEC_WRITE: accepted at the root's threshold, whose pass stored
                for (int lvl = 0; lvl < d; ++lvl) {
                    const float4 res = s_res[tid - node + at];   // lane gbase + at of this wave
                    const int cnt_here = __float_as_int(res.x);
                    q.iter++;
                    const bool more = cnt_here > S;
                    const bool narrow = __builtin_fabsf(q.high - q.low) < 0.000001f;   // found there moves mid
                    search_step(q, cnt_here, S, delta, res.y, res.z, iv, n_high);
                    stored = INSITU_SPEC_WRITE && lvl == 0 && q.found && !narrow && q.iter >= spec_from;
                    if (q.found || q.iter >= 64) break;
                    at = more ? 2 * at + 1 : 2 * at + 2;
                }
                if (q.iter < 64) free_walk(q, iv, n_high, S, delta);
                s_iv[home] = iv;
                s_nh[home] = n_high;
                INSITU_T_MARK(6)   // (the tree walk and the free walk)
                if (q.iter + 1 > 64) {   // :405 -- the next pass would exceed the reference's cap
                    q.iter++;
                    nseg = 0;            // (nothing written: a speculative pass's stores are not the output)
                    done = true;
                } else if (stored) {     // the write pass is the pass just done (same threshold, same bits)
                    q.iter++;
                    done = true;
                } else {
                    if (q.found) q.written = true;
                    th = search_thr(sq_threshold(q.found ? q.mid : tree_threshold(q.low, q.high, q.mid, node)), P.xfer.cmag, q);
                    st.reset();
                    k = 0;
                    nseg = 0;
                    stp = step_first;
#ifdef INSITU_DEBUG_REPLAYS
                    dbg_rounds++;
#endif
                }
            }
            if (done) {
                if (node == 0) {
                    if (P.passes) P.passes[(size_t)bslot * P.passes_stride + pix] = (uint8_t)q.iter;   // finish_ray
                    P.seg_pending[(size_t)bslot * P.passes_stride + pix] = (uint16_t)((nseg < S ? nseg : S) | kPendingDeferred);
                }
                active = false;
            }
        }
        if (round_end && !active && P.debug_rays && node == 0) {
            unsigned long long* e = P.debug_rays + 4 * (size_t)s_dbg_slot[home];
            e[0] = s_dbg_t0[home];
            e[1] = wall_clock64();
            e[2] = (unsigned long long)q.iter | ((unsigned long long)n << 8) | ((unsigned long long)G << 24);
#ifdef INSITU_DEBUG_REPLAYS
            e[2] |= (unsigned long long)dbg_rounds << 32;
#endif
            e[3] = pix | ((unsigned long long)bslot << 32);
        }
    }
    INSITU_T_FLUSH()
}

// rows 2 and 3 of pv in LDS after the search loop's per-lane arrays (ndc_at_rows)
__device__ __forceinline__ void stage_pv_rows(const VdiGenParams& P, float4* smem) {
    float4* s_pv = smem + lut_cm_slots(P.xfer.n_cm) + lut_tf_slots(P.xfer.n_tf) + 1024 + 64;
    if (threadIdx.x == 0) {
        s_pv[0] = make_float4(P.pv[2], P.pv[6], P.pv[10], P.pv[14]);
        s_pv[1] = make_float4(P.pv[3], P.pv[7], P.pv[11], P.pv[15]);
    }
    __syncthreads();
}

template <bool FILTERED, bool MERGED>
__global__ __launch_bounds__(256, INSITU_SEARCH_MIN_WAVES) void vdi_search_kernel(const VdiGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    stage_luts(P.xfer, smem, reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm)));
    stage_pv_rows(P, smem);
    search_loop<FILTERED, MERGED>(P, smem);
}

// The stored supersegments the generator left pending: their octree cell counts
// (AccumulateVDI.comp:143-177) and, for the search kernel's rays, their adjusted colours
// (AccumulateVDI.comp:50-54, from the raw curV and step count stored in the slot).  One lane per
// pixel, one wave per 8x8 tile of one brick.  Counting is order-independent and the colour is the
// same function of the same operands, so the results are identical to doing both inline; done
// here, the work runs with the lanes of a tile together instead of with the one lane closing a
// supersegment in the middle of a replay.
// The 64 pixels of a tile normally share one grid cell (8x8 pixels per cell, DistributedVolumes.kt:342),
// so their counts meet in a per-wave LDS histogram over the S z intervals and reach HBM as at most
// S atomics per tile instead of one contended atomic per (supersegment, interval).
__global__ __launch_bounds__(256, INSITU_FINISH_MIN_BLOCKS) void vdi_finish_kernel(const VdiGenParams P) {
    extern __shared__ uint32_t s_hist[];   // S counters per wave
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* hist = s_hist + wave * P.S;
    for (int j = lane; j < P.S; j += 64) hist[j] = 0u;
    const int b = (int)blockIdx.y;
    const int tile = (int)blockIdx.x * 4 + wave;
    const int yt = tile % P.ytiles, ct = tile / P.ytiles;
    const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
    const int xl = xt * 8 + (lane & 7), gy = yt * 8 + (lane >> 3);
    const bool valid = d < P.nstrips && xl < P.strip_w && gy < P.H;
    const int gx = d * P.strip_w + xl;
    const uint32_t pend = valid ? P.seg_pending[(size_t)b * P.passes_stride + (size_t)gy * (size_t)P.W + (size_t)gx] : 0u;
    const bool deferred = (pend & kPendingDeferred) != 0u;
    const bool count_cells = (pend & kPendingCounted) == 0u;   // vdi_march counted its cells inline
    const int cnt = (deferred || count_cells) ? (int)(pend & kPendingCount) : 0;
    const unsigned long long act = __ballot(cnt > 0);
    if (act == 0ull) return;   // wave-uniform
    Ray R{};
    ray_dirs(P, gx, gy, R);
    const bool in_grid = R.cx >= 0 && R.cx < P.ncx && R.cy >= 0 && R.cy < P.ncy;
    const int cell = R.cy * P.ncx + R.cx;
    const int first = __builtin_ctzll(act);
    const int cell0 = __shfl(cell, first);
    const bool uniform = __ballot(cnt > 0 && (cell != cell0 || !in_grid)) == 0ull;
    uint32_t* oct = P.octree + (size_t)b * P.octree_stride;
    __builtin_amdgcn_wave_barrier();
    if (cnt > 0) {
        const RayOut o = ray_out(P, gx, gy, b);
        const size_t e0 = (size_t)(o.color - P.color);
        // supersegments in batches of 4: the loads of a batch are issued together, so a pixel waits
        // for memory once per batch rather than once per supersegment (slots past cnt are not read)
        for (int i0 = 0; i0 < cnt; i0 += 4) {
            float2 se[4];
            float4 cv[4];
            uint16_t st[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int i = i0 + u < cnt ? i0 + u : cnt - 1;   // (a repeated slot is read, not used)
                const size_t e = e0 + (size_t)i * o.slot_stride;
                se[u] = P.depth[e];
                if (deferred) {
                    cv[u] = P.color[e];
                    st[u] = P.seg_steps[e];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i0 + u >= cnt) break;
                const size_t e = e0 + (size_t)(i0 + u) * o.slot_stride;
                float2 d = se[u];
                if (deferred) {
                    // the generator stored the ray parameters of the boundaries: their NDC z
                    // (AccumulateVDI.comp:214-217 at the opening sample, :243-248 one step past the
                    // last non-transparent one), and raw colours: adjusted here (:50-54)
                    d = make_float2(ndc_at(P, R.wfront, R.wback, d.x), ndc_at(P, R.wfront, R.wback, d.y));
                    P.depth[e] = d;
                    const f4 a = exact_adjusted(f4{cv[u].x, cv[u].y, cv[u].z, cv[u].w}, (int)st[u], R.wfront, R.wback, P.nw);
                    P.color[e] = make_float4(a.x, a.y, a.z, a.w);
                }
                if (count_cells && uniform) {
                    int sc, ec;
                    octree_range(P, R.uvx, R.uvy, d.x, d.y, sc, ec);
                    for (int j = sc; j <= ec && j < P.S; ++j) atomicAdd(&hist[j], 1u);
                } else if (count_cells) {
                    octree_update(P, oct, R.uvx, R.uvy, d.x, d.y, R.cx, R.cy);
                }
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (uniform) {
        for (int j = lane; j < P.S; j += 64) {
            const uint32_t v = hist[j];
            if (v) atomicAdd(&oct[(uint32_t)j * (uint32_t)(P.ncx * P.ncy) + (uint32_t)cell0], v);
        }
    }
}

hipError_t launch_vdi_finish(const VdiGenParams& p, hipStream_t s) {
    if (!p.seg_pending || !p.seg_steps) return hipErrorInvalidValue;
    const int tiles = p.ytiles * p.nstrips * p.strip_tiles;
    hipLaunchKernelGGL(vdi_finish_kernel, dim3((tiles + 3) / 4, p.B), dim3(256), 4 * sizeof(uint32_t) * p.S, s, p);
    return hipGetLastError();
}

size_t vdi_generator_lds_bytes(int n_tf, int n_cm) {
    const size_t a = sample_lds_bytes(n_tf, n_cm), b = merge_lds_bytes(n_tf, n_cm), c = search_lds_bytes(n_tf, n_cm);
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

hipError_t vdi_search_resident_lanes(int n_tf, int n_cm, int device, int* lanes) {
    // every instantiation the renders launch with search_lanes (filtered / exact, brick / merged rays): the
    // fewest blocks any of them keeps resident, so the group sizes never assume lanes a launch does not get
    int blocks_per_cu = 1 << 30, cus = 0;
    hipError_t e = hipSuccess;
    const size_t lds = search_lds_bytes(n_tf, n_cm);
    for (const void* k : {reinterpret_cast<const void*>(vdi_search_kernel<true, false>),
                          reinterpret_cast<const void*>(vdi_search_kernel<false, false>),
                          reinterpret_cast<const void*>(vdi_search_kernel<true, true>),
                          reinterpret_cast<const void*>(vdi_search_kernel<false, true>)}) {
        int n = 0;
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, lds);
        if (e != hipSuccess) return e;
        blocks_per_cu = n < blocks_per_cu ? n : blocks_per_cu;
    }
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return e;
    *lanes = blocks_per_cu * cus * 256;
    return hipSuccess;
}

hipError_t launch_vdi_prepare(const VdiGenParams& p, hipStream_t s) {
    const int tiles = p.ytiles * p.nstrips * p.strip_tiles;
    hipError_t e = hipMemsetAsync(p.ctr, 0, sizeof(GenCounters), s);
    if (e == hipSuccess && p.pipe_flag) {   // the search's drain trigger (GenCounters::pipe_flag)
        e = hipStreamWriteValue64(s, &p.ctr->pipe_flag, (uint64_t)(uintptr_t)p.pipe_flag, 0);
        if (e == hipSuccess) e = hipStreamWriteValue64(s, &p.ctr->pipe_seq, p.pipe_seq, 0);
    }
    if (e != hipSuccess || !p.tile_ids) return e;
    // longest tiles first: keys (and the frame's cache demand), one sort
    const int n = p.B * tiles;
    const int sup = p.super_tile, sup2 = sup * sup;
    if (sup != 1 && sup != 2 && sup != 4) return hipErrorInvalidValue;
    const int nsuper = ((p.nstrips * p.strip_tiles + sup - 1) / sup) * ((p.ytiles + sup - 1) / sup);
    const int wpb = sup2 > 4 ? sup2 : 4;   // waves per block: whole super-tiles
    const int spb = wpb / sup2;
    if (sup == 1 && !p.measure_cache && !p.tile_len_exact)
        hipLaunchKernelGGL(vdi_tile_len_sub_kernel, dim3((tiles + 15) / 16, p.B), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL(vdi_tile_len_kernel, dim3((nsuper + spb - 1) / spb, p.B), dim3(64 * wpb), 0, s, p);
    size_t tb = p.sort_tmp_bytes;
    return sort_tiles_desc(p.sort_tmp, tb, p.tile_keys, p.tile_keys + n, p.tile_ids, p.tile_ids + n, n, s);
}

// the first half of a render: tile keys and sort (unless p.prepared), then the sampling kernel (or, merged
// volumes, the merge kernel) over every local brick; p.split_event is recorded after it
hipError_t launch_vdi_sample(const VdiGenParams& p, hipStream_t s) {
    const int tiles = p.ytiles * p.nstrips * p.strip_tiles;
    const dim3 grid((tiles + 3) / 4, p.B);
    const size_t lds = sample_lds_bytes(p.xfer.n_tf, p.xfer.n_cm);
    if (p.B < 1 || p.B > kMaxBricks || !p.seg_pending || !p.seg_steps || !p.ctr) return hipErrorInvalidValue;
    for (int b = 1; b < p.B; ++b)   // one voxel type per launch (the kernel is templated on it)
        if (p.bricks[b].dtype != p.bricks[0].dtype) return hipErrorInvalidValue;
    if (p.cache) {
        if (!p.queue || p.search_lanes <= 0 || p.search_depth < 0 || p.search_depth > kMaxSearchDepth)
            return hipErrorInvalidValue;
    }
    hipError_t e = hipSuccess;
    if (!p.prepared) {
        e = launch_vdi_prepare(p, s);
        if (e != hipSuccess) return e;
    }
    const bool f = !p.exact_search;
    if (p.nvolumes > 0) {   // several volumes, one VDI (one output block per strip, B == 1)
        if (p.B != 1 || p.nvolumes > kMaxBricks) return hipErrorInvalidValue;
        for (int b = 1; b < p.nvolumes; ++b)
            if (p.bricks[b].dtype != p.bricks[0].dtype) return hipErrorInvalidValue;
        const dim3 mgrid((tiles + 3) / 4);
        const size_t lds_merge = merge_lds_bytes(p.xfer.n_tf, p.xfer.n_cm);
        switch (p.bricks[0].dtype) {
        case VOX_U8:
            if (f) hipLaunchKernelGGL((vdi_merge_kernel<VOX_U8, true>), mgrid, dim3(256), lds_merge, s, p);
            else hipLaunchKernelGGL((vdi_merge_kernel<VOX_U8, false>), mgrid, dim3(256), lds_merge, s, p);
            break;
        case VOX_U16:
            if (f) hipLaunchKernelGGL((vdi_merge_kernel<VOX_U16, true>), mgrid, dim3(256), lds_merge, s, p);
            else hipLaunchKernelGGL((vdi_merge_kernel<VOX_U16, false>), mgrid, dim3(256), lds_merge, s, p);
            break;
        case VOX_F32:
            if (f) hipLaunchKernelGGL((vdi_merge_kernel<VOX_F32, true>), mgrid, dim3(256), lds_merge, s, p);
            else hipLaunchKernelGGL((vdi_merge_kernel<VOX_F32, false>), mgrid, dim3(256), lds_merge, s, p);
            break;
        default: return hipErrorInvalidValue;
        }
    } else {
        dim3 sgrid = grid;
        if (p.tile_ids) sgrid = dim3((p.B * tiles + 3) / 4, 1);   // a 1-D grid over the sorted list
        switch (p.bricks[0].dtype) {
        case VOX_U8:
            if (f) hipLaunchKernelGGL((vdi_sample_kernel<VOX_U8, true>), sgrid, dim3(256), lds, s, p);
            else hipLaunchKernelGGL((vdi_sample_kernel<VOX_U8, false>), sgrid, dim3(256), lds, s, p);
            break;
        case VOX_U16:
            if (f) hipLaunchKernelGGL((vdi_sample_kernel<VOX_U16, true>), sgrid, dim3(256), lds, s, p);
            else hipLaunchKernelGGL((vdi_sample_kernel<VOX_U16, false>), sgrid, dim3(256), lds, s, p);
            break;
        case VOX_F32:
            if (f) hipLaunchKernelGGL((vdi_sample_kernel<VOX_F32, true>), sgrid, dim3(256), lds, s, p);
            else hipLaunchKernelGGL((vdi_sample_kernel<VOX_F32, false>), sgrid, dim3(256), lds, s, p);
            break;
        default: return hipErrorInvalidValue;
        }
    }
    e = hipGetLastError();
    if (e == hipSuccess && p.split_event) e = hipEventRecord(p.split_event, s);
    return e;
}

// the second half: the persistent threshold search over the rays the first pass queued (no-op without a cache)
hipError_t launch_vdi_search(const VdiGenParams& p, hipStream_t s) {
    if (!p.cache) return hipSuccess;
    const bool f = !p.exact_search;
    const size_t lds_search = search_lds_bytes(p.xfer.n_tf, p.xfer.n_cm);
    if (p.nvolumes > 0) {
        if (f) hipLaunchKernelGGL((vdi_search_kernel<true, true>), dim3(p.search_blocks), dim3(256), lds_search, s, p);
        else hipLaunchKernelGGL((vdi_search_kernel<false, true>), dim3(p.search_blocks), dim3(256), lds_search, s, p);
        return hipGetLastError();
    }
    if (f) hipLaunchKernelGGL((vdi_search_kernel<true, false>), dim3(p.search_blocks), dim3(256), lds_search, s, p);
    else hipLaunchKernelGGL((vdi_search_kernel<false, false>), dim3(p.search_blocks), dim3(256), lds_search, s, p);
#ifdef INSITU_DIAG_TIME
    {
        unsigned long long h[8] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dtime), sizeof h);
        const unsigned long long z[8] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dtime), z, sizeof z);
        const double tot = (double)(h[0] + h[1] + h[2] + h[3] + h[4]);
        const double tot8 = tot + (double)(h[5] + h[6]);
        std::fprintf(stderr, "[dtime] search wave cycles %.4g: claim %.3f take %.3f regroup %.3f replay %.3f checks+publish %.3f walk %.3f thr+done %.3f\n",
                     tot8, h[5] / tot8, h[0] / tot8, h[1] / tot8, h[2] / tot8, h[3] / tot8, h[6] / tot8, h[4] / tot8);
    }
#endif
#ifdef INSITU_DIAG
    {
        unsigned long long h[16] = {};
        (void)hipStreamSynchronize(s);
        (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(g_diag), sizeof h);
        const unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), z, sizeof z);
        std::fprintf(stderr, "[diag] filtered decisions %llu, exact fallbacks %llu (%.3f%%); wave calls %llu, with a fallback %llu (%.2f%%)\n",
                     h[0], h[1], 100.0 * (double)h[1] / (double)(h[0] ? h[0] : 1), h[4], h[5],
                     100.0 * (double)h[5] / (double)(h[4] ? h[4] : 1));
        std::fprintf(stderr, "[diag] search trips %llu, replaying lanes per trip %.2f; round-end blocks %llu (%.3f per trip), lanes per block %.2f\n",
                     h[6], (double)h[2] / (double)(h[6] ? h[6] : 1), h[7], (double)h[7] / (double)(h[6] ? h[6] : 1),
                     (double)h[3] / (double)(h[7] ? h[7] : 1));
        std::fprintf(stderr, "[diag] close blocks %llu (%.3f per trip), writing lanes %llu (%.2f per block with any)\n",
                     h[12], (double)h[12] / (double)(h[6] ? h[6] : 1), h[8], (double)h[8] / (double)(h[12] ? h[12] : 1));
    }
#endif
    return hipGetLastError();
}

hipError_t launch_vdi_generate(const VdiGenParams& p, hipStream_t s) {
    hipError_t e = launch_vdi_sample(p, s);
    return e == hipSuccess ? launch_vdi_search(p, s) : e;
}

}  // namespace insitu
