// composite.hip -- sort-last compositing for gfx950.
//
// vdi_flatten_kernel: per pixel of this rank's screen strip, a k-way merge of the V
// received supersegment lists in the order determineNextSupseg picks them
// (VDICompositor.comp:58-91: smallest non-zero start depth, lowest list index on ties),
// each blended with accumulateSupseg (VDIGenerator.comp:147-185).  The list fronts (start
// depth + entry offset) live in registers, so every supersegment is read exactly once.
// vdi_composite_kernel: VDICompositor.comp:152-469, the re-supersegmenting compositor of VDI
// mode: the same merge order, gaps as transparent samples, the supersegment test and its own
// threshold binary search, S_out output supersegments per pixel.
// plain_composite_kernel: PlainImageCompositor.comp:35-92 over V one-entry lists.
#include "insitu_device.h"
#include "insitu_filter.h"
#include "insitu_kernels.h"

#pragma clang fp contract(off)

namespace insitu {

// The front of list L for this lane's pixel: first entry `base`, entries apart by `stride`, `count`
// of them.  Compact lists need the wave's 64 counts for the prefix sum, so every lane of the wave
// calls this (invalid pixels with valid == false count 0).
__device__ __forceinline__ void list_front(const VdiList& L, int tile, int lane, bool valid, int gy, int xl, int S,
                                           uint32_t e0, uint32_t slot_stride, uint32_t& base, uint32_t& stride,
                                           int& count) {
    if (L.cnt8) {   // (uniform) compact tile of the variable-length exchange
        int c = valid ? (int)L.cnt8[(size_t)tile * 64 + (size_t)lane] : 0;
        c = c < S ? c : S;   // (the sender clamps too: a corrupt count must not walk past the S slots)
        int incl = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        base = L.toff[tile] + (uint32_t)(incl - c);
        stride = 1u;
        count = c;
    } else {
        base = e0;
        stride = slot_stride;
        count = !valid ? 0 : (L.cnt16 ? (int)(L.cnt16[(size_t)gy * (size_t)L.cnt_pitch + (size_t)(L.cnt_x0 + xl)] & kPendingCount) : S);
        count = count < S ? count : S;
    }
}

template <int VMAX>
__global__ __launch_bounds__(256) void vdi_flatten_kernel(const FlattenParams P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ytiles = (P.H + 7) >> 3;
    const int tile = xcd_block((int)blockIdx.x, (int)gridDim.x) * 4 + wave;
    const int yt = tile % ytiles, xt = tile / ytiles;
    if (xt >= P.strip_tiles) return;   // wave-uniform
    const int xx = lane & 7, xl = xt * 8 + xx, gy = yt * 8 + (lane >> 3);
    const bool valid = xl < P.strip_w && gy < P.H;
    const int gx = P.x_offset + xl;
    const int S = P.S, V = P.V;
    const uint32_t e0 = (((uint32_t)xt * (uint32_t)S) * (uint32_t)P.H + (uint32_t)gy) * 8u + (uint32_t)xx;

    float fs[VMAX];      // start depth at the front of each list (0 = exhausted/empty)
    uint32_t fo[VMAX];   // entry offset of that front
    uint32_t st[VMAX];   // entry stride of the list
    int rem[VMAX];       // entries left in the list, the front included
#pragma unroll
    for (int j = 0; j < VMAX; ++j) {
        fo[j] = 0u;
        st[j] = 0u;
        rem[j] = 0;
        if (j < V) list_front(P.lists[j], tile, lane, valid, gy, xl, S, e0, (uint32_t)P.H * 8u, fo[j], st[j], rem[j]);
    }
    if (!valid) return;
#pragma unroll
    for (int j = 0; j < VMAX; ++j) fs[j] = rem[j] > 0 ? P.lists[j].dep[fo[j]].x : 0.0f;

    // accumulateSupseg pixel constants (VDIGenerator.comp:152-153)
    const float ndc_x = __builtin_fmaf((float)gx / (float)P.W, 2.0f, -1.0f);
    const float ndc_y = __builtin_fmaf((float)gy / (float)P.H, 2.0f, -1.0f);
    float base[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) base[r] = __builtin_fmaf(P.ipv[4 + r], ndc_y, P.ipv[r] * ndc_x);

    float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f, C3 = 0.0f;
    for (;;) {
        // determineNextSupseg (VDICompositor.comp:58-91): smallest non-zero front start, lowest index on ties
        float low = 100000.0f;
        int idx = -1;
#pragma unroll
        for (int j = 0; j < VMAX; ++j) {
            const float c = fs[j];
            if (c < low && c != 0.0f) { low = c; idx = j; }
        }
        if (idx < 0) break;
        const float2* dp = nullptr;
        const float4* cp = nullptr;
        uint32_t off = 0, stride = 0;
        int left = 0;
#pragma unroll
        for (int j = 0; j < VMAX; ++j)
            if (j == idx) { dp = P.lists[j].dep; cp = P.lists[j].col; off = fo[j]; stride = st[j]; left = rem[j]; }
        const float2 se = dp[off];
        const float4 colour = cp[off];
        // advance that list
        const uint32_t noff = off + stride;
        const float nxt = left > 1 ? dp[noff].x : 0.0f;
#pragma unroll
        for (int j = 0; j < VMAX; ++j)
            if (j == idx) { fo[j] = noff; rem[j] = left - 1; fs[j] = nxt; }
        // accumulateSupseg(colour, start, end)
        f4 sw, ew;
        sw.x = __builtin_fmaf(P.ipv[12], 1.0f, __builtin_fmaf(P.ipv[8], se.x, base[0]));
        sw.y = __builtin_fmaf(P.ipv[13], 1.0f, __builtin_fmaf(P.ipv[9], se.x, base[1]));
        sw.z = __builtin_fmaf(P.ipv[14], 1.0f, __builtin_fmaf(P.ipv[10], se.x, base[2]));
        sw.w = __builtin_fmaf(P.ipv[15], 1.0f, __builtin_fmaf(P.ipv[11], se.x, base[3]));
        ew.x = __builtin_fmaf(P.ipv[12], 1.0f, __builtin_fmaf(P.ipv[8], se.y, base[0]));
        ew.y = __builtin_fmaf(P.ipv[13], 1.0f, __builtin_fmaf(P.ipv[9], se.y, base[1]));
        ew.z = __builtin_fmaf(P.ipv[14], 1.0f, __builtin_fmaf(P.ipv[10], se.y, base[2]));
        ew.w = __builtin_fmaf(P.ipv[15], 1.0f, __builtin_fmaf(P.ipv[11], se.y, base[3]));
        sw = persp_div(sw);
        ew = persp_div(ew);
        const float len = len4(sw.x - ew.x, sw.y - ew.y, sw.z - ew.z, sw.w - ew.w);
        const float adj = adjust_opacity(colour.w, len);
        const float t = 1.0f - C3;
        C0 = __builtin_fmaf(t * colour.x, adj, C0);
        C1 = __builtin_fmaf(t * colour.y, adj, C1);
        C2 = __builtin_fmaf(t * colour.z, adj, C2);
        C3 = __builtin_fmaf(t, adj, C3);
        if (C3 == 1.0f) break;   // further blends add exactly zero (finite inputs)
    }
    P.out[(uint32_t)gy * (uint32_t)P.strip_w + (uint32_t)xl] =
        unorm8(C0) | (unorm8(C1) << 8) | (unorm8(C2) << 16) | (unorm8(C3) << 24);
}

hipError_t launch_vdi_flatten(const FlattenParams& p, hipStream_t s) {
    const int tiles = ((p.H + 7) / 8) * p.strip_tiles;
    const int blocks = (tiles + 3) / 4;
    if (p.V <= 8) hipLaunchKernelGGL(vdi_flatten_kernel<8>, dim3(blocks), dim3(256), 0, s, p);
    else if (p.V <= 16) hipLaunchKernelGGL(vdi_flatten_kernel<16>, dim3(blocks), dim3(256), 0, s, p);
    else if (p.V <= kMaxLists) hipLaunchKernelGGL(vdi_flatten_kernel<kMaxLists>, dim3(blocks), dim3(256), 0, s, p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

// VDICompositor.comp:152-469 for one pixel per lane; the output goes to the strip block layout
// [xt][i][y][xx] with S_out slots, zero-filled past the written ones (VDICompositor.comp:461-468).
//
// Every search pass walks the k-way merge of the V lists (determineNextSupseg, :58-91) in the same
// order -- a pass's state only decides whether a transparent gap is inserted before an entry, never
// which entry comes next -- and each entry's adjusted alpha (:286-295: its own start/end distance and
// opacity) and the world positions of its depths are the same in every pass.  So the first walk stores
// the merged sequence with that alpha and those positions in the merge cache (lane-interleaved,
// coalesced), and the search passes replay it: no front scans, no dependent list loads, no division
// for a world position, no pow for an entry's own opacity.  A wave that gets no cache space merges on
// every pass, with exact decisions (same operations, same results).
//
// The search (the generator's machinery, vdi_generate.hip): the supersegment test `diff >= thresh`
// (:338-350) is decided from the filtered estimate of diff^2 (insitu_filter.h; hardware rsq / log / exp /
// rcp on the same exact world positions and accumulated colour) when it is farther from the threshold
// than the rigorous margin, else by the exact contract path; each pass records the segmentation
// interval of its threshold-dependent decisions, and the search steps (:427-458) whose thresholds fall
// in the interval of the pass at `low` or at `high` are taken without a replay (their passes would make
// the same decisions); a pass that has closed more than S_out supersegments is decided and stops.
// Results are bit-identical to the exact, pass-by-pass form (tests/test_gpu_parity.py).
struct CompSearch {
    float low, high, mid;
    int iter;
    bool found;
};
// VDICompositor.comp:427-458 after a pass that did not write (delta = 3, :220)
__device__ __forceinline__ void comp_search_update(CompSearch& q, int n, int S_out) {
    constexpr int delta = 3;
    if (__builtin_fabsf(q.high - q.low) < 0.000001f) {
        q.found = true;
        q.mid = (n == 0) ? q.low : q.high;
        return;
    } else if (n > S_out) {
        q.low = q.mid;
    } else if (n < S_out - delta) {
        q.high = q.mid;
    } else {
        q.found = true;
        return;
    }
    q.mid = (q.low + q.high) / 2.0f;
}

#ifndef INSITU_COMP_DEEP_WINDOW
#define INSITU_COMP_DEEP_WINDOW 3e-3f   // search range below which the exact window spans it (as INSITU_DEEP_WINDOW)
#endif

#ifndef INSITU_COMP_MIN_WAVES
#define INSITU_COMP_MIN_WAVES 4   // waves per SIMD of vdi_composite_kernel for V <= 8 lists (4: 128 VGPRs with spills, -0.12 ms against 3)
#endif
template <int VMAX, bool FILTERED>
__global__ __launch_bounds__(256, VMAX <= 8 ? INSITU_COMP_MIN_WAVES : 1) void vdi_composite_kernel(const CompositeParams P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ytiles = (P.H + 7) >> 3;
    const int tile = xcd_block((int)blockIdx.x, (int)gridDim.x) * 4 + wave;
    const int yt = tile % ytiles, xt = tile / ytiles;
    if (xt >= P.strip_tiles) return;   // wave-uniform
    const int xx = lane & 7, xl = xt * 8 + xx, gy = yt * 8 + (lane >> 3);
    const bool valid = xl < P.strip_w && gy < P.H;
    const int gx = P.x_offset + xl;
    const int S = P.S, V = P.V, S_out = P.S_out;
    const uint32_t ostride = (uint32_t)P.H * 8u;
    const uint32_t e0 = (((uint32_t)xt * (uint32_t)S) * (uint32_t)P.H + (uint32_t)gy) * 8u + (uint32_t)xx;
    const uint32_t o0 = (((uint32_t)xt * (uint32_t)S_out) * (uint32_t)P.H + (uint32_t)gy) * 8u + (uint32_t)xx;
    uint32_t lb[VMAX], ls[VMAX];   // first entry and stride of each list
    int lc[VMAX];                  // entries of each list
    int total_in = 0;
#pragma unroll
    for (int j = 0; j < VMAX; ++j) {
        lb[j] = 0u;
        ls[j] = 0u;
        lc[j] = 0;
        if (j < V) list_front(P.lists[j], tile, lane, valid, gy, xl, S, e0, (uint32_t)P.H * 8u, lb[j], ls[j], lc[j]);
        total_in += lc[j];
    }
    // merge-cache space for the wave: 64 x its longest merged sequence (one 64-bit atomic)
    float4* seq = nullptr;
    if (P.seq) {
        int mx = total_in;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o));
        const unsigned long long want = (unsigned long long)mx * 64ull;
        unsigned long long base = 0;
        if (lane == 0 && want) base = atomicAdd(P.seq_cursor, want);
        base = __shfl(base, 0);
        if (want && base + want <= P.seq_cap) seq = P.seq + kCompEntryF4 * (size_t)(base + (unsigned long long)lane);
    }
    if (!valid) return;
    float4* oc = P.out_color + o0;
    float2* od = P.out_depth + o0;

    const float ndc_x = __builtin_fmaf((float)(P.ndc_local ? xl : gx) / (float)P.W, 2.0f, -1.0f);   // :204-205
    const float ndc_y = __builtin_fmaf((float)gy / (float)P.H, 2.0f, -1.0f);
    float base[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) base[r] = __builtin_fmaf(P.ipv[4 + r], ndc_y, P.ipv[r] * ndc_x);
    auto world = [&](float z) {   // ivp_orig * vec4(ndc_x, ndc_y, z, 1), divided by w
        f4 w;
        w.x = __builtin_fmaf(P.ipv[12], 1.0f, __builtin_fmaf(P.ipv[8], z, base[0]));
        w.y = __builtin_fmaf(P.ipv[13], 1.0f, __builtin_fmaf(P.ipv[9], z, base[1]));
        w.z = __builtin_fmaf(P.ipv[14], 1.0f, __builtin_fmaf(P.ipv[10], z, base[2]));
        w.w = __builtin_fmaf(P.ipv[15], 1.0f, __builtin_fmaf(P.ipv[11], z, base[3]));
        return persp_div(w);
    };
    // squared distance of two world positions: len4's operand (dist = sqrt of it, :317-322)
    auto dist2 = [](const f4& a, const f4& b) {
        const float x = a.x - b.x, y = a.y - b.y, z = a.z - b.z, w = a.w - b.w;
        return __builtin_fmaf(w, w, __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)));
    };
    auto dist = [&](const f4& a, const f4& b) { return __builtin_sqrtf(dist2(a, b)); };
    // :286-295, an entry's own adjusted alpha
    auto entry_alpha = [&](const f4& ws, const f4& we, float ca) {
        return gmax(adjust_opacity(ca, dist(ws, we)), 0.000001f);
    };

    // the merge (determineNextSupseg, :58-91): the next entry of the merged sequence, or idx < 0
    float fs[VMAX];
    uint32_t fo[VMAX];
    int rem[VMAX];
    auto merge_reset = [&]() {
#pragma unroll
        for (int j = 0; j < VMAX; ++j) {
            fo[j] = lb[j];
            rem[j] = lc[j];
            fs[j] = rem[j] > 0 ? P.lists[j].dep[fo[j]].x : 0.0f;
        }
    };
    auto merge_next = [&](float& sd, float& ed, f4& col) {
        float lowd = 100000.0f;
        int idx = -1;
#pragma unroll
        for (int j = 0; j < VMAX; ++j) {
            const float c = fs[j];
            if (c < lowd && c != 0.0f) { lowd = c; idx = j; }
        }
        sd = 0.0f;
        ed = 0.0f;
        col = f4{0.0f, 0.0f, 0.0f, 0.0f};
        if (idx >= 0) {
            const float2* dp = nullptr;
            const float4* cp = nullptr;
            uint32_t off = 0;
#pragma unroll
            for (int j = 0; j < VMAX; ++j)
                if (j == idx) { dp = P.lists[j].dep; cp = P.lists[j].col; off = fo[j]; }
            const float2 se = dp[off];
            const float4 cc = cp[off];
            sd = se.x;
            ed = se.y;
            col = f4{cc.x, cc.y, cc.z, cc.w};
        }
        return idx;
    };
    auto merge_advance = [&](int idx) {
#pragma unroll
        for (int j = 0; j < VMAX; ++j)
            if (j == idx) {
                fo[j] += ls[j];
                rem[j] -= 1;
                fs[j] = rem[j] > 0 ? P.lists[j].dep[fo[j]].x : 0.0f;
            }
    };

    // the colour bound of the filtered decisions (insitu_filter.h, filter_margin): c = max(1, 2C, 2CA)
    // with C = the largest |colour| and A the largest |alpha| of the pixel's entries -- every adjusted
    // colour of an open supersegment is a weighted mean of its entries' colours (gaps add nothing) and
    // the compared entry colour is premultiplied by its alpha.  inf: exact decisions only.
    float cpix = __builtin_inff();
    int nent = 0;   // entries in the cached sequence
    if (seq) {      // the first walk: the merged sequence, each entry's adjusted alpha and world positions
        float cmax = 0.0f, amax = 0.0f;
        merge_reset();
        for (;;) {
            float sd, ed;
            f4 col;
            const int idx = merge_next(sd, ed, col);
            if (idx < 0) break;
            const f4 ws = world(sd), we = world(ed);
            float4* q = seq + kCompEntryF4 * 64 * (size_t)nent;
            q[0] = make_float4(sd, ed, entry_alpha(ws, we, col.w), 0.0f);
            q[1] = make_float4(col.x, col.y, col.z, col.w);
            cmax = __builtin_fmaxf(cmax, __builtin_fmaxf(__builtin_fabsf(col.x), __builtin_fmaxf(__builtin_fabsf(col.y),
                                                                                           __builtin_fabsf(col.z))));
            amax = __builtin_fmaxf(amax, __builtin_fabsf(col.w));
            nent++;
            if (ed == 0.0f) break;   // the pass ends at this entry (:277)
            merge_advance(idx);
        }
        const float cb = __builtin_fmaxf(1.0f, __builtin_fmaxf(2.0f * cmax, 2.0f * cmax * amax));
        if (FILTERED && cb < 1.0e6f) cpix = cb;   // (non-finite colours: exact decisions)
    }
#ifdef INSITU_COMP_ABL_WALK
    // timing ablation only (wrong results): the merging walk that fills the merge cache, no search passes
    if (seq) {
        oc[0] = make_float4(cpix, (float)nent, 0.0f, 0.0f);
        return;
    }
#endif

    // the terminal sample of :277 (past the last entry): the same for every pass
    const f4 w0 = world(0.0f);
    const float alpha0 = entry_alpha(w0, w0, 0.0f);
    int nseg = 0;
    CompSearch q{0.0f, 1.732f, (1.732f + 0.0f) / 2.0f, 0, false};                    // :209-211
    // The search, with one pass loop per entry source (CACHED: the merge cache, the next entry loaded while
    // the current one is decided -- the replay is bound by the latency of its entry loads; else the merge
    // itself); the two copies make the same decisions in the same order.
    auto search = [&](auto cached_c) {
        constexpr bool CACHED = decltype(cached_c)::value;
        bool written = false;
        // segmentation intervals of the passes at `low` and at `high` (squared-difference space), and the
        // count of the pass at `high` (vdi_generate.hip, free_walk)
        float4 iv{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};
        int n_high = 0;
        while (!q.found || !written) {                                               // :225
            q.iter++;
            if (q.iter > 64) break;
            if (q.found) written = true;
            const bool write = written;
            // the pass's decision thresholds (insitu_filter.h); deep in the search the exact window spans the
            // whole remaining range (vdi_generate.hip, search_thr), so the recorded interval is exact there
            Thr th = make_thr(sq_threshold(q.mid), cpix);
            if (!q.found && q.high - q.low < INSITU_COMP_DEEP_WINDOW) {
                th.hi = __builtin_fmaxf(th.hi, make_thr(sq_threshold(q.high), cpix).hi);
                th.lo = __builtin_fminf(th.lo, make_thr(sq_threshold(q.low), cpix).lo);
            }
            int nterm = 0;
            bool open = false;
            float ssStart = 0.0f, ssEnd = 0.0f, ssEndTT = 0.0f;
            f4 wS{0.0f, 0.0f, 0.0f, 0.0f}, wE{0.0f, 0.0f, 0.0f, 0.0f};   // world(ssStart), world(ssEnd)
            f4 curV{0.0f, 0.0f, 0.0f, 0.0f};
            float lo = 0.0f, hi = __builtin_inff(), lo_a = -1.0f, hi_a = __builtin_inff();   // the pass's interval
            // One step of the walk (:256-417) over the entry {startDepth, endDepth, alpha, colour, world
            // positions}: a transparent gap before the entry (:299-315), or the entry itself.  Returns true
            // when the step consumed the entry (not a gap); `stop` when the pass ends (:277, or decided).
            bool stop = false;
            auto walk_step = [&](float startDepth, float endDepth, float adj_alpha, f4 colour, f4 wsd, f4 wed) {
                const bool complete = endDepth == 0.0f;                              // :277
                bool transparent = false;
                if (open) {
                    if (startDepth > ssEnd) {                                        // :299-315
                        transparent = true;
                        colour = f4{0.0f, 0.0f, 0.0f, 0.0f};
                        adj_alpha = 0.0f;
                        endDepth = startDepth;
                        wed = wsd;
                        startDepth = ssEnd;
                    }
                    // :317-350 -- the supersegment test, filtered; a terminal entry always closes
                    bool close = complete;
                    if (!complete) {
                        const float len2 = dist2(wS, wE);
                        bool decided = false;
                        if constexpr (FILTERED) {
                            // estimate of diff^2 (:325-338): adjusted opacity through v_rsq / v_log / v_exp, the
                            // adjusted colour through v_rcp (vdi_generate.hip, approx_diff_sq)
                            const float aw = 1.0f - __builtin_amdgcn_exp2f(__builtin_amdgcn_rsqf(len2) *
                                                                           __builtin_amdgcn_logf(1.0f - curV.w));
                            const float k = __builtin_amdgcn_rcpf(curV.w) * aw;
                            const float est = sumsq3(curV.x * k - colour.x * colour.w, curV.y * k - colour.y * colour.w,
                                                     curV.z * k - colour.z * colour.w);
                            const bool yes = est >= th.hi && est < 1.0e30f, no = est < th.lo;
                            // (selects, not stores through a chosen variable: keeps the four bounds in registers)
                            hi_a = yes ? __builtin_fminf(hi_a, est) : hi_a;
                            lo_a = no ? __builtin_fmaxf(lo_a, est) : lo_a;
                            decided = yes || no;
                            close = yes;
                        }
                        if (!decided) {   // the exact contract path (:317-338)
                            const float inva = 1.0f / curV.w;                        // :325-326
                            const f4 adj{curV.x * inva, curV.y * inva, curV.z * inva,
                                         adjust_opacity(curV.w, 1.0f / __builtin_sqrtf(len2))};
                            const float d2 = sumsq3(adj.x * adj.w - colour.x * colour.w, adj.y * adj.w - colour.y * colour.w,
                                                    adj.z * adj.w - colour.z * colour.w);   // :338, :93-98 (squared)
                            close = d2 >= th.sq;
                            hi = close ? __builtin_fminf(hi, d2) : hi;
                            lo = close ? lo : __builtin_fmaxf(lo, d2);
                        }
                    }
                    if (close) {                                                     // :350-384
                        nterm++;
                        open = false;
                        if (write) {
                            const float inva = 1.0f / curV.w;
                            const f4 adj{curV.x * inva, curV.y * inva, curV.z * inva,
                                         adjust_opacity(curV.w, 1.0f / dist(wS, world(ssEndTT)))};
                            if (nseg < S_out) {                                      // :146-148, OOB dropped
                                oc[(uint32_t)nseg * ostride] = make_float4(adj.x, adj.y, adj.z, adj.w);
                                od[(uint32_t)nseg * ostride] = make_float2(ssStart, ssEndTT);
                            }
                            nseg++;
                        }
                    } else {                                                         // :385-392
                        const float t = 1.0f - curV.w;                               // :328-330
                        curV = f4{__builtin_fmaf(t * colour.x, adj_alpha, curV.x), __builtin_fmaf(t * colour.y, adj_alpha, curV.y),
                                  __builtin_fmaf(t * colour.z, adj_alpha, curV.z), __builtin_fmaf(t, adj_alpha, curV.w)};
                        ssEnd = endDepth;
                        wE = wed;
                        if (!transparent) ssEndTT = endDepth;
                    }
                }
                if (!open && !transparent) {                                         // :395-408
                    ssStart = startDepth;
                    ssEnd = endDepth;
                    ssEndTT = endDepth;
                    wS = wsd;
                    wE = wed;
                    curV = f4{colour.x * adj_alpha, colour.y * adj_alpha, colour.z * adj_alpha, adj_alpha};
                    open = true;
                }
                // a search pass that has closed more than S_out supersegments is decided (:427-458 only asks
                // n > S_out, n < S_out - delta, or n == 0): the rest of it is skipped
                stop = complete || (!write && nterm > S_out);
                return !transparent;
            };
            if constexpr (CACHED) {
                // entries e and e + 1 in the register sets A and B, each reloaded with entry e + 2 as soon as
                // it is consumed: the walk alternates A, B (an entry takes one or two steps: a gap may come
                // first), so a load has a whole entry's decisions to land, and no register copies are needed
                float4 a0{}, a1{}, b0{}, b1{};
                auto load_entry = [&](int j, float4& x0, float4& x1) {
                    const float4* qe = seq + kCompEntryF4 * 64 * (size_t)j;
                    x0 = qe[0];
                    x1 = qe[1];
                };
                // the entry in (x0, x1) if it exists, else the terminal sample of :277 (past the last entry);
                // the world positions of its depths are recomputed (world(): the same operations on the same
                // values as the first walk, so the same bits -- a few dozen VALU per entry against 32 more
                // bytes of merge-cache traffic per entry and pass: composite 3.81 -> 3.18 ms, round 5)
                auto walk_entry = [&](bool exists, const float4& x0, const float4& x1) {
                    const f4 wsd = world(x0.x), wed = world(x0.y);
                    for (;;) {   // at most two steps: a gap, then the entry
                        const bool consumed = exists ? walk_step(x0.x, x0.y, x0.z, f4{x1.x, x1.y, x1.z, x1.w}, wsd, wed)
                                                     : walk_step(0.0f, 0.0f, alpha0, f4{0.0f, 0.0f, 0.0f, 0.0f}, w0, w0);
                        if (consumed || stop) return;
                    }
                };
                // (loads past the last entry read the last one again -- unconditional loads, so the register
                // sets are never merged with their old values; the wave's cache space holds entry 0 of every
                // lane, so a lane without entries reads its own slot)
                const int elast = nent > 0 ? nent - 1 : 0;
                load_entry(0, a0, a1);
                load_entry(min(1, elast), b0, b1);
                for (int e = 0;; e += 2) {
                    walk_entry(e < nent, a0, a1);
                    if (stop) break;
                    load_entry(min(e + 2, elast), a0, a1);
                    walk_entry(e + 1 < nent, b0, b1);
                    if (stop) break;
                    load_entry(min(e + 3, elast), b0, b1);
                }
            } else {
                merge_reset();
                for (;;) {
                    float sd, ed;
                    f4 col;
                    const int idx = merge_next(sd, ed, col);
                    if (idx >= 0) {
                        const f4 ws = world(sd), we = world(ed);
                        const float al = entry_alpha(ws, we, col.w);
                        for (;;) {   // a gap, then the entry
                            const bool consumed = walk_step(sd, ed, al, col, ws, we);
                            if (consumed || stop) break;
                        }
                        if (stop) break;
                        merge_advance(idx);
                    } else {
                        for (;;) {
                            const bool consumed = walk_step(0.0f, 0.0f, alpha0, f4{0.0f, 0.0f, 0.0f, 0.0f}, w0, w0);
                            if (consumed || stop) break;
                        }
                        break;   // (the terminal sample always ends the pass)
                    }
                }
            }
            if (!written) {                                                          // :427-458
                if constexpr (FILTERED) {   // bounds from the recorded extreme estimates (insitu_filter.h)
                    lo = __builtin_fmaxf(lo, seg_lo_bound(lo_a, cpix));
                    hi = __builtin_fminf(hi, seg_hi_bound(hi_a, cpix));
                }
                if (!(__builtin_fabsf(q.high - q.low) < 0.000001f)) {   // the bound the step moves keeps the interval
                    if (nterm > S_out) {
                        iv.x = lo;
                        iv.y = hi;
                    } else if (nterm < S_out - 3) {
                        iv.z = lo;
                        iv.w = hi;
                        n_high = nterm;
                    }
                }
                comp_search_update(q, nterm, S_out);
                // the steps whose thresholds the intervals decide, without a pass (same decisions, same count)
                while (!q.found && q.iter < 64) {
                    const float t = sq_threshold(q.mid);
                    int n;
                    if (t > iv.x && t <= iv.y) n = S_out + 1;
                    else if (t > iv.z && t <= iv.w) n = n_high;
                    else break;
                    q.iter++;
                    comp_search_update(q, n, S_out);
                }
            }
        }
    };
    if (seq) search(std::true_type{});
    else search(std::false_type{});
    if (P.out_count) {   // the slots past the count are zeros to every reader (insitu_read, the root's flatten)
        P.out_count[(uint32_t)gy * (uint32_t)P.strip_w + (uint32_t)xl] = (uint16_t)(nseg < S_out ? nseg : S_out);
    } else {
        for (int i = nseg; i < S_out; ++i) {                                         // :461-468
            oc[(uint32_t)i * ostride] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            od[(uint32_t)i * ostride] = make_float2(0.0f, 0.0f);
        }
    }
    if (P.passes) P.passes[(uint32_t)gy * (uint32_t)P.strip_w + (uint32_t)xl] = (uint8_t)q.iter;
}

hipError_t launch_vdi_composite(const CompositeParams& p, hipStream_t s) {
    const int tiles = ((p.H + 7) / 8) * p.strip_tiles;
    const int blocks = (tiles + 3) / 4;
    if (p.S_out < 1 || p.S < 1) return hipErrorInvalidValue;
    const bool f = !p.exact;
    if (p.V <= 8) {
        if (f) hipLaunchKernelGGL((vdi_composite_kernel<8, true>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((vdi_composite_kernel<8, false>), dim3(blocks), dim3(256), 0, s, p);
    } else if (p.V <= 16) {
        if (f) hipLaunchKernelGGL((vdi_composite_kernel<16, true>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((vdi_composite_kernel<16, false>), dim3(blocks), dim3(256), 0, s, p);
    } else if (p.V <= kMaxLists) {
        if (f) hipLaunchKernelGGL((vdi_composite_kernel<kMaxLists, true>), dim3(blocks), dim3(256), 0, s, p);
        else hipLaunchKernelGGL((vdi_composite_kernel<kMaxLists, false>), dim3(blocks), dim3(256), 0, s, p);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <int VMAX>
__global__ __launch_bounds__(256) void plain_composite_kernel(const PlainCompParams P) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t npx = (uint32_t)P.rows * (uint32_t)P.dim0;
    if (i >= npx) return;
    const int V = P.V;
    float dv[VMAX];
    bool used[VMAX];
#pragma unroll
    for (int j = 0; j < VMAX; ++j) {
        dv[j] = (j < V) ? decode_depth_rgba8(P.depths[j][i]) : 0.0f;
        used[j] = (j >= V);
    }
    float C0 = 0.0f, C1 = 0.0f, C2 = 0.0f, C3 = 0.0f;
    for (int it = 0; it < V; ++it) {
        float low = 200.0f;
        int idx = -1;
#pragma unroll
        for (int j = 0; j < VMAX; ++j) {
            if (used[j]) continue;
            const float d = dv[j];
            if (d < low && d != 0.0f) { low = d; idx = j; }
        }
        float c0 = 0.0f, c1 = 0.0f, c2 = 0.0f, c3 = 0.0f;
        if (idx >= 0) {
            uint32_t p = 0;
#pragma unroll
            for (int j = 0; j < VMAX; ++j)
                if (j == idx) { p = P.colors[j][i]; used[j] = true; }
            c0 = (float)(p & 0xffu) / 255.0f;
            c1 = (float)((p >> 8) & 0xffu) / 255.0f;
            c2 = (float)((p >> 16) & 0xffu) / 255.0f;
            c3 = (float)(p >> 24) / 255.0f;
        }
        const float t = 1.0f - C3;   // PlainImageCompositor.comp:81-82
        C0 = __builtin_fmaf(t * c0, c3, C0);
        C1 = __builtin_fmaf(t * c1, c3, C1);
        C2 = __builtin_fmaf(t * c2, c3, C2);
        C3 = __builtin_fmaf(t, c3, C3);
    }
    P.out[i] = unorm8(C0) | (unorm8(C1) << 8) | (unorm8(C2) << 16) | (unorm8(C3) << 24);
}

hipError_t launch_plain_composite(const PlainCompParams& p, hipStream_t s) {
    const uint32_t npx = (uint32_t)p.rows * (uint32_t)p.dim0;
    const dim3 grid((npx + 255) / 256);
    if (p.V <= 8) hipLaunchKernelGGL(plain_composite_kernel<8>, grid, dim3(256), 0, s, p);
    else if (p.V <= kMaxLists) hipLaunchKernelGGL(plain_composite_kernel<kMaxLists>, grid, dim3(256), 0, s, p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

__global__ void assemble_columns_kernel(const uint32_t* strips, int nstrips, int H, int strip_w, uint32_t* image) {
    const uint32_t W = (uint32_t)nstrips * (uint32_t)strip_w;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * (uint32_t)H) return;
    const uint32_t y = i / W, x = i - y * W;
    const uint32_t d = x / (uint32_t)strip_w, xl = x - d * (uint32_t)strip_w;
    image[i] = strips[((size_t)d * (size_t)H + y) * (size_t)strip_w + xl];
}

hipError_t launch_assemble_columns(const uint32_t* strips, int nstrips, int H, int strip_w, uint32_t* image,
                                   hipStream_t s) {
    const uint32_t n = (uint32_t)nstrips * (uint32_t)strip_w * (uint32_t)H;
    hipLaunchKernelGGL(assemble_columns_kernel, dim3((n + 255) / 256), dim3(256), 0, s, strips, nstrips, H, strip_w,
                       image);
    return hipGetLastError();
}

// our [d][b][xt][i][y][xx] layout -> reference (S,H,W) rgba32f + (2S,H,W) r32f of brick b, columns
// [x0, x0 + nx) (the whole image: x0 = 0, nx = W); slots past the pixel's count read as zero, as the
// reference's zero-filled images (VDIGenerator.comp:553-590, VDICompositor.comp:461-468).  The count of
// pixel (strip d, row y, strip column xl) of brick b is pend[b * pend_stride + d * pend_dstride + y * pend_pitch + xl]
// (sub-VDIs: per brick [y][x] of the full width, i.e. dstride strip_w, pitch W; composited VDIs: per strip
// [y][xl], dstride H * strip_w, pitch strip_w); null: every slot stored
__global__ void vdi_to_reference_kernel(const float4* color, const float2* depth, const uint16_t* pend,
                                        size_t pend_stride, size_t pend_dstride, size_t pend_pitch, int W, int x0,
                                        int nx, int H, int S, int strip_w, int strip_tiles, int B, int b,
                                        float4* ref_color, float* ref_depth) {
    const size_t n = (size_t)nx * (size_t)H * (size_t)S;
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    // r = ((x - x0)*H + y)*S + i
    const int i = (int)(r % (size_t)S);
    const size_t px = r / (size_t)S;
    const int y = (int)(px % (size_t)H), x = x0 + (int)(px / (size_t)H);
    const int d = x / strip_w, xl = x - d * strip_w, xt = xl >> 3, xx = xl & 7;
    const size_t blockE = (size_t)strip_tiles * (size_t)S * (size_t)H * 8;
    const size_t e = ((size_t)d * (size_t)B + (size_t)b) * blockE +
                     (((size_t)xt * (size_t)S + (size_t)i) * (size_t)H + (size_t)y) * 8 + (size_t)xx;
    const int cnt = pend ? (int)(pend[(size_t)b * pend_stride + (size_t)d * pend_dstride + (size_t)y * pend_pitch + (size_t)xl] &
                                 kPendingCount)
                         : S;
    const bool stored = i < cnt;
    ref_color[r] = stored ? color[e] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float2 se = stored ? depth[e] : make_float2(0.0f, 0.0f);
    ref_depth[2 * r] = se.x;
    ref_depth[2 * r + 1] = se.y;
}

hipError_t launch_vdi_to_reference(const float4* color, const float2* depth, const uint16_t* pend, size_t pend_stride,
                                   size_t pend_dstride, size_t pend_pitch, int W, int x0, int nx, int H, int S, int strip_w,
                                   int strip_tiles, int B, int b, float4* ref_color, float* ref_depth, hipStream_t s) {
    const size_t n = (size_t)nx * (size_t)H * (size_t)S;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(vdi_to_reference_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, color, depth, pend,
                       pend_stride, pend_dstride, pend_pitch, W, x0, nx, H, S, strip_w, strip_tiles, B, b, ref_color,
                       ref_depth);
    return hipGetLastError();
}

// one list of this rank's strip as the compositors read it (own slots with counts, a received compact
// message, or a host-path block) -> the reference layout of that received block: colour (strip_w, H, S)
// rgba32f and depth (strip_w, H, 2S) r32f, x slowest, empty slots zero -- one block of the SetOfVDI set
// uploadForCompositing receives (DistributedVolumes.kt:945, dumped at :974-975).  One wave per 8x8 tile.
__global__ __launch_bounds__(256) void vdi_list_to_reference_kernel(const VdiList L, int S, int H, int strip_w,
                                                                     int strip_tiles, float4* ref_color,
                                                                     float2* ref_depth) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int ytiles = (H + 7) >> 3;
    const int tile = (int)blockIdx.x * 4 + wave;
    const int yt = tile % ytiles, xt = tile / ytiles;
    if (xt >= strip_tiles) return;   // wave-uniform
    const int xx = lane & 7, xl = xt * 8 + xx, gy = yt * 8 + (lane >> 3);
    const bool valid = xl < strip_w && gy < H;
    const uint32_t e0 = (((uint32_t)xt * (uint32_t)S) * (uint32_t)H + (uint32_t)gy) * 8u + (uint32_t)xx;
    uint32_t base = 0, stride = 0;
    int count = 0;
    list_front(L, tile, lane, valid, gy, xl, S, e0, (uint32_t)H * 8u, base, stride, count);
    if (!valid) return;
    const size_t r0 = ((size_t)xl * (size_t)H + (size_t)gy) * (size_t)S;
    for (int i = 0; i < S; ++i) {
        const bool stored = i < count;
        const uint32_t e = base + (uint32_t)i * stride;
        ref_color[r0 + i] = stored ? L.col[e] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        ref_depth[r0 + i] = stored ? L.dep[e] : make_float2(0.0f, 0.0f);
    }
}

hipError_t launch_vdi_list_to_reference(const VdiList& L, int S, int H, int strip_w, int strip_tiles, float4* ref_color,
                                        float2* ref_depth, hipStream_t s) {
    const int tiles = strip_tiles * ((H + 7) / 8);
    if (tiles == 0) return hipSuccess;
    hipLaunchKernelGGL(vdi_list_to_reference_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, s, L, S, H,
                       strip_w, strip_tiles, ref_color, ref_depth);
    return hipGetLastError();
}

// reference-layout strip block of one source -- colour (strip_w, H, S) rgba32f and depth (strip_w, H, 2S)
// r32f, x slowest (what distributeVDIs hands over, DistributedVolumes.kt:860) -> our [xt][i][y][xx] block,
// and per pixel the count of slots before the first empty start ([y][xl]): determineNextSupseg
// (VDICompositor.comp:58-91) never picks a front whose start is 0, so a list ends there
__global__ void vdi_from_reference_kernel(const float4* ref_color, const float* ref_depth, int H, int S, int strip_w,
                                          float4* color, float2* depth, uint16_t* counts) {
    const size_t n = (size_t)strip_w * (size_t)H * (size_t)S;
    const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const int i = (int)(r % (size_t)S);
    const size_t px = r / (size_t)S;
    const int y = (int)(px % (size_t)H), xl = (int)(px / (size_t)H);
    const size_t e = (((size_t)(xl >> 3) * (size_t)S + (size_t)i) * (size_t)H + (size_t)y) * 8 + (size_t)(xl & 7);
    color[e] = ref_color[r];
    depth[e] = make_float2(ref_depth[2 * r], ref_depth[2 * r + 1]);
    if (i == 0) {
        int c = 0;
        while (c < S && ref_depth[2 * (px * (size_t)S + (size_t)c)] != 0.0f) ++c;
        counts[(size_t)y * (size_t)strip_w + (size_t)xl] = (uint16_t)c;
    }
}

hipError_t launch_vdi_from_reference(const float4* ref_color, const float* ref_depth, int H, int S, int strip_w,
                                     int strip_tiles, float4* color, float2* depth, uint16_t* counts, hipStream_t s) {
    const size_t n = (size_t)strip_w * (size_t)H * (size_t)S;
    (void)strip_tiles;
    hipLaunchKernelGGL(vdi_from_reference_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, ref_color,
                       ref_depth, H, S, strip_w, color, depth, counts);
    return hipGetLastError();
}

// Variable-length exchange: one wave per 8x8 tile of a strip block bound for another rank.  The
// tile's 64 counts meet in a wave prefix sum, one atomic on the destination's cursor places the
// tile's entries (pixel-major), the counts and the tile's first entry go to the meta block.  Only
// stored supersegments travel; the slotted blocks hold S slots per pixel, most of them empty.
__global__ __launch_bounds__(256) void vdi_compact_kernel(const CompactParams P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int d = (int)blockIdx.z, b = (int)blockIdx.y;
    if (d == P.skip_d) return;   // block-uniform: this rank's own strip is not sent
    const int tiles = P.strip_tiles * P.ytiles;
    const int tile = (int)blockIdx.x * 4 + wave;
    if (tile >= tiles) return;   // wave-uniform
    const int xt = tile / P.ytiles, yt = tile - xt * P.ytiles;
    const int xl = xt * 8 + (lane & 7), gy = yt * 8 + (lane >> 3);
    const bool valid = xl < P.strip_w && gy < P.H;
    const int gx = d * P.strip_w + xl;
    int c = valid ? (int)(P.pend[(size_t)b * P.pend_stride + (size_t)gy * (size_t)P.W + (size_t)gx] & kPendingCount) : 0;
    c = c < P.S ? c : P.S;
    int incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
    }
    const uint32_t total = (uint32_t)__shfl(incl, 63);
    uint32_t base = 0;
    if (lane == 63 && total) base = atomicAdd(&P.cursor[d], total);
    base = __shfl(base, 63);
    uint8_t* meta = P.out_meta + (size_t)d * P.meta_bytes;
    meta[((size_t)b * (size_t)tiles + (size_t)tile) * 64 + (size_t)lane] = (uint8_t)c;
    uint32_t* toff = reinterpret_cast<uint32_t*>(meta + (size_t)P.B * (size_t)tiles * 64);
    if (lane == 0) toff[(size_t)b * (size_t)tiles + (size_t)tile] = base;
    const size_t src = ((size_t)d * (size_t)P.B + (size_t)b) * P.blockE +
                       (((size_t)xt * (size_t)P.S) * (size_t)P.H + (size_t)gy) * 8 + (size_t)(lane & 7);
    const size_t dst = (size_t)d * (size_t)P.B * P.blockE + (size_t)base + (size_t)(incl - c);
    const size_t sstride = (size_t)P.H * 8;
    for (int i = 0; i < c; ++i) {
        P.out_col[dst + (size_t)i] = P.col[src + (size_t)i * sstride];
        P.out_dep[dst + (size_t)i] = P.dep[src + (size_t)i * sstride];
    }
}

hipError_t launch_vdi_compact(const CompactParams& p, hipStream_t s) {
    const int tiles = p.strip_tiles * p.ytiles;
    hipLaunchKernelGGL(vdi_compact_kernel, dim3((tiles + 3) / 4, p.B, p.nstrips), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace insitu
