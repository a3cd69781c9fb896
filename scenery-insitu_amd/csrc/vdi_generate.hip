// vdi_generate.hip -- VDI generation for gfx950: VDIGenerator.comp + AccumulateVDI.comp.
//
// One lane = one ray (pixel); one wave = one 8x8 pixel tile; 4 waves per 256-thread block
// stacked along y.  The per-ray threshold binary search (VDIGenerator.comp:404-539)
// re-marches the ray until the supersegment count fits S; the accepted threshold is then
// used for a final pass that writes the supersegments (VDIGenerator.comp:204-225) and
// counts octree cells (AccumulateVDI.comp:158-177).  Transfer function and colour map are
// staged in LDS once per block; the brick is read through L1/L2/MALL.
#include "insitu_sampling.h"

#pragma clang fp contract(off)

namespace insitu {

// VDIGenerator.comp:244-254
__device__ __forceinline__ int find_z_interval_view(float z_view, float interval_size, int ncz) {
    float dist_from_front = __builtin_fabsf(z_view - (-1.0f * 0.1f));
    float q = __builtin_floorf(dist_from_front / interval_size);
    if (!(q < (float)ncz)) return ncz;
    return (int)q;
}

struct RayOut {
    float4* color;   // entry 0 of this pixel's block; slot i at + i*H*8
    float2* depth;
    uint32_t slot_stride;
};

__device__ __forceinline__ void octree_update(const VdiGenParams& P, uint32_t* octree, float uvx, float uvy,
                                              float start, float end, int cx, int cy) {
    f4 sw = persp_div(mat_vec(P.ipv, f4{uvx, uvy, start, 1.0f}));
    f4 ew = persp_div(mat_vec(P.ipv, f4{uvx, uvy, end, 1.0f}));
    float sz = mat_row(P.view, 2, sw);
    float ez = mat_row(P.view, 2, ew);
    int sc = find_z_interval_view(sz, P.interval_size, P.S);
    int ec = find_z_interval_view(ez, P.interval_size, P.S);
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

// VDIGenerator.comp:278-372 for one brick (a1)
__device__ __forceinline__ Ray ray_setup(const VdiGenParams& P, const BrickDesc& brick, int gx, int gy) {
    Ray r;
    r.cx = (int)__builtin_floorf(((float)gx / (float)P.W) * (float)P.ncx);   // VDIGenerator.comp:286-287
    r.cy = (int)__builtin_floorf(((float)gy / (float)P.H) * (float)P.ncy);
    const float tcx = (float)gx / (float)P.W, tcy = (float)gy / (float)P.H;
    r.uvx = __builtin_fmaf(tcx, 2.0f, -1.0f);
    r.uvy = __builtin_fmaf(tcy, 2.0f, -1.0f);
    r.wfront = persp_div(mat_vec(P.ipv, f4{r.uvx, r.uvy, -1.0f, 1.0f}));
    r.wback = persp_div(mat_vec(P.ipv, f4{r.uvx, r.uvy, 1.0f, 1.0f}));
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

// Raymarch passes of one ray (VDIGenerator.comp:380-590 with AccumulateVDI.comp at :476).
// cache != null: pass 1 records, per sample inside the brick, {LUT coordinate, adjusted opacity w,
// NDC z of the next sample position}; passes 2.. replay the state machine from those values --
// the same float values the sampling pass would recompute, so results are bit-identical.
template <int DT>
__device__ void vdi_march(const VdiGenParams& P, const BrickDesc& brick, uint32_t* octree, uint8_t* passes,
                          const float* s_tf, const float4* s_cm, int gx, int gy, const Ray& R, RayOut o,
                          float* __restrict__ cache) {
    const float nw = P.nw;
    const int S = P.S;
    const f4 wfront = R.wfront, wback = R.wback;
    const float localNear = R.localNear, localFar = R.localFar;
    const int numSteps = R.numSteps;
    int supersegmentNum = 0;
    int iter = 0;
    if (R.hit) {
        float low_thresh = 0.0f, high_thresh = 1.732f;
        bool supsegs_written = false, thresh_found = false;
        const int desired_supsegs = S;
        const int delta = (int)__builtin_floorf(0.15f * (float)S);
        float mid_thresh = 0.0001f;
        bool first_iteration = true;
        int i0 = 0, i1 = -1;          // samples inside the brick (contiguous), found by pass 1
        float ndc_first = 0.0f;       // NDC z of sample i0
        while (!thresh_found || !supsegs_written) {
            iter++;
            if (iter > 64) break;
            if (thresh_found) supsegs_written = true;
            const float thresh = mid_thresh;
            int num_terminations = 0;
            bool open = false;
            float startPt = 0.0f, endPt = 0.0f;
            bool transparent = false;
            f4 adj{0.0f, 0.0f, 0.0f, 0.0f};
            float ndc_step = 0.0f;
            int steps_in = 0, steps_tt = 0;
            f4 curV{0.0f, 0.0f, 0.0f, 0.0f};
            // the per-sample state machine (AccumulateVDI.comp:12-335) given the sample's colour x,
            // adjusted opacity w, its own NDC z (when opening) and the next position's NDC z
#define INSITU_ACCUMULATE(X, W_, NDC_HERE, NDC_NEXT, LAST)                                                        \
    {                                                                                                             \
        const f4 xv = (X);                                                                                         \
        if (xv.x > -0.5f || (LAST)) {                                                                              \
            const float wv = (W_);                                                                                 \
            if (wv <= 0.0f) transparent = true;                                                                    \
            if (open) {                                                                                           \
                const f4 jp = v4mix(wfront, wback, nw * (float)steps_in);                                         \
                const float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);    \
                const float inva = 1.0f / curV.w;                                                                 \
                adj.x = curV.x * inva;                                                                            \
                adj.y = curV.y * inva;                                                                            \
                adj.z = curV.z * inva;                                                                            \
                adj.w = adjust_opacity(curV.w, 1.0f / segLen);                                                    \
                const float ax = adj.x * adj.w, ay = adj.y * adj.w, az = adj.z * adj.w;                           \
                const float bx = xv.x * xv.w, by = xv.y * xv.w, bz = xv.z * xv.w;                                       \
                const float diff = len3(ax - bx, ay - by, az - bz);                                               \
                if (diff >= thresh) {                                                                             \
                    num_terminations++;                                                                           \
                    open = false;                                                                                 \
                    endPt = ndc_step;                                                                             \
                    steps_in = 0;                                                                                 \
                    steps_tt = 0;                                                                                 \
                    if (thresh_found) {                                                                           \
                        if (supersegmentNum < S) {                                                                \
                            const uint32_t off = (uint32_t)supersegmentNum * o.slot_stride;                       \
                            o.color[off] = make_float4(adj.x, adj.y, adj.z, adj.w);                               \
                            o.depth[off] = make_float2(startPt, endPt);                                           \
                        }                                                                                         \
                        octree_update(P, octree, R.uvx, R.uvy, startPt, endPt, R.cx, R.cy);                       \
                        supersegmentNum++;                                                                        \
                    }                                                                                             \
                }                                                                                                 \
            }                                                                                                     \
            if (!open && !transparent) {                                                                          \
                open = true;                                                                                      \
                startPt = (NDC_HERE);                                                                             \
                curV = f4{0.0f, 0.0f, 0.0f, 0.0f};                                                                \
            }                                                                                                     \
            if (open) {                                                                                           \
                const float t = 1.0f - curV.w;                                                                    \
                curV.x = __builtin_fmaf(t * xv.x, wv, curV.x);                                                      \
                curV.y = __builtin_fmaf(t * xv.y, wv, curV.y);                                                      \
                curV.z = __builtin_fmaf(t * xv.z, wv, curV.z);                                                      \
                curV.w = __builtin_fmaf(t, wv, curV.w);                                                            \
                steps_in++;                                                                                       \
                if (!transparent) {                                                                               \
                    steps_tt = steps_in;                                                                          \
                    ndc_step = (NDC_NEXT);                                                                        \
                }                                                                                                 \
            }                                                                                                     \
            if ((LAST) && open) {                                                                                 \
                const f4 jp = v4mix(wfront, wback, nw * (float)steps_tt);                                         \
                const float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);    \
                const float inva = 1.0f / curV.w;                                                                 \
                adj.x = curV.x * inva;                                                                            \
                adj.y = curV.y * inva;                                                                            \
                adj.z = curV.z * inva;                                                                            \
                adj.w = adjust_opacity(curV.w, 1.0f / segLen);                                                    \
                num_terminations++;                                                                               \
                open = false;                                                                                     \
                endPt = ndc_step;                                                                                 \
                steps_in = 0;                                                                                     \
                if (thresh_found) {                                                                               \
                    if (supersegmentNum < S) {                                                                    \
                        const uint32_t off = (uint32_t)supersegmentNum * o.slot_stride;                           \
                        o.color[off] = make_float4(adj.x, adj.y, adj.z, adj.w);                                   \
                        o.depth[off] = make_float2(startPt, endPt);                                               \
                    }                                                                                             \
                    octree_update(P, octree, R.uvx, R.uvy, startPt, endPt, R.cx, R.cy);                           \
                    supersegmentNum++;                                                                            \
                }                                                                                                 \
            }                                                                                                     \
        }                                                                                                         \
    }
            if (cache != nullptr && iter > 1) {
                // replay pass: only the samples inside the brick, values from the cache
                float prev_ndc = ndc_first;
                for (int i = i0; i <= i1; ++i) {
                    const float* e = cache + 3 * (size_t)i;
                    const float es = e[0], ew = e[1], en = e[2];
                    transparent = false;
                    INSITU_ACCUMULATE(classify_sample(es, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm), ew, prev_ndc, en,
                                      i == numSteps - 1)
                    prev_ndc = en;
                }
            } else {
                const bool fill = cache != nullptr;   // iter == 1
                float step = R.tnear;
                f4 wprev = v4mix(wfront, wback, step - nw);
                for (int i = 0; i < numSteps; ++i, step += nw) {
                    const bool lastSample = (i == numSteps - 1);
                    const f4 wpos = v4mix(wfront, wback, step);
                    if (step > localNear && step < localFar) {
                        transparent = false;
                        const float sc = sample_coord<DT>(brick, wpos);
                        const f4 x = classify_sample(sc, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
                        float w = 0.0f;
                        if (x.x > -0.5f || lastSample)
                            w = adjust_opacity(
                                x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
                        const float ndc_next = persp_div(mat_vec(P.pv, v4mix(wfront, wback, step + nw))).z;
                        if (fill) {
                            if (i1 < i0) {   // first sample inside the brick
                                i0 = i;
                                ndc_first = persp_div(mat_vec(P.pv, wpos)).z;
                            }
                            i1 = i;
                            float* e = cache + 3 * (size_t)i;
                            e[0] = sc;
                            e[1] = w;
                            e[2] = ndc_next;
                        }
                        INSITU_ACCUMULATE(x, w, persp_div(mat_vec(P.pv, wpos)).z, ndc_next, lastSample)
                    }
                    wprev = wpos;
                }
            }
#undef INSITU_ACCUMULATE
            if (!supsegs_written) {
                if (__builtin_fabsf(high_thresh - low_thresh) < 0.000001f) {
                    thresh_found = true;
                    mid_thresh = (num_terminations == 0) ? low_thresh : high_thresh;
                    continue;
                } else if (num_terminations > desired_supsegs) {
                    low_thresh = mid_thresh;
                } else if (num_terminations < (desired_supsegs - delta)) {
                    high_thresh = mid_thresh;
                } else {
                    thresh_found = true;
                    continue;
                }
                if (first_iteration) {
                    first_iteration = false;
                    if (num_terminations < desired_supsegs) {
                        thresh_found = true;
                        continue;
                    }
                }
                mid_thresh = (low_thresh + high_thresh) / 2.0f;
            }
        }
    }
    for (int i = supersegmentNum; i < S; ++i) {   // VDIGenerator.comp:553-590
        const uint32_t off = (uint32_t)i * o.slot_stride;
        o.color[off] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        o.depth[off] = make_float2(0.0f, 0.0f);
    }
    if (passes) passes[(uint32_t)gy * (uint32_t)P.W + (uint32_t)gx] = (uint8_t)iter;
}

template <int DT>
__global__ __launch_bounds__(256) void vdi_generate_kernel(const VdiGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + P.xfer.n_cm);
    stage_luts(P.xfer, s_cm, s_tf);

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = blockIdx.x * 4 + wave;
    const int yt = tile % P.ytiles;
    const int ct = tile / P.ytiles;                   // global column tile
    const int d = ct / P.strip_tiles, xt = ct % P.strip_tiles;
    const int xx = lane & 7, yy = lane >> 3;
    const int xl = xt * 8 + xx, gy = yt * 8 + yy;
    const bool valid = d < P.nstrips && xl < P.strip_w && gy < P.H;
    const int gx = d * P.strip_w + xl;
    const int b = blockIdx.y;
    const BrickDesc& brick = P.bricks[b];
    Ray R{};
    if (valid) R = ray_setup(P, brick, gx, gy);

    // sample-cache allocation for the whole wave: prefix scan of the lanes' sample counts,
    // one 64-bit atomic per wave (all 64 lanes are active here)
    float* cache = nullptr;
    if (P.cache) {
        const uint32_t need = (valid && R.hit && R.numSteps <= 65536) ? (uint32_t)R.numSteps : 0u;
        uint32_t incl = need;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o);
            if (lane >= o) incl += y;
        }
        const uint32_t total = __shfl(incl, 63);
        unsigned long long base = 0;
        if (lane == 63 && total) base = atomicAdd((unsigned long long*)P.cache_cursor, (unsigned long long)total);
        base = __shfl(base, 63);
        if (need && base + total <= (unsigned long long)P.cache_entries)
            cache = P.cache + 3 * (size_t)(base + incl - need);
    }
    if (!valid) return;
    const size_t blockE = (size_t)P.strip_tiles * (size_t)P.S * (size_t)P.H * 8;
    const size_t blk = (size_t)d * (size_t)P.B + (size_t)b;
    const size_t e0 = blk * blockE + (((size_t)xt * (size_t)P.S) * (size_t)P.H + (size_t)gy) * 8 + (size_t)xx;
    RayOut o{P.color + e0, P.depth + e0, (uint32_t)P.H * 8u};
    vdi_march<DT>(P, brick, P.octree + (size_t)b * P.octree_stride,
                  P.passes ? P.passes + (size_t)b * P.passes_stride : nullptr, s_tf, s_cm, gx, gy, R, o, cache);
}

hipError_t launch_vdi_generate(const VdiGenParams& p, hipStream_t s) {
    const int tiles = p.ytiles * p.nstrips * p.strip_tiles;
    const dim3 grid((tiles + 3) / 4, p.B);
    const size_t lds = (size_t)p.xfer.n_cm * sizeof(float4) + (size_t)p.xfer.n_tf * sizeof(float);
    if (p.B < 1 || p.B > kMaxBricks) return hipErrorInvalidValue;
    for (int b = 1; b < p.B; ++b)   // one voxel type per launch (the kernel is templated on it)
        if (p.bricks[b].dtype != p.bricks[0].dtype) return hipErrorInvalidValue;
    if (p.cache) {
        hipError_t e = hipMemsetAsync(p.cache_cursor, 0, sizeof(unsigned long long), s);
        if (e != hipSuccess) return e;
    }
    switch (p.bricks[0].dtype) {
    case VOX_U8: hipLaunchKernelGGL(vdi_generate_kernel<VOX_U8>, grid, dim3(256), lds, s, p); break;
    case VOX_U16: hipLaunchKernelGGL(vdi_generate_kernel<VOX_U16>, grid, dim3(256), lds, s, p); break;
    case VOX_F32: hipLaunchKernelGGL(vdi_generate_kernel<VOX_F32>, grid, dim3(256), lds, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
