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

template <int DT>
__device__ void vdi_ray(const VdiGenParams& P, const BrickDesc& brick, uint32_t* octree, uint8_t* passes,
                        const float* s_tf, const float4* s_cm, int gx, int gy, RayOut o) {
    const int W = P.W, H = P.H;
    const float nw = P.nw;
    const int cx = (int)__builtin_floorf(((float)gx / (float)W) * (float)P.ncx);
    const int cy = (int)__builtin_floorf(((float)gy / (float)H) * (float)P.ncy);
    const float tcx = (float)gx / (float)W, tcy = (float)gy / (float)H;
    const float uvx = __builtin_fmaf(tcx, 2.0f, -1.0f), uvy = __builtin_fmaf(tcy, 2.0f, -1.0f);
    const f4 wfront = persp_div(mat_vec(P.ipv, f4{uvx, uvy, -1.0f, 1.0f}));
    const f4 wback = persp_div(mat_vec(P.ipv, f4{uvx, uvy, 1.0f, 1.0f}));
    float tnear = 1.0f, tfar = 0.0f, n, f;
    bool vis = false;
    float localNear = 0.0f, localFar = 0.0f;
    intersect_bbox(brick, wfront, wback, n, f);
    f = gmin(P.tmax, f);
    if (n < f) {
        localNear = n;
        localFar = f;
        tnear = gmin(tnear, gmax(0.0f, n));
        tfar = gmax(tfar, f);
        vis = true;
    }
    const int S = P.S;
    int supersegmentNum = 0;
    int iter = 0;
    if (tnear < tfar) {
        float dsteps = __builtin_truncf((tfar - tnear) / nw);
        const int numSteps = (dsteps > 2.0e9f) ? 2000000000 : (int)dsteps;
        float low_thresh = 0.0f, high_thresh = 1.732f;
        bool supsegs_written = false, thresh_found = false;
        const int desired_supsegs = S;
        const int delta = (int)__builtin_floorf(0.15f * (float)S);
        float mid_thresh = 0.0001f;
        bool first_iteration = true;
        while (!thresh_found || !supsegs_written) {
            iter++;
            if (iter > 64) break;
            if (thresh_found) supsegs_written = true;
            const float thresh = mid_thresh;
            int num_terminations = 0;
            bool open = false;
            float startPt = 0.0f, endPt = 0.0f;
            bool lastSample = false, transparent = false;
            f4 adj{0.0f, 0.0f, 0.0f, 0.0f};
            float step = tnear;
            f4 wprev = v4mix(wfront, wback, step - nw);
            float ndc_step = 0.0f;
            int steps_in = 0, steps_tt = 0;
            f4 curV{0.0f, 0.0f, 0.0f, 0.0f};
            for (int i = 0; i < numSteps; ++i, step += nw) {
                if (i == numSteps - 1) lastSample = true;
                const f4 wpos = v4mix(wfront, wback, step);
                if (vis && step > localNear && step < localFar) {
                    transparent = false;
                    const f4 x = sample_volume<DT>(brick, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm, wpos);
                    if (x.x > -0.5f || lastSample) {
                        const float w = adjust_opacity(
                            x.w, len4(wpos.x - wprev.x, wpos.y - wprev.y, wpos.z - wprev.z, wpos.w - wprev.w));
                        if (w <= 0.0f) transparent = true;
                        if (open) {
                            const f4 jp = v4mix(wfront, wback, nw * (float)steps_in);
                            const float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);
                            const float inva = 1.0f / curV.w;
                            adj.x = curV.x * inva;
                            adj.y = curV.y * inva;
                            adj.z = curV.z * inva;
                            adj.w = adjust_opacity(curV.w, 1.0f / segLen);
                            const float ax = adj.x * adj.w, ay = adj.y * adj.w, az = adj.z * adj.w;
                            const float bx = x.x * x.w, by = x.y * x.w, bz = x.z * x.w;
                            const float diff = len3(ax - bx, ay - by, az - bz);
                            if (diff >= thresh) {
                                num_terminations++;
                                open = false;
                                endPt = ndc_step;
                                steps_in = 0;
                                steps_tt = 0;
                                if (thresh_found) {
                                    if (supersegmentNum < S) {
                                        const uint32_t off = (uint32_t)supersegmentNum * o.slot_stride;
                                        o.color[off] = make_float4(adj.x, adj.y, adj.z, adj.w);
                                        o.depth[off] = make_float2(startPt, endPt);
                                    }
                                    octree_update(P, octree, uvx, uvy, startPt, endPt, cx, cy);
                                    supersegmentNum++;
                                }
                            }
                        }
                        if (!open && !transparent) {
                            open = true;
                            const f4 ndc = persp_div(mat_vec(P.pv, wpos));
                            startPt = ndc.z;
                            curV = f4{0.0f, 0.0f, 0.0f, 0.0f};
                        }
                        if (open) {
                            const float t = 1.0f - curV.w;
                            curV.x = __builtin_fmaf(t * x.x, w, curV.x);
                            curV.y = __builtin_fmaf(t * x.y, w, curV.y);
                            curV.z = __builtin_fmaf(t * x.z, w, curV.z);
                            curV.w = __builtin_fmaf(t, w, curV.w);
                            steps_in++;
                            if (!transparent) {
                                steps_tt = steps_in;
                                const f4 wnext = v4mix(wfront, wback, step + nw);
                                const f4 ndc = persp_div(mat_vec(P.pv, wnext));
                                ndc_step = ndc.z;
                            }
                        }
                        if (lastSample && open) {
                            const f4 jp = v4mix(wfront, wback, nw * (float)steps_tt);
                            const float segLen = len4(jp.x - wfront.x, jp.y - wfront.y, jp.z - wfront.z, jp.w - wfront.w);
                            const float inva = 1.0f / curV.w;
                            adj.x = curV.x * inva;
                            adj.y = curV.y * inva;
                            adj.z = curV.z * inva;
                            adj.w = adjust_opacity(curV.w, 1.0f / segLen);
                            num_terminations++;
                            open = false;
                            endPt = ndc_step;
                            steps_in = 0;
                            if (thresh_found) {
                                if (supersegmentNum < S) {
                                    const uint32_t off = (uint32_t)supersegmentNum * o.slot_stride;
                                    o.color[off] = make_float4(adj.x, adj.y, adj.z, adj.w);
                                    o.depth[off] = make_float2(startPt, endPt);
                                }
                                octree_update(P, octree, uvx, uvy, startPt, endPt, cx, cy);
                                supersegmentNum++;
                            }
                        }
                    }
                }
                wprev = wpos;
            }
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
    for (int i = supersegmentNum; i < S; ++i) {
        const uint32_t off = (uint32_t)i * o.slot_stride;
        o.color[off] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        o.depth[off] = make_float2(0.0f, 0.0f);
    }
    if (passes) passes[(uint32_t)gy * (uint32_t)W + (uint32_t)gx] = (uint8_t)iter;
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
    if (d >= P.nstrips) return;
    const int xx = lane & 7, yy = lane >> 3;
    const int xl = xt * 8 + xx, gy = yt * 8 + yy;
    if (xl >= P.strip_w || gy >= P.H) return;
    const int gx = d * P.strip_w + xl;
    const size_t blockE = (size_t)P.strip_tiles * (size_t)P.S * (size_t)P.H * 8;
    const int b = blockIdx.y;
    const size_t blk = (size_t)d * (size_t)P.B + (size_t)b;
    const size_t e0 = blk * blockE + (((size_t)xt * (size_t)P.S) * (size_t)P.H + (size_t)gy) * 8 + (size_t)xx;
    RayOut o{P.color + e0, P.depth + e0, (uint32_t)P.H * 8u};
    vdi_ray<DT>(P, P.bricks[b], P.octree + (size_t)b * P.octree_stride,
                P.passes ? P.passes + (size_t)b * P.passes_stride : nullptr, s_tf, s_cm, gx, gy, o);
}

hipError_t launch_vdi_generate(const VdiGenParams& p, hipStream_t s) {
    const int tiles = p.ytiles * p.nstrips * p.strip_tiles;
    const dim3 grid((tiles + 3) / 4, p.B);
    const size_t lds = (size_t)p.xfer.n_cm * sizeof(float4) + (size_t)p.xfer.n_tf * sizeof(float);
    if (p.B < 1 || p.B > kMaxBricks) return hipErrorInvalidValue;
    for (int b = 1; b < p.B; ++b)   // one voxel type per launch (the kernel is templated on it)
        if (p.bricks[b].dtype != p.bricks[0].dtype) return hipErrorInvalidValue;
    switch (p.bricks[0].dtype) {
    case VOX_U8: hipLaunchKernelGGL(vdi_generate_kernel<VOX_U8>, grid, dim3(256), lds, s, p); break;
    case VOX_U16: hipLaunchKernelGGL(vdi_generate_kernel<VOX_U16>, grid, dim3(256), lds, s, p); break;
    case VOX_F32: hipLaunchKernelGGL(vdi_generate_kernel<VOX_F32>, grid, dim3(256), lds, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
