// plain_generate.hip -- plain-image raymarch for gfx950: VolumeRaycaster.comp +
// AccumulatePlainImage.comp.  One lane per pixel, single pass, front-to-back blend with
// early ray termination at alpha >= 1 (AccumulatePlainImage.comp:11-13): a wave leaves
// its step loop once every lane has terminated (the loop exit is the wave ballot).  All of a rank's
// bricks in one launch; the voxel loads of the next sample are issued before the current one blends.
// Output: packed rgba8 colour and EncodeFloatRGBA(tnear) depth, in the exchange layout
// [d][b][rows][dim0] (strip d = texture rows [d*rows, (d+1)*rows)).
#include "insitu_sampling.h"

#pragma clang fp contract(off)

namespace insitu {

template <int DT>
__global__ __launch_bounds__(256) void plain_generate_kernel(const PlainGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + lut_cm_slots(P.xfer.n_cm));
    stage_luts(P.xfer, s_cm, s_tf);

    // all bricks in one launch (blockIdx.y), 16x16 pixel blocks of 8x8 wave tiles in an XCD-aware order
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bx16 = (P.dim0 + 15) / 16;
    const int blk = xcd_block((int)blockIdx.x, (int)gridDim.x);
    const int b = (int)blockIdx.y;
    const BrickDesc& brick = P.bricks[b];
    const int gx = (blk % bx16) * 16 + (wave & 1) * 8 + (lane & 7);
    const int gy = (blk / bx16) * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (gx >= P.dim0 || gy >= P.dim1) return;

    const float tcx = (float)gx / (float)P.dim0, tcy = (float)gy / (float)P.dim1;   // VolumeRaycaster.comp:96
    const float uvx = __builtin_fmaf(tcx, 2.0f, -1.0f), uvy = __builtin_fmaf(tcy, 2.0f, -1.0f);
    const f4 wfront = persp_div(mat_vec(P.ipv, f4{uvx, uvy, -1.0f, 1.0f}));
    const f4 wback = persp_div(mat_vec(P.ipv, f4{uvx, uvy, 1.0f, 1.0f}));
    float tnear = 1.0f, tfar = 0.0f, n, f;
    bool vis = false;
    intersect_bbox(brick, wfront, wback, n, f);   // VolumeRaycaster.comp:112-125
    f = gmin(P.tmax, f);
    if (n < f) {
        tnear = gmin(tnear, gmax(0.0f, n));
        tfar = gmax(tfar, f);
        vis = true;
    }
    uint32_t col = 0, dep = 0;
    if (tnear < tfar) {
        const float nw = P.nw, fwnw = P.fwnw;
        int numSteps;
        if (fwnw > 0.00001f) {   // VolumeRaycaster.comp:132-135
            float q = det_ln(__builtin_fmaf(tfar, fwnw, nw) / __builtin_fmaf(tnear, fwnw, nw)) / det_ln(1.0f + fwnw);
            numSteps = (q > 2.0e9f) ? 2000000000 : (int)q;
        } else {
            float q = __builtin_truncf((tfar - tnear) / nw + 1.0f);
            numSteps = (q > 2.0e9f) ? 2000000000 : (int)q;
        }
        f4 v{0.0f, 0.0f, 0.0f, 0.0f};
        if (vis && numSteps > 0) {
            // software-pipelined: the voxel loads of sample i+1 are in flight while sample i blends
            // (the sample after an early termination is loaded and dropped)
            float step = tnear;
            VoxelFetch cur;
            fetch_voxels<DT, false>(brick, v4mix(wfront, wback, step), cur);
            for (int i = 0; i < numSteps; ++i) {
                const float step_n = step + __builtin_fmaf(step, fwnw, nw);   // :139
                VoxelFetch nxt;
                fetch_voxels<DT, false>(brick, v4mix(wfront, wback, step_n), nxt);
                const f4 x = classify_sample(voxel_coord(brick, cur), s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm);
                const float t = 1.0f - v.w;   // AccumulatePlainImage.comp:8-9
                v.x = __builtin_fmaf(t * x.x, x.w, v.x);
                v.y = __builtin_fmaf(t * x.y, x.w, v.y);
                v.z = __builtin_fmaf(t * x.z, x.w, v.z);
                v.w = __builtin_fmaf(t, x.w, v.w);
                if (v.w >= 1.0f) break;       // ERT (AccumulatePlainImage.comp:11-13)
                cur = nxt;
                step = step_n;
            }
        }
        col = unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | (unorm8(v.w) << 24);
        dep = encode_depth_rgba8(tnear);
    }
    const int d = gy / P.rows, yl = gy - d * P.rows;
    const size_t o = (((size_t)d * (size_t)P.B + (size_t)b) * (size_t)P.rows + (size_t)yl) * (size_t)P.dim0 + (size_t)gx;
    P.color[o] = col;
    P.depth[o] = dep;
}

hipError_t launch_plain_generate(const PlainGenParams& p, hipStream_t s) {
    if (p.B < 1 || p.B > kMaxBricks) return hipErrorInvalidValue;
    for (int b = 1; b < p.B; ++b)
        if (p.bricks[b].dtype != p.bricks[0].dtype) return hipErrorInvalidValue;
    const dim3 grid((unsigned)(((p.dim0 + 15) / 16) * ((p.dim1 + 15) / 16)), (unsigned)p.B);
    const size_t lds = lut_lds_bytes(p.xfer.n_tf, p.xfer.n_cm);
    switch (p.bricks[0].dtype) {
    case VOX_U8: hipLaunchKernelGGL(plain_generate_kernel<VOX_U8>, grid, dim3(256), lds, s, p); break;
    case VOX_U16: hipLaunchKernelGGL(plain_generate_kernel<VOX_U16>, grid, dim3(256), lds, s, p); break;
    case VOX_F32: hipLaunchKernelGGL(plain_generate_kernel<VOX_F32>, grid, dim3(256), lds, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
