// plain_generate.hip -- plain-image raymarch for gfx950: VolumeRaycaster.comp +
// AccumulatePlainImage.comp.  One lane per pixel, single pass, front-to-back blend with
// early ray termination at alpha >= 1 (AccumulatePlainImage.comp:11-13): a wave leaves
// its step loop once every lane has terminated (the loop exit is the wave ballot).
// Output: packed rgba8 colour and EncodeFloatRGBA(tnear) depth, in the exchange layout
// [d][b][rows][dim0] (strip d = texture rows [d*rows, (d+1)*rows)).
#include "insitu_device.h"
#include "insitu_kernels.h"

#pragma clang fp contract(off)

namespace insitu {

template <int DT>
__device__ __forceinline__ float load_voxel_p(const void* base, uint32_t idx) {
    if constexpr (DT == VOX_U8) return (float)static_cast<const uint8_t*>(base)[idx];
    else if constexpr (DT == VOX_U16) return (float)static_cast<const uint16_t*>(base)[idx];
    else return static_cast<const float*>(base)[idx];
}

template <int DT>
__device__ __forceinline__ f4 sample_volume_p(const BrickDesc& b, const float* s_tf, int n_tf, const float4* s_cm,
                                              int n_cm, f4 wpos) {
    f4 p = mat_vec(b.im, wpos);
    int x0, x1, y0, y1, z0, z1;
    float fx, fy, fz;
    texel_pair(p.x, b.nx, x0, x1, fx);
    texel_pair(p.y, b.ny, y0, y1, fy);
    texel_pair(p.z, b.nz, z0, z1, fz);
    const uint32_t sy = (uint32_t)b.nx, sz = (uint32_t)b.nx * (uint32_t)b.ny;
    const uint32_t r00 = (uint32_t)z0 * sz + (uint32_t)y0 * sy, r10 = (uint32_t)z0 * sz + (uint32_t)y1 * sy;
    const uint32_t r01 = (uint32_t)z1 * sz + (uint32_t)y0 * sy, r11 = (uint32_t)z1 * sz + (uint32_t)y1 * sy;
    float c00 = gmix(load_voxel_p<DT>(b.data, r00 + x0), load_voxel_p<DT>(b.data, r00 + x1), fx);
    float c10 = gmix(load_voxel_p<DT>(b.data, r10 + x0), load_voxel_p<DT>(b.data, r10 + x1), fx);
    float c01 = gmix(load_voxel_p<DT>(b.data, r01 + x0), load_voxel_p<DT>(b.data, r01 + x1), fx);
    float c11 = gmix(load_voxel_p<DT>(b.data, r11 + x0), load_voxel_p<DT>(b.data, r11 + x1), fx);
    float val = gmix(gmix(c00, c10, fy), gmix(c01, c11, fy), fz);
    float s = __builtin_fmaf(val, b.conv_k, b.conv_off) + 0.001f;
    int i0, i1;
    float fr;
    texel_pair(__builtin_fmaf(s, (float)n_tf, -0.5f), n_tf, i0, i1, fr);
    float a = gmix(s_tf[i0], s_tf[i1], fr);
    texel_pair(__builtin_fmaf(s, (float)n_cm, -0.5f), n_cm, i0, i1, fr);
    float4 c0 = s_cm[i0], c1 = s_cm[i1];
    return f4{gmix(c0.x, c1.x, fr), gmix(c0.y, c1.y, fr), gmix(c0.z, c1.z, fr), a};
}

template <int DT>
__global__ __launch_bounds__(256) void plain_generate_kernel(const PlainGenParams P) {
    extern __shared__ __attribute__((aligned(16))) float4 smem[];
    float4* s_cm = smem;
    float* s_tf = reinterpret_cast<float*>(smem + P.xfer.n_cm);
    for (int i = threadIdx.x; i < P.xfer.n_cm; i += blockDim.x)
        s_cm[i] = make_float4(P.xfer.cmap[4 * i], P.xfer.cmap[4 * i + 1], P.xfer.cmap[4 * i + 2], P.xfer.cmap[4 * i + 3]);
    for (int i = threadIdx.x; i < P.xfer.n_tf; i += blockDim.x) s_tf[i] = P.xfer.tf[i];
    __syncthreads();

    // 16x16 pixel block, 8x8 tile per wave
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int gx = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int gy = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    if (gx >= P.dim0 || gy >= P.dim1) return;

    const float tcx = (float)gx / (float)P.dim0, tcy = (float)gy / (float)P.dim1;   // VolumeRaycaster.comp:96
    const float uvx = __builtin_fmaf(tcx, 2.0f, -1.0f), uvy = __builtin_fmaf(tcy, 2.0f, -1.0f);
    const f4 wfront = persp_div(mat_vec(P.ipv, f4{uvx, uvy, -1.0f, 1.0f}));
    const f4 wback = persp_div(mat_vec(P.ipv, f4{uvx, uvy, 1.0f, 1.0f}));
    float tnear = 1.0f, tfar = 0.0f, n, f;
    bool vis = false;
    {
        // VolumeRaycaster.comp:112-125 (intersectBox as VDIGenerator.comp:64-78)
        f4 mf = mat_vec(P.brick.im, wfront), mb = mat_vec(P.brick.im, wback);
        float ro[3] = {mf.x, mf.y, mf.z}, rd[3] = {mb.x - mf.x, mb.y - mf.y, mb.z - mf.z};
        float bmax[3] = {(float)P.brick.nx, (float)P.brick.ny, (float)P.brick.nz};
        float tmn[3], tmx[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float invR = 1.0f / rd[k];
            float tbot = invR * (0.0f - ro[k]);
            float ttop = invR * (bmax[k] - ro[k]);
            tmn[k] = gmin(ttop, tbot);
            tmx[k] = gmax(ttop, tbot);
        }
        n = gmax(gmax(tmn[0], tmn[1]), gmax(tmn[0], tmn[2]));
        f = gmin(gmin(tmx[0], tmx[1]), gmin(tmx[0], tmx[2]));
    }
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
        float step = tnear;
        f4 v{0.0f, 0.0f, 0.0f, 0.0f};
        if (vis) {
            for (int i = 0; i < numSteps; ++i, step = step + __builtin_fmaf(step, fwnw, nw)) {
                const f4 wpos = v4mix(wfront, wback, step);
                const f4 x = sample_volume_p<DT>(P.brick, s_tf, P.xfer.n_tf, s_cm, P.xfer.n_cm, wpos);
                const float t = 1.0f - v.w;   // AccumulatePlainImage.comp:8-9
                v.x = __builtin_fmaf(t * x.x, x.w, v.x);
                v.y = __builtin_fmaf(t * x.y, x.w, v.y);
                v.z = __builtin_fmaf(t * x.z, x.w, v.z);
                v.w = __builtin_fmaf(t, x.w, v.w);
                if (v.w >= 1.0f) break;       // ERT (AccumulatePlainImage.comp:11-13)
            }
        }
        col = unorm8(v.x) | (unorm8(v.y) << 8) | (unorm8(v.z) << 16) | (unorm8(v.w) << 24);
        dep = encode_depth_rgba8(tnear);
    }
    const int d = gy / P.rows, yl = gy - d * P.rows;
    const size_t o = (((size_t)d * (size_t)P.B + (size_t)P.b) * (size_t)P.rows + (size_t)yl) * (size_t)P.dim0 + (size_t)gx;
    P.color[o] = col;
    P.depth[o] = dep;
}

hipError_t launch_plain_generate(const PlainGenParams& p, hipStream_t s) {
    dim3 grid((p.dim0 + 15) / 16, (p.dim1 + 15) / 16);
    const size_t lds = (size_t)p.xfer.n_cm * sizeof(float4) + (size_t)p.xfer.n_tf * sizeof(float);
    switch (p.brick.dtype) {
    case VOX_U8: hipLaunchKernelGGL(plain_generate_kernel<VOX_U8>, grid, dim3(256), lds, s, p); break;
    case VOX_U16: hipLaunchKernelGGL(plain_generate_kernel<VOX_U16>, grid, dim3(256), lds, s, p); break;
    case VOX_F32: hipLaunchKernelGGL(plain_generate_kernel<VOX_F32>, grid, dim3(256), lds, s, p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
