// insitu_sampling.h -- the scenery volume-sampling segment (sampleVolume / convert /
// intersectBoundingBox) for gfx950, shared by the VDI and plain raymarch kernels.
//
// Bricks live in HBM in a blocked layout: 8x8x8-voxel blocks (2 KiB for fp32), blocks in
// x-fastest order, voxels x-fastest inside a block.  A trilinear footprint (2x2x2 voxels)
// then touches 1-2 128-byte lines per z-slice instead of one line per (y,z) row, and stays
// inside one 4 KiB page.  Filled from the simulation's linear array by brick_ingest_kernel
// (ingest.hip).  Arithmetic follows the numerical contract of insitu_device.h.
#pragma once
#include "insitu_device.h"
#include "insitu_kernels.h"

#pragma clang fp contract(off)

namespace insitu {

template <int DT>
__device__ __forceinline__ float load_voxel(const void* base, uint32_t idx) {
#ifdef INSITU_ABL_NOLOAD
    (void)base;   // ablation (timing only, wrong results): the address arithmetic without the loads
    return (float)(idx & 255u) * 0.001f;
#endif
    if constexpr (DT == VOX_U8) return (float)static_cast<const uint8_t*>(base)[idx];
    else if constexpr (DT == VOX_U16) return (float)static_cast<const uint16_t*>(base)[idx];
    else return static_cast<const float*>(base)[idx];
}

// offset contribution of voxel coordinate i along one axis in the blocked layout
__device__ __forceinline__ uint32_t axis_offset(int i, uint32_t block_stride, uint32_t voxel_stride) {
    return (uint32_t)(i >> 3) * block_stride + (uint32_t)(i & 7) * voxel_stride;
}

// trilinear interpolation at voxel-space (u,v,w), voxel centres at integers, clamp to edge
template <int DT>
__device__ __forceinline__ float trilinear(const BrickDesc& b, float u, float v, float w) {
    int x0, x1, y0, y1, z0, z1;
    float fx, fy, fz;
    texel_pair(u, b.nx, x0, x1, fx);
    texel_pair(v, b.ny, y0, y1, fy);
    texel_pair(w, b.nz, z0, z1, fz);
    const uint32_t sby = 512u * (uint32_t)b.nbx, sbz = sby * (uint32_t)b.nby;
    const uint32_t ax0 = axis_offset(x0, 512u, 1u), ax1 = axis_offset(x1, 512u, 1u);
    const uint32_t ay0 = axis_offset(y0, sby, 8u), ay1 = axis_offset(y1, sby, 8u);
    const uint32_t az0 = axis_offset(z0, sbz, 64u), az1 = axis_offset(z1, sbz, 64u);
    const uint32_t r00 = ay0 + az0, r10 = ay1 + az0, r01 = ay0 + az1, r11 = ay1 + az1;
    const float v000 = load_voxel<DT>(b.data, r00 + ax0), v100 = load_voxel<DT>(b.data, r00 + ax1);
    const float v010 = load_voxel<DT>(b.data, r10 + ax0), v110 = load_voxel<DT>(b.data, r10 + ax1);
    const float v001 = load_voxel<DT>(b.data, r01 + ax0), v101 = load_voxel<DT>(b.data, r01 + ax1);
    const float v011 = load_voxel<DT>(b.data, r11 + ax0), v111 = load_voxel<DT>(b.data, r11 + ax1);
    const float c00 = gmix(v000, v100, fx);
    const float c10 = gmix(v010, v110, fx);
    const float c01 = gmix(v001, v101, fx);
    const float c11 = gmix(v011, v111, fx);
    return gmix(gmix(c00, c10, fy), gmix(c01, c11, fy), fz);
}

// LUT coordinate of a sample: raw + 0.001 with raw = trilinear * conv_k + conv_off
template <int DT>
__device__ __forceinline__ float sample_coord(const BrickDesc& b, f4 wpos) {
    const f4 p = mat_vec(b.im, wpos);
    const float val = trilinear<DT>(b, p.x, p.y, p.z);
    return __builtin_fmaf(val, b.conv_k, b.conv_off) + 0.001f;
}

// The same sample split in two so a raymarch loop can issue the 8 voxel loads of sample i+1
// before it computes sample i (the loads are independent of the segment state): fetch_voxels
// loads, voxel_coord finishes what sample_coord computes -- the identical float operations.
struct VoxelFetch {
    float v[8];
    float fx, fy, fz;
};

template <int DT>
__device__ __forceinline__ void fetch_voxels(const BrickDesc& b, f4 wpos, VoxelFetch& f) {
    const f4 p = mat_vec(b.im, wpos);
    int x0, x1, y0, y1, z0, z1;
    texel_pair(p.x, b.nx, x0, x1, f.fx);
    texel_pair(p.y, b.ny, y0, y1, f.fy);
    texel_pair(p.z, b.nz, z0, z1, f.fz);
    const uint32_t sby = 512u * (uint32_t)b.nbx, sbz = sby * (uint32_t)b.nby;
    const uint32_t ax0 = axis_offset(x0, 512u, 1u), ax1 = axis_offset(x1, 512u, 1u);
    const uint32_t ay0 = axis_offset(y0, sby, 8u), ay1 = axis_offset(y1, sby, 8u);
    const uint32_t az0 = axis_offset(z0, sbz, 64u), az1 = axis_offset(z1, sbz, 64u);
    const uint32_t r00 = ay0 + az0, r10 = ay1 + az0, r01 = ay0 + az1, r11 = ay1 + az1;
    f.v[0] = load_voxel<DT>(b.data, r00 + ax0);
    f.v[1] = load_voxel<DT>(b.data, r00 + ax1);
    f.v[2] = load_voxel<DT>(b.data, r10 + ax0);
    f.v[3] = load_voxel<DT>(b.data, r10 + ax1);
    f.v[4] = load_voxel<DT>(b.data, r01 + ax0);
    f.v[5] = load_voxel<DT>(b.data, r01 + ax1);
    f.v[6] = load_voxel<DT>(b.data, r11 + ax0);
    f.v[7] = load_voxel<DT>(b.data, r11 + ax1);
}

__device__ __forceinline__ float voxel_coord(const BrickDesc& b, const VoxelFetch& f) {
    const float c00 = gmix(f.v[0], f.v[1], f.fx);
    const float c10 = gmix(f.v[2], f.v[3], f.fx);
    const float c01 = gmix(f.v[4], f.v[5], f.fx);
    const float c11 = gmix(f.v[6], f.v[7], f.fx);
    const float val = gmix(gmix(c00, c10, f.fy), gmix(c01, c11, f.fy), f.fz);
    return __builtin_fmaf(val, b.conv_k, b.conv_off) + 0.001f;
}

// The LUTs live in LDS padded by their edge texels: slot j holds texel clamp(j - 1, 0, n - 1) for j in
// [0, n + 2].  A lookup at texel coordinate t then takes slots floor(t) + 1 and floor(t) + 2 with
// floor(t) clamped to [-1, n] as a float (NaN -> -1, as texel_pair) and needs none of texel_pair's
// four integer clamps: the same two texels, the same weight, fewer instructions per sample.
__host__ __device__ constexpr int lut_cm_slots(int n_cm) { return n_cm + 3; }             // float4 slots
__host__ __device__ constexpr int lut_tf_slots(int n_tf) { return (n_tf + 3 + 3) >> 2; }  // in float4 units
__host__ __device__ constexpr size_t lut_lds_bytes(int n_tf, int n_cm) {
    return (size_t)(lut_cm_slots(n_cm) + lut_tf_slots(n_tf)) * 16;
}

__device__ __forceinline__ void lut_pair(float t, int n, int& j, float& frac) {
    float fl = __builtin_floorf(t);
    frac = t - fl;
    fl = __builtin_fminf(__builtin_fmaxf(fl, -1.0f), (float)n);   // fmax(NaN, -1) = -1
    j = (int)fl + 1;
}

// transfer function + colour map at LUT coordinate s: (colormap(s).rgb, TF(s)); padded LDS LUTs
__device__ __forceinline__ f4 classify_sample(float s, const float* s_tf, int n_tf, const float4* s_cm, int n_cm) {
    int j;
    float fr;
    lut_pair(__builtin_fmaf(s, (float)n_tf, -0.5f), n_tf, j, fr);
    const float a = gmix(s_tf[j], s_tf[j + 1], fr);
    lut_pair(__builtin_fmaf(s, (float)n_cm, -0.5f), n_cm, j, fr);
    const float4 c0 = s_cm[j], c1 = s_cm[j + 1];
    return f4{gmix(c0.x, c1.x, fr), gmix(c0.y, c1.y, fr), gmix(c0.z, c1.z, fr), a};
}

// scenery sampleVolume (AccumulateVDI.comp:4, AccumulatePlainImage.comp:3) under the contract:
// raw = trilinear * conv_k + conv_off; a = TF(raw + 0.001); rgb = colormap(raw + 0.001)
template <int DT>
__device__ __forceinline__ f4 sample_volume(const BrickDesc& b, const float* s_tf, int n_tf, const float4* s_cm,
                                            int n_cm, f4 wpos) {
    return classify_sample(sample_coord<DT>(b, wpos), s_tf, n_tf, s_cm, n_cm);
}

// VDIGenerator.comp:64-78 intersectBox on (im*wfront, im*wback - im*wfront, 0, dims)
__device__ __forceinline__ void intersect_bbox(const BrickDesc& b, f4 wfront, f4 wback, float& tnear, float& tfar) {
    const f4 mf = mat_vec(b.im, wfront);
    const f4 mb = mat_vec(b.im, wback);
    const float ro[3] = {mf.x, mf.y, mf.z};
    const float rd[3] = {mb.x - mf.x, mb.y - mf.y, mb.z - mf.z};
    const float bmax[3] = {(float)b.nx, (float)b.ny, (float)b.nz};
    float tmn[3], tmx[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float invR = 1.0f / rd[k];
        const float tbot = invR * (0.0f - ro[k]);
        const float ttop = invR * (bmax[k] - ro[k]);
        tmn[k] = gmin(ttop, tbot);
        tmx[k] = gmax(ttop, tbot);
    }
    tnear = gmax(gmax(tmn[0], tmn[1]), gmax(tmn[0], tmn[2]));
    tfar = gmin(gmin(tmx[0], tmx[1]), gmin(tmx[0], tmx[2]));
}

// stage the transfer function and colour map in LDS (once per block), padded by their edge texels
// (lut_pair): colour map at s_cm[0 .. n_cm + 2], TF at s_tf[0 .. n_tf + 2]
__device__ __forceinline__ void stage_luts(const TransferDesc& x, float4* s_cm, float* s_tf) {
    for (int j = threadIdx.x; j < x.n_cm + 3; j += blockDim.x) {
        const int i = j - 1 < 0 ? 0 : (j - 1 > x.n_cm - 1 ? x.n_cm - 1 : j - 1);
        s_cm[j] = make_float4(x.cmap[4 * i], x.cmap[4 * i + 1], x.cmap[4 * i + 2], x.cmap[4 * i + 3]);
    }
    for (int j = threadIdx.x; j < x.n_tf + 3; j += blockDim.x) {
        const int i = j - 1 < 0 ? 0 : (j - 1 > x.n_tf - 1 ? x.n_tf - 1 : j - 1);
        s_tf[j] = x.tf[i];
    }
    __syncthreads();
}

}  // namespace insitu
