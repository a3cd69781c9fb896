// insitu_sampling.h -- the scenery volume-sampling segment (sampleVolume / convert /
// intersectBoundingBox) for gfx950, shared by the VDI and plain raymarch kernels.
//
// Bricks live in HBM in a blocked layout with a halo: 9x9x9-voxel blocks, block (bx,by,bz) holding
// voxels [8bx, 8bx+8] x [8by, 8by+8] x [8bz, 8bz+8] (its 8^3 own voxels plus the first plane of the
// next block along each axis; past the brick edge the edge voxel repeated), blocks x-fastest, voxels
// x-fastest inside a block.  A trilinear footprint (2x2x2 voxels) then lies in ONE block, and its
// x-pairs are adjacent: a sample is four 8-byte loads (fp32) instead of eight 4-byte gathers -- half
// the addresses for the texture-address unit, which the 8-gather form kept busy --
// touching 2-4 lines inside one 3 KiB block.  Filled from the simulation's linear array by
// brick_ingest_kernel (ingest.hip).  Arithmetic follows the numerical contract of insitu_device.h.
#pragma once
#include "insitu_device.h"
#include "insitu_kernels.h"

#pragma clang fp contract(off)

namespace insitu {

constexpr uint32_t kBlockEdge = 9;     // voxels per block edge, halo included
constexpr uint32_t kBlockVox = 729;    // voxels per block

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

// voxels idx and idx + 1 (adjacent along x inside a block); fp32 as one 8-byte load at 4-byte
// alignment (gfx950 global loads need dword alignment only)
template <int DT>
__device__ __forceinline__ void load_pair(const void* base, uint32_t idx, float& lo, float& hi) {
#ifdef INSITU_ABL_NOLOAD
    lo = load_voxel<DT>(base, idx);
    hi = load_voxel<DT>(base, idx + 1);
    return;
#endif
    if constexpr (DT == VOX_F32) {
        typedef float v2f_a4 __attribute__((ext_vector_type(2), aligned(4)));
        const v2f_a4 v = *reinterpret_cast<const v2f_a4*>(static_cast<const float*>(base) + idx);
        lo = v.x;
        hi = v.y;
    } else {
        lo = load_voxel<DT>(base, idx);
        hi = load_voxel<DT>(base, idx + 1);
    }
}

// A sample split in two so a raymarch loop can issue the voxel loads of sample i+1 before it
// computes sample i (the loads are independent of the segment state): fetch_voxels loads,
// voxel_coord finishes the trilinear interpolation and the converter.
struct VoxelFetch {
    float v[8];
    float fx, fy, fz;
    bool xedge;   // x1 == x0 (clamp to edge along x): the pairs' upper voxels are replaced by the lower ones
};

// texel_pair (insitu_device.h) as min / max: floor(t) clamped to [-1, n] (NaN -> -1), i0 = clamp(i, 0, n - 1),
// i1 = clamp(i + 1, 0, n - 1) -- the same texels and fraction, fewer compares and selects
__device__ __forceinline__ void texel_pair_mm(float t, int n, int& i0, int& i1, float& frac) {
    const float fl = __builtin_floorf(t);
    frac = t - fl;
    const int i = (int)__builtin_fminf(__builtin_fmaxf(fl, -1.0f), (float)n);   // fmaxf(NaN, -1) = -1
    i0 = min(max(i, 0), n - 1);
    i1 = min(max(i + 1, 0), n - 1);
}

// the 2x2x2 footprint at voxel-space (u, v, w) (voxel centres at integers, clamp to edge): voxels
// (x0|x1, y0|y1, z0|z1) of texel_pair, all inside block (x0/8, y0/8, z0/8).  The loads are issued here and
// not waited on: x1 == x0 (the brick's x faces) is applied by voxel_coord, after the voxels arrived (a
// branch here made the wave wait for its loads at once whenever one lane sat on an x face).
// EDGE_SELECT = false: the x faces as a branch right after the loads (the plain raymarch: there the compiler
// then keeps two samples' loads in flight, 4.2 against 5.5 ms per frame with the select)
template <int DT, bool EDGE_SELECT = true>
__device__ __forceinline__ void fetch_footprint(const BrickDesc& b, float u, float v, float w, VoxelFetch& f) {
    int x0, x1, y0, y1, z0, z1;
    texel_pair_mm(u, b.nx, x0, x1, f.fx);
    texel_pair_mm(v, b.ny, y0, y1, f.fy);
    texel_pair_mm(w, b.nz, z0, z1, f.fz);
    const uint32_t bx = (uint32_t)x0 >> 3, by = (uint32_t)y0 >> 3, bz = (uint32_t)z0 >> 3;
    const uint32_t base = ((bz * (uint32_t)b.nby + by) * (uint32_t)b.nbx + bx) * kBlockVox + ((uint32_t)x0 & 7u);
    // y1, z1 are y0 or y0 + 1 (<= 8 inside the block); x1 is x0 + 1 except at the edges, where it
    // equals x0: the upper edge reads the repeated edge voxel of the halo, the lower one takes v0
    const uint32_t oy0 = ((uint32_t)y0 & 7u) * kBlockEdge, oy1 = ((uint32_t)y1 - (by << 3)) * kBlockEdge;
    const uint32_t oz0 = ((uint32_t)z0 & 7u) * (kBlockEdge * kBlockEdge);
    const uint32_t oz1 = ((uint32_t)z1 - (bz << 3)) * (kBlockEdge * kBlockEdge);
#ifdef INSITU_ABL_QUAD
    // timing ablation only (wrong values): two 16-byte loads per sample, the address count of a layout that
    // stores each voxel's 2x2 x-y footprint together (the quad layout the ablation prices)
    if constexpr (DT == VOX_F32) {
        typedef float v4f_a4 __attribute__((ext_vector_type(4), aligned(4)));
        const v4f_a4 qa = *reinterpret_cast<const v4f_a4*>(static_cast<const float*>(b.data) + base + oz0 + oy0);
        const v4f_a4 qb = *reinterpret_cast<const v4f_a4*>(static_cast<const float*>(b.data) + base + oz1 + oy0);
        f.v[0] = qa.x; f.v[1] = qa.y; f.v[2] = qa.z; f.v[3] = qa.w;
        f.v[4] = qb.x; f.v[5] = qb.y; f.v[6] = qb.z; f.v[7] = qb.w;
        (void)oy1;
    } else
#endif
    {
    load_pair<DT>(b.data, base + oz0 + oy0, f.v[0], f.v[1]);
    load_pair<DT>(b.data, base + oz0 + oy1, f.v[2], f.v[3]);
    load_pair<DT>(b.data, base + oz1 + oy0, f.v[4], f.v[5]);
    load_pair<DT>(b.data, base + oz1 + oy1, f.v[6], f.v[7]);
    }
    if constexpr (EDGE_SELECT) {
        f.xedge = x1 == x0;
    } else {
        f.xedge = false;
        if (x1 == x0) {
            f.v[1] = f.v[0];
            f.v[3] = f.v[2];
            f.v[5] = f.v[4];
            f.v[7] = f.v[6];
        }
    }
}

template <int DT, bool EDGE_SELECT = true>
__device__ __forceinline__ void fetch_voxels(const BrickDesc& b, f4 wpos, VoxelFetch& f) {
    const f4 p = mat_vec(b.im, wpos);
    fetch_footprint<DT, EDGE_SELECT>(b, p.x, p.y, p.z, f);
}

// LUT coordinate of the fetched sample: raw + 0.001 with raw = trilinear * conv_k + conv_off
__device__ __forceinline__ float voxel_coord(const BrickDesc& b, const VoxelFetch& f) {
    const float c00 = gmix(f.v[0], f.xedge ? f.v[0] : f.v[1], f.fx);
    const float c10 = gmix(f.v[2], f.xedge ? f.v[2] : f.v[3], f.fx);
    const float c01 = gmix(f.v[4], f.xedge ? f.v[4] : f.v[5], f.fx);
    const float c11 = gmix(f.v[6], f.xedge ? f.v[6] : f.v[7], f.fx);
    const float val = gmix(gmix(c00, c10, f.fy), gmix(c01, c11, f.fy), f.fz);
    return __builtin_fmaf(val, b.conv_k, b.conv_off) + 0.001f;
}

// trilinear interpolation at voxel-space (u,v,w), voxel centres at integers, clamp to edge
template <int DT>
__device__ __forceinline__ float trilinear(const BrickDesc& b, float u, float v, float w) {
    VoxelFetch f;
    fetch_footprint<DT>(b, u, v, w, f);
    const float c00 = gmix(f.v[0], f.xedge ? f.v[0] : f.v[1], f.fx);
    const float c10 = gmix(f.v[2], f.xedge ? f.v[2] : f.v[3], f.fx);
    const float c01 = gmix(f.v[4], f.xedge ? f.v[4] : f.v[5], f.fx);
    const float c11 = gmix(f.v[6], f.xedge ? f.v[6] : f.v[7], f.fx);
    return gmix(gmix(c00, c10, f.fy), gmix(c01, c11, f.fy), f.fz);
}

// LUT coordinate of a sample: raw + 0.001 with raw = trilinear * conv_k + conv_off
template <int DT>
__device__ __forceinline__ float sample_coord(const BrickDesc& b, f4 wpos) {
    VoxelFetch f;
    fetch_voxels<DT>(b, wpos, f);
    return voxel_coord(b, f);
}

// The LUTs live in LDS padded by their edge texels: slot j holds texel clamp(j - 1, 0, n - 1) for j in
// [0, n + 2].  A lookup at texel coordinate t then takes slots floor(t) + 1 and floor(t) + 2 with
// floor(t) clamped to [-1, n] as a float (NaN -> -1, as texel_pair) and needs none of texel_pair's
// four integer clamps: the same two texels, the same weight, fewer instructions per sample.
//
// LDS image (INSITU_LUT_LAYOUT).  Every lane of a wave looks up its own coordinate, so the reads are
// gathers whose cost is LDS cycles: per lane-group one cycle plus one per extra address on a busy
// bank (MI355X_MICROARCH.md LDS).  The two slots a lookup blends are stored next to each other as
// one PAIR entry, so a lookup is a single wide read instead of two:
//   0: colour map float4 slots, TF float slots (ds_read2_b32 + 2 x ds_read_b128: 12 cycles per wave
//      conflict-free, TF banks mod 32)
//   1: TF pairs float2 {slot j, slot j+1} (ds_read_b64: 2 cycles, banks mod 64) and colour-map pairs of
//      32 B {r_j, g_j, b_j, r_j+1}, {g_j+1, b_j+1, -, -} (ds_read_b128 + ds_read_b64: 6 cycles) -- the
//      colour map's alpha is never read (the TF gives the opacity)
//   2: TF pairs as 1, colour-map pairs as three float2 arrays R, G, B (3 x ds_read_b64: 6 cycles)
//   3: TF pairs as 1, colour-map float4 slots as 0 (ds_read_b64 + 2 x ds_read_b128)
//   4: TF pairs as 1, colour-map pairs as {r_j, g_j, r_j+1, g_j+1} float4s and {b_j, b_j+1} float2s
//      (ds_read_b128 + ds_read_b64: the red/green blends are one packed fma pair)
// Same texels, same weights, same float operations: the layout changes no result.
#ifndef INSITU_LUT_LAYOUT
#define INSITU_LUT_LAYOUT 2
#endif
__host__ __device__ constexpr int lut_cm_slots(int n_cm) {   // float4 slots of the colour-map part
    return (INSITU_LUT_LAYOUT == 0 || INSITU_LUT_LAYOUT == 3) ? n_cm + 3
           : (INSITU_LUT_LAYOUT == 1 ? 2 * (n_cm + 2)
              : (INSITU_LUT_LAYOUT == 4 ? (n_cm + 2) + (n_cm + 3) / 2 : (3 * (n_cm + 2) + 1) / 2));
}
__host__ __device__ constexpr int lut_tf_slots(int n_tf) {   // in float4 units
    return INSITU_LUT_LAYOUT == 0 ? (n_tf + 3 + 3) >> 2 : (n_tf + 2 + 1) >> 1;
}
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
#if INSITU_LUT_LAYOUT == 4
    // both lookups' texel coordinates, fractions and blends in pairs {TF, colour map}
    const f2v tc = pk_fma(f2v{s, s}, f2v{(float)n_tf, (float)n_cm}, f2v{-0.5f, -0.5f});
    const f2v fl = f2v{__builtin_floorf(tc.x), __builtin_floorf(tc.y)};
    const f2v fr = tc - fl;
    const int jt = (int)__builtin_fminf(__builtin_fmaxf(fl.x, -1.0f), (float)n_tf) + 1;   // lut_pair
    const int jc = (int)__builtin_fminf(__builtin_fmaxf(fl.y, -1.0f), (float)n_cm) + 1;
    const float2 tp = reinterpret_cast<const float2*>(s_tf)[jt];
    const float4 rg = s_cm[jc];
    const float2 bb = reinterpret_cast<const float2*>(s_cm + (n_cm + 2))[jc];
    const f2v omf = f2v{1.0f, 1.0f} - fr;
    const f2v ab = pk_fma(f2v{tp.y, bb.y}, fr, f2v{tp.x, bb.x} * omf);                      // {alpha, blue}
    const f2v c_rg = pk_fma(f2v{rg.z, rg.w}, f2v{fr.y, fr.y}, f2v{rg.x, rg.y} * omf.y);     // {red, green}
    return f4{c_rg.x, c_rg.y, ab.y, ab.x};
#else
    int j;
    float fr;
    lut_pair(__builtin_fmaf(s, (float)n_tf, -0.5f), n_tf, j, fr);
#if INSITU_LUT_LAYOUT == 0
    const float a = gmix(s_tf[j], s_tf[j + 1], fr);
#else
    const float2 tp = reinterpret_cast<const float2*>(s_tf)[j];
    const float a = gmix(tp.x, tp.y, fr);
#endif
    lut_pair(__builtin_fmaf(s, (float)n_cm, -0.5f), n_cm, j, fr);
#if INSITU_LUT_LAYOUT == 0 || INSITU_LUT_LAYOUT == 3
    const float4 c0 = s_cm[j], c1 = s_cm[j + 1];
    return f4{gmix(c0.x, c1.x, fr), gmix(c0.y, c1.y, fr), gmix(c0.z, c1.z, fr), a};
#elif INSITU_LUT_LAYOUT == 1
    const float4 p0 = s_cm[2 * j];
    const float2 p1 = *reinterpret_cast<const float2*>(s_cm + 2 * j + 1);
    return f4{gmix(p0.x, p0.w, fr), gmix(p0.y, p1.x, fr), gmix(p0.z, p1.y, fr), a};
#else
    const float2* R = reinterpret_cast<const float2*>(s_cm);
    const float2 r = R[j], g = R[(n_cm + 2) + j], b = R[2 * (n_cm + 2) + j];
    return f4{gmix(r.x, r.y, fr), gmix(g.x, g.y, fr), gmix(b.x, b.y, fr), a};
#endif
#endif
}

#ifdef INSITU_ABL_CLASSIFY2
// timing ablation only: classify_sample's index and blend arithmetic with the LDS reads replaced by
// values computed from the indices (wrong colours)
__device__ __forceinline__ f4 classify_fake(float s, int n_tf, int n_cm) {
    int j;
    float fr;
    lut_pair(__builtin_fmaf(s, (float)n_tf, -0.5f), n_tf, j, fr);
    const float t0 = (float)j * 1e-3f;
    const float a = gmix(t0, t0 + 1e-3f, fr);
    lut_pair(__builtin_fmaf(s, (float)n_cm, -0.5f), n_cm, j, fr);
    const float c0 = (float)j * 1e-3f;
    return f4{gmix(c0, c0 + 1e-3f, fr), gmix(c0 + 2e-3f, c0 + 3e-3f, fr), gmix(c0 + 4e-3f, c0 + 5e-3f, fr), a};
}
#endif

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
// (lut_pair), in the INSITU_LUT_LAYOUT image
__device__ __forceinline__ void stage_luts(const TransferDesc& x, float4* s_cm, float* s_tf) {
    auto cm_tex = [&](int slot) {   // colour-map texel of padded slot `slot`
        const int i = slot - 1 < 0 ? 0 : (slot - 1 > x.n_cm - 1 ? x.n_cm - 1 : slot - 1);
        return make_float4(x.cmap[4 * i], x.cmap[4 * i + 1], x.cmap[4 * i + 2], x.cmap[4 * i + 3]);
    };
    auto tf_tex = [&](int slot) {
        const int i = slot - 1 < 0 ? 0 : (slot - 1 > x.n_tf - 1 ? x.n_tf - 1 : slot - 1);
        return x.tf[i];
    };
#if INSITU_LUT_LAYOUT == 0
    for (int j = threadIdx.x; j < x.n_cm + 3; j += blockDim.x) s_cm[j] = cm_tex(j);
    for (int j = threadIdx.x; j < x.n_tf + 3; j += blockDim.x) s_tf[j] = tf_tex(j);
#else
#if INSITU_LUT_LAYOUT == 3
    for (int j = threadIdx.x; j < x.n_cm + 3; j += blockDim.x) s_cm[j] = cm_tex(j);
#else
    for (int j = threadIdx.x; j < x.n_cm + 2; j += blockDim.x) {
        const float4 a = cm_tex(j), b = cm_tex(j + 1);
#if INSITU_LUT_LAYOUT == 4
        s_cm[j] = make_float4(a.x, a.y, b.x, b.y);
        reinterpret_cast<float2*>(s_cm + (x.n_cm + 2))[j] = make_float2(a.z, b.z);
#elif INSITU_LUT_LAYOUT == 1
        s_cm[2 * j] = make_float4(a.x, a.y, a.z, b.x);
        s_cm[2 * j + 1] = make_float4(b.y, b.z, 0.0f, 0.0f);
#else
        float2* R = reinterpret_cast<float2*>(s_cm);
        R[j] = make_float2(a.x, b.x);
        R[(x.n_cm + 2) + j] = make_float2(a.y, b.y);
        R[2 * (x.n_cm + 2) + j] = make_float2(a.z, b.z);
#endif
    }
#endif
    for (int j = threadIdx.x; j < x.n_tf + 2; j += blockDim.x)
        reinterpret_cast<float2*>(s_tf)[j] = make_float2(tf_tex(j), tf_tex(j + 1));
#endif
    __syncthreads();
}

}  // namespace insitu
