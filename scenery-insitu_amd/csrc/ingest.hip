// ingest.hip -- brick ingest for gfx950: the simulation's x-fastest array (OpenFPM grid view,
// DistributedVolumeRenderer.kt:136-160 / DistributedVolumes.kt:243-250) -> the blocked 8^3
// layout the raymarch kernels sample (insitu_sampling.h).  Re-run every N frames (the reference's
// updateVolumes, DistributedVolumeRenderer.kt:521-527), so it is a bandwidth kernel: one workgroup
// moves a row of 8 blocks along x (8 z-slices x 8 rows x 64 voxels): every wave reads whole 64-voxel
// rows (one contiguous 256-byte request for fp32), the tile is transposed through LDS (rows padded
// to 65 elements: the 8 rows of a block face fall in different banks), and the 8 blocks -- contiguous
// in the blocked layout -- are written as one 16 KiB run.  Padding voxels (dims not a multiple of 8)
// are written as 0 and never sampled (clamp to edge).
#include "insitu_kernels.h"

namespace insitu {

template <typename T>
__global__ __launch_bounds__(256) void brick_ingest_kernel(const T* __restrict__ src, T* __restrict__ dst, int nx,
                                                           int ny, int nz, int nbx, int nby) {
    __shared__ T tile[64][65];   // [z * 8 + y][x within the 8 blocks]
    const int xg = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
    const int lane = (int)(threadIdx.x & 63u), wave = (int)(threadIdx.x >> 6);
    const int gx = xg * 64 + lane;
#pragma unroll 4
    for (int r = wave; r < 64; r += 4) {   // r = z * 8 + y
        const int gy = by * 8 + (r & 7), gz = bz * 8 + (r >> 3);
        T v = T(0);
        if (gx < nx && gy < ny && gz < nz) v = src[((uint32_t)gz * (uint32_t)ny + (uint32_t)gy) * (uint32_t)nx + (uint32_t)gx];
        tile[r][lane] = v;
    }
    __syncthreads();
    const int nblk = min(8, nbx - xg * 8);   // blocks of this row that exist
    const uint32_t base = (((uint32_t)bz * (uint32_t)nby + (uint32_t)by) * (uint32_t)nbx + (uint32_t)xg * 8u) * 512u;
#pragma unroll 4
    for (int i = (int)threadIdx.x; i < nblk * 512; i += 256) {
        const int b = i >> 9, intra = i & 511;
        const int lx = intra & 7, ly = (intra >> 3) & 7, lz = intra >> 6;
        dst[base + (uint32_t)i] = tile[lz * 8 + ly][b * 8 + lx];
    }
}

hipError_t launch_brick_ingest(const void* src, void* dst, int dtype, int nx, int ny, int nz, hipStream_t s) {
    const int nbx = (nx + 7) / 8, nby = (ny + 7) / 8, nbz = (nz + 7) / 8;
    const uint64_t total64 = (uint64_t)nbx * nby * nbz * 512u;
    if (total64 >= (1ull << 32) || nby > 65535 || nbz > 65535) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((nbx + 7) / 8), (unsigned)nby, (unsigned)nbz);
    switch (dtype) {
    case VOX_U8:
        hipLaunchKernelGGL(brick_ingest_kernel<uint8_t>, grid, dim3(256), 0, s, (const uint8_t*)src, (uint8_t*)dst, nx,
                           ny, nz, nbx, nby);
        break;
    case VOX_U16:
        hipLaunchKernelGGL(brick_ingest_kernel<uint16_t>, grid, dim3(256), 0, s, (const uint16_t*)src,
                           (uint16_t*)dst, nx, ny, nz, nbx, nby);
        break;
    case VOX_F32:
        hipLaunchKernelGGL(brick_ingest_kernel<float>, grid, dim3(256), 0, s, (const float*)src, (float*)dst, nx, ny,
                           nz, nbx, nby);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
