// ingest.hip -- brick ingest for gfx950: the simulation's x-fastest array (OpenFPM grid view,
// DistributedVolumeRenderer.kt:136-160 / DistributedVolumes.kt:243-250) -> the blocked layout with
// halo the raymarch kernels sample (insitu_sampling.h: 9^3-voxel blocks, each holding its 8^3 voxels
// plus the first plane of the next block per axis, the edge voxel repeated past the brick).  Re-run
// every N frames (the reference's updateVolumes, DistributedVolumeRenderer.kt:521-527), so it is a
// bandwidth kernel: one workgroup builds a row of 8 blocks along x -- it reads the 9 z-slices x 9
// rows x 65 voxels they cover (whole source rows, clamped at the brick edge) into LDS and writes the
// 8 blocks, contiguous in the blocked layout, as one 23 KiB run (fp32).
#include "insitu_kernels.h"

namespace insitu {

template <typename T>
__global__ __launch_bounds__(256) void brick_ingest_kernel(const T* __restrict__ src, T* __restrict__ dst, int nx,
                                                           int ny, int nz, int nbx, int nby) {
    constexpr int E = 9, EE = 81, BV = 729;   // block edge with halo, face, voxels
    __shared__ T tile[EE][66];                // [z * 9 + y][x: 64 voxels of 8 blocks + 1 halo (+1 pad)]
    const int xg = (int)blockIdx.x, by = (int)blockIdx.y, bz = (int)blockIdx.z;
    for (int i = (int)threadIdx.x; i < EE * 65; i += 256) {
        const int r = i / 65, c = i - r * 65;
        const int gx = min(xg * 64 + c, nx - 1), gy = min(by * 8 + r % E, ny - 1), gz = min(bz * 8 + r / E, nz - 1);
        tile[r][c] = src[((uint32_t)gz * (uint32_t)ny + (uint32_t)gy) * (uint32_t)nx + (uint32_t)gx];
    }
    __syncthreads();
    const int nblk = min(8, nbx - xg * 8);   // blocks of this row that exist
    const uint32_t base = (((uint32_t)bz * (uint32_t)nby + (uint32_t)by) * (uint32_t)nbx + (uint32_t)xg * 8u) * (uint32_t)BV;
    for (int i = (int)threadIdx.x; i < nblk * BV; i += 256) {
        const int b = i / BV, intra = i - b * BV;
        const int lz = intra / EE, rem = intra - lz * EE;
        const int ly = rem / E, lx = rem - ly * E;
        dst[base + (uint32_t)i] = tile[lz * E + ly][b * 8 + lx];
    }
}

hipError_t launch_brick_ingest(const void* src, void* dst, int dtype, int nx, int ny, int nz, hipStream_t s) {
    const int nbx = (nx + 7) / 8, nby = (ny + 7) / 8, nbz = (nz + 7) / 8;
    const uint64_t total64 = (uint64_t)nbx * nby * nbz * 729u;
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
