// ingest.hip -- brick ingest for gfx950: the simulation's x-fastest array (OpenFPM grid view,
// DistributedVolumeRenderer.kt:136-160 / DistributedVolumes.kt:243-250) -> the blocked 8^3
// layout the raymarch kernels sample (insitu_sampling.h).  One lane per destination voxel:
// 64 lanes write one 8x8 (x,y) face of a block contiguously and read 8 runs of 8 voxels.
// Padding voxels (dims not a multiple of 8) are written as 0 and never sampled (clamp to edge).
#include "insitu_kernels.h"

namespace insitu {

template <typename T>
__global__ __launch_bounds__(256) void brick_ingest_kernel(const T* __restrict__ src, T* __restrict__ dst, int nx,
                                                           int ny, int nz, int nbx, int nby, uint32_t total) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t blk = i >> 9, intra = i & 511u;
        const int lx = (int)(intra & 7u), ly = (int)((intra >> 3) & 7u), lz = (int)(intra >> 6);
        const int bx = (int)(blk % (uint32_t)nbx);
        const int by = (int)((blk / (uint32_t)nbx) % (uint32_t)nby);
        const int bz = (int)(blk / ((uint32_t)nbx * (uint32_t)nby));
        const int x = bx * 8 + lx, y = by * 8 + ly, z = bz * 8 + lz;
        T v = T(0);
        if (x < nx && y < ny && z < nz) v = src[((uint32_t)z * (uint32_t)ny + (uint32_t)y) * (uint32_t)nx + (uint32_t)x];
        dst[i] = v;
    }
}

hipError_t launch_brick_ingest(const void* src, void* dst, int dtype, int nx, int ny, int nz, hipStream_t s) {
    const int nbx = (nx + 7) / 8, nby = (ny + 7) / 8, nbz = (nz + 7) / 8;
    const uint64_t total64 = (uint64_t)nbx * nby * nbz * 512u;
    if (total64 >= (1ull << 32)) return hipErrorInvalidValue;
    const uint32_t total = (uint32_t)total64;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((total64 + 255) / 256, 256u * 64u);
    switch (dtype) {
    case VOX_U8:
        hipLaunchKernelGGL(brick_ingest_kernel<uint8_t>, dim3(blocks), dim3(256), 0, s, (const uint8_t*)src,
                           (uint8_t*)dst, nx, ny, nz, nbx, nby, total);
        break;
    case VOX_U16:
        hipLaunchKernelGGL(brick_ingest_kernel<uint16_t>, dim3(blocks), dim3(256), 0, s, (const uint16_t*)src,
                           (uint16_t*)dst, nx, ny, nz, nbx, nby, total);
        break;
    case VOX_F32:
        hipLaunchKernelGGL(brick_ingest_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)src,
                           (float*)dst, nx, ny, nz, nbx, nby, total);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace insitu
