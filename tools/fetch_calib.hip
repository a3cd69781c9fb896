// Calibration of rocprofv3's FETCH_SIZE for the search kernel's access pattern (the x2
// gfx950 correction of MI355X_MICROARCH.md is calibrated for 16-B/lane coalesced streaming reads only).
// Known byte counts, buffers far past the 256 MiB Infinity Cache:
//   stream16   every lane one 16-B load, coalesced (the guide's calibrated case: FETCH_SIZE = bytes / 2)
//   scatter32  every lane 32 B (two 16-B loads of one 32-B chunk) at a pseudo-random chunk: the search
//              kernel's cache-chunk replay (each read in a 128-B line no other read of the launch touches,
//              up to hash collisions)
//   scatter8   every lane one 8-B load at a pseudo-random 8-B slot (merged mode's step indices)
// Each kernel prints nothing; the host prints the requested bytes and distinct-line bytes per launch, and
// rocprofv3 --pmc FETCH_SIZE (one pass) gives the counter per launch: tools/fetch_calib.py divides.
// build: hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o tools/fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix64(uint64_t x) {   // splitmix64 finaliser
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

__global__ void stream16(const float4* __restrict__ src, uint64_t n, float* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    if (i < n) { const float4 v = src[i]; acc = v.x + v.y + v.z + v.w; }
    if (acc == 1234.5f) out[0] = acc;   // (never: keeps the load)
}

__global__ void scatter32(const float4* __restrict__ src, uint64_t nchunks, uint64_t nreads, uint64_t seed, float* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    if (i < nreads) {
        const uint64_t c = mix64(i ^ seed) % nchunks;
        const float4 a = src[2 * c], b = src[2 * c + 1];
        acc = a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w;
    }
    if (acc == 1234.5f) out[0] = acc;
}

__global__ void scatter8(const float2* __restrict__ src, uint64_t nslots, uint64_t nreads, uint64_t seed, float* out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float acc = 0.0f;
    if (i < nreads) { const float2 v = src[mix64(i ^ seed) % nslots]; acc = v.x + v.y; }
    if (acc == 1234.5f) out[0] = acc;
}

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
    const size_t bytes = (size_t)4 << 30;   // 4 GiB: every pattern far past the Infinity Cache
    void* buf = nullptr;
    float* out = nullptr;
    CHK(hipMalloc(&buf, bytes));
    CHK(hipMalloc(&out, sizeof(float)));
    CHK(hipMemset(buf, 0, bytes));
    CHK(hipDeviceSynchronize());
    const uint64_t n16 = bytes / 16;                  // stream16: the whole buffer once
    const uint64_t nchunks = bytes / 32, n32 = (uint64_t)1 << 24;   // 16 M reads of 32 B over 128 M chunks
    const uint64_t nslots = bytes / 8, n8 = (uint64_t)1 << 24;
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(stream16, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, 0, (const float4*)buf, n16, out);
        hipLaunchKernelGGL(scatter32, dim3((unsigned)((n32 + 255) / 256)), dim3(256), 0, 0, (const float4*)buf, nchunks, n32,
                           (uint64_t)rep * 0x9e3779b97f4a7c15ull, out);
        hipLaunchKernelGGL(scatter8, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, 0, (const float2*)buf, nslots, n8,
                           (uint64_t)rep * 0x632be59bd9b4e019ull, out);
        CHK(hipGetLastError());
        CHK(hipDeviceSynchronize());
    }
    // requested bytes per launch, and the 128-B lines they touch (distinct up to hash collisions)
    std::printf("{\"stream16\": {\"bytes\": %llu, \"lines_bytes\": %llu}, "
                "\"scatter32\": {\"bytes\": %llu, \"lines_bytes\": %llu}, "
                "\"scatter8\": {\"bytes\": %llu, \"lines_bytes\": %llu}}\n",
                (unsigned long long)(n16 * 16), (unsigned long long)(n16 * 16),
                (unsigned long long)(n32 * 32), (unsigned long long)(n32 * 128),
                (unsigned long long)(n8 * 8), (unsigned long long)(n8 * 128));
    CHK(hipFree(buf));
    CHK(hipFree(out));
    return 0;
}
