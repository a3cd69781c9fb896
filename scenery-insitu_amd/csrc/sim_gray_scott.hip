// sim_gray_scott.hip -- the synthetic simulation that stands in for OpenFPM's Gray-Scott example
// (README.md:4, artwork/*.gif): explicit-Euler 3-D reaction-diffusion on a periodic n^3 grid, one
// fused kernel per time step (both fields read once, written once) instead of the ~20 elementwise
// tensor ops of the torch formulation in insitu_amd/scene.py.  NOT part of the rendering path: it only
// produces the bricks the benchmark renders (libinsitu_sim.so, loaded by scene.gray_scott for device
// tensors).  Same formula and operation order as scene.gray_scott:
//   lap(a) = a[z-1] + a[z+1] + a[y-1] + a[y+1] + a[x-1] + a[x+1] - 6a   (left to right)
//   uvv = u*v*v;  u' = u + dt*(Du*lap(u) - uvv + F*(1-u));  v' = v + dt*(Dv*lap(v) + uvv - (F+k)*v)
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace {

__global__ __launch_bounds__(256) void gray_scott_step_kernel(const float* __restrict__ u, const float* __restrict__ v,
                                                              float* __restrict__ u2, float* __restrict__ v2, int n,
                                                              float F, float Fk, float Du, float Dv, float dt) {
    const uint32_t nn = (uint32_t)n;
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y, z = blockIdx.z;
    if (x >= nn) return;
    const uint32_t i = (z * nn + y) * nn + x;
    const uint32_t zm = ((z + nn - 1) % nn * nn + y) * nn + x, zp = ((z + 1) % nn * nn + y) * nn + x;
    const uint32_t ym = (z * nn + (y + nn - 1) % nn) * nn + x, yp = (z * nn + (y + 1) % nn) * nn + x;
    const uint32_t xm = i - x + (x + nn - 1) % nn, xp = i - x + (x + 1) % nn;
    const float uc = u[i], vc = v[i];
    const float lu = (((((u[zm] + u[zp]) + u[ym]) + u[yp]) + u[xm]) + u[xp]) - 6.0f * uc;
    const float lv = (((((v[zm] + v[zp]) + v[ym]) + v[yp]) + v[xm]) + v[xp]) - 6.0f * vc;
    const float uvv = (uc * vc) * vc;
    u2[i] = uc + dt * ((Du * lu - uvv) + F * (1.0f - uc));
    v2[i] = vc + dt * ((Dv * lv + uvv) - Fk * vc);
}

}  // namespace

extern "C" {

// `steps` explicit-Euler steps of the n^3 fields u, v (device pointers, index [z][y][x]), ping-ponging
// through u2, v2; the result is left in u, v.  0 = success.
int insitu_sim_gray_scott(float* u, float* v, float* u2, float* v2, int n, int steps, float F, float k, float Du,
                          float Dv, float dt, void* stream) {
    if (!u || !v || !u2 || !v2 || n < 3 || n > 1625 || steps < 0) return -1;   // n^3 < 2^32
    hipStream_t s = (hipStream_t)stream;
    const uint64_t total = (uint64_t)n * n * n;
    const dim3 grid((unsigned)((n + 255) / 256), (unsigned)n, (unsigned)n);
    const float Fk = F + k;
    for (int t = 0; t < steps; ++t) {
        hipLaunchKernelGGL(gray_scott_step_kernel, grid, dim3(256), 0, s, u, v, u2, v2, n, F, Fk, Du, Dv, dt);
        float* a = u; u = u2; u2 = a;
        float* b = v; v = v2; v2 = b;
    }
    if (steps & 1) {   // the last step wrote the scratch pair: copy back
        if (hipMemcpyAsync(u2, u, total * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) return -3;
        if (hipMemcpyAsync(v2, v, total * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) return -3;
    }
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"
