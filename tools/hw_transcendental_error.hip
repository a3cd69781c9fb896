// Measures the error of gfx950's hardware log2 / exp2 (v_log_f32 / v_exp_f32) exhaustively over
// the arguments the filtered supersegment test gives them (vdi_generate.hip, approx_diff_sq):
//   log2(x) for every float x in [2^-26, 1)        (x = 1 - accumulated opacity)
//   exp2(y) for every float y in [-160, 0]          (y = log2(1 - a) / segment length)
// against log2 / exp2 evaluated in double precision (correct to far below a float ulp).
// Prints one JSON line: the worst absolute and relative errors, and the worst error in units of the
// float ulp of the exact value.  The bound the filter margin is built on.
// build: hipcc -O3 --offload-arch=gfx950 tools/hw_transcendental_error.hip -o /tmp/hwerr
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

struct Acc {
    unsigned long long max_abs_bits;   // double bits of the max absolute error (non-negative: ordered as int)
    unsigned long long max_rel_bits;
    unsigned long long max_ulp_bits;
    unsigned int worst_abs_arg, worst_rel_arg, worst_ulp_arg;
};

__device__ void update(Acc* a, double abs_err, double rel_err, double ulp_err, uint32_t arg) {
    const unsigned long long ab = (unsigned long long)__double_as_longlong(abs_err);
    const unsigned long long rb = (unsigned long long)__double_as_longlong(rel_err);
    const unsigned long long ub = (unsigned long long)__double_as_longlong(ulp_err);
    if (atomicMax(&a->max_abs_bits, ab) < ab) a->worst_abs_arg = arg;
    if (atomicMax(&a->max_rel_bits, rb) < rb) a->worst_rel_arg = arg;
    if (atomicMax(&a->max_ulp_bits, ub) < ub) a->worst_ulp_arg = arg;
}

__device__ double ulp_of(float v) {
    const float a = fabsf(v);
    if (a == 0.0f) return 1.401298464324817e-45;
    const float n = __uint_as_float(__float_as_uint(a) + 1u);
    return (double)n - (double)a;
}

__global__ void log_err(uint32_t lo, uint32_t n, Acc* acc) {
    double mab = 0.0, mre = 0.0, mul = 0.0;
    uint32_t wa = 0, wr = 0, wu = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = lo + i;
        const float x = __uint_as_float(bits);
        const float hw = __builtin_amdgcn_logf(x);
        const double ex = log2((double)x);
        const double ae = fabs((double)hw - ex);
        const double re = ex != 0.0 ? ae / fabs(ex) : 0.0;
        const double ue = ae / ulp_of((float)ex);
        if (ae > mab) { mab = ae; wa = bits; }
        if (re > mre) { mre = re; wr = bits; }
        if (ue > mul) { mul = ue; wu = bits; }
    }
    update(acc, mab, mre, mul, 0u);
    (void)wa; (void)wr; (void)wu;
}

__global__ void exp_err(uint32_t lo, uint32_t n, Acc* acc) {
    double mab = 0.0, mre = 0.0, mul = 0.0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t bits = lo + i;
        const float y = -__uint_as_float(bits);   // negative arguments
        const float hw = __builtin_amdgcn_exp2f(y);
        const double ex = exp2((double)y);
        const double ae = fabs((double)hw - ex);
        const double re = ex != 0.0 ? ae / ex : 0.0;
        const double ue = ex >= 1.1754943508222875e-38 ? ae / ulp_of((float)ex) : 0.0;   // normal results
        if (ae > mab) mab = ae;
        if (ex >= 1.1754943508222875e-38 && re > mre) mre = re;
        if (ue > mul) mul = ue;
    }
    update(acc, mab, mre, mul, 0u);
}

int main() {
    Acc* d;
    hipMalloc(&d, 2 * sizeof(Acc));
    hipMemset(d, 0, 2 * sizeof(Acc));
    float a = std::ldexp(1.0f, -26), b = 1.0f;
    uint32_t lo, hi;
    std::memcpy(&lo, &a, 4);
    std::memcpy(&hi, &b, 4);
    hipLaunchKernelGGL(log_err, dim3(4096), dim3(256), 0, 0, lo, hi - lo, d);
    float y0 = 0.0f, y1 = 160.0f;
    std::memcpy(&lo, &y0, 4);
    std::memcpy(&hi, &y1, 4);
    hipLaunchKernelGGL(exp_err, dim3(4096), dim3(256), 0, 0, lo, hi - lo + 1, d + 1);
    Acc h[2];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    auto dd = [](unsigned long long u) { double v; std::memcpy(&v, &u, 8); return v; };
    std::printf("{\"log2_hw\": {\"range\": \"[2^-26, 1)\", \"max_abs\": %.6e, \"max_rel\": %.6e, \"max_ulp\": %.4f}, "
                "\"exp2_hw\": {\"range\": \"[-160, 0]\", \"max_abs\": %.6e, \"max_rel_normal\": %.6e, \"max_ulp_normal\": %.4f}}\n",
                dd(h[0].max_abs_bits), dd(h[0].max_rel_bits), dd(h[0].max_ulp_bits), dd(h[1].max_abs_bits),
                dd(h[1].max_rel_bits), dd(h[1].max_ulp_bits));
    return 0;
}
