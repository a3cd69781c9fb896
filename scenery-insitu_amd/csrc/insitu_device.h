// insitu_device.h -- gfx950 device helpers shared by the VDI hot-path kernels.
//
// Numerical contract (DESIGN.md "Numerical contract"): IEEE binary32, round to nearest,
// subnormals kept, correctly rounded '/' and sqrt (hipcc default), fused multiply-add
// ONLY where written as fmaf() below, everything else rounds per operation.  The build
// passes -ffp-contract=off and this header repeats it as a pragma so no translation unit
// can silently fuse.  pow/log2/exp2 are the fixed polynomial algorithms below rather than
// v_log_f32/v_exp_f32, so results are reproducible bit for bit on any host.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace insitu {

struct f4 {
    float x, y, z, w;
};

__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }
// GLSL mix(x,y,a) = x*(1-a) + y*a, contracted into one fma
__device__ __forceinline__ float gmix(float x, float y, float a) { return __builtin_fmaf(y, a, x * (1.0f - a)); }

// Packed fp32 (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32): two lanes of independent IEEE operations
// in one instruction -- per component the same rounded multiply, add or fused multiply-add as the
// scalar form, so the same bits, in half the vector instructions.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pk_fma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v lo2(const f4& v) { return f2v{v.x, v.y}; }
__device__ __forceinline__ f2v hi2(const f4& v) { return f2v{v.z, v.w}; }
__device__ __forceinline__ f4 join2(f2v a, f2v b) { return f4{a.x, a.y, b.x, b.y}; }

// column-major mat4 * vec4, ((c0*x + c1*y) + c2*z) + c3*w, rows in pairs
__device__ __forceinline__ f4 mat_vec(const float* m, f4 v) {
    const f2v r01 = pk_fma(f2v{m[12], m[13]}, f2v{v.w, v.w},
                           pk_fma(f2v{m[8], m[9]}, f2v{v.z, v.z},
                                  pk_fma(f2v{m[4], m[5]}, f2v{v.y, v.y}, f2v{m[0], m[1]} * v.x)));
    const f2v r23 = pk_fma(f2v{m[14], m[15]}, f2v{v.w, v.w},
                           pk_fma(f2v{m[10], m[11]}, f2v{v.z, v.z},
                                  pk_fma(f2v{m[6], m[7]}, f2v{v.y, v.y}, f2v{m[2], m[3]} * v.x)));
    return join2(r01, r23);
}
// only row r of a mat4 * vec4
__device__ __forceinline__ float mat_row(const float* m, int r, f4 v) {
    return __builtin_fmaf(m[12 + r], v.w, __builtin_fmaf(m[8 + r], v.z, __builtin_fmaf(m[4 + r], v.y, m[r] * v.x)));
}
__device__ __forceinline__ f4 v4mix(f4 a, f4 b, float t) {   // gmix per component, in pairs
    const float u = 1.0f - t;
    return join2(pk_fma(lo2(b), f2v{t, t}, lo2(a) * u), pk_fma(hi2(b), f2v{t, t}, hi2(a) * u));
}
__device__ __forceinline__ float len4(float x, float y, float z, float w) {
    return __builtin_sqrtf(__builtin_fmaf(w, w, __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x))));
}
__device__ __forceinline__ float len3(float x, float y, float z) {
    return __builtin_sqrtf(__builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x)));
}
__device__ __forceinline__ f4 persp_div(f4 v) {
    float r = 1.0f / v.w;
    return f4{v.x * r, v.y * r, v.z * r, v.w * r};
}

// XCD-aware block order: the hardware deals consecutive workgroups round-robin to the 8 XCDs,
// each with its own L2.  Renumber in chunks of C blocks: the C blocks one XCD runs back to back
// get C consecutive logical blocks (neighbouring screen tiles, which read neighbouring brick
// blocks, share that XCD's L2), while consecutive chunks still rotate over the XCDs (screen
// regions with heavy rays are spread over all of them).  A tail that does not fill 8*C blocks
// keeps the hardware order.
__device__ __forceinline__ int xcd_block(int b, int nblocks, int C = 16) {
    const int span = 8 * C;
    if (b >= (nblocks / span) * span) return b;
    const int x = b & 7, i = b >> 3;
    return ((i / C) * 8 + x) * C + (i % C);
}

// ---- deterministic log2 / exp2 / pow (pow(x,y) := exp2(y*log2(x)), GLSL definition) ----
// Branch-free forms: the main path is evaluated for every input and special inputs (0, inf,
// NaN, negative, out-of-range exponents) are selected afterwards, so a wave never splits its
// exec mask here.  Results are identical, input for input, to the branching restatement in
// oracle/insitu_oracle.c (orc_log2/orc_exp2); tests/test_device_math.py checks that on the host.
__host__ __device__ __forceinline__ float det_log2(float x) {
    const bool sub = x < 1.17549435e-38f;
    const float xs = sub ? x * 8388608.0f : x;
    const uint32_t u = __builtin_bit_cast(uint32_t, xs);
    int e = (int)((u >> 23) & 0xffu) - 127 + (sub ? -23 : 0);
    float m = __builtin_bit_cast(float, (u & 0x007fffffu) | 0x3f800000u);
    const bool big = m > 1.41421354f;
    m = big ? m * 0.5f : m;
    e += big ? 1 : 0;
    const float f = m - 1.0f;
#ifdef __HIP_DEVICE_COMPILE__
    // f / (2 + f) by the hardware's correctly rounded division sequence without its scaling and fix-up
    // steps, which are the identity here: f lies in [-0.293, 0.415] and 2 + f in [1.70, 2.42] for every x
    // (m is in [0.707, 1.414]; a NaN or inf x is selected away below), so no operand is near under- or
    // overflow -- the same operations on the same values, the same correctly rounded quotient
    const float dd = 2.0f + f;
    float y = __builtin_amdgcn_rcpf(dd);
    y = __builtin_fmaf(__builtin_fmaf(-dd, y, 1.0f), y, y);
    float s = f * y;
    s = __builtin_fmaf(__builtin_fmaf(-dd, s, f), y, s);
    s = __builtin_fmaf(__builtin_fmaf(-dd, s, f), y, s);
#else
    const float s = f / (2.0f + f);
#endif
    const float z = s * s;
    float p = __builtin_fmaf(z, 0.0909090936f, 0.111111112f);
    p = __builtin_fmaf(z, p, 0.142857149f);
    p = __builtin_fmaf(z, p, 0.200000003f);
    p = __builtin_fmaf(z, p, 0.333333343f);
    const float s2 = s + s;
    const float ln = __builtin_fmaf(s2 * z, p, s2);
    float r = __builtin_fmaf(ln, 1.44269502f, (float)e);
    r = (x == __builtin_inff()) ? __builtin_inff() : r;
    r = (x == 0.0f) ? -__builtin_inff() : r;
    r = (x >= 0.0f) ? r : __builtin_nanf("");
    return r;
}

__host__ __device__ __forceinline__ float det_exp2(float y) {
    const float n = __builtin_rintf(y);
    const float f = y - n;
    float p = 1.52527336e-05f;
    p = __builtin_fmaf(p, f, 1.54035297e-04f);
    p = __builtin_fmaf(p, f, 1.33335581e-03f);
    p = __builtin_fmaf(p, f, 9.61812911e-03f);
    p = __builtin_fmaf(p, f, 5.55041087e-02f);
    p = __builtin_fmaf(p, f, 2.40226507e-01f);
    p = __builtin_fmaf(p, f, 6.93147182e-01f);
    p = __builtin_fmaf(p, f, 1.0f);
    const float nc = __builtin_fminf(__builtin_fmaxf(n, -200.0f), 200.0f);   // NaN -> 200 (selected away)
    const int ni = (int)nc;
    // 2^ni as (p * 2^ea) * b: one multiply in the normal range, two beyond it (as orc_exp2)
    const int ea = ni > 127 ? 127 : (ni >= -126 ? ni : ni + 64);
    const float b = ni > 127 ? 2.0f : (ni >= -126 ? 1.0f : __builtin_bit_cast(float, (uint32_t)(127 - 64) << 23));
    float r = (p * __builtin_bit_cast(float, (uint32_t)(ea + 127) << 23)) * b;
    r = (y < -150.0f) ? 0.0f : r;
    r = (y >= 128.0f) ? __builtin_inff() : r;
    r = (y != y) ? y : r;
    return r;
}

__host__ __device__ __forceinline__ float det_pow(float x, float y) { return det_exp2(y * det_log2(x)); }
__host__ __device__ __forceinline__ float det_ln(float x) { return det_log2(x) * 0.693147182f; }

// Smallest float y with sqrt_rn(y) >= t (t >= 0): since correctly rounded sqrt is monotone,
// `sqrt(y) >= t` is exactly `y >= sq_threshold(t)`, which turns the supersegment test
// length(...) >= threshold (AccumulateVDI.comp:74, VDICompositor.comp:350) into a compare of
// the squared length -- same decisions, no per-sample square root.
// Definition (the search form, kept as the reference for the closed form below):
__host__ __device__ __forceinline__ float sq_threshold_search(float t) {
    if (!(t > 0.0f)) return 0.0f;
    float y = t * t;
    while (y > 0.0f && __builtin_sqrtf(y) >= t) y = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) - 1u);
    while (!(__builtin_sqrtf(y) >= t)) y = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) + 1u);
    return y;
}
// Closed form for normal t: sqrt_rn(y) >= t iff sqrt(y) > mid = (pred(t) + t) / 2, or sqrt(y) == mid
// and the tie rounds to t (t's significand even).  mid has <= 25 significant bits, so M = mid^2 is
// exact in double, and the answer is the smallest float above M (or equal to it on an even t).
// Identical to sq_threshold_search for every t in [2^-60, 2^60] (tests/test_device_math.py checks
// all of [2^-20, 4] exhaustively); other t take the search form.
__host__ __device__ __forceinline__ float sq_threshold(float t) {
    if (!(t >= 8.67361738e-19f && t <= 1.15292150e18f)) return sq_threshold_search(t);
    const uint32_t ut = __builtin_bit_cast(uint32_t, t);
    const float tm = __builtin_bit_cast(float, ut - 1u);          // pred(t)
    const double mid = ((double)tm + (double)t) * 0.5;            // exact
    const double M = mid * mid;                                   // exact (<= 50 bits)
    float y = (float)M;                                           // nearest float
    const bool even = (ut & 1u) == 0u;
    if ((double)y < M || ((double)y == M && !even)) y = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, y) + 1u);
    return y;
}
__device__ __forceinline__ float sumsq3(float x, float y, float z) {
    return __builtin_fmaf(z, z, __builtin_fmaf(y, y, x * x));
}

// VDIGenerator.comp:80-82
__device__ __forceinline__ float adjust_opacity(float a, float len) { return 1.0f - det_pow(1.0f - a, len); }

__device__ __forceinline__ uint32_t unorm8(float x) {
    float q = (x > 0.0f) ? ((x < 1.0f) ? x : 1.0f) : 0.0f;
    return (uint32_t)(int)__builtin_floorf(__builtin_fmaf(q, 255.0f, 0.5f));
}

// floor + clamp-to-edge texel pair
__device__ __forceinline__ void texel_pair(float t, int n, int& i0, int& i1, float& frac) {
    float fl = __builtin_floorf(t);
    frac = t - fl;
    if (!(fl >= -1.0f)) fl = -1.0f;
    if (fl > (float)n) fl = (float)n;
    int i = (int)fl;
    i0 = i < 0 ? 0 : (i > n - 1 ? n - 1 : i);
    int j = i + 1;
    i1 = j < 0 ? 0 : (j > n - 1 ? n - 1 : j);
}

// VolumeRaycaster.comp:63-69 EncodeFloatRGBA -> packed rgba8
__device__ __forceinline__ uint32_t encode_depth_rgba8(float v) {
    float e0 = 1.0f * v, e1 = 255.0f * v, e2 = 65025.0f * v, e3 = 16581375.0f * v;
    e0 = e0 - __builtin_floorf(e0);
    e1 = e1 - __builtin_floorf(e1);
    e2 = e2 - __builtin_floorf(e2);
    e3 = e3 - __builtin_floorf(e3);
    const float c = 1.0f / 255.0f;
    float r0 = __builtin_fmaf(-e1, c, e0);
    float r1 = __builtin_fmaf(-e2, c, e1);
    float r2 = __builtin_fmaf(-e3, c, e2);
    float r3 = __builtin_fmaf(-e3, 0.0f, e3);
    return unorm8(r0) | (unorm8(r1) << 8) | (unorm8(r2) << 16) | (unorm8(r3) << 24);
}

// PlainImageCompositor.comp:25-29 DecodeFloatRGBA of a packed rgba8 texel
__device__ __forceinline__ float decode_depth_rgba8(uint32_t p) {
    const float d0 = 1.0f, d1 = 1.0f / 255.0f, d2 = 1.0f / 65025.0f, d3 = 1.0f / 16581375.0f;
    float v0 = (float)(p & 0xffu) / 255.0f, v1 = (float)((p >> 8) & 0xffu) / 255.0f;
    float v2 = (float)((p >> 16) & 0xffu) / 255.0f, v3 = (float)(p >> 24) / 255.0f;
    return __builtin_fmaf(v3, d3, __builtin_fmaf(v2, d2, __builtin_fmaf(v1, d1, v0 * d0)));
}

}  // namespace insitu
