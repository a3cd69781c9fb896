// insitu_filter.h -- filtered supersegment decisions (the generator's search passes and the
// VDICompositor's): decide `diff >= threshold` from a cheap estimate of diff^2 when it is farther from the
// threshold than a rigorous error margin, otherwise by the exact contract computation.  Shared by
// vdi_generate.hip and composite.hip; the derivation is at filter_margin below.
#pragma once
#include "insitu_device.h"

#pragma clang fp contract(off)

namespace insitu {

// ---- filtered supersegment test -------------------------------------------------------------
#ifndef INSITU_HW_TRANSCENDENTALS
#define INSITU_HW_TRANSCENDENTALS 1   // estimate's log2/exp2: 1 = hardware (default: -12 % frame time), 0 = polynomial
#endif
// A search pass only needs the DECISION `diff >= threshold` per sample (VDIGenerator.comp:497-529
// reads num_terminations; the state curV never depends on the adjusted colour).  The filtered
// form first estimates diff^2 with hardware reciprocals (v_rcp / v_rsq, <= 1 ulp) in place of
// the three correctly rounded divisions and the square root of the exact form; when the estimate
// is farther than a rigorous error margin from the threshold the decision is certain, otherwise
// (and for any non-finite or extreme value) the exact contract computation decides.
//
// Error budget of the estimate against the contract value.  With c = max(1, |adjusted colour|,
// |premultiplied sample colour|): adjusted colour 2^-22 relative (rcp vs division); adjusted
// opacity <= 5e-7 absolute (the exponent y = len^-1 * log2(1 - a) is 2^-21 relative off, and
// |d exp2(y)| <= ln2 |y| 2^y 2^-21 <= 2^-21 / e, plus det_exp2's own rounding at two arguments);
// so each premultiplied difference d_i is off by at most E0 = 1e-6 c (plus 2^-23 |d_i| from the
// subtraction).  Then |est - exact| <= 2 E0 sum|d_i| + 3 E0^2 + 2^-20 est <= 2 E0 sqrt(3 est) +
// 3 E0^2 + 2^-20 est.  The margin takes E0 four times larger:
//     m = c (1.4e-5 sqrt(est) + 5e-11 c) + 1e-6 est,
// i.e. relative to the difference itself (1.4e-7 at diff^2 = 1e-4), not to the colour range: near
// small thresholds the estimate almost always decides.  Written supersegments always take the
// exact adjusted colour.  tests/test_gpu_parity.py checks filtered == exact on whole frames.
//
// c is a constant of the transfer function (TransferDesc::cmag, computed by the host): with C the
// largest |rgb| component of the colour map and A the largest |alpha| of the TF, every sample colour
// is a lerp of two colour-map texels (|x.rgb| <= C up to one rounding) and the open supersegment's
// adjusted colour curV.rgb / curV.a is a weighted mean of sample colours: each accumulation step adds
// t*x*w to curV.rgb and t*w to curV.a, so |curV.rgb| <= C curV.a (1 + 3 n 2^-24) after n <= 65535
// steps, i.e. within 1.2 % of C.  Hence c = max(1, 2C, 2CA) bounds both the adjusted colour and the
// premultiplied sample colour x.rgb * x.a with room to spare, and the per-sample max() chain is gone.
__device__ __forceinline__ float filter_margin(float est, float c) {
    // c (1.4e-5 sqrt(est) + 5e-11 c) + 1e-6 est, as two fmas around the square root (c uniform)
    return __builtin_fmaf(1.4e-5f * c, __builtin_amdgcn_sqrtf(est), __builtin_fmaf(1e-6f, est, 5e-11f * c * c));
}

// The decision thresholds of the estimate, once per pass instead of a margin per sample.  With
// f(a) = a - m(a) and g(a) = a + m(a) (m = filter_margin in real arithmetic), the estimate a decides
// "close" when f(a) >= thresh_sq and "no close" when g(a) < thresh_sq.  Both are increasing where
// it matters (g everywhere; f for a > 4.9e-11 c^2, and f < 0 below its root, so f(a) >= t > 0 only
// past the root), hence the tests are a >= hi and a < lo with hi, lo the roots of f = t and g = t:
// computed in float and moved 16 ulps outward (hi up, lo down).  The per-sample
// test is then two compares: no square root, no margin arithmetic.
struct Thr {
    float sq;   // sq_threshold(threshold): the exact decision is diff^2 >= sq
    float hi;   // estimate >= hi: certainly closes
    float lo;   // estimate <  lo: certainly does not close
};

__device__ __forceinline__ float ulps_up(float x, int n) { return __uint_as_float(__float_as_uint(x) + (uint32_t)n); }

__device__ __forceinline__ Thr make_thr(float t_sq, float c) {
    // hi root s = (p + sqrt(p^2 + 4A(q + t))) / 2A; lo root s = 2(t - q) / (p + sqrt(p^2 + 4B(t - q)))
    // (no cancellation), with hardware v_sqrt / v_rcp (<= 1 ulp each): each square is within ~10 ulps,
    // and the 16-ulp outward moves cover that (2e-6 relative, far inside the margin's own band,
    // >= 1.6e-5 c relative)
    const float p = 1.4e-5f * c, q = 5e-11f * c * c;
    const float A = 1.0f - 1e-6f, B = 1.0f + 1e-6f;
    Thr r;
    r.sq = t_sq;
    const float sh = (p + __builtin_amdgcn_sqrtf(__builtin_fmaf(p, p, 4.0f * A * (q + t_sq)))) *
                     __builtin_amdgcn_rcpf(2.0f * A);
    r.hi = ulps_up(sh * sh, 16);
    r.lo = 0.0f;   // the estimate is >= 0: 0 means never "certainly no close"
    if (q <= 0.5f * t_sq) {   // t - q then has at most one rounding relative to itself
        const float d = t_sq - q;
        const float sl = (2.0f * d) * __builtin_amdgcn_rcpf(p + __builtin_amdgcn_sqrtf(__builtin_fmaf(p, p, 4.0f * B * d)));
        const float l = sl * sl;
        if (__float_as_uint(l) > 16u) r.lo = __uint_as_float(__float_as_uint(l) - 16u);
    }
    return r;
}

// a Thr every lane computed from the same uniform values, kept in scalar registers
__device__ __forceinline__ Thr uniform_thr(const Thr& t) {
    return Thr{__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.sq))),
               __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.hi))),
               __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(t.lo)))};
}

// the segmentation-interval bounds from the extreme estimates of a PRE pass: lo_a = the largest
// estimate of a certain non-closing decision, hi_a = the smallest of a certain closing one.  Every
// such non-closing exact diff^2 is <= g(its estimate) <= g(lo_a) (g increasing); every such closing
// one is >= f(its estimate) >= f(hi_a) when f(hi_a) >= 0 (all recorded estimates then lie where f
// increases), and a negative hi admits no threshold at all.  Exact decisions keep their exact values
// (deep in the search the thresholds are ulps apart and only exact bounds separate them)
__device__ __forceinline__ float seg_lo_bound(float lo_a, float c) {
    return lo_a < 0.0f ? lo_a : lo_a + filter_margin(lo_a, c);
}
__device__ __forceinline__ float seg_hi_bound(float hi_a, float c) {
    return (hi_a < 1.0e30f) ? hi_a - filter_margin(hi_a, c) : hi_a;
}


}  // namespace insitu
