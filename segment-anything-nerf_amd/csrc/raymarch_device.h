// raymarch_device.h -- per-ray device steps of the NeRF ray-march loop.
//
// Each function restates one op sequence of nerf/renderer.py as torch runs it
// on the CPU (the oracle the parity tests compare against): separate roundings
// per elementwise op (this library is compiled with -ffp-contract=off; fused
// multiply-adds appear only where written as __builtin_fmaf), cumulative sums
// accumulated in double like ATen's CPU cumsum, first-index argmax on ties.
#pragma once

#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>

namespace samnerf {

// nerf/renderer.py:122-139 -- slab test against the AABB; no hit -> 1e9.
__device__ __forceinline__ void near_far_aabb(const float o[3], const float d[3], const float* aabb,
                                              float min_near, float& near, float& far) {
    float n = -INFINITY, f = INFINITY;
    bool nan_n = false, nan_f = false;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float dd = d[c] + 1e-15f;
        const float t0 = (aabb[c] - o[c]) / dd;
        const float t1 = (aabb[3 + c] - o[c]) / dd;
        const float lo = t0 < t1 ? t0 : t1;   // torch.where(tmin < tmax, tmin, tmax)
        const float hi = t0 > t1 ? t0 : t1;   // torch.where(tmin > tmax, tmin, tmax)
        nan_n |= isnan(lo);
        nan_f |= isnan(hi);
        n = fmaxf(n, lo);
        f = fminf(f, hi);
    }
    if (nan_n) n = NAN;                       // amax / amin propagate NaN
    if (nan_f) f = NAN;
    if (f < n) { n = 1e9f; f = 1e9f; }
    near = fmaxf(n, min_near);                // torch.clamp(min=) (NaN stays NaN below)
    if (isnan(n)) near = n;
    far = f;
}

// spacing_fn / spacing_fn_inv (renderer.py:250-253)
__device__ __forceinline__ float spacing(float x) { return x < 1.0f ? x / 2.0f : 1.0f - 1.0f / (2.0f * x); }
__device__ __forceinline__ float spacing_inv(float x) {
    return x < 0.5f ? 2.0f * x : 1.0f / (2.0f - 2.0f * x);
}
// real_bins = spacing_inv(s_near * (1 - bin) + s_far * bin)   (renderer.py:278)
__device__ __forceinline__ float real_bin(float sn, float sf, float b) {
    return spacing_inv(sn * (1.0f - b) + sf * b);
}

// contract (renderer.py:60-69): L-inf contraction to [-2, 2].
__device__ __forceinline__ void contract3(float& x, float& y, float& z) {
    const float ax = fabsf(x), ay = fabsf(y), az = fabsf(z);
    float mag = ax;
    int idx = 0;
    if (ay > mag) { mag = ay; idx = 1; }
    if (az > mag) { mag = az; idx = 2; }
    if (isnan(ax) || isnan(ay) || isnan(az)) mag = NAN;
    if (mag < 1.0f) return;
    const float s = 1.0f / mag;
    const float sk = (2.0f - 1.0f / mag) / mag;
    x = x * (idx == 0 ? sk : s);
    y = y * (idx == 1 ? sk : s);
    z = z * (idx == 2 ? sk : s);
}

// torch.nan_to_num: NaN -> 0, +-inf -> +-FLT_MAX
// (branch-free: a clamp and one select, no divergent blocks in the
// unrolled compositing chains)
__device__ __forceinline__ float nan_to_num(float v) {
    const float c = fmaxf(fminf(v, FLT_MAX), -FLT_MAX);
    return v == v ? c : 0.0f;
}

// One compositing step (renderer.py:310-326): given delta*sigma of sample k
// and the running double cumsum of the previous ones, the weight.
__device__ __forceinline__ float composite_step(float ds, double& cum, bool last) {
    if (last) ds = INFINITY;
    const float alpha = 1.0f - expf(-ds);
    const float trans = expf(-(float)cum);
    cum += (double)ds;
    return nan_to_num(alpha * trans);
}

// torch.sum over a contiguous float row exactly as ATen's CPU kernel orders
// it (vectorized_inner_sum: Vectorized<float> of 8 lanes, 4 accumulators
// taking vectors round-robin, combined in sequence, scalar tail first, then
// the 8 lanes in sequence) -- the order tests/test_oracle.py pins against
// torch.sum.  Used for the pdf normaliser of sample_pdf (renderer.py:92) so
// searchsorted indices match the reference on identical inputs.
template <class XF>
__device__ __forceinline__ float torch_row_sum(int n, XF X) {
    float acc[4][8];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int l = 0; l < 8; ++l) acc[m][l] = 0.0f;
    const int nv = n / 8;
    int v = 0;
    for (; v + 4 <= nv; v += 4)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[m][l] = acc[m][l] + X((v + m) * 8 + l);
#pragma unroll
    for (int m = 0; m < 3; ++m)
        if (v + m < nv)
#pragma unroll
            for (int l = 0; l < 8; ++l) acc[m][l] = acc[m][l] + X((v + m) * 8 + l);
    float t = 0.0f;
    for (int k = nv * 8; k < n; ++k) t = t + X(k);
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        float a = acc[0][l];
#pragma unroll
        for (int m = 1; m < 4; ++m) a = a + acc[m][l];
        t = t + a;
    }
    return t;
}

// Inverse-CDF resampling of one ray (renderer.py:84-119, perturb = False) by a
// merge walk: cdf is the clamped double cumsum of (w + 0.01) / sum, u the
// sorted linspace table, so searchsorted(right=True) is the number of cdf
// entries <= u_j.  `wsum` = torch_row_sum of (w_i + 0.01).
// U(j) returns u_j, W(i) weight i, BINS(i) bin i of the ray; EMIT(j, value, inds).
template <class UF, class WF, class BF, class EF>
__device__ __forceinline__ void sample_pdf_walk(int T0, int T, UF U, float wsum, WF W, BF BINS,
                                                EF EMIT) {
    int i = 0;          // cdf entries consumed so far (all <= the current u)
    double cum = 0.0;
    float cdf_prev = 0.0f, cdf_cur = 0.0f;   // cdf[i-1], cdf[i]
    int j = 0;
    for (int step = 0; step < T0 + 1 + T; ++step) {
        if (j >= T) break;
        const float u = U(j);
        if (i <= T0 && cdf_cur <= u) {
            ++i;
            cdf_prev = cdf_cur;
            if (i <= T0) {
                const float pdf = (W(i - 1) + 0.01f) / wsum;
                cum += (double)pdf;
                cdf_cur = fminf((float)cum, 1.0f);
            }
        } else {
            const int below = i - 1;                 // i >= 1 always (cdf[0] = 0 <= u)
            const int above = i <= T0 ? i : T0;
            const float g0 = cdf_prev;
            const float g1 = i <= T0 ? cdf_cur : cdf_prev;
            const float b0 = BINS(below), b1 = BINS(above);
            float t = nan_to_num((u - g0) / (g1 - g0));
            t = fminf(fmaxf(t, 0.0f), 1.0f);
            EMIT(j, b0 + t * (b1 - b0), i);
            ++j;
        }
    }
}

// torch.norm over the last dim of a 3-vector, then divide (renderer.py:295,
// sphere_harmonics.py:82).
__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
    const float n = sqrtf(x * x + y * y + z * z);
    x = x / n;
    y = y / n;
    z = z / n;
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + expf(-x)); }

}  // namespace samnerf
