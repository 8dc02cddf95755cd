// train_optim.hip -- the optimiser step of the SAM-distillation training step
// (BASELINE config 5: nerf/utils.py:1831 scaler.step(optimizer) with
// Adam(lr=1e-2, eps=1e-15), main.py:296) as ONE pass over
// every parameter tensor.
//
// torch.optim.Adam (foreach) runs the update as 7 multi-tensor kernels per
// parameter group (lerp, mul, addcmul, sqrt, div, add, addcdiv), each reading
// and writing whole tensors: over the 42 M-float s_grid table that is ~0.78 ms
// per step (profiles/r1_train_kernel_stats.csv) against the 7 x 4 B x 42 M =
// 1.18 GB one pass needs (~0.2 ms at HBM rate).  Here every element is read
// (param, grad, exp_avg, exp_avg_sq) and written (param, exp_avg, exp_avg_sq)
// exactly once, 16-B vector accesses, all tensors of the step in one launch.
//
// Arithmetic per element, in torch's _multi_tensor_adam order (float):
//   g      = grad (+ weight_decay * param)
//   m      = lerp(m, g, 1 - beta1)          (ATen lerp: m + w * (g - m), w < 0.5)
//   v      = v * beta2 + (1 - beta2) * g * g
//   denom  = sqrt(v) / sqrt(1 - beta2^t) + eps
//   param += (-lr / (1 - beta1^t)) * m / denom
// Same values up to the rounding of the fused forms torch's kernels use
// (tests/test_gpu_train.py compares with torch.optim.Adam).
#include <algorithm>
#include <cmath>

#include "samnerf_common.h"

using namespace samnerf;

namespace {

constexpr int kMaxTensors = 16;
constexpr uint32_t kThreads = 256;
constexpr uint32_t kVecPerThread = 4;                      // float4 per thread per block pass
constexpr uint64_t kElemsPerBlock = (uint64_t)kThreads * kVecPerThread * 4;

struct AdamTable {
    float* param[kMaxTensors];
    const float* grad[kMaxTensors];
    float* m[kMaxTensors];
    float* v[kMaxTensors];
    uint64_t n[kMaxTensors];
    uint32_t block0[kMaxTensors + 1];   // first block of tensor i (prefix sums)
    uint32_t vec4;                      // bit i: tensor i takes 16-B accesses
    uint32_t count;
};

struct AdamHyper {
    float w1;          // 1 - beta1 (lerp weight)
    float beta2, one_m_beta2;
    float bc2_sqrt;    // sqrt(1 - beta2^t)
    float eps;
    float step_size;   // -lr / (1 - beta1^t)
    float wd;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h) {
    if (h.wd != 0.0f) g = g + h.wd * p;
    m = m + h.w1 * (g - m);
    v = v * h.beta2;
    v = v + (h.one_m_beta2 * g) * g;
    const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
    p = p + h.step_size * (m / denom);
}

__global__ void __launch_bounds__(kThreads) k_adam(AdamTable t, AdamHyper h) {
    const uint32_t b = blockIdx.x;
    int i = 0;
#pragma unroll 1
    while (i + 1 < (int)t.count && b >= t.block0[i + 1]) ++i;       // scalar: uniform per block
    const uint64_t base = (uint64_t)(b - t.block0[i]) * kElemsPerBlock;
    const uint64_t n = t.n[i];
    float* __restrict__ P = t.param[i];
    const float* __restrict__ G = t.grad[i];
    float* __restrict__ M = t.m[i];
    float* __restrict__ V = t.v[i];
    if ((t.vec4 >> i) & 1u) {
#pragma unroll
        for (uint32_t k = 0; k < kVecPerThread; ++k) {
            const uint64_t e = base + ((uint64_t)k * kThreads + threadIdx.x) * 4u;
            if (e >= n) break;
            float4 p = *reinterpret_cast<const float4*>(P + e);
            const float4 g = *reinterpret_cast<const float4*>(G + e);
            float4 m = *reinterpret_cast<const float4*>(M + e);
            float4 v = *reinterpret_cast<const float4*>(V + e);
            adam_elem(p.x, g.x, m.x, v.x, h);
            adam_elem(p.y, g.y, m.y, v.y, h);
            adam_elem(p.z, g.z, m.z, v.z, h);
            adam_elem(p.w, g.w, m.w, v.w, h);
            *reinterpret_cast<float4*>(P + e) = p;
            *reinterpret_cast<float4*>(M + e) = m;
            *reinterpret_cast<float4*>(V + e) = v;
        }
    } else {
        for (uint32_t k = 0; k < kVecPerThread * 4; ++k) {
            const uint64_t e = base + (uint64_t)k * kThreads + threadIdx.x;
            if (e >= n) break;
            float p = P[e], m = M[e], v = V[e];
            adam_elem(p, G[e], m, v, h);
            P[e] = p;
            M[e] = m;
            V[e] = v;
        }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" int samnerf_adam_step(const samnerf_adam_tensor* tensors, uint32_t n_tensors, double lr,
                                 double beta1, double beta2, double eps, double weight_decay,
                                 uint32_t step, samnerf_stream_t stream) {
    if (n_tensors && !tensors) return fail(SAMNERF_EINVAL, "adam_step: null tensor table");
    if (step == 0) return fail(SAMNERF_EINVAL, "adam_step: step counts from 1");
    if (!(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0))
        return fail(SAMNERF_EINVAL, "adam_step: betas must lie in [0, 1)");
    // every scalar in double from the caller's (Python) values, rounded to
    // float once, as torch hands its scalars to the foreach kernels (1 - beta2
    // taken in float would differ by 1.3e-5 relative)
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    AdamHyper h;
    h.w1 = (float)(1.0 - beta1);
    h.beta2 = (float)beta2;
    h.one_m_beta2 = (float)(1.0 - beta2);
    h.bc2_sqrt = (float)std::sqrt(bc2);
    h.eps = (float)eps;
    h.step_size = (float)(-lr / bc1);
    h.wd = (float)weight_decay;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint32_t i = 0;
    while (i < n_tensors) {
        AdamTable t{};
        uint32_t blocks = 0;
        for (; i < n_tensors && t.count < (uint32_t)kMaxTensors; ++i) {
            const samnerf_adam_tensor& x = tensors[i];
            if (!x.grad || x.n == 0) continue;                  // torch skips params without grad
            if (!x.param || !x.exp_avg || !x.exp_avg_sq)
                return fail(SAMNERF_EINVAL, "adam_step: tensor %u has a null buffer", i);
            const uint32_t c = t.count++;
            t.param[c] = x.param;
            t.grad[c] = x.grad;
            t.m[c] = x.exp_avg;
            t.v[c] = x.exp_avg_sq;
            t.n[c] = x.n;
            if (x.n % 4 == 0 && aligned16(x.param) && aligned16(x.grad) && aligned16(x.exp_avg) &&
                aligned16(x.exp_avg_sq))
                t.vec4 |= 1u << c;
            t.block0[c] = blocks;
            const uint64_t nb = (x.n + kElemsPerBlock - 1) / kElemsPerBlock;
            if (blocks + nb > 0x7fffffffull) return fail(SAMNERF_EINVAL, "adam_step: tensors too large");
            blocks += (uint32_t)nb;
        }
        t.block0[t.count] = blocks;
        if (blocks == 0) continue;
        k_adam<<<blocks, kThreads, 0, s>>>(t, h);
        const int rc = check_launch("adam_step");
        if (rc) return rc;
    }
    return SAMNERF_OK;
}
