// sh_freq_encoder.hip -- drop-in SH and frequency encoders for gfx950.
//
// Replaces the reference's _shencoder (shencoder/src/shencoder.cu:358-439) and
// _freqencoder (freqencoder/src/freqencoder.cu:30-129).  SH evaluates the
// basis by recurrence (sh_device.h) with the degree as a template parameter;
// the frequency encoder computes one output element per thread like the
// reference but with an accurate sinf (the reference's -use_fast_math
// __sinf loses accuracy as 2^f * x grows; parity tolerance in the tests).
#include "samnerf_common.h"
#include "sh_device.h"

using namespace samnerf;

namespace {

template <int DEG>
__global__ void __launch_bounds__(256)
k_sh_forward(const float* __restrict__ inputs, float* __restrict__ outputs, uint32_t B,
             uint32_t D, float* __restrict__ dy_dx) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    constexpr int C2 = DEG * DEG;
    const float x = inputs[(size_t)b * D], y = inputs[(size_t)b * D + 1],
                z = inputs[(size_t)b * D + 2];
    float out[C2];
    if (dy_dx) {
        float gx[C2], gy[C2], gz[C2];
        sh_values_grad<DEG>(x, y, z, out, gx, gy, gz);
        float* dd = dy_dx + (size_t)b * D * C2;
#pragma unroll
        for (int i = 0; i < C2; ++i) {
            dd[i] = gx[i];
            dd[C2 + i] = gy[i];
            dd[2 * C2 + i] = gz[i];
        }
    } else {
        sh_values<DEG>(x, y, z, out);
    }
    float* o = outputs + (size_t)b * C2;
#pragma unroll
    for (int i = 0; i < C2; ++i) o[i] = out[i];
}

// grad_inputs[t] += sum_ch grad[b, ch] * dy_dx[b, d, ch]   (shencoder.cu:358-382)
__global__ void __launch_bounds__(256)
k_sh_backward(const float* __restrict__ grad, const float* __restrict__ dy_dx,
              float* __restrict__ grad_inputs, uint32_t B, uint32_t D, uint32_t C2) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t b = t / D;
    if (b >= B) return;
    const uint32_t d = t - b * D;
    const float* g = grad + (size_t)b * C2;
    const float* j = dy_dx + ((size_t)b * D + d) * C2;
    float r = grad_inputs[t];
    for (uint32_t ch = 0; ch < C2; ++ch) r = __builtin_fmaf(g[ch], j[ch], r);
    grad_inputs[t] = r;
}

__global__ void __launch_bounds__(256)
k_freq_forward(const float* __restrict__ inputs, uint32_t B, uint32_t D, uint32_t C,
               float* __restrict__ outputs) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint64_t)B * C) return;
    const uint32_t b = (uint32_t)(t / C), c = (uint32_t)(t % C);
    const float* x = inputs + (size_t)b * D;
    float v;
    if (c < D) {
        v = x[c];
    } else {
        const uint32_t blk = c / D - 1u, d = c % D;
        const float arg = ldexpf(x[d], (int)(blk >> 1)) + (float)(blk & 1u) * 1.57079632679489662f;
        v = sinf(arg);
    }
    outputs[t] = v;
}

__global__ void __launch_bounds__(256)
k_freq_backward(const float* __restrict__ grad, const float* __restrict__ outputs, uint32_t B,
                uint32_t D, uint32_t deg, uint32_t C, float* __restrict__ grad_inputs) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    const float* g = grad + (size_t)b * C;
    const float* o = outputs + (size_t)b * C;
    float r = g[d];
    for (uint32_t f = 0; f < deg; ++f) {
        const uint32_t s = D + 2u * f * D, k = s + D;
        const float q = __builtin_fmaf(g[s + d], o[k + d], -(g[k + d] * o[s + d]));
        r = __builtin_fmaf(ldexpf(1.0f, (int)f), q, r);
    }
    grad_inputs[t] = r;
}

}  // namespace

extern "C" {

int samnerf_sh_encode_forward(const float* inputs, float* outputs, uint32_t B, uint32_t D,
                              uint32_t C, float* dy_dx, samnerf_stream_t stream) {
    if (!inputs || !outputs) return fail(SAMNERF_EINVAL, "SHEncoder: null tensor pointer");
    if (D != 3) return fail(SAMNERF_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SAMNERF_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (B == 0) return SAMNERF_OK;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint32_t g = div_up(B, 256);
    switch (C) {
        case 1: k_sh_forward<1><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 2: k_sh_forward<2><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 3: k_sh_forward<3><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 4: k_sh_forward<4><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 5: k_sh_forward<5><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 6: k_sh_forward<6><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 7: k_sh_forward<7><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
        case 8: k_sh_forward<8><<<g, 256, 0, s>>>(inputs, outputs, B, D, dy_dx); break;
    }
    return check_launch("sh_encode_forward");
}

int samnerf_sh_encode_backward(const float* grad, const float* inputs, uint32_t B, uint32_t D,
                               uint32_t C, const float* dy_dx, float* grad_inputs,
                               samnerf_stream_t stream) {
    (void)inputs;
    if (!grad || !dy_dx || !grad_inputs)
        return fail(SAMNERF_EINVAL, "SHEncoder backward: null tensor pointer");
    if (D != 3) return fail(SAMNERF_EINVAL, "SH encoder only support input dim == 3");
    if (C < 1 || C > 8) return fail(SAMNERF_EINVAL, "SH encoder only supports degree in [1, 8]");
    if (B == 0) return SAMNERF_OK;
    k_sh_backward<<<div_up((uint64_t)B * D, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        grad, dy_dx, grad_inputs, B, D, C * C);
    return check_launch("sh_encode_backward");
}

int samnerf_freq_encode_forward(const float* inputs, uint32_t B, uint32_t D, uint32_t deg,
                                uint32_t C, float* outputs, samnerf_stream_t stream) {
    if (!inputs || !outputs) return fail(SAMNERF_EINVAL, "FreqEncoder: null tensor pointer");
    if (C != D + 2u * D * deg) return fail(SAMNERF_EINVAL, "FreqEncoder: C != D + 2*D*degree");
    if (B == 0) return SAMNERF_OK;
    k_freq_forward<<<div_up((uint64_t)B * C, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        inputs, B, D, C, outputs);
    return check_launch("freq_encode_forward");
}

int samnerf_freq_encode_backward(const float* grad, const float* outputs, uint32_t B, uint32_t D,
                                 uint32_t deg, uint32_t C, float* grad_inputs,
                                 samnerf_stream_t stream) {
    if (!grad || !outputs || !grad_inputs)
        return fail(SAMNERF_EINVAL, "FreqEncoder backward: null tensor pointer");
    if (C != D + 2u * D * deg) return fail(SAMNERF_EINVAL, "FreqEncoder: C != D + 2*D*degree");
    if (B == 0) return SAMNERF_OK;
    k_freq_backward<<<div_up((uint64_t)B * D, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        grad, outputs, B, D, deg, C, grad_inputs);
    return check_launch("freq_encode_backward");
}

}  // extern "C"
