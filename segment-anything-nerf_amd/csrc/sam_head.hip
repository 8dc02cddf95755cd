// sam_head.hip -- the SAM-feature head on gfx950 matrix cores.
//
// samvit_mlp = Sequential(SkipConnMLP(163, 256, 256, 5, skip_layers=[2],
// bias=True), LayerNorm(256)) (nerf/network.py:36-75, :120-123), applied per
// ray to f = cat(f_sam, f_image, image, depth) (nerf/renderer.py:377-385).
//
// fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32 (exact f32 FMA chains,
// cdna_hip_programming.md section 3 "FP32-input MFMA") so the head keeps the
// 1e-3 parity budget that bf16 operands would spend.
//   * one workgroup = 32 rays x all 256 output columns, 4 waves, each wave two
//     32x32 accumulator tiles;
//   * activations live in LDS (odd row strides: conflict-free ds_read_b32 for
//     the A operand, lane = row), the 5 layers run back to back in the same
//     workgroup, bias + leaky_relu(0.01) and the final LayerNorm fused;
//   * weights are re-packed once per call so each B fragment group (4 k-steps
//     of one 32-column tile) is one contiguous 1 KiB wave load (16 B per lane)
//     from L2.
#include "samnerf_common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace samnerf {

namespace {

constexpr int kRows = 32;          // rays per workgroup
constexpr int kXPad = 168;         // 163 head inputs padded to a multiple of 8
constexpr int kXStride = 169;      // odd LDS strides
constexpr int kHStride = 257;
constexpr int kIn = 163;
constexpr int kRowIn = 164;        // row stride of the input rows written by raymarch
// padded K of each layer (physical LDS k positions)
constexpr int kK[5] = {kXPad, 256, 256 + kXPad, 256, 256};
constexpr int kGroups[5] = {kXPad / 8, 256 / 8, (256 + kXPad) / 8, 256 / 8, 256 / 8};
constexpr int kLogicalIn[5] = {kIn, 256, 256 + kIn, 256, 256};

__host__ __device__ constexpr int group_base(int layer) {
    int b = 0;
    for (int i = 0; i < layer; ++i) b += kGroups[i];
    return b;
}
constexpr int kTotalGroups = group_base(5);

// physical k -> logical input column of the layer's weight (or -1 = zero).
__device__ __forceinline__ int logical_k(int layer, int kp) {
    if (layer == 0) return kp < kIn ? kp : -1;
    if (layer == 2) {
        if (kp < 256) return kp;
        const int x = kp - 256;
        return x < kIn ? 256 + x : -1;
    }
    return kp;
}

// packed[layer][tile 0..7][group][lane 0..63][4]
__global__ void __launch_bounds__(256)
k_pack(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
       const float* __restrict__ w3, const float* __restrict__ w4, float* __restrict__ packed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;   // one float4 per thread
    const uint32_t total = 8u * kTotalGroups * 64u;
    if (t >= total) return;
    const uint32_t lane = t & 63u;
    uint32_t rest = t >> 6;
    // rest = tile * kTotalGroups + global_group
    const uint32_t tile = rest / kTotalGroups;
    const uint32_t gg = rest % kTotalGroups;
    int layer = 0;
    while (layer < 4 && (int)gg >= group_base(layer + 1)) ++layer;
    const int g = (int)gg - group_base(layer);
    const float* W = layer == 0 ? w0 : layer == 1 ? w1 : layer == 2 ? w2 : layer == 3 ? w3 : w4;
    const int col = (int)(tile * 32u + (lane & 31u));
    const int h = (int)(lane >> 5);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int kp = 2 * (4 * g + e) + h;
        const int k = logical_k(layer, kp);
        v[e] = k >= 0 ? W[(size_t)col * kLogicalIn[layer] + k] : 0.0f;
    }
    float4* dst = reinterpret_cast<float4*>(packed) +
                  ((size_t)tile * kTotalGroups + gg) * 64u + lane;
    *dst = make_float4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float leaky(float x) { return x >= 0.0f ? x : x * 0.01f; }

template <int LAYER>
__device__ __forceinline__ void run_layer(const float* __restrict__ packed,
                                          const float* __restrict__ bias, float* X, float* Hs,
                                          int wave, int lane, floatx16& acc0, floatx16& acc1) {
    const int r = lane & 31, h = lane >> 5;
    const int t0 = 2 * wave, t1 = 2 * wave + 1;
    const float4* p0 = reinterpret_cast<const float4*>(packed) +
                       ((size_t)t0 * kTotalGroups + group_base(LAYER)) * 64 + lane;
    const float4* p1 = reinterpret_cast<const float4*>(packed) +
                       ((size_t)t1 * kTotalGroups + group_base(LAYER)) * 64 + lane;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc0[i] = 0.0f;
        acc1[i] = 0.0f;
    }
    float4 b0 = p0[0], b1 = p1[0];
    for (int g = 0; g < kGroups[LAYER]; ++g) {
        float4 n0 = b0, n1 = b1;
        if (g + 1 < kGroups[LAYER]) {   // prefetch the next group's B fragments
            n0 = p0[(size_t)(g + 1) * 64];
            n1 = p1[(size_t)(g + 1) * 64];
        }
        const float bb0[4] = {b0.x, b0.y, b0.z, b0.w};
        const float bb1[4] = {b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int kp = 2 * (4 * g + e) + h;
            float a;
            if constexpr (LAYER == 0) a = X[r * kXStride + kp];
            else if constexpr (LAYER == 2) a = kp < 256 ? Hs[r * kHStride + kp] : X[r * kXStride + kp - 256];
            else a = Hs[r * kHStride + kp];
            acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb0[e], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb1[e], acc1, 0, 0, 0);
        }
        b0 = n0;
        b1 = n1;
    }
    __syncthreads();                      // every wave has read Hs
    if constexpr (LAYER < 4) {
        const float bc0 = bias[t0 * 32 + r], bc1 = bias[t1 * 32 + r];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            Hs[row * kHStride + t0 * 32 + r] = leaky(acc0[i] + bc0);
            Hs[row * kHStride + t1 * 32 + r] = leaky(acc1[i] + bc1);
        }
    } else {
        const float bc0 = bias[t0 * 32 + r], bc1 = bias[t1 * 32 + r];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (i & 3) + 8 * (i >> 2) + 4 * h;
            Hs[row * kHStride + t0 * 32 + r] = acc0[i] + bc0;
            Hs[row * kHStride + t1 * 32 + r] = acc1[i] + bc1;
        }
    }
    __syncthreads();
}

struct HeadArgs {
    const float* rows;     // [N, 164]
    uint32_t N;
    const float* packed;
    const float* b[5];
    const float* ln_w;
    const float* ln_b;
    float* out;            // [N, 256]
};

__global__ void __launch_bounds__(256) k_sam_head(HeadArgs a) {
    __shared__ float X[kRows * kXStride];
    __shared__ float Hs[kRows * kHStride];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t ray0 = blockIdx.x * kRows;

    for (int i = tid; i < kRows * kXPad; i += 256) {
        const int r = i / kXPad, c = i % kXPad;
        const uint32_t ray = ray0 + r;
        float v = 0.0f;
        if (ray < a.N && c < kIn) v = a.rows[(size_t)ray * kRowIn + c];
        X[r * kXStride + c] = v;
    }
    __syncthreads();

    floatx16 acc0, acc1;
    run_layer<0>(a.packed, a.b[0], X, Hs, wave, lane, acc0, acc1);
    run_layer<1>(a.packed, a.b[1], X, Hs, wave, lane, acc0, acc1);
    run_layer<2>(a.packed, a.b[2], X, Hs, wave, lane, acc0, acc1);
    run_layer<3>(a.packed, a.b[3], X, Hs, wave, lane, acc0, acc1);
    run_layer<4>(a.packed, a.b[4], X, Hs, wave, lane, acc0, acc1);

    // LayerNorm(256, eps=1e-5): 8 threads per row, 32 columns each.
    const int row = tid >> 3, q = tid & 7;
    const float* hr = Hs + row * kHStride + q * 32;
    double s = 0.0;
    for (int c = 0; c < 32; ++c) s += (double)hr[c];
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) s += __shfl_xor(s, m, 8);
    const double mean = s / 256.0;
    double v = 0.0;
    for (int c = 0; c < 32; ++c) {
        const double dlt = (double)hr[c] - mean;
        v += dlt * dlt;
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) v += __shfl_xor(v, m, 8);
    const float rstd = (float)(1.0 / sqrt(v / 256.0 + 1e-5));
    const float mf = (float)mean;
    const uint32_t ray = ray0 + row;
    if (ray < a.N) {
        float* o = a.out + (size_t)ray * 256 + q * 32;
        for (int c = 0; c < 32; c += 4) {
            float4 y;
            y.x = ((hr[c + 0] - mf) * rstd) * a.ln_w[q * 32 + c + 0] + a.ln_b[q * 32 + c + 0];
            y.y = ((hr[c + 1] - mf) * rstd) * a.ln_w[q * 32 + c + 1] + a.ln_b[q * 32 + c + 1];
            y.z = ((hr[c + 2] - mf) * rstd) * a.ln_w[q * 32 + c + 2] + a.ln_b[q * 32 + c + 2];
            y.w = ((hr[c + 3] - mf) * rstd) * a.ln_w[q * 32 + c + 3] + a.ln_b[q * 32 + c + 3];
            *reinterpret_cast<float4*>(o + c) = y;
        }
    }
}

}  // namespace

size_t sam_head_packed_floats() { return (size_t)8 * kTotalGroups * 64 * 4; }

int sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                     float* packed, hipStream_t s) {
    const uint32_t nvec = 8u * kTotalGroups * 64u;
    k_pack<<<div_up(nvec, 256), 256, 0, s>>>(m->sam_w[0], m->sam_w[1], m->sam_w[2], m->sam_w[3],
                                             m->sam_w[4], packed);
    HeadArgs a;
    a.rows = rows;
    a.N = N;
    a.packed = packed;
    for (int i = 0; i < 5; ++i) a.b[i] = m->sam_b[i];
    a.ln_w = m->ln_w;
    a.ln_b = m->ln_b;
    a.out = samvit;
    k_sam_head<<<div_up(N, kRows), 256, 0, s>>>(a);
    return check_launch("sam_head");
}

}  // namespace samnerf
