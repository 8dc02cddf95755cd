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


// ===================================================================== bf16x3
// Split-precision head: x = x_hi + x_lo with x_hi = bf16(x), x_lo =
// bf16(x - x_hi); A.B ~= A_lo.B_hi + A_hi.B_lo + A_hi.B_hi on
// v_mfma_f32_32x32x16_bf16 (fp32 accumulate).  Relative error per product
// ~2^-16 (the dropped A_lo.B_lo term and the rounding of the lo parts),
// i.e. ~1e-5 on the head output against the 1e-3 budget, at 3 bf16 MFMAs per
// 16-deep k-block instead of 8 fp32 ones (5.3x fewer matrix cycles).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kXkB = 176;                 // head input padded to 11 k-blocks of 16
constexpr int kRowB = 264;                // LDS row stride in bf16 (528 B = 16 mod 256: conflict-free b128 reads)
constexpr int kThreadsB = 512;            // 8 waves = the 8 output column tiles
// k-block segments: 0 = W0 (x, 11), 1 = W1 (16), 2 = W2[:, :256] (h, 16),
// 3 = W3 (16), 4 = W4 (16), 5 = W2[:, 256:] (x part of the skip layer, 11)
constexpr int kKbB[6] = {11, 16, 16, 16, 16, 11};
constexpr int kbBase(int seg) {
    int b = 0;
    for (int i = 0; i < seg; ++i) b += kKbB[i];
    return b;
}
constexpr int kKbTotal = kbBase(6);       // 86

__device__ __forceinline__ uint32_t bf16_rne(float x) {
    uint32_t u = __float_as_uint(x);
    u += 0x7FFFu + ((u >> 16) & 1u);
    return u >> 16;
}
__device__ __forceinline__ void split_bf16(float x, uint32_t& hi, uint32_t& lo) {
    hi = bf16_rne(x);
    lo = bf16_rne(x - __uint_as_float(hi << 16));
}

// packed_{hi,lo}[tile 8][global k-block 86][lane 64] : 8 bf16 (16 B) each
__global__ void __launch_bounds__(256)
k_pack_bf3(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
           const float* __restrict__ w3, const float* __restrict__ w4, uint4* __restrict__ phi,
           uint4* __restrict__ plo) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 8u * kKbTotal * 64u) return;
    const uint32_t lane = t & 63u, rest = t >> 6;
    const uint32_t tile = rest / kKbTotal, gkb = rest % kKbTotal;
    int seg = 0;
    while (seg < 5 && (int)gkb >= kbBase(seg + 1)) ++seg;
    const int kb = (int)gkb - kbBase(seg);
    const float* W = seg == 0 ? w0 : seg == 1 ? w1 : (seg == 2 || seg == 5) ? w2 : seg == 3 ? w3 : w4;
    const int ldw = seg == 0 ? kIn : (seg == 2 || seg == 5) ? 256 + kIn : 256;
    const int col = (int)(tile * 32u + (lane & 31u));
    uint32_t hi[8], lo[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kp = kb * 16 + 8 * (int)(lane >> 5) + j;
        int k = kp;                                   // logical weight column
        if (seg == 0) k = kp < kIn ? kp : -1;
        if (seg == 5) k = kp < kIn ? 256 + kp : -1;
        const float v = k >= 0 ? W[(size_t)col * ldw + k] : 0.0f;
        split_bf16(v, hi[j], lo[j]);
    }
    phi[t] = make_uint4(hi[0] | hi[1] << 16, hi[2] | hi[3] << 16, hi[4] | hi[5] << 16, hi[6] | hi[7] << 16);
    plo[t] = make_uint4(lo[0] | lo[1] << 16, lo[2] | lo[3] << 16, lo[4] | lo[5] << 16, lo[6] | lo[7] << 16);
}

struct HeadArgsB {
    const float* rows;
    uint32_t N;
    const uint4* phi;
    const uint4* plo;
    const float* b[5];
    const float* ln_w;
    const float* ln_b;
    float* out;
};

#define MFMA_BF16(A, B, C) __builtin_amdgcn_mfma_f32_32x32x16_bf16((A), (B), (C), 0, 0, 0)

// One workgroup = RT row tiles of 32 rays, 8 waves; wave ct owns output
// columns 32ct..32ct+31 of every layer for ALL the block's rows, so each
// weight fragment it streams from L2 feeds 3 x RT MFMAs (the head is bound by
// that stream: ~11 KB of fragments per ray at RT = 4).  The skip layer's input
// half W2[:, 256:] . x is accumulated during layer 0 (while x is resident), so
// the activations need one in-place hi/lo buffer.
template <int SEG, int RT>
__device__ __forceinline__ void kloop_bf3(const HeadArgsB& a, const uint16_t* Ph, const uint16_t* Pl,
                                          int ct, int lane, floatx16 (&acc)[RT]) {
    const int r = lane & 31, h = lane >> 5;
    const uint4* ph = a.phi + ((size_t)ct * kKbTotal + kbBase(SEG)) * 64 + lane;
    const uint4* pl = a.plo + ((size_t)ct * kKbTotal + kbBase(SEG)) * 64 + lane;
    uint4 bh = ph[0], bl = pl[0];
#pragma unroll 1
    for (int kb = 0; kb < kKbB[SEG]; ++kb) {
        uint4 nh = bh, nl = bl;
        if (kb + 1 < kKbB[SEG]) {           // prefetch the next k-block's B fragments (L2)
            nh = ph[(kb + 1) * 64];
            nl = pl[(kb + 1) * 64];
        }
        const int kk = kb * 16 + 8 * h;
        bf16x8 ah[RT], al[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            ah[t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Ph + (t * 32 + r) * kRowB + kk));
            al[t] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(Pl + (t * 32 + r) * kRowB + kk));
        }
        const bf16x8 b_h = __builtin_bit_cast(bf16x8, bh), b_l = __builtin_bit_cast(bf16x8, bl);
        // small terms first, RT independent accumulators between dependent MFMAs
#pragma unroll
        for (int t = 0; t < RT; ++t) acc[t] = MFMA_BF16(al[t], b_h, acc[t]);
#pragma unroll
        for (int t = 0; t < RT; ++t) acc[t] = MFMA_BF16(ah[t], b_l, acc[t]);
#pragma unroll
        for (int t = 0; t < RT; ++t) acc[t] = MFMA_BF16(ah[t], b_h, acc[t]);
        bh = nh;
        bl = nl;
    }
}

// bias + activation, written back in place as bf16 hi/lo planes (or fp32 for
// the LayerNorm), after every wave has finished reading the planes.
template <bool LAST, int RT>
__device__ __forceinline__ void epilogue_bf3(const float* __restrict__ bias, uint16_t* Ph, uint16_t* Pl,
                                             float* F, int ct, int lane, const floatx16 (&acc)[RT]) {
    const int r = lane & 31, h = lane >> 5;
    const int col = ct * 32 + r;
    const float bc = bias[col];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = t * 32 + (i & 3) + 8 * (i >> 2) + 4 * h;
            const float v = acc[t][i] + bc;
            if constexpr (!LAST) {
                uint32_t hi, lo;
                split_bf16(leaky(v), hi, lo);
                Ph[row * kRowB + col] = (uint16_t)hi;
                Pl[row * kRowB + col] = (uint16_t)lo;
            } else {
                F[row * kHStride + col] = v;
            }
        }
    }
}

template <int RT>
constexpr size_t head_lds_bytes() { return (size_t)2 * RT * 32 * kRowB * sizeof(uint16_t); }

template <int RT>
__global__ void __launch_bounds__(kThreadsB) k_sam_head_bf3(HeadArgsB a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
    constexpr int kRows = RT * 32;
    uint16_t* Ph = lds;                       // bf16 hi plane [kRows][kRowB]
    uint16_t* Pl = lds + kRows * kRowB;       // bf16 lo plane
    float* F = reinterpret_cast<float*>(lds); // fp32 pre-LayerNorm tile [kRows][257] (aliases the planes)
    static_assert((size_t)kRows * kHStride * 4 <= head_lds_bytes<RT>(), "LN tile must fit the planes");
    const int tid = threadIdx.x, ct = tid >> 6, lane = tid & 63;
    const uint32_t ray0 = blockIdx.x * kRows;
    for (int i = tid; i < kRows * kXkB; i += kThreadsB) {
        const int rr = i / kXkB, c = i % kXkB;
        const uint32_t ray = ray0 + rr;
        float v = 0.0f;
        if (ray < a.N && c < kIn) v = a.rows[(size_t)ray * kRowIn + c];
        uint32_t hi, lo;
        split_bf16(v, hi, lo);
        Ph[rr * kRowB + c] = (uint16_t)hi;
        Pl[rr * kRowB + c] = (uint16_t)lo;
    }
    __syncthreads();

    floatx16 acc[RT], skip[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) { acc[t] = floatx16{}; skip[t] = floatx16{}; }
    kloop_bf3<0, RT>(a, Ph, Pl, ct, lane, acc);        // layer 0: W0 . x
    kloop_bf3<5, RT>(a, Ph, Pl, ct, lane, skip);       // layer 2's W2[:, 256:] . x
    __syncthreads();
    epilogue_bf3<false, RT>(a.b[0], Ph, Pl, F, ct, lane, acc);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[t] = floatx16{};
    kloop_bf3<1, RT>(a, Ph, Pl, ct, lane, acc);        // layer 1
    __syncthreads();
    epilogue_bf3<false, RT>(a.b[1], Ph, Pl, F, ct, lane, acc);
    __syncthreads();
    kloop_bf3<2, RT>(a, Ph, Pl, ct, lane, skip);       // layer 2: + W2[:, :256] . h
    __syncthreads();
    epilogue_bf3<false, RT>(a.b[2], Ph, Pl, F, ct, lane, skip);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[t] = floatx16{};
    kloop_bf3<3, RT>(a, Ph, Pl, ct, lane, acc);        // layer 3
    __syncthreads();
    epilogue_bf3<false, RT>(a.b[3], Ph, Pl, F, ct, lane, acc);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[t] = floatx16{};
    kloop_bf3<4, RT>(a, Ph, Pl, ct, lane, acc);        // layer 4 (no activation)
    __syncthreads();
    epilogue_bf3<true, RT>(a.b[4], Ph, Pl, F, ct, lane, acc);
    __syncthreads();

    // LayerNorm(256, eps=1e-5): TPR threads per row, in double
    constexpr int TPR = kThreadsB / kRows, CPT = 256 / TPR;
    const int row = tid / TPR, q = tid % TPR;
    const float* hr = F + row * kHStride + q * CPT;
    double s = 0.0;
    for (int c = 0; c < CPT; ++c) s += (double)hr[c];
#pragma unroll
    for (int m = 1; m < TPR; m <<= 1) s += __shfl_xor(s, m, TPR);
    const double mean = s / 256.0;
    double v = 0.0;
    for (int c = 0; c < CPT; ++c) {
        const double dlt = (double)hr[c] - mean;
        v += dlt * dlt;
    }
#pragma unroll
    for (int m = 1; m < TPR; m <<= 1) v += __shfl_xor(v, m, TPR);
    const float rstd = (float)(1.0 / sqrt(v / 256.0 + 1e-5));
    const float mf = (float)mean;
    const uint32_t ray = ray0 + row;
    if (ray < a.N) {
        float* o = a.out + (size_t)ray * 256 + q * CPT;
        const float* lw = a.ln_w + q * CPT;
        const float* lb = a.ln_b + q * CPT;
        for (int c = 0; c < CPT; c += 4) {
            float4 y;
            y.x = ((hr[c + 0] - mf) * rstd) * lw[c + 0] + lb[c + 0];
            y.y = ((hr[c + 1] - mf) * rstd) * lw[c + 1] + lb[c + 1];
            y.z = ((hr[c + 2] - mf) * rstd) * lw[c + 2] + lb[c + 2];
            y.w = ((hr[c + 3] - mf) * rstd) * lw[c + 3] + lb[c + 3];
            *reinterpret_cast<float4*>(o + c) = y;
        }
    }
}

template <int RT>
int launch_head_bf3(const HeadArgsB& a, hipStream_t s) {
    static bool attr = false;                 // > 64 KB of dynamic LDS needs opting in once
    if (!attr) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sam_head_bf3<RT>),
                                hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)head_lds_bytes<RT>()) != hipSuccess)
            return fail(SAMNERF_ELAUNCH, "sam_head: cannot reserve %zu B of LDS", head_lds_bytes<RT>());
        attr = true;
    }
    k_sam_head_bf3<RT><<<div_up(a.N, RT * 32u), kThreadsB, head_lds_bytes<RT>(), s>>>(a);
    return check_launch("sam_head_bf3");
}

}  // namespace

size_t sam_head_packed_floats() {
    const size_t f32 = (size_t)8 * kTotalGroups * 64 * 4;
    const size_t bf3 = (size_t)2 * 8 * kKbTotal * 64 * 4;      // hi + lo uint4 planes
    return f32 > bf3 ? f32 : bf3;
}

int sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                     float* packed, hipStream_t s) {
    if (m->head_mode == 0) {                                     // bf16x3 (default)
        const uint32_t nvec = 8u * kKbTotal * 64u;
        uint4* phi = reinterpret_cast<uint4*>(packed);
        uint4* plo = phi + nvec;
        k_pack_bf3<<<div_up(nvec, 256), 256, 0, s>>>(m->sam_w[0], m->sam_w[1], m->sam_w[2],
                                                     m->sam_w[3], m->sam_w[4], phi, plo);
        HeadArgsB a;
        a.rows = rows;
        a.N = N;
        a.phi = phi;
        a.plo = plo;
        for (int i = 0; i < 5; ++i) a.b[i] = m->sam_b[i];
        a.ln_w = m->ln_w;
        a.ln_b = m->ln_b;
        a.out = samvit;
        // 128 rays per block when that still gives >= 2 blocks per CU, else 64
        return N >= 128u * 512u ? launch_head_bf3<4>(a, s) : launch_head_bf3<2>(a, s);
    }
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
