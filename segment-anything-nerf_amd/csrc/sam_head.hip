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
// Split-precision head (default): x = x_hi + x_lo with x_hi = bf16(x), x_lo =
// bf16(x - x_hi); A.B ~= A_lo.B_hi + A_hi.B_lo + A_hi.B_hi on
// v_mfma_f32_32x32x16_bf16 (fp32 accumulate).  Relative error per product
// ~2^-16 (the dropped A_lo.B_lo term and the rounding of the lo parts), i.e.
// ~1e-5 on the head output against the 1e-3 budget, at 3 bf16 MFMAs per
// 16-deep k-block instead of 8 fp32 ones.
//
// Orientation: out^T[256 units x 32 rays] = W . act^T -- A = weights (rows =
// output units, 8 tiles of 32), B = activations (columns = the wave's 32
// rays).  A 32x32 accumulator holds, in lane (j, h) register q, unit
// rho(q) + 4h of ray j, rho(q) = (q&3) + 8(q>>2); k-block kb of a 256-wide
// input takes registers 8(kb&1)..+7 of tile kb>>1, so after bias/activation
// and the hi/lo split a layer's accumulators ARE the next layer's B operands
// (weights are packed permuted to match, hidden_unit()).  Activations never
// leave the registers; the x input (needed again by the skip layer) stays
// resident as bf16 hi/lo.  Weights stream through LDS: one "step" = one
// k-block of one layer for all 8 output tiles = 16 KiB of hi/lo fragments,
// double-buffered and shared by the block's 4 waves (one per SIMD).
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float float2v __attribute__((ext_vector_type(2)));

constexpr int kXkb = 11;                      // 163 inputs -> 11 k-blocks of 16
constexpr int kHkb = 16;                      // 256 -> 16 k-blocks
// step segments in consumption order: L0 (x) | L1 (h) | L2 x-part | L2 h-part | L3 | L4
constexpr int kSegKb[6] = {kXkb, kHkb, kXkb, kHkb, kHkb, kHkb};
constexpr int segBase(int seg) {
    int b = 0;
    for (int i = 0; i < seg; ++i) b += kSegKb[i];
    return b;
}
constexpr int kSteps = segBase(6);            // 86
constexpr int kStepVec = 2 * 8 * 64;          // uint4 per step: [hi/lo][tile][lane]
constexpr int kRaysV5 = 128;                  // 4 waves x 32 rays

__device__ __forceinline__ int rho(int q) { return (q & 3) + 8 * (q >> 2); }
__device__ __forceinline__ int hidden_unit(int kb, int h, int m) {
    return 32 * (kb >> 1) + rho(8 * (kb & 1) + m) + 4 * h;
}

__device__ __forceinline__ void split_pair(float x, float y, uint32_t& hi, uint32_t& lo) {
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2v){x, y}, bf16x2v));
    const float hx = __uint_as_float(hi << 16), hy = __uint_as_float(hi & 0xffff0000u);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((float2v){x - hx, y - hy}, bf16x2v));
}
__device__ __forceinline__ void split8(const float* v, uint4& hi, uint4& lo) {
    split_pair(v[0], v[1], hi.x, lo.x);
    split_pair(v[2], v[3], hi.y, lo.y);
    split_pair(v[4], v[5], hi.z, lo.z);
    split_pair(v[6], v[7], hi.w, lo.w);
}

// packed[step 86][hi/lo][tile 8][lane 64] : 8 bf16 (16 B) each
__global__ void __launch_bounds__(256)
k_pack_bf3(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
           const float* __restrict__ w3, const float* __restrict__ w4, uint4* __restrict__ packed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;   // one (step, tile, lane)
    if (t >= (uint32_t)kSteps * 8u * 64u) return;
    const int lane = (int)(t & 63u), tile = (int)((t >> 6) & 7u), step = (int)(t >> 9);
    int seg = 0;
    while (seg < 5 && step >= segBase(seg + 1)) ++seg;
    const int kb = step - segBase(seg);
    const int i = lane & 31, h = lane >> 5, unit = tile * 32 + i;
    float v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int kx = 16 * kb + 8 * h + m;           // x input column (natural order)
        const int kh = hidden_unit(kb, h, m);         // hidden input unit (accumulator order)
        float w;
        switch (seg) {
            case 0: w = kx < kIn ? w0[unit * kIn + kx] : 0.0f; break;
            case 1: w = w1[unit * 256 + kh]; break;
            case 2: w = kx < kIn ? w2[unit * (256 + kIn) + 256 + kx] : 0.0f; break;
            case 3: w = w2[unit * (256 + kIn) + kh]; break;
            case 4: w = w3[unit * 256 + kh]; break;
            default: w = w4[unit * 256 + kh]; break;
        }
        v[m] = w;
    }
    uint4 hi, lo;
    split8(v, hi, lo);
    packed[(size_t)step * kStepVec + tile * 64 + lane] = hi;
    packed[(size_t)step * kStepVec + 512 + tile * 64 + lane] = lo;
}

struct HeadArgsB {
    const float* rows;
    uint32_t N;
    const uint4* packed;
    const float* b[5];
    const float* ln_w;
    const float* ln_b;
    float* out;
};

#define MFMA_BF16(A, B, C) __builtin_amdgcn_mfma_f32_32x32x16_bf16((A), (B), (C), 0, 0, 0)

__device__ __forceinline__ floatx16 mfma3(uint4 ah, uint4 al, uint4 bh, uint4 bl, floatx16 c) {
    const bf16x8 Ah = __builtin_bit_cast(bf16x8, ah), Al = __builtin_bit_cast(bf16x8, al);
    const bf16x8 Bh = __builtin_bit_cast(bf16x8, bh), Bl = __builtin_bit_cast(bf16x8, bl);
    c = MFMA_BF16(Al, Bh, c);
    c = MFMA_BF16(Ah, Bl, c);
    return MFMA_BF16(Ah, Bh, c);
}

typedef __attribute__((address_space(1))) const void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// Weight stream: step s's 16 KiB of fragments go global -> LDS by direct DMA
// (global_load_lds_dwordx4, no VGPRs), into one of 3 buffers, two steps
// ahead; each wave moves 4 KiB (4 wave-instructions of 64 x 16 B).  The step
// boundary waits only for the step about to be read (counted vmcnt, one step
// stays in flight across the raw barrier), per cdna_hip_programming.md
// "Pipelining across barriers".
struct HeadStepper {
    const uint4* __restrict__ packed;
    uint4* Wb;            // LDS [3][kStepVec]
    int wave, lane;
    int step;

    // The DMA is issued from inline asm so that the compiler does not see an
    // LDS write of unknown extent in flight (it would drain vmcnt(0) before
    // every ds_read); the waits are counted by hand in run().  No ordinary
    // vector-memory load is issued inside the step loop.
    __device__ __forceinline__ void issue(int s) {
        const uint4* src = packed + (size_t)s * kStepVec + wave * 256 + lane;
        const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>(Wb + (s % 3) * kStepVec + wave * 256);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t d = __builtin_amdgcn_readfirstlane(dst + c * 1024u);
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(src + c * 64), "s"(d)
                : "memory");
        }
    }

    // one k-block of the current layer for all 8 output tiles.  (Holding the
    // next step's fragments in registers, read under this step's MFMAs with
    // the skip layer's h-part moved first to make room, measured no faster:
    // 0.581 vs 0.575 ms per view, with 21 VGPRs spilled.)
    __device__ __forceinline__ void run(floatx16 (&acc)[8], const uint4& bh, const uint4& bl) {
        const bool ahead = step + 2 < kSteps;
        if (ahead) issue(step + 2);
        const uint4* cur = Wb + (step % 3) * kStepVec + lane;
        uint4 fh[8], fl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            fh[t] = cur[t * 64];
            fl[t] = cur[512 + t * 64];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma3(fh[t], fl[t], bh, bl, acc[t]);
        if (ahead) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");   // step + 1 landed
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ++step;
    }
};

// SAMNERF_HEAD_STAGE=1: the same stream staged through VGPRs by ordinary
// loads (mask_head.hip's MaskStager): each thread loads its four 16-B pieces
// of step s + 1 at the start of step s and writes them to the other half of a
// 2-step LDS ring after step s's MFMAs, then the barrier.  500 VGPRs, no
// spills, but slower here: 0.58 -> 0.82 ms per view (one step of lookahead
// exposes the load latency before the store; the DMA runs two steps ahead
// without registers).  The mask head, whose DMA form spilled, gains from it.
#ifndef SAMNERF_HEAD_STAGE
#define SAMNERF_HEAD_STAGE 0
#endif
struct HeadStager {
    const uint4* __restrict__ packed;
    uint4* Wb;            // LDS [2][kStepVec]
    int tid, lane;
    int step;
    uint4 stg[4];

    __device__ __forceinline__ void load(int s) {
        const uint4* src = packed + (size_t)s * kStepVec + tid;
#pragma unroll
        for (int c = 0; c < 4; ++c) stg[c] = src[c * 256];
    }
    __device__ __forceinline__ void store(int s) {
        uint4* dst = Wb + (s & 1) * kStepVec + tid;
#pragma unroll
        for (int c = 0; c < 4; ++c) dst[c * 256] = stg[c];
    }
    __device__ __forceinline__ void begin() {
        load(0);
        store(0);
        __syncthreads();
    }
    __device__ __forceinline__ void run(floatx16 (&acc)[8], const uint4& bh, const uint4& bl) {
        const bool ahead = step + 1 < kSteps;
        if (ahead) load(step + 1);
        const uint4* cur = Wb + (step & 1) * kStepVec + lane;
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = mfma3(cur[t * 64], cur[512 + t * 64], bh, bl, acc[t]);
        if (ahead) store(step + 1);
        __syncthreads();
        ++step;
    }
};

__device__ __forceinline__ float leaky(float x, bool act) { return act && x < 0.0f ? x * 0.01f : x; }

// bias (+ leaky_relu) on the accumulators, then the hi/lo split into the next
// layer's B operands (k-block kb = 2t + s <- registers 8s..8s+7 of tile t)
__device__ __forceinline__ void epilogue(const floatx16 (&acc)[8], const float* Bs, int h,
                                         uint4 (&ah)[kHkb], uint4 (&al)[kHkb]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        float v[16];
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {      // registers 4mm..4mm+3 = units 32t + 8mm + 4h + 0..3
            const float4 bb = *reinterpret_cast<const float4*>(Bs + 32 * t + 8 * mm + 4 * h);
            v[4 * mm + 0] = leaky(acc[t][4 * mm + 0] + bb.x, true);
            v[4 * mm + 1] = leaky(acc[t][4 * mm + 1] + bb.y, true);
            v[4 * mm + 2] = leaky(acc[t][4 * mm + 2] + bb.z, true);
            v[4 * mm + 3] = leaky(acc[t][4 * mm + 3] + bb.w, true);
        }
        split8(v, ah[2 * t], al[2 * t]);
        split8(v + 8, ah[2 * t + 1], al[2 * t + 1]);
    }
}

// One tile's epilogue (bias + leaky_relu, then the hi/lo split): the B
// operands of k-blocks 2t and 2t + 1 of the next layer.
__device__ __forceinline__ void epilogue_tile(const floatx16& acc, const float* Bs, int t, int h, uint4& h0,
                                              uint4& l0, uint4& h1, uint4& l1) {
    float v[16];
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
        const float4 bb = *reinterpret_cast<const float4*>(Bs + 32 * t + 8 * mm + 4 * h);
        v[4 * mm + 0] = leaky(acc[4 * mm + 0] + bb.x, true);
        v[4 * mm + 1] = leaky(acc[4 * mm + 1] + bb.y, true);
        v[4 * mm + 2] = leaky(acc[4 * mm + 2] + bb.z, true);
        v[4 * mm + 3] = leaky(acc[4 * mm + 3] + bb.w, true);
    }
    split8(v, h0, l0);
    split8(v + 8, h1, l1);
}

// SAMNERF_HEAD_LAZY=1: two accumulator sets that alternate by layer, and each
// layer's epilogue done tile by tile just before the next layer's k-blocks
// that read it (k-blocks 2t, 2t + 1 read tile t), so the VALU epilogue runs
// beside the previous step's MFMAs instead of between layers with the matrix
// cores idle (the round-1 VERDICT's suggestion).  The B operands no longer sit
// in 128 registers for a whole layer, which pays for the second set.
#ifndef SAMNERF_HEAD_LAZY
#define SAMNERF_HEAD_LAZY 0
#endif

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_sam_head_bf3(HeadArgsB a) {
    // one LDS object (a second __shared__ object can de-pipeline the DMA
    // waits): 3 x 16 KiB weight steps, then biases and LN weight/bias
    constexpr int kRingSteps = SAMNERF_HEAD_STAGE ? 2 : 3;
    __shared__ uint4 smem[kRingSteps * kStepVec + (7 * 256) / 4];
    uint4* Wb = smem;
    float* Bs = reinterpret_cast<float*>(smem + kRingSteps * kStepVec);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 31, h = lane >> 5;
    const uint32_t ray = blockIdx.x * kRaysV5 + wave * 32u + j;
    const bool live = ray < a.N;

    for (int i = tid; i < 5 * 256; i += 256) Bs[i] = a.b[i >> 8][i & 255];
    Bs[5 * 256 + tid] = a.ln_w[tid];
    Bs[6 * 256 + tid] = a.ln_b[tid];

    // x (head input row) as B operands: k-block kb, lane half h -> columns
    // 16kb + 8h .. +7; loaded again for the skip layer rather than held in
    // 88 VGPRs through layer 1
    const float* xr = a.rows + (size_t)(live ? ray : 0u) * kRowIn;
    auto load_x = [&](int kb, uint4& xh, uint4& xl) {
        float v[8];
        const int c0 = 16 * kb + 8 * h;
        if (c0 + 8 <= kRowIn) {
            const float4 p = *reinterpret_cast<const float4*>(xr + c0);
            const float4 q = *reinterpret_cast<const float4*>(xr + c0 + 4);
            v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
            v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = c0 + m < kRowIn ? xr[c0 + m] : 0.0f;
        }
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!live || c0 + m >= kIn) v[m] = 0.0f;      // column 163 of a row is padding
        split8(v, xh, xl);
    };
    uint4 xh[kXkb], xl[kXkb];
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) load_x(kb, xh[kb], xl[kb]);
#if SAMNERF_HEAD_STAGE
    HeadStager st{a.packed, Wb, tid, lane, 0, {}};
    st.begin();
#else
    HeadStepper st{a.packed, Wb, wave, lane, 0};
    st.issue(0);
    st.issue(1);
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");          // step 0 landed
    __syncthreads();
#endif
#if SAMNERF_HEAD_LAZY
    floatx16 accA[8], accB[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) accA[t] = floatx16{};
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(accA, xh[kb], xl[kb]);        // layer 0 -> A
    // one hidden layer from `src` (its pre-activations) into `dst`
    auto hidden = [&](floatx16 (&src)[8], floatx16 (&dst)[8], const float* bias) {
        uint4 ch0, cl0, ch1, cl1;
#pragma unroll
        for (int kb = 0; kb < kHkb; ++kb) {
            if ((kb & 1) == 0) epilogue_tile(src[kb >> 1], bias, kb >> 1, h, ch0, cl0, ch1, cl1);
            if (kb & 1) st.run(dst, ch1, cl1);
            else st.run(dst, ch0, cl0);
        }
    };
#pragma unroll
    for (int t = 0; t < 8; ++t) accB[t] = floatx16{};
    hidden(accA, accB, Bs + 0 * 256);                                      // layer 1 -> B
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) load_x(kb, xh[kb], xl[kb]);
#pragma unroll
    for (int t = 0; t < 8; ++t) accA[t] = floatx16{};
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(accA, xh[kb], xl[kb]);       // layer 2: x part -> A
    hidden(accB, accA, Bs + 1 * 256);                                      //          h part
#pragma unroll
    for (int t = 0; t < 8; ++t) accB[t] = floatx16{};
    hidden(accA, accB, Bs + 2 * 256);                                      // layer 3 -> B
#pragma unroll
    for (int t = 0; t < 8; ++t) accA[t] = floatx16{};
    hidden(accB, accA, Bs + 3 * 256);                                      // layer 4 -> A
    floatx16 (&acc)[8] = accA;
#else
    floatx16 acc[8];
    uint4 ah[kHkb], al[kHkb];
    auto zero = [&]() {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = floatx16{};
    };

    zero();                                                   // layer 0: W0 . x
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
    epilogue(acc, Bs + 0 * 256, h, ah, al);
    zero();                                                   // layer 1
#pragma unroll
    for (int kb = 0; kb < kHkb; ++kb) st.run(acc, ah[kb], al[kb]);
    epilogue(acc, Bs + 1 * 256, h, ah, al);
    zero();                                                   // layer 2: W2 . cat(h, x)
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) load_x(kb, xh[kb], xl[kb]);
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
#pragma unroll
    for (int kb = 0; kb < kHkb; ++kb) st.run(acc, ah[kb], al[kb]);
    epilogue(acc, Bs + 2 * 256, h, ah, al);
    zero();                                                   // layer 3
#pragma unroll
    for (int kb = 0; kb < kHkb; ++kb) st.run(acc, ah[kb], al[kb]);
    epilogue(acc, Bs + 3 * 256, h, ah, al);
    zero();                                                   // layer 4 (no activation)
#pragma unroll
    for (int kb = 0; kb < kHkb; ++kb) st.run(acc, ah[kb], al[kb]);
#endif

    // + bias, LayerNorm(256, eps=1e-5) per ray: this lane holds 128 of the
    // ray's units, the other half-wave (lane ^ 32) the rest; sums in double
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            acc[t][q] += Bs[4 * 256 + 32 * t + rho(q) + 4 * h];
            s += (double)acc[t][q];
        }
    s += __shfl_xor(s, 32);
    const double mean = s / 256.0;
    double var = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const double dlt = (double)acc[t][q] - mean;
            var += dlt * dlt;
        }
    var += __shfl_xor(var, 32);
    const float rstd = (float)(1.0 / sqrt(var / 256.0 + 1e-5));
    const float mf = (float)mean;
    if (!live) return;
    float* o = a.out + (size_t)ray * 256;
    const float* lw = Bs + 5 * 256;
    const float* lb = Bs + 6 * 256;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const int u = 32 * t + 8 * mm + 4 * h;
            float4 y;
            y.x = ((acc[t][4 * mm + 0] - mf) * rstd) * lw[u + 0] + lb[u + 0];
            y.y = ((acc[t][4 * mm + 1] - mf) * rstd) * lw[u + 1] + lb[u + 1];
            y.z = ((acc[t][4 * mm + 2] - mf) * rstd) * lw[u + 2] + lb[u + 2];
            y.w = ((acc[t][4 * mm + 3] - mf) * rstd) * lw[u + 3] + lb[u + 3];
            *reinterpret_cast<float4*>(o + u) = y;
        }
}

}  // namespace

size_t sam_head_packed_floats() {
    const size_t f32 = (size_t)8 * kTotalGroups * 64 * 4;
    const size_t bf3 = (size_t)kSteps * kStepVec * 4;        // uint4 fragments
    return f32 > bf3 ? f32 : bf3;
}

int sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                     float* packed, hipStream_t s) {
    if (m->head_mode == 0) {                                     // bf16x3 (default)
        uint4* pk = reinterpret_cast<uint4*>(packed);
        const uint32_t nfrag = (uint32_t)kSteps * 8u * 64u;
        k_pack_bf3<<<div_up(nfrag, 256), 256, 0, s>>>(m->sam_w[0], m->sam_w[1], m->sam_w[2],
                                                      m->sam_w[3], m->sam_w[4], pk);
        HeadArgsB a;
        a.rows = rows;
        a.N = N;
        a.packed = pk;
        for (int i = 0; i < 5; ++i) a.b[i] = m->sam_b[i];
        a.ln_w = m->ln_w;
        a.ln_b = m->ln_b;
        a.out = samvit;
        k_sam_head_bf3<<<div_up(N, (uint32_t)kRaysV5), 256, 0, s>>>(a);
        return check_launch("sam_head_bf3");
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
