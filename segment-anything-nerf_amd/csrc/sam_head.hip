// sam_head.hip -- the SAM-feature head on gfx950 matrix cores.
//
// samvit_mlp = Sequential(SkipConnMLP(163, 256, 256, 5, skip_layers=[2],
// bias=True), LayerNorm(256)) (nerf/network.py:36-75, :120-123), applied per
// ray to f = cat(f_sam, f_image, image, depth) (nerf/renderer.py:377-385).
//
// fp32 in / fp32 accumulate on v_mfma_f32_32x32x2_f32 (exact f32 FMA chains,
// cdna_hip_programming.md section 3 "FP32-input MFMA") so the head keeps the
// 1e-3 parity budget that bf16 operands would spend.  This is
// head_mode 1; the default (head_mode 0) is the f16x3 head below.
//   * one workgroup = 32 rays x all 256 output columns, 4 waves, each wave two
//     32x32 accumulator tiles;
//   * activations live in LDS (odd row strides: conflict-free ds_read_b32 for
//     the A operand, lane = row), the 5 layers run back to back in the same
//     workgroup, bias + leaky_relu(0.01) and the final LayerNorm fused;
//   * weights are re-packed once per call so each B fragment group (4 k-steps
//     of one 32-column tile) is one contiguous 1 KiB wave load (16 B per lane)
//     from L2.
#include "samnerf_common.h"
#include "f16x3.h"

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
    float* out;            // [N, 256], row stride ld
    uint32_t ld;           // 256, or the gather tile's row (samnerf_render_forward_tile)
    bool vec_out;          // rows 16-B aligned: float4 stores
};

// samvit output store of 4 consecutive features: one 16-B store when the rows
// are 16-B aligned (the [N, 256] output), four 4-B stores inside a gather tile
// whose rows are not (kernel-uniform branch)
__device__ __forceinline__ void store_out4(float* p, const float4& y, bool vec) {
    if (vec) {
        *reinterpret_cast<float4*>(p) = y;
    } else {
        p[0] = y.x;
        p[1] = y.y;
        p[2] = y.z;
        p[3] = y.w;
    }
}

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
        float* o = a.out + (size_t)ray * a.ld + q * 32;
        for (int c = 0; c < 32; c += 4) {
            float4 y;
            y.x = ((hr[c + 0] - mf) * rstd) * a.ln_w[q * 32 + c + 0] + a.ln_b[q * 32 + c + 0];
            y.y = ((hr[c + 1] - mf) * rstd) * a.ln_w[q * 32 + c + 1] + a.ln_b[q * 32 + c + 1];
            y.z = ((hr[c + 2] - mf) * rstd) * a.ln_w[q * 32 + c + 2] + a.ln_b[q * 32 + c + 2];
            y.w = ((hr[c + 3] - mf) * rstd) * a.ln_w[q * 32 + c + 3] + a.ln_b[q * 32 + c + 3];
            store_out4(o + c, y, a.vec_out);
        }
    }
}


// ===================================================================== f16x3
// fp32-equivalent head (default, f16x3.h): each fp32 product as three fp16
// MFMA products on power-of-two scaled operands -- each weight tensor scaled
// at packing (k_head_wmax + k_pack_h16), each ray's activations at run time
// from their max over the layer's inputs.  Error against float64 at the
// level of an exact fp32 GEMM (tools/f16x3_error.py), at 3 v_mfma_f32_32x32x16_f16
// per 16-deep k-block instead of 8 fp32 MFMAs of twice the cycles.
//
// Orientation: out^T[256 units x 32 rays] = W . act^T -- A = weights (rows =
// output units, 8 tiles of 32), B = activations (columns = the wave's 32
// rays).  A 32x32 accumulator holds, in lane (j, h) register q, unit
// rho(q) + 4h of ray j, rho(q) = (q&3) + 8(q>>2); k-block kb of a 256-wide
// input takes registers 8(kb&1)..+7 of tile kb>>1, so after bias/activation,
// scaling and the hi/lo split a layer's accumulators ARE the next layer's B
// operands (weights are packed permuted to match, hidden_unit()).  Activations
// never leave the registers; the x input (needed again by the skip layer) is
// re-read from the rows.  Weights stream through LDS: one "step" = one k-block
// of one layer for all 8 output tiles = 16 KiB of hi/lo fragments, three
// buffers shared by the block's 4 waves (one per SIMD).
constexpr int kXkb = 11;                      // 163 inputs -> 11 k-blocks of 16
constexpr int kHkb = 16;                      // 256 -> 16 k-blocks
// step segments in consumption order: L0 (x) | L1 (h) | L2 x-part | L2 h-part | L3 | L4
constexpr int kSegKb[6] = {kXkb, kHkb, kXkb, kHkb, kHkb, kHkb};
constexpr int kSegLayer[6] = {0, 1, 2, 2, 3, 4};
constexpr int segBase(int seg) {
    int b = 0;
    for (int i = 0; i < seg; ++i) b += kSegKb[i];
    return b;
}
constexpr int kSteps = segBase(6);            // 86
constexpr int kStepVec = 2 * 8 * 64;          // uint4 per step: [hi/lo][tile][lane]
constexpr int kRaysV5 = 128;                  // 4 waves x 32 rays
constexpr int kPackedVec = kSteps * kStepVec; // uint4 of fragments; then kexp [5] ints
// Copies of the packed fragments: every workgroup streams the same 16 KiB
// step at about the same time, so with one copy the whole chip's requests for
// a step land on the few L2 channels that hold it; workgroup b reads copy
// (b >> 3) % kHeadCopies (b & 7 is its XCD), spreading each XCD's requests
// over kHeadCopies x as many channels.  The copies hold the same bits.
// Measured (round 4, interleaved A/B of whole builds, 512^2 view): 8 copies
// 0.569 ms per head launch against 0.566 with one -- the step stream is not
// channel-bound -- so the product keeps one (the switch stays for A/B builds).
#ifndef SAMNERF_HEAD_COPIES
#define SAMNERF_HEAD_COPIES 1
#endif
constexpr int kHeadCopies = SAMNERF_HEAD_COPIES;

__device__ __forceinline__ int rho(int q) { return (q & 3) + 8 * (q >> 2); }
__device__ __forceinline__ int hidden_unit(int kb, int h, int m) {
    return 32 * (kb >> 1) + rho(8 * (kb & 1) + m) + 4 * h;
}

// weight of segment `seg`, k-block kb, lane half h, element m for output unit
__device__ __forceinline__ float seg_weight(const float* const* W, int seg, int kb, int h, int m, int unit) {
    const int kx = 16 * kb + 8 * h + m;           // x input column (natural order)
    const int kh = hidden_unit(kb, h, m);         // hidden input unit (accumulator order)
    switch (seg) {
        case 0: return kx < kIn ? W[0][unit * kIn + kx] : 0.0f;
        case 1: return W[1][unit * 256 + kh];
        case 2: return kx < kIn ? W[2][unit * (256 + kIn) + 256 + kx] : 0.0f;
        case 3: return W[2][unit * (256 + kIn) + kh];
        case 4: return W[3][unit * 256 + kh];
        default: return W[4][unit * 256 + kh];
    }
}

// packed[step 86][hi/lo][tile 8][lane 64] (8 f16 = 16 B each), then kexp[5]:
// each weight tensor scaled by the power of two that puts its max |w| in
// [2^13, 2^14) (f16x3.h), kexp = log2 of that scale.  k_head_wmax finds the
// five maxima as kWmaxParts partial maxima per tensor (5 x 32 workgroups: the
// one-workgroup-per-tensor form took 32 us per view, a serial chain of ~100
// loads per thread), k_pack_h16 folds a tensor's partials per workgroup, keeps
// kexp and writes the fragments (one thread per fragment).
constexpr int kWmaxParts = 32;
struct PackArgs {
    const float* W[5];
    uint4* packed;
    int* kexp;
    float* part;             // [5][kWmaxParts] partial maxima
};
__global__ void __launch_bounds__(256) k_head_wmax(PackArgs a) {
    __shared__ float wm[4];
    const int layer = blockIdx.y, tid = threadIdx.x;
    const int n = 256 * kLogicalIn[layer];
    const int chunk = (n + kWmaxParts - 1) / kWmaxParts;
    const int i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
    const float* W = a.W[layer];
    float m = 0.0f;
#pragma unroll 4
    for (int i = i0 + tid; i < i1; i += 256) m = fmaxf(m, fabsf(W[i]));
    m = wave_max64(m);
    if ((tid & 63) == 0) wm[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) a.part[layer * kWmaxParts + blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}
__global__ void __launch_bounds__(256) k_pack_h16(PackArgs a) {
    __shared__ int kx;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;   // one (step, tile, lane)
    // a workgroup's 256 fragments are half of one step: one layer
    const int bstep = (int)((blockIdx.x * blockDim.x) >> 9);
    int bseg = 0;
    while (bseg < 5 && bstep >= segBase(bseg + 1)) ++bseg;
    const int layer = kSegLayer[bseg];
    if (threadIdx.x < 64) {
        float m = threadIdx.x < kWmaxParts ? a.part[layer * kWmaxParts + threadIdx.x] : 0.0f;
        m = wave_max64(m);
        if (threadIdx.x == 0) {
            kx = scale_exp_of_max(m);
            a.kexp[layer] = kx;                 // the same value from every workgroup of the layer
        }
    }
    __syncthreads();
    if (t >= (uint32_t)kSteps * 8u * 64u) return;
    const int lane = (int)(t & 63u), tile = (int)((t >> 6) & 7u), step = (int)(t >> 9);
    int seg = 0;
    while (seg < 5 && step >= segBase(seg + 1)) ++seg;
    const int kb = step - segBase(seg);
    const int j = lane & 31, h = lane >> 5, unit = tile * 32 + j;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = seg_weight(a.W, seg, kb, h, e, unit);
    uint4 hi, lo;
    split8_f16(v, exp2i(kx), hi, lo);
#pragma unroll
    for (int c = 0; c < kHeadCopies; ++c) {
        a.packed[(size_t)c * kPackedVec + (size_t)step * kStepVec + tile * 64 + lane] = hi;
        a.packed[(size_t)c * kPackedVec + (size_t)step * kStepVec + 512 + tile * 64 + lane] = lo;
    }
}

struct HeadArgsH {
    const float* rows;
    uint32_t N;
    const uint4* packed;
    const int* kexp;
    const float* b[5];
    const float* ln_w;
    const float* ln_b;
    float* out;            // [N, 256], row stride ld
    uint32_t ld;
    bool vec_out;
    unsigned long long* stamps;   // diagnostic form 13 only: [block][wave][16] s_memtime marks
};

// Weight stream: step s's 16 KiB of fragments go global -> LDS by direct DMA
// (global_load_lds_dwordx4, no VGPRs), into one of 3 buffers, two steps
// ahead; each wave moves 4 KiB (4 wave-instructions of 64 x 16 B).  The step
// boundary waits only for the step about to be read (counted vmcnt, one step
// stays in flight across the raw barrier), per cdna_hip_programming.md
// "Pipelining across barriers".
// vmcnt(N) for N = 0, 2, 4, 8, 16 (the waits are counted by hand: the DMA is inline asm);
// wait_vmn: any N that folds to a constant (0..63)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N == 0 || N == 2 || N == 4 || N == 5 || N == 6 || N == 8 || N == 16, "vmcnt literal");
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
}

// 16 B per lane, global -> LDS at lds_byte_addr + 16 lane (direct DMA, no
// VGPRs; counted in vmcnt, waited by hand)
__device__ __forceinline__ void lds_dma16(const void* src, uint32_t lds_byte_addr) {
    const uint32_t d = __builtin_amdgcn_readfirstlane(lds_byte_addr);
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(src), "s"(d)
        : "memory");
}

__device__ __forceinline__ void wait_vmn(int n) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory");
}

// The weight stream in "super-steps" of KPS k-blocks (KPS x 16 KiB): NBUF
// LDS buffers, the DMA NBUF - 1 super-steps ahead, one barrier per
// super-step (the k-blocks of a super-step may straddle a layer boundary: the
// barrier only guards the weight buffers).  SPREAD: the DMA pieces are issued
// between the MFMAs (one after every second tile) instead of before them.
template <int NBUF, bool SPREAD, int KPS_>
struct HeadStepper {
    // KPS_ 0: the diagnostic no-DMA form (one k-block per barrier, the weight
    // stream skipped: wrong results, for timing what the DMA costs)
    static constexpr int KPS = KPS_ ? KPS_ : 1;
    static constexpr bool kNoDma = KPS_ == 0;
    static constexpr int kSuper = (kSteps + KPS - 1) / KPS;
    static constexpr int kPieces = 4 * KPS;                  // 1-KiB pieces per wave and super-step
    const uint4* __restrict__ packed;
    uint4* Wb;            // LDS [NBUF][KPS][kStepVec]
    int wave, lane;
    int step;             // k-block

    // The DMA is issued from inline asm so that the compiler does not see an
    // LDS write of unknown extent in flight (it would drain vmcnt(0) before
    // every ds_read); the waits are counted by hand in run().  No ordinary
    // vector-memory load is issued inside the step loop.
    __device__ __forceinline__ void piece(int S, int c) {
        if constexpr (kNoDma) return;
        const size_t chunk = (size_t)wave * 256 * KPS + (size_t)c * 64;
        const uint4* src = packed + (size_t)S * KPS * kStepVec + chunk + lane;
        const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>(Wb + (S % NBUF) * KPS * kStepVec + chunk);
        const uint32_t d = __builtin_amdgcn_readfirstlane(dst);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(src), "s"(d)
            : "memory");
    }
    __device__ __forceinline__ void issue(int S) {
#pragma unroll
        for (int c = 0; c < kPieces; ++c) piece(S, c);
    }
    __device__ __forceinline__ void begin() {
#pragma unroll
        for (int q = 0; q < NBUF - 1; ++q) issue(q);
        wait_vm<kPieces * (NBUF - 2)>();                      // super-step 0 landed
        __syncthreads();
    }

    // one k-block of the current layer for all 8 output tiles
    __device__ __forceinline__ void run(floatx16 (&acc)[8], const uint4& bh, const uint4& bl) {
        const int S = step / KPS, sub = step % KPS;
        const bool ahead = S + NBUF - 1 < kSuper;
        if (!SPREAD && sub == 0 && ahead) issue(S + NBUF - 1);
        const uint4* cur = Wb + ((S % NBUF) * KPS + sub) * kStepVec + lane;
        uint4 fh[8], fl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            fh[t] = cur[t * 64];
            fl[t] = cur[512 + t * 64];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            acc[t] = mfma_f16x3(fh[t], fl[t], bh, bl, acc[t]);
            if (SPREAD && (t & 1) && ahead) {
                __builtin_amdgcn_sched_barrier(0);
                piece(S + NBUF - 1, 4 * sub + (t >> 1));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (sub == KPS - 1 || step + 1 == kSteps) {
            if (ahead) wait_vm<kPieces * (NBUF - 2)>();      // super-step S + 1 landed
            else wait_vm<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        }
        ++step;
    }
};

// leaky_relu(0.01) as max(x, 0.01 x): the same value for every x (x >= 0, -0.0
// included, gives x; x < 0 gives 0.01 x), two VALU instead of three; x is an
// arithmetic result (canonical), so fmaxf needs no canonicalising move
__device__ __forceinline__ float leaky(float x, bool act) { return act ? fmaxf(x, x * 0.01f) : x; }

// The accumulators of a layer back to fp32 values in place: times `inv` (the
// inverse of the column's input scale and of the weight tensor's scale: a
// power of two, so acc * inv is exact) + bias in one rounding, leaky_relu when
// `act`; returns this lane's max |value| (the ray's other units are on lane ^ 32).
__device__ __forceinline__ float finish_layer(floatx16 (&acc)[8], const float* Bs, float inv, int h, bool act) {
    float m = 0.0f;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {       // registers 4mm..4mm+3 = units 32t + 8mm + 4h + 0..3
            const float4 bb = *reinterpret_cast<const float4*>(Bs + 32 * t + 8 * mm + 4 * h);
            const float b4[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                acc[t][4 * mm + e] = leaky(__builtin_fmaf(acc[t][4 * mm + e], inv, b4[e]), act);
#pragma unroll
            for (int e = 0; e < 4; e += 2) m = max_abs3(m, acc[t][4 * mm + e], acc[t][4 * mm + e + 1]);
        }
    return m;
}

// the values (times s) as the next layer's B operands: k-block kb = 2t + c
// <- registers 8c..8c+7 of tile t
__device__ __forceinline__ void split_layer(const floatx16 (&acc)[8], float s, uint4 (&ah)[kHkb],
                                            uint4 (&al)[kHkb]) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = acc[t][q];
        split8_f16(v, s, ah[2 * t], al[2 * t]);
        split8_f16(v + 8, s, ah[2 * t + 1], al[2 * t + 1]);
    }
}

// LAZY (diagnostic form 12, measured 3 % slower): a layer's values stay fp32
// through the next layer and each k-block's B operands are split right before
// its step, inside the MFMA shadow, instead of at the layer boundary
// STAMP (diagnostic form 13): s_memtime at the phase boundaries of every wave
// (kernel start, stream primed, each layer's steps, each layer boundary, the
// LayerNorm), written by lane 0 at the end: where the cycles of a wave go
template <int NBUF, bool SPREAD, int KPS, bool LAZY = false, bool STAMP = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_sam_head_h16(HeadArgsH a) {
    unsigned long long ts[16];
    auto mark = [&](int i) {
        if constexpr (STAMP) {
            __builtin_amdgcn_sched_barrier(0);
            ts[i] = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    mark(0);
    unsigned long long rt0 = 0;
    if constexpr (STAMP) rt0 = __builtin_amdgcn_s_memrealtime();
    // one LDS object (a second __shared__ object can de-pipeline the DMA
    // waits): 3 x 16 KiB weight steps, then biases [5][256], LN weight / bias,
    // the weight tensors' inverse scales [5]
    constexpr int kBufVec = NBUF * (KPS ? KPS : 1) * kStepVec;
    __shared__ uint4 smem[kBufVec + (7 * 256 + 8) / 4];
    uint4* Wb = smem;
    float* Bs = reinterpret_cast<float*>(smem + kBufVec);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 31, h = lane >> 5;
    const uint32_t ray = blockIdx.x * kRaysV5 + wave * 32u + j;
    const bool live = ray < a.N;

    for (int i = tid; i < 5 * 256; i += 256) Bs[i] = a.b[i >> 8][i & 255];
    float* const Wi = Bs + 7 * 256;                       // 2^-kexp[l]
    if (tid < 5) Wi[tid] = exp2i(-a.kexp[tid]);
    Bs[5 * 256 + tid] = a.ln_w[tid];
    Bs[6 * 256 + tid] = a.ln_b[tid];

    // x (head input row) as B operands: k-block kb, lane half h -> columns
    // 16kb + 8h .. +7; read again for the skip layer rather than held in 88
    // VGPRs through layer 1
    const float* xr = a.rows + (size_t)(live ? ray : 0u) * kRowIn;
    auto x8 = [&](int kb, float (&v)[8]) {
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
    };
    float xmax = 0.0f;                                    // the ray's max |x| (both half-waves)
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) {
        float v[8];
        x8(kb, v);
#pragma unroll
        for (int m = 0; m < 8; ++m) xmax = fmaxf(xmax, fabsf(v[m]));
    }
    xmax = fmaxf(xmax, __shfl_xor(xmax, 32));
    auto load_x = [&](float s, uint4 (&xh)[kXkb], uint4 (&xl)[kXkb]) {
#pragma unroll
        for (int kb = 0; kb < kXkb; ++kb) {
            float v[8];
            x8(kb, v);
            split8_f16(v, s, xh[kb], xl[kb]);
        }
    };
    uint4 xh[kXkb], xl[kXkb];
    Scale2 sc = scale_of_max(xmax);
    load_x(sc.s, xh, xl);
    HeadStepper<NBUF, SPREAD, KPS> st{};
    st.packed = a.packed;
    st.Wb = Wb;
    st.wave = wave;
    st.lane = lane;
    st.step = 0;
    st.begin();
    mark(1);

    floatx16 acc[8];
    uint4 ah[LAZY ? 1 : kHkb], al[LAZY ? 1 : kHkb];
    floatx16 hv[LAZY ? 8 : 1];                                // LAZY: the previous layer's values
    auto zero = [&]() {
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = floatx16{};
    };
    // the layer's values, then the next layer's B operands at the scale of
    // their max (and of `extra`, another input of the same layer)
    auto next = [&](int layer, float extra) {
        float m = finish_layer(acc, Bs + layer * 256, sc.inv * Wi[layer], h, true);
        m = fmaxf(fmaxf(m, __shfl_xor(m, 32)), extra);
        sc = scale_of_max(m);
        if constexpr (LAZY) {
#pragma unroll
            for (int t = 0; t < 8; ++t) hv[t] = acc[t];
        } else {
            split_layer(acc, sc.s, ah, al);
        }
    };
    // one layer's 16 hidden-input k-blocks
    auto h_segment = [&]() {
#pragma unroll
        for (int kb = 0; kb < kHkb; ++kb) {
            if constexpr (LAZY) {
                float v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = hv[kb >> 1][8 * (kb & 1) + q];
                uint4 bh, bl;
                split8_f16(v, sc.s, bh, bl);
                st.run(acc, bh, bl);
            } else {
                st.run(acc, ah[kb], al[kb]);
            }
        }
    };

    zero();                                                   // layer 0: W0 . x
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
    mark(2);
    next(0, 0.0f);
    mark(3);
    zero();                                                   // layer 1
    h_segment();
    mark(4);
    next(1, xmax);                                            // layer 2 reads cat(h, x): one scale
    zero();                                                   // layer 2: W2 . cat(h, x)
    load_x(sc.s, xh, xl);
    mark(5);
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
    h_segment();
    mark(6);
    next(2, 0.0f);
    mark(7);
    zero();                                                   // layer 3
    h_segment();
    mark(8);
    next(3, 0.0f);
    mark(9);
    zero();                                                   // layer 4 (no activation)
    h_segment();
    mark(10);
    finish_layer(acc, Bs + 4 * 256, sc.inv * Wi[4], h, false);
    mark(11);

    // LayerNorm(256, eps=1e-5) per ray: this lane holds 128 of the ray's
    // units, the other half-wave (lane ^ 32) the rest; sums in double
    double s = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) s += (double)acc[t][q];
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
    mark(12);
    if constexpr (STAMP) {
        // where the wave ran: HW_ID (wave, SIMD, CU, SH, SE bits) in ts[15], XCC_ID in ts[14]
        ts[15] = (unsigned long long)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        ts[14] = (unsigned long long)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
        ts[13] = __builtin_amdgcn_s_memrealtime() - rt0;     // 100 MHz ticks over marks 0 .. 12
        if (lane == 0)
            for (int i = 0; i < 16; ++i) a.stamps[((size_t)blockIdx.x * 4 + wave) * 16 + i] = ts[i];
    }
    if (!live) return;
    float* o = a.out + (size_t)ray * a.ld;
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
            store_out4(o + u, y, a.vec_out);
        }
}

// ======================================================= f16x3, persistent
// The product head: k_sam_head_h16's arithmetic (the same MFMA products in
// the same order, the same scales, finishing and LayerNorm: bit-identical
// output) in a persistent workgroup per CU that walks its 128-ray tiles
// (tile = blockIdx.x + i * gridDim.x).  Per tile, k_sam_head_h16 spent ~20 k
// of its ~145 k cycles per wave in the prologue (the rows' HBM latency, the
// weight stream priming) and ~12 k between blocks (tools/head_stamps.py); here
//   * the weight ring runs on across tiles: the last two steps of tile i
//     stream steps 0 and 1 of tile i + 1 (the weights are the same for every
//     tile), ring buffer = global step mod 3 (`rot` = the tile's first buffer);
//   * the next tile's rows (one contiguous 82 KiB: 128 rows of 164 floats) go
//     global -> LDS by DMA during steps kXFirst .. kXFirst + 20, one 1 KiB
//     piece per wave and step after the step's weight pieces, into the x
//     region that the current tile last reads at layer 2's skip input
//     (step 11's barrier long passed); layer 0 and the skip input read x
//     from LDS (conflict-free: row stride 656 B = 41 slots);
//   * the output stores of tile i drain under tile i + 1's first step.
// LDS: 64 KiB ring (4 buffers: the DMA three steps ahead, so an x piece has
// three steps to arrive from HBM) + 84 KiB x + 7 KiB biases / LayerNorm / scales.
// Measured (profiles/r3_head_clock.txt): 9 % fewer cycles per tile (142 k vs
// 156 k per wave), but the head runs at the power limit -- its clock falls
// from 1.89 to 1.77 GHz when it runs back to back -- so alone it is no
// faster (0.687 vs 0.678 ms); inside the view (2.1 GHz) it saves 0.04 ms per
// view (2.955 vs 2.99 ms; tools/view_ab.py SAMNERF_HEAD_V=4 times the
// per-tile form against it).  Bit-identical.
constexpr int kTileBytes = kRaysV5 * kRowIn * 4;    // 83,968 B = 82 KiB
constexpr int kXPieces = 21;                        // per wave: 84 pieces per tile, 82 carry rows
constexpr int kXVec = 4 * kXPieces * 64;            // uint4 of the x region
constexpr int kXFirst = 40;                         // x pieces in steps 40 .. 60 (layer 2's h part, layer 3)
static_assert(4 * kXPieces * 1024 >= kTileBytes, "x region holds a tile");
static_assert(kXFirst > kXkb + kHkb + kXkb && kXFirst + kXPieces + 3 < kSteps, "x stream window");

template <int NBUF>
struct HeadStreamQ {
    const uint4* packed;
    uint4* Wb;                 // LDS ring [NBUF][kStepVec]
    const char* rows;          // head-input rows (global)
    const char* rows_end;      // their last 16 B
    uint32_t xs;               // LDS byte address of the x region
    uint32_t next_tile;        // whose rows the x pieces carry
    int wave, lane;
    int rot;                   // ring buffer of the tile's step 0 (uniform)
    int step;                  // in-tile step (constant per call site: every loop is unrolled)

    __device__ __forceinline__ int buf(int s) const {
        const int b = rot + s % NBUF;
        return b >= NBUF ? b - NBUF : b;
    }
    // piece c (0..3) of in-tile step s (s >= kSteps: the next tile's step s - kSteps)
    __device__ __forceinline__ void wpiece(int s, int c) {
        const uint4* base = packed + (size_t)(s % kSteps) * kStepVec + (size_t)wave * 256 + (size_t)c * 64;
        lds_dma16(base + lane, (uint32_t)reinterpret_cast<uintptr_t>(Wb + buf(s) * kStepVec + wave * 256 + c * 64));
    }
    __device__ __forceinline__ void xpiece(int q) {
        const uint32_t p = (uint32_t)(wave * kXPieces + q);
        const char* base = rows + (size_t)next_tile * kTileBytes + (size_t)p * 1024u;
        const char* src = base + (size_t)lane * 16u;
        src = src > rows_end ? rows_end : src;            // pieces past the rows reload the last 16 B
        lds_dma16(src, xs + p * 1024u);
    }
    static __device__ __forceinline__ constexpr bool xstep(int s) { return s >= kXFirst && s < kXFirst + kXPieces; }

    // one k-block of the current layer for all 8 output tiles
    __device__ __forceinline__ void run(floatx16 (&acc)[8], const uint4& bh, const uint4& bl) {
        const int s = step;
        const uint4* cur = Wb + buf(s) * kStepVec + lane;
        uint4 fh[8], fl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            fh[t] = cur[t * 64];
            fl[t] = cur[512 + t * 64];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            acc[t] = mfma_f16x3(fh[t], fl[t], bh, bl, acc[t]);
            if (t & 1) {
                __builtin_amdgcn_sched_barrier(0);
                wpiece(s + NBUF - 1, t >> 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (xstep(s)) {
            __builtin_amdgcn_sched_barrier(0);
            xpiece(s - kXFirst);
            __builtin_amdgcn_sched_barrier(0);
        }
        // step s + 1 landed: younger than its pieces (issued in step s + 2 - NBUF)
        // are that step's x piece and the pieces of the steps after it
        int n = 4 * (NBUF - 2);
#pragma unroll
        for (int k = s + 2 - NBUF; k <= s; ++k) n += xstep(k) ? 1 : 0;
        wait_vmn(n);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ++step;
    }
};

// VEC: the output rows are 16-B aligned (the [N, 256] samvit array): float4
// stores.  The gather-tile form (samnerf_render_forward_tile, rows of 261
// floats) is its own instantiation with 4-B stores: a run-time choice in the
// one kernel cost the product head 0.575 -> 0.67 ms per view (measured A/B,
// the epilogue's packed fp32 math was lost to the second store path).
template <int NBUF, bool STAMP = false, bool VEC = true>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_sam_head_h16q(HeadArgsH a, uint32_t ntiles) {
    unsigned long long t0 = 0, rt0 = 0;                   // STAMP: the wave's clock over its life
    if constexpr (STAMP) {
        t0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
    }
    __shared__ uint4 smem[NBUF * kStepVec + kXVec + (7 * 256 + 8) / 4];
    uint4* const Wb = smem;
    float* const Xs = reinterpret_cast<float*>(smem + NBUF * kStepVec);
    float* const Bs = reinterpret_cast<float*>(smem + NBUF * kStepVec + kXVec);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 31, h = lane >> 5;

    for (int i = tid; i < 5 * 256; i += 256) Bs[i] = a.b[i >> 8][i & 255];
    float* const Wi = Bs + 7 * 256;                       // 2^-kexp[l]
    if (tid < 5) Wi[tid] = exp2i(-a.kexp[tid]);
    Bs[5 * 256 + tid] = a.ln_w[tid];
    Bs[6 * 256 + tid] = a.ln_b[tid];

    HeadStreamQ<NBUF> st;
    st.packed = a.packed + (size_t)((blockIdx.x >> 3) % kHeadCopies) * kPackedVec;
    st.Wb = Wb;
    st.rows = reinterpret_cast<const char*>(a.rows);
    st.rows_end = st.rows + (size_t)a.N * kRowIn * 4 - 16;
    st.xs = (uint32_t)reinterpret_cast<uintptr_t>(Xs);
    st.next_tile = blockIdx.x;
    st.wave = __builtin_amdgcn_readfirstlane(wave);
    st.lane = lane;
    st.rot = 0;
    st.step = 0;
    // the first tile's rows, then weight steps 0 and 1; rows and step 0 landed
#pragma unroll
    for (int q = 0; q < kXPieces; ++q) st.xpiece(q);
#pragma unroll
    for (int q = 0; q + 1 < NBUF; ++q)
#pragma unroll
        for (int c = 0; c < 4; ++c) st.wpiece(q, c);
    wait_vmn(4 * (NBUF - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();

    const float* xr = Xs + (wave * 32 + j) * kRowIn;      // this lane's row of the tile
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        st.next_tile = tile + gridDim.x;
        st.step = 0;
        // the stream's bases made opaque per tile: otherwise the compiler hoists
        // the 344 piece addresses of a tile out of the tile loop (spilled)
        asm volatile("" : "+s"(st.packed), "+s"(st.rows));
        const uint32_t ray = tile * kRaysV5 + wave * 32u + j;
        const bool live = ray < a.N;
        auto x8 = [&](int kb, float (&v)[8]) {
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
                if (!live || c0 + m >= kIn) v[m] = 0.0f;  // column 163 of a row is padding
        };
        float xmax = 0.0f;
#pragma unroll
        for (int kb = 0; kb < kXkb; ++kb) {
            float v[8];
            x8(kb, v);
#pragma unroll
            for (int m = 0; m < 8; ++m) xmax = fmaxf(xmax, fabsf(v[m]));
        }
        xmax = fmaxf(xmax, __shfl_xor(xmax, 32));
        auto load_x = [&](float sc_s, uint4 (&xh)[kXkb], uint4 (&xl)[kXkb]) {
#pragma unroll
            for (int kb = 0; kb < kXkb; ++kb) {
                float v[8];
                x8(kb, v);
                split8_f16(v, sc_s, xh[kb], xl[kb]);
            }
        };
        uint4 xh[kXkb], xl[kXkb];
        Scale2 sc = scale_of_max(xmax);
        load_x(sc.s, xh, xl);

        floatx16 acc[8];
        uint4 ah[kHkb], al[kHkb];
        auto zero = [&]() {
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] = floatx16{};
        };
        auto next = [&](int layer, float extra) {
            float m = finish_layer(acc, Bs + layer * 256, sc.inv * Wi[layer], h, true);
            m = fmaxf(fmaxf(m, __shfl_xor(m, 32)), extra);
            sc = scale_of_max(m);
            split_layer(acc, sc.s, ah, al);
        };
        auto h_segment = [&]() {
#pragma unroll
            for (int kb = 0; kb < kHkb; ++kb) st.run(acc, ah[kb], al[kb]);
        };

        zero();                                               // layer 0: W0 . x
#pragma unroll
        for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
        next(0, 0.0f);
        zero();                                               // layer 1
        h_segment();
        next(1, xmax);                                        // layer 2 reads cat(h, x): one scale
        zero();                                               // layer 2: W2 . cat(h, x)
        load_x(sc.s, xh, xl);
#pragma unroll
        for (int kb = 0; kb < kXkb; ++kb) st.run(acc, xh[kb], xl[kb]);
        h_segment();
        next(2, 0.0f);
        zero();                                               // layer 3
        h_segment();
        next(3, 0.0f);
        zero();                                               // layer 4 (no activation)
        h_segment();
        finish_layer(acc, Bs + 4 * 256, sc.inv * Wi[4], h, false);

        // LayerNorm(256, eps=1e-5), as k_sam_head_h16
        double s = 0.0;
#pragma unroll
        for (int t = 0; t < 8; ++t)
#pragma unroll
            for (int q = 0; q < 16; ++q) s += (double)acc[t][q];
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
        if (live) {
            float* o = a.out + (size_t)ray * a.ld;
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
                    store_out4(o + u, y, VEC);
                }
        }
        st.rot = (st.rot + kSteps) % NBUF;
    }
    wait_vmn(0);
    if constexpr (STAMP) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), rt1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            unsigned long long* o = a.stamps + ((size_t)blockIdx.x * 4 + wave) * 16;
            for (int i = 0; i < 16; ++i) o[i] = 0;
            o[12] = t1 - t0;
            o[13] = rt1 - rt0;
        }
    }                                             // the DMA past the last tile drained
}

#ifndef SAMNERF_HEAD_W8
#define SAMNERF_HEAD_W8 1                     // 0: k_sam_head_h16q, 2: two 4-wave workgroups per CU
#endif
#if defined(SAMNERF_DIAG_VARIANTS) || SAMNERF_HEAD_W8
// ============================================ f16x3, 16-ray waves, 2 per SIMD
// The head at two waves per SIMD: one wave per SIMD
// (k_sam_head_h16q) leaves the matrix pipe idle while the wave does its
// layer-boundary VALU (bias, leaky_relu, column max, hi / lo split of 128
// values per lane), its LDS reads and its step barrier, so the head sat at
// ~0.4 of its MFMA issue rate.  Here a 128-ray tile is 8 waves of 16 rays on
// v_mfma_f32_16x16x32_f16 (4 accumulator registers per 16 x 16 tile, 16 tiles
// = the 256 units: 64 registers where the 32-ray form holds 128), so two
// waves fit a SIMD's 512 registers and one wave's boundary work runs beside
// the other wave's MFMAs.  The waves are independent (own rays, all 256
// units): no exchange between them, only the shared weight stream.
//
// Orientation: out^T[16 units x 16 rays] per tile; A = weights (lane (i, g)
// = unit 16 t + i, inputs 8 g .. 8 g + 7 of the 32-deep k-block), B =
// activations (lane (j, g) = ray j, the same 8 inputs), D lane (j, g) =
// units 16 t + 4 g + r (r = 0..3) of ray j.  A hidden layer's k-block b takes
// D registers of tiles 2 b and 2 b + 1 -- input position 8 g + m of k-block b
// is unit 32 b + 4 g + m (m < 4) or 32 b + 16 + 4 g + m - 4 -- so the weights
// are packed permuted to match (w8_unit) and a layer's accumulators ARE the
// next layer's B operands, as in the 32-ray form.
//
// Weight stream: a step = one 32-deep k-block x 8 of the 16 output tiles
// (16 KiB of hi / lo fragments, [hi/lo][tile][lane]); 88 steps per tile (x
// layers 6 k-blocks: 163 inputs padded to 192).  4-buffer ring by LDS DMA, two
// 1-KiB pieces per wave and step, issued between the step's MFMAs; the tile's
// rows come into LDS by DMA during steps 30 .. 40 of the previous tile (11
// pieces per wave; the pieces past the 84-KiB x region go to a 1-KiB sink so
// that every wave issues the same count -- the hand-counted vmcnt waits rely on
// it).  The waves dispatched second take s_setprio 1 for the whole kernel
// (MI355X_MICROARCH.md "Two waves per SIMD", item 4).
//
// Arithmetic: the same f16x3 products (power-of-two scaled operands, per-ray
// column scales, per-tensor weight scales) over 32-deep instead of 16-deep
// k-blocks: fp32-equivalent like the 32-ray form, not bit-identical to it (the
// accumulation order differs; tests/test_gpu_render.py::
// test_sam_head_w8_form_is_fp32_equivalent).
//
// Measured (round 5, profiles/r5l_head_forms.txt): the head alone, back to
// back, 0.608 ms against 0.697 for k_sam_head_h16q (-13 %; the two
// 4-wave-workgroups form 0.676); inside the view 0.54 against 0.565 ms, but
// the view was not faster then (2.856-2.890 against 2.851-2.866 ms): the
// chip is at its power limit through the view (2.1-2.2 GHz).  Round 6, after
// the proposal / k_final VALU cuts, three interleaved rounds of the view with
// the live shader clock (profiles/r6d_head_w8_ab.txt): 8-wave workgroups
// 2.773-2.836 ms (head 0.504-0.509) against 2.800-2.894 (0.551-0.569) for
// k_sam_head_h16q at the same clocks, every round; the two 4-wave-workgroups
// form loses (2.878-2.899).  So the 8-wave form is the product
// (SAMNERF_HEAD_W8 = 1); h16q stays the default of SAMNERF_HEAD_W8 = 0 builds
// and the diagnostic forms (SAMNERF_HEAD_V other than 30 / 31).
namespace w8 {
constexpr int kXkb = 6;                               // 163 inputs -> 6 k-blocks of 32
constexpr int kHkb = 8;                               // 256 -> 8
constexpr int kSegKb[6] = {kXkb, kHkb, kXkb, kHkb, kHkb, kHkb};
constexpr int kSegLayer[6] = {0, 1, 2, 2, 3, 4};
constexpr int segBase(int seg) {
    int b = 0;
    for (int i = 0; i < seg; ++i) b += kSegKb[i];
    return b;
}
constexpr int kKb = segBase(6);                       // 44 k-blocks
constexpr int kSteps = 2 * kKb;                       // 88: (k-block, half of the tiles)
constexpr int kStepVec = 2 * 8 * 64;                  // uint4 per step
constexpr int kPackedVec = kSteps * kStepVec;
constexpr int kRays = 16;                             // per wave
constexpr int kWaves = 8;
constexpr int kXPieces = 11;                          // per wave and tile: 88 >= 82 KiB of rows
constexpr int kXRegion = 84;                          // KiB of the x region
constexpr int kXFirst = 30;                           // x pieces in steps 30 .. 40 (x last read before step 28)
static_assert(kXPieces * kWaves * 1024 >= kTileBytes, "x pieces cover a tile");
static_assert(kXRegion * 1024 >= kTileBytes && kXRegion * 1024 <= kXVec * 16, "x region");
static_assert(kXFirst > 2 * (kXkb + kHkb) + 1 && kXFirst + kXPieces + 3 < kSteps, "x stream window");

// the input of a hidden layer's k-block b at position 8 g + m (accumulator order)
__host__ __device__ constexpr int hunit(int b, int g, int m) { return 32 * b + (m < 4 ? 4 * g + m : 16 + 4 * g + m - 4); }

__device__ __forceinline__ float weight(const float* const* W, int kb, int unit, int g, int m) {
    int seg = 0;
    while (seg < 5 && kb >= segBase(seg + 1)) ++seg;
    const int b = kb - segBase(seg);
    const int kx = 32 * b + 8 * g + m;
    switch (seg) {
        case 0: return kx < kIn ? W[0][unit * kIn + kx] : 0.0f;
        case 1: return W[1][unit * 256 + hunit(b, g, m)];
        case 2: return kx < kIn ? W[2][unit * (256 + kIn) + 256 + kx] : 0.0f;
        case 3: return W[2][unit * (256 + kIn) + hunit(b, g, m)];
        case 4: return W[3][unit * 256 + hunit(b, g, m)];
        default: return W[4][unit * 256 + hunit(b, g, m)];
    }
}
}  // namespace w8

// packed[step 88][hi/lo][tile 8][lane 64], then kexp[5]; a workgroup's 256
// fragments are half a step (one layer), as k_pack_h16
__global__ void __launch_bounds__(256) k_pack_w8(PackArgs a) {
    __shared__ int kx;
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const int bstep = (int)((blockIdx.x * blockDim.x) >> 9);
    int bseg = 0;
    while (bseg < 5 && (bstep >> 1) >= w8::segBase(bseg + 1)) ++bseg;
    const int layer = w8::kSegLayer[bseg];
    if (threadIdx.x < 64) {
        float m = threadIdx.x < kWmaxParts ? a.part[layer * kWmaxParts + threadIdx.x] : 0.0f;
        m = wave_max64(m);
        if (threadIdx.x == 0) {
            kx = scale_exp_of_max(m);
            a.kexp[layer] = kx;
        }
    }
    __syncthreads();
    if (t >= (uint32_t)w8::kSteps * 8u * 64u) return;
    const int lane = (int)(t & 63u), tile = (int)((t >> 6) & 7u), step = (int)(t >> 9);
    const int kb = step >> 1, unit = 16 * (8 * (step & 1) + tile) + (lane & 15), g = lane >> 4;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = w8::weight(a.W, kb, unit, g, e);
    uint4 hi, lo;
    split8_f16(v, exp2i(kx), hi, lo);
    a.packed[(size_t)step * w8::kStepVec + tile * 64 + lane] = hi;
    a.packed[(size_t)step * w8::kStepVec + 512 + tile * 64 + lane] = lo;
}


template <int NBUF, int WAVES>
struct HeadStreamW8 {
    static constexpr int kPieces = 16 / WAVES;          // 1-KiB weight pieces per wave and step
    const uint4* packed;
    uint4* Wb;                 // LDS ring [NBUF][kStepVec]
    const char* rows;
    const char* rows_end;      // their last 16 B
    uint32_t xs;               // LDS byte address of the x region
    uint32_t sink;             // LDS byte address of the 1-KiB sink
    uint32_t next_tile;
    int wave, lane;
    int rot;
    int step;

    __device__ __forceinline__ int buf(int s) const {
        const int b = rot + s % NBUF;
        return b >= NBUF ? b - NBUF : b;
    }
    // piece c (0..1) of in-tile step s (s >= kSteps: the next tile's)
    __device__ __forceinline__ void wpiece(int s, int c) {
        const int o = wave * 64 * kPieces + c * 64;
        const uint4* base = packed + (size_t)(s % w8::kSteps) * w8::kStepVec + (size_t)o;
        lds_dma16(base + lane, (uint32_t)reinterpret_cast<uintptr_t>(Wb + buf(s) * w8::kStepVec + o));
    }
    __device__ __forceinline__ void xpiece(int q) {
        const uint32_t p = (uint32_t)(wave * w8::kXPieces + q);
        const char* src = rows + (size_t)next_tile * kTileBytes + (size_t)p * 1024u + (size_t)lane * 16u;
        src = src > rows_end ? rows_end : src;
        lds_dma16(src, p < (uint32_t)w8::kXRegion ? xs + p * 1024u : sink);
    }
    // the rows stream into LDS only in the 8-wave form (WAVES 4: read from global)
    static __device__ __forceinline__ constexpr bool xstep(int s) {
        return WAVES == 8 && s >= w8::kXFirst && s < w8::kXFirst + w8::kXPieces;
    }

    // k-block step s: tiles 8 HALF .. 8 HALF + 7 of the current layer
    template <int HALF>
    __device__ __forceinline__ void run(floatx4 (&acc)[16], const uint4& bh, const uint4& bl) {
        const int s = step;
        const uint4* cur = Wb + buf(s) * w8::kStepVec + lane;
        uint4 fh[8], fl[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            fh[t] = cur[t * 64];
            fl[t] = cur[512 + t * 64];
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            acc[8 * HALF + t] = mfma16_f16x3(fh[t], fl[t], bh, bl, acc[8 * HALF + t]);
            if (t % (8 / kPieces) == 8 / kPieces - 1) {
                __builtin_amdgcn_sched_barrier(0);
                wpiece(s + NBUF - 1, t / (8 / kPieces));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (xstep(s)) {
            __builtin_amdgcn_sched_barrier(0);
            xpiece(s - w8::kXFirst);
            __builtin_amdgcn_sched_barrier(0);
        }
        // step s + 1 landed: younger than its pieces (issued in step s + 2 -
        // NBUF) are the x pieces of steps s + 2 - NBUF .. s and the weight
        // pieces of the steps after it
        int n = kPieces * (NBUF - 2);
#pragma unroll
        for (int k = s + 2 - NBUF; k <= s; ++k) n += xstep(k) ? 1 : 0;
        wait_vmn(n);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ++step;
    }
};

// a layer's accumulators back to fp32 values in place (times `inv`, + bias,
// leaky_relu when `act`); returns the lane's max |value|
__device__ __forceinline__ float finish_w8(floatx4 (&acc)[16], const float* Bs, float inv, int g, bool act) {
    float m = 0.0f;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const float4 bb = *reinterpret_cast<const float4*>(Bs + 16 * t + 4 * g);
        const float b4[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[t][r] = leaky(__builtin_fmaf(acc[t][r], inv, b4[r]), act);
        m = max_abs3(m, acc[t][0], acc[t][1]);
        m = max_abs3(m, acc[t][2], acc[t][3]);
    }
    return m;
}

// the values (times s) as the next layer's B operands: k-block b <- tiles 2 b, 2 b + 1
__device__ __forceinline__ void split_w8(const floatx4 (&acc)[16], float s, uint4 (&ah)[w8::kHkb],
                                         uint4 (&al)[w8::kHkb]) {
#pragma unroll
    for (int b = 0; b < w8::kHkb; ++b) {
        const float v[8] = {acc[2 * b][0], acc[2 * b][1], acc[2 * b][2], acc[2 * b][3],
                            acc[2 * b + 1][0], acc[2 * b + 1][1], acc[2 * b + 1][2], acc[2 * b + 1][3]};
        split8_f16<true>(v, s, ah[b], al[b]);
    }
}

// max over the 4 lanes of a ray (j, j + 16, j + 32, j + 48)
__device__ __forceinline__ float ray_max4(float m) {
    m = fmaxf(m, __shfl_xor(m, 16));
    return fmaxf(m, __shfl_xor(m, 32));
}
__device__ __forceinline__ double ray_sum4(double v) {
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}

constexpr int kW8SinkVec = 64;                        // uint4 of the 1-KiB sink

// WAVES 8: one 512-thread workgroup per CU, 128-ray tiles, the rows by LDS
// DMA.  WAVES 4: two independent 256-thread workgroups per CU (64-ray tiles,
// LDS 71 KiB each, the rows read from global at the tile's start and at layer
// 2): the two waves of a SIMD belong to different workgroups and drift out of
// phase, so one's layer boundary can run under the other's MFMAs; the
// weight stream is read twice per CU.
template <int NBUF, int WAVES, bool VEC = true>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_sam_head_w8(HeadArgsH a, uint32_t ntiles) {
    constexpr bool XLDS = WAVES == 8;
    constexpr int kTileRays = WAVES * w8::kRays;
    constexpr int kX = XLDS ? kXVec + kW8SinkVec : 0;
    __shared__ uint4 smem[NBUF * w8::kStepVec + kX + (7 * 256 + 8) / 4];
    uint4* const Wb = smem;
    float* const Xs = reinterpret_cast<float*>(smem + NBUF * w8::kStepVec);
    float* const Bs = reinterpret_cast<float*>(smem + NBUF * w8::kStepVec + kX);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 15, g = lane >> 4;
    if (XLDS && wave >= 4) __builtin_amdgcn_s_setprio(1);   // the second-dispatched half, static

    for (int i = tid; i < 5 * 256; i += 64 * WAVES) Bs[i] = a.b[i >> 8][i & 255];
    float* const Wi = Bs + 7 * 256;                       // 2^-kexp[l]
    if (tid < 5) Wi[tid] = exp2i(-a.kexp[tid]);
    if (tid < 256) {
        Bs[5 * 256 + tid] = a.ln_w[tid];
        Bs[6 * 256 + tid] = a.ln_b[tid];
    }

    HeadStreamW8<NBUF, WAVES> st;
    st.packed = a.packed;
    st.Wb = Wb;
    st.rows = reinterpret_cast<const char*>(a.rows);
    st.rows_end = st.rows + (size_t)a.N * kRowIn * 4 - 16;
    st.xs = (uint32_t)reinterpret_cast<uintptr_t>(Xs);
    st.sink = (uint32_t)reinterpret_cast<uintptr_t>(smem + NBUF * w8::kStepVec + kXVec);
    st.next_tile = blockIdx.x;
    st.wave = __builtin_amdgcn_readfirstlane(wave);
    st.lane = lane;
    st.rot = 0;
    st.step = 0;
    if constexpr (XLDS) {
#pragma unroll
        for (int q = 0; q < w8::kXPieces; ++q) st.xpiece(q);
    }
#pragma unroll
    for (int q = 0; q + 1 < NBUF; ++q)
#pragma unroll
        for (int c = 0; c < st.kPieces; ++c) st.wpiece(q, c);
    wait_vmn(st.kPieces * (NBUF - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();

    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        st.next_tile = tile + gridDim.x;
        st.step = 0;
        asm volatile("" : "+s"(st.packed), "+s"(st.rows));
        const uint32_t ray = tile * kTileRays + wave * w8::kRays + j;
        const bool live = ray < a.N;
        // this lane's row: in LDS (WAVES 8) or global (a dead lane reads row 0)
        const float* xr = XLDS ? Xs + (wave * w8::kRays + j) * kRowIn : a.rows + (size_t)(live ? ray : 0u) * kRowIn;
        auto x8 = [&](int kb, float (&v)[8]) {
            const int c0 = 32 * kb + 8 * g;
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
        };
        float xmax = 0.0f;
#pragma unroll
        for (int kb = 0; kb < w8::kXkb; ++kb) {
            float v[8];
            x8(kb, v);
#pragma unroll
            for (int m = 0; m < 8; ++m) xmax = fmaxf(xmax, fabsf(v[m]));
        }
        xmax = ray_max4(xmax);
        uint4 xh[w8::kXkb], xl[w8::kXkb];
        auto load_x = [&](float sc_s) {
#pragma unroll
            for (int kb = 0; kb < w8::kXkb; ++kb) {
                float v[8];
                x8(kb, v);
                split8_f16<true>(v, sc_s, xh[kb], xl[kb]);
            }
        };
        Scale2 sc = scale_of_max(xmax);
        load_x(sc.s);

        floatx4 acc[16];
        uint4 ah[w8::kHkb], al[w8::kHkb];
        auto zero = [&]() {
#pragma unroll
            for (int t = 0; t < 16; ++t) acc[t] = floatx4{};
        };
        auto next = [&](int layer, float extra) {
            float m = finish_w8(acc, Bs + layer * 256, sc.inv * Wi[layer], g, true);
            m = fmaxf(ray_max4(m), extra);
            sc = scale_of_max(m);
            split_w8(acc, sc.s, ah, al);
        };
        auto x_segment = [&]() {
#pragma unroll
            for (int kb = 0; kb < w8::kXkb; ++kb) {
                st.template run<0>(acc, xh[kb], xl[kb]);
                st.template run<1>(acc, xh[kb], xl[kb]);
            }
        };
        auto h_segment = [&]() {
#pragma unroll
            for (int kb = 0; kb < w8::kHkb; ++kb) {
                st.template run<0>(acc, ah[kb], al[kb]);
                st.template run<1>(acc, ah[kb], al[kb]);
            }
        };

        zero();                                               // layer 0: W0 . x
        x_segment();
        next(0, 0.0f);
        zero();                                               // layer 1
        h_segment();
        next(1, xmax);                                        // layer 2 reads cat(h, x): one scale
        zero();                                               // layer 2: W2 . cat(h, x)
        load_x(sc.s);
        x_segment();
        h_segment();
        next(2, 0.0f);
        zero();                                               // layer 3
        h_segment();
        next(3, 0.0f);
        zero();                                               // layer 4 (no activation)
        h_segment();
        finish_w8(acc, Bs + 4 * 256, sc.inv * Wi[4], g, false);

        // LayerNorm(256, eps=1e-5)
        double s = 0.0;
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) s += (double)acc[t][r];
        s = ray_sum4(s);
        const double mean = s / 256.0;
        double var = 0.0;
#pragma unroll
        for (int t = 0; t < 16; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double dlt = (double)acc[t][r] - mean;
                var += dlt * dlt;
            }
        var = ray_sum4(var);
        const float rstd = (float)(1.0 / sqrt(var / 256.0 + 1e-5));
        const float mf = (float)mean;
        if (live) {
            float* o = a.out + (size_t)ray * a.ld;
            const float* lw = Bs + 5 * 256;
            const float* lb = Bs + 6 * 256;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int u = 16 * t + 4 * g;
                float4 y;
                y.x = ((acc[t][0] - mf) * rstd) * lw[u + 0] + lb[u + 0];
                y.y = ((acc[t][1] - mf) * rstd) * lw[u + 1] + lb[u + 1];
                y.z = ((acc[t][2] - mf) * rstd) * lw[u + 2] + lb[u + 2];
                y.w = ((acc[t][3] - mf) * rstd) * lw[u + 3] + lb[u + 3];
                store_out4(o + u, y, VEC);
            }
        }
        st.rot = (st.rot + w8::kSteps) % NBUF;
    }
    wait_vmn(0);                                          // the DMA past the last tile drained
}
#endif  // SAMNERF_DIAG_VARIANTS || SAMNERF_HEAD_W8

#ifdef SAMNERF_DIAG_VARIANTS
// ============================================================ f16x3, paired
// The same arithmetic as k_sam_head_h16 (every accumulator tile sees the same
// f16x3 MFMA products in the same order, the same scales, the same finishing
// and LayerNorm sums: bit-identical output) at 2 or 4 waves per SIMD instead
// of 1: a 32-ray group's 8 output tiles are shared by WPG = 8 / TPW waves,
// each holding TPW accumulator tiles, and the group's B operands (the layer
// input, hi / lo fp16 fragments) live in LDS, written once per layer by the
// waves that produced them and read by all of the group's waves each step.
// The x rows (layer 0 and the skip input of layer 2) are read and split per
// k-block, one k-block ahead.  While one wave waits on LDS, the barrier or
// its DMA issue, the other waves of its SIMD issue MFMAs.
//   LDS (one object, 160 KiB): 2 weight steps of 16 KiB (the step being read
//   and the one in flight) + 4 groups x 32 KiB of B fragments; biases and
//   LayerNorm parameters are read from global memory (L2) at layer ends.
//   Layer boundary: finish the own tiles (bias, leaky_relu), exchange the
//   per-ray max through the weight buffer that is idle between the layer's
//   last step and the next step's DMA, split at the common scale, write the
//   B fragments; two barriers.
template <int TPW>
struct PairCfg {
    static constexpr int WPG = 8 / TPW;                  // waves per 32-ray group
    static constexpr int NW = 4 * WPG;                   // waves per block (4 groups)
    static constexpr int NT = 64 * NW;
    static constexpr int PIECES = 16 / NW;               // 1-KiB DMA pieces per wave and step
};
constexpr int kBVec = kHkb * 2 * 64;                     // uint4 of one group's B fragments (32 KiB)
constexpr int kPairSmemVec = 2 * kStepVec + 4 * kBVec;   // 10,240 uint4 = 160 KiB

// every LDS access of this wave done, then the workgroup barrier
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

template <int TPW>
__global__ void __launch_bounds__(PairCfg<TPW>::NT)
__attribute__((amdgpu_waves_per_eu(PairCfg<TPW>::WPG, PairCfg<TPW>::WPG)))
k_sam_head_h16p(HeadArgsH a) {
    using C = PairCfg<TPW>;
    __shared__ uint4 smem[kPairSmemVec];
    uint4* const Wb = smem;                                   // [2][kStepVec] weight steps
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int grp = wave / C::WPG, part = wave % C::WPG;
    const int t0 = part * TPW;                                // first own output tile
    uint4* const Bg = smem + 2 * kStepVec + grp * kBVec;      // [kb][hi/lo][lane]
    const int j = lane & 31, h = lane >> 5;
    const uint32_t ray = blockIdx.x * kRaysV5 + grp * 32u + j;
    const bool live = ray < a.N;
    const float* xr = a.rows + (size_t)(live ? ray : 0u) * kRowIn;

    // weight step s -> buffer s & 1; this wave moves PIECES KiB of it
    auto issue = [&](int s) {
        const uint4* src = a.packed + (size_t)s * kStepVec + wave * (64 * C::PIECES) + lane;
        const uint32_t dst = (uint32_t)reinterpret_cast<uintptr_t>(Wb + (s & 1) * kStepVec + wave * (64 * C::PIECES));
#pragma unroll
        for (int c = 0; c < C::PIECES; ++c) lds_dma16(src + c * 64, dst + c * 1024u);
    };
    // raw x columns 16kb + 8h .. +7 of the row (masked where consumed, so the
    // loads stay in flight across a step)
    auto xload = [&](int kb, float4& p, float4& q) {
        if (kb < kXkb - 1) {
            p = *reinterpret_cast<const float4*>(xr + 16 * kb + 8 * h);
            q = *reinterpret_cast<const float4*>(xr + 16 * kb + 8 * h + 4);
        } else {                                              // columns 160..163 (h = 0) only
            p = *reinterpret_cast<const float4*>(xr + 160);
            q = p;
        }
    };
    auto xvals = [&](int kb, const float4& p, const float4& q, float (&v)[8]) {
        v[0] = p.x; v[1] = p.y; v[2] = p.z; v[3] = p.w;
        v[4] = q.x; v[5] = q.y; v[6] = q.z; v[7] = q.w;
        const int c0 = 16 * kb + 8 * h;
#pragma unroll
        for (int m = 0; m < 8; ++m)
            if (!live || c0 + m >= kIn) v[m] = 0.0f;          // column 163 of a row is padding
    };

    int s = 0;                                                // next weight step
    issue(0);
    float xmax = 0.0f;
#pragma unroll
    for (int kb = 0; kb < kXkb; ++kb) {
        float4 p, q;
        float v[8];
        xload(kb, p, q);
        xvals(kb, p, q, v);
#pragma unroll
        for (int m = 0; m < 8; ++m) xmax = fmaxf(xmax, fabsf(v[m]));
    }
    xmax = fmaxf(xmax, __shfl_xor(xmax, 32));
    float Wi[5];
#pragma unroll
    for (int l = 0; l < 5; ++l) Wi[l] = exp2i(-a.kexp[l]);
    Scale2 sc = scale_of_max(xmax);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");         // step 0 landed
    lds_barrier();

    floatx16 acc[TPW];
    auto zero = [&]() {
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = floatx16{};
    };
    // one k-block of the current layer for the own tiles; ends with step s + 1
    // landed and visible, buffer s & 1 free
    auto mma = [&](const uint4& bh, const uint4& bl) {
        const uint4* cur = Wb + (s & 1) * kStepVec + lane;
        uint4 fh[TPW], fl[TPW];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            fh[t] = cur[(t0 + t) * 64];
            fl[t] = cur[512 + (t0 + t) * 64];
        }
#pragma unroll
        for (int t = 0; t < TPW; ++t) acc[t] = mfma_f16x3(fh[t], fl[t], bh, bl, acc[t]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        lds_barrier();
        ++s;
    };
    // layer input x (layer 0, or the skip part of layer 2) at scale sc.s
    auto x_segment = [&]() {
        float4 p, q;
        xload(0, p, q);
#pragma unroll
        for (int kb = 0; kb < kXkb; ++kb) {
            float v[8];
            xvals(kb, p, q, v);                               // waits for this k-block's loads only
            uint4 bh, bl;
            split8_f16(v, sc.s, bh, bl);
            if (s + 1 < kSteps) issue(s + 1);
            if (kb + 1 < kXkb) xload(kb + 1, p, q);
            mma(bh, bl);
        }
    };
    auto h_segment = [&]() {
#pragma unroll
        for (int kb = 0; kb < kHkb; ++kb) {
            const uint4 bh = Bg[(2 * kb) * 64 + lane], bl = Bg[(2 * kb + 1) * 64 + lane];
            if (s + 1 < kSteps) issue(s + 1);
            mma(bh, bl);
        }
    };
    // bias (+ leaky_relu) of the own tiles, the ray's max |value| over all 8
    // tiles (with `extra`), the common scale, and the next layer's B fragments
    auto next = [&](int layer, float extra) {
        const float inv = sc.inv * Wi[layer];
        const float* bias = a.b[layer];
        float m = 0.0f;
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int mm = 0; mm < 4; ++mm) {
                const float4 bb = *reinterpret_cast<const float4*>(bias + 32 * (t0 + t) + 8 * mm + 4 * h);
                const float b4[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    acc[t][4 * mm + e] = leaky(__builtin_fmaf(acc[t][4 * mm + e], inv, b4[e]), true);
#pragma unroll
                for (int e = 0; e < 4; e += 2) m = max_abs3(m, acc[t][4 * mm + e], acc[t][4 * mm + e + 1]);
            }
        m = fmaxf(m, __shfl_xor(m, 32));
        float* X = reinterpret_cast<float*>(Wb + ((s + 1) & 1) * kStepVec);   // idle until step s + 1's DMA
        if (h == 0) X[(grp * C::WPG + part) * 32 + j] = m;
        lds_barrier();
        float mm2 = 0.0f;
#pragma unroll
        for (int p = 0; p < C::WPG; ++p) mm2 = fmaxf(mm2, X[(grp * C::WPG + p) * 32 + j]);
        sc = scale_of_max(fmaxf(mm2, extra));
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
            float v[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) v[q] = acc[t][q];
            uint4 hi, lo;
            split8_f16(v, sc.s, hi, lo);
            Bg[(2 * (2 * (t0 + t))) * 64 + lane] = hi;
            Bg[(2 * (2 * (t0 + t)) + 1) * 64 + lane] = lo;
            split8_f16(v + 8, sc.s, hi, lo);
            Bg[(2 * (2 * (t0 + t) + 1)) * 64 + lane] = hi;
            Bg[(2 * (2 * (t0 + t) + 1) + 1) * 64 + lane] = lo;
        }
        lds_barrier();
    };

    zero();                                                   // layer 0: W0 . x
    x_segment();
    next(0, 0.0f);
    zero();                                                   // layer 1
    h_segment();
    next(1, xmax);                                            // layer 2 reads cat(h, x): one scale
    zero();                                                   // layer 2: W2 . cat(h, x)
    x_segment();
    h_segment();
    next(2, 0.0f);
    zero();                                                   // layer 3
    h_segment();
    next(3, 0.0f);
    zero();                                                   // layer 4 (no activation)
    h_segment();

    // layer 4 outputs (bias, no activation) into the group's B region as
    // fp32, [tile][register quad][lane]; every wave of the group then forms
    // the LayerNorm sums over all 8 tiles in k_sam_head_h16's order
    float4* Y = reinterpret_cast<float4*>(Bg);
    {
        const float inv = sc.inv * Wi[4];
        const float* bias = a.b[4];
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
            for (int mm = 0; mm < 4; ++mm) {
                const float4 bb = *reinterpret_cast<const float4*>(bias + 32 * (t0 + t) + 8 * mm + 4 * h);
                float4 y;
                y.x = __builtin_fmaf(acc[t][4 * mm + 0], inv, bb.x);
                y.y = __builtin_fmaf(acc[t][4 * mm + 1], inv, bb.y);
                y.z = __builtin_fmaf(acc[t][4 * mm + 2], inv, bb.z);
                y.w = __builtin_fmaf(acc[t][4 * mm + 3], inv, bb.w);
                Y[((t0 + t) * 4 + mm) * 64 + lane] = y;
            }
    }
    lds_barrier();
    // (one tile's values at a time: the empty asm keeps the compiler from
    // holding all 128 of the lane's values in registers across the loops)
    double sum = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const float4 y = Y[(t * 4 + mm) * 64 + lane];
            sum += (double)y.x;
            sum += (double)y.y;
            sum += (double)y.z;
            sum += (double)y.w;
        }
        asm volatile("" ::: "memory");
    }
    sum += __shfl_xor(sum, 32);
    const double mean = sum / 256.0;
    double var = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const float4 y = Y[(t * 4 + mm) * 64 + lane];
            const float yy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const double dlt = (double)yy[e] - mean;
                var += dlt * dlt;
            }
        }
        asm volatile("" ::: "memory");
    }
    var += __shfl_xor(var, 32);
    const float rstd = (float)(1.0 / sqrt(var / 256.0 + 1e-5));
    const float mf = (float)mean;
    if (!live) return;
    float* o = a.out + (size_t)ray * a.ld;
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const int u = 32 * (t0 + t) + 8 * mm + 4 * h;
            const float4 v = Y[((t0 + t) * 4 + mm) * 64 + lane];
            const float4 lw = *reinterpret_cast<const float4*>(a.ln_w + u);
            const float4 lb = *reinterpret_cast<const float4*>(a.ln_b + u);
            float4 y;
            y.x = ((v.x - mf) * rstd) * lw.x + lb.x;
            y.y = ((v.y - mf) * rstd) * lw.y + lb.y;
            y.z = ((v.z - mf) * rstd) * lw.z + lb.z;
            y.w = ((v.w - mf) * rstd) * lw.w + lb.w;
            store_out4(o + u, y, a.vec_out);
        }
}

#endif  // SAMNERF_DIAG_VARIANTS

}  // namespace

// compute units of the current device (the persistent head's grid)
static int device_cus() {
    static int cus[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

// the 16-ray two-waves-per-SIMD head (k_sam_head_w8): SAMNERF_HEAD_W8=1 (the
// product) / 2 at build time, or diagnostic forms 30 / 31; any other
// SAMNERF_HEAD_V in the diagnostic build selects a k_sam_head_h16 form
[[maybe_unused]] static int head_w8() {      // 0: k_sam_head_h16q, 1: 8-wave workgroups, 2: two 4-wave workgroups per CU
#ifdef SAMNERF_DIAG_VARIANTS
    const char* v = diag_env("SAMNERF_HEAD_V");
    if (v) return atoi(v) == 30 ? 1 : atoi(v) == 31 ? 2 : 0;
#endif
    return SAMNERF_HEAD_W8;
}

size_t sam_head_packed_floats() {
    const size_t f32 = (size_t)8 * kTotalGroups * 64 * 4;
    const size_t h16 = (size_t)kPackedVec * 4 * kHeadCopies + 8 + 5 * kWmaxParts;   // fragment copies, log2 scales, partial maxima
    const size_t hw8 = (size_t)88 * 1024 * 4 + 8 + 5 * kWmaxParts;   // k_sam_head_w8's 88 steps (diagnostic forms)
    const size_t m = f32 > h16 ? f32 : h16;
    return m > hw8 ? m : hw8;
}

int sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                     float* packed, hipStream_t s, uint32_t ld, bool pack) {
    const bool vec = ld % 4u == 0u && reinterpret_cast<uintptr_t>(samvit) % 16u == 0u;
#if defined(SAMNERF_DIAG_VARIANTS) || SAMNERF_HEAD_W8
    if (m->head_mode == 0 && head_w8()) {                        // f16x3, 16-ray waves
        PackArgs p;
        for (int i = 0; i < 5; ++i) p.W[i] = m->sam_w[i];
        p.packed = reinterpret_cast<uint4*>(packed);
        p.kexp = reinterpret_cast<int*>(packed + (size_t)w8::kPackedVec * 4);
        p.part = packed + (size_t)w8::kPackedVec * 4 + 8;
        if (pack) {                       // (the diagnostic library always packs: pack_weights)
            k_head_wmax<<<dim3(kWmaxParts, 5), 256, 0, s>>>(p);
            k_pack_w8<<<div_up((uint32_t)w8::kSteps * 8u * 64u, 256), 256, 0, s>>>(p);
        }
        HeadArgsH a{};
        a.rows = rows;
        a.N = N;
        a.packed = p.packed;
        a.kexp = p.kexp;
        for (int i = 0; i < 5; ++i) a.b[i] = m->sam_b[i];
        a.ln_w = m->ln_w;
        a.ln_b = m->ln_b;
        a.out = samvit;
        a.ld = ld;
        a.vec_out = vec;
        if (head_w8() == 2) {                                    // two 64-ray workgroups per CU
            const uint32_t blocks = div_up(N, 64u);
            const uint32_t grid = blocks < 2u * (uint32_t)device_cus() ? blocks : 2u * (uint32_t)device_cus();
            if (vec) k_sam_head_w8<4, 4><<<grid, 256, 0, s>>>(a, blocks);
            else k_sam_head_w8<4, 4, false><<<grid, 256, 0, s>>>(a, blocks);
        } else {
            const uint32_t blocks = div_up(N, (uint32_t)kRaysV5);
            const uint32_t grid = blocks < (uint32_t)device_cus() ? blocks : (uint32_t)device_cus();
            if (vec) k_sam_head_w8<4, 8><<<grid, 512, 0, s>>>(a, blocks);
            else k_sam_head_w8<4, 8, false><<<grid, 512, 0, s>>>(a, blocks);
        }
        return check_launch("sam_head_w8");
    }
#endif
    if (m->head_mode == 0) {                                     // f16x3 (default)
        PackArgs p;
        for (int i = 0; i < 5; ++i) p.W[i] = m->sam_w[i];
        p.packed = reinterpret_cast<uint4*>(packed);
        p.kexp = reinterpret_cast<int*>(packed + (size_t)kPackedVec * 4 * kHeadCopies);
        p.part = packed + (size_t)kPackedVec * 4 * kHeadCopies + 8;
        if (pack) {                       // else the workspace holds them (samnerf_model::reuse_packed)
            k_head_wmax<<<dim3(kWmaxParts, 5), 256, 0, s>>>(p);
            k_pack_h16<<<div_up((uint32_t)kSteps * 8u * 64u, 256), 256, 0, s>>>(p);
        }
        HeadArgsH a;
        a.rows = rows;
        a.N = N;
        a.packed = p.packed;
        a.kexp = p.kexp;
        for (int i = 0; i < 5; ++i) a.b[i] = m->sam_b[i];
        a.ln_w = m->ln_w;
        a.ln_b = m->ln_b;
        a.out = samvit;
        a.ld = ld;
        a.vec_out = vec;
        a.stamps = nullptr;
        const uint32_t blocks = div_up(N, (uint32_t)kRaysV5);
#ifdef SAMNERF_DIAG_VARIANTS
        // measured forms (tools/head_bench.py, profiles/r3_head_forms.txt), all
        // bit-identical; 1 = the round-2 schedule (DMA before the MFMAs), 2 / 3
        // = the paired 2 / 4-waves-per-SIMD forms (0.78 / 0.84 vs 0.72 ms),
        // 5 / 7 / 8 = two k-blocks per barrier, 6 / 8 = four buffers, 11 = no
        // weight DMA (timing only), 12 = lazy split, 13 = phase stamps,
        // 4 = one block per tile (k_sam_head_h16, round 3), 20 = persistent
        // with 3 buffers, 21 = the product with clock stamps
        const char* v = diag_env("SAMNERF_HEAD_V");
        const int form = v ? atoi(v) : 0;
        const uint32_t grid = blocks < (uint32_t)device_cus() ? blocks : (uint32_t)device_cus();
        if (form == 20) k_sam_head_h16q<3><<<grid, 256, 0, s>>>(a, blocks);
        else if (form == 21 || form == 13) {                   // stamps (tools/head_stamps.py)
            const char* p = diag_env("SAMNERF_HEAD_STAMPS");
            a.stamps = reinterpret_cast<unsigned long long*>(p ? strtoull(p, nullptr, 16) : 0ull);
            if (!a.stamps) return fail(SAMNERF_EINVAL, "sam_head form %d needs SAMNERF_HEAD_STAMPS", form);
            if (form == 21) k_sam_head_h16q<4, true><<<grid, 256, 0, s>>>(a, blocks);
            else k_sam_head_h16<3, true, 1, false, true><<<blocks, 256, 0, s>>>(a);
        }
        else if (form == 1) k_sam_head_h16<3, false, 1><<<blocks, 256, 0, s>>>(a);
        else if (form == 2) k_sam_head_h16p<4><<<blocks, PairCfg<4>::NT, 0, s>>>(a);
        else if (form == 3) k_sam_head_h16p<2><<<blocks, PairCfg<2>::NT, 0, s>>>(a);
        else if (form == 5) k_sam_head_h16<3, false, 2><<<blocks, 256, 0, s>>>(a);
        else if (form == 6) k_sam_head_h16<4, true, 1><<<blocks, 256, 0, s>>>(a);
        else if (form == 7) k_sam_head_h16<3, true, 2><<<blocks, 256, 0, s>>>(a);
        else if (form == 8) k_sam_head_h16<4, true, 2><<<blocks, 256, 0, s>>>(a);
        else if (form == 11) k_sam_head_h16<3, true, 0><<<blocks, 256, 0, s>>>(a);
        else if (form == 12) k_sam_head_h16<3, true, 1, true><<<blocks, 256, 0, s>>>(a);
        else if (form == 4) k_sam_head_h16<3, true, 1><<<blocks, 256, 0, s>>>(a);   // one block per tile
        else
#endif
        {
            const uint32_t grid = blocks < (uint32_t)device_cus() ? blocks : (uint32_t)device_cus();
            if (vec) k_sam_head_h16q<4><<<grid, 256, 0, s>>>(a, blocks);   // persistent, one workgroup per CU
            else k_sam_head_h16q<4, false, false><<<grid, 256, 0, s>>>(a, blocks);
        }
        return check_launch("sam_head_h16");
    }
    const uint32_t nvec = 8u * kTotalGroups * 64u;
    if (pack)
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
    a.ld = ld;
    a.vec_out = vec;
    k_sam_head<<<div_up(N, kRows), 256, 0, s>>>(a);
    return check_launch("sam_head");
}

}  // namespace samnerf

extern "C" {

size_t samnerf_sam_head_workspace_size(void) { return samnerf::sam_head_packed_floats() * sizeof(float); }

int samnerf_sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                             void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    using namespace samnerf;
    if (!m) return fail(SAMNERF_EINVAL, "sam_head_forward: null model");
    if (!m->with_sam) return fail(SAMNERF_EINVAL, "sam_head_forward: model has no SAM head (with_sam = 0)");
    for (int i = 0; i < 5; ++i)
        if (!m->sam_w[i] || !m->sam_b[i]) return fail(SAMNERF_EINVAL, "sam_head_forward: null head weight");
    if (!m->ln_w || !m->ln_b) return fail(SAMNERF_EINVAL, "sam_head_forward: null LayerNorm weight");
    if (m->head_mode != 0 && m->head_mode != 1)
        return fail(SAMNERF_EINVAL, "sam_head_forward: head_mode must be 0 or 1, got %d", m->head_mode);
    if (N == 0) return SAMNERF_OK;
    if (!rows || !samvit || !workspace) return fail(SAMNERF_EINVAL, "sam_head_forward: null pointer");
    const size_t need = samnerf_sam_head_workspace_size();
    if (workspace_bytes < need)
        return fail(SAMNERF_EWORKSPACE, "sam_head_forward: workspace needs %zu bytes, got %zu", need,
                    workspace_bytes);
    return sam_head_forward(m, rows, N, samvit, static_cast<float*>(workspace),
                            reinterpret_cast<hipStream_t>(stream), 256u, true);
}

}  // extern "C"
