// mask_head.hip -- the --with_mask instance head (mask_mlp_type 'default') on
// gfx950 matrix cores, fused after the ray march.
//
// Reference (nerf/network.py:125-133, nerf/renderer.py:322-323, :392-395,
// :451-452): per final sample k of a ray
//     point_mask_k = SkipConnMLP(143 -> 256 -> 256 -> K, bias=False, leaky_relu)
//                        (cat(m_grid(x_k) [16 levels x 8 channels], geo_feat_k [15]))
//     instance_mask_logits = sum_k weights_k.detach() * point_mask_k
// The head is non-linear, so the sum cannot move in front of it: it runs on
// all 32 samples of every ray (~6.5 MFLOP per ray, 3x the SAM head's GEMM
// work per ray x 32 samples / 10).  The reference materialises [N, 32, 143]
// and [N, 32, 256] twice per 16K-ray chunk; here nothing per sample leaves
// the registers except the weight stream.
//
// One workgroup = 128 ray slots (4 waves x 32), looping over the 32 samples.
// Per sample a wave gathers its 32 rays' m_grid features straight into the
// B operands of layer 0 (lane half h of k-block kb < 8 = level 2 kb + h, its 8
// channels = one 32-B corner row per corner: lookup_level3<8>), k-block 8 =
// geo_feat (k_final stores it per sample when the model has a mask head).
// Orientation is k_sam_head_h16's (sam_head.hip): out^T[256 units x 32 rays] =
// W . act^T, 8 accumulator tiles per wave whose registers are the next layer's
// B operands, weights in 16 KiB steps through LDS shared by the 4 waves.  27
// steps per sample:
// layer 0 (9 k-blocks x 8 tiles), layer 1 (16 x 8), layer 2 (16 k-blocks x
// the one output tile, 8 per step).  The weighted sum over samples stays in
// the output tile's registers.
//
// Precision (head_mode): 0 = f16x3 (f16x3.h: 3 fp16 MFMAs per 16-deep k-block
// on power-of-two scaled operands, fp32-equivalent: per-tensor weight scales,
// per-sample-column activation scales); 1 = exact fp32 (8
// v_mfma_f32_32x32x2_f32 per k-block, the step holds the fp32 weights in the
// same 32 B per lane and tile).
#include <algorithm>

#include "f16x3.h"
#include "samnerf_common.h"

using namespace samnerf;

namespace {


constexpr int kMIn = 143;                     // 128 m_grid features + 15 geo
constexpr int kL0kb = 9;                      // 8 level pairs + geo (15 + 1 pad)
constexpr int kHkb = 16;                      // 256 -> 16 k-blocks
constexpr int kStepsPerSample = kL0kb + kHkb + 2;   // 27
constexpr int kStepVec = 2 * 8 * 64;          // uint4 per step
constexpr int kSlots = 128;                   // ray slots per workgroup
constexpr int kPackVec = kStepsPerSample * kStepVec;   // uint4 of one copy of the weight fragments
// Copies of the fragments: every workgroup streams the same steps at about
// the same time; workgroup b reads copy (b >> 3) % kMaskCopies so that each
// XCD's requests spread over that many times as many L2 channels (the
// SAM head's kHeadCopies).  The copies hold the same bits.  Measured no
// faster (9.13 vs 9.04 ms per mask view with the VGPR-staged stream), so one.
#ifndef SAMNERF_MASK_COPIES
#define SAMNERF_MASK_COPIES 1
#endif
constexpr int kMaskCopies = SAMNERF_MASK_COPIES;
constexpr int kT = 32;                        // final samples per ray
__device__ __forceinline__ int rho(int q) { return (q & 3) + 8 * (q >> 2); }
__device__ __forceinline__ int hidden_unit(int kb, int h, int m) {
    return 32 * (kb >> 1) + rho(8 * (kb & 1) + m) + 4 * h;
}

// 8 values of one lane's k-block as the B operand pair: f16x3 hi / lo of the
// values times s, or (EXACT) the fp32 values themselves, 4 in each uint4
template <bool EXACT>
__device__ __forceinline__ void to_operand(const float* v, float s, uint4& a, uint4& b) {
    if constexpr (EXACT) {
        a = make_uint4(__float_as_uint(v[0]), __float_as_uint(v[1]), __float_as_uint(v[2]), __float_as_uint(v[3]));
        b = make_uint4(__float_as_uint(v[4]), __float_as_uint(v[5]), __float_as_uint(v[6]), __float_as_uint(v[7]));
    } else {
        split8_f16(v, s, a, b);
    }
}

__device__ __forceinline__ float u4f(const uint4& u, int i) {
    return __uint_as_float(i == 0 ? u.x : i == 1 ? u.y : i == 2 ? u.z : u.w);
}

// acc += A . B over one 16-deep k-block
template <bool EXACT>
__device__ __forceinline__ floatx16 kblock(uint4 a0, uint4 a1, uint4 b0, uint4 b1, floatx16 c) {
    if constexpr (EXACT) {
        // instruction s: lane (i, h) A = W[i][input (kb, h, s)], B = x[input (kb, h, s)]
#pragma unroll
        for (int s = 0; s < 8; ++s)
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(s < 4 ? u4f(a0, s) : u4f(a1, s - 4),
                                                    s < 4 ? u4f(b0, s) : u4f(b1, s - 4), c, 0, 0, 0);
        return c;
    } else {
        return mfma_f16x3(a0, a1, b0, b1, c);
    }
}

// packed[step 27][part 2][slot 8][lane 64] uint4: steps 0-8 layer 0 (slot =
// output tile), 9-24 layer 1 (slot = tile), 25-26 layer 2 (slot = k-block
// 8 (step - 25) + slot of the single output tile).  Lane (i, h), 8 values m
// of k-block kb: W[32 t + i][input (kb, h, m)], input = 16 kb + 8 h + m for
// layer 0 (m_grid level 2 kb + h channel m; kb 8: geo 8 h + m at column 128 +
// 8 h + m, column 143 = padding), hidden_unit(kb, h, m) for layers 1-2.
__device__ __forceinline__ float mask_weight(const float* __restrict__ w0, const float* __restrict__ w1,
                                             const float* __restrict__ w2, uint32_t K, int step, int slot,
                                             int lane, int m) {
    const int i = lane & 31, h = lane >> 5;
    if (step < kL0kb) {                                   // layer 0: tile = slot
        const int col = 16 * step + 8 * h + m;
        return col < kMIn ? w0[(32 * slot + i) * kMIn + col] : 0.0f;
    }
    if (step < kL0kb + kHkb) {                            // layer 1
        const int kb = step - kL0kb;
        return w1[(32 * slot + i) * 256 + hidden_unit(kb, h, m)];
    }
    const int kb = 8 * (step - kL0kb - kHkb) + slot;      // layer 2: one tile
    return (uint32_t)i < K ? w2[i * 256 + hidden_unit(kb, h, m)] : 0.0f;
}

__device__ __forceinline__ int step_layer(int step) { return step < kL0kb ? 0 : step < kL0kb + kHkb ? 1 : 2; }

// exact fp32 weights (head_mode 1), one thread per (step, slot, lane)
__global__ void __launch_bounds__(256)
k_mask_pack_f32(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
                uint32_t K, uint4* __restrict__ packed) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (uint32_t)kStepsPerSample * 8u * 64u) return;
    const int lane = (int)(t & 63u), slot = (int)((t >> 6) & 7u), step = (int)(t >> 9);
    float v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = mask_weight(w0, w1, w2, K, step, slot, lane, m);
    uint4 a, b;
    to_operand<true>(v, 1.0f, a, b);
#pragma unroll
    for (int c = 0; c < kMaskCopies; ++c) {
        packed[(size_t)c * kPackVec + (size_t)step * kStepVec + slot * 64 + lane] = a;
        packed[(size_t)c * kPackVec + (size_t)step * kStepVec + 512 + slot * 64 + lane] = b;
    }
}

// f16x3 weights (head_mode 0): one workgroup finds each tensor's max |w|, then
// packs the fragments scaled by that tensor's power of two; kexp[3] (after
// the fragments) = the tensors' log2 scales
__global__ void __launch_bounds__(1024)
k_mask_pack_h16(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
                uint32_t K, uint4* __restrict__ packed) {
    __shared__ float wm[3][16];
    __shared__ int ke[3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float m0 = 0.0f, m1 = 0.0f, m2 = 0.0f;
    for (int i = tid; i < 256 * kMIn; i += 1024) m0 = fmaxf(m0, fabsf(w0[i]));
    for (int i = tid; i < 256 * 256; i += 1024) m1 = fmaxf(m1, fabsf(w1[i]));
    for (int i = tid; i < (int)K * 256; i += 1024) m2 = fmaxf(m2, fabsf(w2[i]));
    m0 = wave_max64(m0);
    m1 = wave_max64(m1);
    m2 = wave_max64(m2);
    if (lane == 0) {
        wm[0][wave] = m0;
        wm[1][wave] = m1;
        wm[2][wave] = m2;
    }
    __syncthreads();
    if (tid < 3) {
        float m = 0.0f;
        for (int w = 0; w < 16; ++w) m = fmaxf(m, wm[tid][w]);
        ke[tid] = scale_exp_of_max(m);
    }
    __syncthreads();
    for (int t = tid; t < kStepsPerSample * 8 * 64; t += 1024) {
        const int lane2 = t & 63, slot = (t >> 6) & 7, step = t >> 9;
        float v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = mask_weight(w0, w1, w2, K, step, slot, lane2, m);
        uint4 a, b;
        to_operand<false>(v, exp2i(ke[step_layer(step)]), a, b);
#pragma unroll
        for (int c = 0; c < kMaskCopies; ++c) {
            packed[(size_t)c * kPackVec + (size_t)step * kStepVec + slot * 64 + lane2] = a;
            packed[(size_t)c * kPackVec + (size_t)step * kStepVec + 512 + slot * 64 + lane2] = b;
        }
    }
    if (tid < 3) reinterpret_cast<int*>(packed + (size_t)kMaskCopies * kPackVec)[tid] = ke[tid];
}

struct MaskArgs {
    GridDesc<16> grid;       // m_grid
    const float* u_in;       // [32][3][N] grid-space sample positions (slot order)
    const float* w_in;       // [32][N] final weights
    const float* geo_in;     // [32][16][N] grid_mlp output rows (row 0 = sigma, unused)
    uint32_t N, K;
    RayTiles tiles;
    const uint4* packed;
    const int* kexp;         // f16x3: the three weight tensors' log2 scales
    float* out;              // [N][K] (ray order)
};

// The round-2/3 weight stream (SAMNERF_MASK_RING=0 builds only), staged
// through VGPRs: steps go in groups of kGroup; the block's 256 threads load the
// next group (kGroup x 16 KiB, four 16-B loads per thread and step) at the
// start of a group, write it to the other half of a 2-group LDS ring after the
// group's MFMAs, then one barrier per group.  (Round 2: a dword LDS-DMA ring
// measured slower than this form; two steps per group spilled 52-93 VGPRs.)
constexpr uint32_t kGroup = 1;
struct MaskStager {
    const uint4* __restrict__ packed;
    uint4* Wb;            // [2][kGroup][kStepVec]
    int tid, lane;
    uint32_t step;
    uint32_t total;
    uint4 stg[4 * kGroup];

    __device__ __forceinline__ void load(uint32_t g) {          // group g = steps g kGroup ..
#pragma unroll
        for (uint32_t i = 0; i < kGroup; ++i) {
            const uint32_t s = g * kGroup + i;
            const uint4* src = packed + (size_t)(s % kStepsPerSample) * kStepVec + tid;
#pragma unroll
            for (int c = 0; c < 4; ++c) stg[4 * i + c] = s < total ? src[c * 256] : make_uint4(0, 0, 0, 0);
        }
    }
    __device__ __forceinline__ void store(uint32_t g) {
        uint4* dst = Wb + (size_t)(g & 1u) * kGroup * kStepVec + tid;
#pragma unroll
        for (uint32_t i = 0; i < kGroup; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) dst[i * kStepVec + c * 256] = stg[4 * i + c];
    }
    __device__ __forceinline__ void begin() {
        load(0);
        store(0);
        __syncthreads();
    }
    __device__ __forceinline__ const uint4* start() {
        const uint32_t g = step / kGroup, i = step % kGroup;
        if (i == 0 && (g + 1) * kGroup < total) load(g + 1);
        return Wb + ((size_t)(g & 1u) * kGroup + i) * kStepVec + lane;
    }
    __device__ __forceinline__ void finish() {
        const uint32_t g = step / kGroup, i = step % kGroup;
        if (i == kGroup - 1 || step + 1 == total) {
            if ((g + 1) * kGroup < total) store(g + 1);
            __syncthreads();
        }
        ++step;
    }

    template <bool EXACT>
    __device__ __forceinline__ void run8(floatx16 (&acc)[8], const uint4& b0, const uint4& b1) {
        const uint4* cur = start();
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = kblock<EXACT>(cur[t * 64], cur[512 + t * 64], b0, b1, acc[t]);
        finish();
    }
    template <bool EXACT>
    __device__ __forceinline__ void run1(floatx16& acc, const uint4* b0, const uint4* b1) {
        const uint4* cur = start();
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = kblock<EXACT>(cur[k * 64], cur[512 + k * 64], b0[k], b1[k], acc);
        finish();
    }
};

// The weight stream by LDS DMA (global_load_lds_dwordx4: 16 B per lane
// straight into LDS, no staging registers): a kRing-step ring, step s + kRing
// - 1 requested at the start of step s, so a step's fragments have kRing - 1
// steps of MFMA work to arrive in.  A step is 16 KiB = 4 DMA instructions per
// wave.  At the end of step s each wave waits until step s + 1's requests are done
// (vmcnt counted by hand: the later steps' 4 (kRing - 2) requests may stay in
// flight; vector-memory completions count in order, and other loads issued
// in between only make the wait stricter), then one barrier makes every
// wave's part visible.  The slot a request overwrites was last read in step
// s - 1, which every wave finished before the previous barrier.
// Measured (round 4, 512^2 mask view, interleaved A/B of whole builds): the
// VGPR-staged stream 9.04-9.13 ms per view, this ring 3-deep 8.59, 5-deep 8.36
// (LDS: 5 x 16 KiB ring + 4 x 18 KiB layer-0 operands).  Attribution builds of
// the VGPR-staged form: without the m_grid gathers 7.92 ms, without the weight
// loads 8.77, without the step barriers 8.63 -- the gathers at each sample's
// start are the largest single stall.
#ifndef SAMNERF_MASK_RING
#define SAMNERF_MASK_RING 5
#endif
constexpr int kRing = SAMNERF_MASK_RING;
static_assert(kRing == 0 || (kRing >= 3 && kRing <= 5), "finish() counts vmcnt for 3-5 deep rings");
struct MaskStagerDma {
    const uint4* __restrict__ packed;
    uint4* Wb;            // [kRing][kStepVec]
    int tid, lane, wave;
    uint32_t step;
    uint32_t total;

    // wave w moves uint4 256 w .. 256 w + 255 of step s (4 x 1 KiB); the
    // step's offset is opaque so that the 27 steps' addresses are formed here,
    // not hoisted out of the sample loop (27 x 4 address pairs spilled)
    __device__ __forceinline__ void request(uint32_t s) {
        uint32_t so = (s % kStepsPerSample) * (uint32_t)(kStepVec * 16);
        asm volatile("" : "+s"(so));
        const char* base = reinterpret_cast<const char*>(packed) + so;
        const uint32_t vo = (uint32_t)(wave * 256 + lane) * 16u;
        const uint32_t d = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(Wb + (size_t)(s % kRing) * kStepVec + wave * 256));
        uint32_t keep, t1, t2, t3;
        // no "memory" clobber: the ring slot written here is not read before
        // finish()'s wait and barrier (volatile asm keeps its place among them)
        asm volatile(
            "v_add_u32 %1, 1024, %4\n\tv_add_u32 %2, 2048, %4\n\tv_add_u32 %3, 3072, %4\n\t"
            "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %6\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %4, %5\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, %5\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %2, %5\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %3, %5\n\ts_mov_b32 m0, %0"
            : "=&s"(keep), "=&v"(t1), "=&v"(t2), "=&v"(t3)
            : "v"(vo), "s"(base), "s"(d));
    }
    __device__ __forceinline__ void begin() {
        for (uint32_t s = 0; s + 1 < (uint32_t)kRing && s < total; ++s) request(s);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    __device__ __forceinline__ const uint4* start() {
        if (step + kRing - 1 < total) request(step + kRing - 1);
        return Wb + (size_t)(step % kRing) * kStepVec + lane;
    }
    __device__ __forceinline__ void finish() {
        if (step + kRing - 1 < total) {
            if constexpr (kRing == 3) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            else if constexpr (kRing == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        ++step;
    }

    template <bool EXACT>
    __device__ __forceinline__ void run8(floatx16 (&acc)[8], const uint4& b0, const uint4& b1) {
        const uint4* cur = start();
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = kblock<EXACT>(cur[t * 64], cur[512 + t * 64], b0, b1, acc[t]);
        finish();
    }
    template <bool EXACT>
    __device__ __forceinline__ void run1(floatx16& acc, const uint4* b0, const uint4* b1) {
        const uint4* cur = start();
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = kblock<EXACT>(cur[k * 64], cur[512 + k * 64], b0[k], b1[k], acc);
        finish();
    }
};

// leaky_relu(0.01) as max(x, 0.01 x): the same value for every x (x >= 0,
// -0.0 included, gives x; x < 0 gives 0.01 x; NaN stays NaN).  The max is a
// plain v_max_f32: fmaxf on an accumulator (not a known arithmetic result)
// would add a canonicalising v_max per value, and the compare-and-select form
// takes three VALU.  The multiply comes first and reads x, so the compiler
// has already placed x's MFMA-result wait states before the asm reads it.
// Only for outputs that reach an MFMA through further VALU (the f16x3 split):
// hipcc pads one wait state after an asm statement, an MFMA operand needs two.
__device__ __forceinline__ float leaky(float x) {
    const float t = x * 0.01f;
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(t));
    return r;
}

// leaky_relu on the accumulators, then the next layer's B operands (k-block
// kb = 2t + s <- registers 8s..8s+7 of tile t, hidden_unit order).  f16x3:
// scaled by 2^k, k from the sample column's max |value| (both half-waves);
// returns k (leaky_relu is positively homogeneous, so the raw accumulators'
// scale carries through it)
template <bool EXACT>
__device__ __forceinline__ int epilogue(floatx16 (&acc)[8], uint4 (&a0)[kHkb], uint4 (&a1)[kHkb]) {
    float m = 0.0f;
#pragma unroll
    for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            // exact fp32: the value feeds an MFMA B operand directly, and an
            // asm statement's output gets one wait state from hipcc where the
            // MFMA needs two (tools/isa_hazards.py R1) -- fmaxf, which the
            // compiler schedules and pads (and canonicalises), instead
            if constexpr (EXACT) acc[t][q] = fmaxf(acc[t][q], acc[t][q] * 0.01f);
            else acc[t][q] = leaky(acc[t][q]);
            if constexpr (!EXACT) m = fmaxf(m, fabsf(acc[t][q]));
        }
    int k = 0;
    if constexpr (!EXACT) k = scale_exp_of_max(fmaxf(m, __shfl_xor(m, 32)));
    const float s = EXACT ? 1.0f : exp2i(k);
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        float v[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) v[q] = acc[t][q];
        to_operand<EXACT>(v, s, a0[2 * t], a1[2 * t]);
        to_operand<EXACT>(v + 8, s, a0[2 * t + 1], a1[2 * t + 1]);
    }
    return k;
}

// lookup_level3<8> in two halves, so that one level's loads can run under a
// weight step's MFMAs: the 8 corner rows (2 x 16 B each) and weights, then
// the weighted sum in lookup_level3's order (the same bits)
struct Gather8 {
    float4 e[8][2];
    float w[8];
};
__device__ __forceinline__ void gather8_issue(const float* __restrict__ emb, const LevelDesc& d, float ux, float uy,
                                              float uz, Gather8& g) {
    uint32_t off[8];
    corner_rows<8>(d, ux, uy, uz, off, g.w);
    const char* base = reinterpret_cast<const char*>(emb);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        g.e[c][0] = *reinterpret_cast<const float4*>(base + off[c]);
        g.e[c][1] = *reinterpret_cast<const float4*>(base + off[c] + 16u);
    }
}
__device__ __forceinline__ void gather8_finish(const Gather8& g, float* acc) {
    f2v a[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = f2v{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const f2v wc = {g.w[c], g.w[c]};
        a[0] = __builtin_elementwise_fma(wc, f2v{g.e[c][0].x, g.e[c][0].y}, a[0]);
        a[1] = __builtin_elementwise_fma(wc, f2v{g.e[c][0].z, g.e[c][0].w}, a[1]);
        a[2] = __builtin_elementwise_fma(wc, f2v{g.e[c][1].x, g.e[c][1].y}, a[2]);
        a[3] = __builtin_elementwise_fma(wc, f2v{g.e[c][1].z, g.e[c][1].w}, a[3]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        acc[2 * i] = a[i].x;
        acc[2 * i + 1] = a[i].y;
    }
}

constexpr int kXVec = kL0kb * 2 * 64;          // uint4 per wave: layer-0 B operands [kb][part][lane]
constexpr int kDescVec = (16 * (int)sizeof(LevelDesc) + 15) / 16;

template <bool EXACT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_mask_head(MaskArgs a) {
    // one LDS object: the kRing-step weight ring | each wave's layer-0 B operands
    // of the current sample (the gathers land there, not in 72 VGPRs that
    // would live through layer 0 next to the accumulators, fragments and
    // activations: with them the kernel spilled ~350 registers) | the m_grid
    // level descriptors (read per lane: a select between two kernel-argument
    // descriptors became per-lane loads from the kernarg segment)
    constexpr uint32_t kRingUsed = kRing ? (uint32_t)kRing : 2u * kGroup;
    __shared__ uint4 smem[kRingUsed * kStepVec + 4 * kXVec + kDescVec];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 31, h = lane >> 5;
    const uint32_t slot = blockIdx.x * kSlots + wave * 32u + j;
    const bool live = slot < a.N;
    const uint32_t ss = live ? slot : a.N - 1u, N = a.N;
    uint4* const Xw = smem + kRingUsed * kStepVec + wave * kXVec;
    LevelDesc* const sLv = reinterpret_cast<LevelDesc*>(smem + kRingUsed * kStepVec + 4 * kXVec);
    if (tid < 16) sLv[tid] = a.grid.lv[tid];

    const uint4* const pk = a.packed + (size_t)((blockIdx.x >> 3) % kMaskCopies) * kPackVec;
#if SAMNERF_MASK_RING
    MaskStagerDma st{pk, smem, tid, lane, wave, 0u, (uint32_t)kT * kStepsPerSample};
#else
    MaskStager st{pk, smem, tid, lane, 0u, (uint32_t)kT * kStepsPerSample, {}};
#endif
    st.begin();

    floatx16 sum = {};                                       // sum_k w_k * logits_k
    floatx16 acc[8];
    uint4 a0[kHkb], a1[kHkb];
    // f16x3: log2 scales of the weight tensors (uniform)
    const int kw0 = EXACT ? 0 : a.kexp[0], kw1 = EXACT ? 0 : a.kexp[1], kw2 = EXACT ? 0 : a.kexp[2];
    // The inputs of a sample: lane half h of k-block kb = m_grid level 2 kb + h
    // (8 channels), k-block 8 = geo_feat; Xw holds them as fp32 (8 per lane
    // and k-block, two uint4), split into B operands as each k-block is
    // consumed (f16x3: at the scale of the column's max |input|, xm).  The 8
    // levels' loads go out in two batches of 4 (64 rows per lane in flight,
    // 256 VGPRs -- the accumulators and hidden-layer operands are dead at a
    // sample's start), two memory round trips per sample where one level at a
    // time took eight (the m_grid gathers were the largest single stall).
#pragma unroll 1
    for (int k = 0; k < kT; ++k) {
        // `ko` is opaque so that the per-sample addresses are formed here, not
        // carried through the loop as 64-bit induction pointers
        uint32_t ko = (uint32_t)k;
        asm volatile("" : "+s"(ko));
        const float* up = a.u_in + (size_t)ko * 3u * N + ss;
        const float ux = up[0], uy = up[N], uz = up[2u * N];
        const float w = live ? a.w_in[(size_t)ko * N + ss] : 0.0f;
        float xm = 0.0f;
        auto store_level = [&](int kb, const float* f) {
            uint4 xa, xb;
            to_operand<true>(f, 1.0f, xa, xb);
            Xw[(2 * kb) * 64 + lane] = xa;
            Xw[(2 * kb + 1) * 64 + lane] = xb;
#pragma unroll
            for (int m = 0; m < 8; ++m) xm = fmaxf(xm, fabsf(f[m]));
        };
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            Gather8 g[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) gather8_issue(a.grid.emb, sLv[2 * (4 * half + i) + h], ux, uy, uz, g[i]);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float f[8];
                gather8_finish(g[i], f);
                store_level(4 * half + i, f);
            }
        }
        {
            float g[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int gi = 8 * h + m;                    // geo_feat index; 15 = padding
                g[m] = gi < 15 ? a.geo_in[((size_t)ko * 16u + gi + 1) * N + ss] : 0.0f;
            }
            store_level(8, g);
        }
        const int k0 = EXACT ? 0 : scale_exp_of_max(fmaxf(xm, __shfl_xor(xm, 32)));
        const float s0 = EXACT ? 1.0f : exp2i(k0);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = floatx16{};
#pragma unroll
        for (int kb = 0; kb < kL0kb; ++kb) {
            uint4 b0 = Xw[(2 * kb) * 64 + lane], b1 = Xw[(2 * kb + 1) * 64 + lane];
            if constexpr (!EXACT) {
                const float v[8] = {__uint_as_float(b0.x), __uint_as_float(b0.y), __uint_as_float(b0.z),
                                    __uint_as_float(b0.w), __uint_as_float(b1.x), __uint_as_float(b1.y),
                                    __uint_as_float(b1.z), __uint_as_float(b1.w)};
                to_operand<false>(v, s0, b0, b1);
            }
            st.run8<EXACT>(acc, b0, b1);
        }
        const int k1 = epilogue<EXACT>(acc, a0, a1);
#pragma unroll
        for (int t = 0; t < 8; ++t) acc[t] = floatx16{};
#pragma unroll
        for (int kb = 0; kb < kHkb; ++kb) st.run8<EXACT>(acc, a0[kb], a1[kb]);
        const int k2 = epilogue<EXACT>(acc, a0, a1);
        floatx16 o = {};
        st.run1<EXACT>(o, a0, a1);
        st.run1<EXACT>(o, a0 + 8, a1 + 8);
        // f16x3: o carries 2^(k0 + kw0 + k1 + kw1 + k2 + kw2); w * 2^-e is exact
        const float wo = EXACT ? w : w * exp2i(-(k0 + kw0 + k1 + kw1 + k2 + kw2));
#pragma unroll
        for (int q = 0; q < 16; ++q) sum[q] = __builtin_fmaf(wo, o[q], sum[q]);
    }
    if (!live) return;
    float* dst = a.out + (size_t)a.tiles(slot) * a.K;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const uint32_t u = (uint32_t)(rho(q) + 4 * h);
        if (u < a.K) dst[u] = sum[q];
    }
}

// ============================================ f16x3, 16-ray waves, 2 per SIMD
// (round 6; SAMNERF_MASK_W8, the SAM head's k_sam_head_w8 structure applied
// to the mask head).  k_mask_head holds 426 registers per
// 32-ray wave, one wave per SIMD, so each sample's m_grid gathers and its
// MFMAs run one after the other on every SIMD (the gathers were the largest
// single stall, see the ring's note above).  Here a workgroup is 8 waves of
// 16 ray slots (128 slots, as before) on v_mfma_f32_16x16x32_f16: a layer's
// 256 units are 16 accumulator tiles of 4 registers (64 where the 32-ray form
// holds 128), so two waves share a SIMD and one wave's gathers, splits and
// leaky_relu run under the other's MFMAs.
//
// Lane (j, g): ray slot j of the wave, input group g (8 inputs of a 32-deep
// k-block).  Layer 0's k-block b < 4 is m_grid levels 4 b .. 4 b + 3 (lane
// group g: level 4 b + g, its 8 channels = one 32-B corner row per corner),
// k-block 4 is geo_feat (g 0: 0-7, g 1: 8-14 + pad, g 2-3: zero padding).
// A hidden layer's k-block b is the accumulator tiles 2 b, 2 b + 1 (hunit,
// the weights packed permuted to match), as in k_sam_head_w8.  Weight steps
// of 16 KiB (8 tiles x 32-deep k-block, hi / lo): layer 0 10 steps (5
// k-blocks x 2 halves of the tiles), layer 1 16, layer 2 OT (one per 16-unit
// output tile, its 8 k-blocks in the step's 8 slots): 26 + OT per sample,
// streamed through a 4-step LDS ring by LDS DMA (2 x 1 KiB per wave and step).
// Arithmetic: the f16x3 products with per-tensor weight scales and per-ray
// activation scales, as k_mask_head, over 32-deep instead of 16-deep k-blocks:
// fp32-equivalent, not bit-identical to it (tests/test_gpu_mask.py: the
// reference's goldens and the unfused op sequence within 1e-3, ragged
// launches bit-equal to the full launch).
// Measured (profiles/r6m_mask_w8_ab.txt, r6n_mask_w8_ab.txt, interleaved):
// the --with_mask 512^2 view 7.57-7.71 ms against 7.84-7.94 for k_mask_head
// (-3.5 %); 169 registers, no scratch.  Not the 2x two waves per SIMD could
// give: the per-step barrier keeps a workgroup's 8 waves in lockstep, so the
// two waves of a SIMD gather and multiply at the same time; two independent
// 4-wave workgroups per CU (SAMNERF_MASK_W8=2) drift apart but must keep the
// inputs in registers (no LDS for two rings and two input stages) and spill:
// 9.1-9.2 ms.  Two levels' corner rows in flight instead of one: the same
// time (200 registers); the next sample's gathers issued under this
// sample's layer-1 MFMAs (software-pipelined into the free LDS input stage):
// 7.55-7.59 against 7.44-7.53 ms (profiles/r6o_mask_pipe_ab.txt) -- the
// gathers are not what bounds this form.
#ifndef SAMNERF_MASK_W8
#define SAMNERF_MASK_W8 1
#endif
namespace mw8 {
constexpr int kRays = 16;                                      // ray slots per wave
constexpr int kL0 = 5, kH = 8;                                   // layer-0 / hidden k-blocks (32 deep)
constexpr int kNbuf = 4;
constexpr int steps(int ot) { return 2 * kL0 + 2 * kH + ot; }
__host__ __device__ constexpr int hunit(int b, int g, int m) { return 32 * b + (m < 4 ? 4 * g + m : 16 + 4 * g + m - 4); }
}  // namespace mw8

// packed[step][hi/lo][slot 8][lane 64] (step layout above), then kexp[3]
template <int OT>
__global__ void __launch_bounds__(1024)
k_mask_pack_w8(const float* __restrict__ w0, const float* __restrict__ w1, const float* __restrict__ w2,
               uint32_t K, uint4* __restrict__ packed) {
    __shared__ float wm[3][16];
    __shared__ int ke[3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float m0 = 0.0f, m1 = 0.0f, m2 = 0.0f;
    for (int i = tid; i < 256 * kMIn; i += 1024) m0 = fmaxf(m0, fabsf(w0[i]));
    for (int i = tid; i < 256 * 256; i += 1024) m1 = fmaxf(m1, fabsf(w1[i]));
    for (int i = tid; i < (int)K * 256; i += 1024) m2 = fmaxf(m2, fabsf(w2[i]));
    m0 = wave_max64(m0);
    m1 = wave_max64(m1);
    m2 = wave_max64(m2);
    if (lane == 0) {
        wm[0][wave] = m0;
        wm[1][wave] = m1;
        wm[2][wave] = m2;
    }
    __syncthreads();
    if (tid < 3) {
        float m = 0.0f;
        for (int w = 0; w < 16; ++w) m = fmaxf(m, wm[tid][w]);
        ke[tid] = scale_exp_of_max(m);
    }
    __syncthreads();
    constexpr int S = mw8::steps(OT);
    for (int t = tid; t < S * 8 * 64; t += 1024) {
        const int l = t & 63, slot = (t >> 6) & 7, step = t >> 9;
        const int i = l & 15, g = l >> 4;
        int layer;
        float v[8];
        if (step < 2 * mw8::kL0) {                     // layer 0: k-block step / 2, tiles 8 (step & 1) + slot
            layer = 0;
            const int unit = 16 * (8 * (step & 1) + slot) + i;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int col = 32 * (step >> 1) + 8 * g + m;
                v[m] = col < kMIn ? w0[unit * kMIn + col] : 0.0f;
            }
        } else if (step < 2 * (mw8::kL0 + mw8::kH)) {  // layer 1
            layer = 1;
            const int q = step - 2 * mw8::kL0, unit = 16 * (8 * (q & 1) + slot) + i;
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = w1[unit * 256 + mw8::hunit(q >> 1, g, m)];
        } else {                                       // layer 2: output tile step - 26, k-block = slot
            layer = 2;
            const int unit = 16 * (step - 2 * (mw8::kL0 + mw8::kH)) + i;
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = (uint32_t)unit < K ? w2[unit * 256 + mw8::hunit(slot, g, m)] : 0.0f;
        }
        uint4 a, b;
        to_operand<false>(v, exp2i(ke[layer]), a, b);
        packed[(size_t)step * kStepVec + slot * 64 + l] = a;
        packed[(size_t)step * kStepVec + 512 + slot * 64 + l] = b;
    }
    if (tid < 3) reinterpret_cast<int*>(packed + (size_t)S * kStepVec)[tid] = ke[tid];
}

template <int OT, int WAVES>
struct MaskStreamW8 {
    static constexpr int S = mw8::steps(OT);
    static constexpr int kPieces = 16 / WAVES;          // 1-KiB pieces per wave and step
    const uint4* __restrict__ packed;
    uint4* Wb;            // [kNbuf][kStepVec]
    int wave, lane;
    uint32_t step, total;

    // wave w moves uint4 64 kPieces w .. of step s (kPieces x 1 KiB) into
    // ring slot s % kNbuf by LDS DMA; the step's offset is opaque (formed
    // here, not hoisted as per-step pointers).  No VGPR is written inside the
    // statements: a VGPR output could land on a register an MFMA issued just
    // before still reads or writes, which hipcc does not pad for an asm
    // statement (tools/isa_hazards.py R2 / R3)
    __device__ __forceinline__ void request(uint32_t s) {
        uint32_t so = (s % (uint32_t)S) * (uint32_t)(kStepVec * 16);
        asm volatile("" : "+s"(so));
        const char* base = reinterpret_cast<const char*>(packed) + so;
        const uint32_t vo = (uint32_t)(wave * 64 * kPieces + lane) * 16u;
        const uint32_t d = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(Wb + (size_t)(s % (uint32_t)mw8::kNbuf) * kStepVec + wave * 64 * kPieces));
#pragma unroll
        for (int c = 0; c < kPieces; ++c) {
            const uint32_t vc = vo + 1024u * (uint32_t)c;
            uint32_t keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(vc), "s"(base), "s"(d + 1024u * (uint32_t)c));
        }
    }
    __device__ __forceinline__ void begin() {
        for (uint32_t s = 0; s + 1 < (uint32_t)mw8::kNbuf && s < total; ++s) request(s);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    __device__ __forceinline__ const uint4* start() {
        if (step + mw8::kNbuf - 1 < total) request(step + mw8::kNbuf - 1);
        return Wb + (size_t)(step % (uint32_t)mw8::kNbuf) * kStepVec + lane;
    }
    // step + 1's pieces landed: younger than them are at most the kPieces
    // (kNbuf - 2) pieces of the steps after it (other loads in between only make the wait
    // stricter); at the end of the stream everything
    __device__ __forceinline__ void finish() {
        if (step + mw8::kNbuf - 1 < total) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPieces * (mw8::kNbuf - 2)) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        ++step;
    }
    // one 32-deep k-block of the current layer for tiles 8 HALF .. 8 HALF + 7
    // (fragments in two batches of 4 tiles: 32 registers, not 64, at the
    // layer-1 peak -- accumulators, operands and fragments -- of a 256-register wave)
    template <int HALF>
    __device__ __forceinline__ void run(floatx4 (&acc)[16], const uint4& bh, const uint4& bl) {
        const uint4* cur = start();
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            uint4 fh[4], fl[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                fh[t] = cur[(4 * q + t) * 64];
                fl[t] = cur[512 + (4 * q + t) * 64];
            }
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[8 * HALF + 4 * q + t] = mfma16_f16x3(fh[t], fl[t], bh, bl, acc[8 * HALF + 4 * q + t]);
            if (q == 0) __builtin_amdgcn_sched_barrier(0);
        }
        finish();
    }
    // one output tile: its 8 k-blocks from the step's 8 slots
    __device__ __forceinline__ void run_out(floatx4& o, const uint4 (&ah)[mw8::kH], const uint4 (&al)[mw8::kH]) {
        const uint4* cur = start();
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            uint4 fh[4], fl[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                fh[k] = cur[(4 * q + k) * 64];
                fl[k] = cur[512 + (4 * q + k) * 64];
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) o = mfma16_f16x3(fh[k], fl[k], ah[4 * q + k], al[4 * q + k], o);
            if (q == 0) __builtin_amdgcn_sched_barrier(0);
        }
        finish();
    }
};

__device__ __forceinline__ float ray_max4_mw8(float m) {             // lanes j, j + 16, j + 32, j + 48
    m = fmaxf(m, __shfl_xor(m, 16));
    return fmaxf(m, __shfl_xor(m, 32));
}

// leaky's max in place on the accumulator register ("+v"): the statement
// then writes only a register whose MFMA result the multiply before it has
// already waited for -- with a separate output, hipcc was free to pick a
// register a still-running MFMA of the layer reads as SrcC (write-after-read,
// tools/isa_hazards.py R3, found when this kernel was written)
__device__ __forceinline__ void leaky_inplace(float& x) {
    const float t = x * 0.01f;
    asm("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(t));
}

// leaky_relu on a layer's 16 tiles, then the next layer's B operands (k-block
// b <- tiles 2 b, 2 b + 1) at the ray's scale; returns its exponent
__device__ __forceinline__ int epilogue_w8(floatx4 (&acc)[16], uint4 (&ah)[mw8::kH], uint4 (&al)[mw8::kH]) {
    float m = 0.0f;
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            float v = acc[t][r];
            leaky_inplace(v);
            acc[t][r] = v;
            m = fmaxf(m, fabsf(acc[t][r]));
        }
    const int k = scale_exp_of_max(ray_max4_mw8(m));
    const float s = exp2i(k);
#pragma unroll
    for (int b = 0; b < mw8::kH; ++b) {
        const float v[8] = {acc[2 * b][0], acc[2 * b][1], acc[2 * b][2], acc[2 * b][3],
                            acc[2 * b + 1][0], acc[2 * b + 1][1], acc[2 * b + 1][2], acc[2 * b + 1][3]};
        split8_f16<true>(v, s, ah[b], al[b]);
    }
    return k;
}

// WAVES 8: one 512-thread workgroup per CU (128 ray slots), the layer-0
// inputs through LDS.  WAVES 4: two independent 256-thread workgroups per CU
// (64 slots each, its own weight ring and step barriers, the inputs in
// registers): the two waves of a SIMD belong to different workgroups and
// drift out of phase, so one's gathers run under the other's MFMAs, where the
// 8 waves of one workgroup move in lockstep from barrier to barrier.
template <int OT, int WAVES>
__global__ void __launch_bounds__(64 * WAVES) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_mask_head_w8(MaskArgs a) {
    // LDS: the weight ring | (WAVES 8) each wave's layer-0 inputs of the
    // current sample (fp32, [k-block][part][lane]) | the level descriptors
    constexpr bool XLDS = WAVES == 8;
    constexpr int kXw = XLDS ? mw8::kL0 * 2 * 64 : 0;
    __shared__ uint4 smem[mw8::kNbuf * kStepVec + WAVES * kXw + kDescVec];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int j = lane & 15, g = lane >> 4;
    const uint32_t slot = blockIdx.x * (uint32_t)(WAVES * mw8::kRays) + (uint32_t)(wave * mw8::kRays + j);
    const bool live = slot < a.N;
    const uint32_t ss = live ? slot : a.N - 1u, N = a.N;
    uint4* const Xw = smem + mw8::kNbuf * kStepVec + wave * kXw;
    LevelDesc* const sLv = reinterpret_cast<LevelDesc*>(smem + mw8::kNbuf * kStepVec + WAVES * kXw);
    if (tid < 16) sLv[tid] = a.grid.lv[tid];
    MaskStreamW8<OT, WAVES> st{a.packed, smem, wave, lane, 0u, (uint32_t)kT * (uint32_t)mw8::steps(OT)};
    st.begin();

    const int kw = a.kexp[0] + a.kexp[1] + a.kexp[2];             // the weight tensors' log2 scales
    floatx4 sum[OT];
#pragma unroll
    for (int o = 0; o < OT; ++o) sum[o] = floatx4{};
    floatx4 acc[16];
    uint4 ah[mw8::kH], al[mw8::kH];
    // 32-bit byte offsets from the uniform array bases (saddr loads; the host
    // launches this form for N < 2^21: 2 KiB of geo rows per ray)
    const char* const ub = reinterpret_cast<const char*>(a.u_in);
    const char* const wb = reinterpret_cast<const char*>(a.w_in);
    const char* const gb = reinterpret_cast<const char*>(a.geo_in);
    auto ld = [](const char* b, uint32_t off) { return *reinterpret_cast<const float*>(b + off); };
    const char* const eb = reinterpret_cast<const char*>(a.grid.emb);
    // sample kk's position (slot order, [32][3][N])
    auto position = [&](uint32_t kk, float& px, float& py, float& pz) {
        asm volatile("" : "+s"(kk));
        const uint32_t uo = (kk * 3u * N + ss) * 4u;
        px = ld(ub, uo), py = ld(ub, uo + 4u * N), pz = ld(ub, uo + 8u * N);
    };
    // level 4 b + g's 8 corner rows (issue) and their sum in lookup_level3's
    // corner order (as gather8_finish); gq: this lane's group, opaque per call
    // (the descriptors re-read from LDS, not hoisted through the loop)
    struct Rows {
        float4 e[8][2];
        float cw[8];
    };
    auto issue_level = [&](int b, float px, float py, float pz, Rows& r) {
        uint32_t gq = (uint32_t)g;
        asm volatile("" : "+v"(gq));
        uint32_t off[8];
        corner_rows<8>(sLv[4 * b + gq], px, py, pz, off, r.cw);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            r.e[c][0] = *reinterpret_cast<const float4*>(eb + off[c]);
            r.e[c][1] = *reinterpret_cast<const float4*>(eb + off[c] + 16u);
        }
    };
    auto sum_level = [&](const Rows& r, float* f) {
        f2v acc2[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc2[i] = f2v{0.0f, 0.0f};
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const f2v wc = {r.cw[c], r.cw[c]};
            acc2[0] = __builtin_elementwise_fma(wc, f2v{r.e[c][0].x, r.e[c][0].y}, acc2[0]);
            acc2[1] = __builtin_elementwise_fma(wc, f2v{r.e[c][0].z, r.e[c][0].w}, acc2[1]);
            acc2[2] = __builtin_elementwise_fma(wc, f2v{r.e[c][1].x, r.e[c][1].y}, acc2[2]);
            acc2[3] = __builtin_elementwise_fma(wc, f2v{r.e[c][1].z, r.e[c][1].w}, acc2[3]);
        }
        f[0] = acc2[0].x, f[1] = acc2[0].y, f[2] = acc2[1].x, f[3] = acc2[1].y;
        f[4] = acc2[2].x, f[5] = acc2[2].y, f[6] = acc2[3].x, f[7] = acc2[3].y;
    };
    float xr[XLDS ? 1 : mw8::kL0][8];                              // WAVES 4: the inputs in registers
    auto put = [&](int b, const float* f, float& xm) {
        if constexpr (XLDS) {
            Xw[(2 * b) * 64 + lane] = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]),
                                                 __float_as_uint(f[2]), __float_as_uint(f[3]));
            Xw[(2 * b + 1) * 64 + lane] = make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]),
                                                     __float_as_uint(f[6]), __float_as_uint(f[7]));
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) xr[b][m] = f[m];
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) xm = fmaxf(xm, fabsf(f[m]));
    };
    auto geo = [&](uint32_t kk, float& xm) {
        uint32_t gq = (uint32_t)g;
        asm volatile("" : "+v"(gq));
        asm volatile("" : "+s"(kk));
        float f[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t gi = 8u * gq + (uint32_t)m;             // geo_feat index; >= 15: padding
            f[m] = gi < 15u ? ld(gb, ((kk * 16u + gi + 1u) * N + ss) * 4u) : 0.0f;
        }
        put(4, f, xm);
    };
    // all of sample kk's inputs, one level's rows in flight at a time
    auto inputs = [&](uint32_t kk, float& xm) {
        float px, py, pz;
        position(kk, px, py, pz);
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            Rows r;
            issue_level(b, px, py, pz, r);
            float f[8];
            sum_level(r, f);
            put(b, f, xm);
            __builtin_amdgcn_sched_barrier(0);
        }
        geo(kk, xm);
    };
#pragma unroll 1
    for (int k = 0; k < kT; ++k) {
        uint32_t ko = (uint32_t)k;
        asm volatile("" : "+s"(ko));
        const float w = live ? ld(wb, (ko * N + ss) * 4u) : 0.0f;
        float xm = 0.0f;
        inputs(ko, xm);
        const int k0 = scale_exp_of_max(ray_max4_mw8(xm));
        const float s0 = exp2i(k0);
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = floatx4{};
#pragma unroll
        for (int b = 0; b < mw8::kL0; ++b) {
            float v[8];
            if constexpr (XLDS) {
                const uint4 u0 = Xw[(2 * b) * 64 + lane], u1 = Xw[(2 * b + 1) * 64 + lane];
                v[0] = __uint_as_float(u0.x), v[1] = __uint_as_float(u0.y), v[2] = __uint_as_float(u0.z);
                v[3] = __uint_as_float(u0.w), v[4] = __uint_as_float(u1.x), v[5] = __uint_as_float(u1.y);
                v[6] = __uint_as_float(u1.z), v[7] = __uint_as_float(u1.w);
            } else {
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = xr[b][m];
            }
            uint4 xh, xl;
            split8_f16<true>(v, s0, xh, xl);
            st.template run<0>(acc, xh, xl);
            st.template run<1>(acc, xh, xl);
        }
        const int k1 = epilogue_w8(acc, ah, al);
#pragma unroll
        for (int t = 0; t < 16; ++t) acc[t] = floatx4{};
#pragma unroll
        for (int b = 0; b < mw8::kH; ++b) {
            st.template run<0>(acc, ah[b], al[b]);
            st.template run<1>(acc, ah[b], al[b]);
        }
        const int k2 = epilogue_w8(acc, ah, al);
        // the logits carry 2^(k0 + k1 + k2 + the weight scales); w * 2^-e is exact
        const float wo = w * exp2i(-(k0 + k1 + k2 + kw));
#pragma unroll
        for (int o = 0; o < OT; ++o) {
            floatx4 lo = {};
            st.run_out(lo, ah, al);
#pragma unroll
            for (int r = 0; r < 4; ++r) sum[o][r] = __builtin_fmaf(wo, lo[r], sum[o][r]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!live) return;
    float* dst = a.out + (size_t)a.tiles(slot) * a.K;
#pragma unroll
    for (int o = 0; o < OT; ++o)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t u = (uint32_t)(16 * o + 4 * g + r);
            if (u < a.K) dst[u] = sum[o][r];
        }
}

}  // namespace

namespace samnerf {

size_t mask_head_packed_floats() {
    const size_t h32 = (size_t)kMaskCopies * kPackVec * 4 + 4;
    const size_t hw8 = (size_t)mw8::steps(2) * kStepVec * 4 + 4;             // k_mask_head_w8's steps
    return h32 > hw8 ? h32 : hw8;
}

int mask_head_forward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                      const float* geo_f, uint32_t N, float* out, RayTiles tiles, float* packed,
                      hipStream_t s) {
    uint4* pk = reinterpret_cast<uint4*>(packed);
    const uint32_t nfrag = (uint32_t)kStepsPerSample * 8u * 64u;
    MaskArgs a;
    a.grid = grid;
    a.u_in = u_f;
    a.w_in = w_f;
    a.geo_in = geo_f;
    a.N = N;
    a.K = m->mask_out;
    a.tiles = tiles;
    a.packed = pk;
    a.kexp = reinterpret_cast<const int*>(pk + (size_t)kMaskCopies * kPackVec);
    a.out = out;
    if (m->head_mode == 1) {
        k_mask_pack_f32<<<div_up(nfrag, 256), 256, 0, s>>>(m->mask_w[0], m->mask_w[1], m->mask_w[2],
                                                           m->mask_out, pk);
        k_mask_head<true><<<div_up(N, (uint32_t)kSlots), 256, 0, s>>>(a);
    } else if (SAMNERF_MASK_W8 && N < (1u << 21)) {
        // 1: one 8-wave workgroup per CU (7.57-7.60 ms per mask view against
        // 7.86-7.94 for k_mask_head, profiles/r6m_mask_w8_ab.txt); 2: two
        // 4-wave workgroups per CU (the inputs in registers spill: 9.1-9.2 ms)
        constexpr int W = SAMNERF_MASK_W8 == 2 ? 4 : 8;
        const uint32_t grid = div_up(N, (uint32_t)(W * mw8::kRays));
        if (m->mask_out > 16u) {
            k_mask_pack_w8<2><<<1, 1024, 0, s>>>(m->mask_w[0], m->mask_w[1], m->mask_w[2], m->mask_out, pk);
            a.kexp = reinterpret_cast<const int*>(pk + (size_t)mw8::steps(2) * kStepVec);
            k_mask_head_w8<2, W><<<grid, 64 * W, 0, s>>>(a);
        } else {
            k_mask_pack_w8<1><<<1, 1024, 0, s>>>(m->mask_w[0], m->mask_w[1], m->mask_w[2], m->mask_out, pk);
            a.kexp = reinterpret_cast<const int*>(pk + (size_t)mw8::steps(1) * kStepVec);
            k_mask_head_w8<1, W><<<grid, 64 * W, 0, s>>>(a);
        }
    } else {
        k_mask_pack_h16<<<1, 1024, 0, s>>>(m->mask_w[0], m->mask_w[1], m->mask_w[2], m->mask_out, pk);
        k_mask_head<false><<<div_up(N, (uint32_t)kSlots), 256, 0, s>>>(a);
    }
    return check_launch("mask_head");
}

}  // namespace samnerf
