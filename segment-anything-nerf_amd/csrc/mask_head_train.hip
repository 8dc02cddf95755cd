// mask_head_train.hip -- the --with_mask training step's instance head
// ('default' mask_mlp_type) with its backward, exact fp32 on matrix cores.
//
// Reference (nerf/utils.py:941-977 under nerf/renderer.py:392-395, :451-452,
// heads at nerf/network.py:125-133): per final sample k of ray n
//     x_k  = cat(m_grid(xyz_k) [16 levels x 8 channels], geo_feat_k.detach() [15])
//     o_k  = W2 leaky(W1 leaky(W0 x_k))          (SkipConnMLP, bias=False)
//     instance_mask_logits_n = sum_k weights_k.detach() * o_k
// trained through softmax / clamp / NLL (utils.py:958-973): the gradient
// reaches mask_mlp's three weights and m_grid's embeddings only (weights and
// geo_feat are detached, the sample positions carry no gradient).  torch runs
// this as ~350 kernels per step (m_grid forward / backward through the
// encoder, [N, 32, 143] and [N, 32, 256] materialised twice, GEMMs, leaky
// backward); here:
//   k_mt_pack    the weights in 16x16x4 A-fragment order, forward and transposed;
//   k_mt_fwd     16 rows (samples) per workgroup: the m_grid gathers + geo_feat
//                into LDS, the three layers on v_mfma_f32_16x16x4_f32, x / h1 /
//                h2 / o saved (unit-major, row-contiguous) for the backward;
//   k_mt_logits  logits[n] = sum_k w_k o_k in sample order;
//   k_mt_bwd     16 rows per workgroup: g_o = w_k dL/dlogits_n, dz2 = (W2^T g_o) *
//                leaky'(h2), dz1 = (W1^T dz2) * leaky'(h1), dx = W0^T dz1, and
//                the trilinear scatter of dx's m_grid part into the embedding
//                gradient (float atomics per corner and channel as the
//                reference encoder's backward, gridencoder.cu:252-349, one per
//                run of the block's rows that share a corner row);
//   k_mt_dw      dW0 = dz1^T x, dW1 = dz2^T h1, dW2 = g_o^T h2 over all rows: one
//                32x32 output tile x 1,024 rows per wave, float atomics.
// Rows are sample-major (row = k * N + slot), the order in which the render
// (k_final, GEO form) leaves positions, weights and geo_feat in its workspace.
// head_mode 1: every product is an fp32 MFMA (exact fma chains), so the
// gradients match torch's fp32 autograd up to summation order.  head_mode 0
// (the default, as the inference heads; round 5): the forward's GEMMs in
// f16x3 (k_mt_fwd16 below: fp32-equivalent products on the fp16 matrix
// cores); the backward and dW stay exact fp32 in both modes (measured: the
// f16x3 forms of those are bound by the scatter and the row loads, not the
// matrix cores, and were not faster).
#include <algorithm>

#include "f16x3.h"
#include "fp32_chain.h"
#include "samnerf_common.h"

using namespace samnerf;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRows = 16;                     // rows per workgroup (fwd / bwd)
constexpr int kT = 32;                        // final samples per ray
constexpr int kIn0 = 143;                     // 128 m_grid features + 15 geo_feat
constexpr int kKp[3] = {144, 256, 256};       // padded fan-in per layer
constexpr int kOp[3] = {256, 256, 32};        // padded fan-out per layer
#ifndef SAMNERF_MT_CHUNK
#define SAMNERF_MT_CHUNK 1024
#endif
// dW's work items take the rows of a chunk in groups of 8 x kDwU (kDwU = 2
// below): a chunk size that is not a multiple of 16 would silently drop rows
static_assert(SAMNERF_MT_CHUNK % 16 == 0, "SAMNERF_MT_CHUNK must be a multiple of 16 (8 x kDwU)");
constexpr uint32_t kChunk = SAMNERF_MT_CHUNK; // rows per dW work item

__host__ __device__ constexpr int pack_base(int l) {     // floats before layer l (either pack)
    int b = 0;
    for (int i = 0; i < l; ++i) b += kKp[i] * kOp[i];
    return b;
}
constexpr int kPackFloats = pack_base(3);

struct MaskW {
    const float* w[3];       // [256,143] [256,256] [K,256]
    uint32_t K;
};
__host__ __device__ inline int logical_in(int l) { return l == 0 ? kIn0 : 256; }
__host__ __device__ inline int logical_out(int l, uint32_t K) { return l == 2 ? (int)K : 256; }

// wf[l][tile t < Op/16][step s < Kp/4][lane]: A of out = W x (16x16x4):
//   A[i = lane & 15][k = lane >> 4] = W_l[16t + i][4s + k]
// wb[l][tile t < Kp/16][step s < Op/4][lane]: A of dx = W^T g:
//   A[i][k] = W_l[4s + k][16t + i]
__global__ void __launch_bounds__(256) k_mt_pack(MaskW mw, float* __restrict__ wf, float* __restrict__ wb) {
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= (uint32_t)kPackFloats) return;
    int l = 0;
    while (l < 2 && (int)e >= pack_base(l + 1)) ++l;
    const uint32_t o = e - (uint32_t)pack_base(l);
    const uint32_t lane = o & 63u, i = lane & 15u, k = lane >> 4, ts = o >> 6;
    const float* W = mw.w[l];
    const int li = logical_in(l), lo = logical_out(l, mw.K);
    {
        const uint32_t S = (uint32_t)kKp[l] / 4u, t = ts / S, s = ts % S;
        const int r = (int)(16u * t + i), c = (int)(4u * s + k);
        wf[e] = (r < lo && c < li) ? W[(size_t)r * li + c] : 0.0f;
    }
    {
        const uint32_t S = (uint32_t)kOp[l] / 4u, t = ts / S, s = ts % S;
        const int r = (int)(4u * s + k), c = (int)(16u * t + i);
        wb[e] = (r < lo && c < li) ? W[(size_t)r * li + c] : 0.0f;
    }
}

__device__ __forceinline__ float leaky(float x) { return x >= 0.0f ? x : x * 0.01f; }

struct Saved {
    float* x;      // [144][Rp]
    float* h1;     // [256][Rp] (post leaky_relu)
    float* h2;     // [256][Rp]
    float* o;      // [32][Rp]  point mask logits
    float* go;     // [32][Rp]  d loss / d o
    float* g2;     // [256][Rp] d loss / d z2
    float* g1;     // [256][Rp] d loss / d z1
    uint32_t R, Rp;
};

struct SampleIn {
    GridDesc<16> grid;       // m_grid (L16 C8)
    const float* u;          // [32][3][N] grid-space positions (slot order)
    const float* w;          // [32][N] final weights
    const float* geo;        // [32][16][N] grid_mlp output rows (row 0 = sigma, unused)
    uint32_t N;
};

struct FwdArgs {
    SampleIn in;
    const float* wf;
    Saved sv;
};

// out[Op x 16] = W_l in[Kp x 16]: wave w owns output tiles w, w + 4, ..;
// B operand = in[(4s + k) * 16 + j] from LDS.  Returns through `store`.
template <int L, typename Store>
__device__ __forceinline__ void fwd_layer(const float* __restrict__ wf, const float* in, int w, int lane,
                                          Store store) {
    constexpr int NT = kOp[L] / 16, MT = (NT + 3) / 4, S = kKp[L] / 4;
    if (w >= NT) return;                                   // layer 2: waves 0, 1
    const int j = lane & 15, k = lane >> 4;
    f32x4 acc[MT];
    const float* Ap[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        acc[m] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        Ap[m] = wf + pack_base(L) + (size_t)(w + 4 * m) * S * 64 + lane;
    }
    mfma_chain<MT, S, 4>(acc, Ap, in + k * kRows + j);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) store(16 * (w + 4 * m) + 4 * k + r, j, acc[m][r]);
}

// the m_grid features (16 levels x 8 channels) and geo_feat of the block's 16
// rows into X[c * 16 + j]; thread (level tid >> 4, row tid & 15)
__device__ __forceinline__ void gather_x(const SampleIn& in, const LevelDesc* sLv, uint32_t r0, uint32_t R,
                                         float* X) {
    const int tid = threadIdx.x, j = tid & 15, l = tid >> 4;
    const uint32_t r = r0 + (uint32_t)j;
    const bool live = r < R;
    const uint32_t k = live ? r / in.N : 0u, s = live ? r % in.N : 0u;
    const float* up = in.u + (size_t)k * 3u * in.N + s;
    float f[8];
    lookup_level3<8>(in.grid.emb, sLv[l], up[0], up[in.N], up[2u * in.N], f);
#pragma unroll
    for (int c = 0; c < 8; ++c) X[(8 * l + c) * kRows + j] = live ? f[c] : 0.0f;
    // geo_feat: thread (g = tid >> 4 = 0..15, row j); index 15 = padding
    const float gv = (live && l < 15) ? in.geo[((size_t)k * 16u + (uint32_t)l + 1u) * in.N + s] : 0.0f;
    X[(128 + l) * kRows + j] = gv;
}

__global__ void __launch_bounds__(256) k_mt_fwd(FwdArgs a) {
    __shared__ float X[kKp[0] * kRows];
    __shared__ float H1[256 * kRows];
    __shared__ float H2[256 * kRows];
    __shared__ LevelDesc sLv[16];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t r0 = blockIdx.x * kRows;
    const Saved& sv = a.sv;
    if (tid < 16) sLv[tid] = a.in.grid.lv[tid];
    __syncthreads();
    gather_x(a.in, sLv, r0, sv.R, X);
    __syncthreads();
    for (int idx = tid; idx < kKp[0] * kRows; idx += 256)
        sv.x[(size_t)(idx / kRows) * sv.Rp + r0 + (idx % kRows)] = X[idx];
    fwd_layer<0>(a.wf, X, w, lane, [&](int u, int j, float z) {
        const float h = r0 + (uint32_t)j < sv.R ? leaky(z) : 0.0f;
        H1[u * kRows + j] = h;
        sv.h1[(size_t)u * sv.Rp + r0 + j] = h;
    });
    __syncthreads();
    fwd_layer<1>(a.wf, H1, w, lane, [&](int u, int j, float z) {
        const float h = r0 + (uint32_t)j < sv.R ? leaky(z) : 0.0f;
        H2[u * kRows + j] = h;
        sv.h2[(size_t)u * sv.Rp + r0 + j] = h;
    });
    __syncthreads();
    fwd_layer<2>(a.wf, H2, w, lane, [&](int u, int j, float z) {
        sv.o[(size_t)u * sv.Rp + r0 + j] = r0 + (uint32_t)j < sv.R ? z : 0.0f;
    });
}

// logits[tiles(s)][u] = sum_k w[k][s] * o[u][k N + s], k in sample order
__global__ void __launch_bounds__(256) k_mt_logits(const float* __restrict__ wk, const float* __restrict__ o,
                                                   uint32_t N, uint32_t K, uint32_t Rp, RayTiles tiles,
                                                   float* __restrict__ logits) {
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= N * K) return;
    const uint32_t s = e % N, u = e / N;
    float acc = 0.0f;
    for (int k = 0; k < kT; ++k) acc += wk[(size_t)k * N + s] * o[(size_t)u * Rp + (size_t)k * N + s];
    logits[(size_t)tiles(s) * K + u] = acc;
}

struct BwdArgs {
    SampleIn in;
    const float* wb;
    const float* glog;       // [N][K] d loss / d instance_mask_logits (ray order)
    RayTiles tiles;
    uint32_t K;
    Saved sv;
    float* gemb;             // m_grid embedding gradient (accumulated)
    float* rep;              // kRep copies of the coarse levels' gradient rows
    uint32_t rep_levels;     // levels 0 .. rep_levels - 1 scatter into the copies
    uint32_t rep_floats;     // floats of those levels' rows (one copy)
};

// The coarse levels' rows are hot: every sample lands in one of a few
// thousand cells, so their float atomics queue on few addresses (attribution
// build: levels 0-3 alone cost 0.37 ms of the 3.16 ms training step, levels
// 4-15 together 0.56).  As the RGB training's scatter (rgb_train.hip kRep),
// those levels add into kRep copies of their rows, the copy picked by the
// block's XCD (blocks go to the 8 XCDs round-robin), and k_mt_rep_sum folds
// the copies into the gradient in a fixed order.  Measured (tools/gpu_r4r.sh,
// 3 interleaved A/B pairs): 3.16 -> 2.99 ms per 128 x 128 training step; the
// copies cost 16 MiB of workspace.
constexpr uint32_t kRep = 8, kRepRows = 65536;          // rows of the replicated levels, at most

// gemb[i] += sum_c rep[c][i] for i < n
__global__ void __launch_bounds__(256) k_mt_rep_sum(const float* __restrict__ rep, uint32_t n,
                                                    float* __restrict__ gemb) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    float acc = 0.0f;
#pragma unroll
    for (uint32_t c = 0; c < kRep; ++c) acc += rep[(size_t)c * n + i];
    gemb[i] += acc;
}

// dx[Kp x 16] = W_l^T g[Op x 16]: output tiles t = w, w + 4, .. of NT (tiles
// past NT repeat the last and are dropped: the chain stays branch-free)
template <int L, int NT, typename Store>
__device__ __forceinline__ void bwd_layer(const float* __restrict__ wb, const float* g, int w, int lane,
                                          Store store) {
    constexpr int MT = (NT + 3) / 4, S = kOp[L] / 4;
    const int j = lane & 15, k = lane >> 4;
    f32x4 acc[MT];
    const float* Ap[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        acc[m] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        const int t = min(w + 4 * m, NT - 1);
        Ap[m] = wb + pack_base(L) + (size_t)t * S * 64 + lane;
    }
    mfma_chain<MT, S, 4>(acc, Ap, g + k * kRows + j);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int t = w + 4 * m;
        if (t >= NT) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) store(16 * t + 4 * k + r, j, acc[m][r]);
    }
}

// the trilinear scatter of dx's m_grid part (Q [128][16] of the block's rows)
// into the embedding gradient (k_mt_bwd)
__device__ __forceinline__ void mt_scatter(const BwdArgs& a, const LevelDesc* sLv, const float* Q, uint32_t r0,
                                           int w, int lane) {
    const Saved& sv = a.sv;
    const uint32_t N = a.in.N;
    // trilinear scatter: wave w takes levels w, w + 4, .., lane = (corner c,
    // channel ch), the block's 16 rows in order: each float atomic instruction
    // adds to 8 corner rows of 32 contiguous bytes (a thread per (row, level)
    // with 64 atomics of its own sent 64 lanes to 64 different rows: ~17x
    // slower per byte, MI355X_MICROARCH.md "Global float atomics").  The rows
    // are neighbouring rays at one sample index, so on the coarse levels
    // consecutive rows fall in the same cell: a lane keeps adding to its
    // corner row while the row repeats and sends one atomic per run.
    const int c = lane >> 3, ch = lane & 7;
#ifdef SAMNERF_AB_MT_NOSCATTER   // timing attribution only: no m_grid gradient
    return;
#endif
    for (int l = w; l < 16; l += 4) {
#ifdef SAMNERF_AB_MT_SCATTER_LEVELS   // timing attribution only: scatter levels [lo, hi) only
        if (l < (SAMNERF_AB_MT_SCATTER_LEVELS >> 8) || l >= (SAMNERF_AB_MT_SCATTER_LEVELS & 255)) continue;
#endif
        float* const tgt = (uint32_t)l < a.rep_levels ? a.rep + (blockIdx.x & (kRep - 1u)) * a.rep_floats : a.gemb;
        uint32_t run = 0xffffffffu;                           // the lane's current corner row (byte offset)
        float acc = 0.0f;
        for (int j = 0; j < kRows; ++j) {
            const uint32_t r = r0 + (uint32_t)j;
            if (r >= sv.R) break;                             // wave-uniform: the tail block's last rows
            const uint32_t k = r / N, s = r % N;
            const float* up = a.in.u + (size_t)k * 3u * N + s;
            uint32_t o;
            float wc;
            corner_row_of<8>(sLv[l], up[0], up[N], up[2u * N], (uint32_t)c, o, wc);
            const float v = wc * Q[(8 * l + ch) * kRows + j];
            if (o == run) {
                acc += v;
            } else {
                if (run != 0xffffffffu) atomicAdd(tgt + run / 4u + ch, acc);
                run = o;
                acc = v;
            }
        }
        if (run != 0xffffffffu) atomicAdd(tgt + run / 4u + ch, acc);
    }
}

__global__ void __launch_bounds__(256) k_mt_bwd(BwdArgs a) {
    __shared__ float P[256 * kRows];
    __shared__ float Q[256 * kRows];
    __shared__ LevelDesc sLv[16];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t r0 = blockIdx.x * kRows;
    const Saved& sv = a.sv;
    const uint32_t N = a.in.N;
    if (tid < 16) sLv[tid] = a.in.grid.lv[tid];
    // g_o[u][j] = w_row * dL/dlogits[ray][u] (u < K), into P (32 x 16)
    for (int idx = tid; idx < 32 * kRows; idx += 256) {
        const int u = idx / kRows, j = idx % kRows;
        const uint32_t r = r0 + (uint32_t)j;
        float g = 0.0f;
        if (r < sv.R && (uint32_t)u < a.K) {
            const uint32_t k = r / N, s = r % N;
            g = a.in.w[(size_t)k * N + s] * a.glog[(size_t)a.tiles(s) * a.K + u];
        }
        P[idx] = g;
        sv.go[(size_t)u * sv.Rp + r] = g;
    }
    __syncthreads();
    // torch's leaky_relu backward: grad * (result > 0 ? 1 : slope)
    bwd_layer<2, 16>(a.wb, P, w, lane, [&](int v, int j, float d) {
        const uint32_t r = r0 + (uint32_t)j;
        const float h = sv.h2[(size_t)v * sv.Rp + r];
        const float gz = r < sv.R ? (h > 0.0f ? d : d * 0.01f) : 0.0f;
        Q[v * kRows + j] = gz;
        sv.g2[(size_t)v * sv.Rp + r] = gz;
    });
    __syncthreads();
    bwd_layer<1, 16>(a.wb, Q, w, lane, [&](int v, int j, float d) {
        const uint32_t r = r0 + (uint32_t)j;
        const float h = sv.h1[(size_t)v * sv.Rp + r];
        const float gz = r < sv.R ? (h > 0.0f ? d : d * 0.01f) : 0.0f;
        P[v * kRows + j] = gz;
        sv.g1[(size_t)v * sv.Rp + r] = gz;
    });
    __syncthreads();
    // dx of the m_grid part (tiles 0..7 of 9; geo_feat is detached) into Q
    bwd_layer<0, 8>(a.wb, P, w, lane, [&](int v, int j, float d) { Q[v * kRows + j] = d; });
    __syncthreads();
    mt_scatter(a, sLv, Q, r0, w, lane);
}

// ------------------------------------------------------ f16x3 forward
// head_mode 0 (the default, as the inference heads): the forward's three
// layers as f16x3 on v_mfma_f32_16x16x32_f16 (f16x3.h: each fp32 product as
// three fp16 MFMA products of power-of-two scaled operands -- the weight
// tensors scaled per tensor at packing, each row's inputs per row from their
// max), 16 rows per workgroup as k_mt_fwd; fp32-equivalent, not k_mt_fwd's
// bits (the accumulation order differs).  A layer is: the input rows' maxima
// (LDS atomics on the magnitude bits), a split pass writing the B fragments
// of the whole layer input into LDS once ([k-step][hi/lo][lane]), then each
// wave's output tiles over the k-steps with the weights' A fragments from the
// packed copy, and the store of the unscaled value.
// Measured (round 5, 4,096-ray training step, tools/train_profile.py): the
// forward 0.485 -> 0.34 ms; the same scheme for the backward's dx chain
// (k_mt_bwd: 1.15 -> 1.28 ms -- its 16 KiB of B fragments cost a workgroup
// per CU, and the kernel is bound by the m_grid scatter, not the GEMMs) and
// for dW (0.516 -> 0.486 ms: the row loads, not the MFMAs, bound it) was not
// kept: the backward stays exact fp32 in both modes.
constexpr int kKp16[3] = {160, 256, 256};                 // fan-in padded to 32
__host__ __device__ constexpr int f16_tiles(int L) { return kOp[L] / 16; }
__host__ __device__ constexpr int f16_steps(int L) { return kKp16[L] / 32; }
__host__ __device__ constexpr int f16_vec(int L) { return f16_tiles(L) * f16_steps(L) * 2 * 64; }
__host__ __device__ constexpr int f16_base(int L) {       // uint4 before layer L
    int b = 0;
    for (int i = 0; i < L; ++i) b += f16_vec(i);
    return b;
}
constexpr int kPack16Vec = f16_base(3);
constexpr int kW16Parts = 32;                             // partial maxima per tensor

// partial max |w| of tensor blockIdx.y over its part blockIdx.x
__global__ void __launch_bounds__(256) k_mt_wmax16(MaskW mw, float* __restrict__ part) {
    __shared__ float wm[4];
    const int L = blockIdx.y, tid = threadIdx.x;
    const int n = logical_out(L, mw.K) * logical_in(L), chunk = (n + kW16Parts - 1) / kW16Parts;
    const int i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
    float m = 0.0f;
    for (int i = i0 + tid; i < i1; i += 256) m = fmaxf(m, fabsf(mw.w[L][i]));
    m = wave_max64(m);
    if ((tid & 63) == 0) wm[tid >> 6] = m;
    __syncthreads();
    if (tid == 0) part[L * kW16Parts + blockIdx.x] = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
}

// packed[L][tile][step][hi/lo][lane]: lane (i, g), 8 values m:
//   A[i][k] = W_L[16 t + i][32 s + 8 g + m] times 2^kexp[L], zero outside the
// logical shape; kexp[L] from the tensor's partial maxima
__global__ void __launch_bounds__(256) k_mt_pack16(MaskW mw, const float* __restrict__ part, int* __restrict__ kexp,
                                                   uint4* __restrict__ pk) {
    const int e = (int)(blockIdx.x * 256u + threadIdx.x);            // one (hi, lo) pair
    if (e >= kPack16Vec / 2) return;
    int L = 0, rem = e;
    while (L < 2 && rem >= f16_vec(L) / 2) rem -= f16_vec(L++) / 2;
    float wmax = 0.0f;
    for (int q = 0; q < kW16Parts; ++q) wmax = fmaxf(wmax, part[L * kW16Parts + q]);
    const int kx = scale_exp_of_max(wmax);
    if (rem == 0) kexp[L] = kx;
    const int lane = rem & 63, ts = rem >> 6, S = f16_steps(L), t = ts / S, s = ts % S;
    const int i = lane & 15, g = lane >> 4;
    const int lo_ = logical_out(L, mw.K), li = logical_in(L);
    const float* W = mw.w[L];
    float v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int r = 16 * t + i, c = 32 * s + 8 * g + m;
        v[m] = (r < lo_ && c < li) ? W[(size_t)r * li + c] : 0.0f;
    }
    uint4 hi, lo;
    split8_f16(v, exp2i(kx), hi, lo);
    uint4* o = pk + f16_base(L) + (size_t)(t * S + s) * 128;
    o[lane] = hi;
    o[64 + lane] = lo;
}

// max |v| of a row into rmax[j] (magnitude bits order as unsigned integers)
__device__ __forceinline__ void row_max_bits(uint32_t* rmax, int j, float v) {
    atomicMax(rmax + j, __float_as_uint(fabsf(v)));
}

// One f16x3 layer over the block's 16 rows: out[NT tiles of 16][16] from
// in[K][16] (LDS, row j = column j of B).  All 256 threads: the split of the
// input into B fragments (Bf, LDS [step][hi/lo][64] uint4) at each row's
// scale, then wave w takes output tiles w, w + 4, .. (< NT) over the k-steps.
// store(u, j, value) gets the unscaled fp32 result for unit u of row j.
template <int L, int NT, typename Store>
__device__ __forceinline__ void gemm16(const uint4* __restrict__ pk, const int* __restrict__ kexp, const float* in,
                                       const uint32_t* rmax, uint4* Bf, int tid, Store store) {
    constexpr int S = f16_steps(L), NTT = f16_tiles(L), MT = (NT + 3) / 4;
    static_assert(NT <= NTT, "tiles");
    // split: item (step s, B lane (j, g)) = in[32 s + 8 g + m][j], m = 0..7
    for (int it = tid; it < S * 64; it += 256) {
        const int s = it >> 6, bl = it & 63, j = bl & 15, g = bl >> 4;
        float v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = in[(32 * s + 8 * g + m) * kRows + j];
        uint4 hi, lo;
        split8_f16(v, exp2i(scale_exp_of_max(__uint_as_float(rmax[j]))), hi, lo);
        Bf[(2 * s) * 64 + bl] = hi;
        Bf[(2 * s + 1) * 64 + bl] = lo;
    }
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63, j = lane & 15, g = lane >> 4;
    if (w >= NT) return;
    const uint4* A = pk + f16_base(L) + lane;
    floatx4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    uint4 ah[2][MT], al[2][MT];
    auto load = [&](int b, int s) {
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int t = min(w + 4 * m, NT - 1);            // past NT: repeat the last (dropped)
            ah[b][m] = A[(size_t)(t * S + s) * 128];
            al[b][m] = A[(size_t)(t * S + s) * 128 + 64];
        }
    };
    load(0, 0);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (s + 1 < S) load((s + 1) & 1, s + 1);
        const uint4 bh = Bf[(2 * s) * 64 + lane], bl = Bf[(2 * s + 1) * 64 + lane];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = mfma16_f16x3(ah[s & 1][m], al[s & 1][m], bh, bl, acc[m]);
    }
    const float iw = exp2i(-kexp[L]), ir = exp2i(-scale_exp_of_max(__uint_as_float(rmax[j])));
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int t = w + 4 * m;
        if (t >= NT) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) store(16 * t + 4 * g + r, j, (acc[m][r] * iw) * ir);
    }
}

struct Fwd16Args {
    SampleIn in;
    const uint4* pk;
    const int* kexp;
    Saved sv;
};


__global__ void __launch_bounds__(256) k_mt_fwd16(Fwd16Args a) {
    __shared__ float XH2[256 * kRows];                    // x (160 rows), then h2
    __shared__ float H1[256 * kRows];
    __shared__ uint4 Bf[8 * 2 * 64];
    __shared__ uint32_t rmax[3][kRows];
    __shared__ LevelDesc sLv[16];
    const int tid = threadIdx.x;
    const uint32_t r0 = blockIdx.x * kRows;
    const Saved& sv = a.sv;
    if (tid < 16) sLv[tid] = a.in.grid.lv[tid];
    if (tid < 3 * kRows) rmax[tid / kRows][tid % kRows] = 0u;
    for (int idx = kKp[0] * kRows + tid; idx < kKp16[0] * kRows; idx += 256) XH2[idx] = 0.0f;
    __syncthreads();
    gather_x(a.in, sLv, r0, sv.R, XH2);
    __syncthreads();
    for (int idx = tid; idx < kKp[0] * kRows; idx += 256) {
        const float v = XH2[idx];
        sv.x[(size_t)(idx / kRows) * sv.Rp + r0 + (idx % kRows)] = v;
        row_max_bits(rmax[0], idx % kRows, v);
    }
    __syncthreads();
    gemm16<0, 16>(a.pk, a.kexp, XH2, rmax[0], Bf, tid, [&](int u, int j, float z) {
        const float h = r0 + (uint32_t)j < sv.R ? leaky(z) : 0.0f;
        H1[u * kRows + j] = h;
        sv.h1[(size_t)u * sv.Rp + r0 + j] = h;
        row_max_bits(rmax[1], j, h);
    });
    __syncthreads();
    gemm16<1, 16>(a.pk, a.kexp, H1, rmax[1], Bf, tid, [&](int u, int j, float z) {
        const float h = r0 + (uint32_t)j < sv.R ? leaky(z) : 0.0f;
        XH2[u * kRows + j] = h;
        sv.h2[(size_t)u * sv.Rp + r0 + j] = h;
        row_max_bits(rmax[2], j, h);
    });
    __syncthreads();
    gemm16<2, 2>(a.pk, a.kexp, XH2, rmax[2], Bf, tid, [&](int u, int j, float z) {
        sv.o[(size_t)u * sv.Rp + r0 + j] = r0 + (uint32_t)j < sv.R ? z : 0.0f;
    });
}


struct DwArgs {
    Saved sv;
    uint32_t K;
    float* gw[3];            // [256][143] [256][256] [K][256], zeroed, accumulated
};

constexpr int kDwTilesK[3] = {5, 8, 8};                  // 32-wide input tiles per layer
constexpr int kDwTilesU[3] = {8, 8, 1};                  // 32-wide output tiles per layer
__host__ __device__ constexpr int dw_items_before(int l) {
    int b = 0;
    for (int i = 0; i < l; ++i) b += kDwTilesU[i] * kDwTilesK[i];
    return b;
}
constexpr int kDwTiles = dw_items_before(3);             // 112 output tiles of 32 x 32

// dW_l[u][c] += sum over a chunk of rows of G_l[u][r] X_l[c][r] (G: dz1 / dz2
// / g_o, X: x / h1 / h2); one wave per (output tile, chunk).  The rows of an
// MFMA's k pair can be any two: lane half h of group m takes rows
// c0 + 8m + 4h .. +3 over four MFMAs, one 16-B load per operand.
__global__ void __launch_bounds__(256) k_mt_dw(DwArgs a) {
    const uint32_t item = blockIdx.x * 4u + (threadIdx.x >> 6);
    const uint32_t chunks = a.sv.Rp / kChunk;
    if (item >= (uint32_t)kDwTiles * chunks) return;
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    const uint32_t tile = item % kDwTiles, chunk = item / kDwTiles;
    int l = 0;
    while (l < 2 && (int)tile >= dw_items_before(l + 1)) ++l;
    const int lt = (int)tile - dw_items_before(l);
    const int ut = lt / kDwTilesK[l], kt = lt % kDwTilesK[l];
    const uint32_t c0 = chunk * kChunk;
    const int u = 32 * ut + i, c = 32 * kt + i;              // A row (unit) / B column (input)
    const Saved& sv = a.sv;
    const float* G = l == 0 ? sv.g1 : l == 1 ? sv.g2 : sv.go;
    const float* X = l == 0 ? sv.x : l == 1 ? sv.h1 : sv.h2;
    const bool gok = u < kOp[l], xok = c < kKp[l];
    const float* Ga = G + (size_t)(gok ? u : 0) * sv.Rp + c0 + 4 * h;
    const float* Xb = X + (size_t)(xok ? c : 0) * sv.Rp + c0 + 4 * h;
    f32x16 acc = {};
    // the rows in groups of kDwU loop trips, two register buffers in ping-pong
    // (fp32_chain.h's scheme): a group's loads are in flight while the
    // previous group's MFMAs run, where one load pair then its four MFMAs
    // waited for L2 on every trip.  The MFMA order is unchanged.
    constexpr int kDwU = 2, kDwG = (int)(kChunk / 8u) / kDwU;
    const float4 zero4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    auto load = [&](float4 (&ga)[kDwU], float4 (&xb)[kDwU], int grp) {
#pragma unroll
        for (int u = 0; u < kDwU; ++u) {
            const int m = grp * kDwU + u;
            ga[u] = *reinterpret_cast<const float4*>(Ga + 8 * m);   // rows clamped in range:
            xb[u] = *reinterpret_cast<const float4*>(Xb + 8 * m);   // unconditional loads
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    auto mma = [&](const float4 (&ga)[kDwU], const float4 (&xb)[kDwU]) {
#pragma unroll
        for (int u = 0; u < kDwU; ++u) {
            const float4 g = gok ? ga[u] : zero4, x = xok ? xb[u] : zero4;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(g.x, x.x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(g.y, x.y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(g.z, x.z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(g.w, x.w, acc, 0, 0, 0);
        }
    };
    float4 g0[kDwU], x0[kDwU], g1[kDwU], x1[kDwU];
    load(g0, x0, 0);
#pragma unroll 1
    for (int grp = 0; grp < kDwG; grp += 2) {
        load(g1, x1, min(grp + 1, kDwG - 1));
        mma(g0, x0);
        if (grp + 1 < kDwG) {
            load(g0, x0, min(grp + 2, kDwG - 1));
            mma(g1, x1);
        }
    }
    // acc register q of lane (col i, half h) = dW[32ut + (q & 3) + 8 (q >> 2) + 4h][32kt + i]
    const int lo = logical_out(l, a.K), li = logical_in(l);
    if (c >= li) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int row = 32 * ut + (q & 3) + 8 * (q >> 2) + 4 * h;
        if (row < lo) atomicAdd(a.gw[l] + (size_t)row * li + c, acc[q]);
    }
}


struct Layout {
    float *wf, *wb;
    uint4* pk16;             // f16x3 fragments (head_mode 0), kPack16Vec uint4
    int* kexp16;             // their per-tensor log2 scales, then 3 x kW16Parts partial maxima
    float* rep;              // kRep x kRepRows x 8 floats (the coarse levels' gradient copies)
    Saved sv;
    size_t bytes;
};

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

Layout carve(uint32_t N, void* base) {
    Layout L{};
    const uint32_t R = N * (uint32_t)kT;
    L.sv.R = R;
    L.sv.Rp = (R + kChunk - 1u) / kChunk * kChunk;
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t floats) {
        float* q = base ? reinterpret_cast<float*>(p + off) : nullptr;
        off += al256(floats * sizeof(float));
        return q;
    };
    const size_t Rp = L.sv.Rp;
    L.wf = take(kPackFloats);
    L.wb = take(kPackFloats);
    L.pk16 = reinterpret_cast<uint4*>(take((size_t)kPack16Vec * 4u));
    L.kexp16 = reinterpret_cast<int*>(take(4 + 3 * kW16Parts));
    L.rep = take((size_t)kRep * kRepRows * 8u);
    L.sv.x = take((size_t)kKp[0] * Rp);
    L.sv.h1 = take((size_t)256 * Rp);
    L.sv.h2 = take((size_t)256 * Rp);
    L.sv.o = take((size_t)32 * Rp);
    L.sv.go = take((size_t)32 * Rp);
    L.sv.g2 = take((size_t)256 * Rp);
    L.sv.g1 = take((size_t)256 * Rp);
    L.bytes = off;
    return L;
}

int mask_weights(const samnerf_model* m, MaskW& mw) {
    if (!m || !m->with_mask || m->mask_kind != 0)
        return fail(SAMNERF_EINVAL, "mask_train: the model has no 'default' mask head");
    if (m->mask_out < 1 || m->mask_out > 32)
        return fail(SAMNERF_EINVAL, "mask_train: mask_out %u outside 1..32", m->mask_out);
    for (int i = 0; i < 3; ++i) {
        if (!m->mask_w[i]) return fail(SAMNERF_EINVAL, "mask_train: null mask_mlp weight");
        mw.w[i] = m->mask_w[i];
    }
    mw.K = m->mask_out;
    return SAMNERF_OK;
}

// ------------------------------------------------- adaptive heads (kinds 1-2)
// 'adaptive' / 'density' (network.py:167-180, renderer.py:424-436; the
// reference's own scripts/train_mask.sh:16,20,21) and 'adaptive' / 'rgb'
// (network.py:148-160, renderer.py:400-413): bias-free Linear layers on
// concatenations [intermediate ; m] with no activation,
//     m0 = W0 g,  m_i = W_i [x_i ; m_{i-1}],  logits = W_last m_{last-1},
// where g = grid_output.detach() and the x_i are grid_mlp's (and, for 'rgb',
// the per-sample view_mlp's) saved intermediates, all detached
// (network.py:28-33).  Linear in the per-sample inputs, so with
// X = sum_k weights_k.detach() x_k (k_final<AD> writes X per ray, in the
// column order of the effective matrix: g 32 | h1 64 | h2 64 | o3 16 | v1 32 |
// v2 32) the ray's logits are the chain applied to X, and the gradient of
// every W_i is sum over rays of g_i (x) in_i(X) with g_i the chain's backward
// of dL/dlogits -- the same sums the reference's per-sample chain and
// weighted sum produce, reassociated (rounding-level differences).  Only the
// mask_mlp weights receive gradient (every input is detached).
//   k_adt_fwd   16 rays per workgroup: the chain, m_0 .. m_{L-2} saved, logits;
//   k_adt_bwd   16 rays per workgroup: g_{L-1} = dL/dlogits, g_{i-1} =
//               W_i[:, m part]^T g_i, saved;
//   k_adt_dw    dW_i = sum_r g_i[r] in_i[r]^T, one 32 x 32 output tile of one
//               layer per workgroup over all rays in ray order (fixed order:
//               bitwise reproducible, no atomics).
// fp32 VALU fma chains (4,096 rays x ~60 K MACs: the render dominates).
constexpr int kAdU = 96;                      // hidden width (network.py:147 mask_mlp_dim)
constexpr int kAdX = 240;                     // X row (raymarch.hip kAeff)
constexpr int kAdRays = 16;                   // rays per workgroup (fwd / bwd)
constexpr int kAdMaxL = 8;

struct AdLayer {
    int xo, xw;          // the X part of the input: columns [xo, xo + xw) of X (0 width: none)
    int mw;              // the m part (the previous layer's output): 96 or 0
    int out;             // 96, or K for the last layer
    const float* W;      // [out][xw + mw], torch layout: cat([x part, m part]) (renderer.py:402-433)
};

struct AdArgs {
    AdLayer L[kAdMaxL];
    int nl;
    uint32_t N;
    const float* X;      // [N][kAdX] (ray order)
    float* m;            // [nl - 1][N][96] saved layer outputs
    float* g;            // [nl - 1][N][96] their gradients (bwd)
    const float* G;      // [N][K] dL/dlogits (bwd)
    float* logits;       // [N][K] (fwd)
};

int ad_layers(const samnerf_model* m, AdLayer* L) {
    const int K = (int)m->mask_out;
    if (m->mask_kind == 1) {                    // density: g | h1 | h2 | o3, then two plain layers
        const AdLayer t[6] = {{0, 32, 0, kAdU, m->mask_w[0]},   {32, 64, kAdU, kAdU, m->mask_w[1]},
                              {96, 64, kAdU, kAdU, m->mask_w[2]}, {160, 16, kAdU, kAdU, m->mask_w[3]},
                              {0, 0, kAdU, kAdU, m->mask_w[4]},   {0, 0, kAdU, K, m->mask_w[5]}};
        for (int i = 0; i < 6; ++i) L[i] = t[i];
        return 6;
    }
    const AdLayer t[8] = {{0, 32, 0, kAdU, m->mask_w[0]},    {32, 64, kAdU, kAdU, m->mask_w[1]},
                          {96, 64, kAdU, kAdU, m->mask_w[2]},  {160, 16, kAdU, kAdU, m->mask_w[3]},
                          {176, 32, kAdU, kAdU, m->mask_w[4]}, {208, 32, kAdU, kAdU, m->mask_w[5]},
                          {0, 0, kAdU, kAdU, m->mask_w[6]},    {0, 0, kAdU, K, m->mask_w[7]}};
    for (int i = 0; i < 8; ++i) L[i] = t[i];
    return 8;
}

// 192 threads: unit u = t % 96 of rays (t / 96) * 8 .. + 7 of the block's 16
__global__ void __launch_bounds__(192) k_adt_fwd(AdArgs a) {
    __shared__ float Xs[kAdRays][kAdX];
    __shared__ float Ms[2][kAdRays][kAdU];
    const int t = threadIdx.x, u = t % kAdU, rh = t / kAdU;
    const uint32_t r0 = blockIdx.x * kAdRays, N = a.N;
    for (int e = t; e < kAdRays * kAdX; e += 192) {
        const uint32_t r = r0 + e / kAdX;
        Xs[e / kAdX][e % kAdX] = r < N ? a.X[(size_t)r * kAdX + e % kAdX] : 0.0f;
    }
    __syncthreads();
    int cur = 0;
    for (int l = 0; l < a.nl; ++l) {
        const AdLayer& L = a.L[l];
        const int ld = L.xw + L.mw;
        float acc[8] = {};
        if (u < L.out) {
            const float* w = L.W + (size_t)u * ld;
            for (int k = 0; k < L.xw; ++k) {
                const float wk = w[k];
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(wk, Xs[rh * 8 + i][L.xo + k], acc[i]);
            }
            for (int k = 0; k < L.mw; ++k) {
                const float wk = w[L.xw + k];
#pragma unroll
                for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(wk, Ms[cur][rh * 8 + i][k], acc[i]);
            }
        }
        const bool last = l == a.nl - 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t r = r0 + rh * 8 + i;
            if (u >= L.out || r >= N) continue;
            if (last) a.logits[(size_t)r * L.out + u] = acc[i];
            else {
                Ms[cur ^ 1][rh * 8 + i][u] = acc[i];
                a.m[((size_t)l * N + r) * kAdU + u] = acc[i];
            }
        }
        __syncthreads();
        cur ^= 1;
    }
}

__global__ void __launch_bounds__(192) k_adt_bwd(AdArgs a) {
    __shared__ float Gs[2][kAdRays][kAdU];
    const int t = threadIdx.x, u = t % kAdU, rh = t / kAdU;
    const uint32_t r0 = blockIdx.x * kAdRays, N = a.N;
    const int K = a.L[a.nl - 1].out;
    for (int e = t; e < kAdRays * K; e += 192) {
        const uint32_t r = r0 + e / K;
        Gs[0][e / K][e % K] = r < N ? a.G[(size_t)r * K + e % K] : 0.0f;
    }
    __syncthreads();
    int cur = 0;
    for (int l = a.nl - 1; l >= 1; --l) {        // g_{l-1} = W_l[:, m part]^T g_l
        const AdLayer& L = a.L[l];
        const int ld = L.xw + L.mw;
        float acc[8] = {};
        for (int o = 0; o < L.out; ++o) {
            const float wk = L.W[(size_t)o * ld + L.xw + u];
#pragma unroll
            for (int i = 0; i < 8; ++i) acc[i] = __builtin_fmaf(wk, Gs[cur][rh * 8 + i][o], acc[i]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const uint32_t r = r0 + rh * 8 + i;
            Gs[cur ^ 1][rh * 8 + i][u] = acc[i];
            if (r < N) a.g[((size_t)(l - 1) * N + r) * kAdU + u] = acc[i];
        }
        __syncthreads();
        cur ^= 1;
    }
}

// dW_l[o][c] = sum_r g_l[r][o] in_l[r][c], in_l = [X part ; m_{l-1}]; one
// 32 x 32 tile per workgroup (tile list from the host), 32-ray LDS tiles, a
// 2 x 2 register tile per thread, rays summed in order
struct AdTile {
    int layer, o0, c0;
};
constexpr int kAdMaxTiles = 160;
struct AdDwArgs {
    AdArgs a;
    float* dW[kAdMaxL];
    AdTile tile[kAdMaxTiles];
};

__global__ void __launch_bounds__(256) k_adt_dw(AdDwArgs d) {
    __shared__ float Gt[32][33], It[32][33];          // [ray][o], [ray][c]
    const AdArgs& a = d.a;
    const AdTile tl = d.tile[blockIdx.x];
    const AdLayer& L = a.L[tl.layer];
    const int ld = L.xw + L.mw, tid = threadIdx.x, ti = tid >> 4, tj = tid & 15;
    const uint32_t N = a.N;
    const bool lastl = tl.layer == a.nl - 1;
    float acc[2][2] = {};
    for (uint32_t rb = 0; rb < N; rb += 32) {
        for (int e = tid; e < 32 * 32; e += 256) {
            const int rr = e >> 5, j = e & 31;
            const uint32_t r = rb + rr;
            const int o = tl.o0 + j, c = tl.c0 + j;
            float gv = 0.0f, iv = 0.0f;
            if (r < N && o < L.out)
                gv = lastl ? a.G[(size_t)r * L.out + o] : a.g[((size_t)tl.layer * N + r) * kAdU + o];
            if (r < N && c < ld)
                iv = c < L.xw ? a.X[(size_t)r * kAdX + L.xo + c]
                              : a.m[((size_t)(tl.layer - 1) * N + r) * kAdU + (c - L.xw)];
            Gt[rr][j] = gv;
            It[rr][j] = iv;
        }
        __syncthreads();
#pragma unroll 8
        for (int rr = 0; rr < 32; ++rr) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_fmaf(Gt[rr][ti * 2 + i], It[rr][tj * 2 + j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int o = tl.o0 + ti * 2 + i, c = tl.c0 + tj * 2 + j;
            if (o < L.out && c < ld) d.dW[tl.layer][(size_t)o * ld + c] = acc[i][j];
        }
}

size_t ad_ws_floats(uint32_t N) { return (size_t)2 * (kAdMaxL - 1) * N * kAdU; }

}  // namespace

namespace samnerf {

size_t mask_train_workspace_bytes(uint32_t N) {
    return std::max(carve(N, nullptr).bytes, ad_ws_floats(N) * sizeof(float));
}

// model-aware: the 'default' head's activation carve (and its
// per-XCD gradient copies) or the adaptive chain's 2 x 7 x 96 floats per ray
size_t mask_train_workspace_bytes(int mask_kind, uint32_t N) {
    return mask_kind == 0 ? carve(N, nullptr).bytes : ad_ws_floats(N) * sizeof(float);
}

// The adaptive heads (mask_kind 1 / 2): X [N][240] per-ray input sums from the
// render (k_final<AD>, ray order)
int adaptive_train_forward(const samnerf_model* m, const float* X, uint32_t N, float* logits, void* ws,
                           size_t ws_bytes, hipStream_t s) {
    if (ws_bytes < ad_ws_floats(N) * sizeof(float))
        return fail(SAMNERF_EWORKSPACE, "mask_train_forward: workspace too small");
    AdArgs a{};
    a.nl = ad_layers(m, a.L);
    for (int i = 0; i < a.nl; ++i)
        if (!a.L[i].W) return fail(SAMNERF_EINVAL, "mask_train_forward: null mask_mlp weight %d", i);
    a.N = N;
    a.X = X;
    a.m = static_cast<float*>(ws);
    a.g = a.m + (size_t)(kAdMaxL - 1) * N * kAdU;
    a.logits = logits;
    k_adt_fwd<<<div_up(N, (uint32_t)kAdRays), 192, 0, s>>>(a);
    return check_launch("mask_train_forward (adaptive)");
}

int adaptive_train_backward(const samnerf_model* m, const float* X, uint32_t N, const float* grad_logits,
                            float* const* grad_w, void* ws, size_t ws_bytes, hipStream_t s) {
    if (ws_bytes < ad_ws_floats(N) * sizeof(float))
        return fail(SAMNERF_EWORKSPACE, "mask_train_backward: workspace too small");
    AdDwArgs d{};
    AdArgs& a = d.a;
    a.nl = ad_layers(m, a.L);
    a.N = N;
    a.X = X;
    a.m = static_cast<float*>(ws);
    a.g = a.m + (size_t)(kAdMaxL - 1) * N * kAdU;
    a.G = grad_logits;
    for (int i = 0; i < a.nl; ++i) {
        if (!grad_w[i]) return fail(SAMNERF_EINVAL, "mask_train_backward: null gradient %d", i);
        d.dW[i] = grad_w[i];
    }
    k_adt_bwd<<<div_up(N, (uint32_t)kAdRays), 192, 0, s>>>(a);
    int nt = 0;
    for (int l = 0; l < a.nl; ++l) {
        const int ld = a.L[l].xw + a.L[l].mw;
        for (int o0 = 0; o0 < a.L[l].out; o0 += 32)
            for (int c0 = 0; c0 < ld; c0 += 32) {
                if (nt == kAdMaxTiles) return fail(SAMNERF_EINVAL, "mask_train_backward: tile table full");
                d.tile[nt++] = AdTile{l, o0, c0};
            }
    }
    k_adt_dw<<<nt, 256, 0, s>>>(d);
    return check_launch("mask_train_backward (adaptive)");
}

// positions / weights / geo_feat of the render's final samples (sample-major,
// slot order) and its ray order
int mask_train_forward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                       const float* geo_f, uint32_t N, RayTiles tiles, float* logits, void* ws,
                       size_t ws_bytes, hipStream_t s) {
    MaskW mw;
    int rc = mask_weights(m, mw);
    if (rc) return rc;
    const Layout L = carve(N, ws);
    if (ws_bytes < L.bytes)
        return fail(SAMNERF_EWORKSPACE, "mask_train_forward: workspace needs %zu bytes, got %zu", L.bytes,
                    ws_bytes);
    // the exact fp32 fragments: the forward of head_mode 1, the backward of both
    k_mt_pack<<<div_up(kPackFloats, 256), 256, 0, s>>>(mw, L.wf, L.wb);
    if (m->head_mode == 0) {                        // f16x3 forward (fp32-equivalent)
        float* part = reinterpret_cast<float*>(L.kexp16 + 4);
        k_mt_wmax16<<<dim3(kW16Parts, 3), 256, 0, s>>>(mw, part);
        k_mt_pack16<<<div_up(kPack16Vec / 2, 256), 256, 0, s>>>(mw, part, L.kexp16, L.pk16);
        Fwd16Args a;
        a.in = SampleIn{grid, u_f, w_f, geo_f, N};
        a.pk = L.pk16;
        a.kexp = L.kexp16;
        a.sv = L.sv;
        k_mt_fwd16<<<L.sv.Rp / kRows, 256, 0, s>>>(a);   // rows R .. Rp saved as zeros (k_mt_dw)
    } else {                                        // exact fp32
        FwdArgs a;
        a.in = SampleIn{grid, u_f, w_f, geo_f, N};
        a.wf = L.wf;
        a.sv = L.sv;
        k_mt_fwd<<<L.sv.Rp / kRows, 256, 0, s>>>(a);   // rows R .. Rp saved as zeros (k_mt_dw)
    }
    k_mt_logits<<<div_up((uint64_t)N * mw.K, 256), 256, 0, s>>>(w_f, L.sv.o, N, mw.K, L.sv.Rp, tiles, logits);
    return check_launch("mask_train_forward");
}

int mask_train_backward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                        const float* geo_f, uint32_t N, RayTiles tiles, const float* grad_logits,
                        float* const* grad_w, float* grad_m_grid, void* ws, size_t ws_bytes, hipStream_t s) {
    MaskW mw;
    int rc = mask_weights(m, mw);
    if (rc) return rc;
    const Layout L = carve(N, ws);
    if (ws_bytes < L.bytes)
        return fail(SAMNERF_EWORKSPACE, "mask_train_backward: workspace needs %zu bytes, got %zu", L.bytes,
                    ws_bytes);
    if (hipMemsetAsync(grad_w[0], 0, sizeof(float) * 256 * kIn0, s) != hipSuccess ||
        hipMemsetAsync(grad_w[1], 0, sizeof(float) * 256 * 256, s) != hipSuccess ||
        hipMemsetAsync(grad_w[2], 0, sizeof(float) * mw.K * 256, s) != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "mask_train_backward: zeroing the weight gradients failed");
    BwdArgs b;
    b.in = SampleIn{grid, u_f, w_f, geo_f, N};
    b.wb = L.wb;
    b.glog = grad_logits;
    b.tiles = tiles;
    b.K = mw.K;
    b.sv = L.sv;
    b.gemb = grad_m_grid;
    // the leading levels whose rows fit kRepRows go through the copies
    b.rep = L.rep;
    b.rep_levels = 0u;
    while (b.rep_levels < 4u && grid.lv[b.rep_levels + 1u].off <= kRepRows) ++b.rep_levels;
    b.rep_floats = grid.lv[b.rep_levels].off * 8u;
    if (b.rep_levels &&
        hipMemsetAsync(L.rep, 0, sizeof(float) * kRep * b.rep_floats, s) != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "mask_train_backward: zeroing the gradient copies failed");
    k_mt_bwd<<<L.sv.Rp / kRows, 256, 0, s>>>(b);
    if (b.rep_levels) k_mt_rep_sum<<<div_up(b.rep_floats, 256), 256, 0, s>>>(L.rep, b.rep_floats, grad_m_grid);
    if ((rc = check_launch("mask_train_backward"))) return rc;
    DwArgs d;
    d.sv = L.sv;
    d.K = mw.K;
    for (int i = 0; i < 3; ++i) d.gw[i] = grad_w[i];
    k_mt_dw<<<div_up((uint64_t)kDwTiles * (L.sv.Rp / kChunk), 4), 256, 0, s>>>(d);
    return check_launch("mask_train_backward (dW)");
}

}  // namespace samnerf
