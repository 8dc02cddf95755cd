// sam_head_train.hip -- the SAM head of the distillation step (BASELINE
// config 5), forward with saved activations and the full backward, on fp32
// matrix cores.
//
// samvit_mlp = Sequential(SkipConnMLP(163, 256, 256, 5, skip_layers=[2],
// bias=True), LayerNorm(256)) (nerf/network.py:36-75, :120-123) applied to the
// head input rows of the fused render; the step backpropagates MSE(samvit,
// gt) through it (nerf/utils.py:1098-1106).  torch runs this as ~30 kernels
// for 4,096 rays (GEMMs of 4096 x 256 x K, leaky_relu and its backward,
// LayerNorm forward / backward, bias reductions, zero fills: ~0.4 ms of the
// 1.5 ms step, profiles/r2_train_kernel_stats.csv).  Here:
//   k_ht_pack  weights into MFMA fragment order, forward and transposed
//   k_ht_fwd   16 rays per workgroup, all 5 layers + LayerNorm, activations
//              kept in LDS and saved for the backward;
//   k_ht_bwd   LayerNorm backward, then dX = W^T G through the 5 layers with
//              the leaky_relu derivative; writes the gradient of the head
//              input (its f_sam part feeds the s_grid scatter), per-workgroup
//              LN-parameter partials, and zeroes the parameter gradients;
//   k_ht_dw    dW_l = G_l^T X_l over all rays: one 32x32 output tile x 256
//              rays per wave, float atomics into the weight gradients; the
//              bias gradients (row sums of G_l) and the LN partials per
//              256-ray chunk.  No address takes more than one atomic per
//              chunk: the first version summed the bias gradients with one
//              atomic per workgroup and address in k_ht_bwd (256 same-address
//              atomics each at 4,096 rays), which made k_ht_bwd 436 us.
// Every product is v_mfma_f32_16x16x4_f32 / v_mfma_f32_32x32x2_f32: exact fp32
// (an fma chain in k order, cdna_hip_programming.md "FP32-input MFMA"), so
// the gradients match torch's fp32 autograd to summation-order rounding.
// 16 rays per workgroup: 256 workgroups for a 4,096-ray step fill the chip.
#include <algorithm>
#include <cstring>

#include "fp32_chain.h"
#include "samnerf_common.h"

using namespace samnerf;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kIn = 163;            // head inputs (f_sam 128, f_image 31, image 3, depth 1)
constexpr int kRowIn = 164;         // row stride of the render's head-input rows
constexpr int kRays = 16;           // rays per workgroup (forward / backward)
constexpr int kKp[5] = {176, 256, 432, 256, 256};        // padded fan-in per layer
constexpr int kKl[5] = {163, 256, 419, 256, 256};        // logical fan-in (torch weight columns)

__host__ __device__ constexpr int fwd_base(int l) {      // floats before layer l (forward pack)
    int b = 0;
    for (int i = 0; i < l; ++i) b += 256 * kKp[i];
    return b;
}
constexpr int kPackFloats = fwd_base(5);                  // same count for the transposed pack

// logical weight column of padded input k of layer l, or -1 (zero padding)
__host__ __device__ constexpr int kcol(int l, int k) {
    return l == 0 ? (k < kIn ? k : -1) : l == 2 ? (k < 256 + kIn ? k : -1) : k;
}

struct HeadW {
    const float* w[5];
    const float* b[5];
    const float* ln_w;
    const float* ln_b;
};

// Wf[l][tile t 0..15][step s 0..Kp/4-1][lane]: A of out = W x, 16x16x4:
//   A[i = lane & 15][k = lane >> 4] = W_l[16t + i][4s + k]
// Wb[l][tile t 0..Kp/16-1][step s 0..63][lane]: A of dX = W^T G:
//   A[i][k] = W_l[4s + k][16t + i]
__global__ void __launch_bounds__(256) k_ht_pack(HeadW hw, float* __restrict__ wf, float* __restrict__ wb) {
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= (uint32_t)kPackFloats) return;
    int l = 0;
    while (l < 4 && (int)e >= fwd_base(l + 1)) ++l;
    const uint32_t o = e - (uint32_t)fwd_base(l);
    const uint32_t lane = o & 63u, i = lane & 15u, k = lane >> 4;
    const float* W = hw.w[l];
    const int kl = kKl[l];
    {   // forward: o = (t * Kp/4 + s) * 64 + lane
        const uint32_t ts = o >> 6, S = (uint32_t)kKp[l] / 4u;
        const uint32_t t = ts / S, s = ts % S;
        const int col = kcol(l, (int)(4u * s + k));
        wf[e] = col >= 0 ? W[(size_t)(16u * t + i) * kl + col] : 0.0f;
    }
    {   // transposed: o = (t * 64 + s) * 64 + lane
        const uint32_t ts = o >> 6;
        const uint32_t t = ts >> 6, s = ts & 63u;
        const int col = kcol(l, (int)(16u * t + i));
        wb[e] = col >= 0 ? W[(size_t)(4u * s + k) * kl + col] : 0.0f;
    }
}

__device__ __forceinline__ float leaky(float x) { return x >= 0.0f ? x : x * 0.01f; }

struct FwdArgs {
    HeadW hw;
    const float* rows;     // [N][164]
    const float* wf;       // forward pack
    uint32_t N, Np;        // rays, padded ray stride of the saved buffers
    float* samvit;         // [N][256]
    float* hsave;          // [5][256][Np]: h0..h3 (post leaky_relu), y (pre LayerNorm)
    float* stats;          // [Np][2]: mean, rstd
};

// out[256 x 16] = act(W_l in[Kp x 16] + b): wave w owns the output tiles
// 4w..4w+3 (units 64w..64w+63); B operand = in[(4s + k) * 16 + j] from LDS.
template <int L>
__device__ __forceinline__ void fwd_layer(const FwdArgs& a, const float* in, float* out, int w, int lane,
                                          uint32_t ray0) {
    constexpr int S = kKp[L] / 4;
    const int j = lane & 15, k = lane >> 4;
    f32x4 acc[4];
    const float* Ap[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        acc[t] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        Ap[t] = a.wf + fwd_base(L) + (size_t)(4 * w + t) * S * 64 + lane;
    }
    mfma_chain<4, S, 4>(acc, Ap, in + k * kRays + j);
    const bool live = ray0 + (uint32_t)j < a.N;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int u = 16 * (4 * w + t) + 4 * k + r;
            const float z = acc[t][r] + a.hw.b[L][u];
            const float h = L < 4 ? leaky(z) : z;
            out[u * kRays + j] = h;
            a.hsave[((size_t)L * 256 + u) * a.Np + ray0 + j] = live ? h : 0.0f;
        }
}

__global__ void __launch_bounds__(256) k_ht_fwd(FwdArgs a) {
    __shared__ float P[256 * kRays];
    __shared__ float Q[432 * kRays];                     // rows 0..255: h1 / h3; 256..431: x
    __shared__ float red[16 * kRays];
    __shared__ float st[2 * kRays];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t ray0 = blockIdx.x * kRays;
    for (int idx = tid; idx < kRays * 176; idx += 256) {  // x, transposed into Q[256 + c][ray]
        const int jr = idx / 176, c = idx % 176;
        const uint32_t ray = ray0 + jr;
        Q[(256 + c) * kRays + jr] = (c < kIn && ray < a.N) ? a.rows[(size_t)ray * kRowIn + c] : 0.0f;
    }
    __syncthreads();
    fwd_layer<0>(a, Q + 256 * kRays, P, w, lane, ray0);
    __syncthreads();
    fwd_layer<1>(a, P, Q, w, lane, ray0);
    __syncthreads();
    fwd_layer<2>(a, Q, P, w, lane, ray0);
    __syncthreads();
    fwd_layer<3>(a, P, Q, w, lane, ray0);
    __syncthreads();
    fwd_layer<4>(a, Q, P, w, lane, ray0);
    __syncthreads();
    // LayerNorm(256, eps 1e-5) per ray over P[u][ray]: two passes
    const int j = tid & 15, p = tid >> 4;
    float s1 = 0.0f;
#pragma unroll
    for (int u = 0; u < 16; ++u) s1 += P[(16 * p + u) * kRays + j];
    red[p * kRays + j] = s1;
    __syncthreads();
    if (tid < kRays) {
        float m = 0.0f;
        for (int q = 0; q < 16; ++q) m += red[q * kRays + tid];
        st[tid] = m / 256.0f;
    }
    __syncthreads();
    float s2 = 0.0f;
    const float mj = st[j];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
        const float d = P[(16 * p + u) * kRays + j] - mj;
        s2 += d * d;
    }
    red[p * kRays + j] = s2;
    __syncthreads();
    if (tid < kRays) {
        float v = 0.0f;
        for (int q = 0; q < 16; ++q) v += red[q * kRays + tid];
        const float rstd = 1.0f / sqrtf(v / 256.0f + 1e-5f);
        st[kRays + tid] = rstd;
        const uint32_t ray = ray0 + tid;
        a.stats[(size_t)ray * 2 + 0] = ray < a.N ? st[tid] : 0.0f;
        a.stats[(size_t)ray * 2 + 1] = ray < a.N ? rstd : 0.0f;
    }
    __syncthreads();
    const int u = tid;
    const float gw = a.hw.ln_w[u], gb = a.hw.ln_b[u];
    for (int jj = 0; jj < kRays; ++jj) {
        const uint32_t ray = ray0 + jj;
        if (ray >= a.N) break;
        a.samvit[(size_t)ray * 256 + u] = (P[u * kRays + jj] - st[jj]) * st[kRays + jj] * gw + gb;
    }
}

struct BwdArgs {
    HeadW hw;
    const float* wb;        // transposed pack
    const float* gout;      // [N][256] d loss / d samvit
    const float* hsave;     // [5][256][Np]
    const float* stats;     // [Np][2]
    uint32_t N, Np;
    float* G;               // [5][256][Np] d loss / d z_l (pre-activation), for k_ht_dw
    float* grows;           // [N][164]: d loss / d head input (column 163 written 0)
    float* lnpart;          // [blocks][512]: per-workgroup sums of g * yhat (LN weight), g (LN bias)
    float* zero[12];        // parameter gradients, zeroed here and accumulated by k_ht_dw
    uint32_t zero_n[12];
};

// zero the parameter gradients (k_ht_dw, stream-ordered after this kernel,
// accumulates into them)
__device__ __forceinline__ void zero_grads(const BwdArgs& a) {
    const uint32_t stride = gridDim.x * blockDim.x;
    for (int t = 0; t < 12; ++t)
        for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < a.zero_n[t]; e += stride) a.zero[t][e] = 0.0f;
}

// dX[Kp x 16] = W_l^T G[256 x 16]: output tiles t = w, w + 4, .. of Kp/16.
// MODE 0: the next G = dX * leaky'(h_{l-1}) into out (+ save for k_ht_dw)
// MODE 1 (layer 2): rows < 256 as MODE 0, rows >= 256 raw into out (skip)
// MODE 2 (layer 0): grows = dX + skip (out holds the skip rows at 256 + c)
template <int L, int MODE>
__device__ __forceinline__ void bwd_layer(const BwdArgs& a, const float* in, float* out, int w, int lane,
                                          uint32_t ray0) {
    constexpr int NT = kKp[L] / 16;
    constexpr int MT = (NT + 3) / 4;
    const int j = lane & 15, k = lane >> 4;
    const uint32_t ray = ray0 + (uint32_t)j;
    const bool live = ray < a.N;
    f32x4 acc[MT];
    const float* Ap[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        acc[m] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
        // tiles past NT (layers 0 and 2: 11 and 27 tiles over 4 waves) repeat
        // the last tile and are dropped below: the chain stays branch-free
        const int t = min(w + 4 * m, NT - 1);
        Ap[m] = a.wb + fwd_base(L) + (size_t)t * 64 * 64 + lane;
    }
    mfma_chain<MT, 64, 4>(acc, Ap, in + k * kRays + j);
#pragma unroll
    for (int m = 0; m < MT; ++m) {
        const int t = w + 4 * m;
        if (t >= NT) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int v = 16 * t + 4 * k + r;               // input unit of layer L
            const float dx = acc[m][r];
            if (MODE == 2) {
                if (v < kIn && live) a.grows[(size_t)ray * kRowIn + v] = dx + out[(256 + v) * kRays + j];
                if (v == kIn && live) a.grows[(size_t)ray * kRowIn + v] = 0.0f;
                continue;
            }
            if (MODE == 1 && v >= 256) {                    // d / d x through the skip
                out[v * kRays + j] = dx;
                continue;
            }
            // torch's in-place leaky_relu backward: grad * (result > 0 ? 1 : slope)
            const float h = a.hsave[((size_t)(L - 1) * 256 + v) * a.Np + ray];
            const float gz = live ? (h > 0.0f ? dx : dx * 0.01f) : 0.0f;
            out[v * kRays + j] = gz;
            a.G[((size_t)(L - 1) * 256 + v) * a.Np + ray] = gz;
        }
    }
}

__global__ void __launch_bounds__(256) k_ht_bwd(BwdArgs a) {
    __shared__ float P[256 * kRays];
    __shared__ float Q[432 * kRays];
    __shared__ float red[2][4][kRays];
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const uint32_t ray0 = blockIdx.x * kRays;
    zero_grads(a);
    // LayerNorm backward: thread u holds unit u of the 16 rays
    {
        const int u = tid;
        const float gw = a.hw.ln_w[u];
        float yh[kRays], gyh[kRays];
        float dgw = 0.0f, dgb = 0.0f;
#pragma unroll
        for (int jj = 0; jj < kRays; ++jj) {
            const uint32_t ray = ray0 + jj;
            const bool live = ray < a.N;
            const float g = live ? a.gout[(size_t)ray * 256 + u] : 0.0f;
            const float y = a.hsave[((size_t)4 * 256 + u) * a.Np + ray];
            yh[jj] = live ? (y - a.stats[(size_t)ray * 2]) * a.stats[(size_t)ray * 2 + 1] : 0.0f;
            gyh[jj] = g * gw;
            dgw += g * yh[jj];
            dgb += g;
        }
        a.lnpart[(size_t)blockIdx.x * 512 + u] = dgw;
        a.lnpart[(size_t)blockIdx.x * 512 + 256 + u] = dgb;
        // per ray: sums over the 256 units of gyh and gyh * yh (wave, then 4 waves)
#pragma unroll
        for (int jj = 0; jj < kRays; ++jj) {
            float s1 = gyh[jj], s2 = gyh[jj] * yh[jj];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                s1 += __shfl_xor(s1, o);
                s2 += __shfl_xor(s2, o);
            }
            if (lane == 0) {
                red[0][w][jj] = s1;
                red[1][w][jj] = s2;
            }
        }
        __syncthreads();
#pragma unroll
        for (int jj = 0; jj < kRays; ++jj) {
            const uint32_t ray = ray0 + jj;
            const float m1 = (red[0][0][jj] + red[0][1][jj] + red[0][2][jj] + red[0][3][jj]) / 256.0f;
            const float m2 = (red[1][0][jj] + red[1][1][jj] + red[1][2][jj] + red[1][3][jj]) / 256.0f;
            const float rstd = ray < a.N ? a.stats[(size_t)ray * 2 + 1] : 0.0f;
            const float gy = rstd * (gyh[jj] - m1 - yh[jj] * m2);
            P[u * kRays + jj] = gy;
            a.G[((size_t)4 * 256 + u) * a.Np + ray] = gy;
        }
    }
    __syncthreads();
    bwd_layer<4, 0>(a, P, Q, w, lane, ray0);      // -> G3
    __syncthreads();
    bwd_layer<3, 0>(a, Q, P, w, lane, ray0);      // -> G2
    __syncthreads();
    bwd_layer<2, 1>(a, P, Q, w, lane, ray0);      // -> G1 (rows < 256) + skip d x (rows 256..431)
    __syncthreads();
    bwd_layer<1, 0>(a, Q, P, w, lane, ray0);      // -> G0
    __syncthreads();
    bwd_layer<0, 2>(a, P, Q, w, lane, ray0);      // -> d rows = W0^T G0 + skip
}

struct DwArgs {
    const float* G;         // [5][256][Np]
    const float* hsave;     // [5][256][Np]
    const float* rows;      // [N][164]
    const float* lnpart;    // [blocks][512] from k_ht_bwd
    uint32_t N, Np, chunks; // chunks of 256 rays
    uint32_t blocks;        // k_ht_bwd workgroups
    uint32_t parts;         // partial sums per output: min(chunks, kDwParts)
    float* slab;            // [parts][kDwTiles][32 x 32] | [parts][5][256] bias | [parts][512] LN
    float* gw[5];           // weight gradients [256][K_l] (accumulated)
    float* gb[5];           // bias gradients (accumulated)
    float* gln_w;
    float* gln_b;
};

constexpr int kDwTilesK[5] = {6, 8, 14, 8, 8};          // 32-wide column tiles of Kp_l
__host__ __device__ constexpr int dw_items_before(int l) {
    int b = 0;
    for (int i = 0; i < l; ++i) b += 8 * kDwTilesK[i];
    return b;
}
constexpr int kDwTiles = dw_items_before(5);              // 352 output tiles of 32 x 32

// dW_l[u][k] = sum over the rays of G_l[u][r] X_l[k][r], in a FIXED order
// (round 5: the gradients of a step repeat bit for bit -- the round-2..4 form
// added each 256-ray chunk's tile with float atomics, in whatever order the
// waves finished).  One wave per (output tile, part): part p sums chunks p,
// p + parts, .. in order into its accumulators and stores the tile to the
// slab; k_ht_dw_sum adds the parts in order.  The sum runs over rays, so the
// rays of an MFMA's k pair can be any two: lane half h of group m takes rays
// c0 + 8m + 4h .. +3 over four MFMAs, one 16-B load per operand.  The waves
// of the first column tile (kt 0) also sum their G rows: the bias gradient.
// After the tiles, 8 waves per part sum the part's LN partials.
constexpr uint32_t kDwParts = 16;
constexpr size_t kDwSlabTile = (size_t)kDwTiles * 1024;   // floats per part: the weight tiles
__host__ __device__ constexpr size_t dw_slab_floats(uint32_t parts) {
    return (size_t)parts * (kDwSlabTile + 5 * 256 + 512);
}

__global__ void __launch_bounds__(256) k_ht_dw(DwArgs a) {
    const uint32_t item = blockIdx.x * 4u + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, i = lane & 31, h = lane >> 5;
    float* const sbias = a.slab + (size_t)a.parts * kDwSlabTile;       // [parts][5][256]
    float* const sln = sbias + (size_t)a.parts * 5 * 256;              // [parts][512]
    if (item >= (uint32_t)kDwTiles * a.parts) {
        const uint32_t e = item - (uint32_t)kDwTiles * a.parts;
        if (e >= 8u * a.parts) return;
        const uint32_t part = e >> 3, v = ((e & 7u) << 6) + (uint32_t)lane;       // v: 0..511
        float sum = 0.0f;
        for (uint32_t chunk = part; chunk < a.chunks; chunk += a.parts) {
            const uint32_t b0 = chunk * (256u / kRays), b1 = min(b0 + 256u / kRays, a.blocks);
            for (uint32_t b = b0; b < b1; ++b) sum += a.lnpart[(size_t)b * 512 + v];
        }
        sln[(size_t)part * 512 + v] = sum;
        return;
    }
    const uint32_t tile = item % kDwTiles, part = item / kDwTiles;
    int l = 0;
    while (l < 4 && (int)tile >= dw_items_before(l + 1)) ++l;
    const int lt = (int)tile - dw_items_before(l);
    const int ut = lt / kDwTilesK[l], kt = lt % kDwTilesK[l];
    const int u = 32 * ut + i, kk = 32 * kt + i;           // A row (unit) / B column (input) of this lane
    // B source: saved activations (unit-major, ray-contiguous) or the rows
    const bool from_x = (l == 0) || (l == 2 && kk >= 256);
    const int xc = l == 0 ? kk : kk - 256;                  // x column for from_x
    const bool xok = xc < kIn;
    f32x16 acc = {};
    float bsum = 0.0f;
    for (uint32_t chunk = part; chunk < a.chunks; chunk += a.parts) {
        const uint32_t c0 = chunk * 256u;
        const float* Ga = a.G + ((size_t)l * 256 + u) * a.Np + c0 + 4 * h;
        const float* Hb = (l == 0 || from_x) ? nullptr
                                             : a.hsave + ((size_t)(l - 1) * 256 + kk) * a.Np + c0 + 4 * h;
        for (int m = 0; m < 32; ++m) {
            const float4 ga = *reinterpret_cast<const float4*>(Ga + 8 * m);
            if (kt == 0) bsum += (ga.x + ga.y) + (ga.z + ga.w);
            float xb[4];
            if (from_x) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const uint32_t ray = c0 + 8u * m + 4u * h + e;
                    xb[e] = (xok && ray < a.N) ? a.rows[(size_t)ray * kRowIn + xc] : 0.0f;
                }
            } else {
                const float4 hb = *reinterpret_cast<const float4*>(Hb + 8 * m);
                xb[0] = hb.x; xb[1] = hb.y; xb[2] = hb.z; xb[3] = hb.w;
            }
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ga.x, xb[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ga.y, xb[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ga.z, xb[2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ga.w, xb[3], acc, 0, 0, 0);
        }
    }
    if (kt == 0) {
        bsum = sum_halves(bsum);
        if (h == 0) sbias[((size_t)part * 5 + l) * 256 + u] = bsum;
    }
    // acc register q of lane (col i, half h) = dW[32ut + (q & 3) + 8 (q >> 2) + 4h][32kt + i]
    float* const st = a.slab + ((size_t)part * kDwTiles + tile) * 1024;
#pragma unroll
    for (int q = 0; q < 16; ++q) st[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + i] = acc[q];
}

// the parts of every weight / bias / LN gradient added in part order into
// the (zeroed) gradients: one thread per output value
__global__ void __launch_bounds__(256) k_ht_dw_sum(DwArgs a) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t base = 0;
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        const uint32_t n = 256u * (uint32_t)kKl[l];
        if (t >= base && t < base + n) {
            const uint32_t row = (t - base) / (uint32_t)kKl[l], col = (t - base) % (uint32_t)kKl[l];
            // padded input column of logical column col (layer 0: the same; layer 2: the same)
            const uint32_t tile = (uint32_t)dw_items_before(l) + (row >> 5) * kDwTilesK[l] + (col >> 5);
            const size_t off = (size_t)tile * 1024 + (row & 31u) * 32 + (col & 31u);
            float sum = 0.0f;
            for (uint32_t p = 0; p < a.parts; ++p) sum += a.slab[(size_t)p * kDwSlabTile + off];
            a.gw[l][t - base] += sum;
            return;
        }
        base += n;
    }
    const float* sbias = a.slab + (size_t)a.parts * kDwSlabTile;
    if (t < base + 5u * 256u) {
        const uint32_t l = (t - base) >> 8, u = (t - base) & 255u;
        float sum = 0.0f;
        for (uint32_t p = 0; p < a.parts; ++p) sum += sbias[((size_t)p * 5 + l) * 256 + u];
        a.gb[l][u] += sum;
        return;
    }
    base += 5u * 256u;
    if (t < base + 512u) {
        const uint32_t v = t - base;
        const float* sln = sbias + (size_t)a.parts * 5 * 256;
        float sum = 0.0f;
        for (uint32_t p = 0; p < a.parts; ++p) sum += sln[(size_t)p * 512 + v];
        if (v < 256u) a.gln_w[v] += sum;
        else a.gln_b[v - 256u] += sum;
    }
}
constexpr uint32_t kDwOutputs = 256u * (163u + 256u + 419u + 256u + 256u) + 5u * 256u + 512u;

struct Layout {
    float* wf;
    float* wb;
    float* hsave;
    float* stats;
    float* G;
    float* lnpart;
    float* slab;            // k_ht_dw's partial sums (dw_slab_floats)
    uint32_t Np;
    size_t bytes;
};

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

Layout carve(uint32_t N, void* base) {
    Layout L{};
    L.Np = (N + 255u) & ~255u;
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t floats) {
        float* q = base ? reinterpret_cast<float*>(p + off) : nullptr;
        off += al256(floats * sizeof(float));
        return q;
    };
    L.wf = take(kPackFloats);
    L.wb = take(kPackFloats);
    L.hsave = take((size_t)5 * 256 * L.Np);
    L.stats = take((size_t)2 * L.Np);
    L.G = take((size_t)5 * 256 * L.Np);
    L.lnpart = take((size_t)512 * div_up(N, kRays));
    L.slab = take(dw_slab_floats(std::min<uint32_t>(L.Np / 256u, kDwParts)));
    L.bytes = off;
    return L;
}

int head_weights(const samnerf_model* m, HeadW& hw) {
    if (!m || !m->with_sam) return fail(SAMNERF_EINVAL, "head_train: model has no SAM head");
    for (int i = 0; i < 5; ++i) {
        if (!m->sam_w[i] || !m->sam_b[i]) return fail(SAMNERF_EINVAL, "head_train: null head weight");
        hw.w[i] = m->sam_w[i];
        hw.b[i] = m->sam_b[i];
    }
    if (!m->ln_w || !m->ln_b) return fail(SAMNERF_EINVAL, "head_train: null LayerNorm parameter");
    hw.ln_w = m->ln_w;
    hw.ln_b = m->ln_b;
    return SAMNERF_OK;
}

}  // namespace

extern "C" {

size_t samnerf_head_train_workspace_size(uint32_t N) { return carve(N, nullptr).bytes; }

int samnerf_head_train_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                               void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    HeadW hw;
    int rc = head_weights(m, hw);
    if (rc) return rc;
    if (N == 0) return SAMNERF_OK;
    if (!rows || !samvit || !workspace) return fail(SAMNERF_EINVAL, "head_train_forward: null pointer");
    const Layout L = carve(N, workspace);
    if (workspace_bytes < L.bytes)
        return fail(SAMNERF_EWORKSPACE, "head_train_forward: workspace needs %zu bytes, got %zu", L.bytes,
                    workspace_bytes);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    k_ht_pack<<<div_up(kPackFloats, 256), 256, 0, s>>>(hw, L.wf, L.wb);
    FwdArgs a{hw, rows, L.wf, N, L.Np, samvit, L.hsave, L.stats};
    // rays N .. Np of the saved buffers are written as zeros by the last
    // workgroups only up to the workgroup boundary; the rest must read as 0
    if (L.Np > div_up(N, kRays) * (uint32_t)kRays) {
        for (int l = 0; l < 5; ++l)
            (void)hipMemsetAsync(L.hsave + (size_t)l * 256 * L.Np, 0, sizeof(float) * 256 * L.Np, s);
    }
    k_ht_fwd<<<div_up(N, kRays), 256, 0, s>>>(a);
    return check_launch("head_train_forward");
}

int samnerf_head_train_backward(const samnerf_model* m, const float* rows, const float* grad_samvit,
                                uint32_t N, float* grad_rows, float* const* grad_w,
                                float* const* grad_b, float* grad_ln_w, float* grad_ln_b,
                                void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    HeadW hw;
    int rc = head_weights(m, hw);
    if (rc) return rc;
    if (N == 0) return SAMNERF_OK;
    if (!rows || !grad_samvit || !grad_rows || !grad_w || !grad_b || !grad_ln_w || !grad_ln_b || !workspace)
        return fail(SAMNERF_EINVAL, "head_train_backward: null pointer");
    for (int i = 0; i < 5; ++i)
        if (!grad_w[i] || !grad_b[i]) return fail(SAMNERF_EINVAL, "head_train_backward: null gradient");
    const Layout L = carve(N, workspace);
    if (workspace_bytes < L.bytes)
        return fail(SAMNERF_EWORKSPACE, "head_train_backward: workspace needs %zu bytes", L.bytes);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (L.Np > div_up(N, kRays) * (uint32_t)kRays)
        (void)hipMemsetAsync(L.G, 0, sizeof(float) * 5 * 256 * L.Np, s);
    BwdArgs b{};
    b.hw = hw;
    b.wb = L.wb;
    b.gout = grad_samvit;
    b.hsave = L.hsave;
    b.stats = L.stats;
    b.N = N;
    b.Np = L.Np;
    b.G = L.G;
    b.grows = grad_rows;
    b.lnpart = L.lnpart;
    for (int i = 0; i < 5; ++i) {
        b.zero[i] = grad_w[i];
        b.zero_n[i] = 256u * (uint32_t)kKl[i];
        b.zero[5 + i] = grad_b[i];
        b.zero_n[5 + i] = 256u;
    }
    b.zero[10] = grad_ln_w;
    b.zero[11] = grad_ln_b;
    b.zero_n[10] = b.zero_n[11] = 256u;
    const uint32_t blocks = div_up(N, kRays);
    k_ht_bwd<<<blocks, 256, 0, s>>>(b);
    if ((rc = check_launch("head_train_backward"))) return rc;
    DwArgs d{};
    d.G = L.G;
    d.hsave = L.hsave;
    d.rows = rows;
    d.N = N;
    d.Np = L.Np;
    d.chunks = L.Np / 256u;
    d.lnpart = L.lnpart;
    d.blocks = blocks;
    for (int i = 0; i < 5; ++i) {
        d.gw[i] = grad_w[i];
        d.gb[i] = grad_b[i];
    }
    d.gln_w = grad_ln_w;
    d.gln_b = grad_ln_b;
    d.parts = std::min<uint32_t>(d.chunks, kDwParts);
    d.slab = L.slab;
    k_ht_dw<<<div_up((uint64_t)(kDwTiles + 8) * d.parts, 4), 256, 0, s>>>(d);
    k_ht_dw_sum<<<div_up(kDwOutputs, 256), 256, 0, s>>>(d);
    return check_launch("head_train_backward (dW)");
}

}  // extern "C"
