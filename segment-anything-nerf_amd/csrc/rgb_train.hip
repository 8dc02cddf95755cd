// rgb_train.hip -- one RGB training step of the reference's Trainer
// (nerf/utils.py:897-937: render with perturb=True and update_proposal, MSE +
// lambda_proposal * proposal_loss + lambda_distort * distort_loss (+
// lambda_entropy * entropy), backward) as gfx950 kernels: the forward keeps
// what the backward needs, the backward is written out by hand -- no autograd
// graph, no [N, T, C] temporaries, ~25 launches instead of the ~700 ATen
// kernels of the torch path (nerf/renderer.py run_torch + autograd).  Entry
// points: samnerf_rgb_train_forward / _backward (an autograd pair: the train-
// mode NeRFRenderer.run) and samnerf_rgb_train_step (both plus the Trainer's
// MSE / entropy terms in one call).
//
// Forward
//   proposal stages     the fused render's own kernels (raymarch.hip
//                       proposal_forward): ds, weights and bins of both stages
//   k_rt_final_fwd      one thread per final sample (ray-major): bins ->
//                       position -> contract -> grid L16C2 gather (packed /
//                       pair-load form, bit-identical to the reference's) ->
//                       grid_mlp (exact fp32, weights in LDS); saves u, grid
//                       features, both hidden layers and the 16 outputs
//   k_rt_composite_h    a half-wave per ray: compositing (renderer.py:309-335),
//                       SH(4), f_image, view_mlp, sigmoid, background; the
//                       per-ray distortion term
//   k_rt_prop_ray_w<T>  per ray (a wave) and stage: proposal_loss (renderer.py:30-57)
//                       and its gradient w.r.t. the stage's weights (the final
//                       stage's are detached) through the stage's compositing
//                       (unit loss weight; the backward scales it)
// Backward
//   k_rt_final_bwd_ray_h  a half-wave per ray: d(image), d(weights_sum), d(depth) -> view_mlp
//                       -> f_image -> weights (+ distortion) -> delta*sigma
//                       (reverse scan) -> trunc_exp -> d(grid_mlp out)
//   k_rt_final_bwd      per sample: grid_mlp backward, d(grid features) scattered
//                       into grid.embeddings' gradient (float atomics, as
//                       kernel_grid_backward, gridencoder.cu:252-349; shaped
//                       per wave: run merge, lane quads, zero-wave skip)
//   k_rt_prop_bwd<T>    per proposal sample: prop_mlp backward, prop grid
//                       scatter, prop_mlp weight gradients as wave sums
//   k_rt_rep_sum        the coarse levels (hot rows) scatter into per-XCD
//                       copies of their rows; this adds the copies in order
//   k_rt_outer          grid_mlp / view_mlp weight gradients dW = sum_s dY[:, s]
//                       X[:, s]^T (split-K, 4 x 4 register tiles, slab rows
//                       summed in a fixed order by k_rt_outer_sum)
//   k_rt_rgb_loss_grad, k_rt_loss   the one-call step's MSE / entropy terms and
//                       their upstream gradients; fixed-order loss means
// Arithmetic is fp32 throughout (the reference's precision); the forward
// repeats the fused render's op order (bins, positions, gathers, compositing),
// so its proposal stages are bit-identical to samnerf_render_forward's.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "raymarch_device.h"
#include "samnerf_common.h"
#include "sh_device.h"
#include "wave_box.h"

using namespace samnerf;

namespace {

constexpr int kT = 32;                                    // final samples per ray
constexpr int kG0 = 64 * 32, kG1 = 64 * 64, kG2 = 16 * 64; // grid_mlp [64,32] [64,64] [16,64]
constexpr int kGW = kG0 + kG1 + kG2;

// torch.linspace(start, end, steps) on the CPU (samnerf_linspace_host; the
// same formula as raymarch.hip's stage-0 bins)
struct LinSpace {
    float start, end, step;
    uint32_t steps;
    __device__ __forceinline__ float operator()(int j) const {
        return (uint32_t)j < steps / 2u ? __builtin_fmaf(step, (float)j, start)
                                        : __builtin_fmaf(-step, (float)(steps - 1u - j), end);
    }
};

LinSpace make_linspace(float start, float end, uint32_t steps) {
    LinSpace l;
    l.start = start;
    l.end = end;
    l.steps = steps;
    l.step = steps > 1 ? (end - start) / (float)(steps - 1u) : 0.0f;
    return l;
}

struct RtArgs {
    const float* rays_o;
    const float* rays_d;
    uint32_t N;
    float bound, b2, inv_b2;
    float bg;
    GridDesc<16> grid;
    const float* G[3];        // grid_mlp
    const float* V[3];        // view_mlp
    const float* snf;         // [2][N]
    const float* bins2;       // [33][N]
    // upstream gradients of the render's outputs (the backward's inputs):
    const float* g_img;       // [N][3] d loss / d image
    const float* g_ws;        // [N] d loss / d weights_sum, or null
    const float* g_depth;     // [N] d loss / d depth, or null
    const float* g_w;         // [N][32] d loss / d weights (results['weights']), or null
    const float* g_loss;      // [2] d loss / d (proposal_loss, distort_loss) (device), or null
    float inv_n;              // 1 / N
    // per final sample s = 32 r + k (ray-major): [channel][S], S = 32 N
    float* pos;               // [3] grid-space u
    float* feat;              // [32] grid features
    float* h1;                // [64] relu(G0 feat)
    float* h2;                // [64] relu(G1 h1)
    float* out;               // [16] G2 h2: sigma pre-activation, geo_feat
    float* delta;             // [1] real_bins[k+1] - real_bins[k]
    float* tmid;              // [1] rays_t
    float* dout;              // [16]
    float* dh1;               // [64]
    float* dh2;               // [64]
    // per ray: [channel][N]
    float* w;                 // [32] final weights
    float* fimg;              // [31] f_image
    float* v1;                // [32] view_mlp hidden
    float* v2;                // [32]
    float* sig;               // [3] sigmoid(view_mlp)
    float* dz;                // [3]
    float* dv1;               // [32]
    float* dv2;               // [32]
    float* terms;             // [4]: mse (sum of 3), proposal, distortion, entropy
    float* image;             // [N][3]
    float* depth;             // [N]
    float* wsum;              // [N]
    float* weights;           // [N][32] the final weights as results['weights'] (renderer.py:350), or null
    float* grad_grid;         // [rows][2]
    float* grad_rep;          // [kRep][rep_floats]: the coarse levels' gradient, one copy per XCD
    uint32_t rep_levels, rep_floats;
};

__device__ __forceinline__ float grid_u(const RtArgs& a, float x) {
    return a.inv_b2 != 0.0f ? (x + a.bound) * a.inv_b2 : (x + a.bound) / a.b2;
}

__device__ __forceinline__ void load_grid_mlp(const RtArgs& a, float* sw) {
    for (int i = threadIdx.x; i < kG0; i += blockDim.x) sw[i] = a.G[0][i];
    for (int i = threadIdx.x; i < kG1; i += blockDim.x) sw[kG0 + i] = a.G[1][i];
    for (int i = threadIdx.x; i < kG2; i += blockDim.x) sw[kG0 + kG1 + i] = a.G[2][i];
    __syncthreads();
}

// Sum over the 64 lanes in a fixed order (DPP within rows of 16, then the row
// broadcasts), as wave_box.h's reductions: wave-uniform result.
__device__ __forceinline__ float wave_sum(float v) {
    v += dpp_f<0xB1>(v);                                   // quad_perm [1,0,3,2]
    v += dpp_f<0x4E>(v);                                   // quad_perm [2,3,0,1]
    v += dpp_f<0x141>(v);                                  // row_half_mirror
    v += dpp_f<0x140>(v);                                  // row_mirror: row totals
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xa, 0xf, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x143, 0xc, 0xf, false));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// Scatter one sample's d(features) of a C = 2 level into the gradient table
// (kernel_grid_backward's atomics, gridencoder.cu:252-349).  Float atomics
// execute at the memory side, priced per 64-B request (MI355X_MICROARCH.md
// "Global float atomics": 64 lanes in 64 rows is ~17x slower than 256
// contiguous bytes), so the per-sample kernels run ray-major -- a wave is 64
// consecutive samples of two rays, neighbours in space -- and the adds are
// shaped before they leave:
//  (1) runs of equal rows in consecutive lanes (consecutive samples of a ray
//      often share cells) are summed by a segmented scan and the run's last
//      lane adds the sum;
//  (2) the corners c and c + 1 (x and x + 1) sit in one 64-B segment 7 times in
//      8 on dense AND hashed levels (x ^ (x + 1) only flips low bits), so a quad
//      of lanes emits one sample's corner pair -- both channels of both rows,
//      16 bytes, one request -- through a per-wave LDS transpose, instead of one
//      channel of 64 rows per instruction.
// Every lane of the wave must call it (live = false past the end); `stage` is
// the wave's 384-float LDS slice.
__device__ __forceinline__ void scatter_level_c2(float* __restrict__ gtab, const LevelDesc& d, float ux,
                                                 float uy, float uz, float g0, float g1, bool live,
                                                 float* stage) {
    // a wave whose samples all carry a zero gradient adds nothing (samples
    // behind the last weighted one, whole rays outside the scene)
    if (!__any(live && (g0 != 0.0f || g1 != 0.0f))) return;
    uint32_t off[8];
    float cw[8];
    corner_rows<2>(d, ux, uy, uz, off, cw);
    const uint32_t lane = threadIdx.x & 63u, j = lane & 3u, quad = lane & ~3u;
    float4* sv = reinterpret_cast<float4*>(stage);             // [lane] 4 values
    uint2* so = reinterpret_cast<uint2*>(stage + 256);         // [lane] 2 row offsets
    constexpr uint32_t kDead = 0xFFFFFFFFu;
#pragma unroll
    for (int c = 0; c < 8; c += 2) {
        float v[4];
        uint32_t o[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            o[h] = off[c + h];
            float v0 = cw[c + h] * g0, v1 = cw[c + h] * g1;
            // runs of equal rows in consecutive lanes (samples along a ray)
            // summed by a segmented scan; the run's last lane keeps the sum
            const uint32_t po = __shfl_up(o[h], 1);
            const bool pl = __shfl_up((int)live, 1) != 0;
            bool seg = lane == 0u || !live || !pl || po != o[h];   // run head
            const bool head = seg;
#pragma unroll
            for (uint32_t sd = 1; sd < 64u; sd <<= 1) {
                const float a0 = __shfl_up(v0, sd), a1 = __shfl_up(v1, sd);
                const bool af = __shfl_up((int)seg, sd) != 0;
                if (lane >= sd && !seg) {
                    v0 += a0;
                    v1 += a1;
                    seg = af;
                }
            }
            const bool next_head = __shfl_down((int)head, 1) != 0;
            const bool alive = live && (lane == 63u || next_head);
            v[2 * h] = v0;
            v[2 * h + 1] = v1;
            if (!alive) o[h] = kDead;
        }
        sv[lane] = make_float4(v[0], v[1], v[2], v[3]);
        so[lane] = make_uint2(o[0], o[1]);
        wave_lds_sync();
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const uint32_t src = quad | q;
            const float val = stage[src * 4u + j];
            const uint32_t oo = reinterpret_cast<const uint32_t*>(so)[src * 2u + (j >> 1)];
            if (oo != kDead) atomicAdd(gtab + (oo >> 2) + (j & 1u), val);
        }
        wave_lds_sync();
    }
}

// The coarse levels' rows are hot: every ray crosses them, so their adds
// queue at the memory side on a few addresses (skipping the scatter of final
// levels 0-1 saves 190 us of k_rt_final_bwd's 1.2 ms for 6 % of its atomic
// requests; proposal level 0, 100 us per stage for 7 %;
// tools/r2/gpu_r2s4b.sh).  Those levels scatter into kRep copies of their
// rows instead, the copy picked by the block's XCD (blocks are dealt to the 8
// XCDs round-robin), and k_rt_rep_sum adds the copies in a fixed order.
#ifndef RT_KREP
#define RT_KREP 8   // diagnostics may build other copy counts (a power of two)
#endif
constexpr uint32_t kRep = RT_KREP, kRepRows = 600000;

__device__ __forceinline__ float* level_table(float* grad, float* rep, uint32_t rep_levels, uint32_t rep_floats,
                                              int l) {
    return (uint32_t)l < rep_levels ? rep + (blockIdx.x & (kRep - 1u)) * rep_floats : grad;
}

// grad[i] = sum_c rep[c][i] for i < n (the coarse rows get no other adds)
__global__ void __launch_bounds__(256) k_rt_rep_sum(const float* __restrict__ rep, uint32_t n,
                                                    float* __restrict__ grad) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    float acc = 0.0f;
#pragma unroll
    for (uint32_t c = 0; c < kRep; ++c) acc += rep[(size_t)c * n + i];
    grad[i] = acc;
}

// ------------------------------------------------------------- forward --

// One thread per final sample, ray-major (s = 32 r + k).
// renderer.py:278-286 (bins -> position -> contract), network.py:221-229
// (grid -> grid_mlp; trunc_exp is applied by the compositing kernel).
// 3 waves per SIMD (168 VGPRs, no spills) instead of the compiler's 186 VGPRs
// and 2: the gathers' latency hides better, 240 -> 216 us per 8K-ray step
// (tools/r2/gpu_r2s4m.sh); 4 waves spill 150 VGPRs.  Builds may override it.
#ifndef RT_FWD_WAVES
#define RT_FWD_WAVES 3
#endif
#ifndef RT_BWD_WAVES   // the same for k_rt_final_bwd
#define RT_BWD_WAVES 0
#endif
__global__ void __launch_bounds__(256)
#if RT_FWD_WAVES
__attribute__((amdgpu_waves_per_eu(RT_FWD_WAVES, RT_FWD_WAVES)))
#endif
k_rt_final_fwd(RtArgs a) {
    __shared__ float sw[kGW];
    load_grid_mlp(a, sw);
    const uint32_t N = a.N;
    const size_t S = (size_t)kT * N, s = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (s >= S) return;
    const uint32_t r = (uint32_t)(s / kT), k = (uint32_t)(s % kT);
    const size_t ks = (size_t)k * N + r;
    float o[3], d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        o[c] = a.rays_o[(size_t)r * 3 + c];
        d[c] = a.rays_d[(size_t)r * 3 + c];
    }
    const float sn = a.snf[r], sf = a.snf[N + r];
    const float rbp = real_bin(sn, sf, a.bins2[ks]), rbn = real_bin(sn, sf, a.bins2[ks + N]);
    const float t = (rbn + rbp) / 2.0f;
    float x = o[0] + d[0] * t, y = o[1] + d[1] * t, z = o[2] + d[2] * t;
    contract3(x, y, z);
    const float ux = grid_u(a, x), uy = grid_u(a, y), uz = grid_u(a, z);
    a.pos[s] = ux;
    a.pos[S + s] = uy;
    a.pos[2 * S + s] = uz;
    a.delta[s] = rbn - rbp;
    a.tmid[s] = t;
    float f[32];
#pragma unroll
    for (int l = 0; l < 16; ++l) lookup_level3<2>(a.grid.emb, a.grid.lv[l], ux, uy, uz, f + 2 * l);
#pragma unroll
    for (int i = 0; i < 32; ++i) a.feat[i * S + s] = f[i];
    float h[64];
#pragma unroll
    for (int q = 0; q < 64; ++q) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 32; ++i) acc = __builtin_fmaf(sw[q * 32 + i], f[i], acc);
        h[q] = fmaxf(acc, 0.0f);
        a.h1[q * S + s] = h[q];
    }
#pragma unroll 4
    for (int q = 0; q < 64; ++q) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 64; ++i) acc = __builtin_fmaf(sw[kG0 + q * 64 + i], h[i], acc);
        a.h2[q * S + s] = fmaxf(acc, 0.0f);
    }
    float h2v[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) h2v[i] = a.h2[i * S + s];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 64; ++i) acc = __builtin_fmaf(sw[kG0 + kG1 + q * 64 + i], h2v[i], acc);
        a.out[q * S + s] = acc;
    }
}

// SH(4) of the ray's direction, normalised twice (renderer.py:295 and
// sphere_harmonics.py:79-82), as k_final
__device__ __forceinline__ void ray_sh(const RtArgs& a, uint32_t r, float* sh) {
    float dx = a.rays_d[(size_t)r * 3], dy = a.rays_d[(size_t)r * 3 + 1], dz = a.rays_d[(size_t)r * 3 + 2];
    normalize3(dx, dy, dz);
    normalize3(dx, dy, dz);
    sh_values<4>(dx, dy, dz, sh);
}

// The Trainer's own terms for the one-call step (utils.py:917, 926-929): per
// ray MSE and entropy, and their gradients w.r.t. image and weights_sum -- the
// upstream gradients a torch criterion would hand the render's backward.
__global__ void __launch_bounds__(256) k_rt_rgb_loss_grad(RtArgs a, const float* __restrict__ gt, float c_ent,
                                                          float* __restrict__ g_img, float* __restrict__ g_ws) {
    const uint32_t N = a.N, r = blockIdx.x * 256u + threadIdx.x;
    if (r >= N) return;
    const float c_mse = (float)(2.0 / 3.0) * a.inv_n;
    float mse = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float e = a.image[(size_t)r * 3 + c] - gt[(size_t)r * 3 + c];
        mse = mse + e * e;
        g_img[(size_t)r * 3 + c] = c_mse * e;
    }
    const float ws = a.wsum[r];
    const float we = fminf(fmaxf(ws, 1e-5f), 1.0f - 1e-5f);
    a.terms[r] = mse;
    a.terms[3 * N + r] = -we * log2f(we) - (1.0f - we) * log2f(1.0f - we);
    // clamp(ws, 1e-5, 1 - 1e-5) passes the gradient inside its range
    g_ws[r] = (c_ent != 0.0f && ws >= 1e-5f && ws <= 1.0f - 1e-5f) ? c_ent * (log2f(1.0f - ws) - log2f(ws))
                                                                      : 0.0f;
}

// Half-wave (32-lane) helpers: lane k of a half = sample k of its ray.
template <class V>
__device__ __forceinline__ V half_sum(V v) {
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) v += __shfl_xor(v, m, 32);
    return v;
}
template <class V>
__device__ __forceinline__ V half_incl_scan(V v, uint32_t k) {
#pragma unroll
    for (uint32_t sd = 1; sd < 32u; sd <<= 1) {
        const V o = __shfl_up(v, sd, 32);
        if (k >= sd) v += o;
    }
    return v;
}
template <class V>
__device__ __forceinline__ V half_incl_suffix(V v, uint32_t k) {
#pragma unroll
    for (uint32_t sd = 1; sd < 32u; sd <<= 1) {
        const V o = __shfl_down(v, sd, 32);
        if (k + sd < 32u) v += o;
    }
    return v;
}

// Compositing with one half-wave per ray (8 rays per block; renderer.py:309-358,
// last_sample background, plus the per-ray distortion term): lane k
// composites sample k (the exclusive double cumsum of delta * sigma as a scan,
// as composite_step orders it), the ray's sums are half-wave reductions, and
// the view MLP runs unit-per-lane (v1 / v2 unit q on lane q).  (The first form,
// one thread per ray, ran 128 waves for 8K rays: it and its backward took
// 0.25 ms of the step; these 0.02.)
__global__ void __launch_bounds__(256) k_rt_composite_h(RtArgs a) {
    const uint32_t N = a.N, k = threadIdx.x & 31u;
    const uint32_t r0 = blockIdx.x * 8u + (threadIdx.x >> 5);
    if (r0 >= N) return;                                   // whole half (no barriers below)
    const uint32_t r = r0;
    const size_t S = (size_t)kT * N, s = (size_t)r * kT + k, ks = (size_t)k * N + r;
    const bool last = k == (uint32_t)kT - 1u;
    const float sigma = expf(a.out[s]);                    // trunc_exp forward
    const float ds = last ? INFINITY : a.delta[s] * sigma;
    const double dsd = last ? 0.0 : (double)ds;
    const double cum = half_incl_scan(dsd, k) - dsd;       // before sample k
    const float w = nan_to_num((1.0f - expf(-ds)) * expf(-(float)cum));
    a.w[ks] = w;
    if (a.weights) a.weights[s] = w;
    const double wsd = half_sum((double)w);
    const double dep = half_sum((double)(w * a.tmid[s]));
    float fg[15];
#pragma unroll
    for (int j = 0; j < 15; ++j) fg[j] = half_sum(w * a.out[(size_t)(1 + j) * S + s]);
    // distortion (renderer.py:17-27 via eff_distloss): per sample
    // w_k m_k W_<k - w_k WM_<k, and s_k w_k^2
    const float b0 = a.bins2[ks], b1 = a.bins2[ks + N];
    const float iv = b1 - b0, mid = b0 + iv / 2.0f, wm = w * mid;
    const float Wx = half_incl_scan(w, k) - w, WMx = half_incl_scan(wm, k) - wm;
    const float bi = half_sum(k > 0 ? (wm * Wx - w * WMx) : 0.0f);
    const float uni = half_sum(iv * (w * w));
    const float ws = (float)wsd;
    float sh[16];
    ray_sh(a, r, sh);
    float fi[31];
#pragma unroll
    for (int j = 0; j < 15; ++j) fi[j] = fg[j];
#pragma unroll
    for (int j = 0; j < 16; ++j) fi[15 + j] = sh[j] * ws;
#pragma unroll
    for (int j = 0; j < 31; ++j)
        if (k == (uint32_t)j) a.fimg[(size_t)j * N + r] = fi[j];
    // view MLP, unit q on lane q
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 31; ++i) acc = __builtin_fmaf(a.V[0][k * 31 + i], fi[i], acc);
    const float v1 = fmaxf(acc, 0.0f);
    a.v1[(size_t)k * N + r] = v1;
    acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc = __builtin_fmaf(a.V[1][k * 32 + i], __shfl(v1, i, 32), acc);
    const float v2 = fmaxf(acc, 0.0f);
    a.v2[(size_t)k * N + r] = v2;
    float z[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) z[c] = half_sum(a.V[2][c * 32 + k] * v2);
    if (k < 3u) {
        const float zc = k == 0 ? z[0] : k == 1 ? z[1] : z[2];
        const float sg = sigmoidf(zc);
        a.sig[(size_t)k * N + r] = sg;
        a.image[(size_t)r * 3 + k] = sg + (1.0f - ws) * a.bg;
    }
    if (k == 0) {
        a.depth[r] = (float)dep;
        a.wsum[r] = ws;
        a.terms[N + r] = 0.0f;
        a.terms[2 * N + r] = 2.0f * bi + uni / 3.0f;
    }
}

// The per-ray backward with one half-wave per ray: d(image), d(weights_sum),
// d(depth) -> sigmoid -> the view MLP backward
// unit-per-lane (dv2 / dv1 unit on its lane, d f_image component j on lane j),
// then sample k on lane k: d(loss)/d(w_k), the distortion terms from prefix
// scans, and the compositing reverse scan as a suffix scan.
__global__ void __launch_bounds__(256) k_rt_final_bwd_ray_h(RtArgs a) {
    const uint32_t N = a.N, k = threadIdx.x & 31u;
    const uint32_t r = blockIdx.x * 8u + (threadIdx.x >> 5);
    if (r >= N) return;
    const size_t S = (size_t)kT * N, s = (size_t)r * kT + k, ks = (size_t)k * N + r;
    const bool last = k == (uint32_t)kT - 1u;
    float dimg[3], dz[3], dws = a.g_ws ? a.g_ws[r] : 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        dimg[c] = a.g_img[(size_t)r * 3 + c];
        dws = dws - dimg[c] * a.bg;                         // image += (1 - weights_sum) * bg
        const float sg = a.sig[(size_t)c * N + r];
        dz[c] = dimg[c] * (1.0f - sg) * sg;                 // sigmoid backward
    }
    if (k < 3u) a.dz[(size_t)k * N + r] = k == 0 ? dz[0] : k == 1 ? dz[1] : dz[2];
    const float gdep = a.g_depth ? a.g_depth[r] : 0.0f;     // depth = sum_k w_k t_k
    const float c_dist = a.g_loss ? a.g_loss[1] * a.inv_n : 0.0f;
    // view MLP backward: unit q on lane q (ascending-q sums as the VALU form)
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < 3; ++c) acc = __builtin_fmaf(a.V[2][c * 32 + k], dz[c], acc);
    const float dv2 = a.v2[(size_t)k * N + r] > 0.0f ? acc : 0.0f;
    a.dv2[(size_t)k * N + r] = dv2;
    acc = 0.0f;
#pragma unroll
    for (int q = 0; q < 32; ++q) acc = __builtin_fmaf(a.V[1][q * 32 + k], __shfl(dv2, q, 32), acc);
    const float dv1 = a.v1[(size_t)k * N + r] > 0.0f ? acc : 0.0f;
    a.dv1[(size_t)k * N + r] = dv1;
    acc = 0.0f;
    const uint32_t jj = k < 31u ? k : 30u;
#pragma unroll
    for (int q = 0; q < 32; ++q) acc = __builtin_fmaf(a.V[0][q * 31 + jj], __shfl(dv1, q, 32), acc);
    const float dfi_k = acc;                               // d f_image[k], k < 31
    float dfi[31];
#pragma unroll
    for (int j = 0; j < 31; ++j) dfi[j] = __shfl(dfi_k, j, 32);
    float sh[16];
    ray_sh(a, r, sh);
    float g = dws;
#pragma unroll
    for (int j = 0; j < 16; ++j) g = __builtin_fmaf(dfi[15 + j], sh[j], g);   // d f_image[15:] / d w_k = sh
    // this sample: forward again, d(loss)/d(w_k)
    const float ds = last ? INFINITY : a.delta[s] * expf(a.out[s]);
    const double dsd = last ? 0.0 : (double)ds;
    const double cum = half_incl_scan(dsd, k) - dsd;
    const float e = expf(-ds), Tk = expf(-(float)cum);
    const float raw = (1.0f - e) * Tk;
    const float w = nan_to_num(raw);
    g = __builtin_fmaf(gdep, a.tmid[s], g);
#pragma unroll
    for (int j = 0; j < 15; ++j) {
        const size_t q = (size_t)(1 + j) * S + s;
        g = __builtin_fmaf(dfi[j], a.out[q], g);
        a.dout[q] = w * dfi[j];
    }
    if (c_dist != 0.0f) {
        // d/dw_k [2 sum_i sum_{j<i} w_i w_j (m_i - m_j) + 1/3 sum_i s_i w_i^2]
        // = 2 (m_k W_<k - WM_<k + WM_>k - m_k W_>k) + 2/3 s_k w_k: the partial
        // sums in double (the torch form sums its cumsums in double on the
        // CPU), and the differences of those nearly equal terms too
        const float b0 = a.bins2[ks], b1 = a.bins2[ks + N], iv = b1 - b0, m = b0 + iv / 2.0f, wm = w * m;
        const double wd = (double)w, wmd = (double)wm, md = (double)m;
        const double Wi = half_incl_scan(wd, k), WMi = half_incl_scan(wmd, k);
        const double Wt = __shfl(Wi, 31, 32), WMt = __shfl(WMi, 31, 32);
        const double before = md * (Wi - wd) - (WMi - wmd);
        const double after = (WMt - WMi) - md * (Wt - Wi);
        g = __builtin_fmaf(c_dist, (float)(2.0 * (before + after)) + (2.0f / 3.0f) * iv * w, g);
    }
    if (a.g_w) g = g + a.g_w[(size_t)r * kT + k];          // a loss on results['weights'] itself
    const bool fin = isfinite(raw);                        // nan_to_num_ backward
    const float dw = fin ? g : 0.0f;
    // sum_{j>k} dw_j raw_j: the exclusive suffix sum in double (ATen sums the
    // backward of the compositing cumsum in double on the CPU; in fp32, with
    // the inclusive sum minus the own term, the cancellation below lost ~1e-2
    // of the density gradients against a float64 twin)
    const double drd = fin ? (double)(dw * raw) : 0.0;
    const double after_k = half_incl_suffix(drd, k) - drd;
    float dx = 0.0f;
    if (!last) {
        const float dds = (float)((double)(dw * (e * Tk)) - after_k);
        const float x = a.out[s];
        dx = (dds * a.delta[s]) * expf(fminf(fmaxf(x, -15.0f), 15.0f));   // trunc_exp backward
    }
    a.dout[s] = dx;
}

// ------------------------------------------------------------ backward --

// One thread per final sample: grid_mlp backward (ReLU masks from the saved
// activations) and the grid scatter.
__global__ void __launch_bounds__(256)
#if RT_BWD_WAVES
__attribute__((amdgpu_waves_per_eu(RT_BWD_WAVES, RT_BWD_WAVES)))
#endif
k_rt_final_bwd(RtArgs a) {
    __shared__ float sw[kGW];
    __shared__ float sstage[4][384];
    float* stage = sstage[threadIdx.x >> 6];
    load_grid_mlp(a, sw);
    const uint32_t N = a.N;
    const size_t S = (size_t)kT * N, s0 = (size_t)blockIdx.x * 256u + threadIdx.x;
    if ((s0 & ~(size_t)63) >= S) return;                    // whole wave past the end
    const bool live = s0 < S;                               // other lanes stay for the merges
    const size_t s = live ? s0 : S - 1u;
    float dy[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dy[q] = a.dout[q * S + s];
    float g2[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = __builtin_fmaf(sw[kG0 + kG1 + q * 64 + i], dy[q], acc);
        g2[i] = a.h2[i * S + s] > 0.0f ? acc : 0.0f;
        if (live) a.dh2[i * S + s] = g2[i];
    }
    float g1[64];
#ifdef RT_BWD_G1_UNROLL   // diagnostics: g1 in registers (fully unrolled) instead of scratch
#pragma unroll
#else
#pragma unroll 4
#endif
    for (int i = 0; i < 64; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < 64; ++q) acc = __builtin_fmaf(sw[kG0 + q * 64 + i], g2[q], acc);
        g1[i] = a.h1[i * S + s] > 0.0f ? acc : 0.0f;
        if (live) a.dh1[i * S + s] = g1[i];
    }
    const float ux = a.pos[s], uy = a.pos[S + s], uz = a.pos[2 * S + s];
#pragma unroll 1
    for (int l = 0; l < 16; ++l) {
        float df0 = 0.0f, df1 = 0.0f;
#pragma unroll
        for (int q = 0; q < 64; ++q) {
            df0 = __builtin_fmaf(sw[q * 32 + 2 * l], g1[q], df0);
            df1 = __builtin_fmaf(sw[q * 32 + 2 * l + 1], g1[q], df1);
        }
#ifdef RT_DIAG_LMASK   // diagnostics only (tools/diag): scatter a subset of the levels
        if (!((RT_DIAG_LMASK >> l) & 1)) continue;
#endif
        scatter_level_c2(level_table(a.grad_grid, a.grad_rep, a.rep_levels, a.rep_floats, l), a.grid.lv[l], ux,
                         uy, uz, df0, df1, live, stage);
    }
}

// dW[m][n] += sum_{s in chunk} A[i * S + s] * B[j * S + s] for m, n <= 64: a
// block owns the whole m x n output for its chunk of samples (each operand row
// read once), 32-sample LDS tiles stored k-major, a 4 x 4 register tile per
// thread (16 FMAs per 8 LDS reads).  Each block stores its partial m x n sum
// in a slab row and k_rt_outer_sum adds the rows in block order: float
// atomics from every block into the same few KB serialise at the memory side
// (0.2 ms per call measured), and this way the weight gradients are bitwise
// reproducible.
__host__ __device__ constexpr uint32_t outer_chunk(size_t S) {
    // about 1,024 blocks (4 per CU: latency hiding for the dependent loads),
    // chunks of at least 256 samples, a multiple of the 32-sample tile
    return (uint32_t)(((S + 1023) / 1024 + 255) / 256 * 256);
}

template <bool V4>
__global__ void __launch_bounds__(256) k_rt_outer(const float* __restrict__ A, const float* __restrict__ B,
                                                  uint32_t m, uint32_t n, size_t S, uint32_t chunk,
                                                  float* __restrict__ slab) {
    __shared__ float4 As[32][17], Bs[32][17];              // [k][i / 4], one float4 of padding
    const uint32_t tid = threadIdx.x, ti = tid >> 4, tj = tid & 15u;
    const size_t s0 = (size_t)blockIdx.x * chunk;
    const size_t s1 = s0 + chunk < S ? s0 + chunk : S;
    float acc[4][4] = {};
    float* as = reinterpret_cast<float*>(As);
    float* bs = reinterpret_cast<float*>(Bs);
    // 64 rows x 32 samples of each operand per tile, the sample fastest;
    // V4 (S % 4 == 0): one 16-B load per lane and operand covers 4 samples of
    // a row (2 per tile), else 8 scalar loads; the next tile's loads are in
    // flight while this one is multiplied
    constexpr int NL = V4 ? 2 : 8;
    float4 pa[NL], pb[NL];
    auto fetch = [&](size_t sb) {
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            if constexpr (V4) {
                const uint32_t idx = tid + 256u * q, row = idx >> 3, k4 = (idx & 7u) * 4u;
                const size_t sc = sb + k4;
                const bool ok = sc < s1;                    // s1 and sc are multiples of 4
                pa[q] = (row < m && ok) ? *reinterpret_cast<const float4*>(A + (size_t)row * S + sc)
                                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                pb[q] = (row < n && ok) ? *reinterpret_cast<const float4*>(B + (size_t)row * S + sc)
                                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            } else {
                const uint32_t idx = tid + 256u * q, row = idx >> 5, kk = idx & 31u;
                const size_t sc = sb + kk;
                pa[q].x = (row < m && sc < s1) ? A[(size_t)row * S + sc] : 0.0f;
                pb[q].x = (row < n && sc < s1) ? B[(size_t)row * S + sc] : 0.0f;
            }
        }
    };
    fetch(s0);
    for (size_t sb = s0; sb < s1; sb += 32) {
#pragma unroll
        for (int q = 0; q < NL; ++q) {
            if constexpr (V4) {
                const uint32_t idx = tid + 256u * q, row = idx >> 3, k4 = (idx & 7u) * 4u;
                as[(k4 + 0) * 68 + row] = pa[q].x;
                as[(k4 + 1) * 68 + row] = pa[q].y;
                as[(k4 + 2) * 68 + row] = pa[q].z;
                as[(k4 + 3) * 68 + row] = pa[q].w;
                bs[(k4 + 0) * 68 + row] = pb[q].x;
                bs[(k4 + 1) * 68 + row] = pb[q].y;
                bs[(k4 + 2) * 68 + row] = pb[q].z;
                bs[(k4 + 3) * 68 + row] = pb[q].w;
            } else {
                const uint32_t idx = tid + 256u * q, row = idx >> 5, kk = idx & 31u;
                as[kk * 68 + row] = pa[q].x;
                bs[kk * 68 + row] = pb[q].x;
            }
        }
        __syncthreads();
        if (sb + 32 < s1) fetch(sb + 32);
#pragma unroll 8
        for (int k = 0; k < 32; ++k) {
            const float4 x = As[k][ti], y = Bs[k][tj];
            const float xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_fmaf(xa[i], ya[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t oi = ti * 4u + i, oj = tj * 4u + j;
            if (oi < m && oj < n) slab[(size_t)blockIdx.x * m * n + (size_t)oi * n + oj] = acc[i][j];
        }
}

// out[e] = sum over slab rows in a fixed order: 16 outputs x 16 row groups per
// block, the groups combined in order through LDS
__global__ void __launch_bounds__(256) k_rt_outer_sum(const float* __restrict__ slab, uint32_t stride,
                                                      uint32_t off, uint32_t mn, uint32_t blocks,
                                                      float* __restrict__ out) {
    __shared__ float part[16][17];
    const uint32_t tid = threadIdx.x, eo = tid & 15u, g = tid >> 4, e = blockIdx.x * 16u + eo;
    float acc = 0.0f;
    if (e < mn) {
#pragma unroll 8
        for (uint32_t b = g; b < blocks; b += 16u) acc += slab[(size_t)b * stride + off + e];
    }
    part[g][eo] = acc;
    __syncthreads();
    if (g == 0 && e < mn) {
        float t = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += part[q][eo];
        out[e] = t;
    }
}

struct PropBwdArgs {
    const float* rays_o;
    const float* rays_d;
    uint32_t N;
    float bound, b2, inv_b2;
    GridDesc<16> grid;        // prop_encoders[stage]
    const float* P0;          // [16,10]
    const float* P1;          // [1,16]
    const float* snf;
    LinSpace bins0;           // stage 0, perturb off
    const float* pbins0;      // stage 0, perturb on: [N][129]
    const float* bins_in;     // stage 1: [65][N]
    const float* ws;          // [T][N] the stage's weights
    const float* ds;          // [T][N] its delta * sigma
    const float* bins2;       // [33][N] final bins (detached)
    const float* wf;          // [32][N] final weights (detached)
    float c_prop;             // 1 / (32 N): the forward stores the gradient of the unweighted loss
    const float* g_loss;      // [2] upstream gradients (device); [0] scales the proposal backward
    float* dds;               // [T][N]
    float* terms;             // [4][N] (row 1 accumulates the proposal loss)
    // per sample s = T r + k: [channel][T N]
    float* slab;              // [blocks][176] per-block prop_mlp gradient sums
    float* grad_grid;         // [rows][2]
    float* grad_rep;          // as RtArgs
    uint32_t rep_levels, rep_floats;
};

template <int T, bool FIRST>
__device__ __forceinline__ float stage_bin_t(const PropBwdArgs& a, int i, uint32_t r) {
    if constexpr (FIRST) return a.pbins0 ? a.pbins0[(size_t)r * (T + 1) + i] : a.bins0(i);
    else return a.bins_in[(size_t)i * a.N + r];
}

// torch.searchsorted(arr[0..n), v, right=True) by the binary search of ATen's
// kernels (cus_upper_bound): the same index even where arr is not sorted
template <class F>
__device__ __forceinline__ int upper_bound_t(int n, float v, F arr) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        if (!(v < arr(mid))) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Inclusive prefix sum over the 64 lanes (Hillis-Steele, 6 shuffles).
template <class V>
__device__ __forceinline__ V wave_incl_scan(V v, uint32_t lane) {
#pragma unroll
    for (uint32_t sd = 1; sd < 64u; sd <<= 1) {
        const V o = __shfl_up(v, sd);
        if (lane >= sd) v += o;
    }
    return v;
}

// Inclusive suffix sum (lanes >= this one), the same steps downwards.
template <class V>
__device__ __forceinline__ V wave_incl_suffix(V v, uint32_t lane) {
#pragma unroll
    for (uint32_t sd = 1; sd < 64u; sd <<= 1) {
        const V o = __shfl_down(v, sd);
        if (lane + sd < 64u) v += o;
    }
    return v;
}

// loss_interlevel(bins_ref, w_ref, bins, w) of renderer.py:35-49 and its
// gradient w.r.t. the stage weights (w = cw1[hi + 1] - cw1[lo] is a signed
// range sum: a difference array), then the stage's compositing backward (the
// final stage's reverse scan), with one WAVE per ray (4 rays per block): the ray's T weights
// and optical depths spread over the lanes (E = T / 64 consecutive ones each),
// the cumulative sums as wave scans, the 32 final intervals' searchsorted
// pairs on lanes 0-31 with the difference array in LDS (float atomics: the
// order of two adds into one entry is free), the compositing reverse scan as a
// suffix scan.  The first form (one thread per ray) ran 128 waves for 8K rays
// on 1,024 SIMDs, a serial chain each: 0.21 ms for both stages, step 3.67 ->
// 3.57 ms with this one.
template <int T, bool FIRST>
__global__ void __launch_bounds__(256) k_rt_prop_ray_w(PropBwdArgs a) {
    constexpr int E = T / 64;
    __shared__ float Cw[4][T + 2];
    __shared__ float D[4][T + 2];
    const uint32_t N = a.N, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint32_t r = blockIdx.x * 4u + wv;
    if (r >= N) return;                                    // whole wave (no block barrier below)
    float* cw = Cw[wv];
    float* dd = D[wv];
    // cw = [0, cumsum(w1)] (renderer.py:38-39)
    float w1[E], run = 0.0f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        w1[e] = a.ws[(size_t)(lane * E + e) * N + r];
        run += w1[e];
    }
    float pre = wave_incl_scan(run, lane) - run;           // exclusive: before this lane's chunk
#pragma unroll
    for (int e = 0; e < E; ++e) {
        pre += w1[e];
        cw[lane * E + e + 1] = pre;
        dd[lane * E + e] = 0.0f;
    }
    if (lane == 0) {
        cw[0] = 0.0f;
        dd[T] = 0.0f;
    }
    wave_lds_sync();
    // the 32 final intervals (renderer.py:40-49)
    float loss = 0.0f;
    if (lane < (uint32_t)kT) {
        const uint32_t i = lane;
        const float t0lo = a.bins2[(size_t)i * N + r], t0hi = a.bins2[(size_t)(i + 1) * N + r];
        int lo = upper_bound_t(T, t0lo, [&](int q) { return stage_bin_t<T, FIRST>(a, q, r); }) - 1;
        int hi = upper_bound_t(T, t0hi, [&](int q) { return stage_bin_t<T, FIRST>(a, q + 1, r); });
        lo = min(max(lo, 0), T - 1);
        hi = min(max(hi, 0), T - 1);
        const float w = cw[hi + 1] - cw[lo];
        const float w0 = a.wf[(size_t)i * N + r];
        const float x = w0 - w;
        if (x > 0.0f) {
            const float den = w0 + 1e-8f;
            loss = (x * x) / den;
            const float g = -2.0f * x / den * a.c_prop;
            atomicAdd(dd + lo, g);
            atomicAdd(dd + hi + 1, -g);
        }
    }
    loss = wave_sum(loss);
    wave_lds_sync();
    if (lane == 0) a.terms[N + r] += loss / (float)kT;
    // dw1 = prefix of the difference array; the compositing forward again
    // (cum of ds in double, as the forward kernels) and the reverse scan
    float dwl[E], dsl[E], dsum = 0.0f;
    double csum = 0.0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        const int j = lane * E + e;
        dwl[e] = dd[j];
        dsum += dwl[e];
        dsl[e] = j == T - 1 ? INFINITY : a.ds[(size_t)j * N + r];
        csum += j == T - 1 ? 0.0 : (double)dsl[e];
    }
    float dpre = wave_incl_scan(dsum, lane) - dsum;
    double cpre = wave_incl_scan(csum, lane) - csum;
    float raw[E], ev[E], tail = 0.0f;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        dpre += dwl[e];
        const float ds = dsl[e];
        const float ex = expf(-ds), Tj = expf(-(float)cpre);
        cpre += lane * E + e == T - 1 ? 0.0 : (double)ds;
        const float rw = (1.0f - ex) * Tj;
        const float dw = isfinite(rw) ? dpre : 0.0f;
        raw[e] = isfinite(rw) ? dw * rw : 0.0f;
        ev[e] = dw * (ex * Tj);
        tail += raw[e];
    }
    // suffix sums of dw_k raw_k from the far end (the later lanes' chunks,
    // then this chunk backwards): d ds_j = dw_j e^-ds_j T_j - sum_{k>j} dw_k raw_k
    float acc = wave_incl_suffix(tail, lane) - tail;
#pragma unroll
    for (int e = E - 1; e >= 0; --e) {
        const int j = lane * E + e;
        a.dds[(size_t)j * N + r] = j < T - 1 ? ev[e] - acc : 0.0f;
        acc += raw[e];
    }
}

// One thread per proposal sample, ray-major (s = T r + k): the density network of
// the stage (network.py:248-259) re-evaluated, then its backward.
constexpr uint32_t kPropW = 176;            // prop_mlp gradients: [16,10] then [1,16]

template <int T, bool FIRST>
__global__ void __launch_bounds__(256) k_rt_prop_bwd(PropBwdArgs a) {
    __shared__ float sstage[4][384];
    __shared__ float sred[4][kPropW];
    const uint32_t wv = threadIdx.x >> 6;
    float* stage = sstage[wv];
    const uint32_t N = a.N;
    const size_t S = (size_t)T * N, s0 = (size_t)blockIdx.x * 256u + threadIdx.x;
    if ((s0 & ~(size_t)63) >= S) {                          // whole wave past the end
        for (uint32_t i = threadIdx.x & 63u; i < kPropW; i += 64u) sred[wv][i] = 0.0f;
        __syncthreads();
        if (threadIdx.x < kPropW)
            a.slab[(size_t)blockIdx.x * kPropW + threadIdx.x] =
                sred[0][threadIdx.x] + sred[1][threadIdx.x] + sred[2][threadIdx.x] + sred[3][threadIdx.x];
        return;
    }
    const bool live = s0 < S;                               // other lanes stay for the merges
    const size_t s = live ? s0 : S - 1u;                    // ray-major: s = T r + k
    const uint32_t r = (uint32_t)(s / T), k = (uint32_t)(s % T);
    float o[3], d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        o[c] = a.rays_o[(size_t)r * 3 + c];
        d[c] = a.rays_d[(size_t)r * 3 + c];
    }
    const float sn = a.snf[r], sf = a.snf[N + r];
    const float rbp = real_bin(sn, sf, stage_bin_t<T, FIRST>(a, (int)k, r));
    const float rbn = real_bin(sn, sf, stage_bin_t<T, FIRST>(a, (int)k + 1, r));
    const float t = (rbn + rbp) / 2.0f;
    float x = o[0] + d[0] * t, y = o[1] + d[1] * t, z = o[2] + d[2] * t;
    contract3(x, y, z);
    auto gu = [&](float v) { return a.inv_b2 != 0.0f ? (v + a.bound) * a.inv_b2 : (v + a.bound) / a.b2; };
    const float ux = gu(x), uy = gu(y), uz = gu(z);
    float f[10];
#pragma unroll
    for (int l = 0; l < 5; ++l) lookup_level3<2>(a.grid.emb, a.grid.lv[l], ux, uy, uz, f + 2 * l);
    float h[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 10; ++i) acc = __builtin_fmaf(a.P0[q * 10 + i], f[i], acc);
        h[q] = fmaxf(acc, 0.0f);
    }
    float sv = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) sv = __builtin_fmaf(a.P1[i], h[i], sv);
    const float dsig = (a.dds[(size_t)k * N + r] * a.g_loss[0]) * (rbn - rbp);
    const float dx = dsig * expf(fminf(fmaxf(sv, -15.0f), 15.0f));
    float dh[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) dh[q] = h[q] > 0.0f ? a.P1[q] * dx : 0.0f;
    float df[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        float acc = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) acc = __builtin_fmaf(a.P0[q * 10 + i], dh[q], acc);
        df[i] = acc;
    }
#pragma unroll
    for (int l = 0; l < 5; ++l)
#ifdef RT_DIAG_PMASK   // diagnostics only (tools/diag)
        if ((RT_DIAG_PMASK >> l) & 1)
#endif
        scatter_level_c2(level_table(a.grad_grid, a.grad_rep, a.rep_levels, a.rep_floats, l), a.grid.lv[l], ux,
                         uy, uz, df[2 * l], df[2 * l + 1], live, stage);
    // the prop_mlp weight gradients dP0 = sum dh f^T, dP1 = sum dx h^T: wave
    // sums (fixed order), the block's four waves added in order into its slab
    // row (k_rt_outer_sum adds the rows) -- no [16 + 10 + 16 + 1][T N] round trip
    const float lv = live ? 1.0f : 0.0f;
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const float dq = dh[q] * lv;
#pragma unroll
        for (int i = 0; i < 10; ++i) {
            const float v = wave_sum(dq * f[i]);
            if (lane == 0) sred[wv][q * 10 + i] = v;
        }
        const float v = wave_sum((dx * lv) * h[q]);
        if (lane == 0) sred[wv][160 + q] = v;
    }
    __syncthreads();
    if (threadIdx.x < kPropW)
        a.slab[(size_t)blockIdx.x * kPropW + threadIdx.x] =
            sred[0][threadIdx.x] + sred[1][threadIdx.x] + sred[2][threadIdx.x] + sred[3][threadIdx.x];
}

// Means of the per-ray loss terms (fixed-order sums in double): terms rows
// 0..3 = mse (sum of 3 channels), proposal, distortion, entropy.  loss5 (or
// null) = the four means and the total of utils.py:917-931; loss2 (or null) =
// (proposal, distortion), the render's own loss outputs.  nt = rows to reduce.
__global__ void __launch_bounds__(1024) k_rt_loss(const float* terms, uint32_t N, int t0, int nt, float lp,
                                                  float ld, float le, int with_prop, float* loss5, float* loss2) {
    // one block of 1024: every row's strided partial sums in independent
    // chains, then one tree over the rows together (a single block is all
    // there is, so the loads must not wait on each other)
    __shared__ double red[4][1024];
    __shared__ float mean[4];
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    uint32_t r = threadIdx.x;
    for (; r + 3072u < N; r += 4096u) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (t >= nt) break;
            const float* row = terms + (size_t)(t0 + t) * N + r;
            const float v0 = row[0], v1 = row[1024], v2 = row[2048], v3 = row[3072];
            acc[t] += ((double)v0 + (double)v1) + ((double)v2 + (double)v3);
        }
    }
    for (; r < N; r += 1024u)
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (t < nt) acc[t] += (double)terms[(size_t)(t0 + t) * N + r];
#pragma unroll
    for (int t = 0; t < 4; ++t) red[t][threadIdx.x] = acc[t];
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
#pragma unroll
            for (int t = 0; t < 4; ++t) red[t][threadIdx.x] += red[t][threadIdx.x + w];
        __syncthreads();
    }
    if ((int)threadIdx.x < nt) {
        const int t = t0 + (int)threadIdx.x;
        mean[t] = (float)(red[threadIdx.x][0] / (double)N / (t == 0 ? 3.0 : 1.0));
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (loss2) {
        loss2[0] = mean[1];
        loss2[1] = mean[2];
    }
    if (loss5) {
        for (int t = 0; t < 4; ++t) loss5[t] = mean[t];
        float total = mean[0];
        if (with_prop && lp > 0.0f) total = total + lp * mean[1];
        if (ld > 0.0f) total = total + ld * mean[2];
        if (le > 0.0f) total = total + le * mean[3];
        loss5[4] = total;
    }
}

__global__ void k_rt_set2(float* p, float x, float y) {
    p[0] = x;
    p[1] = y;
}

struct RtWorkspace {
    ProposalOut p;
    float* dds0;
    float* dds1;
    float* fin[10];          // pos feat h1 h2 out delta tmid dout dh1 dh2
    float* ray[10];          // w fimg v1 v2 sig dz dv1 dv2 terms, step scratch (g_img 3 | g_ws | g_loss 2)
    float* slab;             // k_rt_outer partial sums
    float* rep;              // kRep copies of the coarse levels' gradient rows
    uint32_t rep_levels[3], rep_floats[3];   // final grid, proposal grids 0 and 1
    size_t bytes;
};

constexpr int kFinCh[10] = {3, 32, 64, 64, 16, 1, 1, 16, 64, 64};
constexpr int kRayCh[10] = {32, 31, 32, 32, 3, 3, 32, 32, 4, 6};

// the leading levels whose rows fit kRepRows (SAMNERF_RT_REP_ROWS overrides it: A/B timing)
uint32_t rep_rows_cap() {
    static const uint32_t cap = [] {
        const char* e = diag_env("SAMNERF_RT_REP_ROWS");
        return e ? (uint32_t)std::strtoul(e, nullptr, 10) : kRepRows;
    }();
    return cap;
}

void rep_span(const int32_t* offsets, int levels, uint32_t& n_levels, uint32_t& floats) {
    n_levels = 0;
    const uint32_t cap = rep_rows_cap();
    while ((int)n_levels < levels && offsets && (uint32_t)offsets[n_levels + 1] <= cap) ++n_levels;
    floats = n_levels ? (uint32_t)offsets[n_levels] * 2u : 0u;
}

RtWorkspace carve_rt(const samnerf_model* m, uint32_t N, void* base) {
    RtWorkspace w{};
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t floats) {
        float* q = base ? reinterpret_cast<float*>(p + off) : nullptr;
        off += (floats * sizeof(float) + 255) & ~(size_t)255;
        return q;
    };
    const size_t n = N;
    w.p.snf = take(2 * n);
    w.p.rec = reinterpret_cast<float4*>(take(8 * n));
    w.p.ds0 = take(128 * n);
    w.p.w0 = take(128 * n);
    w.p.bins1 = take(65 * n);
    w.p.ds1 = take(64 * n);
    w.p.w1 = take(64 * n);
    w.p.bins2 = take(33 * n);
    w.dds0 = take(128 * n);
    w.dds1 = take(64 * n);
    for (int i = 0; i < 10; ++i) w.fin[i] = take((size_t)kFinCh[i] * kT * n);
    for (int i = 0; i < 10; ++i) w.ray[i] = take((size_t)kRayCh[i] * n);
    // the largest slab: grid_mlp.1 (64 x 64) over 32 N samples, or a proposal
    // MLP (16 x 10) over 128 N
    const size_t sf = (size_t)kT * n, sp = (size_t)128 * n;
    const size_t sb = std::max((size_t)div_up(sf, outer_chunk(sf)) * 4096, (size_t)div_up(sp, 256) * kPropW);
    w.slab = take(sb);
    rep_span(m->grid.offsets_host, 16, w.rep_levels[0], w.rep_floats[0]);
    for (int p = 0; p < 2; ++p) rep_span(m->prop[p].offsets_host, 5, w.rep_levels[1 + p], w.rep_floats[1 + p]);
    w.rep = take((size_t)kRep * std::max(w.rep_floats[0], std::max(w.rep_floats[1], w.rep_floats[2])));
    w.bytes = off;
    return w;
}

// out[m][n] = sum_s A[:, s] B[:, s]^T (overwritten); slab >= blocks * m * n floats
void outer(const float* A, const float* B, uint32_t m, uint32_t n, size_t S, float* out, float* slab,
           hipStream_t s) {
    const uint32_t chunk = outer_chunk(S), blocks = div_up(S, chunk);
    if (S % 4 == 0) k_rt_outer<true><<<blocks, 256, 0, s>>>(A, B, m, n, S, chunk, slab);
    else k_rt_outer<false><<<blocks, 256, 0, s>>>(A, B, m, n, S, chunk, slab);
    k_rt_outer_sum<<<div_up(m * n, 16), 256, 0, s>>>(slab, m * n, 0u, m * n, blocks, out);
}


// What forward and backward share: the model's argument blocks over one workspace.
struct RtCall {
    TrainGeometry geo;
    RtArgs a;
    PropBwdArgs pb;
};

int rt_setup(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N, float bg,
             RtWorkspace& w, RtCall& c) {
    if (m->num_steps[0] != 128 || m->num_steps[1] != 64 || m->num_steps[2] != 32)
        return fail(SAMNERF_EINVAL, "rgb_train: built for num_steps = [128, 64, 32]");
    if (m->with_sam || m->with_mask || m->sum_after_mlp)
        return fail(SAMNERF_EINVAL, "rgb_train: RGB models only (no SAM / mask head, no sum_after_mlp; "
                    "renderer.py:348 adds the training losses only then)");
    if ((uint64_t)N * 128u >= (1ull << 31)) return fail(SAMNERF_EINVAL, "rgb_train: too many rays");
    for (int i = 0; i < 3; ++i)
        if (!m->grid_mlp[i] || !m->view_mlp[i]) return fail(SAMNERF_EINVAL, "rgb_train: null MLP weight");
    int rc = train_geometry(m, c.geo);
    if (rc) return rc;
    RtArgs& a = c.a;
    a = RtArgs{};
    a.rays_o = rays_o;
    a.rays_d = rays_d;
    a.N = N;
    a.bound = c.geo.bound;
    a.b2 = c.geo.b2;
    a.inv_b2 = c.geo.inv_b2;
    a.bg = bg;
    a.grid = c.geo.grid;
    for (int i = 0; i < 3; ++i) {
        a.G[i] = m->grid_mlp[i];
        a.V[i] = m->view_mlp[i];
    }
    a.snf = w.p.snf;
    a.bins2 = w.p.bins2;
    a.inv_n = (float)(1.0 / (double)N);
    a.pos = w.fin[0];
    a.feat = w.fin[1];
    a.h1 = w.fin[2];
    a.h2 = w.fin[3];
    a.out = w.fin[4];
    a.delta = w.fin[5];
    a.tmid = w.fin[6];
    a.dout = w.fin[7];
    a.dh1 = w.fin[8];
    a.dh2 = w.fin[9];
    a.w = w.ray[0];
    a.fimg = w.ray[1];
    a.v1 = w.ray[2];
    a.v2 = w.ray[3];
    a.sig = w.ray[4];
    a.dz = w.ray[5];
    a.dv1 = w.ray[6];
    a.dv2 = w.ray[7];
    a.terms = w.ray[8];
    PropBwdArgs& pb = c.pb;
    pb = PropBwdArgs{};
    pb.rays_o = rays_o;
    pb.rays_d = rays_d;
    pb.N = N;
    pb.bound = c.geo.bound;
    pb.b2 = c.geo.b2;
    pb.inv_b2 = c.geo.inv_b2;
    pb.snf = w.p.snf;
    pb.bins0 = make_linspace(0.0f, 1.0f, 129);
    pb.pbins0 = m->perturb[0];
    pb.bins_in = w.p.bins1;
    pb.bins2 = w.p.bins2;
    pb.wf = a.w;
    pb.c_prop = (float)(1.0 / (32.0 * N));
    pb.terms = a.terms;
    pb.slab = w.slab;
    return SAMNERF_OK;
}

void rt_prop_stage(const samnerf_model* m, RtCall& c, const RtWorkspace& w, int stage) {
    PropBwdArgs& pb = c.pb;
    pb.grid = c.geo.prop[stage];
    pb.P0 = m->prop_mlp[stage][0];
    pb.P1 = m->prop_mlp[stage][1];
    pb.ws = stage ? w.p.w1 : w.p.w0;
    pb.ds = stage ? w.p.ds1 : w.p.ds0;
    pb.dds = stage ? w.dds1 : w.dds0;
}

// forward: proposal stages, final samples, compositing; with_prop: the
// proposal loss and its (unit-weight) gradient through the stages' compositing
int rt_forward(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N, const float* cnf,
               uint32_t n_cnf, bool with_prop, float* image, float* depth, float* weights_sum, float* weights,
               RtCall& c, const RtWorkspace& w, hipStream_t s) {
    int rc = proposal_forward(m, c.geo, rays_o, rays_d, N, cnf, n_cnf, w.p, s);
    if (rc) return rc;
    c.a.image = image;
    c.a.depth = depth;
    c.a.wsum = weights_sum;
    c.a.weights = weights;
    k_rt_final_fwd<<<div_up((uint64_t)kT * N, 256), 256, 0, s>>>(c.a);
    k_rt_composite_h<<<div_up(N, 8), 256, 0, s>>>(c.a);
    if (with_prop) {
        rt_prop_stage(m, c, w, 0);
        k_rt_prop_ray_w<128, true><<<div_up(N, 4), 256, 0, s>>>(c.pb);
        rt_prop_stage(m, c, w, 1);
        k_rt_prop_ray_w<64, false><<<div_up(N, 4), 256, 0, s>>>(c.pb);
    }
    return SAMNERF_OK;
}

// backward given the upstream gradients in c.a (g_img, g_ws, g_depth, g_loss)
int rt_backward(const samnerf_model* m, uint32_t N, bool with_prop, const samnerf_rgb_grads* g, RtCall& c,
                const RtWorkspace& w, hipStream_t s) {
    if (!g || !g->grid) return fail(SAMNERF_EINVAL, "rgb_train: null grid gradient");
    for (int i = 0; i < 3; ++i)
        if (!g->grid_mlp[i] || !g->view_mlp[i]) return fail(SAMNERF_EINVAL, "rgb_train: null MLP gradient");
    if (with_prop)
        for (int p = 0; p < 2; ++p)
            if (!g->prop[p] || !g->prop_mlp[p][0] || !g->prop_mlp[p][1])
                return fail(SAMNERF_EINVAL, "rgb_train: null proposal gradient");
    // gradients are overwritten: the grid tables are zero-filled and scattered
    // into (torch accumulates into zeroed .grad), the MLP weights' written whole
    // by k_rt_outer_sum
    auto zero = [&](float* p, size_t floats) { return hipMemsetAsync(p, 0, floats * sizeof(float), s); };
    bool ok = zero(g->grid, (size_t)m->grid.offsets_host[16] * 2) == hipSuccess;
    if (with_prop)
        for (int p = 0; p < 2; ++p)
            ok = ok && zero(g->prop[p], (size_t)m->prop[p].offsets_host[5] * 2) == hipSuccess;
    if (!ok) return fail(SAMNERF_ELAUNCH, "rgb_train: gradient zero-fill failed");
    // the coarse levels through kRep copies (k_rt_rep_sum writes their rows)
    auto rep_scatter = [&](uint32_t levels, uint32_t floats, float*& rep, uint32_t& rl, uint32_t& rf) {
        rep = w.rep;
        rl = levels;
        rf = floats;
        return !floats || zero(w.rep, (size_t)kRep * floats) == hipSuccess;
    };
    auto rep_sum = [&](uint32_t floats, float* grad) {
        if (floats) k_rt_rep_sum<<<div_up(floats, 256), 256, 0, s>>>(w.rep, floats, grad);
    };
    RtArgs& a = c.a;
    a.grad_grid = g->grid;
    if (!rep_scatter(w.rep_levels[0], w.rep_floats[0], a.grad_rep, a.rep_levels, a.rep_floats))
        return fail(SAMNERF_ELAUNCH, "rgb_train: gradient zero-fill failed");
    k_rt_final_bwd_ray_h<<<div_up(N, 8), 256, 0, s>>>(a);
    k_rt_final_bwd<<<div_up((uint64_t)kT * N, 256), 256, 0, s>>>(a);
    rep_sum(w.rep_floats[0], g->grid);
    const size_t S = (size_t)kT * N;
    outer(a.dh1, a.feat, 64, 32, S, g->grid_mlp[0], w.slab, s);
    outer(a.dh2, a.h1, 64, 64, S, g->grid_mlp[1], w.slab, s);
    outer(a.dout, a.h2, 16, 64, S, g->grid_mlp[2], w.slab, s);
    outer(a.dv1, a.fimg, 32, 31, N, g->view_mlp[0], w.slab, s);
    outer(a.dv2, a.v1, 32, 32, N, g->view_mlp[1], w.slab, s);
    outer(a.dz, a.v2, 3, 32, N, g->view_mlp[2], w.slab, s);
    if (with_prop) {                      // proposal_loss only: the bins are detached
        PropBwdArgs& pb = c.pb;
        pb.g_loss = a.g_loss;
        for (int st = 0; st < 2; ++st) {
            rt_prop_stage(m, c, w, st);
            pb.grad_grid = g->prop[st];
            if (!rep_scatter(w.rep_levels[1 + st], w.rep_floats[1 + st], pb.grad_rep, pb.rep_levels, pb.rep_floats))
                return fail(SAMNERF_ELAUNCH, "rgb_train: gradient zero-fill failed");
            const uint32_t T = st ? 64u : 128u;
            const uint32_t blocks = div_up((uint64_t)T * N, 256);
            if (st) k_rt_prop_bwd<64, false><<<blocks, 256, 0, s>>>(pb);
            else k_rt_prop_bwd<128, true><<<blocks, 256, 0, s>>>(pb);
            rep_sum(w.rep_floats[1 + st], g->prop[st]);
            k_rt_outer_sum<<<div_up(160, 16), 256, 0, s>>>(w.slab, kPropW, 0u, 160u, blocks, g->prop_mlp[st][0]);
            k_rt_outer_sum<<<1, 256, 0, s>>>(w.slab, kPropW, 160u, 16u, blocks, g->prop_mlp[st][1]);
        }
    }
    return SAMNERF_OK;
}

bool perturb_ok(const samnerf_model* m) { return !m->perturb[0] == !m->perturb[1] && !m->perturb[0] == !m->perturb[2]; }

}  // namespace

extern "C" {

size_t samnerf_rgb_train_workspace_size(const samnerf_model* model, uint32_t N) {
    if (!model) return 0;
    return carve_rt(model, N, nullptr).bytes;
}

int samnerf_rgb_train_forward(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N,
                              const float* cam_near_far, uint32_t n_cnf, float bg_color, int with_proposal,
                              float* image, float* depth, float* weights_sum, float* weights, float* losses,
                              void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m) return fail(SAMNERF_EINVAL, "rgb_train_forward: null model");
    if (N == 0) return SAMNERF_OK;
    if (!rays_o || !rays_d || !image || !depth || !weights_sum || !losses)
        return fail(SAMNERF_EINVAL, "rgb_train_forward: null pointer");
    if (cam_near_far && n_cnf != 1 && n_cnf != N)
        return fail(SAMNERF_EINVAL, "rgb_train_forward: cam_near_far must have 1 or N rows");
    if (!perturb_ok(m))
        return fail(SAMNERF_EINVAL, "rgb_train_forward: perturb needs all three position arrays or none");
    RtWorkspace w = carve_rt(m, N, workspace);
    if (!workspace || workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "rgb_train_forward: workspace needs %zu bytes, got %zu", w.bytes,
                    workspace_bytes);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    RtCall c;
    int rc = rt_setup(m, rays_o, rays_d, N, bg_color, w, c);
    if (rc) return rc;
    if ((rc = rt_forward(m, rays_o, rays_d, N, cam_near_far, n_cnf, with_proposal != 0, image, depth,
                         weights_sum, weights, c, w, s)))
        return rc;
    k_rt_loss<<<1, 1024, 0, s>>>(c.a.terms, N, 1, 2, 0.0f, 0.0f, 0.0f, 0, nullptr, losses);
    return check_launch("rgb_train_forward");
}

int samnerf_rgb_train_backward(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N,
                               float bg_color, int with_proposal, const float* grad_image,
                               const float* grad_weights_sum, const float* grad_depth, const float* grad_weights,
                               const float* grad_losses, const samnerf_rgb_grads* grads, void* workspace,
                               size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m) return fail(SAMNERF_EINVAL, "rgb_train_backward: null model");
    if (N == 0) return SAMNERF_OK;
    if (!rays_o || !rays_d || !grad_image) return fail(SAMNERF_EINVAL, "rgb_train_backward: null pointer");
    if (with_proposal && !grad_losses)
        return fail(SAMNERF_EINVAL, "rgb_train_backward: the proposal backward needs grad_losses");
    RtWorkspace w = carve_rt(m, N, workspace);
    if (!workspace || workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "rgb_train_backward: workspace needs %zu bytes, got %zu", w.bytes,
                    workspace_bytes);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    RtCall c;
    int rc = rt_setup(m, rays_o, rays_d, N, bg_color, w, c);
    if (rc) return rc;
    c.a.image = nullptr;
    c.a.depth = nullptr;
    c.a.wsum = nullptr;
    c.a.g_img = grad_image;
    c.a.g_ws = grad_weights_sum;
    c.a.g_depth = grad_depth;
    c.a.g_w = grad_weights;
    c.a.g_loss = grad_losses;
    if ((rc = rt_backward(m, N, with_proposal != 0, grads, c, w, s))) return rc;
    return check_launch("rgb_train_backward");
}

int samnerf_rgb_train_step(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N,
                           const float* cam_near_far, uint32_t n_cnf, const float* gt_rgb,
                           const samnerf_rgb_train_opts* opts, float* image, float* depth,
                           float* weights_sum, float* loss, const samnerf_rgb_grads* grads,
                           void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m || !opts || !grads) return fail(SAMNERF_EINVAL, "rgb_train_step: null pointer");
    if (N == 0) return SAMNERF_OK;
    if (!rays_o || !rays_d || !gt_rgb || !image || !depth || !weights_sum || !loss)
        return fail(SAMNERF_EINVAL, "rgb_train_step: null pointer");
    if (cam_near_far && n_cnf != 1 && n_cnf != N)
        return fail(SAMNERF_EINVAL, "rgb_train_step: cam_near_far must have 1 or N rows");
    if (!perturb_ok(m))
        return fail(SAMNERF_EINVAL, "rgb_train_step: perturb needs all three position arrays or none");
    RtWorkspace w = carve_rt(m, N, workspace);
    if (!workspace || workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "rgb_train_step: workspace needs %zu bytes, got %zu", w.bytes,
                    workspace_bytes);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool with_prop = opts->update_proposal && opts->lambda_proposal > 0.0f;
    RtCall c;
    int rc = rt_setup(m, rays_o, rays_d, N, opts->bg_color, w, c);
    if (rc) return rc;
    if ((rc = rt_forward(m, rays_o, rays_d, N, cam_near_far, n_cnf, with_prop, image, depth, weights_sum, nullptr,
                         c, w, s)))
        return rc;
    // the Trainer's loss (utils.py:917-931) and its upstream gradients
    float* g_img = w.ray[9];
    float* g_ws = g_img + 3 * (size_t)N;
    float* g_loss = g_ws + N;
    const float c_ent = opts->lambda_entropy > 0.0f ? (float)(opts->lambda_entropy / (double)N) : 0.0f;
    k_rt_rgb_loss_grad<<<div_up(N, 256), 256, 0, s>>>(c.a, gt_rgb, c_ent, g_img, g_ws);
    k_rt_set2<<<1, 1, 0, s>>>(g_loss, with_prop ? opts->lambda_proposal : 0.0f,
                              opts->lambda_distort > 0.0f ? opts->lambda_distort : 0.0f);
    k_rt_loss<<<1, 1024, 0, s>>>(c.a.terms, N, 0, 4, opts->lambda_proposal, opts->lambda_distort,
                                opts->lambda_entropy, with_prop ? 1 : 0, loss, nullptr);
    c.a.g_img = g_img;
    c.a.g_ws = g_ws;
    c.a.g_depth = nullptr;
    c.a.g_w = nullptr;
    c.a.g_loss = g_loss;
    if ((rc = rt_backward(m, N, with_prop, grads, c, w, s))) return rc;
    return check_launch("rgb_train_step");
}

}  // extern "C"
