// raymarch.hip -- the NeRF ray-march inner loop (nerf/renderer.py:221-390 +
// nerf/network.py:221-259) as fused gfx950 kernels, plus the stand-alone step
// kernels used by the parity tests.
//
// Fused pipeline for N rays (all intermediates stay in one workspace; nothing
// of shape [N, T, C] is ever materialised, unlike the reference's ~350 ATen
// ops per chunk):
//   k_prop_sigma<128>       one thread per (ray, sample): near/far + uniform
//                           bins + prop0 grid/MLP -> ds = delta * sigma
//   k_prop_pdf<128, 65>     per ray: compositing (double cumsum) + torch-
//                           ordered normaliser + cdf (one thread), inverse-CDF
//                           (four threads, quarter merge walks) -> 65 bins
//   k_prop_sigma/pdf<64,33> the same for prop1 -> 33 bins
//   k_final<32>             final samples: hash grid L16C2 + sigma/geo MLP +
//                           SH(4) + compositing + view MLP -> image, depth,
//                           weights_sum, head-input row; keeps (u_k, w_k)
//   k_sgrid<32>             s_grid L16C8 gather, weighted by w_k -> f_sam
//   sam_head (sam_head.hip) SkipConnMLP(163->256 x5) + LayerNorm on MFMA
// Rays are independent and every ray does the same work (fixed 128/64/32
// samples), so no compaction or load balancing is needed; the
// proposal gathers run one thread per sample (enough waves to hide gather
// latency even at the 32K rays of one rank of an 8-GPU view).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "f16x3.h"
#include "raymarch_device.h"
#include "samnerf_common.h"
#include "sh_device.h"
#include "wave_box.h"

using namespace samnerf;

namespace samnerf {
int sam_head_forward(const samnerf_model* m, const float* rows, uint32_t N, float* samvit,
                     float* packed, hipStream_t s, uint32_t ld = 256u, bool pack = true);
size_t sam_head_packed_floats();
int mask_head_forward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                      const float* geo_f, uint32_t N, float* out, RayTiles tiles, float* packed,
                      hipStream_t s);
size_t mask_head_packed_floats();
size_t mask_train_workspace_bytes(uint32_t N);
size_t mask_train_workspace_bytes(int mask_kind, uint32_t N);
int mask_train_forward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                       const float* geo_f, uint32_t N, RayTiles tiles, float* logits, void* ws,
                       size_t ws_bytes, hipStream_t s);
int mask_train_backward(const samnerf_model* m, const GridDesc<16>& grid, const float* u_f, const float* w_f,
                        const float* geo_f, uint32_t N, RayTiles tiles, const float* grad_logits,
                        float* const* grad_w, float* grad_m_grid, void* ws, size_t ws_bytes, hipStream_t s);
int adaptive_train_forward(const samnerf_model* m, const float* X, uint32_t N, float* logits, void* ws,
                           size_t ws_bytes, hipStream_t s);
int adaptive_train_backward(const samnerf_model* m, const float* X, uint32_t N, const float* grad_logits,
                            float* const* grad_w, void* ws, size_t ws_bytes, hipStream_t s);
}  // namespace samnerf

namespace {

constexpr uint32_t kRow = 164;     // head input row: f_sam 128 | f_image 31 | image 3 | depth 1 | pad

// torch.linspace(start, end, steps) element j (CPU float algorithm; see
// samnerf_linspace_host).
struct Lin {
    float start, end, step;
    uint32_t steps;
    __device__ __forceinline__ float operator()(int j) const {
        return (uint32_t)j < steps / 2u ? __builtin_fmaf(step, (float)j, start)
                                        : __builtin_fmaf(-step, (float)(steps - 1u - j), end);
    }
};

Lin make_lin(float start, float end, uint32_t steps) {
    Lin l;
    l.start = start;
    l.end = end;
    l.steps = steps;
    l.step = steps > 1 ? (end - start) / (float)(steps - 1u) : 0.0f;
    return l;
}

// XCD-aware block order.  Blocks are dispatched round-robin over the 8 XCDs
// (block b runs on XCD b % 8), each with its own 4 MB L2.  A launch over n
// ray chunks uses xcd_blocks(n) blocks and block b takes chunk xcd_chunk(b,
// n): XCD x gets the contiguous chunks [x*per, (x+1)*per) -- a band of the
// view -- so the grid cells that neighbouring rays share meet in one L2
// instead of eight.  Chunks >= n are empty.
__host__ __device__ constexpr uint32_t xcd_per(uint32_t n) { return (n + 7u) / 8u; }
__host__ __device__ constexpr uint32_t xcd_blocks(uint32_t n) { return xcd_per(n) * 8u; }
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t b, uint32_t n) {
    return (b & 7u) * xcd_per(n) + (b >> 3);
}

// Grid-space coordinate u = (x + bound) / (2 bound) (grid.py:156) with the
// reference's rounding.  When 2*bound is a power of two the host passes its
// exact reciprocal (inv_b2 != 0) and the division becomes a multiplication
// with the identical result; otherwise it is an IEEE division.
struct GridScale {
    float bound, b2, inv_b2;
    __device__ __forceinline__ float operator()(float x) const {
        return inv_b2 != 0.0f ? (x + bound) * inv_b2 : (x + bound) / b2;
    }
};

GridScale make_grid_scale(float bound) {
    GridScale g;
    g.bound = bound;
    g.b2 = 2.0f * bound;
    int e = 0;
    const float m = std::frexp(g.b2, &e);                 // b2 = m * 2^e, m in [0.5, 1)
    g.inv_b2 = (m == 0.5f && std::isfinite(g.b2)) ? std::ldexp(1.0f, 1 - e) : 0.0f;
    return g;
}

// MLP layer y = W x (torch layout W[out][in]), fma chain in input order.
template <int OUT, int IN, bool RELU>
__device__ __forceinline__ void dense(const float* __restrict__ W, const float* x, float* y) {
#pragma unroll
    for (int o = 0; o < OUT; ++o) {
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < IN; ++i) a = __builtin_fmaf(W[o * IN + i], x[i], a);
        y[o] = RELU ? fmaxf(a, 0.0f) : a;
    }
}

// The same layer with two output units per v_pk_fma_f32 (each lane of it is
// the scalar fma chain of dense(), so the bits are unchanged).
template <int OUT, int IN, bool RELU>
__device__ __forceinline__ void dense_pk(const float* __restrict__ W, const float* x, float* y) {
    static_assert(OUT % 2 == 0, "output pairs");
#pragma unroll
    for (int o = 0; o < OUT; o += 2) {
        f2v a = {0.0f, 0.0f};
#pragma unroll
        for (int i = 0; i < IN; ++i)
            a = __builtin_elementwise_fma(f2v{W[o * IN + i], W[(o + 1) * IN + i]}, f2v{x[i], x[i]}, a);
        y[o] = RELU ? fmaxf(a.x, 0.0f) : a.x;
        y[o + 1] = RELU ? fmaxf(a.y, 0.0f) : a.y;
    }
}

// Levels are issued in groups of GROUP (8 corner loads each) separated by a
// scheduling barrier, bounding the loads in flight (and their VGPRs) per lane.
template <int L, int C, bool REF, int GROUP = 4>
__device__ __forceinline__ void grid_features(const GridDesc<16>& g, float ux, float uy, float uz,
                                              float* feat) {
#pragma unroll
    for (int l = 0; l < L; ++l) {
        if constexpr (REF) lookup_level3_ref<C>(g.emb, g.lv[l], ux, uy, uz, feat + l * C);
        else lookup_level3<C>(g.emb, g.lv[l], ux, uy, uz, feat + l * C);
        if ((l + 1) % GROUP == 0 && l + 1 < L) __builtin_amdgcn_sched_barrier(0);
    }
}

// Gather forms (SAMNERF_LOOKUP, lookup_mode): direct packed / direct per-
// corner reference / de-duplicated box; auto picks per stage.
constexpr int kLookPacked = 0, kLookRef = 1, kLookBox4 = 3;
constexpr int kLookAuto = 4;     // host-side only

struct PropArgs {
    const float* rays_o;
    const float* rays_d;
    const float* cnf;
    uint32_t N, n_cnf;
    RayTiles tiles;        // slot -> ray (rays_o / rays_d / cnf are in ray order)
    float aabb[6];
    float min_near;
    GridScale gs;
    GridDesc<16> grid;
    const float* W0;       // [16, 10]
    const float* W1;       // [1, 16]
    Lin bins0;             // stage 0: linspace(0, 1, T+1)
    Lin u;                 // sample_pdf positions for the next stage
    // perturb=True (samnerf_model.perturb, ray order): the stage-0 bins [N][T+1]
    // and sample_pdf's u [N][TN] as the reference computes them from
    // torch.rand_like; null: linspace (bins0 / u above)
    const float* pbins0;
    const float* pu;
    const float* bins_in;  // [T+1][N] (stages > 0)
    float* snf;            // [2][N] spacing(near), spacing(far)
    // [N][2] slot-ordered ray records {o.xyz, spacing(near)}, {d.xyz,
    // spacing(far)} (k_snf; null: not written).  The proposal sigma kernels
    // read a sample's ray in two coalesced 16-B loads from its slot, instead of
    // mapping slot -> ray (RayTiles) and gathering rays_o / rays_d / snf in
    // four loads of 64-bit addresses: the proposal stages are bound by vector
    // issue and the vector-memory address path.
    float4* rec;
    float* wtmp;           // [T][N]: ds per sample
    float* bins_out;       // [TN][N]
    int32_t* inds_out;     // [TN][N] searchsorted indices, or null (parity taps only)
    float* w_out;          // [T][N] composited weights, or null (parity taps only)
    uint32_t pdf_seq;      // diagnostic build, SAMNERF_PDF_SEQ=1: every ray on the sequential phase A
};

// Bin i of a stage's input for slot r (ray `ray`): stage 0 linspace(0, 1, T+1)
// or its perturbed copy (renderer.py:264-271), later stages the previous
// stage's resampled bins (slot-major workspace).
template <int T, bool FIRST>
__device__ __forceinline__ float stage_bin(const PropArgs& a, int i, uint32_t r, uint32_t ray) {
    if constexpr (FIRST) return a.pbins0 ? a.pbins0[(size_t)ray * (T + 1) + i] : a.bins0(i);
    else return a.bins_in[(size_t)i * a.N + r];
}

// Proposal stage, part 1: one thread per (ray, sample).  A wave is 64
// neighbouring rays at one sample index (their corner gathers share cache
// lines) and a block is 4 consecutive sample indices of those rays.  XCD x
// (blocks b with b % 8 == x) owns a contiguous band of ray groups, all T/4
// sample groups of each, so they share its L2.  Writes ds_k =
// (real_bin_{k+1} - real_bin_k) * trunc_exp(density) (renderer.py:282-300)
// to wtmp[k][r]; the serial part of compositing is in k_prop_pdf.
template <int T>
constexpr uint32_t prop_sigma_blocks(uint32_t N) {
    return xcd_blocks((N + 63u) / 64u) * (T / 4);
}

//
// LOOK = kLookPacked / kLookRef: direct corner gathers (lookup_level3 /
// lookup_level3_ref).  LOOK = kLookBox4: de-duplicated gathers (wave_box.h):
// the 64 positions of a wave span a few cells of each proposal level (the
// padded corner box of a 512^2 view's wave holds at most 64 rows at every
// level), so the wave loads each level's box once (one row per lane) into
// its LDS slice and reads its 40 corners from there: 5 vector-memory
// instructions per sample instead of 40.  Same rows, weights and FMA order:
// identical bits.
constexpr uint32_t kPropBoxSlots = 128;      // rows per level slice (8 B each)

// KD / KH (round 5): the proposal grid's level classes as compile-time
// masks (bit l: level l dense / hashed; the reference's proposal grids,
// network.py:96-104 at the default sizes, are DDDHH and DDHHH), with a
// power-of-two grid scale.  The run-time form (KD = KH = 0) takes each
// level's dense / hashed branch on a uniform flag, and the branches split the
// levels into separate blocks: each level's loads were issued and waited for
// before the next level's (5 memory round trips per sample).  With the
// classes known the 5 levels' 28 loads issue together, then the weighted
// corner sums (gather_issue_c2 / gather_finish_c2, the k_final lookups: the
// same rows, weights and FMA order as lookup_level3, so the same bits).
template <uint32_t KD, uint32_t KH>
__device__ __forceinline__ void prop_lookup_lay(const PropArgs& a, float x, float y, float z, float* feat);

#ifndef SAMNERF_PROP_WAVES
#define SAMNERF_PROP_WAVES 0
#endif
template <int T, bool FIRST, int LOOK, uint32_t KD = 0, uint32_t KH = 0>
__global__ void __launch_bounds__(256)
#if SAMNERF_PROP_WAVES
__attribute__((amdgpu_waves_per_eu(SAMNERF_PROP_WAVES, SAMNERF_PROP_WAVES)))
#endif
k_prop_sigma(PropArgs a) {
    static_assert(T % 4 == 0, "T must be a multiple of 4");
    constexpr uint32_t Q = T / 4;
    const uint32_t b = blockIdx.x, i = b >> 3;
    const uint32_t q = i % Q, g = (b & 7u) * xcd_per((a.N + 63u) / 64u) + i / Q;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t r0 = g * 64u + lane, k = q * 4u + (threadIdx.x >> 6);
    if (g * 64u >= a.N) return;                     // whole wave past the end
    // box form: every lane stays active for the wave reductions (lanes past
    // the end recompute ray N - 1 and store nothing)
    if (LOOK != kLookBox4 && r0 >= a.N) return;
    const bool live = r0 < a.N;
    const uint32_t r = live ? r0 : a.N - 1u;              // slot
    const uint32_t N = a.N;
    // the LAY forms read k_snf's slot-ordered ray record (the ray id is then
    // needed only for perturb's per-ray bins); the others map slot -> ray
    constexpr bool REC = (KD | KH) == 0x1Fu && LOOK == kLookPacked;
    float o[3], d[3], sn, sf;
    if constexpr (REC) {
        const char* rbase = reinterpret_cast<const char*>(a.rec);     // 32-bit offsets: saddr loads
        const float4 ra = *reinterpret_cast<const float4*>(rbase + r * 32u),
                     rb = *reinterpret_cast<const float4*>(rbase + r * 32u + 16u);
        o[0] = ra.x, o[1] = ra.y, o[2] = ra.z, sn = ra.w;
        d[0] = rb.x, d[1] = rb.y, d[2] = rb.z, sf = rb.w;
    } else {
        const uint32_t ray = a.tiles(r);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            o[c] = a.rays_o[(size_t)ray * 3 + c];
            d[c] = a.rays_d[(size_t)ray * 3 + c];
        }
        sn = a.snf[r], sf = a.snf[N + r];                   // k_snf (stage 0) / stage 0 (stage 1)
    }
    // the ray id: only perturb's per-ray bins need it (FIRST)
    const uint32_t pray = (FIRST && a.pbins0) ? a.tiles(r) : 0u;
    const float b0 = stage_bin<T, FIRST>(a, (int)k, r, pray), b1 = stage_bin<T, FIRST>(a, (int)k + 1, r, pray);
    const float rb_prev = real_bin(sn, sf, b0), rb_next = real_bin(sn, sf, b1);
    const float t = (rb_next + rb_prev) / 2.0f;
    float x = o[0] + d[0] * t, y = o[1] + d[1] * t, z = o[2] + d[2] * t;
    contract3(x, y, z);
    float feat[10];
    if constexpr (LOOK == kLookBox4) {
        __shared__ float2 smem[4][5 * kPropBoxSlots];
        float* slice = reinterpret_cast<float*>(smem[threadIdx.x >> 6]);
        const float ux = a.gs(x), uy = a.gs(y), uz = a.gs(z);
        const URange ur = wave_urange(ux, uy, uz);
        const bool ordered = wave_positions_ordered(ux, uy, uz);
        // lane l < 5 sizes level l's box (pbox_lane reads res, fres, ftop)
        const LevelDesc* lv = a.grid.lv;
        LevelDesc mine = lv[0];
#pragma unroll
        for (int l = 1; l < 5; ++l) {
            const bool me = lane == (uint32_t)l;
            mine.res = me ? lv[l].res : mine.res;
            mine.fres = me ? lv[l].fres : mine.fres;
            mine.ftop = me ? lv[l].ftop : mine.ftop;
        }
        uint32_t p0, p1, p2;
        pbox_lane(mine, ur, p0, p1, p2);
        PBox bx[5];
#pragma unroll
        for (int l = 0; l < 5; ++l) bx[l] = pbox_read(p0, p1, p2, l);
        const char* base = reinterpret_cast<const char*>(a.grid.emb);
#pragma unroll
        for (int l = 0; l < 5; ++l)
            if (bx[l].slots <= kPropBoxSlots)
                stage_pbox<2>(base, a.grid.lv[l], bx[l], slice + l * kPropBoxSlots * 2, lane);
        wave_lds_sync();
#pragma unroll
        for (int l = 0; l < 5; ++l) {
            const float* sl = slice + l * kPropBoxSlots * 2;
            if (bx[l].slots > kPropBoxSlots)
                lookup_level3<2>(a.grid.emb, a.grid.lv[l], ux, uy, uz, feat + 2 * l);
            else if (ordered)
                lookup_level3_pbox<2, false>(a.grid.emb, a.grid.lv[l], bx[l], sl, ux, uy, uz, feat + 2 * l);
            else
                lookup_level3_pbox<2, true>(a.grid.emb, a.grid.lv[l], bx[l], sl, ux, uy, uz, feat + 2 * l);
        }
    } else if constexpr ((KD | KH) == 0x1Fu && LOOK == kLookPacked) {
        prop_lookup_lay<KD, KH>(a, x, y, z, feat);
    } else {
        grid_features<5, 2, LOOK == kLookRef>(a.grid, a.gs(x), a.gs(y), a.gs(z), feat);
    }
    float h[16], sv;
    if constexpr (LOOK == kLookRef) dense<16, 10, true>(a.W0, feat, h);
    else dense_pk<16, 10, true>(a.W0, feat, h);
    dense<1, 16, false>(a.W1, h, &sv);
    // the only store, after the weight reads: an earlier store could alias
    // W0/W1 and would demote the uniform weight reads to per-lane vector loads
    if (live) a.wtmp[(size_t)k * N + r] = (rb_next - rb_prev) * expf(sv);          // trunc_exp forward
}

// Stage 0 ray setup, one thread per ray: near/far from the AABB slab test
// (renderer.py:122-139, 229-236) and their spacing (renderer.py:250-253).
__global__ void __launch_bounds__(256) k_snf(PropArgs a) {
    const uint32_t r = blockIdx.x * 256u + threadIdx.x;  // slot
    if (r >= a.N) return;
    const uint32_t ray = a.tiles(r);
    float o[3], d[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        o[c] = a.rays_o[(size_t)ray * 3 + c];
        d[c] = a.rays_d[(size_t)ray * 3 + c];
    }
    float near, far;
    near_far_aabb(o, d, a.aabb, a.min_near, near, far);
    if (a.cnf) {  // renderer.py:234-236
        const uint32_t q = a.n_cnf == 1 ? 0u : ray;
        const float cn = a.cnf[q * 2], cf = a.cnf[q * 2 + 1];
        near = (isnan(near) || isnan(cn)) ? NAN : fmaxf(near, cn);
        far = (isnan(far) || isnan(cf)) ? NAN : fminf(far, cf);
    }
    const float sn = spacing(near), sf = spacing(far);
    a.snf[r] = sn;
    a.snf[a.N + r] = sf;
    if (a.rec) {
        a.rec[2 * (size_t)r] = make_float4(o[0], o[1], o[2], sn);
        a.rec[2 * (size_t)r + 1] = make_float4(d[0], d[1], d[2], sf);
    }
}

// Proposal stage, part 2 (renderer.py:84-119 and 300-307), 64 rays per block.
// Phase A, one thread per ray, in the reference's sequential order: composite
// weights with the double cumulative sum, the torch-ordered pdf normaliser,
// and cdf[i] = min(float(double cumsum of (w + 0.01) / sum), 1), written in
// place over the ray's LDS row.  Phase B, 4 threads per ray: each takes a
// contiguous quarter of the TN outputs, finds its first searchsorted(right)
// position by binary search, and merge-walks its quarter -- the same cdf
// values and the same interpolation as one walk over the whole ray, so the
// indices and bins are identical, with a quarter of the dependent steps.
template <int T, int TN, bool FIRST>
__device__ __forceinline__ void prop_pdf_phases(const PropArgs& a, float* sw, uint32_t r0, uint32_t nr);
#ifndef SAMNERF_PDF_SPLIT
#define SAMNERF_PDF_SPLIT 1                  // phase A split over the block's 4 waves (below)
#endif
#ifndef SAMNERF_PDF_SPLIT_MIN
#define SAMNERF_PDF_SPLIT_MIN 128            // from this many samples per ray
#endif

template <int T, int TN, bool FIRST>
__global__ void __launch_bounds__(256)
// T = 128: 4 waves per SIMD, the 4 blocks per CU the ds rows' LDS allows
// (the split phase A otherwise takes 146 VGPRs, 3 waves)
__attribute__((amdgpu_waves_per_eu(T >= 128 ? 4 : 1, T >= 128 ? 4 : 8)))
k_prop_pdf(PropArgs a) {
    constexpr int SW = T + 1;                 // T + 1 cdf entries per row (odd stride)
    __shared__ float sw[64 * SW];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, part = tid >> 6;
    const uint32_t r0 = xcd_chunk(blockIdx.x, (a.N + 63u) / 64u) * 64u, N = a.N;
    if (r0 >= N) return;
    const uint32_t nr = min(64u, N - r0);
    float* row = sw + lane * SW;
    // All four waves stage the ds rows (sample-major wtmp, coalesced across
    // the wave): T/4 independent loads per thread in flight at once, instead
    // of one thread per ray loading its whole row in dependent batches.
    // (Staging the input bins of stage > 0 as well doubles the LDS of
    // k_prop_pdf<64> and halves its occupancy: measured slower.  32 rays per
    // block -- twice the resident phase-A waves -- measured no faster: 0.593
    // -> 0.611 ms prop0 at a full view, 0.103 -> 0.101 ms at 32K rays.)
    if (lane < nr) {
        constexpr int TQ = T / 4;
        float v[TQ];
#pragma unroll
        for (int k = 0; k < TQ; ++k) v[k] = a.wtmp[(size_t)(part * TQ + k) * N + r0 + lane];
#pragma unroll
        for (int k = 0; k < TQ; ++k) row[part * TQ + k] = v[k];
    }
    __syncthreads();
    prop_pdf_phases<T, TN, FIRST>(a, sw, r0, nr);
}

// Exact-sum window of a run of float terms (phase A's double cumulative
// sums): the exponent fields of its non-zero terms and whether any term is
// subnormal, infinite or NaN.  When every term is normal or zero and the
// exponents of the largest and smallest non-zero term differ by at most 22,
// every partial sum of up to 128 of them is a multiple of the smallest
// term's ulp below 2^(e_max + 8), i.e. exactly representable in double
// (53 bits): then each partial sum is the exact real sum, whatever order it
// was formed in, and a prefix taken as (sum of the earlier quarters) + (this
// quarter's terms in order) is bit for bit the sequential prefix.
struct SumWindow {
    uint32_t emin = 0xFFu, emax = 0u, bad = 0u;
    __device__ __forceinline__ void add(float v) {
        const uint32_t e = (__float_as_uint(v) >> 23) & 0xFFu;
        const bool nz = (__float_as_uint(v) & 0x7FFFFFFFu) != 0u;
        bad |= (nz && (e == 0u || e == 0xFFu)) ? 1u : 0u;
        emin = nz ? min(emin, e) : emin;
        emax = nz ? max(emax, e) : emax;
    }
    __device__ __forceinline__ uint32_t pack() const { return bad << 16 | emax << 8 | emin; }
};
__device__ __forceinline__ bool sum_window_exact(const uint32_t* w4) {
    uint32_t emin = 0xFFu, emax = 0u, bad = 0u;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        emin = min(emin, w4[p] & 0xFFu);
        emax = max(emax, (w4[p] >> 8) & 0xFFu);
        bad |= w4[p] >> 16;
    }
    return bad == 0u && (emax < emin || emax - emin <= 22u);
}

// Phases A and B of the proposal pdf over 64 rays whose ds rows sit in LDS
// (row stride T + 1); every thread of the block calls it after a barrier.
//
// Phase A (SAMNERF_PDF_SPLIT, round 6): the four waves of the block take a
// quarter of each ray's samples.  The reference's two serial chains -- the
// double cumulative sum of ds behind the transmittance, and the double
// cumulative sum of the pdf behind the cdf -- are prefix sums: each wave sums
// its quarter in order, the quarter sums meet in LDS, and each wave runs its
// quarter from the sum of the quarters before it.  That is the sequential
// result bit for bit when the ray's terms pass the exact-sum window
// (SumWindow), checked per ray at run time; a ray that does not (ds spanning
// more than 2^22, or non-finite) takes the whole sequential chain in wave 0
// as before.  The pdf terms (w + 0.01) / sum with w in [0, 1] always pass.
// One serial chain of 128 steps per ray, one wave per SIMD at the LDS-bound
// occupancy, was the latency that bounded k_prop_pdf.
template <int T, int TN, bool FIRST>
__device__ __forceinline__ void prop_pdf_phases(const PropArgs& a, float* sw, uint32_t r0, uint32_t nr) {
    constexpr int SW = T + 1;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, part = tid >> 6, N = a.N;
    float* row = sw + lane * SW;
    // stage 0 only: at T = 64 the split's barriers and registers cost more
    // than the 64-step chains it shortens (prop1 0.304-0.308 against
    // 0.299-0.303 ms sequential; prop0 0.552-0.560 against 0.580-0.588)
    constexpr bool kSplit = SAMNERF_PDF_SPLIT && T >= SAMNERF_PDF_SPLIT_MIN;
    if constexpr (kSplit) {
    constexpr int Q = T / 4;
    __shared__ double qsum[4][64];            // per quarter and ray: the quarter's double sum
    __shared__ uint32_t qwin[4][64];          // and its SumWindow
    const bool rl = lane < nr;
    const int k0 = (int)part * Q;
    // A1: ds quarter sums (the last sample's ds is replaced by +inf and the
    // sum after it is never read: not part of the window)
    {
        SumWindow win;
        double q = 0.0;
        if (rl) {
#pragma unroll 8
            for (int k = k0; k < k0 + Q; ++k) {
                if (k == T - 1) break;
                const float ds = row[k];
                win.add(ds);
                q += (double)ds;
            }
        }
        qsum[part][lane] = q;
        qwin[part][lane] = win.pack();
    }
    __syncthreads();
    // A2: composite.  Exact rays: each wave its quarter from the earlier
    // quarters' sum; the others: wave 0 the whole ray, in order.
    if (rl) {
        const uint32_t w4[4] = {qwin[0][lane], qwin[1][lane], qwin[2][lane], qwin[3][lane]};
        if (!a.pdf_seq && sum_window_exact(w4)) {
            double cum = 0.0;
            for (int p = 0; p < (int)part; ++p) cum += qsum[p][lane];
#pragma unroll 8
            for (int k = k0; k < k0 + Q; ++k) row[k] = composite_step(row[k], cum, k == T - 1);
        } else if (part == 0) {
            double cum = 0.0;
#pragma unroll 8
            for (int k = 0; k < T; ++k) row[k] = composite_step(row[k], cum, k == T - 1);
        }
    }
    __syncthreads();
    // A3: the weights out (taps) and the torch-ordered normaliser (each wave
    // for itself, over all T weights), then -- after a barrier, so no wave
    // still reads weights -- each wave replaces its quarter's weights by their
    // pdf (w + 0.01) / sum in place and forms the quarter's double sum
    float wsum = 0.0f;
    if (rl) {
        if (a.w_out)
            for (int k = k0; k < k0 + Q; ++k) a.w_out[(size_t)k * N + r0 + lane] = row[k];
        wsum = torch_row_sum(T, [&](int i) { return row[i] + 0.01f; });
    }
    __syncthreads();
    float pfirst = 0.0f;                      // this quarter's first pdf (A4 reads it from here)
    {
        SumWindow win;
        double q = 0.0;
        if (rl) {
#pragma unroll 8
            for (int k = k0; k < k0 + Q; ++k) {
                const float pdf = (row[k] + 0.01f) / wsum;
                row[k] = pdf;
                win.add(pdf);
                q += (double)pdf;
            }
            pfirst = row[k0];
        }
        qsum[part][lane] = q;
        qwin[part][lane] = win.pack();
    }
    __syncthreads();
    // A4: cdf[i + 1] = min(float(double cumsum of pdf), 1) in place: wave p
    // writes entries k0 + 1 .. k0 + Q, of which only k0 + Q is a pdf another
    // wave reads -- the next wave's first, which it holds in pfirst
    if (rl) {
        const uint32_t w4[4] = {qwin[0][lane], qwin[1][lane], qwin[2][lane], qwin[3][lane]};
        if (!a.pdf_seq && sum_window_exact(w4)) {
            double c = 0.0;
            for (int p = 0; p < (int)part; ++p) c += qsum[p][lane];
            if (part == 0) row[0] = 0.0f;
            float pnext = pfirst;
#pragma unroll 8
            for (int i = 0; i < Q; ++i) {
                const float pi = pnext;
                if (i + 1 < Q) pnext = row[k0 + i + 1];
                c += (double)pi;
                row[k0 + i + 1] = fminf((float)c, 1.0f);
            }
        } else if (part == 0) {
            // not exact (a NaN pdf): wave 0 the whole chain in order, the
            // other waves write nothing of this ray (every pdf is in LDS:
            // no wave wrote a cdf entry of it)
            double c = 0.0;
            float pnext = row[0];
            row[0] = 0.0f;
            for (int i = 0; i < T; ++i) {
                const float pi = pnext;
                if (i + 1 < T) pnext = row[i + 1];
                c += (double)pi;
                row[i + 1] = fminf((float)c, 1.0f);
            }
        }
    }
    } else {
    if (part == 0 && lane < nr) {
        // unrolled by 8: the LDS reads run ahead of the double-precision
        // chains (a full unroll takes 248 VGPRs and halves occupancy)
        double cum = 0.0;
#pragma unroll 8
        for (int k = 0; k < T; ++k) row[k] = composite_step(row[k], cum, k == T - 1);
        if (a.w_out)
            for (int k = 0; k < T; ++k) a.w_out[(size_t)k * N + r0 + lane] = row[k];
        const float wsum = torch_row_sum(T, [&](int i) { return row[i] + 0.01f; });
        double c = 0.0;
        float wnext = row[0];
        row[0] = 0.0f;
#pragma unroll 8
        for (int i = 0; i < T; ++i) {
            const float wi = wnext;
            if (i + 1 < T) wnext = row[i + 1];
            const float pdf = (wi + 0.01f) / wsum;
            c += (double)pdf;
            row[i + 1] = fminf((float)c, 1.0f);
        }
    }
    }
    __syncthreads();
    if (lane >= nr) return;
    const uint32_t r = r0 + lane, ray = a.tiles(r);
    auto bin = [&](int i) -> float { return stage_bin<T, FIRST>(a, i, r, ray); };
    // u_j: linspace, or the perturbed positions (nondecreasing up to rounding:
    // u_j < (j+1)/TN <= u_{j+1} before it, hence the backward step below)
    const float* pu = a.pu ? a.pu + (size_t)ray * TN : nullptr;
    auto uj = [&](int j) -> float { return pu ? pu[j] : a.u(j); };
    constexpr int QN = TN / 4;
    const int j0 = (int)part * QN, j1 = part == 3 ? TN : j0 + QN;
    // first index with cdf > u_j0 (cdf is nondecreasing, cdf[0] = 0 <= u)
    const float u0 = uj(j0);
    int lo = 1, hi = T + 1;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (row[mid] <= u0) lo = mid + 1;
        else hi = mid;
    }
    int i = lo;
    for (int j = j0; j < j1; ++j) {
        const float u = uj(j);
        if (pu)
            while (i > 1 && row[i - 1] > u) --i;
        while (i <= T && row[i] <= u) ++i;
        const int below = i - 1, above = i <= T ? i : T;
        const float g0 = row[below], g1 = row[above];
        const float b0 = bin(below), b1 = bin(above);
        float t = nan_to_num((u - g0) / (g1 - g0));
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        a.bins_out[(size_t)j * N + r] = b0 + t * (b1 - b0);
        if (a.inds_out) a.inds_out[(size_t)j * N + r] = i;    // torch.searchsorted(cdf, u, right=True)
    }
}

// The proposal stage in one kernel (round 2, DESIGN.md 5 "intermediates"): a
// block owns 64 ray slots and all T samples -- wave w evaluates samples w,
// w + 4, .. of its 64 rays (each ray's origin, direction and near/far loaded
// once, not once per sample) and writes ds into the LDS rows k_prop_pdf
// staged from HBM -- then the same pdf phases.  ds ([T][N], 134 MB per 512^2
// view at T = 128) never leaves the CU.  Bit-identical to the two-kernel form
// but 1.9x slower (prop0 1.10 vs 0.59 ms): 33 KB of LDS and 125 VGPRs per
// block leave 4 waves per SIMD instead of k_prop_sigma's 8 to hide the gather
// latency, and the serial pdf phase holds the block's slots while 3 of its 4
// waves wait at the barrier.  A selectable variant (SAMNERF_PROP_FUSED=1).
template <int T, int TN, bool FIRST>
__global__ void __launch_bounds__(256) k_prop_fused(PropArgs a) {
    constexpr int SW = T + 1;
    __shared__ float sw[64 * SW];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, part = tid >> 6;
    const uint32_t r0 = xcd_chunk(blockIdx.x, (a.N + 63u) / 64u) * 64u, N = a.N;
    if (r0 >= N) return;
    const uint32_t nr = min(64u, N - r0);
    if (lane < nr) {
        const uint32_t r = r0 + lane, ray = a.tiles(r);
        float o[3], d[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            o[c] = a.rays_o[(size_t)ray * 3 + c];
            d[c] = a.rays_d[(size_t)ray * 3 + c];
        }
        const float sn = a.snf[r], sf = a.snf[N + r];
        float* row = sw + lane * SW;
#pragma unroll 2
        for (int kk = 0; kk < T / 4; ++kk) {
            const int k = (int)part + 4 * kk;
            const float b0 = stage_bin<T, FIRST>(a, k, r, ray), b1 = stage_bin<T, FIRST>(a, k + 1, r, ray);
            const float rb_prev = real_bin(sn, sf, b0), rb_next = real_bin(sn, sf, b1);
            const float t = (rb_next + rb_prev) / 2.0f;
            float x = o[0] + d[0] * t, y = o[1] + d[1] * t, z = o[2] + d[2] * t;
            contract3(x, y, z);
            float feat[10];
            grid_features<5, 2, false>(a.grid, a.gs(x), a.gs(y), a.gs(z), feat);
            float h[16], sv;
            dense_pk<16, 10, true>(a.W0, feat, h);
            dense<1, 16, false>(a.W1, h, &sv);
            row[k] = (rb_next - rb_prev) * expf(sv);      // trunc_exp forward
        }
    }
    __syncthreads();
    prop_pdf_phases<T, TN, FIRST>(a, sw, r0, nr);
}

struct FinalArgs {
    const float* rays_o;
    const float* rays_d;
    uint32_t N;
    GridScale gs;
    float bg;
    // The main grid's level descriptors by value (kernarg), copied into LDS
    // at kernel start; each half-wave reads its slot's descriptor from there.
    // Round 1 read them from a copy in the workspace (written by a one-thread
    // kernel before each render): the kernel's stores may alias that table,
    // so the compiler could not use the scalar cache, and the per-half-wave
    // select became one 64-lane 16-B load per descriptor -- ~33 extra VMEM
    // instructions per wave and sample competing with the gathers for the
    // texture-address path (profiles/r2b PMC: 90 VMEM reads per wave-sample),
    // and the source of the prefetch nondeterminism.  Kernarg
    // scalar loads + selects in the loop measured slower (1.23 vs 0.92 ms:
    // SGPR-bound reloads, lgkmcnt waits); LDS: 0.82 ms.
    GridDesc<16> grid;
    uint32_t kdense[2], khashed[2];   // wave-uniform slot classes of k-blocks 0 / 1 (host-side)
    // LAY 1's hashed slots (round 6): byte offset of the slot's half-wave-0
    // level (emb + hoff8 is a uniform SGPR base); half-wave 1's level is the
    // next one, hbit = its byte distance 8 S (S = the levels' common power-of-
    // two size, above every masked row bit), hm8 = 8 (S - 1)  (final_layout
    // admits LAY 1 only when every hashed slot is laid out so)
    uint32_t hoff8[2][4];
    uint32_t hbit, hm8;
    const float* grid_emb;  // == grid.emb, as a kernel argument so gathers are global_load (not flat)
    const float* G0;   // grid_mlp [64,32]
    const float* G1;   // [64,64]
    const float* G2;   // [16,64]
    const uint4* gpack;     // f16x3: the grid_mlp fragments [hi / lo][kFSlots][64] (k_pack_grid_mlp)
    const int* gexp;        // f16x3: log2 scale of G0 / G1 / G2's fragments
    const float* V0;   // view_mlp [32,31]
    const float* V1;   // [32,32]
    const float* V2;   // [3,32]
    const float* bins_in;   // [T+1][N]
    const float* snf;       // [2][N]
    float* u_out;      // [T][3][N] grid-space sample positions
    float* w_out;      // [T][N] final weights
    float* image;      // [N,3], row stride img_ld
    float* depth;      // [N], stride scal_ld
    float* wsum;       // [N], stride scal_ld
    uint32_t img_ld, scal_ld;   // 3 / 1, or the gather tile's row (samnerf_render_forward_tile)
    float* rows;       // [N, kRow] or null
    RayTiles tiles;    // slot -> ray: rays_o / rays_d and the per-ray outputs are in ray order
    // N1 (flagged, non-parity; samnerf_model.t_thresh): optical depth
    // -ln(t_thresh) past which a ray is opaque; a wave whose rays all are
    // stops marching.  INFINITY: off (the default, the reference's semantics).
    float exit_depth;
    float* geo_out;    // GEO: [T][16][N] the grid_mlp output rows of every sample (mask head input)
    // AD (adaptive mask heads): the head is linear in the per-sample grid
    // features and MLP intermediates, so sum_k w_k head(x_k) = E . sum_k w_k x_k
    const float* aeff; // [K][240] E, blocks g 32 | h1 64 | h2 64 | o3 16 | v1 32 | v2 32 (k_mask_eff)
    float* mlog;       // [N][K] instance_mask_logits (ray order)
    float* xsum;       // [N][kAeff] the per-ray sums sum_k w_k x_k in E's column order (ray
                       // order), the adaptive head's input for its training (mask_head_train.hip)
    uint32_t mask_out;
    // N1 ray compaction (EXIT form): this pass marches samples [i0, i1) of
    // the slots in list_in (n_in of them, a device count; null: every slot);
    // a ray still open at i1 keeps its running sums in st_d / st_f and sets
    // its bit in its wave's ballot mask (wave_mask, one 64-bit word per
    // wave); k_n1_scan / k_n1_scatter then build the next pass's list in
    // slot order (so a compacted wave's rays stay neighbours in the image).
    // The others finish in this pass (outputs written, later samples
    // zeroed).  Defaults: i0 0, i1 T, no lists.
    int i0, i1;
    const uint32_t* list_in;
    const uint32_t* n_in;
    uint64_t* wave_mask;   // [ceil(N / 32)] (non-null: a non-final pass)
    struct {               // host side: the passes' buffers (workspace, t_thresh > 0)
        uint32_t* list;    // [2][N] slot lists
        uint32_t* cnt;     // [2] their lengths
        uint64_t* mask;    // [ceil(N / 32)] ballot masks
        uint32_t* base;    // [ceil(N / 32)] scan
    } n1;
    double* st_d;      // [3][N] optical depth, sum w, sum w t (slot order)
    float* st_f;       // [16][N] sum w * grid_mlp rows
    // parity taps (samnerf_taps; null in every product render): sigma of
    // every sample [T][N], and the corner rows of every level of the samples
    // of slots r % tap_stride == 0, [N / tap_stride][T][16][8]
    float* sigma_tap;
    uint32_t* rows_tap;
    uint32_t tap_stride;
};

constexpr int kAeff = 240;          // columns of the adaptive heads' effective matrix

// ---- grid_mlp on f16x3 MFMAs (v_mfma_f32_32x32x16_f16, fp32 accumulate).
// Transposed orientation: A = weights (rows = hidden units), B = activations
// (columns = 32 rays), so a layer's accumulator is the next layer's B operand
// as it stands.  Lane (j, h) of a 32x32 accumulator holds rows rho(q) + 4h,
// rho(q) = (q&3) + 8(q>>2); k-block kb of a 64-wide input takes registers
// 8(kb&1)..8(kb&1)+7 of tile kb>>1, and the weights are stored permuted to
// match (hidden_unit).  Each product is split x = hi + lo (fp16 RNE, on
// power-of-two scaled operands) and A.B = A_lo.B_hi + A_hi.B_lo + A_hi.B_hi
// (f16x3.h): fp32-equivalent, at 3 MFMAs of 32 cycles per 16-deep k-block
// instead of 8 fp32 MFMAs of 64.

constexpr int kF1 = 0;               // grid_mlp.0: slot kb*2 + ob      (kb < 2)  W[64,32]
constexpr int kF2 = 4;               // grid_mlp.1: slot 4 + kb*2 + ob  (kb < 4)  W[64,64]
constexpr int kF3 = 12;              // grid_mlp.2: slot 12 + kb        (kb < 4)  W[16,64]
constexpr int kFSlots = 16;          // x 64 lanes x (8 f16 hi + 8 f16 lo)
// view_mlp on v_mfma_f32_32x32x2_f32 (once per ray): [q 16][lane] each
constexpr int kV1 = 0;               // view_mlp.0  q<8: geo acc rows, q>=8: sh pairs
constexpr int kV2 = 1024;            // view_mlp.1  W[32,32]
constexpr int kV3 = 2048;            // view_mlp.2  W[3,32]
constexpr int kVTotal = 3072;

__device__ __forceinline__ int rho(int q) { return (q & 3) + 8 * (q >> 2); }

// input unit of a 64-wide layer fed by accumulator tiles (kb, half h, element m)
__device__ __forceinline__ int hidden_unit(int kb, int h, int m) {
    return (kb >> 1) * 32 + rho(8 * (kb & 1) + m) + 4 * h;
}

// Level gathered by half-wave h in slot q of k-block kb (its B operand of the
// first layer holds that level's two channels at k = 2q, 2q + 1).  Adjacent
// levels share a slot: the dense levels (the coarse ones) then pair up in
// both half-waves, so their slots take gather_issue_c2's uniform dense path.
__host__ __device__ constexpr int final_level(int kb, int h, int q) { return 8 * kb + 2 * q + h; }

__device__ float grid_weight(const FinalArgs& a, int slot, int lane, int m) {
    const int i = lane & 31, h = lane >> 5;
    if (slot < kF2) {                          // input k = 2*level + channel, level = final_level(kb, h, m / 2)
        const int kb = slot >> 1, ob = slot & 1;
        return a.G0[(ob * 32 + i) * 32 + 2 * final_level(kb, h, m >> 1) + (m & 1)];
    }
    if (slot < kF3) {
        const int t = slot - kF2, kb = t >> 1, ob = t & 1;
        return a.G1[(ob * 32 + i) * 64 + hidden_unit(kb, h, m)];
    }
    const int kb = slot - kF3;
    return i < 16 ? a.G2[i * 64 + hidden_unit(kb, h, m)] : 0.0f;
}

__device__ float view_weight(const FinalArgs& a, int idx) {
    const int lane = idx & 63, i = lane & 31, h = lane >> 5;
    if (idx < kV2) {                           // f_image = [geo (units 1..15), sh * wsum]
        const int r = idx >> 6;
        if (r < 8) {
            const int unit = rho(r) + 4 * h;   // grid_mlp output row; unit 0 is sigma
            return unit >= 1 ? a.V0[i * 31 + unit - 1] : 0.0f;
        }
        return a.V0[i * 31 + 15 + 2 * (r - 8) + h];
    }
    if (idx < kV3) {
        const int r = (idx - kV2) >> 6;
        return a.V1[i * 32 + rho(r) + 4 * h];
    }
    const int r = (idx - kV3) >> 6;
    return i < 3 ? a.V2[i * 32 + rho(r) + 4 * h] : 0.0f;
}

// Exact-fp32 grid_mlp (head_mode 1) on v_mfma_f32_32x32x2_f32: one weight
// per lane and k-step, A[i][k = h] for the lane (i, h), 128 k-steps:
//   layer 1  step = ob*16 + kb*8 + m        (m: register of the gathered f[8])
//   layer 2  step = 32 + ob*32 + t*16 + q   (q: register of accumulator tile t)
//   layer 3  step = 96 + t*16 + q
// Each MFMA is the fma chain of its two k terms in k order (exact fp32).
constexpr int kXSteps = 128;

__device__ float grid_weight_exact(const FinalArgs& a, int step, int lane) {
    const int i = lane & 31, h = lane >> 5;
    if (step < 32) {
        const int ob = step >> 4, kb = (step >> 3) & 1, m = step & 7;
        return a.G0[(ob * 32 + i) * 32 + 2 * final_level(kb, h, m >> 1) + (m & 1)];
    }
    if (step < 96) {
        const int s = step - 32, ob = s >> 5, t = (s >> 4) & 1, q = s & 15;
        return a.G1[(ob * 32 + i) * 64 + t * 32 + rho(q) + 4 * h];
    }
    const int s = step - 96, t = s >> 4, q = s & 15;
    return i < 16 ? a.G2[i * 64 + t * 32 + rho(q) + 4 * h] : 0.0f;
}

#define MFMA32(A, B, C) __builtin_amdgcn_mfma_f32_32x32x2f32((A), (B), (C), 0, 0, 0)

// grid_mlp fragments for the f16x3 form (head_mode 0, f16x3.h), once per
// render (one workgroup): each weight tensor scaled by the power of two that
// puts its max |w| in [2^13, 2^14) (scale_exp_of_max), in grid_weight's slot layout, hi then lo;
// gexp[l] = log2 of tensor l's scale.  (A per-tensor scale: the scaled
// accumulators of a sample column then differ from the true values by one
// factor, so each layer's outputs are rescaled straight from their max.)
__global__ void __launch_bounds__(256) k_pack_grid_mlp(FinalArgs a, uint4* gpack, int* gexp) {
    __shared__ float wm[3][4];
    __shared__ int ke[3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float m0 = 0.0f, m1 = 0.0f, m2 = 0.0f;
    // unrolled: the 28 loads per thread issue together (one memory round trip)
#pragma unroll
    for (int i = tid; i < 64 * 32; i += 256) m0 = fmaxf(m0, fabsf(a.G0[i]));
#pragma unroll
    for (int i = tid; i < 64 * 64; i += 256) m1 = fmaxf(m1, fabsf(a.G1[i]));
#pragma unroll
    for (int i = tid; i < 16 * 64; i += 256) m2 = fmaxf(m2, fabsf(a.G2[i]));
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
        const float m = fmaxf(fmaxf(wm[tid][0], wm[tid][1]), fmaxf(wm[tid][2], wm[tid][3]));
        ke[tid] = scale_exp_of_max(m);
        gexp[tid] = ke[tid];
    }
    __syncthreads();
    for (int idx = tid; idx < kFSlots * 64; idx += 256) {
        const int slot = idx >> 6, layer = slot < kF2 ? 0 : slot < kF3 ? 1 : 2;
        float v[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) v[m] = grid_weight(a, slot, idx & 63, m);
        split8_f16(v, exp2i(ke[layer]), gpack[idx], gpack[kFSlots * 64 + idx]);
    }
}

// Trilinear lookup of both channels of NL L16C2 levels whose descriptors
// differ between the half-waves (lane-varying; no divergent branch): the row
// of corner (x, y, z) is x + y*res + z*res^2 (dense) or (x ^ y*P1 ^ z*P2) &
// (size-1) (hashed), built from per-axis terms.  All 8*NL corner loads are
// issued before the first is consumed (one memory round trip per call; the
// compiler otherwise waits for each level before issuing the next).
// Gathered corner rows of NL levels (both channels) and their fractions:
// the issue half of gather_levels_c2, so a caller can start the loads of the
// next sample before consuming them (k_final's cross-iteration prefetch).
template <int NL>
struct GatherC2 {
    float2 e[NL][8];
    float fx[NL], fy[NL], fz[NL];
};

// Wave-uniform classes of the NL level slots of one call: bit l of `dense`
// = the level of slot l is dense in both half-waves, of `hashed` = hashed in
// both.  Such a slot skips the per-lane dense/hash selects, and a dense one
// fetches its x-adjacent corner pairs with one 16-B load each (the rows
// (x, y, z) and (x + 1, y, z) are adjacent).  Mixed slots keep the
// lane-varying form.
struct SlotKinds {
    uint32_t dense, hashed;
};

// Hashed slots of a LAY 1 k-block (k_final, round 6): the table base of each
// slot's half-wave-0 level (uniform), this lane's half-wave bit (0, or the
// byte distance to the next level) and the byte mask.  A corner's byte offset
// from the slot base is then X8 ^ Y8 ^ Z8 with the per-axis terms pre-shifted
// by 3 and pre-masked (AND distributes over XOR) and the half-wave bit folded
// into X8 (it sits above every masked bit): one v_xor_b32 per corner where
// v_bitop3 + v_add_lshl_u32 took 6.6 cycles (profiles/r5v_valu_rate.json).
// Same rows as the reference's (x ^ y P1 ^ z P2) & (S - 1) at offset off.
struct HashSlots {
    const char* base[4];
    uint32_t hx, m8;
};

// tap (parity taps only, samnerf_taps.rows2; null otherwise): the level-
// relative row each corner weight multiplies, tap[l * tap_ls + c] for slot l
// and corner c (bit 0 x, 1 y, 2 z, as gridencoder.cu:61-79 / the oracle's
// corner order) -- the rows the loads below read.  A dense pair's top cell
// reads (top - 1, top) with weights (0, 1), recorded as such.
template <int NL>
__device__ __forceinline__ void gather_issue_c2(const float2* __restrict__ emb, const LevelDesc* d,
                                                float ux, float uy, float uz, GatherC2<NL>& g,
                                                SlotKinds kinds = SlotKinds{0u, 0u},
                                                uint32_t* tap = nullptr, int tap_ls = 8,
                                                const HashSlots* hs = nullptr) {
    // byte offsets of every corner (dense-pair slots: of the 4 pairs) first,
    // then all loads, so they are in flight together
    uint32_t row[NL][8];
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        uint32_t cx, cy, cz;
        locate_axis(ux, d[l], cx, g.fx[l]);
        locate_axis(uy, d[l], cy, g.fy[l]);
        locate_axis(uz, d[l], cz, g.fz[l]);
        const uint32_t top = d[l].res - 1u;
        const uint32_t ny = min(cy + 1u, top), nz = min(cz + 1u, top);
        if ((kinds.dense >> l) & 1u) {
            // pair (cx, cx + 1); in the top cell (cx = top, so fx = 0) the pair
            // (top - 1, top) is loaded and the x weights swapped (fx := 1):
            // corner 0 then adds 0 * row(top - 1), an exact no-op (the running
            // sum is never -0), and corner 1 adds row(top) with corner 0's
            // original weight (1 * wy) * wz -- the same bits as the reference
            const bool edge = cx == top;
            g.fx[l] = edge ? 1.0f : g.fx[l];
            const uint32_t bx = d[l].off + (edge ? cx - 1u : cx);
            const uint32_t r2 = d[l].res * d[l].res;
            const uint32_t Y[2] = {(uint32_t)__umul24(cy, d[l].res), (uint32_t)__umul24(ny, d[l].res)};
            const uint32_t Z[2] = {(uint32_t)__umul24(cz, r2), (uint32_t)__umul24(nz, r2)};
#pragma unroll
            for (int p = 0; p < 4; ++p) row[l][p] = (bx + Y[p & 1] + Z[p >> 1]) << 3;
        } else if (((kinds.hashed >> l) & 1u) && hs) {
            // byte offsets from the slot base hs->base[l] (HashSlots)
            const uint32_t m8 = hs->m8;
            const uint32_t X[2] = {(cx << 3) | hs->hx, ((uint32_t)min(cx + 1u, top) << 3) | hs->hx};
            const uint32_t Y[2] = {(cy * (kPrime1 << 3)) & m8, (ny * (kPrime1 << 3)) & m8};
            const uint32_t Z[2] = {(cz * (kPrime2 << 3)) & m8, (nz * (kPrime2 << 3)) & m8};
#pragma unroll
            for (int c = 0; c < 8; ++c) row[l][c] = X[c & 1] ^ Y[(c >> 1) & 1] ^ Z[c >> 2];
        } else if ((kinds.hashed >> l) & 1u) {
            const uint32_t mask = d[l].size - 1u;
            const uint32_t X[2] = {cx, min(cx + 1u, top)};
            const uint32_t Y[2] = {cy * kPrime1, ny * kPrime1};
            const uint32_t Z[2] = {cz * kPrime2, nz * kPrime2};
#pragma unroll
            for (int c = 0; c < 8; ++c)
                row[l][c] = (d[l].off + ((X[c & 1] ^ Y[(c >> 1) & 1] ^ Z[c >> 2]) & mask)) << 3;
        } else {
            const bool hashed = d[l].flags & kHashed;
            const uint32_t my = hashed ? kPrime1 : d[l].res, mz = hashed ? kPrime2 : d[l].res * d[l].res;
            // per-lane choice between the hashed and the dense row as a bitwise
            // blend on an opaque all-ones / zero mask: written as a select the
            // compiler turned each of the 8 corners into a divergent
            // exec-masked branch pair
            uint32_t hsel = hashed ? 0xffffffffu : 0u;
            asm volatile("" : "+v"(hsel));
            const uint32_t hmask = hsel & (d[l].size - 1u), dmask = ~hsel;
            const uint32_t X[2] = {cx, min(cx + 1u, top)};
            const uint32_t Y[2] = {cy * my, ny * my};
            const uint32_t Z[2] = {cz * mz, nz * mz};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t xs = X[c & 1], ys = Y[(c >> 1) & 1], zs = Z[c >> 2];
                row[l][c] = (d[l].off + (((xs ^ ys ^ zs) & hmask) | ((xs + ys + zs) & dmask))) << 3;
            }
        }
    }
    if (tap) {
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            if ((kinds.dense >> l) & 1u) {
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const uint32_t r0 = (row[l][p] >> 3) - d[l].off;
                    tap[l * tap_ls + 2 * p] = r0;
                    tap[l * tap_ls + 2 * p + 1] = r0 + 1u;
                }
            } else if (((kinds.hashed >> l) & 1u) && hs) {
#pragma unroll
                for (int c = 0; c < 8; ++c) tap[l * tap_ls + c] = (row[l][c] & hs->m8) >> 3;
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) tap[l * tap_ls + c] = (row[l][c] >> 3) - d[l].off;
            }
        }
    }
    // 32-bit byte offsets from the uniform table base (saddr loads)
    const char* base = reinterpret_cast<const char*>(emb);
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        if ((kinds.dense >> l) & 1u) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const f4a8 v = *reinterpret_cast<const f4a8*>(base + row[l][p]);
                g.e[l][2 * p] = make_float2(v.x, v.y);
                g.e[l][2 * p + 1] = make_float2(v.z, v.w);
            }
        } else {
            const char* lb = (((kinds.hashed >> l) & 1u) && hs) ? hs->base[l] : base;
#pragma unroll
            for (int c = 0; c < 8; ++c) g.e[l][c] = *reinterpret_cast<const float2*>(lb + row[l][c]);
        }
    }
}

// Weighted corner sums with the reference's weights (wx * wy) * wz.  PK: both
// channels on one v_pk_fma_f32 per corner (each lane the scalar fma: same
// bits).  The forms schedule differently: PK measured faster in k_final's
// S = 1 form (1.04 -> 1.00 ms per view), scalar in its prefetching S = 2 form
// (0.26 vs 0.29 ms at 32K rays).
template <int NL, bool PK = false>
__device__ __forceinline__ void gather_finish_c2(const GatherC2<NL>& g, float* f) {
#pragma unroll
    for (int l = 0; l < NL; ++l) {
        if constexpr (PK) {
            f2v wc[4];
            corner_weights_pk(g.fx[l], g.fy[l], g.fz[l], wc);
            f2v acc = {0.0f, 0.0f};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float w = corner_w(wc, c);
                acc = __builtin_elementwise_fma(f2v{w, w}, f2v{g.e[l][c].x, g.e[l][c].y}, acc);
            }
            f[2 * l] = acc.x;
            f[2 * l + 1] = acc.y;
        } else {
            f2v wc[4];
            corner_weights_pk(g.fx[l], g.fy[l], g.fz[l], wc);
            float f0 = 0.0f, f1 = 0.0f;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float w = corner_w(wc, c);
                f0 = __builtin_fmaf(w, g.e[l][c].x, f0);
                f1 = __builtin_fmaf(w, g.e[l][c].y, f1);
            }
            f[2 * l] = f0;
            f[2 * l + 1] = f1;
        }
    }
}

// Trilinear lookup of both channels of NL L16C2 levels whose descriptors
// differ between the half-waves (lane-varying; no divergent branch): the row
// of corner (x, y, z) is x + y*res + z*res^2 (dense) or (x ^ y*P1 ^ z*P2) &
// (size-1) (hashed), built from per-axis terms.  All 8*NL corner loads are
// issued before the first is consumed (one memory round trip per call; the
// compiler otherwise waits for each level before issuing the next).
template <int NL, bool PK = false>
__device__ __forceinline__ void gather_levels_c2(const float2* __restrict__ emb, const LevelDesc* d,
                                                 float ux, float uy, float uz, float* f,
                                                 SlotKinds kinds = SlotKinds{0u, 0u},
                                                 uint32_t* tap = nullptr, int tap_ls = 8) {
    GatherC2<NL> g;
    gather_issue_c2<NL>(emb, d, ux, uy, uz, g, kinds, tap, tap_ls);
    gather_finish_c2<NL, PK>(g, f);
}

// k_prop_sigma's lookup with compile-time level classes (KD / KH): the 5
// levels' loads issued together, then the packed corner sums
// PROP_UNI (round 5): a dense level whose cell is the same for all the
// wave's lanes (the coarse proposal levels: 64 neighbouring rays at one
// sample) reads its 4 corner pairs once through the scalar cache instead of
// 4 vector gathers -- the proposal stages are bound by the vector-memory
// address path.  Same rows, weights and FMA order (same bits).
#ifndef SAMNERF_PROP_UNI
#define SAMNERF_PROP_UNI 1
#endif
// PROP_TWO (round 5, late; removed in round 6): a dense level whose lanes sit
// in two cells read both cells' corner pairs through the scalar cache and
// took each lane's by v_cndmask -- bit-identical but slower (prop0 0.575 ->
// 0.62 ms, profiles/r5two_prop_two_cell_ab.txt): the second cell's scalar
// loads add latency the vector path hides.

// Round 6, the same rows, weights and FMA order (same
// bits), fewer VALU cycles per sample:
//  * hashed levels: the table base of the level (emb + 8 off) is a uniform
//    SGPR pair, and the per-axis hash terms are kept pre-shifted and
//    pre-masked in bytes -- X8 = 8 x, Y8 = (y P1 8) & M8, Z8 = (z P2 8) & M8
//    with M8 = 8 (size - 1), since AND distributes over XOR and the shift
//    commutes with both -- so a corner's byte offset 8 ((x ^ y P1 ^ z P2) &
//    (size - 1)) is ONE v_xor_b32 (2.2 cycles per wave64 instruction,
//    profiles/r5v_valu_rate.json) where v_bitop3 + v_add_lshl_u32 took 6.6
//    (the host admits the form only with res <= size, so X8 needs no mask);
//  * uniform dense levels: the corner sums read the scalar-loaded rows as
//    SGPR operands of the packed FMAs in their own branch.  The round-5 form
//    joined them with the vector path's rows before one shared sum, and the
//    join copied 16 SGPRs to VGPRs per level (v_mov_b32 at 4.1 cycles; the
//    compiler also merged the fourth corner pair into a vector load).
#ifndef SAMNERF_PROP_SPLIT
#define SAMNERF_PROP_SPLIT 1
#endif
template <uint32_t KD, uint32_t KH>
__device__ __forceinline__ void prop_lookup_lay(const PropArgs& a, float x, float y, float z, float* feat) {
    const float ux = (x + a.gs.bound) * a.gs.inv_b2, uy = (y + a.gs.bound) * a.gs.inv_b2,
                uz = (z + a.gs.bound) * a.gs.inv_b2;
    if constexpr (!SAMNERF_PROP_UNI) {
        GatherC2<5> g;
        gather_issue_c2<5>(reinterpret_cast<const float2*>(a.grid.emb), a.grid.lv, ux, uy, uz, g,
                           SlotKinds{KD, KH});
        gather_finish_c2<5, true>(g, feat);
        return;
    }
    const char* base = reinterpret_cast<const char*>(a.grid.emb);
    const uint64_t live = __builtin_amdgcn_read_exec();
    float fx[5], fy[5], fz[5];
    uint32_t row[5][8];
    bool uni[5];
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        uni[l] = false;
        if ((KD >> l) & 1u) {
            const LevelDesc& d = a.grid.lv[l];
            uint32_t cx, cy, cz;
            locate_axis(ux, d, cx, fx[l]);
            locate_axis(uy, d, cy, fy[l]);
            locate_axis(uz, d, cz, fz[l]);
            const uint32_t top = d.res - 1u;
            const uint32_t ny = min(cy + 1u, top), nz = min(cz + 1u, top);
            // one cell for every live lane (wave-uniform: a ballot)
            const uint32_t c0 = __builtin_amdgcn_readfirstlane(cx), c1 = __builtin_amdgcn_readfirstlane(cy),
                           c2 = __builtin_amdgcn_readfirstlane(cz);
            const bool same0 = cx == c0 && cy == c1 && cz == c2;
            uni[l] = __builtin_amdgcn_ballot_w64(same0) == live;
            const bool edge = cx == top;                   // gather_issue_c2's top-cell pair
            fx[l] = edge ? 1.0f : fx[l];
            const uint32_t bx = d.off + (edge ? cx - 1u : cx);
            const uint32_t r2 = d.res * d.res;
            const uint32_t Y[2] = {(uint32_t)__umul24(cy, d.res), (uint32_t)__umul24(ny, d.res)};
            const uint32_t Z[2] = {(uint32_t)__umul24(cz, r2), (uint32_t)__umul24(nz, r2)};
#pragma unroll
            for (int p = 0; p < 4; ++p) row[l][p] = (bx + Y[p & 1] + Z[p >> 1]) << 3;
        }
    }
    // Dense levels first: the non-uniform ones' vector loads, then each
    // uniform level's rows by scalar loads and its sum straight from the SGPRs
    // (summed where the vector rows are, the compiler merged the two into one
    // sum of phi'd VGPRs: 8 v_mov_b64 per level), then the vector sums; then
    // the hashed levels' loads and sums.  PROP_SPLIT 0 issues the hashed loads
    // with the dense ones (one memory round trip, 122-126 VGPRs: 4 waves per
    // SIMD instead of 6).
    f4a8 vd[5][4];
    float2 vh[5][8];
    auto issue_hashed = [&]() {
#pragma unroll
        for (int l = 0; l < 5; ++l) {
            if (!((KD >> l) & 1u)) {
                const LevelDesc& d = a.grid.lv[l];
                uint32_t cx, cy, cz;
                locate_axis(ux, d, cx, fx[l]);
                locate_axis(uy, d, cy, fy[l]);
                locate_axis(uz, d, cz, fz[l]);
                const uint32_t top = d.res - 1u;
                const uint32_t ny = min(cy + 1u, top), nz = min(cz + 1u, top);
                const uint32_t m8 = (d.size - 1u) << 3;
                const uint32_t X[2] = {cx << 3, (uint32_t)min(cx + 1u, top) << 3};
                const uint32_t Y[2] = {(cy * (kPrime1 << 3)) & m8, (ny * (kPrime1 << 3)) & m8};
                const uint32_t Z[2] = {(cz * (kPrime2 << 3)) & m8, (nz * (kPrime2 << 3)) & m8};
#pragma unroll
                for (int c = 0; c < 8; ++c) row[l][c] = X[c & 1] ^ Y[(c >> 1) & 1] ^ Z[c >> 2];
                const char* lb = base + (size_t)d.off * 8u;                // uniform: SGPR base
#pragma unroll
                for (int c = 0; c < 8; ++c) vh[l][c] = *reinterpret_cast<const float2*>(lb + row[l][c]);
            }
        }
    };
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        if (((KD >> l) & 1u) && !uni[l]) {
#pragma unroll
            for (int p = 0; p < 4; ++p) vd[l][p] = *reinterpret_cast<const f4a8*>(base + row[l][p]);
        }
    }
    if (!SAMNERF_PROP_SPLIT) issue_hashed();
    // corner pair p of a dense level holds corners 2p (x) and 2p + 1 (x + 1)
    auto dense_sum = [&](int l, const f4a8* v) {
        f2v w[4];
        corner_weights_pk(fx[l], fy[l], fz[l], w);
        f2v acc = {0.0f, 0.0f};
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const float w0 = corner_w(w, 2 * p), w1 = corner_w(w, 2 * p + 1);
            acc = __builtin_elementwise_fma(f2v{w0, w0}, f2v{v[p].x, v[p].y}, acc);
            acc = __builtin_elementwise_fma(f2v{w1, w1}, f2v{v[p].z, v[p].w}, acc);
        }
        return acc;
    };
    f2v fl[5];                 // per level (an array of 10 floats updated in branches became one
                               // phi'd aggregate: v_mov chains at every join)
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        if (((KD >> l) & 1u) && uni[l]) {
            // the scalar cache: wave-uniform rows, through a constant-address-
            // space pointer (the compiler may not turn them into vector loads)
            f4a8 sd[4];
#pragma unroll
            for (int p = 0; p < 4; ++p)
                sd[p] = *(const __attribute__((address_space(4))) f4a8*)(
                    base + (uint32_t)__builtin_amdgcn_readfirstlane(row[l][p]));
            fl[l] = dense_sum(l, sd);
        }
    }
#pragma unroll
    for (int l = 0; l < 5; ++l)
        if (((KD >> l) & 1u) && !uni[l]) fl[l] = dense_sum(l, vd[l]);
    if (SAMNERF_PROP_SPLIT) issue_hashed();
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        if (!((KD >> l) & 1u)) {
            f2v w[4];
            corner_weights_pk(fx[l], fy[l], fz[l], w);
            f2v acc = {0.0f, 0.0f};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float wt = corner_w(w, c);
                acc = __builtin_elementwise_fma(f2v{wt, wt}, f2v{vh[l][c].x, vh[l][c].y}, acc);
            }
            fl[l] = acc;
        }
    }
#pragma unroll
    for (int l = 0; l < 5; ++l) {
        feat[2 * l] = fl[l].x;
        feat[2 * l + 1] = fl[l].y;
    }
}

__device__ __forceinline__ LevelDesc select_level(const LevelDesc& p, const LevelDesc& q, bool hi) {
    return LevelDesc{hi ? q.off : p.off, hi ? q.size : p.size, hi ? q.res : p.res, hi ? q.flags : p.flags,
                     hi ? q.fres : p.fres, hi ? q.ftop : p.ftop};
}

// One wave marches 32 (ray, slot) columns: with S slots per ray, lane (j, h)
// owns slot j / R of ray j % R (R = 32 / S rays per wave), i.e. samples
// slot, slot + S, slot + 2S, ...  For k-block kb it gathers both channels of
// levels final_level(kb, h, 0..3) = 8kb + h, 8kb + 2 + h, .. -- exactly its B
// operand of the first layer (grid_weight permutes the weight columns to
// match) -- so the hash grid feeds the matrix cores
// with no data movement.  grid_mlp 32->64->64->16 runs on f16x3 MFMAs,
// view_mlp 31->32->32->3 (once per ray) on fp32 MFMAs.  Compositing: each
// step the S slots of a ray exchange their optical depths by shuffle and
// every lane forms the ray's exclusive cumulative sum in sample order (the
// reference's sequential double cumsum, exactly), so the stored weights are
// final; per-slot partial sums of w, w*t and w*features are added at the end.
// S > 1 only serves small N (one rank's share of a view): S-times more waves,
// while a wave still gathers at adjacent samples of neighbouring rays.
// Occupancy: the S = 1 form without the cross-sample prefetch runs at 3 waves
// per SIMD (168 VGPRs, 10 spilled): more waves hide the gather latency better
// than the prefetch did at 2 (0.797 vs 0.826 ms per view); the S = 2 / 4 forms
// spill 20+ registers at 3 waves and stay at 2 (0.139 vs 0.158 ms at 32K rays).
#ifndef SAMNERF_DIAG_FINAL_WAVES
#define SAMNERF_DIAG_FINAL_WAVES 3
#endif
#ifndef SAMNERF_FINAL_JOINT
#define SAMNERF_FINAL_JOINT 1
#endif
#ifndef SAMNERF_FINAL_VG
#define SAMNERF_FINAL_VG 0
#endif
template <int S_, bool PLAIN_ = true>
constexpr int final_waves() { return (S_ == 1 && PLAIN_) ? SAMNERF_DIAG_FINAL_WAVES : 2; }

// EXIT: the N1 early-exit form, its own instantiation at 2 waves per SIMD:
// the exit in the sample loop raised the 3-wave form's spills from 10 to 22
// VGPRs (and cost the default kernel 0.80 -> 0.92 ms per view while it was a
// run-time check in the one instantiation)
// GEO: also store every sample's grid_mlp output rows (geo_feat) for the
// mask head (its own instantiation, only for renders of a mask model).
// SA: --sum_after_mlp (renderer.py:339-342): the view MLP runs on every
// sample's colour features, image = sigmoid(sum_k w_k view_mlp(colour_k)).
// AD: the adaptive mask heads (1 'density', 2 'rgb', S = 1 only): per-ray
// weighted sums of the grid features and the grid_mlp (and, SA, view_mlp)
// intermediates, then instance_mask_logits = E . sums (the head is linear).
// The EXIT / GEO / SA forms run at 2 waves per SIMD, the AD forms at 1.
template <int S_, bool PLAIN_, int AD_>
constexpr int final_waves_of() { return AD_ ? 1 : final_waves<S_, PLAIN_>(); }

// LAY: the main grid's level layout as the kernel sees it.
//   0  run time: slot classes from the kernel arguments (kdense / khashed),
//      the grid scale's division / multiplication picked per call;
//   1  the reference architecture's grid (network.py:82-86: L16 C2, 2^19
//      rows per level, base resolution 16 -> levels 0-4 dense, 5-15 hashed)
//      with a power-of-two grid scale: k-block 0's slots are dense, dense,
//      mixed, hashed, k-block 1's all hashed -- compile-time constants, so the
//      sample loop is straight-line code (no per-slot uniform branches for the
//      scheduler to stop at, no per-slot selects) and the grid scale is one
//      multiply.  The host picks 1 when the model's descriptors match
//      (final_layout), else 0; both give the same bits.
// TAP: the parity-tap stores (sigma of every sample, the corner rows) are
// compiled in.  Product renders run TAP = false: the tap address arithmetic
// and its branches are not in their sample loop at all.
constexpr uint32_t kLay1Dense[2] = {0x3u, 0x0u}, kLay1Hashed[2] = {0x8u, 0xFu};

template <int T, int S, bool EXACT, bool EXIT = false, bool GEO = false, bool SA = false, int AD = 0,
          int LAY = 0, bool TAP = true>
__global__ void __launch_bounds__(256)
__attribute__((amdgpu_waves_per_eu(final_waves_of<S, !EXIT && !GEO && !SA, AD>(),
                                   final_waves_of<S, !EXIT && !GEO && !SA, AD>())))
k_final(FinalArgs a) {
    static_assert(AD == 0 || S == 1, "adaptive mask forms: one segment");
    static_assert(AD != 2 || SA, "the 'rgb' adaptive head reads the per-sample view MLP (sum_after_mlp)");
    static_assert(S == 1 || S == 2 || S == 4, "segments per ray");
    static_assert(kXSteps * 64 == 2 * kFSlots * 64 * 4, "exact weights reuse the f16x3 slots");
    constexpr int R = 32 / S, TS = T / S;
    __shared__ uint4 Fbuf[2 * kFSlots * 64];          // f16x3: hi | lo fragments; exact: fp32 steps
    // VG: the view MLP's weights read from global memory (L2) at the end of
    // the ray instead of staged in LDS -- it runs once per ray (not per
    // sample) outside the SA forms, and without its 12 KiB a block's LDS
    // (33 KiB) lets 4 blocks share a CU
    constexpr bool VG = SAMNERF_FINAL_VG && !SA;
    __shared__ float Vl[VG ? 1 : kVTotal];
    __shared__ LevelDesc sLv[16];
    if (threadIdx.x < 16) sLv[threadIdx.x] = a.grid.lv[threadIdx.x];
    uint4* const Fh = Fbuf;
    uint4* const Fl = Fbuf + kFSlots * 64;
    float* const Fx = reinterpret_cast<float*>(Fbuf);
    if constexpr (EXACT) {
        for (int idx = threadIdx.x; idx < kXSteps * 64; idx += 256)
            Fx[idx] = grid_weight_exact(a, idx >> 6, idx & 63);
    } else {
        for (int idx = threadIdx.x; idx < 2 * kFSlots * 64; idx += 256) Fbuf[idx] = a.gpack[idx];
    }
    if constexpr (!VG)
        for (int idx = threadIdx.x; idx < kVTotal; idx += 256) Vl[idx] = view_weight(a, idx);
    auto VW = [&](int idx) { return VG ? view_weight(a, idx) : Vl[idx]; };
    // f16x3: log2 scales of the three weight tensors' fragments
    const int ke0 = EXACT ? 0 : a.gexp[0], ke1 = EXACT ? 0 : a.gexp[1], ke2 = EXACT ? 0 : a.gexp[2];
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int hh = lane >> 5, jj = lane & 31;
    const int seg = jj / R;                              // slot of this column
    const uint32_t chunk = xcd_chunk(blockIdx.x, (a.N + 4u * R - 1u) / (4u * R));
    const uint32_t ray0 = chunk * (4u * R) + wave * (uint32_t)R;
    // EXIT with a list: the wave's columns are list entries ray0 .. (slots)
    const bool listed = EXIT && a.list_in != nullptr;
    const uint32_t n_act = listed ? *a.n_in : a.N;
    if (ray0 >= n_act) return;                           // wave-uniform
    const uint32_t c_idx = ray0 + (uint32_t)(jj % R);
    const bool live = c_idx < n_act;
    const uint32_t rr = listed ? a.list_in[live ? c_idx : n_act - 1] : (live ? c_idx : a.N - 1);
    const uint32_t r = listed ? rr : c_idx;              // this column's slot
    const bool sample_writer = live && hh == 0;          // u_out / w_out of this segment
    const bool writer = sample_writer && seg == 0;       // per-ray outputs
    const uint32_t N = a.N;
    const float2* __restrict__ emb = reinterpret_cast<const float2*>(a.grid_emb);

    float o[3], d[3];
    {
        const uint32_t ray = a.tiles(rr);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            o[c] = a.rays_o[(size_t)ray * 3 + c];
            d[c] = a.rays_d[(size_t)ray * 3 + c];
        }
    }
    const int i_begin = EXIT ? a.i0 : 0, i_end = EXIT ? min(a.i1, TS) : TS;
    const float sn = a.snf[rr], sf = a.snf[N + rr];
    float rb_prev = real_bin(sn, sf, a.bins_in[(size_t)(i_begin * S + seg) * N + rr]);
    double cum = 0.0, wsum = 0.0, depth = 0.0;            // cum: optical depth before this step
    float fg[8];                                          // sum_k w_k * grid_mlp rows (acc layout)
#pragma unroll
    for (int q = 0; q < 8; ++q) fg[q] = 0.0f;
    if (EXIT && i_begin > 0) {                            // N1 compaction: a later pass
        cum = a.st_d[rr];
        wsum = a.st_d[N + rr];
        depth = a.st_d[2 * (size_t)N + rr];
#pragma unroll
        for (int q = 0; q < 8; ++q) fg[q] = a.st_f[(size_t)(q + 8 * hh) * N + rr];
    }
    float sh[16];                                         // SH(4) of the normalised direction
    auto sh_of_ray = [&]() {
        float dx = d[0], dy = d[1], dz = d[2];
        normalize3(dx, dy, dz);
        normalize3(dx, dy, dz);
        sh_values<4>(dx, dy, dz, sh);
    };
    float rgb[3] = {0.0f, 0.0f, 0.0f};                    // SA: sum_k w_k * view_mlp(colour_k)
    if constexpr (SA) sh_of_ray();
    // AD: sum_k w_k x_k of the adaptive heads' inputs, this lane's components
    float gacc[AD ? 16 : 1], h1acc[AD ? 32 : 1], h2acc[AD ? 32 : 1], v1acc[AD == 2 ? 16 : 1],
        v2acc[AD == 2 ? 16 : 1];
    if constexpr (AD > 0) {
#pragma unroll
        for (int q = 0; q < 16; ++q) gacc[q] = 0.0f;
#pragma unroll
        for (int q = 0; q < 32; ++q) h1acc[q] = h2acc[q] = 0.0f;
    }
    if constexpr (AD == 2) {
#pragma unroll
        for (int q = 0; q < 16; ++q) v1acc[q] = v2acc[q] = 0.0f;
    }

    // level descriptors of k-block kb for this half-wave (LDS reads,
    // re-evaluated where used rather than held in VGPRs)
    auto levels = [&](int kb, LevelDesc* dl) {
#pragma unroll
        for (int q = 0; q < 4; ++q) dl[q] = sLv[final_level(kb, hh, q)];
    };
    // wave-uniform slot classes (kernel arguments)
    auto kinds = [&](int kb) {
        if constexpr (LAY == 1) return SlotKinds{kLay1Dense[kb], kLay1Hashed[kb]};
        else return SlotKinds{a.kdense[kb], a.khashed[kb]};
    };
    // grid-space coordinate (LAY 1: the host checked inv_b2 != 0)
    auto gscale = [&](float x) { return LAY == 1 ? (x + a.gs.bound) * a.gs.inv_b2 : a.gs(x); };
    // rb_prev of sample i is rb_next of sample i - 1 when S == 1 (same bits;
    // saves a division), recomputed from the bins otherwise
    // the sample's position from its two raw bins (b0 read only when S > 1:
    // for S == 1 rbp is the previous sample's rbn, or the pre-loop rb_prev)
    auto position_of = [&](int i, float b0, float b1, float& rbp, float& rbn, float& ux, float& uy,
                           float& uz) {
        const int k = i * S + seg;
        if (S > 1) rbp = real_bin(sn, sf, b0);
        rbn = real_bin(sn, sf, b1);
        const float t = (rbn + rbp) / 2.0f;
        float x = o[0] + d[0] * t, y = o[1] + d[1] * t, z = o[2] + d[2] * t;
        contract3(x, y, z);
        ux = gscale(x);
        uy = gscale(y);
        uz = gscale(z);
    };
    // the sample's positions for k_sgrid (stored after its first gathers are
    // issued: the stores share vmcnt with the loads, so stores issued first
    // would hold up the first gather's consumption by their write latency)
    auto store_position = [&](int i, float ux, float uy, float uz) {
        const int k = i * S + seg;
        if (sample_writer) {
            a.u_out[((size_t)k * 3 + 0) * N + r] = ux;
            a.u_out[((size_t)k * 3 + 1) * N + r] = uy;
            a.u_out[((size_t)k * 3 + 2) * N + r] = uz;
        }
    };
    auto position = [&](int i, float& rbp, float& rbn, float& ux, float& uy, float& uz) {
        const int k = i * S + seg;
        position_of(i, S > 1 ? a.bins_in[(size_t)k * N + rr] : 0.0f, a.bins_in[(size_t)(k + 1) * N + rr], rbp,
                    rbn, ux, uy, uz);
    };
    // the next sample's raw bins are loaded one sample ahead, so the gathers
    // of a sample start without a dependent global load in front (the load
    // of sample i + 1's bins is in flight behind sample i's work)
    float nb0 = 0.0f, nb1 = 0.0f;
    {
        const int kb0 = i_begin * S + seg;
        if (S > 1) nb0 = a.bins_in[(size_t)kb0 * N + rr];
        nb1 = a.bins_in[(size_t)(kb0 + 1) * N + rr];
    }

    int exit_at = i_end;                                  // EXIT: first step not marched
    for (int i = i_begin; i < i_end; ++i) {
        const int k = i * S + seg;
        float rb_next, ux, uy, uz;
        {
            const float b0 = nb0, b1 = nb1;
            if (i + 1 < i_end) {
                const int kn = (i + 1) * S + seg;
                if (S > 1) nb0 = a.bins_in[(size_t)kn * N + rr];
                nb1 = a.bins_in[(size_t)(kn + 1) * N + rr];
            }
            position_of(i, b0, b1, rb_prev, rb_next, ux, uy, uz);
        }
        const float t = (rb_next + rb_prev) / 2.0f;
        // weight fragments are re-read from LDS each sample rather than
        // hoisted into VGPRs for the whole loop (opaque offset defeats LICM)
        int wo = lane;
        asm volatile("" : "+v"(wo));
        const uint4* FH = Fh + wo;
        const uint4* FL = Fl + wo;
        const float* FX = Fx + wo;

        floatx16 h1a = {}, h1b = {};
        float fk[AD ? 16 : 1];                           // AD: this sample's grid features (by k-block)
        // f16x3 (f16x3.h): each layer's B operands are scaled by the power of
        // two that puts the sample column's max |input| in [2^13, 2^14);
        // e_h1 / e_h2 / e_o3 = log2 of the factor a layer's accumulators carry
        // over the true values (input scales + weight-tensor scales).  Layer 1
        // (the default, SAMNERF_FINAL_JOINT = 1, round 5) gathers both k-blocks
        // first and takes ONE scale from the column's max over all 32 inputs
        // (16 levels x 2 channels): the dense and hashed levels share it, so a
        // level far below the column max keeps fewer significant bits in its
        // fp16 halves -- down to 2^-27 of the max it stays normal fp16, and the
        // f16x3 products stay within the error bound of an exact fp32 GEMM
        // (tests/test_gpu_render.py::test_final_joint_scale_over_wide_level_ranges
        // against the exact-fp32 form on levels 2^-20 .. 1 apart).  The
        // one-block-at-a-time form (SAMNERF_FINAL_JOINT = 0: the second block
        // rescales the accumulators by an exact power of two when its max needs
        // a scale two or more binades lower) remains as a build switch.
        int k1 = 0, e_h1 = 0, e_h2 = 0;
        // this half-wave's 8 features of k-block kb (levels 8 kb + hh + 2 q)
        auto gather_kb = [&](int kb, float* f, bool first) {
            LevelDesc dl[4];
            levels(kb, dl);
            uint32_t* rt = nullptr;                      // parity taps only
            if (TAP && a.rows_tap && live && r % a.tap_stride == 0u)
                rt = a.rows_tap + ((size_t)(r / a.tap_stride) * T + k) * 128u + (8 * kb + hh) * 8;
            GatherC2<4> g;
            HashSlots hs;
            if constexpr (LAY == 1) {
#pragma unroll
                for (int q = 0; q < 4; ++q) hs.base[q] = reinterpret_cast<const char*>(a.grid_emb) + a.hoff8[kb][q];
                hs.hx = hh ? a.hbit : 0u;
                hs.m8 = a.hm8;
            }
            gather_issue_c2<4>(emb, dl, ux, uy, uz, g, kinds(kb), rt, 16, LAY == 1 ? &hs : nullptr);
            if (first) store_position(i, ux, uy, uz);
            gather_finish_c2<4, S == 1>(g, f);
        };
#if SAMNERF_FINAL_JOINT
        // f16x3, layer 1 in one piece (round 5): both k-blocks gathered first
        // -- k-block 0 (the dense pair loads, 24 loads) before k-block 1 (32),
        // so only its 8 features wait through the second gather, where the
        // one-block-at-a-time form held layer 1's 32 accumulators there --
        // then ONE scale from the column's max over all 32 inputs, and the 12
        // MFMAs in the k-block 1, 0 order of every round.  (No rescale of the
        // accumulators between the blocks any more: the same f16x3 products
        // at one power-of-two scale, fp32-equivalent as before; the bits are
        // those of this form.)
        constexpr bool kJoint = !EXACT;
#else
        constexpr bool kJoint = false;
#endif
        if constexpr (kJoint) {
            float f0[8], f1[8];
            gather_kb(0, f0, true);
            gather_kb(1, f1, false);
            if constexpr (AD > 0) {
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    fk[m] = f0[m];
                    fk[8 + m] = f1[m];
                }
            }
            float m = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; e += 2) m = max_abs3(max_abs3(m, f0[e], f0[e + 1]), f1[e], f1[e + 1]);
            k1 = scale_exp_of_max(max_halves(m));
            const float sc = exp2i(k1);
            uint4 bh, bl;
            split8_f16(f1, sc, bh, bl);
            h1a = mfma_f16x3(FH[(kF1 + 2) * 64], FL[(kF1 + 2) * 64], bh, bl, h1a);
            h1b = mfma_f16x3(FH[(kF1 + 3) * 64], FL[(kF1 + 3) * 64], bh, bl, h1b);
            split8_f16(f0, sc, bh, bl);
            h1a = mfma_f16x3(FH[kF1 * 64], FL[kF1 * 64], bh, bl, h1a);
            h1b = mfma_f16x3(FH[(kF1 + 1) * 64], FL[(kF1 + 1) * 64], bh, bl, h1b);
        }
#pragma unroll
        for (int kbi = 0; kbi < (kJoint ? 0 : 2); ++kbi) {
            // k-block 1 (levels 8-15) first, then 0: the accumulation order
            // of every round (a cross-sample prefetch of k-block 1 set it)
            const int kb = 1 - kbi;
            float f[8];
            gather_kb(kb, f, kbi == 0);
            if constexpr (AD > 0) {
#pragma unroll
                for (int m = 0; m < 8; ++m) fk[kb * 8 + m] = f[m];
            }
            if constexpr (EXACT) {
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    h1a = MFMA32(FX[(kb * 8 + m) * 64], f[m], h1a);
                    h1b = MFMA32(FX[(16 + kb * 8 + m) * 64], f[m], h1b);
                }
            } else {
                float m = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; e += 2) m = max_abs3(m, f[e], f[e + 1]);
                m = max_halves(m);
                const int kk = scale_exp_of_max(m);
                if (kbi == 0) {
                    k1 = kk;
                } else if (kk < k1 - 1) {                // (within 2x the first block's max: fits fp16
                                                         // at its scale); lanes of a column agree
                    const float r = exp2i(kk - k1);
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        h1a[q] *= r;
                        h1b[q] *= r;
                    }
                    k1 = kk;
                }
                uint4 bh, bl;
                split8_f16(f, exp2i(k1), bh, bl);
                h1a = mfma_f16x3(FH[(kF1 + 2 * kb) * 64], FL[(kF1 + 2 * kb) * 64], bh, bl, h1a);
                h1b = mfma_f16x3(FH[(kF1 + 2 * kb + 1) * 64], FL[(kF1 + 2 * kb + 1) * 64], bh, bl, h1b);
            }
        }
        if constexpr (!EXACT) e_h1 = k1 + ke0;
        float s2 = 1.0f;
        if constexpr (!EXACT) {                          // max of relu(h1): the raw max, floored at 0
            int mb = 0;                                  // max of relu(h1) on the float bits
#pragma unroll
            for (int i = 0; i < 16; ++i) mb = max_relu3(mb, h1a[i], h1b[i]);
            const float m = max_halves(__builtin_bit_cast(float, mb));
            const int k2 = scale_exp_of_max(m);
            s2 = exp2i(k2);
            e_h2 = e_h1 + k2 + ke1;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            h1a[i] = relu_bits(h1a[i]);
            h1b[i] = relu_bits(h1b[i]);
        }
        floatx16 h2a = {}, h2b = {};
        if constexpr (EXACT) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float v = t ? h1b[q] : h1a[q];
                    h2a = MFMA32(FX[(32 + t * 16 + q) * 64], v, h2a);
                    h2b = MFMA32(FX[(64 + t * 16 + q) * 64], v, h2b);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                float v[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = (kb >> 1) ? h1b[8 * (kb & 1) + m] : h1a[8 * (kb & 1) + m];
                uint4 bh, bl;
                split8_f16(v, s2, bh, bl);
                h2a = mfma_f16x3(FH[(kF2 + 2 * kb) * 64], FL[(kF2 + 2 * kb) * 64], bh, bl, h2a);
                h2b = mfma_f16x3(FH[(kF2 + 2 * kb + 1) * 64], FL[(kF2 + 2 * kb + 1) * 64], bh, bl, h2b);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        float s3 = 1.0f;
        int e_o3 = 0;
        if constexpr (!EXACT) {
            int mb = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) mb = max_relu3(mb, h2a[i], h2b[i]);
            const float m = max_halves(__builtin_bit_cast(float, mb));
            const int k3 = scale_exp_of_max(m);
            s3 = exp2i(k3);
            e_o3 = e_h2 + k3 + ke2;
        }
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            h2a[i] = relu_bits(h2a[i]);
            h2b[i] = relu_bits(h2b[i]);
        }
        floatx16 o3 = {};
        if constexpr (EXACT) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
#pragma unroll
                for (int q = 0; q < 16; ++q) o3 = MFMA32(FX[(96 + t * 16 + q) * 64], t ? h2b[q] : h2a[q], o3);
                __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                float v[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) v[m] = (kb >> 1) ? h2b[8 * (kb & 1) + m] : h2a[8 * (kb & 1) + m];
                uint4 bh, bl;
                split8_f16(v, s3, bh, bl);
                o3 = mfma_f16x3(FH[(kF3 + kb) * 64], FL[(kF3 + kb) * 64], bh, bl, o3);
                __builtin_amdgcn_sched_barrier(0);
            }
            // back to the true outputs (rows 0..15 = registers 0..7 of both halves)
            const float inv = exp2i(-e_o3);
#pragma unroll
            for (int q = 0; q < 8; ++q) o3[q] = o3[q] * inv;
        }

        // sigma pre-activation = row 0, held by the lower half-wave
        float s_lo, s_hi;
        halves(o3[0], s_lo, s_hi);                       // s_lo: row 0 of this column in both halves
#ifdef SAMNERF_AB_FASTEXP   // timing A/B only
#define KF_EXP __expf
#else
#define KF_EXP expf
#endif
        const float sigma = KF_EXP(s_lo);
        // composite (renderer.py:300-307): w_k = alpha_k * exp(-sum_{j<k} ds_j),
        // the sum in double and in sample order across the ray's S slots
        const float ds = k == T - 1 ? INFINITY : (rb_next - rb_prev) * sigma;
        double before = cum;
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) {
            const float d2 = S > 1 ? __shfl(ds, (jj % R) + R * s2 + 32 * hh) : ds;
            if (s2 < seg) before += (double)d2;
            cum += (double)d2;
        }
        const float w = nan_to_num((1.0f - KF_EXP(-ds)) * KF_EXP(-(float)before));
        if (sample_writer) a.w_out[(size_t)k * N + r] = w;
        if (TAP && a.sigma_tap && sample_writer) a.sigma_tap[(size_t)k * N + r] = sigma;
        wsum += (double)w;
        depth += (double)(w * t);
#pragma unroll
        for (int q = 0; q < 8; ++q) fg[q] = fg[q] + w * o3[q];
        if constexpr (AD > 0) {
#pragma unroll
            for (int m = 0; m < 16; ++m) gacc[m] = gacc[m] + w * fk[m];
            // f16x3: the accumulators carry 2^e_h1 / 2^e_h2 (w * 2^-e is exact)
            const float w1 = EXACT ? w : w * exp2i(-e_h1), w2 = EXACT ? w : w * exp2i(-e_h2);
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                h1acc[q] = h1acc[q] + w1 * h1a[q];
                h1acc[16 + q] = h1acc[16 + q] + w1 * h1b[q];
                h2acc[q] = h2acc[q] + w2 * h2a[q];
                h2acc[16 + q] = h2acc[16 + q] + w2 * h2b[q];
            }
        }
        if (GEO && live) {                               // rows rho(q) + 4 hh of this sample
#pragma unroll
            for (int q = 0; q < 8; ++q) a.geo_out[((size_t)k * 16 + rho(q) + 4 * hh) * N + r] = o3[q];
        }
        if constexpr (SA) {                              // view MLP on this sample's colour
            floatx16 p1 = {};
#pragma unroll
            for (int q = 0; q < 8; ++q) p1 = MFMA32(Vl[kV1 + q * 64 + lane], o3[q], p1);
#pragma unroll
            for (int s2 = 0; s2 < 8; ++s2) p1 = MFMA32(Vl[kV1 + (8 + s2) * 64 + lane], sh[2 * s2 + hh], p1);
#pragma unroll
            for (int q = 0; q < 16; ++q) p1[q] = relu_bits(p1[q]);
            floatx16 p2 = {};
#pragma unroll
            for (int q = 0; q < 16; ++q) p2 = MFMA32(Vl[kV2 + q * 64 + lane], p1[q], p2);
#pragma unroll
            for (int q = 0; q < 16; ++q) p2[q] = relu_bits(p2[q]);
            floatx16 p3 = {};
#pragma unroll
            for (int q = 0; q < 16; ++q) p3 = MFMA32(Vl[kV3 + q * 64 + lane], p2[q], p3);
#pragma unroll
            for (int c = 0; c < 3; ++c) rgb[c] = rgb[c] + w * p3[c];   // rows 0..2, lower half
            if constexpr (AD == 2) {                     // view_mlp intermediates (post-ReLU)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    v1acc[q] = v1acc[q] + w * p1[q];
                    v2acc[q] = v2acc[q] + w * p2[q];
                }
            }
        }
        rb_prev = rb_next;
        // N1 early exit: once the transmittance of every ray of the wave is
        // below t_thresh, the samples left (whose weights sum to that
        // transmittance, the last one absorbing the rest) are dropped: their
        // weights are stored as 0 (k_sgrid skips all-zero samples) and their
        // positions as the grid centre (in range for any gather).  Nothing of
        // the sample is held past its MFMAs for this (holding the position
        // spilled 16 more VGPRs at 3 waves per SIMD).
        if (EXIT && i + 1 < i_end) {
            const bool open = live && !(cum > (double)a.exit_depth);
            if (__builtin_amdgcn_ballot_w64(open) == 0) {
                exit_at = i + 1;
                break;
            }
        }
    }
    // N1 compaction: rays still open at the end of a non-final pass go on
    bool cont = false;
    if constexpr (EXIT) {
        cont = a.wave_mask != nullptr && live && !(cum > (double)a.exit_depth);
        if (cont) {                                      // running sums for the next pass
            if (hh == 0) {
                a.st_d[rr] = cum;
                a.st_d[N + rr] = wsum;
                a.st_d[2 * (size_t)N + rr] = depth;
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) a.st_f[(size_t)(q + 8 * hh) * N + rr] = fg[q];
        }
        const uint64_t m = __builtin_amdgcn_ballot_w64(cont && hh == 0);   // lanes 0..31 = the rays
        if (a.wave_mask && lane == 0) a.wave_mask[ray0 / 32u] = m;
    }
    if (EXIT && sample_writer && !cont) {
        for (int i2 = exit_at; i2 < TS; ++i2) {
            const int k2 = i2 * S + seg;
            a.w_out[(size_t)k2 * N + r] = 0.0f;
            a.u_out[((size_t)k2 * 3 + 0) * N + r] = 0.5f;
            a.u_out[((size_t)k2 * 3 + 1) * N + r] = 0.5f;
            a.u_out[((size_t)k2 * 3 + 2) * N + r] = 0.5f;
        }
    }

    if constexpr (S > 1) {                               // add the slots' partial sums
        double pw = 0.0, pd = 0.0;
        float pf[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pf[q] = 0.0f;
#pragma unroll
        for (int s2 = 0; s2 < S; ++s2) {
            const int src = (jj % R) + R * s2 + 32 * hh;
            pw += __shfl(wsum, src);
            pd += __shfl(depth, src);
#pragma unroll
            for (int q = 0; q < 8; ++q) pf[q] += __shfl(fg[q], src);
        }
        wsum = pw;
        depth = pd;
#pragma unroll
        for (int q = 0; q < 8; ++q) fg[q] = pf[q];
        if constexpr (SA) {
            float pr[3] = {0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s2 = 0; s2 < S; ++s2) {
                const int src = (jj % R) + R * s2 + 32 * hh;
#pragma unroll
                for (int c = 0; c < 3; ++c) pr[c] += __shfl(rgb[c], src);
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) rgb[c] = pr[c];
        }
    }

    if (EXIT && __builtin_amdgcn_ballot_w64(live && !cont) == 0) return;   // nothing finishes here
    // view MLP on the accumulated colour features: rows 1..15 of fg are
    // f_image[0..14] (geo), f_image[15..30] = sh * sum(w) (colour = cat(geo, sh)
    // with sh constant along the ray, renderer.py:338; a rounding-level
    // reassociation of the reference's sum of products)
    if constexpr (!SA) sh_of_ray();
    const float ws = (float)wsum, dp = (float)depth;
    floatx16 v3 = {};
    if constexpr (!SA) {
        floatx16 v1 = {};
#pragma unroll
        for (int q = 0; q < 8; ++q) v1 = MFMA32(VW(kV1 + q * 64 + lane), fg[q], v1);
#pragma unroll
        for (int s = 0; s < 8; ++s) v1 = MFMA32(VW(kV1 + (8 + s) * 64 + lane), sh[2 * s + hh] * ws, v1);
#pragma unroll
        for (int i = 0; i < 16; ++i) v1[i] = relu_bits(v1[i]);
        floatx16 v2 = {};
#pragma unroll
        for (int q = 0; q < 16; ++q) v2 = MFMA32(VW(kV2 + q * 64 + lane), v1[q], v2);
#pragma unroll
        for (int i = 0; i < 16; ++i) v2[i] = relu_bits(v2[i]);
#pragma unroll
        for (int q = 0; q < 16; ++q) v3 = MFMA32(VW(kV3 + q * 64 + lane), v2[q], v3);
    }

    if constexpr (AD > 0) {
        // instance_mask_logits[c] = E[c] . sums: this lane's components, then
        // the other half-wave's (lane ^ 32 holds the ray's other rows)
        const uint32_t K = a.mask_out;
        for (uint32_t c = 0; c < K; ++c) {
            const float* E = a.aeff + (size_t)c * kAeff;
            float sacc = 0.0f;
#pragma unroll
            for (int m = 0; m < 16; ++m)
                sacc += E[2 * final_level(m >> 3, hh, (m & 7) >> 1) + (m & 1)] * gacc[m];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int u = rho(q) + 4 * hh;
                sacc += E[32 + u] * h1acc[q] + E[64 + u] * h1acc[16 + q];
                sacc += E[96 + u] * h2acc[q] + E[128 + u] * h2acc[16 + q];
                if constexpr (AD == 2) sacc += E[176 + u] * v1acc[q] + E[208 + u] * v2acc[q];
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) sacc += E[160 + rho(q) + 4 * hh] * fg[q];
            sacc = sum_halves(sacc);
            if (live && hh == 0) a.mlog[(size_t)a.tiles(r) * K + c] = sacc;
        }
        if (live && a.xsum) {                            // this lane's components of X (training)
            float* X = a.xsum + (size_t)a.tiles(r) * kAeff;
#pragma unroll
            for (int m = 0; m < 16; ++m) X[2 * final_level(m >> 3, hh, (m & 7) >> 1) + (m & 1)] = gacc[m];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int u = rho(q) + 4 * hh;
                X[32 + u] = h1acc[q];
                X[64 + u] = h1acc[16 + q];
                X[96 + u] = h2acc[q];
                X[128 + u] = h2acc[16 + q];
                if constexpr (AD == 2) {
                    X[176 + u] = v1acc[q];
                    X[208 + u] = v2acc[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 8; ++q) X[160 + rho(q) + 4 * hh] = fg[q];
        }
    }
    if (!live || seg != 0 || cont) return;
    const uint32_t ray = a.tiles(r);                     // per-ray outputs in ray order
    float* row = a.rows ? a.rows + (size_t)ray * kRow : nullptr;
    if (row) {                                 // geo units owned by this half-wave
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const int unit = rho(q) + 4 * hh;
            if (unit >= 1) row[128 + unit - 1] = fg[q];
        }
    }
    if (hh != 0) return;
    float img[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {                // rows 0..2 of v3 = registers 0..2, lower half
        img[c] = sigmoidf(SA ? rgb[c] : v3[c]) + (1.0f - ws) * a.bg;
        a.image[(size_t)ray * a.img_ld + c] = img[c];
    }
    a.depth[(size_t)ray * a.scal_ld] = dp;
    a.wsum[(size_t)ray * a.scal_ld] = ws;
    if (row) {
#pragma unroll
        for (int i = 0; i < 16; ++i) row[143 + i] = sh[i] * ws;
        row[159] = img[0];
        row[160] = img[1];
        row[161] = img[2];
        row[162] = dp;
        row[163] = 0.0f;
    }
}

struct SgridArgs {
    uint32_t N;
    RayTiles tiles;      // slot -> ray of the rows
    GridDesc<16> grid;
    const float* u_in;   // [T][3][N]
    const float* w_in;   // [T][N]
    float* rows;         // [N, kRow]
    // parity taps (samnerf_taps.srows; null in every product render): the
    // corner rows of every level of the samples of slots r % tap_stride == 0,
    // [N / tap_stride][T][16][8] (k_sgrid_box4)
    uint32_t* rows_tap;
    uint32_t tap_stride;
    // diagnostic build only (SAMNERF_SGRID_PATHS = hex device address of 8
    // uint64): per (wave, sample, level) of k_sgrid_box4, [0] uniform-cell,
    // [1] staged box, [2] direct gathers; [3] wave-samples skipped (all
    // weights 0); [4] box slots and [5] box cells of the staged boxes; null
    // in every other render
    unsigned long long* paths;
};

// f_sam = sum_k w_k * s_grid(x_k).  A block is one level x 64 neighbouring
// rays x 4 sample quarters: thread (q, ray) sums samples q*T/4 .. q*T/4 + T/4
// - 1 (its next sample's position/weight prefetched behind the current
// gather), and the quarters are added through LDS.  A wave is 64 rays at one
// (level, sample), so corner rows are shared across lanes.
// MODE: kLookPacked (lookup_level3), kLookRef (lookup_level3_ref, scalar
// accumulation); k_sgrid_box4 below is the de-duplicated form.  All give
// identical bits.

template <int T, int MODE>
__global__ void __launch_bounds__(256) k_sgrid(SgridArgs a) {
    constexpr int TQ = T / 4;
    __shared__ float part[3][8][64];
    const uint32_t lane = threadIdx.x & 63u, q = threadIdx.x >> 6;
    const uint32_t r = xcd_chunk(blockIdx.x, (a.N + 63u) / 64u) * 64u + lane;   // gridDim.x % 8 == 0
    const uint32_t level = blockIdx.y;
    const bool live = r < a.N;
    const uint32_t N = a.N, rr = live ? r : N - 1;
    const LevelDesc lv = a.grid.lv[level];
    float acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = 0.0f;
    const int k0 = (int)q * TQ;
    float ux = a.u_in[((size_t)k0 * 3 + 0) * N + rr];
    float uy = a.u_in[((size_t)k0 * 3 + 1) * N + rr];
    float uz = a.u_in[((size_t)k0 * 3 + 2) * N + rr];
    float w = a.w_in[(size_t)k0 * N + rr];
    for (int k = k0; k < k0 + TQ; ++k) {
        const int kn = k + 1 < k0 + TQ ? k + 1 : k;          // prefetch (clamped)
        const float nx = a.u_in[((size_t)kn * 3 + 0) * N + rr];
        const float ny = a.u_in[((size_t)kn * 3 + 1) * N + rr];
        const float nz = a.u_in[((size_t)kn * 3 + 2) * N + rr];
        const float nw = a.w_in[(size_t)kn * N + rr];
        float f[8];
        // a sample with weight 0 on every ray of the wave adds nothing (N1's
        // dropped samples; acc + 0 * f == acc for the finite features)
        if (__builtin_amdgcn_ballot_w64(w != 0.0f) == 0) {
        } else if constexpr (MODE == kLookRef) {
            lookup_level3_ref<8>(a.grid.emb, lv, ux, uy, uz, f);
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = acc[c] + w * f[c];
        } else {
            lookup_level3<8>(a.grid.emb, lv, ux, uy, uz, f);
            const f2v wv = {w, w};            // acc + w * f, two channels per packed mul / add
#pragma unroll
            for (int c = 0; c < 8; c += 2) {
                const f2v s = f2v{acc[c], acc[c + 1]} + wv * f2v{f[c], f[c + 1]};
                acc[c] = s.x;
                acc[c + 1] = s.y;
            }
        }
        ux = nx;
        uy = ny;
        uz = nz;
        w = nw;
    }
    if (q > 0) {
#pragma unroll
        for (int c = 0; c < 8; ++c) part[q - 1][c][lane] = acc[c];
    }
    __syncthreads();
    if (q > 0 || !live) return;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = ((acc[c] + part[0][c][lane]) + part[1][c][lane]) + part[2][c][lane];
    float4* dst = reinterpret_cast<float4*>(a.rows + (size_t)a.tiles(r) * kRow + level * 8u);
    dst[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
    dst[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
}

// k_sgrid with de-duplicated gathers (SAMNERF_LOOKUP=box4, wave_box.h).  A
// block is 64 neighbouring rays x 4 sample quarters at one group of 4
// levels (gridDim.y = 4): wave q sums samples q*T/4 .. q*T/4 + T/4 - 1 for
// levels 4g .. 4g+3 (32 accumulators per lane).  Per sample the wave reduces
// its positions' range once, lanes 0-3 evaluate the 4 levels' padded corner
// boxes, and per level the wave loads each distinct corner row once into its
// 8 KiB LDS slice and reads the 8 corners of every lane from there: the
// vector-memory path carries one address per distinct row instead of 16 per
// lane.  Same rows, weights, FMA order and quarter split as k_sgrid, so the
// bits are identical.
constexpr uint32_t kBoxSlots = 256;          // 32 B slots per wave (8 KiB)

// 4 waves per SIMD (128 VGPRs, 7 spilled) instead of the 3 the compiler's
// default 142 VGPRs allow: the VALU-bound box gathers hide their LDS and
// staging latency better -- 0.835 -> 0.72 ms per view, 0.126 -> 0.112 ms at
// one rank's 32K rays (round 2)
#ifndef SAMNERF_DIAG_SGRID_WAVES
#define SAMNERF_DIAG_SGRID_WAVES 4
#endif
// TAP: the parity-tap instantiation (samnerf_taps.srows): the same kernel plus
// the corner-row stores, its own instantiation because the tap code raised the
// product form's spills (20 -> 60 bytes of scratch at 4 waves per SIMD); the
// tapped render's outputs are checked bit-identical to the product's.
// SGRID_UNI (round 5): a level whose box is one cell for the whole wave
// reads that cell's 8 corner rows through the scalar cache
// (lookup_level3_uniform) -- the coarse levels, where a wave's 64 neighbouring
// rays at one sample share a cell most of the time; the box path's LDS reads
// (8 corners x 32 B per lane) bound the kernel
#ifndef SAMNERF_SGRID_UNI
#define SAMNERF_SGRID_UNI 1
#endif
constexpr bool SGRID_UNI = SAMNERF_SGRID_UNI;

template <int T, bool TAP = false>
__global__ void __launch_bounds__(256)
#if SAMNERF_DIAG_SGRID_WAVES
__attribute__((amdgpu_waves_per_eu(SAMNERF_DIAG_SGRID_WAVES, SAMNERF_DIAG_SGRID_WAVES)))
#endif
k_sgrid_box4(SgridArgs a) {
    constexpr int TQ = T / 4;
    __shared__ float4 smem[4][kBoxSlots * 2];          // per wave: the box slice
    const uint32_t lane = threadIdx.x & 63u, q = threadIdx.x >> 6;
    const uint32_t r = xcd_chunk(blockIdx.x, (a.N + 63u) / 64u) * 64u + lane;
    const uint32_t g = blockIdx.y;                      // levels 4g .. 4g+3
    const bool live = r < a.N;
    const uint32_t N = a.N, rr = live ? r : N - 1;
    const LevelDesc L[4] = {a.grid.lv[4 * g], a.grid.lv[4 * g + 1], a.grid.lv[4 * g + 2],
                            a.grid.lv[4 * g + 3]};
    const uint32_t li = lane & 3u;                      // this lane's level for the box pass
    const LevelDesc mine = {li == 0 ? L[0].off : li == 1 ? L[1].off : li == 2 ? L[2].off : L[3].off,
                            li == 0 ? L[0].size : li == 1 ? L[1].size : li == 2 ? L[2].size : L[3].size,
                            li == 0 ? L[0].res : li == 1 ? L[1].res : li == 2 ? L[2].res : L[3].res,
                            0u,
                            li == 0 ? L[0].fres : li == 1 ? L[1].fres : li == 2 ? L[2].fres : L[3].fres,
                            li == 0 ? L[0].ftop : li == 1 ? L[1].ftop : li == 2 ? L[2].ftop : L[3].ftop};
    float* slice = reinterpret_cast<float*>(smem[q]);
    const char* base = reinterpret_cast<const char*>(a.grid.emb);
    float acc[4][8];
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[l][c] = 0.0f;
    const int k0 = (int)q * TQ;
    // 32-bit byte offsets (the host launches this form only for 384 N < 2^32):
    // uniform base + lane offset loads, no 64-bit address arithmetic per sample
    const char* ub = reinterpret_cast<const char*>(a.u_in);
    const char* wb = reinterpret_cast<const char*>(a.w_in);
    const uint32_t N4 = N * 4u;
    auto ld = [](const char* b, uint32_t off) { return *reinterpret_cast<const float*>(b + off); };
    float ux = ld(ub, ((uint32_t)k0 * 3u + 0u) * N4 + rr * 4u);
    float uy = ld(ub, ((uint32_t)k0 * 3u + 1u) * N4 + rr * 4u);
    float uz = ld(ub, ((uint32_t)k0 * 3u + 2u) * N4 + rr * 4u);
    float w = ld(wb, (uint32_t)k0 * N4 + rr * 4u);
    for (int k = k0; k < k0 + TQ; ++k) {
        const uint32_t kn = (uint32_t)(k + 1 < k0 + TQ ? k + 1 : k);          // prefetch (clamped)
        const float nx = ld(ub, (kn * 3u + 0u) * N4 + rr * 4u);
        const float ny = ld(ub, (kn * 3u + 1u) * N4 + rr * 4u);
        const float nz = ld(ub, (kn * 3u + 2u) * N4 + rr * 4u);
        const float nw = ld(wb, kn * N4 + rr * 4u);
        // samples with weight 0 on all 64 rays (N1's dropped samples) add nothing
#ifdef SAMNERF_DIAG_VARIANTS
        if (a.paths && lane == 0u && __builtin_amdgcn_ballot_w64(w != 0.0f) == 0) atomicAdd(a.paths + 3, 1ull);
#endif
        if (__builtin_amdgcn_ballot_w64(w != 0.0f) != 0) {
            const f2v wv = {w, w};
            auto add = [&](int l, const float* f) {
#pragma unroll
                for (int c = 0; c < 8; c += 2) {
                    const f2v s2 = f2v{acc[l][c], acc[l][c + 1]} + wv * f2v{f[c], f[c + 1]};
                    acc[l][c] = s2.x;
                    acc[l][c + 1] = s2.y;
                }
            };
            const URange ur = wave_urange(ux, uy, uz);
            const bool ordered = wave_positions_ordered(ux, uy, uz);
            uint32_t p0, p1, p2;
            pbox_lane(mine, ur, p0, p1, p2);
            // per level: the box's rows staged through registers into the
            // wave's slice, then every lane's 8 corners read from LDS; a box
            // over kBoxSlots slots gathers directly.  (Round 4 measured a
            // one-pass form -- the 4 boxes by LDS DMA into the one slice, one
            // memory round trip per sample, a level whose box did not fit
            // beside the others gathering directly -- at 0.86 against 0.665 ms
            // per view, interleaved A/B of whole builds.)
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                const PBox b = pbox_read(p0, p1, p2, l);
                float f[8];
                uint32_t* rt = nullptr;                     // parity taps only
                if (TAP && live && r % a.tap_stride == 0u)
                    rt = a.rows_tap + ((size_t)(r / a.tap_stride) * T + k) * 128u + (4 * g + l) * 8;
#ifdef SAMNERF_DIAG_VARIANTS
                if (a.paths && lane == 0u) {
                    const int path = (SGRID_UNI && b.uni && ordered) ? 0 : b.slots <= kBoxSlots ? 1 : 2;
                    atomicAdd(a.paths + path, 1ull);
                    if (path == 1) {
                        atomicAdd(a.paths + 4, (unsigned long long)b.slots);
                        atomicAdd(a.paths + 5, (unsigned long long)(b.ex * b.ey * b.ez));
                    }
                }
#endif
                if (SGRID_UNI && b.uni && ordered) {
                    // one cell for the whole wave: its 8 corner rows through the
                    // scalar cache, no box staging, no LDS reads (round 5)
                    const uint32_t dx = b.ex - 1u, dy = b.ey - 1u, dz = b.ez - 1u;
                    uint32_t rows[8];
#pragma unroll
                    for (int c = 0; c < 8; ++c)
                        rows[c] = dense_or_hash_row(b.x0 + (c & 1) * dx, b.y0 + ((c >> 1) & 1) * dy,
                                                    b.z0 + (c >> 2) * dz, L[l]);
                    if (rt) {
#pragma unroll
                        for (int c = 0; c < 8; ++c) rt[c] = rows[c];
                    }
                    lookup_level3_uniform<8>(a.grid.emb, L[l], rows, ux, uy, uz, f);
                } else if (b.slots <= kBoxSlots) {
                    wave_lds_sync();                        // previous level's reads done
                    stage_pbox<8>(base, L[l], b, slice, lane);
                    wave_lds_sync();
                    if (ordered)
                        lookup_level3_pbox<8, false>(a.grid.emb, L[l], b, slice, ux, uy, uz, f, rt);
                    else
                        lookup_level3_pbox<8, true>(a.grid.emb, L[l], b, slice, ux, uy, uz, f, rt);
                } else {
                    if (rt) tap_direct_rows<8>(L[l], ux, uy, uz, rt);
                    lookup_level3<8>(a.grid.emb, L[l], ux, uy, uz, f);
                }
                add(l, f);
            }
        }
        ux = nx;
        uy = ny;
        uz = nz;
        w = nw;
    }
    // quarters 1-3 hand their sums to quarter 0 through the (now free) slices
    __syncthreads();
    float* part = reinterpret_cast<float*>(smem);          // [3][32][64]
    if (q > 0) {
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int c = 0; c < 8; ++c) part[((q - 1) * 32 + l * 8 + c) * 64 + lane] = acc[l][c];
    }
    __syncthreads();
    if (q > 0 || !live) return;
    float* dst = a.rows + (size_t)a.tiles(r) * kRow + g * 32u;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        float v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int i = l * 8 + c;
            v[c] = ((acc[l][c] + part[(0 * 32 + i) * 64 + lane]) + part[(1 * 32 + i) * 64 + lane]) +
                   part[(2 * 32 + i) * 64 + lane];
        }
        reinterpret_cast<float4*>(dst + l * 8)[0] = make_float4(v[0], v[1], v[2], v[3]);
        reinterpret_cast<float4*>(dst + l * 8)[1] = make_float4(v[4], v[5], v[6], v[7]);
    }
}

// Backward of k_sgrid for the distillation step: grad_emb[row] += w_k *
// corner_weight * g[ray, level*8 + c].  One thread per (ray, level, channel):
// a wave is 8 neighbouring rays x 8 channels, so one atomic wave-instruction
// adds 8 rows of 32 contiguous bytes.
//
// The global float atomics are the cost: they execute at the memory side at
// roughly one wave-instruction per 50 ns per CU whatever the lanes hold
// (MI355X_MICROARCH.md), and the round-1 form issued 8 per wave and sample (one
// per corner, duplicates among the 8 rays merged by a butterfly).  Here the
// wave first sums its 64 corner contributions per channel in LDS over the
// exact box of corner cells the 8 rays touch (wave_box.h's idea, reversed),
// then compacts the non-zero cells (ballot + prefix) and adds each distinct
// cell row once: ceil(distinct rows / 8) atomics per wave and sample --
// ~2.4x fewer over the 16 levels of a training view (distinct corner rows of
// 8 rays: ~10 at the coarse levels, ~50 at level 15).  Boxes of more than 64
// cells (scattered rays) take the per-corner form.  Measured on a cfg-5 step
// the box form is SLOWER (0.70 vs 0.56 ms): the atomic instruction count is
// not what binds the per-corner form; the box's six wave reductions, LDS
// atomics and three wave syncs per sample cost more than the atomics they
// save.  The per-corner form stays the default (max_cells = 0); the box form
// is kept selectable (SAMNERF_SGRID_BWD=box) and tested against it.
constexpr uint32_t kBwdBoxCells = 64;

// DET (samnerf_sgrid_backward_det): the per-corner form's adds go
// to a 64-bit fixed-point accumulator instead of the fp32 table -- integer
// atomics are associative, so every total is the same whatever order the
// waves reach it in -- at the scale 2^det_shift (sgrid_det_shift: |any row's
// total| * 2^shift < 2^61); k_sgrid_det_finish adds the totals to the fp32
// gradient.  The per-wave butterfly merge is a fixed order, so it stays.
struct DetAcc {
    unsigned long long* acc;   // [rows][8] int64 (two's complement), null: the fp32 atomics
    const uint32_t* hdr;       // hdr[0]: max |grad_fsam| (float bits), k_sgrid_det_max;
                               // hdr[1]: non-zero when grad_fsam holds a NaN or an Inf
    int log2n;                 // ceil(log2 N)
};

// A gradient with a NaN or an Inf has no fixed-point scale (frexpf(inf) is
// unspecified and a NaN converts to INT64_MIN), and the reference's atomics
// (gridencoder.cu:252-349) propagate it into every row the ray reaches: such
// a call takes the fp32 atomic form (wave-uniform: one header word), whose
// sums carry the NaN / Inf like the reference's.  Bits repeat only for finite
// gradients, which is all the deterministic mode promises.
__device__ __forceinline__ bool sgrid_det_nonfinite(const DetAcc& d) { return d.hdr[1] != 0u; }

// 2^shift of the fixed point: max |g| < 2^e and at most N rays of weights
// summing to <= 1 reach a row, so |total| < 2^(log2n + e) and |total| 2^shift
// < 2^61 (two bits of margin)
__device__ __forceinline__ int sgrid_det_shift(const DetAcc& d) {
    int e = 0;
    frexpf(__uint_as_float(d.hdr[0]), &e);
    return 61 - d.log2n - e;
}

template <int T, bool DET = false>
__global__ void __launch_bounds__(256)
k_sgrid_backward(uint32_t N, RayTiles tiles, GridDesc<16> g, const float* __restrict__ u_in,
                 const float* __restrict__ w_in, const float* __restrict__ grad, uint32_t gstride,
                 float* __restrict__ gemb, uint32_t max_cells, uint32_t run_res, DetAcc det = {}) {
    __shared__ float box[4][kBwdBoxCells * 8];           // per wave: cell x channel sums
    __shared__ uint32_t list[4][kBwdBoxCells];           // per wave: rows of the non-zero cells
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t r = (uint32_t)(t >> 3), ch = (uint32_t)(t & 7u), lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t level = blockIdx.y;
    if (((t & ~(uint64_t)63) >> 3) >= N) return;          // whole wave past the end
#ifdef SG_DIAG_MINLEVEL   // diagnostics only (tools/r2/gpu_r2s4h.sh): scatter levels >= this
    if (level < SG_DIAG_MINLEVEL) return;
#endif
    const bool live = r < N;                                // lanes stay for the reductions
    const uint32_t rr = live ? r : N - 1;
    const LevelDesc d = g.lv[level];
    const float gv = live ? grad[(size_t)tiles(rr) * gstride + level * 8u + ch] : 0.0f;
    float* base = gemb + (size_t)d.off * 8u + ch;
    float* slice = box[wv];
    uint32_t* rows = list[wv];
    const uint32_t top = d.res - 1u;
    // blockIdx.z: this block's share of the samples (more waves in flight: the
    // per-sample chain -- loads, box reductions, LDS sums, atomics -- is
    // latency-bound at 8 rays per wave)
    const int k0 = (int)(blockIdx.z * T / gridDim.z), k1 = (int)((blockIdx.z + 1) * T / gridDim.z);
    // levels up to run_res: a lane walks its ray's samples in order, and the
    // previous sample's 8 corner rows stay pending in registers -- a new corner
    // on a pending row absorbs its sum, only rows the ray has left are added to
    // memory (consecutive samples of a ray share cells at the coarse levels)
    const bool run = !DET && max_cells == 0u && d.res <= run_res;     // block-uniform
    const bool fixed = DET && !sgrid_det_nonfinite(det);  // uniform: the header word
    const double dscale = fixed ? ldexp(1.0, sgrid_det_shift(det)) : 0.0;
    unsigned long long* const dbase = fixed ? det.acc + (size_t)d.off * 8u + ch : nullptr;
    uint32_t prow[8];
    float pval[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        prow[c] = 0xFFFFFFFFu;
        pval[c] = 0.0f;
    }
    for (int k = k0; k < k1; ++k) {
        const float ux = u_in[((size_t)k * 3 + 0) * N + rr];
        const float uy = u_in[((size_t)k * 3 + 1) * N + rr];
        const float uz = u_in[((size_t)k * 3 + 2) * N + rr];
        const float wk = w_in[(size_t)k * N + rr];
        if (__builtin_amdgcn_ballot_w64(wk != 0.0f) == 0) continue;   // N1's dropped samples
        const float wg = wk * gv;
        uint32_t cx, cy, cz;
        float fx, fy, fz;
        locate_axis(ux, d, cx, fx);
        locate_axis(uy, d, cy, fy);
        locate_axis(uz, d, cz, fz);
        const uint32_t nx = min(cx + 1u, top), ny = min(cy + 1u, top), nz = min(cz + 1u, top);
        // the wave's box of corner cells (cells are never negative: int order)
        const uint32_t x0 = (uint32_t)wave_imin((int)cx), x1 = (uint32_t)wave_imax((int)nx);
        const uint32_t y0 = (uint32_t)wave_imin((int)cy), y1 = (uint32_t)wave_imax((int)ny);
        const uint32_t z0 = (uint32_t)wave_imin((int)cz), z1 = (uint32_t)wave_imax((int)nz);
        const uint32_t ex = x1 - x0 + 1u, ey = y1 - y0 + 1u, ez = z1 - z0 + 1u;
        const uint32_t cells = ex * ey * ez;                 // wave-uniform
        if (!DET && cells <= max_cells) {
            // 1. zero the slice (lane = cell), 2. LDS-add the corners
            reinterpret_cast<float4*>(slice + lane * 8u)[0] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            reinterpret_cast<float4*>(slice + lane * 8u)[1] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            wave_lds_sync();
            const uint32_t X[2] = {cx - x0, nx - x0};
            const uint32_t Y[2] = {(cy - y0) * ex, (ny - y0) * ex};
            const uint32_t Z[2] = {(cz - z0) * ex * ey, (nz - z0) * ex * ey};
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float wx = (c & 1) ? fx : 1.0f - fx;
                const float wy = (c & 2) ? fy : 1.0f - fy;
                const float wz = (c & 4) ? fz : 1.0f - fz;
                const uint32_t cell = X[c & 1] + Y[(c >> 1) & 1] + Z[c >> 2];
                atomicAdd(slice + cell * 8u + ch, ((wx * wy) * wz) * wg);
            }
            wave_lds_sync();
            // 3. compact the non-zero cells (lane = cell): ballot + prefix
            const float4 va = reinterpret_cast<const float4*>(slice + lane * 8u)[0];
            const float4 vb = reinterpret_cast<const float4*>(slice + lane * 8u)[1];
            const bool nzc = lane < cells && (va.x != 0.0f || va.y != 0.0f || va.z != 0.0f ||
                                              va.w != 0.0f || vb.x != 0.0f || vb.y != 0.0f ||
                                              vb.z != 0.0f || vb.w != 0.0f);
            const uint64_t mask = __builtin_amdgcn_ballot_w64(nzc);
            const uint32_t n = (uint32_t)__builtin_popcountll(mask);
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
            if (nzc) {
                const uint32_t bx = lane % ex, by = (lane / ex) % ey, bz = lane / (ex * ey);
                rows[rank] = (dense_or_hash_row(x0 + bx, y0 + by, z0 + bz, d) << 6) | lane;
            }
            wave_lds_sync();
            // 4. one global atomic per distinct cell row and channel, 8 cells
            //    (x 8 channels) per wave-instruction
            for (uint32_t j = 0; j < n; j += 8u) {
                const uint32_t idx = j + (lane >> 3);
                if (idx < n) {
                    const uint32_t e = rows[idx];
                    atomicAdd(base + (size_t)(e >> 6) * 8u, slice[(e & 63u) * 8u + ch]);
                }
            }
            wave_lds_sync();                                  // reads done before the next zeroing
        } else if (run) {
            uint32_t nrow[8];
            float nval[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float wx = (c & 1) ? fx : 1.0f - fx;
                const float wy = (c & 2) ? fy : 1.0f - fy;
                const float wz = (c & 4) ? fz : 1.0f - fz;
                nrow[c] = dense_or_hash_row((c & 1) ? nx : cx, (c & 2) ? ny : cy, (c & 4) ? nz : cz, d);
                nval[c] = ((wx * wy) * wz) * wg;
            }
#pragma unroll
            for (int p = 0; p < 8; ++p) {
                bool hit = false;
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const bool h = !hit && prow[p] == nrow[c];
                    nval[c] += h ? pval[p] : 0.0f;
                    hit = hit || h;
                }
                if (!hit && live && prow[p] != 0xFFFFFFFFu) atomicAdd(base + (size_t)prow[p] * 8u, pval[p]);
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                prow[c] = nrow[c];
                pval[c] = nval[c];
            }
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const float wx = (c & 1) ? fx : 1.0f - fx;
                const float wy = (c & 2) ? fy : 1.0f - fy;
                const float wz = (c & 4) ? fz : 1.0f - fz;
                const uint32_t row = dense_or_hash_row((c & 1) ? nx : cx, (c & 2) ? ny : cy,
                                                       (c & 4) ? nz : cz, d);
                float val = ((wx * wy) * wz) * wg;
                // merge equal rows of the wave's 8 rays over a 3-level butterfly
                // so one lane per row and channel issues the atomic
                bool alive = live;
#pragma unroll
                for (int sd = 8; sd < 64; sd <<= 1) {
                    const uint32_t orow = __shfl_xor(row, sd);
                    const float oval = __shfl_xor(val, sd);
                    const int oalive = __shfl_xor((int)alive, sd);
                    if (alive && oalive && orow == row) {
                        if (lane & sd) alive = false;
                        else val += oval;
                    }
                }
                if (alive) {
                    if (DET && fixed)
                        atomicAdd(dbase + (size_t)row * 8u,
                                  (unsigned long long)__double2ll_rn((double)val * dscale));
                    else
                        atomicAdd(base + (size_t)row * 8u, val);
                }
            }
        }
    }
    if (run && live)
#pragma unroll
        for (int c = 0; c < 8; ++c)
            if (prow[c] != 0xFFFFFFFFu) atomicAdd(base + (size_t)prow[c] * 8u, pval[c]);
}

// max |grad_fsam[ray, 0:128]| into hdr[0] and a non-finite flag into hdr[1]
// (both zeroed by the host): float bits of non-negative values order as
// unsigned integers, so the atomic max is exact
__global__ void __launch_bounds__(256)
k_sgrid_det_max(const float* __restrict__ grad, uint32_t N, uint32_t gstride, uint32_t* hdr) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    float m = 0.0f;
    bool bad = false;
    if (t < (uint64_t)N * 32u) {                     // 4 features per thread
        const float4 v = *reinterpret_cast<const float4*>(grad + (size_t)(t >> 5) * gstride + (t & 31u) * 4u);
        m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
        bad = !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
    }
    m = wave_max64(m);
    const bool any_bad = __builtin_amdgcn_ballot_w64(bad) != 0;
    if ((threadIdx.x & 63u) == 0u) {
        if (m > 0.0f && isfinite(m)) atomicMax(hdr, __float_as_uint(m));
        if (any_bad) atomicOr(hdr + 1, 1u);
    }
}

// the fixed-point totals into the fp32 gradient (accumulated into, as the
// atomic form), the accumulator left zero for the next call
__global__ void __launch_bounds__(256)
k_sgrid_det_finish(DetAcc det, float* __restrict__ gemb, uint64_t n) {
    if (sgrid_det_nonfinite(det)) return;            // the fp32 atomics ran: the accumulator is untouched
    const double inv = ldexp(1.0, -sgrid_det_shift(det));
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        const long long v = (long long)det.acc[i];
        if (v != 0) {
            gemb[i] = gemb[i] + (float)((double)v * inv);
            det.acc[i] = 0ull;
        }
    }
}

// The shader clock over a stretch of the stream (samnerf_clock_stamp, the
// bench's timed views): workgroup b stamps its XCC id, s_memtime (one tick
// per shader cycle, MI355X_MICROARCH.md) and s_memrealtime (100 MHz).  The
// read-only counter instructions only (scalar reads; the stores are vector).
__global__ void __launch_bounds__(64) k_clock_stamp(unsigned long long* out) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long rt = __builtin_amdgcn_s_memrealtime();
    // XCC_ID: hwreg 20, bits [3:0] (gfx940+)
    const unsigned xcc = __builtin_amdgcn_s_getreg((20u) | (0u << 6) | ((4u - 1u) << 11));
    if (threadIdx.x == 0) {
        out[3 * blockIdx.x + 0] = xcc;
        out[3 * blockIdx.x + 1] = t;
        out[3 * blockIdx.x + 2] = rt;
    }
}

// ------------------------------------------------------- step kernels ----

__global__ void __launch_bounds__(256)
k_get_rays(float r00, float r01, float r02, float r10, float r11, float r12, float r20, float r21,
           float r22, float tx, float ty, float tz, float fx, float fy, float cx, float cy,
           uint32_t W, uint32_t row0, uint32_t n, float* __restrict__ rays_o,
           float* __restrict__ rays_d) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    const uint32_t p = row0 * W + t;
    const float i = (float)(p % W) + 0.5f;   // linspace(0, W-1, W) holds exact integers
    const float j = (float)(p / W) + 0.5f;
    const float xs = (i - cx) / fx;
    const float ys = -((j - cy) / fy);
    const float zs = -1.0f;
    // directions @ R^T  (utils.py:255-256)
    // outputs hold only this band: local ray index t
    rays_d[(size_t)t * 3 + 0] = __builtin_fmaf(zs, r02, __builtin_fmaf(ys, r01, xs * r00));
    rays_d[(size_t)t * 3 + 1] = __builtin_fmaf(zs, r12, __builtin_fmaf(ys, r11, xs * r10));
    rays_d[(size_t)t * 3 + 2] = __builtin_fmaf(zs, r22, __builtin_fmaf(ys, r21, xs * r20));
    rays_o[(size_t)t * 3 + 0] = tx;
    rays_o[(size_t)t * 3 + 1] = ty;
    rays_o[(size_t)t * 3 + 2] = tz;
}

struct Aabb {
    float v[6];
};

__global__ void __launch_bounds__(256)
k_near_far(const float* __restrict__ o, const float* __restrict__ d, uint32_t N, Aabb box,
           float min_near, float* __restrict__ nears, float* __restrict__ fars) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    float oo[3] = {o[r * 3], o[r * 3 + 1], o[r * 3 + 2]};
    float dd[3] = {d[r * 3], d[r * 3 + 1], d[r * 3 + 2]};
    float n, f;
    near_far_aabb(oo, dd, box.v, min_near, n, f);
    nears[r] = n;
    fars[r] = f;
}

__global__ void __launch_bounds__(256)
k_contract(const float* __restrict__ x, float* __restrict__ z, uint32_t N) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    float a = x[r * 3], b = x[r * 3 + 1], c = x[r * 3 + 2];
    contract3(a, b, c);
    z[r * 3] = a;
    z[r * 3 + 1] = b;
    z[r * 3 + 2] = c;
}

__global__ void __launch_bounds__(256)
k_sample_pdf(const float* __restrict__ bins, const float* __restrict__ weights, uint32_t N,
             uint32_t T0, uint32_t T, Lin u, float* __restrict__ out, int32_t* __restrict__ inds) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    const float* w = weights + (size_t)r * T0;
    const float* b = bins + (size_t)r * (T0 + 1);
    const float wsum = torch_row_sum((int)T0, [&](int i) { return w[i] + 0.01f; });
    sample_pdf_walk(
        (int)T0, (int)T, u, wsum, [&](int i) { return w[i]; },
        [&](int i) { return b[i]; },
        [&](int j, float v, int ind) {
            out[(size_t)r * T + j] = v;
            if (inds) inds[(size_t)r * T + j] = ind;
        });
}

__global__ void __launch_bounds__(256)
k_composite(const float* __restrict__ rb, const float* __restrict__ sig, uint32_t N, uint32_t T,
            float* __restrict__ w) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= N) return;
    double cum = 0.0;
    for (uint32_t k = 0; k < T; ++k) {
        const float ds = (rb[(size_t)r * (T + 1) + k + 1] - rb[(size_t)r * (T + 1) + k]) *
                         sig[(size_t)r * T + k];
        w[(size_t)r * T + k] = composite_step(ds, cum, k == T - 1);
    }
}

}  // namespace


// ------------------------------------------------------------------ host --

namespace {

struct Workspace {
    float* snf;
    float4* rec;       // [N][2] slot-ordered ray records (k_snf, PropArgs::rec)
    float* bins1;
    float* bins2;
    float* wtmp;
    float* u_f;
    float* w_f;
    float* rows;
    float* packed;
    uint4* gpack;      // f16x3 grid_mlp fragments [2][kFSlots][64] (head_mode 0)
    int* gexp;         // their tensors' log2 scales [3]
    float* geo_f;      // [32][16][N] grid_mlp output rows per sample (with_mask, kind 0)
    float* mpacked;    // mask head weight stream (with_mask, kind 0)
    float* aeff;       // [K][240] adaptive heads' effective matrix (with_mask, kinds 1-2)
    float* mlog;       // [N][K] adaptive heads' logits (with_mask, kinds 1-2)
    float* xsum;       // [N][kAeff] their per-ray input sums (with_mask, kinds 1-2; training)
    uint32_t* n1_list; // [2][N] N1 compaction: the passes' slot lists (t_thresh > 0)
    uint32_t* n1_cnt;  // [2] their lengths
    uint64_t* n1_mask; // [ceil(N / 32)] the waves' ballot masks of open rays
    uint32_t* n1_base; // [ceil(N / 32)] their exclusive scan
    double* n1_std;    // [3][N] running optical depth / sum w / sum w t of open rays
    float* n1_stf;     // [16][N] running sum w * grid_mlp rows
    size_t bytes;
};

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// Gather variants, for A/B measurement and the bit-identity tests:
// SAMNERF_LOOKUP = packed (default) | ref | box (k_sgrid only; the proposal
// stages use packed).  Read per call (getenv is cheap next to a launch).
int lookup_mode() {
    const char* v = diag_env("SAMNERF_LOOKUP");
    if (!v || !*v) return kLookAuto;
    if (!strcmp(v, "ref")) return kLookRef;
    if (!strcmp(v, "box")) return kLookBox4;
    if (!strcmp(v, "box4")) return kLookBox4;
    return kLookPacked;
}

thread_local hipEvent_t g_stage_events[8];
thread_local uint32_t g_n_stage_events = 0;
thread_local samnerf_taps g_taps = {};
thread_local uint32_t g_taps_n = 0;
thread_local bool g_taps_on = false;
// the compiled forms the last render of this thread launched
// (samnerf_last_forms): [0] / [1] the proposal stages' level classes (KD |
// KH << 8, 0 for the run-time form), [2] k_final's layout (final_layout)
thread_local uint32_t g_last_forms[4] = {};

void mark_stage(uint32_t i, hipStream_t s) {
    if (i < g_n_stage_events && g_stage_events[i]) (void)hipEventRecord(g_stage_events[i], s);
}

// Default k_sgrid form by launch size: the de-duplicated box gathers win
// on a full view (TA-bound direct gathers): 0.83 vs 1.05 ms at 262,144 rays.
// Since the integer-bit range reduction and v_med3 clamp they also win on one
// rank's share of a sharded view: 0.120 vs 0.132 ms at 32,768 rays, 0.228 vs
// 0.262 at 65,536 (bands of the 512x512 view, bench --rank-share 8 / 4).
// Below 32,768 rays (not measured) the direct form stays.
constexpr uint32_t kBox4MinRays = 32768;

// k_final's cross-sample prefetch of k-block 1's gathers (rounds 1-3, a
// diagnostic form only since round 2: for S = 1 three waves per SIMD without
// it beat two with it, 0.797 vs 0.826 ms per view; for S = 2 / 4 it spilled,
// 0.288 vs 0.260 ms at 32,768 rays) was removed in round 4: its f16x3 forms
// rendered one sample of one 16-lane group differently in about one launch in
// four, mostly the first of a process (|d sigma| up to 7e-3 relative; the
// exact-fp32 prefetch form and every product form bit-stable over the same
// runs; not traced to a cause -- tools/pf_diag.py).
// k_final's wave-uniform slot paths (dense pair loads, select-free hashed
// rows): on by default; SAMNERF_FINAL_CLASSES=0 takes the lane-varying form
// everywhere (same bits: the A/B parity test).
uint32_t final_classes() {
    const char* v = diag_env("SAMNERF_FINAL_CLASSES");
    return (v && atoi(v) == 0) ? 0u : 1u;
}

// k_final's LAY (1: the reference grid's slot classes and a power-of-two
// grid scale, compile-time; 0: run time).  SAMNERF_FINAL_LAY=0 (diagnostic
// build) forces the run-time form, for the bit-identity test.
int final_layout(const FinalArgs& fa) {
    const char* v = diag_env("SAMNERF_FINAL_LAY");
    if (v && atoi(v) == 0) return 0;
    for (int kb = 0; kb < 2; ++kb)
        if (fa.kdense[kb] != kLay1Dense[kb] || fa.khashed[kb] != kLay1Hashed[kb]) return 0;
    if (fa.hbit == 0u) return 0;                      // hashed slots not laid out for HashSlots
    return fa.gs.inv_b2 != 0.0f ? 1 : 0;
}

// LAY 1's HashSlots layout (FinalArgs::hoff8 / hbit / hm8): every hashed slot
// holds two consecutive levels of one power-of-two size S (the reference's
// 2^19 hash tables) with res <= S; else hbit = 0 and LAY 1 is not used.
void set_hash_slots(FinalArgs& fa, const GridDesc<16>& g) {
    fa.hbit = fa.hm8 = 0u;
    uint32_t S = 0u;
    for (int kb = 0; kb < 2; ++kb)
        for (int q = 0; q < 4; ++q) {
            fa.hoff8[kb][q] = 0u;
            if (!((fa.khashed[kb] >> q) & 1u)) continue;
            const LevelDesc& a = g.lv[final_level(kb, 0, q)];
            const LevelDesc& b = g.lv[final_level(kb, 1, q)];
            if (!S) S = a.size;
            if (a.size != S || b.size != S || (S & (S - 1u)) || b.off != a.off + S || a.res > S || b.res > S ||
                (uint64_t)S * 8u > (1ull << 31))
                return;
            fa.hoff8[kb][q] = a.off * 8u;
        }
    if (!S) return;
    fa.hbit = S * 8u;
    fa.hm8 = (S - 1u) * 8u;
}

// The per-render packing launches (grid_mlp fragments, the SAM head's weight
// stream) run unless the caller vouches that the workspace already holds this
// model's packed weights (samnerf_model::reuse_packed); the diagnostic build,
// whose kernel forms switch with the environment, always packs.
bool pack_weights(const samnerf_model* m) {
#ifdef SAMNERF_DIAG_VARIANTS
    return true;
#else
    return m->reuse_packed == 0;
#endif
}

// k_sgrid_box4 packs cell indices and extents into 10 bits
bool box4_ok(const GridDesc<16>& g) {
    for (int l = 0; l < 16; ++l)
        if (g.lv[l].res > 1023u) return false;
    return true;
}

// Proposal gather form: direct by default (packed / auto), the box form for
// SAMNERF_LOOKUP = box / box4.  The box form trades the kernel's 40 corner
// gathers for ~200 VALU instructions of range reduction, box staging and LDS
// addressing per sample; the direct form is only slightly TA-bound (704 TA
// vs 575 VALU cycles per wave) so the box form is slower, 0.88 vs 0.83 ms.
template <int T, bool FIRST>
void launch_prop_sigma(int look, uint32_t N, hipStream_t s, const PropArgs& pa) {
    const uint32_t nb = prop_sigma_blocks<T>(N);
    // the reference's proposal grids with a power-of-two grid scale: the
    // compile-time level classes (SAMNERF_PROP_LAY=0, diagnostic build: the
    // run-time form, for the bit-identity test)
    uint32_t kd = 0, kh = 0;
    for (int l = 0; l < 5; ++l) {
        kd |= (pa.grid.lv[l].flags & kHashed) ? 0u : 1u << l;
        kh |= (pa.grid.lv[l].flags & kHashed) ? 1u << l : 0u;
    }
    const char* pl = diag_env("SAMNERF_PROP_LAY");
    // the LAY forms' byte-offset hash terms need res <= size on hashed levels
    bool small_res = true;
    for (int l = 0; l < 5; ++l)
        if ((pa.grid.lv[l].flags & kHashed) && pa.grid.lv[l].res > pa.grid.lv[l].size) small_res = false;
    const bool lay = (look == kLookPacked || look == kLookAuto) && pa.gs.inv_b2 != 0.0f &&
                     !(pl && atoi(pl) == 0) && small_res && pa.rec;
    const bool lay_ok = lay && ((kd == 0x07u && kh == 0x18u) || (kd == 0x03u && kh == 0x1Cu));
    g_last_forms[T == 128 ? 0 : 1] = lay_ok ? kd | kh << 8 : 0u;
    if (lay && kd == 0x07u && kh == 0x18u) {
        k_prop_sigma<T, FIRST, kLookPacked, 0x07u, 0x18u><<<nb, 256, 0, s>>>(pa);
        return;
    }
    if (lay && kd == 0x03u && kh == 0x1Cu) {
        k_prop_sigma<T, FIRST, kLookPacked, 0x03u, 0x1Cu><<<nb, 256, 0, s>>>(pa);
        return;
    }
    if (look == kLookRef) k_prop_sigma<T, FIRST, kLookRef><<<nb, 256, 0, s>>>(pa);
    else if (look == kLookBox4 && box4_ok(pa.grid))
        k_prop_sigma<T, FIRST, kLookBox4><<<nb, 256, 0, s>>>(pa);
    else k_prop_sigma<T, FIRST, kLookPacked><<<nb, 256, 0, s>>>(pa);
}

// The adaptive mask heads (network.py:143-191, renderer.py:399-434) are
// chains of bias-free Linears on concatenations [intermediate ; m]: linear in
// the per-sample inputs, so sum_k w_k head(x_k) = E . sum_k w_k x_k with E the
// product of the chain, K x 240 (blocks g 32 | h1 64 | h2 64 | o3 16 | v1 32 |
// v2 32).  One block multiplies it out from the output layer back:
// P = W_last W_prev, then per concatenating layer [A | B]: E_block = P A,
// P = P B.  (A reassociation of the reference's layer-by-layer products:
// rounding-level differences.)
struct EffArgs {
    const float* w[8];
    uint32_t K;
    int kind;          // 1 density (6 layers), 2 rgb (8 layers)
    float* aeff;
};

__global__ void __launch_bounds__(256) k_mask_eff(EffArgs a) {
    __shared__ float P[2][32 * 96];
    const int tid = threadIdx.x;
    const int K = (int)a.K, nl = a.kind == 2 ? 8 : 6;
    int cur = 0;
    for (int e = tid; e < K * 96; e += 256) P[0][e] = a.w[nl - 1][e];
    __syncthreads();
    // out[r][c] = sum_i P[r][i] W[i][c0 + c] (W: 96 rows of `ld` columns)
    auto mul = [&](const float* W, int ld, int c0, int nc, float* out, int out_ld) {
        for (int e = tid; e < K * nc; e += 256) {
            const int r = e / nc, c = e % nc;
            float acc = 0.0f;
            for (int i = 0; i < 96; ++i) acc = __builtin_fmaf(P[cur][r * 96 + i], W[i * ld + c0 + c], acc);
            out[r * out_ld + c] = acc;
        }
        __syncthreads();
    };
    auto next = [&](const float* W, int ld, int c0) {
        mul(W, ld, c0, 96, P[cur ^ 1], 96);
        cur ^= 1;
    };
    float* E = a.aeff;
    next(a.w[nl - 2], 96, 0);                            // P = W_last W_{last-1}
    if (a.kind == 2) {
        mul(a.w[5], 128, 0, 32, E + 208, kAeff);         // [v2 | m4]
        next(a.w[5], 128, 32);
        mul(a.w[4], 128, 0, 32, E + 176, kAeff);         // [v1 | m3]
        next(a.w[4], 128, 32);
    } else {
        for (int e = tid; e < K * 64; e += 256) E[(e / 64) * kAeff + 176 + e % 64] = 0.0f;
    }
    mul(a.w[3], 112, 0, 16, E + 160, kAeff);             // [o3 | m2]
    next(a.w[3], 112, 16);
    mul(a.w[2], 160, 0, 64, E + 96, kAeff);              // [h2 | m1]
    next(a.w[2], 160, 64);
    mul(a.w[1], 160, 0, 64, E + 32, kAeff);              // [h1 | m0]
    next(a.w[1], 160, 64);
    mul(a.w[0], 32, 0, 32, E, kAeff);                    // m0 = W0 g
}

// k_final by ray-segment form S and prefetch; EXACT = the exact-fp32
// grid_mlp of head_mode 1.  The non-prefetching forms by segment count:
// N1 compaction between k_final passes: exclusive scan of the waves' open
// counts (popcount of their ballot masks; one workgroup, the waves of the
// pass in order), then each wave's open slots are written at its base in
// lane order: the next list keeps slot order (the image's tile order).
__global__ void __launch_bounds__(1024) k_n1_scan(const uint64_t* __restrict__ mask, const uint32_t* n_in,
                                                  uint32_t n_all, uint32_t* __restrict__ base,
                                                  uint32_t* __restrict__ n_out) {
    __shared__ uint32_t part[1024];
    const uint32_t n = n_in ? *n_in : n_all;
    const uint32_t nw = (n + 31u) / 32u, tid = threadIdx.x;
    const uint32_t per = (nw + 1023u) / 1024u, b0 = tid * per, b1 = min(b0 + per, nw);
    uint32_t sum = 0;
    for (uint32_t i = b0; i < b1; ++i) sum += (uint32_t)__popcll(mask[i]);
    part[tid] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < 1024u; off <<= 1) {          // inclusive scan (Hillis-Steele)
        const uint32_t v = tid >= off ? part[tid - off] : 0u;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    uint32_t run = part[tid] - sum;                           // exclusive
    for (uint32_t i = b0; i < b1; ++i) {
        base[i] = run;
        run += (uint32_t)__popcll(mask[i]);
    }
    if (tid == 1023u) *n_out = part[1023];
}

__global__ void __launch_bounds__(256) k_n1_scatter(const uint64_t* __restrict__ mask,
                                                    const uint32_t* __restrict__ base,
                                                    const uint32_t* __restrict__ list_in,
                                                    const uint32_t* n_in, uint32_t n_all,
                                                    uint32_t* __restrict__ list_out) {
    const uint32_t n = n_in ? *n_in : n_all;
    const uint32_t c = blockIdx.x * 256u + threadIdx.x;       // list entry (32 per wave of k_final)
    if (c >= n) return;
    const uint32_t w = c / 32u, l = c % 32u;
    const uint64_t m = mask[w];
    if (!((m >> l) & 1ull)) return;
    list_out[base[w] + (uint32_t)__popcll(m & ((1ull << l) - 1ull))] = list_in ? list_in[c] : c;
}

// N1: sample chunks of the compacted march (k_final passes; the diagnostic
// build's SAMNERF_N1_CHUNKS).  1 = the wave-level exit alone, the product
// form: on the opaque-sphere 512^2 view the compacted passes measured slower
// -- k_final 0.97 ms in one pass, 1.37 ms in 2 passes (0.61 + 0.77), 1.53 ms
// in 4 (0.32 + 0.35 + 0.54 + 0.31), profiles/r3_n1_compaction.txt: a
// compacted wave's rays come from several 8 x 4 pixel tiles, its gathers
// touch more distinct rows, and each pass re-reads the state and refills
// the weights, while the wave exit keeps every wave's rays neighbours.
inline int n1_chunks() {
    const char* v = diag_env("SAMNERF_N1_CHUNKS");
    const int c = v ? atoi(v) : 1;
    return (c == 1 || c == 2 || c == 4 || c == 8) ? c : 1;
}

template <bool EXACT, bool EXIT, bool GEO, bool SA>
void launch_final_np(int seg, uint32_t N, hipStream_t s, const FinalArgs& fa) {
    if (seg == 1) k_final<32, 1, EXACT, EXIT, GEO, SA><<<xcd_blocks(div_up(N, 128)), 256, 0, s>>>(fa);
    else if (seg == 2) k_final<32, 2, EXACT, EXIT, GEO, SA><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(fa);
    else k_final<32, 4, EXACT, EXIT, GEO, SA><<<xcd_blocks(div_up(N, 32)), 256, 0, s>>>(fa);
}

template <bool EXACT>
void launch_final(int seg, uint32_t N, hipStream_t s, const FinalArgs& fa, bool sa, int ad) {
    g_last_forms[2] = 0u;
    // LAY 1 (the reference grid's compile-time slot layout) wherever the grid
    // matches it and no taps are set; the taps' forms keep the run-time layout
    const bool lay1 = final_layout(fa) == 1 && !fa.sigma_tap && !fa.rows_tap;
    if (ad) {                                            // adaptive mask heads: S = 1
        const uint32_t nb = xcd_blocks(div_up(N, 128));
        g_last_forms[2] = lay1 ? 1u : 0u;
        if (ad == 2) {
            if (lay1) k_final<32, 1, EXACT, false, false, true, 2, 1, false><<<nb, 256, 0, s>>>(fa);
            else k_final<32, 1, EXACT, false, false, true, 2><<<nb, 256, 0, s>>>(fa);
        } else if (sa) {
            if (lay1) k_final<32, 1, EXACT, false, false, true, 1, 1, false><<<nb, 256, 0, s>>>(fa);
            else k_final<32, 1, EXACT, false, false, true, 1><<<nb, 256, 0, s>>>(fa);
        } else {
            if (lay1) k_final<32, 1, EXACT, false, false, false, 1, 1, false><<<nb, 256, 0, s>>>(fa);
            else k_final<32, 1, EXACT, false, false, false, 1><<<nb, 256, 0, s>>>(fa);
        }
        return;
    }
    if (sa) {                                            // --sum_after_mlp (RGB / mask models)
        if (fa.geo_out) launch_final_np<EXACT, false, true, true>(seg, N, s, fa);
        else launch_final_np<EXACT, false, false, true>(seg, N, s, fa);
        return;
    }
    if (fa.geo_out) {                                    // mask model: geo_feat per sample
        if (seg == 1 && lay1) {
            g_last_forms[2] = 1u;
            k_final<32, 1, EXACT, false, true, false, 0, 1, false><<<xcd_blocks(div_up(N, 128)), 256, 0, s>>>(fa);
        } else {
            launch_final_np<EXACT, false, true, false>(seg, N, s, fa);
        }
        return;
    }
    if (fa.exit_depth < INFINITY) {                      // N1 (no prefetch form)
        // a pass marches [p cs, (p + 1) cs) of the TS = 32 / seg steps of each
        // slot (passes over chunks only with seg == 1: n1_passes)
        const int chunks = seg == 1 && fa.n1.list ? n1_chunks() : 1;
        const int cs = (32 / seg) / chunks;
        uint32_t* list[2] = {fa.n1.list, fa.n1.list + N};
        for (int p = 0; p < chunks; ++p) {              // ray compaction between sample chunks
            FinalArgs f = fa;
            f.i0 = p * cs;
            f.i1 = (p + 1) * cs;
            f.list_in = p ? list[(p - 1) & 1] : nullptr;
            f.n_in = p ? fa.n1.cnt + ((p - 1) & 1) : nullptr;
            f.wave_mask = p + 1 < chunks ? fa.n1.mask : nullptr;
            launch_final_np<EXACT, true, false, false>(chunks > 1 ? 1 : seg, N, s, f);
            if (p + 1 < chunks) {
                k_n1_scan<<<1, 1024, 0, s>>>(fa.n1.mask, f.n_in, N, fa.n1.base, fa.n1.cnt + (p & 1));
                k_n1_scatter<<<div_up(N, 256), 256, 0, s>>>(fa.n1.mask, fa.n1.base, f.list_in, f.n_in, N,
                                                            list[p & 1]);
            }
        }
        return;
    }
    // the plain forms: LAY 1 when the grid matches it, TAP only while taps are
    // set (S = 1 only: the taps' renders are whole views; S > 1 tapped renders
    // take the run-time layout)
    const bool tap = fa.sigma_tap || fa.rows_tap;
    const bool lay = final_layout(fa) == 1;
    g_last_forms[2] = lay && (seg == 1 || !tap) ? 1u : 0u;
    const uint32_t nb1 = xcd_blocks(div_up(N, 128)), nb2 = xcd_blocks(div_up(N, 64)),
                   nb4 = xcd_blocks(div_up(N, 32));
    if (seg == 1) {
        if (lay && !tap) k_final<32, 1, EXACT, false, false, false, 0, 1, false><<<nb1, 256, 0, s>>>(fa);
        else if (lay) k_final<32, 1, EXACT, false, false, false, 0, 1, true><<<nb1, 256, 0, s>>>(fa);
        else k_final<32, 1, EXACT><<<nb1, 256, 0, s>>>(fa);
    } else if (seg == 2) {
        if (lay && !tap) k_final<32, 2, EXACT, false, false, false, 0, 1, false><<<nb2, 256, 0, s>>>(fa);
        else k_final<32, 2, EXACT><<<nb2, 256, 0, s>>>(fa);
    } else {
        if (lay && !tap) k_final<32, 4, EXACT, false, false, false, 0, 1, false><<<nb4, 256, 0, s>>>(fa);
        else k_final<32, 4, EXACT><<<nb4, 256, 0, s>>>(fa);
    }
}

Workspace carve(const samnerf_model* m, uint32_t N, void* base) {
    Workspace w;
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t floats) {
        float* q = base ? reinterpret_cast<float*>(p + off) : nullptr;
        off += align256(floats * sizeof(float));
        return q;
    };
    const size_t n = N;
    // the packed weights first: their offsets do not depend on N, so a
    // render of another ray count on the same workspace finds them where
    // the packing render left them (samnerf_model::reuse_packed)
    w.gpack = reinterpret_cast<uint4*>(take((size_t)2 * kFSlots * 64 * 4));
    w.gexp = reinterpret_cast<int*>(take(4));
    w.packed = take(m->with_sam ? sam_head_packed_floats() : 0);
    w.snf = take(2 * n);
    w.rec = reinterpret_cast<float4*>(take(8 * n));
    w.bins1 = take((m->num_steps[1] + 1) * n);
    w.bins2 = take((m->num_steps[2] + 1) * n);
    w.wtmp = take((size_t)std::max(m->num_steps[0], m->num_steps[1]) * n);
    w.u_f = take(3 * (size_t)m->num_steps[2] * n);
    w.w_f = take((size_t)m->num_steps[2] * n);
    w.rows = take((size_t)kRow * n);
    const bool mdef = m->with_mask && m->mask_kind == 0, madapt = m->with_mask && m->mask_kind > 0;
    w.geo_f = take(mdef ? (size_t)16 * m->num_steps[2] * n : 0);
    w.mpacked = take(mdef ? mask_head_packed_floats() : 0);
    w.aeff = take(madapt ? (size_t)32 * kAeff : 0);
    w.mlog = take(madapt ? (size_t)m->mask_out * n : 0);
    w.xsum = take(madapt && m->with_mask == 2 ? (size_t)kAeff * n : 0);   // training renders only
    const bool n1 = m->t_thresh > 0.0f;
    w.n1_list = reinterpret_cast<uint32_t*>(take(n1 ? 2 * n : 0));
    w.n1_cnt = reinterpret_cast<uint32_t*>(take(n1 ? 2 : 0));
    w.n1_mask = reinterpret_cast<uint64_t*>(take(n1 ? 2 * ((n + 31) / 32) : 0));
    w.n1_base = reinterpret_cast<uint32_t*>(take(n1 ? (n + 31) / 32 : 0));
    w.n1_std = reinterpret_cast<double*>(take(n1 ? 6 * n : 0));
    w.n1_stf = take(n1 ? 16 * n : 0);
    w.bytes = off;
    return w;
}

// Parity taps: the final samples' weights and positions, which the render
// keeps in its workspace, copied out after the stages that read them.
int copy_final_taps(const samnerf_taps& tp, const Workspace& w, uint32_t N, hipStream_t s) {
    const size_t n = N;
    if (tp.w2 && hipMemcpyAsync(tp.w2, w.w_f, 32 * n * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "render: copying the w2 tap failed");
    if (tp.u2 && hipMemcpyAsync(tp.u2, w.u_f, 96 * n * sizeof(float), hipMemcpyDeviceToDevice, s) != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "render: copying the u2 tap failed");
    return SAMNERF_OK;
}

int make_grid_desc(const samnerf_grid& g, uint32_t C, uint32_t L, GridDesc<16>& d,
                   const char* name) {
    if (!g.embeddings || !g.offsets_host)
        return fail(SAMNERF_EINVAL, "render: %s has null embeddings/offsets", name);
    if (g.level_dim != C || g.num_levels != L)
        return fail(SAMNERF_EINVAL, "render: %s must be L%u C%u (got L%u C%u)", name, L, C,
                    g.num_levels, g.level_dim);
    const ResTable rt = make_res_table(L, g.S, g.base_resolution);
    d.emb = g.embeddings;
    for (uint32_t l = 0; l < 16; ++l) {
        if (l < L) {
            const uint32_t off = (uint32_t)g.offsets_host[l];
            const uint32_t size = (uint32_t)(g.offsets_host[l + 1] - g.offsets_host[l]);
            d.lv[l] = make_level(off, size, rt.res[l], 0u);
            const bool hashed = d.lv[l].flags & kHashed;
            if (!hashed && (uint64_t)rt.res[l] * rt.res[l] * rt.res[l] > size)
                return fail(SAMNERF_EINVAL, "render: %s level %u is neither dense nor hashed", name, l);
            if (hashed && (size & (size - 1u)))
                return fail(SAMNERF_EINVAL, "render: %s level %u hashes into a non power-of-two table",
                            name, l);
            if ((uint64_t)(off + size) * C * sizeof(float) > (1ull << 32))
                return fail(SAMNERF_EINVAL, "render: %s exceeds 4 GiB (32-bit gather offsets)", name);
        } else {
            d.lv[l] = LevelDesc{0, 1, 1, 0, 1.0f, 0.0f};
        }
    }
    return SAMNERF_OK;
}

}  // namespace

// The proposal stages of a training render (rgb_train.hip): the same kernels
// as samnerf_render_forward's stages 0 and 1, ray order (no tiling), writing
// every intermediate the RGB backward reads to the caller's buffers.
namespace samnerf {

int train_geometry(const samnerf_model* m, TrainGeometry& g) {
    int rc;
    GridDesc<16> d;
    if ((rc = make_grid_desc(m->grid, 2, 16, d, "grid"))) return rc;
    g.grid = d;
    for (int p = 0; p < 2; ++p) {
        if ((rc = make_grid_desc(m->prop[p], 2, 5, d, p ? "prop_encoders.1" : "prop_encoders.0")))
            return rc;
        g.prop[p] = d;
    }
    const GridScale gs = make_grid_scale(m->grid_bound);
    g.bound = gs.bound;
    g.b2 = gs.b2;
    g.inv_b2 = gs.inv_b2;
    return SAMNERF_OK;
}

int proposal_forward(const samnerf_model* m, const TrainGeometry& g, const float* rays_o,
                     const float* rays_d, uint32_t N, const float* cnf, uint32_t n_cnf,
                     const ProposalOut& o, hipStream_t s) {
    PropArgs pa{};
    pa.rays_o = rays_o;
    pa.rays_d = rays_d;
    pa.cnf = cnf;
    pa.N = N;
    {
        const char* ps = diag_env("SAMNERF_PDF_SEQ");
        pa.pdf_seq = ps && atoi(ps) != 0 ? 1u : 0u;
    }
    pa.tiles = RayTiles{0u, 0u, 32u};
    pa.n_cnf = n_cnf;
    for (int i = 0; i < 6; ++i) pa.aabb[i] = m->aabb[i];
    pa.min_near = m->min_near;
    pa.gs = make_grid_scale(m->grid_bound);
    pa.snf = o.snf;
    pa.rec = o.rec;
    pa.grid = g.prop[0];
    pa.W0 = m->prop_mlp[0][0];
    pa.W1 = m->prop_mlp[0][1];
    pa.bins0 = make_lin(0.0f, 1.0f, 129);
    pa.u = make_lin((float)(0.5 / 65), (float)(1.0 - 0.5 / 65), 65);
    pa.pbins0 = m->perturb[0];
    pa.pu = m->perturb[1];
    pa.bins_out = o.bins1;
    pa.wtmp = o.ds0;
    pa.w_out = o.w0;
    k_snf<<<div_up(N, 256), 256, 0, s>>>(pa);
    launch_prop_sigma<128, true>(kLookPacked, N, s, pa);
    k_prop_pdf<128, 65, true><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    pa.grid = g.prop[1];
    pa.W0 = m->prop_mlp[1][0];
    pa.W1 = m->prop_mlp[1][1];
    pa.u = make_lin((float)(0.5 / 33), (float)(1.0 - 0.5 / 33), 33);
    pa.pu = m->perturb[2];
    pa.bins_in = o.bins1;
    pa.bins_out = o.bins2;
    pa.wtmp = o.ds1;
    pa.w_out = o.w1;
    launch_prop_sigma<64, false>(kLookPacked, N, s, pa);
    k_prop_pdf<64, 33, false><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    return check_launch("proposal_forward");
}

}  // namespace samnerf

extern "C" {

int samnerf_get_rays(const float* pose, float fx, float fy, float cx, float cy, uint32_t H,
                     uint32_t W, uint32_t row0, uint32_t rows, float* rays_o, float* rays_d,
                     samnerf_stream_t stream) {
    if (!pose || !rays_o || !rays_d) return fail(SAMNERF_EINVAL, "get_rays: null pointer");
    if (row0 + rows > H) return fail(SAMNERF_EINVAL, "get_rays: rows out of range");
    const uint32_t n = rows * W;
    if (n == 0) return SAMNERF_OK;
    k_get_rays<<<div_up(n, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        pose[0], pose[1], pose[2], pose[4], pose[5], pose[6], pose[8], pose[9], pose[10], pose[3],
        pose[7], pose[11], fx, fy, cx, cy, W, row0, n, rays_o, rays_d);
    return check_launch("get_rays");
}

int samnerf_near_far(const float* rays_o, const float* rays_d, uint32_t N, const float* aabb,
                     float min_near, float* nears, float* fars, samnerf_stream_t stream) {
    if (!rays_o || !rays_d || !aabb || !nears || !fars)
        return fail(SAMNERF_EINVAL, "near_far: null pointer");
    if (N == 0) return SAMNERF_OK;
    Aabb box;
    for (int i = 0; i < 6; ++i) box.v[i] = aabb[i];
    k_near_far<<<div_up(N, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        rays_o, rays_d, N, box, min_near, nears, fars);
    return check_launch("near_far");
}

int samnerf_contract(const float* x, float* z, uint32_t N, samnerf_stream_t stream) {
    if (!x || !z) return fail(SAMNERF_EINVAL, "contract: null pointer");
    if (N == 0) return SAMNERF_OK;
    k_contract<<<div_up(N, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(x, z, N);
    return check_launch("contract");
}

int samnerf_sample_pdf(const float* bins, const float* weights, uint32_t N, uint32_t T0,
                       uint32_t T, float* out, int32_t* inds, samnerf_stream_t stream) {
    if (!bins || !weights || !out) return fail(SAMNERF_EINVAL, "sample_pdf: null pointer");
    if (T0 == 0 || T == 0) return fail(SAMNERF_EINVAL, "sample_pdf: empty bins");
    if (N == 0) return SAMNERF_OK;
    // renderer.py:97: u = linspace(0.5 / T, 1 - 0.5 / T, T), bounds from Python doubles
    const Lin u = make_lin((float)(0.5 / T), (float)(1.0 - 0.5 / T), T);
    k_sample_pdf<<<div_up(N, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        bins, weights, N, T0, T, u, out, inds);
    return check_launch("sample_pdf");
}

int samnerf_composite_weights(const float* real_bins, const float* sigmas, uint32_t N, uint32_t T,
                              float* weights, samnerf_stream_t stream) {
    if (!real_bins || !sigmas || !weights) return fail(SAMNERF_EINVAL, "composite: null pointer");
    if (N == 0 || T == 0) return SAMNERF_OK;
    k_composite<<<div_up(N, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        real_bins, sigmas, N, T, weights);
    return check_launch("composite_weights");
}

size_t samnerf_render_workspace_size(const samnerf_model* model, uint32_t N) {
    if (!model) return 0;
    return carve(model, N, nullptr).bytes;
}

}  // extern "C"

namespace {

// Where the per-ray outputs go: separate arrays (samnerf_render_forward) or
// the rows of one gather tile (samnerf_render_forward_tile).
struct OutLayout {
    float* image;
    float* depth;
    float* wsum;
    float* samvit;
    uint32_t img_ld, scal_ld, sv_ld;
};

int render_impl(const samnerf_model* m, const float* rays_o, const float* rays_d, uint32_t N,
                const float* cam_near_far, uint32_t n_cnf, float bg_color, const OutLayout& ol,
                float* feature_rows, void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    float* const image = ol.image;
    float* const depth = ol.depth;
    float* const weights_sum = ol.wsum;
    float* const samvit = ol.samvit;
    if (m->num_steps[0] != 128 || m->num_steps[1] != 64 || m->num_steps[2] != 32)
        return fail(SAMNERF_EINVAL, "render: fused path is built for num_steps = [128, 64, 32]");
    // with_sam and samvit == NULL: the caller does not want the features
    // (renderer.py computes them and drops them when return_feats == 0), so the
    // s_grid composite runs only if feature_rows are requested and the head not
    // at all
    if (cam_near_far && n_cnf != 1 && n_cnf != N)
        return fail(SAMNERF_EINVAL, "render: cam_near_far must have 1 or N rows");
    if (!m->perturb[0] != !m->perturb[1] || !m->perturb[0] != !m->perturb[2])
        return fail(SAMNERF_EINVAL, "render: perturb needs all three position arrays or none");
    Workspace w = carve(m, N, workspace);
    if (!workspace || workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "render: workspace needs %zu bytes, got %zu", w.bytes,
                    workspace_bytes);
    for (int i = 0; i < 3; ++i)
        if (!m->grid_mlp[i] || !m->view_mlp[i]) return fail(SAMNERF_EINVAL, "render: null MLP weight");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    float* rows = feature_rows ? feature_rows : w.rows;

    GridDesc<16> gp0, gp1, gg, gs;
    int rc;
    if ((rc = make_grid_desc(m->prop[0], 2, 5, gp0, "prop_encoders.0"))) return rc;
    if ((rc = make_grid_desc(m->prop[1], 2, 5, gp1, "prop_encoders.1"))) return rc;
    if ((rc = make_grid_desc(m->grid, 2, 16, gg, "grid"))) return rc;
    if (m->with_sam && (rc = make_grid_desc(m->s_grid, 8, 16, gs, "s_grid"))) return rc;

    const uint32_t nb = div_up(N, 256);
    // (parity taps: the tapped intermediates stay in slot order, the caller
    // maps slots to rays -- fused.py ray_of_slots -- so the taps see the
    // product's tiled launch)
    const RayTiles tiles = make_ray_tiles(N, m->view_width);
    PropArgs pa{};
    pa.rays_o = rays_o;
    pa.rays_d = rays_d;
    pa.cnf = cam_near_far;
    pa.N = N;
    {
        const char* ps = diag_env("SAMNERF_PDF_SEQ");
        pa.pdf_seq = ps && atoi(ps) != 0 ? 1u : 0u;
    }
    pa.tiles = tiles;
    pa.n_cnf = n_cnf;
    for (int i = 0; i < 6; ++i) pa.aabb[i] = m->aabb[i];
    pa.min_near = m->min_near;
    pa.gs = make_grid_scale(m->grid_bound);
    pa.snf = w.snf;
    pa.rec = w.rec;
    pa.wtmp = w.wtmp;
    // parity taps (samnerf_set_taps): the stages write their intermediates to
    // the caller's buffers instead of the workspace; the kernels are the same
    if (g_taps_on && g_taps_n != N)
        return fail(SAMNERF_EINVAL, "render: taps were set for %u rays, the call renders %u", g_taps_n, N);
    const samnerf_taps tp = g_taps_on ? g_taps : samnerf_taps{};
    float* const bins1 = tp.bins1 ? tp.bins1 : w.bins1;
    float* const bins2 = tp.bins2 ? tp.bins2 : w.bins2;

    // stage 0: 128 uniform samples -> 65 bins (renderer.py:263-267, :274-275)
    pa.grid = gp0;
    pa.W0 = m->prop_mlp[0][0];
    pa.W1 = m->prop_mlp[0][1];
    pa.bins0 = make_lin(0.0f, 1.0f, 129);
    pa.u = make_lin((float)(0.5 / 65), (float)(1.0 - 0.5 / 65), 65);
    pa.bins_in = nullptr;
    pa.pbins0 = m->perturb[0];
    pa.pu = m->perturb[1];
    pa.bins_out = bins1;
    pa.wtmp = tp.ds0 ? tp.ds0 : w.wtmp;
    pa.inds_out = tp.inds1;
    pa.w_out = tp.w0;
    const int look = lookup_mode();
    mark_stage(0, s);
    k_snf<<<div_up(N, 256), 256, 0, s>>>(pa);
    // SAMNERF_PROP_FUSED=1: one kernel per proposal stage, ds kept in LDS
    // (k_prop_fused; bit-identical, but measured 1.9x slower -- prop0 1.10 vs
    // 0.59 ms per view -- so the two-kernel form stays the default)
    const char* pfv = diag_env("SAMNERF_PROP_FUSED");
    const bool pfused = !g_taps_on && look == kLookAuto && pfv && pfv[0] == '1';
    if (pfused) {
        k_prop_fused<128, 65, true><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    } else {
        launch_prop_sigma<128, true>(look, N, s, pa);
        k_prop_pdf<128, 65, true><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    }

    // stage 1: 64 samples -> 33 bins
    pa.grid = gp1;
    pa.W0 = m->prop_mlp[1][0];
    pa.W1 = m->prop_mlp[1][1];
    pa.u = make_lin((float)(0.5 / 33), (float)(1.0 - 0.5 / 33), 33);
    pa.pu = m->perturb[2];
    pa.bins_in = bins1;
    pa.bins_out = bins2;
    pa.wtmp = tp.ds1 ? tp.ds1 : w.wtmp;
    pa.inds_out = tp.inds2;
    pa.w_out = tp.w1;
    mark_stage(1, s);
    if (pfused) {
        k_prop_fused<64, 33, false><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    } else {
        launch_prop_sigma<64, false>(look, N, s, pa);
        k_prop_pdf<64, 33, false><<<xcd_blocks(div_up(N, 64)), 256, 0, s>>>(pa);
    }

    // stage 2: 32 samples through the full network
    FinalArgs fa{};
    fa.rays_o = rays_o;
    fa.rays_d = rays_d;
    fa.N = N;
    fa.tiles = tiles;
    fa.gs = make_grid_scale(m->grid_bound);
    fa.bg = bg_color;
    fa.grid = gg;
    fa.grid_emb = gg.emb;
    // slot q of k-block kb holds levels final_level(kb, 0 / 1, q): dense in
    // both half-waves -> pair loads, hashed in both -> select-free rows
    for (int kb = 0; kb < 2; ++kb) {
        fa.kdense[kb] = fa.khashed[kb] = 0u;
        for (int q = 0; q < 4 && final_classes(); ++q) {
            const bool ha = gg.lv[final_level(kb, 0, q)].flags & kHashed;
            const bool hb = gg.lv[final_level(kb, 1, q)].flags & kHashed;
            fa.kdense[kb] |= (!ha && !hb) ? 1u << q : 0u;
            fa.khashed[kb] |= (ha && hb) ? 1u << q : 0u;
        }
    }
    set_hash_slots(fa, gg);
    fa.G0 = m->grid_mlp[0];
    fa.G1 = m->grid_mlp[1];
    fa.G2 = m->grid_mlp[2];
    fa.V0 = m->view_mlp[0];
    fa.V1 = m->view_mlp[1];
    fa.V2 = m->view_mlp[2];
    fa.bins_in = bins2;
    fa.snf = w.snf;
    fa.u_out = w.u_f;
    fa.w_out = w.w_f;
    fa.image = image;
    fa.depth = depth;
    fa.wsum = weights_sum;
    fa.img_ld = ol.img_ld;
    fa.scal_ld = ol.scal_ld;
    if (!(m->t_thresh >= 0.0f && m->t_thresh < 1.0f))
        return fail(SAMNERF_EINVAL, "render_forward: t_thresh %g outside [0, 1)", (double)m->t_thresh);
    fa.exit_depth = m->t_thresh > 0.0f ? -logf(m->t_thresh) : INFINITY;
    if (tp.row_stride == 0 && (tp.rows2 || tp.srows))
        return fail(SAMNERF_EINVAL, "render: taps rows2 / srows need row_stride > 0");
    fa.sigma_tap = tp.sigma2;
    fa.rows_tap = tp.rows2;
    fa.tap_stride = tp.row_stride ? tp.row_stride : 1u;
    fa.i0 = 0;
    fa.i1 = 32;                                          // steps per slot, 32 / seg (set below; EXIT only)
    if (m->t_thresh > 0.0f) {                            // N1: ray compaction buffers (k_final passes)
        fa.n1.list = w.n1_list;
        fa.n1.cnt = w.n1_cnt;
        fa.n1.mask = w.n1_mask;
        fa.n1.base = w.n1_base;
        fa.st_d = w.n1_std;
        fa.st_f = w.n1_stf;
    }
    int ad = 0;
    if (m->with_mask) {
        if (m->t_thresh > 0.0f)
            return fail(SAMNERF_EINVAL, "render_forward: the mask head and t_thresh do not combine");
        if (m->mask_kind < 0 || m->mask_kind > 2)
            return fail(SAMNERF_EINVAL, "render_forward: mask_kind %d", m->mask_kind);
        if (m->mask_out < 1 || m->mask_out > 32)
            return fail(SAMNERF_EINVAL, "render_forward: mask_out %u outside 1..32", m->mask_out);
        const int nl = m->mask_kind == 0 ? 3 : m->mask_kind == 1 ? 6 : 8;
        for (int i = 0; i < nl; ++i)
            if (!m->mask_w[i]) return fail(SAMNERF_EINVAL, "render_forward: null mask_mlp weight %d", i);
        if (m->mask_kind == 0) {
            fa.geo_out = w.geo_f;
        } else {
            if (m->mask_kind == 2 && !m->sum_after_mlp)
                return fail(SAMNERF_EINVAL, "render_forward: the adaptive 'rgb' head needs sum_after_mlp");
            EffArgs ea{};
            for (int i = 0; i < nl; ++i) ea.w[i] = m->mask_w[i];
            ea.K = m->mask_out;
            ea.kind = m->mask_kind;
            ea.aeff = w.aeff;
            k_mask_eff<<<1, 256, 0, s>>>(ea);
            fa.aeff = w.aeff;
            fa.mlog = w.mlog;
            fa.xsum = m->with_mask == 2 ? w.xsum : nullptr;   // training render: the head's inputs
            fa.mask_out = m->mask_out;
            ad = m->mask_kind;
        }
    }
    const bool sam_rows = m->with_sam && (samvit || feature_rows);
    fa.rows = sam_rows || feature_rows ? rows : nullptr;
    mark_stage(2, s);
    // segments per ray: enough waves to fill the resident slots (2 per SIMD)
    // (SAMNERF_FINAL_S = 1 | 2 | 4 overrides, for measurement)
    const char* fs = diag_env("SAMNERF_FINAL_S");
    // N1's compaction passes (diagnostic build) need whole rays: one segment
    const bool n1_passes = m->t_thresh > 0.0f && n1_chunks() > 1;
    const int seg = fs ? atoi(fs) : (n1_passes || N >= 65536u ? 1 : N >= 32768u ? 2 : 4);
    fa.i1 = 32 / seg;
    if (m->sum_after_mlp && (m->t_thresh > 0.0f || sam_rows))
        return fail(SAMNERF_EINVAL, "render_forward: sum_after_mlp renders RGB (+ mask) only: no SAM "
                    "features (the reference's branch crashes, SURVEY 0.2) and no t_thresh");
    if (m->head_mode == 1) {
        launch_final<true>(seg, N, s, fa, m->sum_after_mlp != 0, ad);
    } else {
        fa.gpack = w.gpack;
        fa.gexp = w.gexp;
        if (pack_weights(m)) k_pack_grid_mlp<<<1, 256, 0, s>>>(fa, w.gpack, w.gexp);
        launch_final<false>(seg, N, s, fa, m->sum_after_mlp != 0, ad);
    }

    if (sam_rows) {
        SgridArgs sa{};
        sa.N = N;
        sa.tiles = tiles;
        sa.grid = gs;
        sa.u_in = w.u_f;
        sa.w_in = w.w_f;
        sa.rows = rows;
        sa.rows_tap = tp.srows;
        sa.tap_stride = tp.row_stride ? tp.row_stride : 1u;
        {
            const char* pp = diag_env("SAMNERF_SGRID_PATHS");
            sa.paths = pp ? reinterpret_cast<unsigned long long*>(strtoull(pp, nullptr, 16)) : nullptr;
        }
        mark_stage(3, s);
        const dim3 sg(xcd_blocks(div_up(N, 64)), 16);
        const dim3 sb(xcd_blocks(div_up(N, 64)), 4);
        if (look == kLookRef) {
            k_sgrid<32, kLookRef><<<sg, 256, 0, s>>>(sa);
        } else if ((look == kLookBox4 || (look == kLookAuto && N >= kBox4MinRays)) && box4_ok(gs) &&
                   (uint64_t)N * 384u < (1ull << 32)) {
            if (sa.rows_tap) k_sgrid_box4<32, true><<<sb, 256, 0, s>>>(sa);
            else k_sgrid_box4<32><<<sb, 256, 0, s>>>(sa);
        } else {
            k_sgrid<32, kLookPacked><<<sg, 256, 0, s>>>(sa);
        }
        if ((rc = check_launch("render"))) return rc;
        mark_stage(4, s);
        if (samvit) rc = sam_head_forward(m, rows, N, samvit, w.packed, s, ol.sv_ld, pack_weights(m));
        mark_stage(5, s);
        if (rc == SAMNERF_OK) rc = copy_final_taps(tp, w, N, s);
        return rc;
    }
    mark_stage(3, s);
    mark_stage(4, s);
    mark_stage(5, s);
    if ((rc = check_launch("render"))) return rc;
    return copy_final_taps(tp, w, N, s);
}

}  // namespace

extern "C" {

int samnerf_render_forward(const samnerf_model* m, const float* rays_o, const float* rays_d,
                           uint32_t N, const float* cam_near_far, uint32_t n_cnf, float bg_color,
                           float* image, float* depth, float* weights_sum, float* samvit,
                           float* feature_rows, void* workspace, size_t workspace_bytes,
                           samnerf_stream_t stream) {
    // N = 0 is a no-op whatever the buffers (an empty torch tensor has a null
    // data pointer)
    if (!m) return fail(SAMNERF_EINVAL, "render: null pointer");
    if (N == 0) return SAMNERF_OK;
    if (!rays_o || !rays_d || !image || !depth || !weights_sum)
        return fail(SAMNERF_EINVAL, "render: null pointer");
    const OutLayout ol{image, depth, weights_sum, samvit, 3u, 1u, 256u};
    return render_impl(m, rays_o, rays_d, N, cam_near_far, n_cnf, bg_color, ol, feature_rows, workspace,
                       workspace_bytes, stream);
}

int samnerf_render_forward_tile(const samnerf_model* m, const float* rays_o, const float* rays_d,
                                uint32_t N, const float* cam_near_far, uint32_t n_cnf, float bg_color,
                                float* tile, uint32_t ld, int feats, float* feature_rows, void* workspace,
                                size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m) return fail(SAMNERF_EINVAL, "render_tile: null pointer");
    if (N == 0) return SAMNERF_OK;
    if (!rays_o || !rays_d || !tile) return fail(SAMNERF_EINVAL, "render_tile: null pointer");
    const bool sv = feats && m->with_sam;
    if (ld < (sv ? 261u : 5u))
        return fail(SAMNERF_EINVAL, "render_tile: row of %u floats cannot hold the outputs (needs %u)", ld,
                    sv ? 261u : 5u);
    const OutLayout ol{tile, tile + 3, tile + 4, sv ? tile + 5 : nullptr, ld, ld, ld};
    return render_impl(m, rays_o, rays_d, N, cam_near_far, n_cnf, bg_color, ol, feature_rows, workspace,
                       workspace_bytes, stream);
}

int samnerf_set_stage_events(void* const* events, uint32_t n) {
    if (n > 8) return fail(SAMNERF_EINVAL, "set_stage_events: at most 8 events");
    g_n_stage_events = events ? n : 0u;
    for (uint32_t i = 0; i < g_n_stage_events; ++i)
        g_stage_events[i] = reinterpret_cast<hipEvent_t>(events[i]);
    return SAMNERF_OK;
}

int samnerf_last_forms(uint32_t* out, uint32_t n) {
    for (uint32_t i = 0; out && i < n && i < 4; ++i) out[i] = g_last_forms[i];
    return 4;
}

int samnerf_clock_stamp(uint64_t* out, samnerf_stream_t stream) {
    if (!out) return fail(SAMNERF_EINVAL, "clock_stamp: null pointer");
    k_clock_stamp<<<256, 64, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        reinterpret_cast<unsigned long long*>(out));
    return check_launch("clock_stamp");
}

int samnerf_set_taps(const samnerf_taps* taps, uint32_t N) {
    g_taps_on = taps != nullptr;
    g_taps = taps ? *taps : samnerf_taps{};
    g_taps_n = taps ? N : 0u;
    return SAMNERF_OK;
}

int samnerf_mask_forward(const samnerf_model* m, uint32_t N, float* logits, const void* workspace,
                         size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m) return fail(SAMNERF_EINVAL, "mask_forward: null model");
    if (!m->with_mask) return fail(SAMNERF_EINVAL, "mask_forward: model has no mask head (with_mask = 0)");
    if (N == 0) return SAMNERF_OK;
    if (!logits || !workspace) return fail(SAMNERF_EINVAL, "mask_forward: null pointer");
    if (m->mask_out < 1 || m->mask_out > 32)
        return fail(SAMNERF_EINVAL, "mask_forward: mask_out %u outside 1..32", m->mask_out);
    if (m->num_steps[2] != 32) return fail(SAMNERF_EINVAL, "mask_forward: fused path is built for 32 final samples");
    Workspace w = carve(m, N, const_cast<void*>(workspace));
    if (workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "mask_forward: workspace needs %zu bytes, got %zu", w.bytes,
                    workspace_bytes);
    if (m->mask_kind != 0) {                            // adaptive: k_final wrote them
        if (hipMemcpyAsync(logits, w.mlog, sizeof(float) * m->mask_out * (size_t)N, hipMemcpyDeviceToDevice,
                           reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
            return fail(SAMNERF_ELAUNCH, "mask_forward: copy failed");
        return SAMNERF_OK;
    }
    for (int i = 0; i < 3; ++i)
        if (!m->mask_w[i]) return fail(SAMNERF_EINVAL, "mask_forward: null mask_mlp weight");
    GridDesc<16> gm;
    int rc = make_grid_desc(m->m_grid, 8, 16, gm, "m_grid");
    if (rc) return rc;
    const RayTiles tiles = make_ray_tiles(N, m->view_width);
    return mask_head_forward(m, gm, w.u_f, w.w_f, w.geo_f, N, logits, tiles, w.mpacked,
                             reinterpret_cast<hipStream_t>(stream));
}

size_t samnerf_mask_train_workspace_size(uint32_t N) { return mask_train_workspace_bytes(N); }

size_t samnerf_mask_train_workspace_size_model(const samnerf_model* m, uint32_t N) {
    if (!m || !m->with_mask || m->mask_kind < 0 || m->mask_kind > 2) return mask_train_workspace_bytes(N);
    return mask_train_workspace_bytes(m->mask_kind, N);
}

// the render workspace's final samples of a 'default' mask model, checked
static int mask_train_inputs(const samnerf_model* m, uint32_t N, const void* render_ws, size_t render_bytes,
                             Workspace& w, GridDesc<16>& gm, const char* what) {
    if (!m) return fail(SAMNERF_EINVAL, "%s: null model", what);
    if (!m->with_mask || m->mask_kind < 0 || m->mask_kind > 2)
        return fail(SAMNERF_EINVAL, "%s: model has no fused mask head (with_mask = 1, mask_kind 0-2)", what);
    if (m->mask_out < 1 || m->mask_out > 32)
        return fail(SAMNERF_EINVAL, "%s: mask_out %u outside 1..32", what, m->mask_out);
    if (m->num_steps[2] != 32) return fail(SAMNERF_EINVAL, "%s: fused path is built for 32 final samples", what);
    if (!render_ws) return fail(SAMNERF_EINVAL, "%s: null render workspace", what);
    w = carve(m, N, const_cast<void*>(render_ws));
    if (render_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "%s: render workspace needs %zu bytes, got %zu", what, w.bytes,
                    render_bytes);
    if (m->mask_kind != 0 && m->with_mask != 2)
        return fail(SAMNERF_EINVAL, "%s: the adaptive heads train on a render with with_mask = 2 (it keeps "
                    "the per-ray input sums)", what);
    return m->mask_kind == 0 ? make_grid_desc(m->m_grid, 8, 16, gm, "m_grid") : SAMNERF_OK;
}

int samnerf_mask_train_forward(const samnerf_model* m, uint32_t N, float* logits, const void* render_ws,
                               size_t render_bytes, void* workspace, size_t workspace_bytes,
                               samnerf_stream_t stream) {
    Workspace w;
    GridDesc<16> gm;
    int rc = mask_train_inputs(m, N, render_ws, render_bytes, w, gm, "mask_train_forward");
    if (rc) return rc;
    if (N == 0) return SAMNERF_OK;
    if (!logits || !workspace) return fail(SAMNERF_EINVAL, "mask_train_forward: null pointer");
    if (m->mask_kind != 0)                               // adaptive: the chain on the per-ray sums
        return adaptive_train_forward(m, w.xsum, N, logits, workspace, workspace_bytes,
                                      reinterpret_cast<hipStream_t>(stream));
    const RayTiles tiles = make_ray_tiles(N, m->view_width);
    return mask_train_forward(m, gm, w.u_f, w.w_f, w.geo_f, N, tiles, logits, workspace, workspace_bytes,
                              reinterpret_cast<hipStream_t>(stream));
}

int samnerf_mask_train_backward(const samnerf_model* m, uint32_t N, const float* grad_logits,
                                float* const* grad_mask_w, float* grad_m_grid, const void* render_ws,
                                size_t render_bytes, void* workspace, size_t workspace_bytes,
                                samnerf_stream_t stream) {
    Workspace w;
    GridDesc<16> gm;
    int rc = mask_train_inputs(m, N, render_ws, render_bytes, w, gm, "mask_train_backward");
    if (rc) return rc;
    if (N == 0) return SAMNERF_OK;
    if (!grad_logits || !grad_mask_w || !workspace)
        return fail(SAMNERF_EINVAL, "mask_train_backward: null pointer");
    if (m->mask_kind != 0)                               // adaptive: no grid gradient (all inputs detached)
        return adaptive_train_backward(m, w.xsum, N, grad_logits, grad_mask_w, workspace, workspace_bytes,
                                       reinterpret_cast<hipStream_t>(stream));
    if (!grad_m_grid) return fail(SAMNERF_EINVAL, "mask_train_backward: null m_grid gradient");
    for (int i = 0; i < 3; ++i)
        if (!grad_mask_w[i]) return fail(SAMNERF_EINVAL, "mask_train_backward: null gradient");
    const RayTiles tiles = make_ray_tiles(N, m->view_width);
    return mask_train_backward(m, gm, w.u_f, w.w_f, w.geo_f, N, tiles, grad_logits, grad_mask_w, grad_m_grid,
                               workspace, workspace_bytes, reinterpret_cast<hipStream_t>(stream));
}

// rows of the s_grid table (the deterministic backward's accumulator holds 8
// int64 per row, then an 8-entry header)
static uint64_t sgrid_rows(const samnerf_model* m) {
    return m && m->with_sam && m->s_grid.offsets_host ? (uint64_t)m->s_grid.offsets_host[m->s_grid.num_levels]
                                                      : 0u;
}

size_t samnerf_sgrid_accum_size(const samnerf_model* m) {
    const uint64_t rows = sgrid_rows(m);
    return rows ? (size_t)(rows * 8u + 8u) * sizeof(int64_t) : 0u;
}

int samnerf_sgrid_backward_det(const samnerf_model* m, const float* grad_fsam, uint32_t N,
                               float* grad_embeddings, int64_t* accum, size_t accum_bytes,
                               const void* workspace, size_t workspace_bytes, samnerf_stream_t stream) {
    if (!m || !grad_fsam || !grad_embeddings || !workspace || !accum)
        return fail(SAMNERF_EINVAL, "sgrid_backward_det: null pointer");
    if (!m->with_sam) return fail(SAMNERF_EINVAL, "sgrid_backward_det: model has no s_grid");
    Workspace w = carve(m, N, const_cast<void*>(workspace));
    if (workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "sgrid_backward_det: workspace too small");
    if (accum_bytes < samnerf_sgrid_accum_size(m))
        return fail(SAMNERF_EWORKSPACE, "sgrid_backward_det: accumulator needs %zu bytes, got %zu",
                    samnerf_sgrid_accum_size(m), accum_bytes);
    if (N == 0) return SAMNERF_OK;
    GridDesc<16> gs;
    int rc = make_grid_desc(m->s_grid, 8, 16, gs, "s_grid");
    if (rc) return rc;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uint64_t n = sgrid_rows(m) * 8u;
    DetAcc det;
    det.acc = reinterpret_cast<unsigned long long*>(accum);
    uint32_t* hdr = reinterpret_cast<uint32_t*>(accum + n);
    det.hdr = hdr;
    det.log2n = 0;
    while ((1ull << det.log2n) < (uint64_t)N) ++det.log2n;
    if (hipMemsetAsync(hdr, 0, 2 * sizeof(uint32_t), s) != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "sgrid_backward_det: header reset failed");
    k_sgrid_det_max<<<div_up((uint64_t)N * 32u, 256), 256, 0, s>>>(grad_fsam, N, kRow, hdr);
    k_sgrid_backward<32, true><<<dim3(div_up((uint64_t)N * 8, 256), 16, 1), 256, 0, s>>>(
        N, make_ray_tiles(N, m->view_width), gs, w.u_f, w.w_f, grad_fsam, kRow, grad_embeddings, 0u, 0u, det);
    k_sgrid_det_finish<<<2048, 256, 0, s>>>(det, grad_embeddings, n);
    return check_launch("sgrid_backward_det");
}

int samnerf_sgrid_backward(const samnerf_model* m, const float* grad_fsam, uint32_t N,
                           float* grad_embeddings, const void* workspace, size_t workspace_bytes,
                           samnerf_stream_t stream) {
    if (!m || !grad_fsam || !grad_embeddings || !workspace)
        return fail(SAMNERF_EINVAL, "sgrid_backward: null pointer");
    if (!m->with_sam) return fail(SAMNERF_EINVAL, "sgrid_backward: model has no s_grid");
    Workspace w = carve(m, N, const_cast<void*>(workspace));
    if (workspace_bytes < w.bytes)
        return fail(SAMNERF_EWORKSPACE, "sgrid_backward: workspace too small");
    if (N == 0) return SAMNERF_OK;
    GridDesc<16> gs;
    int rc = make_grid_desc(m->s_grid, 8, 16, gs, "s_grid");
    if (rc) return rc;
    for (int l = 0; l < 16; ++l)       // box cells carry row << 6 | cell in 32 bits
        if (gs.lv[l].size > (1u << 26))
            return fail(SAMNERF_EINVAL, "sgrid_backward: level %d has more than 2^26 rows", l);
    // SAMNERF_SGRID_BWD=box: the LDS-box aggregation (A/B and tests; measured
    // slower than the per-corner atomics, 0.70 vs 0.56 ms per cfg-5 step, so
    // not the default); SAMNERF_SGRID_BWD_SPLIT: sample groups per ray
    // (blockIdx.z; 1 = the round-1 form, 4-16 measured no faster)
    // SAMNERF_SGRID_BWD=run: the along-ray merge on every level
    // (SAMNERF_SGRID_RUN_RES: up to this level resolution).  Measured slower on
    // a cfg-5 step: 1.29 ms per step with the per-corner form, 1.62 with the
    // merge on every level, 1.50 on levels up to res 64 (tools/r2/gpu_r2s3n.sh):
    // a wave's 8 neighbouring rays share corner rows at one sample index (the
    // butterfly) more often than consecutive samples of one ray do, and the
    // merge gives the butterfly up.  Kept selectable and tested.
    const char* mode = diag_env("SAMNERF_SGRID_BWD");
    const uint32_t max_cells = (mode && !strcmp(mode, "box")) ? kBwdBoxCells : 0u;
    const char* rr = diag_env("SAMNERF_SGRID_RUN_RES");
    uint32_t run_res = rr ? (uint32_t)atoi(rr) : 0u;
    if (mode && !strcmp(mode, "run") && !rr) run_res = 0xFFFFFFFFu;
    const char* sp = diag_env("SAMNERF_SGRID_BWD_SPLIT");
    const uint32_t split = sp ? (uint32_t)std::max(1, std::min(32, atoi(sp))) : 1u;
    k_sgrid_backward<32><<<dim3(div_up((uint64_t)N * 8, 256), 16, split), 256, 0,
                           reinterpret_cast<hipStream_t>(stream)>>>(N, make_ray_tiles(N, m->view_width),
                                                                     gs, w.u_f, w.w_f, grad_fsam,
                                                                     kRow, grad_embeddings, max_cells,
                                                                     run_res);
    return check_launch("sgrid_backward");
}

}  // extern "C"
