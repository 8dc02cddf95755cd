// samnerf_common.h -- shared host/device helpers for the gfx950 HIP library.
//
// Error convention of the C ABI (include/samnerf_hip.h): every entry point
// returns 0 on success or a negative SAMNERF_E* code and records a message
// retrievable with samnerf_last_error().  Argument errors mirror the
// reference's TORCH_CHECK / std::runtime_error messages
// (gridencoder/src/gridencoder.cu:15-18, :392, :409).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#include "../../include/samnerf_hip.h"

namespace samnerf {

int fail(int code, const char* fmt, ...);

// A/B variant switches of the kernels (the bit-identity tests' alternative
// forms and the measured-slower variants): read from the environment only in
// the diagnostic build (-DSAMNERF_DIAG_VARIANTS, libsamnerf_hip_diag.so, which
// build.py makes beside the product library for the tests).  The product
// library ignores the environment: one path per configuration.
inline const char* diag_env(const char* name) {
#ifdef SAMNERF_DIAG_VARIANTS
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}
int check_launch(const char* what);

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Hash primes of the coherent spatial hash (gridencoder.cu:49).
constexpr uint32_t kPrime1 = 2654435761u;
constexpr uint32_t kPrime2 = 805459861u;
constexpr uint32_t kPrimes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                 2097192037u, 1434869437u, 2165219737u};

// Indexing resolution per level, float formula of gridencoder.cu:133.  Host
// side so the device never evaluates exp2f (which only needs to be exact on
// integral arguments, SURVEY.md H4, but this removes the question).
struct ResTable {
    uint32_t res[32];
};
ResTable make_res_table(uint32_t L, float S, uint32_t H);

// One level of a hash grid, fully resolved on the host (fused path).
struct LevelDesc {
    uint32_t off;      // first row of the level in the embeddings table
    uint32_t size;     // rows in the level
    uint32_t res;      // indexing resolution
    uint32_t flags;    // bit0: hashed, bit1: size is a power of two
    float fres, ftop;  // (float)res, (float)(res - 1): no per-lane conversions
};
constexpr uint32_t kHashed = 1u, kPow2 = 2u;

// Level geometry exactly as gridencoder.cu:61-79 decides it for D = 3: the
// dense row index uses strides 1, res, res^2 while the running stride fits the
// table; a hash grid whose stride outgrows the table hashes instead.
LevelDesc make_level(uint32_t off, uint32_t size, uint32_t res, uint32_t gridtype);

template <int MAXL>
struct GridDesc {
    const float* emb;
    LevelDesc lv[MAXL];
};

// What the RGB training step (rgb_train.hip) takes from the fused render
// (raymarch.hip): the model's grids resolved as the render resolves them, the
// grid-space scale, and the proposal stages run by the render's own kernels
// with their intermediates written to the caller's buffers (sample-major
// [k][N], ray order).
struct TrainGeometry {
    GridDesc<16> grid;         // L16 C2
    GridDesc<16> prop[2];      // L5 C2
    float bound, b2, inv_b2;   // u = (x + bound) * inv_b2, or / b2 when inv_b2 == 0
};
struct ProposalOut {
    float* snf;                // [2][N] spacing(near), spacing(far)
    float4* rec;               // [N][2] slot-ordered ray records (PropArgs::rec)
    float* ds0;                // [128][N] delta * sigma of stage 0
    float* w0;                 // [128][N] its composited weights
    float* bins1;              // [65][N] resampled bins
    float* ds1;                // [64][N]
    float* w1;                 // [64][N]
    float* bins2;              // [33][N] the final stage's bins
};
int train_geometry(const samnerf_model* m, TrainGeometry& g);
int proposal_forward(const samnerf_model* m, const TrainGeometry& g, const float* rays_o,
                     const float* rays_d, uint32_t N, const float* cnf, uint32_t n_cnf,
                     const ProposalOut& o, hipStream_t s);

// ------------------------------------------------------------ device math --

// pos = clamp(fma(u, res, -0.5), 0, res-1); cell = floor; frac = pos - cell.
// nvcc contracts `u*res - 0.5` (gridencoder.cu:148), so the fma is explicit.
// p >= 0 after the clamp, so the truncating conversion is the floor and
// v_fract_f32 (p - floor(p), clamped below 1) is p - cell exactly: one VALU
// less per axis than floor, convert and subtract, the same bits.
__device__ __forceinline__ void locate_axis(float u, uint32_t res, uint32_t& cell, float& frac) {
    float p = __builtin_fmaf(u, (float)res, -0.5f);
    p = fminf(fmaxf(p, 0.0f), (float)(res - 1u));
    cell = (uint32_t)p;
    frac = __builtin_amdgcn_fractf(p);
}

// fminf(fmaxf(p, 0), top) for top >= 0 as one v_med3_f32 (fminf / fmaxf
// also canonicalise an operand loaded from memory: 3 VALU -> 1).  Same
// value for every p: med3 of a NaN input is min3 = 0 (IEEE minNum skips the
// quiet NaN), as fminf(fmaxf(NaN, 0), top) = 0; p = fma(u, res, -0.5) is
// never -0.
__device__ __forceinline__ float clamp_med3(float p, float top) {
    return __builtin_amdgcn_fmed3f(p, 0.0f, top);
}

// ReLU as one v_max_i32 on the float's bits: fmaxf(x, 0) on an MFMA
// accumulator (not known to be canonical) costs a canonicalising v_max first
// (and LLVM turns med3(x, 0, inf) back into that).  Same value as fmaxf for
// every non-NaN x (negative and -0.0 -> +0.0); a positive NaN passes through,
// as in torch.relu.
__device__ __forceinline__ float relu_bits(float x) {
    return __int_as_float(max(__float_as_int(x), 0));
}

// The same with the level's float resolution precomputed: frac = p -
// floorf(p) is p - (float)cell exactly (p in [0, res - 1], res < 2^24), and
// for p >= 0 that is v_fract_f32 (no floor instruction; the conversion
// truncates, which is the floor).
__device__ __forceinline__ void locate_axis(float u, const LevelDesc& d, uint32_t& cell, float& frac) {
    float p = __builtin_fmaf(u, d.fres, -0.5f);
    p = clamp_med3(p, d.ftop);
    cell = (uint32_t)p;
    frac = __builtin_amdgcn_fractf(p);
}

// Fused-path row index.  The host (make_grid_desc) only admits levels that
// are either dense with res^3 <= size (row < size, the reference's
// `% size` is the identity) or hashed into a power-of-two table (`% size` is a
// mask), so no integer division is ever emitted.
__device__ __forceinline__ uint32_t dense_or_hash_row(uint32_t x, uint32_t y, uint32_t z,
                                                      const LevelDesc& d) {
    if (d.flags & kHashed) return (x ^ (y * kPrime1) ^ (z * kPrime2)) & (d.size - 1u);
    return x + y * d.res + z * (d.res * d.res);
}

// Cross-half-wave exchange (lane i <-> lane i ^ 32) as one
// v_permlane32_swap_b32, a VALU op on gfx950, instead of __shfl_xor(v, 32)'s
// ds_bpermute_b32 (an LDS round trip and an lgkmcnt wait in the middle of the
// MLP chains).  With vdst = vsrc = v the swap leaves lo = v[i & 31] and
// hi = v[i | 32] in every lane i.
__device__ __forceinline__ void halves(float v, float& lo, float& hi) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
}
// fmaxf(v, __shfl_xor(v, 32)) (operands in lane order; only ever fed to
// scale_exp_of_max, which ignores the sign of a zero)
__device__ __forceinline__ float max_halves(float v) {
    float lo, hi;
    halves(v, lo, hi);
    return fmaxf(lo, hi);
}
// v + __shfl_xor(v, 32), the same bits in both halves (IEEE + commutes)
__device__ __forceinline__ float sum_halves(float v) {
    float lo, hi;
    halves(v, lo, hi);
    return lo + hi;
}
// __shfl_xor(v, 32)
__device__ __forceinline__ float xor_half(float v) {
    float lo, hi;
    halves(v, lo, hi);
    return (threadIdx.x & 32u) ? lo : hi;
}

template <int N>
struct alignas(16) VecF {
    float v[N];
};

// Load C contiguous floats (C in {1,2,4,8}) with the widest aligned access.
template <int C>
__device__ __forceinline__ void load_row(const float* __restrict__ p, float* out) {
    if constexpr (C == 1) {
        out[0] = p[0];
    } else if constexpr (C == 2) {
        float2 a = *reinterpret_cast<const float2*>(p);
        out[0] = a.x; out[1] = a.y;
    } else {
#pragma unroll
        for (int i = 0; i < C; i += 4) {
            float4 a = *reinterpret_cast<const float4*>(p + i);
            out[i] = a.x; out[i + 1] = a.y; out[i + 2] = a.z; out[i + 3] = a.w;
        }
    }
}

// Load C contiguous floats at a 32-bit byte offset from a uniform base: the
// address is base (SGPRs) + zero-extended offset (one VGPR), i.e. the
// global_load saddr form, with no per-lane 64-bit address arithmetic.  Only
// for tables the host has checked to be < 4 GiB (make_grid_desc).
template <int C>
__device__ __forceinline__ void load_row_b(const char* __restrict__ base, uint32_t off, float* out) {
    if constexpr (C == 2) {
        const float2 v = *reinterpret_cast<const float2*>(base + off);
        out[0] = v.x;
        out[1] = v.y;
    } else if constexpr (C == 8) {
        const float4 a = *reinterpret_cast<const float4*>(base + off);
        const float4 b = *reinterpret_cast<const float4*>(base + off + 16u);
        out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
        out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
    } else {
#pragma unroll
        for (int i = 0; i < C; ++i) out[i] = *reinterpret_cast<const float*>(base + off + 4u * i);
    }
}

typedef float f2v __attribute__((ext_vector_type(2)));

// The 8 trilinear corner weights (wx * wy) * wz of corner c (bit d <-> axis d,
// gridencoder.cu:168-201), two per packed multiply: wc[c >> 1] holds corners
// c & ~1 (.x) and c | 1 (.y).  Each lane of v_pk_mul_f32 is the scalar IEEE
// multiply, so the weights are the bits of the scalar form.
__device__ __forceinline__ void corner_weights_pk(float fx, float fy, float fz, f2v* wc) {
    const float wx0 = 1.0f - fx, wy0 = 1.0f - fy, wz0 = 1.0f - fz;
    const f2v xw = {wx0, fx};
    const f2v wxy01 = xw * f2v{wy0, wy0}, wxy23 = xw * f2v{fy, fy};
    wc[0] = wxy01 * f2v{wz0, wz0};
    wc[1] = wxy23 * f2v{wz0, wz0};
    wc[2] = wxy01 * f2v{fz, fz};
    wc[3] = wxy23 * f2v{fz, fz};
}

__device__ __forceinline__ float corner_w(const f2v* wc, int c) { return (c & 1) ? wc[c >> 1].y : wc[c >> 1].x; }

// Byte offsets (from the table base) of the 8 corner rows of the cell holding
// (ux, uy, uz) and their trilinear weights, corner c = bit d <-> axis d
// (gridencoder.cu:168-201).  Built from per-axis terms: 4 multiplies per
// level instead of 2 per corner, 24-bit multiplies for dense levels (res^3 <=
// size < 2^30 keeps every factor below 2^24), the level's first row folded
// into the x terms.  Same rows as dense_or_hash_row (uint32 wrap-around sums
// are associative) and the same weights ((wx * wy) * wz) as the reference.
template <int C>
__device__ __forceinline__ void corner_rows(const LevelDesc& d, float ux, float uy, float uz,
                                            uint32_t* off, float* w) {
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d, cx, fx);
    locate_axis(uy, d, cy, fy);
    locate_axis(uz, d, cz, fz);
    const uint32_t top = d.res - 1u;
    const uint32_t nx = min(cx + 1u, top), ny = min(cy + 1u, top), nz = min(cz + 1u, top);
    constexpr uint32_t RB = C * 4u;
    if (d.flags & kHashed) {
        const uint32_t m = d.size - 1u;
        const uint32_t y0 = cy * kPrime1, y1 = ny * kPrime1, z0 = cz * kPrime2, z1 = nz * kPrime2;
        const uint32_t xy[4] = {cx ^ y0, nx ^ y0, cx ^ y1, nx ^ y1};
#pragma unroll
        for (int c = 0; c < 8; ++c) off[c] = (d.off + ((xy[c & 3] ^ ((c & 4) ? z1 : z0)) & m)) * RB;
    } else {
        const uint32_t r2 = d.res * d.res;
        const uint32_t y0 = __umul24(cy, d.res), y1 = __umul24(ny, d.res);
        const uint32_t z0 = __umul24(cz, r2), z1 = __umul24(nz, r2);
        const uint32_t x0 = d.off + cx, x1 = d.off + nx;
        const uint32_t xy[4] = {x0 + y0, x1 + y0, x0 + y1, x1 + y1};
#pragma unroll
        for (int c = 0; c < 8; ++c) off[c] = (xy[c & 3] + ((c & 4) ? z1 : z0)) * RB;
    }
    if constexpr (C == 2) {
        f2v wc[4];
        corner_weights_pk(fx, fy, fz, wc);
#pragma unroll
        for (int c = 0; c < 8; ++c) w[c] = corner_w(wc, c);
    } else {
        // scalar products for the C = 8 fallback of k_sgrid_box4: the packed
        // form shifts its register allocation into spills in the sample loop
        const float wx0 = 1.0f - fx, wy0 = 1.0f - fy, wz0 = 1.0f - fz;
        const float wxy[4] = {wx0 * wy0, fx * wy0, wx0 * fy, fx * fy};
#pragma unroll
        for (int c = 0; c < 8; ++c) w[c] = wxy[c & 3] * ((c & 4) ? fz : wz0);
    }
}

// One corner (bit 0 x, 1 y, 2 z of c, lane-varying) of corner_rows<C>: the
// same byte offset and the same weight bits -- (wx * wy) * wz in that order,
// the row's terms combined as there (xor and integer adds are associative) --
// for a lane that needs only its own corner (the mask-training scatter: lane
// = (corner, channel)); a third of corner_rows' instructions.
template <uint32_t C>
__device__ __forceinline__ void corner_row_of(const LevelDesc& d, float ux, float uy, float uz, uint32_t c,
                                              uint32_t& off, float& w) {
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d, cx, fx);
    locate_axis(uy, d, cy, fy);
    locate_axis(uz, d, cz, fz);
    const uint32_t top = d.res - 1u;
    const uint32_t x = (c & 1u) ? min(cx + 1u, top) : cx, y = (c & 2u) ? min(cy + 1u, top) : cy,
                   z = (c & 4u) ? min(cz + 1u, top) : cz;
    const uint32_t row = (d.flags & kHashed) ? (x ^ (y * kPrime1) ^ (z * kPrime2)) & (d.size - 1u)
                                             : x + (uint32_t)__umul24(y, d.res) + (uint32_t)__umul24(z, d.res * d.res);
    off = (d.off + row) * (C * 4u);
    const float wx = (c & 1u) ? fx : 1.0f - fx, wy = (c & 2u) ? fy : 1.0f - fy, wz = (c & 4u) ? fz : 1.0f - fz;
    w = (wx * wy) * wz;
}

// Trilinear lookup of one level (D = 3, linear interpolation, no
// align_corners): the 8 corners in the reference's order, FMA accumulation
// into `acc` on packed-fp32 FMAs (two channels per v_pk_fma_f32; each lane
// of it is the same IEEE fma as the scalar form, so the bits are unchanged).
// Fused-path tables only (32-bit byte offsets, see load_row_b).
typedef float f4a8 __attribute__((ext_vector_type(4), aligned(8)));

// Dense C = 2 level: corners c and c | 1 (x and x + 1 at the same y, z) are
// adjacent 8-byte rows, so one 16-byte load fetches both -- 4 vector-memory
// instructions per level instead of 8, and the texture-address unit's cost is
// per lane and instruction, not per byte.  At the top x cell (cx = res - 1,
// nx = cx, so fx = 0) the pair (top - 1, top) is loaded and the x weights
// swapped (fx := 1): corner 0 then adds 0 * row(top - 1), an exact no-op (the
// running sum starts at +0 and is never -0; rows are finite), and corner 1
// adds row(top) with corner 0's original weight (1 * wy) * wz.  Same bits as
// lookup_level3 (the SAMNERF_LOOKUP=ref parity test), no per-corner selects.
__device__ __forceinline__ void lookup_dense_c2_paired(const float* __restrict__ emb,
                                                       const LevelDesc& d, float ux, float uy,
                                                       float uz, float* acc) {
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d, cx, fx);
    locate_axis(uy, d, cy, fy);
    locate_axis(uz, d, cz, fz);
    const uint32_t top = d.res - 1u;
    const uint32_t ny = min(cy + 1u, top), nz = min(cz + 1u, top);
    const bool edge = cx == top;
    fx = edge ? 1.0f : fx;
    const uint32_t bx = d.off + (edge ? cx - 1u : cx);
    const uint32_t r2 = d.res * d.res;
    const uint32_t y0 = __umul24(cy, d.res), y1 = __umul24(ny, d.res);
    const uint32_t z0 = __umul24(cz, r2), z1 = __umul24(nz, r2);
    const uint32_t pr[4] = {bx + y0 + z0, bx + y1 + z0, bx + y0 + z1, bx + y1 + z1};
    const char* base = reinterpret_cast<const char*>(emb);
    f4a8 v[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) v[p] = *reinterpret_cast<const f4a8*>(base + pr[p] * 8u);
    f2v wc[4];
    corner_weights_pk(fx, fy, fz, wc);
    f2v a = {0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const f4a8& q = v[c >> 1];              // pair (y, z) = (c >> 1 & 1, c >> 2)
        const f2v e = (c & 1) ? f2v{q.z, q.w} : f2v{q.x, q.y};
        const float w = corner_w(wc, c);
        a = __builtin_elementwise_fma(f2v{w, w}, e, a);
    }
    acc[0] = a.x;
    acc[1] = a.y;
}

template <int C>
__device__ __forceinline__ void lookup_level3(const float* __restrict__ emb, const LevelDesc& d,
                                              float ux, float uy, float uz, float* acc) {
    static_assert(C % 2 == 0, "packed accumulation needs an even channel count");
    if constexpr (C == 2) {
        if (!(d.flags & kHashed)) {
            lookup_dense_c2_paired(emb, d, ux, uy, uz, acc);
            return;
        }
    }
    uint32_t off[8];
    float w[8];
    corner_rows<C>(d, ux, uy, uz, off, w);
    const char* base = reinterpret_cast<const char*>(emb);
    f2v a[C / 2];
#pragma unroll
    for (int i = 0; i < C / 2; ++i) a[i] = f2v{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float e[C];
        load_row_b<C>(base, off[c], e);
        const f2v wc = {w[c], w[c]};
#pragma unroll
        for (int i = 0; i < C / 2; ++i)
            a[i] = __builtin_elementwise_fma(wc, f2v{e[2 * i], e[2 * i + 1]}, a[i]);
    }
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
        acc[2 * i] = a[i].x;
        acc[2 * i + 1] = a[i].y;
    }
}

// The per-corner form (one row computation and one scalar FMA per corner and
// channel): kept as the reference variant of lookup_level3 for the A/B
// parity test (SAMNERF_LOOKUP=ref).
template <int C>
__device__ __forceinline__ void lookup_level3_ref(const float* __restrict__ emb, const LevelDesc& d,
                                                  float ux, float uy, float uz, float* acc) {
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d.res, cx, fx);
    locate_axis(uy, d.res, cy, fy);
    locate_axis(uz, d.res, cz, fz);
    const uint32_t top = d.res - 1u;
    const uint32_t nx = min(cx + 1u, top), ny = min(cy + 1u, top), nz = min(cz + 1u, top);
    const char* base = reinterpret_cast<const char*>(emb);
#pragma unroll
    for (int i = 0; i < C; ++i) acc[i] = 0.0f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float wx = (c & 1) ? fx : 1.0f - fx;
        const float wy = (c & 2) ? fy : 1.0f - fy;
        const float wz = (c & 4) ? fz : 1.0f - fz;
        const float w = (wx * wy) * wz;
        const uint32_t row = dense_or_hash_row((c & 1) ? nx : cx, (c & 2) ? ny : cy,
                                               (c & 4) ? nz : cz, d);
        float e[C];
        load_row_b<C>(base, (d.off + row) * (uint32_t)(C * 4), e);
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] = __builtin_fmaf(w, e[i], acc[i]);
    }
}

// Ray tiling (samnerf_model.view_width).  The kernels work on ray SLOTS: a
// wave of the proposal / s_grid kernels is 64 consecutive slots, a k_final
// wave 32.  With the view's width W known, slot s is the ray of pixel
// (x, y) of an 8 x 4 tile -- tile s / 32 in row-major tile order, pixel s % 32
// row-major inside it -- so a wave's samples cover a compact patch of the
// scene instead of a 32- or 64-pixel row segment: at fine levels the corner
// boxes shrink and more gathers hit rows a neighbour already brought into L1
// (tools/diag/tile_probe.py: 3.14 -> 2.97 ms per default-init view, final
// 1.41 -> 1.20 ms on the opaque-sphere scene).  Per-sample intermediates
// (near/far, bins, ds, u_f, w_f) live in slot order; the rays are read and the
// per-ray outputs (image, depth, weights_sum, head rows) written at ray_of(s),
// so callers see ray order.  w == 0: identity (W not a multiple of 8, or N not
// a multiple of 4 W rows).
// tpr_log2: log2(tpr) when tpr is a power of two (the 512-wide views: a shift
// where the generic unsigned division by the uniform tpr is ~20 VALU -- once
// per sample in k_prop_sigma), else 32 (the division)
struct RayTiles {
    uint32_t w;           // view width in pixels (0: identity)
    uint32_t tpr;         // tiles per tile row = w / 8
    uint32_t tpr_log2;
    __device__ __forceinline__ uint32_t operator()(uint32_t s) const {
        if (w == 0u) return s;
        const uint32_t tile = s >> 5, in = s & 31u;
        const uint32_t trow = tpr_log2 < 32u ? tile >> tpr_log2 : tile / tpr, tcol = tile - trow * tpr;
        return (trow * 4u + (in >> 3)) * w + tcol * 8u + (in & 7u);
    }
};

inline RayTiles make_ray_tiles(uint32_t N, uint32_t W) {
    RayTiles t{0u, 0u, 32u};
    if (W >= 8u && W % 8u == 0u && N % (4u * W) == 0u) {
        t.w = W;
        t.tpr = W / 8u;
        if ((t.tpr & (t.tpr - 1u)) == 0u) t.tpr_log2 = (uint32_t)__builtin_ctz(t.tpr);
    }
    return t;
}

}  // namespace samnerf
