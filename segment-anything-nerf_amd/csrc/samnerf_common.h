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

#include "../../include/samnerf_hip.h"

namespace samnerf {

int fail(int code, const char* fmt, ...);
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

// ------------------------------------------------------------ device math --

// pos = clamp(fma(u, res, -0.5), 0, res-1); cell = floor; frac = pos - cell.
// nvcc contracts `u*res - 0.5` (gridencoder.cu:148), so the fma is explicit.
__device__ __forceinline__ void locate_axis(float u, uint32_t res, uint32_t& cell, float& frac) {
    float p = __builtin_fmaf(u, (float)res, -0.5f);
    p = fminf(fmaxf(p, 0.0f), (float)(res - 1u));
    cell = (uint32_t)floorf(p);
    frac = p - (float)cell;
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

// Trilinear lookup of one level (D = 3, linear interpolation, no
// align_corners): the 8 corners in the reference's order (bit d <-> axis d,
// gridencoder.cu:171-192), FMA accumulation into `acc`.  Fused-path tables
// only (32-bit byte offsets, see load_row_b).
template <int C>
__device__ __forceinline__ void lookup_level3(const float* __restrict__ emb, const LevelDesc& d,
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

}  // namespace samnerf
