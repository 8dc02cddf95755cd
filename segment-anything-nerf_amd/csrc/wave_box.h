// wave_box.h -- de-duplicated hash-grid gathers through LDS.
//
// A gather wave-instruction of the march kernels is 64 neighbouring rays at
// one sample index.  Their positions lie close together, so the 8 x 64 corner
// rows a wave reads at one level are far fewer distinct rows, but every lane
// still costs the vector memory path its own address and bytes.  The box
// path reads each distinct row once instead:
//   1. the wave reduces the grid-space range [lo, hi] of its positions
//      (DPP + readlane, wave-uniform result);
//   2. per level, the cell range of that range is exact (locate_axis is
//      monotonic in u), so the box of corner cells [x0, x1] x [y0, y1] x
//      [z0, z1] holds every corner any lane needs;
//   3. if the box has at most CAP slots, the wave loads it once into its own
//      LDS slice and every lane reads its 8 corners from LDS; a bigger box
//      takes the direct gathers.
// Rows, weights and FMA order are lookup_level3's, so results are
// bit-identical to the direct path (k_sgrid_box4 in raymarch.hip).  A lane whose corners fall outside the
// box anyway (a NaN position clamps to cell 0, and fminf/fmaxf skip NaN in
// the range) gathers directly.
#pragma once

#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include "samnerf_common.h"

namespace samnerf {

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}

// min / max over the 64 lanes (all lanes must be active); wave-uniform
// result.  Within a row of 16: quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror; across rows: readlane 0/16/32/48.
__device__ __forceinline__ float wave_fmin(float v) {
    v = fminf(v, dpp_f<0xB1>(v));
    v = fminf(v, dpp_f<0x4E>(v));
    v = fminf(v, dpp_f<0x141>(v));
    v = fminf(v, dpp_f<0x140>(v));
    const int b = __float_as_int(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(b, 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(b, 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(b, 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(b, 48));
    return fminf(fminf(r0, r1), fminf(r2, r3));
}

__device__ __forceinline__ float wave_fmax(float v) {
    v = fmaxf(v, dpp_f<0xB1>(v));
    v = fmaxf(v, dpp_f<0x4E>(v));
    v = fmaxf(v, dpp_f<0x141>(v));
    v = fmaxf(v, dpp_f<0x140>(v));
    const int b = __float_as_int(v);
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(b, 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(b, 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(b, 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(b, 48));
    return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}

// Wave-uniform grid-space range of the lanes' positions.
struct URange {
    float lo[3], hi[3];
};

template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}

// Signed-integer min / max of float bit patterns over the 64 lanes: the DPP
// steps fold into v_min_i32 / v_max_i32 (fminf / fmaxf need a canonicalising
// v_max per operand), the cross-row step is scalar.
__device__ __forceinline__ int wave_imin(int v) {
    v = min(v, dpp_i<0xB1>(v));
    v = min(v, dpp_i<0x4E>(v));
    v = min(v, dpp_i<0x141>(v));
    v = min(v, dpp_i<0x140>(v));
    const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return min(min(r0, r1), min(r2, r3));
}

__device__ __forceinline__ int wave_imax(int v) {
    v = max(v, dpp_i<0xB1>(v));
    v = max(v, dpp_i<0x4E>(v));
    v = max(v, dpp_i<0x141>(v));
    v = max(v, dpp_i<0x140>(v));
    const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return max(max(r0, r1), max(r2, r3));
}

// The range feeds only cell_of, which clamps below at cell 0.  Signed-integer
// order of float bits is the float order on non-negative values and puts
// every negative value (-0.0 included) below them, so the integer min / max
// select a value in the same cell as the float min / max: a negative result
// occurs exactly when the float result is negative (or -0.0), and both clamp
// to cell 0.  NaN lanes are neutral (INT_MAX in the min, INT_MIN in the max),
// as fminf / fmaxf skip NaN; an all-NaN wave yields NaN bits / -0.0, cell 0
// like the float reduction's NaN.
// The six reductions run in lockstep (independent DPP chains, so no hazard
// wait states between steps); across the rows of 16, row_bcast:15 and
// row_bcast:31 fold the row results into row 3 and one readlane of lane 63
// takes the total (round 1: four readlanes, two copies and a min3 per value).
__device__ __forceinline__ URange wave_urange(float ux, float uy, float uz) {
    const float u[3] = {ux, uy, uz};
    int lo[3], hi[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int b = __float_as_int(u[c]);
        const bool nan = u[c] != u[c];
        lo[c] = nan ? INT_MAX : b;
        hi[c] = nan ? INT_MIN : b;
    }
#define SAMNERF_URANGE_STEP(EXPR_LO, EXPR_HI)                                   \
    _Pragma("unroll") for (int c = 0; c < 3; ++c) {                             \
        lo[c] = min(lo[c], EXPR_LO);                                            \
        hi[c] = max(hi[c], EXPR_HI);                                            \
    }
    SAMNERF_URANGE_STEP(dpp_i<0xB1>(lo[c]), dpp_i<0xB1>(hi[c]))        // quad_perm [1,0,3,2]
    SAMNERF_URANGE_STEP(dpp_i<0x4E>(lo[c]), dpp_i<0x4E>(hi[c]))        // quad_perm [2,3,0,1]
    SAMNERF_URANGE_STEP(dpp_i<0x141>(lo[c]), dpp_i<0x141>(hi[c]))      // row_half_mirror
    SAMNERF_URANGE_STEP(dpp_i<0x140>(lo[c]), dpp_i<0x140>(hi[c]))      // row_mirror: row totals
    // rows 1, 3 take lane 15 of the row below, rows 2, 3 lane 31 (the other
    // rows see the identity, so min / max fold into one DPP instruction each)
    SAMNERF_URANGE_STEP(__builtin_amdgcn_update_dpp(INT_MAX, lo[c], 0x142, 0xa, 0xf, false),
                        __builtin_amdgcn_update_dpp(INT_MIN, hi[c], 0x142, 0xa, 0xf, false))
    SAMNERF_URANGE_STEP(__builtin_amdgcn_update_dpp(INT_MAX, lo[c], 0x143, 0xc, 0xf, false),
                        __builtin_amdgcn_update_dpp(INT_MIN, hi[c], 0x143, 0xc, 0xf, false))
#undef SAMNERF_URANGE_STEP
    URange r;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        r.lo[c] = __int_as_float(__builtin_amdgcn_readlane(lo[c], 63));
        r.hi[c] = __int_as_float(__builtin_amdgcn_readlane(hi[c], 63));
    }
    return r;
}

__device__ __forceinline__ uint32_t cell_of(float u, const LevelDesc& d) {
    float p = __builtin_fmaf(u, d.fres, -0.5f);
    p = clamp_med3(p, d.ftop);
    return (uint32_t)p;                       // p >= 0: truncation is the floor
}

}  // namespace samnerf

namespace samnerf {

// ---- power-of-two padded boxes, evaluated lane-parallel -----------------
// The x and y extents are rounded up to powers of two so that slot decoding
// and local corner indices are shifts and masks.  A wave that handles NL
// levels evaluates level i's box in lane i (one pass of VALU work for all
// levels) and reads the fields back with three readlanes.

__device__ __forceinline__ uint32_t log2_ceil(uint32_t v) { return v <= 1u ? 0u : 32u - __clz(v - 1u); }

struct PBox {
    uint32_t x0, y0, z0, ex, ey, ez, lx, ly, slots;
    uint32_t uni;          // every lane's position in the one cell (x0, y0, z0): the box is its corners
};

// Packed per-lane form: p0 = x0 | y0 << 10 | z0 << 20, p1 = ex | ey << 10 |
// ez << 20, p2 = lx | ly << 8 (every cell index and extent < 1024: the host
// admits only grids with res <= 1023 on this path).
__device__ __forceinline__ void pbox_lane(const LevelDesc& d, const URange& u, uint32_t& p0,
                                          uint32_t& p1, uint32_t& p2) {
    const uint32_t top = d.res - 1u;
    const uint32_t x0 = cell_of(u.lo[0], d), y0 = cell_of(u.lo[1], d), z0 = cell_of(u.lo[2], d);
    const uint32_t hx = cell_of(u.hi[0], d), hy = cell_of(u.hi[1], d), hz = cell_of(u.hi[2], d);
    const uint32_t x1 = min(hx + 1u, top);
    const uint32_t y1 = min(hy + 1u, top);
    const uint32_t z1 = min(hz + 1u, top);
    const uint32_t ex = x1 - x0 + 1u, ey = y1 - y0 + 1u, ez = z1 - z0 + 1u;
    p0 = x0 | (y0 << 10) | (z0 << 20);
    p1 = ex | (ey << 10) | (ez << 20);
    p2 = log2_ceil(ex) | (log2_ceil(ey) << 8) | ((hx == x0 && hy == y0 && hz == z0) ? 1u << 16 : 0u);
}

__device__ __forceinline__ PBox pbox_read(uint32_t p0, uint32_t p1, uint32_t p2, int lane) {
    const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)p0, lane);
    const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)p1, lane);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)p2, lane);
    PBox r;
    r.x0 = a & 1023u;
    r.y0 = (a >> 10) & 1023u;
    r.z0 = a >> 20;
    r.ex = b & 1023u;
    r.ey = (b >> 10) & 1023u;
    r.ez = b >> 20;
    r.lx = c & 255u;
    r.ly = (c >> 8) & 255u;
    r.uni = c >> 16;
    r.slots = r.ez << (r.lx + r.ly);
    return r;
}

// Stage the box's rows (C floats each) into `slice`, slot j = bx | by << lx
// | bz << (lx + ly); padding slots are left unwritten (never read).
template <int C>
__device__ __forceinline__ void stage_pbox(const char* __restrict__ base, const LevelDesc& d,
                                           const PBox& b, float* slice, uint32_t lane) {
    const uint32_t xm = (1u << b.lx) - 1u, ym = (1u << b.ly) - 1u;
    for (uint32_t j = lane; j < b.slots; j += 64u) {
        const uint32_t bx = j & xm, t = j >> b.lx, by = t & ym, bz = t >> b.ly;
        if (bx < b.ex && by < b.ey) {
            const uint32_t row = dense_or_hash_row(b.x0 + bx, b.y0 + by, b.z0 + bz, d);
            float e[C];
            load_row_b<C>(base, (d.off + row) * (uint32_t)(C * 4), e);
            if constexpr (C == 2) {
                *reinterpret_cast<float2*>(slice + j * 2) = make_float2(e[0], e[1]);
            } else {
#pragma unroll
                for (int i = 0; i < C; i += 4)
                    *reinterpret_cast<float4*>(slice + j * C + i) = make_float4(e[i], e[i + 1], e[i + 2], e[i + 3]);
            }
        }
    }
}

// Orders a wave's LDS stores before its later LDS loads of other lanes'
// slots (and the loads before the next stores): the LDS queue of one wave is
// in order, this only keeps the compiler from moving the accesses across.
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// True if no lane's position is NaN (all lanes active).  Then every lane's
// corners lie in the exact box and lookup_level3_pbox<C, false> may skip the
// per-lane inside test.
__device__ __forceinline__ bool wave_positions_ordered(float ux, float uy, float uz) {
    return __builtin_amdgcn_ballot_w64(ux != ux || uy != uy || uz != uz) == 0;
}

// Parity taps (samnerf_taps.srows; never in a product render): the
// level-relative rows of the 8 corners a direct lookup_level3<C> reads.
template <int C>
__device__ __forceinline__ void tap_direct_rows(const LevelDesc& d, float ux, float uy, float uz,
                                                uint32_t* tap) {
    uint32_t off[8];
    float w[8];
    corner_rows<C>(d, ux, uy, uz, off, w);
#pragma unroll
    for (int c = 0; c < 8; ++c) tap[c] = off[c] / (uint32_t)(C * 4) - d.off;
}

// lookup_level3 when every lane of the wave is in one cell (PBox::uni, no NaN
// lane): the 8 corner rows are wave-uniform, so they are read once through
// the scalar cache (s_load, no vector-memory or LDS traffic) and each lane
// weights them with its own fractions -- the same rows (the top-clamped
// corners of the cell), weights and FMA order as lookup_level3 (same bits).
// row[c]: the level-relative row of corner c (wave-uniform).
template <int C>
__device__ __forceinline__ void lookup_level3_uniform(const float* __restrict__ emb, const LevelDesc& d,
                                                      const uint32_t* row, float ux, float uy, float uz,
                                                      float* acc) {
    static_assert(C == 8, "uniform-cell lookup: C = 8 rows (32 B)");
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d, cx, fx);
    locate_axis(uy, d, cy, fy);
    locate_axis(uz, d, cz, fz);
    f2v wc[4];
    corner_weights_pk(fx, fy, fz, wc);
    f2v a[C / 2];
#pragma unroll
    for (int i = 0; i < C / 2; ++i) a[i] = f2v{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float4* p = reinterpret_cast<const float4*>(emb + (size_t)(d.off + row[c]) * C);
        const float4 v0 = p[0], v1 = p[1];
        const float w = corner_w(wc, c);
        const f2v wv = {w, w};
        a[0] = __builtin_elementwise_fma(wv, f2v{v0.x, v0.y}, a[0]);
        a[1] = __builtin_elementwise_fma(wv, f2v{v0.z, v0.w}, a[1]);
        a[2] = __builtin_elementwise_fma(wv, f2v{v1.x, v1.y}, a[2]);
        a[3] = __builtin_elementwise_fma(wv, f2v{v1.z, v1.w}, a[3]);
    }
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
        acc[2 * i] = a[i].x;
        acc[2 * i + 1] = a[i].y;
    }
}

// lookup_level3 from a staged padded box (same rows, weights, FMA order);
// with CHECK, a lane whose corners are outside the box gathers directly.
// tap (parity taps only; null otherwise): the row staged into each LDS slot
// the 8 corners read (stage_pbox's slot -> cell decoding), level-relative.
template <int C, bool CHECK = true>
__device__ __forceinline__ void lookup_level3_pbox(const float* __restrict__ emb, const LevelDesc& d,
                                                   const PBox& b, const float* slice, float ux,
                                                   float uy, float uz, float* acc,
                                                   uint32_t* tap = nullptr) {
    uint32_t cx, cy, cz;
    float fx, fy, fz;
    locate_axis(ux, d, cx, fx);
    locate_axis(uy, d, cy, fy);
    locate_axis(uz, d, cz, fz);
    const uint32_t top = d.res - 1u;
    const uint32_t nx = min(cx + 1u, top), ny = min(cy + 1u, top), nz = min(cz + 1u, top);
    const uint32_t lx0 = cx - b.x0, lx1 = nx - b.x0;
    const uint32_t ly0 = cy - b.y0, ly1 = ny - b.y0;
    const uint32_t lz0 = cz - b.z0, lz1 = nz - b.z0;
    if constexpr (CHECK) {
        const bool inside = lx0 < b.ex && lx1 < b.ex && ly0 < b.ey && ly1 < b.ey && lz0 < b.ez && lz1 < b.ez;
        if (!inside) {
            if (tap) tap_direct_rows<C>(d, ux, uy, uz, tap);
            lookup_level3<C>(emb, d, ux, uy, uz, acc);
            return;
        }
    }
    // corner c's slot byte offset: the (x, y, z) = (0, 0, 0) corner plus
    // per-axis steps of 0 (clamped top cell) or one slot row, one add each
    constexpr uint32_t RB = C * 4u;                     // bytes per slot
    const uint32_t lxy = b.lx + b.ly;
    const uint32_t o0 = (lx0 + (ly0 << b.lx) + (lz0 << lxy)) * RB;
    const uint32_t DX = (lx1 - lx0) * RB, DY = ((ly1 - ly0) << b.lx) * RB, DZ = ((lz1 - lz0) << lxy) * RB;
    uint32_t off[8];
    off[0] = o0;
    off[1] = o0 + DX;
    off[2] = o0 + DY;
    off[3] = off[2] + DX;
    off[4] = o0 + DZ;
    off[5] = off[4] + DX;
    off[6] = off[4] + DY;
    off[7] = off[6] + DX;
    if (tap) {
        const uint32_t xm = (1u << b.lx) - 1u, ym = (1u << b.ly) - 1u;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const uint32_t j = off[c] / RB;
            tap[c] = dense_or_hash_row(b.x0 + (j & xm), b.y0 + ((j >> b.lx) & ym), b.z0 + (j >> lxy), d);
        }
    }
    f2v wc[4];
    corner_weights_pk(fx, fy, fz, wc);
    const char* sb = reinterpret_cast<const char*>(slice);
    f2v a[C / 2];
#pragma unroll
    for (int i = 0; i < C / 2; ++i) a[i] = f2v{0.0f, 0.0f};
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float w = corner_w(wc, c);
        const f2v wv = {w, w};
        if constexpr (C == 2) {
            const float2 v = *reinterpret_cast<const float2*>(sb + off[c]);
            a[0] = __builtin_elementwise_fma(wv, f2v{v.x, v.y}, a[0]);
        } else {
#pragma unroll
            for (int i = 0; i < C; i += 4) {
                const float4 v = *reinterpret_cast<const float4*>(sb + off[c] + i * 4);
                a[i / 2] = __builtin_elementwise_fma(wv, f2v{v.x, v.y}, a[i / 2]);
                a[i / 2 + 1] = __builtin_elementwise_fma(wv, f2v{v.z, v.w}, a[i / 2 + 1]);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
        acc[2 * i] = a[i].x;
        acc[2 * i + 1] = a[i].y;
    }
}

}  // namespace samnerf
