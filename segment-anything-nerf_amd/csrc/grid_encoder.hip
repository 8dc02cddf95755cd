// grid_encoder.hip -- drop-in multiresolution hash/tiled grid encoder for gfx950.
//
// Same contract as the reference's _gridencoder module
// (gridencoder/src/gridencoder.cu:381-713) behind a C ABI, re-designed for
// CDNA4 wave64:
//   * resolution table computed on the host (no device exp2f),
//   * one thread per (point, level), 256-thread blocks, rows loaded with the
//     widest aligned vector access (float2 / float4) instead of per-channel
//     scalar loads,
//   * backward: one thread per (point, level, channel) so the atomics of a
//     corner row come from adjacent lanes (contiguous bytes per wave
//     instruction, MI355X_MICROARCH.md "Global float atomics"),
//   * launches on the caller's stream instead of the legacy default stream.
// Index semantics (corner order, uint32 wrap, hash primes, % size) are the
// reference's, bit for bit (tests/test_gpu_encoders.py).
#include <cstdio>
#include <type_traits>

#include "samnerf_common.h"

using namespace samnerf;

namespace {

template <uint32_t D>
__device__ __forceinline__ uint32_t grid_row(uint32_t gridtype, uint32_t size, uint32_t res,
                                             const uint32_t* cell) {
    uint32_t stride = 1u, row = 0u;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        if (stride <= size) {
            row += cell[d] * stride;
            stride *= res;
        }
    }
    if (gridtype == 0u && stride > size) {
        row = 0u;
#pragma unroll
        for (uint32_t d = 0; d < D; ++d) row ^= cell[d] * kPrimes[d];
    }
    return row % size;
}
// NB: the reference's loop stops at the first stride that exceeds the table;
// the `if` above is equivalent because once stride > size it never shrinks
// (res >= 1), so later iterations are skipped in both forms.

template <uint32_t D>
__device__ __forceinline__ bool outside(const float* x) {
    bool o = false;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) o |= (x[d] < 0.0f) | (x[d] > 1.0f);
    return o;
}

template <uint32_t D>
__device__ __forceinline__ void place(const float* x, uint32_t res, bool align_corners,
                                      uint32_t interp, float* frac, float* dfrac, uint32_t* cell) {
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        float p;
        uint32_t g;
        if (align_corners) {
            p = x[d] * (float)(res - 1u);
            g = min((uint32_t)floorf(p), res - 2u);
        } else {
            p = fminf(fmaxf(__builtin_fmaf(x[d], (float)res, -0.5f), 0.0f), (float)(res - 1u));
            g = (uint32_t)floorf(p);
        }
        p -= (float)g;
        if (interp == 1u) {
            dfrac[d] = (6.0f * p) * (1.0f - p);
            p = (p * p) * __builtin_fmaf(-2.0f, p, 3.0f);
        } else {
            dfrac[d] = 1.0f;
        }
        frac[d] = p;
        cell[d] = g;
    }
}

template <uint32_t D>
__device__ __forceinline__ float corner_weight(uint32_t c, uint32_t res, const float* frac,
                                               const uint32_t* cell, uint32_t* cc) {
    float w = 1.0f;
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        if (c & (1u << d)) {
            w *= frac[d];
            cc[d] = min(cell[d] + 1u, res - 1u);
        } else {
            w *= 1.0f - frac[d];
            cc[d] = cell[d];
        }
    }
    return w;
}

template <uint32_t C>
__device__ __forceinline__ void load_vec(const float* __restrict__ p, float* e) {
    if constexpr (C == 1) {
        e[0] = p[0];
    } else if constexpr (C == 2) {
        float2 a = *reinterpret_cast<const float2*>(p);
        e[0] = a.x; e[1] = a.y;
    } else {
#pragma unroll
        for (uint32_t i = 0; i < C; i += 4) {
            float4 a = *reinterpret_cast<const float4*>(p + i);
            e[i] = a.x; e[i + 1] = a.y; e[i + 2] = a.z; e[i + 3] = a.w;
        }
    }
}

template <uint32_t C>
__device__ __forceinline__ void store_vec(float* __restrict__ p, const float* e) {
    if constexpr (C == 1) {
        p[0] = e[0];
    } else if constexpr (C == 2) {
        *reinterpret_cast<float2*>(p) = make_float2(e[0], e[1]);
    } else {
#pragma unroll
        for (uint32_t i = 0; i < C; i += 4)
            *reinterpret_cast<float4*>(p + i) = make_float4(e[i], e[i + 1], e[i + 2], e[i + 3]);
    }
}

// ---------------------------------------------------------------- forward --
template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_forward(const float* __restrict__ inputs, const float* __restrict__ emb,
               const int32_t* __restrict__ offsets, float* __restrict__ outputs, uint32_t B,
               uint32_t L, ResTable rt, float* __restrict__ dy_dx, uint32_t gridtype,
               bool align_corners, uint32_t interp) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t level = blockIdx.y;
    if (b >= B) return;
    const uint32_t base = (uint32_t)offsets[level];
    const uint32_t size = (uint32_t)offsets[level + 1] - base;
    const uint32_t res = rt.res[level];
    const float* table = emb + (size_t)base * C;

    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) x[d] = inputs[(size_t)b * D + d];
    float* out = outputs + ((size_t)level * B + b) * C;
    float* dd = dy_dx ? dy_dx + ((size_t)b * L + level) * D * C : nullptr;

    float acc[C];
#pragma unroll
    for (uint32_t i = 0; i < C; ++i) acc[i] = 0.0f;

    if (outside<D>(x)) {
        store_vec<C>(out, acc);
        if (dd)
            for (uint32_t i = 0; i < D * C; ++i) dd[i] = 0.0f;
        return;
    }

    float frac[D], dfrac[D];
    uint32_t cell[D], cc[D];
    place<D>(x, res, align_corners, interp, frac, dfrac, cell);

#pragma unroll
    for (uint32_t c = 0; c < (1u << D); ++c) {
        const float w = corner_weight<D>(c, res, frac, cell, cc);
        const uint32_t row = grid_row<D>(gridtype, size, res, cc);
        float e[C];
        load_vec<C>(table + (size_t)row * C, e);
#pragma unroll
        for (uint32_t i = 0; i < C; ++i) acc[i] = __builtin_fmaf(w, e[i], acc[i]);
    }
    store_vec<C>(out, acc);

    if (dd) {
        const float span = (float)(align_corners ? res - 1u : res);
#pragma unroll
        for (uint32_t gd = 0; gd < D; ++gd) {
            float g[C];
#pragma unroll
            for (uint32_t i = 0; i < C; ++i) g[i] = 0.0f;
#pragma unroll
            for (uint32_t c = 0; c < (1u << (D - 1u)); ++c) {
                float w = span;
#pragma unroll
                for (uint32_t nd = 0; nd < D - 1u; ++nd) {
                    const uint32_t d = nd >= gd ? nd + 1u : nd;
                    if (c & (1u << nd)) {
                        w *= frac[d];
                        cc[d] = min(cell[d] + 1u, res - 1u);
                    } else {
                        w *= 1.0f - frac[d];
                        cc[d] = cell[d];
                    }
                }
                cc[gd] = cell[gd];
                const uint32_t lo = grid_row<D>(gridtype, size, res, cc);
                cc[gd] = min(cell[gd] + 1u, res - 1u);
                const uint32_t hi = grid_row<D>(gridtype, size, res, cc);
                float el[C], eh[C];
                load_vec<C>(table + (size_t)lo * C, el);
                load_vec<C>(table + (size_t)hi * C, eh);
#pragma unroll
                for (uint32_t i = 0; i < C; ++i)
                    g[i] = __builtin_fmaf(w * (eh[i] - el[i]), dfrac[gd], g[i]);
            }
            store_vec<C>(dd + gd * C, g);
        }
    }
}

// --------------------------------------------------------------- backward --
// One thread per (point, level, channel): lanes c = 0..C-1 of a point update
// the C contiguous floats of the same corner row together, and equal rows of
// the wave's other points are merged before the atomic (fewer memory-side
// requests; the sum is reassociated, within the backward's float-atomic
// tolerance).
template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grid_backward(const float* __restrict__ grad, const float* __restrict__ inputs,
                const int32_t* __restrict__ offsets, float* __restrict__ grad_emb, uint32_t B,
                ResTable rt, uint32_t gridtype, bool align_corners, uint32_t interp) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t level = blockIdx.y;
    const uint32_t b = (uint32_t)(t / C), ch = (uint32_t)(t % C);
    const uint32_t lane = threadIdx.x & 63u;
    if ((t & ~(uint64_t)63) / C >= B) return;              // whole wave past the end
    const uint32_t bb = b < B ? b : B - 1;                  // lanes stay for the shuffles
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) x[d] = inputs[(size_t)bb * D + d];
    const bool live = b < B && !outside<D>(x);
    const uint32_t base = (uint32_t)offsets[level];
    const uint32_t size = (uint32_t)offsets[level + 1] - base;
    const uint32_t res = rt.res[level];
    float frac[D], dfrac[D];
    uint32_t cell[D], cc[D];
    place<D>(x, res, align_corners, interp, frac, dfrac, cell);
    const float g = live ? grad[((size_t)level * B + bb) * C + ch] : 0.0f;
    float* gtab = grad_emb + (size_t)base * C + ch;
#pragma unroll
    for (uint32_t c = 0; c < (1u << D); ++c) {
        const float w = corner_weight<D>(c, res, frac, cell, cc);
        const uint32_t row = grid_row<D>(gridtype, size, res, cc);
        float val = w * g;
        // neighbouring points of a wave often hit the same corner row: merge
        // equal rows (same channel = lanes C apart) over a butterfly so one
        // lane per row issues the memory-side atomic
        bool alive = live;
#pragma unroll
        for (uint32_t sd = C; sd < 64u; sd <<= 1) {
            const uint32_t orow = __shfl_xor(row, (int)sd);
            const float oval = __shfl_xor(val, (int)sd);
            const int oalive = __shfl_xor((int)alive, (int)sd);
            if (alive && oalive && orow == row) {
                if (lane & sd) alive = false;
                else val += oval;
            }
        }
        if (alive) atomicAdd(gtab + (size_t)row * C, val);
    }
}

template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_input_backward(const float* __restrict__ grad, const float* __restrict__ dy_dx,
                 float* __restrict__ grad_inputs, uint32_t B, uint32_t L) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    float r = 0.0f;
    for (uint32_t l = 0; l < L; ++l)
#pragma unroll
        for (uint32_t ch = 0; ch < C; ++ch)
            r = __builtin_fmaf(grad[((size_t)l * B + b) * C + ch],
                               dy_dx[(((size_t)b * L + l) * D + d) * C + ch], r);
    grad_inputs[t] = r;
}

// ---------------------------------------------------------------------- TV --
template <uint32_t D, uint32_t C>
__global__ void __launch_bounds__(256)
k_grad_tv(const float* __restrict__ inputs, const float* __restrict__ emb,
          float* __restrict__ grad, const int32_t* __restrict__ offsets, float weight,
          uint32_t B, ResTable rt, uint32_t gridtype, bool align_corners) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t level = blockIdx.y;
    if (b >= B) return;
    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) x[d] = inputs[(size_t)b * D + d];
    if (outside<D>(x)) return;
    const uint32_t base = (uint32_t)offsets[level];
    const uint32_t size = (uint32_t)offsets[level + 1] - base;
    const uint32_t res = rt.res[level];
    const float* table = emb + (size_t)base * C;
    float* gtab = grad + (size_t)base * C;
    float frac[D], dfrac[D];
    uint32_t cell[D];
    place<D>(x, res, align_corners, 0u, frac, dfrac, cell);
    const uint32_t here = grid_row<D>(gridtype, size, res, cell);
    float e0[C], sum[C], sq[C];
    load_vec<C>(table + (size_t)here * C, e0);
#pragma unroll
    for (uint32_t i = 0; i < C; ++i) sum[i] = sq[i] = 0.0f;
    const float w = weight / (float)(2u * D);
#pragma unroll
    for (uint32_t d = 0; d < D; ++d) {
        const uint32_t keep = cell[d];
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            if (side == 0 ? keep < res : keep > 0u) {
                cell[d] = side == 0 ? keep + 1u : keep - 1u;
                float e[C];
                load_vec<C>(table + (size_t)grid_row<D>(gridtype, size, res, cell) * C, e);
#pragma unroll
                for (uint32_t i = 0; i < C; ++i) {
                    const float v = e0[i] - e[i];
                    sum[i] += v;
                    sq[i] = __builtin_fmaf(v, v, sq[i]);
                }
            }
        }
        cell[d] = keep;
    }
#pragma unroll
    for (uint32_t i = 0; i < C; ++i)
        atomicAdd(gtab + (size_t)here * C + i, (w * sum[i]) * rsqrtf(sq[i] + 1e-9f));
}

// ---------------------------------------------------------------------- WD --
__global__ void __launch_bounds__(256)
k_grad_wd(const float* __restrict__ emb, float* __restrict__ grad,
          const int32_t* __restrict__ offsets, float weight, uint64_t n, uint32_t C, uint32_t L) {
    const uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const uint32_t row = (uint32_t)(e / C);
    uint32_t lo = 0, hi = L, level = 0;
    while (lo < hi) {            // last level whose first row <= row
        const uint32_t m = (lo + hi) >> 1;
        if ((uint32_t)offsets[m] <= row) { level = m; lo = m + 1u; } else { hi = m; }
    }
    const uint32_t size = (uint32_t)(offsets[level + 1] - offsets[level]);
    grad[e] += ((2.0f * weight) * emb[e]) / (float)size;
}

// ------------------------------------------------------------ dispatchers --
template <uint32_t D, class F>
int dispatch_c(uint32_t C, F& f) {
    switch (C) {
        case 1: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 1>{});
        case 2: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 2>{});
        case 4: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 4>{});
        case 8: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 8>{});
        case 16: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 16>{});
        case 32: return f(std::integral_constant<uint32_t, D>{}, std::integral_constant<uint32_t, 32>{});
        default: return fail(SAMNERF_EINVAL, "GridEncoding: C must be 1, 2, 4, 8, 16 or 32.");
    }
}

template <class F>
int dispatch_dc(uint32_t D, uint32_t C, F&& f) {
    switch (D) {
        case 2: return dispatch_c<2>(C, f);
        case 3: return dispatch_c<3>(C, f);
        case 4: return dispatch_c<4>(C, f);
        case 5: return dispatch_c<5>(C, f);
        default: return fail(SAMNERF_EINVAL, "GridEncoding: D must be 2, 3, 4 or 5.");
    }
}

int check_common(const void* a, const void* b, const void* c, uint32_t L, uint32_t max_level) {
    if (!a || !b || !c) return fail(SAMNERF_EINVAL, "GridEncoding: null tensor pointer");
    if (L == 0 || L > 32) return fail(SAMNERF_EINVAL, "GridEncoding: L must be in [1, 32]");
    if (max_level > L) return fail(SAMNERF_EINVAL, "GridEncoding: max_level > L");
    return SAMNERF_OK;
}

}  // namespace

extern "C" {

int samnerf_grid_encode_forward(const float* inputs, const float* embeddings,
                                const int32_t* offsets, float* outputs, uint32_t B, uint32_t D,
                                uint32_t C, uint32_t L, uint32_t max_level, float S, uint32_t H,
                                float* dy_dx, uint32_t gridtype, int align_corners,
                                uint32_t interp, samnerf_stream_t stream) {
    int rc = check_common(inputs, embeddings, offsets, L, max_level);
    if (rc) return rc;
    if (!outputs) return fail(SAMNERF_EINVAL, "GridEncoding: null outputs");
    if (B == 0 || max_level == 0) return SAMNERF_OK;
    const ResTable rt = make_res_table(L, S, H);
    const dim3 grid(div_up(B, 256), max_level);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    rc = dispatch_dc(D, C, [&](auto d, auto c) {
        k_grid_forward<decltype(d)::value, decltype(c)::value><<<grid, 256, 0, s>>>(
            inputs, embeddings, offsets, outputs, B, L, rt, dy_dx, gridtype, align_corners != 0,
            interp);
        return 0;
    });
    return rc ? rc : check_launch("grid_encode_forward");
}

int samnerf_grid_encode_backward(const float* grad, const float* inputs, const float* embeddings,
                                 const int32_t* offsets, float* grad_embeddings, uint32_t B,
                                 uint32_t D, uint32_t C, uint32_t L, uint32_t max_level, float S,
                                 uint32_t H, const float* dy_dx, float* grad_inputs,
                                 uint32_t gridtype, int align_corners, uint32_t interp,
                                 samnerf_stream_t stream) {
    int rc = check_common(grad, inputs, offsets, L, max_level);
    if (rc) return rc;
    (void)embeddings;
    if (!grad_embeddings) return fail(SAMNERF_EINVAL, "GridEncoding: null grad_embeddings");
    if ((dy_dx == nullptr) != (grad_inputs == nullptr))
        return fail(SAMNERF_EINVAL, "GridEncoding: dy_dx and grad_inputs must be given together");
    if (B == 0) return SAMNERF_OK;
    const ResTable rt = make_res_table(L, S, H);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    rc = dispatch_dc(D, C, [&](auto d, auto c) {
        constexpr uint32_t kD = decltype(d)::value, kC = decltype(c)::value;
        if (max_level > 0) {
            const dim3 grid(div_up((uint64_t)B * kC, 256), max_level);
            k_grid_backward<kD, kC><<<grid, 256, 0, s>>>(grad, inputs, offsets, grad_embeddings,
                                                        B, rt, gridtype, align_corners != 0,
                                                        interp);
        }
        if (dy_dx)
            k_input_backward<kD, kC><<<div_up((uint64_t)B * kD, 256), 256, 0, s>>>(
                grad, dy_dx, grad_inputs, B, L);
        return 0;
    });
    return rc ? rc : check_launch("grid_encode_backward");
}

int samnerf_grad_total_variation(const float* inputs, const float* embeddings, float* grad,
                                 const int32_t* offsets, float weight, uint32_t B, uint32_t D,
                                 uint32_t C, uint32_t L, float S, uint32_t H, uint32_t gridtype,
                                 int align_corners, samnerf_stream_t stream) {
    int rc = check_common(inputs, embeddings, offsets, L, L);
    if (rc) return rc;
    if (!grad) return fail(SAMNERF_EINVAL, "GridEncoding: null grad");
    if (B == 0) return SAMNERF_OK;
    const ResTable rt = make_res_table(L, S, H);
    const dim3 grid(div_up(B, 256), L);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    rc = dispatch_dc(D, C, [&](auto d, auto c) {
        k_grad_tv<decltype(d)::value, decltype(c)::value><<<grid, 256, 0, s>>>(
            inputs, embeddings, grad, offsets, weight, B, rt, gridtype, align_corners != 0);
        return 0;
    });
    return rc ? rc : check_launch("grad_total_variation");
}

int samnerf_grad_weight_decay(const float* embeddings, float* grad, const int32_t* offsets,
                              float weight, uint32_t B, uint32_t C, uint32_t L,
                              samnerf_stream_t stream) {
    int rc = check_common(embeddings, grad, offsets, L, L);
    if (rc) return rc;
    const uint64_t n = (uint64_t)B * C;
    if (n == 0) return SAMNERF_OK;
    k_grad_wd<<<div_up(n, 256), 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
        embeddings, grad, offsets, weight, n, C, L);
    return check_launch("grad_weight_decay");
}

}  // extern "C"
