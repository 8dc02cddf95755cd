// fp32_chain.h -- exact-fp32 MFMA accumulation chains of the training heads
// (sam_head_train.hip, mask_head_train.hip).
//
// acc[m] += sum over KS k-steps s of A_m(s) B(s) on v_mfma_f32_16x16x4_f32
// (an fma chain in k order, cdna_hip_programming.md "FP32-input MFMA"): the A
// fragment of tile m at step s is Ap[m][s * 64] (an L2-resident weight pack
// in fragment order), B(s) = bl[s * 64] (LDS).  The A loads of the next U
// steps are issued before the MFMAs of the current U (register double
// buffer), so a wave waits for L2 once per chain instead of once per step:
// the first version, one load then its MFMA, left the SAM head's backward at
// ~380 us of L2 latency for 4,096 rays.
#pragma once

#include <hip/hip_runtime.h>

namespace samnerf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int MT, int U>
__device__ __forceinline__ void chain_load(float (&buf)[U][MT], const float* const (&Ap)[MT], int g) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
        for (int m = 0; m < MT; ++m) buf[u][m] = Ap[m][(g * U + u) * 64];
    // keep the whole group's loads ahead of the MFMAs that follow (the
    // scheduler otherwise sinks them between the MFMAs and reuses registers,
    // leaving ~2 steps of loads in flight)
    __builtin_amdgcn_sched_barrier(0);
}

template <int MT, int U>
__device__ __forceinline__ void chain_mfma(f32x4 (&acc)[MT], const float (&buf)[U][MT], const float* bl, int g) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const float b = bl[(g * U + u) * 64];
#pragma unroll
        for (int m = 0; m < MT; ++m) acc[m] = mfma16(buf[u][m], b, acc[m]);
    }
}

// Two register buffers in ping-pong, no copies between them (a rotating
// cur = nxt copy made the compiler wait for the fresh loads right after
// issuing them).  Past the last group the load repeats it (unused).
template <int MT, int KS, int U>
__device__ __forceinline__ void mfma_chain(f32x4 (&acc)[MT], const float* const (&Ap)[MT], const float* bl) {
    static_assert(KS % U == 0, "k-steps must split into groups of U");
    constexpr int G = KS / U;
    float b0[U][MT], b1[U][MT];
    chain_load<MT, U>(b0, Ap, 0);
#pragma unroll 1
    for (int g = 0; g < G; g += 2) {
        chain_load<MT, U>(b1, Ap, min(g + 1, G - 1));
        chain_mfma<MT, U>(acc, b0, bl, g);
        if (g + 1 < G) {
            chain_load<MT, U>(b0, Ap, min(g + 2, G - 1));
            chain_mfma<MT, U>(acc, b1, bl, g + 1);
        }
    }
}

}  // namespace samnerf
