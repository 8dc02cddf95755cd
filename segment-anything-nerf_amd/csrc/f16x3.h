// f16x3.h -- fp32-equivalent GEMM operands on the fp16 matrix cores.
//
// The MLPs of the path (grid_mlp, the SAM head, the mask head) are fp32 in
// the reference (nerf/network.py:9-75).  gfx950 runs fp32-input MFMA at 1/16
// of the fp16 rate, so these GEMMs run as three fp16 products per fp32
// product ("f16x3"): each operand x is split x = hi + lo with
//   hi = f16_rne(x),  lo = f16_rne(x - hi)       (x - hi is exact in fp32)
// and A.B = A_lo.B_hi + A_hi.B_lo + A_hi.B_hi on v_mfma_f32_32x32x16_f16
// (fp32 accumulate; the dropped A_lo.B_lo is 2^-22 of the product).  hi + lo
// carries 22 significant bits, so each product is within ~2^-21 of the exact
// one -- below the fp32 rounding of the accumulation it feeds over K = 16..419
// terms (tools/f16x3_error.py: the same max error against float64 as an exact
// fp32 MFMA GEMM, 36x below the bf16 split it replaces).
//
// fp16's narrow exponent range (normal from 2^-14, max 65504) is handled by
// exact power-of-two scaling: every weight tensor is scaled so its largest
// |w| lies in [2^13, 2^14) (packing time, log2 of the scale kept), and every
// activation COLUMN (one ray or sample) the same way at run time, from the max
// over the column's K inputs.  Scaling by 2^e commutes with rounding, so the
// scaled product is the unscaled one times 2^(e_row + e_col) exactly; the
// consumer multiplies the accumulator by the two inverse scales.  With the
// column maximum at 2^13, elements down to 2^-27 of it stay normal fp16 and the
// absolute error floor is 2^-38 of the maximum.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace samnerf {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// Power-of-two scale s and its inverse for a column (or row) whose largest
// magnitude is `maxabs` (>= 0): maxabs * s in [2^13, 2^14) -- one binade below
// fp16's top, so values up to 4x the maximum a scale was chosen for still fit
// (the headroom k_final's one-block-at-a-time layer 1, SAMNERF_FINAL_JOINT = 0,
// relies on; the default joint form takes one scale over both k-blocks).  The exponent is
// clamped so that both s and 1/s are normal floats (all-zero or tiny columns
// get s = 2^125; inf / NaN columns s = 2^-115 and stay inf / NaN).
struct Scale2 {
    float s, inv;
};
__host__ __device__ __forceinline__ Scale2 scale_of_max(float maxabs) {
    uint32_t e = __builtin_bit_cast(uint32_t, maxabs) >> 23;          // biased exponent (sign bit clear)
    e = e < 15u ? 15u : (e > 255u ? 255u : e);
    Scale2 r;
    r.s = __builtin_bit_cast(float, (267u - e) << 23);             // 2^(140 - e)
    r.inv = __builtin_bit_cast(float, (e - 13u) << 23);             // 2^(e - 140)
    return r;
}

// The same as an exponent k (s = 2^k, k in [-115, 125]) and 2^k as a float
// for any k (clamped to the normal range): scales tracked across layers.
__device__ __forceinline__ int scale_exp_of_max(float maxabs) {
    uint32_t e = __builtin_bit_cast(uint32_t, maxabs) >> 23;
    e = e < 15u ? 15u : (e > 255u ? 255u : e);
    return 140 - (int)e;
}
__device__ __forceinline__ float exp2i(int k) {
    k = k < -126 ? -126 : (k > 127 ? 127 : k);
    return __builtin_bit_cast(float, (uint32_t)(k + 127) << 23);
}

// hi / lo halves of 8 values times s (s a power of two, so x * s is exact),
// packed as two f16 per dword: hi = f16(x s), lo = f16(x s - hi), each one
// v_fma_mix (fp32 fma of f32 / f16 sources rounded once to f16): 4
// instructions per pair where multiply, convert, convert back, subtract and
// convert took 6.  The same bits as that sequence (x s and x s - hi are exact
// in fp32, so both round the same value once).
//
// Wait states (nothing inside an asm string is padded by hipcc): both mix
// forms write half of their destination and keep the other half (a
// read-modify-write of the dword), and a VALU that reads a VGPR right after
// such a partial write needs one wait state (gfx950's dst-sel forwarding
// hazard).  So every dword's partial writes and reads here are 4 instructions
// apart: the four hi dwords' low halves, then their high halves, then the lo
// dwords' low halves (reading the hi dwords), then their high halves; the
// string ends with s_nop 1 because its outputs feed MFMA A/B operands, which
// need two wait states after a VALU write (the guide's VALU -> MFMA operand
// rule; it also covers the last partial write).  The round-1 to round-3 form
// (hi, then lo, of each pair back to back) read the hi dword one instruction
// after its partial write: on a busy SIMD another wave's instruction usually
// sat between them, so the outputs were right on most launches and wrong on a
// few (the k_final prefetch variants' "nondeterminism"); the
// first round-4 form still wrote each hi dword's two halves back to back.
#if defined(SAMNERF_F16X3_NOASM)
// The same split in plain C (v_pk_mul_f32, v_cvt_pk_f16_f32, conversions back,
// a subtraction, v_cvt_pk_f16_f32 again): full-dword writes the compiler
// schedules and pads itself; the same bits (x s and x s - hi are exact).
template <bool LEAD = false>   // compiler code: hipcc pads its hazards
__device__ __forceinline__ void split8_f16(const float* v, float s, uint4& hi, uint4& lo) {
    uint32_t h[4], l[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const float a = v[2 * p] * s, b = v[2 * p + 1] * s;
        const f16x2v hh = {(_Float16)a, (_Float16)b};
        const f16x2v ll = {(_Float16)(a - (float)hh.x), (_Float16)(b - (float)hh.y)};
        h[p] = __builtin_bit_cast(uint32_t, hh);
        l[p] = __builtin_bit_cast(uint32_t, ll);
    }
    hi = make_uint4(h[0], h[1], h[2], h[3]);
    lo = make_uint4(l[0], l[1], l[2], l[3]);
}
#elif defined(SAMNERF_AB_OLDSPLIT)   // timing A/B only: the round-3 form (hazard-exposed)
__device__ __forceinline__ void split_pair_f16_old(float x, float y, float s, uint32_t& hi, uint32_t& lo) {
    uint32_t h, l;
    asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
        "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
        "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
        : "=&v"(h), "=&v"(l)
        : "v"(x), "v"(y), "v"(s));
    hi = h;
    lo = l;
}
template <bool LEAD = false>   // timing variants: no leading pad
__device__ __forceinline__ void split8_f16(const float* v, float s, uint4& hi, uint4& lo) {
    split_pair_f16_old(v[0], v[1], s, hi.x, lo.x);
    split_pair_f16_old(v[2], v[3], s, hi.y, lo.y);
    split_pair_f16_old(v[4], v[5], s, hi.z, lo.z);
    split_pair_f16_old(v[6], v[7], s, hi.w, lo.w);
}
#elif !defined(SAMNERF_SPLIT_MIX)
// Round 5: the same split on full-dword conversions.  v_fma_mix issues at a
// quarter of v_fma_f32's rate on gfx950 (8.2 cycles per wave64 instruction
// against 2.2; v_cvt_pk_f16_f32 / v_cvt_f32_f16 4.1, v_mul_f32 / v_sub_f32
// 2.2: tools/valu_rate.hip, profiles/r5v_valu_rate.json), so 16 mixes
// (131 cycles per 8 values) cost more than a = x s, hi = cvt_pk(a), the hi
// halves back to fp32, d = a - f32(hi), lo = cvt_pk(d): 32 instructions, 101
// cycles.  The same bits: x s, f32(hi) and a - f32(hi) are exact, and each
// half is rounded to fp16 once (RNE), as the mix does.  Every write is a
// whole dword (no dst-sel hazard), each result is read at least 4
// instructions after it is written, and the closing s_nop 1 covers the VALU
// -> MFMA operand rule for the last lo dword.  hipcc does not pad an MFMA
// whose result registers the statement's outputs reuse (it cannot see into
// the string): LEAD = true opens it with s_nop 7, the 8 wait states a 4-pass
// XDL result needs before a VALU writes the same registers -- the call sites
// whose schedule puts the statement right behind MFMAs (k_sam_head_w8, found
// by tests/test_isa_hazards.py) take it.
#define SAMNERF_SPLIT8_ASM \
    "v_mul_f32 %[a0], %[v0], %[s]\n\t" \
    "v_mul_f32 %[a1], %[v1], %[s]\n\t" \
    "v_mul_f32 %[a2], %[v2], %[s]\n\t" \
    "v_mul_f32 %[a3], %[v3], %[s]\n\t" \
    "v_mul_f32 %[a4], %[v4], %[s]\n\t" \
    "v_mul_f32 %[a5], %[v5], %[s]\n\t" \
    "v_mul_f32 %[a6], %[v6], %[s]\n\t" \
    "v_mul_f32 %[a7], %[v7], %[s]\n\t" \
    "v_cvt_pk_f16_f32 %[h0], %[a0], %[a1]\n\t" \
    "v_cvt_pk_f16_f32 %[h1], %[a2], %[a3]\n\t" \
    "v_cvt_pk_f16_f32 %[h2], %[a4], %[a5]\n\t" \
    "v_cvt_pk_f16_f32 %[h3], %[a6], %[a7]\n\t" \
    "v_cvt_f32_f16 %[t0], %[h0]\n\t" \
    "v_cvt_f32_f16 %[t2], %[h1]\n\t" \
    "v_cvt_f32_f16 %[t4], %[h2]\n\t" \
    "v_cvt_f32_f16 %[t6], %[h3]\n\t" \
    "v_cvt_f32_f16_sdwa %[t1], %[h0] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
    "v_cvt_f32_f16_sdwa %[t3], %[h1] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
    "v_cvt_f32_f16_sdwa %[t5], %[h2] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
    "v_cvt_f32_f16_sdwa %[t7], %[h3] dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1\n\t" \
    "v_sub_f32 %[t0], %[a0], %[t0]\n\t" \
    "v_sub_f32 %[t2], %[a2], %[t2]\n\t" \
    "v_sub_f32 %[t4], %[a4], %[t4]\n\t" \
    "v_sub_f32 %[t6], %[a6], %[t6]\n\t" \
    "v_sub_f32 %[t1], %[a1], %[t1]\n\t" \
    "v_sub_f32 %[t3], %[a3], %[t3]\n\t" \
    "v_sub_f32 %[t5], %[a5], %[t5]\n\t" \
    "v_sub_f32 %[t7], %[a7], %[t7]\n\t" \
    "v_cvt_pk_f16_f32 %[l0], %[t0], %[t1]\n\t" \
    "v_cvt_pk_f16_f32 %[l1], %[t2], %[t3]\n\t" \
    "v_cvt_pk_f16_f32 %[l2], %[t4], %[t5]\n\t" \
    "v_cvt_pk_f16_f32 %[l3], %[t6], %[t7]\n\t" \
    "s_nop 1"
#define SAMNERF_SPLIT8_OUT \
    [h0] "=&v"(h0), [h1] "=&v"(h1), [h2] "=&v"(h2), [h3] "=&v"(h3), [l0] "=&v"(l0), [l1] "=&v"(l1), \
    [l2] "=&v"(l2), [l3] "=&v"(l3), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3), \
    [a4] "=&v"(a4), [a5] "=&v"(a5), [a6] "=&v"(a6), [a7] "=&v"(a7), [t0] "=&v"(t0), [t1] "=&v"(t1), \
    [t2] "=&v"(t2), [t3] "=&v"(t3), [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7)
#define SAMNERF_SPLIT8_IN \
    [v0] "v"(v[0]), [v1] "v"(v[1]), [v2] "v"(v[2]), [v3] "v"(v[3]), [v4] "v"(v[4]), [v5] "v"(v[5]), \
    [v6] "v"(v[6]), [v7] "v"(v[7]), [s] "v"(s)
template <bool LEAD = false>
__device__ __forceinline__ void split8_f16(const float* v, float s, uint4& hi, uint4& lo) {
    uint32_t h0, h1, h2, h3, l0, l1, l2, l3;
    float a0, a1, a2, a3, a4, a5, a6, a7, t0, t1, t2, t3, t4, t5, t6, t7;
    if constexpr (LEAD) asm("s_nop 7\n\t" SAMNERF_SPLIT8_ASM : SAMNERF_SPLIT8_OUT : SAMNERF_SPLIT8_IN);
    else asm(SAMNERF_SPLIT8_ASM : SAMNERF_SPLIT8_OUT : SAMNERF_SPLIT8_IN);
    hi = make_uint4(h0, h1, h2, h3);
    lo = make_uint4(l0, l1, l2, l3);
}
#else   // SAMNERF_SPLIT_MIX: rounds 1-5's v_fma_mix form (timing A/B)
template <bool LEAD = false>   // timing variants: no leading pad
__device__ __forceinline__ void split8_f16(const float* v, float s, uint4& hi, uint4& lo) {
    uint32_t h0, h1, h2, h3, l0, l1, l2, l3;
    asm("v_fma_mixlo_f16 %0, %8, %16, 0\n\t"
        "v_fma_mixlo_f16 %1, %10, %16, 0\n\t"
        "v_fma_mixlo_f16 %2, %12, %16, 0\n\t"
        "v_fma_mixlo_f16 %3, %14, %16, 0\n\t"
        "v_fma_mixhi_f16 %0, %9, %16, 0\n\t"
        "v_fma_mixhi_f16 %1, %11, %16, 0\n\t"
        "v_fma_mixhi_f16 %2, %13, %16, 0\n\t"
        "v_fma_mixhi_f16 %3, %15, %16, 0\n\t"
        "v_fma_mixlo_f16 %4, %8, %16, -%0 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %5, %10, %16, -%1 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %6, %12, %16, -%2 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixlo_f16 %7, %14, %16, -%3 op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %4, %9, %16, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %5, %11, %16, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %6, %13, %16, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "v_fma_mixhi_f16 %7, %15, %16, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
        "s_nop 1"
        : "=&v"(h0), "=&v"(h1), "=&v"(h2), "=&v"(h3), "=&v"(l0), "=&v"(l1), "=&v"(l2), "=&v"(l3)
        : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]),
          "v"(s));
    hi = make_uint4(h0, h1, h2, h3);
    lo = make_uint4(l0, l1, l2, l3);
}
#endif

// running max |a|, |b| into m (one v_max3_f32 with |.| source modifiers)
__device__ __forceinline__ float max_abs3(float m, float a, float b) {
#if defined(SAMNERF_F16X3_NOASM)
    return fmaxf(m, fmaxf(fabsf(a), fabsf(b)));
#endif
    float r;
    asm("v_max3_f32 %0, %1, |%2|, |%3|" : "=v"(r) : "v"(m), "v"(a), "v"(b));
    return r;
}
// running max of relu(a), relu(b) on the float bits (m >= 0 as int; a
// negative float is a negative int): one v_max3_i32
__device__ __forceinline__ int max_relu3(int m, float a, float b) {
    return max(m, max(__builtin_bit_cast(int, a), __builtin_bit_cast(int, b)));
}

// C += A.B in f16x3 (small terms first)
__device__ __forceinline__ floatx16 mfma_f16x3(uint4 ah, uint4 al, uint4 bh, uint4 bl, floatx16 c) {
    const f16x8 Ah = __builtin_bit_cast(f16x8, ah), Al = __builtin_bit_cast(f16x8, al);
    const f16x8 Bh = __builtin_bit_cast(f16x8, bh), Bl = __builtin_bit_cast(f16x8, bl);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(Al, Bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(Ah, Bh, c, 0, 0, 0);
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// C += A.B in f16x3 on the 16 x 16 x 32 form (small terms first): lane
// (i, g) holds A[row i][k = 8 g .. 8 g + 7] and B[k = 8 g ..][column i], D
// lane (j, g) column j, rows 4 g .. 4 g + 3
__device__ __forceinline__ floatx4 mfma16_f16x3(uint4 ah, uint4 al, uint4 bh, uint4 bl, floatx4 c) {
    const f16x8 Ah = __builtin_bit_cast(f16x8, ah), Al = __builtin_bit_cast(f16x8, al);
    const f16x8 Bh = __builtin_bit_cast(f16x8, bh), Bl = __builtin_bit_cast(f16x8, bl);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(Al, Bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah, Bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(Ah, Bh, c, 0, 0, 0);
}

// max |x| of a wave-wide reduction over the 64 lanes (for weight rows)
__device__ __forceinline__ float wave_max64(float m) {
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) m = fmaxf(m, __shfl_xor(m, k));
    return m;
}

}  // namespace samnerf
