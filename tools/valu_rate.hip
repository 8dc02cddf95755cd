// tools/valu_rate.hip -- VALU issue rate of one MI355X SIMD, measured: how many
// wave64 vector instructions per clock per SIMD a stream of independent
// instructions sustains at 1, 2, 3, 4 and 8 resident waves per SIMD.  The
// march kernels' rooflines price their VALU work at this rate (bench.py
// rooflines(), MI355X_MICROARCH.md: 2 cycles per v_fma_f32 on SIMD-32, 4 for
// one wave alone) and the committed PMC passes of this program relate the
// SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU counters to it (profiles/r4_valu_rate.*).
//
// Each lane runs 16 independent accumulation chains (no dependency stalls:
// the chains are 16 instructions apart), `iters` times, of one instruction
// kind: v_fma_f32, v_pk_fma_f32 (two fp32 per lane), v_exp_f32 (a
// transcendental), v_xor_b32 / v_add_u32 (integer).  The grid is 256 x w
// workgroups of 256 threads (one wave per SIMD each), so every SIMD holds w
// waves; the clock is the in-kernel one (s_memtime / s_memrealtime, median
// over workgroups), written by a vector store.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/valu_rate tools/valu_rate.hip
// run:   tools/bin/valu_rate > profiles/r4_valu_rate.json
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

constexpr int kChains = 16;
constexpr int kBlock = 256;
typedef float f2v __attribute__((ext_vector_type(2)));

enum Kind { kFma = 0, kPkFma = 1, kExp = 2, kInt = 3, kMulLo = 4, kMix = 5, kMaxI = 6, kBitop3 = 7,
           kCvtPk = 8, kCvtF32 = 9, kCvtF32Hi = 10, kMaxF = 11, kMed3 = 12,
           kMulF = 13, kAddLshl = 14, kCndmask = 15, kFract = 16, kCvtU32 = 17, kMadU24 = 18, kLshl = 19, kCndS = 20, kCndV = 21 };
constexpr int kKinds = 22;

template <int K>
__global__ void __launch_bounds__(kBlock) k_valu(float seed, uint32_t iters, float* __restrict__ out,
                                                 unsigned long long* __restrict__ stamps) {
    float a[kChains];
    f2v p[kChains];
    uint32_t u[kChains];
#pragma unroll
    for (int j = 0; j < kChains; ++j) {
        a[j] = seed + (float)(threadIdx.x + j);
        p[j] = f2v{a[j], a[j] * 0.5f};
        u[j] = (uint32_t)threadIdx.x * 2654435761u + (uint32_t)j;
    }
    const float m = seed * 1e-3f + 0.999f, c = seed * 1e-7f;
    const unsigned long long smask = __builtin_amdgcn_read_exec() & 0x5555555555555555ull;
    const f2v mm = {m, m}, cc = {c, c};
    unsigned long long t0, r0, t1, r1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // the instructions are written as asm so that the compiler neither packs
    // the scalar chains into v_pk_fma_f32 nor folds anything; 4 chain steps per
    // loop trip keep the loop's SALU overhead off the VALU stream
    for (uint32_t it = 0; it < iters; it += 4) {
#pragma unroll
        for (int rep = 0; rep < 4; ++rep)
#pragma unroll
            for (int j = 0; j < kChains; ++j) {
                if constexpr (K == kFma) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(m), "v"(c));
                else if constexpr (K == kPkFma)
                    asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[j]) : "v"(mm), "v"(cc));
                else if constexpr (K == kExp) asm volatile("v_exp_f32 %0, %0" : "+v"(a[j]));
                else if constexpr (K == kInt)
                    asm volatile("v_xor_b32 %0, 0x9e3779b9, %0\n\tv_add_u32 %0, %0, %1" : "+v"(u[j]) : "v"(it));
                else if constexpr (K == kMulLo) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[j]) : "v"(it));
                // the f16x3 split's instruction: a half-dword write (read-modify-write of %0)
                else if constexpr (K == kMix) asm volatile("v_fma_mixlo_f16 %0, %1, %2, 0" : "+v"(u[j]) : "v"(m), "v"(c));
                else if constexpr (K == kMaxI) asm volatile("v_max_i32 %0, %0, %1" : "+v"(u[j]) : "v"(it));
                else if constexpr (K == kBitop3)
                    asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(u[j]) : "v"(it), "v"(u[(j + 1) % kChains]));
                // conversions of a split without v_fma_mix: f32 pair -> packed f16, f16 -> f32 (low / high half)
                else if constexpr (K == kCvtPk) asm volatile("v_cvt_pk_f16_f32 %0, %1, %0" : "+v"(u[j]) : "v"(m));
                else if constexpr (K == kCvtF32) asm volatile("v_cvt_f32_f16 %0, %0" : "+v"(u[j]));
                else if constexpr (K == kCvtF32Hi) asm volatile("v_cvt_f32_f16_sdwa %0, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1" : "+v"(u[j]));
                else if constexpr (K == kMaxF) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[j]) : "v"(m));
                else if constexpr (K == kMed3) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(m), "v"(c));
                // the index arithmetic of the corner rows
                else if constexpr (K == kMulF) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(m));
                else if constexpr (K == kAddLshl) asm volatile("v_add_lshl_u32 %0, %0, %1, 3" : "+v"(u[j]) : "v"(it));
                else if constexpr (K == kCndmask)
                    asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[j]) : "v"(it) : "vcc");
                else if constexpr (K == kFract) asm volatile("v_fract_f32 %0, %0" : "+v"(a[j]));
                else if constexpr (K == kCvtU32) asm volatile("v_cvt_u32_f32 %0, %0" : "+v"(u[j]));
                else if constexpr (K == kMadU24) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(u[j]) : "v"(it));
                else if constexpr (K == kLshl) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u[j]));
                // v_cndmask on a 64-bit SGPR condition (e64), and on a compare result written each step
                else if constexpr (K == kCndS)
                    asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[j]) : "v"(it), "s"(smask));
                else asm volatile("v_cmp_gt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[j]) : "v"(it) : "vcc");
            }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    float s = 0.0f;
#pragma unroll
    for (int j = 0; j < kChains; ++j) s += a[j] + p[j].x + p[j].y + (float)u[j];
    out[blockIdx.x * kBlock + threadIdx.x] = s;
    if (threadIdx.x < 2)                                  // lanes 0, 1: a lane-indexed (vector) store
        stamps[2 * blockIdx.x + threadIdx.x] = threadIdx.x ? r1 - r0 : t1 - t0;
}

struct Result {
    double ms, clock_ghz, inst_per_clk_simd, cycles_per_inst;
};

template <int K>
Result run(int cus, int waves_per_simd, uint32_t iters) {
    const uint32_t blocks = (uint32_t)cus * waves_per_simd;
    float* out;
    unsigned long long* stamps;
    CHECK(hipMalloc(&out, (size_t)blocks * kBlock * 4));
    CHECK(hipMalloc(&stamps, (size_t)blocks * 2 * 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 2; ++w) k_valu<K><<<blocks, kBlock>>>(1.0f, iters, out, stamps);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(a));
        k_valu<K><<<blocks, kBlock>>>(1.0f, iters, out, stamps);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        best = std::min(best, ms);
    }
    std::vector<unsigned long long> st((size_t)blocks * 2);
    CHECK(hipMemcpy(st.data(), stamps, st.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (uint32_t i = 0; i < blocks; ++i)
        if (st[2 * i + 1] > 0) clk.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 0.1);   // GHz
    std::sort(clk.begin(), clk.end());
    const double ghz = clk.empty() ? 2.4 : clk[clk.size() / 2];
    // wave instructions of the timed loop (one per chain per iteration)
    const double insts = (double)blocks * (kBlock / 64) * kChains * iters;
    Result r;
    r.ms = best;
    r.clock_ghz = ghz;
    r.inst_per_clk_simd = insts / (best * 1e-3) / (ghz * 1e9) / (cus * 4.0);
    r.cycles_per_inst = 1.0 / r.inst_per_clk_simd;
    CHECK(hipFree(out));
    CHECK(hipFree(stamps));
    return r;
}

int main(int argc, char** argv) {
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 4096;
    const int waves[5] = {1, 2, 3, 4, 8};
    const char* kinds[kKinds] = {"v_fma_f32", "v_pk_fma_f32", "v_exp_f32", "v_xor_b32+v_add_u32",
                                 "v_mul_lo_u32", "v_fma_mixlo_f16", "v_max_i32", "v_bitop3_b32",
                                 "v_cvt_pk_f16_f32", "v_cvt_f32_f16", "v_cvt_f32_f16_sdwa_hi", "v_max_f32", "v_med3_f32",
                                 "v_mul_f32", "v_add_lshl_u32", "v_cndmask_b32_vcc_clobber_artifact", "v_fract_f32", "v_cvt_u32_f32",
                                 "v_mad_u32_u24", "v_lshlrev_b32", "v_cndmask_b32_e64_sgpr", "v_cmp+v_cndmask_vcc"};
    printf("{\"what\": \"independent wave64 VALU instructions per clock per SIMD by resident waves per SIMD "
           "(tools/valu_rate.hip)\", \"cus\": %d, \"iters\": %u, \"kinds\": {", cus, iters);
    for (int k = 0; k < kKinds; ++k) {
        printf("%s\"%s\": {", k ? ", " : "", kinds[k]);
        for (int i = 0; i < 5; ++i) {
            // the integer form issues two instructions per chain step
            Result r = k == kFma ? run<kFma>(cus, waves[i], iters)
                     : k == kPkFma ? run<kPkFma>(cus, waves[i], iters)
                     : k == kExp ? run<kExp>(cus, waves[i], iters / 2)
                     : k == kInt ? run<kInt>(cus, waves[i], iters)
                     : k == kMulLo ? run<kMulLo>(cus, waves[i], iters / 2)
                     : k == kMix ? run<kMix>(cus, waves[i], iters)
                     : k == kMaxI ? run<kMaxI>(cus, waves[i], iters)
                     : k == kBitop3 ? run<kBitop3>(cus, waves[i], iters)
                     : k == kCvtPk ? run<kCvtPk>(cus, waves[i], iters)
                     : k == kCvtF32 ? run<kCvtF32>(cus, waves[i], iters)
                     : k == kCvtF32Hi ? run<kCvtF32Hi>(cus, waves[i], iters)
                     : k == kMaxF ? run<kMaxF>(cus, waves[i], iters)
                     : k == kMed3 ? run<kMed3>(cus, waves[i], iters)
                     : k == kMulF ? run<kMulF>(cus, waves[i], iters)
                     : k == kAddLshl ? run<kAddLshl>(cus, waves[i], iters)
                     : k == kCndmask ? run<kCndmask>(cus, waves[i], iters)
                     : k == kFract ? run<kFract>(cus, waves[i], iters)
                     : k == kCvtU32 ? run<kCvtU32>(cus, waves[i], iters)
                     : k == kMadU24 ? run<kMadU24>(cus, waves[i], iters)
                     : k == kLshl ? run<kLshl>(cus, waves[i], iters)
                     : k == kCndS ? run<kCndS>(cus, waves[i], iters)
                                  : run<kCndV>(cus, waves[i], iters);
            if (k == kInt || k == kCndV) {
                r.inst_per_clk_simd *= 2.0;
                r.cycles_per_inst = 1.0 / r.inst_per_clk_simd;
            }
            printf("%s\"%d\": {\"ms\": %.4f, \"clock_ghz\": %.3f, \"inst_per_clk_per_simd\": %.4f, "
                   "\"cycles_per_inst\": %.3f}",
                   i ? ", " : "", waves[i], r.ms, r.clock_ghz, r.inst_per_clk_simd, r.cycles_per_inst);
            fflush(stdout);
        }
        printf("}");
    }
    printf("}}\n");
    return 0;
}
