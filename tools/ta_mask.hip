// tools/ta_mask.hip -- cost of an L1-resident gather instruction by width and
// by active lanes.  The proposal stages' gathers hit the vector L1 ~98 % of
// the time (r5m PMC: TCP_TCC_READ_REQ / TCP_TOTAL_CACHE_ACCESSES) and keep its
// address path ~72 % busy, so what a hashed-level x-pair load would save
// depends on whether an exec-masked instruction (odd-x lanes' second corner)
// costs its active lanes or the whole wave.  Patterns, each 16 gathers per
// loop trip from a 16 KiB table (L1-resident), random per lane:
//   x2      global_load_dwordx2, 64 lanes
//   x4      global_load_dwordx4, 64 lanes
//   x2_half global_load_dwordx2 with the odd lanes masked off (32 lanes)
//   pair    one x4 (64 lanes) + one x2 on the odd lanes: the x-pair form of
//           two x2 corner loads
//   x2_g8   global_load_dwordx2, 64 lanes in 8 groups of 8 that share an address
//   x2_uni  global_load_dwordx2, all 64 lanes one address
// Printed: wave-instructions per clock per CU and clocks per 64-lane
// instruction (ns from events, the in-kernel clock as in ta_rate.hip).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/ta_mask tools/ta_mask.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

constexpr int kPerLane = 16;
constexpr uint32_t kTableBytes = 16384;
constexpr int kBlock = 256;
enum Pattern { kX2 = 0, kX4 = 1, kX2Half = 2, kPair = 3, kX2G8 = 4, kX2Uni = 5 };

template <int P>
__global__ void __launch_bounds__(kBlock) k_gather(const char* __restrict__ table, const uint32_t* __restrict__ offs,
                                                   uint32_t iters, uint32_t* __restrict__ out,
                                                   unsigned long long* __restrict__ stamps) {
    const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
    const bool odd = threadIdx.x & 1u;
    uint32_t o[kPerLane];
    // the groups read their first lane's offset (x2_g8: lanes 8g .. 8g+7; x2_uni: the wave)
    const uint32_t src = P == kX2G8 ? (tid & ~7u) : P == kX2Uni ? (tid & ~63u) : tid;
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) o[j] = offs[(size_t)j * gridDim.x * kBlock + src];   // 16-B aligned
    uint32_t acc = 0;
    unsigned long long t0, r0, t1, r1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    for (uint32_t it = 0; it < iters; ++it) {
        const char* b = table + ((it & 1u) << 4);     // keeps the loads in the loop
        // one exec-masked region per trip (16 loads issued, then consumed), as
        // a kernel's level batch would be
        if constexpr (P == kX2 || P == kX2G8 || P == kX2Uni) {
#pragma unroll
            for (int j = 0; j < kPerLane; ++j) {
                const uint2 v = *reinterpret_cast<const uint2*>(b + o[j]);
                acc ^= v.x ^ v.y;
            }
        } else if constexpr (P == kX4 || P == kPair) {
#pragma unroll
            for (int j = 0; j < kPerLane; ++j) {
                const uint4 v = *reinterpret_cast<const uint4*>(b + o[j]);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
        if constexpr (P == kX2Half || P == kPair) {
            if (P == kX2Half ? !odd : odd) {
#pragma unroll
                for (int j = 0; j < kPerLane; ++j) {
                    const uint2 w = *reinterpret_cast<const uint2*>(b + (o[j] ^ 4096u));
                    acc ^= w.x ^ w.y;
                }
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    out[tid] = acc;
    if (threadIdx.x < 2) stamps[2 * blockIdx.x + threadIdx.x] = threadIdx.x ? r1 - r0 : t1 - t0;
}

template <int P>
void run(const char* name, const char* table, const uint32_t* offs, uint32_t blocks, uint32_t iters, int cus,
         bool first) {
    uint32_t* out;
    unsigned long long* stamps;
    CHECK(hipMalloc(&out, (size_t)blocks * kBlock * 4));
    CHECK(hipMalloc(&stamps, (size_t)blocks * 2 * 8));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) k_gather<P><<<blocks, kBlock>>>(table, offs, iters, out, stamps);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(a));
        k_gather<P><<<blocks, kBlock>>>(table, offs, iters, out, stamps);
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
        if (st[2 * i + 1] > 0) clk.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 0.1);
    std::sort(clk.begin(), clk.end());
    const double ghz = clk.empty() ? 2.4 : clk[clk.size() / 2];
    // "corner-pair slots": 16 per lane and trip, each 1 (x2, x4, x2_half) or 2 (pair) instructions
    const double slots = (double)blocks * (kBlock / 64) * kPerLane * iters;
    const double clk_per_slot_cu = (best * 1e-3) * (ghz * 1e9) * cus / slots;
    printf("%s\"%s\": {\"ms\": %.4f, \"clock_ghz\": %.3f, \"clk_per_slot_per_cu\": %.3f}", first ? "" : ", ", name,
           best, ghz, clk_per_slot_cu);
    fflush(stdout);
    CHECK(hipFree(out));
    CHECK(hipFree(stamps));
}

int main() {
    const uint32_t blocks = 8192, iters = 64;
    const size_t n_lanes = (size_t)blocks * kBlock;
    char* table;
    CHECK(hipMalloc(&table, kTableBytes + 64));
    CHECK(hipMemset(table, 0x5a, kTableBytes + 64));
    std::mt19937 rng(99);
    std::vector<uint32_t> offs_h((size_t)kPerLane * n_lanes);
    for (auto& x : offs_h) x = (rng() % (kTableBytes / 2 / 16)) * 16u;   // 16-B aligned, first half
    uint32_t* offs;
    CHECK(hipMalloc(&offs, offs_h.size() * 4));
    CHECK(hipMemcpy(offs, offs_h.data(), offs_h.size() * 4, hipMemcpyHostToDevice));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"what\": \"L1-resident (16 KiB) random gathers: clocks per CU per slot of 64 lanes by width and active "
           "lanes (tools/ta_mask.hip)\", \"cus\": %d, \"patterns\": {", cus);
    run<kX2>("x2", table, offs, blocks, iters, cus, true);
    run<kX4>("x4", table, offs, blocks, iters, cus, false);
    run<kX2Half>("x2_half", table, offs, blocks, iters, cus, false);
    run<kPair>("pair_x4_plus_x2_odd", table, offs, blocks, iters, cus, false);
    run<kX2G8>("x2_groups_of_8", table, offs, blocks, iters, cus, false);
    run<kX2Uni>("x2_uniform", table, offs, blocks, iters, cus, false);
    printf("}}\n");
    CHECK(hipFree(offs));
    CHECK(hipFree(table));
    return 0;
}
