// tools/ta_rate.hip -- texture-address (vector-memory gather) rate of one MI355X
// CU, measured: how many lane-addresses per clock per CU a stream of 64-lane
// gather instructions sustains when the data is L2-resident.  The fused
// hash-grid kernels (k_prop_sigma, k_final) issue such gathers; bench.py prices
// them against the rate this program measures (profiles/r3_ta_rate.json).
//
// Each lane holds 16 precomputed word offsets into a 1 MiB table; iteration
// `it` adds a wave-uniform shift (an SGPR), so the loop issues 16 gathers and
// 16 xors per iteration and no address arithmetic per lane (global_load with
// a 32-bit VGPR offset from a scalar base).  Patterns: random dword / dwordx2 /
// dwordx4 per lane (every lane its own 64-B line: the hash-grid case) and
// contiguous dwords (a wave reads 256 consecutive bytes).  The clock is the
// in-kernel one (s_memtime ticks / s_memrealtime 100 MHz ticks, median over
// workgroups; MI355X_MICROARCH.md "DVFS give-back" item 6), written by one
// lane per workgroup with a vector store.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/ta_rate tools/ta_rate.hip
// run:   tools/bin/ta_rate > profiles/r3_ta_rate.json
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
constexpr uint32_t kTableWords = 1u << 18;          // 1 MiB of offsets' range
constexpr uint32_t kShiftWords = 1u << 18;          // + up to 1 MiB of uniform shift
constexpr int kBlock = 256;

template <int W>
struct Vec;
template <>
struct Vec<1> {
    typedef uint32_t T;
    __device__ static uint32_t fold(T v) { return v; }
};
template <>
struct Vec<2> {
    typedef uint2 T;
    __device__ static uint32_t fold(T v) { return v.x ^ v.y; }
};
template <>
struct Vec<4> {
    typedef uint4 T;
    __device__ static uint32_t fold(T v) { return v.x ^ v.y ^ v.z ^ v.w; }
};

template <int W>
__global__ void __launch_bounds__(kBlock) k_gather(const uint32_t* __restrict__ table,
                                                   const uint32_t* __restrict__ offs, uint32_t iters,
                                                   uint32_t* __restrict__ out,
                                                   unsigned long long* __restrict__ stamps) {
    typedef typename Vec<W>::T T;
    const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
    uint32_t o[kPerLane];
#pragma unroll
    for (int j = 0; j < kPerLane; ++j) o[j] = offs[(size_t)j * gridDim.x * kBlock + tid];   // byte offsets
    uint32_t acc = 0;
    unsigned long long t0, r0, t1, r1;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0), "=s"(r0) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    for (uint32_t it = 0; it < iters; ++it) {
        // wave-uniform shift (multiple of 64 words keeps every pattern's alignment)
        const uint32_t* base = table + ((it * 4099u * 64u) & (kShiftWords - 1u) & ~63u);
        const char* b = reinterpret_cast<const char*>(base);
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) acc ^= Vec<W>::fold(*reinterpret_cast<const T*>(b + o[j]));
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1), "=s"(r1) :: "memory");
    __builtin_amdgcn_sched_barrier(0);
    out[tid] = acc;
    if (threadIdx.x < 2)                                  // lanes 0, 1: a lane-indexed (vector) store
        stamps[2 * blockIdx.x + threadIdx.x] = threadIdx.x ? r1 - r0 : t1 - t0;
}

struct Result {
    double ms, lanes_per_clk_cu, clock_ghz, lanes_per_clk_cu_nominal;
};

template <int W>
Result run(const uint32_t* table, const std::vector<uint32_t>& offs_h, uint32_t blocks, uint32_t iters) {
    uint32_t *offs, *out;
    unsigned long long* stamps;
    CHECK(hipMalloc(&offs, offs_h.size() * 4));
    CHECK(hipMalloc(&out, (size_t)blocks * kBlock * 4));
    CHECK(hipMalloc(&stamps, (size_t)blocks * 2 * 8));
    CHECK(hipMemcpy(offs, offs_h.data(), offs_h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) k_gather<W><<<blocks, kBlock>>>(table, offs, iters, out, stamps);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        CHECK(hipEventRecord(a));
        k_gather<W><<<blocks, kBlock>>>(table, offs, iters, out, stamps);
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
    const double lanes = (double)blocks * kBlock * kPerLane * iters;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    Result r;
    r.ms = best;
    r.clock_ghz = ghz;
    r.lanes_per_clk_cu = lanes / (best * 1e-3) / (ghz * 1e9) / cus;
    r.lanes_per_clk_cu_nominal = lanes / (best * 1e-3) / (2.4e9) / cus;
    CHECK(hipFree(offs));
    CHECK(hipFree(out));
    CHECK(hipFree(stamps));
    return r;
}

int main() {
    const uint32_t blocks = 8192, iters = 64;             // 32 waves per CU, 16 x 64 gathers per lane
    const size_t n_lanes = (size_t)blocks * kBlock;
    uint32_t* table;
    CHECK(hipMalloc(&table, (size_t)(kTableWords + kShiftWords + 64) * 4));
    CHECK(hipMemset(table, 0x5a, (size_t)(kTableWords + kShiftWords + 64) * 4));
    std::mt19937 rng(1234);
    auto random_offs = [&](uint32_t align) {
        std::vector<uint32_t> v((size_t)kPerLane * n_lanes);
        for (auto& x : v) x = (rng() % (kTableWords / align)) * align * 4u;      // bytes
        return v;
    };
    std::vector<uint32_t> contig((size_t)kPerLane * n_lanes);
    for (int j = 0; j < kPerLane; ++j)
        for (size_t t = 0; t < n_lanes; ++t) {
            const size_t wave = t / 64, lane = t % 64;
            contig[(size_t)j * n_lanes + t] = (uint32_t)((((wave * kPerLane + j) * 64u) % kTableWords + lane) * 4u);
        }
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"what\": \"64-lane gathers from an L2-resident 1 MiB table: lane-addresses per clock per CU "
           "(tools/ta_rate.hip)\", \"cus\": %d, \"waves_per_cu\": %u, \"patterns\": {", cus,
           blocks * (kBlock / 64) / (uint32_t)cus);
    const char* names[4] = {"random_dword", "random_dwordx2", "random_dwordx4", "contiguous_dword"};
    for (int p = 0; p < 4; ++p) {
        Result r;
        if (p == 0) r = run<1>(table, random_offs(1), blocks, iters);
        else if (p == 1) r = run<2>(table, random_offs(2), blocks, iters);
        else if (p == 2) r = run<4>(table, random_offs(4), blocks, iters);
        else r = run<1>(table, contig, blocks, iters);
        printf("%s\"%s\": {\"ms\": %.4f, \"clock_ghz\": %.3f, \"lane_addr_per_clk_per_cu\": %.3f, "
               "\"lane_addr_per_clk_per_cu_at_2p4ghz\": %.3f}",
               p ? ", " : "", names[p], r.ms, r.clock_ghz, r.lanes_per_clk_cu, r.lanes_per_clk_cu_nominal);
        fflush(stdout);
    }
    printf("}}\n");
    CHECK(hipFree(table));
    return 0;
}
