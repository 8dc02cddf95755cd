// common.cpp -- host-side helpers of libsamnerf_hip.so (error state, level
// tables, torch-exact linspace).
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "samnerf_common.h"

namespace samnerf {

static thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(SAMNERF_ELAUNCH, "%s: launch failed: %s", what, hipGetErrorString(e));
    return SAMNERF_OK;
}

ResTable make_res_table(uint32_t L, float S, uint32_t H) {
    ResTable t;
    for (uint32_t l = 0; l < 32; ++l) {
        // gridencoder.cu:133 -- (uint32_t)ceil(exp2f(level * S) * H) in float
        float scale = std::exp2f((float)l * S);
        t.res[l] = l < L ? (uint32_t)std::ceil(scale * (float)H) : 0u;
    }
    return t;
}

LevelDesc make_level(uint32_t off, uint32_t size, uint32_t res, uint32_t gridtype) {
    LevelDesc d;
    d.off = off;
    d.size = size;
    d.res = res;
    d.fres = (float)res;
    d.ftop = (float)(res - 1u);
    // Running stride of get_grid_index (gridencoder.cu:63-76), uint32 wrap.
    uint32_t stride = 1u, dims = 0u;
    while (dims < 3u && stride <= size) {
        stride *= res;
        ++dims;
    }
    bool hashed = (gridtype == 0u && stride > size);
    d.flags = (hashed ? kHashed : 0u) | (((size & (size - 1u)) == 0u) ? kPow2 : 0u);
    // The fused path only handles hash grids whose dense levels index all three
    // axes (true for every NeRFNetwork grid); tiled grids go through the
    // drop-in encoder, which evaluates get_grid_index generically.
    return d;
}

}  // namespace samnerf

extern "C" {

const char* samnerf_version(void) { return "samnerf_hip 0.3 (gfx950)"; }

// 1 in the diagnostic build whose kernels read the A/B variant switches from
// the environment (samnerf_common.h diag_env), 0 in the product library
int samnerf_diag_variants(void) {
#ifdef SAMNERF_DIAG_VARIANTS
    return 1;
#else
    return 0;
#endif
}

const char* samnerf_last_error(void) { return samnerf::g_err; }

// torch.linspace on the CPU for float32 (ATen RangeFactoriesKernel): step in
// float, the first half fma(step, i, start), the second half
// fma(-step, steps-1-i, end).  Verified bit-exact against torch.linspace in
// tests/test_capi.py.
void samnerf_linspace_host(float start, float end, uint32_t steps, float* out) {
    if (steps == 0) return;
    if (steps == 1) {
        out[0] = start;
        return;
    }
    const float step = (end - start) / (float)(steps - 1u);
    const uint32_t half = steps / 2u;
    for (uint32_t i = 0; i < steps; ++i)
        out[i] = i < half ? std::fmaf(step, (float)i, start)
                          : std::fmaf(-step, (float)(steps - 1u - i), end);
}

}  // extern "C"
