/*
 * oracle/encoders_oracle.c -- CPU restatement of the reference's native encoders.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing on the product path may link or call this
 * file: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * load it, and only as the checker / the timed CPU baseline.
 *
 * What it restates (reference paths relative to the reference root):
 *   grid forward        gridencoder/src/gridencoder.cu:82-249   (kernel_grid)
 *   grid backward       gridencoder/src/gridencoder.cu:252-349  (kernel_grid_backward)
 *   input backward      gridencoder/src/gridencoder.cu:352-378  (kernel_input_backward)
 *   total variation     gridencoder/src/gridencoder.cu:525-631  (kernel_grad_tv)
 *   weight decay        gridencoder/src/gridencoder.cu:670-703  (kernel_grad_wd)
 *   SH forward/backward shencoder/src/shencoder.cu:27-382
 *   freq fwd/backward   freqencoder/src/freqencoder.cu:30-94
 *
 * Floating-point contract.  The reference is compiled by nvcc with its default
 * --fmad=true, so `a*b + c` patterns become one fused multiply-add.  This file
 * is compiled with -ffp-contract=off and spells every such contraction as an
 * explicit fmaf(), exactly where nvcc contracts (gridencoder.cu:148 position,
 * :191 accumulation, :239 dy_dx accumulation, :373 input backward).  With that,
 * the integer corner indices and the forward features are reproducible bit for
 * bit on identical float inputs.
 *
 * Spherical harmonics are evaluated with the associated-Legendre recurrence and
 * forward-mode derivatives (dual numbers) instead of the reference's expanded
 * polynomials; the basis (Condon-Shortley phase, real form, ordering
 * l*l + l + m) is pinned against SciPy in tests/test_oracle.py.  Values agree
 * with the expanded polynomials to float rounding, not bit for bit.
 *
 * The backward kernels run sequentially here (b, level, corner order), so the
 * oracle's gradients are deterministic; the device ones are order-dependent
 * float atomics, compared with a tolerance.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#define MAXD 8

/* ---------------------------------------------------------------- grid ---- */

typedef struct {
    uint32_t size;      /* rows in this level's table (offsets[l+1]-offsets[l]) */
    uint32_t res;       /* indexing resolution (float formula, gridencoder.cu:133) */
} level_info;

static level_info level_of(const int32_t *offsets, uint32_t level, float S, uint32_t H) {
    level_info li;
    li.size = (uint32_t)(offsets[level + 1] - offsets[level]);
    /* ceil(exp2f(level*S)*H) evaluated in float, exactly like the device code */
    float scale = exp2f((float)level * S);
    li.res = (uint32_t)ceilf(scale * (float)H);
    return li;
}

/* gridencoder.cu:45-79: dense index while the running stride fits the table,
 * otherwise (hash grids) the coherent prime hash; always reduced mod size. */
static uint32_t corner_row(uint32_t gridtype, uint32_t size, uint32_t res,
                           const uint32_t *cell, uint32_t D) {
    static const uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                       2097192037u, 1434869437u, 2165219737u};
    uint32_t stride = 1u, row = 0u, d = 0u;
    while (d < D && stride <= size) {
        row += cell[d] * stride;
        stride *= res;
        ++d;
    }
    if (gridtype == 0u && stride > size) {
        row = 0u;
        for (uint32_t k = 0; k < D; ++k) row ^= cell[k] * primes[k];
    }
    return row % size;
}

static int out_of_unit_cube(const float *x, uint32_t D) {
    for (uint32_t d = 0; d < D; ++d)
        if (x[d] < 0.0f || x[d] > 1.0f) return 1;
    return 0;
}

/* Cell coordinate + fractional position (gridencoder.cu:141-160). */
static void locate(const float *x, uint32_t D, uint32_t res, int align_corners,
                   uint32_t interp, float *frac, float *dfrac, uint32_t *cell) {
    for (uint32_t d = 0; d < D; ++d) {
        float p;
        uint32_t g;
        if (align_corners) {
            p = x[d] * (float)(res - 1u);
            g = (uint32_t)floorf(p);
            if (g > res - 2u) g = res - 2u;
        } else {
            p = fmaf(x[d], (float)res, -0.5f);          /* nvcc contracts :148 */
            p = fminf(fmaxf(p, 0.0f), (float)(res - 1u));
            g = (uint32_t)floorf(p);
        }
        p -= (float)g;
        if (interp == 1u) {
            if (dfrac) dfrac[d] = (6.0f * p) * (1.0f - p);
            p = (p * p) * fmaf(-2.0f, p, 3.0f);
        } else if (dfrac) {
            dfrac[d] = 1.0f;
        }
        frac[d] = p;
        cell[d] = g;
    }
}

/* Trilinear (D-linear) corner weight and cell for corner bit pattern `c`. */
static float corner(uint32_t c, uint32_t D, uint32_t res, const float *frac,
                    const uint32_t *cell, uint32_t *out_cell) {
    float w = 1.0f;
    for (uint32_t d = 0; d < D; ++d) {
        if (c & (1u << d)) {
            w *= frac[d];
            out_cell[d] = (cell[d] + 1u < res - 1u) ? cell[d] + 1u : res - 1u;
        } else {
            w *= 1.0f - frac[d];
            out_cell[d] = cell[d];
        }
    }
    return w;
}

/* outputs: [L, B, C]; dy_dx: [B, L, D, C] or NULL.  Levels >= max_level are
 * left untouched (the caller zero-fills, grid.py:52). */
void oracle_grid_encode_forward(const float *inputs, const float *embeddings,
                                const int32_t *offsets, float *outputs,
                                uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                uint32_t max_level, float S, uint32_t H,
                                float *dy_dx, uint32_t gridtype,
                                int align_corners, uint32_t interp,
                                uint32_t *corner_rows /* optional [L,B,2^D] */) {
    for (uint32_t level = 0; level < max_level; ++level) {
        level_info li = level_of(offsets, level, S, H);
        const float *table = embeddings + (size_t)offsets[level] * C;
        /* points are independent: parallel over b (results do not depend on
         * the thread count) -- only for the bench's CPU-baseline timing */
#pragma omp parallel for schedule(static)
        for (uint32_t b = 0; b < B; ++b) {
            const float *x = inputs + (size_t)b * D;
            float *out = outputs + ((size_t)level * B + b) * C;
            float *dd = dy_dx ? dy_dx + ((size_t)b * L + level) * D * C : NULL;
            if (out_of_unit_cube(x, D)) {
                for (uint32_t ch = 0; ch < C; ++ch) out[ch] = 0.0f;
                if (dd) memset(dd, 0, sizeof(float) * D * C);
                if (corner_rows)
                    for (uint32_t c = 0; c < (1u << D); ++c)
                        corner_rows[((size_t)level * B + b) * (1u << D) + c] = 0xffffffffu;
                continue;
            }
            float frac[MAXD], dfrac[MAXD];
            uint32_t cell[MAXD], cc[MAXD];
            locate(x, D, li.res, align_corners, interp, frac, dfrac, cell);

            float acc[64];
            for (uint32_t ch = 0; ch < C; ++ch) acc[ch] = 0.0f;
            for (uint32_t c = 0; c < (1u << D); ++c) {
                float w = corner(c, D, li.res, frac, cell, cc);
                uint32_t row = corner_row(gridtype, li.size, li.res, cc, D);
                if (corner_rows)
                    corner_rows[((size_t)level * B + b) * (1u << D) + c] = row;
                const float *e = table + (size_t)row * C;
                for (uint32_t ch = 0; ch < C; ++ch) acc[ch] = fmaf(w, e[ch], acc[ch]); /* :191 */
            }
            for (uint32_t ch = 0; ch < C; ++ch) out[ch] = acc[ch];

            if (dd) {
                const float span = (float)(align_corners ? li.res - 1u : li.res);
                for (uint32_t gd = 0; gd < D; ++gd) {
                    float g[64];
                    for (uint32_t ch = 0; ch < C; ++ch) g[ch] = 0.0f;
                    for (uint32_t c = 0; c < (1u << (D - 1u)); ++c) {
                        float w = span;
                        for (uint32_t nd = 0; nd < D - 1u; ++nd) {
                            uint32_t d = nd >= gd ? nd + 1u : nd;
                            if (c & (1u << nd)) {
                                w *= frac[d];
                                cc[d] = (cell[d] + 1u < li.res - 1u) ? cell[d] + 1u : li.res - 1u;
                            } else {
                                w *= 1.0f - frac[d];
                                cc[d] = cell[d];
                            }
                        }
                        cc[gd] = cell[gd];
                        uint32_t lo = corner_row(gridtype, li.size, li.res, cc, D);
                        cc[gd] = (cell[gd] + 1u < li.res - 1u) ? cell[gd] + 1u : li.res - 1u;
                        uint32_t hi = corner_row(gridtype, li.size, li.res, cc, D);
                        for (uint32_t ch = 0; ch < C; ++ch) {
                            float diff = table[(size_t)hi * C + ch] - table[(size_t)lo * C + ch];
                            g[ch] = fmaf(w * diff, dfrac[gd], g[ch]);            /* :239 */
                        }
                    }
                    for (uint32_t ch = 0; ch < C; ++ch) dd[gd * C + ch] = g[ch];
                }
            }
        }
    }
}

/* grad: [L, B, C]; grad_embeddings: [rows, C] accumulated into (caller zeroes). */
void oracle_grid_encode_backward(const float *grad, const float *inputs,
                                 const float *embeddings, const int32_t *offsets,
                                 float *grad_embeddings, uint32_t B, uint32_t D,
                                 uint32_t C, uint32_t L, uint32_t max_level,
                                 float S, uint32_t H, const float *dy_dx,
                                 float *grad_inputs, uint32_t gridtype,
                                 int align_corners, uint32_t interp) {
    (void)embeddings;
    for (uint32_t level = 0; level < max_level; ++level) {
        level_info li = level_of(offsets, level, S, H);
        float *gtab = grad_embeddings + (size_t)offsets[level] * C;
        for (uint32_t b = 0; b < B; ++b) {
            const float *x = inputs + (size_t)b * D;
            if (out_of_unit_cube(x, D)) continue;
            float frac[MAXD];
            uint32_t cell[MAXD], cc[MAXD];
            locate(x, D, li.res, align_corners, interp, frac, NULL, cell);
            const float *g = grad + ((size_t)level * B + b) * C;
            for (uint32_t c = 0; c < (1u << D); ++c) {
                float w = corner(c, D, li.res, frac, cell, cc);
                uint32_t row = corner_row(gridtype, li.size, li.res, cc, D);
                for (uint32_t ch = 0; ch < C; ++ch)
                    gtab[(size_t)row * C + ch] += w * g[ch];
            }
        }
    }
    if (dy_dx && grad_inputs) {
        for (uint32_t b = 0; b < B; ++b)
            for (uint32_t d = 0; d < D; ++d) {
                float r = 0.0f;
                for (uint32_t l = 0; l < L; ++l)
                    for (uint32_t ch = 0; ch < C; ++ch)
                        r = fmaf(grad[((size_t)l * B + b) * C + ch],
                                 dy_dx[(((size_t)b * L + l) * D + d) * C + ch], r); /* :373 */
                grad_inputs[(size_t)b * D + d] = r;
            }
    }
}

/* gridencoder.cu:525-631 -- in-place TV gradient at `inputs`, all L levels. */
void oracle_grad_total_variation(const float *inputs, const float *embeddings,
                                 float *grad, const int32_t *offsets, float weight,
                                 uint32_t B, uint32_t D, uint32_t C, uint32_t L,
                                 float S, uint32_t H, uint32_t gridtype,
                                 int align_corners) {
    const float w = weight / (float)(2u * D);
    for (uint32_t level = 0; level < L; ++level) {
        level_info li = level_of(offsets, level, S, H);
        const float *table = embeddings + (size_t)offsets[level] * C;
        float *gtab = grad + (size_t)offsets[level] * C;
        for (uint32_t b = 0; b < B; ++b) {
            const float *x = inputs + (size_t)b * D;
            if (out_of_unit_cube(x, D)) continue;
            float frac[MAXD];
            uint32_t cell[MAXD];
            locate(x, D, li.res, align_corners, 0u, frac, NULL, cell);
            uint32_t here = corner_row(gridtype, li.size, li.res, cell, D);
            float sum[64], sq[64];
            for (uint32_t ch = 0; ch < C; ++ch) sum[ch] = sq[ch] = 0.0f;
            for (uint32_t d = 0; d < D; ++d) {
                uint32_t keep = cell[d];
                if (keep < li.res) {
                    cell[d] = keep + 1u;
                    uint32_t nb = corner_row(gridtype, li.size, li.res, cell, D);
                    for (uint32_t ch = 0; ch < C; ++ch) {
                        float v = table[(size_t)here * C + ch] - table[(size_t)nb * C + ch];
                        sum[ch] += v;
                        sq[ch] = fmaf(v, v, sq[ch]);
                    }
                }
                if (keep > 0u) {
                    cell[d] = keep - 1u;
                    uint32_t nb = corner_row(gridtype, li.size, li.res, cell, D);
                    for (uint32_t ch = 0; ch < C; ++ch) {
                        float v = table[(size_t)here * C + ch] - table[(size_t)nb * C + ch];
                        sum[ch] += v;
                        sq[ch] = fmaf(v, v, sq[ch]);
                    }
                }
                cell[d] = keep;
            }
            for (uint32_t ch = 0; ch < C; ++ch)
                gtab[(size_t)here * C + ch] += (w * sum[ch]) * (1.0f / sqrtf(sq[ch] + 1e-9f));
        }
    }
}

/* gridencoder.cu:670-703 -- level-normalised L2 gradient over all rows. */
void oracle_grad_weight_decay(const float *embeddings, float *grad,
                              const int32_t *offsets, float weight, uint32_t rows,
                              uint32_t C, uint32_t L) {
    for (uint64_t e = 0; e < (uint64_t)rows * C; ++e) {
        uint32_t n = (uint32_t)(e / C);
        uint32_t level = 0;
        for (uint32_t m = 0; m < L; ++m)
            if ((uint32_t)offsets[m] <= n) level = m;
        uint32_t size = (uint32_t)(offsets[level + 1] - offsets[level]);
        grad[e] += ((2.0f * weight) * embeddings[e]) / (float)size;
    }
}

/* ------------------------------------------------------------------ SH ---- */

/* Dual number: value and d/dx, d/dy, d/dz. */
typedef struct { float v, dx, dy, dz; } dual;

static dual dmul(dual a, dual b) {
    dual r = {a.v * b.v, a.dx * b.v + a.v * b.dx, a.dy * b.v + a.v * b.dy,
              a.dz * b.v + a.v * b.dz};
    return r;
}
static dual dscale(dual a, float s) { dual r = {a.v * s, a.dx * s, a.dy * s, a.dz * s}; return r; }
static dual dsub(dual a, dual b) { dual r = {a.v - b.v, a.dx - b.dx, a.dy - b.dy, a.dz - b.dz}; return r; }
static dual dadd(dual a, dual b) { dual r = {a.v + b.v, a.dx + b.dx, a.dy + b.dy, a.dz + b.dz}; return r; }

/* Normalisation K_l^m * (sqrt(2) if m != 0), in double then rounded. */
static double sh_norm(int l, int m) {
    double f = 1.0;
    for (int k = l - m + 1; k <= l + m; ++k) f *= (double)k;      /* (l+m)!/(l-m)! */
    double k = sqrt((2.0 * l + 1.0) / (4.0 * M_PI) / f);
    return m == 0 ? k : k * sqrt(2.0);
}

/* Real SH with Condon-Shortley phase, degree < 9, output index l*l + l + m. */
static void sh_eval(float x, float y, float z, uint32_t degree, float *out, float *dx,
                    float *dy, float *dz) {
    dual X = {x, 1, 0, 0}, Y = {y, 0, 1, 0}, Z = {z, 0, 0, 1};
    dual cm[9], sm[9];                      /* Re/Im of (x + i y)^m */
    cm[0] = (dual){1, 0, 0, 0};
    sm[0] = (dual){0, 0, 0, 0};
    for (int m = 1; m < (int)degree; ++m) {
        cm[m] = dsub(dmul(X, cm[m - 1]), dmul(Y, sm[m - 1]));
        sm[m] = dadd(dmul(X, sm[m - 1]), dmul(Y, cm[m - 1]));
    }
    for (int m = 0; m < (int)degree; ++m) {
        /* Q_l^m = P_l^m / sin^m, starting at Q_m^m = (-1)^m (2m-1)!! */
        double dfact = 1.0;
        for (int k = 2 * m - 1; k > 1; k -= 2) dfact *= k;
        dual q_prev = {0, 0, 0, 0};
        dual q = {(float)((m & 1) ? -dfact : dfact), 0, 0, 0};
        for (int l = m; l < (int)degree; ++l) {
            if (l > m) {
                /* ((2l-1) z Q_{l-1} - (l+m-1) Q_{l-2}) / (l-m) */
                dual t = dsub(dscale(dmul(Z, q), (float)(2 * l - 1)),
                              dscale(q_prev, (float)(l + m - 1)));
                t = dscale(t, 1.0f / (float)(l - m));
                q_prev = q;
                q = t;
            }
            float k = (float)sh_norm(l, m);
            dual pos = dscale(dmul(q, cm[m]), k);
            int ip = l * l + l + m;
            out[ip] = pos.v;
            if (dx) { dx[ip] = pos.dx; dy[ip] = pos.dy; dz[ip] = pos.dz; }
            if (m > 0) {
                dual neg = dscale(dmul(q, sm[m]), k);
                int in = l * l + l - m;
                out[in] = neg.v;
                if (dx) { dx[in] = neg.dx; dy[in] = neg.dy; dz[in] = neg.dz; }
            }
        }
    }
}

/* inputs [B, D=3] (already unit length, sphere_harmonics.py:82); outputs
 * [B, C*C]; dy_dx [B, D, C*C] or NULL.  C is the degree (1..8). */
void oracle_sh_encode_forward(const float *inputs, float *outputs, uint32_t B,
                              uint32_t D, uint32_t C, float *dy_dx) {
    const uint32_t C2 = C * C;
#pragma omp parallel for schedule(static)
    for (uint32_t b = 0; b < B; ++b) {
        const float *v = inputs + (size_t)b * D;
        float *dd = dy_dx ? dy_dx + (size_t)b * D * C2 : NULL;
        sh_eval(v[0], v[1], v[2], C, outputs + (size_t)b * C2, dd, dd ? dd + C2 : NULL,
                dd ? dd + 2 * C2 : NULL);
    }
}

/* grad [B, C*C]; grad_inputs [B, D] accumulated into (caller zeroes). */
void oracle_sh_encode_backward(const float *grad, const float *inputs, uint32_t B,
                               uint32_t D, uint32_t C, const float *dy_dx,
                               float *grad_inputs) {
    (void)inputs;
    const uint32_t C2 = C * C;
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t d = 0; d < D; ++d) {
            float r = grad_inputs[(size_t)b * D + d];
            for (uint32_t ch = 0; ch < C2; ++ch)
                r = fmaf(grad[(size_t)b * C2 + ch], dy_dx[((size_t)b * D + d) * C2 + ch], r);
            grad_inputs[(size_t)b * D + d] = r;
        }
}

/* ---------------------------------------------------------------- freq ---- */

/* outputs [B, C], C = D + 2*D*deg: [x, sin(2^0 x), cos(2^0 x), sin(2^1 x), ...]
 * with each block D wide (freqencoder.cu:30-58).  Accurate sinf here; the
 * reference's __sinf is a fast approximation (tolerance in the tests). */
void oracle_freq_encode_forward(const float *inputs, uint32_t B, uint32_t D,
                                uint32_t deg, uint32_t C, float *outputs) {
    const float half_pi = 1.57079632679489662f;
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t c = 0; c < C; ++c) {
            float *o = outputs + (size_t)b * C + c;
            if (c < D) { *o = inputs[(size_t)b * D + c]; continue; }
            uint32_t blk = c / D - 1u, d = c % D;
            float arg = ldexpf(inputs[(size_t)b * D + d], (int)(blk / 2u)) +
                        (float)(blk % 2u) * half_pi;
            *o = sinf(arg);
        }
    (void)deg;
}

/* grad [B, C]; outputs [B, C] (forward result); grad_inputs [B, D]. */
void oracle_freq_encode_backward(const float *grad, const float *outputs, uint32_t B,
                                 uint32_t D, uint32_t deg, uint32_t C,
                                 float *grad_inputs) {
    for (uint32_t b = 0; b < B; ++b)
        for (uint32_t d = 0; d < D; ++d) {
            const float *g = grad + (size_t)b * C;
            const float *o = outputs + (size_t)b * C;
            float r = g[d];
            for (uint32_t f = 0; f < deg; ++f) {
                uint32_t s = D + 2u * f * D, k = s + D;
                float t = fmaf(g[s + d], o[k + d], -(g[k + d] * o[s + d]));
                r = fmaf(ldexpf(1.0f, (int)f), t, r);
            }
            grad_inputs[(size_t)b * D + d] = r;
        }
}
