// sh_device.h -- real spherical harmonics (Condon-Shortley phase) on gfx950.
//
// Basis and ordering of the reference's kernel_sh (shencoder/src/shencoder.cu:27-123):
// output l*l + l + m for degree l < DEG, m in [-l, l].  Evaluated with the
// associated-Legendre recurrence on Q_l^m = P_l^m / sin^m and the
// Re/Im parts of (x + i y)^m, carrying d/dx, d/dy, d/dz as dual numbers when
// the Jacobian is requested (shencoder.cu:125-355 writes the same
// derivatives of the polynomial in x, y, z).  Normalisation constants are
// folded at compile time.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>

namespace samnerf {

// K_l^m (times sqrt(2) for m != 0), as a constexpr table for l, m < 8.
constexpr double cx_sqrt(double x) {
    double r = x > 1.0 ? x : 1.0;
    for (int i = 0; i < 80; ++i) r = 0.5 * (r + x / r);
    return r;
}
constexpr double sh_k(int l, int m) {
    double f = 1.0;
    for (int k = l - m + 1; k <= l + m; ++k) f *= (double)k;
    double k = cx_sqrt((2.0 * l + 1.0) / (4.0 * 3.14159265358979323846) / f);
    return m == 0 ? k : k * 1.41421356237309504880;
}
constexpr double sh_q0(int m) {  // Q_m^m = (-1)^m (2m-1)!!
    double d = 1.0;
    for (int k = 2 * m - 1; k > 1; k -= 2) d *= k;
    return (m & 1) ? -d : d;
}

// All recurrence constants, evaluated at compile time.
struct ShConst {
    float k[8][8];     // sh_k(l, m)
    float q0[8];       // Q_m^m
    float inv[9];      // 1 / n
};
constexpr ShConst make_sh_const() {
    ShConst c{};
    for (int l = 0; l < 8; ++l)
        for (int m = 0; m <= l; ++m) c.k[l][m] = (float)sh_k(l, m);
    for (int m = 0; m < 8; ++m) c.q0[m] = (float)sh_q0(m);
    for (int n = 1; n < 9; ++n) c.inv[n] = (float)(1.0 / (double)n);
    return c;
}
constexpr ShConst kShConst = make_sh_const();

struct Dual {
    float v, dx, dy, dz;
};
__device__ __forceinline__ Dual dmul(Dual a, Dual b) {
    return {a.v * b.v, a.dx * b.v + a.v * b.dx, a.dy * b.v + a.v * b.dy, a.dz * b.v + a.v * b.dz};
}
__device__ __forceinline__ Dual dsc(Dual a, float s) { return {a.v * s, a.dx * s, a.dy * s, a.dz * s}; }
__device__ __forceinline__ Dual dsub(Dual a, Dual b) {
    return {a.v - b.v, a.dx - b.dx, a.dy - b.dy, a.dz - b.dz};
}
__device__ __forceinline__ Dual dadd(Dual a, Dual b) {
    return {a.v + b.v, a.dx + b.dx, a.dy + b.dy, a.dz + b.dz};
}

// Values only (the fused renderer's direction encoding, DEG = 4 there).
template <int DEG>
__device__ __forceinline__ void sh_values(float x, float y, float z, float* out) {
    float cm[DEG], sm[DEG];
    cm[0] = 1.0f;
    sm[0] = 0.0f;
#pragma unroll
    for (int m = 1; m < DEG; ++m) {
        cm[m] = x * cm[m - 1] - y * sm[m - 1];
        sm[m] = x * sm[m - 1] + y * cm[m - 1];
    }
#pragma unroll
    for (int m = 0; m < DEG; ++m) {
        float qp = 0.0f, q = kShConst.q0[m];
#pragma unroll
        for (int l = m; l < DEG; ++l) {
            if (l > m) {
                float t = ((float)(2 * l - 1) * (z * q) - (float)(l + m - 1) * qp) *
                          kShConst.inv[l - m];
                qp = q;
                q = t;
            }
            const float k = kShConst.k[l][m];
            out[l * l + l + m] = (q * cm[m]) * k;
            if (m > 0) out[l * l + l - m] = (q * sm[m]) * k;
        }
    }
}

// Values + Jacobian (rows d/dx, d/dy, d/dz), any degree <= 8.
template <int DEG>
__device__ __forceinline__ void sh_values_grad(float x, float y, float z, float* out, float* dx,
                                               float* dy, float* dz) {
    const Dual X{x, 1, 0, 0}, Y{y, 0, 1, 0}, Z{z, 0, 0, 1};
    Dual cm[DEG], sm[DEG];
    cm[0] = {1, 0, 0, 0};
    sm[0] = {0, 0, 0, 0};
#pragma unroll
    for (int m = 1; m < DEG; ++m) {
        cm[m] = dsub(dmul(X, cm[m - 1]), dmul(Y, sm[m - 1]));
        sm[m] = dadd(dmul(X, sm[m - 1]), dmul(Y, cm[m - 1]));
    }
#pragma unroll
    for (int m = 0; m < DEG; ++m) {
        Dual qp{0, 0, 0, 0}, q{kShConst.q0[m], 0, 0, 0};
#pragma unroll
        for (int l = m; l < DEG; ++l) {
            if (l > m) {
                Dual t = dsub(dsc(dmul(Z, q), (float)(2 * l - 1)), dsc(qp, (float)(l + m - 1)));
                t = dsc(t, kShConst.inv[l - m]);
                qp = q;
                q = t;
            }
            const float k = kShConst.k[l][m];
            const Dual p = dsc(dmul(q, cm[m]), k);
            const int ip = l * l + l + m;
            out[ip] = p.v;
            if (dx) { dx[ip] = p.dx; dy[ip] = p.dy; dz[ip] = p.dz; }
            if (m > 0) {
                const Dual n = dsc(dmul(q, sm[m]), k);
                const int in = l * l + l - m;
                out[in] = n.v;
                if (dx) { dx[in] = n.dx; dy[in] = n.dy; dz[in] = n.dz; }
            }
        }
    }
}

}  // namespace samnerf
