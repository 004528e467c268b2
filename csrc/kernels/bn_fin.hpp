// BN finalize math shared by the standalone finalize kernels (bn.hip) and the in-kernel
// finalize of the convolution's statistics epilogues (conv.hip): per channel, from the f64 sums
// of the kStatSlots slots, the forward batch statistics / affine coefficients / running stats,
// or the backward dgamma / dbeta and the three backward-apply coefficients.  One definition,
// so both paths produce bit-identical results.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kfk {

// forward: s = sum x, q = sum x^2 over `rows` elements of channel c.  The per-channel inputs come
// in as values (g, b: gamma / beta or 1 / 0; rm, rv: the running stats, used when run_mean is set)
// so that a caller can issue their loads together with the slot loads: loaded here, behind the
// stores, every one was a serial memory round trip (bn_sums_finalize measured 5.7 us for ~6 of them).
__device__ __forceinline__ void bn_fin_fwd_channel(int c, int C, double s, double q, int64_t rows, float g, float b,
                                                   float rm, float rv, float *mean, float *invstd, float *run_mean,
                                                   float *run_var, float momentum, float eps, float *coef) {
    const double m = s / rows;
    double var = q / rows - m * m;
    if (var < 0) var = 0;
    const float is = rsqrtf(static_cast<float>(var) + eps);
    const float sc = g * is;
    mean[c] = static_cast<float>(m);
    invstd[c] = is;
    if (run_mean) {
        const double unbiased = rows > 1 ? var * rows / (rows - 1) : var;
        run_mean[c] = (1.f - momentum) * rm + momentum * static_cast<float>(m);
        run_var[c] = (1.f - momentum) * rv + momentum * static_cast<float>(unbiased);
    }
    coef[c] = sc;
    coef[C + c] = b - static_cast<float>(m) * sc;
}

// backward: s0 = sum dz, s1 = sum dz * x (dz = the gradient of the BN output under the ReLU gate);
// g = gamma (or 1), mu / is = the forward batch mean / inverse std of channel c, as values.
__device__ __forceinline__ void bn_fin_bwd_channel(int c, int C, double s0, double s1, int64_t rows, float g,
                                                   float mu, float is, float *dgamma, float *dbeta, float *coef,
                                                   bool training) {
    const double db = s0, dg = static_cast<double>(is) * (s1 - static_cast<double>(mu) * db);
    dgamma[c] = static_cast<float>(dg);
    dbeta[c] = static_cast<float>(db);
    const float a = g * is;
    if (training) {
        const float inv_m = 1.f / static_cast<float>(rows);
        const float k2 = -a * static_cast<float>(dg) * is * inv_m;
        coef[c] = a;
        coef[C + c] = k2;
        coef[2 * C + c] = -a * static_cast<float>(db) * inv_m - k2 * mu;
    } else {
        coef[c] = a;
        coef[C + c] = 0.f;
        coef[2 * C + c] = 0.f;
    }
}

// pointer forms (the in-launch finalize of conv.hip): the loads behind the caller's own
__device__ __forceinline__ void bn_fin_fwd_channel_p(int c, int C, double s, double q, int64_t rows,
                                                     const float *gamma, const float *beta, float *mean,
                                                     float *invstd, float *run_mean, float *run_var, float momentum,
                                                     float eps, float *coef) {
    bn_fin_fwd_channel(c, C, s, q, rows, gamma ? gamma[c] : 1.f, beta ? beta[c] : 0.f, run_mean ? run_mean[c] : 0.f,
                       run_mean ? run_var[c] : 0.f, mean, invstd, run_mean, run_var, momentum, eps, coef);
}

__device__ __forceinline__ void bn_fin_bwd_channel_p(int c, int C, double s0, double s1, int64_t rows,
                                                     const float *gamma, const float *mean, const float *invstd,
                                                     float *dgamma, float *dbeta, float *coef, bool training) {
    bn_fin_bwd_channel(c, C, s0, s1, rows, gamma ? gamma[c] : 1.f, mean[c], invstd[c], dgamma, dbeta, coef,
                       training);
}

}  // namespace kfk
