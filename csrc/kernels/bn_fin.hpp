// BN finalize math shared by the standalone finalize kernels (bn.hip) and the in-kernel
// finalize of the convolution's statistics epilogues (conv.hip): per channel, from the f64 sums
// of the kStatSlots slots, the forward batch statistics / affine coefficients / running stats,
// or the backward dgamma / dbeta and the three backward-apply coefficients.  One definition,
// so both paths produce bit-identical results.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace kfk {

// forward: s = sum x, q = sum x^2 over `rows` elements of channel c
__device__ __forceinline__ void bn_fin_fwd_channel(int c, int C, double s, double q, int64_t rows, const float *gamma,
                                                   const float *beta, float *mean, float *invstd, float *run_mean,
                                                   float *run_var, float momentum, float eps, float *coef) {
    const double m = s / rows;
    double var = q / rows - m * m;
    if (var < 0) var = 0;
    const float is = rsqrtf(static_cast<float>(var) + eps);
    mean[c] = static_cast<float>(m);
    invstd[c] = is;
    if (run_mean) {
        const double unbiased = rows > 1 ? var * rows / (rows - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * static_cast<float>(m);
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * static_cast<float>(unbiased);
    }
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    const float sc = g * is;
    coef[c] = sc;
    coef[C + c] = b - static_cast<float>(m) * sc;
}

// backward: s0 = sum dz, s1 = sum dz * x (dz = the gradient of the BN output under the ReLU gate)
__device__ __forceinline__ void bn_fin_bwd_channel(int c, int C, double s0, double s1, int64_t rows,
                                                   const float *gamma, const float *mean, const float *invstd,
                                                   float *dgamma, float *dbeta, float *coef, bool training) {
    const double db = s0, dg = static_cast<double>(invstd[c]) * (s1 - static_cast<double>(mean[c]) * db);
    dgamma[c] = static_cast<float>(dg);
    dbeta[c] = static_cast<float>(db);
    const float g = gamma ? gamma[c] : 1.f;
    const float a = g * invstd[c];
    if (training) {
        const float inv_m = 1.f / static_cast<float>(rows);
        const float k2 = -a * static_cast<float>(dg) * invstd[c] * inv_m;
        coef[c] = a;
        coef[C + c] = k2;
        coef[2 * C + c] = -a * static_cast<float>(db) * inv_m - k2 * mean[c];
    } else {
        coef[c] = a;
        coef[C + c] = 0.f;
        coef[2 * C + c] = 0.f;
    }
}

}  // namespace kfk
