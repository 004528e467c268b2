// Shared device helpers for the kungfu-amd CDNA4 (gfx950) kernels.
//
// Conventions for every bandwidth-bound kernel here (cdna_hip_programming.md
// §6 G11/G13, App. B):
//   * 256-thread blocks (4 waves of 64), 16-byte vector loads/stores per lane,
//   * grid = min(ceil(n / (256 * VEC)), 2048) with a grid-stride loop, so a
//     launch fills all 256 CUs and long tensors amortise launch cost,
//   * f32 accumulation for bf16/f16 data, round-to-nearest-even on store,
//   * wave64 reductions via __shfl_xor (64-lane), then LDS across the 4 waves.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace kfk {

// Developer A/B switches (kungfu_amd/knobs.py kind "dev"): `name` is read from the environment
// only when KUNGFU_DEV_KNOBS=1 is set too; otherwise the measured default `def` holds, so a
// stale shell variable cannot change a production run.
inline int dev_knob(const char *name, int def) {
    static const bool dev = [] {
        const char *e = std::getenv("KUNGFU_DEV_KNOBS");
        return e && *e && std::atoi(e) != 0;
    }();
    if (!dev) return def;
    const char *e = std::getenv(name);
    return e && *e ? std::atoi(e) : def;
}

constexpr int kBlock = 256;
constexpr int kWave = 64;
constexpr int kMaxGrid = 2048;

inline int grid_for(size_t n_vec) {
    size_t g = (n_vec + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > static_cast<size_t>(kMaxGrid)) g = kMaxGrid;
    return static_cast<int>(g);
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float(static_cast<uint32_t>(h) << 16); }

// f32 -> bf16, round to nearest even (finite inputs; NaN payloads are not preserved).  Integer
// rounding, NOT gfx950's v_cvt_pk_bf16_f32: the same bits for every finite input
// (tools/diag/cvt_check.hip, 2^26 patterns), but the instruction measured far slower in the kernels
// -- the NT GEMM with it 6.5x slower (101.7 vs 15.7 ms over 108 launches), ResNet-50 21.17 vs
// 20.35 ms/step, BERT-base 26.8 vs 15.95 ms/step (tools/runs/gpu_r6_t13.sh / t14, same box).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>(u >> 16);
}
// (lo, hi) -> one 32-bit word, lo in the low half
__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
    return static_cast<uint32_t>(f32_to_bf16(lo)) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
}

__device__ __forceinline__ float f16_to_f32(uint16_t h) {
    _Float16 x;
    __builtin_memcpy(&x, &h, 2);
    return static_cast<float>(x);
}

__device__ __forceinline__ uint16_t f32_to_f16(float f) {
    _Float16 x = static_cast<_Float16>(f);
    uint16_t h;
    __builtin_memcpy(&h, &x, 2);
    return h;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide sum of up to two values; result valid in thread 0.
template <int N>
__device__ __forceinline__ void block_sum(float (&v)[N], float (*lds)[kBlock / kWave]) {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        v[i] = wave_sum(v[i]);
        if (lane == 0) lds[i][wid] = v[i];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            float s = 0;
#pragma unroll
            for (int w = 0; w < kBlock / kWave; ++w) s += lds[i][w];
            v[i] = s;
        }
    }
}

enum DT : int { DT_U8 = 0, DT_I32 = 6, DT_I64 = 7, DT_F16 = 8, DT_BF16 = 9, DT_F32 = 10, DT_F64 = 11 };
enum OP : int { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2, OP_PROD = 3 };

// gelu'(x) = Phi(x) + x phi(x) with ONE exponential: erf(x / sqrt 2) by Abramowitz-Stegun 7.1.26
// (|error| < 1.5e-7, far below a bf16 ulp of the result) whose e^{-x^2/2} factor is phi's own.
// ~12 vector instructions instead of erff + expf (~40): the fused pass below is memory-bound.
__device__ __forceinline__ float gelu_grad_fast(float x) {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float e = __expf(-0.5f * x * x);  // = e^{-z^2}
    const float t = __frcp_rn(1.f + 0.3275911f * z);
    const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f +
                                                                                            t * 1.061405429f))));
    const float erf_abs = 1.f - poly * e;
    const float cdf = 0.5f * (1.f + (x < 0.f ? -erf_abs : erf_abs));
    return cdf + x * (e * 0.39894228040143268f);
}

// Phi(x) = 0.5 (1 + erf(x / sqrt 2)) by the same Abramowitz-Stegun form (one exponential)
__device__ __forceinline__ float gelu_cdf_fast(float x) {
    const float z = fabsf(x) * 0.70710678118654752f;
    const float e = __expf(-0.5f * x * x);
    const float t = __frcp_rn(1.f + 0.3275911f * z);
    const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f +
                                                                                            t * 1.061405429f))));
    const float erf_abs = 1.f - poly * e;
    return 0.5f * (1.f + (x < 0.f ? -erf_abs : erf_abs));
}

}  // namespace kfk
