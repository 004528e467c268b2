// Conv bias + ReLU for NHWC bf16 activations (VGG-16's conv -> bias -> ReLU), for gfx950.
//
// Why: VGG-16 at 256 images per GPU spends ~11 ms of a 54 ms step in separate torch passes
// around its 13 MFMA convolutions: bias add (new tensor), in-place clamp, threshold
// backward, and a channel reduce for the bias gradient (profiles/r17_vgg16_b256.md).
// All are HBM-bound, so the fusion is about bytes:
//
//   forward   y = max(y + b, 0) in place on the conv output            (read 2 + write 2 B)
//   backward  dz = dy * (y > 0) and db[c] = sum dz[:, c] in one pass   (read 4 + write 2 B)
//
// The ReLU gate comes from y itself (y > 0 <=> y + b > 0 before the clamp), y being kept
// alive anyway as the next layer's conv input.
//
// Layout: rows = N*H*W, C contiguous, one lane = one 16-byte vector of 8 channels,
// CVEC = C/8 divides the 256-thread block, so every grid stride is a multiple of CVEC and
// a lane's channel group is fixed: per-channel bias / gradient accumulators stay in
// registers.  The bias-gradient block partials are reduced through LDS and added with one
// f32 global atomic per channel per block (vector memory atomics).
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

__device__ __forceinline__ void unpack8v(const uint4 &v, float (&f)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

__device__ __forceinline__ uint4 pack8v(const float (&f)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w[i] = static_cast<uint32_t>(f32_to_bf16(f[2 * i])) | (static_cast<uint32_t>(f32_to_bf16(f[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

template <int CVEC, bool RELU>
__global__ __launch_bounds__(kBlock) void bias_act_fwd_kernel(uint4 *__restrict__ y, const float *__restrict__ bias,
                                                              int64_t nvec) {
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = bias[cv * 8 + k];
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = tid; i < nvec; i += stride) {
        float f[8];
        unpack8v(y[i], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            f[k] += b[k];
            if (RELU) f[k] = !(f[k] <= 0.f) ? f[k] : 0.f;  // NaN stays NaN (torch.relu)
        }
        y[i] = pack8v(f);
    }
}

template <int CVEC, bool RELU>
__global__ __launch_bounds__(kBlock) void bias_act_bwd_kernel(const uint4 *__restrict__ dy,
                                                              const uint4 *__restrict__ y, uint4 *__restrict__ dz,
                                                              float *__restrict__ dbias, int64_t nvec) {
    constexpr int C = CVEC * 8, RPI = kBlock / CVEC;
    __shared__ float lds[kBlock * 8];
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = tid; i < nvec; i += stride) {
        float g[8];
        unpack8v(dy[i], g);
        if (RELU) {
            float v[8];
            unpack8v(y[i], v);
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = v[k] > 0.f ? g[k] : 0.f;
            dz[i] = pack8v(g);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += g[k];
    }
    // threadIdx.x = r * CVEC + cv (kBlock % CVEC == 0): fold the RPI rows of each channel
    const int r0 = threadIdx.x / CVEC;
#pragma unroll
    for (int k = 0; k < 8; ++k) lds[r0 * C + cv * 8 + k] = acc[k];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += kBlock) {
        float s = 0.f;
        for (int r = 0; r < RPI; ++r) s += lds[r * C + c];
        atomicAdd(dbias + c, s);
    }
}

template <class F>
void dispatch_bias_cvec(int cvec, F &&f) {
    switch (cvec) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    case 8: f(std::integral_constant<int, 8>()); break;
    case 16: f(std::integral_constant<int, 16>()); break;
    case 32: f(std::integral_constant<int, 32>()); break;
    case 64: f(std::integral_constant<int, 64>()); break;
    case 128: f(std::integral_constant<int, 128>()); break;
    case 256: f(std::integral_constant<int, 256>()); break;
    default: throw std::invalid_argument("bias_act: C/8 must be a power of two <= 256");
    }
}

// Enough blocks to fill the chip with the grid a multiple of nothing in particular:
// the stride gridDim*256 is a multiple of every supported CVEC.
int bias_grid(int64_t nvec) {
    int64_t g = (nvec + kBlock - 1) / kBlock;
    if (g > 4096) g = 4096;
    return static_cast<int>(g < 1 ? 1 : g);
}

}  // namespace

bool bias_act_supported(int C) {
    if (C % 8) return false;
    const int cv = C / 8;
    return cv >= 1 && cv <= 256 && (cv & (cv - 1)) == 0;
}

void launch_bias_act_forward(uint16_t *y, const float *bias, int64_t rows, int C, bool relu, hipStream_t s) {
    const int64_t nvec = rows * (C / 8);
    if (nvec == 0) return;
    dispatch_bias_cvec(C / 8, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        uint4 *yv = reinterpret_cast<uint4 *>(y);
        if (relu) bias_act_fwd_kernel<CV, true><<<bias_grid(nvec), kBlock, 0, s>>>(yv, bias, nvec);
        else bias_act_fwd_kernel<CV, false><<<bias_grid(nvec), kBlock, 0, s>>>(yv, bias, nvec);
    });
}

void launch_bias_act_backward(const uint16_t *dy, const uint16_t *y, uint16_t *dz, float *dbias, int64_t rows, int C,
                              bool relu, hipStream_t s) {
    const int64_t nvec = rows * (C / 8);
    (void)hipMemsetAsync(dbias, 0, sizeof(float) * C, s);
    if (nvec == 0) return;
    dispatch_bias_cvec(C / 8, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        const uint4 *dv = reinterpret_cast<const uint4 *>(dy), *yv = reinterpret_cast<const uint4 *>(y);
        uint4 *zv = reinterpret_cast<uint4 *>(dz);
        if (relu) bias_act_bwd_kernel<CV, true><<<bias_grid(nvec), kBlock, 0, s>>>(dv, yv, zv, dbias, nvec);
        else bias_act_bwd_kernel<CV, false><<<bias_grid(nvec), kBlock, 0, s>>>(dv, yv, zv, dbias, nvec);
    });
}

}  // namespace kfk
