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
// registers.  The bias gradient is deterministic and needs no zeroed output: each block
// folds its rows through LDS and WRITES its [C] partial (plain vector stores, no atomics),
// then colsum_rows_kernel sums the <= 4096 block partials per channel in a fixed order
// (two levels: 64 rows per workgroup, then the <= 64 level sums).
//
// Round 5: the previous form zeroed the f32 gradient with
// hipMemsetAsync and added block partials with f32 atomics.  It was the only in-step
// hipMemsetAsync of the engine and the only piece of VGG-16's per-layer path that the
// fused stack does not share; under whole-step capture that path gave a different loss
// in every run and went NaN in ~1 of 4 runs, while eager was bit-stable.  The memset
// node is not needed any more and the sum no longer depends on atomic arrival order.
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
        w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
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
                                                              float *__restrict__ partial, int64_t nvec) {
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
    float *part = partial + static_cast<int64_t>(blockIdx.x) * C;
    for (int c = threadIdx.x; c < C; c += kBlock) {
        float s = 0.f;
        for (int r = 0; r < RPI; ++r) s += lds[r * C + c];
        part[c] = s;
    }
}

// Deterministic column sums of an f32 [R, C] partial matrix (C % 4 == 0), in a fixed order:
// workgroup w sums rows [w * rpw, (w + 1) * rpw) into out[w][:].  Lanes are (row group, channel
// quad): CQ = C / 4 quads, RG = 256 / CQ row groups when CQ < 256, each lane adding every RG-th row
// of its range with 16-byte loads (adjacent lanes = adjacent quads: coalesced), the RG lane partials
// then folded through LDS in row-group order.  Two launches (R -> R / 64 -> 1) replace one lane per
// channel walking all <= 4096 block partials (latency-bound: ~4 ms per VGG-16 step, r5t6).
__global__ __launch_bounds__(kBlock) void colsum_rows_kernel(const float *__restrict__ in, float *__restrict__ out,
                                                             int R, int C, int rpw) {
    __shared__ float4 lds[kBlock];
    const int CQ = C >> 2;
    const int RG = CQ >= kBlock ? 1 : kBlock / CQ;
    const int r0 = blockIdx.x * rpw;
    const int r1 = min(R, r0 + rpw);
    const int rg = threadIdx.x / min(CQ, kBlock);
    for (int cq0 = 0; cq0 < CQ; cq0 += kBlock) {
        const int cq = cq0 + threadIdx.x % min(CQ, kBlock);
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (cq < CQ) {
            const float4 *col = reinterpret_cast<const float4 *>(in) + cq;
#pragma unroll 4
            for (int r = r0 + rg; r < r1; r += RG) {
                const float4 v = col[static_cast<int64_t>(r) * CQ];
                a.x += v.x;
                a.y += v.y;
                a.z += v.z;
                a.w += v.w;
            }
        }
        if (RG == 1) {
            if (cq < CQ) reinterpret_cast<float4 *>(out)[static_cast<int64_t>(blockIdx.x) * CQ + cq] = a;
            continue;
        }
        lds[threadIdx.x] = a;
        __syncthreads();
        if (rg == 0) {
            for (int g = 1; g < RG; ++g) {
                const float4 v = lds[g * CQ + threadIdx.x];
                a.x += v.x;
                a.y += v.y;
                a.z += v.z;
                a.w += v.w;
            }
            reinterpret_cast<float4 *>(out)[static_cast<int64_t>(blockIdx.x) * CQ + cq] = a;
        }
        __syncthreads();
    }
}

constexpr int kColsumRows = 64;  // rows per workgroup of the first column-sum level

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

int bias_act_backward_blocks(int64_t rows, int C) {
    const int blocks = bias_grid(rows * (C / 8));
    return blocks + (blocks + kColsumRows - 1) / kColsumRows;  // block partials + the first sum level
}

void launch_bias_act_backward(const uint16_t *dy, const uint16_t *y, uint16_t *dz, float *dbias, float *partial,
                              int64_t rows, int C, bool relu, hipStream_t s) {
    const int64_t nvec = rows * (C / 8);
    const int blocks = bias_grid(nvec);
    if (nvec > 0) {
        dispatch_bias_cvec(C / 8, [&](auto cvc) {
            constexpr int CV = decltype(cvc)::value;
            const uint4 *dv = reinterpret_cast<const uint4 *>(dy), *yv = reinterpret_cast<const uint4 *>(y);
            uint4 *zv = reinterpret_cast<uint4 *>(dz);
            if (relu) bias_act_bwd_kernel<CV, true><<<blocks, kBlock, 0, s>>>(dv, yv, zv, partial, nvec);
            else bias_act_bwd_kernel<CV, false><<<blocks, kBlock, 0, s>>>(dv, yv, zv, partial, nvec);
        });
    }
    // nvec == 0: zero partial rows are summed (the column sum writes dbias = 0 then)
    const int R = nvec > 0 ? blocks : 0;
    if (R > kColsumRows) {
        const int R2 = (R + kColsumRows - 1) / kColsumRows;
        float *mid = partial + static_cast<int64_t>(blocks) * C;
        colsum_rows_kernel<<<R2, kBlock, 0, s>>>(partial, mid, R, C, kColsumRows);
        colsum_rows_kernel<<<1, kBlock, 0, s>>>(mid, dbias, R2, C, R2);
    } else {
        colsum_rows_kernel<<<1, kBlock, 0, s>>>(partial, dbias, R, C, kColsumRows);
    }
}

}  // namespace kfk
