// Fused NHWC BatchNorm (+ residual add) (+ ReLU), forward and backward,
// bf16 activations / f32 statistics and parameters, for gfx950.
//
// Why: on MI355X a channels_last bf16 ResNet-50 step spends ~55% of its time in
// MIOpen batch-norm kernels plus separate PyTorch ReLU / residual-add /
// threshold-backward kernels (profiles/r1_baseline_torch_resnet50_*.md), all
// HBM-bound.  Fusing them cuts the bytes moved per BN layer by ~30-40% and
// the launches by ~3x.
//
// Layout: x is [rows = N*H*W, C] with C contiguous (channels_last).  Each lane
// owns one 16-byte vector = 8 channels; CVEC = C/8 lanes cover a row and a
// 256-thread block covers RPI = 256/CVEC rows per iteration.  Because every
// grid stride is a multiple of CVEC, a thread's channel group is fixed for the
// whole kernel: per-channel coefficients live in registers, no LDS staging.
//
// Passes (bytes per element, bf16):
//   forward   stats (read x: 2)  + apply (read x [+res], write y: 4 [6])
//   backward  reduce (read dy, y, x: 6) + apply (read dy, y, x, write dx [+dres]: 8 [10])
// vs. MIOpen BN + torch relu/add/threshold_backward: ~10 [16] forward, ~16 [19] backward.
//
// Statistics are two-stage and deterministic: per-chunk partial sums (f32)
// then a per-channel fold in f64 (no float atomics).
#include "common.hpp"
#include "kernels.hpp"

namespace kfk {

namespace {

__device__ __forceinline__ void unpack8(const uint4 &v, float (&f)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}

__device__ __forceinline__ uint4 pack8(const float (&f)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        w[i] = static_cast<uint32_t>(f32_to_bf16(f[2 * i])) | (static_cast<uint32_t>(f32_to_bf16(f[2 * i + 1])) << 16);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

struct Chunking {
    int64_t rows_per_chunk;
    int nchunks;
};

constexpr int kMaxChunks = 512;
constexpr int kFoldCh = 32;                   // channels per fold block
constexpr int kFoldLanes = kBlock / kFoldCh;  // chunk lanes per channel

// Fold partial[v][chunk][C] over chunks for kFoldCh channels per block:
// 32 channel lanes x 8 chunk lanes, coalesced 128-B rows, f64 accumulation,
// then an LDS reduce across chunk lanes.  Result valid for lane kl == 0.
template <int NV>
__device__ __forceinline__ void fold_partials(const float *partial, int nchunks, int C, int c, int kl,
                                              double (&out)[NV]) {
    __shared__ double red[NV][kFoldLanes][kFoldCh];
    const int ci = threadIdx.x % kFoldCh;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        double s = 0;
        if (c < C) {
            const float *p = partial + static_cast<int64_t>(v) * nchunks * C + c;
#pragma unroll 8
            for (int k = kl; k < nchunks; k += kFoldLanes) s += p[static_cast<int64_t>(k) * C];
        }
        red[v][kl][ci] = s;
    }
    __syncthreads();
    if (kl == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            double s = 0;
#pragma unroll
            for (int j = 0; j < kFoldLanes; ++j) s += red[v][j][ci];
            out[v] = s;
        }
    }
}

inline Chunking chunking(const BNShape &sh) {
    const int cvec = sh.channels / 8;
    const int rpi = kBlock / cvec;
    int64_t row_bytes = static_cast<int64_t>(sh.channels) * 2;
    int64_t rpc = (64 * 1024 + row_bytes - 1) / row_bytes;  // >= 64 KiB per block
    rpc = ((rpc + rpi - 1) / rpi) * rpi;
    int64_t n = (sh.rows + rpc - 1) / rpc;
    // <= 2 blocks per CU: enough bytes in flight (4 x 16 B loads per lane per
    // step) while keeping the partials fold short.
    if (n > kMaxChunks) {
        rpc = (sh.rows + kMaxChunks - 1) / kMaxChunks;
        rpc = ((rpc + rpi - 1) / rpi) * rpi;
        n = (sh.rows + rpc - 1) / rpc;
    }
    if (n < 1) n = 1;
    return {rpc, static_cast<int>(n)};
}

// Block-reduce NV per-thread 8-channel accumulators into partial[chunk][C] arrays.
template <int CVEC, int NV>
__device__ __forceinline__ void reduce_to_partials(float (&acc)[NV][8], float *lds, float *partial, int C,
                                                   int nchunks_total) {
    constexpr int RPI = kBlock / CVEC;
    const int tid = threadIdx.x, cv = tid % CVEC, r0 = tid / CVEC;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        float *dst = lds + (v * RPI + r0) * C + cv * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) dst[k] = acc[v][k];
    }
    __syncthreads();
    for (int c = tid; c < C; c += kBlock) {
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < RPI; ++r) s += lds[(v * RPI + r) * C + c];
            partial[(static_cast<int64_t>(v) * nchunks_total + blockIdx.x) * C + c] = s;
        }
    }
}

// ---------------------------------------------------------------- forward stats

template <int CVEC>
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const uint4 *__restrict__ x, int64_t rows,
                                                          int64_t rows_per_chunk, float *partial) {
    constexpr int RPI = kBlock / CVEC;
    constexpr int C = CVEC * 8;
    __shared__ float lds[2 * RPI * C];  // 2 * 256 * 8 floats = 16 KiB
    const int tid = threadIdx.x, cv = tid % CVEC, r0 = tid / CVEC;
    float acc[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[0][k] = acc[1][k] = 0.f;
    const int64_t r_begin = static_cast<int64_t>(blockIdx.x) * rows_per_chunk;
    int64_t r_end = r_begin + rows_per_chunk;
    if (r_end > rows) r_end = rows;
    int64_t r = r_begin + r0;
    // 4 independent 16-B loads in flight per lane
    for (; r + 3 * RPI < r_end; r += 4 * RPI) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = x[(r + u * RPI) * CVEC + cv];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            float f[8];
            unpack8(v[u], f);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                acc[0][k] += f[k];
                acc[1][k] += f[k] * f[k];
            }
        }
    }
    for (; r < r_end; r += RPI) {
        float f[8];
        unpack8(x[r * CVEC + cv], f);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[0][k] += f[k];
            acc[1][k] += f[k] * f[k];
        }
    }
    reduce_to_partials<CVEC, 2>(acc, lds, partial, C, gridDim.x);
}

// Fold partials (parallel over chunks), emit mean/invstd, running stats and
// the affine coefficients scale = gamma*invstd, shift = beta - mean*scale.
__global__ __launch_bounds__(kBlock) void bn_stats_finalize(const float *partial, int nchunks, int C, int64_t rows,
                                                            const float *gamma, const float *beta, float *mean,
                                                            float *invstd, float *run_mean, float *run_var,
                                                            float momentum, float eps, float *coef) {
    const int c = blockIdx.x * kFoldCh + threadIdx.x % kFoldCh, kl = threadIdx.x / kFoldCh;
    double sums[2];
    fold_partials<2>(partial, nchunks, C, c, kl, sums);
    if (kl != 0 || c >= C) return;
    double s = sums[0], q = sums[1];
    double m = s / rows;
    double var = q / rows - m * m;
    if (var < 0) var = 0;
    float is = rsqrtf(static_cast<float>(var) + eps);
    mean[c] = static_cast<float>(m);
    invstd[c] = is;
    if (run_mean) {
        double unbiased = rows > 1 ? var * rows / (rows - 1) : var;
        run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * static_cast<float>(m);
        run_var[c] = (1.f - momentum) * run_var[c] + momentum * static_cast<float>(unbiased);
    }
    float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    float sc = g * is;
    coef[c] = sc;
    coef[C + c] = b - static_cast<float>(m) * sc;
}

// Eval mode: coefficients from running stats.
__global__ void bn_eval_coef(int C, const float *gamma, const float *beta, const float *run_mean,
                             const float *run_var, float eps, float *mean, float *invstd, float *coef) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    float is = rsqrtf(run_var[c] + eps);
    float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    mean[c] = run_mean[c];
    invstd[c] = is;
    coef[c] = g * is;
    coef[C + c] = b - run_mean[c] * g * is;
}

// ---------------------------------------------------------------- forward apply

template <int CVEC, bool RES, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const uint4 *__restrict__ x, const uint4 *__restrict__ res,
                                                          const float *__restrict__ coef, uint4 *__restrict__ y,
                                                          int64_t nvec) {
    constexpr int C = CVEC * 8;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sc[k] = coef[cv * 8 + k];
        sh[k] = coef[C + cv * 8 + k];
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;  // multiple of CVEC
    for (int64_t i = tid; i < nvec; i += stride) {
        float f[8];
        unpack8(x[i], f);
        float rr[8];
        if (RES) unpack8(res[i], rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float v = f[k] * sc[k] + sh[k];
            if (RES) v += rr[k];
            if (RELU) v = v > 0.f ? v : 0.f;
            f[k] = v;
        }
        y[i] = pack8(f);
    }
}

// ---------------------------------------------------------------- backward

template <int CVEC, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(const uint4 *__restrict__ dy,
                                                               const uint4 *__restrict__ y,
                                                               const uint4 *__restrict__ x,
                                                               const float *__restrict__ mean,
                                                               const float *__restrict__ invstd, int64_t rows,
                                                               int64_t rows_per_chunk, float *partial) {
    constexpr int RPI = kBlock / CVEC;
    constexpr int C = CVEC * 8;
    __shared__ float lds[2 * RPI * C];
    const int tid = threadIdx.x, cv = tid % CVEC, r0 = tid / CVEC;
    float mu[8], is[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        mu[k] = mean[cv * 8 + k];
        is[k] = invstd[cv * 8 + k];
    }
    float acc[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[0][k] = acc[1][k] = 0.f;
    const int64_t r_begin = static_cast<int64_t>(blockIdx.x) * rows_per_chunk;
    int64_t r_end = r_begin + rows_per_chunk;
    if (r_end > rows) r_end = rows;
    // Accumulate sum(dz) and sum(dz * x); dgamma = invstd*(sum(dz*x) - mean*sum(dz))
    // is formed in the finalize (one FMA per element here instead of three).
    int64_t r = r_begin + r0;
    for (; r + RPI < r_end; r += 2 * RPI) {
        uint4 vg[2], vx[2], vy[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int64_t i = (r + u * RPI) * CVEC + cv;
            vg[u] = dy[i];
            vx[u] = x[i];
            if (RELU) vy[u] = y[i];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            float g[8], xv[8];
            unpack8(vg[u], g);
            unpack8(vx[u], xv);
            if (RELU) {
                float yv[8];
                unpack8(vy[u], yv);
#pragma unroll
                for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                acc[0][k] += g[k];
                acc[1][k] += g[k] * xv[k];
            }
        }
    }
    for (; r < r_end; r += RPI) {
        const int64_t i = r * CVEC + cv;
        float g[8], xv[8];
        unpack8(dy[i], g);
        unpack8(x[i], xv);
        if (RELU) {
            float yv[8];
            unpack8(y[i], yv);
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[0][k] += g[k];
            acc[1][k] += g[k] * xv[k];
        }
    }
    (void)mu;
    (void)is;
    reduce_to_partials<CVEC, 2>(acc, lds, partial, C, gridDim.x);
}

// dbeta = sum dz, dgamma = sum dz*xhat; dx = k1*dz + k2*x + k3.
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize(const float *partial, int nchunks, int C, int64_t rows,
                                                          const float *gamma, const float *mean, const float *invstd,
                                                          float *dgamma, float *dbeta, float *coef, bool training) {
    const int c = blockIdx.x * kFoldCh + threadIdx.x % kFoldCh, kl = threadIdx.x / kFoldCh;
    double sums[2];
    fold_partials<2>(partial, nchunks, C, c, kl, sums);
    if (kl != 0 || c >= C) return;
    // sums[1] = sum(dz * x)  ->  dgamma = invstd * (sum(dz*x) - mean * sum(dz))
    double db = sums[0], dg = static_cast<double>(invstd[c]) * (sums[1] - static_cast<double>(mean[c]) * db);
    dgamma[c] = static_cast<float>(dg);
    dbeta[c] = static_cast<float>(db);
    float g = gamma ? gamma[c] : 1.f;
    float a = g * invstd[c];
    if (training) {
        float inv_m = 1.f / static_cast<float>(rows);
        float k2 = -a * static_cast<float>(dg) * invstd[c] * inv_m;
        coef[c] = a;
        coef[C + c] = k2;
        coef[2 * C + c] = -a * static_cast<float>(db) * inv_m - k2 * mean[c];
    } else {
        coef[c] = a;
        coef[C + c] = 0.f;
        coef[2 * C + c] = 0.f;
    }
}

template <int CVEC, bool RELU, bool DRES>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(const uint4 *__restrict__ dy,
                                                              const uint4 *__restrict__ y,
                                                              const uint4 *__restrict__ x,
                                                              const float *__restrict__ coef, uint4 *__restrict__ dx,
                                                              uint4 *__restrict__ dres, int64_t nvec) {
    constexpr int C = CVEC * 8;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float k1[8], k2[8], k3[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        k1[k] = coef[cv * 8 + k];
        k2[k] = coef[C + cv * 8 + k];
        k3[k] = coef[2 * C + cv * 8 + k];
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
    for (int64_t i = tid; i < nvec; i += stride) {
        float g[8], xv[8];
        unpack8(dy[i], g);
        unpack8(x[i], xv);
        if (RELU) {
            float yv[8];
            unpack8(y[i], yv);
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
        }
        if (DRES) dres[i] = pack8(g);
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = k1[k] * g[k] + k2[k] * xv[k] + k3[k];
        dx[i] = pack8(o);
    }
}

template <typename F>
void dispatch_cvec(int cvec, F &&f) {
    switch (cvec) {
    case 8: f(std::integral_constant<int, 8>()); break;
    case 16: f(std::integral_constant<int, 16>()); break;
    case 32: f(std::integral_constant<int, 32>()); break;
    case 64: f(std::integral_constant<int, 64>()); break;
    case 128: f(std::integral_constant<int, 128>()); break;
    case 256: f(std::integral_constant<int, 256>()); break;
    default: break;
    }
}

int apply_grid(int64_t nvec, int cvec) {
    int64_t g = (nvec + kBlock - 1) / kBlock;
    if (g > kMaxGrid) g = kMaxGrid;
    if (g < 1) g = 1;
    (void)cvec;  // kBlock is a multiple of every supported CVEC, so any grid keeps cv fixed
    return static_cast<int>(g);
}

}  // namespace

bool bn_supported_channels(int C) {
    if (C % 8) return false;
    int cv = C / 8;
    return cv >= 8 && cv <= 256 && (cv & (cv - 1)) == 0;
}

int bn_num_chunks(BNShape sh) { return chunking(sh).nchunks; }

void launch_bn_forward(const uint16_t *x, const uint16_t *res, const float *gamma, const float *beta, uint16_t *y,
                       BNShape sh, bool relu, bool training, float *run_mean, float *run_var, float momentum,
                       float eps, float *partial, float *mean, float *invstd, float *coef, hipStream_t s) {
    const int C = sh.channels, cvec = C / 8;
    const int64_t nvec = sh.rows * cvec;
    if (training) {
        Chunking ch = chunking(sh);
        dispatch_cvec(cvec, [&](auto cvc) {
            constexpr int CV = decltype(cvc)::value;
            bn_stats_kernel<CV><<<ch.nchunks, kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x), sh.rows,
                                                              ch.rows_per_chunk, partial);
        });
        bn_stats_finalize<<<(C + kFoldCh - 1) / kFoldCh, kBlock, 0, s>>>(partial, ch.nchunks, C, sh.rows, gamma, beta,
                                                                         mean, invstd,
                                                          run_mean, run_var, momentum, eps, coef);
    } else {
        bn_eval_coef<<<(C + 255) / 256, 256, 0, s>>>(C, gamma, beta, run_mean, run_var, eps, mean, invstd, coef);
    }
    int g = apply_grid(nvec, cvec);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        const uint4 *xv = reinterpret_cast<const uint4 *>(x);
        const uint4 *rv = reinterpret_cast<const uint4 *>(res);
        uint4 *yv = reinterpret_cast<uint4 *>(y);
        if (res) {
            if (relu) bn_apply_kernel<CV, true, true><<<g, kBlock, 0, s>>>(xv, rv, coef, yv, nvec);
            else bn_apply_kernel<CV, true, false><<<g, kBlock, 0, s>>>(xv, rv, coef, yv, nvec);
        } else {
            if (relu) bn_apply_kernel<CV, false, true><<<g, kBlock, 0, s>>>(xv, rv, coef, yv, nvec);
            else bn_apply_kernel<CV, false, false><<<g, kBlock, 0, s>>>(xv, rv, coef, yv, nvec);
        }
    });
}

void launch_bn_backward(const uint16_t *dy, const uint16_t *y, const uint16_t *x, const float *mean,
                        const float *invstd, const float *gamma, BNShape sh, bool relu, bool training,
                        float *partial, float *dgamma, float *dbeta, float *coef, uint16_t *dx, uint16_t *dres,
                        hipStream_t s) {
    const int C = sh.channels, cvec = C / 8;
    const int64_t nvec = sh.rows * cvec;
    Chunking ch = chunking(sh);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        const uint4 *d = reinterpret_cast<const uint4 *>(dy), *yy = reinterpret_cast<const uint4 *>(y),
                    *xx = reinterpret_cast<const uint4 *>(x);
        if (relu)
            bn_bwd_reduce_kernel<CV, true><<<ch.nchunks, kBlock, 0, s>>>(d, yy, xx, mean, invstd, sh.rows,
                                                                         ch.rows_per_chunk, partial);
        else
            bn_bwd_reduce_kernel<CV, false><<<ch.nchunks, kBlock, 0, s>>>(d, yy, xx, mean, invstd, sh.rows,
                                                                          ch.rows_per_chunk, partial);
    });
    bn_bwd_finalize<<<(C + kFoldCh - 1) / kFoldCh, kBlock, 0, s>>>(partial, ch.nchunks, C, sh.rows, gamma, mean,
                                                                   invstd, dgamma, dbeta, coef, training);
    int g = apply_grid(nvec, cvec);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        const uint4 *d = reinterpret_cast<const uint4 *>(dy), *yy = reinterpret_cast<const uint4 *>(y),
                    *xx = reinterpret_cast<const uint4 *>(x);
        uint4 *o = reinterpret_cast<uint4 *>(dx), *r = reinterpret_cast<uint4 *>(dres);
        if (relu) {
            if (dres) bn_bwd_apply_kernel<CV, true, true><<<g, kBlock, 0, s>>>(d, yy, xx, coef, o, r, nvec);
            else bn_bwd_apply_kernel<CV, true, false><<<g, kBlock, 0, s>>>(d, yy, xx, coef, o, r, nvec);
        } else {
            if (dres) bn_bwd_apply_kernel<CV, false, true><<<g, kBlock, 0, s>>>(d, yy, xx, coef, o, r, nvec);
            else bn_bwd_apply_kernel<CV, false, false><<<g, kBlock, 0, s>>>(d, yy, xx, coef, o, r, nvec);
        }
    });
}

}  // namespace kfk
