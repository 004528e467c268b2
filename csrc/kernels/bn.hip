// Fused NHWC BatchNorm (+ residual add) (+ ReLU) (+ 3x3/s2 max-pool), forward and
// backward, bf16 activations / f32 statistics and parameters, for gfx950.
//
// Why: on MI355X a channels_last bf16 ResNet-50 step spends ~55% of its time in
// MIOpen batch-norm kernels plus separate PyTorch ReLU / residual-add /
// threshold-backward / max-pool kernels (profiles/r1_baseline_torch_resnet50_*.md),
// all HBM-bound.  Every byte not moved is time saved, so:
//
//   * the ReLU mask is never re-read from y in backward: for BN+ReLU it is
//     recomputed from x with the forward coefficients (x is read anyway), for
//     BN+add+ReLU a 1-bit-per-element mask is written in forward (1/16 of y);
//   * the ResNet stem BN+ReLU+MaxPool(3,2,1) is one forward kernel (the 112x112
//     post-BN map is never written) and one backward gather (no scatter, no
//     112x112 pool-gradient tensor);
//   * statistics folds are wide (8 channels x 32 chunk lanes per block) so the
//     tiny finalize kernels are not latency bound, and num_batches_tracked is
//     bumped inside the finalize instead of by a separate launch.
//
// Layout: x is [rows = N*H*W, C] with C contiguous (channels_last).  Each lane
// owns one 16-byte vector = 8 channels; CVEC = C/8 lanes cover a row and a
// 256-thread block covers RPI = 256/CVEC rows per iteration.  Because every
// grid stride is a multiple of CVEC, a thread's channel group is fixed for the
// whole kernel: per-channel coefficients live in registers, no LDS staging.
//
// Bytes per element (bf16 = 2):
//   forward   stats (x: 2) + apply (x [+res] -> y [+mask]: 4 [6.125])
//   backward  reduce (dy, x [+mask]: 4 [4.125]) + apply (dy, x -> dx [+dres]: 6 [8.125])
//
// Statistics are two-stage and deterministic: per-chunk partial sums (f32)
// then a per-channel fold in f64 (no float atomics).
#include "bn_fin.hpp"
#include "common.hpp"
#include "kernels.hpp"

#include <cstdlib>
#include <stdexcept>

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
        w[i] = pack_bf16x2(f[2 * i], f[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
}

// Non-temporal 16-byte accesses (bn_nt_mode(): bit 0 loads, bit 1 stores), for the apply passes
// that stream every byte exactly once.  A uniform runtime flag: both paths are in one kernel.
typedef unsigned int kf_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint4 *p, bool nt) {
    if (nt) {
        const kf_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const kf_u32x4 *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    }
    return *p;
}

__device__ __forceinline__ void st16(uint4 *p, const uint4 &v, bool nt) {
    if (nt) {
        kf_u32x4 w;
        w.x = v.x;
        w.y = v.y;
        w.z = v.z;
        w.w = v.w;
        __builtin_nontemporal_store(w, reinterpret_cast<kf_u32x4 *>(p));
    } else {
        *p = v;
    }
}

// default 1 (non-temporal loads): ResNet-50 step 21.73 -> 21.39 ms on MI355X, while
// non-temporal stores did not pay in the full step (profiles/README.md, r3f)
// (the round-3 timing experiment that skipped the sums-finalize launches -- an upper bound of
// 1.0 ms/step on what folding them elsewhere could save -- is retired with its knob, round 5)
bool bn_skip_finalize() { return false; }

// non-temporal loads, plain stores (bit 0 loads, bit 1 stores; the round-3 A/B above)
int bn_nt_mode() { return 1; }

int bn_max_grid(int def) { return def; }

struct Chunking {
    int64_t rows_per_chunk;
    int nchunks;
};

// Threads per block for a row of CVEC 16-byte vectors: the largest multiple of CVEC that
// fits 256 (all 256 when CVEC divides it).  Every grid stride is then a multiple of CVEC, so
// a lane's channel group stays fixed -- for any C % 8 == 0 (Inception's 80, 96, 160, 192,
// 320, 384, 448 channels included), not only powers of two.
template <int CVEC>
constexpr int bn_threads() {
    return (kBlock / CVEC) * CVEC;
}

constexpr int kMaxChunks = 512;
constexpr int kFoldCh = 8;                    // channels per fold block
constexpr int kFoldLanes = kBlock / kFoldCh;  // chunk lanes per channel (32)

// Fold partial[v][chunk][C] over chunks for kFoldCh channels per block:
// 8 channel lanes x 32 chunk lanes (<= 16 independent loads per lane for 512
// chunks), f64 accumulation, then an LDS reduce across chunk lanes.  Result
// valid for lane kl == 0.
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
#pragma unroll 16
            for (int k = kl; k < nchunks; k += kFoldLanes) s += p[static_cast<int64_t>(k) * C];
        }
        red[v][kl][ci] = s;
    }
    __syncthreads();
    // tree over the 32 chunk lanes
#pragma unroll
    for (int w = kFoldLanes / 2; w > 0; w >>= 1) {
        if (kl < w) {
#pragma unroll
            for (int v = 0; v < NV; ++v) red[v][kl][ci] += red[v][kl + w][ci];
        }
        __syncthreads();
    }
    if (kl == 0) {
#pragma unroll
        for (int v = 0; v < NV; ++v) out[v] = red[v][0][ci];
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
    for (int c = tid; c < C; c += bn_threads<CVEC>()) {
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
                                                            float momentum, float eps, float *coef,
                                                            int64_t *num_batches) {
    const int c = blockIdx.x * kFoldCh + threadIdx.x % kFoldCh, kl = threadIdx.x / kFoldCh;
    double sums[2];
    fold_partials<2>(partial, nchunks, C, c, kl, sums);
    if (num_batches && blockIdx.x == 0 && threadIdx.x == 0) num_batches[0] += 1;
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

// Same outputs from f64 per-channel sums produced by a convolution epilogue
// (conv.hip, EPI bit 0): kStatSlots slots of [sum x (C), sum x^2 (C)]; the sums are
// re-zeroed for the next producer (self-cleaning workspace, no memset launch).
__global__ __launch_bounds__(256) void bn_sums_finalize(double *__restrict__ sums, int C, int64_t rows,
                                                        const float *__restrict__ gamma,
                                                        const float *__restrict__ beta, float *mean, float *invstd,
                                                        float *run_mean, float *run_var, float momentum, float eps,
                                                        float *coef, int64_t *num_batches) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (num_batches && c == 0) num_batches[0] += 1;
    if (c >= C) return;
    // every input issued before any store: the slot sums and the channel's parameters / running
    // stats (loaded behind the zeroing and output stores, each was a serial round trip: 5.7 us)
    const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    const float rm = run_mean ? run_mean[c] : 0.f, rv = run_mean ? run_var[c] : 0.f;
    const double *sp = sums + c;
    double vs[kStatSlots], vq[kStatSlots];
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        vs[k] = sp[k * 2 * C];
        vq[k] = sp[k * 2 * C + C];
    }
    double s = 0, q = 0;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        s += vs[k];
        q += vq[k];
    }
    double *zp = sums + c;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        zp[k * 2 * C] = 0.0;
        zp[k * 2 * C + C] = 0.0;
    }
    bn_fin_fwd_channel(c, C, s, q, rows, g, b, rm, rv, mean, invstd, run_mean, run_var, momentum, eps, coef);
}

// Several BNs' sums-finalizes in ONE launch (blockIdx.y = which BN): the deferred branch BNs of an
// Inception block's concatenation are all finalized before any of their applies (ops/fused_bn.py
// _BNConcatFn), 2-6 launches of ~5 us each that were back-to-back anyway.
__global__ __launch_bounds__(256) void bn_sums_finalize_multi(BnFinBatch b) {
    const BnFinDesc &d = b.d[blockIdx.y];
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (d.nbt && c == 0) d.nbt[0] += 1;
    if (c >= d.C) return;
    const int C = d.C;
    const float g = d.gamma ? d.gamma[c] : 1.f, bb = d.beta ? d.beta[c] : 0.f;
    const float rm = d.run_mean ? d.run_mean[c] : 0.f, rv = d.run_mean ? d.run_var[c] : 0.f;
    const double *sp = d.sums + c;
    double vs[kStatSlots], vq[kStatSlots];
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        vs[k] = sp[k * 2 * C];
        vq[k] = sp[k * 2 * C + C];
    }
    double s = 0, q = 0;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        s += vs[k];
        q += vq[k];
    }
    double *zp = d.sums + c;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        zp[k * 2 * C] = 0.0;
        zp[k * 2 * C + C] = 0.0;
    }
    bn_fin_fwd_channel(c, C, s, q, d.rows, g, bb, rm, rv, d.mean, d.invstd, d.run_mean, d.run_var, d.momentum, d.eps,
                       d.coef);
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

// y = act(x*scale + shift [+ res]); with RES && RELU also a 1-bit mask per
// element (one byte per 8-channel vector) for the backward.  RESC: the residual is itself a
// BN input -- res*rscale + rshift with the coefficients rcoef (the downsample branch's BN, so
// its output is never materialised).
// SOUT: y is a channel slice of a wider NHWC tensor (row stride y_ldv 16-byte vectors): the
// branch outputs of an Inception block written straight into their concatenation.
template <int CVEC, bool RES, bool RELU, bool RESC = false, bool SOUT = false>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const uint4 *__restrict__ x, const uint4 *__restrict__ res,
                                                          const float *__restrict__ coef, uint4 *__restrict__ y,
                                                          uint8_t *__restrict__ mask, int64_t nvec,
                                                          const float *__restrict__ rcoef = nullptr, int ntm = 0,
                                                          int64_t y_ldv = 0) {
    constexpr int C = CVEC * 8;
    const bool ntl = ntm & 1, nts = ntm & 2;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * bn_threads<CVEC>() + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sc[k] = coef[cv * 8 + k];
        sh[k] = coef[C + cv * 8 + k];
        if (RESC) {
            rsc[k] = rcoef[cv * 8 + k];
            sh[k] += rcoef[C + cv * 8 + k];
        }
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * bn_threads<CVEC>();  // multiple of CVEC
    // two vectors per trip, both loads issued before either is used (bytes in flight per lane)
    constexpr int U = 2;
    for (int64_t i0 = tid; i0 < nvec; i0 += U * stride) {
        uint4 xr[U], rr4[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < nvec) {
                xr[u] = ld16(x + i, ntl);
                if (RES) rr4[u] = ld16(res + i, ntl);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= nvec) break;
            float f[8];
            unpack8(xr[u], f);
            float rr[8];
            if (RES) unpack8(rr4[u], rr);
            uint32_t m = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float v = f[k] * sc[k] + sh[k];
                if (RESC) v += rr[k] * rsc[k];
                else if (RES) v += rr[k];
                if (RELU) {
                    m |= (v > 0.f ? 1u : 0u) << k;
                    v = v > 0.f ? v : 0.f;
                }
                f[k] = v;
            }
            if constexpr (SOUT) st16(y + (i / CVEC) * y_ldv + cv, pack8(f), nts);
            else st16(y + i, pack8(f), nts);
            if (RES && RELU) mask[i] = static_cast<uint8_t>(m);
        }
    }
}

// ---------------------------------------------------------------- stem: BN + ReLU + MaxPool(3, 2, 1)

// One lane per (pooled pixel, 8-channel vector): 9 window loads (served mostly
// from L2 -- neighbouring outputs share 3-6 of them), BN+ReLU per element, max.
// Emits the pooled bf16 map and the window argmax (0..8) per element as bytes.
template <int CVEC>
// xarg (optional): the pre-BN input value of each window's chosen element, so the backward's
// BN sums can run over the pooled map (bn_pool_bwd_sums_kernel) instead of a full-resolution gather.
__global__ __launch_bounds__(kBlock) void bn_pool_apply_kernel(const uint4 *__restrict__ x,
                                                               const float *__restrict__ coef, uint4 *__restrict__ yp,
                                                               uint2 *__restrict__ arg, int H, int W, int OH, int OW,
                                                               int64_t nout_vec, uint4 *__restrict__ xarg) {
    constexpr int C = CVEC * 8;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * bn_threads<CVEC>() + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sc[k] = coef[cv * 8 + k];
        sh[k] = coef[C + cv * 8 + k];
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * bn_threads<CVEC>();
    for (int64_t i = tid; i < nout_vec; i += stride) {
        const int64_t p = i / CVEC;
        const int ow = static_cast<int>(p % OW);
        const int64_t t = p / OW;
        const int oh = static_cast<int>(t % OH);
        const int64_t n = t / OH;
        float best[8], xb[8];
        uint32_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            best[k] = -1.f;  // post-ReLU values are >= 0
            a[k] = 0;
            xb[k] = 0.f;
        }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int h = 2 * oh - 1 + kh;
            if (h < 0 || h >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int w = 2 * ow - 1 + kw;
                if (w < 0 || w >= W) continue;
                float f[8];
                unpack8(x[((n * H + h) * W + w) * CVEC + cv], f);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    float v = f[k] * sc[k] + sh[k];
                    v = v > 0.f ? v : 0.f;
                    if (v > best[k]) {
                        best[k] = v;
                        a[k] = kh * 3 + kw;
                        xb[k] = f[k];
                    }
                }
            }
        }
        yp[i] = pack8(best);
        arg[i] = make_uint2(a[0] | (a[1] << 8) | (a[2] << 16) | (a[3] << 24),
                            a[4] | (a[5] << 8) | (a[6] << 16) | (a[7] << 24));
        if (xarg) xarg[i] = pack8(xb);  // exact: bf16 inputs re-packed
    }
}

// BN backward sums of the stem's BN+ReLU+MaxPool in POOLED space: every window hands its
// gradient to exactly one input element (its argmax), so
//   sum_p dz[p] = sum_w dy[w] * relu'(x_w),   sum_p dz[p] x[p] = sum_w dy[w] * relu'(x_w) * x_w
// with x_w = xarg[w] -- two reads of the pooled map instead of the full-resolution gather
// (exact up to f32 summation order).  Sums go to f64 slots [kStatSlots][2][C].
template <int CVEC>
__global__ __launch_bounds__(kBlock) void bn_pool_bwd_sums_kernel(const uint4 *__restrict__ dy,
                                                                  const uint4 *__restrict__ xarg,
                                                                  const float *__restrict__ fcoef,
                                                                  double *__restrict__ sums, int64_t nvec) {
    constexpr int C = CVEC * 8, NT = bn_threads<CVEC>();
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float sc[8], sh[8], s1[8], s2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sc[k] = fcoef[cv * 8 + k];
        sh[k] = fcoef[C + cv * 8 + k];
        s1[k] = s2[k] = 0.f;
    }
    const int64_t stride = static_cast<int64_t>(gridDim.x) * NT;
    for (int64_t i = tid; i < nvec; i += stride) {
        float g[8], xv[8];
        unpack8(dy[i], g);
        unpack8(xarg[i], xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const float dz = xv[k] * sc[k] + sh[k] > 0.f ? g[k] : 0.f;
            s1[k] += dz;
            s2[k] += dz * xv[k];
        }
    }
    __shared__ float red[kBlock][17];
    if (threadIdx.x < NT) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            red[threadIdx.x][k] = s1[k];
            red[threadIdx.x][8 + k] = s2[k];
        }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
        const int cvi = c >> 3, k = c & 7;
        double a1 = 0, a2 = 0;
        for (int u = cvi; u < NT; u += CVEC) {
            a1 += red[u][k];
            a2 += red[u][8 + k];
        }
        double *sl = sums + (blockIdx.x % kStatSlots) * 2 * C;
        atomicAdd(sl + c, a1);
        atomicAdd(sl + C + c, a2);
    }
}

// ---------------------------------------------------------------- backward gradient sources

// dy read directly ([rows, C]).
// Two-phase interface so the reduce loop can put several rows of loads in
// flight before any arithmetic: fetch() issues the loads, get() unpacks.
struct DirectGrad {
    const uint4 *dy;
    bool nt = false;
    using Raw = uint4;
    template <int CVEC>
    __device__ __forceinline__ Raw fetch(int64_t i, int64_t /*row*/, int /*cv*/) const {
        return ld16(dy + i, nt);
    }
    __device__ __forceinline__ void get(const Raw &r, float (&g)[8]) const { unpack8(r, g); }
};

// dy is a channel slice of a wider channels-last tensor (row stride ldv 16-byte vectors): the
// gradient of a branch of a channel concatenation (Inception) read in place, no copy.
struct StridedGrad {
    const uint4 *dy;
    int64_t ldv;
    using Raw = uint4;
    template <int CVEC>
    __device__ __forceinline__ Raw fetch(int64_t /*i*/, int64_t row, int cv) const {
        return dy[row * ldv + cv];
    }
    __device__ __forceinline__ void get(const Raw &r, float (&g)[8]) const { unpack8(r, g); }
};

// dy of the BN output gathered from the max-pool gradient: input pixel (h, w)
// receives dy_pool of every window (<= 2x2 of them) whose argmax it is.
struct PoolGrad {
    const uint4 *dyp;  // [N, OH, OW, C]
    const uint2 *arg;  // [N, OH, OW, C] bytes
    int H, W, OH, OW;
    uint64_t m_hw, m_w;  // floor(p / d) = (p * m) >> 40 (exact for p * d < 2^40): no integer division
    // Raw = the up to 4 covering windows' argmax bytes and gradients, loaded branch-free
    // (invalid candidates re-read window 0 and carry kk = 0xff, which no argmax byte equals),
    // so fetch() only issues loads and several rows' gathers stay in flight together; get()
    // does the compare-and-add once the data is needed.
    struct Raw {
        uint2 am[4];
        uint4 d[4];
        uint32_t kk;  // 4 packed candidate window offsets (0..8, or 0xff)
    };
    __device__ __forceinline__ void get(const Raw &r, float (&g)[8]) const {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const uint32_t kk = (r.kk >> (8 * c)) & 0xffu;
            float d[8];
            unpack8(r.d[c], d);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t ak = ((k < 4 ? r.am[c].x : r.am[c].y) >> (8 * (k & 3))) & 0xffu;
                g[k] += ak == kk ? d[k] : 0.f;
            }
        }
    }
    // rows < 2^31 (checked on the host): 32-bit index math only.
    template <int CVEC>
    __device__ __forceinline__ Raw fetch(int64_t /*i*/, int64_t row64, int cv) const {
        const uint32_t row = static_cast<uint32_t>(row64);
        const uint32_t hw = static_cast<uint32_t>(H) * static_cast<uint32_t>(W);
        const uint32_t n = static_cast<uint32_t>((static_cast<uint64_t>(row) * m_hw) >> 40);
        const uint32_t rem = row - n * hw;
        const int h = static_cast<int>((static_cast<uint64_t>(rem) * m_w) >> 40);
        const int w = static_cast<int>(rem) - h * W;
        // windows oh with 2 oh - 1 <= h <= 2 oh + 1: h >> 1 always, (h + 1) >> 1 when h is odd
        const int oh_lo = h >> 1, oh_hi = (h + 1) >> 1;
        const int ow_lo = w >> 1, ow_hi = (w + 1) >> 1;
        Raw r;
        r.kk = 0;
        const uint32_t base = (n * OH) * OW;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int oh = (c & 2) ? oh_hi : oh_lo, ow = (c & 1) ? ow_hi : ow_lo;
            const bool ok = (!(c & 2) || oh_hi != oh_lo) && (!(c & 1) || ow_hi != ow_lo) && oh < OH && ow < OW;
            const uint32_t kk = ok ? static_cast<uint32_t>((h + 1 - 2 * oh) * 3 + (w + 1 - 2 * ow)) : 0xffu;
            const uint32_t o = ((base + (ok ? oh : oh_lo) * OW + (ok ? ow : ow_lo)) * CVEC) + cv;
            r.am[c] = arg[o];
            r.d[c] = dyp[o];
            r.kk |= kk << (8 * c);
        }
        return r;
    }
    template <int CVEC>
    __device__ __forceinline__ void load(int64_t i, int64_t row, int cv, float (&g)[8]) const {
        get(fetch<CVEC>(i, row, cv), g);
    }
};

enum ReluMode : int { RM_NONE = 0, RM_COEF = 1, RM_BITS = 2 };

// Zero g where the forward ReLU was inactive.
template <int RM>
__device__ __forceinline__ void relu_gate(float (&g)[8], const float (&xv)[8], const float (&sc)[8],
                                          const float (&sh)[8], const uint8_t *mask, int64_t i) {
    if (RM == RM_COEF) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = (xv[k] * sc[k] + sh[k]) > 0.f ? g[k] : 0.f;
    } else if (RM == RM_BITS) {
        const uint32_t m = mask[i];
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = ((m >> k) & 1u) ? g[k] : 0.f;
    }
}

template <int CVEC, int RM>
__device__ __forceinline__ void load_fwd_coef(const float *fcoef, int cv, float (&sc)[8], float (&sh)[8]) {
    constexpr int C = CVEC * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        sc[k] = RM == RM_COEF ? fcoef[cv * 8 + k] : 0.f;
        sh[k] = RM == RM_COEF ? fcoef[C + cv * 8 + k] : 0.f;
    }
}

// ---------------------------------------------------------------- backward reduce

// Accumulate sum(dz) and sum(dz * x); dgamma = invstd*(sum(dz*x) - mean*sum(dz))
// is formed in the finalize (one FMA per element here instead of three).
template <int CVEC, int RM, class G>
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(G grad, const uint4 *__restrict__ x,
                                                               const float *__restrict__ fcoef,
                                                               const uint8_t *__restrict__ mask, int64_t rows,
                                                               int64_t rows_per_chunk, float *partial, int ntm = 0) {
    const bool ntl = ntm & 1;
    constexpr int RPI = kBlock / CVEC;
    constexpr int C = CVEC * 8;
    __shared__ float lds[2 * RPI * C];
    const int tid = threadIdx.x, cv = tid % CVEC, r0 = tid / CVEC;
    float sc[8], sh[8];
    load_fwd_coef<CVEC, RM>(fcoef, cv, sc, sh);
    float acc[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[0][k] = acc[1][k] = 0.f;
    const int64_t r_begin = static_cast<int64_t>(blockIdx.x) * rows_per_chunk;
    int64_t r_end = r_begin + rows_per_chunk;
    if (r_end > rows) r_end = rows;
    int64_t r = r_begin + r0;
    // U rows per lane in flight (2 x 16-B loads each) before any arithmetic
    constexpr int U = 4;
    for (; r + (U - 1) * RPI < r_end; r += U * RPI) {
        typename G::Raw gr[U];
        uint4 xr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t row = r + u * RPI, i = row * CVEC + cv;
            gr[u] = grad.template fetch<CVEC>(i, row, cv);
            xr[u] = ld16(x + i, ntl);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float g[8], xv[8];
            grad.get(gr[u], g);
            unpack8(xr[u], xv);
            relu_gate<RM>(g, xv, sc, sh, mask, (r + u * RPI) * CVEC + cv);
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
        grad.get(grad.template fetch<CVEC>(i, r, cv), g);
        unpack8(x[i], xv);
        relu_gate<RM>(g, xv, sc, sh, mask, i);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            acc[0][k] += g[k];
            acc[1][k] += g[k] * xv[k];
        }
    }
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

// Several BNs' backward finalizes in ONE launch (blockIdx.y = which BN): the branch BNs of an
// Inception block's concatenation (ops/fused_bn.py _BNConcatFn.backward).
__global__ __launch_bounds__(kBlock) void bn_bwd_finalize_multi(BnBwdFinBatch b) {
    const BnBwdFinDesc &d = b.d[blockIdx.y];
    const int C = d.C;
    if (static_cast<int>(blockIdx.x) * kFoldCh >= C) return;  // a narrower BN of the batch: uniform exit
    const int c = blockIdx.x * kFoldCh + threadIdx.x % kFoldCh, kl = threadIdx.x / kFoldCh;
    double sums[2];
    fold_partials<2>(d.partial, d.nchunks, C, c, kl, sums);
    if (kl != 0 || c >= C) return;
    double db = sums[0], dg = static_cast<double>(d.invstd[c]) * (sums[1] - static_cast<double>(d.mean[c]) * db);
    d.dgamma[c] = static_cast<float>(dg);
    d.dbeta[c] = static_cast<float>(db);
    float g = d.gamma ? d.gamma[c] : 1.f;
    float a = g * d.invstd[c];
    const float inv_m = 1.f / static_cast<float>(d.rows);
    const float k2 = -a * static_cast<float>(dg) * d.invstd[c] * inv_m;
    d.coef[c] = a;
    d.coef[C + c] = k2;
    d.coef[2 * C + c] = -a * static_cast<float>(db) * inv_m - k2 * d.mean[c];
}

// Same coefficients from the f64 slotted sums of a data-gradient conv epilogue
// (conv.hip kEpiBwd*): sum dz, sum dz*x; the slots are re-zeroed.
__global__ __launch_bounds__(256) void bn_bwd_finalize_sums(double *__restrict__ sums, int C, int64_t rows,
                                                            const float *__restrict__ gamma,
                                                            const float *__restrict__ mean,
                                                            const float *__restrict__ invstd, float *dgamma,
                                                            float *dbeta, float *coef, bool training) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float g = gamma ? gamma[c] : 1.f, mu = mean[c], is = invstd[c];  // issued with the slot loads
    const double *sp = sums + c;
    double v0[kStatSlots], v1[kStatSlots];
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        v0[k] = sp[k * 2 * C];
        v1[k] = sp[k * 2 * C + C];
    }
    double s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        s0 += v0[k];
        s1 += v1[k];
    }
    double *zp = sums + c;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        zp[k * 2 * C] = 0.0;
        zp[k * 2 * C + C] = 0.0;
    }
    bn_fin_bwd_channel(c, C, s0, s1, rows, g, mu, is, dgamma, dbeta, coef, training);
}

// ---------------------------------------------------------------- backward apply

// DRES && dsx: the residual gradient also feeds a second BN (the downsample branch's, input dsx,
// no ReLU): its backward sums sum(dres) and sum(dres * dsx) (of the bf16-rounded dres, as that
// BN's own pass would read it) go to the f64 slots dsums, so that BN skips its reduce pass.
template <int CVEC, int RM, bool DRES, class G>
__global__ __launch_bounds__(kBlock) void bn_bwd_apply_kernel(G grad, const uint4 *__restrict__ x,
                                                              const float *__restrict__ fcoef,
                                                              const uint8_t *__restrict__ mask,
                                                              const float *__restrict__ coef, uint4 *__restrict__ dx,
                                                              uint4 *__restrict__ dres, int64_t nvec,
                                                              const uint4 *__restrict__ dsx = nullptr,
                                                              double *__restrict__ dsums = nullptr, int ntm = 0) {
    constexpr int C = CVEC * 8;
    const bool ntl = ntm & 1, nts = ntm & 2;
    const int64_t tid = static_cast<int64_t>(blockIdx.x) * bn_threads<CVEC>() + threadIdx.x;
    const int cv = static_cast<int>(tid % CVEC);
    float k1[8], k2[8], k3[8], sc[8], sh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        k1[k] = coef[cv * 8 + k];
        k2[k] = coef[C + cv * 8 + k];
        k3[k] = coef[2 * C + cv * 8 + k];
    }
    load_fwd_coef<CVEC, RM>(fcoef, cv, sc, sh);
    float d1[8], d2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d1[k] = d2[k] = 0.f;
    const bool dsum = DRES && dsx != nullptr;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * bn_threads<CVEC>();
    // two vectors per trip, every load issued before any is used (bytes in flight per lane)
    constexpr int U = 2;
    for (int64_t i0 = tid; i0 < nvec; i0 += U * stride) {
        typename G::Raw gr[U];
        uint4 xr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i < nvec) {
                gr[u] = grad.template fetch<CVEC>(i, i / CVEC, cv);
                xr[u] = ld16(x + i, ntl);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = i0 + u * stride;
            if (i >= nvec) break;
            float g[8], xv[8];
            grad.get(gr[u], g);
            unpack8(xr[u], xv);
            relu_gate<RM>(g, xv, sc, sh, mask, i);
            if (DRES) {
                const uint4 gr = pack8(g);
                st16(dres + i, gr, nts);
                if (dsum) {
                    float gq[8], sx[8];
                    unpack8(gr, gq);
                    unpack8(dsx[i], sx);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        d1[k] += gq[k];
                        d2[k] += gq[k] * sx[k];
                    }
                }
            }
            float o[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = k1[k] * g[k] + k2[k] * xv[k] + k3[k];
            st16(dx + i, pack8(o), nts);
        }
    }
    if (dsum) {
        constexpr int NT = bn_threads<CVEC>();
        __shared__ float red[kBlock][17];
        if (threadIdx.x < NT) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                red[threadIdx.x][k] = d1[k];
                red[threadIdx.x][8 + k] = d2[k];
            }
        }
        __syncthreads();
        for (int c = threadIdx.x; c < C; c += NT) {
            const int cvi = c >> 3, k = c & 7;
            double a1 = 0, a2 = 0;
            for (int u = cvi; u < NT; u += CVEC) {
                a1 += red[u][k];
                a2 += red[u][8 + k];
            }
            double *sl = dsums + (blockIdx.x % kStatSlots) * 2 * C;
            atomicAdd(sl + c, a1);
            atomicAdd(sl + C + c, a2);
        }
    }
}

template <typename F>
void dispatch_cvec(int cvec, F &&f) {
    switch (cvec) {
    case 4: f(std::integral_constant<int, 4>()); break;
    case 6: f(std::integral_constant<int, 6>()); break;
    case 10: f(std::integral_constant<int, 10>()); break;
    case 12: f(std::integral_constant<int, 12>()); break;
    case 20: f(std::integral_constant<int, 20>()); break;
    case 24: f(std::integral_constant<int, 24>()); break;
    case 40: f(std::integral_constant<int, 40>()); break;
    case 48: f(std::integral_constant<int, 48>()); break;
    case 56: f(std::integral_constant<int, 56>()); break;
    case 8: f(std::integral_constant<int, 8>()); break;
    case 16: f(std::integral_constant<int, 16>()); break;
    case 32: f(std::integral_constant<int, 32>()); break;
    case 64: f(std::integral_constant<int, 64>()); break;
    case 128: f(std::integral_constant<int, 128>()); break;
    case 256: f(std::integral_constant<int, 256>()); break;
    default: break;
    }
}

// blocks of bn_threads<CVEC>() threads (a multiple of CVEC, so any grid keeps cv fixed)
int apply_grid(int64_t nvec, int cvec) {
    const int nt = (kBlock / cvec) * cvec;
    int64_t g = (nvec + nt - 1) / nt;
    const int mg = bn_max_grid(kMaxGrid);
    if (g > mg) g = mg;
    if (g < 1) g = 1;
    return static_cast<int>(g);
}

void launch_stats(const uint16_t *x, BNShape sh, const float *gamma, const float *beta, float *run_mean,
                  float *run_var, float momentum, float eps, float *partial, float *mean, float *invstd, float *coef,
                  int64_t *num_batches, hipStream_t s) {
    const int C = sh.channels, cvec = C / 8;
    Chunking ch = chunking(sh);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        bn_stats_kernel<CV><<<ch.nchunks, bn_threads<CV>(), 0, s>>>(reinterpret_cast<const uint4 *>(x), sh.rows,
                                                          ch.rows_per_chunk, partial);
    });
    bn_stats_finalize<<<(C + kFoldCh - 1) / kFoldCh, kBlock, 0, s>>>(partial, ch.nchunks, C, sh.rows, gamma, beta,
                                                                     mean, invstd, run_mean, run_var, momentum, eps,
                                                                     coef, num_batches);
}

template <class G>
void launch_backward_impl(G grad, const uint16_t *x, const float *fcoef, const uint8_t *mask, const float *mean,
                          const float *invstd, const float *gamma, BNShape sh, int rm, bool training, float *partial,
                          float *dgamma, float *dbeta, float *coef, uint16_t *dx, uint16_t *dres, hipStream_t s,
                          double *sums = nullptr, const uint16_t *dres_x = nullptr, double *dres_sums = nullptr,
                          bool prefinalized = false, int phase = 0) {
    // phase 0: everything; 1: the reduce pass only (statistics path, no sums); 2: the apply pass only
    // (coef already finalized -- bn_bwd_finalize_multi); 3: statistics + finalize, no apply (the
    // caller consumes coef itself: the stem's fused weight gradient)
    const int C = sh.channels, cvec = C / 8;
    const int64_t nvec = sh.rows * cvec;
    Chunking ch = chunking(sh);
    const uint4 *xx = reinterpret_cast<const uint4 *>(x);
    if (phase == 2) {
    } else if (sums) {
        if (!prefinalized && !bn_skip_finalize())
        bn_bwd_finalize_sums<<<(C + 255) / 256, 256, 0, s>>>(sums, C, sh.rows, gamma, mean, invstd, dgamma, dbeta,
                                                             coef, training);
    } else {
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        auto go = [&](auto rmc) {
            constexpr int RM = decltype(rmc)::value;
            bn_bwd_reduce_kernel<CV, RM, G>
                <<<ch.nchunks, bn_threads<CV>(), 0, s>>>(grad, xx, fcoef, mask, sh.rows, ch.rows_per_chunk, partial,
                                                          bn_nt_mode());
        };
        if (rm == RM_COEF) go(std::integral_constant<int, RM_COEF>());
        else if (rm == RM_BITS) go(std::integral_constant<int, RM_BITS>());
        else go(std::integral_constant<int, RM_NONE>());
    });
    if (phase == 1) return;
    bn_bwd_finalize<<<(C + kFoldCh - 1) / kFoldCh, kBlock, 0, s>>>(partial, ch.nchunks, C, sh.rows, gamma, mean,
                                                                   invstd, dgamma, dbeta, coef, training);
    }
    if (phase == 3) return;
    const int g = apply_grid(nvec, cvec);
    uint4 *o = reinterpret_cast<uint4 *>(dx), *r = reinterpret_cast<uint4 *>(dres);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        auto go = [&](auto rmc, auto drc) {
            constexpr int RM = decltype(rmc)::value;
            constexpr bool DR = decltype(drc)::value;
            bn_bwd_apply_kernel<CV, RM, DR, G><<<g, bn_threads<CV>(), 0, s>>>(
                grad, xx, fcoef, mask, coef, o, r, nvec, DR ? reinterpret_cast<const uint4 *>(dres_x) : nullptr,
                DR ? dres_sums : nullptr, bn_nt_mode());
        };
        using T = std::true_type;
        using F = std::false_type;
        if (rm == RM_COEF) {
            if (dres) go(std::integral_constant<int, RM_COEF>(), T());
            else go(std::integral_constant<int, RM_COEF>(), F());
        } else if (rm == RM_BITS) {
            if (dres) go(std::integral_constant<int, RM_BITS>(), T());
            else go(std::integral_constant<int, RM_BITS>(), F());
        } else {
            if (dres) go(std::integral_constant<int, RM_NONE>(), T());
            else go(std::integral_constant<int, RM_NONE>(), F());
        }
    });
}

}  // namespace

void launch_bn_bwd_finalize_multi(const BnBwdFinBatch &b, hipStream_t s) {
    if (b.n <= 0) return;
    if (b.n > kBnFinMax) throw std::invalid_argument("bn_bwd_finalize_multi: too many BNs");
    int cmax = 0;
    for (int i = 0; i < b.n; ++i) cmax = b.d[i].C > cmax ? b.d[i].C : cmax;
    bn_bwd_finalize_multi<<<dim3((cmax + kFoldCh - 1) / kFoldCh, b.n), kBlock, 0, s>>>(b);
}

void launch_bn_sums_finalize_multi(const BnFinBatch &b, hipStream_t s) {
    if (b.n <= 0) return;
    if (b.n > kBnFinMax) throw std::invalid_argument("bn_sums_finalize_multi: too many BNs");
    int cmax = 0;
    for (int i = 0; i < b.n; ++i) cmax = b.d[i].C > cmax ? b.d[i].C : cmax;
    if (bn_skip_finalize()) return;
    bn_sums_finalize_multi<<<dim3((cmax + 255) / 256, b.n), 256, 0, s>>>(b);
}

bool bn_supported_channels(int C) {
    if (C % 8) return false;
    switch (C / 8) {
    case 4: case 6: case 8: case 10: case 12: case 16: case 20: case 24: case 32: case 40: case 48: case 56:
    case 64: case 128: case 256:
        return true;
    default:
        return false;
    }
}

int bn_num_chunks(BNShape sh) { return chunking(sh).nchunks; }

void launch_bn_forward(const uint16_t *x, const uint16_t *res, const float *gamma, const float *beta, uint16_t *y,
                       uint8_t *mask, BNShape sh, bool relu, bool training, float *run_mean, float *run_var,
                       float momentum, float eps, float *partial, float *mean, float *invstd, float *coef,
                       int64_t *num_batches, hipStream_t s, double *sums, const float *res_coef, bool apply,
                       int64_t y_ld, bool prefinalized) {
    const int C = sh.channels, cvec = C / 8;
    if (y_ld > 0 && (y_ld % 8 || y_ld < C || res || !relu))
        throw std::invalid_argument("bn_forward: a strided output needs BN+ReLU without residual, row stride % 8");
    const int64_t nvec = sh.rows * cvec;
    if (training && sums) {
        if (!prefinalized && !bn_skip_finalize())
        bn_sums_finalize<<<(C + 255) / 256, 256, 0, s>>>(sums, C, sh.rows, gamma, beta, mean, invstd, run_mean,
                                                         run_var, momentum, eps, coef, num_batches);
    } else if (training) {
        launch_stats(x, sh, gamma, beta, run_mean, run_var, momentum, eps, partial, mean, invstd, coef, num_batches,
                     s);
    } else {
        bn_eval_coef<<<(C + 255) / 256, 256, 0, s>>>(C, gamma, beta, run_mean, run_var, eps, mean, invstd, coef);
    }
    if (!apply) return;
    const int g = apply_grid(nvec, cvec);
    const int ntm = bn_nt_mode();
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        constexpr int NT = bn_threads<CV>();
        const uint4 *xv = reinterpret_cast<const uint4 *>(x);
        const uint4 *rv = reinterpret_cast<const uint4 *>(res);
        uint4 *yv = reinterpret_cast<uint4 *>(y);
        if (res && res_coef) {
            if (relu) bn_apply_kernel<CV, true, true, true><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, res_coef, ntm);
            else bn_apply_kernel<CV, true, false, true><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, res_coef, ntm);
        } else if (res) {
            if (relu) bn_apply_kernel<CV, true, true><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, nullptr, ntm);
            else bn_apply_kernel<CV, true, false><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, nullptr, ntm);
        } else if (y_ld > 0 && y_ld != C) {
            bn_apply_kernel<CV, false, true, false, true><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, nullptr, ntm,
                                                                          y_ld / 8);
        } else {
            if (relu) bn_apply_kernel<CV, false, true><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, nullptr, ntm);
            else bn_apply_kernel<CV, false, false><<<g, NT, 0, s>>>(xv, rv, coef, yv, mask, nvec, nullptr, ntm);
        }
    });
}

void launch_bn_backward(const uint16_t *dy, const uint16_t *x, const float *fcoef, const uint8_t *mask,
                        const float *mean, const float *invstd, const float *gamma, BNShape sh, bool relu,
                        bool training, float *partial, float *dgamma, float *dbeta, float *coef, uint16_t *dx,
                        uint16_t *dres, hipStream_t s, double *sums, const uint16_t *dres_x, double *dres_sums,
                        int64_t dy_ld, bool prefinalized, int phase) {
    const int rm = !relu ? RM_NONE : (mask ? RM_BITS : RM_COEF);
    if (dy_ld > 0 && dy_ld != sh.channels) {
        if (dy_ld % 8) throw std::invalid_argument("bn_backward: dy row stride must be a multiple of 8");
        launch_backward_impl(StridedGrad{reinterpret_cast<const uint4 *>(dy), dy_ld / 8}, x, fcoef, mask, mean, invstd,
                             gamma, sh, rm, training, partial, dgamma, dbeta, coef, dx, dres, s, sums, dres_x,
                             dres_sums, prefinalized, phase);
        return;
    }
    launch_backward_impl(DirectGrad{reinterpret_cast<const uint4 *>(dy), (bn_nt_mode() & 1) != 0}, x, fcoef, mask, mean, invstd, gamma, sh, rm,
                         training, partial, dgamma, dbeta, coef, dx, dres, s, sums, dres_x, dres_sums, prefinalized, phase);
}

bool bn_pool_supported(BNShape sh, int H, int W) {
    return bn_supported_channels(sh.channels) && H >= 2 && W >= 2 && sh.rows % (static_cast<int64_t>(H) * W) == 0 &&
           sh.rows * (sh.channels / 8) < (int64_t(1) << 31);  // PoolGrad uses 32-bit index math
}

void launch_bn_pool_forward(const uint16_t *x, const float *gamma, const float *beta, uint16_t *yp, uint8_t *arg,
                            BNShape sh, int H, int W, bool training, float *run_mean, float *run_var, float momentum,
                            float eps, float *partial, float *mean, float *invstd, float *coef, int64_t *num_batches,
                            hipStream_t s, double *sums, uint16_t *xarg) {
    const int C = sh.channels, cvec = C / 8;
    if (training && sums) {
        if (!bn_skip_finalize())
        bn_sums_finalize<<<(C + 255) / 256, 256, 0, s>>>(sums, C, sh.rows, gamma, beta, mean, invstd, run_mean,
                                                         run_var, momentum, eps, coef, num_batches);
    } else if (training) {
        launch_stats(x, sh, gamma, beta, run_mean, run_var, momentum, eps, partial, mean, invstd, coef, num_batches,
                     s);
    } else {
        bn_eval_coef<<<(C + 255) / 256, 256, 0, s>>>(C, gamma, beta, run_mean, run_var, eps, mean, invstd, coef);
    }
    const int OH = pool_out(H), OW = pool_out(W);
    const int64_t N = sh.rows / (static_cast<int64_t>(H) * W);
    const int64_t nout = N * OH * OW * cvec;
    const int g = apply_grid(nout, cvec);
    dispatch_cvec(cvec, [&](auto cvc) {
        constexpr int CV = decltype(cvc)::value;
        bn_pool_apply_kernel<CV><<<g, bn_threads<CV>(), 0, s>>>(reinterpret_cast<const uint4 *>(x), coef,
                                                      reinterpret_cast<uint4 *>(yp), reinterpret_cast<uint2 *>(arg), H,
                                                      W, OH, OW, nout, reinterpret_cast<uint4 *>(xarg));
    });
}

void launch_bn_pool_backward(const uint16_t *dyp, const uint8_t *arg, const uint16_t *x, const float *fcoef,
                             const float *mean, const float *invstd, const float *gamma, BNShape sh, int H, int W,
                             bool training, float *partial, float *dgamma, float *dbeta, float *coef, uint16_t *dx,
                             hipStream_t s, const uint16_t *xarg, double *sums, bool apply) {
    if (xarg && sums && training) {
        const int C = sh.channels, cvec = C / 8;
        const int64_t nvec = sh.rows / (static_cast<int64_t>(H) * W) * pool_out(H) * pool_out(W) * cvec;
        const int g = apply_grid(nvec, cvec);
        dispatch_cvec(cvec, [&](auto cvc) {
            constexpr int CV = decltype(cvc)::value;
            bn_pool_bwd_sums_kernel<CV><<<g, bn_threads<CV>(), 0, s>>>(
                reinterpret_cast<const uint4 *>(dyp), reinterpret_cast<const uint4 *>(xarg), fcoef, sums, nvec);
        });
    } else {
        sums = nullptr;
    }
    const uint64_t m_hw = (uint64_t(1) << 40) / (static_cast<uint64_t>(H) * W) + 1;
    const uint64_t m_w = (uint64_t(1) << 40) / static_cast<uint64_t>(W) + 1;
    if (static_cast<uint64_t>(sh.rows) * H * W >= (uint64_t(1) << 40))
        throw std::invalid_argument("bn_pool_backward: too many rows for the 40-bit division");
    PoolGrad pg{reinterpret_cast<const uint4 *>(dyp), reinterpret_cast<const uint2 *>(arg), H, W, pool_out(H),
                pool_out(W), m_hw, m_w};
    launch_backward_impl(pg, x, fcoef, nullptr, mean, invstd, gamma, sh, RM_COEF, training, partial, dgamma, dbeta,
                         coef, dx, nullptr, s, sums, nullptr, nullptr, false, apply ? 0 : 3);
}

}  // namespace kfk
