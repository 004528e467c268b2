// 2x2 / stride-2 max-pool on NHWC bf16 (VGG-16's five pools), forward and backward, for gfx950.
//
// Why: torch's NHWC max-pool writes an int64 argmax per output (4x the bytes of the bf16
// output) and its backward zero-fills dx and scatters into it: 6.3 ms of a 50 ms VGG-16 step
// (profiles/r17_vgg16_b256_biasrelu.md).  The 2x2/s2 windows do not overlap, so:
//
//   forward   read the 4 window vectors, write the max                    (no argmax tensor)
//   backward  re-read the 4 window vectors and dy, write all 4 dx vectors (a gather: every
//             dx element written exactly once, no zero-fill, no atomics)
//
// The window element that receives the gradient is the first maximum in (0,0), (0,1),
// (1,0), (1,1) order -- the forward's choice recomputed from x.  One lane = one 16-byte
// vector of 8 channels of one output pixel.
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

__device__ __forceinline__ float lo16(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi16(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

struct PoolGeo {
    int H, W, OH, OW, CV;
    int64_t nout;  // N * OH * OW * CV
};

// vector index of window element (dy, dx) for output vector i
__device__ __forceinline__ int64_t window_base(const PoolGeo &g, int64_t i, int &cv) {
    cv = static_cast<int>(i % g.CV);
    int64_t t = i / g.CV;
    const int ow = static_cast<int>(t % g.OW);
    t /= g.OW;
    const int oh = static_cast<int>(t % g.OH);
    const int64_t n = t / g.OH;
    return ((n * g.H + 2 * oh) * g.W + 2 * ow) * g.CV + cv;
}

__device__ __forceinline__ uint32_t bits_of(const uint4 &v, int k) {
    return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w;
}

__global__ __launch_bounds__(kBlock) void maxpool2_fwd_kernel(const uint4 *__restrict__ x, uint4 *__restrict__ y,
                                                              PoolGeo g) {
    const int64_t rowv = static_cast<int64_t>(g.W) * g.CV;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < g.nout;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        int cv;
        const int64_t b = window_base(g, i, cv);
        const uint4 v[4] = {x[b], x[b + g.CV], x[b + rowv], x[b + rowv + g.CV]};
        uint32_t out[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float ml = lo16(bits_of(v[0], k)), mh = hi16(bits_of(v[0], k));
            uint32_t bl = bits_of(v[0], k) & 0xffffu, bh = bits_of(v[0], k) >> 16;
#pragma unroll
            for (int p = 1; p < 4; ++p) {
                const uint32_t w = bits_of(v[p], k);
                // NaN propagates like torch's max-pool: a NaN always takes the window
                if (lo16(w) > ml || isnan(lo16(w))) ml = lo16(w), bl = w & 0xffffu;
                if (hi16(w) > mh || isnan(hi16(w))) mh = hi16(w), bh = w >> 16;
            }
            out[k] = bl | (bh << 16);
        }
        y[i] = make_uint4(out[0], out[1], out[2], out[3]);
    }
}

// GATE: x is a ReLU output and dx goes on as that ReLU's input gradient: the window maximum
// passes dy only where it is > 0 (NaN passes, like torch.relu's backward), and the per-channel
// sums of dx (the preceding conv's bias gradient) go to the f64 slots stats[slot][0][C].
// The grid stride is a multiple of CV (kBlock % CV == 0), so a thread keeps one channel group.
template <bool GATE>
__global__ __launch_bounds__(kBlock) void maxpool2_bwd_kernel(const uint4 *__restrict__ x,
                                                              const uint4 *__restrict__ dy, uint4 *__restrict__ dx,
                                                              PoolGeo g, double *__restrict__ stats) {
    float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int64_t rowv = static_cast<int64_t>(g.W) * g.CV;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < g.nout;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        int cv;
        const int64_t b = window_base(g, i, cv);
        const int64_t off[4] = {b, b + g.CV, b + rowv, b + rowv + g.CV};
        const uint4 v[4] = {x[off[0]], x[off[1]], x[off[2]], x[off[3]]};
        const uint4 gv = dy[i];
        uint32_t o[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            // first maximum per half-word, as the forward chose it
            float ml = lo16(bits_of(v[0], k)), mh = hi16(bits_of(v[0], k));
            int pl = 0, ph = 0;
#pragma unroll
            for (int p = 1; p < 4; ++p) {
                const uint32_t w = bits_of(v[p], k);
                if (lo16(w) > ml || isnan(lo16(w))) ml = lo16(w), pl = p;
                if (hi16(w) > mh || isnan(hi16(w))) mh = hi16(w), ph = p;
            }
            uint32_t gw = bits_of(gv, k);
            if constexpr (GATE) {
                if (ml <= 0.f) gw &= 0xffff0000u;
                if (mh <= 0.f) gw &= 0xffffu;
                csum[2 * k] += lo16(gw);
                csum[2 * k + 1] += hi16(gw);
            }
#pragma unroll
            for (int p = 0; p < 4; ++p)
                o[p][k] = (p == pl ? (gw & 0xffffu) : 0u) | (p == ph ? (gw & 0xffff0000u) : 0u);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) dx[off[p]] = make_uint4(o[p][0], o[p][1], o[p][2], o[p][3]);
    }
    if constexpr (GATE) {
        __shared__ float red[kBlock][9];  // padded: the CV threads of a channel group are spread
        const int t = threadIdx.x;
#pragma unroll
        for (int k = 0; k < 8; ++k) red[t][k] = csum[k];
        __syncthreads();
        for (int c = t; c < g.CV * 8; c += kBlock) {
            const int cvi = c >> 3, k = c & 7;  // fold channel 8 cvi + k
            double a = 0;
            for (int u = cvi; u < kBlock; u += g.CV) a += red[u][k];
            atomicAdd(stats + (blockIdx.x % kStatSlots) * 2 * (g.CV * 8) + c, a);
        }
    }
}


// ---------------------------------------------------------------- 3x3 pools (Inception-v3)
//
// max 3x3 / stride 2 / pad P (P = 0: Inception's reduction pools): the windows overlap, so
// the forward also writes the window argmax (0..8) as one byte per element (8 bytes per
// 16-byte output vector, 1/2 of y -- vs torch's int64 per element, 8x of y) and the backward
// is a gather over the <= 2x2 windows covering each input pixel (no zero-fill, no atomics,
// every dx element written once).  NaN takes the window, as in torch.
//
// avg 3x3 / stride 1 / pad 1, count_include_pad (the Inception pool branches): a 9-tap
// stencil with divisor 9; its gradient is the same stencil applied to dy.
struct Pool3Geo {
    int H, W, OH, OW, CV, P;
    int64_t nout;  // N * OH * OW * CV
};

__global__ __launch_bounds__(kBlock) void maxpool3s2_fwd_kernel(const uint4 *__restrict__ x, uint4 *__restrict__ y,
                                                                uint2 *__restrict__ arg, Pool3Geo g) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < g.nout;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int cv = static_cast<int>(i % g.CV);
        int64_t t = i / g.CV;
        const int ow = static_cast<int>(t % g.OW);
        t /= g.OW;
        const int oh = static_cast<int>(t % g.OH);
        const int64_t n = t / g.OH;
        float best[8];
        uint32_t a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            best[k] = -INFINITY;
            a[k] = 0;
        }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
            const int h = 2 * oh - g.P + kh;
            if (h < 0 || h >= g.H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) {
                const int w = 2 * ow - g.P + kw;
                if (w < 0 || w >= g.W) continue;
                const uint4 v = x[((n * g.H + h) * g.W + w) * g.CV + cv];
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float f = (k & 1) ? hi16(bits_of(v, k >> 1)) : lo16(bits_of(v, k >> 1));
                    if (f > best[k] || isnan(f)) {  // torch: a later NaN takes over
                        best[k] = f;
                        a[k] = kh * 3 + kw;
                    }
                }
            }
        }
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = pack_bf16x2(best[2 * k], best[2 * k + 1]);
        y[i] = make_uint4(o[0], o[1], o[2], o[3]);
        arg[i] = make_uint2(a[0] | (a[1] << 8) | (a[2] << 16) | (a[3] << 24),
                            a[4] | (a[5] << 8) | (a[6] << 16) | (a[7] << 24));
    }
}

// one lane per input vector: gather dy of every window (oh, ow) that contains (h, w) and
// whose argmax byte points at it.  nin = N * H * W * CV.
__global__ __launch_bounds__(kBlock) void maxpool3s2_bwd_kernel(const uint4 *__restrict__ dy,
                                                                const uint2 *__restrict__ arg, uint4 *__restrict__ dx,
                                                                Pool3Geo g, int64_t nin) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < nin;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int cv = static_cast<int>(i % g.CV);
        int64_t t = i / g.CV;
        const int w = static_cast<int>(t % g.W);
        t /= g.W;
        const int h = static_cast<int>(t % g.H);
        const int64_t n = t / g.H;
        // windows with 2*oh - P <= h <= 2*oh - P + 2
        const int hp = h + g.P, wp = w + g.P;
        int oh0 = (hp - 2 + 1) / 2, oh1 = hp / 2, ow0 = (wp - 2 + 1) / 2, ow1 = wp / 2;
        if (hp - 2 < 0) oh0 = 0;
        if (wp - 2 < 0) ow0 = 0;
        if (oh1 > g.OH - 1) oh1 = g.OH - 1;
        if (ow1 > g.OW - 1) ow1 = g.OW - 1;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
        for (int oh = oh0; oh <= oh1; ++oh)
            for (int ow = ow0; ow <= ow1; ++ow) {
                const int64_t o = ((n * g.OH + oh) * g.OW + ow) * g.CV + cv;
                const uint2 am = arg[o];
                const uint4 d = dy[o];
                const uint32_t me = static_cast<uint32_t>((hp - 2 * oh) * 3 + (wp - 2 * ow));
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const uint32_t ak = ((k < 4 ? am.x : am.y) >> (8 * (k & 3))) & 0xffu;
                    const float f = (k & 1) ? hi16(bits_of(d, k >> 1)) : lo16(bits_of(d, k >> 1));
                    acc[k] += ak == me ? f : 0.f;
                }
            }
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = pack_bf16x2(acc[2 * k], acc[2 * k + 1]);
        dx[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// y = (1/9) * sum of the 3x3 window (zero padding, count_include_pad), same H x W
__global__ __launch_bounds__(kBlock) void avgpool3s1_kernel(const uint4 *__restrict__ x, uint4 *__restrict__ y, int H,
                                                            int W, int CV, int64_t n) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int cv = static_cast<int>(i % CV);
        int64_t t = i / CV;
        const int w = static_cast<int>(t % W);
        t /= W;
        const int h = static_cast<int>(t % H);
        const int64_t nn = t / H;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll
        for (int dh = -1; dh <= 1; ++dh) {
            const int hh = h + dh;
            if (hh < 0 || hh >= H) continue;
#pragma unroll
            for (int dw = -1; dw <= 1; ++dw) {
                const int ww = w + dw;
                if (ww < 0 || ww >= W) continue;
                const uint4 v = x[((nn * H + hh) * W + ww) * CV + cv];
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    acc[k] += (k & 1) ? hi16(bits_of(v, k >> 1)) : lo16(bits_of(v, k >> 1));
            }
        }
        constexpr float inv9 = 1.f / 9.f;
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = pack_bf16x2(acc[2 * k] * inv9, acc[2 * k + 1] * inv9);
        y[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// Global average pool (the ResNet / Inception head), NHWC: y[n, c] = mean over the HW pixels.
// One thread per (n, 8-channel group); adjacent threads read adjacent 16-byte vectors of a
// pixel, the HW pixels are walked with 4 loads in flight.
__global__ __launch_bounds__(kBlock) void gap_fwd_kernel(const uint4 *__restrict__ x, uint4 *__restrict__ y, int HW,
                                                         int CV, int64_t n, float inv) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int cv = static_cast<int>(i % CV);
        const int64_t nn = i / CV;
        const uint4 *p = x + nn * HW * CV + cv;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = 0.f;
        int q = 0;
        for (; q + 4 <= HW; q += 4) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = p[static_cast<int64_t>(q + u) * CV];
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int k = 0; k < 8; ++k) acc[k] += (k & 1) ? hi16(bits_of(v[u], k >> 1)) : lo16(bits_of(v[u], k >> 1));
        }
        for (; q < HW; ++q) {
            const uint4 v = p[static_cast<int64_t>(q) * CV];
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] += (k & 1) ? hi16(bits_of(v, k >> 1)) : lo16(bits_of(v, k >> 1));
        }
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = pack_bf16x2(acc[2 * k] * inv, acc[2 * k + 1] * inv);
        y[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

// dx[n, p, c] = dy[n, c] / HW for every pixel p: one 16-byte store per thread
__global__ __launch_bounds__(kBlock) void gap_bwd_kernel(const uint4 *__restrict__ dy, uint4 *__restrict__ dx, int HW,
                                                         int CV, int64_t n, float inv) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * kBlock) {
        const int cv = static_cast<int>(i % CV);
        const int64_t nn = i / (static_cast<int64_t>(CV) * HW);
        const uint4 d = dy[nn * CV + cv];
        uint32_t o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            o[k] = static_cast<uint32_t>(f32_to_bf16(lo16(bits_of(d, k)) * inv)) |
                   (static_cast<uint32_t>(f32_to_bf16(hi16(bits_of(d, k)) * inv)) << 16);
        dx[i] = make_uint4(o[0], o[1], o[2], o[3]);
    }
}

PoolGeo pool_geo(int64_t N, int H, int W, int C) {
    if (C % 8 || H % 2 || W % 2) throw std::invalid_argument("maxpool2x2: needs C % 8 == 0 and even H, W");
    PoolGeo g;
    g.H = H, g.W = W, g.OH = H / 2, g.OW = W / 2, g.CV = C / 8;
    g.nout = N * g.OH * g.OW * g.CV;
    return g;
}

int pool_grid(int64_t n) {
    int64_t b = (n + kBlock - 1) / kBlock;
    if (b > 8192) b = 8192;
    return static_cast<int>(b < 1 ? 1 : b);
}

}  // namespace

void launch_maxpool2x2_forward(const uint16_t *x, uint16_t *y, int64_t N, int H, int W, int C, hipStream_t s) {
    const PoolGeo g = pool_geo(N, H, W, C);
    if (g.nout == 0) return;
    maxpool2_fwd_kernel<<<pool_grid(g.nout), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x),
                                                              reinterpret_cast<uint4 *>(y), g);
}

void launch_maxpool2x2_backward(const uint16_t *x, const uint16_t *dy, uint16_t *dx, int64_t N, int H, int W, int C,
                                hipStream_t s, double *gate_stats) {
    const PoolGeo g = pool_geo(N, H, W, C);
    if (g.nout == 0) return;
    if (gate_stats) {
        if (kBlock % g.CV != 0) throw std::invalid_argument("maxpool2x2 gate: C/8 must divide 256");
        maxpool2_bwd_kernel<true><<<pool_grid(g.nout), kBlock, 0, s>>>(
            reinterpret_cast<const uint4 *>(x), reinterpret_cast<const uint4 *>(dy), reinterpret_cast<uint4 *>(dx), g,
            gate_stats);
        return;
    }
    maxpool2_bwd_kernel<false><<<pool_grid(g.nout), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x),
                                                                     reinterpret_cast<const uint4 *>(dy),
                                                                     reinterpret_cast<uint4 *>(dx), g, nullptr);
}

int maxpool3s2_out(int h, int pad) { return (h + 2 * pad - 3) / 2 + 1; }

void launch_maxpool3s2_forward(const uint16_t *x, uint16_t *y, uint8_t *arg, int64_t N, int H, int W, int C, int pad,
                               hipStream_t s) {
    if (C % 8) throw std::invalid_argument("maxpool3x3s2: needs C % 8 == 0");
    Pool3Geo g;
    g.H = H, g.W = W, g.P = pad, g.CV = C / 8, g.OH = maxpool3s2_out(H, pad), g.OW = maxpool3s2_out(W, pad);
    g.nout = N * g.OH * g.OW * g.CV;
    if (g.nout <= 0) return;
    maxpool3s2_fwd_kernel<<<pool_grid(g.nout), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x),
                                                                reinterpret_cast<uint4 *>(y),
                                                                reinterpret_cast<uint2 *>(arg), g);
}

void launch_maxpool3s2_backward(const uint16_t *dy, const uint8_t *arg, uint16_t *dx, int64_t N, int H, int W, int C,
                                int pad, hipStream_t s) {
    if (C % 8) throw std::invalid_argument("maxpool3x3s2: needs C % 8 == 0");
    Pool3Geo g;
    g.H = H, g.W = W, g.P = pad, g.CV = C / 8, g.OH = maxpool3s2_out(H, pad), g.OW = maxpool3s2_out(W, pad);
    g.nout = N * g.OH * g.OW * g.CV;
    const int64_t nin = N * H * W * g.CV;
    if (nin <= 0) return;
    maxpool3s2_bwd_kernel<<<pool_grid(nin), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(dy),
                                                             reinterpret_cast<const uint2 *>(arg),
                                                             reinterpret_cast<uint4 *>(dx), g, nin);
}

void launch_avgpool3s1(const uint16_t *x, uint16_t *y, int64_t N, int H, int W, int C, hipStream_t s) {
    if (C % 8) throw std::invalid_argument("avgpool3x3s1: needs C % 8 == 0");
    const int64_t n = N * H * W * (C / 8);
    if (n <= 0) return;
    avgpool3s1_kernel<<<pool_grid(n), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x), reinterpret_cast<uint4 *>(y),
                                                       H, W, C / 8, n);
}

void launch_global_avgpool_forward(const uint16_t *x, uint16_t *y, int64_t N, int HW, int C, hipStream_t s) {
    if (C % 8 || HW <= 0) throw std::invalid_argument("global_avgpool: needs C % 8 == 0");
    const int64_t n = N * (C / 8);
    if (n <= 0) return;
    gap_fwd_kernel<<<pool_grid(n), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x), reinterpret_cast<uint4 *>(y), HW,
                                                    C / 8, n, 1.f / HW);
}

void launch_global_avgpool_backward(const uint16_t *dy, uint16_t *dx, int64_t N, int HW, int C, hipStream_t s) {
    if (C % 8 || HW <= 0) throw std::invalid_argument("global_avgpool: needs C % 8 == 0");
    const int64_t n = N * HW * (C / 8);
    if (n <= 0) return;
    gap_bwd_kernel<<<pool_grid(n), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(dy), reinterpret_cast<uint4 *>(dx), HW,
                                                    C / 8, n, 1.f / HW);
}

}  // namespace kfk
