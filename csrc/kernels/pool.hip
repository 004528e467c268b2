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

__global__ __launch_bounds__(kBlock) void maxpool2_bwd_kernel(const uint4 *__restrict__ x,
                                                              const uint4 *__restrict__ dy, uint4 *__restrict__ dx,
                                                              PoolGeo g) {
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
            const uint32_t gw = bits_of(gv, k);
#pragma unroll
            for (int p = 0; p < 4; ++p)
                o[p][k] = (p == pl ? (gw & 0xffffu) : 0u) | (p == ph ? (gw & 0xffff0000u) : 0u);
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) dx[off[p]] = make_uint4(o[p][0], o[p][1], o[p][2], o[p][3]);
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
                                hipStream_t s) {
    const PoolGeo g = pool_geo(N, H, W, C);
    if (g.nout == 0) return;
    maxpool2_bwd_kernel<<<pool_grid(g.nout), kBlock, 0, s>>>(reinterpret_cast<const uint4 *>(x),
                                                              reinterpret_cast<const uint4 *>(dy),
                                                              reinterpret_cast<uint4 *>(dx), g);
}

}  // namespace kfk
