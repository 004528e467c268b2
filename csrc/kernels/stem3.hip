// Small image-stem convolution on CDNA4 matrix cores, for gfx950: a KH x KW (<= 4 x 4) window over
// a 3-channel image, 32 output channels, any stride / zero padding -- Inception-v3's Conv2d_1a
// (3x3, stride 2, no padding, 3 -> 32), the last convolution of the Inception step that ran on MIOpen
// (fwd 0.10 + weight gradient 0.23 ms per 256-image step, profiles/r4z_inception_v3_summary.md, plus
// the f32 -> bf16 image cast and the BN's statistics pass it needed).
//
// Layout: the image is read as it is (f32 or bf16 NHWC, 3 channels: no cast / pad pass); the im2col
// K index is k = kh*16 + kw*4 + c (kw padded to 4, c to 4: zero weights), so one lane's 8-element MFMA
// fragment is 2 neighbouring pixels of one window row (3 channels each, converted to bf16 on load).
// K <= 64 = two K-steps of v_mfma_f32_16x16x32_bf16.
//
// Forward: a wave computes 64 output pixels x 32 channels per trip (4 x 2 MFMA tiles, 2 K-steps) with
// the weights held in registers for the whole kernel; the product is computed transposed (weights as
// the MFMA A operand), and the weight rows are permuted so that each lane ends with 8 CONSECUTIVE
// channels of one pixel (rows 4q+t of the two 16-channel blocks are channels 8q+t and 8q+4+t) -- one
// 16-byte bf16 store, a pixel's 64 bytes from 4 lanes -- and the following BN's per-channel sum /
// sum of squares of the bf16 outputs are reduced with lane shuffles and LDS, then added to the BN's
// f64 slotted workspace (as conv.hip) once per workgroup.
// Weight gradient: per trip a workgroup stages 256 pixels (64 per wave) of dy and of the im2col rows
// TRANSPOSED into LDS (feature-major, 16-byte pixel runs: the MFMA's K dimension is the pixels), so
// the fragments are ds_read_b128 row reads; each wave accumulates its 32 x 64 tile over the trips,
// the workgroup folds its 4 waves and writes one f32 partial; stem3_wgrad_reduce_kernel sums the
// partials in a fixed order (deterministic) and unpacks [co][kh][kw][c].
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int kCo = 32;
constexpr int kKp = 64;       // padded K: 4 kh x 4 kw x 4 c
constexpr int kRowS = 144;    // LDS bytes per transposed row (64 pixels x 2 B + 16 pad)

struct S3Geo {
    int N, H, W, OH, OW, M, KH, KW, stride, ph, pw;
};

typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;

// two f32 -> packed bf16 pair (round to nearest even: v_cvt_pk_bf16_f32), schedulable like any other op
__device__ __forceinline__ uint32_t pk2(float a, float b) {
    const bf16x2 v = __builtin_convertvector(f32x2{a, b}, bf16x2);
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ float ldf(const float *p) { return *p; }
__device__ __forceinline__ float ldf(const uint16_t *p) { return __uint_as_float(static_cast<uint32_t>(*p) << 16); }

// One K-chunk of the im2col row of output pixel p, unconverted: window row ih, columns iw0, iw0+1, the 3
// channels of each; out-of-image pixels and chunks past the window are zero
template <class T>
__device__ __forceinline__ void im2col_raw(const T *__restrict__ x, const S3Geo &g, int n, int ih, int iw0, bool valid,
                                           float (&v)[6]) {
#pragma unroll
    for (int c = 0; c < 6; ++c) v[c] = 0.f;
    if (valid && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H)) {
        const T *row = x + (static_cast<int64_t>(n) * g.H + ih) * g.W * 3;
        if (static_cast<unsigned>(iw0) < static_cast<unsigned>(g.W)) {
#pragma unroll
            for (int c = 0; c < 3; ++c) v[c] = ldf(row + iw0 * 3 + c);
        }
        if (static_cast<unsigned>(iw0 + 1) < static_cast<unsigned>(g.W)) {
#pragma unroll
            for (int c = 0; c < 3; ++c) v[3 + c] = ldf(row + (iw0 + 1) * 3 + c);
        }
    }
}

// the 8 bf16 of a chunk (a zero 4th channel per pixel)
__device__ __forceinline__ uint4 pack_chunk(const float (&v)[6]) {
    return make_uint4(pk2(v[0], v[1]), pk2(v[2], 0.f), pk2(v[3], v[4]), pk2(v[5], 0.f));
}

template <class T>
__device__ __forceinline__ uint4 im2col_chunk(const T *__restrict__ x, const S3Geo &g, int n, int ih, int iw0,
                                              bool valid) {
    float v[6];
    im2col_raw(x, g, n, ih, iw0, valid, v);
    return pack_chunk(v);
}

// MFMA row rho (0..31 over the two 16-row blocks) -> output channel: lane rows 4q+t of block j hold
// channel 8q + 4j + t, so a lane's 8 results are 8 consecutive channels
__device__ __forceinline__ int perm_ch(int rho) { return ((rho & 15) >> 2) * 8 + (rho >> 4) * 4 + (rho & 3); }

template <class T>
__global__ __launch_bounds__(256) void stem3_fwd_kernel(const T *__restrict__ x, const uint4 *__restrict__ wp,
                                                        uint4 *__restrict__ y, double *__restrict__ stats, S3Geo g) {
    __shared__ float red[4][2][kCo];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, r = lane & 15;
    // weights as the MFMA A operand: rows = output channels, K chunk q of K-step s
    bf16x8 wa[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const uint4 v = wp[(perm_ch(j * 16 + r) * kKp + s * 32 + q * 8) / 8];
            __builtin_memcpy(&wa[j][s], &v, 16);
        }
    // this lane's K chunks: (s, q) -> window row kh, first column kw0
    int ckh[2], ckw[2];
    bool cval[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int k0 = s * 32 + q * 8;
        ckh[s] = k0 >> 4;
        ckw[s] = (k0 & 15) >> 2;
        cval[s] = ckh[s] < g.KH && ckw[s] < g.KW;
    }
    float s1[2][4], s2[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) s1[j][t] = s2[j][t] = 0.f;
    const int ntiles = (g.M + 63) / 64;
    for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += gridDim.x * 4) {
        f32x4 acc[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = tile * 64 + i * 16 + r;
            int n = 0, ih0 = 0, iw0 = 0;
            const bool pin = p < g.M;
            if (pin) {
                const int ow = p % g.OW, t = p / g.OW, oh = t % g.OH;
                n = t / g.OH;
                ih0 = oh * g.stride - g.ph;
                iw0 = ow * g.stride - g.pw;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const uint4 v = im2col_chunk(x, g, n, ih0 + ckh[s], iw0 + ckw[s], pin && cval[s]);
                bf16x8 b;
                __builtin_memcpy(&b, &v, 16);
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[j][s], b, acc[j][i], 0, 0, 0);
            }
        }
        // lane holds channels 8q + 4j + (0..3) of pixel i*16 + r: one 16-byte store of 8 channels
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = tile * 64 + i * 16 + r;
            if (p >= g.M) continue;
            uint32_t w[4];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                w[2 * j] = pk2(acc[j][i][0], acc[j][i][1]);
                w[2 * j + 1] = pk2(acc[j][i][2], acc[j][i][3]);
            }
            y[static_cast<int64_t>(p) * (kCo / 8) + q] = make_uint4(w[0], w[1], w[2], w[3]);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const float v[4] = {__uint_as_float(w[2 * j] << 16), __uint_as_float(w[2 * j] & 0xffff0000u),
                                    __uint_as_float(w[2 * j + 1] << 16), __uint_as_float(w[2 * j + 1] & 0xffff0000u)};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    s1[j][t] += v[t];
                    s2[j][t] += v[t] * v[t];
                }
            }
        }
    }
    if (stats == nullptr) return;
    // fold the 16 pixel lanes of each channel quad, then the 4 waves, then one f64 add per channel
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) {
                s1[j][t] += __shfl_xor(s1[j][t], o, 64);
                s2[j][t] += __shfl_xor(s2[j][t], o, 64);
            }
        }
    if (r == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                red[wave][0][8 * q + 4 * j + t] = s1[j][t];
                red[wave][1][8 * q + 4 * j + t] = s2[j][t];
            }
    }
    __syncthreads();
    if (threadIdx.x < 2 * kCo) {
        const int which = threadIdx.x / kCo, c = threadIdx.x % kCo;
        double a = 0.0;
        for (int w = 0; w < 4; ++w) a += red[w][which][c];
        atomicAdd(stats + (blockIdx.x % kStatSlots) * 2 * kCo + which * kCo + c, a);
    }
}

// dy [M, 32] bf16, x [N, H, W, 3] f32 / bf16 -> part[block][32][64] f32 (one per workgroup)
template <class T>
__global__ __launch_bounds__(256) void stem3_wgrad_kernel(const uint4 *__restrict__ dy, const T *__restrict__ x,
                                                          float *__restrict__ part, S3Geo g) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4 * (kCo + kKp) * kRowS];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, r = lane & 15;
    uint8_t *dyT = lds + wave * (kCo + kKp) * kRowS;  // [32 co][64 px]
    uint8_t *colT = dyT + kCo * kRowS;                 // [64 k][64 px]
    const int nkb = (g.KH * 16 + 15) / 16;             // 16-wide k blocks that carry the window
    f32x4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[j][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nblk = (g.M + 255) / 256;
    // next trip's dy row and raw im2col chunks, loaded into registers while this trip's MFMAs run
    uint4 d[4];
    float xv[4][2][6];
    auto fetch = [&](int blk) {
        const int p = blk * 256 + wave * 64 + lane;
        const bool pin = blk < nblk && p < g.M;
#pragma unroll
        for (int u = 0; u < 4; ++u) d[u] = pin ? dy[static_cast<int64_t>(p) * 4 + u] : make_uint4(0u, 0u, 0u, 0u);
        int n = 0, ih0 = 0, iw0 = 0;
        if (pin) {
            const int ow = p % g.OW, t = p / g.OW, oh = t % g.OH;
            n = t / g.OH;
            ih0 = oh * g.stride - g.ph;
            iw0 = ow * g.stride - g.pw;
        }
#pragma unroll
        for (int kh = 0; kh < 4; ++kh)
#pragma unroll
            for (int h = 0; h < 2; ++h) im2col_raw(x, g, n, ih0 + kh, iw0 + 2 * h, pin && kh < g.KH && 2 * h < g.KW, xv[kh][h]);
    };
    fetch(blockIdx.x);
    for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // uniform trip count per workgroup
        // dy row of this lane's pixel -> column `lane` of dyT
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t w4[4] = {d[u].x, d[u].y, d[u].z, d[u].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                *reinterpret_cast<uint16_t *>(dyT + (u * 8 + 2 * e) * kRowS + lane * 2) = static_cast<uint16_t>(w4[e]);
                *reinterpret_cast<uint16_t *>(dyT + (u * 8 + 2 * e + 1) * kRowS + lane * 2) =
                    static_cast<uint16_t>(w4[e] >> 16);
            }
        }
        // im2col row of this lane's pixel -> column `lane` of colT (rows k = kh*16 + kw*4 + c)
#pragma unroll
        for (int kh = 0; kh < 4; ++kh) {
            if (kh >= g.KH) break;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint4 v = pack_chunk(xv[kh][h]);
                const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int k = kh * 16 + h * 8 + 2 * e;
                    *reinterpret_cast<uint16_t *>(colT + k * kRowS + lane * 2) = static_cast<uint16_t>(w4[e]);
                    *reinterpret_cast<uint16_t *>(colT + (k + 1) * kRowS + lane * 2) = static_cast<uint16_t>(w4[e] >> 16);
                }
            }
        }
        fetch(blk + gridDim.x);
        __syncthreads();
        // dW[co][k] += sum over this wave's 64 pixels: two 32-pixel K-steps
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 a[2];
#pragma unroll
            for (int j = 0; j < 2; ++j) a[j] = *reinterpret_cast<const bf16x8 *>(dyT + (j * 16 + r) * kRowS + (s * 32 + q * 8) * 2);
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                if (b >= nkb) break;
                const bf16x8 c = *reinterpret_cast<const bf16x8 *>(colT + (b * 16 + r) * kRowS + (s * 32 + q * 8) * 2);
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[j][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[j], c, acc[j][b], 0, 0, 0);
            }
        }
        __syncthreads();  // the next trip overwrites the images
    }
    // fold the 4 waves through LDS (the images are dead): lane holds C[co = j*16 + 4q + t][k = b*16 + r]
    float *fr = reinterpret_cast<float *>(lds);  // [4 waves][32][64]
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int t = 0; t < 4; ++t) fr[(wave * kCo + j * 16 + q * 4 + t) * kKp + b * 16 + r] = acc[j][b][t];
    __syncthreads();
    float *dst = part + static_cast<int64_t>(blockIdx.x) * kCo * kKp;
    for (int e = threadIdx.x; e < kCo * kKp; e += 256)
        dst[e] = (fr[e] + fr[kCo * kKp + e]) + (fr[2 * kCo * kKp + e] + fr[3 * kCo * kKp + e]);
}

// Level 1 of the partial sum: mid[rg][e] = sum of partial rows [rg*16, rg*16+16) (e over the 32 x 64
// padded tile); coalesced across threads, 16 loads per thread
__global__ __launch_bounds__(256) void stem3_wgrad_fold_kernel(const float *__restrict__ part, int blocks,
                                                               float *__restrict__ mid) {
    const int e = blockIdx.x * 256 + threadIdx.x, rg = blockIdx.y;
    float a = 0.f;
    const int b1 = min(blocks, rg * 16 + 16);
    for (int b = rg * 16; b < b1; ++b) a += part[static_cast<int64_t>(b) * kCo * kKp + e];
    mid[rg * kCo * kKp + e] = a;
}

// dw[co][kh][kw][c] (PyTorch [Cout, Cin, KH, KW] memory in channels_last = [co][kh][kw][c]) = the sum of
// the level-1 rows, in order (deterministic); f32 or bf16 output
__global__ __launch_bounds__(256) void stem3_wgrad_reduce_kernel(const float *__restrict__ mid, int rows,
                                                                 void *__restrict__ dw, int out_f32, int KH, int KW) {
    const int e = blockIdx.x * 256 + threadIdx.x;  // [co][kh][kw][c] element
    const int nout = kCo * KH * KW * 3;
    if (e >= nout) return;
    const int c = e % 3, t = e / 3, kw = t % KW, t2 = t / KW, kh = t2 % KH, co = t2 / KH;
    const int k = kh * 16 + kw * 4 + c;
    float a = 0.f;
    for (int rg = 0; rg < rows; ++rg) a += mid[(static_cast<int64_t>(rg) * kCo + co) * kKp + k];
    if (out_f32) static_cast<float *>(dw)[e] = a;
    else static_cast<uint16_t *>(dw)[e] = f32_to_bf16(a);
}

// w [co][kh][kw][c] bf16 (channels_last [32, 3, KH, KW]) -> wp [32][64] (k = kh*16 + kw*4 + c, zeros)
__global__ void stem3_pack_weight_kernel(const uint16_t *__restrict__ w, uint16_t *__restrict__ wp, int KH, int KW) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kCo * kKp) return;
    const int co = e / kKp, k = e % kKp, kh = k >> 4, kw = (k >> 2) & 3, c = k & 3;
    uint16_t v = 0;
    if (kh < KH && kw < KW && c < 3) v = w[((co * KH + kh) * KW + kw) * 3 + c];
    wp[e] = v;
}

S3Geo make_geo(int N, int H, int W, int KH, int KW, int stride, int ph, int pw) {
    if (KH < 1 || KH > 4 || KW < 1 || KW > 4 || stride < 1 || ph < 0 || pw < 0 || ph >= KH || pw >= KW)
        throw std::invalid_argument("stem3: window <= 4x4, stride >= 1, 0 <= padding < window");
    S3Geo g;
    g.N = N, g.H = H, g.W = W, g.KH = KH, g.KW = KW, g.stride = stride, g.ph = ph, g.pw = pw;
    g.OH = (H + 2 * ph - KH) / stride + 1;
    g.OW = (W + 2 * pw - KW) / stride + 1;
    if (g.OH < 1 || g.OW < 1) throw std::invalid_argument("stem3: empty output");
    const int64_t m = static_cast<int64_t>(N) * g.OH * g.OW;
    if (m >= (int64_t(1) << 31) || static_cast<int64_t>(N) * H * W >= (int64_t(1) << 31))
        throw std::invalid_argument("stem3: too many pixels");
    g.M = static_cast<int>(m);
    return g;
}

}  // namespace

int stem3_out(int h, int k, int stride, int pad) { return (h + 2 * pad - k) / stride + 1; }

void launch_stem3_pack_weight(const uint16_t *w, uint16_t *wp, int KH, int KW, hipStream_t s) {
    stem3_pack_weight_kernel<<<(kCo * kKp + 255) / 256, 256, 0, s>>>(w, wp, KH, KW);
}

void launch_stem3_forward(const void *x, bool x_f32, const uint16_t *wp, uint16_t *y, double *stats, int N, int H,
                          int W, int KH, int KW, int stride, int ph, int pw, hipStream_t s) {
    const S3Geo g = make_geo(N, H, W, KH, KW, stride, ph, pw);
    const int tiles = (g.M + 63) / 64;
    int grid = (tiles + 3) / 4;
    if (grid > 2048) grid = 2048;
    const uint4 *w4 = reinterpret_cast<const uint4 *>(wp);
    uint4 *y4 = reinterpret_cast<uint4 *>(y);
    if (x_f32) stem3_fwd_kernel<float><<<grid, 256, 0, s>>>(static_cast<const float *>(x), w4, y4, stats, g);
    else stem3_fwd_kernel<uint16_t><<<grid, 256, 0, s>>>(static_cast<const uint16_t *>(x), w4, y4, stats, g);
}

int stem3_wgrad_blocks(int N, int H, int W, int KH, int KW, int stride, int ph, int pw) {
    const S3Geo g = make_geo(N, H, W, KH, KW, stride, ph, pw);
    const int nblk = (g.M + 255) / 256;
    return nblk < 512 ? nblk : 512;  // two resident per CU (55 KB LDS each); one partial row each, then a 16-row fold
}

int64_t stem3_wgrad_workspace(int N, int H, int W, int KH, int KW, int stride, int ph, int pw) {
    const int blocks = stem3_wgrad_blocks(N, H, W, KH, KW, stride, ph, pw);
    return static_cast<int64_t>(blocks + (blocks + 15) / 16) * kCo * kKp;
}

void launch_stem3_wgrad(const uint16_t *dy, const void *x, bool x_f32, void *dw, bool out_f32, float *part, int N,
                        int H, int W, int KH, int KW, int stride, int ph, int pw, hipStream_t s) {
    const S3Geo g = make_geo(N, H, W, KH, KW, stride, ph, pw);
    const int blocks = stem3_wgrad_blocks(N, H, W, KH, KW, stride, ph, pw);
    const uint4 *d4 = reinterpret_cast<const uint4 *>(dy);
    if (x_f32) stem3_wgrad_kernel<float><<<blocks, 256, 0, s>>>(d4, static_cast<const float *>(x), part, g);
    else stem3_wgrad_kernel<uint16_t><<<blocks, 256, 0, s>>>(d4, static_cast<const uint16_t *>(x), part, g);
    const int rows = (blocks + 15) / 16;
    float *mid = part + static_cast<int64_t>(blocks) * kCo * kKp;
    stem3_wgrad_fold_kernel<<<dim3(kCo * kKp / 256, rows), 256, 0, s>>>(part, blocks, mid);
    const int nout = kCo * KH * KW * 3;
    stem3_wgrad_reduce_kernel<<<(nout + 255) / 256, 256, 0, s>>>(mid, rows, dw, out_f32 ? 1 : 0, KH, KW);
}

}  // namespace kfk
