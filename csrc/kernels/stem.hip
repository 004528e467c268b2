// ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels, NHWC bf16) on CDNA4
// matrix cores, for gfx950: forward with the following BN's batch statistics fused into the
// epilogue, and the weight gradient.  (The stem input is the image: no data gradient.)
//
// Why: MIOpen ran this layer at ~80 TF/s (370 us forward + 354 us weight gradient + a 97 us
// BN statistics pass per 256-image step, profiles/r12_*.md) because K = 3*7*7 = 147 fits no
// library tiling.  Here the 3 input channels are padded to 4 (one 8-byte load per pixel,
// ``stem_pad4``) and K is laid out (kh, kw, c) with kw padded to 8: one kh row of the
// 7x7 window is 8 pixels x 4 channels = 32 bf16 = exactly one K-step of
// v_mfma_f32_16x16x32_bf16, so the im2col is 7 K-steps of 8-byte pixel loads.  The padded
// kw = 7 / c = 3 weights are zero (``stem_pack_weight``).
//
// Forward: 256-pixel x 64-channel tiles (4 waves, 64x64 wave tiles); a tile's whole
// 7x8-pixel window is loaded into registers at once and staged into a double-buffered LDS
// image (64-byte rows, 16-byte chunks XOR-swizzled by row so ds_read_b128 is conflict-free);
// the packed weights sit in LDS (464-byte rows: conflict-free); the product is computed
// transposed so the epilogue stores 4-channel bf16 quads straight from the accumulators and
// reduces the per-channel sum / sum of squares with lane shuffles (f64 atomics into the BN's
// slotted workspace, as conv.hip).
// Weight gradient: split-K over pixels (64 pixels per K-step); operands read with the
// transposing ds_read_b64_tr_b16 as in conv_wgrad.hip (dy image 128-byte rows, im2col
// image 512-byte rows, 32-byte column groups XOR-swizzled), per-split f32 partial tiles
// summed, unpacked to [64][7][7][3] and rounded by a second kernel.
//
// Reference parity: none (the reference trains tf.keras ResNet-50 with stock TF kernels,
// benchmarks/system/benchmark_kungfu.py:96).
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kKH = 7;           // window rows (one K-step each)
constexpr int kKPad = 224;       // K = 7 kh x 8 kw x 4 c
constexpr int kBRow = 464;       // LDS bytes per packed weight row (448 + 16)
constexpr int kCout = 64;

struct StemGeo {
    int N, H, W, OH, OW, M;
    uint64_t m_hw, m_ow;  // floor division magics (see conv_wgrad.hip)
};

__device__ __forceinline__ int fdiv(int p, uint64_t m) {
    return static_cast<int>((static_cast<uint64_t>(static_cast<uint32_t>(p)) * m) >> 40);
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

// two f32 -> packed bf16 pair (round to nearest even): one v_cvt_pk_bf16_f32 on gfx950.  Shadows
// common.hpp's integer-rounding pack_bf16x2 inside this file: here (stem forward epilogue, the BNP dx)
// the instruction measured faster (r6t15: ResNet-50 20.24-20.27 vs 20.35-20.42 ms/step with attention /
// stem / stem3 on it), while in gemm.hip's epilogues it measured 6.5x slower (r6t14)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    const bf16x2 v = __builtin_convertvector(f32x2{a, b}, bf16x2);
    return __builtin_bit_cast(uint32_t, v);
}

__device__ __forceinline__ void unpack8(const uint4 &v, float (&f)[8]) {
    const uint32_t *u = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(u[k] << 16);
        f[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
    }
}

// x [P, 3] -> x4 [P, 4] (4th channel 0); two pixels per thread (12-byte aligned reads).
__global__ void stem_pad4_kernel(const uint32_t *__restrict__ x, uint4 *__restrict__ x4, int64_t npairs,
                                 const uint16_t *__restrict__ xtail, int64_t npix) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < npairs;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t a = x[3 * i], b = x[3 * i + 1], c = x[3 * i + 2];
        // a = (c0, c1) of p0, b = (c2 of p0, c0 of p1), c = (c1, c2) of p1
        x4[i] = make_uint4(a, b & 0xffffu, (b >> 16) | (c << 16), c >> 16);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (npix & 1)) {  // odd pixel count: last pixel
        const int64_t p = npix - 1;
        uint16_t *o = reinterpret_cast<uint16_t *>(x4) + 4 * p;
        o[0] = xtail[3 * p];
        o[1] = xtail[3 * p + 1];
        o[2] = xtail[3 * p + 2];
        o[3] = 0;
    }
}

// f32 input (the image before autocast): cast and pad in one pass, one pixel per thread.
__global__ void stem_pad4_f32_kernel(const float *__restrict__ x, uint2 *__restrict__ x4, int64_t npix) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < npix;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const uint32_t c0 = f32_to_bf16(x[3 * i]), c1 = f32_to_bf16(x[3 * i + 1]), c2 = f32_to_bf16(x[3 * i + 2]);
        x4[i] = make_uint2(c0 | (c1 << 16), c2);
    }
}

// w [64][7][7][3] (channels_last [64, 3, 7, 7]) -> wp [64][7][8][4], zero padded.
__global__ void stem_pack_weight_kernel(const uint16_t *__restrict__ w, uint16_t *__restrict__ wp) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kCout * kKPad; i += gridDim.x * blockDim.x) {
        const int co = i / kKPad, k = i - co * kKPad;
        const int kh = k >> 5, kw = (k >> 2) & 7, c = k & 3;
        wp[i] = (kw < 7 && c < 3) ? w[((co * 7 + kh) * 7 + kw) * 3 + c] : static_cast<uint16_t>(0);
    }
}

// ---------------------------------------------------------------------------------- forward
constexpr int kFwdBM = 256;
constexpr int kAStage = kFwdBM * 64;  // 16 KB

__device__ __forceinline__ int a_img_off(int row, int chunk) { return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4); }

// One 256-pixel x 64-channel tile per workgroup.  The MFMA computes the tile transposed
// (A = weights: rows = output channels; B = im2col: columns = pixels), so each lane's
// accumulator holds 4 consecutive channels of one pixel: stored as 8-byte bf16 quads
// straight from registers (no LDS round trip; L2 merges the quads of a 128-byte pixel row).
__global__ __launch_bounds__(256) void stem_fwd_kernel(const uint16_t *__restrict__ x4, const uint16_t *__restrict__ wp,
                                                       uint16_t *__restrict__ y, double *__restrict__ stats,
                                                       StemGeo g) {
    constexpr int BM = kFwdBM, BN = kCout, NT = 256;
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kAStage + kCout * kBRow];
    uint8_t *bimg = lds + 2 * kAStage;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
    const int mt = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
    const int m0 = mt * BM;

    // packed weights -> LDS (once)
    for (int q = tid; q < kCout * 28; q += NT) {
        const int co = q / 28, c = q - co * 28;
        *reinterpret_cast<uint4 *>(bimg + co * kBRow + c * 16) =
            *reinterpret_cast<const uint4 *>(wp + co * kKPad + c * 8);
    }

    // A staging: thread -> window column kw = tid & 7, rows (tid >> 3) + 32 i
    const int kw = tid & 7;
    int off[8], woff[8];
    uint32_t okm[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int r = (tid >> 3) + 32 * i;
        const int m = m0 + r;
        woff[i] = a_img_off(r, kw >> 1) + 8 * (kw & 1);
        off[i] = 0;
        okm[i] = 0;
        if (m < g.M) {
            const int n = fdiv(m, g.m_hw);
            const int rem = m - n * g.OH * g.OW;
            const int oh = fdiv(rem, g.m_ow);
            const int ow = rem - oh * g.OW;
            const int ih0 = oh * 2 - 3, iw = ow * 2 - 3 + kw;
            off[i] = ((n * g.H + ih0) * g.W + iw) * 4;
            if (iw >= 0 && iw < g.W) {
                uint32_t bits = 0;
#pragma unroll
                for (int kh = 0; kh < kKH; ++kh)
                    if (static_cast<unsigned>(ih0 + kh) < static_cast<unsigned>(g.H)) bits |= 1u << kh;
                okm[i] = bits;
            }
        }
    }
    // all 7 window rows' loads issued up front: the K loop is 7 short steps
    uint2 regs[kKH][8];
#pragma unroll
    for (int kh = 0; kh < kKH; ++kh)
#pragma unroll
        for (int i = 0; i < 8; ++i)
            regs[kh][i] = ((okm[i] >> kh) & 1u) ? *reinterpret_cast<const uint2 *>(x4 + (off[i] + kh * g.W * 4))
                                               : make_uint2(0u, 0u);

    f32x4 acc[4][4];  // [channel tile i][pixel tile j]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int kh = 0; kh < kKH; ++kh) {
        uint8_t *abase = lds + (kh & 1) * kAStage;
#pragma unroll
        for (int i = 0; i < 8; ++i) *reinterpret_cast<uint2 *>(abase + woff[i]) = regs[kh][i];
        __syncthreads();  // also orders this buffer's reuse: its previous readers passed the last barrier
        bf16x8 wf[4], xf[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = i * 16 + (lane & 15);
            wf[i] = *reinterpret_cast<const bf16x8 *>(bimg + co * kBRow + 16 * (kh * 4 + (lane >> 4)));
            const int m = wave * 64 + i * 16 + (lane & 15);
            xf[i] = *reinterpret_cast<const bf16x8 *>(abase + a_img_off(m, lane >> 4));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[i], xf[j], acc[i][j], 0, 0, 0);
    }

    // ---- epilogue: lane holds channels 16 i + 4 (lane >> 4) + r of pixel wave*64 + 16 j + (lane & 15)
    float s1[4][4], s2[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int m = m0 + wave * 64 + j * 16 + (lane & 15);
        if (m < g.M) {
            uint16_t *dst = y + static_cast<int64_t>(m) * BN + (lane >> 4) * 4;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                uint16_t h[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    h[r] = f32_to_bf16(acc[i][j][r]);
                    const float f = bf16_to_f32(h[r]);  // statistics of the stored (rounded) values
                    s1[i][r] += f;
                    s2[i][r] += f * f;
                }
                *reinterpret_cast<uint2 *>(dst + i * 16) =
                    make_uint2(h[0] | (static_cast<uint32_t>(h[1]) << 16), h[2] | (static_cast<uint32_t>(h[3]) << 16));
            }
        }
    }
    if (stats) {
        // sum over the 16 pixels of a lane group (lanes with equal lane >> 4), then over waves
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s1[i][r] += __shfl_xor(s1[i][r], o, 64);
                    s2[i][r] += __shfl_xor(s2[i][r], o, 64);
                }
        __syncthreads();  // the A buffers are free: reuse as the [wave][2][64] reduction scratch
        float *red = reinterpret_cast<float *>(lds);
        if ((lane & 15) == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = i * 16 + (lane >> 4) * 4 + r;
                    red[(wave * 2) * BN + co] = s1[i][r];
                    red[(wave * 2 + 1) * BN + co] = s2[i][r];
                }
        }
        __syncthreads();
        if (tid < 2 * BN) {
            const int which = tid / BN, co = tid % BN;
            double t = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) t += red[(w * 2 + which) * BN + co];
            atomicAdd(stats + (mt % kStatSlots) * 2 * BN + which * BN + co, t);
        }
    }
}

// Workgroup barrier for LDS hand-offs only: __syncthreads()'s fence also waits for every
// outstanding global load and store (vmcnt(0)), which would drain the input-row prefetch
// queue and the output stores at every row.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
}

// ------------------------------------------------------------- forward, row-based formulation
// One output row (n, oh) = 112 pixels x 64 channels reads 7 input rows (ih = 2 oh - 3 + kh);
// consecutive output rows share 5 of them.  Each workgroup walks a run of output rows keeping
// the input rows in a 16-slot LDS ring (2 new rows per output row, prefetched into registers
// during the previous row's MFMAs), so every input pixel is loaded once per workgroup instead
// of ~12 times (the 7x7 / stride-2 window overlap) as in the per-pixel im2col staging above.
// An input row sits in its slot with 3 zero pixels on the left: the 16-byte operand of
// (output pixel ow, window columns kw, kw + 1) then starts at pixel 2 ow + kw, 16-byte
// aligned for the even kw an MFMA fragment starts at.
constexpr int kRowPad = 3;
constexpr int kRowPx = 232;                 // 3 + 224 + 5 (covers 2 * 111 + 7 + 3)
constexpr int kRowBytes = kRowPx * 8;
constexpr int kRing = 16;

__global__ __launch_bounds__(512) void stem_fwd_rows_kernel(const uint16_t *__restrict__ x4,
                                                            const uint16_t *__restrict__ wp,
                                                            uint16_t *__restrict__ y, double *__restrict__ stats,
                                                            StemGeo g, int rows_per_wg) {
    constexpr int BN = kCout;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kCout * kBRow + kRing * kRowBytes];
    uint8_t *bimg = lds;
    uint8_t *ring = lds + kCout * kBRow;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int R = g.N * g.OH;
    const int r_begin = blockIdx.x * rows_per_wg;
    const int r_end = r_begin + rows_per_wg < R ? r_begin + rows_per_wg : R;

    for (int q = tid; q < kCout * 28; q += 512) {
        const int co = q / 28, c = q - co * 28;
        *reinterpret_cast<uint4 *>(bimg + co * kBRow + c * 16) =
            *reinterpret_cast<const uint4 *>(wp + co * kKPad + c * 8);
    }
    // row loader: thread t < kRowPx owns padded pixel t of a row (8 bytes)
    const int px = tid - kRowPad;
    const bool pxok = tid < kRowPx && px >= 0 && px < g.W;
    // Loads are unconditional (clamped to a valid pixel) and masked only when stored: a load
    // inside a branch makes the compiler drain the whole memory counter (vmcnt(0)) at the join,
    // which would serialise the prefetch queue below.
    const int pxc = px < 0 ? 0 : (px >= g.W ? g.W - 1 : px);
    auto row_value = [&](int n, int ih) -> uint2 {
        const int ihc = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih);
        return *reinterpret_cast<const uint2 *>(x4 + ((static_cast<int64_t>(n) * g.H + ihc) * g.W + pxc) * 4);
    };
    auto row_store = [&](int ih, uint2 v) {
        const bool ok = pxok && ih >= 0 && ih < g.H;
        if (!ok) v = make_uint2(0u, 0u);
        if (tid < kRowPx) *reinterpret_cast<uint2 *>(ring + ((ih + kRing) & (kRing - 1)) * kRowBytes + tid * 8) = v;
    };

    // stats: lane holds channels 16 i + 4 (lane >> 4) + r
    float s1[4][4], s2[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;

    // the packed weights as MFMA A fragments, resident in registers for the whole run; their
    // LDS image is then reused as the per-row output staging tile
    uint8_t *cimg = bimg;
    static_assert(128 * (kCout * 2 + 16) <= kCout * kBRow, "output row tile fits the weight image");
    lds_barrier();
    bf16x8 wf[kKH][4];
#pragma unroll
    for (int kh = 0; kh < kKH; ++kh)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            wf[kh][i] = *reinterpret_cast<const bf16x8 *>(bimg + (i * 16 + (lane & 15)) * kBRow +
                                                          16 * (kh * 4 + (lane >> 4)));

    int n = 0, oh = 0;
    if (r_begin < r_end) {
        n = r_begin / g.OH;
        oh = r_begin - n * g.OH;
    }
    // input-row queue: the two new rows of output row oh + d are loaded at row oh + d - 3
    // (three rows of MFMA work hide the load latency) and stored into the ring at row oh + d - 1
    // (slots rotate by renaming in a loop unrolled by 3: step(A, B, C), step(B, C, A), ...;
    // copying a register that a load is still filling would make the compiler wait for it)
    struct Q {
        uint2 a, b;
    };
    bool fresh = true;
    auto step = [&](int r, Q &qa, Q &qb, Q &qc) {
        if (fresh) {
#pragma unroll
            for (int kh = 0; kh < kKH; ++kh) row_store(2 * oh - 3 + kh, row_value(n, 2 * oh - 3 + kh));
            // queue: rows of output rows oh + 1, oh + 2 (same image)
            qa.a = row_value(n, 2 * oh + 4);
            qa.b = row_value(n, 2 * oh + 5);
            qb.a = row_value(n, 2 * oh + 6);
            qb.b = row_value(n, 2 * oh + 7);
            lds_barrier();
        }
        const bool next_same = r + 1 < r_end && oh + 1 < g.OH;
        // issue the loads for output row oh + 3
        // (beyond the run / image these are clamped loads that are never stored)
        qc.a = row_value(n, 2 * oh + 8);
        qc.b = row_value(n, 2 * oh + 9);
        // 8 waves: wave w owns output pixels [16 w, 16 w + 16) of the row, all 64 channels
        f32x4 acc[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int ow_t0 = wave * 16;
        const bool live = ow_t0 < g.OW;
        if (live) {
            // all 7 im2col fragments of the row first (one LDS latency), then the 28 MFMAs
            bf16x8 xf[kKH];
            int owr = ow_t0 + (lane & 15);
            owr = owr < g.OW ? owr : g.OW - 1;  // padding columns: any in-row data, never stored
#pragma unroll
            for (int kh = 0; kh < kKH; ++kh)
                xf[kh] = *reinterpret_cast<const bf16x8 *>(ring + ((2 * oh - 3 + kh + kRing) & (kRing - 1)) * kRowBytes +
                                                           16 * (owr + (lane >> 4)));
#pragma unroll
            for (int kh = 0; kh < kKH; ++kh)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kh][i], xf[kh], acc[i], 0, 0, 0);
        }
        // lane holds channels 16 i + 4 (lane >> 4) + [0, 4) of pixel ow: 8-byte quads into an
        // LDS [ow][64 ch] row image, then full 128-byte pixel rows out with 16-byte stores
        // (scattered 8-byte global stores cost 2x the whole kernel)
        constexpr int CROW = BN * 2 + 16;
        {
            const int ow = ow_t0 + (lane & 15);
            if (ow < g.OW) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    // v_cvt_pk_bf16_f32 (RNE, two values per instruction); statistics of the stored values
                    const uint32_t lo = pack_bf16x2(acc[i][0], acc[i][1]);
                    const uint32_t hi = pack_bf16x2(acc[i][2], acc[i][3]);
                    const float f0 = __uint_as_float(lo << 16), f1 = __uint_as_float(lo & 0xffff0000u);
                    const float f2 = __uint_as_float(hi << 16), f3 = __uint_as_float(hi & 0xffff0000u);
                    s1[i][0] += f0;
                    s1[i][1] += f1;
                    s1[i][2] += f2;
                    s1[i][3] += f3;
                    s2[i][0] += f0 * f0;
                    s2[i][1] += f1 * f1;
                    s2[i][2] += f2 * f2;
                    s2[i][3] += f3 * f3;
                    *reinterpret_cast<uint2 *>(cimg + ow * CROW + (i * 16 + (lane >> 4) * 4) * 2) = make_uint2(lo, hi);
                }
            }
        }
        lds_barrier();
        {
            uint4 *dst = reinterpret_cast<uint4 *>(y + (static_cast<int64_t>(n) * g.OH + oh) * g.OW * BN);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int v = tid + 512 * u;
                if (v < g.OW * 8) dst[v] = *reinterpret_cast<const uint4 *>(cimg + (v >> 3) * CROW + (v & 7) * 16);
            }
        }
        if (next_same) {  // rows 2 oh + 4, 2 oh + 5 (output row oh + 1): not in this row's window
            row_store(2 * oh + 4, qa.a);
            row_store(2 * oh + 5, qa.b);
        }
        lds_barrier();
        fresh = !next_same;
        if (++oh == g.OH) {
            oh = 0;
            ++n;
        }
    };
    Q q0, q1, q2;
    for (int r = r_begin; r < r_end; r += 3) {
        step(r, q0, q1, q2);
        if (r + 1 >= r_end) break;
        step(r + 1, q1, q2, q0);
        if (r + 2 >= r_end) break;
        step(r + 2, q2, q0, q1);
    }
    if (stats) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int o = 1; o < 16; o <<= 1) {
                    s1[i][q] += __shfl_xor(s1[i][q], o, 64);
                    s2[i][q] += __shfl_xor(s2[i][q], o, 64);
                }
        float *red = reinterpret_cast<float *>(ring);  // the last barrier passed: ring is free
        if ((lane & 15) == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int co = i * 16 + (lane >> 4) * 4 + q;
                    red[(wave * 2) * BN + co] = s1[i][q];
                    red[(wave * 2 + 1) * BN + co] = s2[i][q];
                }
        }
        lds_barrier();
        if (tid < 2 * BN) {
            const int which = tid / BN, co = tid % BN;
            double t = 0;
#pragma unroll
            for (int w = 0; w < 8; ++w) t += red[(w * 2 + which) * BN + co];
            atomicAdd(stats + (blockIdx.x % kStatSlots) * 2 * BN + which * BN + co, t);
        }
    }
}

// ------------------------------------------------------------------------- weight gradient
constexpr int kBK = 64;               // pixels per K-step
constexpr int kARow = 128;            // dy image: 64 channels
constexpr int kIRow = 512;            // im2col image: 256 k (224 used)
constexpr int kWStage = kBK * (kARow + kIRow);  // 40 KB

template <int ROW>
__device__ __forceinline__ int hswz(int row) {
    if constexpr (ROW == 128) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    else return (row & 3) | (((row >> 3) & 1) << 2);  // 256- and 512-byte rows: 8 groups per bank row
}

__device__ __forceinline__ bf16x8 tr_frag(const uint8_t *p0, const uint8_t *p1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

// grid = splits; tile = 64 co x 256 k (wave w: k in [64w, 64w + 64); wave 3 uses k < 224 only)
__global__ __launch_bounds__(256) void stem_wgrad_kernel(const uint16_t *__restrict__ dy,
                                                         const uint16_t *__restrict__ x4, float *__restrict__ part,
                                                         StemGeo g, int kps) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kWStage];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int split = blockIdx.x;
    const int p_begin = split * kps * kBK;
    int nsteps = (g.M - p_begin + kBK - 1) / kBK;
    if (nsteps > kps) nsteps = kps;

    // staging: dy rows (tid >> 2), 16-byte chunks 2 (tid & 3) + {0, 1};
    //          im2col: pixel (tid >> 2), window slots q = (tid & 3) + 4 i (kh = q / 8, kw = q % 8)
    const int spx = tid >> 2, ssub = tid & 3;
    struct Regs {
        uint4 d[2];
        uint2 im[14];
    };
    auto gload = [&](Regs &R, int ks) {
        const int p = p_begin + ks * kBK + spx;
        const bool ok = p < g.M;
#pragma unroll
        for (int u = 0; u < 2; ++u)
            R.d[u] = ok ? *reinterpret_cast<const uint4 *>(dy + static_cast<int64_t>(p) * kCout + (2 * ssub + u) * 8)
                         : make_uint4(0u, 0u, 0u, 0u);
        int n = 0, oh = 0, ow = 0;
        if (ok) {
            n = fdiv(p, g.m_hw);
            const int rem = p - n * g.OH * g.OW;
            oh = fdiv(rem, g.m_ow);
            ow = rem - oh * g.OW;
        }
        const int ih0 = oh * 2 - 3, iw0 = ow * 2 - 3;
        const int base = ((n * g.H + ih0) * g.W + iw0) * 4;
#pragma unroll
        for (int i = 0; i < 14; ++i) {
            const int q = ssub + 4 * i, kh = q >> 3, kw = q & 7;
            const bool in = ok && static_cast<unsigned>(ih0 + kh) < static_cast<unsigned>(g.H) &&
                            static_cast<unsigned>(iw0 + kw) < static_cast<unsigned>(g.W);
            R.im[i] = in ? *reinterpret_cast<const uint2 *>(x4 + (base + (kh * g.W + kw) * 4)) : make_uint2(0u, 0u);
        }
    };
    auto swrite = [&](const Regs &R, int buf) {
        uint8_t *ab = lds + buf * kWStage;
        uint8_t *ib = ab + kBK * kARow;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int c = 2 * ssub + u;  // 16-byte chunk of the 128-byte row
            const int grp = (c >> 1) ^ hswz<kARow>(spx);
            *reinterpret_cast<uint4 *>(ab + spx * kARow + grp * 32 + (c & 1) * 16) = R.d[u];
        }
#pragma unroll
        for (int i = 0; i < 14; ++i) {
            const int q = ssub + 4 * i, kh = q >> 3, kw = q & 7;
            const int byte = kh * 64 + kw * 8;  // k = kh*32 + kw*4 (+c) -> 2 bytes per k
            const int grp = (byte >> 5) ^ hswz<kIRow>(spx);
            *reinterpret_cast<uint2 *>(ib + spx * kIRow + grp * 32 + (byte & 31)) = R.im[i];
        }
    };

    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    const int row0 = 8 * fg + fq;
    int aoff[4], boff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        aoff[i] = row0 * kARow + 32 * (i ^ hswz<kARow>(row0)) + 8 * fp;
        boff[i] = row0 * kIRow + 32 * ((wave * 4 + i) ^ hswz<kIRow>(row0)) + 8 * fp;
    }
    const int jmax = wave == 3 ? 2 : 4;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const uint8_t *ab = lds + buf * kWStage;
        const uint8_t *ib = ab + kBK * kARow;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            bf16x8 af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                af[i] = tr_frag(ab + aoff[i] + 32 * s * kARow, ab + aoff[i] + (32 * s + 4) * kARow);
                bfr[i] = tr_frag(ib + boff[i] + 32 * s * kIRow, ib + boff[i] + (32 * s + 4) * kIRow);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (j < jmax) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
    };

    Regs R;
    if (nsteps > 0) {
        gload(R, 0);
        swrite(R, 0);
    }
    __syncthreads();
    for (int ks = 0; ks < nsteps; ++ks) {
        if (ks + 1 < nsteps) gload(R, ks + 1);
        compute(ks & 1);
        if (ks + 1 < nsteps) swrite(R, (ks + 1) & 1);
        __syncthreads();
    }
    // partial tile: part[split][co][k], k < 224
    float *dst = part + static_cast<int64_t>(split) * kCout * kKPad;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (j < jmax)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = i * 16 + (lane >> 4) * 4 + r;
                    const int k = wave * 64 + j * 16 + (lane & 15);
                    dst[co * kKPad + k] = acc[i][j][r];
                }
}

// dw[co][kh][kw][c] (c < 3, kw < 7) = sum_s part[s][co][kh*32 + kw*4 + c]; block = 16 outputs x 16 split groups
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float *__restrict__ part, int splits,
                                                                uint16_t *__restrict__ dw) {
    __shared__ float red[256];
    const int t = threadIdx.x, o = t & 15, sg = t >> 4;
    const int e = blockIdx.x * 16 + o;  // output element (co, kh, kw, c) in dw order
    constexpr int NOUT = kCout * 7 * 7 * 3;
    float s = 0.f;
    int k = 0, co = 0;
    if (e < NOUT) {
        co = e / 147;
        const int r = e - co * 147, kh = r / 21, r2 = r - kh * 21, kw = r2 / 3, c = r2 - kw * 3;
        k = kh * 32 + kw * 4 + c;
        for (int sp = sg; sp < splits; sp += 16) s += part[(static_cast<int64_t>(sp) * kCout + co) * kKPad + k];
    }
    red[t] = s;
    __syncthreads();
    if (sg == 0 && e < NOUT) {
        for (int q = 1; q < 16; ++q) s += red[o + 16 * q];
        dw[e] = f32_to_bf16(s);
    }
}

// ------------------------------------------------------- weight gradient, row-based formulation
// dW[co][kh*32 + kw*4 + c] = sum over output rows (n, oh) and pixels ow of
//     dy[n, oh, ow, co] * x4[n, 2 oh - 3 + kh, 2 ow - 3 + kw, c]
// Per output row: GEMM M = 64 co, N = 32 per kh, K = 112 ow (padded to 128).  7 waves, wave =
// kh.  A = dy^T read with ds_read_b64_tr_b16 from the dy row image ([ow][64 co], 128-byte rows,
// rows 112..127 zero); B = the stride-2 window of input row 2 oh - 3 + kh, read with the same
// transposing read straight from the input-row ring (lane (q, p) of a 16-lane group supplies
// pixel 2 (ow0 + q) + kw0 + p: 4 channels = 8 bytes) -- no im2col image at all.
constexpr int kDyRow = 128 * kARow;  // dy row image: 128 ow x 128 B

// BNP (round 6): the dy operand is not read but FORMED while staging -- the gradient of the stem's
// conv output through BN(batch stats) + ReLU + MaxPool(3, 2, 1):
//     g  = sum of dyp over the (<= 2x2) pooled windows whose argmax is this element  (the pool gather)
//     dz = g if y * fscale + fshift > 0 else 0                                         (the ReLU gate)
//     dx = k1 * dz + k2 * y + k3                      (BN backward, k = bn_bwd_finalize's coefficients)
// with y the conv output (read where the plain kernel reads dy: same layout, same bytes).  The
// same f32 expressions as bn.hip's bn_bwd_apply_kernel<PoolGrad>, so dx rounds to the same bf16 and
// the weight gradient equals the layered path's; but the 411 MB BN input gradient of a 256-image
// batch is never written nor read back (the layered pass was 256 us + a 167 us weight gradient).
// The pooled gradient and argmax rows are staged through a 2-slot LDS ring (pooled row p in slot
// p & 1; conv row h needs rows h >> 1 and (h + 1) >> 1) and gathered from there: each pooled byte
// is read from HBM once.  (Gathering the <= 4 candidates per pixel from global memory instead --
// 8 dependent loads per 16-byte chunk at one workgroup per CU -- ran the kernel at 418 us.)
struct StemBnp {
    const uint4 *dyp;    // pooled gradient [N, PH, PW, 64]
    const uint2 *arg;    // window argmax bytes [N, PH, PW, 64]
    const float *fcoef;  // forward BN [scale(64); shift(64)]
    const float *bcoef;  // backward BN [k1(64); k2(64); k3(64)]
    int PH, PW;
};
constexpr int kPoolD = 64 * 128;               // slot: dyp row [PW <= 64][64] bf16 ...
constexpr int kPoolSlot = kPoolD + 64 * 64;    // ... + argmax row [PW][64] bytes

__device__ __forceinline__ void unpack8f(const uint4 &v, float (&f)[8]) {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f[2 * i] = __uint_as_float(u[i] << 16);
        f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
}

// 16-bit lane masks of the argmax bytes equal to kk: for the 4 bytes of a (channels 4 q .. 4 q + 3),
// lo = [ch 0 | ch 1] and hi = [ch 2 | ch 3] as 0xffff / 0 halves (SWAR zero-byte test of a ^ kk, then
// v_perm_b32's sign-replicating selectors 8..11 spread each byte's flag; ~8 ops for 4 channels against
// 8 compares + 8 selects)
__device__ __forceinline__ void argmax_masks(uint32_t a, uint32_t kk, uint32_t &lo, uint32_t &hi) {
    const uint32_t x = a ^ (kk * 0x01010101u);
    const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);  // 0x80 in each zero byte
    const uint32_t zs = z << 8;  // flags of bytes 0 / 2 at bits 15 / 31
    // perm(src0 = z, src1 = zs): sel 8 = zs bit 15 (byte 0), 9 = zs bit 31 (byte 2), 10 = z bit 15 (byte 1),
    // 11 = z bit 31 (byte 3)
    lo = __builtin_amdgcn_perm(z, zs, 0x0a0a0808u);
    hi = __builtin_amdgcn_perm(z, zs, 0x0b0b0909u);
}

// g = the pooled gradient gathered back to conv-output pixel (h, w), 8 channels cv * 8.., from the LDS
// ring: the windows (oh, ow) with oh in {h >> 1, (h + 1) >> 1} and ow in {w >> 1, (w + 1) >> 1}, in
// bn.hip PoolGrad's order, each adding its dyp where its argmax byte names (h, w).  PoolGrad adds a 0
// for a window that cannot cover (h, w); here such windows are skipped -- at compile time for the
// column (ODDW: w is odd, so two columns) and by the wave-uniform row parity (hodd) -- which gives the
// same sum (adding +0 to a sum that starts at +0 changes nothing): 2.25 windows per pixel, not 4.
// The window offset of (h, w) in window (oh, ow), kk = (h + 1 - 2 oh) * 3 + (w + 1 - 2 ow), is a
// constant per (row parity, window row, column parity, window column).
template <bool ODDW>
__device__ __forceinline__ void pool_grad8(const uint8_t *pool, int PH, int PW, int h, bool hodd, int w, int cv,
                                           float (&g)[8]) {
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = 0.f;
    const int oh_lo = h >> 1, ow_lo = w >> 1;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const int oh = oh_lo + rr;
        if (rr == 1 && !(hodd && oh < PH)) break;  // wave-uniform
        const uint8_t *slot = pool + (oh & 1) * kPoolSlot;
        const uint32_t krow = hodd ? (rr ? 0u : 6u) : 3u;  // 3 (h + 1 - 2 oh)
#pragma unroll
        for (int cc = 0; cc < (ODDW ? 2 : 1); ++cc) {
            int ow = ow_lo + cc;
            // the last odd column of an even-width map has no right window: read window ow_lo, never match
            const bool ok = cc == 0 || ow < PW;
            const uint32_t kk = ok ? krow + (ODDW ? (cc ? 0u : 2u) : 1u) : 0xffu;
            ow = ok ? ow : ow_lo;
            const int e = ow * 8 + cv;
            const uint4 dv = *reinterpret_cast<const uint4 *>(slot + e * 16);
            const uint2 am = *reinterpret_cast<const uint2 *>(slot + kPoolD + e * 8);
            uint32_t m0, m1, m2, m3;
            argmax_masks(am.x, kk, m0, m1);
            argmax_masks(am.y, kk, m2, m3);
            float d[8];
            unpack8f(make_uint4(dv.x & m0, dv.y & m1, dv.z & m2, dv.w & m3), d);
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] += d[k];
        }
    }
}

// the forward / backward BN coefficients [fs; fh; k1; k2; k3] x 64 channels, staged once into LDS
// (register-resident they cost 40 VGPRs across the MFMA loop and pushed the kernel into spills)
constexpr int kBnpCoef = 5 * kCout;

// dx (8 channels cv * 8.., bf16) of one conv-output pixel from its y vector and gathered pooled gradient;
// kc = the LDS coefficient table
__device__ __forceinline__ uint4 bnp_dx(const float *kc, int cv, const uint4 &yv, float (&g)[8]) {
    float xv[8];
    unpack8f(yv, xv);
    float o[8];
    // (scalar reads of the table, not a [5][8] array: the array was promoted to LDS)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const float *t = kc + cv * 8 + k;
        g[k] = (xv[k] * t[0] + t[kCout]) > 0.f ? g[k] : 0.f;
        o[k] = t[2 * kCout] * g[k] + t[3 * kCout] * xv[k] + t[4 * kCout];
    }
    return make_uint4(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3]), pack_bf16x2(o[4], o[5]),
                      pack_bf16x2(o[6], o[7]));
}

template <bool BNP>
__global__ __launch_bounds__(448) void stem_wgrad_rows_kernel(const uint16_t *__restrict__ dy,
                                                              const uint16_t *__restrict__ x4,
                                                              float *__restrict__ part, StemGeo g, int rows_per_wg,
                                                              StemBnp bp) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kRing * kRowBytes + 2 * kDyRow + (BNP ? kBnpCoef * 4 + 2 * kPoolSlot : 0)];
    uint8_t *ring = lds;
    uint8_t *dyimg = lds + kRing * kRowBytes;
    float *kc = reinterpret_cast<float *>(lds + kRing * kRowBytes + 2 * kDyRow);  // BNP only
    uint8_t *pool = lds + kRing * kRowBytes + 2 * kDyRow + kBnpCoef * 4;       // BNP only: the pooled-row ring
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;  // wave = kh
    const int R = g.N * g.OH;
    const int r_begin = blockIdx.x * rows_per_wg;
    const int r_end = r_begin + rows_per_wg < R ? r_begin + rows_per_wg : R;

    // zero both dy images once (rows >= OW stay zero: the K padding)
    for (int v = tid; v < 2 * kDyRow / 16; v += 448)
        reinterpret_cast<uint4 *>(dyimg)[v] = make_uint4(0u, 0u, 0u, 0u);
    if constexpr (BNP) {
        if (tid < kBnpCoef) kc[tid] = tid < 2 * kCout ? bp.fcoef[tid] : bp.bcoef[tid - 2 * kCout];
    }
    lds_barrier();  // the zero fill (and table) before any dy row lands in the images

    // input-row loader (as the forward): thread t < kRowPx owns padded pixel t
    const int px = tid - kRowPad;
    const bool pxok = tid < kRowPx && px >= 0 && px < g.W;
    const int pxc = px < 0 ? 0 : (px >= g.W ? g.W - 1 : px);
    auto row_value = [&](int n, int ih) -> uint2 {
        const int ihc = ih < 0 ? 0 : (ih >= g.H ? g.H - 1 : ih);
        return *reinterpret_cast<const uint2 *>(x4 + ((static_cast<int64_t>(n) * g.H + ihc) * g.W + pxc) * 4);
    };
    auto row_store = [&](int ih, uint2 v) {
        const bool ok = pxok && ih >= 0 && ih < g.H;
        if (!ok) v = make_uint2(0u, 0u);
        if (tid < kRowPx) *reinterpret_cast<uint2 *>(ring + ((ih + kRing) & (kRing - 1)) * kRowBytes + tid * 8) = v;
    };
    // dy row loader: two of the OW x 8 16-byte chunks (ow, channel group c) per thread -- chunks tid and
    // tid + 448; BNP: (2 j, c) and (2 j + 1, c) for j = tid >> 3, c = tid & 7 (an even and an odd column:
    // the pool gather is specialised by column parity; OW <= 112).  Two named registers, not a [2] array:
    // with the BNP staging below the arrays stayed in scratch.
    const int cv0 = BNP ? (tid >> 3) * 16 + (tid & 7) : tid, cv1 = BNP ? cv0 + 8 : tid + 448;
    const int dv0 = cv0 < g.OW * 8 ? cv0 : g.OW * 8 - 1;  // clamped (masked at the store)
    const int dv1 = cv1 < g.OW * 8 ? cv1 : g.OW * 8 - 1;
    auto dy_load = [&](int r, uint4 &d0, uint4 &d1) {
        const uint4 *src = reinterpret_cast<const uint4 *>(dy + static_cast<int64_t>(r) * g.OW * kCout);
        d0 = src[dv0];
        d1 = src[dv1];
    };
    // BNP: pooled row p of image n (PW x 8 16-byte chunks of dyp, 8-byte chunks of argmax: chunk v = tid +
    // 448 u) -> registers -> its LDS slot p & 1
    struct PRow {  // native vectors: HIP's uint4 struct copies were left in scratch across the step
        u32x4 d0, d1;
        u32x2 a0, a1;
    };
    const u32x4 *dyp4 = reinterpret_cast<const u32x4 *>(bp.dyp);
    const u32x2 *arg2 = reinterpret_cast<const u32x2 *>(bp.arg);
    const int pv1 = tid + 448 < bp.PW * 8 ? tid + 448 : bp.PW * 8 - 1;  // chunk tid + 448, clamped
    auto prow_load = [&](int nn, int p, PRow &pr) {
        const int64_t base = (static_cast<int64_t>(nn) * bp.PH + p) * bp.PW * 8;
        const int v0 = tid < bp.PW * 8 ? tid : bp.PW * 8 - 1;
        pr.d0 = dyp4[base + v0];
        pr.a0 = arg2[base + v0];
        pr.d1 = dyp4[base + pv1];
        pr.a1 = arg2[base + pv1];
    };
    auto prow_store = [&](int p, const PRow &pr) {
        uint8_t *slot = pool + (p & 1) * kPoolSlot;
        if (tid < bp.PW * 8) {
            *reinterpret_cast<u32x4 *>(slot + tid * 16) = pr.d0;
            *reinterpret_cast<u32x2 *>(slot + kPoolD + tid * 8) = pr.a0;
        }
        if (tid + 448 < bp.PW * 8) {
            *reinterpret_cast<u32x4 *>(slot + (tid + 448) * 16) = pr.d1;
            *reinterpret_cast<u32x2 *>(slot + kPoolD + (tid + 448) * 8) = pr.a1;
        }
    };
    // stage dy row hh (conv row hh of the current image; BNP: formed from y = d and the pooled ring)
    auto dy_put = [&](int buf, int v, const uint4 &val) {
        const int ow = v >> 3, c = v & 7;
        *reinterpret_cast<uint4 *>(dyimg + buf * kDyRow + ow * kARow + ((c >> 1) ^ hswz<kARow>(ow)) * 32 + (c & 1) * 16) =
            val;
    };
    auto dy_store = [&](int buf, const uint4 &d0, const uint4 &d1, int hh) {
        if constexpr (BNP) {
            const bool hodd = hh & 1;
            const int c = tid & 7, ow0 = cv0 >> 3;
            if (cv0 < g.OW * 8) {
                float gg[8];
                pool_grad8<false>(pool, bp.PH, bp.PW, hh, hodd, ow0, c, gg);
                dy_put(buf, cv0, bnp_dx(kc, c, d0, gg));
            }
            if (cv1 < g.OW * 8) {
                float gg[8];
                pool_grad8<true>(pool, bp.PH, bp.PW, hh, hodd, ow0 + 1, c, gg);
                dy_put(buf, cv1, bnp_dx(kc, c, d1, gg));
            }
        } else {
            if (cv0 < g.OW * 8) dy_put(buf, cv0, d0);
            if (cv1 < g.OW * 8) dy_put(buf, cv1, d1);
        }
    };

    // fragment addressing (transposing reads): lane = 16 fg + 4 fq + fp
    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    const int row0 = 8 * fg + fq;
    int aoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = row0 * kARow + 32 * (i ^ hswz<kARow>(row0)) + 8 * fp;

    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};

    int n = 0, oh = 0;
    if (r_begin < r_end) {
        n = r_begin / g.OH;
        oh = r_begin - n * g.OH;
    }
    // Prefetch queue, 3 output rows deep: slot A holds output row r + 1's two new input rows and
    // dy row (stored into the ring / the other dy image at the end of row r), B row r + 2, and
    // row r + 3's loads are issued into C.  The loop is unrolled by 3 and rotates the slots by
    // renaming (step(A, B, C), step(B, C, A), step(C, A, B)): copying a register that a load is
    // still filling would make the compiler wait for that load.
    struct Q {
        uint2 a, b;
        uint4 d0, d1;
    };
    auto rclamp = [&](int rr) { return rr < R ? rr : R - 1; };
    bool fresh = true;
    int buf = 0;
    auto step = [&](int r, Q &qa, Q &qb, Q &qc) {
        if (fresh) {
            uint4 dc0, dc1;
            if constexpr (BNP) {
                // pooled rows oh >> 1 and the next: those of conv rows oh and oh + 1 (later ones are
                // loaded one step ahead, below)
                const int p0 = oh >> 1;
                PRow a, b;
                prow_load(n, p0, a);
                if (p0 + 1 < bp.PH) prow_load(n, p0 + 1, b);
                prow_store(p0, a);
                if (p0 + 1 < bp.PH) prow_store(p0 + 1, b);
                lds_barrier();
            }
            dy_load(r, dc0, dc1);
            dy_load(rclamp(r + 1), qa.d0, qa.d1);
            dy_load(rclamp(r + 2), qb.d0, qb.d1);
#pragma unroll
            for (int kh = 0; kh < kKH; ++kh) row_store(2 * oh - 3 + kh, row_value(n, 2 * oh - 3 + kh));
            qa.a = row_value(n, 2 * oh + 4);
            qa.b = row_value(n, 2 * oh + 5);
            qb.a = row_value(n, 2 * oh + 6);
            qb.b = row_value(n, 2 * oh + 7);
            dy_store(buf, dc0, dc1, oh);
            lds_barrier();
        }
        const bool next_same = r + 1 < r_end && oh + 1 < g.OH;
        // BNP: at an odd conv row, pooled row (oh + 3) / 2 -- first needed by conv row oh + 2 -- into the
        // slot of row (oh - 1) / 2, whose last reader (conv row oh) is staged.  Issued first: the wait for
        // it at this step's end leaves the later row prefetches in flight
        PRow pn;
        const int pnext = (oh + 3) >> 1;
        const bool pload = BNP && (oh & 1) && next_same && pnext < bp.PH;
        if constexpr (BNP) {
            if (pload) prow_load(n, pnext, pn);
            __builtin_amdgcn_sched_barrier(0);
        }
        qc.a = row_value(n, 2 * oh + 8);  // the new input rows of output row oh + 3
        qc.b = row_value(n, 2 * oh + 9);
        dy_load(rclamp(r + 3), qc.d0, qc.d1);

        if (wave < kKH) {
            const int kh = wave;
            const uint8_t *rowp = ring + ((2 * oh - 3 + kh + kRing) & (kRing - 1)) * kRowBytes;
            const uint8_t *ab = dyimg + buf * kDyRow;
#pragma unroll
            for (int s = 0; s < 4; ++s) {  // 32 output pixels per substep
                bf16x8 af[4], bfr[2];
#pragma unroll
                for (int i = 0; i < 4; ++i) af[i] = tr_frag(ab + aoff[i] + 32 * s * kARow, ab + aoff[i] + (32 * s + 4) * kARow);
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    // rows q: ow = 32 s + 8 fg + fq (+4); cols 4 fp: kw = 4 j + fp, channels 0..3
                    int ow0 = 32 * s + 8 * fg + fq, ow1 = ow0 + 4;
                    ow0 = ow0 < g.OW ? ow0 : g.OW - 1;  // K padding: dy rows are zero there
                    ow1 = ow1 < g.OW ? ow1 : g.OW - 1;
                    bfr[j] = tr_frag(rowp + (2 * ow0 + 4 * j + fp) * 8, rowp + (2 * ow1 + 4 * j + fp) * 8);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
        if (next_same) {  // rows of output row oh + 1 and its dy row, into the free slots / buffer
            row_store(2 * oh + 4, qa.a);
            row_store(2 * oh + 5, qa.b);
            if constexpr (BNP) {
                if (pload) prow_store(pnext, pn);
            }
            dy_store(buf ^ 1, qa.d0, qa.d1, oh + 1);
        }
        lds_barrier();
        buf ^= 1;
        fresh = !next_same;
        if (++oh == g.OH) {
            oh = 0;
            ++n;
        }
    };
    Q q0, q1, q2;
    for (int r = r_begin; r < r_end; r += 3) {
        step(r, q0, q1, q2);
        if (r + 1 >= r_end) break;
        step(r + 1, q1, q2, q0);
        if (r + 2 >= r_end) break;
        step(r + 2, q2, q0, q1);
    }
    // partial tile of this workgroup: part[blockIdx][co][k < 224]
    if (wave < kKH) {
        float *dst = part + static_cast<int64_t>(blockIdx.x) * kCout * kKPad;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int co = i * 16 + (lane >> 4) * 4 + q;
                    dst[co * kKPad + wave * 32 + j * 16 + (lane & 15)] = acc[i][j][q];
                }
    }
}

uint64_t magic40(int d) { return (uint64_t(1) << 40) / static_cast<uint64_t>(d) + 1; }

StemGeo make_geo(int N, int H, int W) {
    StemGeo g;
    g.N = N, g.H = H, g.W = W;
    g.OH = (H + 6 - 7) / 2 + 1;
    g.OW = (W + 6 - 7) / 2 + 1;
    g.M = N * g.OH * g.OW;
    g.m_hw = magic40(g.OH * g.OW);
    g.m_ow = magic40(g.OW);
    return g;
}

void check_geo(const StemGeo &g) {
    if (g.M <= 0 || static_cast<int64_t>(g.M) * g.OH * g.OW >= (int64_t(1) << 40) ||
        static_cast<int64_t>(g.N) * g.H * g.W * 4 >= (int64_t(1) << 31))
        throw std::invalid_argument("stem: shape out of range");
}

}  // namespace

void launch_stem_pad4(const uint16_t *x, uint16_t *x4, int64_t npix, hipStream_t s) {
    const int64_t npairs = npix / 2;
    int64_t grid = (npairs + 255) / 256;
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    stem_pad4_kernel<<<static_cast<int>(grid), 256, 0, s>>>(reinterpret_cast<const uint32_t *>(x),
                                                            reinterpret_cast<uint4 *>(x4), npairs, x, npix);
}

void launch_stem_pad4_f32(const float *x, uint16_t *x4, int64_t npix, hipStream_t s) {
    int64_t grid = (npix + 255) / 256;
    if (grid > 8192) grid = 8192;
    if (grid < 1) grid = 1;
    stem_pad4_f32_kernel<<<static_cast<int>(grid), 256, 0, s>>>(x, reinterpret_cast<uint2 *>(x4), npix);
}

void launch_stem_pack_weight(const uint16_t *w, uint16_t *wp, hipStream_t s) {
    stem_pack_weight_kernel<<<(kCout * kKPad + 255) / 256, 256, 0, s>>>(w, wp);
}

int stem_out(int h) { return (h + 6 - 7) / 2 + 1; }

void launch_stem_forward(const uint16_t *x4, const uint16_t *wp, uint16_t *y, double *stats, int N, int H, int W,
                         hipStream_t s) {
    const StemGeo g = make_geo(N, H, W);
    check_geo(g);
    if (g.W <= kRowPx - 8 && g.OW <= 128) {
        // row-based kernel: one 8-wave workgroup per CU (2 waves / SIMD), each a run of output
        // rows (a whole 112-row image at batch 256)
        const int R = g.N * g.OH;
        int grid = R < 256 ? R : 256;
        const int rpw = (R + grid - 1) / grid;
        grid = (R + rpw - 1) / rpw;
        stem_fwd_rows_kernel<<<grid, 512, 0, s>>>(x4, wp, y, stats, g, rpw);
        return;
    }
    const int grid = (g.M + kFwdBM - 1) / kFwdBM;
    stem_fwd_kernel<<<grid, 256, 0, s>>>(x4, wp, y, stats, g);
}

int64_t stem_wgrad_workspace(int N, int H, int W, int splits) {
    (void)N, (void)H, (void)W;
    return static_cast<int64_t>(splits) * kCout * kKPad;
}

int stem_wgrad_splits(int N, int H, int W) {
    const StemGeo g = make_geo(N, H, W);
    const int ksteps = (g.M + kBK - 1) / kBK;
    int splits = 256;  // the row-based kernel: one workgroup per CU (tools/bench_stem.py)
    if (splits > ksteps) splits = ksteps;
    return splits < 1 ? 1 : splits;
}

bool stem_wgrad_bnp_supported(int N, int H, int W) {
    const StemGeo g = make_geo(N, H, W);
    return g.W <= kRowPx - 8 && g.OW <= 112;  // one even and one odd column per thread
}

void launch_stem_wgrad_bnp(const uint16_t *y, const uint16_t *x4, uint16_t *dw, float *part, int N, int H, int W,
                           int splits, const uint16_t *dyp, const uint8_t *arg, const float *fcoef,
                           const float *bcoef, hipStream_t s) {
    const StemGeo g = make_geo(N, H, W);
    check_geo(g);
    if (!(g.W <= kRowPx - 8 && g.OW <= 112)) throw std::invalid_argument("stem_wgrad_bnp: image too wide for the row kernel");
    const int R = g.N * g.OH;
    if (splits < 1) splits = 1;
    if (splits > R) splits = R;
    const int rpw = (R + splits - 1) / splits;
    splits = (R + rpw - 1) / rpw;
    StemBnp bp{reinterpret_cast<const uint4 *>(dyp), reinterpret_cast<const uint2 *>(arg), fcoef, bcoef,
               (g.OH + 2 - 3) / 2 + 1, (g.OW + 2 - 3) / 2 + 1};
    stem_wgrad_rows_kernel<true><<<splits, 448, 0, s>>>(y, x4, part, g, rpw, bp);
    stem_wgrad_reduce_kernel<<<(kCout * 147 + 15) / 16, 256, 0, s>>>(part, splits, dw);
}

void launch_stem_wgrad(const uint16_t *dy, const uint16_t *x4, uint16_t *dw, float *part, int N, int H, int W,
                       int splits, hipStream_t s) {
    const StemGeo g = make_geo(N, H, W);
    check_geo(g);
    if (g.W <= kRowPx - 8 && g.OW <= 128) {
        // row-based kernel: splits = workgroups, each a run of output rows
        const int R = g.N * g.OH;
        if (splits < 1) splits = 1;
        if (splits > R) splits = R;
        const int rpw = (R + splits - 1) / splits;
        splits = (R + rpw - 1) / rpw;
        stem_wgrad_rows_kernel<false><<<splits, 448, 0, s>>>(dy, x4, part, g, rpw, StemBnp{});
        stem_wgrad_reduce_kernel<<<(kCout * 147 + 15) / 16, 256, 0, s>>>(part, splits, dw);
        return;
    }
    const int ksteps = (g.M + kBK - 1) / kBK;
    if (splits < 1) splits = 1;
    if (splits > ksteps) splits = ksteps;
    const int kps = (ksteps + splits - 1) / splits;
    splits = (ksteps + kps - 1) / kps;  // no empty split
    stem_wgrad_kernel<<<splits, 256, 0, s>>>(dy, x4, part, g, kps);
    stem_wgrad_reduce_kernel<<<(kCout * 147 + 15) / 16, 256, 0, s>>>(part, splits, dw);
}

}  // namespace kfk
