// Weight gradient of the 1x1 / 3x3 NHWC bf16 convolutions (stride 1 or 2) on CDNA4
// matrix cores, for gfx950: a split-K GEMM over output pixels.
//
//   dw[co, kh, kw, ci] = sum_p dy[p, co] * x[n, oh*s + kh - pad, ow*s + kw - pad, ci]
//   GEMM: M = Cout, N = Cin (one tap per tile), K = P = N*OH*OW output pixels
//
// Why: the weight gradients were the last convolution pass on MIOpen (5.4 ms of a 25 ms
// ResNet-50 step plus 0.6 ms of its split-K zero-fills and casts, profiles/README.md).
// Both operands carry the reduction index (the pixel) as their ROW and the GEMM index
// (channel) contiguous, the "NT" layout: tiles are staged global->LDS unchanged
// (16-byte global_load_lds, rows of BM or BN channels) and every MFMA operand is read
// with the gfx950 transposing LDS read ds_read_b64_tr_b16, which hands each lane 4
// pixels of one channel -- no register/ds_write transpose pass.
//
// LDS image: rows of 128 or 256 bytes (64 / 128 channels), 32-byte column groups
// XOR-swizzled by the row (h(row) below) so the 8 rows one 32-lane half of a
// transposing read touches (two 4-row blocks 8 rows apart) land on 8 distinct
// 32-byte bank groups: conflict-free.  The swizzle is applied on the staging source
// address (global_load_lds writes fixed LDS offsets) and on the read address.
//
// Split-K: P is 12.5 K .. 800 K pixels while M x N is at most 2048 x 512, so each
// workgroup reduces a contiguous pixel range; partial f32 tiles go to a workspace in
// the accumulator's native register order (coalesced 16-byte stores) and a second
// kernel sums the splits, converts and scatters to [Cout][KS*KS][Cin] (deterministic).
// Accumulating into an f32 destination (e.g. a flat f32 gradient slot) the splits add
// their tiles with f32 atomics instead: no workspace, no second pass.  Workgroups of one
// split are launched together (same pixel rows in L2) and remapped XCD-contiguously.
//
// Reference parity: the reference has no kernels of its own; it trains
// tf.keras.applications ResNet-50 with TF's stock convolutions
// (benchmarks/system/benchmark_kungfu.py:96).
#include "common.hpp"
#include "kernels.hpp"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace kfk {

const void *zero_page();  // conv.hip

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kBK = 64;  // pixels per K-step

struct WGeo {
    int N, H, W, C, OH, OW, K;
    int P, HW;
    uint64_t m_hw, m_ow;  // floor(p / d) = (p * m) >> 40, exact for p * d < 2^40
    int mtiles, ntiles, taps, tiles, splits, kps;
    int kwin, ph, pw;  // KS == 0 (any window): taps per kernel row and the zero padding
};

// Cache policy of the split-K kernel's LDS-DMA operand loads: non-temporal (aux = 2).  Measured
// on the ResNet-50 step (r3h, tools/gpu_r3_ntconv.sh): +1 % with nt on both operands; the same
// hint on the forward / data-gradient conv kernel's activation loads cost 1.5-2 %.
#ifndef KUNGFU_WGRAD_AUX
#define KUNGFU_WGRAD_AUX 2
#endif
constexpr int kWgradAux = KUNGFU_WGRAD_AUX;

// Buffer-resource staging of wgrad_kernel's operands (num_records = 2 GiB; offset kWBufOOB
// reads zeros).
#ifndef KUNGFU_WGRAD_BUFLD
#define KUNGFU_WGRAD_BUFLD 0
#endif
constexpr uint32_t kWBufOOB = 0x80000000u;
constexpr int kWBufFlags = 0x00020000;

__device__ __forceinline__ __attribute__((address_space(3))) void *wlds_ptr(uint8_t *p) {
    return (__attribute__((address_space(3))) void *)(p);
}

__device__ __forceinline__ int fdiv(int p, uint64_t m) {
    return static_cast<int>((static_cast<uint64_t>(static_cast<uint32_t>(p)) * m) >> 40);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// 32-byte column-group swizzle of an LDS image row (ROW = 128, 256 or 512 bytes; a 512-byte
// row spans two 256-byte bank cycles, so the 3-bit swizzle of 256-byte rows serves it too).
template <int ROW>
__device__ __forceinline__ int hswz(int row) {
    if constexpr (ROW >= 256) return (row & 3) | (((row >> 3) & 1) << 2);
    else if constexpr (ROW == 64) return (row >> 3) & 1;  // 4 rows per 256-byte bank cycle: flip rows 8..15
    else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}

__device__ __forceinline__ bf16x8 tr_frag(const uint8_t *p0, const uint8_t *p1) {
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p1));
    const s16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, v);
}

// WM x WN waves (wave tile 64 co x 16*TN ci), STAGES-deep global_load_lds ring; S = stride.
// KS = 1 | 3 (pad (KS-1)/2), or 0: a KH x KW window with padding (g.kwin, g.ph, g.pw) at run
// time (Inception-v3's 1x7 / 7x1 / 1x3 / 3x1 / 5x5 / 3x3-pad-0).  Channel counts that are not
// multiples of the tile: channels past Cout / Cin read the zero page, their outputs are dropped.
// KB: pixels per staged K-step (64, or 32 with a deeper ring: the 256x256 tile holds only two
// 64-deep stages -- every K-step then waits for ALL its LDS-DMA -- but four 32-deep ones, which
// keep two K-steps in flight across the barrier; gemm.hip uses the same structure).
template <int KS, int S, int WM, int WN, int STAGES, int TN = 4, int KB = 64>
__global__ __launch_bounds__(64 * WM * WN) void wgrad_kernel(const uint16_t *__restrict__ dy,
                                                             const uint16_t *__restrict__ x,
                                                             float *__restrict__ part, void *__restrict__ dw,
                                                             const uint16_t *__restrict__ zero, WGeo g,
                                                             int out_f32, int accumulate, int atomic_out,
                                                             int stagger = 0) {
    constexpr int BM = 64 * WM, BN = 16 * TN * WN, NW = WM * WN, NT = 64 * NW;
    constexpr int PAD = KS > 0 ? (KS - 1) / 2 : 0;
    constexpr int ROWA = BM * 2, ROWB = BN * 2;  // bytes per staged pixel row
    constexpr int CPRA = ROWA / 16, CPRB = ROWB / 16;
    constexpr int RPIA = 64 / CPRA, RPIB = 64 / CPRB;  // rows per 1 KB glds instruction
    constexpr int A_BYTES = KB * ROWA, B_BYTES = KB * ROWB, STAGE = A_BYTES + B_BYTES;
    constexpr int A_INST = KB / RPIA / NW, B_INST = KB / RPIB / NW;
    constexpr int LOADS = A_INST + B_INST;
    static_assert(A_INST >= 1 && B_INST >= 1 && A_INST * NW * RPIA == KB && B_INST * NW * RPIB == KB, "split");
    static_assert(KB == 32 || KB == 64, "K-step of 32 or 64 pixels");
    constexpr bool IDENT = KS == 1 && S == 1;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + (orig >> 3);
    const int split = wg / g.tiles, tile = wg - split * g.tiles;
    const int mn = g.mtiles * g.ntiles;
    const int tap = tile / mn, rem = tile - tap * mn;
    const int mt = rem / g.ntiles, nt = rem - mt * g.ntiles;
    const int kwin = KS > 0 ? KS : g.kwin;
    const int kh = tap / kwin, kw = tap - kh * kwin;
    const int pad_h = KS > 0 ? PAD : g.ph, pad_w = KS > 0 ? PAD : g.pw;
    const int m0 = mt * BM, n0 = nt * BN;
    const int p_begin = split * g.kps * kBK;  // the plan's splits are in 64-pixel steps
    int nsteps = (g.P - p_begin + KB - 1) / KB;
    if (nsteps > g.kps * (kBK / KB)) nsteps = g.kps * (kBK / KB);

    // ---- staging descriptors: lane l of an instruction writes image bytes [16l, 16l+16)
    int a_row[A_INST], a_col[A_INST];
#pragma unroll
    for (int j = 0; j < A_INST; ++j) {
        const int r = (wave * A_INST + j) * RPIA + lane / CPRA;
        const int pc = lane % CPRA;
        const int lc = (((pc >> 1) ^ hswz<ROWA>(r)) << 1) | (pc & 1);
        a_row[j] = r;
        a_col[j] = m0 + lc * 8;
    }
    int b_row[B_INST], b_col[B_INST];
#pragma unroll
    for (int j = 0; j < B_INST; ++j) {
        const int r = (wave * B_INST + j) * RPIB + lane / CPRB;
        const int pc = lane % CPRB;
        const int lc = (((pc >> 1) ^ hswz<ROWB>(r)) << 1) | (pc & 1);
        b_row[j] = r;
        b_col[j] = n0 + lc * 8;
    }

#if KUNGFU_WGRAD_BUFLD
    // LDS-DMA through buffer resources (as conv.hip KUNGFU_CONV_BUFLD): 32-bit byte offsets, an
    // out-of-range lane (pixel past P, channel past Cout / Cin, padding tap) reads zeros past
    // num_records; the launcher checks that dy and x are below 2 GiB
    const __amdgpu_buffer_rsrc_t dyr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(dy), 0, static_cast<int>(kWBufOOB), kWBufFlags);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(x), 0, static_cast<int>(kWBufOOB), kWBufFlags);
#endif
    auto stage = [&](int ks, int buf) {
        const int p0 = p_begin + ks * KB;
        uint8_t *abase = lds + buf * STAGE;
        uint8_t *bbase = abase + A_BYTES;
#pragma unroll
        for (int j = 0; j < A_INST; ++j) {
            const int p = p0 + a_row[j];
#if KUNGFU_WGRAD_BUFLD
            const uint32_t vo = p < g.P && a_col[j] < g.K ? static_cast<uint32_t>(p * g.K + a_col[j]) * 2u : kWBufOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(dyr, wlds_ptr(abase + (wave * A_INST + j) * 1024), 16, vo, 0, 0,
                                                     kWgradAux);
#else
            const uint16_t *src = p < g.P && a_col[j] < g.K ? dy + static_cast<uint32_t>(p * g.K + a_col[j]) : zero;
            __builtin_amdgcn_global_load_lds(src, abase + (wave * A_INST + j) * 1024, 16, 0, kWgradAux);
#endif
        }
#pragma unroll
        for (int j = 0; j < B_INST; ++j) {
            const int p = p0 + b_row[j];
            uint32_t eo = 0xFFFFFFFFu;  // element offset into x, or out of range
            if constexpr (IDENT) {
                if (p < g.P && b_col[j] < g.C) eo = static_cast<uint32_t>(p * g.C + b_col[j]);
            } else {
                const int n = fdiv(p, g.m_hw);
                const int r = p - n * g.HW;
                const int oh = fdiv(r, g.m_ow);
                const int ow = r - oh * g.OW;
                const int ih = oh * S + kh - pad_h, iw = ow * S + kw - pad_w;
                if (p < g.P && b_col[j] < g.C && static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                    static_cast<unsigned>(iw) < static_cast<unsigned>(g.W))
                    eo = static_cast<uint32_t>(((n * g.H + ih) * g.W + iw) * g.C + b_col[j]);
            }
#if KUNGFU_WGRAD_BUFLD
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, wlds_ptr(bbase + (wave * B_INST + j) * 1024), 16,
                                                     eo == 0xFFFFFFFFu ? kWBufOOB : eo * 2u, 0, 0, kWgradAux);
#else
            const uint16_t *src = eo == 0xFFFFFFFFu ? zero : x + eo;
            __builtin_amdgcn_global_load_lds(src, bbase + (wave * B_INST + j) * 1024, 16, 0, kWgradAux);
#endif
        }
    };

    // ---- fragment read addresses (transposing reads; see file comment)
    // lane = 16 g + 4 q + p: block rows kb + q (kb = 32 s + 8 g [+4]), columns 16 c + 4 p.
    const int wm = wave / WN, wn = wave % WN;
    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    const int rowa0 = 8 * fg + fq;  // hswz is the same for rows rowa0 + {0, 4, 32, 36}
    int aoff[4], boff[TN];
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = rowa0 * ROWA + 32 * ((wm * 4 + i) ^ hswz<ROWA>(rowa0)) + 8 * fp;
#pragma unroll
    for (int j = 0; j < TN; ++j) boff[j] = rowa0 * ROWB + 32 * ((wn * TN + j) ^ hswz<ROWB>(rowa0)) + 8 * fp;

    f32x4 acc[4][TN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto mfma_block = [&](const bf16x8 (&af)[4], const bf16x8 (&bfr)[TN]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    };

#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < nsteps) stage(p, p);
    int buf = 0;
    // stagger (fixed per tile in the launcher): the upper half of the waves (one per SIMD with 8 waves) issues its
    // LDS-DMA staging before its fragment reads instead of between its two MFMA clusters, so the two
    // waves sharing a SIMD do not stall on staging issue at the same time
    // stagger 1: stage before the fragment reads; 2: after the second MFMA cluster (upper wave half)
    const bool upper = NW >= 8 && ((wave >> 2) & 1);
    const bool early = (stagger & 3) == 1 && upper, late = (stagger & 3) == 2 && upper;
    if ((stagger & 4) && upper) __builtin_amdgcn_s_setprio(1);  // stagger bit 2: static priority
    for (int ks = 0; ks < nsteps; ++ks) {
        if (ks + STAGES - 1 <= nsteps) wait_vmcnt<LOADS * (STAGES - 2)>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (early && ks + STAGES - 1 < nsteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *abase = lds + buf * STAGE;
        const uint8_t *bbase = abase + A_BYTES;
        bf16x8 af0[4], bf0[TN];
#pragma unroll
        for (int i = 0; i < 4; ++i) af0[i] = tr_frag(abase + aoff[i], abase + aoff[i] + 4 * ROWA);
#pragma unroll
        for (int j = 0; j < TN; ++j) bf0[j] = tr_frag(bbase + boff[j], bbase + boff[j] + 4 * ROWB);
        if constexpr (KB == 64) {
            bf16x8 af1[4], bf1[TN];
#pragma unroll
            for (int i = 0; i < 4; ++i) af1[i] = tr_frag(abase + aoff[i] + 32 * ROWA, abase + aoff[i] + 36 * ROWA);
#pragma unroll
            for (int j = 0; j < TN; ++j) bf1[j] = tr_frag(bbase + boff[j] + 32 * ROWB, bbase + boff[j] + 36 * ROWB);
            mfma_block(af0, bf0);
            __builtin_amdgcn_sched_barrier(0);
            if (!early && !late && ks + STAGES - 1 < nsteps) {
                int nb = buf + STAGES - 1;
                if (nb >= STAGES) nb -= STAGES;
                stage(ks + STAGES - 1, nb);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_block(af1, bf1);
        } else {
            // one 32-deep sub-step: stage the slot read at ks-1 first, then compute
            if (!early && !late && ks + STAGES - 1 < nsteps) {
                int nb = buf + STAGES - 1;
                if (nb >= STAGES) nb -= STAGES;
                stage(ks + STAGES - 1, nb);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_block(af0, bf0);
        }
        if (late && ks + STAGES - 1 < nsteps) {
            __builtin_amdgcn_sched_barrier(0);
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        buf = buf + 1 == STAGES ? 0 : buf + 1;
    }
    wait_vmcnt<0>();

    // ---- epilogue.  C map (16x16): col (ci) = lane & 15, row (co) = (lane >> 4) * 4 + r.
    if (atomic_out) {
        // f32 destination, every split adds its tile in place (no workspace, no reduce pass)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
                    const int ci = n0 + wn * 16 * TN + j * 16 + (lane & 15);
                    if (co >= g.K || ci >= g.C) continue;
                    const int64_t e = (static_cast<int64_t>(co) * g.taps + tap) * g.C + ci;
                    atomicAdd(static_cast<float *>(dw) + e, acc[i][j][r]);
                }
    } else if (g.splits == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = m0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
                    const int ci = n0 + wn * 16 * TN + j * 16 + (lane & 15);
                    if (co >= g.K || ci >= g.C) continue;
                    const int64_t e = (static_cast<int64_t>(co) * g.taps + tap) * g.C + ci;
                    float v = acc[i][j][r];
                    if (out_f32) {
                        float *o = static_cast<float *>(dw) + e;
                        *o = accumulate ? *o + v : v;
                    } else {
                        uint16_t *o = static_cast<uint16_t *>(dw) + e;
                        if (accumulate) v += bf16_to_f32(*o);
                        *o = f32_to_bf16(v);
                    }
                }
    } else {
        f32x4 *dst = reinterpret_cast<f32x4 *>(part + static_cast<int64_t>(wg) * (BM * BN)) + tid;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) dst[(i * TN + j) * NT] = acc[i][j];
    }
}

// ---------------------------------------------------------------------------------------
// Row-image 3x3 / stride-1 weight gradient for narrow channel tiles (64 co x 64 ci per tap).
//
// wgrad_kernel runs one workgroup per TAP: every tap re-stages its own copy of dy and of the
// shifted input, and a 64x64 tile is one wave whose 16 LDS-DMA pieces per K-step cost more
// issue time than its 32 MFMAs (VGG-16 64->64 at 224x224: 247 TF/s; ResNet-50 layer1: 238).
// Here ONE workgroup of 9 waves (wave = tap) shares each K-step's staging:
//   * a K-step is a segment of 64 output pixels: 64 consecutive pixels of one output row
//     (OW >= 64) or R = 64 / OW whole rows (OW < 64);
//   * dy is staged as 64 pixel rows (A operand, as in wgrad_kernel), the input as an image of
//     the (R + 2) input rows x (L + 2) pixels around the segment, zero-padded at the borders;
//   * tap (kh, kw)'s B operand is that image read at row offset kh * (L + 2) + kw: the
//     transposing reads (ds_read_b64_tr_b16) take per-lane row addresses, so the im2col shift
//     is only an address offset -- every input pixel is staged once per segment.
// 33-35 LDS-DMA pieces per K-step are spread over the 9 waves (4 each) against 32 MFMAs per
// wave.  Partial tiles use wgrad_kernel's workspace order (reduced by wgrad_reduce_kernel).
struct RGeo {
    int N, H, W, C, K;
    int L, R, spr, gpi, nseg;  // segment: L pixels per row, R rows; segments per row / per image
    int XW, xrows, xpieces;    // input image: XW = L + 2 pixels per row, xrows rows, 1 KB pieces
    int mtiles, ntiles, tiles, splits, kps;
};

template <int STAGES>
__global__ __launch_bounds__(576) void wgrad_rows_kernel(const uint16_t *__restrict__ dy,
                                                         const uint16_t *__restrict__ x,
                                                         float *__restrict__ part, void *__restrict__ dw,
                                                         const uint16_t *__restrict__ zero, RGeo g, int out_f32,
                                                         int accumulate, int atomic_out, int stagger = 0) {
    constexpr int ROW = 128;            // 64 channels
    constexpr int MAXP = 4;             // pieces per wave per K-step (9 * 4 >= 8 + 25)
    constexpr int STAGE = (8 + 25 + 1) * 1024;  // dy 8 KB | input image <= 25 KB | dummy 1 KB
    constexpr int DUMMY = (8 + 25) * 1024;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[STAGES * STAGE];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = tap
    const int kh = wave / 3, kw = wave - 3 * (wave / 3);
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, rr8 = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (orig >> 3);
    const int mn = g.mtiles * g.ntiles;
    const int split = wg / mn, ctile = wg - split * mn;
    const int mt = ctile / g.ntiles, nt = ctile - mt * g.ntiles;
    const int m0 = mt * 64, n0 = nt * 64;
    const int seg0 = split * g.kps;
    int nsteps = g.nseg - seg0;
    if (nsteps > g.kps) nsteps = g.kps;

    // ---- staging descriptors: wave issues pieces wave + 9u; piece < 8: dy, else input image
    const int total = 8 + g.xpieces;
    int p_kind[MAXP], p_r[MAXP], p_c[MAXP], p_col[MAXP];  // kind 0 dy, 1 x, 2 dummy
#pragma unroll
    for (int u = 0; u < MAXP; ++u) {
        const int pq = wave + 9 * u;
        const int pc = lane & 7;
        if (pq < 8) {
            const int t = pq * 8 + (lane >> 3);  // dy slot
            p_kind[u] = 0;
            p_r[u] = t / g.L;
            p_c[u] = t - p_r[u] * g.L;
            if (p_r[u] >= g.R) p_r[u] = 1 << 20;  // slot past the segment: invalid
            p_col[u] = m0 + ((((pc >> 1) ^ hswz<ROW>(t)) << 1) | (pc & 1)) * 8;
        } else if (pq < total) {
            const int t = (pq - 8) * 8 + (lane >> 3);  // image row
            p_kind[u] = 1;
            p_r[u] = t / g.XW;
            p_c[u] = t - p_r[u] * g.XW;
            if (t >= g.xrows) p_r[u] = 1 << 20;
            p_col[u] = n0 + ((((pc >> 1) ^ hswz<ROW>(t)) << 1) | (pc & 1)) * 8;
        } else {
            p_kind[u] = 2;
            p_r[u] = p_c[u] = p_col[u] = 0;
        }
    }
    const int segs_img = g.gpi * g.spr;
    auto stage = [&](int ks, int buf) {
        const int seg = seg0 + ks;
        const int n = seg / segs_img, rem = seg - n * segs_img;
        const int grp = rem / g.spr, sidx = rem - grp * g.spr;
        const int oh0 = grp * g.R, ow0 = sidx * 64;
        uint8_t *base = lds + buf * STAGE;
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            const int pq = wave + 9 * u;
            const uint16_t *src = zero;
            uint8_t *dst = base + DUMMY;
            if (p_kind[u] == 0) {
                const int oh = oh0 + p_r[u], ow = ow0 + p_c[u];
                if (oh < g.H && ow < g.W) src = dy + static_cast<uint32_t>(((n * g.H + oh) * g.W + ow) * g.K + p_col[u]);
                dst = base + pq * 1024;
            } else if (p_kind[u] == 1) {
                const int ih = oh0 + p_r[u] - 1, iw = ow0 + p_c[u] - 1;
                if (static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                    static_cast<unsigned>(iw) < static_cast<unsigned>(g.W))
                    src = x + static_cast<uint32_t>(((n * g.H + ih) * g.W + iw) * g.C + p_col[u]);
                dst = base + pq * 1024;
            }
            __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
        }
    };

    // ---- fragment addresses.  lane = 16 fg + 4 fq + fp; K-slots j = 8 fg + fq + {0, 4, 32, 36}.
    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    const int rowa0 = 8 * fg + fq;
    int aoff[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) aoff[i] = rowa0 * ROW + 32 * (i ^ hswz<ROW>(rowa0)) + 8 * fp;
    int boff[4][4];  // [sub-read][ci block]
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int j = rowa0 + (s & 1) * 4 + (s >> 1) * 32;
        const int r = j / g.L, c = j - r * g.L;
        const int jrow = r < g.R ? r * g.XW + c : 0;  // slots past the segment read a staged row (dy is 0)
        const int trow = jrow + kh * g.XW + kw;
        const int h = hswz<ROW>(trow);
#pragma unroll
        for (int i = 0; i < 4; ++i) boff[s][i] = 8192 + trow * ROW + 32 * (i ^ h) + 8 * fp;
    }

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma_block = [&](const bf16x8 (&af)[4], const bf16x8 (&bfr)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    };

#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < nsteps) stage(p, p);
    int buf = 0;
    const bool early = stagger && ((wave >> 2) & 1);  // see wgrad_kernel: staggered staging issue
    for (int ks = 0; ks < nsteps; ++ks) {
        if (ks + STAGES - 1 <= nsteps) wait_vmcnt<MAXP * (STAGES - 2)>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (early && ks + STAGES - 1 < nsteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *base = lds + buf * STAGE;
        bf16x8 af0[4], bf0[4], af1[4], bf1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            af0[i] = tr_frag(base + aoff[i], base + aoff[i] + 4 * ROW);
            bf0[i] = tr_frag(base + boff[0][i], base + boff[1][i]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            af1[i] = tr_frag(base + aoff[i] + 32 * ROW, base + aoff[i] + 36 * ROW);
            bf1[i] = tr_frag(base + boff[2][i], base + boff[3][i]);
        }
        mfma_block(af0, bf0);
        __builtin_amdgcn_sched_barrier(0);
        if (!early && ks + STAGES - 1 < nsteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_block(af1, bf1);
        buf = buf + 1 == STAGES ? 0 : buf + 1;
    }
    wait_vmcnt<0>();

    // ---- epilogue (wgrad_kernel's three forms; tile = this wave's tap)
    const int tap = wave, taps = 9;
    if (atomic_out || g.splits == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = m0 + i * 16 + (lane >> 4) * 4 + r;
                    const int ci = n0 + j * 16 + (lane & 15);
                    const int64_t e = (static_cast<int64_t>(co) * taps + tap) * g.C + ci;
                    float v = acc[i][j][r];
                    if (atomic_out) {
                        atomicAdd(static_cast<float *>(dw) + e, v);
                    } else if (out_f32) {
                        float *o = static_cast<float *>(dw) + e;
                        *o = accumulate ? *o + v : v;
                    } else {
                        uint16_t *o = static_cast<uint16_t *>(dw) + e;
                        if (accumulate) v += bf16_to_f32(*o);
                        *o = f32_to_bf16(v);
                    }
                }
    } else {
        const int tile = tap * mn + mt * g.ntiles + nt;
        f32x4 *dst = reinterpret_cast<f32x4 *>(part + (static_cast<int64_t>(split) * g.tiles + tile) * 4096) + lane;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[(i * 4 + j) * 64] = acc[i][j];
    }
}

// ---------------------------------------------------------------------------------------
// Row-image weight gradient for ANY stride-1 KH x KW window with zero padding and channel
// counts % 8 (Inception-v3's narrow multi-tap layers: 32..192 channels, 1x7 / 7x1 / 3x3 /
// 5x5, pad 0 or (K-1)/2), the generalisation of wgrad_rows_kernel above:
//   * output tile 64 co x 64 ci per wave and tap; channels past Cout / Cin are staged from the
//     zero page and their outputs dropped (48 -> one half-empty tile, 80 -> 64 + 16, ...);
//   * a workgroup holds NWV waves = NWV consecutive taps of the window (taps > NWV: the window
//     is split over tap groups, e.g. 5x5 = 9 + 9 + 7 taps; idle waves of the last group only
//     stage) and shares one K-step's staging among them: dy as 64 pixel rows, the input as the
//     (R + KH - 1) x (L + KW - 1) image around the segment of 64 output pixels;
//   * tap (kh, kw) reads the image at row offset kh * XW + kw (transposing LDS reads with
//     per-lane row addresses: the im2col shift is only an address offset).
// CT = the channel tile (both co and ci): 64, or 32 for the channel counts that are not multiples
// of 64 (Inception's 32 / 80 / 96 / 160 / 48: no zero-padded half tiles, 64-byte staged rows, a
// 32 x 32 wave tile) -- CT 32 also writes its split partials in dw layout ([split][co][tap][ci],
// exactly K * taps * C floats, no tile padding), summed by wgrad_dense_reduce_kernel.
// Replaces MIOpen's igemm_wrw for these shapes (r2o_inception_wgrad.txt: 170-275 TF/s there).
struct RRGeo {
    int N, H, W, C, K, OH, OW;
    int KH, KW, ph, pw, taps, tgroups;
    int L, R, spr, gpi, nseg;
    int XW, xrows, xpieces;
    int mtiles, ntiles, tiles, splits, kps;
    int stage;  // LDS bytes per ring stage: dy | image | 1 KB dummy
    int S;      // stride (1, or 2 on the kRowsEx variants)
};

// s_waitcnt until at most n * (S - 2) loads of this wave are in flight (n = its loads per stage,
// wave-uniform, 1..5): the oldest outstanding stage of an S-deep ring has landed
template <int S>
__device__ __forceinline__ void wait_ring(int n) {
    if constexpr (S <= 2) {
        wait_vmcnt<0>();
    } else {
        switch (n) {
            case 1: wait_vmcnt<1 * (S - 2)>(); break;
            case 2: wait_vmcnt<2 * (S - 2)>(); break;
            case 3: wait_vmcnt<3 * (S - 2)>(); break;
            case 4: wait_vmcnt<4 * (S - 2)>(); break;
            case 5: wait_vmcnt<5 * (S - 2)>(); break;
            default: wait_vmcnt<0>();
        }
    }
}

template <int NWV, int STAGES, int CT = 64, bool DENSE = (CT == 32)>
__global__ __launch_bounds__(64 * NWV) void wgrad_rows_rect_kernel(const uint16_t *__restrict__ dy,
                                                                   const uint16_t *__restrict__ x,
                                                                   float *__restrict__ part, void *__restrict__ dw,
                                                                   const uint16_t *__restrict__ zero, RRGeo g,
                                                                   int out_f32, int accumulate, int atomic_out,
                                                                   int stagger = 0) {
    constexpr int ROW = 2 * CT;                    // staged bytes per pixel (CT channels)
    constexpr int TI = CT / 16;                    // 16-wide MFMA blocks per tile side
    constexpr int LPR = ROW / 16;                  // lanes (16 B each) per staged row
    constexpr int RPP = 64 / LPR;                  // rows per 1 KB piece
    constexpr int DYP = 64 / RPP;                  // dy pieces per K-step (64 pixels)
    constexpr int DYB = DYP * 1024;
    constexpr int MAXP = (DYP + 25 + NWV - 1) / NWV;  // 1 KB pieces per wave per K-step (bound)
    static_assert(MAXP <= 5, "wait_ring covers 5 loads per stage");
    extern __shared__ __attribute__((aligned(1024))) uint8_t lds[];  // STAGES x g.stage bytes
    const int STAGE = g.stage;                   // dy | input image (<= 25 KB) | dummy 1 KB
    const int DUMMY = g.stage - 1024;

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q8 = nwg >> 3, rr8 = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < rr8 ? xcd * (q8 + 1) : rr8 * (q8 + 1) + (xcd - rr8) * q8) + (orig >> 3);
    const int mn = g.mtiles * g.ntiles;
    const int per_split = mn * g.tgroups;
    const int split = wg / per_split, rem0 = wg - split * per_split;
    const int tg = rem0 / mn, ctile = rem0 - tg * mn;
    const int mt = ctile / g.ntiles, nt = ctile - mt * g.ntiles;
    const int m0 = mt * CT, n0 = nt * CT;
    const int tap = tg * NWV + wave;  // >= g.taps: staging-only wave
    const bool has_tap = tap < g.taps;
    const int kh = has_tap ? tap / g.KW : 0, kw = has_tap ? tap - kh * g.KW : 0;
    const int seg0 = split * g.kps;
    int nsteps = g.nseg - seg0;
    if (nsteps > g.kps) nsteps = g.kps;

    // ---- staging descriptors: wave issues pieces wave + NWV u; piece < 8: dy, else input image
    const int total = DYP + g.xpieces;
    const int nload = (total + NWV - 1) / NWV;  // pieces per wave per stage (a ring > 2 issues them all)
    int p_kind[MAXP], p_r[MAXP], p_c[MAXP], p_col[MAXP];  // kind 0 dy, 1 x, 2 dummy
    bool p_cok[MAXP];
#pragma unroll
    for (int u = 0; u < MAXP; ++u) {
        const int pq = wave + NWV * u;
        const int pc = lane % LPR;
        p_cok[u] = false;
        if (pq < DYP) {
            const int t = pq * RPP + lane / LPR;  // dy slot
            p_kind[u] = 0;
            p_r[u] = t / g.L;
            p_c[u] = t - p_r[u] * g.L;
            if (p_r[u] >= g.R) p_r[u] = 1 << 20;  // slot past the segment: invalid
            p_col[u] = m0 + ((((pc >> 1) ^ hswz<ROW>(t)) << 1) | (pc & 1)) * 8;
            p_cok[u] = p_col[u] < g.K;
        } else if (pq < total) {
            const int t = (pq - DYP) * RPP + lane / LPR;  // image row
            p_kind[u] = 1;
            p_r[u] = t / g.XW;
            p_c[u] = t - p_r[u] * g.XW;
            if (t >= g.xrows) p_r[u] = 1 << 20;
            p_col[u] = n0 + ((((pc >> 1) ^ hswz<ROW>(t)) << 1) | (pc & 1)) * 8;
            p_cok[u] = p_col[u] < g.C;
        } else {
            p_kind[u] = 2;
            p_r[u] = p_c[u] = p_col[u] = 0;
        }
    }
    const int segs_img = g.gpi * g.spr;
    auto stage = [&](int ks, int buf) {
        const int seg = seg0 + ks;
        const int n = seg / segs_img, rem = seg - n * segs_img;
        const int grp = rem / g.spr, sidx = rem - grp * g.spr;
        const int oh0 = grp * g.R, ow0 = sidx * g.L;
        uint8_t *base = lds + buf * STAGE;
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            if (u >= nload) break;
            const int pq = wave + NWV * u;
            if constexpr (STAGES == 2) {
                // every K-step waits for all of its loads (vmcnt 0), so no dummy issue keeps the
                // count; lanes of channels past Cout / Cin leave their LDS bytes stale (they only
                // reach outputs that are dropped)
                if (p_kind[u] == 2 || !p_cok[u]) continue;
            }
            const uint16_t *src = zero;
            uint8_t *dst = base + DUMMY;
            if (p_kind[u] == 0) {
                const int oh = oh0 + p_r[u], ow = ow0 + p_c[u];
                if (oh < g.OH && ow < g.OW && p_cok[u])
                    src = dy + static_cast<uint32_t>(((n * g.OH + oh) * g.OW + ow) * g.K + p_col[u]);
                dst = base + pq * 1024;
            } else if (p_kind[u] == 1) {
                const int ih = oh0 * g.S + p_r[u] - g.ph, iw = ow0 * g.S + p_c[u] - g.pw;
                if (static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) &&
                    static_cast<unsigned>(iw) < static_cast<unsigned>(g.W) && p_cok[u])
                    src = x + static_cast<uint32_t>(((n * g.H + ih) * g.W + iw) * g.C + p_col[u]);
                dst = base + pq * 1024;
            }
            __builtin_amdgcn_global_load_lds(src, dst, 16, 0, 0);
        }
    };

    // ---- fragment addresses.  lane = 16 fg + 4 fq + fp; K-slots j = 8 fg + fq + {0, 4, 32, 36}.
    const int fg = lane >> 4, fq = (lane >> 2) & 3, fp = lane & 3;
    const int rowa0 = 8 * fg + fq;
    int aoff[TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) aoff[i] = rowa0 * ROW + 32 * (i ^ hswz<ROW>(rowa0)) + 8 * fp;
    int boff[4][TI];  // [sub-read][ci block]
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int j = rowa0 + (s & 1) * 4 + (s >> 1) * 32;
        const int r = j / g.L, c = j - r * g.L;
        // output (r, c) of the segment sits at image row S r, column S c; slots past it read a staged
        // row (their dy is 0)
        const int jrow = r < g.R ? r * g.S * g.XW + g.S * c : 0;
        const int trow = jrow + kh * g.XW + kw;
        const int h = hswz<ROW>(trow);
#pragma unroll
        for (int i = 0; i < TI; ++i) boff[s][i] = DYB + trow * ROW + 32 * (i ^ h) + 8 * fp;
    }

    f32x4 acc[TI][TI];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma_block = [&](const bf16x8 (&af)[TI], const bf16x8 (&bfr)[TI]) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TI; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    };

#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < nsteps) stage(p, p);
    int buf = 0;
    const bool early = stagger && ((wave >> 2) & 1);  // see wgrad_kernel: staggered staging issue
    for (int ks = 0; ks < nsteps; ++ks) {
        if (ks + STAGES - 1 <= nsteps) wait_ring<STAGES>(nload);
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if ((early || !has_tap) && ks + STAGES - 1 < nsteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *base = lds + buf * STAGE;
        if (has_tap) {  // wave-uniform
            bf16x8 af0[TI], bf0[TI], af1[TI], bf1[TI];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                af0[i] = tr_frag(base + aoff[i], base + aoff[i] + 4 * ROW);
                bf0[i] = tr_frag(base + boff[0][i], base + boff[1][i]);
            }
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                af1[i] = tr_frag(base + aoff[i] + 32 * ROW, base + aoff[i] + 36 * ROW);
                bf1[i] = tr_frag(base + boff[2][i], base + boff[3][i]);
            }
            mfma_block(af0, bf0);
            __builtin_amdgcn_sched_barrier(0);
            if (!early && ks + STAGES - 1 < nsteps) {
                int nb = buf + STAGES - 1;
                if (nb >= STAGES) nb -= STAGES;
                stage(ks + STAGES - 1, nb);
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_block(af1, bf1);
        }
        buf = buf + 1 == STAGES ? 0 : buf + 1;
    }
    wait_vmcnt<0>();
    if (!has_tap) return;

    // ---- epilogue (wgrad_kernel's three forms; tile = this wave's tap)
    if constexpr (DENSE) {
        if (!atomic_out && g.splits > 1) {  // dw-layout partial of this split: plain f32 stores
            float *dst = part + static_cast<int64_t>(split) * g.K * g.taps * g.C;
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TI; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co = m0 + i * 16 + (lane >> 4) * 4 + r;
                        const int ci = n0 + j * 16 + (lane & 15);
                        if (co < g.K && ci < g.C) dst[(static_cast<int64_t>(co) * g.taps + tap) * g.C + ci] = acc[i][j][r];
                    }
            return;
        }
    }
    if (atomic_out || g.splits == 1) {
#pragma unroll
        for (int i = 0; i < TI; ++i)
#pragma unroll
            for (int j = 0; j < TI; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = m0 + i * 16 + (lane >> 4) * 4 + r;
                    const int ci = n0 + j * 16 + (lane & 15);
                    if (co >= g.K || ci >= g.C) continue;
                    const int64_t e = (static_cast<int64_t>(co) * g.taps + tap) * g.C + ci;
                    float v = acc[i][j][r];
                    if (atomic_out) {
                        atomicAdd(static_cast<float *>(dw) + e, v);
                    } else if (out_f32) {
                        float *o = static_cast<float *>(dw) + e;
                        *o = accumulate ? *o + v : v;
                    } else {
                        uint16_t *o = static_cast<uint16_t *>(dw) + e;
                        if (accumulate) v += bf16_to_f32(*o);
                        *o = f32_to_bf16(v);
                    }
                }
    } else if constexpr (!DENSE) {
        const int tile = tap * mn + mt * g.ntiles + nt;
        f32x4 *dst = reinterpret_cast<f32x4 *>(part + (static_cast<int64_t>(split) * g.tiles + tile) * 4096) + lane;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) dst[(i * 4 + j) * 64] = acc[i][j];
    }
}

// dw[e] (+)= the sum over the splits of part[split][e] (deterministic: a fixed order for a given
// shape); e over the n = K * taps * C outputs in dw layout, as float4 columns (n % 4 == 0: C % 8).
// Block = 256 threads = (256 >> sgl) columns x (1 << sgl) split groups: group g sums splits g, g + G,
// ... in order, then the G group sums meet in LDS in group order -- a few thousand columns over
// hundreds of splits (Conv2d_2a: 2,304 x 768) still keep every CU's loads in flight.
__global__ __launch_bounds__(256) void wgrad_dense_reduce_kernel(const float *__restrict__ part, int splits, int64_t n,
                                                                 void *__restrict__ dw, int out_f32, int accumulate,
                                                                 int sgl) {
    __shared__ f32x4 red[256];
    const int G = 1 << sgl, COLS = 256 >> sgl;
    const int t = threadIdx.x, c = t & (COLS - 1), grp = t >> (8 - sgl);
    const int64_t n4 = n / 4, col = static_cast<int64_t>(blockIdx.x) * COLS + c;
    f32x4 a = f32x4{0.f, 0.f, 0.f, 0.f};
    if (col < n4) {
        const f32x4 *src = reinterpret_cast<const f32x4 *>(part) + col;
        int sp = grp;
        for (; sp + G < splits; sp += 2 * G) {
            const f32x4 u = src[sp * n4], v = src[(sp + G) * n4];
            a += u;
            a += v;
        }
        if (sp < splits) a += src[sp * n4];
    }
    red[t] = a;
    __syncthreads();
    if (grp != 0 || col >= n4) return;
    f32x4 sum = red[c];
    for (int k = 1; k < G; ++k) sum += red[k * COLS + c];
    const int64_t e = col * 4;
    if (out_f32) {
        f32x4 *o = reinterpret_cast<f32x4 *>(static_cast<float *>(dw) + e);
        if (accumulate) sum += *o;
        *o = sum;
    } else {
        uint16_t *o = static_cast<uint16_t *>(dw) + e;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v = sum[k];
            if (accumulate) v += bf16_to_f32(o[k]);
            o[k] = f32_to_bf16(v);
        }
    }
}

// Sum the split partials (workspace order of wgrad_kernel) and scatter to dw.
// Block = 256 threads = OUT float4 outputs x SG split groups (SG = 256 / OUT, a power of
// two <= splits): a few K outputs with hundreds of splits (the 56x56 layers) still keep
// every CU's loads in flight; the SG partial sums meet in LDS.
template <int WM, int WN, int TN = 4>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float *__restrict__ part, void *__restrict__ dw,
                                                           WGeo g, int out_f32, int accumulate, int sg_log2) {
    constexpr int BM = 64 * WM, BN = 16 * TN * WN, NT = 64 * WM * WN;
    constexpr int TILE4 = BM * BN / 4;
    __shared__ f32x4 red[256];
    const int SG = 1 << sg_log2, OUT = 256 >> sg_log2;
    const int t = threadIdx.x, o = t & (OUT - 1), sg = t >> (8 - sg_log2);
    const int64_t total = static_cast<int64_t>(g.tiles) * TILE4;
    const int64_t idx = static_cast<int64_t>(blockIdx.x) * OUT + o;
    const int64_t stride_split = total;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
    if (idx < total) {
        const f32x4 *src = reinterpret_cast<const f32x4 *>(part) + idx;
        int sp = sg;
        for (; sp + 3 * SG < g.splits; sp += 4 * SG) {
            const f32x4 a = src[sp * stride_split];
            const f32x4 b = src[(sp + SG) * stride_split];
            const f32x4 c = src[(sp + 2 * SG) * stride_split];
            const f32x4 d = src[(sp + 3 * SG) * stride_split];
            s += (a + b) + (c + d);
        }
        for (; sp < g.splits; sp += SG) s += src[sp * stride_split];
    }
    red[t] = s;
    __syncthreads();
    if (sg == 0 && idx < total) {
        for (int k = 1; k < SG; ++k) s += red[o + k * OUT];
        const int tile = static_cast<int>(idx / TILE4);
        const int rem = static_cast<int>(idx - static_cast<int64_t>(tile) * TILE4);
        const int ij = rem / NT, tid = rem - ij * NT;
        const int mn = g.mtiles * g.ntiles;
        const int tap = tile / mn, r2 = tile - tap * mn;
        const int mt = r2 / g.ntiles, nt = r2 - mt * g.ntiles;
        const int lane = tid & 63, wave = tid >> 6;
        const int wm = wave / WN, wn = wave % WN;
        const int i = ij / TN, j = ij % TN;
        const int ci = nt * BN + wn * 16 * TN + j * 16 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = mt * BM + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
            if (co >= g.K || ci >= g.C) continue;
            const int64_t e = (static_cast<int64_t>(co) * g.taps + tap) * g.C + ci;
            float v = s[r];
            if (out_f32) {
                float *d = static_cast<float *>(dw) + e;
                *d = accumulate ? *d + v : v;
            } else {
                uint16_t *d = static_cast<uint16_t *>(dw) + e;
                if (accumulate) v += bf16_to_f32(*d);
                *d = f32_to_bf16(v);
            }
        }
    }
}

// Staggered staging issue in the row-image kernels (see wgrad_kernel), default on (same-box A/Bs:
// Inception-v3 21.62 -> 21.45 ms/step, VGG-16 34.85 -> 34.62, ResNet-50 neutral);
int rows_stagger(bool /*rect*/) { return 1; }

struct Tile {
    int wm, wn, tn;  // waves (co, ci) and 16-channel ci blocks per wave
    constexpr int bm() const { return 64 * wm; }
    constexpr int bn() const { return 16 * tn * wn; }
};
// variant -> tile (co x ci): 0 128x128, 1 128x64, 2 64x128, 3 64x64, 4 256x128, 5 128x256,
// 6 the row-image kernel (below), 7 256x256 (8 waves of 64x128: twice the MFMAs per staged byte)
constexpr Tile kTiles[] = {{2, 2, 4}, {2, 1, 4}, {1, 2, 4}, {1, 1, 4}, {4, 2, 4}, {2, 4, 4}, {0, 0, 0}, {4, 2, 8}};
constexpr int kNumVariants = 8;
constexpr int kRowsVariant = 6;
// conv_wgrad_rect only: the row-image kernel with segments chosen for the fewest staged rows, an
// LDS ring sized to the segment, dw-layout partials: 8 / 9 / 10 = 32-channel tiles with a 2 / 3 /
// 4-stage ring, 11 / 12 = 64-channel tiles with a 3 / 4-stage ring
constexpr int kRowsExFirst = 8, kRowsExLast = 12;
struct RowsEx {
    int ct, stages;
};
constexpr RowsEx kRowsEx[] = {{32, 2}, {32, 3}, {32, 4}, {64, 3}, {64, 4}};

bool rows_supported(int Cin, int Cout, int ks, int stride) {
    return ks == 3 && stride == 1 && Cin % 64 == 0 && Cout % 64 == 0;
}
// KUNGFU_WGRAD_PLAN (dev knob): 2 (default) = the round-6 plan rules below, 1 = the round-5 ones
int wgrad_plan_rules() {
    static const int v = dev_knob("KUNGFU_WGRAD_PLAN", 2);
    return v;
}

// default for the narrow channel counts (tools/bench_wgrad.py), and (round 6) for every stride-1 3x3:
// ResNet-50's 14 x 14 256->256 and 7 x 7 512->512 measured 113 -> 93 us on it (r6t36), VGG-16's
// 56 x 56 128->256 / 256->256 673 -> 766 / 688 -> 788 TF/s (r6t43, profiles/r6_wgrad_plan.md)
bool rows_default(int Cin, int Cout, int ks, int stride, int64_t /*P*/) {
    if (!rows_supported(Cin, Cout, ks, stride)) return false;
    return (Cin <= 128 && Cout <= 128) || wgrad_plan_rules() >= 2;
}

RGeo rows_segments(int N, int H, int W, int Cin, int Cout) {
    RGeo g{};
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout;
    if (W >= 64) {
        g.L = 64, g.R = 1, g.spr = (W + 63) / 64, g.gpi = H;
    } else {
        g.L = W, g.R = 64 / W, g.spr = 1, g.gpi = (H + g.R - 1) / g.R;
    }
    g.nseg = N * g.gpi * g.spr;
    g.XW = g.L + 2;
    g.xrows = (g.R + 2) * g.XW;
    g.xpieces = (g.xrows + 7) / 8;
    g.mtiles = Cout / 64, g.ntiles = Cin / 64;
    g.tiles = g.mtiles * g.ntiles * 9;
    return g;
}

RGeo make_rgeo(int N, int H, int W, int Cin, int Cout, const WgradPlan &plan) {
    RGeo g = rows_segments(N, H, W, Cin, Cout);
    if (g.xpieces > 25) throw std::invalid_argument("conv_wgrad rows: input image exceeds the stage");
    g.splits = plan.splits;
    g.kps = plan.kps;
    return g;
}

uint64_t magic40(int d) { return (uint64_t(1) << 40) / static_cast<uint64_t>(d) + 1; }

WGeo make_geo(int N, int H, int W, int Cin, int Cout, int ks, int stride, const WgradPlan &plan) {
    // (tap-tiled variants 0-5 only)
    WGeo g;
    const int pad = (ks - 1) / 2;
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout;
    g.OH = (H + 2 * pad - ks) / stride + 1;
    g.OW = (W + 2 * pad - ks) / stride + 1;
    g.HW = g.OH * g.OW;
    g.P = N * g.HW;
    g.m_hw = magic40(g.HW);
    g.m_ow = magic40(g.OW);
    const Tile t = kTiles[plan.variant];
    g.mtiles = Cout / t.bm();
    g.ntiles = Cin / t.bn();
    g.taps = ks * ks;
    g.kwin = ks, g.ph = g.pw = pad;
    g.tiles = g.mtiles * g.ntiles * g.taps;
    g.splits = plan.splits;
    g.kps = plan.kps;
    return g;
}

template <int KS, int S, int WM, int WN, int TN = 4>
void launch_t(const uint16_t *dy, const uint16_t *x, void *dw, float *part, const WGeo &g, bool out_f32,
              bool accumulate, bool atomic_out, hipStream_t s) {
    // 3-deep global_load_lds ring (tools/bench_wgrad.py --sweep: 2 stages starve the 8-wave
    // 256x128 tiles, 4 stages cost the 1-2 wave tiles their second/third workgroup per CU);
    // 2 for the 256x256 tile (64 KB per stage)
    constexpr int STAGE_BYTES = 64 * (64 * WM + 16 * TN * WN) * 2;
    constexpr int STAGES = 3 * STAGE_BYTES <= 160 * 1024 ? 3 : 2;
    // staggered staging issue: on for the 256x256 tiles only -- BERT-base's long-K linear weight
    // gradients +1.5 % step time, ResNet-50's 256x128 tiles -0.8 % with it (tools/gpu_r3_envab.sh)
    const int stagger = TN == 8 ? 1 : 0;
    if (KUNGFU_WGRAD_BUFLD && (static_cast<int64_t>(g.P) * g.K * 2 >= kWBufOOB ||
                               static_cast<int64_t>(g.N) * g.H * g.W * g.C * 2 >= kWBufOOB))
        throw std::invalid_argument("conv_wgrad: dy or x of 2 GiB or more (buffer-resource staging)");
    // 256x256 tiles with four 32-pixel stages instead of two 64-pixel ones: measured no better (r4t1)
    constexpr int kb32 = 0;
    if constexpr (TN == 8) {
        if (kb32) {
            wgrad_kernel<KS, S, WM, WN, 4, TN, 32><<<g.tiles * g.splits, 64 * WM * WN, 0, s>>>(
                dy, x, part, dw, reinterpret_cast<const uint16_t *>(zero_page()), g, out_f32, accumulate, atomic_out,
                stagger);
        } else {
            wgrad_kernel<KS, S, WM, WN, STAGES, TN><<<g.tiles * g.splits, 64 * WM * WN, 0, s>>>(
                dy, x, part, dw, reinterpret_cast<const uint16_t *>(zero_page()), g, out_f32, accumulate,
                atomic_out, stagger);
        }
    } else {
        wgrad_kernel<KS, S, WM, WN, STAGES, TN><<<g.tiles * g.splits, 64 * WM * WN, 0, s>>>(
            dy, x, part, dw, reinterpret_cast<const uint16_t *>(zero_page()), g, out_f32, accumulate, atomic_out,
            stagger);
    }
    if (g.splits > 1 && !atomic_out) {
        const int64_t total = static_cast<int64_t>(g.tiles) * (64 * WM) * (16 * TN * WN) / 4;
        int sgl = 0;  // split groups: enough blocks for the chip, at most 64 groups, <= splits
        while (sgl < 6 && (2 << sgl) <= g.splits && (total << (sgl + 1)) <= int64_t(256) * 2048) ++sgl;
        const int64_t grid = (total + (256 >> sgl) - 1) / (256 >> sgl);
        wgrad_reduce_kernel<WM, WN, TN><<<static_cast<int>(grid), 256, 0, s>>>(part, dw, g, out_f32, accumulate, sgl);
    }
}

template <int KS, int S>
void launch_ks(const uint16_t *dy, const uint16_t *x, void *dw, float *part, const WGeo &g, int variant,
               bool out_f32, bool accumulate, bool atomic_out, hipStream_t s) {
    switch (variant) {
    case 0: launch_t<KS, S, 2, 2>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    case 1: launch_t<KS, S, 2, 1>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    case 2: launch_t<KS, S, 1, 2>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    case 3: launch_t<KS, S, 1, 1>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    case 4: launch_t<KS, S, 4, 2>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    case 5: launch_t<KS, S, 2, 4>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    default: launch_t<KS, S, 4, 2, 8>(dy, x, dw, part, g, out_f32, accumulate, atomic_out, s); break;
    }
}

}  // namespace

int conv_wgrad_variants() { return kNumVariants; }

int64_t conv_wgrad_max_pixels(int N, int H, int W, int Cin, int Cout, int ks, int stride) {
    // the tap-tiled kernel's 40-bit magic division holds < 2^23 output pixels; the row-image
    // kernel only needs 32-bit element offsets (checked by the caller)
    const WgradPlan pl = conv_wgrad_plan(N, H, W, Cin, Cout, ks, stride, -1, -1);
    return pl.variant == kRowsVariant ? (int64_t(1) << 31) : (int64_t(1) << 23);
}

bool conv_wgrad_supported(int Cin, int Cout, int ks, int stride) {
    return (ks == 1 || ks == 3) && (stride == 1 || stride == 2) && Cin % 64 == 0 && Cout % 64 == 0 && Cin >= 64 &&
           Cout >= 64;
}

WgradPlan conv_wgrad_plan(int N, int H, int W, int Cin, int Cout, int ks, int stride, int variant, int splits) {
    WgradPlan pl;
    const int64_t work = static_cast<int64_t>(Cin) * Cout * ks * ks;
    if (variant < 0 && rows_default(Cin, Cout, ks, stride, static_cast<int64_t>(N) * H * W)) variant = kRowsVariant;
    if (variant == kRowsVariant) {
        if (!rows_supported(Cin, Cout, ks, stride)) throw std::invalid_argument("conv_wgrad: rows variant needs 3x3/s1");
        pl.variant = variant;
        const RGeo rg = rows_segments(N, H, W, Cin, Cout);
        const int ct = rg.mtiles * rg.ntiles;
        // one workgroup of 9 waves per CU (round 6; two per CU through round 5): half the split
        // partials to reduce -- 56 x 56 64->64 119 -> 89 us, 28 x 28 128->128 108 -> 84 (r6t36)
        const int per = wgrad_plan_rules() >= 2 ? 256 : 512;
        if (splits < 0) splits = std::max(1, (per + ct / 2) / ct);
        splits = std::max(1, std::min(splits, std::max(1, rg.nseg / 4)));
        pl.kps = (rg.nseg + splits - 1) / splits;
        pl.splits = (rg.nseg + pl.kps - 1) / pl.kps;
        pl.ws_floats = pl.splits > 1 ? static_cast<int64_t>(pl.splits) * ct * 9 * 4096 : 0;
        return pl;
    }
    if (variant < 0) {
        // tools/bench_wgrad.py --sweep (profiles/README.md): 8-wave 256x128 tiles once the
        // GEMM is big enough, else the largest 4/2/1-wave tile the channel counts allow
        // tools/bench_wgrad_1x1.py: 256x256 for the large long-K linear-layer products (BERT-base
        // 768x3072 at 16 K tokens: 133 -> 87 us); ResNet's 1x1 shapes keep 256x128 (their split-K
        // partials of 256x256 tiles cost more than the extra MFMA density saves)
        const int64_t P1 = static_cast<int64_t>(N) * ((H + 2 * ((ks - 1) / 2) - ks) / stride + 1) *
                           ((W + 2 * ((ks - 1) / 2) - ks) / stride + 1);
        // (round 6: and the wide 1x1 products on >= 200,704 output pixels -- 28 x 28 512->256 103 -> 77 us,
        // 56 x 56 256->512 / s2 103 -> 90; ResNet-50 20.09-20.13 -> 20.07 ms/step, r6t36 / r6t37)
        if (Cout % 256 == 0 && Cin % 256 == 0 && ks == 1 && (work >= 1500000 || (wgrad_plan_rules() >= 2 && P1 >= 200704)))
            variant = 7;
        else if (Cout % 256 == 0 && Cin % 128 == 0) variant = 4;
        else if (Cout % 128 == 0 && Cin % 256 == 0 && work >= (wgrad_plan_rules() >= 2 ? 32768 : 131072)) variant = 5;
        // (round 6: 128x256 from 32 K outputs -- 56 x 56 256->128 158 -> 111 us, 28 x 28 512->128 73 -> 60, r6t36)
        else if (Cout % 128 == 0 && Cin % 128 == 0) variant = 0;
        else if (Cout % 128 == 0) variant = 1;
        else if (Cin % 128 == 0) variant = 2;
        else variant = 3;
    }
    const Tile t = kTiles[variant];
    if (t.wm == 0 || Cout % t.bm() != 0 || Cin % t.bn() != 0) throw std::invalid_argument("conv_wgrad: tile/channel mismatch");
    pl.variant = variant;
    const int pad = (ks - 1) / 2;
    const int OH = (H + 2 * pad - ks) / stride + 1, OW = (W + 2 * pad - ks) / stride + 1;
    const int64_t P = static_cast<int64_t>(N) * OH * OW;
    const int ksteps = static_cast<int>((P + kBK - 1) / kBK);
    const int tiles = (Cout / t.bm()) * (Cin / t.bn()) * ks * ks;
    if (splits < 0) {
        // workgroups per launch: one per CU for the 4/8-wave tiles (2 for 3x3), more for the
        // 1-2 wave tiles, so every CU keeps >= ~48 KB of loads in flight; >= 4 K-steps per split
        const int nw = t.wm * t.wn;
        int target = 256 * (nw >= 4 ? 1 : 2);
        if (ks == 3) target *= nw == 1 ? 4 : 2;
        splits = (target + tiles / 2) / tiles;
        // large-pixel 3x3 shapes (VGG-16's 56..224 layers, batch 256): ~100 K-steps per split
        // and up to 512 splits (tools/bench_vgg_wgrad.py: 112x112 128->128 313 -> 477 TF/s,
        // 56x56 128->256 587 -> 761 TF/s; 28x28 and smaller keep the default)
        if (ks == 3 && P >= 800000) splits = std::max(splits, std::min(512, ksteps / 96));
        splits = std::max(1, std::min(splits, ksteps / 4));
    }
    splits = std::max(1, std::min(splits, ksteps));
    pl.kps = (ksteps + splits - 1) / splits;
    pl.splits = (ksteps + pl.kps - 1) / pl.kps;  // no empty split
    pl.ws_floats = pl.splits > 1 ? static_cast<int64_t>(pl.splits) * tiles * t.bm() * t.bn() : 0;
    return pl;
}

void launch_conv_wgrad(const uint16_t *dy, const uint16_t *x, void *dw, float *part, int N, int H, int W, int Cin,
                       int Cout, int ks, int stride, const WgradPlan &plan, bool out_f32, bool accumulate,
                       hipStream_t s, bool atomics) {
    // split-K accumulating into an f32 destination: every split adds its tile with atomics (unless
    // `atomics` is off: then partial tiles + the deterministic reduce, which adds into dw)
    const bool atomic_out = atomics && out_f32 && accumulate && plan.splits > 1;
    if (!conv_wgrad_supported(Cin, Cout, ks, stride)) throw std::invalid_argument("conv_wgrad: unsupported shape");
    if (plan.variant == kRowsVariant) {
        if (!rows_supported(Cin, Cout, ks, stride)) throw std::invalid_argument("conv_wgrad: rows variant needs 3x3/s1");
        const RGeo rg = make_rgeo(N, H, W, Cin, Cout, plan);
        wgrad_rows_kernel<2><<<rg.mtiles * rg.ntiles * rg.splits, 576, 0, s>>>(
            dy, x, part, dw, reinterpret_cast<const uint16_t *>(zero_page()), rg, out_f32, accumulate, atomic_out,
            rows_stagger(false));
        if (rg.splits > 1 && !atomic_out) {
            WGeo g{};
            g.C = Cin, g.K = Cout, g.mtiles = rg.mtiles, g.ntiles = rg.ntiles, g.taps = 9, g.tiles = rg.tiles;
            g.splits = rg.splits;
            const int64_t tot = static_cast<int64_t>(g.tiles) * 1024;
            int sgl = 0;
            while (sgl < 6 && (2 << sgl) <= g.splits && (tot << (sgl + 1)) <= int64_t(256) * 2048) ++sgl;
            const int64_t grid = (tot + (256 >> sgl) - 1) / (256 >> sgl);
            wgrad_reduce_kernel<1, 1><<<static_cast<int>(grid), 256, 0, s>>>(part, dw, g, out_f32, accumulate, sgl);
        }
        return;
    }
    const WGeo g = make_geo(N, H, W, Cin, Cout, ks, stride, plan);
    if (static_cast<int64_t>(g.P) * g.HW >= (int64_t(1) << 40) || g.P >= (1 << 23))
        throw std::invalid_argument("conv_wgrad: too many pixels for the 40-bit division");
    if (g.splits > 1 && !atomic_out && part == nullptr) throw std::invalid_argument("conv_wgrad: split-K needs the workspace");
    if (ks == 1) {
        if (stride == 1) launch_ks<1, 1>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else launch_ks<1, 2>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
    } else {
        if (stride == 1) launch_ks<3, 1>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else launch_ks<3, 2>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
    }
}

// ---- any KH x KW window, padding, channel counts % 8 (Inception-v3) -----------------------

bool conv_wgrad_rect_supported(int Cin, int Cout, int kh, int kw, int stride) {
    return Cin % 8 == 0 && Cout % 8 == 0 && Cin >= 16 && Cout >= 16 && (stride == 1 || stride == 2) && kh >= 1 &&
           kw >= 1 && kh * kw <= 49;
}

namespace {
// tile: 128 rows where the channel count reaches it (less zero padding otherwise)
int rect_variant(int Cin, int Cout) { return Cout >= 128 ? (Cin >= 128 ? 0 : 1) : (Cin >= 128 ? 2 : 3); }

WGeo make_rect_geo(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int stride, int variant) {
    WGeo g{};
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout;
    g.OH = (H + 2 * ph - kh) / stride + 1;
    g.OW = (W + 2 * pw - kw) / stride + 1;
    g.HW = g.OH * g.OW;
    g.P = N * g.HW;
    g.m_hw = magic40(g.HW);
    g.m_ow = magic40(g.OW);
    const Tile t = kTiles[variant];
    g.mtiles = (Cout + t.bm() - 1) / t.bm();
    g.ntiles = (Cin + t.bn() - 1) / t.bn();
    g.taps = kh * kw;
    g.tiles = g.mtiles * g.ntiles * g.taps;
    g.kwin = kw, g.ph = ph, g.pw = pw;
    return g;
}
}  // namespace

namespace {
// the row-image kernel's segments / tap groups for a stride-1 KH x KW window (xpieces > 25: unsupported)
RRGeo rows_rect_geo(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int ct = 64,
                    bool legacy = true, int stride = 1) {
    RRGeo g{};
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout, g.S = stride;
    g.OH = (H + 2 * ph - kh) / stride + 1, g.OW = (W + 2 * pw - kw) / stride + 1;
    g.KH = kh, g.KW = kw, g.ph = ph, g.pw = pw, g.taps = kh * kw;
    const int nwv = g.taps % 7 == 0 ? 7 : 9;
    g.tgroups = (g.taps + nwv - 1) / nwv;
    auto shape = [&](int L, int R) {
        g.L = L, g.R = R, g.spr = (g.OW + L - 1) / L, g.gpi = (g.OH + R - 1) / R;
        g.nseg = N * g.gpi * g.spr;
        g.XW = stride * (g.L - 1) + kw;
        g.xrows = (stride * (g.R - 1) + kh) * g.XW;
    };
    if (legacy) {
        if (g.OW >= 64) shape(64, 1);
        else shape(g.OW, 64 / g.OW);
    } else {
        // 64-byte rows: the R x L segment of 64 slots with the fewest staged rows (dy + image) in
        // total -- R > 1 on the wide maps too (Conv2d_2a's 109-wide rows: 16 x 4 stages 1.7 input
        // rows per output pixel where 64 x 1 stages 3.1)
        int64_t best = -1;
        int bl = 64, br = 1;
        for (int R = 1; R <= 64; ++R) {
            const int L = std::min(g.OW, 64 / R);
            if (L < 1 || (R > 1 && (R - 1) * L >= 64)) break;
            if (R > g.OH + 1) break;
            shape(L, R);
            if (g.xrows * 2 * ct > 25 * 1024) continue;
            const int64_t cost = static_cast<int64_t>(g.nseg) * (64 + g.xrows);
            if (best < 0 || cost < best) best = cost, bl = L, br = R;
        }
        shape(bl, br);
    }
    g.xpieces = (g.xrows * 2 * ct + 1023) / 1024;
    g.mtiles = (Cout + ct - 1) / ct, g.ntiles = (Cin + ct - 1) / ct;
    g.stage = 64 * 2 * ct + (legacy ? 26 : g.xpieces + 1) * 1024;
    g.tiles = g.mtiles * g.ntiles * g.taps;
    return g;
}
}  // namespace

bool conv_wgrad_rows_rect_supported(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw,
                                    int stride) {
    if ((stride != 1 && stride != 2) || kh * kw < 2 || !conv_wgrad_rect_supported(Cin, Cout, kh, kw, stride)) return false;
    if (H + 2 * ph - kh < 0 || W + 2 * pw - kw < 0) return false;
    if (stride == 1) return rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw).xpieces <= 25;
    // stride 2: the kRowsEx variants only (64-channel tiles bound the staged image)
    return rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, 64, false, 2).xpieces <= 25;
}

// Row-image variant per shape, from the Inception-v3 sweep (profiles/r5_inception_wgrad.md): 32-channel
// tiles (8) when both channel counts fit one; the 64-tile kernel as before (6) when both are
// multiples of 64; otherwise 64-channel tiles on the fewest-rows segments with a 4-stage ring (12) on
// the small maps (<= 32 x 32: few segments per workgroup, the ring's depth pays) when it fits in
// 96 KB, else a 3-stage ring (11: two workgroups per CU on the 54 x 54 / 109 x 109 maps)
int conv_wgrad_rows_rect_auto(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int stride) {
    if (Cin <= 32 && Cout <= 32) return 8;
    if (stride == 2) {
        // r5 stride-2 sweep: 25x25 96->96 34 us on 10 (MIOpen 50), 288->384 241 on 8 (tap-tiled 266,
        // MIOpen 324), 12x12 192->192 / 192->320 33 / 41 on 12 (MIOpen 29 / 41)
        if (Cin % 64 != 0 || Cout % 64 != 0) return (H * W <= 1024 && Cout <= 128) ? 10 : 8;
        return 12;
    }
    if (stride == 1 && Cin % 64 == 0 && Cout % 64 == 0) return kRowsVariant;
    const RRGeo rg = rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, 64, false, stride);
    return (H * W <= 1024 && 4 * rg.stage <= 96 * 1024) ? 12 : 11;
}

WgradPlan conv_wgrad_rect_plan(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int stride,
                               int variant) {
    WgradPlan pl;
    if (variant == 13) {
        if (!conv_wgrad_rows_rect_supported(N, H, W, Cin, Cout, kh, kw, ph, pw, stride))
            throw std::invalid_argument("conv_wgrad_rect: row-image variant unsupported for this shape");
        variant = conv_wgrad_rows_rect_auto(N, H, W, Cin, Cout, kh, kw, ph, pw, stride);
    }
    if (variant >= kRowsExFirst && variant <= kRowsExLast) {
        if (!conv_wgrad_rows_rect_supported(N, H, W, Cin, Cout, kh, kw, ph, pw, stride))
            throw std::invalid_argument("conv_wgrad_rect: row-image variant unsupported for this shape");
        const RowsEx vx = kRowsEx[variant - kRowsExFirst];
        const RRGeo rg = rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, vx.ct, false, stride);
        if (rg.xpieces > 25) throw std::invalid_argument("conv_wgrad_rect: image segment too large for this variant");
        pl.variant = variant;
        const int ct = rg.mtiles * rg.ntiles * rg.tgroups;
        // as many workgroups as fit at once: LDS ring per CU, <= 3 of 7-9 waves
        const int occ = std::max(1, std::min(3, 160 * 1024 / (vx.stages * rg.stage)));
        int splits = std::max(1, (256 * occ + ct / 2) / ct);
        splits = std::max(1, std::min(splits, std::max(1, rg.nseg / 4)));
        pl.kps = (rg.nseg + splits - 1) / splits;
        pl.splits = (rg.nseg + pl.kps - 1) / pl.kps;
        pl.ws_floats = pl.splits > 1 ? static_cast<int64_t>(pl.splits) * Cout * rg.taps * Cin : 0;
        return pl;
    }
    if (variant == kRowsVariant) {
        if (stride != 1 || !conv_wgrad_rows_rect_supported(N, H, W, Cin, Cout, kh, kw, ph, pw, stride))
            throw std::invalid_argument("conv_wgrad_rect: row-image variant unsupported for this shape");
        const RRGeo rg = rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw);
        pl.variant = variant;
        const int ct = rg.mtiles * rg.ntiles * rg.tgroups;
        // ~2 workgroups of 7-9 waves per CU, >= 4 segments per split
        int splits = std::max(1, (512 + ct / 2) / ct);
        splits = std::max(1, std::min(splits, std::max(1, rg.nseg / 4)));
        pl.kps = (rg.nseg + splits - 1) / splits;
        pl.splits = (rg.nseg + pl.kps - 1) / pl.kps;
        pl.ws_floats = pl.splits > 1 ? static_cast<int64_t>(pl.splits) * rg.tiles * 4096 : 0;
        return pl;
    }
    pl.variant = rect_variant(Cin, Cout);
    WGeo g = make_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, stride, pl.variant);
    const Tile t = kTiles[pl.variant];
    const int ksteps = (g.P + kBK - 1) / kBK;
    const int nw = t.wm * t.wn;
    int target = 256 * (nw >= 4 ? 1 : 2) * (g.taps > 1 ? 2 : 1);
    int splits = (target + g.tiles / 2) / g.tiles;
    splits = std::max(1, std::min(splits, ksteps / 4));
    splits = std::max(1, std::min(splits, ksteps));
    pl.kps = (ksteps + splits - 1) / splits;
    pl.splits = (ksteps + pl.kps - 1) / pl.kps;
    pl.ws_floats = pl.splits > 1 ? static_cast<int64_t>(pl.splits) * g.tiles * t.bm() * t.bn() : 0;
    return pl;
}

void launch_conv_wgrad_rect(const uint16_t *dy, const uint16_t *x, void *dw, float *part, int N, int H, int W,
                            int Cin, int Cout, int kh, int kw, int ph, int pw, int stride, const WgradPlan &plan,
                            bool out_f32, bool accumulate, hipStream_t s) {
    if (!conv_wgrad_rect_supported(Cin, Cout, kh, kw, stride)) throw std::invalid_argument("conv_wgrad_rect: unsupported");
    const bool atomic_out = out_f32 && accumulate && plan.splits > 1;
    if (plan.variant >= kRowsExFirst && plan.variant <= kRowsExLast) {
        if (!conv_wgrad_rows_rect_supported(N, H, W, Cin, Cout, kh, kw, ph, pw, stride))
            throw std::invalid_argument("conv_wgrad_rect: row-image variant unsupported for this shape");
        const RowsEx vx = kRowsEx[plan.variant - kRowsExFirst];
        RRGeo rg = rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, vx.ct, false, stride);
        rg.splits = plan.splits, rg.kps = plan.kps;
        if (rg.splits > 1 && !atomic_out && part == nullptr) throw std::invalid_argument("conv_wgrad_rect: needs the workspace");
        const int grid = rg.mtiles * rg.ntiles * rg.tgroups * rg.splits;
        const uint16_t *z = reinterpret_cast<const uint16_t *>(zero_page());
        const int lds = vx.stages * rg.stage;
        const bool t7 = rg.taps % 7 == 0;
        static bool attr_set[kRowsExLast - kRowsExFirst + 1][2] = {};  // per instantiation, once
        auto go = [&](auto kern, int nwv) {
            bool &done = attr_set[plan.variant - kRowsExFirst][t7 ? 1 : 0];
            if (!done) {
                (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                          160 * 1024);
                done = true;
            }
            kern<<<grid, 64 * nwv, lds, s>>>(dy, x, part, dw, z, rg, out_f32, accumulate, atomic_out, rows_stagger(true));
        };
        switch (plan.variant) {
            case 8: t7 ? go(wgrad_rows_rect_kernel<7, 2, 32, true>, 7) : go(wgrad_rows_rect_kernel<9, 2, 32, true>, 9); break;
            case 9: t7 ? go(wgrad_rows_rect_kernel<7, 3, 32, true>, 7) : go(wgrad_rows_rect_kernel<9, 3, 32, true>, 9); break;
            case 10: t7 ? go(wgrad_rows_rect_kernel<7, 4, 32, true>, 7) : go(wgrad_rows_rect_kernel<9, 4, 32, true>, 9); break;
            case 11: t7 ? go(wgrad_rows_rect_kernel<7, 3, 64, true>, 7) : go(wgrad_rows_rect_kernel<9, 3, 64, true>, 9); break;
            default: t7 ? go(wgrad_rows_rect_kernel<7, 4, 64, true>, 7) : go(wgrad_rows_rect_kernel<9, 4, 64, true>, 9); break;
        }
        if (rg.splits > 1 && !atomic_out) {
            const int64_t n = static_cast<int64_t>(Cout) * rg.taps * Cin;
            // split groups: up to 64, ~8 splits each, while >= 1,024 blocks of columns... or fewer
            int sgl = 0;
            while (sgl < 6 && (8 << sgl) < rg.splits && (n / 4) * (2 << sgl) <= int64_t(1024) * 256) ++sgl;
            const int cols = 256 >> sgl;
            wgrad_dense_reduce_kernel<<<static_cast<int>((n / 4 + cols - 1) / cols), 256, 0, s>>>(
                part, rg.splits, n, dw, out_f32, accumulate, sgl);
        }
        return;
    }
    if (plan.variant == kRowsVariant) {
        if (stride != 1 || !conv_wgrad_rows_rect_supported(N, H, W, Cin, Cout, kh, kw, ph, pw, stride))
            throw std::invalid_argument("conv_wgrad_rect: row-image variant unsupported for this shape");
        RRGeo rg = rows_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw);
        rg.splits = plan.splits, rg.kps = plan.kps;
        if (rg.splits > 1 && !atomic_out && part == nullptr) throw std::invalid_argument("conv_wgrad_rect: needs the workspace");
        const int grid = rg.mtiles * rg.ntiles * rg.tgroups * rg.splits;
        const uint16_t *z = reinterpret_cast<const uint16_t *>(zero_page());
        static const bool attr = [] {
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(wgrad_rows_rect_kernel<7, 2>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(wgrad_rows_rect_kernel<9, 2>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            return true;
        }();
        (void)attr;
        if (rg.taps % 7 == 0)
            wgrad_rows_rect_kernel<7, 2><<<grid, 64 * 7, 2 * rg.stage, s>>>(dy, x, part, dw, z, rg, out_f32, accumulate,
                                                                          atomic_out, rows_stagger(true));
        else
            wgrad_rows_rect_kernel<9, 2><<<grid, 64 * 9, 2 * rg.stage, s>>>(dy, x, part, dw, z, rg, out_f32, accumulate,
                                                                          atomic_out, rows_stagger(true));
        if (rg.splits > 1 && !atomic_out) {
            WGeo g{};
            g.C = Cin, g.K = Cout, g.mtiles = rg.mtiles, g.ntiles = rg.ntiles, g.taps = rg.taps, g.tiles = rg.tiles;
            g.splits = rg.splits;
            const int64_t tot = static_cast<int64_t>(g.tiles) * 1024;
            int sgl = 0;
            while (sgl < 6 && (2 << sgl) <= g.splits && (tot << (sgl + 1)) <= int64_t(256) * 2048) ++sgl;
            const int64_t rgrid = (tot + (256 >> sgl) - 1) / (256 >> sgl);
            wgrad_reduce_kernel<1, 1><<<static_cast<int>(rgrid), 256, 0, s>>>(part, dw, g, out_f32, accumulate, sgl);
        }
        return;
    }
    WGeo g = make_rect_geo(N, H, W, Cin, Cout, kh, kw, ph, pw, stride, plan.variant);
    g.splits = plan.splits;
    g.kps = plan.kps;
    if (static_cast<int64_t>(g.P) * g.HW >= (int64_t(1) << 40) || g.P >= (1 << 23))
        throw std::invalid_argument("conv_wgrad_rect: too many pixels for the 40-bit division");
    if (g.splits > 1 && !atomic_out && part == nullptr) throw std::invalid_argument("conv_wgrad_rect: needs the workspace");
    const bool k1 = kh == 1 && kw == 1 && ph == 0 && pw == 0, k3 = kh == 3 && kw == 3 && ph == 1 && pw == 1;
    if (stride == 1) {
        if (k1) launch_ks<1, 1>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else if (k3) launch_ks<3, 1>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else launch_ks<0, 1>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
    } else {
        if (k1) launch_ks<1, 2>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else if (k3) launch_ks<3, 2>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
        else launch_ks<0, 2>(dy, x, dw, part, g, plan.variant, out_f32, accumulate, atomic_out, s);
    }
}

}  // namespace kfk
