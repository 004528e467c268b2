// 3x3 (pad 1) and 1x1 (pad 0) convolutions, stride 1 or 2, NHWC bf16, as an implicit
// GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x32_bf16), for gfx950, with optional
// fused epilogues: BN batch statistics of the output, accumulate-into-destination.
//
//   y[m, co] = sum_{kh, kw, ci} x[n, oh*s + kh - 1, ow*s + kw - 1, ci] * w[co, kh, kw, ci]
//   GEMM: M = N*OH*OW output pixels, N = Cout, K = 9 * Cin (tap-major, channel-minor)
//
// Why: ResNet-50 spends ~6.3 ms of a 28.6 ms step in its 16 3x3 convolutions at
// ~450 TF/s through MIOpen/CK (profiles/README.md).  The K dimension of one
// tap is a run of Cin contiguous channels, so every A-tile row is a 128-byte
// segment of the input (or of a zero page at the padding border): the im2col
// is done by the per-lane source address of global_load_lds, never in memory.
//
// Tiling: block = 4 waves (256 threads), wave tile 64x64 (4x4 MFMA 16x16
// tiles, 64 accumulator VGPRs), block tile 128x128 (2x2 waves) or 256x64 (4x1,
// for Cout = 64), BK = 64 channels of one tap per K-step.  A and B tiles are
// staged global->LDS with 16-byte global_load_lds (no VGPR round trip),
// double-buffered, with an XOR swizzle of the 16-byte chunk index by the row
// (chunk ^ (row & 7)) applied on the source address and on the ds_read, so the
// 16 rows a ds_read_b128 touches spread over 8 chunk positions.  Blocks are
// remapped XCD-contiguously (consecutive tiles share input halo rows in L2).
//
// The same kernel computes the stride-1 data gradient: dx = conv3x3(dy, w')
// with w'[ci, kh, kw, co] = w[co, 2-kh, 2-kw, ci] (conv3x3_flip_weight).
//
// This header holds the kernel template and its launch helpers; the instantiations are spread over
// conv.hip (dispatch, weight flips), conv_k1.hip / conv_k3.hip (square windows), conv_rect.hip,
// conv_gemm.hip and conv_s2.hip, so the ~480 kernel instances build in parallel.
#pragma once

#include "bn_fin.hpp"
#include "common.hpp"
#include "kernels.hpp"

#include <cstdlib>
#include <stdexcept>

namespace kfk {

struct Geo {
    int N, H, W, C, OH, OW, K, stride;
    int M;       // N*OH*OW
    int mtiles;  // ceil(M / BM)
    int ntiles;  // K / BN
    // strided data gradient as parity phases (launch_conv_dgrad_s2):
    int wtaps;   // taps per weight row (B row stride = wtaps * C)
    int tapmap;  // -1: tap t reads weight tap t; else weight tap of tap t = nibble t
    int scat;    // 1: output (n, a, b) of the OH x OW phase grid -> pixel (2a + pr, 2b + pc) of a dh x dw image
    int pr, pc;
    int dh, dw;  // scat: the data-gradient image (2OH x 2OW for an even input)
    int ph, pw;  // zero padding (rows, columns)
    int stagger;  // 1: the upper half of 8 waves issues its LDS-DMA staging before its fragment reads
    int prio;     // 1: the upper (second-dispatched) wave half runs at s_setprio 1
};

const void *zero_page();
void check_buf_extent(const Geo &g);
int conv_tile_rules();
int conv_t224();
int conv_stagger();
int conv_prio();
// the square-window launchers (conv_k1.hip / conv_k3.hip): tile variant < 0 = the per-shape default
void launch_conv_k1(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s, int variant);
void launch_conv_k3(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s, int variant);

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__device__ __forceinline__ int wm_of(int wave, int wn) { return wave / wn; }


__device__ __forceinline__ void unpack_bf16x8(const uint4 &v, float (&f)[8]) {
    const uint32_t *u = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(u[k] << 16);
        f[2 * k + 1] = __uint_as_float(u[k] & 0xffff0000u);
    }
}

constexpr int kBK = 64;              // channels per K-step
constexpr int kRowBytes = kBK * 2;   // 128 B per staged row

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ (row & 7); }

// LDS byte address of (row, 16-B chunk) in a staged tile image.
__device__ __forceinline__ int img_off(int row, int chunk) { return row * kRowBytes + (swz_chunk(row, chunk) << 4); }



template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Buffer-resource LDS-DMA staging in conv_kernel (KUNGFU_CONV_BUFLD): num_records = 2 GiB, so
// the out-of-range offset kBufOOB returns zeros; dword 3 = the CDNA raw-buffer format word.
#ifndef KUNGFU_CONV_BUFLD
#define KUNGFU_CONV_BUFLD 1
#endif
constexpr uint32_t kBufOOB = 0x80000000u;
constexpr int kBufFlags = 0x00020000;

__device__ __forceinline__ __attribute__((address_space(3))) void *lds_ptr(uint8_t *p) {
    return (__attribute__((address_space(3))) void *)(p);
}

// In-launch BN finalize (kernels.hpp BNFin): called by every workgroup after its slot atomics.
// Completion-ordered hand-off (MI355X_MICROARCH.md, inter-workgroup visibility: "the workgroup whose
// add came last, told by the value its add returned", sc1 loads of the handed-off words): each wave
// waits for its own atomics (vmcnt counts them), the workgroup joins a barrier, one lane arrives on
// its shard counter (blockIdx % 8) and the last arriver of a shard on the top counter; the last of
// those folds every channel's slots with sc1 loads (the f64 adds were performed at the memory side,
// no L2 holds them) and re-zeroes slots and counters with sc1 stores for the next launch.  No fence:
// the outputs are read by later kernels only.
// `red` (the kernel's own LDS, free once the statistics are out) holds red_doubles doubles and then
// the flag word: a separate __shared__ variable would push the 256x64 tiles' 80 KB past the
// two-workgroups-per-CU LDS budget.
__device__ __forceinline__ void bn_finalize_last(const BNFin *__restrict__ fp, double *sums, int C, int nwg, int orig,
                                                 int tid, int nt, double *red, int red_doubles) {
    int &s_last = *reinterpret_cast<int *>(red + red_doubles);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        const int shard = orig & 7;
        const int nsh = nwg < 8 ? nwg : 8;
        const unsigned nin = static_cast<unsigned>((nwg - shard + 7) / 8);
        int last = 0;
        unsigned *arrive = fp->arrive;
        const unsigned o = __hip_atomic_fetch_add(arrive + shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (o == nin - 1) {
            const unsigned o2 = __hip_atomic_fetch_add(arrive + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = o2 == static_cast<unsigned>(nsh - 1);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    // channel chunks staged through LDS (the main loop's buffers are free): every slot word of the
    // chunk loaded once (sc1, all independent) and re-zeroed, then each channel folded in slot order
    // k = 0..15 -- the order of bn_sums_finalize / bn_bwd_finalize_sums, so bit-identical to them
    constexpr int KS2 = 2 * kStatSlots;
    const int chunk = red_doubles / KS2 < C ? red_doubles / KS2 : C;
    for (int c0 = 0; c0 < C; c0 += chunk) {
        const int ch = C - c0 < chunk ? C - c0 : chunk;
        const int items = KS2 * ch;
#pragma unroll 8
        for (int it = tid; it < items; it += nt) {
            const int kw = it / ch, cc = it - kw * ch;  // kw = 2 k + which
            double *a = sums + static_cast<int64_t>(kw) * C + c0 + cc;
            red[it] = __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(a, 0.0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        for (int cc = tid; cc < ch; cc += nt) {
            double s0 = 0, s1 = 0;
            for (int k = 0; k < kStatSlots; ++k) {
                s0 += red[(2 * k) * ch + cc];
                s1 += red[(2 * k + 1) * ch + cc];
            }
            const int c = c0 + cc;
            if (fp->mode == 1)
                bn_fin_fwd_channel_p(c, C, s0, s1, fp->rows, fp->gamma, fp->beta, fp->mean, fp->invstd, fp->run_mean,
                                   fp->run_var, fp->momentum, fp->eps, fp->coef);
            else
                bn_fin_bwd_channel_p(c, C, s0, s1, fp->rows, fp->gamma, fp->mean, fp->invstd, fp->dgamma, fp->dbeta,
                                   fp->coef, fp->training != 0);
        }
        __syncthreads();
    }
    if (tid < 9) __hip_atomic_store(fp->arrive + tid, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (tid == 0 && fp->mode == 1 && fp->num_batches) fp->num_batches[0] += 1;
}

// The same finalize as a launch of its own (a non-persistent statistics launch: there every
// workgroup would hold its CU through the wait for its atomics).
__global__ void bn_fin_desc_kernel(const BNFin *__restrict__ fp, double *sums, int C) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double v0[kStatSlots], v1[kStatSlots];
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        v0[k] = sums[k * 2 * C + c];
        v1[k] = sums[k * 2 * C + C + c];
    }
    double s0 = 0, s1 = 0;
#pragma unroll
    for (int k = 0; k < kStatSlots; ++k) {
        s0 += v0[k];
        s1 += v1[k];
        sums[k * 2 * C + c] = 0.0;
        sums[k * 2 * C + C + c] = 0.0;
    }
    if (fp->mode == 1) {
        if (c == 0 && fp->num_batches) fp->num_batches[0] += 1;
        bn_fin_fwd_channel_p(c, C, s0, s1, fp->rows, fp->gamma, fp->beta, fp->mean, fp->invstd, fp->run_mean,
                           fp->run_var, fp->momentum, fp->eps, fp->coef);
    } else {
        bn_fin_bwd_channel_p(c, C, s0, s1, fp->rows, fp->gamma, fp->mean, fp->invstd, fp->dgamma, fp->dbeta, fp->coef,
                           fp->training != 0);
    }
}

// The epilogue of one output tile (shared by conv_kernel and conv_rows_kernel): the f32
// accumulators (C^T fragments: lane -> pixel row lane & 15, channels 4 (lane >> 4) + r) go through
// the LDS as a bf16 tile, then 16-byte row stores with the fused epilogue applied on the way; the
// per-channel statistics accumulate in s1 / s2 (this thread's fixed 8-channel group).  The caller
// has waited for its LDS-DMA and passed a barrier (the LDS is reused).
template <int WM, int WN, int TM, int TN, int EPI>
__device__ __forceinline__ void conv_store_tile(const f32x4 (&acc)[TM][TN], uint8_t *lds, uint16_t *__restrict__ y,
                                                const Geo &g, const EpiArgs &ea, int m0, int n0, int tid,
                                                float (&s1)[8], float (&s2)[8]) {
    constexpr int WTM = 16 * TM, WTN = 16 * TN;
    constexpr int BM = WTM * WM, BN = WTN * WN, NT = 64 * WM * WN;
    constexpr int CROW = BN * 2 + 16;  // padded bytes per C row of the epilogue tile
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate | kEpiGeluGrad)) != 0;
    constexpr bool GATE = (EPI & kEpiGate) != 0;
    constexpr bool GELUG = (EPI & kEpiGeluGrad) != 0;
    constexpr bool BIAS = (EPI & (kEpiBiasRelu | kEpiBias)) != 0;
    constexpr int NSUM = (GATE || GELUG) ? 1 : 2;  // the gates need sum(y) only (a bias gradient)
    constexpr int VPR = BN / 8;  // 16-byte vectors per C row
    constexpr int GROUPS = NT / VPR;
    constexpr int ITER = BM * VPR / NT;  // 16-byte output vectors per thread per tile
    static_assert(ITER * NT == BM * VPR, "whole store iterations");
    constexpr bool LD_OLD = (EPI & kEpiAccum) != 0;
    constexpr bool LD_BX = GATE || GELUG || (EPI & (kEpiBwdCoef | kEpiBwdBits)) != 0;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int cv = tid % (BN / 8);  // the epilogue's fixed 8-channel group of this thread
    (void)STATS, (void)NSUM, (void)GROUPS, (void)LD_OLD, (void)LD_BX, (void)lane, (void)wm, (void)wn, (void)CROW,
        (void)BIAS, (void)ITER;

    // ---- epilogue: bf16 tile through LDS, then 16-byte row stores
    // C^T map (16x16): pixel row = lane & 15, channel col = (lane >> 4) * 4 + r.
    float bcol[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            bcol[j][r] = 0.f;
            if constexpr (BIAS) {
                const int c = n0 + wn * WTN + j * 16 + (lane >> 4) * 4 + r;
                if (c < g.K) bcol[j][r] = bf16_to_f32(ea.bias[c]);
            }
        }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = wm * WTM + i * 16 + (lane & 15);
            const int col = wn * WTN + j * 16 + (lane >> 4) * 4;
            float v4[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = acc[i][j][r];
                if constexpr (BIAS) v += bcol[j][r];
                if constexpr ((EPI & kEpiBiasRelu) != 0) v = !(v <= 0.f) ? v : 0.f;  // NaN stays NaN (torch.relu)
                v4[r] = v;
            }
            // (integer rounding: v_cvt_pk_bf16_f32 here measured ResNet-50 20.24 -> 20.72 ms/step, the 56 x 56
            // 3x3 conv 99 -> 163 us, r6t25 / profiles/r6_conv3x3_rows.md)
            *reinterpret_cast<uint2 *>(lds + row * CROW + col * 2) =
                make_uint2(f32_to_bf16(v4[0]) | (static_cast<uint32_t>(f32_to_bf16(v4[1])) << 16),
                           f32_to_bf16(v4[2]) | (static_cast<uint32_t>(f32_to_bf16(v4[3])) << 16));
        }
    __syncthreads();
    // Store loop: thread -> 16-byte vectors (row, cv) with a FIXED 8-channel group cv (NT is a
    // multiple of VPR), so per-channel statistics accumulate in registers across its rows.
    static_assert(NT % VPR == 0, "fixed channel group per thread");
    // The global reads of the epilogue (old value, BN input, masks) of U rows are all issued
    // before any of them is consumed: one load round trip per U rows instead of per row (the
    // loop is otherwise a chain of dependent HBM latencies -- the stores to y may alias later
    // reads as far as the compiler knows).
    // U rows in flight (none to batch without global reads; 2 for the BN-coefficient epilogue on
    // the 256x256 tile, whose 16 coefficient registers would otherwise spill).  (Round 6: issuing
    // every row's epilogue reads behind the prologue staging instead -- operands in registers when
    // the K loop ends -- took the 4-wave tiles to one wave per SIMD and spilled the 8-wave ones:
    // ResNet-50 20.40 -> 21.45 ms/step, profiles/r6_conv_pmc.md.)
    constexpr int U0 = !(LD_OLD || LD_BX) ? 1 : ((EPI & kEpiBwdCoef) && TM * TN >= 32) ? 2 : (ITER >= 4 ? 4 : ITER);
    constexpr int U = ITER % U0 == 0 ? U0 : (ITER % 2 == 0 ? 2 : 1);  // whole groups (ITER = 14 on the 224-row tile)
    static_assert(ITER % U == 0, "whole row groups");
    const bool col_ok = n0 + cv * 8 < g.K;  // this thread's 8 channels exist (Cout % BN != 0)
    float sc[8], sh[8];  // bwd coef: the forward BN's [scale; shift] of this thread's 8 channels
    if constexpr ((EPI & kEpiBwdCoef) != 0) {
        if (col_ok)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            sc[k] = ea.fcoef[n0 + cv * 8 + k];
            sh[k] = ea.fcoef[g.K + n0 + cv * 8 + k];
        }
    }
    for (int it0 = 0; it0 < ITER; it0 += U) {
        uint4 val[U], old[U], bxv[U];
        uint32_t amb[U], bmb[U];
        int64_t ee[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int v = tid + (it0 + u) * NT;
            const int row = v / VPR;
            const int m = m0 + row;
            ok[u] = m < g.M && col_ok;
            int pix = m;
            if (g.scat) {
                const int t = m / g.OW, ow = m - t * g.OW;
                const int n = t / g.OH, a = t - n * g.OH;
                pix = (n * g.dh + 2 * a + g.pr) * g.dw + 2 * ow + g.pc;
            }
            const int64_t e = static_cast<int64_t>(pix) * g.K + n0 + cv * 8;
            ee[u] = e;
            val[u] = *reinterpret_cast<const uint4 *>(lds + row * CROW + cv * 16);
            old[u] = bxv[u] = make_uint4(0u, 0u, 0u, 0u);
            amb[u] = 0u;
            bmb[u] = 0xffu;
            if (ok[u]) {
                if constexpr (LD_OLD) {
                    bool here = true;
                    if constexpr ((EPI & kEpiAccEven) != 0) {
                        // only the even pixels hold a partial sum (a stride-2 1x1 data gradient)
                        const int t = m / g.OW, ow = m - t * g.OW;
                        here = ((ow | (t % g.OH)) & 1) == 0;
                    }
                    if (here) old[u] = *reinterpret_cast<const uint4 *>(y + e);
                    if constexpr ((EPI & kEpiAccMask) != 0) amb[u] = ea.amask[e >> 3];  // 8 channels, 8-aligned e
                }
                if constexpr (LD_BX) bxv[u] = *reinterpret_cast<const uint4 *>(ea.bx + e);
                if constexpr ((EPI & kEpiBwdBits) != 0) bmb[u] = ea.bmask[e >> 3];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            uint4 v = val[u];
            if constexpr (LD_OLD) {
                uint4 o0 = old[u];
                if constexpr ((EPI & kEpiAccMask) != 0) {
                    const uint32_t mb = amb[u];
                    uint32_t *ow = reinterpret_cast<uint32_t *>(&o0);
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        ow[k] &= (((mb >> (2 * k)) & 1u) ? 0xffffu : 0u) | (((mb >> (2 * k + 1)) & 1u) ? 0xffff0000u : 0u);
                }
                const uint32_t *a = reinterpret_cast<const uint32_t *>(&v);
                const uint32_t *b = reinterpret_cast<const uint32_t *>(&o0);
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float lo = bf16_to_f32(static_cast<uint16_t>(a[k] & 0xffffu)) +
                                     bf16_to_f32(static_cast<uint16_t>(b[k] & 0xffffu));
                    const float hi = bf16_to_f32(static_cast<uint16_t>(a[k] >> 16)) +
                                     bf16_to_f32(static_cast<uint16_t>(b[k] >> 16));
                    o[k] = pack_bf16x2(lo, hi);
                }
                v = make_uint4(o[0], o[1], o[2], o[3]);
            }
            if constexpr (GATE) {
                // gradient of a ReLU output: keep y where bx > 0 (NaN passes), sum the kept values
                const uint32_t *bw = reinterpret_cast<const uint32_t *>(&bxv[u]);
                uint32_t *vw = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t keep = (!(__uint_as_float(bw[k] << 16) <= 0.f) ? 0xffffu : 0u) |
                                          (!(__uint_as_float(bw[k] & 0xffff0000u) <= 0.f) ? 0xffff0000u : 0u);
                    vw[k] &= keep;
                }
            }
            if constexpr (GELUG) {
                // gradient of gelu(u): dy * (Phi(u) + u * phi(u)), torch's GeluBackward in f32
                float f[8], uf[8];
                unpack_bf16x8(v, f);
                unpack_bf16x8(bxv[u], uf);
                uint32_t *vw = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float d[2];
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const float t = uf[2 * k + h];
                        const float cdf = 0.5f * (1.f + erff(t * 0.70710678118654752f));
                        const float pdf = __expf(-0.5f * t * t) * 0.39894228040143268f;
                        d[h] = f[2 * k + h] * (cdf + t * pdf);
                    }
                    vw[k] = pack_bf16x2(d[0], d[1]);
                }
            }
            *reinterpret_cast<uint4 *>(y + ee[u]) = v;
            if constexpr (STATS) {
                float f[8];
                unpack_bf16x8(v, f);
                if constexpr (GATE || GELUG) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) s1[k] += f[k];
                } else if constexpr ((EPI & kEpiFwdStats) != 0) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        s1[k] += f[k];
                        s2[k] += f[k] * f[k];
                    }
                } else {
                    // BN backward sums of the BN whose input is ea.bx:
                    //   dz = grad * relu'(.) ; s1 += dz ; s2 += dz * x
                    float xv[8];
                    unpack_bf16x8(bxv[u], xv);
                    const uint32_t mbits = bmb[u];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        bool on;
                        if constexpr ((EPI & kEpiBwdBits) != 0) on = (mbits >> k) & 1u;
                        else on = xv[k] * sc[k] + sh[k] > 0.f;
                        const float dz = on ? f[k] : 0.f;
                        s1[k] += dz;
                        s2[k] += dz * xv[k];
                    }
                }
            }
        }
    }
}

// Per-channel statistics of a workgroup (s1 / s2 of every thread) -> f64 atomics into stats slot
// `slot_sel % kStatSlots`, then the optional in-launch finalize.
template <int WM, int WN, int TM, int TN, int EPI, int LDS_BYTES>
__device__ __forceinline__ void conv_stats_flush(uint8_t *lds, const Geo &g, const EpiArgs &ea, int n0, int tid,
                                                 const float (&s1)[8], const float (&s2)[8], int slot_sel, int nwg,
                                                 int orig) {
    constexpr int WTM = 16 * TM, WTN = 16 * TN;
    constexpr int BM = WTM * WM, BN = WTN * WN, NT = 64 * WM * WN;
    constexpr int CROW = BN * 2 + 16;  // padded bytes per C row of the epilogue tile
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate | kEpiGeluGrad)) != 0;
    constexpr bool GATE = (EPI & kEpiGate) != 0;
    constexpr bool GELUG = (EPI & kEpiGeluGrad) != 0;
    constexpr bool BIAS = (EPI & (kEpiBiasRelu | kEpiBias)) != 0;
    constexpr int NSUM = (GATE || GELUG) ? 1 : 2;  // the gates need sum(y) only (a bias gradient)
    constexpr int VPR = BN / 8;  // 16-byte vectors per C row
    constexpr int GROUPS = NT / VPR;
    constexpr int ITER = BM * VPR / NT;  // 16-byte output vectors per thread per tile
    static_assert(ITER * NT == BM * VPR, "whole store iterations");
    constexpr bool LD_OLD = (EPI & kEpiAccum) != 0;
    constexpr bool LD_BX = GATE || GELUG || (EPI & (kEpiBwdCoef | kEpiBwdBits)) != 0;
    const int lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const int cv = tid % (BN / 8);  // the epilogue's fixed 8-channel group of this thread
    (void)STATS, (void)NSUM, (void)GROUPS, (void)LD_OLD, (void)LD_BX, (void)lane, (void)wm, (void)wn, (void)CROW,
        (void)BIAS, (void)ITER;
    {
        // reduce the NT / VPR threads of each channel group, then f64 atomics into a slot
        float *red = reinterpret_cast<float *>(lds);
        __syncthreads();
        const int grp = tid / VPR;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            red[grp * BN + cv * 8 + k] = s1[k];
            if constexpr (NSUM == 2) red[(GROUPS + grp) * BN + cv * 8 + k] = s2[k];
        }
        __syncthreads();
        for (int col = tid; col < BN; col += NT) {
            double t1 = 0, t2 = 0;
#pragma unroll 4
            for (int p = 0; p < GROUPS; ++p) {
                t1 += red[p * BN + col];
                if constexpr (NSUM == 2) t2 += red[(GROUPS + p) * BN + col];
            }
            double *sl = ea.stats + (slot_sel % kStatSlots) * 2 * g.K;  // spread atomics over slots
            if (n0 + col < g.K) {
                atomicAdd(sl + n0 + col, t1);
                if constexpr (NSUM == 2) atomicAdd(sl + g.K + n0 + col, t2);
            }
        }
        if constexpr (NSUM == 2) {
            if (ea.fin != nullptr)
                bn_finalize_last(ea.fin, ea.stats, g.K, nwg, orig, tid, NT, reinterpret_cast<double *>(lds),
                                 LDS_BYTES / 8 - 2);
        }
    }
}

// WM x WN waves (wave tile 64x64), STAGES-deep global_load_lds ring.
// KS = 3 or 1: square window; KS = 0xHW (>= 16): an H x W window (Inception's 1x7 / 7x1 / 1x3 /
// 3x1 / 5x5, and the parity phases of a stride-2 3x3 data gradient, launch_conv_dgrad_s2).  The
// zero padding is g.ph / g.pw (out-of-range taps read the zero page).  EPI flags (kernels.hpp ConvEpi):
//   kEpiAccum     y += conv (accumulate into the existing bf16 tensor, a residual gradient);
//   kEpiFwdStats  per-channel sum / sum-of-squares of the bf16 outputs (the following BN's
//                 batch statistics) -> f64 atomics into ea.stats[slot][2][K];
//   kEpiBwdCoef / kEpiBwdBits  the output is the gradient of a BN(+ReLU) output whose input
//                 is ea.bx: sum(dz) and sum(dz * x) with dz = grad * relu' from the forward
//                 coefficients ea.fcoef (recomputed) or from the 1-bit mask ea.bmask.
// PERSIST: the grid is smaller than the tile count; each block keeps ONE n-tile and walks
// m-tiles mt0, mt0 + mstride, ... -- its per-channel statistics accumulate in registers
// across all of them and reach the f64 slots with ONE set of atomics per block (instead of
// one per tile: 3.2 M f64 atomics for a 56x56 64->256 conv at batch 256).
template <int KS, int WM, int WN, int STAGES, int EPI, int TM = 4, int TN = 4, bool PERSIST = false>
__global__ __launch_bounds__(64 * WM * WN) void conv_kernel(const uint16_t *__restrict__ x,
                                                            const uint16_t *__restrict__ w,
                                                            uint16_t *__restrict__ y,
                                                            const uint16_t *__restrict__ zero, Geo g,
                                                            EpiArgs ea) {
    // wave tile (16*TM) x (16*TN): TM x TN accumulators of one 16x16x32 MFMA each
    constexpr int WTM = 16 * TM, WTN = 16 * TN;
    constexpr int BM = WTM * WM, BN = WTN * WN, NW = WM * WN, NT = 64 * NW;
    constexpr int KH = KS >= 16 ? (KS >> 4) : KS, KW = KS >= 16 ? (KS & 15) : KS;
    constexpr int TAPS = KH * KW;
    constexpr int A_BYTES = BM * kRowBytes, B_BYTES = BN * kRowBytes;
    constexpr int STAGE = A_BYTES + B_BYTES;
    // A pieces (8 rows each): A_INST per wave; when BM / 8 is not a multiple of the wave count (the
    // 224-row tile) the pieces interleave over the waves (piece j * NW + wave) and the last round is
    // partial -- per-wave load counts then differ, so only the 2-stage ring (vmcnt(0) waits) allows it
    constexpr int A_PIECES = BM / 8;
    constexpr int A_INST = (A_PIECES + NW - 1) / NW;  // glds instructions per wave per A tile (at most)
    constexpr bool A_EVEN = A_INST * NW == A_PIECES;
    constexpr int B_INST = BN / 8 / NW;
    constexpr int LOADS = A_INST + B_INST;
    static_assert(A_INST >= 1 && B_INST >= 1 && A_PIECES * 8 == BM && B_INST * NW * 8 == BN, "tile split");
    static_assert(A_EVEN || STAGES == 2, "uneven A split needs the 2-stage ring");
    constexpr int CROW = BN * 2 + 16;  // padded bytes per C row of the epilogue tile
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate | kEpiGeluGrad)) != 0;
    constexpr bool GATE = (EPI & kEpiGate) != 0;
    constexpr bool GELUG = (EPI & kEpiGeluGrad) != 0;
    constexpr bool BIAS = (EPI & (kEpiBiasRelu | kEpiBias)) != 0;
    constexpr int NSUM = (GATE || GELUG) ? 1 : 2;  // the gates need sum(y) only (a bias gradient)
    constexpr int VPR = BN / 8;  // 16-byte vectors per C row
    constexpr int GROUPS = NT / VPR;
    constexpr int ITER = BM * VPR / NT;  // 16-byte output vectors per thread per tile
    static_assert(ITER * NT == BM * VPR, "whole store iterations");
    constexpr bool LD_OLD = (EPI & kEpiAccum) != 0;
    constexpr bool LD_BX = GATE || GELUG || (EPI & (kEpiBwdCoef | kEpiBwdBits)) != 0;
    // the statistics reduction reuses the C tile's LDS once the last tile is stored
    constexpr int RED_BYTES = STATS ? NSUM * GROUPS * BN * 4 : 0;
    constexpr int EPI_BYTES = BM * CROW > RED_BYTES ? BM * CROW : RED_BYTES;
    constexpr int LDS_BYTES = STAGES * STAGE > EPI_BYTES ? STAGES * STAGE : EPI_BYTES;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware bijective remap: blocks sharing an XCD get consecutive tile ids.
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int mt_first = wg / g.ntiles, nt = wg - mt_first * g.ntiles;
    const int n0 = nt * BN;
    const int mstride = PERSIST ? nwg / g.ntiles : g.mtiles;  // nwg % ntiles == 0 when persistent
    const int cv = tid % (BN / 8);  // the epilogue's fixed 8-channel group of this thread
    float s1[8], s2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
    int mt_last = mt_first;
    for (int mt = mt_first; mt < g.mtiles; mt += mstride) {
    mt_last = mt;
    const int m0 = mt * BM;
    if (mt != mt_first) __syncthreads();  // every thread is done with the previous tile's LDS

    // ---- per-lane staging descriptors (fixed for the whole K loop)
    // lane l of a glds instruction writes image bytes [l*16, l*16+16) of its
    // 8-row slab: row = l/8, image chunk = l%8 -> logical chunk (l%8)^(l/8).
    // A rows: 32-bit element offset of the tap-(0,0) input pixel (linear in the
    // tap: + (kh*W + kw)*C) and a 9-bit in-bounds mask per row.
    const int srow = lane >> 3;
    const int schunk = (lane & 7) ^ srow;
    int a_off[A_INST];
    uint32_t a_ok[A_INST];
#pragma unroll
    for (int j = 0; j < A_INST; ++j) {
        const int piece = A_EVEN ? wave * A_INST + j : j * NW + wave;
        const int r = piece * 8 + srow;
        const int m = m0 + r;
        a_off[j] = 0;
        a_ok[j] = 0;
        if (m < g.M && piece < A_PIECES) {
            const int ow = m % g.OW, t = m / g.OW, oh = t % g.OH, n = t / g.OH;
            const int ih0 = oh * g.stride - g.ph, iw0 = ow * g.stride - g.pw;
            a_off[j] = ((n * g.H + ih0) * g.W + iw0) * g.C + schunk * 8;
            uint32_t ok = 0;
#pragma unroll
            for (int kh = 0; kh < KH; ++kh)
#pragma unroll
                for (int kw = 0; kw < KW; ++kw)
                    if (static_cast<unsigned>(ih0 + kh) < static_cast<unsigned>(g.H) &&
                        static_cast<unsigned>(iw0 + kw) < static_cast<unsigned>(g.W))
                        ok |= 1u << (kh * KW + kw);
            a_ok[j] = ok;
        }
    }
    // Channel counts that are not multiples of the tile (Inception's 48, 80, 96, 160, ...): the
    // K-step's 8-channel chunks past Cin and the B rows past Cout read the zero page.
    int b_off[B_INST];
    uint32_t b_ok = 0;
#pragma unroll
    for (int j = 0; j < B_INST; ++j) {
        const int r = (wave * B_INST + j) * 8 + srow;
        b_off[j] = (n0 + r) * g.wtaps * g.C + schunk * 8;
        if (n0 + r < g.K) b_ok |= 1u << j;
    }
    const int csteps = (g.C + kBK - 1) / kBK;
    const int ksteps = TAPS * csteps;
#if KUNGFU_CONV_BUFLD
    // LDS-DMA through buffer resources: 32-bit byte offsets, out-of-range lanes (padding taps,
    // channel chunks past Cin, B rows past Cout) get offset kBufOOB >= num_records and read
    // zeros -- no 64-bit per-lane addresses, no zero-page select (the launcher checks that x and
    // w are below 2 GiB).
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(x), 0, static_cast<int>(kBufOOB), kBufFlags);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(w), 0, static_cast<int>(kBufOOB), kBufFlags);
#endif
    auto stage = [&](int ks, int buf) {
        const int tap = ks / csteps, cc = ks - tap * csteps;
        const int kh = tap / KW, kw = tap - kh * KW;
        const int toff = (kh * g.W + kw) * g.C + cc * kBK;  // wave-uniform
        const int wtap = g.tapmap < 0 ? tap : (g.tapmap >> (4 * tap)) & 15;
        const bool cin_ok = cc * kBK + schunk * 8 < g.C;
        uint8_t *abase = lds + buf * STAGE;
        uint8_t *bbase = abase + A_BYTES;
#pragma unroll
        for (int j = 0; j < A_INST; ++j) {
            const int piece = A_EVEN ? wave * A_INST + j : j * NW + wave;
            if (!A_EVEN && piece >= A_PIECES) break;  // wave-uniform
            const bool ok = ((a_ok[j] >> tap) & 1u) && cin_ok;
#if KUNGFU_CONV_BUFLD
            const uint32_t vo = ok ? static_cast<uint32_t>(a_off[j] + toff) * 2u : kBufOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, lds_ptr(abase + piece * 1024), 16, vo, 0, 0, 0);
#else
            const uint16_t *src = ok ? x + static_cast<uint32_t>(a_off[j] + toff) : zero;
            __builtin_amdgcn_global_load_lds(src, abase + piece * 1024, 16, 0, 0);
#endif
        }
#pragma unroll
        for (int j = 0; j < B_INST; ++j) {
            const bool ok = ((b_ok >> j) & 1u) && cin_ok;
#if KUNGFU_CONV_BUFLD
            const uint32_t vo = ok ? static_cast<uint32_t>(b_off[j] + wtap * g.C + cc * kBK) * 2u : kBufOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, lds_ptr(bbase + (wave * B_INST + j) * 1024), 16, vo, 0, 0,
                                                     0);
#else
            const uint16_t *src = ok ? w + static_cast<uint32_t>(b_off[j] + wtap * g.C + cc * kBK) : zero;
            __builtin_amdgcn_global_load_lds(src, bbase + (wave * B_INST + j) * 1024, 16, 0, 0);
#endif
        }
    };

    const int wm = wave / WN, wn = wave % WN;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // transposed product (MFMA A operand = the weight fragment): acc[i][j] holds C^T of block (i, j),
    // lane -> output pixel (lane & 15), 4 consecutive output channels 4 (lane >> 4) + r -- one 8-byte
    // LDS store per block in the epilogue instead of four 2-byte ones
    auto mfma_block = [&](const bf16x8 (&af)[TM], const bf16x8 (&bfr)[TN]) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    };

    // prologue: STAGES-1 tiles in flight
#pragma unroll
    for (int p = 0; p < STAGES - 1; ++p)
        if (p < ksteps) stage(p, p);
    int buf = 0;
    // g.stagger 1: the upper wave half stages before its fragment reads; 2: after its second MFMA cluster
    const bool upper = NW >= 8 && ((wave >> 2) & 1);
    const bool early = g.stagger == 1 && upper, late = g.stagger == 2 && upper;
    if (g.prio && upper) __builtin_amdgcn_s_setprio(1);
    for (int ks = 0; ks < ksteps; ++ks) {
        // tile ks landed (this wave's loads); later tiles may stay in flight
        if (ks + STAGES - 1 <= ksteps) wait_vmcnt<LOADS * (STAGES - 2)>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // raw barrier: keeps the other tiles' LDS-DMA in flight
        __builtin_amdgcn_sched_barrier(0);
        if (early && ks + STAGES - 1 < ksteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *abase = lds + buf * STAGE;
        const uint8_t *bbase = abase + A_BYTES;
        // all 16 fragments of the K-step issued up front (substep 1 lands while
        // substep 0's MFMAs run)
        bf16x8 af0[TM], bf0[TN], af1[TM], bf1[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int ra = wm * WTM + i * 16 + (lane & 15);
            af0[i] = *reinterpret_cast<const bf16x8 *>(abase + img_off(ra, lane >> 4));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int rb = wn * WTN + j * 16 + (lane & 15);
            bf0[j] = *reinterpret_cast<const bf16x8 *>(bbase + img_off(rb, lane >> 4));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int ra = wm * WTM + i * 16 + (lane & 15);
            af1[i] = *reinterpret_cast<const bf16x8 *>(abase + img_off(ra, 4 + (lane >> 4)));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int rb = wn * WTN + j * 16 + (lane & 15);
            bf1[j] = *reinterpret_cast<const bf16x8 *>(bbase + img_off(rb, 4 + (lane >> 4)));
        }
        mfma_block(af0, bf0);
        __builtin_amdgcn_sched_barrier(0);
        // next tile's staging (VALU + LDS-DMA issue) between the two MFMA clusters
        if (!early && !late && ks + STAGES - 1 < ksteps) {
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);  // the buffer read in iteration ks-1
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_block(af1, bf1);
        if (late && ks + STAGES - 1 < ksteps) {
            __builtin_amdgcn_sched_barrier(0);
            int nb = buf + STAGES - 1;
            if (nb >= STAGES) nb -= STAGES;
            stage(ks + STAGES - 1, nb);
        }
        buf = buf + 1 == STAGES ? 0 : buf + 1;
    }
    wait_vmcnt<0>();
    __syncthreads();  // all ds_reads of the last tile done before the LDS is reused
    conv_store_tile<WM, WN, TM, TN, EPI>(acc, lds, y, g, ea, m0, n0, tid, s1, s2);
    }  // m-tile loop
    if constexpr (STATS) conv_stats_flush<WM, WN, TM, TN, EPI, LDS_BYTES>(lds, g, ea, n0, tid, s1, s2, mt_last + wg, nwg, orig);
}

// Row-image 3x3 / stride-1 / pad-1 convolution (forward, and the stride-1 data gradient on
// flipped weights): the same GEMM as conv_kernel<3>, M = output pixels, N = Cout, K = 9 * Cin, but
// the A operand is staged ONCE per 64-channel chunk as an image instead of once per tap.
//   * Padded pixel index G(n, ihp, iwp) = (n (H + 2) + ihp)(W + 2) + iwp (ihp = ih + 1, iwp = iw + 1):
//     output pixel m = (n, oh, ow) reads, at tap (kh, kw), the input at G(m) + kh (W + 2) + kw with
//     G(m) = (n (H + 2) + oh)(W + 2) + ow.  A tile of BM consecutive output pixels therefore reads one
//     CONTIGUOUS range of padded indices, [G(m0), G(m_last) + 2 (W + 2) + 2] (image boundaries
//     included: their pad rows are part of the range and read zeros).
//   * That range is staged as IMG rows of 128 bytes (one pixel's 64 channels; padding pixels and
//     rows past the range get the out-of-range buffer offset, i.e. zeros) with the 16-byte chunk
//     swizzle of conv_kernel (chunk ^ (row & 7)); the tap shift is only an address offset of the
//     per-lane fragment reads (ds_read_b128 takes per-lane addresses).
//   * K-steps run chunk-major, tap-minor: only B (BN weight rows of one tap and chunk) goes through
//     the BST-deep ring per step; the image of chunk c + 1 is staged with B of its first tap, into
//     the other of IMGB image buffers (IMGB = 1 when Cin = 64: one chunk).
// Why: conv_kernel re-stages the A tile for each of the 9 taps -- 9x the bytes through the LDS-DMA
// path; at 56 x 56 (64 -> 64) its K-step is 512 MFMA cycles per SIMD against 40 KB of staging, and
// the kernel ran at 23 % MFMA busy (profiles/r6_conv3x3_rows.md).  Here the staged bytes per tile
// fall from 9 (BM + BN) to about 1.1 BM + 9 BN rows per chunk.
// The epilogue and the statistics flush are conv_kernel's (conv_store_tile / conv_stats_flush).
template <int WM, int WN, int BST, int EPI, int TM, int TN, int IMG, int IMGB, bool PERSIST>
__global__ __launch_bounds__(64 * WM * WN) void conv_rows_kernel(const uint16_t *__restrict__ x,
                                                                 const uint16_t *__restrict__ w,
                                                                 uint16_t *__restrict__ y, Geo g, EpiArgs ea) {
    constexpr int WTM = 16 * TM, WTN = 16 * TN;
    constexpr int BM = WTM * WM, BN = WTN * WN, NW = WM * WN, NT = 64 * NW;
    constexpr int B_BYTES = BN * kRowBytes, IMG_BYTES = IMG * kRowBytes;
    constexpr int B_INST = BN / 8 / NW;  // LDS-DMA pieces per wave per B stage (8 rows each)
    constexpr int I_INST = IMG / 8 / NW;  // ... per image
    static_assert(B_INST >= 1 && B_INST * NW * 8 == BN && I_INST * NW * 8 == IMG, "staging split");
    constexpr int CROW = BN * 2 + 16;
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate | kEpiGeluGrad)) != 0;
    constexpr int NSUM = (EPI & (kEpiGate | kEpiGeluGrad)) ? 1 : 2;
    constexpr int RED_BYTES = STATS ? NSUM * (NT / (BN / 8)) * BN * 4 : 0;
    constexpr int EPI_BYTES = BM * CROW > RED_BYTES ? BM * CROW : RED_BYTES;
    constexpr int MAIN_BYTES = IMGB * IMG_BYTES + BST * B_BYTES;
    constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
    __shared__ __attribute__((aligned(1024))) uint8_t lds[LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nwg = gridDim.x, orig = blockIdx.x;
    const int q = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int mt_first = wg / g.ntiles, nt = wg - mt_first * g.ntiles;
    const int n0 = nt * BN;
    const int mstride = PERSIST ? nwg / g.ntiles : g.mtiles;
    float s1[8], s2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
    const int Wp = g.W + 2, HWp = (g.H + 2) * Wp;
    const int csteps = g.C / kBK;  // Cin % 64 == 0 (launcher)
    const int ksteps = 9 * csteps;
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(x), 0, static_cast<int>(kBufOOB), kBufFlags);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(w), 0, static_cast<int>(kBufOOB), kBufFlags);
    const int srow = lane >> 3;
    const int schunk = (lane & 7) ^ srow;  // staged rows start at multiples of 8: row & 7 = srow
    const int wm = wave / WN, wn = wave % WN;
    int mt_last = mt_first;
    for (int mt = mt_first; mt < g.mtiles; mt += mstride) {
        mt_last = mt;
        const int m0 = mt * BM;
        if (mt != mt_first) __syncthreads();
        auto gidx = [&](int m) {
            const int ow = m % g.OW, t = m / g.OW, oh = t % g.OH, n = t / g.OH;
            return n * HWp + oh * Wp + ow;
        };
        const int base = gidx(m0);
        const int mlast = (m0 + BM < g.M ? m0 + BM : g.M) - 1;
        const int nslots = gidx(mlast) - base + 2 * Wp + 3;
        // image staging: element offset of slot s's pixel (this lane's chunk), or -1 (zeros)
        // (decoded once, then stepped by 8 slots per piece: Wp >= 9, so at most one column wrap;
        // integer divisions per piece were ~1.5 k VALU instructions per wave and tile)
        int i_off[I_INST];
        {
            const int s0 = wave * I_INST * 8 + srow;
            int n = (base + s0) / HWp, r = base + s0 - n * HWp;
            int ihp = r / Wp, iwp = r - ihp * Wp;
#pragma unroll
            for (int j = 0; j < I_INST; ++j) {
                const int s = s0 + j * 8;
                const bool ok = s < nslots && n < g.N && ihp >= 1 && ihp <= g.H && iwp >= 1 && iwp <= g.W;
                i_off[j] = ok ? ((n * g.H + ihp - 1) * g.W + iwp - 1) * g.C + schunk * 8 : -1;
                iwp += 8;
                if (iwp >= Wp) {
                    iwp -= Wp;
                    if (++ihp == g.H + 2) {
                        ihp = 0;
                        ++n;
                    }
                }
            }
        }
        int b_off[B_INST];
#pragma unroll
        for (int j = 0; j < B_INST; ++j) b_off[j] = (n0 + (wave * B_INST + j) * 8 + srow) * 9 * g.C + schunk * 8;
        // fragment rows: slot of tap (0, 0) relative to the image (rows past M read a valid slot)
        int frel[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int m = m0 + wm * WTM + i * 16 + (lane & 15);
            frel[i] = gidx(m < g.M ? m : g.M - 1) - base;
        }
        auto stage = [&](int ks) {
            const int cc = ks / 9, tap = ks - cc * 9;
            if (tap == 0) {
                uint8_t *ib = lds + (IMGB == 1 ? 0 : (cc & 1)) * IMG_BYTES;
#pragma unroll
                for (int j = 0; j < I_INST; ++j) {
                    const uint32_t vo = i_off[j] >= 0 ? static_cast<uint32_t>(i_off[j] + cc * kBK) * 2u : kBufOOB;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, lds_ptr(ib + (wave * I_INST + j) * 1024), 16, vo, 0,
                                                             0, 0);
                }
            }
            uint8_t *bb = lds + IMGB * IMG_BYTES + (ks % BST) * B_BYTES;
#pragma unroll
            for (int j = 0; j < B_INST; ++j) {
                const uint32_t vo = static_cast<uint32_t>(b_off[j] + tap * g.C + cc * kBK) * 2u;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(wr, lds_ptr(bb + (wave * B_INST + j) * 1024), 16, vo, 0, 0,
                                                         0);
            }
        };
        f32x4 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        auto mfma_block = [&](const bf16x8 (&af)[TM], const bf16x8 (&bfr)[TN]) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
        };
#pragma unroll
        for (int p = 0; p < BST - 1; ++p)
            if (p < ksteps) stage(p);
        for (int ks = 0; ks < ksteps; ++ks) {
            // B of step ks (and every older load: its chunk's image) landed
            if (ks + BST - 1 <= ksteps) wait_vmcnt<B_INST * (BST - 2)>();
            else wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            const int cc = ks / 9, tap = ks - cc * 9;
            const int kh = tap / 3, kw = tap - kh * 3;
            const int toff = kh * Wp + kw;
            const uint8_t *ib = lds + (IMGB == 1 ? 0 : (cc & 1)) * IMG_BYTES;
            const uint8_t *bb = lds + IMGB * IMG_BYTES + (ks % BST) * B_BYTES;
            bf16x8 af0[TM], bf0[TN], af1[TM], bf1[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int sl = frel[i] + toff;
                af0[i] = *reinterpret_cast<const bf16x8 *>(ib + img_off(sl, lane >> 4));
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int rb = wn * WTN + j * 16 + (lane & 15);
                bf0[j] = *reinterpret_cast<const bf16x8 *>(bb + img_off(rb, lane >> 4));
            }
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int sl = frel[i] + toff;
                af1[i] = *reinterpret_cast<const bf16x8 *>(ib + img_off(sl, 4 + (lane >> 4)));
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int rb = wn * WTN + j * 16 + (lane & 15);
                bf1[j] = *reinterpret_cast<const bf16x8 *>(bb + img_off(rb, 4 + (lane >> 4)));
            }
            mfma_block(af0, bf0);
            __builtin_amdgcn_sched_barrier(0);
            if (ks + BST - 1 < ksteps) stage(ks + BST - 1);  // into the slot read in step ks - 1
            __builtin_amdgcn_sched_barrier(0);
            mfma_block(af1, bf1);
        }
        wait_vmcnt<0>();
        __syncthreads();
        conv_store_tile<WM, WN, TM, TN, EPI>(acc, lds, y, g, ea, m0, n0, tid, s1, s2);
    }  // m-tile loop
    if constexpr (STATS)
        conv_stats_flush<WM, WN, TM, TN, EPI, LDS_BYTES>(lds, g, ea, n0, tid, s1, s2, mt_last + wg, nwg, orig);
}

// Largest image (padded-index range) any BM-pixel tile of this stride-1 3x3 geometry reads.
inline int conv_rows_slots(const Geo &g, int BM) {
    const int Wp = g.W + 2, HWp = (g.H + 2) * Wp;
    auto gidx = [&](int m) {
        const int ow = m % g.OW, t = m / g.OW, oh = t % g.OH, n = t / g.OH;
        return n * HWp + oh * Wp + ow;
    };
    // the range depends on the tile only through m0 mod (OH * OW): one period of tile positions
    const int per_img = g.OH * g.OW;
    int a = per_img, b = BM;
    while (b) {
        const int t = a % b;
        a = b;
        b = t;
    }
    const int64_t period = static_cast<int64_t>(per_img / a) * BM;  // lcm(per_img, BM) pixels
    int worst = 0;
    for (int m0 = 0; m0 < g.M && m0 < period; m0 += BM) {
        const int ml = (m0 + BM < g.M ? m0 + BM : g.M) - 1;
        const int s = gidx(ml) - gidx(m0) + 2 * Wp + 3;
        worst = s > worst ? s : worst;
    }
    return worst;
}

template <int WM, int WN, int BST, int EPI, int TM, int TN, int IMG, int IMGB>
void launch_rows_epi(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, hipStream_t s) {
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    g.mtiles = (g.M + BM - 1) / BM;
    g.ntiles = g.K / BN;
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate)) != 0;
    if constexpr (STATS) {
        constexpr int LDS = IMGB * IMG * 128 + BST * BN * 128;
        constexpr int OCC = (160 * 1024) / LDS < 4 ? (160 * 1024) / LDS : 4;
        const int per_n = 256 * (OCC < 1 ? 1 : OCC) / g.ntiles;
        if (per_n >= 1 && g.mtiles > 2 * per_n) {
            conv_rows_kernel<WM, WN, BST, EPI, TM, TN, IMG, IMGB, true><<<per_n * g.ntiles, 64 * WM * WN, 0, s>>>(
                x, w, y, g, ea);
            return;
        }
    }
    if (ea.fin) {
        EpiArgs e2 = ea;
        e2.fin = nullptr;
        conv_rows_kernel<WM, WN, BST, EPI, TM, TN, IMG, IMGB, false><<<g.mtiles * g.ntiles, 64 * WM * WN, 0, s>>>(
            x, w, y, g, e2);
        bn_fin_desc_kernel<<<(g.K + 255) / 256, 256, 0, s>>>(ea.fin, ea.stats, g.K);
        return;
    }
    conv_rows_kernel<WM, WN, BST, EPI, TM, TN, IMG, IMGB, false><<<g.mtiles * g.ntiles, 64 * WM * WN, 0, s>>>(
        x, w, y, g, ea);
}

// The epilogues of a stride-1 3x3 conv in ResNet / VGG (forward statistics, BN-backward sums with
// the coefficients or the ReLU bits, accumulate, plain); false = not on this kernel.
template <int WM, int WN, int BST, int TM, int TN, int IMG, int IMGB>
bool launch_rows_variant(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                         hipStream_t s) {
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    if (g.K % BN || g.C % kBK || (IMGB == 1 && g.C != kBK) || g.W < 7 || conv_rows_slots(g, BM) > IMG) return false;
    switch (epi) {
    case 0: launch_rows_epi<WM, WN, BST, 0, TM, TN, IMG, IMGB>(x, w, y, g, ea, s); return true;
    case kEpiFwdStats: launch_rows_epi<WM, WN, BST, kEpiFwdStats, TM, TN, IMG, IMGB>(x, w, y, g, ea, s); return true;
    case kEpiBwdCoef: launch_rows_epi<WM, WN, BST, kEpiBwdCoef, TM, TN, IMG, IMGB>(x, w, y, g, ea, s); return true;
    case kEpiBwdBits: launch_rows_epi<WM, WN, BST, kEpiBwdBits, TM, TN, IMG, IMGB>(x, w, y, g, ea, s); return true;
    default: return false;
    }
}

template <int KS, int WM, int WN, int ST, int EPI, int TM = 4, int TN = 4>
void launch_epi(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, hipStream_t s) {
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    if (g.K % 8 || g.C % 8) throw std::invalid_argument("conv: Cin and Cout must be multiples of 8");
    check_buf_extent(g);
    g.mtiles = (g.M + BM - 1) / BM;
    g.ntiles = (g.K + BN - 1) / BN;
    constexpr bool STATS = (EPI & (kEpiFwdStats | kEpiBwdCoef | kEpiBwdBits | kEpiGate)) != 0;
    if constexpr (STATS) {
        // persistent blocks (4 per CU, fewer when the tile's LDS allows less): one atomic
        // statistics flush per block instead of per tile
        constexpr int env_cap = 0;
        constexpr int kRow = 128, STG = ST * (BM + BN) * kRow, CT = BM * (BN * 2 + 16);
        constexpr int LDS = STG > CT ? STG : CT;
        constexpr int OCC = (160 * 1024) / LDS < 4 ? (160 * 1024) / LDS : 4;
        const int cap = env_cap > 0 ? env_cap : 256 * (OCC < 1 ? 1 : OCC);
        const int per_n = cap / g.ntiles;
        if (cap > 0 && per_n >= 1 && g.mtiles > 2 * per_n) {
            conv_kernel<KS, WM, WN, ST, EPI, TM, TN, true><<<per_n * g.ntiles, 64 * WM * WN, 0, s>>>(
                x, w, y, reinterpret_cast<const uint16_t *>(zero_page()), g, ea);
            return;
        }
    }
    if (ea.fin) {
        // one tile per workgroup: finalize in a launch of its own
        EpiArgs e2 = ea;
        e2.fin = nullptr;
        conv_kernel<KS, WM, WN, ST, EPI, TM, TN><<<g.mtiles * g.ntiles, 64 * WM * WN, 0, s>>>(
            x, w, y, reinterpret_cast<const uint16_t *>(zero_page()), g, e2);
        bn_fin_desc_kernel<<<(g.K + 255) / 256, 256, 0, s>>>(ea.fin, ea.stats, g.K);
        return;
    }
    conv_kernel<KS, WM, WN, ST, EPI, TM, TN><<<g.mtiles * g.ntiles, 64 * WM * WN, 0, s>>>(
        x, w, y, reinterpret_cast<const uint16_t *>(zero_page()), g, ea);
}

// Every fused epilogue on one tile shape.
template <int KS, int WM, int WN, int ST, int TM = 4, int TN = 4>
void launch_variant(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s) {
    constexpr int A = kEpiAccum, M = kEpiAccMask, B = kEpiBwdBits, C = kEpiBwdCoef;
    switch (epi) {
    case 0: launch_epi<KS, WM, WN, ST, 0, TM, TN>(x, w, y, g, ea, s); break;
    case kEpiFwdStats: launch_epi<KS, WM, WN, ST, kEpiFwdStats, TM, TN>(x, w, y, g, ea, s); break;
    case A: launch_epi<KS, WM, WN, ST, A, TM, TN>(x, w, y, g, ea, s); break;
    case C: launch_epi<KS, WM, WN, ST, C, TM, TN>(x, w, y, g, ea, s); break;
    case B: launch_epi<KS, WM, WN, ST, B, TM, TN>(x, w, y, g, ea, s); break;
    case A | B: launch_epi<KS, WM, WN, ST, A | B, TM, TN>(x, w, y, g, ea, s); break;
    case A | C: launch_epi<KS, WM, WN, ST, A | C, TM, TN>(x, w, y, g, ea, s); break;
    case A | M: launch_epi<KS, WM, WN, ST, A | M, TM, TN>(x, w, y, g, ea, s); break;
    case A | M | B: launch_epi<KS, WM, WN, ST, A | M | B, TM, TN>(x, w, y, g, ea, s); break;
    case A | kEpiAccEven: launch_epi<KS, WM, WN, ST, A | kEpiAccEven, TM, TN>(x, w, y, g, ea, s); break;
    case A | kEpiAccEven | B: launch_epi<KS, WM, WN, ST, A | kEpiAccEven | B, TM, TN>(x, w, y, g, ea, s); break;
    case kEpiBiasRelu: launch_epi<KS, WM, WN, ST, kEpiBiasRelu, TM, TN>(x, w, y, g, ea, s); break;
    case kEpiGate: launch_epi<KS, WM, WN, ST, kEpiGate, TM, TN>(x, w, y, g, ea, s); break;
    default: throw std::invalid_argument("conv: unsupported epilogue combination");
    }
}

template <int KS>
void launch_ks(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi, hipStream_t s,
               int variant) {
    // default per shape (re-measured with the fused epilogues, tools/bench_conv1x1_variants.py
    // [KS3=1]; VGG's compute-bound 3x3 layers: tools/bench_vgg_conv.py, 1.15-1.17 PF/s): 256x256 /
    // 8 waves whenever Cout % 256 == 0 and there are >= 128 such tiles (64->256 at 56x56 161 ->
    // 123 us, 3x3 256->256 at 14x14 70 -> 57 us; fewer tiles under-fill the chip: 3x3 512->512 at
    // 7x7 62 -> 100 us), else 256x128 / 8 waves (1x1 included: 4-13 % over 128x128), else 256x64
    if (variant < 0) {
        const int64_t tiles256 = ((static_cast<int64_t>(g.M) + 255) / 256) * (g.K / 256);  // (K % 256 == 0 only)
        variant = g.K <= 32 ? 11 : g.K % 256 == 0 && tiles256 >= 128 ? 7 : g.K % 128 == 0 ? 1 : 2;
        if (variant == 7 && g.K % 128 == 0) {
            // tile quantisation: 256x256 tiles run one workgroup per CU (135 KB of LDS), so a grid
            // of T tiles takes ceil(T / 256) rounds; when the 256x128 grid fills its rounds >= 10 %
            // better it wins despite the smaller tile (r5t21: 256->1024 at 14x14 63 -> 51 us; the
            // 56x56 / 28x28 / 7x7 shapes keep 256x256, tools/bench_conv1x1_variants.py)
            const int64_t t7 = tiles256, t1 = t7 * 2;
            const double e7 = static_cast<double>(t7) / (((t7 + 255) / 256) * 256);
            const double e1 = static_cast<double>(t1) / (((t1 + 255) / 256) * 256);
            if (e1 > 1.1 * e7) variant = 1;
        }
        if (conv_tile_rules() >= 2 && g.K % 128 == 0 && g.K > 32) {
            // re-measured with the staggered staging (tools/bench_conv1x1_variants.py, profiles/r3_conv_variants.txt):
            // the accumulating data gradients (ResNet's conv1 dgrad into the residual gradient) run best on
            // 128x128 / 4 waves at every ResNet size (64->256@56 303 -> 290 us, 128->512@28 174 -> 156,
            // 256->1024@14 90 -> 82, 512->2048@7 60 -> 57), and so do the stride-1 3x3 ones with 128 or
            // 512 outputs that are not on 256x256 tiles (128->128@28 101 -> 88, 512->512@7 76 -> 71)
            if ((epi & kEpiAccum) != 0 || (KS == 3 && g.stride == 1 && variant != 7)) variant = 0;
        }
        if (variant == 7 && g.M % 224 == 0 && conv_t224()) {
            // a one- or two-round grid of 256x256 tiles: 224x256 tiles when their rounds cost >= 5 %
            // less (ResNet-50's 14 x 14 layers, M = 50,176: 196 tiles leave 60 of 256 CUs idle, 224
            // tiles of 7/8 the work fill 224 of them)
            const int64_t t7 = ((static_cast<int64_t>(g.M) + 255) / 256) * (g.K / 256), t8 = (g.M / 224) * (g.K / 256);
            if (t7 <= 512 && ((t8 + 255) / 256) * 224 < 0.95 * ((t7 + 255) / 256) * 256) variant = 8;
        }
    }
    // the per-shape defaults only (round 6: the tuning-only tiles -- 256x64 3-stage, 512x64, 128x64,
    // 256x256 of 128x64 waves, the 2- and 4-wave 64x128 -- never won a default, see
    // profiles/r3_conv_variants.txt, and are no longer instantiated)
    switch (variant) {
    case 0: if (g.K % 128 == 0) { launch_variant<KS, 2, 2, 2>(x, w, y, g, ea, epi, s); break; }  // 128x128
            [[fallthrough]];
    case 1: if (g.K % 128 == 0) { launch_variant<KS, 4, 2, 3>(x, w, y, g, ea, epi, s); break; }  // 256x128
            [[fallthrough]];
    case 2: launch_variant<KS, 4, 1, 2>(x, w, y, g, ea, epi, s); break;                          // 256x64
    case 7: if (g.K % 256) throw std::invalid_argument("conv variant 7: Cout % 256");
            launch_variant<KS, 4, 2, 2, 4, 8>(x, w, y, g, ea, epi, s); break;                  // 256x256, 8w, 64x128
    case 8: if (g.K % 256) throw std::invalid_argument("conv variant 8: Cout % 256");
            launch_variant<KS, 2, 4, 2, 7, 4>(x, w, y, g, ea, epi, s); break;                  // 224x256, 8w, 112x64
    case 11: launch_variant<KS, 4, 1, 2, 4, 2>(x, w, y, g, ea, epi, s); break;                // 256x32 (Cout <= 32)
    default: throw std::invalid_argument("conv: tile variant must be -1, 0, 1, 2, 7, 8 or 11");
    }
}


}  // namespace

}  // namespace kfk
