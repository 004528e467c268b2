// Fused multi-head self-attention (forward + backward) for BERT-sized sequences on gfx950:
// S = 64 or 128 tokens, head dim 64, bf16, dropout on the attention probabilities, no mask.
//
// Why: at S = 128 the whole per-(sequence, head) problem is 16 KB per operand, yet torch's
// flash-attention backward on ROCm took 248 us per layer for BERT-base at batch 128 (12.5 % of
// a 26.7 ms step, r2f profile) and the q/k/v gradient concatenation another 90 us.  One
// workgroup per (sequence, head) keeps Q, K, V (and dO) in LDS, computes every product on the
// MFMA cores (v_mfma_f32_16x16x32_bf16) and touches HBM once per operand:
//
//   forward   S^T = K Q^T (wave w: query rows 32w..32w+31; each lane holds 4 consecutive keys of
//             a query), row softmax in registers (2 cross-group shuffles), dropout mask from a counter hash of (seed, sequence*heads + head,
//             query, key) -- nothing stored -- P_drop staged in LDS, O^T = V^T P_drop^T so each
//             lane ends with 4 consecutive head dims of one query (8-byte stores straight
//             into [B, S, H*64]); the row log-sum-exp is kept for the backward.
//   backward  per query block: P = exp(S*scale - lse), dP = dO V^T, D = rowsum(dO o O),
//             dS = P o (dP o keep/(1-p) - D); dQ^T = K^T dS^T.  Then per key block (after one
//             barrier): dV^T = dO^T P_drop, dK^T = Q^T dS, all from LDS images read with the
//             transposing ds_read_b64_tr_b16 -- dq, dk, dv written straight into the
//             [B, S, 3, H, 64] layout of the fused qkv projection (no concatenation).
//
// LDS images: row-major tiles whose 32-byte column groups are XOR-swizzled by the row (the
// conv_wgrad.hip scheme), filled by 16-byte global_load_lds for the HBM operands.
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int DH = 64;  // head dim

// swizzle of the 32-byte column group by the row: 128-byte rows (64 bf16) / 256-byte rows
template <int ROW>
__device__ __forceinline__ int hsw(int row) {
    if constexpr (ROW == 256) return (row & 3) | (((row >> 3) & 1) << 2);
    else return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
}
template <int ROW>
__device__ __forceinline__ int off(int row, int col) {
    return row * ROW + (((col >> 4) ^ hsw<ROW>(row)) << 5) + (col & 15) * 2;
}

__device__ __forceinline__ bf16x8 rd128(const uint8_t *p) { return *reinterpret_cast<const bf16x8 *>(p); }

// operand fragment from an image whose ROWS are the MFMA K index: lane 16g+4q+p reads row
// k0 + 8g + q (+4), columns c0 + 4p..4p+3; lane i of the 16-group receives column c0 + i
template <int ROW>
__device__ __forceinline__ bf16x8 tr_frag(const uint8_t *img, int k0, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r = k0 + 8 * g + q, c = c0 + 4 * p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + off<ROW>(r, c)));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(img + off<ROW>(r + 4, c)));
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// operand fragment from an image whose COLUMNS are the MFMA K index: lane l reads row
// r0 + (l & 15), columns k0 + 8 (l >> 4) .. +7
template <int ROW>
__device__ __forceinline__ bf16x8 row_frag(const uint8_t *img, int r0, int k0, int lane) {
    return rd128(img + off<ROW>(r0 + (lane & 15), k0 + 8 * (lane >> 4)));
}

__device__ __forceinline__ f32x4 mfma(const bf16x8 &a, const bf16x8 &b, const f32x4 &c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2{a, b}), bf16x2));
}

// Dropout keep test: a counter hash of (seed, sequence*heads + head, query, key).  The same
// function is reproduced in torch by the tests (kungfu_amd/ops/attention.py: dropout_keep).
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t bh, uint32_t q, uint32_t k, uint32_t thresh) {
    uint32_t x = ((q << 16) | k) ^ seed;
    x *= 0x9E3779B1u;
    x ^= bh * 0x85EBCA77u + (x >> 15);
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x >= thresh;
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Stage NIMG images of S rows x 64 bf16 (128-byte rows) with 16-byte global_load_lds: image t
// row r comes from src[t] + r * stride[t]; the NW waves split the 1 KB (8-row) pieces.
template <int S, int NIMG, int NW = 4>
__device__ __forceinline__ void stage_images(uint8_t *lds, const uint16_t *const (&src)[NIMG],
                                             const int (&stride)[NIMG], int wave, int lane) {
    constexpr int PIECES = S / 8;
    static_assert((NIMG * PIECES) % NW == 0, "pieces per wave");
    const int pch = lane & 7;
#pragma unroll
    for (int u = 0; u < NIMG * PIECES / NW; ++u) {
        const int gp = wave + NW * u;
        const int t = gp / PIECES, pc = gp - t * PIECES;
        const int r = pc * 8 + (lane >> 3);
        const int col = ((((pch >> 1) ^ hsw<128>(r)) << 1) | (pch & 1)) * 8;
        const uint16_t *s = src[t] + static_cast<int64_t>(r) * stride[t] + col;
        __builtin_amdgcn_global_load_lds(s, lds + t * S * 128 + pc * 1024, 16, 0, 0);
    }
}

struct AttnArgs {
    const uint16_t *qkv;  // [B, S, 3, H, 64]
    uint16_t *out;        // [B, S, H, 64]
    float *lse;           // [B, H, S]
    const uint16_t *dout; // [B, S, H, 64]
    uint16_t *dqkv;       // [B, S, 3, H, 64]
    int H;
    float scale;
    uint32_t seed, thresh;
    float inv_keep;
    const uint32_t *seed_base;  // device word mixed into the seed (graph replays advance it), or null
};

// the per-call seed mixed with the device seed base (dropout_seed_base)
__device__ __forceinline__ uint32_t call_seed(const AttnArgs &a) {
    return a.seed_base ? a.seed ^ (a.seed_base[0] * 0x85EBCA6Bu) : a.seed;
}

template <int S>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnArgs a) {
    constexpr int PROW = 2 * S;    // P image row bytes
    constexpr int QW = S / 4;      // query rows per wave
    constexpr int TQ = QW / 16, TK = S / 16;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[3 * S * 128 + S * PROW];
    uint8_t *Qi = lds, *Ki = lds + S * 128, *Vi = lds + 2 * S * 128, *Pi = lds + 3 * S * 128;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t seed = call_seed(a);
    const int bh = blockIdx.x, b = bh / a.H, h = bh - b * a.H;
    const int D = a.H * DH, RS = 3 * D;  // qkv row stride (elements)
    const uint16_t *base = a.qkv + static_cast<int64_t>(b) * S * RS + h * DH;
    const uint16_t *src[3] = {base, base + D, base + 2 * D};
    const int strd[3] = {RS, RS, RS};
    stage_images<S, 3>(lds, src, strd, wave, lane);
    wait_vmcnt<0>();
    __syncthreads();

    const int q0 = wave * QW;
    // S^T = K Q^T: acc[j][i] holds keys 16 j + 4 (lane >> 4) + r of query q0 + 16 i + (lane & 15), so a
    // query's softmax is 32 in-lane values + 2 cross-group shuffles, and its 4 consecutive keys of a
    // P row leave in ONE 8-byte LDS store (the S = Q K^T layout needed 16-lane butterflies and a
    // 2-byte store per element)
    f32x4 acc[TK][TQ];
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
        for (int i = 0; i < TQ; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DH / 32; ++s) {
        bf16x8 qa[TQ], kb[TK];
#pragma unroll
        for (int i = 0; i < TQ; ++i) qa[i] = row_frag<128>(Qi, q0 + 16 * i, 32 * s, lane);
#pragma unroll
        for (int j = 0; j < TK; ++j) kb[j] = row_frag<128>(Ki, 16 * j, 32 * s, lane);
#pragma unroll
        for (int j = 0; j < TK; ++j)
#pragma unroll
            for (int i = 0; i < TQ; ++i) acc[j][i] = mfma(kb[j], qa[i], acc[j][i]);
    }
    const int lg = lane >> 4, lc = lane & 15;
#pragma unroll
    for (int i = 0; i < TQ; ++i) {
        const int row = q0 + 16 * i + lc;  // the query
        float m = -INFINITY;
#pragma unroll
        for (int j = 0; j < TK; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) m = fmaxf(m, acc[j][i][r] * a.scale);
        m = fmaxf(m, __shfl_xor(m, 16));
        m = fmaxf(m, __shfl_xor(m, 32));
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < TK; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float e = __expf(acc[j][i][r] * a.scale - m);
                acc[j][i][r] = e;
                sum += e;
            }
        sum += __shfl_xor(sum, 16);
        sum += __shfl_xor(sum, 32);
        const float inv = 1.f / sum;
        if (lg == 0) a.lse[static_cast<int64_t>(bh) * S + row] = m + __logf(sum);
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int kb0 = 16 * j + 4 * lg;
            float p[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[j][i][r] * inv;
                p[r] = keep_elem(seed, bh, row, kb0 + r, a.thresh) ? v * a.inv_keep : 0.f;
            }
            *reinterpret_cast<uint2 *>(Pi + off<PROW>(row, kb0)) = make_uint2(pack2(p[0], p[1]), pack2(p[2], p[3]));
        }
    }
    __syncthreads();
    // O^T[d][q] = sum_key V[key][d] P[q][key]: lane -> 4 consecutive d of one query
    f32x4 o[4][TQ];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < TQ; ++i) o[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S / 32; ++s) {
        bf16x8 va[4], pb[TQ];
#pragma unroll
        for (int c = 0; c < 4; ++c) va[c] = tr_frag<128>(Vi, 32 * s, 16 * c, lane);
#pragma unroll
        for (int i = 0; i < TQ; ++i) pb[i] = row_frag<PROW>(Pi, q0 + 16 * i, 32 * s, lane);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int i = 0; i < TQ; ++i) o[c][i] = mfma(va[c], pb[i], o[c][i]);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < TQ; ++i) {
            const int q = q0 + 16 * i + lc;
            uint16_t *dst = a.out + (static_cast<int64_t>(b) * S + q) * D + h * DH + 16 * c + 4 * lg;
            *reinterpret_cast<uint2 *>(dst) = make_uint2(pack2(o[c][i][0], o[c][i][1]), pack2(o[c][i][2], o[c][i][3]));
        }
}

// NW waves: 8 at S = 128 -- the 128 KB of LDS allow one workgroup per CU, so 4 waves would leave
// one wave per SIMD with nothing to overlap its exp / dropout-hash VALU work or LDS waits against
template <int S, int NW>
__global__ __launch_bounds__(64 * NW) void attn_bwd_kernel(AttnArgs a) {
    constexpr int PROW = 2 * S;
    constexpr int QW = S / NW;
    static_assert(QW % 16 == 0, "query rows per wave");
    constexpr int TQ = QW / 16, TK = S / 16;
    __shared__ __attribute__((aligned(1024))) uint8_t lds[4 * S * 128 + 2 * S * PROW];
    __shared__ float dsum[S];
    uint8_t *Qi = lds, *Ki = lds + S * 128, *Vi = lds + 2 * S * 128, *Oi = lds + 3 * S * 128;  // Oi: dO
    uint8_t *Pi = lds + 4 * S * 128, *Si = Pi + S * PROW;                                      // P_drop, dS
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t seed = call_seed(a);
    const int bh = blockIdx.x, b = bh / a.H, h = bh - b * a.H;
    const int D = a.H * DH, RS = 3 * D;
    const uint16_t *base = a.qkv + static_cast<int64_t>(b) * S * RS + h * DH;
    const uint16_t *dob = a.dout + static_cast<int64_t>(b) * S * D + h * DH;
    const uint16_t *src[4] = {base, base + D, base + 2 * D, dob};
    const int strd[4] = {RS, RS, RS, D};
    stage_images<S, 4, NW>(lds, src, strd, wave, lane);
    // D[q] = sum_d dO[q][d] * O[q][d]: TPR lanes per row (64 / TPR dims each), from global
    {
        constexpr int TPR = NW * 64 / 128 < 1 ? 1 : NW * 64 / 128;  // 2 (256 threads) or 4 (512)
        constexpr int NV = 8 / TPR;                                   // 16-byte vectors per lane
        const int q = threadIdx.x / TPR, part = threadIdx.x % TPR;
        if (q < S) {
            const uint4 *po = reinterpret_cast<const uint4 *>(a.out + (static_cast<int64_t>(b) * S + q) * D + h * DH + 8 * NV * part);
            const uint4 *pd = reinterpret_cast<const uint4 *>(dob + static_cast<int64_t>(q) * D + 8 * NV * part);
            float t = 0.f;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const uint4 ov = po[k], dv = pd[k];
                const uint32_t *ow = reinterpret_cast<const uint32_t *>(&ov);
                const uint32_t *dw = reinterpret_cast<const uint32_t *>(&dv);
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    t += __uint_as_float(ow[e] << 16) * __uint_as_float(dw[e] << 16) +
                         __uint_as_float(ow[e] & 0xffff0000u) * __uint_as_float(dw[e] & 0xffff0000u);
            }
#pragma unroll
            for (int o = 1; o < TPR; o <<= 1) t += __shfl_xor(t, o);
            if (part == 0) dsum[q] = t;
        }
    }
    wait_vmcnt<0>();
    __syncthreads();

    const int lg = lane >> 4, lc = lane & 15;
    // ---- phase 1: query rows q0 .. q0 + QW - 1
    const int q0 = wave * QW;
    // transposed products (as the forward): sc[j][i] / dp[j][i] hold keys 16 j + 4 lg + r of query
    // q0 + 16 i + lc -- one lse / D load per query and 8-byte P / dS row stores
    f32x4 sc[TK][TQ], dp[TK][TQ];
#pragma unroll
    for (int j = 0; j < TK; ++j)
#pragma unroll
        for (int i = 0; i < TQ; ++i) sc[j][i] = dp[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < DH / 32; ++s) {
        bf16x8 qa[TQ], ga[TQ], kb[TK], vb[TK];
#pragma unroll
        for (int i = 0; i < TQ; ++i) {
            qa[i] = row_frag<128>(Qi, q0 + 16 * i, 32 * s, lane);
            ga[i] = row_frag<128>(Oi, q0 + 16 * i, 32 * s, lane);
        }
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            kb[j] = row_frag<128>(Ki, 16 * j, 32 * s, lane);
            vb[j] = row_frag<128>(Vi, 16 * j, 32 * s, lane);
        }
#pragma unroll
        for (int j = 0; j < TK; ++j)
#pragma unroll
            for (int i = 0; i < TQ; ++i) {
                sc[j][i] = mfma(kb[j], qa[i], sc[j][i]);
                dp[j][i] = mfma(vb[j], ga[i], dp[j][i]);
            }
    }
#pragma unroll
    for (int i = 0; i < TQ; ++i) {
        const int row = q0 + 16 * i + lc;  // the query
        const float l = a.lse[static_cast<int64_t>(bh) * S + row];
        const float dd = dsum[row];
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int kb0 = 16 * j + 4 * lg;
            float pv[4], sv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float p = __expf(sc[j][i][r] * a.scale - l);
                const bool kp = keep_elem(seed, bh, row, kb0 + r, a.thresh);
                const float dpd = kp ? dp[j][i][r] * a.inv_keep : 0.f;
                pv[r] = kp ? p * a.inv_keep : 0.f;
                sv[r] = p * (dpd - dd);
            }
            *reinterpret_cast<uint2 *>(Pi + off<PROW>(row, kb0)) = make_uint2(pack2(pv[0], pv[1]), pack2(pv[2], pv[3]));
            *reinterpret_cast<uint2 *>(Si + off<PROW>(row, kb0)) = make_uint2(pack2(sv[0], sv[1]), pack2(sv[2], sv[3]));
        }
    }
    __syncthreads();
    // dQ^T[d][q] = scale * sum_key K[key][d] dS[q][key]
    {
        f32x4 o[4][TQ];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int i = 0; i < TQ; ++i) o[c][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S / 32; ++s) {
            bf16x8 ka[4], sb[TQ];
#pragma unroll
            for (int c = 0; c < 4; ++c) ka[c] = tr_frag<128>(Ki, 32 * s, 16 * c, lane);
#pragma unroll
            for (int i = 0; i < TQ; ++i) sb[i] = row_frag<PROW>(Si, q0 + 16 * i, 32 * s, lane);
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int i = 0; i < TQ; ++i) o[c][i] = mfma(ka[c], sb[i], o[c][i]);
        }
#pragma unroll
        for (int i = 0; i < TQ; ++i)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int q = q0 + 16 * i + lc;
                uint16_t *dst = a.dqkv + (static_cast<int64_t>(b) * S + q) * RS + h * DH + 16 * c + 4 * lg;
                *reinterpret_cast<uint2 *>(dst) = make_uint2(pack2(o[c][i][0] * a.scale, o[c][i][1] * a.scale),
                                                             pack2(o[c][i][2] * a.scale, o[c][i][3] * a.scale));
            }
    }
    // ---- phase 2: key rows k0 .. k0 + QW - 1
    const int k0 = wave * QW;
    f32x4 dv[4][TQ], dk[4][TQ];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int j = 0; j < TQ; ++j) dv[c][j] = dk[c][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S / 32; ++s) {
        bf16x8 ga[4], qa[4], pb[TQ], sb[TQ];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            ga[c] = tr_frag<128>(Oi, 32 * s, 16 * c, lane);
            qa[c] = tr_frag<128>(Qi, 32 * s, 16 * c, lane);
        }
#pragma unroll
        for (int j = 0; j < TQ; ++j) {
            pb[j] = tr_frag<PROW>(Pi, 32 * s, k0 + 16 * j, lane);
            sb[j] = tr_frag<PROW>(Si, 32 * s, k0 + 16 * j, lane);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < TQ; ++j) {
                dv[c][j] = mfma(ga[c], pb[j], dv[c][j]);
                dk[c][j] = mfma(qa[c], sb[j], dk[c][j]);
            }
    }
#pragma unroll
    for (int j = 0; j < TQ; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int key = k0 + 16 * j + lc;
            uint16_t *row = a.dqkv + (static_cast<int64_t>(b) * S + key) * RS + h * DH + 16 * c + 4 * lg;
            *reinterpret_cast<uint2 *>(row + D) = make_uint2(pack2(dk[c][j][0] * a.scale, dk[c][j][1] * a.scale),
                                                             pack2(dk[c][j][2] * a.scale, dk[c][j][3] * a.scale));
            *reinterpret_cast<uint2 *>(row + 2 * D) =
                make_uint2(pack2(dv[c][j][0], dv[c][j][1]), pack2(dv[c][j][2], dv[c][j][3]));
        }
}

// 8 waves per S = 128 backward workgroup (4: one wave per SIMD, measured slower, r4t15)
int attn_bwd_waves() { return 8; }

AttnArgs make_args(const uint16_t *qkv, uint16_t *out, float *lse, const uint16_t *dout, uint16_t *dqkv, int H,
                   float scale, uint32_t seed, float p_drop) {
    AttnArgs a;
    a.qkv = qkv, a.out = out, a.lse = lse, a.dout = dout, a.dqkv = dqkv, a.H = H, a.scale = scale, a.seed = seed;
    a.seed_base = dropout_seed_base();
    const double t = static_cast<double>(p_drop) * 4294967296.0;
    a.thresh = p_drop <= 0.f ? 0u : (t >= 4294967295.0 ? 0xffffffffu : static_cast<uint32_t>(t));
    a.inv_keep = p_drop < 1.f ? 1.f / (1.f - p_drop) : 0.f;
    return a;
}

}  // namespace

bool attention_supported(int S, int head_dim) { return head_dim == DH && (S == 64 || S == 128); }

void launch_attention_forward(const uint16_t *qkv, uint16_t *out, float *lse, int B, int S, int H, float scale,
                              uint32_t seed, float p_drop, hipStream_t s) {
    if (!attention_supported(S, DH)) throw std::invalid_argument("attention: S must be 64 or 128");
    const AttnArgs a = make_args(qkv, out, lse, nullptr, nullptr, H, scale, seed, p_drop);
    if (S == 128) attn_fwd_kernel<128><<<B * H, 256, 0, s>>>(a);
    else attn_fwd_kernel<64><<<B * H, 256, 0, s>>>(a);
}

void launch_attention_backward(const uint16_t *qkv, const uint16_t *out, const float *lse, const uint16_t *dout,
                               uint16_t *dqkv, int B, int S, int H, float scale, uint32_t seed, float p_drop,
                               hipStream_t s) {
    if (!attention_supported(S, DH)) throw std::invalid_argument("attention: S must be 64 or 128");
    AttnArgs a = make_args(qkv, const_cast<uint16_t *>(out), const_cast<float *>(lse), dout, dqkv, H, scale, seed,
                           p_drop);
    if (S == 128) {
        if (attn_bwd_waves() == 8) attn_bwd_kernel<128, 8><<<B * H, 512, 0, s>>>(a);
        else attn_bwd_kernel<128, 4><<<B * H, 256, 0, s>>>(a);
    } else {
        attn_bwd_kernel<64, 4><<<B * H, 256, 0, s>>>(a);
    }
}

}  // namespace kfk
