// Fused residual-add + LayerNorm for transformer blocks (BERT-base, D = 768), bf16 in/out,
// f32 statistics, for gfx950.
//
//   forward   s = x + r (optional r);  y = (s - mean) * rstd * gamma + beta      (bf16 y, s)
//   backward  g = dy * gamma;  ds = rstd * (g - mean(g) - xhat * mean(g * xhat))
//             dgamma = sum_rows dy * xhat,  dbeta = sum_rows dy                    (f32)
//
// Why: under bf16 autocast torch runs LayerNorm in f32 (an f32 output the next GEMM casts
// back to bf16), the residual add in f32, and the backward as three kernels (input
// gradient, per-block gamma/beta partials, their reduction): ~5 ms of a 30 ms BERT-base
// step (profiles/r2b_bert_base_gns.md).  Here the residual stream stays bf16 and each
// direction is one pass over the activations plus a tiny column reduction.
//
// Residual dropout (BERT's dropout(dense(x)) before the add): with p > 0 the residual input r
// is dropped and scaled in the forward, r' = keep(e) ? r / (1 - p) : 0, from a counter hash
// of (seed, element index) -- no mask tensor; the backward recomputes keep(e) and writes
// dr = keep(e) ? ds / (1 - p) : 0 beside ds (replacing torch's dropout and masked-scale passes).
//
// Layout: rows of D contiguous elements (D % 256 == 0, D <= 4096).  One wave64 per row;
// lane l owns the 4-element groups l, l + 64, l + 128, ... (8-byte accesses, coalesced
// across the wave), so each lane's columns are FIXED: the backward accumulates its
// dgamma/dbeta columns in registers across all the rows its wave visits (grid-stride),
// then one block reduction writes [blocks][2][D] f32 partials for a column-sum kernel.
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

constexpr int kLnWaves = 4;  // waves (rows in flight) per block

__device__ __forceinline__ void unpack4(const uint2 &v, float (&f)[4]) {
    f[0] = __uint_as_float(v.x << 16);
    f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16);
    f[3] = __uint_as_float(v.y & 0xffff0000u);
}

__device__ __forceinline__ uint2 pack4(const float (&f)[4]) {
    return make_uint2(pack_bf16x2(f[0], f[1]),
                      pack_bf16x2(f[2], f[3]));
}

struct LnDrop {
    uint32_t seed = 0, thresh = 0;  // keep(e) <=> hash(seed, e) >= thresh (thresh = p * 2^32)
    float inv_keep = 1.f;
    bool on = false;
    const uint32_t *base = nullptr;  // device seed base (dropout_seed_base), mixed in at kernel entry
};

// the kernel-entry seed: the call's host seed mixed with the device seed base
__device__ __forceinline__ void ln_seed(LnDrop &d) {
    if (d.on && d.base) d.seed ^= d.base[0] * 0x85EBCA6Bu;
}

__device__ __forceinline__ bool ln_keep(const LnDrop &d, int64_t e) {
    uint32_t h = static_cast<uint32_t>(e) * 0x9E3779B1u ^ static_cast<uint32_t>(e >> 32) * 0x7FEB352Du ^ d.seed;
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return h >= d.thresh;
}

template <int G>  // G = D / 256 four-element groups per lane
__global__ __launch_bounds__(64 * kLnWaves) void ln_fwd_kernel(const uint2 *__restrict__ x,
                                                               const uint2 *__restrict__ r,
                                                               const float *__restrict__ gamma,
                                                               const float *__restrict__ beta, uint2 *__restrict__ y,
                                                               uint2 *__restrict__ s_out, float *__restrict__ mean,
                                                               float *__restrict__ rstd, int64_t rows, float eps,
                                                               LnDrop drop) {
    ln_seed(drop);
    constexpr int D = 256 * G;
    const int lane = threadIdx.x & 63;
    float gm[G][4], bt[G][4];
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            gm[j][k] = gamma[(j * 64 + lane) * 4 + k];
            bt[j][k] = beta[(j * 64 + lane) * 4 + k];
        }
    const int64_t wstride = static_cast<int64_t>(gridDim.x) * kLnWaves;
    for (int64_t row = static_cast<int64_t>(blockIdx.x) * kLnWaves + (threadIdx.x >> 6); row < rows; row += wstride) {
        const int64_t base = row * (D / 4);
        float v[G][4];
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            unpack4(x[base + j * 64 + lane], v[j]);
            if (r) {
                float t[4];
                unpack4(r[base + j * 64 + lane], t);
                if (drop.on) {
                    const int64_t e0 = (base + j * 64 + lane) * 4;
#pragma unroll
                    for (int k = 0; k < 4; ++k) t[k] = ln_keep(drop, e0 + k) ? t[k] * drop.inv_keep : 0.f;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) v[j][k] += t[k];
            }
            // the residual stream is bf16: normalise exactly the values that are stored
            uint2 sv = pack4(v[j]);
            if (s_out) s_out[base + j * 64 + lane] = sv;
            unpack4(sv, v[j]);
#pragma unroll
            for (int k = 0; k < 4; ++k) sum += v[j][k];
        }
        const float mu = wave_sum(sum) * (1.f / D);
        float var = 0.f;
#pragma unroll
        for (int j = 0; j < G; ++j)
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float d = v[j][k] - mu;
                var += d * d;
            }
        const float rs = rsqrtf(wave_sum(var) * (1.f / D) + eps);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = (v[j][k] - mu) * rs * gm[j][k] + bt[j][k];
            y[base + j * 64 + lane] = pack4(o);
        }
        if (lane == 0) {
            mean[row] = mu;
            rstd[row] = rs;
        }
    }
}

// RB: also the column sums of the residual input's gradient (dr, or ds without dropout) as written
// in bf16 -- the bias gradient of the linear layer that produced the residual input (its colsum
// pass is skipped); partial rows [blocks][3][D].
template <int G, bool RB>
__global__ __launch_bounds__(64 * kLnWaves) void ln_bwd_kernel(const uint2 *__restrict__ dy,
                                                               const uint2 *__restrict__ s,
                                                               const float *__restrict__ gamma,
                                                               const float *__restrict__ mean,
                                                               const float *__restrict__ rstd, uint2 *__restrict__ ds,
                                                               float *__restrict__ partial, int64_t rows,
                                                               uint2 *__restrict__ dr, LnDrop drop) {
    ln_seed(drop);
    constexpr int D = 256 * G;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float gm[G][4], dg[G][4], db[G][4], rb[RB ? G : 1][4];
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            gm[j][k] = gamma[(j * 64 + lane) * 4 + k];
            dg[j][k] = db[j][k] = 0.f;
            if constexpr (RB) rb[j][k] = 0.f;
        }
    const int64_t wstride = static_cast<int64_t>(gridDim.x) * kLnWaves;
    for (int64_t row = static_cast<int64_t>(blockIdx.x) * kLnWaves + wave; row < rows; row += wstride) {
        const int64_t base = row * (D / 4);
        const float mu = mean[row], rs = rstd[row];
        float xh[G][4], g[G][4];
        float a1 = 0.f, a2 = 0.f;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            float d[4], xv[4];
            unpack4(dy[base + j * 64 + lane], d);
            unpack4(s[base + j * 64 + lane], xv);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                xh[j][k] = (xv[k] - mu) * rs;
                g[j][k] = d[k] * gm[j][k];
                a1 += g[j][k];
                a2 += g[j][k] * xh[j][k];
                dg[j][k] += d[k] * xh[j][k];
                db[j][k] += d[k];
            }
        }
        const float m1 = wave_sum(a1) * (1.f / D), m2 = wave_sum(a2) * (1.f / D);
#pragma unroll
        for (int j = 0; j < G; ++j) {
            float o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) o[k] = rs * (g[j][k] - m1 - xh[j][k] * m2);
            uint2 pk = pack4(o);
            ds[base + j * 64 + lane] = pk;
            if (dr) {  // gradient of the dropped residual input
                const int64_t e0 = (base + j * 64 + lane) * 4;
#pragma unroll
                for (int k = 0; k < 4; ++k) o[k] = ln_keep(drop, e0 + k) ? o[k] * drop.inv_keep : 0.f;
                pk = pack4(o);
                dr[base + j * 64 + lane] = pk;
            }
            if constexpr (RB) {
                float w[4];
                unpack4(pk, w);  // the bf16 values the producing linear's backward consumes
#pragma unroll
                for (int k = 0; k < 4; ++k) rb[j][k] += w[k];
            }
        }
    }
    // block reduction of the per-lane column sums -> partial[block][NS][D]
    constexpr int NS = RB ? 3 : 2;
    __shared__ float red[kLnWaves][NS][D];
#pragma unroll
    for (int j = 0; j < G; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            red[wave][0][(j * 64 + lane) * 4 + k] = dg[j][k];
            red[wave][1][(j * 64 + lane) * 4 + k] = db[j][k];
            if constexpr (RB) red[wave][2][(j * 64 + lane) * 4 + k] = rb[j][k];
        }
    __syncthreads();
    for (int c = threadIdx.x; c < NS * D; c += 64 * kLnWaves) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < kLnWaves; ++w) t += (&red[w][0][0])[c];
        partial[static_cast<int64_t>(blockIdx.x) * NS * D + c] = t;
    }
}

// out[c] = sum_b partial[b][c] for c < 2D.  Block = 64 consecutive columns x 16 row groups
// (coalesced 256-byte row segments, 16 independent f64 chains per column), then an LDS
// reduction over the groups.
constexpr int kColGroups = 16;
__global__ __launch_bounds__(64 * kColGroups) void ln_colsum_kernel(const float *__restrict__ partial, int nblocks,
                                                                    int cols, float *__restrict__ dgamma,
                                                                    float *__restrict__ dbeta, int D,
                                                                    float *__restrict__ rb_f32 = nullptr,
                                                                    uint16_t *__restrict__ rb_bf16 = nullptr) {
    __shared__ double red[kColGroups][64];
    const int lane = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    double t = 0;
    if (c < cols) {
#pragma unroll 8
        for (int b = grp; b < nblocks; b += kColGroups) t += partial[static_cast<int64_t>(b) * cols + c];
    }
    red[grp][lane] = t;
    __syncthreads();
    if (grp == 0 && c < cols) {
        double u = 0;
#pragma unroll
        for (int g = 0; g < kColGroups; ++g) u += red[g][lane];
        if (c < D) dgamma[c] = static_cast<float>(u);
        else if (c < 2 * D) dbeta[c - D] = static_cast<float>(u);
        else if (rb_f32) rb_f32[c - 2 * D] = static_cast<float>(u);
        else rb_bf16[c - 2 * D] = f32_to_bf16(static_cast<float>(u));
    }
}

template <typename F>
void dispatch_g(int D, F &&f) {
    switch (D / 256) {
    case 1: f(std::integral_constant<int, 1>()); break;
    case 2: f(std::integral_constant<int, 2>()); break;
    case 3: f(std::integral_constant<int, 3>()); break;
    case 4: f(std::integral_constant<int, 4>()); break;
    case 6: f(std::integral_constant<int, 6>()); break;
    case 8: f(std::integral_constant<int, 8>()); break;
    case 12: f(std::integral_constant<int, 12>()); break;
    case 16: f(std::integral_constant<int, 16>()); break;
    default: throw std::invalid_argument("layernorm: D must be 256 x {1,2,3,4,6,8,12,16}");
    }
}

}  // namespace

bool layernorm_supported(int D) {
    const int g = D / 256;
    return D % 256 == 0 && (g == 1 || g == 2 || g == 3 || g == 4 || g == 6 || g == 8 || g == 12 || g == 16);
}

// rows per wave of the backward (grid-stride): more rows -> fewer [blocks][NS][D] partials for the column
// sums, fewer rows -> more waves in flight per CU; 2 / 4 / 8 measured within noise of each other on
// BERT-base (16.17 / 15.98 / 16.07 ms/step, one run each, profiles/r5t39_bert_r*.log)
constexpr int kLnBwdRpw = 8;

int layernorm_bwd_blocks(int64_t rows) {
    int64_t b = (rows + kLnWaves * kLnBwdRpw - 1) / (kLnWaves * kLnBwdRpw);
    if (b > 4096) b = 4096;
    return static_cast<int>(b < 1 ? 1 : b);
}

static LnDrop make_drop(float p, uint32_t seed) {
    LnDrop d;
    if (p > 0.f) {
        if (p >= 1.f) throw std::invalid_argument("layernorm: dropout p must be < 1");
        d.on = true;
        d.seed = seed;
        d.base = dropout_seed_base();
        d.thresh = static_cast<uint32_t>(static_cast<double>(p) * 4294967296.0);
        d.inv_keep = 1.f / (1.f - p);
    }
    return d;
}

void launch_layernorm_forward(const uint16_t *x, const uint16_t *r, const float *gamma, const float *beta, uint16_t *y,
                              uint16_t *s, float *mean, float *rstd, int64_t rows, int D, float eps, hipStream_t st,
                              float p, uint32_t seed) {
    const LnDrop drop = make_drop(r ? p : 0.f, seed);
    if (rows <= 0) return;
    int64_t blocks = (rows + kLnWaves - 1) / kLnWaves;
    if (blocks > 8192) blocks = 8192;
    dispatch_g(D, [&](auto gc) {
        constexpr int G = decltype(gc)::value;
        ln_fwd_kernel<G><<<static_cast<int>(blocks), 64 * kLnWaves, 0, st>>>(
            reinterpret_cast<const uint2 *>(x), reinterpret_cast<const uint2 *>(r), gamma, beta,
            reinterpret_cast<uint2 *>(y), reinterpret_cast<uint2 *>(s), mean, rstd, rows, eps, drop);
    });
}

void launch_layernorm_backward(const uint16_t *dy, const uint16_t *s, const float *gamma, const float *mean,
                               const float *rstd, uint16_t *ds, float *partial, float *dgamma, float *dbeta,
                               int64_t rows, int D, hipStream_t st, uint16_t *dr, float p, uint32_t seed,
                               float *rb_f32, uint16_t *rb_bf16) {
    if (rows <= 0) return;
    const LnDrop drop = make_drop(dr ? p : 0.f, seed);
    const int blocks = layernorm_bwd_blocks(rows);
    const bool rb = rb_f32 || rb_bf16;
    dispatch_g(D, [&](auto gc) {
        constexpr int G = decltype(gc)::value;
        if (rb) {
            // the third partial row must fit the block's LDS reduction: D <= 2048
            if constexpr (G <= 8)
                ln_bwd_kernel<G, true><<<blocks, 64 * kLnWaves, 0, st>>>(
                    reinterpret_cast<const uint2 *>(dy), reinterpret_cast<const uint2 *>(s), gamma, mean, rstd,
                    reinterpret_cast<uint2 *>(ds), partial, rows, reinterpret_cast<uint2 *>(dr), drop);
            else
                throw std::invalid_argument("layernorm_backward: residual bias sums need D <= 2048");
        } else
            ln_bwd_kernel<G, false><<<blocks, 64 * kLnWaves, 0, st>>>(
                reinterpret_cast<const uint2 *>(dy), reinterpret_cast<const uint2 *>(s), gamma, mean, rstd,
                reinterpret_cast<uint2 *>(ds), partial, rows, reinterpret_cast<uint2 *>(dr), drop);
    });
    const int cols = (rb ? 3 : 2) * D;
    ln_colsum_kernel<<<(cols + 63) / 64, 64 * kColGroups, 0, st>>>(partial, blocks, cols, dgamma, dbeta, D, rb_f32,
                                                                   rb_bf16);
}

}  // namespace kfk
