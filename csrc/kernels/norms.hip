// Reductions for the training monitors.
//   K5 gradient noise scale: sum-of-squares of the local (small-batch) and the
//      all-reduced (big-batch) gradient in ONE pass over both buffers, then a
//      device-side epilogue computing G_biased / S_biased, their EMAs and S/G.
//      Reference: srcs/python/kungfu/tensorflow/ops/monitor.py:6-17,
//      srcs/cpp/src/tensorflow/ops/cpu/collective.cpp:212-260,
//      srcs/python/kungfu/tensorflow/optimizers/grad_noise_scale.py:56-88.
//   K6 gradient variance: sum_i |E[g^2]_i - E[g]_i^2| from the all-reduced
//      sums of g and g^2.  Reference: optimizers/grad_variance.py:46-59.
//
// Structure: two-stage, deterministic (no float atomics): stage 1 grid-stride
// with 16-byte loads, wave64 shuffle + LDS block reduce, one partial per block;
// stage 2 a single block folds the partials.
#include "common.hpp"
#include "kernels.hpp"

namespace kfk {

namespace {

template <bool BF16, bool TWO>
__global__ __launch_bounds__(kBlock) void sumsq2_stage1(const void *a, const void *b, size_t n, bool vec,
                                                         float *partials) {
    __shared__ float lds[2][kBlock / kWave];
    float acc[2] = {0.f, 0.f};
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (BF16) {
        size_t n8 = vec ? n / 8 : 0;
        const uint4 *a8 = static_cast<const uint4 *>(a), *b8 = static_cast<const uint4 *>(b);
#pragma unroll 4
        for (size_t i = tid; i < n8; i += stride) {
            uint4 va = a8[i];
            const uint16_t *pa = reinterpret_cast<const uint16_t *>(&va);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                float x = bf16_to_f32(pa[k]);
                acc[0] += x * x;
            }
            if (TWO) {
                uint4 vb = b8[i];
                const uint16_t *pb = reinterpret_cast<const uint16_t *>(&vb);
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    float y = bf16_to_f32(pb[k]);
                    acc[1] += y * y;
                }
            }
        }
        for (size_t i = n8 * 8 + tid; i < n; i += stride) {
            float x = bf16_to_f32(static_cast<const uint16_t *>(a)[i]);
            acc[0] += x * x;
            if (TWO) {
                float y = bf16_to_f32(static_cast<const uint16_t *>(b)[i]);
                acc[1] += y * y;
            }
        }
    } else {
        size_t n4 = vec ? n / 4 : 0;
        const float4 *a4 = static_cast<const float4 *>(a), *b4 = static_cast<const float4 *>(b);
        size_t i = tid;
        // four 16-byte loads per operand in flight per lane (one per trip left most of an HBM
        // round trip exposed: 1.25 TB/s on a BERT-base gradient bucket)
        for (; i + 3 * stride < n4; i += 4 * stride) {
            float4 va[4], vb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                va[u] = a4[i + u * stride];
                if (TWO) vb[u] = b4[i + u * stride];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc[0] += va[u].x * va[u].x + va[u].y * va[u].y + va[u].z * va[u].z + va[u].w * va[u].w;
                if (TWO) acc[1] += vb[u].x * vb[u].x + vb[u].y * vb[u].y + vb[u].z * vb[u].z + vb[u].w * vb[u].w;
            }
        }
        for (; i < n4; i += stride) {
            float4 va = a4[i];
            acc[0] += va.x * va.x + va.y * va.y + va.z * va.z + va.w * va.w;
            if (TWO) {
                float4 vb = b4[i];
                acc[1] += vb.x * vb.x + vb.y * vb.y + vb.z * vb.z + vb.w * vb.w;
            }
        }
        for (size_t i = n4 * 4 + tid; i < n; i += stride) {
            float x = static_cast<const float *>(a)[i];
            acc[0] += x * x;
            if (TWO) {
                float y = static_cast<const float *>(b)[i];
                acc[1] += y * y;
            }
        }
    }
    block_sum<2>(acc, lds);
    if (threadIdx.x == 0) {
        partials[blockIdx.x] = acc[0];
        partials[kMaxGrid + blockIdx.x] = acc[1];
    }
}

__global__ __launch_bounds__(kBlock) void fold2(const float *partials, int nparts, float *out) {
    __shared__ float lds[2][kBlock / kWave];
    float acc[2] = {0.f, 0.f};
    int i = threadIdx.x;
    for (; i + 3 * kBlock < nparts; i += 4 * kBlock) {  // 8 loads in flight per lane, summed in order
        float u[4], v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            u[k] = partials[i + k * kBlock];
            v[k] = partials[kMaxGrid + i + k * kBlock];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            acc[0] += u[k];
            acc[1] += v[k];
        }
    }
    for (; i < nparts; i += kBlock) {
        acc[0] += partials[i];
        acc[1] += partials[kMaxGrid + i];
    }
    block_sum<2>(acc, lds);
    if (threadIdx.x == 0) {
        out[0] = acc[0];
        out[1] = acc[1];
    }
}

__global__ __launch_bounds__(kBlock) void variance_stage1(const float4 *s1, const float4 *s2, const float *s1t,
                                                          const float *s2t, size_t n, float inv, float *partials) {
    __shared__ float lds[1][kBlock / kWave];
    float acc[1] = {0.f};
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    size_t tid = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    size_t n4 = s1 ? n / 4 : 0;
#pragma unroll 4
    for (size_t i = tid; i < n4; i += stride) {
        float4 a = s1[i], b = s2[i];
        float m;
        m = a.x * inv;
        acc[0] += fabsf(b.x * inv - m * m);
        m = a.y * inv;
        acc[0] += fabsf(b.y * inv - m * m);
        m = a.z * inv;
        acc[0] += fabsf(b.z * inv - m * m);
        m = a.w * inv;
        acc[0] += fabsf(b.w * inv - m * m);
    }
    for (size_t i = n4 * 4 + tid; i < n; i += stride) {
        float m = s1t[i] * inv;
        acc[0] += fabsf(s2t[i] * inv - m * m);
    }
    block_sum<1>(acc, lds);
    if (threadIdx.x == 0) partials[blockIdx.x] = acc[0];
}

__global__ void fold1(const float *partials, int nparts, float *out) {
    __shared__ float lds[1][kBlock / kWave];
    float acc[1] = {0.f};
    int i = threadIdx.x;
    for (; i + 3 * kBlock < nparts; i += 4 * kBlock) {
        float u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = partials[i + k * kBlock];
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[0] += u[k];
    }
    for (; i < nparts; i += kBlock) acc[0] += partials[i];
    block_sum<1>(acc, lds);
    if (threadIdx.x == 0) out[0] = acc[0];
}

// state: [ema_G, ema_S, noise_scale, n_updates]
__global__ void gns_update_kernel(const float *sumsq_small, const float *sumsq_big, float b_small, float b_big,
                                  float alpha, float *state) {
    float gs = *sumsq_small, gb = *sumsq_big;
    // one peer (B == b): the estimator is undefined -- keep the state (count unchanged)
    if (!(b_big > b_small)) return;
    float G = (b_big * gb - b_small * gs) / (b_big - b_small);
    float S = (gs - gb) / (1.f / b_small - 1.f / b_big);
    float cnt = state[3];
    float eg = cnt == 0.f ? G : alpha * state[0] + (1.f - alpha) * G;
    float es = cnt == 0.f ? S : alpha * state[1] + (1.f - alpha) * S;
    state[0] = eg;
    state[1] = es;
    state[2] = eg != 0.f ? es / eg : 0.f;
    state[3] = cnt + 1.f;
}

inline bool al16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Per-segment (per-tensor) sum of d^2, d = s2*inv - (s1*inv)^2, over a flat
// buffer whose tensors start at seg_off[k].  Block b owns a contiguous chunk;
// lanes stride by 256 inside it, so loads stay coalesced and each lane's
// segment index only moves forward: one agent-scope float atomic per
// (lane, segment) it touched.
__global__ __launch_bounds__(kBlock) void seg_variance_kernel(const float *s1, const float *s2, int64_t n,
                                                              float inv, const int64_t *seg_off, int nseg,
                                                              int64_t chunk, float *out) {
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * chunk;
    int64_t b1 = b0 + chunk;
    if (b1 > n) b1 = n;
    int64_t i = b0 + threadIdx.x;
    if (i >= b1) return;
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (seg_off[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    int seg = lo;
    int64_t seg_end = seg_off[seg + 1];
    float acc = 0.f;
    for (; i < b1; i += kBlock) {
        while (i >= seg_end) {
            if (acc != 0.f) atomicAdd(out + seg, acc);
            acc = 0.f;
            ++seg;
            seg_end = seg_off[seg + 1];
        }
        float m = s1[i] * inv;
        float d = s2[i] * inv - m * m;
        acc += d * d;
    }
    if (acc != 0.f) atomicAdd(out + seg, acc);
}

}  // namespace

void launch_seg_variance(const float *s1, const float *s2, size_t n, float inv_np, const int64_t *seg_off, int nseg,
                         float *out, hipStream_t s) {
    if (n == 0 || nseg == 0) return;
    int64_t blocks = static_cast<int64_t>((n + kBlock * 16 - 1) / (kBlock * 16));
    if (blocks > kMaxGrid) blocks = kMaxGrid;
    int64_t chunk = (static_cast<int64_t>(n) + blocks - 1) / blocks;
    seg_variance_kernel<<<static_cast<int>(blocks), kBlock, 0, s>>>(s1, s2, static_cast<int64_t>(n), inv_np, seg_off,
                                                                     nseg, chunk, out);
}

void launch_sumsq2(const void *a, const void *b, size_t n, int dtype, float *partials, float *out, hipStream_t s) {
    bool bf = dtype == DT_BF16;
    size_t nvec = bf ? n / 8 : n / 4;
    int g = grid_for(nvec ? nvec : 1);
    bool aligned = al16(a) && (!b || al16(b));
    if (bf) {
        if (b) sumsq2_stage1<true, true><<<g, kBlock, 0, s>>>(a, b, n, aligned, partials);
        else sumsq2_stage1<true, false><<<g, kBlock, 0, s>>>(a, a, n, aligned, partials);
    } else {
        if (b) sumsq2_stage1<false, true><<<g, kBlock, 0, s>>>(a, b, n, aligned, partials);
        else sumsq2_stage1<false, false><<<g, kBlock, 0, s>>>(a, a, n, aligned, partials);
    }
    fold2<<<1, kBlock, 0, s>>>(partials, g, out);
}

void launch_variance(const float *s1, const float *s2, size_t n, float inv_np, float *partials, float *out,
                     hipStream_t s) {
    bool al = al16(s1) && al16(s2);
    int g = grid_for(al ? (n / 4 ? n / 4 : 1) : (n ? n : 1));
    variance_stage1<<<g, kBlock, 0, s>>>(al ? reinterpret_cast<const float4 *>(s1) : nullptr,
                                         reinterpret_cast<const float4 *>(s2), s1, s2, n, inv_np, partials);
    fold1<<<1, kBlock, 0, s>>>(partials, g, out);
}

void launch_gns_update(const float *sumsq_small, const float *sumsq_big, float b_small, float b_big, float alpha,
                       float *state, hipStream_t s) {
    gns_update_kernel<<<1, 1, 0, s>>>(sumsq_small, sumsq_big, b_small, b_big, alpha, state);
}

// ---- column sums of a bf16 [T, O] matrix (a linear layer's bias gradient) ---------------
// Stage 1: block = (row chunk, 64 column vectors of 8): each thread sums its 8 columns over the
// chunk's rows with 4 rows' loads in flight; partial f32 [chunks][O].  Stage 2: one thread per
// column sums the chunk partials in order (deterministic).
namespace {
constexpr int kColVec = 64;  // 8-column vectors per block (512 columns)

__device__ __forceinline__ void add8(const uint4 &q, float (&acc)[8]) {
    const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        acc[2 * k] += __uint_as_float(w[k] << 16);
        acc[2 * k + 1] += __uint_as_float(w[k] & 0xffff0000u);
    }
}

__global__ __launch_bounds__(256) void colsum_stage1(const uint4 *__restrict__ x, int64_t T, int OV, int rows_per,
                                                     float *__restrict__ part) {
    const int v = blockIdx.y * kColVec + (threadIdx.x % kColVec);
    const int rsub = threadIdx.x / kColVec;  // 4 row lanes
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per;
    int64_t r1 = r0 + rows_per;
    if (r1 > T) r1 = T;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    if (v < OV) {
        int64_t r = r0 + rsub;
        for (; r + 12 < r1; r += 16) {
            uint4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = x[(r + 4 * u) * OV + v];
#pragma unroll
            for (int u = 0; u < 4; ++u) add8(q[u], acc);
        }
        for (; r < r1; r += 4) {
            add8(x[r * OV + v], acc);
        }
    }
    __shared__ float red[4][kColVec * 8];
#pragma unroll
    for (int k = 0; k < 8; ++k) red[rsub][(threadIdx.x % kColVec) * 8 + k] = acc[k];
    __syncthreads();
    const int O = OV * 8;
    for (int c = threadIdx.x; c < kColVec * 8; c += 256) {
        const int col = blockIdx.y * kColVec * 8 + c;
        if (col < O) part[static_cast<int64_t>(blockIdx.x) * O + col] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
}


// y = x Phi(x) (erf GELU, torch's F.gelu default) on bf16, 16-byte vectors, two per trip.  Both this
// and torch's erff kernel are vector-issue bound (~2.5 TB/s on BERT-base's 16 K x 3072 FC1 output);
// measured 0.6 % slower end to end than torch's (KUNGFU_GELU_FWD A/B, r4t20): off by default.
__global__ __launch_bounds__(256) void gelu_fwd_kernel(const uint4 *__restrict__ u, uint4 *__restrict__ y,
                                                       int64_t nvec) {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
    for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i0 < nvec; i0 += 2 * stride) {
        uint4 q[2];
#pragma unroll
        for (int h = 0; h < 2; ++h)
            if (i0 + h * stride < nvec) q[h] = u[i0 + h * stride];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            if (i0 + h * stride >= nvec) break;
            const uint32_t *a = reinterpret_cast<const uint32_t *>(&q[h]);
            uint32_t o[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float x0 = __uint_as_float(a[k] << 16), x1 = __uint_as_float(a[k] & 0xffff0000u);
                o[k] = pack_bf16x2(x0 * gelu_cdf_fast(x0), x1 * gelu_cdf_fast(x1));
            }
            y[i0 + h * stride] = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
}

// GELU backward fused with the column sums of its output: du = dy * (Phi(u) + u * phi(u)) (the erf
// form of torch's GeluBackward, f32 math with gelu_grad_fast, one bf16 rounding), and per-chunk column partial sums of the
// bf16 du -- the bias gradient of the linear layer that produced u -- with colsum_stage1's layout
// (fixed 8-column group per thread, 4 row lanes per block, partials [chunk][O]).
__global__ __launch_bounds__(256) void gelu_bwd_colsum_stage1(const uint4 *__restrict__ dy, const uint4 *__restrict__ u,
                                                              uint4 *__restrict__ du, int64_t T, int OV, int rows_per,
                                                              float *__restrict__ part) {
    const int v = blockIdx.y * kColVec + (threadIdx.x % kColVec);
    const int rsub = threadIdx.x / kColVec;
    const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per;
    int64_t r1 = r0 + rows_per;
    if (r1 > T) r1 = T;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    if (v < OV) {
        for (int64_t r = r0 + rsub; r < r1; r += 8) {
            uint4 qd[2], qu[2];
            bool ok[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t rr = r + 4 * h;
                ok[h] = rr < r1;
                if (ok[h]) {
                    qd[h] = dy[rr * OV + v];
                    qu[h] = u[rr * OV + v];
                }
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                if (!ok[h]) continue;
                const uint32_t *a = reinterpret_cast<const uint32_t *>(&qd[h]);
                const uint32_t *b = reinterpret_cast<const uint32_t *>(&qu[h]);
                uint32_t o[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    float d2[2] = {__uint_as_float(a[k] << 16), __uint_as_float(a[k] & 0xffff0000u)};
                    float x2[2] = {__uint_as_float(b[k] << 16), __uint_as_float(b[k] & 0xffff0000u)};
                    uint16_t r2[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        r2[e] = f32_to_bf16(d2[e] * gelu_grad_fast(x2[e]));
                        acc[2 * k + e] += bf16_to_f32(r2[e]);
                    }
                    o[k] = static_cast<uint32_t>(r2[0]) | (static_cast<uint32_t>(r2[1]) << 16);
                }
                du[(r + 4 * h) * OV + v] = make_uint4(o[0], o[1], o[2], o[3]);
            }
        }
    }
    __shared__ float red[4][kColVec * 8];
#pragma unroll
    for (int k = 0; k < 8; ++k) red[rsub][(threadIdx.x % kColVec) * 8 + k] = acc[k];
    __syncthreads();
    const int O = OV * 8;
    for (int c = threadIdx.x; c < kColVec * 8; c += 256) {
        const int col = blockIdx.y * kColVec * 8 + c;
        if (col < O) part[static_cast<int64_t>(blockIdx.x) * O + col] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
    }
}

// one block per 32 columns: kC2Lanes chunk lanes per column each sum every kC2Lanes-th chunk partial
// (coalesced: the 32 columns of a row are adjacent), then the lane sums meet in LDS in a fixed order
// (deterministic).  32 lanes (1024 threads): ~11 loads per lane for GELU's 341 chunks -- with 8 lanes the
// 43-load chains made this ~10 us launch latency-bound (25 launches per BERT-base step).
constexpr int kC2Lanes = 32;
__global__ __launch_bounds__(32 * kC2Lanes) void colsum_stage2(const float *__restrict__ part, int chunks, int O,
                                                               float *out_f32, uint16_t *out_bf16) {
    __shared__ float red[kC2Lanes][33];
    const int cl = threadIdx.x & 31, lane = threadIdx.x >> 5;
    const int c = blockIdx.x * 32 + cl;
    float s0 = 0.f, s1 = 0.f;
    if (c < O) {
        int k = lane;
        for (; k + kC2Lanes < chunks; k += 2 * kC2Lanes) {  // two independent chains
            s0 += part[static_cast<int64_t>(k) * O + c];
            s1 += part[static_cast<int64_t>(k + kC2Lanes) * O + c];
        }
        if (k < chunks) s0 += part[static_cast<int64_t>(k) * O + c];
    }
    red[lane][cl] = s0 + s1;
    __syncthreads();
    if (lane == 0 && c < O) {
        float t = 0.f;
#pragma unroll
        for (int l = 0; l < kC2Lanes; ++l) t += red[l][cl];
        if (out_f32) out_f32[c] = t;
        else out_bf16[c] = f32_to_bf16(t);
    }
}
}  // namespace

int colsum_chunks(int64_t T, int O) {
    // ~512 stage-1 blocks (2 per CU), >= 16 rows per chunk
    const int colblocks = (O / 8 + kColVec - 1) / kColVec;
    int64_t c = 512 / colblocks;
    const int64_t cap = (T + 15) / 16;
    if (c > cap) c = cap;
    return static_cast<int>(c < 1 ? 1 : (c > 1024 ? 1024 : c));
}

void launch_colsum_bf16(const uint16_t *x, int64_t T, int O, float *part, float *out_f32, uint16_t *out_bf16,
                        hipStream_t s) {
    const int OV = O / 8, chunks = colsum_chunks(T, O);
    const int rows_per = static_cast<int>((T + chunks - 1) / chunks);
    dim3 g1(chunks, (OV + kColVec - 1) / kColVec);
    colsum_stage1<<<g1, 256, 0, s>>>(reinterpret_cast<const uint4 *>(x), T, OV, rows_per, part);
    colsum_stage2<<<(O + 31) / 32, 32 * kC2Lanes, 0, s>>>(part, chunks, O, out_f32, out_bf16);
}

void launch_colsum_fold(const float *part, int rows, int O, float *out_f32, uint16_t *out_bf16, hipStream_t s) {
    colsum_stage2<<<(O + 31) / 32, 32 * kC2Lanes, 0, s>>>(part, rows, O, out_f32, out_bf16);
}

void launch_gelu_forward(const uint16_t *u, uint16_t *y, int64_t n, hipStream_t s) {
    if (n % 8) throw std::invalid_argument("gelu_forward: element count must be a multiple of 8");
    const int64_t nvec = n / 8;
    int64_t g = (nvec + 511) / 512;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    gelu_fwd_kernel<<<static_cast<int>(g), 256, 0, s>>>(reinterpret_cast<const uint4 *>(u), reinterpret_cast<uint4 *>(y),
                                                        nvec);
}

int gelu_colsum_chunks(int64_t T, int O) {
    // the erf/exp math makes this pass VALU-heavy: ~8 workgroups per CU (vs colsum's 2), >= 16 rows each
    const int colblocks = (O / 8 + kColVec - 1) / kColVec;
    int64_t c = 2048 / colblocks;
    const int64_t cap = (T + 15) / 16;
    if (c > cap) c = cap;
    return static_cast<int>(c < 1 ? 1 : (c > 2048 ? 2048 : c));
}

void launch_gelu_bwd_colsum(const uint16_t *dy, const uint16_t *u, uint16_t *du, int64_t T, int O, float *part,
                            float *out_f32, uint16_t *out_bf16, hipStream_t s) {
    const int OV = O / 8, chunks = gelu_colsum_chunks(T, O);
    const int rows_per = static_cast<int>((T + chunks - 1) / chunks);
    dim3 g1(chunks, (OV + kColVec - 1) / kColVec);
    gelu_bwd_colsum_stage1<<<g1, 256, 0, s>>>(reinterpret_cast<const uint4 *>(dy), reinterpret_cast<const uint4 *>(u),
                                              reinterpret_cast<uint4 *>(du), T, OV, rows_per, part);
    colsum_stage2<<<(O + 31) / 32, 32 * kC2Lanes, 0, s>>>(part, chunks, O, out_f32, out_bf16);
}

}  // namespace kfk
