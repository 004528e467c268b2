// Softmax cross-entropy over bf16 logits, fused (BERT's masked-LM loss: 2,560 rows x 30,522
// classes per BERT-base step).
//
// Why: the stock path casts the bf16 logits to f32 (a 312 MB write), runs log_softmax (read 312 MB,
// write 312 MB) and nll; the backward zero-fills and scatters an f32 gradient, runs the log_softmax
// backward (read 624 MB, write 312 MB) and casts the result back to bf16 -- ~2 GB of traffic and
// ~0.9 ms per step in 10 launches (profiles/r4t13_bert_base_summary.md: loss/softmax + casts).
// Here the forward reads the bf16 row once (online max / sum of exponentials, f32) and keeps one
// f32 log-sum-exp per row; the backward reads the row again and writes the bf16 gradient
//   d logits[r, v] = (exp(x[r, v] - lse[r]) - [v == label[r]]) * scale
// with `scale` = d loss / (number of counted rows), read from device memory (no host sync).
//
// One workgroup (256 threads) per row; 4-byte (2 x bf16) loads: a row of an odd-by-2 vocabulary
// (30,522) is 4-byte but not 16-byte aligned.  Rows whose label is outside [0, V) (PyTorch's
// ignore_index, -100) contribute a zero loss and a zero gradient.
#include "common.hpp"
#include "kernels.hpp"

#include <stdexcept>

namespace kfk {

namespace {

constexpr int kXBlock = 256;

__device__ __forceinline__ void online_merge(float &m, float &s, float m2, float s2) {
    const float mm = fmaxf(m, m2);
    if (mm == -INFINITY) return;  // both empty
    s = s * __expf(m - mm) + s2 * __expf(m2 - mm);
    m = mm;
}

__global__ __launch_bounds__(kXBlock) void xent_fwd_kernel(const uint32_t *__restrict__ x, const int64_t *__restrict__ labels,
                                                          int V, float *__restrict__ lse, float *__restrict__ loss) {
    const int r = blockIdx.x;
    const int V2 = V / 2;
    const uint32_t *row = x + static_cast<int64_t>(r) * V2;
    float m = -INFINITY, s = 0.f;
    for (int i = threadIdx.x; i < V2; i += kXBlock) {
        const uint32_t w = row[i];
        const float a = __uint_as_float(w << 16), b = __uint_as_float(w & 0xffff0000u);
        const float mx = fmaxf(a, b);
        if (mx > m) {
            s = s * __expf(m - mx);
            m = mx;
        }
        s += __expf(a - m) + __expf(b - m);
    }
    // wave reduction, then across the 4 waves
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
        online_merge(m, s, m2, s2);
    }
    __shared__ float sm[kXBlock / 64], ss[kXBlock / 64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        sm[wave] = m;
        ss[wave] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = sm[0], S = ss[0];
        for (int w = 1; w < kXBlock / 64; ++w) online_merge(M, S, sm[w], ss[w]);
        const float l = M + __logf(S);
        lse[r] = l;
        const int64_t lab = labels[r];
        float xl = 0.f;
        if (lab >= 0 && lab < V) {
            const uint16_t *xb = reinterpret_cast<const uint16_t *>(row);
            xl = bf16_to_f32(xb[lab]);
        }
        loss[r] = (lab >= 0 && lab < V) ? l - xl : 0.f;
    }
}

__global__ __launch_bounds__(kXBlock) void xent_bwd_kernel(const uint32_t *__restrict__ x, const int64_t *__restrict__ labels,
                                                          const float *__restrict__ lse, const float *__restrict__ scale,
                                                          int V, uint32_t *__restrict__ dx) {
    const int r = blockIdx.x;
    const int V2 = V / 2;
    const int64_t lab = labels[r];
    const bool counted = lab >= 0 && lab < V;
    const float l = lse[r], g = counted ? scale[0] : 0.f;
    const uint32_t *row = x + static_cast<int64_t>(r) * V2;
    uint32_t *drow = dx + static_cast<int64_t>(r) * V2;
    for (int i = threadIdx.x; i < V2; i += kXBlock) {
        const uint32_t w = row[i];
        float a = __expf(__uint_as_float(w << 16) - l), b = __expf(__uint_as_float(w & 0xffff0000u) - l);
        if (2 * i == lab) a -= 1.f;
        if (2 * i + 1 == lab) b -= 1.f;
        drow[i] = pack_bf16x2(a * g, b * g);
    }
}

// Rows padded to a multiple of 8 classes (ld % 8 == 0: the vocabulary-projection GEMM's padded
// logits, gemm_nt_ld): 16-byte loads, four in flight per lane; classes >= V of the last chunk masked.
__device__ __forceinline__ void bf8_unpack(const uint4 v, float (&f)[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = __uint_as_float(w[k] << 16);
        f[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
    }
}

__global__ __launch_bounds__(kXBlock) void xent_fwd_vec_kernel(const uint16_t *__restrict__ x,
                                                              const int64_t *__restrict__ labels, int V, int64_t ld,
                                                              float *__restrict__ lse, float *__restrict__ loss) {
    const int r = blockIdx.x;
    const uint16_t *row = x + r * ld;
    const uint4 *rv = reinterpret_cast<const uint4 *>(row);
    const int nch = (V + 7) / 8;
    float m = -INFINITY, s = 0.f;
    auto fold = [&](const uint4 v, int c) {
        float f[8];
        bf8_unpack(v, f);
        float mx = -INFINITY;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (c * 8 + k >= V) f[k] = -INFINITY;
            mx = fmaxf(mx, f[k]);
        }
        if (mx > m) {
            s = s * __expf(m - mx);
            m = mx;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s += __expf(f[k] - m);
    };
    int c = threadIdx.x;
    for (; c + 3 * kXBlock < nch; c += 4 * kXBlock) {
        const uint4 v0 = rv[c], v1 = rv[c + kXBlock], v2 = rv[c + 2 * kXBlock], v3 = rv[c + 3 * kXBlock];
        fold(v0, c);
        fold(v1, c + kXBlock);
        fold(v2, c + 2 * kXBlock);
        fold(v3, c + 3 * kXBlock);
    }
    for (; c < nch; c += kXBlock) fold(rv[c], c);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
        online_merge(m, s, m2, s2);
    }
    __shared__ float sm[kXBlock / 64], ss[kXBlock / 64];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) {
        sm[wave] = m;
        ss[wave] = s;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        float M = sm[0], S = ss[0];
        for (int w = 1; w < kXBlock / 64; ++w) online_merge(M, S, sm[w], ss[w]);
        const float l = M + __logf(S);
        lse[r] = l;
        const int64_t lab = labels[r];
        const bool counted = lab >= 0 && lab < V;
        loss[r] = counted ? l - bf16_to_f32(row[lab]) : 0.f;
    }
}

__global__ __launch_bounds__(kXBlock) void xent_bwd_vec_kernel(const uint16_t *__restrict__ x,
                                                              const int64_t *__restrict__ labels,
                                                              const float *__restrict__ lse,
                                                              const float *__restrict__ scale, int V, int64_t ld,
                                                              uint16_t *__restrict__ dx) {
    const int r = blockIdx.x;
    const int64_t lab = labels[r];
    const bool counted = lab >= 0 && lab < V;
    const float l = lse[r], g = counted ? scale[0] : 0.f;
    const uint4 *rv = reinterpret_cast<const uint4 *>(x + r * ld);
    uint4 *dv = reinterpret_cast<uint4 *>(dx + r * ld);
    const int nch = (V + 7) / 8;
    auto grad = [&](const uint4 v, int c) {
        float f[8];
        bf8_unpack(v, f);
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int e = c * 8 + 2 * k;
            float a = e < V ? __expf(f[2 * k] - l) : 0.f, b = e + 1 < V ? __expf(f[2 * k + 1] - l) : 0.f;
            if (e == lab) a -= 1.f;
            if (e + 1 == lab) b -= 1.f;
            w[k] = pack_bf16x2(a * g, b * g);
        }
        return make_uint4(w[0], w[1], w[2], w[3]);
    };
    int c = threadIdx.x;
    for (; c + 3 * kXBlock < nch; c += 4 * kXBlock) {
        const uint4 v0 = rv[c], v1 = rv[c + kXBlock], v2 = rv[c + 2 * kXBlock], v3 = rv[c + 3 * kXBlock];
        dv[c] = grad(v0, c);
        dv[c + kXBlock] = grad(v1, c + kXBlock);
        dv[c + 2 * kXBlock] = grad(v2, c + 2 * kXBlock);
        dv[c + 3 * kXBlock] = grad(v3, c + 3 * kXBlock);
    }
    for (; c < nch; c += kXBlock) dv[c] = grad(rv[c], c);
}

}  // namespace

void launch_xent_forward(const uint16_t *x, const int64_t *labels, int64_t R, int V, float *lse, float *loss,
                         hipStream_t s, int64_t ld) {
    if (ld > 0) {  // padded rows: ld % 8 == 0, ld >= V, 16-byte aligned base
        if (ld % 8 || ld < V || V <= 0 || reinterpret_cast<uintptr_t>(x) % 16)
            throw std::invalid_argument("xent: padded rows need ld % 8 == 0, ld >= V and a 16-byte aligned base");
        if (R <= 0) return;
        xent_fwd_vec_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(x, labels, V, ld, lse, loss);
        return;
    }
    if (V % 2 || V <= 0) throw std::invalid_argument("xent: the class count must be even");
    if (R <= 0) return;
    xent_fwd_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(reinterpret_cast<const uint32_t *>(x), labels, V, lse, loss);
}

void launch_xent_backward(const uint16_t *x, const int64_t *labels, const float *lse, const float *scale, int64_t R,
                          int V, uint16_t *dx, hipStream_t s, int64_t ld) {
    if (ld > 0) {  // dx has the same padded row stride; the masked classes of the last chunk are written as 0
        if (ld % 8 || ld < V || V <= 0 || reinterpret_cast<uintptr_t>(x) % 16 || reinterpret_cast<uintptr_t>(dx) % 16)
            throw std::invalid_argument("xent: padded rows need ld % 8 == 0, ld >= V and 16-byte aligned bases");
        if (R <= 0) return;
        xent_bwd_vec_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(x, labels, lse, scale, V, ld, dx);
        return;
    }
    if (V % 2 || V <= 0) throw std::invalid_argument("xent: the class count must be even");
    if (R <= 0) return;
    xent_bwd_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(reinterpret_cast<const uint32_t *>(x), labels, lse, scale,
                                                           V, reinterpret_cast<uint32_t *>(dx));
}

}  // namespace kfk
