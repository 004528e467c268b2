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
        drow[i] = static_cast<uint32_t>(f32_to_bf16(a * g)) | (static_cast<uint32_t>(f32_to_bf16(b * g)) << 16);
    }
}

}  // namespace

void launch_xent_forward(const uint16_t *x, const int64_t *labels, int64_t R, int V, float *lse, float *loss,
                         hipStream_t s) {
    if (V % 2 || V <= 0) throw std::invalid_argument("xent: the class count must be even");
    if (R <= 0) return;
    xent_fwd_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(reinterpret_cast<const uint32_t *>(x), labels, V, lse, loss);
}

void launch_xent_backward(const uint16_t *x, const int64_t *labels, const float *lse, const float *scale, int64_t R,
                          int V, uint16_t *dx, hipStream_t s) {
    if (V % 2 || V <= 0) throw std::invalid_argument("xent: the class count must be even");
    if (R <= 0) return;
    xent_bwd_kernel<<<static_cast<int>(R), kXBlock, 0, s>>>(reinterpret_cast<const uint32_t *>(x), labels, lse, scale,
                                                           V, reinterpret_cast<uint32_t *>(dx));
}

}  // namespace kfk
