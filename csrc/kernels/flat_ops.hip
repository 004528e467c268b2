// Flat-buffer elementwise kernels: K1 reduce, K8 fused SGD / Adam steps,
// K3/K4 axpby (SMA blend, pair averaging), K2 scale, K6 square.
//
// All are HBM-bound streaming kernels: 16-byte loads per lane (float4 or
// 8 x bf16), grid-stride over <= 2048 blocks of 256 threads, scalar tail.
// Reference computations: srcs/go/kungfu/base/op.cpp:57-93 (K1),
// srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:103-109 (K2+K8),
// sma_sgd.py:60-67 (K3), async_sgd.py:128-133 (K4), grad_variance.py:46-59 (K6).
#include "common.hpp"
#include "kernels.hpp"

namespace kfk {

namespace {

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// ---------------------------------------------------------------- K1 reduce

template <typename T> struct Sum { __device__ static T ap(T a, T b) { return a + b; } };
template <typename T> struct Min { __device__ static T ap(T a, T b) { return b < a ? b : a; } };
template <typename T> struct Max { __device__ static T ap(T a, T b) { return a < b ? b : a; } };
template <typename T> struct Prod { __device__ static T ap(T a, T b) { return a * b; } };

template <typename T, template <typename> class Op>
__global__ __launch_bounds__(kBlock) void reduce_plain(T *__restrict__ z, const T *__restrict__ x,
                                                       const T *__restrict__ y, size_t n) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride)
        z[i] = Op<T>::ap(x[i], y[i]);
}

// 16-byte vectorised f32 path.
template <template <typename> class Op>
__global__ __launch_bounds__(kBlock) void reduce_f32x4(float4 *z, const float4 *x, const float4 *y, size_t n4) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
        float4 a = x[i], b = y[i], c;
        c.x = Op<float>::ap(a.x, b.x);
        c.y = Op<float>::ap(a.y, b.y);
        c.z = Op<float>::ap(a.z, b.z);
        c.w = Op<float>::ap(a.w, b.w);
        z[i] = c;
    }
}

// half types: 8 elements (16 B) per lane, f32 math.
template <bool BF16, template <typename> class Op>
__global__ __launch_bounds__(kBlock) void reduce_half8(uint4 *z, const uint4 *x, const uint4 *y, size_t n8) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n8; i += stride) {
        uint4 a = x[i], b = y[i], c;
        const uint16_t *pa = reinterpret_cast<const uint16_t *>(&a);
        const uint16_t *pb = reinterpret_cast<const uint16_t *>(&b);
        uint16_t *pc = reinterpret_cast<uint16_t *>(&c);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float fa = BF16 ? bf16_to_f32(pa[k]) : f16_to_f32(pa[k]);
            float fb = BF16 ? bf16_to_f32(pb[k]) : f16_to_f32(pb[k]);
            float fc = Op<float>::ap(fa, fb);
            pc[k] = BF16 ? f32_to_bf16(fc) : f32_to_f16(fc);
        }
        z[i] = c;
    }
}

template <bool BF16, template <typename> class Op>
__global__ void reduce_half_tail(uint16_t *z, const uint16_t *x, const uint16_t *y, size_t begin, size_t n) {
    size_t i = begin + blockIdx.x * kBlock + threadIdx.x;
    if (i < n) {
        float fa = BF16 ? bf16_to_f32(x[i]) : f16_to_f32(x[i]);
        float fb = BF16 ? bf16_to_f32(y[i]) : f16_to_f32(y[i]);
        float fc = Op<float>::ap(fa, fb);
        z[i] = BF16 ? f32_to_bf16(fc) : f32_to_f16(fc);
    }
}

template <template <typename> class Op>
void reduce_dispatch(void *z, const void *x, const void *y, size_t n, int dtype, hipStream_t s) {
    switch (dtype) {
    case DT_F32: {
        size_t n4 = 0;
        if (aligned16(z) && aligned16(x) && aligned16(y)) {
            n4 = n / 4;
            if (n4)
                reduce_f32x4<Op><<<grid_for(n4), kBlock, 0, s>>>(static_cast<float4 *>(z),
                                                                 static_cast<const float4 *>(x),
                                                                 static_cast<const float4 *>(y), n4);
        }
        size_t done = n4 * 4;
        if (done < n)
            reduce_plain<float, Op><<<grid_for(n - done), kBlock, 0, s>>>(
                static_cast<float *>(z) + done, static_cast<const float *>(x) + done,
                static_cast<const float *>(y) + done, n - done);
        return;
    }
    case DT_BF16:
    case DT_F16: {
        size_t n8 = 0;
        bool bf = dtype == DT_BF16;
        if (aligned16(z) && aligned16(x) && aligned16(y)) {
            n8 = n / 8;
            if (n8) {
                if (bf)
                    reduce_half8<true, Op><<<grid_for(n8), kBlock, 0, s>>>(
                        static_cast<uint4 *>(z), static_cast<const uint4 *>(x), static_cast<const uint4 *>(y), n8);
                else
                    reduce_half8<false, Op><<<grid_for(n8), kBlock, 0, s>>>(
                        static_cast<uint4 *>(z), static_cast<const uint4 *>(x), static_cast<const uint4 *>(y), n8);
            }
        }
        size_t done = n8 * 8;
        if (done < n) {
            int g = static_cast<int>((n - done + kBlock - 1) / kBlock);
            if (bf)
                reduce_half_tail<true, Op><<<g, kBlock, 0, s>>>(static_cast<uint16_t *>(z),
                                                                static_cast<const uint16_t *>(x),
                                                                static_cast<const uint16_t *>(y), done, n);
            else
                reduce_half_tail<false, Op><<<g, kBlock, 0, s>>>(static_cast<uint16_t *>(z),
                                                                 static_cast<const uint16_t *>(x),
                                                                 static_cast<const uint16_t *>(y), done, n);
        }
        return;
    }
#define KFK_PLAIN(D, T)                                                                                     \
    case D:                                                                                                 \
        reduce_plain<T, Op><<<grid_for(n), kBlock, 0, s>>>(static_cast<T *>(z), static_cast<const T *>(x), \
                                                           static_cast<const T *>(y), n);                   \
        return;
        KFK_PLAIN(DT_U8, uint8_t)
        KFK_PLAIN(DT_I32, int32_t)
        KFK_PLAIN(DT_I64, int64_t)
        KFK_PLAIN(DT_F64, double)
#undef KFK_PLAIN
    default: return;
    }
}

// ---------------------------------------------------------------- K8 SGD

template <bool NESTEROV, bool MOM>
__global__ __launch_bounds__(kBlock) void sgd_f32x4(float4 *__restrict__ w, const float4 *__restrict__ g,
                                                    float4 *__restrict__ m, ushort4 *__restrict__ shadow, size_t n4,
                                                    float lr, const float *lr_dev, float mu, float damp, float wd,
                                                    float gscale, bool first) {
    if (lr_dev) lr = *lr_dev;
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
        float4 wv = w[i], gv = g[i];
        float *pw = reinterpret_cast<float *>(&wv);
        const float *pg = reinterpret_cast<const float *>(&gv);
        float4 mv;
        float *pm = reinterpret_cast<float *>(&mv);
        if (MOM && !first) mv = m[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float d = pg[k] * gscale + wd * pw[k];
            if (MOM) {
                pm[k] = first ? d : mu * pm[k] + (1.f - damp) * d;
                d = NESTEROV ? d + mu * pm[k] : pm[k];
            }
            pw[k] -= lr * d;
        }
        w[i] = wv;
        if (MOM) m[i] = mv;
        if (shadow) {
            ushort4 sv;
            sv.x = f32_to_bf16(pw[0]);
            sv.y = f32_to_bf16(pw[1]);
            sv.z = f32_to_bf16(pw[2]);
            sv.w = f32_to_bf16(pw[3]);
            shadow[i] = sv;
        }
    }
}

template <bool NESTEROV, bool MOM>
__global__ void sgd_f32_tail(float *w, const float *g, float *m, uint16_t *shadow, size_t begin, size_t n, float lr,
                             const float *lr_dev, float mu, float damp, float wd, float gscale, bool first) {
    if (lr_dev) lr = *lr_dev;
    size_t i = begin + blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float d = g[i] * gscale + wd * w[i];
    if (MOM) {
        float mm = first ? d : mu * m[i] + (1.f - damp) * d;
        m[i] = mm;
        d = NESTEROV ? d + mu * mm : mm;
    }
    w[i] -= lr * d;
    if (shadow) shadow[i] = f32_to_bf16(w[i]);
}

// ---------------------------------------------------------------- Adam

template <bool ADAMW>
__global__ __launch_bounds__(kBlock) void adam_f32x4(float4 *__restrict__ w, const float4 *__restrict__ g,
                                                     float4 *__restrict__ m, float4 *__restrict__ v, size_t n4,
                                                     float lr, const float *lr_dev, float b1, float b2, float eps,
                                                     float wd, float gscale, const float *step_dev,
                                                     ushort4 *__restrict__ shadow) {
    if (lr_dev) lr = *lr_dev;
    float t = *step_dev;
    float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
    float step = lr / bc1, rbc2 = rsqrtf(bc2);
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
        float4 wv = w[i], gv = g[i], mv = m[i], vv = v[i];
        float *pw = reinterpret_cast<float *>(&wv);
        const float *pg = reinterpret_cast<const float *>(&gv);
        float *pm = reinterpret_cast<float *>(&mv);
        float *pv = reinterpret_cast<float *>(&vv);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float gg = pg[k] * gscale;
            if (ADAMW) pw[k] *= (1.f - lr * wd);
            else gg += wd * pw[k];
            pm[k] = b1 * pm[k] + (1.f - b1) * gg;
            pv[k] = b2 * pv[k] + (1.f - b2) * gg * gg;
            float denom = sqrtf(pv[k]) * rbc2 + eps;
            pw[k] -= step * pm[k] / denom;
        }
        w[i] = wv;
        m[i] = mv;
        v[i] = vv;
        // the bf16 compute shadow of the new weights (parallel/flat.py: the forward's cast is skipped)
        if (shadow) shadow[i] = make_ushort4(f32_to_bf16(pw[0]), f32_to_bf16(pw[1]), f32_to_bf16(pw[2]), f32_to_bf16(pw[3]));
    }
}

template <bool ADAMW>
__global__ void adam_f32_tail(float *w, const float *g, float *m, float *v, size_t begin, size_t n, float lr,
                              const float *lr_dev, float b1, float b2, float eps, float wd, float gscale,
                              const float *step_dev, uint16_t *shadow) {
    if (lr_dev) lr = *lr_dev;
    size_t i = begin + blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    float t = *step_dev;
    float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
    float gg = g[i] * gscale;
    float ww = w[i];
    if (ADAMW) ww *= (1.f - lr * wd);
    else gg += wd * ww;
    float mm = b1 * m[i] + (1.f - b1) * gg;
    float vv = b2 * v[i] + (1.f - b2) * gg * gg;
    m[i] = mm;
    v[i] = vv;
    w[i] = ww - (lr / bc1) * mm / (sqrtf(vv) * rsqrtf(bc2) + eps);
    if (shadow) shadow[i] = f32_to_bf16(w[i]);
}

// ---------------------------------------------------------------- axpby / scale / square

__global__ __launch_bounds__(kBlock) void axpby_f32x4(float4 *y, const float4 *x, float4 *z, size_t n4, float a,
                                                      float b) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
        float4 yv = y[i], xv = x[i];
        yv.x = a * yv.x + b * xv.x;
        yv.y = a * yv.y + b * xv.y;
        yv.z = a * yv.z + b * xv.z;
        yv.w = a * yv.w + b * xv.w;
        y[i] = yv;
        if (z) z[i] = yv;
    }
}

__global__ __launch_bounds__(kBlock) void axpby_bf16x8(uint4 *y, const uint4 *x, uint4 *z, size_t n8, float a,
                                                       float b) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n8; i += stride) {
        uint4 yv = y[i], xv = x[i];
        uint16_t *py = reinterpret_cast<uint16_t *>(&yv);
        const uint16_t *px = reinterpret_cast<const uint16_t *>(&xv);
#pragma unroll
        for (int k = 0; k < 8; ++k) py[k] = f32_to_bf16(a * bf16_to_f32(py[k]) + b * bf16_to_f32(px[k]));
        y[i] = yv;
        if (z) z[i] = yv;
    }
}

template <bool BF16>
__global__ void axpby_tail(void *y, const void *x, void *z, size_t begin, size_t n, float a, float b) {
    size_t i = begin + blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (BF16) {
        uint16_t *yy = static_cast<uint16_t *>(y);
        float r = a * bf16_to_f32(yy[i]) + b * bf16_to_f32(static_cast<const uint16_t *>(x)[i]);
        yy[i] = f32_to_bf16(r);
        if (z) static_cast<uint16_t *>(z)[i] = yy[i];
    } else {
        float *yy = static_cast<float *>(y);
        yy[i] = a * yy[i] + b * static_cast<const float *>(x)[i];
        if (z) static_cast<float *>(z)[i] = yy[i];
    }
}

template <int DTYPE>
__global__ __launch_bounds__(kBlock) void scale_kernel(void *x, size_t n, float alpha) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        if (DTYPE == DT_F32) static_cast<float *>(x)[i] *= alpha;
        else if (DTYPE == DT_BF16) {
            uint16_t *p = static_cast<uint16_t *>(x);
            p[i] = f32_to_bf16(bf16_to_f32(p[i]) * alpha);
        } else {
            uint16_t *p = static_cast<uint16_t *>(x);
            p[i] = f32_to_f16(f16_to_f32(p[i]) * alpha);
        }
    }
}

__global__ __launch_bounds__(kBlock) void scale_f32x4(float4 *x, size_t n4, float alpha) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) {
        float4 v = x[i];
        v.x *= alpha;
        v.y *= alpha;
        v.z *= alpha;
        v.w *= alpha;
        x[i] = v;
    }
}

template <bool BF16>
__global__ __launch_bounds__(kBlock) void square_kernel(float *dst, const void *src, size_t n) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n; i += stride) {
        float v = BF16 ? bf16_to_f32(static_cast<const uint16_t *>(src)[i]) : static_cast<const float *>(src)[i];
        dst[i] = v * v;
    }
}


// ---------------------------------------------------------------- cast copy
// dst = scale * src with a dtype change (f32 <-> bf16): the S-SGD engine's bf16
// gradient wire format (bucket -> comm buffer before the all-reduce, back after).
// 8 elements per lane: two float4 on the f32 side, one 16-byte bf16 vector.
template <int SRC, int DST>
__global__ __launch_bounds__(kBlock) void cast8_kernel(void *__restrict__ dst, const void *__restrict__ src, size_t n8,
                                                       float scale) {
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x; i < n8; i += stride) {
        float v[8];
        if (SRC == DT_F32) {
            const float4 *s = static_cast<const float4 *>(src) + 2 * i;
            const float4 a = s[0], b = s[1];
            v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
        } else {
            const uint4 r = static_cast<const uint4 *>(src)[i];
            const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                v[2 * k] = __uint_as_float(w[k] << 16);
                v[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= scale;
        if (DST == DT_F32) {
            float4 *d = static_cast<float4 *>(dst) + 2 * i;
            d[0] = make_float4(v[0], v[1], v[2], v[3]);
            d[1] = make_float4(v[4], v[5], v[6], v[7]);
        } else {
            uint4 o;
            o.x = f32_to_bf16(v[0]) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
            o.y = f32_to_bf16(v[2]) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
            o.z = f32_to_bf16(v[4]) | (static_cast<uint32_t>(f32_to_bf16(v[5])) << 16);
            o.w = f32_to_bf16(v[6]) | (static_cast<uint32_t>(f32_to_bf16(v[7])) << 16);
            static_cast<uint4 *>(dst)[i] = o;
        }
    }
}

__global__ void cast_tail_kernel(void *dst, const void *src, size_t begin, size_t n, int sdt, int ddt, float scale) {
    size_t i = begin + static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (i >= n) return;
    float v = sdt == DT_F32 ? static_cast<const float *>(src)[i] : bf16_to_f32(static_cast<const uint16_t *>(src)[i]);
    v *= scale;
    if (ddt == DT_F32) static_cast<float *>(dst)[i] = v;
    else static_cast<uint16_t *>(dst)[i] = f32_to_bf16(v);
}

}  // namespace

void launch_reduce(void *z, const void *x, const void *y, size_t n, int dtype, int op, hipStream_t s) {
    if (n == 0) return;
    switch (op) {
    case OP_SUM: reduce_dispatch<Sum>(z, x, y, n, dtype, s); break;
    case OP_MIN: reduce_dispatch<Min>(z, x, y, n, dtype, s); break;
    case OP_MAX: reduce_dispatch<Max>(z, x, y, n, dtype, s); break;
    case OP_PROD: reduce_dispatch<Prod>(z, x, y, n, dtype, s); break;
    }
}

void launch_sgd(float *w, const float *g, float *m, uint16_t *shadow, size_t n, float lr, const float *lr_dev,
                float mu, float damp, float wd, float gscale, bool nesterov, bool first, hipStream_t s) {
    if (n == 0) return;
    bool mom = mu != 0.f && m != nullptr;
    size_t n4 = (aligned16(w) && aligned16(g) && (!mom || aligned16(m)) &&
                 (!shadow || (reinterpret_cast<uintptr_t>(shadow) & 7u) == 0))
                    ? n / 4
                    : 0;
#define KFK_SGD(NES, MOM)                                                                                           \
    do {                                                                                                            \
        if (n4)                                                                                                     \
            sgd_f32x4<NES, MOM><<<grid_for(n4), kBlock, 0, s>>>(                                                    \
                reinterpret_cast<float4 *>(w), reinterpret_cast<const float4 *>(g), reinterpret_cast<float4 *>(m), \
                reinterpret_cast<ushort4 *>(shadow), n4, lr, lr_dev, mu, damp, wd, gscale, first);                 \
        if (n4 * 4 < n)                                                                                             \
            sgd_f32_tail<NES, MOM><<<static_cast<int>((n - n4 * 4 + kBlock - 1) / kBlock), kBlock, 0, s>>>(          \
                w, g, m, shadow, n4 * 4, n, lr, lr_dev, mu, damp, wd, gscale, first);                              \
    } while (0)
    if (!mom) KFK_SGD(false, false);
    else if (nesterov) KFK_SGD(true, true);
    else KFK_SGD(false, true);
#undef KFK_SGD
}

void launch_adam(float *w, const float *g, float *m, float *v, size_t n, float lr, const float *lr_dev, float b1,
                 float b2, float eps, float wd, bool adamw, float gscale, const float *step_dev, hipStream_t s,
                 uint16_t *shadow) {
    if (n == 0) return;
    size_t n4 = (aligned16(w) && aligned16(g) && aligned16(m) && aligned16(v) &&
                 (!shadow || (reinterpret_cast<uintptr_t>(shadow) & 7u) == 0))
                    ? n / 4
                    : 0;
#define KFK_ADAM(AW)                                                                                               \
    do {                                                                                                           \
        if (n4)                                                                                                    \
            adam_f32x4<AW><<<grid_for(n4), kBlock, 0, s>>>(                                                        \
                reinterpret_cast<float4 *>(w), reinterpret_cast<const float4 *>(g), reinterpret_cast<float4 *>(m), \
                reinterpret_cast<float4 *>(v), n4, lr, lr_dev, b1, b2, eps, wd, gscale, step_dev,                  \
                reinterpret_cast<ushort4 *>(shadow));                                                              \
        if (n4 * 4 < n)                                                                                            \
            adam_f32_tail<AW><<<static_cast<int>((n - n4 * 4 + kBlock - 1) / kBlock), kBlock, 0, s>>>(              \
                w, g, m, v, n4 * 4, n, lr, lr_dev, b1, b2, eps, wd, gscale, step_dev, shadow);                     \
    } while (0)
    if (adamw) KFK_ADAM(true);
    else KFK_ADAM(false);
#undef KFK_ADAM
}

void launch_axpby(void *y, const void *x, void *z, size_t n, float a, float b, int dtype, hipStream_t s) {
    if (n == 0) return;
    bool al = aligned16(y) && aligned16(x) && (!z || aligned16(z));
    if (dtype == DT_F32) {
        size_t n4 = al ? n / 4 : 0;
        if (n4)
            axpby_f32x4<<<grid_for(n4), kBlock, 0, s>>>(static_cast<float4 *>(y), static_cast<const float4 *>(x),
                                                         static_cast<float4 *>(z), n4, a, b);
        if (n4 * 4 < n)
            axpby_tail<false><<<static_cast<int>((n - n4 * 4 + kBlock - 1) / kBlock), kBlock, 0, s>>>(
                y, x, z, n4 * 4, n, a, b);
    } else {
        size_t n8 = al ? n / 8 : 0;
        if (n8)
            axpby_bf16x8<<<grid_for(n8), kBlock, 0, s>>>(static_cast<uint4 *>(y), static_cast<const uint4 *>(x),
                                                          static_cast<uint4 *>(z), n8, a, b);
        if (n8 * 8 < n)
            axpby_tail<true><<<static_cast<int>((n - n8 * 8 + kBlock - 1) / kBlock), kBlock, 0, s>>>(
                y, x, z, n8 * 8, n, a, b);
    }
}

void launch_scale(void *x, size_t n, float alpha, int dtype, hipStream_t s) {
    if (n == 0) return;
    if (dtype == DT_F32) {
        size_t n4 = aligned16(x) ? n / 4 : 0;
        if (n4) scale_f32x4<<<grid_for(n4), kBlock, 0, s>>>(static_cast<float4 *>(x), n4, alpha);
        if (n4 * 4 < n)
            scale_kernel<DT_F32><<<grid_for(n - n4 * 4), kBlock, 0, s>>>(static_cast<float *>(x) + n4 * 4,
                                                                         n - n4 * 4, alpha);
    } else if (dtype == DT_BF16) scale_kernel<DT_BF16><<<grid_for(n), kBlock, 0, s>>>(x, n, alpha);
    else scale_kernel<DT_F16><<<grid_for(n), kBlock, 0, s>>>(x, n, alpha);
}

void launch_square(float *dst, const void *src, size_t n, int dtype, hipStream_t s) {
    if (n == 0) return;
    if (dtype == DT_BF16) square_kernel<true><<<grid_for(n), kBlock, 0, s>>>(dst, src, n);
    else square_kernel<false><<<grid_for(n), kBlock, 0, s>>>(dst, src, n);
}

void launch_cast(void *dst, const void *src, size_t n, int src_dt, int dst_dt, float scale, hipStream_t s) {
    if (n == 0) return;
    size_t n8 = 0;
    if (aligned16(dst) && aligned16(src)) {
        n8 = n / 8;
        if (n8) {
            if (src_dt == DT_F32 && dst_dt == DT_BF16)
                cast8_kernel<DT_F32, DT_BF16><<<grid_for(n8), kBlock, 0, s>>>(dst, src, n8, scale);
            else if (src_dt == DT_BF16 && dst_dt == DT_F32)
                cast8_kernel<DT_BF16, DT_F32><<<grid_for(n8), kBlock, 0, s>>>(dst, src, n8, scale);
            else if (src_dt == DT_F32)
                cast8_kernel<DT_F32, DT_F32><<<grid_for(n8), kBlock, 0, s>>>(dst, src, n8, scale);
            else
                cast8_kernel<DT_BF16, DT_BF16><<<grid_for(n8), kBlock, 0, s>>>(dst, src, n8, scale);
        }
    }
    size_t done = n8 * 8;
    if (done < n) {
        int g = static_cast<int>((n - done + kBlock - 1) / kBlock);
        cast_tail_kernel<<<g, kBlock, 0, s>>>(dst, src, done, n, src_dt, dst_dt, scale);
    }
}

// Embedding gradient: grad[ids[t], :] += dy[t, :] (grad f32 [V, D], zeroed by the caller; dy f32
// or bf16 [T, D]).  A thread owns 4 columns of a run of `ch` consecutive tokens and sums them in
// registers while the id repeats, issuing one f32 atomic per column at every id change
// (hardware global_atomic_add_f32, -munsafe-fp-atomics).  Long runs for small vocabularies (the
// segment ids: 2 rows; per-address atomic chains of T/ch instead of T), short ones for large
// ones (random token ids: nothing to merge, many threads).  A fixed launch shape -- unlike a sort
// + unique-by-key segment reduction, whose work size comes from the data -- so a hipGraph can
// replay it.  The summation order is not deterministic.
namespace {
template <bool BF16>
__device__ __forceinline__ void emb_load4(const void *dy, int64_t e, float v[4]) {
    if constexpr (BF16) {
        const uint2 r = reinterpret_cast<const uint2 *>(dy)[e];
        v[0] = bf16_to_f32(static_cast<uint16_t>(r.x & 0xffff));
        v[1] = bf16_to_f32(static_cast<uint16_t>(r.x >> 16));
        v[2] = bf16_to_f32(static_cast<uint16_t>(r.y & 0xffff));
        v[3] = bf16_to_f32(static_cast<uint16_t>(r.y >> 16));
    } else {
        const float4 r = reinterpret_cast<const float4 *>(dy)[e];
        v[0] = r.x, v[1] = r.y, v[2] = r.z, v[3] = r.w;
    }
}

template <bool BF16>
__global__ __launch_bounds__(kBlock) void embedding_bwd_kernel(float *__restrict__ grad, const int64_t *__restrict__ ids,
                                                              const void *__restrict__ dy, int64_t T, int D4, int64_t V,
                                                              int ch) {
    const int64_t chunks = (T + ch - 1) / ch;
    const int64_t total = chunks * D4;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int64_t q = i / D4;
        const int c4 = static_cast<int>(i - q * D4);
        const int64_t t0 = q * ch, t1 = t0 + ch < T ? t0 + ch : T;
        int64_t cur = ids[t0];
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        constexpr int U = 4;  // tokens whose id and gradient loads are in flight together
        for (int64_t tb = t0; tb < t1; tb += U) {
            int64_t idu[U];
            float v[U][4];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (tb + u < t1) {
                    idu[u] = ids[tb + u];
                    emb_load4<BF16>(dy, (tb + u) * D4 + c4, v[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (tb + u >= t1) break;
                if (idu[u] != cur) {
                    if (cur >= 0 && cur < V) {  // padding / out-of-range ids contribute nothing
                        float *g = grad + cur * (static_cast<int64_t>(D4) * 4) + c4 * 4;
#pragma unroll
                        for (int k = 0; k < 4; ++k) atomicAdd(g + k, acc[k]);
                    }
                    cur = idu[u];
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] = 0.f;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) acc[k] += v[u][k];
            }
        }
        if (cur >= 0 && cur < V) {
            float *g = grad + cur * (static_cast<int64_t>(D4) * 4) + c4 * 4;
#pragma unroll
            for (int k = 0; k < 4; ++k) atomicAdd(g + k, acc[k]);
        }
    }
}
}  // namespace

void launch_embedding_backward(float *grad, const int64_t *ids, const void *dy, bool dy_bf16, int64_t T, int D,
                               int64_t V, hipStream_t s, int ch) {
    if (T <= 0) return;
    if (D % 4) throw std::invalid_argument("embedding_backward: D must be a multiple of 4");
    if (ch <= 0) {  // long runs only where rows repeat a lot and there are tokens to spare
        const int64_t per_row = T / (V > 0 ? V : 1);
        ch = per_row >= 512 ? 64 : 4;  // segment ids (V = 2, T = 16 K): 64 -> 25 us, 128 -> 42, 4 -> 212
    }
    const int64_t total = (T + ch - 1) / ch * (D / 4);
    int64_t g = (total + kBlock - 1) / kBlock;
    if (g > 8192) g = 8192;
    if (dy_bf16)
        embedding_bwd_kernel<true><<<static_cast<int>(g), kBlock, 0, s>>>(grad, ids, dy, T, D / 4, V, ch);
    else
        embedding_bwd_kernel<false><<<static_cast<int>(g), kBlock, 0, s>>>(grad, ids, dy, T, D / 4, V, ch);
}

namespace {
const uint32_t *g_dropout_seed_base = nullptr;
}
void set_dropout_seed_base(const uint32_t *p) { g_dropout_seed_base = p; }
const uint32_t *dropout_seed_base() { return g_dropout_seed_base; }

}  // namespace kfk
