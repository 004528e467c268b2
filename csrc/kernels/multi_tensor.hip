// K7: multi-tensor pack / unpack between a list of tensors and one flat buffer,
// with a fused scale and dtype cast (f32 <-> bf16 <-> f16).
// Reference: fuse/defuse, srcs/python/kungfu/tensorflow/ops/__init__.py:29-46 and the
// fused NCCL path in optimizers/sync_sgd.py:87-92.
//
// One launch for the whole tensor list: the descriptor table (ptr, offset,
// numel) sorted by offset is staged into LDS once per block; each thread walks
// 4 consecutive flat elements and finds its tensor by binary search in LDS.
// Flat-side accesses are coalesced; the engine's hot path avoids pack/unpack
// entirely by keeping gradients as views of the flat bucket buffers.
#include "common.hpp"
#include "kernels.hpp"

namespace kfk {

namespace {

constexpr int kMaxLdsDesc = 1024;  // 24 KiB of LDS

__device__ __forceinline__ float load_as_f32(const void *p, size_t i, int dt) {
    if (dt == DT_F32) return static_cast<const float *>(p)[i];
    if (dt == DT_BF16) return bf16_to_f32(static_cast<const uint16_t *>(p)[i]);
    return f16_to_f32(static_cast<const uint16_t *>(p)[i]);
}

__device__ __forceinline__ void store_from_f32(void *p, size_t i, int dt, float v) {
    if (dt == DT_F32) static_cast<float *>(p)[i] = v;
    else if (dt == DT_BF16) static_cast<uint16_t *>(p)[i] = f32_to_bf16(v);
    else static_cast<uint16_t *>(p)[i] = f32_to_f16(v);
}

__device__ __forceinline__ int find_tensor(const int64_t *d, int n, int64_t idx) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (d[3 * mid + 1] <= idx) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

template <bool PACK>
__global__ __launch_bounds__(kBlock) void multi_copy(const int64_t *__restrict__ desc, int n_tensors, size_t total,
                                                     void *flat, int flat_dt, int t_dt, float scale) {
    __shared__ int64_t sd[3 * kMaxLdsDesc];
    const bool in_lds = n_tensors <= kMaxLdsDesc;
    if (in_lds) {
        for (int i = threadIdx.x; i < 3 * n_tensors; i += kBlock) sd[i] = desc[i];
        __syncthreads();
    }
    const int64_t *d = in_lds ? sd : desc;
    size_t stride = static_cast<size_t>(gridDim.x) * kBlock * 4;
    for (size_t base = (static_cast<size_t>(blockIdx.x) * kBlock + threadIdx.x) * 4; base < total; base += stride) {
        int t = find_tensor(d, n_tensors, static_cast<int64_t>(base));
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            size_t i = base + k;
            if (i >= total) break;
            while (t + 1 < n_tensors && d[3 * (t + 1) + 1] <= static_cast<int64_t>(i)) ++t;
            int64_t off = d[3 * t + 1], numel = d[3 * t + 2];
            int64_t j = static_cast<int64_t>(i) - off;
            if (j < 0 || j >= numel) continue;  // gap between tensors (alignment padding)
            void *tp = reinterpret_cast<void *>(d[3 * t]);
            if (PACK) store_from_f32(flat, i, flat_dt, scale * load_as_f32(tp, j, t_dt));
            else store_from_f32(tp, j, t_dt, scale * load_as_f32(flat, i, flat_dt));
        }
    }
}

}  // namespace

void launch_pack(const int64_t *desc, int n_tensors, size_t total, void *flat, int flat_dtype, int src_dtype,
                 float scale, hipStream_t s) {
    if (total == 0 || n_tensors == 0) return;
    multi_copy<true><<<grid_for((total + 3) / 4), kBlock, 0, s>>>(desc, n_tensors, total, flat, flat_dtype,
                                                                  src_dtype, scale);
}

void launch_unpack(const int64_t *desc, int n_tensors, size_t total, const void *flat, int flat_dtype,
                   int dst_dtype, float scale, hipStream_t s) {
    if (total == 0 || n_tensors == 0) return;
    multi_copy<false><<<grid_for((total + 3) / 4), kBlock, 0, s>>>(desc, n_tensors, total, const_cast<void *>(flat),
                                                                   flat_dtype, dst_dtype, scale);
}

}  // namespace kfk

// ---------------------------------------------------------------------------
// Bucket gradient accumulation: flat[off_t + j] += scale * src_t[j] for up to
// GradAccTable::kMax tensors in ONE launch.  The table travels in the kernel
// arguments (no descriptor upload, hipGraph-capturable); blocks are assigned
// to tensors by a prefix sum of per-tensor block counts, so each block streams
// a contiguous 8 Ki-element chunk of one tensor with 16-byte accesses (bf16
// sources: 8 elements per lane per iteration).  Used by the S-SGD engine to
// land the bf16 weight gradients of a whole bucket into the f32 flat gradient
// buffer right before its all-reduce (replaces a cast + an add per tensor).
namespace kfk {
namespace {

constexpr int kAccElemsPerBlock = kBlock * 8 * 4;

template <int SRC_DT>
__global__ __launch_bounds__(kBlock) void grad_accumulate_kernel(GradAccTable tab, float *__restrict__ flat) {
    const int b = blockIdx.x;
    int t = 0;
    while (t + 1 < tab.n && tab.blk_start[t + 1] <= b) ++t;
    const int64_t numel = tab.numel[t];
    const int64_t begin = static_cast<int64_t>(b - tab.blk_start[t]) * kAccElemsPerBlock;
    int64_t end = begin + kAccElemsPerBlock;
    if (end > numel) end = numel;
    float *dst = flat + tab.off[t];
    const float sc = tab.scale;
    const bool vec_ok = (reinterpret_cast<uintptr_t>(tab.src[t]) & 15) == 0 && (tab.off[t] & 3) == 0;
    int64_t j = begin + static_cast<int64_t>(threadIdx.x) * 8;
    if (vec_ok) {
        for (; j + 8 <= end; j += kBlock * 8) {
            float v[8];
            if (SRC_DT == DT_BF16) {
                const uint4 r = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(tab.src[t]) + j);
                const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    v[2 * i] = __uint_as_float(w[i] << 16);
                    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
                }
            } else {
                const float4 *s = reinterpret_cast<const float4 *>(static_cast<const float *>(tab.src[t]) + j);
                const float4 a = s[0], c = s[1];
                v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = c.x, v[5] = c.y, v[6] = c.z, v[7] = c.w;
            }
            float4 *d = reinterpret_cast<float4 *>(dst + j);
            float4 d0 = d[0], d1 = d[1];
            d0.x += sc * v[0], d0.y += sc * v[1], d0.z += sc * v[2], d0.w += sc * v[3];
            d1.x += sc * v[4], d1.y += sc * v[5], d1.z += sc * v[6], d1.w += sc * v[7];
            d[0] = d0;
            d[1] = d1;
        }
    }
    // scalar remainder (tail of the tensor, or unaligned source)
    for (; j < end; j += kBlock * 8) {
        for (int k = 0; k < 8 && j + k < end; ++k) {
            const float s = SRC_DT == DT_BF16 ? bf16_to_f32(static_cast<const uint16_t *>(tab.src[t])[j + k])
                                             : static_cast<const float *>(tab.src[t])[j + k];
            dst[j + k] += sc * s;
        }
    }
}

}  // namespace

int grad_accumulate_blocks(int64_t numel) {
    return static_cast<int>((numel + kAccElemsPerBlock - 1) / kAccElemsPerBlock);
}

void launch_grad_accumulate(const GradAccTable &tab, float *flat, hipStream_t s) {
    if (tab.n <= 0) return;
    const int blocks = tab.blk_start[tab.n];
    if (blocks <= 0) return;
    if (tab.src_dtype == DT_BF16) grad_accumulate_kernel<DT_BF16><<<blocks, kBlock, 0, s>>>(tab, flat);
    else grad_accumulate_kernel<DT_F32><<<blocks, kBlock, 0, s>>>(tab, flat);
}

}  // namespace kfk
