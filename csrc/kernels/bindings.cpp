// torch binding of the CDNA4 kernels and the RCCL controller: kungfu_amd._hip
//
// Every op enqueues on the current HIP stream of the tensor's device (or an
// explicit stream handle) and never synchronises the host.
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <torch/extension.h>

#include "kernels.hpp"
#include "rccl_comm.hpp"

#include <memory>
#include <tuple>
#include <vector>
#include <cstring>
#include <csignal>
#include <execinfo.h>
#include <unistd.h>

namespace {

int dtype_code(const at::Tensor &t) {
    switch (t.scalar_type()) {
    case at::kByte: return 0;
    case at::kChar: return 4;
    case at::kInt: return 6;
    case at::kLong: return 7;
    case at::kHalf: return 8;
    case at::kBFloat16: return 9;
    case at::kFloat: return 10;
    case at::kDouble: return 11;
    case at::kBool: return 12;
    default: TORCH_CHECK(false, "kungfu_amd._hip: unsupported dtype ", t.scalar_type());
    }
    return -1;
}

hipStream_t stream_of(const at::Tensor &t, int64_t stream) {
    if (stream) return reinterpret_cast<hipStream_t>(stream);
    return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void check_gpu(const at::Tensor &t, const char *name) {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void reduce_op(at::Tensor z, at::Tensor x, at::Tensor y, int64_t op) {
    check_gpu(z, "z");
    check_gpu(x, "x");
    check_gpu(y, "y");
    TORCH_CHECK(x.numel() == y.numel() && z.numel() == x.numel(), "reduce: size mismatch");
    TORCH_CHECK(x.scalar_type() == y.scalar_type() && z.scalar_type() == x.scalar_type(), "reduce: dtype mismatch");
    c10::DeviceGuard g(z.device());
    kfk::launch_reduce(z.data_ptr(), x.data_ptr(), y.data_ptr(), x.numel(), dtype_code(x), static_cast<int>(op),
                       stream_of(z, 0));
}

void sgd_step(at::Tensor w, at::Tensor g, c10::optional<at::Tensor> m, c10::optional<at::Tensor> shadow, double lr,
              c10::optional<at::Tensor> lr_t, double mu, double damp, double wd, double gscale, bool nesterov,
              bool first) {
    check_gpu(w, "w");
    check_gpu(g, "g");
    TORCH_CHECK(w.scalar_type() == at::kFloat && g.scalar_type() == at::kFloat, "sgd_step: f32 buffers required");
    TORCH_CHECK(w.numel() == g.numel(), "sgd_step: size mismatch");
    float *mp = nullptr;
    if (m && m->defined()) {
        check_gpu(*m, "m");
        TORCH_CHECK(m->numel() == w.numel() && m->scalar_type() == at::kFloat, "sgd_step: bad momentum buffer");
        mp = m->data_ptr<float>();
    }
    uint16_t *sp = nullptr;
    if (shadow && shadow->defined()) {
        TORCH_CHECK(shadow->scalar_type() == at::kBFloat16 && shadow->numel() == w.numel(), "sgd_step: bad shadow");
        sp = reinterpret_cast<uint16_t *>(shadow->data_ptr());
    }
    const float *lrp = nullptr;
    if (lr_t && lr_t->defined()) {
        TORCH_CHECK(lr_t->is_cuda() && lr_t->scalar_type() == at::kFloat, "sgd_step: lr tensor must be f32 on GPU");
        lrp = lr_t->data_ptr<float>();
    }
    c10::DeviceGuard gd(w.device());
    kfk::launch_sgd(w.data_ptr<float>(), g.data_ptr<float>(), mp, sp, w.numel(), static_cast<float>(lr), lrp,
                    static_cast<float>(mu), static_cast<float>(damp), static_cast<float>(wd),
                    static_cast<float>(gscale), nesterov, first, stream_of(w, 0));
}

void adam_step(at::Tensor w, at::Tensor g, at::Tensor m, at::Tensor v, double lr, c10::optional<at::Tensor> lr_t,
               double b1, double b2, double eps, double wd, bool adamw, double gscale, at::Tensor step,
               c10::optional<at::Tensor> shadow) {
    for (auto *t : {&w, &g, &m, &v}) {
        check_gpu(*t, "adam buffer");
        TORCH_CHECK(t->scalar_type() == at::kFloat && t->numel() == w.numel(), "adam_step: f32 buffers of equal size");
    }
    TORCH_CHECK(step.is_cuda() && step.scalar_type() == at::kFloat, "adam_step: step must be an f32 GPU tensor");
    const float *lrp = (lr_t && lr_t->defined()) ? lr_t->data_ptr<float>() : nullptr;
    uint16_t *sh = nullptr;
    if (shadow && shadow->defined()) {
        TORCH_CHECK(shadow->is_cuda() && shadow->scalar_type() == at::kBFloat16 && shadow->is_contiguous() &&
                        shadow->numel() == w.numel() && shadow->device() == w.device(),
                    "adam_step: shadow must be a contiguous bf16 buffer of the weights' size");
        sh = reinterpret_cast<uint16_t *>(shadow->data_ptr());
    }
    c10::DeviceGuard gd(w.device());
    kfk::launch_adam(w.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), w.numel(),
                     static_cast<float>(lr), lrp, static_cast<float>(b1), static_cast<float>(b2),
                     static_cast<float>(eps), static_cast<float>(wd), adamw, static_cast<float>(gscale),
                     step.data_ptr<float>(), stream_of(w, 0), sh);
}

void axpby(at::Tensor y, at::Tensor x, c10::optional<at::Tensor> z, double a, double b) {
    check_gpu(y, "y");
    check_gpu(x, "x");
    TORCH_CHECK(x.numel() == y.numel() && x.scalar_type() == y.scalar_type(), "axpby: mismatch");
    TORCH_CHECK(y.scalar_type() == at::kFloat || y.scalar_type() == at::kBFloat16, "axpby: f32/bf16 only");
    void *zp = nullptr;
    if (z && z->defined()) {
        check_gpu(*z, "z");
        TORCH_CHECK(z->numel() == y.numel() && z->scalar_type() == y.scalar_type(), "axpby: bad z");
        zp = z->data_ptr();
    }
    c10::DeviceGuard gd(y.device());
    kfk::launch_axpby(y.data_ptr(), x.data_ptr(), zp, y.numel(), static_cast<float>(a), static_cast<float>(b),
                      dtype_code(y), stream_of(y, 0));
}

void scale_(at::Tensor x, double alpha) {
    check_gpu(x, "x");
    int dt = dtype_code(x);
    TORCH_CHECK(dt == 8 || dt == 9 || dt == 10, "scale_: float types only");
    c10::DeviceGuard gd(x.device());
    kfk::launch_scale(x.data_ptr(), x.numel(), static_cast<float>(alpha), dt, stream_of(x, 0));
}

void square(at::Tensor dst, at::Tensor src) {
    check_gpu(dst, "dst");
    check_gpu(src, "src");
    TORCH_CHECK(dst.scalar_type() == at::kFloat && dst.numel() == src.numel(), "square: f32 dst of equal size");
    c10::DeviceGuard gd(dst.device());
    kfk::launch_square(dst.data_ptr<float>(), src.data_ptr(), src.numel(), dtype_code(src), stream_of(dst, 0));
}

void cast_copy(at::Tensor dst, at::Tensor src, double scale) {
    check_gpu(dst, "dst");
    check_gpu(src, "src");
    const int sd = dtype_code(src), dd = dtype_code(dst);
    TORCH_CHECK((sd == 9 || sd == 10) && (dd == 9 || dd == 10), "cast_copy: f32/bf16 only");
    TORCH_CHECK(dst.numel() == src.numel() && dst.device() == src.device(), "cast_copy: size/device mismatch");
    c10::DeviceGuard gd(dst.device());
    kfk::launch_cast(dst.data_ptr(), src.data_ptr(), src.numel(), sd, dd, static_cast<float>(scale), stream_of(dst, 0));
}

at::Tensor sumsq2(at::Tensor a, c10::optional<at::Tensor> b) {
    check_gpu(a, "a");
    int dt = dtype_code(a);
    TORCH_CHECK(dt == 9 || dt == 10, "sumsq2: f32/bf16 only");
    const void *bp = nullptr;
    if (b && b->defined()) {
        check_gpu(*b, "b");
        TORCH_CHECK(b->numel() == a.numel() && b->scalar_type() == a.scalar_type(), "sumsq2: mismatch");
        bp = b->data_ptr();
    }
    c10::DeviceGuard gd(a.device());
    auto opts = a.options().dtype(at::kFloat);
    auto partials = at::empty({2 * kfk::kMaxGridHost}, opts);
    auto out = at::empty({2}, opts);
    kfk::launch_sumsq2(a.data_ptr(), bp, a.numel(), dt, partials.data_ptr<float>(), out.data_ptr<float>(),
                       stream_of(a, 0));
    return out;
}

at::Tensor variance(at::Tensor s1, at::Tensor s2, double inv_np) {
    check_gpu(s1, "s1");
    check_gpu(s2, "s2");
    TORCH_CHECK(s1.scalar_type() == at::kFloat && s2.scalar_type() == at::kFloat && s1.numel() == s2.numel(),
                "variance: f32 buffers of equal size");
    c10::DeviceGuard gd(s1.device());
    auto opts = s1.options();
    auto partials = at::empty({kfk::kMaxGridHost}, opts);
    auto out = at::empty({1}, opts);
    kfk::launch_variance(s1.data_ptr<float>(), s2.data_ptr<float>(), s1.numel(), static_cast<float>(inv_np),
                         partials.data_ptr<float>(), out.data_ptr<float>(), stream_of(s1, 0));
    return out;
}

// Per-tensor L2 norms of E[g^2]-E[g]^2 summed over tensors (the reference's
// gradient variance, grad_variance.py:46-59).  seg_off: int64 GPU [nseg+1].
at::Tensor seg_variance(at::Tensor s1, at::Tensor s2, at::Tensor seg_off, double inv_np) {
    check_gpu(s1, "s1");
    check_gpu(s2, "s2");
    TORCH_CHECK(seg_off.is_cuda() && seg_off.scalar_type() == at::kLong && seg_off.numel() >= 2,
                "seg_variance: int64 GPU offsets required");
    TORCH_CHECK(s1.scalar_type() == at::kFloat && s2.scalar_type() == at::kFloat && s1.numel() == s2.numel(),
                "seg_variance: f32 buffers of equal size");
    c10::DeviceGuard gd(s1.device());
    const int nseg = static_cast<int>(seg_off.numel() - 1);
    auto out = at::zeros({nseg}, s1.options());
    kfk::launch_seg_variance(s1.data_ptr<float>(), s2.data_ptr<float>(), s1.numel(), static_cast<float>(inv_np),
                             seg_off.data_ptr<int64_t>(), nseg, out.data_ptr<float>(), stream_of(s1, 0));
    return out.sqrt().sum();
}

void gns_update(at::Tensor sumsq_small, at::Tensor sumsq_big, double b_small, double b_big, double alpha,
                at::Tensor state) {
    TORCH_CHECK(state.is_cuda() && state.scalar_type() == at::kFloat && state.numel() >= 4, "gns_update: bad state");
    c10::DeviceGuard gd(state.device());
    kfk::launch_gns_update(sumsq_small.data_ptr<float>(), sumsq_big.data_ptr<float>(), static_cast<float>(b_small),
                           static_cast<float>(b_big), static_cast<float>(alpha), state.data_ptr<float>(),
                           stream_of(state, 0));
}

// desc: int64 GPU tensor [n, 3] of (ptr, offset, numel), sorted by offset.
void pack(at::Tensor desc, int64_t n_tensors, int64_t src_dtype, at::Tensor flat, double scale) {
    check_gpu(flat, "flat");
    TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong, "pack: desc must be int64 on GPU");
    c10::DeviceGuard gd(flat.device());
    kfk::launch_pack(desc.data_ptr<int64_t>(), static_cast<int>(n_tensors), flat.numel(), flat.data_ptr(),
                     dtype_code(flat), static_cast<int>(src_dtype), static_cast<float>(scale), stream_of(flat, 0));
}

void unpack(at::Tensor desc, int64_t n_tensors, int64_t dst_dtype, at::Tensor flat, double scale) {
    check_gpu(flat, "flat");
    TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong, "unpack: desc must be int64 on GPU");
    c10::DeviceGuard gd(flat.device());
    kfk::launch_unpack(desc.data_ptr<int64_t>(), static_cast<int>(n_tensors), flat.numel(), flat.data_ptr(),
                       dtype_code(flat), static_cast<int>(dst_dtype), static_cast<float>(scale), stream_of(flat, 0));
}

// flat[offsets[i] : offsets[i] + srcs[i].numel()] += scale * srcs[i] (memory order), batched into
// launches of up to GradAccTable::kMax same-dtype tensors.  srcs must be dense (any stride
// permutation); the caller guarantees the flat slot uses the same memory order.
void grad_accumulate(at::Tensor flat, std::vector<at::Tensor> srcs, std::vector<int64_t> offsets, double scale) {
    check_gpu(flat, "flat");
    TORCH_CHECK(flat.scalar_type() == at::kFloat && flat.is_contiguous(), "grad_accumulate: flat must be f32");
    TORCH_CHECK(srcs.size() == offsets.size(), "grad_accumulate: srcs/offsets length mismatch");
    for (const auto &t : srcs)
        TORCH_CHECK(dtype_code(t) == 9 || dtype_code(t) == 10,
                    "grad_accumulate: bf16 or f32 sources only");
    // Sources are consumed on the current stream, the one they were produced
    // on, so the caching allocator's stream-ordered reuse keeps them valid.
    c10::DeviceGuard gd(flat.device());
    auto s = stream_of(flat, 0);
    for (int dt : {9, 10}) {
        kfk::GradAccTable tab;
        tab.src_dtype = dt;
        tab.scale = static_cast<float>(scale);
        tab.blk_start[0] = 0;
        auto flush = [&] {
            kfk::launch_grad_accumulate(tab, flat.data_ptr<float>(), s);
            tab.n = 0;
        };
        for (size_t i = 0; i < srcs.size(); ++i) {
            const auto &t = srcs[i];
            if (dtype_code(t) != dt) continue;
            TORCH_CHECK(t.device() == flat.device(), "grad_accumulate: device mismatch");
            TORCH_CHECK(t.is_non_overlapping_and_dense(), "grad_accumulate: source must be dense");
            TORCH_CHECK(offsets[i] >= 0 && offsets[i] + t.numel() <= flat.numel(), "grad_accumulate: out of range");
            if (t.numel() == 0) continue;
            const int k = tab.n;
            tab.src[k] = t.data_ptr();
            tab.off[k] = offsets[i];
            tab.numel[k] = t.numel();
            tab.blk_start[k + 1] = tab.blk_start[k] + kfk::grad_accumulate_blocks(t.numel());
            tab.n = k + 1;
            if (tab.n == kfk::GradAccTable::kMax) flush();
        }
        flush();
    }
}

// ---- 3x3 implicit-GEMM convolution -------------------------------------------------

at::Tensor conv3x3(at::Tensor x, at::Tensor w, int64_t stride, int64_t variant) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3: x must be a 4-D channels_last bf16 GPU tensor");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                    w.size(1) == x.size(1) && w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3: w must be [Cout, Cin, 3, 3] channels_last bf16");
    const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
    TORCH_CHECK(kfk::conv3x3_supported(C, K, static_cast<int>(stride)), "conv3x3: unsupported channels/stride");
    TORCH_CHECK(static_cast<int64_t>(N) * H * W * std::max(C, K) < (int64_t(1) << 31), "conv3x3: tensor too large");
    const int OH = (H + 2 - 3) / stride + 1, OW = (W + 2 - 3) / stride + 1;
    c10::DeviceGuard gd(x.device());
    auto y = at::empty({N, K, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_conv3x3(reinterpret_cast<const uint16_t *>(x.data_ptr()), reinterpret_cast<const uint16_t *>(w.data_ptr()),
                        reinterpret_cast<uint16_t *>(y.data_ptr()), N, H, W, C, K, static_cast<int>(stride),
                        stream_of(x, 0), static_cast<int>(variant));
    return y;
}

// General 1x1 / 3x3 convolution with fused epilogues (conv.hip).
// stats: f64 [kStatSlots*2*Cout] zero-initialised workspace receiving sum / sum of squares of the
// bf16 outputs per channel (consumed and re-zeroed by bn_forward(..., sums=stats)).
// out: accumulate target (y = out + conv(x, w), written in place and returned).
// bn_x / bn_fcoef / bn_mask (backward): the output is the gradient of a BN(+ReLU) output whose
// input is bn_x; stats then receive sum(dz), sum(dz * x) (dz = grad * relu') for
// bn_backward(..., sums=stats).  bn_mask (1 bit per element) or bn_fcoef (forward
// [scale; shift]) gives the ReLU gate.
// In-launch BN finalize descriptor (kfk::BNFin) packed on the host into a CPU uint8 tensor; the
// caller keeps a device copy and passes it to conv / conv_dgrad_s2 as `fin`.  mode 1 (forward):
//   t = [arrive(int32 >= 9, zeroed), gamma, beta, mean, invstd, coef(2C), running_mean, running_var, num_batches]
// mode 2 (backward): t = [arrive, gamma, mean, invstd, coef(3C), dgamma, dbeta]; f32 per-channel tensors.
at::Tensor bn_fin_desc(int64_t mode, std::vector<at::Tensor> v, int64_t rows, double momentum, double eps,
                       bool training) {
    TORCH_CHECK(mode == 1 || mode == 2, "bn_fin_desc: mode 1 (forward) or 2 (backward)");
    TORCH_CHECK(v.size() == (mode == 1 ? 9u : 7u), "bn_fin_desc: wrong tensor count for the mode");
    TORCH_CHECK(v[0].is_cuda() && v[0].scalar_type() == at::kInt && v[0].numel() >= 9 && v[0].is_contiguous(),
                "bn_fin_desc: arrive must be a zeroed int32 GPU tensor of >= 9 words");
    const int C = static_cast<int>(v[1].numel());
    auto f32 = [&](const at::Tensor &a, int64_t n, const char *what) -> float * {
        TORCH_CHECK(a.defined() && a.scalar_type() == at::kFloat && a.numel() == n && a.is_contiguous() &&
                        a.device() == v[0].device(),
                    "bn_fin_desc: ", what, " must be a contiguous f32 tensor of ", n, " elements on arrive's device");
        return a.data_ptr<float>();
    };
    kfk::BNFin f;
    f.mode = static_cast<int>(mode);
    f.arrive = reinterpret_cast<unsigned *>(v[0].data_ptr<int>());
    f.rows = rows;
    f.training = training ? 1 : 0;
    f.momentum = static_cast<float>(momentum), f.eps = static_cast<float>(eps);
    f.gamma = f32(v[1], C, "gamma");
    if (mode == 1) {
        f.beta = f32(v[2], C, "beta");
        f.mean = f32(v[3], C, "mean");
        f.invstd = f32(v[4], C, "invstd");
        f.coef = f32(v[5], 2 * C, "coef");
        f.run_mean = f32(v[6], C, "running_mean");
        f.run_var = f32(v[7], C, "running_var");
        TORCH_CHECK(v[8].scalar_type() == at::kLong && v[8].numel() == 1, "bn_fin_desc: num_batches must be int64[1]");
        f.num_batches = v[8].data_ptr<int64_t>();
    } else {
        f.mean = f32(v[2], C, "mean");
        f.invstd = f32(v[3], C, "invstd");
        f.coef = f32(v[4], 3 * C, "coef");
        f.dgamma = f32(v[5], C, "dgamma");
        f.dbeta = f32(v[6], C, "dbeta");
    }
    auto out = at::empty({static_cast<int64_t>(sizeof(kfk::BNFin))}, at::TensorOptions().dtype(at::kByte));
    std::memcpy(out.data_ptr<uint8_t>(), &f, sizeof(f));
    return out;
}

static const kfk::BNFin *fin_ptr(const c10::optional<at::Tensor> &fin, const at::Tensor &like, int C) {
    if (!fin || !fin->defined()) return nullptr;
    TORCH_CHECK(fin->is_cuda() && fin->device() == like.device() && fin->scalar_type() == at::kByte &&
                    fin->numel() == static_cast<int64_t>(sizeof(kfk::BNFin)) && fin->is_contiguous(),
                "fin: must be the device copy of a bn_fin_desc descriptor on the conv's device");
    return reinterpret_cast<const kfk::BNFin *>(fin->data_ptr<uint8_t>());
}

at::Tensor conv(at::Tensor x, at::Tensor w, int64_t stride, c10::optional<at::Tensor> stats,
                c10::optional<at::Tensor> out, int64_t variant, c10::optional<at::Tensor> bn_x,
                c10::optional<at::Tensor> bn_fcoef, c10::optional<at::Tensor> bn_mask,
                c10::optional<at::Tensor> bias, bool gate, c10::optional<at::Tensor> acc_mask, bool acc_even,
                c10::optional<at::Tensor> fin) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv: x must be a 4-D channels_last bf16 GPU tensor");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == w.size(3) && w.size(1) == x.size(1) &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.device() == x.device(),
                "conv: w must be [Cout, Cin, KS, KS] channels_last bf16 on x's device");
    const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0), ks = w.size(2);
    TORCH_CHECK(kfk::conv_supported(C, K, ks, static_cast<int>(stride)), "conv: unsupported channels/kernel/stride");
    const int pad = (ks - 1) / 2;
    const int OH = (H + 2 * pad - ks) / stride + 1, OW = (W + 2 * pad - ks) / stride + 1;
    TORCH_CHECK(OH > 0 && OW > 0, "conv: empty output");
    TORCH_CHECK(static_cast<int64_t>(N) * H * W * C < (int64_t(1) << 31) &&
                    static_cast<int64_t>(N) * OH * OW * K < (int64_t(1) << 31),
                "conv: tensor too large for 32-bit offsets");
    c10::DeviceGuard gd(x.device());
    double *sp = nullptr;
    if (stats && stats->defined()) {
        TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->numel() == 2 * K * kfk::kStatSlots &&
                        stats->is_contiguous() && stats->device() == x.device(),
                    "conv: stats must be a contiguous f64 [2*Cout] tensor on x's device");
        sp = stats->data_ptr<double>();
    }
    at::Tensor y;
    bool accum = false;
    if (out && out->defined()) {
        TORCH_CHECK(out->scalar_type() == at::kBFloat16 && out->dim() == 4 && out->size(0) == N && out->size(1) == K &&
                        out->size(2) == OH && out->size(3) == OW &&
                        out->is_contiguous(at::MemoryFormat::ChannelsLast) && out->device() == x.device(),
                    "conv: out must be the [N, Cout, OH, OW] channels_last bf16 output");
        y = *out;
        accum = true;
    } else {
        y = at::empty({N, K, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    }
    kfk::EpiArgs ea;
    ea.stats = sp;
    int epi = accum ? kfk::kEpiAccum : 0;
    const bool bwd = bn_x && bn_x->defined();
    if (bias && bias->defined()) {
        // relu(conv + bias): VGG's conv + bias + ReLU as the conv epilogue
        TORCH_CHECK(!accum && !sp && !bwd && !gate, "conv: bias epilogue excludes out/stats/bn_x/gate");
        TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == K && bias->is_contiguous() &&
                        bias->device() == x.device(),
                    "conv: bias must be a contiguous bf16 [Cout] tensor on x's device");
        ea.bias = reinterpret_cast<const uint16_t *>(bias->data_ptr());
        epi = kfk::kEpiBiasRelu;
    } else if (gate) {
        // gradient of a ReLU output bn_x: y = conv * (bn_x > 0); stats[slot][0] += sum(y)
        TORCH_CHECK(!accum && sp && bwd && !(bn_mask && bn_mask->defined()) && !(bn_fcoef && bn_fcoef->defined()),
                    "conv: gate needs stats and bn_x (the ReLU output), no out/bn_mask/bn_fcoef");
        TORCH_CHECK(bn_x->scalar_type() == at::kBFloat16 && bn_x->sizes() == y.sizes() &&
                        bn_x->is_contiguous(at::MemoryFormat::ChannelsLast) && bn_x->device() == x.device(),
                    "conv: bn_x must be the ReLU output (bf16 channels_last, the output's shape)");
        ea.bx = reinterpret_cast<const uint16_t *>(bn_x->data_ptr());
        epi = kfk::kEpiGate;
    } else if (bwd) {
        TORCH_CHECK(sp, "conv: BN-backward statistics need the stats workspace");
        TORCH_CHECK(bn_x->scalar_type() == at::kBFloat16 && bn_x->sizes() == y.sizes() &&
                        bn_x->is_contiguous(at::MemoryFormat::ChannelsLast) && bn_x->device() == x.device(),
                    "conv: bn_x must be the BN input (bf16 channels_last, the output's shape)");
        ea.bx = reinterpret_cast<const uint16_t *>(bn_x->data_ptr());
        if (bn_mask && bn_mask->defined()) {
            TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == y.numel() / 8 &&
                            bn_mask->device() == x.device(),
                        "conv: bn_mask must hold one byte per 8 output elements");
            ea.bmask = bn_mask->data_ptr<uint8_t>();
            epi |= kfk::kEpiBwdBits;
        } else {
            TORCH_CHECK(bn_fcoef && bn_fcoef->defined() && bn_fcoef->scalar_type() == at::kFloat &&
                            bn_fcoef->numel() >= 2 * K && bn_fcoef->device() == x.device(),
                        "conv: bn_fcoef (forward [scale; shift], f32) or bn_mask required");
            ea.fcoef = bn_fcoef->data_ptr<float>();
            epi |= kfk::kEpiBwdCoef;
        }
    } else if (sp) {
        epi |= kfk::kEpiFwdStats;
    }
    TORCH_CHECK(!(epi & kfk::kEpiFwdStats) || !(epi & kfk::kEpiAccum), "conv: stats + accumulate unsupported");
    if (acc_mask && acc_mask->defined()) {
        // out = out * acc_mask + conv (out: a raw ReLU-output gradient, acc_mask: that ReLU's bits)
        TORCH_CHECK(accum && acc_mask->scalar_type() == at::kByte && acc_mask->numel() == y.numel() / 8 &&
                        acc_mask->device() == x.device() && !(epi & kfk::kEpiBwdCoef),
                    "conv: acc_mask needs out and one byte per 8 output elements");
        ea.amask = acc_mask->data_ptr<uint8_t>();
        epi |= kfk::kEpiAccMask;
    }
    if (acc_even) {
        // out holds a stride-2 1x1 data gradient at its even pixels only (conv_dgrad_s2)
        TORCH_CHECK(accum && stride == 1 && !(epi & (kfk::kEpiAccMask | kfk::kEpiBwdCoef)),
                    "conv: acc_even needs out, stride 1 and no acc_mask / bn_fcoef");
        epi |= kfk::kEpiAccEven;
    }
    ea.fin = fin_ptr(fin, x, K);
    TORCH_CHECK(!ea.fin || (epi & (kfk::kEpiFwdStats | kfk::kEpiBwdCoef | kfk::kEpiBwdBits)),
                "conv: fin needs the statistics epilogue (stats) or the BN-backward sums (stats + bn_x)");
    kfk::launch_conv(reinterpret_cast<const uint16_t *>(x.data_ptr()), reinterpret_cast<const uint16_t *>(w.data_ptr()),
                     reinterpret_cast<uint16_t *>(y.data_ptr()), N, H, W, C, K, ks, static_cast<int>(stride), ea, epi,
                     stream_of(x, 0), static_cast<int>(variant));
    return y;
}

// Linear layer on the MFMA kernel: y[M, N] = x[M, K] @ w[N, K]^T (both row-major bf16).
//   bias:            y += bias (bf16 [N]);
//   out:             y = out += x w^T (accumulate into an existing [M, N] bf16 tensor);
//   gelu_u + stats:  y = (x w^T) * gelu'(gelu_u), stats[slot][0][n] += sum_m y (a bias gradient;
//                    stats: zeroed f64 kStatSlots x 2 x N workspace).
std::vector<at::Tensor> gemm(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> out,
                             c10::optional<at::Tensor> gelu_u,
                             c10::optional<at::Tensor> stats, int64_t variant) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous(),
                "gemm: x must be a contiguous 2-D bf16 GPU tensor");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 2 && w.is_contiguous() && w.size(1) == x.size(1) &&
                    w.device() == x.device(),
                "gemm: w must be a contiguous [N, K] bf16 tensor on x's device");
    const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
    TORCH_CHECK(M < (int64_t(1) << 31) && kfk::gemm_supported(static_cast<int>(M), static_cast<int>(K), static_cast<int>(N)),
                "gemm: unsupported shape (K, N multiples of 64)");
    c10::DeviceGuard gd(x.device());
    kfk::EpiArgs ea;
    int epi = 0;
    at::Tensor y;
    auto check_mn = [&](const at::Tensor &t, const char *what) {
        TORCH_CHECK(t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.size(0) == M && t.size(1) == N &&
                        t.is_contiguous() && t.device() == x.device(),
                    "gemm: ", what, " must be a contiguous [M, N] bf16 tensor on x's device");
    };
    if (out && out->defined()) {
        TORCH_CHECK(!(bias && bias->defined()) && !(gelu_u && gelu_u->defined()),
                    "gemm: out (accumulate) excludes bias / gelu_u");
        check_mn(*out, "out");
        y = *out;
        epi = kfk::kEpiAccum;
    } else {
        y = at::empty({M, N}, x.options());
    }
    if (bias && bias->defined()) {
        TORCH_CHECK(bias->scalar_type() == at::kBFloat16 && bias->numel() == N && bias->is_contiguous() &&
                        bias->device() == x.device(),
                    "gemm: bias must be a contiguous bf16 [N] tensor on x's device");
        ea.bias = reinterpret_cast<const uint16_t *>(bias->data_ptr());
        epi = kfk::kEpiBias;
    }
    if (gelu_u && gelu_u->defined()) {
        TORCH_CHECK(epi == 0, "gemm: gelu_u excludes bias / out");
        check_mn(*gelu_u, "gelu_u");
        TORCH_CHECK(stats && stats->defined() && stats->scalar_type() == at::kDouble && stats->is_contiguous() &&
                        stats->numel() == 2 * N * kfk::kStatSlots && stats->device() == x.device(),
                    "gemm: gelu_u needs the f64 stats workspace (kStatSlots x 2 x N)");
        ea.bx = reinterpret_cast<const uint16_t *>(gelu_u->data_ptr());
        ea.stats = stats->data_ptr<double>();
        epi = kfk::kEpiGeluGrad;
    }
    kfk::launch_gemm(reinterpret_cast<const uint16_t *>(x.data_ptr()), reinterpret_cast<const uint16_t *>(w.data_ptr()),
                     reinterpret_cast<uint16_t *>(y.data_ptr()), static_cast<int>(M), static_cast<int>(K),
                     static_cast<int>(N), ea, epi, stream_of(x, 0), static_cast<int>(variant));
    return {y};
}

// Data gradient of a stride-2 1x1 (pad 0) / 3x3 (pad 1) convolution with an even input:
// dy [N, Cout, OH, OW] -> dx [N, Cin, 2OH, 2OW] (channels_last bf16), wt = conv_flip_weight(w)
// [Cin, Cout, ks, ks].  ks = 3: every pixel written (four parity-phase GEMMs); bn_x + stats
// (+ bn_fcoef or bn_mask) also accumulate the backward sums of the BN whose input is bn_x, as
// conv().  ks = 1: only the even pixels are written -- complete dx with a stride-1 data
// gradient conv(..., out=dx, acc_even=True).
at::Tensor conv_dgrad_s2(at::Tensor dy, at::Tensor wt, int64_t ks, c10::optional<at::Tensor> stats,
                         c10::optional<at::Tensor> bn_x, c10::optional<at::Tensor> bn_fcoef,
                         c10::optional<at::Tensor> bn_mask, int64_t variant, int64_t dh, int64_t dw, int64_t pad,
                         c10::optional<at::Tensor> fin) {
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                    dy.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_dgrad_s2: dy must be a 4-D channels_last bf16 GPU tensor");
    TORCH_CHECK(ks == 1 || ks == 3, "conv_dgrad_s2: ks must be 1 or 3");
    TORCH_CHECK(wt.scalar_type() == at::kBFloat16 && wt.dim() == 4 && wt.size(2) == ks && wt.size(3) == ks &&
                    wt.size(1) == dy.size(1) && wt.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    wt.device() == dy.device(),
                "conv_dgrad_s2: wt must be the flipped [Cin, Cout, ks, ks] channels_last bf16 weight");
    const int N = dy.size(0), K = dy.size(1), OH = dy.size(2), OW = dy.size(3), C = wt.size(0);
    const bool even = dh <= 0;
    if (even) {
        TORCH_CHECK(kfk::conv_supported(K, C, static_cast<int>(ks), 1), "conv_dgrad_s2: unsupported channels");
        dh = 2 * OH, dw = 2 * OW, pad = ks == 3 ? 1 : 0;
    } else {
        // any dx size (ks = 3, pad 0 | 1): channel counts % 8
        TORCH_CHECK(ks == 3 && (pad == 0 || pad == 1) && K % 8 == 0 && C % 8 == 0 && K >= 16 && C >= 16 && dw > 0 &&
                        (dh + 2 * pad - 3) / 2 + 1 == OH && (dw + 2 * pad - 3) / 2 + 1 == OW,
                    "conv_dgrad_s2: dh/dw/pad do not match a 3x3 stride-2 convolution of dy's size (channels % 8)");
    }
    TORCH_CHECK(static_cast<int64_t>(N) * dh * dw * C < (int64_t(1) << 31), "conv_dgrad_s2: tensor too large");
    c10::DeviceGuard gd(dy.device());
    auto dx = at::empty({N, C, dh, dw}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::EpiArgs ea;
    int epi = 0;
    if (bn_x && bn_x->defined()) {
        TORCH_CHECK(ks == 3, "conv_dgrad_s2: BN sums need every pixel (ks = 3)");
        TORCH_CHECK(stats && stats->defined() && stats->scalar_type() == at::kDouble &&
                        stats->numel() == 2 * C * kfk::kStatSlots && stats->is_contiguous() &&
                        stats->device() == dy.device(),
                    "conv_dgrad_s2: BN-backward sums need the f64 stats workspace");
        TORCH_CHECK(bn_x->scalar_type() == at::kBFloat16 && bn_x->sizes() == dx.sizes() &&
                        bn_x->is_contiguous(at::MemoryFormat::ChannelsLast) && bn_x->device() == dy.device(),
                    "conv_dgrad_s2: bn_x must be the BN input (bf16 channels_last, dx's shape)");
        ea.stats = stats->data_ptr<double>();
        ea.bx = reinterpret_cast<const uint16_t *>(bn_x->data_ptr());
        if (bn_mask && bn_mask->defined()) {
            TORCH_CHECK(bn_mask->scalar_type() == at::kByte && bn_mask->numel() == dx.numel() / 8,
                        "conv_dgrad_s2: bn_mask must hold one byte per 8 elements");
            ea.bmask = bn_mask->data_ptr<uint8_t>();
            epi = kfk::kEpiBwdBits;
        } else {
            TORCH_CHECK(bn_fcoef && bn_fcoef->defined() && bn_fcoef->scalar_type() == at::kFloat &&
                            bn_fcoef->numel() >= 2 * C && bn_fcoef->device() == dy.device(),
                        "conv_dgrad_s2: bn_fcoef (forward [scale; shift], f32) or bn_mask required");
            ea.fcoef = bn_fcoef->data_ptr<float>();
            epi = kfk::kEpiBwdCoef;
        }
    }
    ea.fin = fin_ptr(fin, dy, C);
    TORCH_CHECK(!ea.fin || epi != 0, "conv_dgrad_s2: fin needs the BN-backward sums (stats + bn_x)");
    kfk::launch_conv_dgrad_s2(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                              reinterpret_cast<const uint16_t *>(wt.data_ptr()), reinterpret_cast<uint16_t *>(dx.data_ptr()),
                              N, OH, OW, K, C, static_cast<int>(ks), ea, epi, stream_of(dy, 0),
                              static_cast<int>(variant), static_cast<int>(dh), static_cast<int>(dw),
                              static_cast<int>(pad));
    return dx;
}

// Weight gradient of conv(x, w, stride, pad (ks-1)/2): dw [Cout, Cin, ks, ks] channels_last
// (memory [Cout][ks][ks][Cin]).  out: bf16 or f32 destination of that shape/layout (written,
// or added to with accumulate); otherwise a new bf16 tensor.  variant / splits: -1 = planner.
at::Tensor conv_wgrad(at::Tensor dy, at::Tensor x, int64_t ks, int64_t stride, c10::optional<at::Tensor> out,
                      bool accumulate, int64_t variant, int64_t splits, bool atomics) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_wgrad: x must be a 4-D channels_last bf16 GPU tensor");
    const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
    const int pad = static_cast<int>((ks - 1) / 2);
    const int OH = (H + 2 * pad - static_cast<int>(ks)) / static_cast<int>(stride) + 1;
    const int OW = (W + 2 * pad - static_cast<int>(ks)) / static_cast<int>(stride) + 1;
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N &&
                    dy.size(2) == OH && dy.size(3) == OW && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dy.device() == x.device(),
                "conv_wgrad: dy must be the [N, Cout, OH, OW] channels_last bf16 output gradient");
    const int K = dy.size(1);
    TORCH_CHECK(kfk::conv_wgrad_supported(C, K, static_cast<int>(ks), static_cast<int>(stride)),
                "conv_wgrad: unsupported channels/kernel/stride");
    TORCH_CHECK(static_cast<int64_t>(N) * H * W * C < (int64_t(1) << 31) &&
                    static_cast<int64_t>(N) * OH * OW * K < (int64_t(1) << 31),
                "conv_wgrad: tensor too large for 32-bit offsets");
    c10::DeviceGuard gd(x.device());
    at::Tensor dw;
    if (out && out->defined()) {
        TORCH_CHECK((out->scalar_type() == at::kBFloat16 || out->scalar_type() == at::kFloat) && out->dim() == 4 &&
                        out->size(0) == K && out->size(1) == C && out->size(2) == ks && out->size(3) == ks &&
                        out->is_contiguous(at::MemoryFormat::ChannelsLast) && out->device() == x.device(),
                    "conv_wgrad: out must be [Cout, Cin, ks, ks] channels_last bf16/f32 on x's device");
        dw = *out;
    } else {
        TORCH_CHECK(!accumulate, "conv_wgrad: accumulate needs out");
        dw = at::empty({K, C, ks, ks}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    }
    const auto plan = kfk::conv_wgrad_plan(N, H, W, C, K, static_cast<int>(ks), static_cast<int>(stride),
                                           static_cast<int>(variant), static_cast<int>(splits));
    at::Tensor ws;
    if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, x.options().dtype(at::kFloat));
    kfk::launch_conv_wgrad(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                           reinterpret_cast<const uint16_t *>(x.data_ptr()), dw.data_ptr(),
                           plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, N, H, W, C, K, static_cast<int>(ks),
                           static_cast<int>(stride), plan, dw.scalar_type() == at::kFloat, accumulate,
                           stream_of(x, 0), atomics);
    return dw;
}

// Weight gradient of a KH x KW convolution with zero padding (ph, pw): dw [Cout, Cin, KH, KW]
// channels_last bf16 (kfk::conv_wgrad_rect_supported: Inception-v3's windows / channel counts).
at::Tensor conv_wgrad_rect(at::Tensor dy, at::Tensor x, int64_t kh, int64_t kw, int64_t stride, int64_t ph,
                           int64_t pw, int64_t variant) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_wgrad_rect: x must be a 4-D channels_last bf16 GPU tensor");
    const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
    const int OH = (H + 2 * static_cast<int>(ph) - static_cast<int>(kh)) / static_cast<int>(stride) + 1;
    const int OW = (W + 2 * static_cast<int>(pw) - static_cast<int>(kw)) / static_cast<int>(stride) + 1;
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N &&
                    dy.size(2) == OH && dy.size(3) == OW && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dy.device() == x.device(),
                "conv_wgrad_rect: dy must be the [N, Cout, OH, OW] channels_last bf16 output gradient");
    const int K = dy.size(1);
    TORCH_CHECK(kfk::conv_wgrad_rect_supported(C, K, static_cast<int>(kh), static_cast<int>(kw), static_cast<int>(stride)) &&
                    ph >= 0 && pw >= 0 && ph < kh && pw < kw,
                "conv_wgrad_rect: unsupported channels/window/stride/padding");
    TORCH_CHECK(static_cast<int64_t>(N) * H * W * C < (int64_t(1) << 31) &&
                    static_cast<int64_t>(N) * OH * OW * K < (int64_t(1) << 31),
                "conv_wgrad_rect: tensor too large for 32-bit offsets");
    c10::DeviceGuard gd(x.device());
    auto dw = at::empty({K, C, kh, kw}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    const auto plan = kfk::conv_wgrad_rect_plan(N, H, W, C, K, static_cast<int>(kh), static_cast<int>(kw),
                                                static_cast<int>(ph), static_cast<int>(pw), static_cast<int>(stride),
                                                static_cast<int>(variant));
    at::Tensor ws;
    if (plan.ws_floats > 0) ws = at::empty({plan.ws_floats}, x.options().dtype(at::kFloat));
    kfk::launch_conv_wgrad_rect(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                reinterpret_cast<const uint16_t *>(x.data_ptr()), dw.data_ptr(),
                                plan.ws_floats > 0 ? ws.data_ptr<float>() : nullptr, N, H, W, C, K, static_cast<int>(kh),
                                static_cast<int>(kw), static_cast<int>(ph), static_cast<int>(pw),
                                static_cast<int>(stride), plan, false, false, stream_of(x, 0));
    return dw;
}

// fused softmax cross-entropy over bf16 logits [R, V]: (lse [R] f32, per-row loss [R] f32)
// Rows may be padded (x.stride(0) = ld >= V, a multiple of 8, 16-byte aligned base: the vocabulary
// projection's gemm_nt_ld output): the 16-byte-load kernels; those also serve contiguous rows of V % 8 == 0
static int64_t xent_ld(const at::Tensor &x) {
    const int64_t ld = x.stride(0), V = x.size(1);
    const bool al = reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0;
    return (x.stride(1) == 1 && ld >= V && ld % 8 == 0 && al) ? ld : 0;
}

std::vector<at::Tensor> xent_forward(at::Tensor x, at::Tensor labels) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 &&
                    (xent_ld(x) > 0 || (x.is_contiguous() && x.size(1) % 2 == 0)),
                "xent_forward: bf16 [R, V] logits, contiguous with V even or rows padded to a multiple of 8");
    TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                    labels.numel() == x.size(0) && labels.device() == x.device(),
                "xent_forward: int64 labels [R] on the logits' device");
    TORCH_CHECK(x.size(1) < (int64_t(1) << 30) && x.size(0) < (int64_t(1) << 31), "xent_forward: shape too large");
    c10::DeviceGuard gd(x.device());
    auto lse = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
    auto loss = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
    kfk::launch_xent_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()), labels.data_ptr<int64_t>(), x.size(0),
                             static_cast<int>(x.size(1)), lse.data_ptr<float>(), loss.data_ptr<float>(),
                             stream_of(x, 0), xent_ld(x));
    return {lse, loss};
}

// its backward: d logits (bf16 [R, V]) = (softmax - onehot(label)) * scale[0]; padded logits give a
// gradient with the same padded row stride (a [R, V] view of [R, ld], the padding of the last chunk zero)
at::Tensor xent_backward(at::Tensor x, at::Tensor labels, at::Tensor lse, at::Tensor scale) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 &&
                    (xent_ld(x) > 0 || (x.is_contiguous() && x.size(1) % 2 == 0)),
                "xent_backward: bf16 [R, V] logits, contiguous with V even or rows padded to a multiple of 8");
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == x.size(0) &&
                    lse.scalar_type() == at::kFloat && lse.numel() == x.size(0) && scale.scalar_type() == at::kFloat &&
                    scale.numel() >= 1 && labels.device() == x.device() && lse.device() == x.device() &&
                    scale.device() == x.device(),
                "xent_backward: labels int64 [R], lse f32 [R], scale f32 [1] on the logits' device");
    c10::DeviceGuard gd(x.device());
    const int64_t ld = xent_ld(x);
    auto dxp = ld > 0 ? at::empty({x.size(0), ld}, x.options()) : at::empty_like(x);
    kfk::launch_xent_backward(reinterpret_cast<const uint16_t *>(x.data_ptr()), labels.data_ptr<int64_t>(),
                              lse.data_ptr<float>(), scale.data_ptr<float>(), x.size(0), static_cast<int>(x.size(1)),
                              reinterpret_cast<uint16_t *>(dxp.data_ptr()), stream_of(x, 0), ld);
    return ld > 0 && ld != x.size(1) ? dxp.narrow(1, 0, x.size(1)) : dxp;
}

// GELU backward fused with the bias gradient: (du, colsum(du)) for bf16 dy, u [..., O] (O % 8 == 0).
std::vector<at::Tensor> gelu_backward_colsum(at::Tensor dy, at::Tensor u, at::ScalarType dtype) {
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && u.sizes() == dy.sizes() &&
                    u.scalar_type() == at::kBFloat16 && u.is_contiguous() && u.device() == dy.device() &&
                    dy.size(-1) % 8 == 0 && dy.numel() > 0,
                "gelu_backward_colsum: contiguous bf16 dy and u of equal shape, last dim % 8");
    TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16, "gelu_backward_colsum: dtype float32 or bfloat16");
    c10::DeviceGuard gd(dy.device());
    const int O = static_cast<int>(dy.size(-1));
    const int64_t T = dy.numel() / O;
    auto du = at::empty_like(dy);
    auto part = at::empty({static_cast<int64_t>(kfk::gelu_colsum_chunks(T, O)) * O}, dy.options().dtype(at::kFloat));
    auto out = at::empty({O}, dy.options().dtype(dtype));
    kfk::launch_gelu_bwd_colsum(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                reinterpret_cast<const uint16_t *>(u.data_ptr()), reinterpret_cast<uint16_t *>(du.data_ptr()),
                                T, O, part.data_ptr<float>(), dtype == at::kFloat ? out.data_ptr<float>() : nullptr,
                                dtype == at::kBFloat16 ? reinterpret_cast<uint16_t *>(out.data_ptr()) : nullptr,
                                stream_of(dy, 0));
    return {du, out};
}

// Column sums of a contiguous bf16 [T, O] (O % 8 == 0) -> [O] in `dtype` (f32 or bf16).
at::Tensor colsum(at::Tensor x, at::ScalarType dtype) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.is_contiguous() &&
                    x.size(1) % 8 == 0 && x.size(0) > 0,
                "colsum: x must be a contiguous bf16 [T, O] GPU tensor with O % 8 == 0");
    TORCH_CHECK(dtype == at::kFloat || dtype == at::kBFloat16, "colsum: dtype must be float32 or bfloat16");
    c10::DeviceGuard gd(x.device());
    const int64_t T = x.size(0);
    const int O = static_cast<int>(x.size(1));
    auto part = at::empty({static_cast<int64_t>(kfk::colsum_chunks(T, O)) * O}, x.options().dtype(at::kFloat));
    auto out = at::empty({O}, x.options().dtype(dtype));
    kfk::launch_colsum_bf16(reinterpret_cast<const uint16_t *>(x.data_ptr()), T, O, part.data_ptr<float>(),
                            dtype == at::kFloat ? out.data_ptr<float>() : nullptr,
                            dtype == at::kBFloat16 ? reinterpret_cast<uint16_t *>(out.data_ptr()) : nullptr,
                            stream_of(x, 0));
    return out;
}

// Fused self-attention: qkv [B, S, 3*H*64] bf16 contiguous -> (out [B, S, H*64] bf16, lse [B, H, S] f32)
std::vector<at::Tensor> attention_forward(at::Tensor qkv, int64_t heads, double scale, int64_t seed, double p_drop) {
    TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 3 && qkv.is_contiguous() &&
                    qkv.size(2) == 3 * heads * 64 && kfk::attention_supported(qkv.size(1), 64),
                "attention_forward: qkv must be a contiguous bf16 [B, S, 3*H*64] GPU tensor with S in {64, 128}");
    c10::DeviceGuard gd(qkv.device());
    const int B = qkv.size(0), S = qkv.size(1), H = static_cast<int>(heads);
    auto out = at::empty({B, S, H * 64}, qkv.options());
    auto lse = at::empty({B, H, S}, qkv.options().dtype(at::kFloat));
    kfk::launch_attention_forward(reinterpret_cast<const uint16_t *>(qkv.data_ptr()),
                                  reinterpret_cast<uint16_t *>(out.data_ptr()), lse.data_ptr<float>(), B, S, H,
                                  static_cast<float>(scale), static_cast<uint32_t>(seed), static_cast<float>(p_drop),
                                  stream_of(qkv, 0));
    return {out, lse};
}

at::Tensor attention_backward(at::Tensor qkv, at::Tensor out, at::Tensor lse, at::Tensor dout, int64_t heads,
                              double scale, int64_t seed, double p_drop) {
    TORCH_CHECK(qkv.is_cuda() && qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 3 && qkv.is_contiguous() &&
                    qkv.size(2) == 3 * heads * 64 && kfk::attention_supported(qkv.size(1), 64),
                "attention_backward: qkv must be a contiguous bf16 [B, S, 3*H*64] GPU tensor with S in {64, 128}");
    const int B = qkv.size(0), S = qkv.size(1), H = static_cast<int>(heads);
    TORCH_CHECK(out.sizes() == at::IntArrayRef({B, S, H * 64}) && out.is_contiguous() &&
                    out.scalar_type() == at::kBFloat16,
                "attention_backward: out must be the forward's [B, S, H*64] output");
    if (!dout.is_contiguous()) dout = dout.contiguous();
    TORCH_CHECK(dout.sizes() == out.sizes() && dout.scalar_type() == at::kBFloat16, "attention_backward: dout");
    TORCH_CHECK(lse.sizes() == at::IntArrayRef({B, H, S}) && lse.scalar_type() == at::kFloat && lse.is_contiguous(),
                "attention_backward: lse must be the forward's [B, H, S] f32");
    c10::DeviceGuard gd(qkv.device());
    auto dqkv = at::empty_like(qkv);
    kfk::launch_attention_backward(reinterpret_cast<const uint16_t *>(qkv.data_ptr()),
                                   reinterpret_cast<const uint16_t *>(out.data_ptr()), lse.data_ptr<float>(),
                                   reinterpret_cast<const uint16_t *>(dout.data_ptr()),
                                   reinterpret_cast<uint16_t *>(dqkv.data_ptr()), B, S, H, static_cast<float>(scale),
                                   static_cast<uint32_t>(seed), static_cast<float>(p_drop), stream_of(qkv, 0));
    return dqkv;
}

static void check_bias_act(const at::Tensor &y, const char *name) {
    TORCH_CHECK(y.is_cuda() && y.scalar_type() == at::kBFloat16 && y.dim() == 4 &&
                    y.is_contiguous(at::MemoryFormat::ChannelsLast) && kfk::bias_act_supported(y.size(1)),
                name, " must be a 4-D channels_last bf16 GPU tensor with C/8 a power of two <= 256");
}

// y = relu(y + bias) in place (relu=false: y += bias); bias f32 [C]
void bias_act_forward_(at::Tensor y, at::Tensor bias, bool relu) {
    check_bias_act(y, "bias_act_forward_: y");
    TORCH_CHECK(bias.is_cuda() && bias.scalar_type() == at::kFloat && bias.is_contiguous() &&
                    bias.numel() == y.size(1) && bias.device() == y.device(),
                "bias_act_forward_: bias must be a contiguous f32 [C] tensor on y's device");
    c10::DeviceGuard gd(y.device());
    const int64_t rows = y.numel() / y.size(1);
    kfk::launch_bias_act_forward(reinterpret_cast<uint16_t *>(y.data_ptr()), bias.data_ptr<float>(), rows,
                                 static_cast<int>(y.size(1)), relu, stream_of(y, 0));
}

// (dz, dbias): dz = dy * (y > 0) (relu; dz is dy itself without relu), dbias = sum dz over N, H, W (f32)
std::vector<at::Tensor> bias_act_backward(at::Tensor dy, at::Tensor y, bool relu) {
    check_bias_act(y, "bias_act_backward: y");
    check_bias_act(dy, "bias_act_backward: dy");
    TORCH_CHECK(dy.sizes() == y.sizes() && dy.device() == y.device(), "bias_act_backward: dy must match y");
    c10::DeviceGuard gd(y.device());
    const int C = static_cast<int>(y.size(1));
    const int64_t rows = y.numel() / C;
    at::Tensor dz = relu ? at::empty_like(dy, dy.options().memory_format(at::MemoryFormat::ChannelsLast)) : dy;
    at::Tensor db = at::empty({C}, y.options().dtype(at::kFloat));
    at::Tensor part = at::empty({std::max(1, kfk::bias_act_backward_blocks(rows, C)), C}, y.options().dtype(at::kFloat));
    kfk::launch_bias_act_backward(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                  reinterpret_cast<const uint16_t *>(y.data_ptr()),
                                  reinterpret_cast<uint16_t *>(dz.data_ptr()), db.data_ptr<float>(),
                                  part.data_ptr<float>(), rows, C, relu, stream_of(y, 0));
    return {dz, db};
}

static void check_pool_in(const at::Tensor &x, const char *name) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0 && x.size(2) % 2 == 0 &&
                    x.size(3) % 2 == 0,
                name, " must be a 4-D channels_last bf16 GPU tensor with C % 8 == 0 and even H, W");
}

at::Tensor maxpool2x2_forward(at::Tensor x) {
    check_pool_in(x, "maxpool2x2_forward: x");
    c10::DeviceGuard gd(x.device());
    auto y = at::empty({x.size(0), x.size(1), x.size(2) / 2, x.size(3) / 2},
                       x.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_maxpool2x2_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()),
                                   reinterpret_cast<uint16_t *>(y.data_ptr()), x.size(0), static_cast<int>(x.size(2)),
                                   static_cast<int>(x.size(3)), static_cast<int>(x.size(1)), stream_of(x, 0));
    return y;
}

at::Tensor maxpool2x2_backward(at::Tensor x, at::Tensor dy, c10::optional<at::Tensor> gate_stats) {
    check_pool_in(x, "maxpool2x2_backward: x");
    double *gs = nullptr;
    if (gate_stats && gate_stats->defined()) {
        TORCH_CHECK(gate_stats->is_cuda() && gate_stats->scalar_type() == at::kDouble && gate_stats->is_contiguous() &&
                        gate_stats->numel() == 2 * x.size(1) * kfk::kStatSlots && gate_stats->device() == x.device(),
                    "maxpool2x2_backward: gate_stats must be a contiguous f64 [slots * 2 * C] tensor");
        gs = gate_stats->data_ptr<double>();
    }
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == x.size(0) &&
                    dy.size(1) == x.size(1) && dy.size(2) == x.size(2) / 2 && dy.size(3) == x.size(3) / 2 &&
                    dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.device() == x.device(),
                "maxpool2x2_backward: dy must be the channels_last bf16 pooled-output gradient");
    c10::DeviceGuard gd(x.device());
    auto dx = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_maxpool2x2_backward(reinterpret_cast<const uint16_t *>(x.data_ptr()),
                                    reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                    reinterpret_cast<uint16_t *>(dx.data_ptr()), x.size(0), static_cast<int>(x.size(2)),
                                    static_cast<int>(x.size(3)), static_cast<int>(x.size(1)), stream_of(x, 0), gs);
    return dx;
}

static void check_pool3_in(const at::Tensor &x, const char *name) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast) && x.size(1) % 8 == 0 && x.size(2) >= 3 &&
                    x.size(3) >= 3,
                name, " must be a 4-D channels_last bf16 GPU tensor with C % 8 == 0 and H, W >= 3");
}

std::tuple<at::Tensor, at::Tensor> maxpool3s2_forward(at::Tensor x, int64_t pad) {
    check_pool3_in(x, "maxpool3x3s2_forward: x");
    TORCH_CHECK(pad == 0 || pad == 1, "maxpool3x3s2: pad 0 or 1");
    c10::DeviceGuard gd(x.device());
    const int H = x.size(2), W = x.size(3);
    const int OH = kfk::maxpool3s2_out(H, pad), OW = kfk::maxpool3s2_out(W, pad);
    auto y = at::empty({x.size(0), x.size(1), OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    auto arg = at::empty({x.size(0), OH, OW, x.size(1)}, x.options().dtype(at::kByte));
    kfk::launch_maxpool3s2_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()),
                                   reinterpret_cast<uint16_t *>(y.data_ptr()), arg.data_ptr<uint8_t>(), x.size(0), H, W,
                                   static_cast<int>(x.size(1)), static_cast<int>(pad), stream_of(x, 0));
    return {y, arg};
}

at::Tensor maxpool3s2_backward(at::Tensor dy, at::Tensor arg, int64_t H, int64_t W, int64_t pad) {
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 &&
                    dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.size(1) % 8 == 0,
                "maxpool3x3s2_backward: dy must be channels_last bf16 with C % 8 == 0");
    TORCH_CHECK(dy.size(2) == kfk::maxpool3s2_out(H, pad) && dy.size(3) == kfk::maxpool3s2_out(W, pad) &&
                    arg.scalar_type() == at::kByte && arg.numel() == dy.numel() && arg.device() == dy.device(),
                "maxpool3x3s2_backward: shape mismatch");
    c10::DeviceGuard gd(dy.device());
    auto dx = at::empty({dy.size(0), dy.size(1), H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_maxpool3s2_backward(reinterpret_cast<const uint16_t *>(dy.data_ptr()), arg.data_ptr<uint8_t>(),
                                    reinterpret_cast<uint16_t *>(dx.data_ptr()), dy.size(0), static_cast<int>(H),
                                    static_cast<int>(W), static_cast<int>(dy.size(1)), static_cast<int>(pad),
                                    stream_of(dy, 0));
    return dx;
}

// Global average pool of a channels_last bf16 [N, C, H, W] -> [N, C] bf16 (and its backward).
at::Tensor global_avgpool_forward(at::Tensor x) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) % 8 == 0 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "global_avgpool: x must be a channels_last bf16 [N, C, H, W] GPU tensor with C % 8 == 0");
    c10::DeviceGuard gd(x.device());
    auto y = at::empty({x.size(0), x.size(1)}, x.options());
    kfk::launch_global_avgpool_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()),
                                       reinterpret_cast<uint16_t *>(y.data_ptr()), x.size(0),
                                       static_cast<int>(x.size(2) * x.size(3)), static_cast<int>(x.size(1)),
                                       stream_of(x, 0));
    return y;
}

at::Tensor global_avgpool_backward(at::Tensor dy, int64_t H, int64_t W) {
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 && dy.size(1) % 8 == 0 &&
                    H > 0 && W > 0,
                "global_avgpool_backward: dy must be a bf16 [N, C] GPU tensor with C % 8 == 0");
    dy = dy.contiguous();
    c10::DeviceGuard gd(dy.device());
    auto dx = at::empty({dy.size(0), dy.size(1), H, W}, dy.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_global_avgpool_backward(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                        reinterpret_cast<uint16_t *>(dx.data_ptr()), dy.size(0), static_cast<int>(H * W),
                                        static_cast<int>(dy.size(1)), stream_of(dy, 0));
    return dx;
}

at::Tensor avgpool3s1(at::Tensor x) {
    check_pool3_in(x, "avgpool3x3s1: x");
    c10::DeviceGuard gd(x.device());
    auto y = at::empty_like(x, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_avgpool3s1(reinterpret_cast<const uint16_t *>(x.data_ptr()), reinterpret_cast<uint16_t *>(y.data_ptr()),
                           x.size(0), static_cast<int>(x.size(2)), static_cast<int>(x.size(3)),
                           static_cast<int>(x.size(1)), stream_of(x, 0));
    return y;
}

// y, s, mean, rstd = layernorm(x [+ r]) over the last dim (bf16 rows, f32 affine)
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> layernorm_forward(at::Tensor x, c10::optional<at::Tensor> r,
                                                                             at::Tensor gamma, at::Tensor beta,
                                                                             double eps, double p, int64_t seed) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.is_contiguous(),
                "layernorm: x must be a contiguous bf16 GPU tensor");
    const int D = static_cast<int>(x.size(-1));
    TORCH_CHECK(kfk::layernorm_supported(D), "layernorm: unsupported row length ", D);
    TORCH_CHECK(gamma.scalar_type() == at::kFloat && beta.scalar_type() == at::kFloat && gamma.numel() == D &&
                    beta.numel() == D && gamma.is_contiguous() && beta.is_contiguous(),
                "layernorm: f32 gamma/beta of length D");
    const uint16_t *rp = nullptr;
    if (r && r->defined()) {
        TORCH_CHECK(r->scalar_type() == at::kBFloat16 && r->is_contiguous() && r->sizes() == x.sizes(),
                    "layernorm: residual must match x");
        rp = reinterpret_cast<const uint16_t *>(r->data_ptr());
    }
    c10::DeviceGuard gd(x.device());
    const int64_t rows = x.numel() / D;
    auto y = at::empty_like(x);
    auto sv = rp ? at::empty_like(x) : x;
    auto mean = at::empty({rows}, x.options().dtype(at::kFloat));
    auto rstd = at::empty({rows}, x.options().dtype(at::kFloat));
    kfk::launch_layernorm_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()), rp, gamma.data_ptr<float>(),
                                  beta.data_ptr<float>(), reinterpret_cast<uint16_t *>(y.data_ptr()),
                                  rp ? reinterpret_cast<uint16_t *>(sv.data_ptr()) : nullptr, mean.data_ptr<float>(),
                                  rstd.data_ptr<float>(), rows, D, static_cast<float>(eps), stream_of(x, 0),
                                  static_cast<float>(p), static_cast<uint32_t>(seed));
    return {y, sv, mean, rstd};
}

// Returns (ds, dgamma, dbeta, dr): dr (p > 0 only, else undefined) is the gradient of the dropped
// residual input.
// rbias_dtype (float32 / bfloat16, optional): also return the column sums of the residual input's
// gradient (dr, or ds without dropout) in that dtype -- the bias gradient of the linear layer that
// produced the residual input.
std::vector<at::Tensor> layernorm_backward(at::Tensor dy, at::Tensor s, at::Tensor gamma, at::Tensor mean,
                                           at::Tensor rstd, double p, int64_t seed,
                                           c10::optional<at::ScalarType> rbias_dtype) {
    TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.is_contiguous() && s.sizes() == dy.sizes() &&
                    s.scalar_type() == at::kBFloat16 && s.is_contiguous(),
                "layernorm_backward: contiguous bf16 dy and s of equal shape");
    const int D = static_cast<int>(dy.size(-1));
    TORCH_CHECK(kfk::layernorm_supported(D) && gamma.numel() == D, "layernorm_backward: bad D");
    c10::DeviceGuard gd(dy.device());
    const int64_t rows = dy.numel() / D;
    TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_backward: stats size");
    auto ds = at::empty_like(dy);
    const bool rb = rbias_dtype.has_value();
    TORCH_CHECK(!rb || *rbias_dtype == at::kFloat || *rbias_dtype == at::kBFloat16,
                "layernorm_backward: rbias_dtype must be float32 or bfloat16");
    auto partial = at::empty({kfk::layernorm_bwd_blocks(rows), rb ? 3 : 2, D}, dy.options().dtype(at::kFloat));
    at::Tensor rbias;
    if (rb) rbias = at::empty({D}, dy.options().dtype(*rbias_dtype));
    auto dgamma = at::empty({D}, dy.options().dtype(at::kFloat));
    auto dbeta = at::empty({D}, dy.options().dtype(at::kFloat));
    at::Tensor dr;
    if (p > 0) dr = at::empty_like(dy);
    kfk::launch_layernorm_backward(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                                   reinterpret_cast<const uint16_t *>(s.data_ptr()), gamma.data_ptr<float>(),
                                   mean.data_ptr<float>(), rstd.data_ptr<float>(),
                                   reinterpret_cast<uint16_t *>(ds.data_ptr()), partial.data_ptr<float>(),
                                   dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), rows, D, stream_of(dy, 0),
                                   dr.defined() ? reinterpret_cast<uint16_t *>(dr.data_ptr()) : nullptr,
                                   static_cast<float>(p), static_cast<uint32_t>(seed),
                                   rb && *rbias_dtype == at::kFloat ? rbias.data_ptr<float>() : nullptr,
                                   rb && *rbias_dtype == at::kBFloat16 ? reinterpret_cast<uint16_t *>(rbias.data_ptr())
                                                                        : nullptr);
    if (rb) return {ds, dgamma, dbeta, dr, rbias};
    return {ds, dgamma, dbeta, dr};
}

// [Cout, Cin, KS, KS] channels_last -> flipped/transposed [Cin, Cout, KS, KS] channels_last
at::Tensor conv_flip_weight(at::Tensor w) {
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_flip_weight: [Cout, Cin, KH, KW] channels_last bf16 required");
    const int K = w.size(0), C = w.size(1), kh = w.size(2), kw = w.size(3);
    c10::DeviceGuard gd(w.device());
    auto wt = at::empty({C, K, kh, kw}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_conv_flip_weight_taps(reinterpret_cast<const uint16_t *>(w.data_ptr()),
                                      reinterpret_cast<uint16_t *>(wt.data_ptr()), K, C, kh * kw, stream_of(w, 0));
    return wt;
}

// KH x KW convolution with zero padding (ph, pw) on the MFMA kernel (Inception-v3 shapes,
// kfk::conv_rect_supported); stats: optional f64 [kStatSlots*2*Cout] BN-statistics workspace.
at::Tensor conv_rect(at::Tensor x, at::Tensor w, int64_t stride, int64_t ph, int64_t pw,
                     c10::optional<at::Tensor> stats, c10::optional<at::Tensor> out, c10::optional<at::Tensor> bn_x,
                     c10::optional<at::Tensor> bn_fcoef) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
                    x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv_rect: x must be a 4-D channels_last bf16 GPU tensor");
    TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(1) == x.size(1) &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.device() == x.device(),
                "conv_rect: w must be [Cout, Cin, KH, KW] channels_last bf16 on x's device");
    const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
    const int kh = w.size(2), kw = w.size(3);
    TORCH_CHECK(kfk::conv_rect_supported(C, K, kh, kw, static_cast<int>(stride)) && ph >= 0 && pw >= 0 &&
                    ph < kh && pw < kw,
                "conv_rect: unsupported channels/window/stride/padding");
    const int OH = (H + 2 * static_cast<int>(ph) - kh) / static_cast<int>(stride) + 1;
    const int OW = (W + 2 * static_cast<int>(pw) - kw) / static_cast<int>(stride) + 1;
    TORCH_CHECK(OH > 0 && OW > 0, "conv_rect: empty output");
    TORCH_CHECK(static_cast<int64_t>(N) * H * W * C < (int64_t(1) << 31) &&
                    static_cast<int64_t>(N) * OH * OW * K < (int64_t(1) << 31),
                "conv_rect: tensor too large for 32-bit offsets");
    c10::DeviceGuard gd(x.device());
    kfk::EpiArgs ea;
    int epi = 0;
    if (stats && stats->defined()) {
        TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->numel() == 2 * K * kfk::kStatSlots &&
                        stats->is_contiguous() && stats->device() == x.device(),
                    "conv_rect: stats must be the f64 [kStatSlots*2*Cout] workspace");
        ea.stats = stats->data_ptr<double>();
        epi = kfk::kEpiFwdStats;
    }
    const bool bwd = bn_x && bn_x->defined();
    if (bwd) {
        // the output is the gradient of a BN+ReLU output whose input is bn_x (forward coefficients
        // bn_fcoef): stats receives that BN's backward sums (sum dz, sum dz*x) instead
        TORCH_CHECK(ea.stats && bn_x->scalar_type() == at::kBFloat16 && bn_x->size(0) == N && bn_x->size(1) == K &&
                        bn_x->size(2) == OH && bn_x->size(3) == OW &&
                        bn_x->is_contiguous(at::MemoryFormat::ChannelsLast) && bn_x->device() == x.device() &&
                        bn_fcoef && bn_fcoef->defined() && bn_fcoef->scalar_type() == at::kFloat &&
                        bn_fcoef->numel() >= 2 * K && bn_fcoef->device() == x.device(),
                    "conv_rect: bn_x (the BN input, output-shaped) needs stats and bn_fcoef (f32 [scale; shift])");
        ea.bx = reinterpret_cast<const uint16_t *>(bn_x->data_ptr());
        ea.fcoef = bn_fcoef->data_ptr<float>();
        epi = kfk::kEpiBwdCoef;
    }
    at::Tensor y;
    if (out && out->defined()) {
        // y = out + conv(x, w) in place (e.g. sibling convolutions' data gradients into one dx)
        TORCH_CHECK((epi == 0 || bwd) && out->scalar_type() == at::kBFloat16 && out->dim() == 4 && out->size(0) == N &&
                        out->size(1) == K && out->size(2) == OH && out->size(3) == OW &&
                        out->is_contiguous(at::MemoryFormat::ChannelsLast) && out->device() == x.device(),
                    "conv_rect: out must be the [N, Cout, OH, OW] channels_last bf16 output (no stats)");
        y = *out;
        epi |= kfk::kEpiAccum;
    } else {
        y = at::empty({N, K, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    }
    kfk::launch_conv_rect(reinterpret_cast<const uint16_t *>(x.data_ptr()), reinterpret_cast<const uint16_t *>(w.data_ptr()),
                          reinterpret_cast<uint16_t *>(y.data_ptr()), N, H, W, C, K, kh, kw, static_cast<int>(ph),
                          static_cast<int>(pw), static_cast<int>(stride), ea, epi, stream_of(x, 0));
    return y;
}

// dsts[i] = conv_flip_weight(srcs[i]) for a list of bf16 conv weights, in as few launches as
// possible (FlipTable::kMax per launch).  dsts must be preallocated [Cin, Cout, KS, KS] channels_last.
void conv_flip_weights(std::vector<at::Tensor> srcs, std::vector<at::Tensor> dsts) {
    TORCH_CHECK(srcs.size() == dsts.size(), "conv_flip_weights: length mismatch");
    if (srcs.empty()) return;
    c10::DeviceGuard gd(srcs[0].device());
    auto s = stream_of(srcs[0], 0);
    kfk::FlipTable tab;
    tab.start[0] = 0;
    for (size_t i = 0; i < srcs.size(); ++i) {
        const auto &w = srcs[i];
        const auto &d = dsts[i];
        TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 &&
                        w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.device() == srcs[0].device(),
                    "conv_flip_weights: [Cout, Cin, KS, KS] channels_last bf16 sources on one device");
        TORCH_CHECK(d.scalar_type() == at::kBFloat16 && d.dim() == 4 && d.size(0) == w.size(1) &&
                        d.size(1) == w.size(0) && d.size(2) == w.size(2) && d.size(3) == w.size(3) &&
                        d.is_contiguous(at::MemoryFormat::ChannelsLast) && d.device() == w.device(),
                    "conv_flip_weights: destination must be [Cin, Cout, KS, KS] channels_last bf16");
        const int k = tab.n;
        tab.src[k] = reinterpret_cast<const uint16_t *>(w.data_ptr());
        tab.dst[k] = reinterpret_cast<uint16_t *>(d.data_ptr());
        tab.cout[k] = w.size(0);
        tab.cin[k] = w.size(1);
        tab.taps[k] = w.size(2) * w.size(3);
        tab.start[k + 1] = tab.start[k] + w.numel();
        tab.n = k + 1;
        if (tab.n == kfk::FlipTable::kMax) {
            kfk::launch_conv_flip_multi(tab, s);
            tab.n = 0;
        }
    }
    kfk::launch_conv_flip_multi(tab, s);
}

// [Cout, Cin, 3, 3] channels_last -> flipped/transposed [Cin, Cout, 3, 3] channels_last
at::Tensor conv3x3_flip_weight(at::Tensor w) {
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                    w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "conv3x3_flip_weight: [Cout, Cin, 3, 3] channels_last bf16 required");
    const int K = w.size(0), C = w.size(1);
    c10::DeviceGuard gd(w.device());
    auto wt = at::empty({C, K, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_conv3x3_flip_weight(reinterpret_cast<const uint16_t *>(w.data_ptr()),
                                    reinterpret_cast<uint16_t *>(wt.data_ptr()), K, C, stream_of(w, 0));
    return wt;
}

// ---- fused BN(+add)+ReLU ----------------------------------------------------------

kfk::BNShape bn_shape(const at::Tensor &x) {
    TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16, "bn: bf16 GPU tensor required");
    TORCH_CHECK(x.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast), "bn: 4-D channels_last tensor required");
    const int C = static_cast<int>(x.size(1));
    TORCH_CHECK(kfk::bn_supported_channels(C), "bn: unsupported channel count ", C);
    return kfk::BNShape{x.numel() / C, C};
}

struct BNCommon {
    float *rm = nullptr, *rv = nullptr;
    int64_t *nbt = nullptr;
};

BNCommon bn_common(int C, const at::Tensor &weight, const at::Tensor &bias,
                   const c10::optional<at::Tensor> &running_mean, const c10::optional<at::Tensor> &running_var,
                   const c10::optional<at::Tensor> &num_batches, bool training) {
    TORCH_CHECK(weight.scalar_type() == at::kFloat && bias.scalar_type() == at::kFloat && weight.numel() == C &&
                    bias.numel() == C,
                "bn: f32 weight/bias of size C required");
    BNCommon b;
    if (running_mean && running_mean->defined()) {
        TORCH_CHECK(running_var && running_var->defined(), "bn: running_var missing");
        b.rm = running_mean->data_ptr<float>();
        b.rv = running_var->data_ptr<float>();
    }
    TORCH_CHECK(training || b.rm, "bn: eval mode needs running stats");
    if (training && num_batches && num_batches->defined()) {
        TORCH_CHECK(num_batches->scalar_type() == at::kLong && num_batches->numel() == 1 && num_batches->is_cuda(),
                    "bn: num_batches_tracked must be a 1-element int64 GPU tensor");
        b.nbt = num_batches->data_ptr<int64_t>();
    }
    return b;
}

// Batched sums-finalize of several training-mode BNs (each with its producing conv's f64 slotted
// sums): ONE launch; returns [mean, invstd, coef] per BN for bn_forward(..., pre=...).
std::vector<std::vector<at::Tensor>> bn_finalize_multi(std::vector<at::Tensor> xs, std::vector<at::Tensor> sums,
                                                       std::vector<at::Tensor> weights, std::vector<at::Tensor> biases,
                                                       std::vector<c10::optional<at::Tensor>> running_means,
                                                       std::vector<c10::optional<at::Tensor>> running_vars,
                                                       std::vector<c10::optional<at::Tensor>> num_batches,
                                                       std::vector<double> momentum, std::vector<double> eps) {
    const size_t n = xs.size();
    TORCH_CHECK(n >= 1 && n <= static_cast<size_t>(kfk::kBnFinMax) && sums.size() == n && weights.size() == n &&
                    biases.size() == n && running_means.size() == n && running_vars.size() == n &&
                    num_batches.size() == n && momentum.size() == n && eps.size() == n,
                "bn_finalize_multi: 1..8 BNs, every list of the same length");
    kfk::BnFinBatch b{};
    b.n = static_cast<int>(n);
    std::vector<std::vector<at::Tensor>> out;
    for (size_t i = 0; i < n; ++i) {
        auto sh = bn_shape(xs[i]);
        const int C = sh.channels;
        TORCH_CHECK(xs[i].device() == xs[0].device(), "bn_finalize_multi: one device");
        auto c = bn_common(C, weights[i], biases[i], running_means[i], running_vars[i], num_batches[i], true);
        const at::Tensor &s = sums[i];
        TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kDouble && s.numel() == 2 * C * kfk::kStatSlots &&
                        s.is_contiguous() && s.device() == xs[i].device(),
                    "bn_finalize_multi: sums must be the conv epilogue's f64 slotted workspace");
        auto fopt = xs[i].options().dtype(at::kFloat);
        at::Tensor mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt), coef = at::empty({2 * C}, fopt);
        kfk::BnFinDesc &d = b.d[i];
        d.sums = s.data_ptr<double>();
        d.gamma = weights[i].data_ptr<float>(), d.beta = biases[i].data_ptr<float>();
        d.mean = mean.data_ptr<float>(), d.invstd = invstd.data_ptr<float>(), d.coef = coef.data_ptr<float>();
        d.run_mean = c.rm, d.run_var = c.rv, d.nbt = c.nbt;
        d.rows = sh.rows, d.C = C;
        d.momentum = static_cast<float>(momentum[i]), d.eps = static_cast<float>(eps[i]);
        out.push_back({mean, invstd, coef});
    }
    c10::DeviceGuard gd(xs[0].device());
    kfk::launch_bn_sums_finalize_multi(b, stream_of(xs[0], 0));
    return out;
}

// Returns (y, mean, invstd, coef, mask-or-undefined).
std::vector<at::Tensor> bn_forward(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor weight, at::Tensor bias,
                                   c10::optional<at::Tensor> running_mean, c10::optional<at::Tensor> running_var,
                                   double momentum, double eps, bool training, bool relu,
                                   c10::optional<at::Tensor> num_batches, c10::optional<at::Tensor> sums,
                                   c10::optional<at::Tensor> res_coef, bool apply, c10::optional<at::Tensor> out,
                                   c10::optional<std::vector<at::Tensor>> pre) {
    auto sh = bn_shape(x);
    const int C = sh.channels;
    auto b = bn_common(C, weight, bias, running_mean, running_var, num_batches, training);
    const uint16_t *rp = nullptr;
    if (res && res->defined()) {
        TORCH_CHECK(res->sizes() == x.sizes() && res->scalar_type() == at::kBFloat16 &&
                        res->is_contiguous(at::MemoryFormat::ChannelsLast),
                    "bn: residual must match x (bf16, channels_last)");
        rp = reinterpret_cast<const uint16_t *>(res->data_ptr());
    }
    const float *rc = nullptr;
    if (res_coef && res_coef->defined()) {
        TORCH_CHECK(rp && res_coef->scalar_type() == at::kFloat && res_coef->numel() == 2 * C && res_coef->is_contiguous(),
                    "bn: res_coef must be the residual BN's f32 [scale(C); shift(C)] coefficients");
        rc = res_coef->data_ptr<float>();
    }
    c10::DeviceGuard gd(x.device());
    auto fopt = x.options().dtype(at::kFloat);
    at::Tensor y;
    int64_t y_ld = 0;
    if (out && out->defined()) {
        // a channel slice [N, C, H, W] of a wider channels_last bf16 tensor (a concatenation)
        TORCH_CHECK(apply && !rp && relu && out->scalar_type() == at::kBFloat16 && out->dim() == 4 &&
                        out->size(0) == x.size(0) && out->size(1) == C && out->size(2) == x.size(2) &&
                        out->size(3) == x.size(3) && out->stride(1) == 1 && out->stride(3) >= C &&
                        out->stride(3) % 8 == 0 && out->stride(2) == out->size(3) * out->stride(3) &&
                        out->stride(0) == out->size(2) * out->stride(2) &&
                        reinterpret_cast<uintptr_t>(out->data_ptr()) % 16 == 0 && out->device() == x.device(),
                    "bn: out must be a 16-byte aligned channel slice of a channels_last bf16 tensor (BN+ReLU, no residual)");
        y = *out;
        y_ld = out->stride(3);
    } else if (apply) {
        y = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    }
    at::Tensor mean, invstd, coef;
    const bool prefin = pre.has_value();
    if (prefin) {
        // (mean, invstd, coef) already written from `sums` by the producing conv's in-launch finalize
        TORCH_CHECK(pre->size() == 3 && training && sums && sums->defined(), "bn: pre = (mean, invstd, coef) with sums");
        mean = (*pre)[0], invstd = (*pre)[1], coef = (*pre)[2];
        TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() == C && invstd.numel() == C &&
                        coef.numel() == 2 * C && coef.scalar_type() == at::kFloat,
                    "bn: pre tensors must be f32 mean[C], invstd[C], coef[2C]");
    } else {
        mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt), coef = at::empty({2 * C}, fopt);
    }
    at::Tensor mask;
    if (apply && rp && relu) mask = at::empty({sh.rows * (C / 8)}, x.options().dtype(at::kByte));
    double *sp = nullptr;
    if (training && sums && sums->defined()) {
        TORCH_CHECK(sums->is_cuda() && sums->scalar_type() == at::kDouble && sums->numel() == 2 * C * kfk::kStatSlots &&
                        sums->is_contiguous() && sums->device() == x.device(),
                    "bn: sums must be the conv epilogue's f64 [2*C] workspace");
        sp = sums->data_ptr<double>();
    }
    at::Tensor partial;
    if (training && !sp) partial = at::empty({2 * static_cast<int64_t>(kfk::bn_num_chunks(sh)) * C}, fopt);
    kfk::launch_bn_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()), rp, weight.data_ptr<float>(),
                           bias.data_ptr<float>(), apply ? reinterpret_cast<uint16_t *>(y.data_ptr()) : nullptr,
                           mask.defined() ? mask.data_ptr<uint8_t>() : nullptr, sh, relu, training, b.rm, b.rv,
                           static_cast<float>(momentum), static_cast<float>(eps),
                           partial.defined() ? partial.data_ptr<float>() : nullptr, mean.data_ptr<float>(),
                           invstd.data_ptr<float>(), coef.data_ptr<float>(), b.nbt, stream_of(x, 0), sp, rc, apply, y_ld,
                           prefin);
    return {y, mean, invstd, coef, mask};
}

// Returns (dx, dres or undefined, dweight, dbias).
std::vector<at::Tensor> bn_backward(at::Tensor dy, at::Tensor x, at::Tensor mean, at::Tensor invstd,
                                    at::Tensor weight, at::Tensor fcoef, c10::optional<at::Tensor> mask, bool relu,
                                    bool training, bool want_dres, c10::optional<at::Tensor> sums,
                                    c10::optional<at::Tensor> dres_x, c10::optional<at::Tensor> dres_sums,
                                    c10::optional<std::vector<at::Tensor>> pre) {
    auto sh = bn_shape(x);
    const int C = sh.channels;
    // dy may be a channel slice of a wider channels-last tensor (a concatenation's gradient):
    // read in place with its row stride instead of a contiguous copy
    int64_t dy_ld = 0;
    if (!dy.is_contiguous(at::MemoryFormat::ChannelsLast)) {
        const int64_t ld = dy.dim() == 4 ? dy.stride(3) : 0;
        const bool slice = dy.dim() == 4 && dy.stride(1) == 1 && ld >= C && ld % 8 == 0 &&
                           dy.stride(2) == dy.size(3) * ld && dy.stride(0) == dy.size(2) * dy.size(3) * ld &&
                           reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0;
        if (slice) dy_ld = ld;
        else dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
    }
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.sizes() == x.sizes(), "bn_backward: dy must match x");
    TORCH_CHECK(fcoef.scalar_type() == at::kFloat && fcoef.numel() == 2 * C, "bn_backward: fcoef must be 2C f32");
    const uint8_t *mp = nullptr;
    if (mask && mask->defined()) {
        TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() == sh.rows * (C / 8), "bn_backward: bad mask");
        mp = mask->data_ptr<uint8_t>();
    }
    c10::DeviceGuard gd(x.device());
    auto fopt = x.options().dtype(at::kFloat);
    auto dx = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    at::Tensor dres;
    if (want_dres) dres = at::empty_like(x, at::MemoryFormat::ChannelsLast);
    at::Tensor dw, db, coef;
    const bool prefin = pre.has_value();
    if (prefin) {
        // (dgamma, dbeta, coef) already written from `sums` by the dgrad conv's in-launch finalize
        TORCH_CHECK(pre->size() == 3 && sums && sums->defined(), "bn_backward: pre = (dgamma, dbeta, coef) with sums");
        dw = (*pre)[0], db = (*pre)[1], coef = (*pre)[2];
        TORCH_CHECK(dw.scalar_type() == at::kFloat && dw.numel() == C && db.numel() == C && coef.numel() == 3 * C,
                    "bn_backward: pre tensors must be f32 dgamma[C], dbeta[C], coef[3C]");
    } else {
        dw = at::empty({C}, fopt), db = at::empty({C}, fopt), coef = at::empty({3 * C}, fopt);
    }
    double *sp = nullptr;
    if (sums && sums->defined()) {
        TORCH_CHECK(sums->is_cuda() && sums->scalar_type() == at::kDouble && sums->numel() == 2 * C * kfk::kStatSlots &&
                        sums->is_contiguous() && sums->device() == x.device(),
                    "bn_backward: sums must be the conv epilogue's f64 workspace");
        sp = sums->data_ptr<double>();
    }
    at::Tensor partial;
    if (!sp) partial = at::empty({2 * static_cast<int64_t>(kfk::bn_num_chunks(sh)) * C}, fopt);
    const uint16_t *dsx = nullptr;
    double *dsp = nullptr;
    if (dres_x && dres_x->defined()) {
        TORCH_CHECK(want_dres && dres_sums && dres_sums->defined() && dres_x->sizes() == x.sizes() &&
                        dres_x->scalar_type() == at::kBFloat16 && dres_x->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                        dres_sums->scalar_type() == at::kDouble && dres_sums->numel() == 2 * C * kfk::kStatSlots,
                    "bn_backward: dres_x (second BN's input) needs want_dres and its f64 sums workspace");
        dsx = reinterpret_cast<const uint16_t *>(dres_x->data_ptr());
        dsp = dres_sums->data_ptr<double>();
    }
    kfk::launch_bn_backward(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                            reinterpret_cast<const uint16_t *>(x.data_ptr()), fcoef.data_ptr<float>(), mp,
                            mean.data_ptr<float>(), invstd.data_ptr<float>(), weight.data_ptr<float>(), sh, relu,
                            training, partial.defined() ? partial.data_ptr<float>() : nullptr, dw.data_ptr<float>(),
                            db.data_ptr<float>(), coef.data_ptr<float>(), reinterpret_cast<uint16_t *>(dx.data_ptr()),
                            want_dres ? reinterpret_cast<uint16_t *>(dres.data_ptr()) : nullptr, stream_of(x, 0), sp,
                            dsx, dsp, dy_ld, prefin);
    return {dx, dres, dw, db};
}

// Backward of several training BN+ReLUs (no residual, no sums) whose output gradients may be channel
// slices of one concatenation's gradient: every reduce pass, ONE batched finalize, every apply pass.
// Returns [dx, dgamma, dbeta] per BN.
std::vector<std::vector<at::Tensor>> bn_backward_multi(std::vector<at::Tensor> dys, std::vector<at::Tensor> xs,
                                                       std::vector<at::Tensor> means, std::vector<at::Tensor> invstds,
                                                       std::vector<at::Tensor> weights, std::vector<at::Tensor> fcoefs) {
    const size_t n = xs.size();
    TORCH_CHECK(n >= 1 && n <= static_cast<size_t>(kfk::kBnFinMax) && dys.size() == n && means.size() == n &&
                    invstds.size() == n && weights.size() == n && fcoefs.size() == n,
                "bn_backward_multi: 1..8 BNs, every list of the same length");
    c10::DeviceGuard gd(xs[0].device());
    kfk::BnBwdFinBatch fb{};
    fb.n = static_cast<int>(n);
    struct Piece {
        at::Tensor dy, dx, dw, db, coef, partial;
        int64_t ld;
        kfk::BNShape sh;
    };
    std::vector<Piece> ps(n);
    for (size_t i = 0; i < n; ++i) {
        Piece &p = ps[i];
        p.sh = bn_shape(xs[i]);
        const int C = p.sh.channels;
        at::Tensor dy = dys[i];
        p.ld = 0;
        if (!dy.is_contiguous(at::MemoryFormat::ChannelsLast)) {
            const int64_t ld = dy.dim() == 4 ? dy.stride(3) : 0;
            const bool slice = dy.dim() == 4 && dy.stride(1) == 1 && ld >= C && ld % 8 == 0 &&
                               dy.stride(2) == dy.size(3) * ld && dy.stride(0) == dy.size(2) * dy.size(3) * ld &&
                               reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0;
            if (slice) p.ld = ld;
            else dy = dy.contiguous(at::MemoryFormat::ChannelsLast);
        }
        TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.sizes() == xs[i].sizes() && dy.device() == xs[0].device(),
                    "bn_backward_multi: dy must match x");
        TORCH_CHECK(fcoefs[i].scalar_type() == at::kFloat && fcoefs[i].numel() == 2 * C &&
                        means[i].numel() == C && invstds[i].numel() == C && weights[i].numel() == C &&
                        weights[i].scalar_type() == at::kFloat,
                    "bn_backward_multi: f32 fcoef [2C], mean / invstd / weight [C]");
        p.dy = dy;
        auto fopt = xs[i].options().dtype(at::kFloat);
        p.dx = at::empty_like(xs[i], at::MemoryFormat::ChannelsLast);
        p.dw = at::empty({C}, fopt), p.db = at::empty({C}, fopt), p.coef = at::empty({3 * C}, fopt);
        p.partial = at::empty({2 * static_cast<int64_t>(kfk::bn_num_chunks(p.sh)) * C}, fopt);
        kfk::BnBwdFinDesc &d = fb.d[i];
        d.partial = p.partial.data_ptr<float>();
        d.nchunks = kfk::bn_num_chunks(p.sh), d.C = C, d.rows = p.sh.rows;
        d.gamma = weights[i].data_ptr<float>(), d.mean = means[i].data_ptr<float>(), d.invstd = invstds[i].data_ptr<float>();
        d.dgamma = p.dw.data_ptr<float>(), d.dbeta = p.db.data_ptr<float>(), d.coef = p.coef.data_ptr<float>();
    }
    const hipStream_t st = stream_of(xs[0], 0);
    for (int phase : {1, 2}) {
        if (phase == 2) kfk::launch_bn_bwd_finalize_multi(fb, st);
        for (size_t i = 0; i < n; ++i) {
            Piece &p = ps[i];
            kfk::launch_bn_backward(reinterpret_cast<const uint16_t *>(p.dy.data_ptr()),
                                    reinterpret_cast<const uint16_t *>(xs[i].data_ptr()), fcoefs[i].data_ptr<float>(),
                                    nullptr, means[i].data_ptr<float>(), invstds[i].data_ptr<float>(),
                                    weights[i].data_ptr<float>(), p.sh, true, true, p.partial.data_ptr<float>(),
                                    p.dw.data_ptr<float>(), p.db.data_ptr<float>(), p.coef.data_ptr<float>(),
                                    reinterpret_cast<uint16_t *>(p.dx.data_ptr()), nullptr, st, nullptr, nullptr,
                                    nullptr, p.ld, false, phase);
        }
    }
    std::vector<std::vector<at::Tensor>> out;
    for (auto &p : ps) out.push_back({p.dx, p.dw, p.db});
    return out;
}

// Stem BN+ReLU+MaxPool(3,2,1).  Returns (y_pool, mean, invstd, coef, argmax bytes).
std::vector<at::Tensor> bn_pool_forward(at::Tensor x, at::Tensor weight, at::Tensor bias,
                                        c10::optional<at::Tensor> running_mean,
                                        c10::optional<at::Tensor> running_var, double momentum, double eps,
                                        bool training, c10::optional<at::Tensor> num_batches,
                                        c10::optional<at::Tensor> sums) {
    auto sh = bn_shape(x);
    const int C = sh.channels;
    const int H = static_cast<int>(x.size(2)), W = static_cast<int>(x.size(3));
    TORCH_CHECK(kfk::bn_pool_supported(sh, H, W), "bn_pool: unsupported shape");
    double *sp = nullptr;
    if (training && sums && sums->defined()) {
        TORCH_CHECK(sums->is_cuda() && sums->scalar_type() == at::kDouble && sums->numel() == 2 * C * kfk::kStatSlots &&
                        sums->is_contiguous() && sums->device() == x.device(),
                    "bn_pool: sums must be the conv epilogue's f64 [slots*2*C] workspace");
        sp = sums->data_ptr<double>();
    }
    auto b = bn_common(C, weight, bias, running_mean, running_var, num_batches, training);
    c10::DeviceGuard gd(x.device());
    auto fopt = x.options().dtype(at::kFloat);
    const int OH = kfk::pool_out(H), OW = kfk::pool_out(W);
    auto yp = at::empty({x.size(0), C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
    auto arg = at::empty({x.size(0) * OH * OW * C}, x.options().dtype(at::kByte));
    auto mean = at::empty({C}, fopt), invstd = at::empty({C}, fopt), coef = at::empty({2 * C}, fopt);
    at::Tensor partial, xarg;
    if (training) {
        partial = at::empty({2 * static_cast<int64_t>(kfk::bn_num_chunks(sh)) * C}, fopt);
        xarg = at::empty_like(yp, at::MemoryFormat::ChannelsLast);
    }
    kfk::launch_bn_pool_forward(reinterpret_cast<const uint16_t *>(x.data_ptr()), weight.data_ptr<float>(),
                                bias.data_ptr<float>(), reinterpret_cast<uint16_t *>(yp.data_ptr()),
                                arg.data_ptr<uint8_t>(), sh, H, W, training, b.rm, b.rv, static_cast<float>(momentum),
                                static_cast<float>(eps), training ? partial.data_ptr<float>() : nullptr,
                                mean.data_ptr<float>(), invstd.data_ptr<float>(), coef.data_ptr<float>(), b.nbt,
                                stream_of(x, 0), sp,
                                xarg.defined() ? reinterpret_cast<uint16_t *>(xarg.data_ptr()) : nullptr);
    return {yp, mean, invstd, coef, arg, xarg};
}

// ---- ResNet stem (stem.hip) ----
// x [N, 3, H, W] channels_last bf16 -> [N, 4, H, W] channels_last (4th channel zero)
at::Tensor stem_pad4(at::Tensor x) {
    TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) && x.dim() == 4 &&
                    x.size(1) == 3 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_pad4: x must be [N, 3, H, W] channels_last bf16/f32 on the GPU");
    c10::DeviceGuard gd(x.device());
    auto x4 = at::empty({x.size(0), 4, x.size(2), x.size(3)},
                        x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
    const int64_t npix = x.size(0) * x.size(2) * x.size(3);
    if (x.scalar_type() == at::kFloat)
        kfk::launch_stem_pad4_f32(x.data_ptr<float>(), reinterpret_cast<uint16_t *>(x4.data_ptr()), npix,
                                  stream_of(x, 0));
    else
        kfk::launch_stem_pad4(reinterpret_cast<const uint16_t *>(x.data_ptr()),
                              reinterpret_cast<uint16_t *>(x4.data_ptr()), npix, stream_of(x, 0));
    return x4;
}

// w [64, 3, 7, 7] channels_last bf16 -> packed [64, 224] (kh, kw<8, c<4), zero padded
at::Tensor stem_pack_weight(at::Tensor w) {
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 &&
                    w.size(2) == 7 && w.size(3) == 7 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_pack_weight: w must be [64, 3, 7, 7] channels_last bf16");
    c10::DeviceGuard gd(w.device());
    auto wp = at::empty({64, 224}, w.options());
    kfk::launch_stem_pack_weight(reinterpret_cast<const uint16_t *>(w.data_ptr()),
                                 reinterpret_cast<uint16_t *>(wp.data_ptr()), stream_of(w, 0));
    return wp;
}

// y = conv7x7s2p3(x, w) [N, 64, OH, OW] channels_last bf16; stats: BN sums workspace (f64 slots x 2 x 64)
at::Tensor stem_forward(at::Tensor x4, at::Tensor wp, c10::optional<at::Tensor> stats) {
    TORCH_CHECK(x4.is_cuda() && x4.scalar_type() == at::kBFloat16 && x4.dim() == 4 && x4.size(1) == 4 &&
                    x4.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_forward: x4 must be [N, 4, H, W] channels_last bf16");
    TORCH_CHECK(wp.scalar_type() == at::kBFloat16 && wp.numel() == 64 * 224 && wp.is_contiguous() &&
                    wp.device() == x4.device(),
                "stem_forward: wp must be the packed [64, 224] weights");
    const int N = x4.size(0), H = x4.size(2), W = x4.size(3);
    TORCH_CHECK(H >= 4 && W >= 4, "stem_forward: input too small");
    double *sp = nullptr;
    if (stats && stats->defined()) {
        TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->numel() == 2 * 64 * kfk::kStatSlots &&
                        stats->is_contiguous() && stats->device() == x4.device(),
                    "stem_forward: stats must be a contiguous f64 [slots*2*64] tensor");
        sp = stats->data_ptr<double>();
    }
    c10::DeviceGuard gd(x4.device());
    auto y = at::empty({N, 64, kfk::stem_out(H), kfk::stem_out(W)},
                       x4.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_stem_forward(reinterpret_cast<const uint16_t *>(x4.data_ptr()),
                             reinterpret_cast<const uint16_t *>(wp.data_ptr()), reinterpret_cast<uint16_t *>(y.data_ptr()),
                             sp, N, H, W, stream_of(x4, 0));
    return y;
}

// dw [64, 3, 7, 7] channels_last bf16 from dy [N, 64, OH, OW] and x4
at::Tensor stem_wgrad_bnp(at::Tensor y, at::Tensor x4, at::Tensor dyp, at::Tensor arg, at::Tensor fcoef,
                          at::Tensor bcoef, int64_t splits) {
    TORCH_CHECK(x4.is_cuda() && x4.scalar_type() == at::kBFloat16 && x4.dim() == 4 && x4.size(1) == 4 &&
                    x4.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_wgrad_bnp: x4 must be [N, 4, H, W] channels_last bf16");
    const int N = x4.size(0), H = x4.size(2), W = x4.size(3);
    const int OH = kfk::stem_out(H), OW = kfk::stem_out(W);
    TORCH_CHECK(y.scalar_type() == at::kBFloat16 && y.dim() == 4 && y.size(0) == N && y.size(1) == 64 && y.size(2) == OH &&
                    y.size(3) == OW && y.is_contiguous(at::MemoryFormat::ChannelsLast) && y.device() == x4.device(),
                "stem_wgrad_bnp: y must be the [N, 64, OH, OW] channels_last bf16 conv output");
    TORCH_CHECK(dyp.scalar_type() == at::kBFloat16 && dyp.dim() == 4 && dyp.size(0) == N && dyp.size(1) == 64 &&
                    dyp.size(2) == kfk::pool_out(OH) && dyp.size(3) == kfk::pool_out(OW) &&
                    dyp.is_contiguous(at::MemoryFormat::ChannelsLast) && dyp.device() == x4.device(),
                "stem_wgrad_bnp: dyp must be the pooled [N, 64, PH, PW] channels_last bf16 gradient");
    TORCH_CHECK(arg.scalar_type() == at::kByte && arg.numel() == dyp.numel() && arg.device() == x4.device(),
                "stem_wgrad_bnp: arg must hold the window argmax byte of every pooled element");
    TORCH_CHECK(fcoef.scalar_type() == at::kFloat && fcoef.numel() == 128 && bcoef.scalar_type() == at::kFloat &&
                    bcoef.numel() == 192 && fcoef.is_contiguous() && bcoef.is_contiguous(),
                "stem_wgrad_bnp: fcoef [2 x 64] / bcoef [3 x 64] f32");
    TORCH_CHECK(kfk::stem_wgrad_bnp_supported(N, H, W), "stem_wgrad_bnp: image too wide for the row kernel");
    c10::DeviceGuard gd(x4.device());
    const int sp = splits > 0 ? static_cast<int>(splits) : kfk::stem_wgrad_splits(N, H, W);
    auto part = at::empty({kfk::stem_wgrad_workspace(N, H, W, sp)}, x4.options().dtype(at::kFloat));
    auto dw = at::empty({64, 3, 7, 7}, x4.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_stem_wgrad_bnp(reinterpret_cast<const uint16_t *>(y.data_ptr()),
                               reinterpret_cast<const uint16_t *>(x4.data_ptr()),
                               reinterpret_cast<uint16_t *>(dw.data_ptr()), part.data_ptr<float>(), N, H, W, sp,
                               reinterpret_cast<const uint16_t *>(dyp.data_ptr()), arg.data_ptr<uint8_t>(),
                               fcoef.data_ptr<float>(), bcoef.data_ptr<float>(), stream_of(x4, 0));
    return dw;
}

at::Tensor stem_wgrad(at::Tensor dy, at::Tensor x4, int64_t splits) {
    TORCH_CHECK(x4.is_cuda() && x4.scalar_type() == at::kBFloat16 && x4.dim() == 4 && x4.size(1) == 4 &&
                    x4.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem_wgrad: x4 must be [N, 4, H, W] channels_last bf16");
    const int N = x4.size(0), H = x4.size(2), W = x4.size(3);
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == 64 &&
                    dy.size(2) == kfk::stem_out(H) && dy.size(3) == kfk::stem_out(W) &&
                    dy.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.device() == x4.device(),
                "stem_wgrad: dy must be the [N, 64, OH, OW] channels_last bf16 output gradient");
    c10::DeviceGuard gd(x4.device());
    const int sp = splits > 0 ? static_cast<int>(splits) : kfk::stem_wgrad_splits(N, H, W);
    auto part = at::empty({kfk::stem_wgrad_workspace(N, H, W, sp)}, x4.options().dtype(at::kFloat));
    auto dw = at::empty({64, 3, 7, 7}, x4.options().memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_stem_wgrad(reinterpret_cast<const uint16_t *>(dy.data_ptr()),
                           reinterpret_cast<const uint16_t *>(x4.data_ptr()), reinterpret_cast<uint16_t *>(dw.data_ptr()),
                           part.data_ptr<float>(), N, H, W, sp, stream_of(x4, 0));
    return dw;
}

// Small image stem (stem3.hip, Inception's Conv2d_1a): w [32, 3, KH, KW] channels_last bf16 -> packed [32, 64]
at::Tensor stem3_pack_weight(at::Tensor w) {
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kBFloat16 && w.dim() == 4 && w.size(0) == 32 && w.size(1) == 3 &&
                    w.size(2) <= 4 && w.size(3) <= 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast),
                "stem3_pack_weight: w must be [32, 3, KH<=4, KW<=4] channels_last bf16");
    c10::DeviceGuard gd(w.device());
    auto wp = at::empty({32, 64}, w.options().memory_format(at::MemoryFormat::Contiguous));
    kfk::launch_stem3_pack_weight(reinterpret_cast<const uint16_t *>(w.data_ptr()),
                                  reinterpret_cast<uint16_t *>(wp.data_ptr()), w.size(2), w.size(3), stream_of(w, 0));
    return wp;
}

static void check_img3(const at::Tensor &x, const char *name) {
    TORCH_CHECK(x.is_cuda() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) && x.dim() == 4 &&
                    x.size(1) == 3 && x.is_contiguous(at::MemoryFormat::ChannelsLast),
                name, ": x must be the [N, 3, H, W] channels_last f32 / bf16 image");
}

at::Tensor stem3_forward(at::Tensor x, at::Tensor wp, int64_t kh, int64_t kw, int64_t stride, int64_t ph, int64_t pw,
                         c10::optional<at::Tensor> stats) {
    check_img3(x, "stem3_forward");
    TORCH_CHECK(wp.scalar_type() == at::kBFloat16 && wp.numel() == 32 * 64 && wp.is_contiguous() &&
                    wp.device() == x.device(),
                "stem3_forward: wp must be the packed [32, 64] weights");
    const int N = x.size(0), H = x.size(2), W = x.size(3);
    double *sp = nullptr;
    if (stats && stats->defined()) {
        TORCH_CHECK(stats->is_cuda() && stats->scalar_type() == at::kDouble && stats->numel() == 2 * 32 * kfk::kStatSlots &&
                        stats->is_contiguous() && stats->device() == x.device(),
                    "stem3_forward: stats must be a contiguous f64 [slots*2*32] tensor");
        sp = stats->data_ptr<double>();
    }
    c10::DeviceGuard gd(x.device());
    const int OH = kfk::stem3_out(H, kh, stride, ph), OW = kfk::stem3_out(W, kw, stride, pw);
    TORCH_CHECK(OH > 0 && OW > 0, "stem3_forward: empty output");
    auto y = at::empty({N, 32, OH, OW}, x.options().dtype(at::kBFloat16).memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_stem3_forward(x.data_ptr(), x.scalar_type() == at::kFloat, reinterpret_cast<const uint16_t *>(wp.data_ptr()),
                              reinterpret_cast<uint16_t *>(y.data_ptr()), sp, N, H, W, kh, kw, stride, ph, pw,
                              stream_of(x, 0));
    return y;
}

at::Tensor stem3_wgrad(at::Tensor dy, at::Tensor x, int64_t kh, int64_t kw, int64_t stride, int64_t ph, int64_t pw,
                       bool out_f32) {
    check_img3(x, "stem3_wgrad");
    const int N = x.size(0), H = x.size(2), W = x.size(3);
    const int OH = kfk::stem3_out(H, kh, stride, ph), OW = kfk::stem3_out(W, kw, stride, pw);
    TORCH_CHECK(dy.scalar_type() == at::kBFloat16 && dy.dim() == 4 && dy.size(0) == N && dy.size(1) == 32 &&
                    dy.size(2) == OH && dy.size(3) == OW && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
                    dy.device() == x.device(),
                "stem3_wgrad: dy must be the [N, 32, OH, OW] channels_last bf16 output gradient");
    c10::DeviceGuard gd(x.device());
    auto part = at::empty({kfk::stem3_wgrad_workspace(N, H, W, kh, kw, stride, ph, pw)}, x.options().dtype(at::kFloat));
    auto dw = at::empty({32, 3, kh, kw}, x.options().dtype(out_f32 ? at::kFloat : at::kBFloat16)
                                            .memory_format(at::MemoryFormat::ChannelsLast));
    kfk::launch_stem3_wgrad(reinterpret_cast<const uint16_t *>(dy.data_ptr()), x.data_ptr(), x.scalar_type() == at::kFloat,
                            dw.data_ptr(), out_f32, part.data_ptr<float>(), N, H, W, kh, kw, stride, ph, pw,
                            stream_of(x, 0));
    return dw;
}

// Returns (dx, dweight, dbias).
std::vector<at::Tensor> bn_pool_backward(at::Tensor dyp, at::Tensor arg, at::Tensor x, at::Tensor mean,
                                         at::Tensor invstd, at::Tensor weight, at::Tensor fcoef, bool training,
                                         c10::optional<at::Tensor> xarg, bool apply) {
    auto sh = bn_shape(x);
    const int C = sh.channels;
    const int H = static_cast<int>(x.size(2)), W = static_cast<int>(x.size(3));
    const int OH = kfk::pool_out(H), OW = kfk::pool_out(W);
    if (!dyp.is_contiguous(at::MemoryFormat::ChannelsLast)) dyp = dyp.contiguous(at::MemoryFormat::ChannelsLast);
    TORCH_CHECK(dyp.scalar_type() == at::kBFloat16 && dyp.size(0) == x.size(0) && dyp.size(1) == C &&
                    dyp.size(2) == OH && dyp.size(3) == OW,
                "bn_pool_backward: dy shape mismatch");
    TORCH_CHECK(arg.scalar_type() == at::kByte && arg.numel() == dyp.numel(), "bn_pool_backward: bad argmax");
    TORCH_CHECK(fcoef.scalar_type() == at::kFloat && fcoef.numel() == 2 * C, "bn_pool_backward: fcoef must be 2C");
    c10::DeviceGuard gd(x.device());
    auto fopt = x.options().dtype(at::kFloat);
    // apply = false: statistics + finalize only -- dx is not formed (an empty tensor), the backward
    // coefficients [k1; k2; k3] are returned for the caller's own pass (stem_wgrad_bnp)
    auto dx = apply ? at::empty_like(x, at::MemoryFormat::ChannelsLast) : at::empty({0}, x.options());
    auto dw = at::empty({C}, fopt), db = at::empty({C}, fopt), coef = at::empty({3 * C}, fopt);
    auto partial = at::empty({2 * static_cast<int64_t>(kfk::bn_num_chunks(sh)) * C}, fopt);
    const bool pooled = training && xarg && xarg->defined();
    at::Tensor sums;
    if (pooled) {
        TORCH_CHECK(xarg->sizes() == dyp.sizes() && xarg->scalar_type() == at::kBFloat16 &&
                        xarg->is_contiguous(at::MemoryFormat::ChannelsLast),
                    "bn_pool_backward: xarg must be the forward's pooled pre-BN values");
        sums = at::zeros({2 * C * kfk::kStatSlots}, x.options().dtype(at::kDouble));
    }
    kfk::launch_bn_pool_backward(reinterpret_cast<const uint16_t *>(dyp.data_ptr()), arg.data_ptr<uint8_t>(),
                                 reinterpret_cast<const uint16_t *>(x.data_ptr()), fcoef.data_ptr<float>(),
                                 mean.data_ptr<float>(), invstd.data_ptr<float>(), weight.data_ptr<float>(), sh, H, W,
                                 training, partial.data_ptr<float>(), dw.data_ptr<float>(), db.data_ptr<float>(),
                                 coef.data_ptr<float>(), apply ? reinterpret_cast<uint16_t *>(dx.data_ptr()) : nullptr,
                                 stream_of(x, 0),
                                 pooled ? reinterpret_cast<const uint16_t *>(xarg->data_ptr()) : nullptr,
                                 pooled ? sums.data_ptr<double>() : nullptr, apply);
    return {dx, dw, db, coef};
}

// ---- device model store: HIP IPC export / import ------------------------------------
// A dedicated hipMalloc allocation (not a caching-allocator sub-block) so the
// IPC handle maps exactly this buffer; peers open it and pull over xGMI with
// no participation of the owner (one-sided, like the reference's P2P store).

void hcheck(hipError_t e, const char *what) {
    TORCH_CHECK(e == hipSuccess, "hip ", what, ": ", hipGetErrorString(e));
}

at::Tensor ipc_alloc(int64_t numel, int64_t device) {
    c10::DeviceGuard gd(at::Device(at::kCUDA, device));
    void *p = nullptr;
    hcheck(hipMalloc(&p, std::max<int64_t>(numel, 1) * 4), "Malloc");
    hcheck(hipMemset(p, 0, std::max<int64_t>(numel, 1) * 4), "Memset");
    auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device);
    return torch::from_blob(p, {numel}, [](void *q) { (void)hipFree(q); }, opts);
}

py::bytes ipc_handle(at::Tensor t) {
    hipIpcMemHandle_t h;
    hcheck(hipIpcGetMemHandle(&h, t.data_ptr()), "IpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char *>(&h), sizeof(h));
}

at::Tensor ipc_open(py::bytes handle, int64_t numel, int64_t device) {
    std::string hs = handle;
    TORCH_CHECK(hs.size() == sizeof(hipIpcMemHandle_t), "ipc_open: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, hs.data(), sizeof(h));
    c10::DeviceGuard gd(at::Device(at::kCUDA, device));
    void *p = nullptr;
    hcheck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "IpcOpenMemHandle");
    auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device);
    return torch::from_blob(p, {numel}, [](void *q) { (void)hipIpcCloseMemHandle(q); }, opts);
}

// grad[V, D] (f32, accumulated into) += scatter of dy[T, D] (f32 / bf16) by ids[T] (int64)
void embedding_backward(at::Tensor grad, at::Tensor ids, at::Tensor dy, int64_t ch) {
    check_gpu(grad, "grad");
    check_gpu(ids, "ids");
    check_gpu(dy, "dy");
    TORCH_CHECK(grad.scalar_type() == at::kFloat && grad.dim() == 2, "embedding_backward: grad f32 [V, D]");
    TORCH_CHECK(ids.scalar_type() == at::kLong, "embedding_backward: ids int64");
    const int64_t V = grad.size(0), D = grad.size(1), T = ids.numel();
    TORCH_CHECK(dy.numel() == T * D && (dy.scalar_type() == at::kFloat || dy.scalar_type() == at::kBFloat16),
                "embedding_backward: dy f32/bf16 [T, D]");
    TORCH_CHECK(D % 4 == 0, "embedding_backward: D % 4");
    c10::DeviceGuard gd(grad.device());
    kfk::launch_embedding_backward(grad.data_ptr<float>(), ids.data_ptr<int64_t>(), dy.data_ptr(),
                                   dy.scalar_type() == at::kBFloat16, T, static_cast<int>(D), V, stream_of(grad, 0),
                                   static_cast<int>(ch));
}

// gemm.hip: out[M, N] = a[M, K] . b[N, K]^T (+ bias) (+ out when accumulate), bf16.
// C[M, ldc] (only columns < N written, the chunk holding column N - 1 whole) = a . b^T (+ bias), for a
// ragged N (BERT's 30,522-entry vocabulary): rows of C padded to ldc (a multiple of 8) stay 16-byte aligned
at::Tensor gemm_nt_ld(at::Tensor a, at::Tensor b, c10::optional<at::Tensor> bias, int64_t ldc, int64_t bn) {
    TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
                "gemm_nt_ld: bf16 GPU tensors");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
                "gemm_nt_ld: a [M, K], b [N, K] contiguous");
    const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
    if (ldc <= 0) ldc = (N + 7) / 8 * 8;
    TORCH_CHECK(kfk::gemm_nt_ld_supported(M, N, K, ldc), "gemm_nt_ld: unsupported shape M=", M, " N=", N, " K=", K,
                " ldc=", ldc);
    int epi = 0;
    const uint16_t *bp = nullptr;
    if (bias && bias->defined()) {
        TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N &&
                        bias->is_contiguous(),
                    "gemm_nt_ld: bias bf16 [N]");
        bp = reinterpret_cast<const uint16_t *>(bias->data_ptr());
        epi |= kfk::kGemmBias;
    }
    auto c = at::empty({M, ldc}, a.options());
    c10::DeviceGuard gd(a.device());
    kfk::launch_gemm_nt_ld(reinterpret_cast<const uint16_t *>(a.data_ptr()),
                           reinterpret_cast<const uint16_t *>(b.data_ptr()), reinterpret_cast<uint16_t *>(c.data_ptr()),
                           bp, static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), static_cast<int>(ldc), epi,
                           bn > 0 ? static_cast<int>(bn) : 256, c10::hip::getCurrentHIPStream().stream());
    return c;
}

at::Tensor gemm_nt(at::Tensor a, at::Tensor b, c10::optional<at::Tensor> bias, c10::optional<at::Tensor> out,
                   bool accumulate, int64_t bn) {
    TORCH_CHECK(a.is_cuda() && b.is_cuda() && a.scalar_type() == at::kBFloat16 && b.scalar_type() == at::kBFloat16,
                "gemm_nt: bf16 GPU tensors");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
                "gemm_nt: a [M, K], b [N, K] contiguous");
    const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
    TORCH_CHECK(kfk::gemm_nt_supported(M, N, K), "gemm_nt: unsupported shape M=", M, " N=", N, " K=", K);
    int epi = 0;
    const uint16_t *bp = nullptr;
    if (bias && bias->defined()) {
        TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->numel() == N &&
                        bias->is_contiguous(),
                    "gemm_nt: bias bf16 [N]");
        bp = reinterpret_cast<const uint16_t *>(bias->data_ptr());
        epi |= kfk::kGemmBias;
    }
    at::Tensor c;
    if (out && out->defined()) {
        c = *out;
        TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kBFloat16 && c.is_contiguous() && c.numel() == M * N,
                    "gemm_nt: out bf16 [M, N] contiguous");
        if (accumulate) epi |= kfk::kGemmAccum;
    } else {
        TORCH_CHECK(!accumulate, "gemm_nt: accumulate needs out");
        c = at::empty({M, N}, a.options());
    }
    c10::DeviceGuard gd(a.device());
    kfk::launch_gemm_nt(reinterpret_cast<const uint16_t *>(a.data_ptr()), reinterpret_cast<const uint16_t *>(b.data_ptr()),
                        reinterpret_cast<uint16_t *>(c.data_ptr()), bp, static_cast<int>(M), static_cast<int>(N),
                        static_cast<int>(K), epi, static_cast<int>(bn), c10::hip::getCurrentHIPStream().stream());
    return c;
}

// gemm.hip GELU-gradient epilogue: (du [M, N] bf16, db [N]) with du = bf16(bf16(a . b^T) * gelu'(u)) and
// db the column sums of du (f32 or bf16 as bias_dtype) -- the data gradient through GELU of the layer
// whose output u (its pre-activation) fed gelu, and that layer's bias gradient, in one GEMM + fold.
std::vector<at::Tensor> gemm_nt_gelu_grad(at::Tensor a, at::Tensor b, at::Tensor u, c10::optional<at::ScalarType> bias_dtype) {
    TORCH_CHECK(a.is_cuda() && b.is_cuda() && u.is_cuda() && a.scalar_type() == at::kBFloat16 &&
                    b.scalar_type() == at::kBFloat16 && u.scalar_type() == at::kBFloat16,
                "gemm_nt_gelu_grad: bf16 GPU tensors");
    TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && a.is_contiguous() && b.is_contiguous() && a.size(1) == b.size(1),
                "gemm_nt_gelu_grad: a [M, K], b [N, K] contiguous");
    const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
    TORCH_CHECK(u.is_contiguous() && u.numel() == M * N, "gemm_nt_gelu_grad: u [M, N] contiguous");
    TORCH_CHECK(kfk::gemm_nt_supported(M, N, K) && N % 256 == 0, "gemm_nt_gelu_grad: unsupported shape M=", M, " N=", N,
                " K=", K);
    c10::DeviceGuard gd(a.device());
    auto c = at::empty({M, N}, a.options());
    const int rows = kfk::gemm_nt_gelu_grad_rows(static_cast<int>(M));
    auto part = at::empty({rows, N}, a.options().dtype(at::kFloat));
    const bool f32 = !bias_dtype || *bias_dtype == at::kFloat;
    auto db = at::empty({N}, a.options().dtype(f32 ? at::kFloat : at::kBFloat16));
    const auto s = c10::hip::getCurrentHIPStream().stream();
    kfk::launch_gemm_nt_gelu_grad(reinterpret_cast<const uint16_t *>(a.data_ptr()),
                                  reinterpret_cast<const uint16_t *>(b.data_ptr()), reinterpret_cast<uint16_t *>(c.data_ptr()),
                                  reinterpret_cast<const uint16_t *>(u.data_ptr()), part.data_ptr<float>(),
                                  static_cast<int>(M), static_cast<int>(N), static_cast<int>(K), s);
    kfk::launch_colsum_fold(part.data_ptr<float>(), rows, static_cast<int>(N), f32 ? db.data_ptr<float>() : nullptr,
                            f32 ? nullptr : reinterpret_cast<uint16_t *>(db.data_ptr()), s);
    return {c, db};
}

// Collective-interference emulator (comm_emu.hip): stands in for one all-reduce of `bucket`.
void comm_emulate(at::Tensor bucket, at::Tensor scratch, int64_t traffic_bytes, int64_t ctas, double seconds,
                  int64_t stream) {
    check_gpu(bucket, "bucket");
    check_gpu(scratch, "scratch");
    const int64_t bytes = bucket.numel() * bucket.element_size();
    TORCH_CHECK(scratch.numel() * scratch.element_size() >= bytes, "comm_emulate: scratch smaller than the bucket");
    TORCH_CHECK(bytes >= 16 && reinterpret_cast<uintptr_t>(bucket.data_ptr()) % 16 == 0 &&
                    reinterpret_cast<uintptr_t>(scratch.data_ptr()) % 16 == 0,
                "comm_emulate: 16-byte aligned buffers of >= 16 bytes");
    c10::DeviceGuard gd(bucket.device());
    kfk::launch_comm_emulate(bucket.data_ptr(), scratch.data_ptr(), bytes, traffic_bytes, static_cast<int>(ctas),
                             seconds, stream_of(bucket, stream));
}

// Peer access / link of `device` to every visible device (the bench pre-flight's P2P
// matrix): (peer, can_access_peer, link type, hop count); link type per
// hipExtGetLinkTypeAndHopCount (HSA_AMD_LINK_INFO_TYPE_*: 4 = xGMI, 2 = PCIe).
std::vector<std::tuple<int, int, int, int>> device_links(int64_t device) {
    int n = 0;
    hcheck(hipGetDeviceCount(&n), "GetDeviceCount");
    std::vector<std::tuple<int, int, int, int>> out;
    for (int p = 0; p < n; ++p) {
        if (p == device) continue;
        int can = 0;
        uint32_t lt = 0, hops = 0;
        if (hipDeviceCanAccessPeer(&can, static_cast<int>(device), p) != hipSuccess) can = -1;
        if (hipExtGetLinkTypeAndHopCount(static_cast<int>(device), p, &lt, &hops) != hipSuccess) lt = hops = 0;
        out.emplace_back(p, can, static_cast<int>(lt), static_cast<int>(hops));
    }
    return out;
}

// ---- RCCL --------------------------------------------------------------------------

class Comm {
  public:
    Comm(py::bytes id, int rank, int size, int device, double init_timeout_s, int min_ctas, int max_ctas) {
        std::string sid(id);
        py::gil_scoped_release nogil;  // init polls its deadline; other threads keep running
        c_.reset(new kfk::RcclComm(sid, rank, size, device, init_timeout_s, min_ctas, max_ctas));
    }
    py::tuple ctas() const { return py::make_tuple(c_->min_ctas(), c_->max_ctas()); }
    int rank() const { return c_->rank(); }
    int size() const { return c_->size(); }
    bool valid() const { return c_->valid(); }
    bool blocking() const { return c_->blocking(); }
    void all_reduce(at::Tensor in, at::Tensor out, int64_t op, int64_t stream, const std::string &tag) {
        check_gpu(in, "in");
        check_gpu(out, "out");
        TORCH_CHECK(in.numel() == out.numel(), "all_reduce: size mismatch");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->all_reduce(in.data_ptr(), out.data_ptr(), in.numel(), dtype_code(in), static_cast<int>(op),
                       stream_of(in, stream), tag.c_str());
    }
    void broadcast(at::Tensor t, int64_t root, int64_t stream, const std::string &tag) {
        check_gpu(t, "t");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->broadcast(t.data_ptr(), t.data_ptr(), t.numel(), dtype_code(t), static_cast<int>(root),
                      stream_of(t, stream), tag.c_str());
    }
    void reduce(at::Tensor in, at::Tensor out, int64_t op, int64_t root, int64_t stream, const std::string &tag) {
        check_gpu(in, "in");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->reduce(in.data_ptr(), out.data_ptr(), in.numel(), dtype_code(in), static_cast<int>(op),
                   static_cast<int>(root), stream_of(in, stream), tag.c_str());
    }
    void all_gather(at::Tensor in, at::Tensor out, int64_t stream, const std::string &tag) {
        check_gpu(in, "in");
        check_gpu(out, "out");
        TORCH_CHECK(out.numel() == in.numel() * c_->size(), "all_gather: out must hold size*numel(in)");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->all_gather(in.data_ptr(), out.data_ptr(), in.numel(), dtype_code(in), stream_of(in, stream),
                       tag.c_str());
    }
    void reduce_scatter(at::Tensor in, at::Tensor out, int64_t op, int64_t stream, const std::string &tag) {
        check_gpu(in, "in");
        check_gpu(out, "out");
        TORCH_CHECK(in.numel() == out.numel() * c_->size(), "reduce_scatter: in must hold size*numel(out)");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->reduce_scatter(in.data_ptr(), out.data_ptr(), out.numel(), dtype_code(in), static_cast<int>(op),
                           stream_of(in, stream), tag.c_str());
    }
    void send(at::Tensor t, int64_t peer, int64_t stream) {
        check_gpu(t, "t");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->send(t.data_ptr(), t.numel(), dtype_code(t), static_cast<int>(peer), stream_of(t, stream));
    }
    void recv(at::Tensor t, int64_t peer, int64_t stream) {
        check_gpu(t, "t");
        py::gil_scoped_release nogil;  // enq may poll wait_ready (non-blocking comms)
        c_->recv(t.data_ptr(), t.numel(), dtype_code(t), static_cast<int>(peer), stream_of(t, stream));
    }
    void group_start() { c_->group_start(); }
    void group_end() {
        py::gil_scoped_release nogil;
        c_->group_end();
    }
    void watch(int64_t stream, const std::string &what) {
        c_->watch(reinterpret_cast<hipStream_t>(stream), what);
    }
    int async_error() { return c_->async_error(); }
    // Graph all-reduce on the device: one round = one grouped batch of send/recv
    // (kungfu::plan_graph_all_reduce), then the K1 reduce kernel for every received
    // partial (buf[off:off+len] = op(buf[...], scratch[sc:sc+len])).  Every rank must run
    // its own plan of the same strategy graphs (same rounds, matched ops).
    using Xfer = std::tuple<int, int, int64_t, int64_t, int64_t>;  // recv, peer, off, len, scratch
    void graph_run(at::Tensor buf, c10::optional<at::Tensor> scratch, const std::vector<std::vector<Xfer>> &rounds,
                   int64_t op, int64_t stream) {
        check_gpu(buf, "buf");
        TORCH_CHECK(buf.is_contiguous(), "graph_run: buf must be contiguous");
        const int dt = dtype_code(buf);
        const size_t esz = buf.element_size();
        auto *base = static_cast<uint8_t *>(buf.data_ptr());
        uint8_t *sbase = nullptr;
        int64_t sn = 0;
        if (scratch && scratch->defined()) {
            TORCH_CHECK(scratch->is_cuda() && scratch->scalar_type() == buf.scalar_type() && scratch->is_contiguous() &&
                            scratch->device() == buf.device(),
                        "graph_run: scratch must be a contiguous tensor of buf's dtype on its device");
            sbase = static_cast<uint8_t *>(scratch->data_ptr());
            sn = scratch->numel();
        }
        const int64_t n = buf.numel();
        // validate the whole plan before issuing anything
        for (const auto &r : rounds)
            for (const auto &x : r) {
                const int64_t off = std::get<2>(x), len = std::get<3>(x), sc = std::get<4>(x);
                const int peer = std::get<1>(x);
                TORCH_CHECK(off >= 0 && len >= 0 && off + len <= n, "graph_run: range out of bounds");
                TORCH_CHECK(peer >= 0 && peer < c_->size() && peer != c_->rank(), "graph_run: bad peer");
                TORCH_CHECK(!std::get<0>(x) || sc < 0 || (sbase && sc + len <= sn), "graph_run: scratch too small");
            }
        c10::DeviceGuard gd(buf.device());
        auto s = stream_of(buf, stream);
        py::gil_scoped_release nogil;
        for (const auto &r : rounds) {
            if (r.empty()) continue;
            c_->group_start();
            for (const auto &x : r) {
                const int peer = std::get<1>(x);
                const int64_t off = std::get<2>(x), len = std::get<3>(x), sc = std::get<4>(x);
                if (std::get<0>(x)) {
                    uint8_t *dst = sc >= 0 ? sbase + sc * esz : base + off * esz;
                    c_->recv(dst, len, dt, peer, s);
                } else {
                    c_->send(base + off * esz, len, dt, peer, s);
                }
            }
            c_->group_end();
            for (const auto &x : r) {
                const int64_t off = std::get<2>(x), len = std::get<3>(x), sc = std::get<4>(x);
                if (std::get<0>(x) && sc >= 0)
                    kfk::launch_reduce(base + off * esz, base + off * esz, sbase + sc * esz, len, dt,
                                       static_cast<int>(op), s);
            }
        }
        c_->watch(s, "GraphAllReduce(" + std::to_string(rounds.size()) + " rounds, " + std::to_string(n) + " elems)");
    }
    void destroy() {
        py::gil_scoped_release nogil;
        c_->destroy();
    }
    void abort() { c_->abort(); }

  private:
    std::unique_ptr<kfk::RcclComm> c_;
};

}  // namespace

// Native backtrace on SIGSEGV / SIGBUS / SIGABRT (KUNGFU_NATIVE_BACKTRACE=1, a debugging aid: Python's
// faulthandler shows only the Python frames of a crash inside RCCL / HIP).  Chains to the previous
// handler so faulthandler still prints its part.
namespace {
struct sigaction g_prev_segv, g_prev_bus, g_prev_abrt;
void native_bt_handler(int sig, siginfo_t *info, void *uc) {
    static const char hdr[] = "\n[F] kungfu: native backtrace (signal):\n";
    (void)!write(2, hdr, sizeof(hdr) - 1);
    void *frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    struct sigaction *prev = sig == SIGSEGV ? &g_prev_segv : sig == SIGBUS ? &g_prev_bus : &g_prev_abrt;
    sigaction(sig, prev, nullptr);
    if (prev->sa_flags & SA_SIGINFO) {
        if (prev->sa_sigaction) prev->sa_sigaction(sig, info, uc);
    } else if (prev->sa_handler != SIG_DFL && prev->sa_handler != SIG_IGN && prev->sa_handler) {
        prev->sa_handler(sig);
    }
    raise(sig);
}
void install_native_backtrace() {
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = native_bt_handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &g_prev_segv);
    sigaction(SIGBUS, &sa, &g_prev_bus);
    sigaction(SIGABRT, &sa, &g_prev_abrt);
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
    m.def("install_native_backtrace", &install_native_backtrace,
          "print a native backtrace to stderr on SIGSEGV/SIGBUS/SIGABRT (chains to the previous handler)");
    m.doc() = "kungfu-amd CDNA4 kernels (gfx950) and RCCL controller";
    m.def("reduce", &reduce_op, "K1: z = op(x, y)");
    m.def("sgd_step", &sgd_step, "K8: fused SGD/momentum/nesterov/wd step on flat f32 buffers", py::arg("w"),
          py::arg("g"), py::arg("m"), py::arg("shadow"), py::arg("lr"), py::arg("lr_t"), py::arg("mu"),
          py::arg("damp"), py::arg("wd"), py::arg("gscale"), py::arg("nesterov"), py::arg("first"));
    m.def("adam_step", &adam_step, "fused Adam/AdamW step on flat f32 buffers (shadow: also bf16(w) there)",
          py::arg("w"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lr"), py::arg("lr_t"), py::arg("b1"),
          py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("adamw"), py::arg("gscale"), py::arg("step"),
          py::arg("shadow") = py::none());
    m.def("axpby", &axpby, "y = a*y + b*x (optionally also z = y)", py::arg("y"), py::arg("x"), py::arg("z"),
          py::arg("a"), py::arg("b"));
    m.def("scale_", &scale_, "x *= alpha");
    m.def("square", &square, "dst = src^2");
    m.def("cast_copy", &cast_copy, "dst = scale * src with an f32 <-> bf16 cast");
    m.def("sumsq2", &sumsq2, "[sum(a^2), sum(b^2)] in one pass", py::arg("a"), py::arg("b") = py::none());
    m.def("variance", &variance, "sum |s2*inv - (s1*inv)^2|");
    m.def("gns_update", &gns_update, "device-side gradient-noise-scale EMA update");
    m.def("seg_variance", &seg_variance, "sum_k ||E[g^2]-E[g]^2||_2 over flat tensor segments");
    m.def("grad_accumulate", &grad_accumulate, "flat[off_i:] += scale * src_i for a list of bf16/f32 tensors",
          py::arg("flat"), py::arg("srcs"), py::arg("offsets"), py::arg("scale") = 1.0);
    m.def("pack", &pack, "multi-tensor pack into a flat buffer");
    m.def("unpack", &unpack, "multi-tensor unpack from a flat buffer");
    m.def("conv3x3", &conv3x3, "3x3 pad-1 NHWC bf16 convolution (MFMA implicit GEMM)", py::arg("x"), py::arg("w"),
          py::arg("stride") = 1, py::arg("variant") = -1);
    m.def("conv3x3_variants", &kfk::conv3x3_variants);
    m.def("conv", &conv, "1x1/3x3 NHWC bf16 convolution (MFMA implicit GEMM) with fused BN-statistics and "
          "accumulate epilogues", py::arg("x"), py::arg("w"), py::arg("stride") = 1, py::arg("stats") = py::none(),
          py::arg("out") = py::none(), py::arg("variant") = -1, py::arg("bn_x") = py::none(),
          py::arg("bn_fcoef") = py::none(), py::arg("bn_mask") = py::none(), py::arg("bias") = py::none(),
          py::arg("gate") = false, py::arg("acc_mask") = py::none(), py::arg("acc_even") = false,
          py::arg("fin") = py::none());
    m.def("stem3_pack_weight", &stem3_pack_weight, "pack [32, 3, KH, KW] stem weights for stem3_forward");
    m.def("stem3_forward", &stem3_forward, "small image-stem conv (<= 4x4 window, 3 -> 32 channels) with the BN-sums "
          "epilogue", py::arg("x"), py::arg("wp"), py::arg("kh"), py::arg("kw"), py::arg("stride"), py::arg("ph"),
          py::arg("pw"), py::arg("stats") = py::none());
    m.def("stem3_wgrad", &stem3_wgrad, "its weight gradient (MFMA over pixels, deterministic)", py::arg("dy"),
          py::arg("x"), py::arg("kh"), py::arg("kw"), py::arg("stride"), py::arg("ph"), py::arg("pw"),
          py::arg("out_f32") = false);
    m.def("bn_fin_desc", &bn_fin_desc, "pack an in-launch BN finalize descriptor (CPU uint8; copy it to the GPU)",
          py::arg("mode"), py::arg("tensors"), py::arg("rows"), py::arg("momentum") = 0.1, py::arg("eps") = 1e-5,
          py::arg("training") = true);
    m.def("conv_rect", &conv_rect, "KH x KW NHWC bf16 convolution with zero padding (MFMA implicit GEMM; "
          "Inception-v3 windows) with an optional BN-statistics epilogue", py::arg("x"), py::arg("w"),
          py::arg("stride") = 1, py::arg("ph") = 0, py::arg("pw") = 0, py::arg("stats") = py::none(),
          py::arg("out") = py::none(), py::arg("bn_x") = py::none(), py::arg("bn_fcoef") = py::none());
    m.def("conv_rect_supported", &kfk::conv_rect_supported);
    m.def("gemm", &gemm, "linear layer x @ w^T on the MFMA kernel with bias / GELU-gradient(+bias-gradient "
          "sums) / accumulate epilogues", py::arg("x"), py::arg("w"), py::arg("bias") = py::none(),
          py::arg("out") = py::none(), py::arg("gelu_u") = py::none(),
          py::arg("stats") = py::none(), py::arg("variant") = -1);
    m.def("gemm_supported", &kfk::gemm_supported);
    m.def("conv_dgrad_s2", &conv_dgrad_s2, "data gradient of a stride-2 1x1/3x3 NHWC bf16 convolution (parity-phase "
          "MFMA implicit GEMMs)", py::arg("dy"), py::arg("wt"), py::arg("ks"), py::arg("stats") = py::none(),
          py::arg("bn_x") = py::none(), py::arg("bn_fcoef") = py::none(), py::arg("bn_mask") = py::none(),
          py::arg("variant") = -1, py::arg("dh") = 0, py::arg("dw") = 0, py::arg("pad") = 1,
          py::arg("fin") = py::none());
    m.def("xent_forward", &xent_forward, "fused softmax cross-entropy over bf16 logits: (lse, per-row loss)");
    m.def("xent_backward", &xent_backward, "its bf16 logit gradient, scaled by scale[0]");
    m.def("gelu_backward_colsum", &gelu_backward_colsum, "erf-GELU backward du and the column sums of du",
          py::arg("dy"), py::arg("u"), py::arg("dtype"));
    m.def("colsum", &colsum, "column sums of a bf16 [T, O] matrix (bias gradient), deterministic", py::arg("x"),
          py::arg("dtype"));
    m.def("conv_wgrad_rect", &conv_wgrad_rect, "weight gradient of a KH x KW padded NHWC bf16 convolution "
          "(split-K MFMA GEMM, any channel count % 8)", py::arg("dy"), py::arg("x"), py::arg("kh"), py::arg("kw"),
          py::arg("stride") = 1, py::arg("ph") = 0, py::arg("pw") = 0, py::arg("variant") = -1);
    m.def("conv_wgrad_rect_supported", &kfk::conv_wgrad_rect_supported);
    m.def("conv_wgrad_rows_rect_auto", &kfk::conv_wgrad_rows_rect_auto, "the row-image weight-gradient variant "
          "conv_wgrad_rect(..., 13) picks for this shape (args: N, H, W, Cin, Cout, kh, kw, ph, pw, stride)");
    m.def("conv_wgrad_rows_rect_supported", &kfk::conv_wgrad_rows_rect_supported, "row-image weight-gradient kernel "
          "covers this stride-1 window (args: N, H, W, Cin, Cout, kh, kw, ph, pw, stride)");
    m.def("conv_wgrad", &conv_wgrad, "weight gradient of the 1x1/3x3 NHWC bf16 convolution (split-K MFMA GEMM)",
          py::arg("dy"), py::arg("x"), py::arg("ks"), py::arg("stride") = 1, py::arg("out") = py::none(),
          py::arg("accumulate") = false, py::arg("variant") = -1, py::arg("splits") = -1,
          py::arg("atomics") = true);
    m.def("conv_wgrad_supported", &kfk::conv_wgrad_supported);
    m.def("bias_act_supported", &kfk::bias_act_supported);
    m.def("maxpool2x2_forward", &maxpool2x2_forward, "2x2/s2 max-pool, NHWC bf16 (no argmax tensor)");
    m.def("maxpool2x2_backward", &maxpool2x2_backward, "2x2/s2 max-pool gradient (gather from x, dy); gate_stats: "
          "x is a ReLU output, also gate by x > 0 and sum the result per channel", py::arg("x"), py::arg("dy"),
          py::arg("gate_stats") = py::none());
    m.def("maxpool3s2_forward", &maxpool3s2_forward, "3x3/s2 max-pool (pad 0/1), NHWC bf16 -> (y, argmax bytes)");
    m.def("maxpool3s2_backward", &maxpool3s2_backward, "3x3/s2 max-pool gradient (gather via the argmax bytes)");
    m.def("layernorm_supported", &kfk::layernorm_supported);
    m.def("layernorm_forward", &layernorm_forward, "fused residual-add + LayerNorm (bf16 rows) -> (y, s, mean, rstd)",
          py::arg("x"), py::arg("r"), py::arg("gamma"), py::arg("beta"), py::arg("eps"), py::arg("p") = 0.0,
          py::arg("seed") = 0);
    m.def("layernorm_backward", &layernorm_backward,
          "LayerNorm backward -> (ds, dgamma, dbeta, dr or None[, residual-input bias gradient])", py::arg("dy"),
          py::arg("s"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"), py::arg("p") = 0.0, py::arg("seed") = 0,
          py::arg("rbias_dtype") = py::none());
    m.def("global_avgpool_forward", &global_avgpool_forward, "global average pool, NHWC bf16 -> [N, C]");
    m.def("global_avgpool_backward", &global_avgpool_backward, "global average pool backward -> NHWC bf16",
          py::arg("dy"), py::arg("H"), py::arg("W"));
    m.def("avgpool3s1", &avgpool3s1, "3x3/s1/p1 average pool, count_include_pad (also its own gradient on dy)");
    m.def("bias_act_forward_", &bias_act_forward_, "y = relu(y + bias) in place (NHWC bf16, f32 bias)",
          py::arg("y"), py::arg("bias"), py::arg("relu") = true);
    m.def("bias_act_backward", &bias_act_backward, "(dy * (y > 0), its per-channel sum) in one pass",
          py::arg("dy"), py::arg("y"), py::arg("relu") = true);
    m.def("conv_wgrad_variants", &kfk::conv_wgrad_variants);
    m.def("attention_supported", &kfk::attention_supported);
    m.def("attention_forward", &attention_forward, "fused self-attention forward (S 64/128, head dim 64, dropout)",
          py::arg("qkv"), py::arg("heads"), py::arg("scale"), py::arg("seed"), py::arg("p_drop"));
    m.def("attention_backward", &attention_backward, "fused self-attention backward -> dqkv", py::arg("qkv"),
          py::arg("out"), py::arg("lse"), py::arg("dout"), py::arg("heads"), py::arg("scale"), py::arg("seed"),
          py::arg("p_drop"));
    m.def("conv_wgrad_max_pixels", &kfk::conv_wgrad_max_pixels, py::arg("N"), py::arg("H"), py::arg("W"),
          py::arg("Cin"), py::arg("Cout"), py::arg("ks"), py::arg("stride"));
    m.def("conv_wgrad_plan", [](int N, int H, int W, int Cin, int Cout, int ks, int stride, int variant, int splits) {
        const auto p = kfk::conv_wgrad_plan(N, H, W, Cin, Cout, ks, stride, variant, splits);
        return py::make_tuple(p.variant, p.splits, p.kps, p.ws_floats);
    }, py::arg("N"), py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("ks"), py::arg("stride"),
          py::arg("variant") = -1, py::arg("splits") = -1);
    m.def("conv_flip_weight", &conv_flip_weight, "w[co,ci,kh,kw] -> w[ci,co,KS-1-kh,KS-1-kw] (data-gradient weights)");
    m.def("conv_supported", &kfk::conv_supported);
    m.def("conv_flip_weights", &conv_flip_weights, "multi-tensor conv_flip_weight into preallocated outputs");
    m.attr("conv_stat_slots") = kfk::kStatSlots;
    m.def("conv3x3_flip_weight", &conv3x3_flip_weight, "w[co,ci,kh,kw] -> w[ci,co,2-kh,2-kw] (data-gradient weights)");
    m.def("conv3x3_supported", &kfk::conv3x3_supported);
    m.def("bn_supported_channels", &kfk::bn_supported_channels);
    m.def("bn_forward", &bn_forward,
          "fused NHWC BN(+residual)(+ReLU) forward -> (y, mean, invstd, coef, relu mask or None)", py::arg("x"),
          py::arg("res"), py::arg("weight"), py::arg("bias"), py::arg("running_mean"), py::arg("running_var"),
          py::arg("momentum"), py::arg("eps"), py::arg("training"), py::arg("relu"),
          py::arg("num_batches") = py::none(), py::arg("sums") = py::none(), py::arg("res_coef") = py::none(),
          py::arg("apply") = true, py::arg("out") = py::none(), py::arg("pre") = py::none());
    m.def("bn_backward_multi", &bn_backward_multi,
          "backward of several BN+ReLUs (slices of one concatenation's gradient): one batched finalize");
    m.def("bn_finalize_multi", &bn_finalize_multi,
          "batched sums-finalize of several training BNs in one launch -> [[mean, invstd, coef], ...]");
    m.def("bn_backward", &bn_backward, "fused NHWC BN(+residual)(+ReLU) backward -> (dx, dres, dweight, dbias)",
          py::arg("dy"), py::arg("x"), py::arg("mean"), py::arg("invstd"), py::arg("weight"), py::arg("fcoef"),
          py::arg("mask"), py::arg("relu"), py::arg("training"), py::arg("want_dres"), py::arg("sums") = py::none(),
          py::arg("dres_x") = py::none(), py::arg("dres_sums") = py::none(), py::arg("pre") = py::none());
    m.def("bn_pool_supported", [](int64_t C, int64_t H, int64_t W) {
        return kfk::bn_pool_supported(kfk::BNShape{H * W, static_cast<int>(C)}, static_cast<int>(H),
                                      static_cast<int>(W));
    });
    m.def("bn_pool_forward", &bn_pool_forward,
          "stem BN+ReLU+MaxPool(3,2,1) forward -> (y_pool, mean, invstd, coef, argmax)", py::arg("x"),
          py::arg("weight"), py::arg("bias"), py::arg("running_mean"), py::arg("running_var"), py::arg("momentum"),
          py::arg("eps"), py::arg("training"), py::arg("num_batches") = py::none(), py::arg("sums") = py::none());
    m.def("stem_pad4", &stem_pad4, "[N,3,H,W] bf16/f32 -> [N,4,H,W] channels_last bf16 (zero 4th channel)");
    m.def("stem_pack_weight", &stem_pack_weight, "[64,3,7,7] stem weights -> packed [64,224] for stem_forward");
    m.def("stem_forward", &stem_forward, "7x7/2 pad-3 stem conv on MFMA with fused BN statistics",
          py::arg("x4"), py::arg("wp"), py::arg("stats") = py::none());
    m.def("stem_wgrad", &stem_wgrad, "stem conv weight gradient (split-K MFMA)", py::arg("dy"), py::arg("x4"),
          py::arg("splits") = -1);
    m.def("bn_pool_backward", &bn_pool_backward, "stem BN+ReLU+MaxPool backward -> (dx, dweight, dbias, coef)",
          py::arg("dy"), py::arg("arg"), py::arg("x"), py::arg("mean"), py::arg("invstd"), py::arg("weight"),
          py::arg("fcoef"), py::arg("training"), py::arg("xarg") = py::none(), py::arg("apply") = true);
    m.def("stem_wgrad_bnp", &stem_wgrad_bnp, "stem conv weight gradient with dy formed from the BN+ReLU+MaxPool "
          "backward while staging (the BN input gradient is never materialised)", py::arg("y"), py::arg("x4"),
          py::arg("dyp"), py::arg("arg"), py::arg("fcoef"), py::arg("bcoef"), py::arg("splits") = -1);
    m.def("stem_wgrad_bnp_supported", &kfk::stem_wgrad_bnp_supported);
    m.def("ipc_alloc", &ipc_alloc, "dedicated f32 device buffer exportable over HIP IPC");
    m.def("ipc_handle", &ipc_handle, "HIP IPC handle (64 bytes) of an ipc_alloc buffer");
    m.def("ipc_open", &ipc_open, "map a peer's exported buffer as an f32 tensor");
    m.def("gemm_nt", &gemm_nt, py::arg("a"), py::arg("b"), py::arg("bias") = py::none(), py::arg("out") = py::none(),
          py::arg("accumulate") = false, py::arg("bn") = -1,
          "bf16 a[M,K] . b[N,K]^T (+bias) (+out) on the pipelined 256 x bn MFMA GEMM (gemm.hip)");
    m.def("gemm_nt_supported", &kfk::gemm_nt_supported);
    m.def("gemm_nt_ld", &gemm_nt_ld, py::arg("a"), py::arg("b"), py::arg("bias") = py::none(), py::arg("ldc") = 0,
          py::arg("bn") = 256, "C [M, ldc] = a . b^T (+ bias) for any N (columns >= N of C unspecified)");
    m.def("gemm_nt_ld_supported", &kfk::gemm_nt_ld_supported);
    m.def("gemm_nt_gelu_grad", &gemm_nt_gelu_grad, "(du, db): the GELU backward fused into the data-gradient NT GEMM "
          "(du = bf16(bf16(a . b^T) * gelu'(u)), db = column sums of du)", py::arg("a"), py::arg("b"), py::arg("u"),
          py::arg("bias_dtype") = py::none());
    m.def("embedding_backward", &embedding_backward, py::arg("grad"), py::arg("ids"), py::arg("dy"), py::arg("ch") = 0,
          "grad[ids[t]] += dy[t] by f32 atomics (graph-replayable embedding gradient)");
    m.def(
        "set_dropout_seed_base",
        [](c10::optional<at::Tensor> t) {
            if (!t || !t->defined()) {
                kfk::set_dropout_seed_base(nullptr);
                return;
            }
            TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kInt && t->numel() >= 1 && t->is_contiguous(),
                        "set_dropout_seed_base: a contiguous int32 GPU tensor (kept alive by the caller)");
            kfk::set_dropout_seed_base(reinterpret_cast<const uint32_t *>(t->data_ptr()));
        },
        py::arg("base"), "device word mixed into every hashed dropout seed (None: host seeds only)");
    m.def("gemm_nt_pick_bn", &kfk::gemm_nt_pick_bn);
    m.def("comm_emulate", &comm_emulate, py::arg("bucket"), py::arg("scratch"), py::arg("traffic_bytes"),
          py::arg("ctas"), py::arg("seconds"), py::arg("stream") = 0,
          "local footprint of one all-reduce: ctas workgroups stream traffic_bytes, resident for seconds");
    m.def("device_links", &device_links, py::arg("device"),
          "[(peer, can_access_peer, link_type, hops)] of `device` to every other visible device");
    m.def("rccl_unique_id", [] { return py::bytes(kfk::RcclComm::unique_id()); });
    m.def("rccl_version", &kfk::RcclComm::version);
    m.def("rccl_watchdog_info", [] {
        const auto i = kfk::watchdog_info();
        py::dict d;
        d["registered"] = i.registered;
        d["completed"] = i.completed;
        d["pending"] = i.pending;
        d["oldest_s"] = i.oldest_s;
        d["timeout_s"] = i.timeout_s;
        d["abort_on_stall"] = i.abort_on_stall;
        d["stalls_logged"] = i.stalls_logged;
        return d;
    });
    kfk::watchdog_set_freeze_hook([] {
        if (Py_IsInitialized()) PyGILState_Ensure();  // held until the process exits
    });
    m.def("rccl_watchdog_set_label", &kfk::watchdog_set_label);
    m.def("rccl_watchdog_set_timeout", &kfk::watchdog_set_timeout);
    py::class_<kfk::PairPrefetcher>(m, "PairPrefetcher",
                                    "native prefetch thread of the pair-averaging peer model (pair_prefetch.hip)")
        .def(py::init<const std::string &, int, int, const std::string &, const std::string &, int64_t, int>(),
             py::arg("libpath"), py::arg("device"), py::arg("self_rank"), py::arg("rec_name"), py::arg("model_name"),
             py::arg("nbytes"), py::arg("slots") = 3)
        .def(
            "start",
            [](kfk::PairPrefetcher &p, uintptr_t pending_ev, int64_t pending_ver, uintptr_t host_copy, int target,
               std::vector<uintptr_t> src_slots, int64_t own_ver, uintptr_t dst, uintptr_t after_ev,
               uintptr_t host_stage) {
                kfk::PairPrefetcher::Job j;
                j.pending_ev = pending_ev, j.pending_ver = pending_ver, j.host_copy = host_copy, j.target = target;
                j.src_slots = std::move(src_slots), j.own_ver = own_ver, j.dst = dst, j.after_ev = after_ev;
                j.host_stage = host_stage;
                py::gil_scoped_release nogil;  // waits for the previous job
                p.start(j);
            },
            py::arg("pending_ev"), py::arg("pending_ver"), py::arg("host_copy"), py::arg("target"),
            py::arg("src_slots"), py::arg("own_ver"), py::arg("dst"), py::arg("after_ev"), py::arg("host_stage"))
        .def("busy", &kfk::PairPrefetcher::busy)
        .def(
            "finish",
            [](kfk::PairPrefetcher &p, uintptr_t wait_stream) {
                kfk::PairPrefetcher::Result r;
                {
                    py::gil_scoped_release nogil;
                    r = p.finish(wait_stream);
                }
                if (!r.error.empty()) throw std::runtime_error(r.error);
                return py::make_tuple(r.status, r.version, r.own_ver);
            },
            py::arg("wait_stream"), "join the job: (status 0 none / 1 pulled / 2 dropped, version, own advertised version)");

    py::class_<Comm>(m, "RcclComm")
        .def(py::init<py::bytes, int, int, int, double, int, int>(), py::arg("uid"), py::arg("rank"),
             py::arg("size"), py::arg("device"), py::arg("init_timeout_s") = 0.0, py::arg("min_ctas") = 0,
             py::arg("max_ctas") = 0)
        .def("ctas", &Comm::ctas, "(min, max) CTA budget of this communicator (0 = RCCL default)")
        .def("rank", &Comm::rank)
        .def("size", &Comm::size)
        .def("valid", &Comm::valid)
        .def("blocking", &Comm::blocking)
        .def("all_reduce", &Comm::all_reduce, py::arg("input"), py::arg("output"), py::arg("op") = 0,
             py::arg("stream") = 0, py::arg("tag") = "")
        .def("broadcast", &Comm::broadcast, py::arg("tensor"), py::arg("root") = 0, py::arg("stream") = 0,
             py::arg("tag") = "")
        .def("reduce", &Comm::reduce, py::arg("input"), py::arg("output"), py::arg("op") = 0, py::arg("root") = 0,
             py::arg("stream") = 0, py::arg("tag") = "")
        .def("all_gather", &Comm::all_gather, py::arg("input"), py::arg("output"), py::arg("stream") = 0,
             py::arg("tag") = "")
        .def("reduce_scatter", &Comm::reduce_scatter, py::arg("input"), py::arg("output"), py::arg("op") = 0,
             py::arg("stream") = 0, py::arg("tag") = "")
        .def("group_start", &Comm::group_start)
        .def("group_end", &Comm::group_end)
        .def("watch", &Comm::watch, py::arg("stream"), py::arg("what"))
        .def("async_error", &Comm::async_error)
        .def("send", &Comm::send, py::arg("tensor"), py::arg("peer"), py::arg("stream") = 0)
        .def("recv", &Comm::recv, py::arg("tensor"), py::arg("peer"), py::arg("stream") = 0)
        .def("graph_run", &Comm::graph_run, "grouped send/recv rounds + K1 reduce (device graph all-reduce)",
             py::arg("buf"), py::arg("scratch"), py::arg("rounds"), py::arg("op") = 0, py::arg("stream") = 0)
        .def("destroy", &Comm::destroy)
        .def("abort", &Comm::abort);
}
