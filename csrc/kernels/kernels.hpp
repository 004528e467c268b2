// Host-side launchers of the kungfu-amd HIP kernels (no torch dependency).
// Every launcher enqueues on `stream` and never synchronises, so it can be
// captured into a hipGraph.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace kfk {

constexpr int kMaxGridHost = 2048;  // == kMaxGrid in common.hpp (partials scratch size)

// K1: z = op(x, y) elementwise.  dtype/op codes as kungfu::DType / ReduceOp.
void launch_reduce(void *z, const void *x, const void *y, size_t n, int dtype, int op, hipStream_t s);

// Embedding gradient by f32 atomics (flat_ops.hip): grad[ids[t], :] += dy[t, :], D % 4 == 0.
// ch: tokens per thread run (<= 0: by T / V).
void launch_embedding_backward(float *grad, const int64_t *ids, const void *dy, bool dy_bf16, int64_t T, int D,
                               int64_t V, hipStream_t s, int ch = 0);

// Device word mixed into every hashed dropout seed (attention, add+LayerNorm): a graph replay
// re-uses the host seeds recorded at capture, so kungfu_amd.ops.dropout_seed advances this word
// before each replay instead (null: host seeds only).  Defined in flat_ops.hip.
void set_dropout_seed_base(const uint32_t *p);
const uint32_t *dropout_seed_base();

// gemm.hip: C[M, N] = A[M, K] . B[N, K]^T (+ bias[N]) (+ C) in bf16, f32 accumulation, on a
// 256 x bn tile (bn 128 | 192 | 256, <= 0: by shape) with a 3-slab-deep LDS-DMA pipeline.
constexpr int kGemmBias = 1, kGemmAccum = 2, kGemmGeluGrad = 4;
bool gemm_nt_supported(int64_t M, int64_t N, int64_t K);
int gemm_nt_pick_bn(int64_t M, int64_t N);
void launch_gemm_nt(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K,
                    int epi, int bn, hipStream_t s);
// any N >= 1 (rows of B past N read zeros) with C's row stride ldc (% 8 == 0, >= N rounded up to 8):
// the chunk of 8 columns holding column N - 1 is stored whole, into the row padding
bool gemm_nt_ld_supported(int64_t M, int64_t N, int64_t K, int64_t ldc);
void launch_gemm_nt_ld(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K,
                       int ldc, int epi, int bn, hipStream_t s);
// The GELU backward fused into the data-gradient GEMM of the layer that consumes gelu(u):
// c = bf16(bf16(a . b^T) * gelu'(u)) (u: the pre-activation [M, N]) on 256 x 256 tiles (N % 256 == 0),
// and part[gemm_nt_gelu_grad_rows(M)][N] f32 = per-128-row column sums of c -- folded by
// launch_colsum_fold into the bias gradient of the layer that produced u (deterministic)
int gemm_nt_gelu_grad_rows(int M);
void launch_gemm_nt_gelu_grad(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *u, float *part, int M,
                              int N, int K, hipStream_t s);
void launch_colsum_fold(const float *part, int rows, int O, float *out_f32, uint16_t *out_bf16, hipStream_t s);

// comm_emu.hip: the local footprint of one all-reduce of `bytes` (bench.py --emulate-comm):
// `ctas` workgroups copying `traffic_bytes` of the bucket into `scratch` (>= bytes), paced over
// and resident for `seconds`.  The bucket is only read.
void launch_comm_emulate(const void *bucket, void *scratch, int64_t bytes, int64_t traffic_bytes, int ctas,
                         double seconds, hipStream_t s);

// K8: fused SGD step on flat f32 buffers (torch.optim.SGD semantics):
//   d = g*gscale + wd*w ; m = first ? d : mu*m + (1-damp)*d ; d = nesterov ? d + mu*m : m ; w -= lr*d
// lr is read from *lr_dev when lr_dev != nullptr (graph-capture friendly).
// If shadow != nullptr the updated weights are also written as bf16 there.
void launch_sgd(float *w, const float *g, float *m, uint16_t *shadow, size_t n, float lr, const float *lr_dev,
                float mu, float damp, float wd, float gscale, bool nesterov, bool first, hipStream_t s);

// Fused Adam / AdamW step on flat f32 buffers.  step_dev points at a float
// step counter already incremented for this step (bias correction on device).  shadow (optional):
// also writes bf16(w) there -- the bf16 compute copy of the new weights.
void launch_adam(float *w, const float *g, float *m, float *v, size_t n, float lr, const float *lr_dev, float b1,
                 float b2, float eps, float wd, bool adamw, float gscale, const float *step_dev, hipStream_t s,
                 uint16_t *shadow = nullptr);

// K3/K4: y = a*y + b*x (f32 or bf16), optionally also writing the result to z.
void launch_axpby(void *y, const void *x, void *z, size_t n, float a, float b, int dtype, hipStream_t s);

// K2: x *= alpha (f32 / bf16 / f16).
void launch_scale(void *x, size_t n, float alpha, int dtype, hipStream_t s);

// K6 helper: dst = src^2 (f32 out, f32/bf16 in).
void launch_square(float *dst, const void *src, size_t n, int dtype, hipStream_t s);
// dst = scale * src, f32/bf16 -> f32/bf16 (bf16 gradient wire format)
void launch_cast(void *dst, const void *src, size_t n, int src_dt, int dst_dt, float scale, hipStream_t s);

// K5: out[0] = sum(a^2), out[1] = sum(b^2) in one pass (b may be null).
// `partials` needs 2*kMaxGrid floats of scratch.
// Column sums of a row-major bf16 [T, O] matrix (O % 8 == 0) into f32 or bf16 [O]: a linear
// layer's bias gradient.  Deterministic two-stage; part: f32 [colsum_chunks(T) * O] scratch.
int colsum_chunks(int64_t T, int O);
void launch_colsum_bf16(const uint16_t *x, int64_t T, int O, float *part, float *out_f32, uint16_t *out_bf16,
                        hipStream_t s);
// du = gelu'(u) * dy (bf16 [T, O], torch's erf-GELU backward) and the column sums of du (the bias
// gradient of the layer that produced u) in one pass + the colsum second stage.
int gelu_colsum_chunks(int64_t T, int O);  // partial rows of its scratch (part: f32 [chunks * O])
// Native prefetch thread of the pair-averaging peer model (pair_prefetch.hip).
class PairPrefetcher {
  public:
    struct Job {
        uintptr_t pending_ev = 0;  // snapshot event to host-wait before advertising (0: nothing to advertise)
        int64_t pending_ver = 0;   // its version
        uintptr_t host_copy = 0;   // host copy of the snapshot to save too (peers on other hosts), or 0
        int target = 0;            // peer to pull from
        std::vector<uintptr_t> src_slots;  // the target's ring slots (device pointers); empty: via host store
        int64_t own_ver = 0;       // own advertised version before this job (self-pull record)
        uintptr_t dst = 0;         // device destination
        uintptr_t after_ev = 0;    // event the copy waits for (the previous pull's consumer), or 0
        uintptr_t host_stage = 0;  // pinned host staging buffer for host-store pulls
    };
    struct Result {
        int status = 0;  // 0: nothing pulled, 1: pulled, 2: dropped (possibly torn)
        int64_t version = 0, own_ver = 0;
        std::string error;
    };
    PairPrefetcher(const std::string &libpath, int device, int self_rank, const std::string &rec_name,
                   const std::string &model_name, int64_t nbytes, int slots);
    ~PairPrefetcher();
    PairPrefetcher(const PairPrefetcher &) = delete;
    PairPrefetcher &operator=(const PairPrefetcher &) = delete;
    void start(const Job &job);
    bool busy();
    Result finish(uintptr_t wait_stream);  // joins the job; on success `wait_stream` waits on the copy

  private:
    struct Impl;
    Impl *d_;
};

// Softmax cross-entropy over bf16 logits [R, V] (V even; xent.hip): per-row log-sum-exp and loss
// (0 where the label is outside [0, V)); backward writes the bf16 gradient scaled by *scale.
// ld > 0: rows padded to ld classes (ld % 8 == 0, 16-byte aligned; 16-byte loads), dx likewise.
void launch_xent_forward(const uint16_t *x, const int64_t *labels, int64_t R, int V, float *lse, float *loss,
                         hipStream_t s, int64_t ld = 0);
void launch_xent_backward(const uint16_t *x, const int64_t *labels, const float *lse, const float *scale, int64_t R,
                          int V, uint16_t *dx, hipStream_t s, int64_t ld = 0);

// y = gelu(u) (erf form, bf16, n % 8 == 0; norms.hip)
void launch_gelu_bwd_colsum(const uint16_t *dy, const uint16_t *u, uint16_t *du, int64_t T, int O, float *part,
                            float *out_f32, uint16_t *out_bf16, hipStream_t s);
void launch_sumsq2(const void *a, const void *b, size_t n, int dtype, float *partials, float *out, hipStream_t s);

// K6: out[0] = sum_i | s2[i]*inv - (s1[i]*inv)^2 |  (s1 = sum g, s2 = sum g^2 over np ranks)
void launch_variance(const float *s1, const float *s2, size_t n, float inv_np, float *partials, float *out,
                     hipStream_t s);

// K6 (reference form): out[k] += sum over tensor k of (s2*inv - (s1*inv)^2)^2;
// seg_off is a device int64 array of nseg+1 tensor start offsets; out must be zeroed.
// The gradient variance is then sum_k sqrt(out[k]).
void launch_seg_variance(const float *s1, const float *s2, size_t n, float inv_np, const int64_t *seg_off, int nseg,
                         float *out, hipStream_t s);

// K5 epilogue on device: from sumsq(small-batch grad) and sumsq(big-batch grad)
// compute biased G/S estimates, update their EMAs in state[0..1] and write the
// noise scale S/G into state[2].  state[3] counts updates.
void launch_gns_update(const float *sumsq_small, const float *sumsq_big, float b_small, float b_big, float alpha,
                       float *state, hipStream_t s);

// K7: multi-tensor pack/unpack.  desc is a device array of n_tensors
// {ptr (int64), offset (elements), numel} triples; flat is contiguous.
// pack:   flat[off:off+numel] = scale * src (dtype cast src_dtype -> flat_dtype)
// unpack: dst = scale * flat[off:off+numel]
void launch_pack(const int64_t *desc, int n_tensors, size_t total, void *flat, int flat_dtype, int src_dtype,
                 float scale, hipStream_t s);
void launch_unpack(const int64_t *desc, int n_tensors, size_t total, const void *flat, int flat_dtype,
                   int dst_dtype, float scale, hipStream_t s);

// Bucket gradient accumulation: flat[off[t] + j] += scale * src[t][j], all
// sources of one dtype (bf16 or f32), one launch per table.  blk_start is the
// prefix sum of grad_accumulate_blocks(numel[t]) (blk_start[0] = 0).
struct GradAccTable {
    static constexpr int kMax = 48;
    int n = 0;
    int src_dtype = 0;
    float scale = 1.f;
    const void *src[kMax];
    int64_t off[kMax];
    int64_t numel[kMax];
    int blk_start[kMax + 1];
};
int grad_accumulate_blocks(int64_t numel);
void launch_grad_accumulate(const GradAccTable &tab, float *flat, hipStream_t s);

// 3x3 convolution, pad 1, stride 1|2, NHWC bf16 (x [N,H,W,Cin], w [Cout,3,3,Cin],
// y [N,OH,OW,Cout]) as an MFMA implicit GEMM (conv.hip).  Cin, Cout multiples of 64.
bool conv3x3_supported(int Cin, int Cout, int stride);
// variant: tile/pipeline choice (-1 = default for the shape; 0..conv3x3_variants()-1 for tuning).
void launch_conv3x3(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout,
                    int stride, hipStream_t s, int variant = -1);
int conv3x3_variants();
// General KS x KS (KS = 1 or 3, pad (KS-1)/2) convolution with fused epilogues:
// stats != nullptr: f64 atomics of per-output-channel sum / sum of squares of the bf16
// outputs into stats[0..K) / stats[K..2K) (the caller zeroes them; bn_stats_from_sums
// consumes and re-zeroes them); accumulate: y += conv(x, w) instead of y = conv(x, w).
// The stats workspace is kStatSlots x [2][K] f64 (tiles add into slot tile % kStatSlots,
// keeping atomic contention per address low); bn_forward(sums=...) folds the slots.
constexpr int kStatSlots = 16;
bool conv_supported(int Cin, int Cout, int ks, int stride);
// kEpiBiasRelu: y = relu(conv + bias) (bf16 bias, VGG's conv+bias+ReLU in the conv's epilogue);
// kEpiGate: the output is the gradient of a ReLU output ea.bx: y = conv * (bx > 0) (NaN in bx
// passes, like torch.relu's backward) and stats[slot][0][c] += sum(y) (that layer's bias gradient).
// kEpiAccMask (with kEpiAccum): y = old * amask + conv -- the residual gradient dz = dout * relu'
// formed from the raw output gradient and the 1-bit ReLU mask on the fly, so the BN3+add+ReLU
// backward need not write dz (ResNet identity blocks).
// Linear-layer (GEMM) epilogues, launch_gemm only:
//   kEpiBias      y = conv + bias (bf16 bias, added in f32 before the one rounding);
//   kEpiGeluGrad  the output is the gradient of a GELU output whose input is ea.bx (= u):
//                 y = bf16(conv) * gelu'(u) and stats[slot][0][c] += sum(y) (the bias gradient
//                 of the layer that produced u).
enum ConvEpi : int {
    kEpiFwdStats = 1, kEpiAccum = 2, kEpiBwdCoef = 4, kEpiBwdBits = 8, kEpiBiasRelu = 16, kEpiGate = 32,
    kEpiAccMask = 64, kEpiAccEven = 128, kEpiBias = 256, kEpiGeluGrad = 1024
    // (round 6: the BN normalise-on-load A operand, 2048, is gone -- +2.56 ms/step on ResNet-50,
    // profiles/r5_prebn.md; the FC1 bias + GELU forward epilogue, 512, too -- slower end to end than
    // hipBLASLt + the GELU pass, profiles/r5t34_bert_g*.log)
};
// In-launch BN finalize of a statistics epilogue (kEpiFwdStats / kEpiBwdCoef / kEpiBwdBits): every
// workgroup waits for its slot atomics, arrives on a two-level counter (per blockIdx % 8 shard,
// then across shards), and the LAST arriver folds the kStatSlots slots (sc1 loads: the f64 adds
// were performed at the memory side), writes what bn_sums_finalize / bn_bwd_finalize_sums would,
// re-zeroes the slots and the counter -- the separate finalize launch (and its kernel boundary)
// is gone.  The BN apply that follows is told the coefficients are already there.  Passed as a
// pointer to a device copy (bn_fin_desc packs one on the host).
struct BNFin {
    int mode = 0;                // 0 off, 1 forward batch statistics, 2 backward sums
    unsigned *arrive = nullptr;  // 9 zeroed words, left zeroed
    int64_t rows = 0;            // elements per channel
    int training = 1;            // backward: training-mode BN
    const float *gamma = nullptr, *beta = nullptr;
    float *mean = nullptr, *invstd = nullptr;  // forward: written; backward: read
    float *run_mean = nullptr, *run_var = nullptr;
    int64_t *num_batches = nullptr;
    float momentum = 0.f, eps = 0.f;
    float *coef = nullptr;                      // forward [scale; shift] (2C), backward (3C)
    float *dgamma = nullptr, *dbeta = nullptr;  // backward
};
struct EpiArgs {
    // device-resident descriptor (a kernel-argument copy of BNFin costs every statistics kernel
    // ~25 spilled SGPRs: the compiler loads all kernel arguments up front)
    const BNFin *fin = nullptr;
    const uint8_t *amask = nullptr;  // kEpiAccMask: ReLU mask of `old`, one byte per 8 channels
    const uint16_t *bias = nullptr;  // kEpiBiasRelu / kEpiBias: bf16 [K]
    double *stats = nullptr;         // kStatSlots x [2][K] f64 (zeroed; consumed + re-zeroed by the BN)
    const uint16_t *bx = nullptr;    // bwd: the BN's input x, same [M, K] layout as the output
    const float *fcoef = nullptr;    // bwd coef: forward [scale(K); shift(K)]
    const uint8_t *bmask = nullptr;  // bwd bits: ReLU mask, one byte per 8 channels
};
void launch_conv(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout, int ks,
                 int stride, const EpiArgs &ea, int epi, hipStream_t s, int variant = -1);
// kEpiAccEven (with kEpiAccum): accumulate only at pixels with even (h, w) -- the only ones a
// stride-2 1x1 data gradient wrote (launch_conv_dgrad_s2) -- and plain-store the others.
// Data gradient of a stride-2 KS x KS (KS = 1 pad 0 | 3 pad 1) convolution with an even input
// (H = 2*OH, W = 2*OW): dy [N, OH, OW, Cout] -> dx [N, 2OH, 2OW, Cin], wt = the flipped weight
// [Cin][KS*KS][Cout] (conv_flip_weight).  KS = 3: four parity-phase implicit GEMMs (1, 2, 2 and
// 4 taps) write every dx pixel once (epi: 0 or kEpiBwdCoef/kEpiBwdBits -- BN backward sums
// over dx, as launch_conv).  KS = 1: only the even pixels are written (the rest is left for a
// kEpiAccEven stride-1 data gradient into the same dx).
// DH / DW (ks = 3): any dx size with padding `pad` (0 or 1) -- e.g. Inception's 3x3/s2/p0 on odd
// inputs (25 -> 12); <= 0 = the even input 2OH x 2OW.  Cin / Cout multiples of 8.
void launch_conv_dgrad_s2(const uint16_t *dy, const uint16_t *wt, uint16_t *dx, int N, int OH, int OW, int Cout,
                          int Cin, int ks, const EpiArgs &ea, int epi, hipStream_t s, int variant = -1, int DH = 0,
                          int DW = 0, int pad = 1);
// KH x KW window with zero padding (ph, pw), stride 1|2 (Inception-v3's 1x1, 3x3 pad 0|1, 1x7,
// 7x1, 1x3, 3x1, 5x5): the same implicit GEMM, K = KH*KW*Cin tap-major; epilogue none or
// kEpiFwdStats.  Cin, Cout multiples of 64.
// Linear layer y[M, N] = x[M, K] w[N, K]^T (+ epilogue) on the same MFMA kernel (a 1x1 conv over
// M "pixels"): epi 0, kEpiBias, kEpiGeluGrad, kEpiAccum (y += product).  K, N % 64.
bool gemm_supported(int M, int K, int N);
void launch_gemm(const uint16_t *x, const uint16_t *w, uint16_t *y, int M, int K, int N, const EpiArgs &ea, int epi,
                 hipStream_t s, int variant = -1);
bool conv_rect_supported(int Cin, int Cout, int kh, int kw, int stride);
void launch_conv_rect(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout,
                      int kh, int kw, int ph, int pw, int stride, const EpiArgs &ea, int epi, hipStream_t s);
// Multi-tensor flip (one launch for a whole model's conv weights).
struct FlipTable {
    static constexpr int kMax = 64;
    int n = 0;
    const uint16_t *src[kMax];
    uint16_t *dst[kMax];
    int cout[kMax], cin[kMax], taps[kMax];
    int64_t start[kMax + 1];
    int tstart[kMax + 1];  // 64x64 transpose tiles (filled by launch_conv_flip_multi)
};
void launch_conv_flip_multi(const FlipTable &tab, hipStream_t s);
// wt[ci,kh,kw,co] = w[co,KS-1-kh,KS-1-kw,ci]: stride-1 data gradient = conv(dy, wt).
void launch_conv_flip_weight(const uint16_t *w, uint16_t *wt, int Cout, int Cin, int ks, hipStream_t s);
// Any KH x KW window: the flattened tap index is reversed (taps = KH*KW).
void launch_conv_flip_weight_taps(const uint16_t *w, uint16_t *wt, int Cout, int Cin, int taps, hipStream_t s);
// wt[ci,kh,kw,co] = w[co,2-kh,2-kw,ci]: stride-1 data gradient = conv3x3(dy, wt).
void launch_conv3x3_flip_weight(const uint16_t *w, uint16_t *wt, int Cout, int Cin, hipStream_t s);

// Weight gradient of the KS x KS (pad (KS-1)/2, stride 1|2) NHWC convolution as a split-K
// MFMA GEMM (conv_wgrad.hip): dw[co, kh, kw, ci] = sum_p dy[p, co] * x[pix(p, kh, kw), ci].
// dw: bf16 (out_f32 = 0) or f32 (out_f32 = 1), [Cout][KS*KS][Cin]; accumulate: dw += result.
// part: f32 workspace of conv_wgrad_workspace(...) floats (unused when that is 0).
struct WgradPlan {
    int variant = 0;  // tile choice
    int splits = 1;   // K (pixel) splits
    int kps = 0;      // K-steps per split
    int64_t ws_floats = 0;
};
bool conv_wgrad_supported(int Cin, int Cout, int ks, int stride);
// output pixels (N*OH*OW) one launch of the default plan handles
int64_t conv_wgrad_max_pixels(int N, int H, int W, int Cin, int Cout, int ks, int stride);
WgradPlan conv_wgrad_plan(int N, int H, int W, int Cin, int Cout, int ks, int stride, int variant = -1,
                          int splits = -1);
void launch_conv_wgrad(const uint16_t *dy, const uint16_t *x, void *dw, float *part, int N, int H, int W, int Cin,
                       int Cout, int ks, int stride, const WgradPlan &plan, bool out_f32, bool accumulate,
                       hipStream_t s, bool atomics = true);
// Any KH x KW window with zero padding (ph, pw), stride 1|2, Cin / Cout multiples of 8
// (Inception-v3's windows and channel counts): same kernel, runtime window, zero-padded tiles.
bool conv_wgrad_rect_supported(int Cin, int Cout, int kh, int kw, int stride);
// variant 6 (stride 1, multi-tap): the row-image kernel (all taps of a workgroup share one staged
// input image per 64-pixel segment), else -1 = the tap-tiled split-K kernel.
WgradPlan conv_wgrad_rect_plan(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int stride,
                               int variant = -1);
// the row-image variant for a stride-1 multi-tap shape (6, or 8 / 11 / 12: see conv_wgrad.hip kRowsEx);
// conv_wgrad_rect(..., variant = 13) runs it
int conv_wgrad_rows_rect_auto(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw, int stride);
bool conv_wgrad_rows_rect_supported(int N, int H, int W, int Cin, int Cout, int kh, int kw, int ph, int pw,
                                    int stride);
void launch_conv_wgrad_rect(const uint16_t *dy, const uint16_t *x, void *dw, float *part, int N, int H, int W,
                            int Cin, int Cout, int kh, int kw, int ph, int pw, int stride, const WgradPlan &plan,
                            bool out_f32, bool accumulate, hipStream_t s);
int conv_wgrad_variants();

// ResNet stem: 7x7 stride-2 pad-3 convolution, 3 -> 64 channels, NHWC bf16 (stem.hip).
// x4 = input padded to 4 channels; wp = weights packed [64][7 kh][8 kw][4 c] (zero padded).
// stats (optional): kStatSlots x [2][64] f64 per-channel sum / sum of squares of the output.
void launch_stem_pad4(const uint16_t *x, uint16_t *x4, int64_t npix, hipStream_t s);
void launch_stem_pad4_f32(const float *x, uint16_t *x4, int64_t npix, hipStream_t s);  // + cast to bf16
void launch_stem_pack_weight(const uint16_t *w, uint16_t *wp, hipStream_t s);
int stem_out(int h);
// Small image stem (stem3.hip): KH x KW <= 4 x 4 window, any stride / padding, 3 -> 32 channels (Inception's
// Conv2d_1a); x = the NHWC 3-channel image (f32 or bf16), wp = stem3 packed weights [32][64]; stats: the BN's
// f64 slots [slots][2][32].
int stem3_out(int h, int k, int stride, int pad);
void launch_stem3_pack_weight(const uint16_t *w, uint16_t *wp, int KH, int KW, hipStream_t s);
void launch_stem3_forward(const void *x, bool x_f32, const uint16_t *wp, uint16_t *y, double *stats, int N, int H,
                          int W, int KH, int KW, int stride, int ph, int pw, hipStream_t s);
int stem3_wgrad_blocks(int N, int H, int W, int KH, int KW, int stride, int ph, int pw);
int64_t stem3_wgrad_workspace(int N, int H, int W, int KH, int KW, int stride, int ph, int pw);  // floats
// dw [32][KH][KW][3] (channels_last [32, 3, KH, KW]), f32 or bf16; deterministic
void launch_stem3_wgrad(const uint16_t *dy, const void *x, bool x_f32, void *dw, bool out_f32, float *part, int N,
                        int H, int W, int KH, int KW, int stride, int ph, int pw, hipStream_t s);
void launch_stem_forward(const uint16_t *x4, const uint16_t *wp, uint16_t *y, double *stats, int N, int H, int W,
                         hipStream_t s);
// dw [64][7][7][3] bf16; part: stem_wgrad_workspace(...) floats.
int stem_wgrad_splits(int N, int H, int W);
int64_t stem_wgrad_workspace(int N, int H, int W, int splits);
// The stem weight gradient with the dy operand formed while staging from the stem's BN + ReLU +
// MaxPool backward (stem.hip BNP): y = the conv output (BN input), dyp / arg = the pooled gradient and
// window argmax, fcoef = forward [scale; shift], bcoef = bn_bwd_finalize's [k1; k2; k3] -- the BN input
// gradient is never materialised.  Row-kernel shapes only (stem_wgrad_bnp_supported).
bool stem_wgrad_bnp_supported(int N, int H, int W);
void launch_stem_wgrad_bnp(const uint16_t *y, const uint16_t *x4, uint16_t *dw, float *part, int N, int H, int W,
                           int splits, const uint16_t *dyp, const uint8_t *arg, const float *fcoef,
                           const float *bcoef, hipStream_t s);
void launch_stem_wgrad(const uint16_t *dy, const uint16_t *x4, uint16_t *dw, float *part, int N, int H, int W,
                       int splits, hipStream_t s);

// Fused NHWC batch-norm(+residual)(+ReLU), bf16 activations, f32 statistics
// (see bn.hip).  x/y/res/dy/dx/dres are [rows, C] bf16 with C contiguous.
struct BNShape {
    int64_t rows;  // N*H*W
    int channels;
};
bool bn_supported_channels(int C);
int bn_num_chunks(BNShape sh);  // partial scratch = 2 * nchunks * C floats
// Training: batch stats -> mean/invstd, running stats update, coef = [scale; shift]
// (2C floats), y = act(x*scale + shift [+ res]).  Eval: running stats.
// With res && relu, mask (rows*C/8 bytes) receives the ReLU bits for the backward.
// num_batches (optional, int64 on device) is incremented in training mode.
// Batched sums-finalize of up to kBnFinMax BNs (the f64 slotted sums of their producing convs): mean,
// invstd, running stats, coef = [scale; shift], num_batches += 1, slots re-zeroed -- one launch.
struct BnFinDesc {
    double *sums;
    const float *gamma, *beta;
    float *mean, *invstd, *run_mean, *run_var, *coef;
    int64_t *nbt;
    int64_t rows;
    int C;
    float momentum, eps;
};
constexpr int kBnFinMax = 8;
struct BnFinBatch {
    BnFinDesc d[kBnFinMax];
    int n;
};
void launch_bn_sums_finalize_multi(const BnFinBatch &b, hipStream_t s);
// Batched backward finalize (statistics path: the reduce pass's partials) of up to kBnFinMax training BNs.
struct BnBwdFinDesc {
    const float *partial;
    int nchunks, C;
    int64_t rows;
    const float *gamma, *mean, *invstd;
    float *dgamma, *dbeta, *coef;
};
struct BnBwdFinBatch {
    BnBwdFinDesc d[kBnFinMax];
    int n;
};
void launch_bn_bwd_finalize_multi(const BnBwdFinBatch &b, hipStream_t s);

void launch_bn_forward(const uint16_t *x, const uint16_t *res, const float *gamma, const float *beta, uint16_t *y,
                       uint8_t *mask, BNShape sh, bool relu, bool training, float *run_mean, float *run_var,
                       float momentum, float eps, float *partial, float *mean, float *invstd, float *coef,
                       int64_t *num_batches, hipStream_t s, double *sums = nullptr, const float *res_coef = nullptr,
                       bool apply = true, int64_t y_ld = 0, bool prefinalized = false);
// (prefinalized: mean / invstd / coef were already written from `sums` by the producing conv's
// in-launch finalize (BNFin) -- no finalize launch here.
// (y_ld > 0: y is a channel slice of a wider NHWC tensor with that row stride (elements); BN+ReLU only.
// (sums: f64 [2C] batch sums from a conv epilogue -> no statistics pass; re-zeroed.
//  res_coef: the residual is res*res_coef[c] + res_coef[C+c] (another BN's input and
//  coefficients); apply = false: statistics / coefficients only, y untouched.)
// dz = dy * relu'(.)  -- from mask bits if given, else recomputed as x*fcoef[0:C] + fcoef[C:2C] > 0
// (fcoef = the forward's coef) ; dgamma/dbeta (f32) ; dx = k1*dz + k2*x + k3 ; dres = dz.
// coef scratch: 3C floats.
void launch_bn_backward(const uint16_t *dy, const uint16_t *x, const float *fcoef, const uint8_t *mask,
                        const float *mean, const float *invstd, const float *gamma, BNShape sh, bool relu,
                        bool training, float *partial, float *dgamma, float *dbeta, float *coef, uint16_t *dx,
                        uint16_t *dres, hipStream_t s, double *sums = nullptr, const uint16_t *dres_x = nullptr,
                        double *dres_sums = nullptr,
                        int64_t dy_ld = 0, bool prefinalized = false, int phase = 0);
// (dres_x / dres_sums: dres also feeds a second, ReLU-free BN with input dres_x -- its backward
//  sums go to dres_sums, zeroed f64 [slots][2][C])
// (sums: f64 kStatSlots x [sum dz; sum dz*x] from a conv epilogue -> no reduce pass; re-zeroed.)

// ResNet stem: y = maxpool3x3s2p1(relu(bn(x))), x = [N, H, W, C] (rows = N*H*W).
// arg receives the window argmax (0..8) per pooled element (bytes).
inline int pool_out(int h) { return (h + 2 - 3) / 2 + 1; }
bool bn_pool_supported(BNShape sh, int H, int W);
void launch_bn_pool_forward(const uint16_t *x, const float *gamma, const float *beta, uint16_t *yp, uint8_t *arg,
                            BNShape sh, int H, int W, bool training, float *run_mean, float *run_var, float momentum,
                            float eps, float *partial, float *mean, float *invstd, float *coef, int64_t *num_batches,
                            hipStream_t s, double *sums = nullptr, uint16_t *xarg = nullptr);
// xarg + sums (zeroed f64 [slots][2][C]): the BN sums come from the pooled map (exact identity,
// see bn_pool_bwd_sums_kernel) instead of the full-resolution reduce pass.
void launch_bn_pool_backward(const uint16_t *dyp, const uint8_t *arg, const uint16_t *x, const float *fcoef,
                             const float *mean, const float *invstd, const float *gamma, BNShape sh, int H, int W,
                             bool training, float *partial, float *dgamma, float *dbeta, float *coef, uint16_t *dx,
                             hipStream_t s, const uint16_t *xarg = nullptr, double *sums = nullptr, bool apply = true);

// Conv bias (+ ReLU) on NHWC bf16 [rows, C] (bias_act.hip): forward in place; backward
// dz = dy * (y > 0) (relu) and dbias[c] = sum over rows (f32, deterministic: per-block partials
// [bias_act_backward_blocks(rows, C), C] f32 then a fixed-order column sum; no memset, no atomics).
bool bias_act_supported(int C);
void launch_bias_act_forward(uint16_t *y, const float *bias, int64_t rows, int C, bool relu, hipStream_t s);
int bias_act_backward_blocks(int64_t rows, int C);
void launch_bias_act_backward(const uint16_t *dy, const uint16_t *y, uint16_t *dz, float *dbias, float *partial,
                              int64_t rows, int C, bool relu, hipStream_t s);

// 2x2 / stride-2 max-pool, NHWC bf16, C % 8 == 0, even H and W (pool.hip); backward
// recomputes the window argmax from x and writes every dx element once.
void launch_maxpool2x2_forward(const uint16_t *x, uint16_t *y, int64_t N, int H, int W, int C, hipStream_t s);
// 3x3 / stride-2 / pad (0 or 1) max-pool with a byte argmax per element, gather backward;
// 3x3 / stride-1 / pad-1 average pool (count_include_pad; its gradient is the same stencil)
int maxpool3s2_out(int h, int pad);
void launch_maxpool3s2_forward(const uint16_t *x, uint16_t *y, uint8_t *arg, int64_t N, int H, int W, int C, int pad,
                               hipStream_t s);
void launch_maxpool3s2_backward(const uint16_t *dy, const uint8_t *arg, uint16_t *dx, int64_t N, int H, int W, int C,
                                int pad, hipStream_t s);
void launch_avgpool3s1(const uint16_t *x, uint16_t *y, int64_t N, int H, int W, int C, hipStream_t s);
// Global average pool over the H*W pixels of an NHWC bf16 tensor (C % 8 == 0): y [N, C];
// backward dx[n, p, c] = dy[n, c] / HW.
void launch_global_avgpool_forward(const uint16_t *x, uint16_t *y, int64_t N, int HW, int C, hipStream_t s);
void launch_global_avgpool_backward(const uint16_t *dy, uint16_t *dx, int64_t N, int HW, int C, hipStream_t s);

// (p > 0: dropout on the residual input r with a hashed keep mask of (seed, element); the
// backward then also writes dr, the dropped residual's gradient.)
// Fused residual-add + LayerNorm over rows of D (layernorm.hip): bf16 x, r (optional), y, s
// (= x + r, saved for backward), f32 gamma/beta/mean/rstd; backward -> ds (bf16) and
// dgamma/dbeta (f32) through [blocks][2][D] f32 partials.
bool layernorm_supported(int D);
int layernorm_bwd_blocks(int64_t rows);
void launch_layernorm_forward(const uint16_t *x, const uint16_t *r, const float *gamma, const float *beta, uint16_t *y,
                              uint16_t *s, float *mean, float *rstd, int64_t rows, int D, float eps, hipStream_t st,
                              float p = 0.f, uint32_t seed = 0);
void launch_layernorm_backward(const uint16_t *dy, const uint16_t *s, const float *gamma, const float *mean,
                               const float *rstd, uint16_t *ds, float *partial, float *dgamma, float *dbeta,
                               int64_t rows, int D, hipStream_t st,
                               uint16_t *dr = nullptr, float p = 0.f, uint32_t seed = 0, float *rb_f32 = nullptr,
                               uint16_t *rb_bf16 = nullptr);  // rb_*: the residual input's column sums (f32 or bf16)
// gate_stats != nullptr: x is a ReLU output, dx = that ReLU's input gradient (window max > 0 only)
// and the per-channel sums of dx go to gate_stats[slot][0][C] (kStatSlots x 2 x C f64, zeroed)
void launch_maxpool2x2_backward(const uint16_t *x, const uint16_t *dy, uint16_t *dx, int64_t N, int H, int W, int C,
                                hipStream_t s, double *gate_stats = nullptr);

// Fused self-attention (attention.hip): qkv [B, S, 3, H, 64] bf16 (the fused projection's
// output), out [B, S, H*64] bf16, lse [B, H, S] f32; dropout p_drop on the probabilities from a
// counter hash of (seed, b*H + h, query, key); S = 64 or 128, head dim 64, no mask.
bool attention_supported(int S, int head_dim);
void launch_attention_forward(const uint16_t *qkv, uint16_t *out, float *lse, int B, int S, int H, float scale,
                              uint32_t seed, float p_drop, hipStream_t s);
// dqkv [B, S, 3, H, 64] (every element written)
void launch_attention_backward(const uint16_t *qkv, const uint16_t *out, const float *lse, const uint16_t *dout,
                               uint16_t *dqkv, int B, int S, int H, float scale, uint32_t seed, float p_drop,
                               hipStream_t s);

}  // namespace kfk
