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
#include "conv_kernel.hpp"

namespace kfk {

namespace {


// w'[ci, kh, kw, co] = w[co, KS-1-kh, KS-1-kw, ci]  (the stride-1 data-gradient weights)
__global__ void conv_flip_kernel(const uint16_t *__restrict__ w, uint16_t *__restrict__ wt, int Cout, int Cin,
                                 int taps) {
    const int64_t n = static_cast<int64_t>(Cout) * taps * Cin;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int co = static_cast<int>(i % Cout);
        int64_t t = i / Cout;
        const int tap = static_cast<int>(t % taps);
        const int ci = static_cast<int>(t / taps);
        wt[i] = w[(static_cast<int64_t>(co) * taps + (taps - 1 - tap)) * Cin + ci];
    }
}

// The same flip as a tiled transpose: one block per (layer, tap, 64 co x 64 ci tile), rows of
// 64 ci read as 32-bit pairs and rows of 64 co written as pairs through a padded LDS tile, so
// both sides are coalesced (the element kernel above gathers with a Cin*taps read stride:
// 169 us for ResNet-50's 47 MB of conv weights).
__global__ __launch_bounds__(256) void conv_flip_tiled_kernel(FlipTable tab) {
    __shared__ uint16_t tile[64][66];
    const int b = blockIdx.x;
    int lo = 0, hi = tab.n - 1;  // last layer with tstart <= b
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (tab.tstart[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    const int Cout = tab.cout[lo], Cin = tab.cin[lo], taps = tab.taps[lo];
    const int tco_n = (Cout + 63) / 64, tci_n = (Cin + 63) / 64;
    int t = b - tab.tstart[lo];
    const int tap = t / (tco_n * tci_n);
    t -= tap * tco_n * tci_n;
    const int co0 = (t / tci_n) * 64, ci0 = (t % tci_n) * 64;
    const uint16_t *src = tab.src[lo];
    uint16_t *dst = tab.dst[lo];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 pairs x 8 rows per pass
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = ty + 8 * k, co = co0 + r, ci = ci0 + 2 * tx;
        if (co < Cout) {
            const uint16_t *p = src + (static_cast<int64_t>(co) * taps + tap) * Cin + ci;
            tile[r][2 * tx] = ci < Cin ? p[0] : 0;
            tile[r][2 * tx + 1] = ci + 1 < Cin ? p[1] : 0;
        }
    }
    __syncthreads();
    const int tap2 = taps - 1 - tap;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int r = ty + 8 * k, ci = ci0 + r, co = co0 + 2 * tx;
        if (ci < Cin) {
            uint16_t *q = dst + (static_cast<int64_t>(ci) * taps + tap2) * Cout + co;
            if (co < Cout) q[0] = tile[2 * tx][r];
            if (co + 1 < Cout) q[1] = tile[2 * tx + 1][r];
        }
    }
}

}  // namespace

void launch_conv_flip_multi(const FlipTable &tab_in, hipStream_t s) {
    if (tab_in.n == 0 || tab_in.start[tab_in.n] == 0) return;
    FlipTable tab = tab_in;
    tab.tstart[0] = 0;
    for (int k = 0; k < tab.n; ++k)
        tab.tstart[k + 1] = tab.tstart[k] + tab.taps[k] * ((tab.cout[k] + 63) / 64) * ((tab.cin[k] + 63) / 64);
    conv_flip_tiled_kernel<<<tab.tstart[tab.n], 256, 0, s>>>(tab);
}

// Channel / stride predicates only: the caller also checks that x and w stay below 2 GiB
// (buffer-resource staging, check_buf_extent; kungfu_amd._lib.buf_ok on the Python side).
bool conv3x3_supported(int Cin, int Cout, int stride) {
    return Cin % 64 == 0 && Cout % 64 == 0 && (stride == 1 || stride == 2) && Cin >= 64;
}

bool conv_supported(int Cin, int Cout, int ks, int stride) {
    return (ks == 1 || ks == 3) && conv3x3_supported(Cin, Cout, stride);
}

// KUNGFU_CONV_TILE_RULES: 1 = the round-2 tile defaults, 2 (default) = the round-3 re-measured ones
// (ResNet-50 21.28-21.30 -> 21.12-21.17 ms/step same-box A/B, Inception-v3 neutral)
int conv_tile_rules() {
    static const int v = dev_knob("KUNGFU_CONV_TILE_RULES", 2);
    return v;
}

// KUNGFU_CONV_T224 (dev knob, default 1): 224x256 tiles for one- or two-round grids of 256x256 tiles
// (launch_ks); 0 = always 256x256
int conv_t224() {
    static const int v = dev_knob("KUNGFU_CONV_T224", 1);
    return v;
}

// Staggered staging issue in the 8-wave tiles: the two waves sharing a SIMD issue their LDS-DMA
// pieces in different phases of the K-step (one before its fragment reads, one between its MFMA
// clusters) instead of stalling on staging issue together.  ResNet-50 +0.8 % (21.43-21.49 ->
// 21.28-21.29 ms/step, same box), Inception-v3 neutral.
int conv_stagger() { return 1; }

// static s_setprio 1 for the upper wave half of the 8-wave tiles: measured neutral (r3), off
int conv_prio() { return 0; }

// 256-byte zero page for padding rows (global_load_lds needs a real address).
const void *zero_page() {
    static void *p = [] {
        void *q = nullptr;
        (void)hipMalloc(&q, 256);
        (void)hipMemset(q, 0, 256);
        return q;
    }();
    return p;
}

// Buffer-resource staging addresses x and w with 32-bit byte offsets below kBufOOB.
void check_buf_extent(const Geo &g) {
    if (KUNGFU_CONV_BUFLD && (static_cast<int64_t>(g.N) * g.H * g.W * g.C * 2 >= kBufOOB ||
                              static_cast<int64_t>(g.K) * (g.wtaps > 0 ? g.wtaps : 1) * g.C * 2 >= kBufOOB))
        throw std::invalid_argument("conv: input or weight of 2 GiB or more (buffer-resource staging)");
}


int conv3x3_variants() { return 12; }

void launch_conv(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout, int ks,
                 int stride, const EpiArgs &ea, int epi, hipStream_t s, int variant) {
    Geo g;
    const int pad = (ks - 1) / 2;
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout, g.stride = stride;
    g.OH = (H + 2 * pad - ks) / stride + 1;
    g.OW = (W + 2 * pad - ks) / stride + 1;
    g.M = N * g.OH * g.OW;
    g.mtiles = g.ntiles = 0;
    g.wtaps = ks * ks, g.tapmap = -1, g.scat = 0, g.pr = g.pc = 0, g.dh = g.dw = 0;
    g.stagger = conv_stagger();
    g.prio = conv_prio();
    g.ph = g.pw = pad;
    if (ks == 1) launch_conv_k1(x, w, y, g, ea, epi, s, variant);
    else launch_conv_k3(x, w, y, g, ea, epi, s, variant);
}

// Rectangular windows (Inception-v3): plain, BN-statistics, accumulate and/or BN-backward-sums
// (the gradient of a BN+ReLU output: sum dz, sum dz*x into the stats slots) epilogue, 256x128 / 8 waves when
// Cout % 128 == 0, else 256x64.

void launch_conv3x3(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout,
                    int stride, hipStream_t s, int variant) {
    launch_conv(x, w, y, N, H, W, Cin, Cout, 3, stride, EpiArgs{}, 0, s, variant);
}

void launch_conv_flip_weight(const uint16_t *w, uint16_t *wt, int Cout, int Cin, int ks, hipStream_t s) {
    launch_conv_flip_weight_taps(w, wt, Cout, Cin, ks * ks, s);
}

void launch_conv_flip_weight_taps(const uint16_t *w, uint16_t *wt, int Cout, int Cin, int taps, hipStream_t s) {
    const int64_t n = static_cast<int64_t>(Cout) * taps * Cin;
    int grid = static_cast<int>((n + 255) / 256);
    if (grid > 4096) grid = 4096;
    conv_flip_kernel<<<grid, 256, 0, s>>>(w, wt, Cout, Cin, taps);
}

void launch_conv3x3_flip_weight(const uint16_t *w, uint16_t *wt, int Cout, int Cin, hipStream_t s) {
    launch_conv_flip_weight(w, wt, Cout, Cin, 3, s);
}


}  // namespace kfk
