// 3x3 (pad 1) convolutions on the MFMA implicit-GEMM kernels: every tile variant x fused epilogue
// instance of conv_kernel, and the row-image kernel for stride 1 (conv_rows_kernel).
// (the kernel templates and their launch helpers: conv_kernel.hpp)
#include "conv_kernel.hpp"

namespace kfk {

namespace {

// Row-image variants (tile BM x BN, waves, B ring depth, image rows, image buffers):
//   20: 512 x 64, 8 waves, B ring 4, 768-row image, 1 buffer (Cin = 64: one chunk) -- 96 + 32 KB
//   21: 256 x 128, 8 waves, B ring 3, 448-row image x 2 -- 112 + 48 KB
//   22: 128 x 128, 4 waves, B ring 4, 288-row image x 2 -- 72 + 64 KB
//   23: 256 x 64, 4 waves, B ring 4, 512-row image, 1 buffer (Cin = 64) -- 64 + 32 KB
//   24: 256 x 64, 4 waves, B ring 2, 512-row image, 1 buffer (Cin = 64) -- 64 + 16 KB: two workgroups per CU
//   25: 256 x 64, 8 waves of 32 x 64, B ring 2, 512-row image, 1 buffer (Cin = 64) -- 80 KB: two per CU
bool launch_rows(const uint16_t *x, const uint16_t *w, uint16_t *y, const Geo &g, const EpiArgs &ea, int epi,
                 hipStream_t s, int variant) {
    switch (variant) {
    case 20: return launch_rows_variant<8, 1, 4, 4, 4, 768, 1>(x, w, y, g, ea, epi, s);
    case 21: return launch_rows_variant<4, 2, 3, 4, 4, 448, 2>(x, w, y, g, ea, epi, s);
    case 22: return launch_rows_variant<2, 2, 4, 4, 4, 288, 2>(x, w, y, g, ea, epi, s);
    case 23: return launch_rows_variant<4, 1, 4, 4, 4, 512, 1>(x, w, y, g, ea, epi, s);
    case 24: return launch_rows_variant<4, 1, 2, 4, 4, 512, 1>(x, w, y, g, ea, epi, s);
    case 25: return launch_rows_variant<8, 1, 2, 2, 4, 512, 1>(x, w, y, g, ea, epi, s);
    default: return false;
    }
}

// KUNGFU_CONV_ROWS (dev knob, default 1): stride-1 3x3 convs with Cin = Cout = 64 (ResNet-50 layer 1)
// on the row-image kernel.  Isolated (batch 256, 56 x 56): forward + BN statistics 112 -> 97 us, data
// gradient + BN-backward sums 147 -> 121-131 us; ResNet-50 step 20.24-20.27 -> 20.17-20.19 ms, same
// box, bit-identical loss (one 64-channel chunk: the same summation order).  The 28 x 28 and smaller
// layers measured no faster on it (r6t22): tap-wise there.
int conv_rows_default() {
    static const int v = dev_knob("KUNGFU_CONV_ROWS", 1);
    return v;
}

}  // namespace

void launch_conv_k3(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s, int variant) {
    const bool rows_ok = g.stride == 1 && g.ph == 1 && g.pw == 1 && g.tapmap < 0 && !g.scat;
    if (variant >= 20) {
        check_buf_extent(g);
        if (!rows_ok || !launch_rows(x, w, y, g, ea, epi, s, variant))
            throw std::invalid_argument("conv: row-image variant unsupported for this shape / epilogue");
        return;
    }
    if (variant < 0 && rows_ok && conv_rows_default()) {
        check_buf_extent(g);
        const int v = g.C == 64 && g.K == 64 ? 24 : -1;  // 28 x 28 and smaller: v21 / v22 measured no faster (r6t22)
        if (v > 0 && launch_rows(x, w, y, g, ea, epi, s, v)) return;
    }
    launch_ks<3>(x, w, y, g, ea, epi, s, variant);
}

}  // namespace kfk
