// Rectangular-window convolutions (Inception-v3's 1x7 / 7x1 / 1x3 / 3x1 / 5x5) on the MFMA conv kernel.
// (the kernel template and its launch helpers: conv_kernel.hpp)
#include "conv_kernel.hpp"

namespace kfk {

namespace {

// Rectangular windows (Inception-v3): plain, BN-statistics, accumulate and/or BN-backward-sums
// (the gradient of a BN+ReLU output: sum dz, sum dz*x into the stats slots) epilogue, 256x128 / 8 waves when
// Cout % 128 == 0, else 256x64.
template <int KS>
void launch_rect_t(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                   hipStream_t s) {
    constexpr int A = kEpiAccum, C = kEpiBwdCoef;
    if (g.K <= 32) {  // narrow outputs (Inception's 32-channel stem / pool branch): 256x32 tiles
        switch (epi) {
        case 0: launch_epi<KS, 4, 1, 2, 0, 4, 2>(x, w, y, g, ea, s); break;
        case kEpiFwdStats: launch_epi<KS, 4, 1, 2, kEpiFwdStats, 4, 2>(x, w, y, g, ea, s); break;
        case A: launch_epi<KS, 4, 1, 2, A, 4, 2>(x, w, y, g, ea, s); break;
        case C: launch_epi<KS, 4, 1, 2, C, 4, 2>(x, w, y, g, ea, s); break;
        case A | C: launch_epi<KS, 4, 1, 2, A | C, 4, 2>(x, w, y, g, ea, s); break;
        default: throw std::invalid_argument("conv_rect: unsupported epilogue");
        }
    } else if (g.K % 128 == 0) {
        switch (epi) {
        case 0: launch_epi<KS, 4, 2, 3, 0>(x, w, y, g, ea, s); break;
        case kEpiFwdStats: launch_epi<KS, 4, 2, 3, kEpiFwdStats>(x, w, y, g, ea, s); break;
        case A: launch_epi<KS, 4, 2, 3, A>(x, w, y, g, ea, s); break;
        case C: launch_epi<KS, 4, 2, 3, C>(x, w, y, g, ea, s); break;
        case A | C: launch_epi<KS, 4, 2, 3, A | C>(x, w, y, g, ea, s); break;
        default: throw std::invalid_argument("conv_rect: unsupported epilogue");
        }
    } else {
        switch (epi) {
        case 0: launch_epi<KS, 4, 1, 2, 0>(x, w, y, g, ea, s); break;
        case kEpiFwdStats: launch_epi<KS, 4, 1, 2, kEpiFwdStats>(x, w, y, g, ea, s); break;
        case A: launch_epi<KS, 4, 1, 2, A>(x, w, y, g, ea, s); break;
        case C: launch_epi<KS, 4, 1, 2, C>(x, w, y, g, ea, s); break;
        case A | C: launch_epi<KS, 4, 1, 2, A | C>(x, w, y, g, ea, s); break;
        default: throw std::invalid_argument("conv_rect: unsupported epilogue");
        }
    }
}


}  // namespace

bool conv_rect_supported(int Cin, int Cout, int kh, int kw, int stride) {
    // channel counts: multiples of 8 (16-byte chunks); the last K-step / N-tile is zero-padded
    if (Cin % 8 || Cout % 8 || Cin < 16 || Cout < 16 || !(stride == 1 || stride == 2)) return false;
    return (kh == 1 && kw == 1) || (kh == 3 && kw == 3) || (kh == 1 && kw == 7) || (kh == 7 && kw == 1) ||
           (kh == 1 && kw == 3) || (kh == 3 && kw == 1) || (kh == 5 && kw == 5);
}

void launch_conv_rect(const uint16_t *x, const uint16_t *w, uint16_t *y, int N, int H, int W, int Cin, int Cout,
                      int kh, int kw, int ph, int pw, int stride, const EpiArgs &ea, int epi, hipStream_t s) {
    if (!conv_rect_supported(Cin, Cout, kh, kw, stride)) throw std::invalid_argument("conv_rect: unsupported shape");
    Geo g;
    g.N = N, g.H = H, g.W = W, g.C = Cin, g.K = Cout, g.stride = stride;
    g.OH = (H + 2 * ph - kh) / stride + 1;
    g.OW = (W + 2 * pw - kw) / stride + 1;
    g.M = N * g.OH * g.OW;
    g.mtiles = g.ntiles = 0;
    g.wtaps = kh * kw, g.tapmap = -1, g.scat = 0, g.pr = g.pc = 0, g.dh = g.dw = 0;
    g.stagger = conv_stagger();
    g.prio = conv_prio();
    g.ph = ph, g.pw = pw;
    if (kh == 1 && kw == 1) {
        launch_conv_k1(x, w, y, g, ea, epi, s, -1);
        return;
    }
    if (kh == 3 && kw == 3) {
        launch_conv_k3(x, w, y, g, ea, epi, s, -1);
        return;
    }
    if (kh == 1 && kw == 7) launch_rect_t<0x17>(x, w, y, g, ea, epi, s);
    else if (kh == 7 && kw == 1) launch_rect_t<0x71>(x, w, y, g, ea, epi, s);
    else if (kh == 1 && kw == 3) launch_rect_t<0x13>(x, w, y, g, ea, epi, s);
    else if (kh == 3 && kw == 1) launch_rect_t<0x31>(x, w, y, g, ea, epi, s);
    else launch_rect_t<0x55>(x, w, y, g, ea, epi, s);
}


}  // namespace kfk
