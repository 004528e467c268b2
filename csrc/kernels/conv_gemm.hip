// Linear layers on the MFMA implicit-GEMM conv kernel (H = W = 1) with the bias / GELU epilogues.
// (the kernel template and its launch helpers: conv_kernel.hpp)
#include "conv_kernel.hpp"

namespace kfk {

namespace {

// Linear layers: M tokens x K in-features -> N out-features, the 1x1 case of the kernel above
// (H = W = 1) with the bias / GELU / GELU-gradient / accumulate epilogues.
template <int WM, int WN, int ST, int TM, int TN>
void launch_gemm_t(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                   hipStream_t s) {
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    if (g.K % BN) throw std::invalid_argument("gemm: out-features not a multiple of the tile");
    g.mtiles = (g.M + BM - 1) / BM;
    g.ntiles = g.K / BN;
    check_buf_extent(g);
    const dim3 grid(g.mtiles * g.ntiles), block(64 * WM * WN);
    const uint16_t *z = reinterpret_cast<const uint16_t *>(zero_page());
    switch (epi) {
    case 0: conv_kernel<1, WM, WN, ST, 0, TM, TN><<<grid, block, 0, s>>>(x, w, y, z, g, ea); break;
    case kEpiBias: conv_kernel<1, WM, WN, ST, kEpiBias, TM, TN><<<grid, block, 0, s>>>(x, w, y, z, g, ea); break;
    case kEpiGeluGrad:
        conv_kernel<1, WM, WN, ST, kEpiGeluGrad, TM, TN><<<grid, block, 0, s>>>(x, w, y, z, g, ea);
        break;
    case kEpiAccum: conv_kernel<1, WM, WN, ST, kEpiAccum, TM, TN><<<grid, block, 0, s>>>(x, w, y, z, g, ea); break;
    default: throw std::invalid_argument("gemm: unsupported epilogue");
    }
}


}  // namespace

bool gemm_supported(int M, int K, int N) {
    // x (M x K) and the (flipped) weight are staged through buffer resources: below 2 GiB of bf16
    return M > 0 && K >= 64 && K % 64 == 0 && N % 64 == 0 && N >= 64 &&
           static_cast<int64_t>(M) * (K > N ? K : N) < (int64_t(1) << 30);
}

void launch_gemm(const uint16_t *x, const uint16_t *w, uint16_t *y, int M, int K, int N, const EpiArgs &ea, int epi,
                 hipStream_t s, int variant) {
    if (!gemm_supported(M, K, N)) throw std::invalid_argument("gemm: unsupported shape");
    Geo g;
    g.N = M, g.H = g.W = 1, g.C = K, g.K = N, g.stride = 1;
    g.OH = g.OW = 1, g.M = M;
    g.mtiles = g.ntiles = 0;
    g.wtaps = 1, g.tapmap = -1, g.scat = 0, g.pr = g.pc = 0, g.ph = g.pw = 0, g.dh = g.dw = 0;
    g.stagger = conv_stagger();
    g.prio = conv_prio();
    if (variant < 0) {
        // enough 256x256 tiles to fill the chip twice, else 256x128, else 128x128 (or 128x64)
        const int64_t t256 = N % 256 ? 0 : ((M + 255) / 256) * (N / 256);
        const int64_t t128 = N % 128 ? 0 : ((M + 255) / 256) * (N / 128);
        variant = t256 >= 512 ? 0 : t128 >= 512 ? 1 : 2;
    }
    switch (variant) {
    case 0: if (N % 256 == 0) { launch_gemm_t<4, 2, 2, 4, 8>(x, w, y, g, ea, epi, s); break; }  // 256x256, 8 waves
            [[fallthrough]];
    case 1: if (N % 128 == 0) { launch_gemm_t<4, 2, 3, 4, 4>(x, w, y, g, ea, epi, s); break; }  // 256x128, 8 waves
            [[fallthrough]];
    case 2: if (N % 128 == 0) { launch_gemm_t<2, 2, 2, 4, 4>(x, w, y, g, ea, epi, s); break; }  // 128x128, 4 waves
            launch_gemm_t<2, 1, 2, 4, 4>(x, w, y, g, ea, epi, s); break;                       // 128x64
    default: if (N % 256) throw std::invalid_argument("gemm variant 3: N % 256");
            launch_gemm_t<2, 4, 2, 8, 4>(x, w, y, g, ea, epi, s); break;                       // 256x256, 128x64 waves
    }
}


}  // namespace kfk
