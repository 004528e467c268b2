// Stride-2 data gradients as parity-phase implicit GEMMs on the MFMA conv kernel.
// (the kernel template and its launch helpers: conv_kernel.hpp)
#include "conv_kernel.hpp"

namespace kfk {

namespace {

// One parity phase of a stride-2 data gradient: the fused epilogues it needs (none, or the BN
// backward sums of the BN that produced the forward input), 256x128 tiles when Cin % 128 == 0.
template <int KS, int WM, int WN, int ST, int TM = 4, int TN = 4>
void launch_phase_t(const uint16_t *dy, const uint16_t *wt, uint16_t *dx, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s) {
    constexpr int C = kEpiBwdCoef, B = kEpiBwdBits;
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    if (g.K % 8 || g.C % 8) throw std::invalid_argument("conv_dgrad_s2: channel counts must be multiples of 8");
    g.mtiles = (g.M + BM - 1) / BM;
    g.ntiles = (g.K + BN - 1) / BN;  // a partial last N tile reads zero B rows, stores its valid columns
    const int grid = g.mtiles * g.ntiles;
    check_buf_extent(g);
    const uint16_t *z = reinterpret_cast<const uint16_t *>(zero_page());
    EpiArgs e2 = ea;
    e2.fin = nullptr;  // one tile per workgroup: the finalize runs as a launch of its own
    if (epi == 0) conv_kernel<KS, WM, WN, ST, 0, TM, TN><<<grid, 64 * WM * WN, 0, s>>>(dy, wt, dx, z, g, e2);
    else if (epi == C) conv_kernel<KS, WM, WN, ST, C, TM, TN><<<grid, 64 * WM * WN, 0, s>>>(dy, wt, dx, z, g, e2);
    else if (epi == B) conv_kernel<KS, WM, WN, ST, B, TM, TN><<<grid, 64 * WM * WN, 0, s>>>(dy, wt, dx, z, g, e2);
    else throw std::invalid_argument("conv_dgrad_s2: unsupported epilogue");
    if (ea.fin) bn_fin_desc_kernel<<<(g.K + 255) / 256, 256, 0, s>>>(ea.fin, ea.stats, g.K);
}

// Tile for the short-K phase GEMMs (variant >= 0 to override; tools/bench_dgrad_s2.py): 128x128
// / 4 waves for the large-M 3x3 phases (>= 1024 such tiles: two blocks per CU overlap one
// block's prologue/epilogue with the other's MFMAs), else 256x128 / 8 waves; 256x64 when
// Cin % 128 != 0.  (One grid holding all four phases, per-block tap count, measured 5-50 %
// slower than four launches.)
template <int KS>
void launch_phase(const uint16_t *dy, const uint16_t *wt, uint16_t *dx, Geo g, const EpiArgs &ea, int epi,
                  hipStream_t s, int v) {
    if (v < 0) {
        const int64_t t128 = ((static_cast<int64_t>(g.M) + 127) / 128) * (g.K / 128);
        v = g.K % 128 ? 2 : (KS != 1 && t128 >= 1024) ? 0 : 1;
    }
    switch (v) {
    case 0: if (g.K % 128 == 0) { launch_phase_t<KS, 2, 2, 2>(dy, wt, dx, g, ea, epi, s); break; }  // 128x128
            [[fallthrough]];
    case 5: launch_phase_t<KS, 2, 1, 2>(dy, wt, dx, g, ea, epi, s); break;                           // 128x64
    case 1: if (g.K % 128 == 0) { launch_phase_t<KS, 4, 2, 3>(dy, wt, dx, g, ea, epi, s); break; }  // 256x128
            [[fallthrough]];
    default: launch_phase_t<KS, 4, 1, 2>(dy, wt, dx, g, ea, epi, s); break;                         // 256x64
    }
}


}  // namespace

void launch_conv_dgrad_s2(const uint16_t *dy, const uint16_t *wt, uint16_t *dx, int N, int OH, int OW, int Cout,
                          int Cin, int ks, const EpiArgs &ea, int epi, hipStream_t s, int variant, int DH, int DW,
                          int pad) {
    // variant: -1 = default; else the tile variant (0 128x128, 1 256x128, 2 256x64, 5 128x64)
    const int tv = variant;
    if (DH <= 0) DH = 2 * OH;
    if (DW <= 0) DW = 2 * OW;
    Geo g;
    g.N = N, g.H = OH, g.W = OW, g.C = Cout, g.K = Cin, g.stride = 1;
    g.mtiles = g.ntiles = 0;
    g.wtaps = ks * ks, g.scat = 1;
    g.dh = DH, g.dw = DW;
    g.stagger = conv_stagger();
    g.prio = conv_prio();
    g.ph = g.pw = 0;
    if (ks == 1) {
        if (DH != 2 * OH || DW != 2 * OW || pad != 0) throw std::invalid_argument("conv_dgrad_s2: 1x1 needs an even input");
        g.OH = OH, g.OW = OW, g.M = N * OH * OW;
        g.tapmap = -1, g.pr = g.pc = 0;
        launch_phase<1>(dy, wt, dx, g, ea, epi, s, tv);
        return;
    }
    if (ks != 3 || (pad != 0 && pad != 1)) throw std::invalid_argument("conv_dgrad_s2: ks 3 needs pad 0 or 1");
    if ((DH + 2 * pad - 3) / 2 + 1 != OH || (DW + 2 * pad - 3) / 2 + 1 != OW)
        throw std::invalid_argument("conv_dgrad_s2: dy / dx sizes do not match a stride-2 3x3 convolution");
    // dx row ih = 2a + pr sees the forward taps with 2 oh + kh = ih + pad: q = pr + pad odd -> kh = 1 at
    // dy row a (one tap); q even -> kh = 2 at row a + q/2 - 1 and kh = 0 at row a + q/2 (two taps, the
    // window starting q/2 - 1 rows past a, i.e. zero padding 1 - q/2).  Same for columns.  Flipped-weight
    // tap index = 2 - kh; every dx pixel is written by exactly one phase.
    if (ea.fin && (DH < 2 || DW < 2)) throw std::invalid_argument("conv_dgrad_s2: in-launch finalize needs dx >= 2x2");
    // the BN-backward sums accumulate over all four phase launches: only the last one finalizes
    EpiArgs ea_early = ea;
    ea_early.fin = nullptr;
    for (int pr = 0; pr < 2; ++pr)
        for (int pc = 0; pc < 2; ++pc) {
            const EpiArgs &eap = (pr == 1 && pc == 1) ? ea : ea_early;
            const int qr = pr + pad, qc = pc + pad;
            const int nh = (qr & 1) ? 1 : 2, nw = (qc & 1) ? 1 : 2;
            const int PH = (DH - pr + 1) / 2, PW = (DW - pc + 1) / 2;
            if (PH <= 0 || PW <= 0) continue;
            int map = 0;
            for (int th = 0; th < nh; ++th)
                for (int tw = 0; tw < nw; ++tw) {
                    const int rh = nh == 1 ? 1 : (th == 0 ? 0 : 2), rw = nw == 1 ? 1 : (tw == 0 ? 0 : 2);
                    map |= (rh * 3 + rw) << (4 * (th * nw + tw));
                }
            g.tapmap = map, g.pr = pr, g.pc = pc;
            g.OH = PH, g.OW = PW, g.M = N * PH * PW;
            g.ph = nh == 1 ? 0 : 1 - qr / 2;
            g.pw = nw == 1 ? 0 : 1 - qc / 2;
            if (nh == 1 && nw == 1) launch_phase<1>(dy, wt, dx, g, eap, epi, s, tv);
            else if (nh == 1) launch_phase<0x12>(dy, wt, dx, g, eap, epi, s, tv);
            else if (nw == 1) launch_phase<0x21>(dy, wt, dx, g, eap, epi, s, tv);
            else launch_phase<0x22>(dy, wt, dx, g, eap, epi, s, tv);
        }
}


}  // namespace kfk
