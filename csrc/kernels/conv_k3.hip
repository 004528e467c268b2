// 3x3 (pad 1) convolutions on the MFMA implicit-GEMM kernel: every tile variant x fused epilogue instance.
// (the kernel template and its launch helpers: conv_kernel.hpp)
#include "conv_kernel.hpp"

namespace kfk {

void launch_conv_k3(const uint16_t *x, const uint16_t *w, uint16_t *y, Geo g, const EpiArgs &ea, int epi,
                    hipStream_t s, int variant) {
    launch_ks<3>(x, w, y, g, ea, epi, s, variant);
}

}  // namespace kfk
