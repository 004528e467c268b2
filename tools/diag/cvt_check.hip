// Compares gfx950's v_cvt_pk_bf16_f32 (common.hpp pack_bf16x2) with the integer round-to-nearest-even
// bit trick on 2^26 f32 patterns spread over the whole range plus edge cases (denormals, halfway values,
// +-0, inf, NaN, max finite): prints the mismatch count per class.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../csrc/kernels/common.hpp"
using namespace kfk;
__device__ __forceinline__ uint16_t soft_bf16(float f) {
    uint32_t u = __float_as_uint(f);
    u += 0x7fffu + ((u >> 16) & 1u);
    return static_cast<uint16_t>(u >> 16);
}
__global__ void cmp(const uint32_t *in, int n, unsigned long long *bad, uint32_t *first) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    const float a = __uint_as_float(in[2 * i]), b = __uint_as_float(in[2 * i + 1]);
    const uint32_t hw = pack_bf16x2(a, b);
    const uint32_t sw = soft_bf16(a) | (static_cast<uint32_t>(soft_bf16(b)) << 16);
    const uint32_t h1 = f32_to_bf16(a);
    const bool nan = (a != a) || (b != b);
    if (hw != sw || (h1 != (sw & 0xffff))) {
        atomicAdd(bad + (nan ? 1 : 0), 1ull);
        if (!nan) atomicCAS(first, 0u, in[2 * i]);
    }
}
int main() {
    const int n = 1 << 26;
    std::vector<uint32_t> h(n);
    uint64_t x = 88172645463325252ull;
    for (int i = 0; i < n; ++i) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; h[i] = static_cast<uint32_t>(x); }
    const uint32_t edge[] = {0u, 0x80000000u, 1u, 0x807fffffu, 0x007fffffu, 0x00008000u, 0x00018000u, 0x3f808000u,
                             0x3f818000u, 0x7f7fffffu, 0x7f800000u, 0xff800000u, 0x7fc00000u, 0x7fffffffu};
    for (int i = 0; i < 14; ++i) h[i] = edge[i];
    for (int i = 14; i < 1 << 20; ++i) h[i] &= 0x807fffffu;  // a million denormals
    uint32_t *d; unsigned long long *bad; uint32_t *first;
    hipMalloc(&d, 4ull * n); hipMalloc(&bad, 16); hipMalloc(&first, 4);
    hipMemcpy(d, h.data(), 4ull * n, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 16); hipMemset(first, 0, 4);
    cmp<<<n / 2 / 256, 256>>>(d, n, bad, first);
    unsigned long long hb[2]; uint32_t f;
    hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost); hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("mismatches: finite %llu, with NaN %llu (first finite mismatch 0x%08x)\n", hb[0], hb[1], f);
    return 0;
}
