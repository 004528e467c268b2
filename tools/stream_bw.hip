// Streaming bandwidth of the BN-apply access pattern (x, res -> y, 1-byte mask per 16 B) on
// MI355X: plain vs non-temporal loads/stores, unroll depth and grid size.  Standalone:
//   hipcc -O3 --offload-arch=gfx950 tools/stream_bw.hip -o /tmp/stream_bw && /tmp/stream_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e = (x);                                                                 \
        if (e != hipSuccess) {                                                              \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

template <bool NTL>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
    if (NTL) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NTS>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
    if (NTS) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U, bool NTL, bool NTS, bool RES>
__global__ __launch_bounds__(256) void apply(const u32x4 *__restrict__ x, const u32x4 *__restrict__ res,
                                             u32x4 *__restrict__ y, unsigned char *__restrict__ mask, long nvec) {
    const long tid = (long)blockIdx.x * 256 + threadIdx.x, stride = (long)gridDim.x * 256;
    for (long i0 = tid; i0 < nvec; i0 += U * stride) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long i = i0 + u * stride;
            if (i < nvec) {
                a[u] = ld<NTL>(x + i);
                if (RES) b[u] = ld<NTL>(res + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            long i = i0 + u * stride;
            if (i >= nvec) break;
            u32x4 v = a[u];
            if (RES) v = v ^ b[u];
            st<NTS>(y + i, v);
            if (RES) mask[i] = (unsigned char)(v.x & 0xff);
        }
    }
}

template <int U, bool NTL, bool NTS, bool RES>
void run(const char *name, const u32x4 *x, const u32x4 *r, u32x4 *y, unsigned char *m, long nvec, int grid) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) apply<U, NTL, NTS, RES><<<grid, 256>>>(x, r, y, m, nvec);
    CK(hipEventRecord(a));
    const int it = 20;
    for (int w = 0; w < it; ++w) apply<U, NTL, NTS, RES><<<grid, 256>>>(x, r, y, m, nvec);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= it;
    double bytes = (double)nvec * 16 * (RES ? 3 : 2) + (RES ? nvec : 0);
    std::printf("%-34s grid %5d: %8.1f us  %6.2f TB/s\n", name, grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
}

int main() {
    const long nvec = 802816L * 256 / 8;  // ResNet-50 layer1 BN3: 256 x 56 x 56 x 256 bf16
    u32x4 *x, *r, *y;
    unsigned char *m;
    CK(hipMalloc(&x, nvec * 16));
    CK(hipMalloc(&r, nvec * 16));
    CK(hipMalloc(&y, nvec * 16));
    CK(hipMalloc(&m, nvec));
    CK(hipMemset(x, 1, nvec * 16));
    CK(hipMemset(r, 2, nvec * 16));
    for (int grid : {1024, 2048, 4096, 8192}) {
        run<2, false, false, true>("res plain U2", x, r, y, m, nvec, grid);
        run<2, true, false, true>("res ntload U2", x, r, y, m, nvec, grid);
        run<2, false, true, true>("res ntstore U2", x, r, y, m, nvec, grid);
        run<2, true, true, true>("res nt both U2", x, r, y, m, nvec, grid);
        run<4, false, false, true>("res plain U4", x, r, y, m, nvec, grid);
        run<4, true, true, true>("res nt both U4", x, r, y, m, nvec, grid);
        run<2, false, false, false>("copy plain U2", x, r, y, m, nvec, grid);
        run<2, true, true, false>("copy nt both U2", x, r, y, m, nvec, grid);
        run<4, false, true, false>("copy ntstore U4", x, r, y, m, nvec, grid);
    }
    return 0;
}
