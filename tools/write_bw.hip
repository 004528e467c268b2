// Write-only / read-only / copy streaming bandwidth on MI355X (16-byte vector accesses, plain and
// non-temporal stores), the ceiling for write-dominated kernels such as the 1x1 expansion convs
// (412 MB written per 53 MB read).  Standalone:
//   hipcc -O3 --offload-arch=gfx950 tools/write_bw.hip -o /tmp/write_bw && /tmp/write_bw
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            std::exit(1);                                                                    \
        }                                                                                    \
    } while (0)

template <bool NT>
__global__ __launch_bounds__(256) void write_k(u32x4 *__restrict__ y, long n4) {
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) {
        if (NT) __builtin_nontemporal_store(v, y + i);
        else y[i] = v;
    }
}

__global__ __launch_bounds__(256) void read_k(const u32x4 *__restrict__ x, long n4, u32x4 *__restrict__ sink) {
    u32x4 a = {0u, 0u, 0u, 0u};
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) a ^= __builtin_nontemporal_load(x + i);
    if (a.x == 0x12345678u) sink[0] = a;
}

template <bool NT>
__global__ __launch_bounds__(256) void copy_k(const u32x4 *__restrict__ x, u32x4 *__restrict__ y, long n4) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += gridDim.x * 256L) {
        const u32x4 v = __builtin_nontemporal_load(x + i);
        if (NT) __builtin_nontemporal_store(v, y + i);
        else y[i] = v;
    }
}

int main() {
    const long bytes = 1L << 30;  // 1 GiB per buffer
    const long n4 = bytes / 16;
    u32x4 *x, *y, *sink;
    CK(hipMalloc(&x, bytes));
    CK(hipMalloc(&y, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(x, 1, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grids[] = {1024, 2048, 4096, 8192};
    for (int g : grids) {
        float best[5] = {1e9f, 1e9f, 1e9f, 1e9f, 1e9f};
        for (int rep = 0; rep < 5; ++rep) {
            for (int k = 0; k < 5; ++k) {
                CK(hipEventRecord(a));
                if (k == 0) write_k<false><<<g, 256>>>(y, n4);
                if (k == 1) write_k<true><<<g, 256>>>(y, n4);
                if (k == 2) read_k<<<g, 256>>>(x, n4, sink);
                if (k == 3) copy_k<false><<<g, 256>>>(x, y, n4);
                if (k == 4) copy_k<true><<<g, 256>>>(x, y, n4);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                if (ms < best[k]) best[k] = ms;
            }
        }
        std::printf("grid %5d: write %.2f TB/s  write-nt %.2f  read %.2f  copy %.2f  copy-nt %.2f (copy counts read + write)\n", g,
                    bytes / best[0] / 1e9, bytes / best[1] / 1e9, bytes / best[2] / 1e9, 2 * bytes / best[3] / 1e9,
                    2 * bytes / best[4] / 1e9);
    }
    return 0;
}
