// Collective-interference emulator for one GPU (bench.py --emulate-comm N).
//
// On a one-GPU box the bucket all-reduces of an N-rank job cannot run, yet what they cost
// the overlapped backward on the real node is mostly local: the RCCL kernels of a ring
// all-reduce occupy C workgroups (one per channel) for the duration of the transfer and
// stream the bucket through this GPU's HBM (reduce-scatter reads the local chunk and the
// chunk a peer wrote over xGMI and writes the sum, all-gather forwards it: about
// 4 (N-1)/N x bucket bytes of local traffic).  This kernel reproduces exactly that
// footprint on the comm stream in place of the collective:
//   * C workgroups of 256 threads (RCCL's block size), resident for the modelled xGMI time
//     2 (N-1)/N x bytes / busbw + latency;
//   * they copy 2 (N-1)/N x bucket bytes from the bucket into a scratch buffer (read +
//     write = the 4 (N-1)/N traffic), paced in 16 slices over that time, and spin between
//     slices with s_sleep (RCCL's waves poll their flags the same way).
// The bucket is only read (gradients stay exact).  The pacing clock is the constant-rate
// wall clock (wall_clock64, hipDeviceAttributeWallClockRate kHz).
// It is a MODEL of contention: it cannot reproduce inter-rank skew or link congestion.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>

#include "kernels.hpp"

namespace kfk {

namespace {

constexpr int kEmuThreads = 256;
constexpr int kEmuSlices = 16;

__global__ __launch_bounds__(kEmuThreads) void comm_emu_kernel(const uint4 *__restrict__ src, uint4 *__restrict__ dst,
                                                               int64_t n16, int64_t per_wg, uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    const int64_t begin = static_cast<int64_t>(blockIdx.x) * per_wg;
    const int64_t slice = (per_wg + kEmuSlices - 1) / kEmuSlices;
    for (int k = 0; k < kEmuSlices; ++k) {
        const int64_t lo = begin + k * slice;
        int64_t hi = lo + slice;
        if (hi > begin + per_wg) hi = begin + per_wg;
        int64_t j = (lo + threadIdx.x) % n16;  // wraps: more traffic than one pass over the bucket
        for (int64_t i = lo + threadIdx.x; i < hi; i += kEmuThreads) {
            dst[j] = src[j];
            j += kEmuThreads;
            while (j >= n16) j -= n16;
        }
        const uint64_t due = t0 + ticks * static_cast<uint64_t>(k + 1) / kEmuSlices;
        while (wall_clock64() < due) __builtin_amdgcn_s_sleep(16);
    }
}

}  // namespace

void launch_comm_emulate(const void *bucket, void *scratch, int64_t bytes, int64_t traffic_bytes, int ctas,
                         double seconds, hipStream_t s) {
    if (ctas < 1 || ctas > 4096) throw std::invalid_argument("comm_emulate: ctas must be in [1, 4096]");
    if (bytes < 16 || traffic_bytes < 0 || seconds < 0) throw std::invalid_argument("comm_emulate: bad sizes");
    static const int rate_khz = [] {
        int dev = 0, r = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&r, hipDeviceAttributeWallClockRate, dev) != hipSuccess || r <= 0) r = 100000;
        return r;
    }();
    const int64_t n16 = bytes / 16;
    const int64_t total16 = traffic_bytes / 16;
    const int64_t per_wg = (total16 + ctas - 1) / ctas;
    const uint64_t ticks = static_cast<uint64_t>(seconds * rate_khz * 1e3);
    comm_emu_kernel<<<ctas, kEmuThreads, 0, s>>>(static_cast<const uint4 *>(bucket), static_cast<uint4 *>(scratch), n16,
                                                per_wg, ticks);
}

}  // namespace kfk
