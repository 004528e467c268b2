// Dedicated bf16 "NT" GEMM for the transformer linear layers:
//     C[M, N] = A[M, K] . B[N, K]^T  (+ bias[N]) (+ C_old)      f32 accumulation, bf16 out
// (BERT: forward y = x W^T with W [out, in]; data gradient dx = dy W with the transposed
// weight W^T [in, out] -- both operands K-contiguous).
//
// Why not the implicit-GEMM conv kernel (conv.hip, launch_gemm): its 256x256 tile has room for
// only two 64-deep LDS stages, so every K-step waits for ALL its LDS-DMA (vmcnt(0)) -- the ~1.0
// PF/s ceiling measured on BERT's shapes (profiles/README.md, round 3) against hipBLASLt's 1.2.
// This kernel keeps the staging pipeline three slabs deep across barriers instead:
//   * 256 x BN tile (BN 256 / 192 / 128), 8 waves as 2 (M) x 4 (N), each wave 128 x BN/4;
//   * K is consumed in 32-deep slabs through a ring of 4 LDS slots (A 16 KB + B BN*64 B each,
//     <= 128 KB): slab s+3 is staged (buffer_load ... lds, 16 B per lane, lane-linear image with
//     the swizzle applied on the SOURCE address) while slab s is computed, and the wait before a
//     slab's reads is a COUNTED vmcnt (two slabs stay in flight across the raw s_barrier) -- the
//     "pipelining across barriers" rule of cdna_hip_programming.md §5;
//   * conflict-free fragment reads: 64-byte slab rows, 16-byte chunk c of row r stored at chunk
//     c ^ ((r >> 2) & 3) (the 16 rows of a ds_read_b128 lane group hit 16 distinct bank quads);
//   * per slab and wave: 12 ds_read_b128 (4 B + 8 A fragments), then two clusters of 16
//     v_mfma_f32_16x16x32_bf16 under s_setprio(1) -- the second A half's reads land under the
//     first cluster (lgkmcnt(4));
//   * the product is computed transposed (MFMA A operand = the B fragment), so each lane holds 4
//     consecutive output COLUMNS of one row: the epilogue packs them into 8-byte LDS writes, then
//     every wave streams its 128 x (BN/4) sub-tile out in full 128-byte row segments (16-byte
//     stores), applying bias / accumulate on the way;
//   * XCD-aware tile order: a bijective remap gives each XCD a contiguous run of tiles, and tiles
//     run N-fastest, so the blocks of one XCD share their A panels in its L2;
//   * operands through buffer resources (32-bit offsets, rows past M read zeros): A and B must
//     each be below 2 GiB (gemm_nt_supported).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>

#include "common.hpp"
#include "kernels.hpp"

namespace kfk {

namespace {

using bf16x8 = __attribute__((ext_vector_type(8))) short;
using f32x4 = __attribute__((ext_vector_type(4))) float;

constexpr int kGM = 256;             // tile rows
constexpr int kSlabK = 32;           // K per slab
constexpr int kSlots = 4;            // LDS ring depth (3 slabs in flight)
constexpr int kRowB = kSlabK * 2;    // 64-byte slab rows
constexpr int kABytes = kGM * kRowB; // 16 KB
constexpr uint32_t kOOB = 0x80000000u;
constexpr int kRsrcFlags = 0x00020000;

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ __attribute__((address_space(3))) void *lds3(uint8_t *p) {
    return (__attribute__((address_space(3))) void *)(p);
}

// byte offset of 16-byte chunk c (0..3) of slab row r
__device__ __forceinline__ int slab_off(int r, int c) { return r * kRowB + ((c ^ ((r >> 2) & 3)) << 4); }

template <int BN, int EPI>
__global__ __launch_bounds__(512) void gemm_nt_kernel(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                      uint16_t *__restrict__ C, const uint16_t *__restrict__ bias,
                                                      int M, int N, int K, int mtiles, int ntiles) {
    constexpr int TN = BN / 64;           // 16-column blocks per wave (4 waves along N)
    constexpr int TM = 8;                 // 16-row blocks per wave (2 waves along M)
    constexpr int BBYTES = BN * kRowB;
    constexpr int SLOT = kABytes + BBYTES;
    constexpr int B_INST = BN / 16;       // 16-row glds instructions for the B slab (12 / 16 / 8)
    constexpr int B_FULL = B_INST / 8;    // per wave, every wave
    constexpr int B_REM = B_INST % 8;     // the first B_REM waves take one more
    constexpr int WCOLS = BN / 4;         // output columns per wave
    constexpr int EROW = 128;             // epilogue LDS row pitch (bytes): up to 64 columns
    constexpr int LDS_RING = kSlots * SLOT;
    constexpr int LDS_EPI = 8 * 128 * EROW;
    constexpr int LDS = LDS_RING > LDS_EPI ? LDS_RING : LDS_EPI;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3;

    // bijective XCD remap: the blocks that share an XCD (orig % 8) get a contiguous run of tiles
    const int nwg = mtiles * ntiles;
    const int orig = blockIdx.x;
    const int q = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
    const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + (orig >> 3);
    const int mt = wgid / ntiles, nt = wgid - mt * ntiles;
    const int m0 = mt * kGM, n0 = nt * BN;

    const __amdgpu_buffer_rsrc_t ar =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(A), 0, static_cast<int>(kOOB), kRsrcFlags);
    const __amdgpu_buffer_rsrc_t br =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(B), 0, static_cast<int>(kOOB), kRsrcFlags);

    // staging: glds instruction i of a wave writes 1 KB = 16 slab rows, lane j -> row j / 4,
    // LDS chunk j % 4, which holds global chunk (j % 4) ^ ((row >> 2) & 3)
    const int srow = lane >> 2;
    const int schk = (lane & 3) ^ ((srow >> 2) & 3);  // rows of one instruction start at a multiple of 16
    uint32_t a_off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int row = (i * 8 + wave) * 16 + srow;
        a_off[i] = m0 + row < M ? static_cast<uint32_t>(((m0 + row) * K + schk * 8) * 2) : kOOB;
    }
    constexpr int BI = B_FULL + (B_REM ? 1 : 0);
    uint32_t b_off[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
        const int row = (i * 8 + wave) * 16 + srow;  // < BN for the instructions this wave issues
        b_off[i] = static_cast<uint32_t>(((n0 + row) * K + schk * 8) * 2);
    }
    const bool b_extra = B_REM && wave < B_REM;
    const int slabs = K / kSlabK;

    auto stage = [&](int s, int slot) {
        uint8_t *abase = lds + slot * SLOT;
        uint8_t *bbase = abase + kABytes;
        const uint32_t kb = static_cast<uint32_t>(s * kSlabK * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const uint32_t vo = a_off[i] == kOOB ? kOOB : a_off[i] + kb;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, lds3(abase + (i * 8 + wave) * 1024), 16, vo, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < B_FULL; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(br, lds3(bbase + (i * 8 + wave) * 1024), 16, b_off[i] + kb, 0, 0,
                                                     0);
        if constexpr (B_REM != 0) {
            if (b_extra)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(br, lds3(bbase + (B_FULL * 8 + wave) * 1024), 16,
                                                         b_off[B_FULL] + kb, 0, 0, 0);
        }
    };

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // prologue: slabs 0..2 in flight
#pragma unroll
    for (int p = 0; p < kSlots - 1; ++p)
        if (p < slabs) stage(p, p);

    const int frow = lane & 15, fchk = lane >> 4;
    for (int s = 0; s < slabs; ++s) {
        const int slot = s & (kSlots - 1);
        // slab s landed: the (at most two) slabs staged after it may stay in flight.  The
        // per-wave count differs when the B slab does not split evenly over the 8 waves.
        if (s + 2 < slabs) {
            if (B_REM == 0 || b_extra) vm_wait<2 * (2 + BI)>();
            else vm_wait<2 * (2 + B_FULL)>();
        } else if (s + 1 < slabs) {
            if (B_REM == 0 || b_extra) vm_wait<2 + BI>();
            else vm_wait<2 + B_FULL>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();  // raw barrier: the later slabs' LDS-DMA stays in flight
        __builtin_amdgcn_sched_barrier(0);
        if (s + kSlots - 1 < slabs) stage(s + kSlots - 1, (s + kSlots - 1) & (kSlots - 1));  // slot read at s-1
        __builtin_amdgcn_sched_barrier(0);
        const uint8_t *abase = lds + slot * SLOT;
        const uint8_t *bbase = abase + kABytes;
        bf16x8 bf[TN], af[TM];
#pragma unroll
        for (int j = 0; j < TN; ++j)
            bf[j] = *reinterpret_cast<const bf16x8 *>(bbase + slab_off(wn * WCOLS + j * 16 + frow, fchk));
#pragma unroll
        for (int i = 0; i < TM; ++i)
            af[i] = *reinterpret_cast<const bf16x8 *>(abase + slab_off(wm * 128 + i * 16 + frow, fchk));
        // transposed product: MFMA A operand = B fragment (n), B operand = A fragment (m), so
        // acc[i][j] holds C^T[n][m]: lane -> m = lane & 15, n = (lane >> 4) * 4 + r.  The
        // compiler's own lgkmcnt waits let the second A half land under the first cluster.
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TM / 2; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = TM / 2; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();  // every wave's last reads done before the ring is reused for the epilogue

    // ---- epilogue: this wave's 128 x WCOLS sub-tile as bf16 into its own LDS region (8-byte
    // writes of 4 consecutive columns; 16-byte chunk index XOR (row & 7)), then 16-byte row stores
    uint8_t *ew = lds + wave * (128 * EROW);
    const int em = lane & 15, en = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = i * 16 + em;
            const int col = j * 16 + en;  // 4 columns col..col+3, inside 16-byte chunk col / 8
            uint32_t lo = static_cast<uint32_t>(f32_to_bf16(acc[i][j][0])) |
                          (static_cast<uint32_t>(f32_to_bf16(acc[i][j][1])) << 16);
            uint32_t hi = static_cast<uint32_t>(f32_to_bf16(acc[i][j][2])) |
                          (static_cast<uint32_t>(f32_to_bf16(acc[i][j][3])) << 16);
            const int chunk = (col >> 3) ^ (row & 7);
            *reinterpret_cast<uint2 *>(ew + row * EROW + chunk * 16 + (col & 7) * 2) = make_uint2(lo, hi);
        }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    // store: CPR 16-byte chunks per row (WCOLS / 8), 64 / CPR rows per instruction
    constexpr int CPR = WCOLS / 8;
    constexpr int RPI = 64 / CPR;  // rows per wave instruction (8 / 10.67 / 16) -- CPR divides 64 for 8 and 4
    const int ch = lane % CPR, rsub = lane / CPR;
    const int gcol = n0 + wn * WCOLS + ch * 8;
    float bv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = 0.f;
    if constexpr ((EPI & kGemmBias) != 0) {
        const uint4 braw = *reinterpret_cast<const uint4 *>(bias + gcol);
        const uint32_t bw[4] = {braw.x, braw.y, braw.z, braw.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            bv[2 * k] = bf16_to_f32(static_cast<uint16_t>(bw[k] & 0xffff));
            bv[2 * k + 1] = bf16_to_f32(static_cast<uint16_t>(bw[k] >> 16));
        }
    }
    const bool lane_ok = rsub < RPI;
#pragma unroll 4
    for (int r0 = 0; r0 < 128; r0 += RPI) {
        const int row = r0 + rsub;
        const int grow = m0 + wm * 128 + row;
        if (!lane_ok || row >= 128 || grow >= M) continue;
        uint4 v = *reinterpret_cast<const uint4 *>(ew + row * EROW + ((ch ^ (row & 7)) << 4));
        uint16_t *dst = C + static_cast<int64_t>(grow) * N + gcol;
        if constexpr (EPI != 0) {
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
            uint32_t o[4] = {0u, 0u, 0u, 0u};
            if constexpr ((EPI & kGemmAccum) != 0) {
                const uint4 ov = *reinterpret_cast<const uint4 *>(dst);
                o[0] = ov.x, o[1] = ov.y, o[2] = ov.z, o[3] = ov.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float x0 = bf16_to_f32(static_cast<uint16_t>(w[k] & 0xffff)) + bv[2 * k];
                float x1 = bf16_to_f32(static_cast<uint16_t>(w[k] >> 16)) + bv[2 * k + 1];
                if constexpr ((EPI & kGemmAccum) != 0) {
                    x0 += bf16_to_f32(static_cast<uint16_t>(o[k] & 0xffff));
                    x1 += bf16_to_f32(static_cast<uint16_t>(o[k] >> 16));
                }
                w[k] = static_cast<uint32_t>(f32_to_bf16(x0)) | (static_cast<uint32_t>(f32_to_bf16(x1)) << 16);
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4 *>(dst) = v;
    }
}

template <int BN>
void launch_bn(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K, int epi,
               hipStream_t s) {
    const int mtiles = (M + kGM - 1) / kGM, ntiles = N / BN;
    const dim3 grid(mtiles * ntiles), block(512);
    switch (epi) {
    case 0: gemm_nt_kernel<BN, 0><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmBias: gemm_nt_kernel<BN, kGemmBias><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmAccum: gemm_nt_kernel<BN, kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmBias | kGemmAccum:
        gemm_nt_kernel<BN, kGemmBias | kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles);
        break;
    default: throw std::invalid_argument("gemm_nt: unsupported epilogue");
    }
}

}  // namespace

bool gemm_nt_supported(int64_t M, int64_t N, int64_t K) {
    return M > 0 && N >= 128 && N % 128 == 0 && K >= 32 && K % 32 == 0 && M * K * 2 < (int64_t(1) << 31) &&
           N * K * 2 < (int64_t(1) << 31) && M * N < (int64_t(1) << 31);
}

int gemm_nt_pick_bn(int64_t M, int64_t N) {
    // fill the 256 CUs in whole waves of one 256-row tile per CU: the widest tile whose count is
    // a multiple of 256 (BERT at 16 K tokens: N 768 / 2304 -> 192, N 3072 -> 256), else the widest
    // that gives >= 2 waves, else 128
    const int64_t mt = (M + kGM - 1) / kGM;
    const int cand[3] = {256, 192, 128};
    for (int bn : cand)
        if (N % bn == 0 && (mt * (N / bn)) % 256 == 0) return bn;
    for (int bn : cand)
        if (N % bn == 0 && mt * (N / bn) >= 512) return bn;
    return N % 256 == 0 && mt * (N / 256) >= 256 ? 256 : 128;
}

void launch_gemm_nt(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K,
                    int epi, int bn, hipStream_t s) {
    if (!gemm_nt_supported(M, N, K)) throw std::invalid_argument("gemm_nt: unsupported shape");
    if ((epi & kGemmBias) && !bias) throw std::invalid_argument("gemm_nt: bias epilogue without bias");
    if (bn <= 0) bn = gemm_nt_pick_bn(M, N);
    if (N % bn) throw std::invalid_argument("gemm_nt: N not a multiple of the tile width");
    switch (bn) {
    case 256: launch_bn<256>(a, b, c, bias, M, N, K, epi, s); break;
    case 192: launch_bn<192>(a, b, c, bias, M, N, K, epi, s); break;
    case 128: launch_bn<128>(a, b, c, bias, M, N, K, epi, s); break;
    default: throw std::invalid_argument("gemm_nt: tile width must be 128, 192 or 256");
    }
}

}  // namespace kfk
