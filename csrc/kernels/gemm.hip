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
constexpr int kSlots = 5;            // LDS ring depth (up to 4 slabs in flight)
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

// byte offset of 16-byte chunk c (0..3) of slab row r.  ds_read_b128 serves a wave in four
// lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}
// (MI355X_MICROARCH.md, LDS); a fragment read has lane -> (row lane & 15, chunk lane >> 4), and
// the bank quad of (r, c) is 4 (r & 3) + position: XOR-ing the chunk with (r >> 2) & 2 gives every
// group 16 distinct quads (conflict-free); (r >> 2) & 3 -- the "obvious" choice -- is 2-way.
__device__ __forceinline__ int slab_swz(int r) { return (r >> 2) & 2; }
__device__ __forceinline__ int slab_off(int r, int c) { return r * kRowB + ((c ^ slab_swz(r)) << 4); }

// stage slab s (K rows s*32 .. s*32+31 of A and B) into ring slot `slot` with LDS-DMA
// (a plain function: as a lambda inside the kernel template hipcc dropped the host stub)
template <int BN>
__device__ __forceinline__ void gemm_stage(uint8_t *lds, __amdgpu_buffer_rsrc_t ar, __amdgpu_buffer_rsrc_t br,
                                           const uint32_t *a_off, const uint32_t *b_off, int wave, bool b_extra,
                                           int s, int slot) {
    constexpr int SLOT = kABytes + BN * kRowB;
    constexpr int B_INST = BN / 16, B_FULL = B_INST / 8, B_REM = B_INST % 8;
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
        __builtin_amdgcn_raw_ptr_buffer_load_lds(br, lds3(bbase + (i * 8 + wave) * 1024), 16, b_off[i] + kb, 0, 0, 0);
    if constexpr (B_REM != 0) {
        if (b_extra)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(br, lds3(bbase + (B_FULL * 8 + wave) * 1024), 16,
                                                     b_off[B_FULL] + kb, 0, 0, 0);
    }
}

// this wave's fragments of one slab: TN B blocks (its output columns) and TM A blocks (its rows).
// Inline-asm ds_read_b128 on purpose: the compiler's own waitcnt insertion waited for ALL
// outstanding LDS reads (lgkmcnt(0)) before every MFMA cluster of the two-set pipeline below,
// including the next slab's reads issued just before -- so the kernel counts them itself
// (gemm_wait_frags) and fences the MFMAs with sched_barrier (cdna_hip_programming.md §5.4 rule 18).
__device__ __forceinline__ bf16x8 ds_read16(const uint8_t *p) {
    bf16x8 v;
    const uint32_t a = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
    return v;
}

template <int TM, int TN>
__device__ __forceinline__ void gemm_frags(const uint8_t *slot, int arow0, int bcol0, int frow, int fchk,
                                           bf16x8 (&af)[TM], bf16x8 (&bf)[TN]) {
    const uint8_t *bbase = slot + kABytes;
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = ds_read16(bbase + slab_off(bcol0 + j * 16 + frow, fchk));
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = ds_read16(slot + slab_off(arow0 + i * 16 + frow, fchk));
}

// the previous set's TM + TN reads have landed; the N newest (the next slab's) may be in flight
template <int N>
__device__ __forceinline__ void gemm_wait_frags() {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// transposed product (MFMA A operand = the B fragment): acc[i][j] holds C^T[n][m] of block (i, j),
// lane -> m = lane & 15, n = (lane >> 4) * 4 + r
template <int TM, int TN>
__device__ __forceinline__ void gemm_mfma(f32x4 (&acc)[TM][TN], const bf16x8 (&af)[TM], const bf16x8 (&bf)[TN]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
}

// ---- 4-wave layout (NW4): 2 x 2 waves, each 128 x BN/2 of the 256 x BN tile -------------------------
// Per K = 32 slab a wave reads 8 A + BN/32 B fragments for 8 * BN/32 MFMAs: at BN = 256 twice the MFMAs per
// LDS byte of the 8-wave layout, whose 12 reads per 32 MFMAs (plus the LDS-DMA writes) kept the LDS
// port as busy as the matrix cores (profiles/r4_gemm_nt.md).  The 256 accumulators live in AGPRs:
// the MFMAs are inline asm with tied "+a" accumulators -- through the builtin, hipcc kept them in
// AGPRs too but re-coalesced the chains with ~216 v_accvgpr_mov per 128 MFMAs.
template <int BN>
__device__ __forceinline__ void gemm_stage4(uint8_t *lds, __amdgpu_buffer_rsrc_t ar, __amdgpu_buffer_rsrc_t br,
                                            const uint32_t *a_off, const uint32_t *b_off, int wave, int s,
                                            int slot, bool ghost) {
    // ghost: a slab past K -- the loads still issue (every step then waits for the same vmcnt, no
    // branch in the main loop) but read nothing (offset past num_records: zeros, no memory access)
    constexpr int SLOT = kABytes + BN * kRowB;
    constexpr int B_PER = BN / 16 / 4;
    uint8_t *abase = lds + slot * SLOT;
    uint8_t *bbase = abase + kABytes;
    const uint32_t kb = static_cast<uint32_t>(s * kSlabK * 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t vo = (ghost || a_off[i] == kOOB) ? kOOB : a_off[i] + kb;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, lds3(abase + (i * 4 + wave) * 1024), 16, vo, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(br, lds3(bbase + (i * 4 + wave) * 1024), 16,
                                                 ghost ? kOOB : b_off[i] + kb, 0, 0, 0);
}

// one row block's TN MFMAs, acc[j] += B_j^T A (transposed product, as gemm_mfma).  `s_nop 1` first:
// the A fragment may have just landed (a just-written operand before an MFMA, cdna_hip_programming.md
// inline-asm item 2); the accumulate chains need no wait.
template <int TN>
__device__ __forceinline__ void mfma_row(f32x4 (&acc)[TN], const bf16x8 (&b)[TN], const bf16x8 &a) {
    static_assert(TN == 8 || TN == 4, "TN");
    if constexpr (TN == 8) {
        asm volatile(
            "s_nop 1\n"
            "v_mfma_f32_16x16x32_bf16 %0, %8, %16, %0\n"
            "v_mfma_f32_16x16x32_bf16 %1, %9, %16, %1\n"
            "v_mfma_f32_16x16x32_bf16 %2, %10, %16, %2\n"
            "v_mfma_f32_16x16x32_bf16 %3, %11, %16, %3\n"
            "v_mfma_f32_16x16x32_bf16 %4, %12, %16, %4\n"
            "v_mfma_f32_16x16x32_bf16 %5, %13, %16, %5\n"
            "v_mfma_f32_16x16x32_bf16 %6, %14, %16, %6\n"
            "v_mfma_f32_16x16x32_bf16 %7, %15, %16, %7"
            : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3]), "+a"(acc[4]), "+a"(acc[5]), "+a"(acc[6]),
              "+a"(acc[7])
            : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]), "v"(b[6]), "v"(b[7]), "v"(a));
    } else {
        asm volatile(
            "s_nop 1\n"
            "v_mfma_f32_16x16x32_bf16 %0, %4, %8, %0\n"
            "v_mfma_f32_16x16x32_bf16 %1, %5, %8, %1\n"
            "v_mfma_f32_16x16x32_bf16 %2, %6, %8, %2\n"
            "v_mfma_f32_16x16x32_bf16 %3, %7, %8, %3"
            : "+a"(acc[0]), "+a"(acc[1]), "+a"(acc[2]), "+a"(acc[3])
            : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(a));
    }
}

}  // namespace

// (outside the anonymous namespace: hipcc leaves the host stubs of kernel templates declared
// there undefined when they are only instantiated from another template)
template <int BN, int EPI>
__global__ __launch_bounds__(512) void gemm_nt_kernel(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                      uint16_t *__restrict__ C, const uint16_t *__restrict__ bias,
                                                      int M, int N, int K, int mtiles, int ntiles,
                                                      const uint16_t *__restrict__ aux = nullptr,
                                                      float *__restrict__ part = nullptr, int ldc = 0) {
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
    // LDS chunk j % 4, which holds global chunk (j % 4) ^ slab_swz(row)
    const int srow = lane >> 2;
    const int schk = (lane & 3) ^ slab_swz(srow);  // rows of one instruction start at a multiple of 16
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
        // rows past N (the last tile of a ragged N) read zeros: an offset past num_records
        b_off[i] = n0 + row < N ? static_cast<uint32_t>(((n0 + row) * K + schk * 8) * 2) : kOOB;
    }
    const bool b_extra = B_REM && wave < B_REM;
    const int slabs = K / kSlabK;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Software pipeline over the 5-slot ring (slab s lives in slot s % 5):
    //   prologue: stage slabs 0..3, wait for slab 0, read its fragments into F0;
    //   step s:   wait for slab s+1 (counted vmcnt: up to two later slabs stay in flight), raw
    //             barrier, stage slab s+4 into slot (s+4) % 5 -- the slot of slab s-1, whose
    //             fragments every wave read in step s-2 and consumed before this barrier --, issue
    //             the fragment reads of slab s+1 into the other register set, then the 32 MFMAs of
    //             slab s: the LDS latency of the next slab hides under this slab's MFMAs.
    // Two register sets (F0 / F1) by a 2x-unrolled loop, so every index is static.
    const int frow = lane & 15, fchk = lane >> 4;
    const int arow0 = wm * 128, bcol0 = wn * WCOLS;
    const bool full_b = B_REM == 0 || b_extra;  // this wave's glds count per slab: 2 + BI or 2 + B_FULL
#pragma unroll
    for (int p = 0; p < kSlots - 1; ++p)
        if (p < slabs) gemm_stage<BN>(lds, ar, br, a_off, b_off, wave, b_extra, p, p);
    // slab 0 landed: min(3, slabs - 1) later slabs may stay in flight
    {
        const int later = slabs - 1 < 3 ? slabs - 1 : 3;
        if (full_b) {
            if (later == 3) vm_wait<3 * (2 + BI)>();
            else if (later == 2) vm_wait<2 * (2 + BI)>();
            else if (later == 1) vm_wait<2 + BI>();
            else vm_wait<0>();
        } else {
            if (later == 3) vm_wait<3 * (2 + B_FULL)>();
            else if (later == 2) vm_wait<2 * (2 + B_FULL)>();
            else if (later == 1) vm_wait<2 + B_FULL>();
            else vm_wait<0>();
        }
    }
    __builtin_amdgcn_s_barrier();
    bf16x8 a0[TM], b0[TN], a1[TM], b1[TN];
    gemm_frags<TM, TN>(lds, arow0, bcol0, frow, fchk, a0, b0);

    // step s: returns with the fragments of slab s+1 in (an, bn) (if it exists)
    int slot_next = 1;  // (s + 1) % 5
    int slot_stage = 4; // (s + 4) % 5
    auto pre = [&](int s) {
        // wait for slab s+1: issued so far are slabs 0 .. min(s + 3, slabs - 1)
        const int later = (slabs - 1 < s + 3 ? slabs - 1 : s + 3) - (s + 1);
        if (full_b) {
            if (later >= 2) vm_wait<2 * (2 + BI)>();
            else if (later == 1) vm_wait<2 + BI>();
            else vm_wait<0>();
        } else {
            if (later >= 2) vm_wait<2 * (2 + B_FULL)>();
            else if (later == 1) vm_wait<2 + B_FULL>();
            else vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();  // raw barrier: the later slabs' LDS-DMA stays in flight
        __builtin_amdgcn_sched_barrier(0);
        if (s + 4 < slabs) gemm_stage<BN>(lds, ar, br, a_off, b_off, wave, b_extra, s + 4, slot_stage);
        __builtin_amdgcn_sched_barrier(0);
    };
    // branch-free between the fragment reads and the MFMAs (a branch there makes the compiler
    // wait for ALL outstanding LDS reads): the last step reads a stale slot it never uses
    for (int s = 0; s < slabs; s += 2) {
        pre(s);
        gemm_frags<TM, TN>(lds + slot_next * SLOT, arow0, bcol0, frow, fchk, a1, b1);
        gemm_wait_frags<TM + TN>();
        gemm_mfma<TM, TN>(acc, a0, b0);
        slot_next = slot_next == kSlots - 1 ? 0 : slot_next + 1;
        slot_stage = slot_stage == kSlots - 1 ? 0 : slot_stage + 1;
        if (s + 1 >= slabs) break;
        pre(s + 1);
        gemm_frags<TM, TN>(lds + slot_next * SLOT, arow0, bcol0, frow, fchk, a0, b0);
        gemm_wait_frags<TM + TN>();
        gemm_mfma<TM, TN>(acc, a1, b1);
        slot_next = slot_next == kSlots - 1 ? 0 : slot_next + 1;
        slot_stage = slot_stage == kSlots - 1 ? 0 : slot_stage + 1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the last (unused) prefetch reads
    __syncthreads();  // every wave's last reads done before the ring is reused for the epilogue

    // ---- epilogue: this wave's 128 x WCOLS sub-tile as bf16 into its own LDS region (8-byte
    // writes of 4 consecutive columns; 16-byte chunk index XOR (row & 7)), then 16-byte row stores
    uint8_t *ew = lds + wave * (128 * EROW);
    constexpr bool GG = (EPI & kGemmGeluGrad) != 0;
    static_assert(!GG || (BN == 256 && EPI == kGemmGeluGrad), "GELU-gradient epilogue: 256-wide tiles, alone");
    // GELU gradient: every u row of this lane (16 x 16 bytes) requested before the LDS pass, so the
    // loads land under it instead of one HBM round trip per few stored rows
    constexpr int GNR = GG ? 128 / (64 / (WCOLS / 8)) : 1;
    uint4 guv[GNR];
    if constexpr (GG) {
        const int gch = lane % (WCOLS / 8), grs = lane / (WCOLS / 8);
        const int gcl = n0 + wn * WCOLS + gch * 8;
#pragma unroll
        for (int q = 0; q < GNR; ++q) {
            const int grow = m0 + wm * 128 + q * (64 / (WCOLS / 8)) + grs;
            guv[q] = grow < M ? *reinterpret_cast<const uint4 *>(aux + static_cast<int64_t>(grow) * N + gcl)
                              : make_uint4(0u, 0u, 0u, 0u);
        }
    }
    const int em = lane & 15, en = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = i * 16 + em;
            const int col = j * 16 + en;  // 4 columns col..col+3, inside 16-byte chunk col / 8
            uint32_t lo = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
            uint32_t hi = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
            const int chunk = (col >> 3) ^ (row & 7);
            *reinterpret_cast<uint2 *>(ew + row * EROW + chunk * 16 + (col & 7) * 2) = make_uint2(lo, hi);
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes land before its reads
    // store: CPR 16-byte chunks per row (WCOLS / 8), 64 / CPR rows per instruction
    constexpr int CPR = WCOLS / 8;
    constexpr int RPI = 64 / CPR;  // rows per wave instruction (8 / 10.67 / 16) -- CPR divides 64 for 8 and 4
    const int ch = lane % CPR, rsub = lane / CPR;
    const int gcol = n0 + wn * WCOLS + ch * 8;
    const int64_t ldo = ldc > 0 ? ldc : N;  // C row stride (>= N rounded up to 8 when N is ragged)
    float bv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) bv[k] = 0.f;
    if constexpr ((EPI & kGemmBias) != 0) {
        if (gcol + 8 <= N) {
            const uint4 braw = *reinterpret_cast<const uint4 *>(bias + gcol);
            const uint32_t bw[4] = {braw.x, braw.y, braw.z, braw.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                bv[2 * k] = bf16_to_f32(static_cast<uint16_t>(bw[k] & 0xffff));
                bv[2 * k + 1] = bf16_to_f32(static_cast<uint16_t>(bw[k] >> 16));
            }
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) bv[k] = gcol + k < N ? bf16_to_f32(bias[gcol + k]) : 0.f;
        }
    }
    // a ragged N: the chunk holding column N - 1 is stored whole (its columns past N land in the row
    // padding, ldc >= N rounded up to 8), chunks past it not at all
    const bool lane_ok = rsub < RPI && gcol < N;
    // GELU-gradient epilogue (kGemmGeluGrad, 256-wide tiles: CPR = 8, one column chunk per lane,
    // rows rsub + 8 k): du = bf16(dh * gelu'(u)) with dh the bf16 GEMM value, and this lane's
    // column sums of the bf16 du (the gelu_bwd_colsum numerics, norms.hip)
    float cs[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cs[k] = 0.f;
#pragma unroll(GG ? 16 : 4)
    for (int r0 = 0; r0 < 128; r0 += RPI) {
        const int row = r0 + rsub;
        const int grow = m0 + wm * 128 + row;
        if (!lane_ok || row >= 128 || grow >= M) continue;
        uint4 v = *reinterpret_cast<const uint4 *>(ew + row * EROW + ((ch ^ (row & 7)) << 4));
        uint16_t *dst = C + grow * ldo + gcol;
        if constexpr (GG) {
            const uint4 uv = guv[r0 / RPI];
            const uint32_t uw[4] = {uv.x, uv.y, uv.z, uv.w};
            uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint16_t r0b = f32_to_bf16(__uint_as_float(w[k] << 16) * gelu_grad_fast(__uint_as_float(uw[k] << 16)));
                const uint16_t r1b = f32_to_bf16(__uint_as_float(w[k] & 0xffff0000u) *
                                                 gelu_grad_fast(__uint_as_float(uw[k] & 0xffff0000u)));
                cs[2 * k] += bf16_to_f32(r0b);
                cs[2 * k + 1] += bf16_to_f32(r1b);
                w[k] = static_cast<uint32_t>(r0b) | (static_cast<uint32_t>(r1b) << 16);
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        } else if constexpr (EPI != 0) {
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
                w[k] = pack_bf16x2(x0, x1);
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4 *>(dst) = v;
    }
    if constexpr (GG) {
        // the 8 lanes of a column chunk (lane bits 3..5 = rsub) fold their rows in a fixed order;
        // one partial row per (M-tile, M-wave): part[2 mt + wm][n]
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            float t = cs[k];
            t += __shfl_xor(t, 8);
            t += __shfl_xor(t, 16);
            t += __shfl_xor(t, 32);
            cs[k] = t;
        }
        if (rsub == 0) {
            float *pp = part + static_cast<int64_t>(2 * mt + wm) * N + gcol;
            *reinterpret_cast<float4 *>(pp) = make_float4(cs[0], cs[1], cs[2], cs[3]);
            *reinterpret_cast<float4 *>(pp + 4) = make_float4(cs[4], cs[5], cs[6], cs[7]);
        }
    }
}

// 4-wave variant: 256 x BN tile (BN 256 / 128), waves 2 (M) x 2 (N) of 128 x BN/2, same ring, swizzle,
// XCD remap and epilogue as gemm_nt_kernel.
template <int BN, int EPI>
__global__ __launch_bounds__(256) void gemm_nt4_kernel(const uint16_t *__restrict__ A, const uint16_t *__restrict__ B,
                                                       uint16_t *__restrict__ C, const uint16_t *__restrict__ bias,
                                                       int M, int N, int K, int mtiles, int ntiles) {
    constexpr int TN = BN / 32;           // 16-column blocks per wave (2 waves along N)
    constexpr int TM = 8;                 // 16-row blocks per wave (2 waves along M)
    constexpr int SLOT = kABytes + BN * kRowB;
    constexpr int B_PER = BN / 64;        // 16-row glds instructions of the B slab per wave
    constexpr int PER = 4 + B_PER;        // glds per wave per slab
    constexpr int WCOLS = BN / 2;         // output columns per wave
    constexpr int EROW = WCOLS * 2;       // epilogue LDS row pitch (bytes)
    constexpr int LDS_RING = kSlots * SLOT;
    constexpr int LDS_EPI = 4 * 128 * EROW;
    constexpr int LDS = LDS_RING > LDS_EPI ? LDS_RING : LDS_EPI;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDS];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
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
    const int srow = lane >> 2;
    const int schk = (lane & 3) ^ slab_swz(srow);
    uint32_t a_off[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int row = (i * 4 + wave) * 16 + srow;
        a_off[i] = m0 + row < M ? static_cast<uint32_t>(((m0 + row) * K + schk * 8) * 2) : kOOB;
    }
    uint32_t b_off[B_PER];
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
        const int row = (i * 4 + wave) * 16 + srow;
        b_off[i] = static_cast<uint32_t>(((n0 + row) * K + schk * 8) * 2);
    }
    const int slabs = K / kSlabK;

    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int frow = lane & 15, fchk = lane >> 4;
    const int arow0 = wm * 128, bcol0 = wn * WCOLS;
    // slabs is even (K % 64 == 0, launch_gemm_nt): every step below runs both halves, no branch
#pragma unroll
    for (int p = 0; p < kSlots - 1; ++p) gemm_stage4<BN>(lds, ar, br, a_off, b_off, wave, p, p, p >= slabs);
    vm_wait<3 * PER>();
    __builtin_amdgcn_s_barrier();
    bf16x8 af[TM], b0[TN], b1[TN];
    gemm_frags<TM, TN>(lds, arow0, bcol0, frow, fchk, af, b0);

    int slot_next = 1, slot_stage = 4;
    auto pre = [&](int s) {
        vm_wait<2 * PER>();  // slab s + 1 landed (ghost slabs keep the count uniform at the tail)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        gemm_stage4<BN>(lds, ar, br, a_off, b_off, wave, s + 4, slot_stage, s + 4 >= slabs);
        __builtin_amdgcn_sched_barrier(0);
    };
    // per slab: the next slab's B fragments into the other B set, then row block i's MFMAs and the
    // next slab's A fragment i read in place behind them; before row block i the reads newer than
    // this slab's A fragment i are its 7 - i successors, the TN next-B reads and i next-A reads
    auto half = [&](bf16x8 (&bc)[TN], bf16x8 (&bn)[TN]) {
        const uint8_t *nslot = lds + slot_next * SLOT;
#pragma unroll
        for (int j = 0; j < TN; ++j) bn[j] = ds_read16(nslot + kABytes + slab_off(bcol0 + j * 16 + frow, fchk));
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            gemm_wait_frags<TN + 7>();
            mfma_row<TN>(acc[i], bc, af[i]);
            __builtin_amdgcn_sched_barrier(0);
            af[i] = ds_read16(nslot + slab_off(arow0 + i * 16 + frow, fchk));
        }
    };
    for (int s = 0; s < slabs; s += 2) {
        pre(s);
        half(b0, b1);
        slot_next = slot_next == kSlots - 1 ? 0 : slot_next + 1;
        slot_stage = slot_stage == kSlots - 1 ? 0 : slot_stage + 1;
        pre(s + 1);
        half(b1, b0);
        slot_next = slot_next == kSlots - 1 ? 0 : slot_next + 1;
        slot_stage = slot_stage == kSlots - 1 ? 0 : slot_stage + 1;
    }
    vm_wait<0>();  // the ghost slabs' loads
    // the last (unused) prefetch reads, and 16 wait states before the accumulators are read (an
    // MFMA's result -> a non-MFMA reader: 12 states for the 8-pass XDL ops)
    asm volatile("s_waitcnt lgkmcnt(0)\n s_nop 7\n s_nop 7" ::: "memory");
    __syncthreads();

    uint8_t *ew = lds + wave * (128 * EROW);
    const int em = lane & 15, en = (lane >> 4) * 4;
    constexpr int CH = EROW / 16;  // 16-byte chunks per epilogue row
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = i * 16 + em;
            const int col = j * 16 + en;
            uint32_t lo = pack_bf16x2(acc[i][j][0], acc[i][j][1]);
            uint32_t hi = pack_bf16x2(acc[i][j][2], acc[i][j][3]);
            const int chunk = ((col >> 3) ^ (row & 7)) & (CH - 1);
            *reinterpret_cast<uint2 *>(ew + row * EROW + chunk * 16 + (col & 7) * 2) = make_uint2(lo, hi);
        }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    constexpr int CPR = WCOLS / 8;
    constexpr int RPI = 64 / CPR;
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
#pragma unroll 4
    for (int r0 = 0; r0 < 128; r0 += RPI) {
        const int row = r0 + rsub;
        const int grow = m0 + wm * 128 + row;
        if (grow >= M) continue;
        uint4 v = *reinterpret_cast<const uint4 *>(ew + row * EROW + (((ch ^ (row & 7)) & (CH - 1)) << 4));
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
                w[k] = pack_bf16x2(x0, x1);
            }
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        *reinterpret_cast<uint4 *>(dst) = v;
    }
}

namespace {

template <int BN>
void launch_bn4(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K, int epi,
                hipStream_t s) {
    const int mtiles = (M + kGM - 1) / kGM, ntiles = N / BN;
    const dim3 grid(mtiles * ntiles), block(256);
    switch (epi) {
    case 0: gemm_nt4_kernel<BN, 0><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmBias: gemm_nt4_kernel<BN, kGemmBias><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmAccum: gemm_nt4_kernel<BN, kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles); break;
    case kGemmBias | kGemmAccum:
        gemm_nt4_kernel<BN, kGemmBias | kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles);
        break;
    default: throw std::invalid_argument("gemm_nt: unsupported epilogue");
    }
}

template <int BN>
void launch_bn(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K, int epi,
               hipStream_t s, int ldc = 0) {
    const int mtiles = (M + kGM - 1) / kGM, ntiles = (N + BN - 1) / BN;
    const dim3 grid(mtiles * ntiles), block(512);
    switch (epi) {
    case 0:
        gemm_nt_kernel<BN, 0><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles, nullptr, nullptr, ldc);
        break;
    case kGemmBias:
        gemm_nt_kernel<BN, kGemmBias><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles, nullptr, nullptr,
                                                            ldc);
        break;
    case kGemmAccum:
        gemm_nt_kernel<BN, kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles, nullptr, nullptr,
                                                             ldc);
        break;
    case kGemmBias | kGemmAccum:
        gemm_nt_kernel<BN, kGemmBias | kGemmAccum><<<grid, block, 0, s>>>(a, b, c, bias, M, N, K, mtiles, ntiles,
                                                                         nullptr, nullptr, ldc);
        break;
    default: throw std::invalid_argument("gemm_nt: unsupported epilogue");
    }
}

}  // namespace

int gemm_nt_gelu_grad_rows(int M) { return 2 * ((M + kGM - 1) / kGM); }

void launch_gemm_nt_gelu_grad(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *u, float *part, int M,
                              int N, int K, hipStream_t s) {
    if (!gemm_nt_supported(M, N, K) || N % 256) throw std::invalid_argument("gemm_nt_gelu_grad: unsupported shape");
    if (!u || !part) throw std::invalid_argument("gemm_nt_gelu_grad: needs the pre-activation and the partials");
    const int mtiles = (M + kGM - 1) / kGM, ntiles = N / 256;
    gemm_nt_kernel<256, kGemmGeluGrad><<<mtiles * ntiles, 512, 0, s>>>(a, b, c, nullptr, M, N, K, mtiles, ntiles, u, part);
}

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

bool gemm_nt_ld_supported(int64_t M, int64_t N, int64_t K, int64_t ldc) {
    return M > 0 && N > 0 && K >= 32 && K % 32 == 0 && ldc % 8 == 0 && ldc >= (N + 7) / 8 * 8 &&
           M * K * 2 < (int64_t(1) << 31) && N * K * 2 < (int64_t(1) << 31) && M * ldc < (int64_t(1) << 40);
}

void launch_gemm_nt_ld(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K,
                       int ldc, int epi, int bn, hipStream_t s) {
    if (!gemm_nt_ld_supported(M, N, K, ldc)) throw std::invalid_argument("gemm_nt_ld: unsupported shape / row stride");
    if ((epi & kGemmBias) && !bias) throw std::invalid_argument("gemm_nt_ld: bias epilogue without bias");
    switch (bn) {
    case 256: launch_bn<256>(a, b, c, bias, M, N, K, epi, s, ldc); break;
    case 192: launch_bn<192>(a, b, c, bias, M, N, K, epi, s, ldc); break;
    case 128: launch_bn<128>(a, b, c, bias, M, N, K, epi, s, ldc); break;
    default: throw std::invalid_argument("gemm_nt_ld: tile width must be 128, 192 or 256");
    }
}

void launch_gemm_nt(const uint16_t *a, const uint16_t *b, uint16_t *c, const uint16_t *bias, int M, int N, int K,
                    int epi, int bn, hipStream_t s) {
    if (!gemm_nt_supported(M, N, K)) throw std::invalid_argument("gemm_nt: unsupported shape");
    if ((epi & kGemmBias) && !bias) throw std::invalid_argument("gemm_nt: bias epilogue without bias");
    if (bn <= 0) bn = gemm_nt_pick_bn(M, N);
    if (bn < 1000 && N % bn) throw std::invalid_argument("gemm_nt: N not a multiple of the tile width");
    // bn 1256 / 1128: the 4-wave layout of the 256 / 128-wide tiles
    if (bn > 1000) {
        if (N % (bn - 1000)) throw std::invalid_argument("gemm_nt: N not a multiple of the tile width");
        if (K % 64) throw std::invalid_argument("gemm_nt: the 4-wave tiles need K % 64 == 0");
        if (bn == 1256) launch_bn4<256>(a, b, c, bias, M, N, K, epi, s);
        else if (bn == 1128) launch_bn4<128>(a, b, c, bias, M, N, K, epi, s);
        else throw std::invalid_argument("gemm_nt: 4-wave tile width must be 1128 or 1256");
        return;
    }
    switch (bn) {
    case 256: launch_bn<256>(a, b, c, bias, M, N, K, epi, s); break;
    case 192: launch_bn<192>(a, b, c, bias, M, N, K, epi, s); break;
    case 128: launch_bn<128>(a, b, c, bias, M, N, K, epi, s); break;
    default: throw std::invalid_argument("gemm_nt: tile width must be 128, 192 or 256");
    }
}

}  // namespace kfk
