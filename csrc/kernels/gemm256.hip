// Large-tile bf16 TN GEMM for gfx950: 256xBN block tile (BN = 256 or 128),
// 8 waves, LDS ring.
//
//   C[M,N] = epi(A[M,K] . B[N,K]^T)      (same contract as gemm.hip)
//
// Why a second kernel: the 128x128 two-barrier loop of gemm.hip tops out
// near 0.9-1.0 PF because every k-step drains its LDS-DMA before the
// barrier (cdna_hip_programming.md §5, "the step-3 structure's ceiling").
// This kernel keeps the DMA in flight across barriers:
//
//  * K is consumed in 32-deep halves; a 4-slot LDS ring (4 x 32 KiB =
//    128 KiB for BN = 256, one block per CU) holds A[256][32] + B[BN][32]
//    per slot.
//  * at half-step h (its fragments already in registers) every wave waits
//    with a *counted* `s_waitcnt vmcnt(8)` -- only half h+1 must have
//    landed, halves h+2 and h+3 stay in flight -- and a raw s_barrier
//    (never __syncthreads, whose implicit vmcnt(0) would drain the ring),
//    restages the slot half h came from with half h+4 (LDS-DMA,
//    global_load_lds_dwordx4), issues the ds_reads of half h+1 into a second
//    register set and runs the 32 MFMAs of half h under them.
//  * 64-B LDS rows, 16-B chunk c of row r stored at chunk c ^ ((r>>1)&3):
//    each ds_read_b128 lane group covers all 16 bank slots (conflict-free,
//    see swz()); the swizzle is applied on the DMA source address because
//    LDS-DMA writes lane-linearly (rule 21).
//  * BN = 256: 8 waves as 2(M) x 4(N), 128x64 outputs per wave = 8x4
//    tiles of v_mfma_f32_16x16x32_bf16; BN = 128 (for N where 256-wide
//    tiles leave CUs idle, e.g. 2048x4096): 4(M) x 2(N) waves of 64x64.
//    Swapped MFMA operands (C^T in registers -> 4 consecutive columns per
//    lane -> 8-B stores, float4 bias).
//  * XCD-aware bijective workgroup remap + 4-tile-row grouping.
#include <algorithm>
#include <type_traits>

#include "common.hpp"
#include "kernels.hpp"

namespace kiosk {
namespace {

constexpr int BM = 256, BKH = 32;
constexpr int kRowBytes = BKH * 2;                 // 64 B per row per half
constexpr int kSlots = 4;

// Per-BN geometry.  LDS slot = A[256][32] + B[BN][32]; an operand half is
// rows/16 DMA pieces of 16 rows x 64 B spread over the 8 waves.
template <int BN, int kWaves = 8>
struct Geo {
  static constexpr int kWavesM = kWaves == 4 ? 2 : (BN == 256 ? 2 : 4);
  static constexpr int kWavesN = kWaves / kWavesM;
  static constexpr int TM = BM / kWavesM / 16;     // 16-row tiles per wave
  static constexpr int TN = BN / kWavesN / 16;     // 16-col tiles per wave
  static constexpr int kABytes = BM * kRowBytes;   // 16 KiB
  static constexpr int kSlotBytes = (BM + BN) * kRowBytes;
  // the 4-wave kernel's ring: 5 units of one operand x 64-deep K-step
  static constexpr int kLdsBytes =
      kWaves == 4 ? 5 * BM * 128 : kSlots * kSlotBytes;
  static constexpr int kPiecesA = BM / 16 / kWaves;
  static constexpr int kPiecesB = BN / 16 / kWaves;
  static constexpr int kLoadsPerHalf = kPiecesA + kPiecesB;  // glds/wave
  static constexpr int kReads = TM + TN;           // ds_read_b128 per half
};

// ds_read_b128 is serviced in 16-lane groups {0-3,12-15,20-27},
// {4-11,16-19,28-31}, ... (MI355X_MICROARCH.md §LDS), not 16 consecutive
// lanes.  With 64-B rows, row r = lane & 15 and chunk = lane >> 4, the XOR
// term (r >> 1) & 3 gives every group 16 distinct 16-B bank slots
// (conflict-free, 4 LDS cycles per read); the earlier (r >> 2) & 3 was
// 2-way conflicted under that grouping.
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 3; }

__device__ __forceinline__ int slot_off(int r, int c) {
  return r * kRowBytes + ((c ^ swz(r)) << 4);
}

// An operand half = DMA pieces of 16 rows x 64 B (1 KiB); wave w issues
// pieces [w * kPieces, (w + 1) * kPieces).
template <int kPieces>
__device__ __forceinline__ void stage_operand(const uint16_t* __restrict__ g,
                                              int ld, int row0, int rows,
                                              int k0, char* lds, int wave,
                                              int lane) {
#pragma unroll
  for (int i = 0; i < kPieces; ++i) {
    const int piece = wave * kPieces + i;
    const int r = piece * 16 + (lane >> 2);
    const int c = (lane & 3) ^ swz(r);
    int grow = row0 + r;
    grow = grow < rows ? grow : rows - 1;
    glds16(g + static_cast<size_t>(grow) * ld + k0 + c * 8,
           lds + piece * 1024);
  }
}

// One DMA piece (16 rows x 64 B) of an operand half: `piece` indexes the
// operand's 1 KiB pieces.
__device__ __forceinline__ void stage_piece(const uint16_t* __restrict__ g,
                                            int ld, int row0, int rows,
                                            int k0, char* lds, int piece,
                                            int lane) {
  const int r = piece * 16 + (lane >> 2);
  const int c = (lane & 3) ^ swz(r);
  int grow = row0 + r;
  grow = grow < rows ? grow : rows - 1;
  glds16(g + static_cast<size_t>(grow) * ld + k0 + c * 8,
         lds + piece * 1024);
}

// Items p in [0, n) are issued in quarter p * 4 / n: how many land in q.
constexpr int per_quarter(int n, int q) {
  int c = 0;
  for (int p = 0; p < n; ++p) c += (p * 4 / n == q);
  return c;
}

// MFMA with the accumulator pinned to AGPRs.  The 4-wave layout keeps a
// 128x128 fp32 tile per wave (256 registers): with the builtin, hipcc
// splits the AV register class badly (operands land in AGPRs, ~200 VGPRs
// spill); the "a" constraint keeps every accumulator in the AGPR file and
// every operand in VGPRs.  Hazards (cdna_hip_programming.md §5.7): the
// operands come from ds_read (hipcc waits lgkmcnt for asm operands), an
// accumulate chain into the same AGPRs needs no wait states, and the
// epilogue's first AGPR read is padded by mfma_drain().
__device__ __forceinline__ void mfma_agpr(f32x4& acc, const bf16x8& a,
                                          const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
               : "+a"(acc)
               : "v"(a), "v"(b));
}

// First K-step of a tile: C = 0 as the inline constant, so the zeroed
// accumulators never exist in VGPRs (a zero-initialised array held there
// across the prologue costs 256 VGPRs and spills).
__device__ __forceinline__ void mfma_agpr_first(f32x4& acc, const bf16x8& a,
                                                const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
               : "=a"(acc)
               : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// Diagnostic builds only (tools/probes/gemm_ablate.hip): bit 0 drops the 4-wave
// kernel's in-loop DMA, bit 1 its in-loop LDS reads.  Results are wrong in such builds; 0 in the product.
#ifndef KIOSK_GEMM_ABLATE
#define KIOSK_GEMM_ABLATE 0
#endif
// 1: every DMA and LDS-read issue of a half-step inside its first 48 MFMAs
// (+0.5..1.4 % over one per 8 / per 4 across all 64)
#ifndef KIOSK_W4_SPREAD
#define KIOSK_W4_SPREAD 1
#endif
// Stagger the four waves' DMA issue slots against each other: without it
// all four issue their pieces at the same MFMA indices right after the
// barrier and queue on the CU's one texture-address path.  2 (default):
// waves 2 and 3 issue KIOSK_W4_STAGGER_OFF MFMAs later -- +2.0 % on the
// bias+GELU up-projection, +1.2 % on the split-K down-projection, +0.4-0.6 %
// at 8192^3 (profiles/r3_stagger/, 5 interleaved rounds); 4 = waves 0..3
// at offsets 0, 1, 3, 4 (slower); 0 = off.  The persistent kernel keeps one
// schedule (two copies of its loop spill).
#ifndef KIOSK_W4_STAGGER
#define KIOSK_W4_STAGGER 2
#endif
#ifndef KIOSK_W4_STAGGER_OFF
#define KIOSK_W4_STAGGER_OFF 3     // MFMAs the later half of the waves lags
#endif
#ifndef KIOSK_W4_STAGGER_SEL
#define KIOSK_W4_STAGGER_SEL 1     // 0: odd waves lag; 1: waves 2, 3 lag
#endif
// Experiment (tools/probes/gemm_ablate.hip A/B, off in the product): stage the
// k-loop's operand pieces through VGPRs -- buffer_load_dwordx4 into
// registers in half-step h, ds_write_b128 into the ring in half-step h + 1 --
// instead of LDS-DMA, whose issue holds the wave ~60 cycles among MFMAs.
#ifndef KIOSK_W4_REGSTAGE
#define KIOSK_W4_REGSTAGE 0
#endif

// Counted waits go through the builtin (not inline asm) so hipcc's waitcnt
// pass sees them and adds no conservative lgkmcnt(0) of its own.  gfx9
// encoding: vmcnt[3:0] | expcnt[6:4] (7 = no wait) | lgkmcnt[11:8] |
// vmcnt[5:4] in bits [15:14].  lgkmcnt is always 0 here.
constexpr int waitcnt_vm(int vm) {
  return (vm & 0xF) | (((vm >> 4) & 3) << 14) | 0x0070;
}

// kFused (4-wave split-K, two K slices): in-launch combine.  Every K-slice
// block writes its fp32 partial tile to P[blockIdx.y]; the block that
// arrives last at its tile's counter re-reads both partials and runs the
// epilogue.  (A "ticket first" variant -- the first block publishes one
// plane, the second keeps its accumulators and waits for it -- measured
// slower than the reduce kernel and spilled: removed, profiles/r2_splitk_ab.)
// kPersist (4-wave only): a grid of one workgroup per CU walks the tiles
// (tile += gridDim.x; the XCD remap keeps each XCD on its own tile range);
// after a tile's main loop the next tile's first four DMA groups are issued
// into the free ring units *before* this tile's epilogue, so they land while
// the epilogue computes and stores.  The next main loop's opening
// `vmcnt(16)` stays correct: waits count ops in issue order, and the
// epilogue's stores are younger than the prefetch.
template <int EPI, int BN, int kWaves, int kFused = 0, int kPersist = 0>
__global__ __launch_bounds__(64 * kWaves, 1) void gemm256_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
    uint16_t* __restrict__ C, const float* __restrict__ bias,
    const uint16_t* __restrict__ R, int M, int N, int K, int lda,
    float* __restrict__ P, int* __restrict__ cnt, int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // split-K: blockIdx.y picks a K/gridDim.y slice (K is the slice length,
  // lda the full row stride); EPI_PARTIAL writes fp32 partials per slice
  const int split = static_cast<int>(blockIdx.y);
  A += static_cast<size_t>(split) * K;
  B += static_cast<size_t>(split) * K;
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  // tile -> its origin: XCD-aware bijective remap, group_m-row grouping
  // (consecutive tiles of an XCD walk group_m tile rows down one tile column
  // before the next column: the B column is re-read from that XCD's L2)
  auto origin = [&](int t, int& om, int& on) {
    const int wg = xcd_remap(t, ntiles);
    const int per_group = group_m * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * group_m;
    const int gsize = min(tiles_m - first_m, group_m);
    const int in_group = wg - group * per_group;
    om = (first_m + in_group % gsize) * BM;
    on = (in_group / gsize) * BN;
  };
  int tile = static_cast<int>(blockIdx.x);
  int m0 = 0, n0 = 0, m0_next = 0, n0_next = 0;
  origin(tile, m0, n0);

  using G = Geo<BN, kWaves>;
  constexpr int TM = G::TM, TN = G::TN, kSlotBytes = G::kSlotBytes;
  constexpr int kLoadsPerHalf = G::kLoadsPerHalf;
  constexpr int kWaitHalf1 = waitcnt_vm(3 * kLoadsPerHalf);
  constexpr int kWaitHalf2 = waitcnt_vm(2 * kLoadsPerHalf);
  constexpr int kWaitAll = waitcnt_vm(0);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave / G::kWavesN, wn = wave % G::kWavesN;
  for (int it = 0;; ++it) {
  // per tile, the lane-derived offsets are recomputed from an opaque lane
  // id (mbcnt, not threadIdx): hoisted out of the persistent tile loop
  // they would stay live across it and spill (no-op for one-tile grids)
  int lane_id = static_cast<int>(threadIdx.x & 63);
  if constexpr (kPersist) {
    lane_id = static_cast<int>(
        __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)));
    asm volatile("" : "+v"(lane_id));
  }
  const int lane = lane_id;
  f32x4 acc[TM][TN];
  if constexpr (kWaves != 4) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int halves = K / BKH;
  // epilogue bias, loaded before the k-loop: its latency is hidden and the
  // tail starts on the arithmetic (lane l owns columns 4(l >> 4)..+3 of
  // each of its 16-wide column tiles)
  float4 bias_pre[TN];
  if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RESIDUAL) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
      bias_pre[j] = *reinterpret_cast<const float4*>(
          bias + n0 + wn * (TN * 16) + j * 16 + (lane >> 4) * 4);
  }
  // Stage half h into its ring slot.  Past the end the source is clamped to
  // the last half (an L2 hit into a slot nobody reads again), so the
  // pipeline has the same shape -- and the same counted wait -- every step.
  auto stage = [&](int h) {
    char* slot = smem + (h & (kSlots - 1)) * kSlotBytes;
    const int k0 = min(h, halves - 1) * BKH;
    stage_operand<G::kPiecesA>(A, lda, m0, M, k0, slot, wave, lane);
    stage_operand<G::kPiecesB>(B, lda, n0, N, k0, slot + G::kABytes, wave,
                               lane);
  };
  const int arow = wm * (TM * 16) + (lane & 15);
  const int brow = wn * (TN * 16) + (lane & 15);
  const int chunk = lane >> 4;
  auto read_frags = [&](int h, bf16x8 (&wb)[TN], bf16x8 (&xa)[TM]) {
    const char* slot = smem + (h & (kSlots - 1)) * kSlotBytes;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      wb[j] = *reinterpret_cast<const bf16x8*>(
          slot + G::kABytes + slot_off(brow + j * 16, chunk));
#pragma unroll
    for (int i = 0; i < TM; ++i)
      xa[i] = *reinterpret_cast<const bf16x8*>(
          slot + slot_off(arow + i * 16, chunk));
  };
  auto mma = [&](const bf16x8 (&wb)[TN], const bf16x8 (&xa)[TM]) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            wb[j], xa[i], acc[i][j], 0, 0, 0);
  };
  // Software pipeline, per half-step h (fragments of half h already in
  // registers; halves h+1..h+3 staged): wait until half h+1 has landed
  // (h+2, h+3 stay in flight) + barrier -- after it no wave still reads the
  // slot of half h -- restage that slot with half h+4, issue the LDS reads
  // of half h+1 into the other register set, and run the 32 MFMAs of half
  // h while the reads and the DMA are in flight.  Branch-free on purpose: a
  // control-flow join between the reads and the MFMAs makes the waitcnt
  // pass drain lgkmcnt first, which serialises the two.
  // SPREAD (BN = 256): the step's DMA pieces and LDS reads are issued in
  // program order as four quarters (pieces, then reads, of quarter q), so
  // hipcc (which keeps LDS-writing DMAs and LDS reads in order) slots a
  // quarter of the MFMAs behind each: no block of 4 DMA issues (~60+ cycles
  // each) ahead of the cluster.  +3..5 % at 256x256, -3..+1 % at 256x128
  // (profiles/r1_gemm/gemm_spread_dma.jsonl), so only the former uses it.
  constexpr bool SPREAD = BN == 256;
  auto stage_q = [&](int h, int q) {
    char* slot = smem + (h & (kSlots - 1)) * kSlotBytes;
    const int k0 = min(h, halves - 1) * BKH;
#pragma unroll
    for (int p = 0; p < kLoadsPerHalf; ++p) {
      if (p * 4 / kLoadsPerHalf != q) continue;
      if (p < G::kPiecesA)
        stage_piece(A, lda, m0, M, k0, slot, wave * G::kPiecesA + p, lane);
      else
        stage_piece(B, lda, n0, N, k0, slot + G::kABytes,
                    wave * G::kPiecesB + (p - G::kPiecesA), lane);
    }
  };
  auto read_q = [&](int h, int q, bf16x8 (&wb)[TN], bf16x8 (&xa)[TM]) {
    const char* slot = smem + (h & (kSlots - 1)) * kSlotBytes;
#pragma unroll
    for (int r = 0; r < G::kReads; ++r) {
      if (r * 4 / G::kReads != q) continue;
      if (r < TN)
        wb[r] = *reinterpret_cast<const bf16x8*>(
            slot + G::kABytes + slot_off(brow + r * 16, chunk));
      else
        xa[r - TN] = *reinterpret_cast<const bf16x8*>(
            slot + slot_off(arow + (r - TN) * 16, chunk));
    }
  };
  // ---- 4-wave main loop (kWaves == 4) --------------------------------
  // Each DMA piece moves 8 whole 128-B rows (one 64-deep K-step of 8 rows:
  // full cache lines; 32-deep half rows cost +6..9 % -- half-line requests,
  // profiles/r1_gemm/gemm_w4_variants.jsonl).  LDS is a ring of 5 units of
  // 32 KiB, one operand (A or B) of one 64-deep step each: group g = 2T + op
  // (op 0 = A, 1 = B, step T) lives in unit g % 5.  The k-loop runs in
  // 32-deep half-steps h (fragments of half h in registers, half h + 1 read
  // from LDS during it); half-step h issues group h + 4 into unit
  // (h + 4) % 5 = (h - 1) % 5, whose data was last read in half-step h - 2
  // (h even) or h - 1 (h odd), both before the barrier opening half-step h.
  // At the start of half-step h, groups 0 .. h + 3 are issued; the reads of
  // half h + 1 need step (h + 1) / 2 resident: groups up to h + 1 (h even,
  // 2 groups = 16 pieces may stay in flight) or h + 2 (h odd, 8 in flight).
  // Every group thus has >= 1 half-step (~1000 MFMA cycles) to land; the
  // half-steps-in-flight probe shows that is enough.  LDS rows are 128 B
  // with 16-B chunk c of row r at c ^ ((r >> 1) & 7): every ds_read_b128
  // lane group then covers 16 distinct bank slots.
  auto mainloop_w4 = [&](auto phase, int steps, bool prefetched) {
    // this wave's DMA slot offset within a half-step (KIOSK_W4_STAGGER)
    constexpr int kOff = decltype(phase)::value;
    constexpr int kUnit = BM * 128;
    int voff_a[8], voff_b[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int r = (wave * 8 + p) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ ((r >> 1) & 7);
      const int ra = m0 + r < M ? m0 + r : M - 1;
      const int rb = n0 + r < N ? n0 + r : N - 1;
      voff_a[p] = (ra * lda + c * 8) * 2;
      voff_b[p] = (rb * lda + c * 8) * 2;
    }
    const auto rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(A), 0, 0x7fffffff, 0x00020000);
    const auto rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t*>(B), 0, 0x7fffffff, 0x00020000);
    // piece p of group g (past the last step the source is clamped to it:
    // same pipeline shape, same counted waits, every step)
    auto dma = [&](int g, int p) {
      const int t = min(g >> 1, steps - 1);
      char* lds = smem + (g % 5) * kUnit + (wave * 8 + p) * 1024;
      if (g & 1)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void_t*)lds, 16,
                                                 voff_b[p], t * 128, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)lds, 16,
                                                 voff_a[p], t * 128, 0, 0);
    };
    // KIOSK_W4_REGSTAGE: piece p of the group in flight, in registers;
    // written to its ring unit three groups before its first read
    // (2: two register buffers by group parity, so a load has two
    // half-steps to land before its write instead of one)
    typedef __attribute__((ext_vector_type(4))) int i32x4;
    constexpr int kBufs = KIOSK_W4_REGSTAGE == 2 ? 2 : 1;
    i32x4 stage[kBufs * 8];
    auto gload = [&](int g, int p, int buf) {
      const int t = min(g >> 1, steps - 1);
      stage[buf * 8 + p] = __builtin_amdgcn_raw_buffer_load_b128(
          (g & 1) ? rsrc_b : rsrc_a, (g & 1) ? voff_b[p] : voff_a[p],
          t * 128, 0);
    };
    const int lane16 = (threadIdx.x & 63) * 16;
    auto swrite = [&](int g, int p, int buf) {
      char* lds = smem + (g % 5) * kUnit + (wave * 8 + p) * 1024 + lane16;
      *reinterpret_cast<i32x4*>(lds) = stage[buf * 8 + p];
    };
    // fragment r of half h: r < TN -> B tile r, else A tile r - TN
    const int fr = lane & 15;
    const int lane_a = (wm * 128 + fr) * 128, lane_b = (wn * 128 + fr) * 128;
    const int sw = (fr >> 1) & 7;
    // per-lane parts of the two halves' read addresses (row + swizzled
    // chunk); the unit base is wave-uniform and the tile offset r * 2048 an
    // immediate, so each read is one ds_read_b128 with offset:N
    const int lane_a0 = lane_a + (((lane >> 4) ^ sw) << 4);
    const int lane_a1 = lane_a + (((4 + (lane >> 4)) ^ sw) << 4);
    const int lane_b0 = lane_b + (((lane >> 4) ^ sw) << 4);
    const int lane_b1 = lane_b + (((4 + (lane >> 4)) ^ sw) << 4);
    auto read = [&](auto hh, int t, int r, bf16x8 (&wb)[TN],
                    bf16x8 (&xa)[TM]) {
      constexpr bool kHi = decltype(hh)::value != 0;
      if (r < TN) {
        const char* base = smem + __builtin_amdgcn_readfirstlane(
                                      ((2 * t + 1) % 5) * kUnit) +
                           (kHi ? lane_b1 : lane_b0);
        wb[r] = *reinterpret_cast<const bf16x8*>(base + r * 2048);
      } else {
        const char* base = smem + __builtin_amdgcn_readfirstlane(
                                      ((2 * t) % 5) * kUnit) +
                           (kHi ? lane_a1 : lane_a0);
        xa[r - TN] = *reinterpret_cast<const bf16x8*>(base + (r - TN) * 2048);
      }
    };
    // half-step h = 2t + odd
    auto half = [&](auto first, auto odd, int t, const bf16x8 (&wb)[TN],
                    const bf16x8 (&xa)[TM], bf16x8 (&wb_next)[TN],
                    bf16x8 (&xa_next)[TM]) {
      constexpr bool kOdd = decltype(odd)::value;
      const int h = 2 * t + kOdd;
      __builtin_amdgcn_sched_barrier(0);
      // regstage: the previous half-step's ds_writes (lgkmcnt 0) must land;
      // the loads in flight are waited for by each write (compiler vmcnt)
      __builtin_amdgcn_s_waitcnt(
          waitcnt_vm(KIOSK_W4_REGSTAGE ? 63 : (kOdd ? 8 : 16)));
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      // half h + 1: step t (h even, second half) or t + 1 (h odd, first)
      const int tn = kOdd ? t + 1 : t;
      using HH = std::integral_constant<int, kOdd ? 0 : 1>;
      // one DMA piece every 8 MFMAs, one LDS read every 4: each issue sits
      // in an MFMA gap, none stalls the matrix pipe behind a block of them
#pragma unroll
      for (int u = 0; u < TM * TN; ++u) {
        if constexpr (decltype(first)::value)
          mfma_agpr_first(acc[u / TN][u % TN], wb[u % TN], xa[u / TN]);
        else
          mfma_agpr(acc[u / TN][u % TN], wb[u % TN], xa[u / TN]);
        if constexpr (KIOSK_W4_SPREAD == 0) {
          if constexpr (!(KIOSK_GEMM_ABLATE & 1))
            if (u % 8 == 0) dma(h + 4, u / 8);
          if constexpr (!(KIOSK_GEMM_ABLATE & 2))
            if (u % 4 == 2) read(HH(), tn, u / 4, wb_next, xa_next);
        } else {
          // all issues in the first 48 MFMAs: the last LDS read has 16
          // MFMAs (~256 cycles) to return before the next half-step's
          // lgkmcnt(0) + barrier
          if constexpr (!(KIOSK_GEMM_ABLATE & 1))
            if (u >= kOff && (u - kOff) % 6 == 0 && (u - kOff) < 48) {
              if constexpr (KIOSK_W4_REGSTAGE == 1) {
                swrite(h + 3, (u - kOff) / 6, 0);
                gload(h + 4, (u - kOff) / 6, 0);
              } else if constexpr (KIOSK_W4_REGSTAGE == 2) {
                // group h + 3 leaves buffer (h + 3) % 2, group h + 5 refills it
                constexpr int kBuf = kOdd ? 0 : 1;
                swrite(h + 3, (u - kOff) / 6, kBuf);
                gload(h + 5, (u - kOff) / 6, kBuf);
              } else {
                dma(h + 4, (u - kOff) / 6);
              }
            }
          if constexpr (!(KIOSK_GEMM_ABLATE & 2))
            if (u % 3 == 1 && u < 48) read(HH(), tn, u / 3, wb_next, xa_next);
        }
      }
    };
    if (!prefetched) {
#pragma unroll
      for (int g = 0; g < (KIOSK_W4_REGSTAGE ? 3 : 4); ++g)
#pragma unroll
        for (int p = 0; p < 8; ++p) dma(g, p);
    }
    if constexpr (KIOSK_W4_REGSTAGE) {
      // group 3 (and 4) go through the registers (written in half-step 0, 1)
#pragma unroll
      for (int p = 0; p < 8; ++p) gload(3, p, kBufs == 2 ? 1 : 0);
      if constexpr (kBufs == 2) {
#pragma unroll
        for (int p = 0; p < 8; ++p) gload(4, p, 0);
      }
    }
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(16));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 wb0[TN], xa0[TM], wb1[TN], xa1[TM];
#pragma unroll
    for (int r = 0; r < TM + TN; ++r)
      read(std::integral_constant<int, 0>(), 0, r, wb0, xa0);
    half(std::true_type(), std::false_type(), 0, wb0, xa0, wb1, xa1);
    half(std::false_type(), std::true_type(), 0, wb1, xa1, wb0, xa0);
    for (int t = 1; t < steps; ++t) {
      half(std::false_type(), std::false_type(), t, wb0, xa0, wb1, xa1);
      half(std::false_type(), std::true_type(), t, wb1, xa1, wb0, xa0);
    }
  };
  auto step = [&](int h, const bf16x8 (&wb)[TN], const bf16x8 (&xa)[TM],
                  bf16x8 (&wb_next)[TN], bf16x8 (&xa_next)[TM]) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(kWaitHalf2);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (SPREAD) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        stage_q(h + 4, q);
        read_q(h + 1, q, wb_next, xa_next);
      }
    } else {
      stage(h + 4);
      read_frags(h + 1, wb_next, xa_next);
    }
    mma(wb, xa);
    // spread the next half's LDS reads through the MFMA cluster: per
    // quarter a quarter of the ds_read_b128s, then a quarter of the MFMAs.
    // Measured +1..4 % over issuing all 12 reads ahead of the cluster
    // (profiles/r1_gemm/gemm_ab_swizzle_interleave.jsonl).
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (SPREAD) {
        // builtin arguments must be literal constants: one call per quarter
        constexpr int c0 = per_quarter(kLoadsPerHalf, 0);
        constexpr int c1 = per_quarter(kLoadsPerHalf, 1);
        constexpr int c2 = per_quarter(kLoadsPerHalf, 2);
        constexpr int c3 = per_quarter(kLoadsPerHalf, 3);
        if (q == 0 && c0) __builtin_amdgcn_sched_group_barrier(0x010, c0, 0);
        if (q == 1 && c1) __builtin_amdgcn_sched_group_barrier(0x010, c1, 0);
        if (q == 2 && c2) __builtin_amdgcn_sched_group_barrier(0x010, c2, 0);
        if (q == 3 && c3) __builtin_amdgcn_sched_group_barrier(0x010, c3, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, G::kReads / 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, TM * TN / 4, 0);
    }
  };

  if constexpr (kWaves == 4) {
    using P0 = std::integral_constant<int, 0>;
    if constexpr (KIOSK_W4_STAGGER == 2 && !kPersist) {
      if (KIOSK_W4_STAGGER_SEL ? (wave >> 1) & 1 : wave & 1)
        mainloop_w4(std::integral_constant<int, KIOSK_W4_STAGGER_OFF>(),
                    K / 64, kPersist && it > 0);
      else
        mainloop_w4(P0(), K / 64, kPersist && it > 0);
    } else if constexpr (KIOSK_W4_STAGGER == 4 && !kPersist) {
      switch (wave & 3) {
        case 0: mainloop_w4(P0(), K / 64, kPersist && it > 0); break;
        case 1:
          mainloop_w4(std::integral_constant<int, 1>(), K / 64,
                      kPersist && it > 0);
          break;
        case 2:
          mainloop_w4(std::integral_constant<int, 3>(), K / 64,
                      kPersist && it > 0);
          break;
        default:
          mainloop_w4(std::integral_constant<int, 4>(), K / 64,
                      kPersist && it > 0);
      }
    } else {
      mainloop_w4(P0(), K / 64, kPersist && it > 0);
    }
  } else {
#pragma unroll
    for (int h = 0; h < kSlots; ++h) stage(h);
    __builtin_amdgcn_s_waitcnt(kWaitHalf1);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 wb0[TN], xa0[TM], wb1[TN], xa1[TM];
    read_frags(0, wb0, xa0);
    for (int h = 0; h < halves; h += 2) {
      step(h, wb0, xa0, wb1, xa1);
      if (h + 1 < halves) step(h + 1, wb1, xa1, wb0, xa0);
    }
  }
  // drain the tail DMAs before the workgroup's LDS can be released
  __builtin_amdgcn_s_waitcnt(kWaitAll);
  if constexpr (kWaves == 4) {
    mfma_drain();
    // every accumulator is re-defined after the drain, so no read of one
    // (epilogue or spill) can be scheduled between its last MFMA and the
    // wait states hipcc does not insert for asm MFMAs
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+a"(acc[i][j]));
  }
  if constexpr (kPersist) {
    // the next tile's groups 0..3 (units 0..3) under this tile's epilogue;
    // every wave is past its last LDS read and the tail DMAs have drained
    // (vmcnt(0) above), so no unit is still read or written
    // branch-free (a branch here splits the 256 live accumulators'
    // ranges and spills): past the last tile the prefetch re-reads this
    // tile's first groups into units nobody reads; the kernel drains them
    // before it exits
    {
      int next = tile + static_cast<int>(gridDim.x);
      next = next < ntiles ? next : tile;
      origin(next, m0_next, n0_next);
      __builtin_amdgcn_s_barrier();
      constexpr int kUnit = BM * 128;
      const int steps = K / 64;
      const auto rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(A), 0, 0x7fffffff, 0x00020000);
      const auto rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint16_t*>(B), 0, 0x7fffffff, 0x00020000);
      // group-major, as the main loop's prologue: groups 0-1 are the
      // oldest 16 ops its opening vmcnt(16) waits for.  Offsets are
      // computed per issue (no arrays live across the epilogue), and the
      // block is fenced off from the epilogue's scheduling
      __builtin_amdgcn_sched_barrier(0);
      int plane = static_cast<int>(
          __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)));
      asm volatile("" : "+v"(plane));   // derived here, not before the loop
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int t = min(g >> 1, steps - 1);
        const int row0 = (g & 1) ? n0_next : m0_next;
        const int rows = (g & 1) ? N : M;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          const int r = (wave * 8 + p) * 8 + (plane >> 3);
          const int c = (plane & 7) ^ ((r >> 1) & 7);
          const int gr = row0 + r < rows ? row0 + r : rows - 1;
          char* lds = smem + g * kUnit + (wave * 8 + p) * 1024;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              (g & 1) ? rsrc_b : rsrc_a, (lds_void_t*)lds, 16,
              (gr * lda + c * 8) * 2, t * 128, 0, 0);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // Epilogue.  Lane l holds row (l & 15), columns 4g..4g+3 (g = l >> 4) of
  // every 16x16 tile.  Lanes l and l ^ 16 (same row, column groups g and
  // g ^ 1) swap one tile's half of a tile pair (v_permlane16_swap, a VALU
  // op), so every lane then owns 8 consecutive columns and issues one 16-B
  // store where it issued two 8-B ones: the epilogue is store-issue-bound
  // (guide T21).
  auto finish = [&](int m, int nb, int j, const f32x4& a, float (&v)[4]) {
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    if constexpr (kFused) {
      // the other slice's plane
      const size_t plane = static_cast<size_t>(split ^ 1);
      const float4 q = *reinterpret_cast<const float4*>(
          P + plane * M * N + static_cast<size_t>(m) * N + nb);
      v[0] += q.x; v[1] += q.y; v[2] += q.z; v[3] += q.w;
    }
    if (EPI != EPI_NONE) {
      const float4 b = bias_pre[j];
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if (EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
    }
    if (EPI == EPI_BIAS_RESIDUAL) {
      const uint2 res = *reinterpret_cast<const uint2*>(
          R + static_cast<size_t>(m) * N + nb);
      v[0] += bf16_to_f32(res.x & 0xffff);
      v[1] += bf16_to_f32(res.x >> 16);
      v[2] += bf16_to_f32(res.y & 0xffff);
      v[3] += bf16_to_f32(res.y >> 16);
    }
  };
  auto pack2 = [](float lo, float hi) {
    return f32_to_bf16(lo) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
  };
  const int g = lane >> 4;
  const bool odd = (g & 1) != 0;
  if constexpr (kFused == 1) {
    // In-launch split-K combine (cdna_hip_programming.md §5, projection
    // GEMM item 2): plain 16-B partial stores -> every wave vmcnt(0) ->
    // barrier -> one lane: agent-scope release fence, vmcnt(0), relaxed
    // agent-scope ticket; the block drawing splits - 1 acquires and reads
    // the other slices.  Correct for any placement of a tile's slices;
    // the counters are zeroed by a memset ahead of every launch.
    const size_t plane = static_cast<size_t>(M) * N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
      if (m >= M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nb = n0 + wn * (TN * 16) + j * 16 + g * 4;
        *reinterpret_cast<float4*>(P + split * plane +
                                   static_cast<size_t>(m) * N + nb) =
            float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      }
      // one row of tiles at a time: bounds the AGPR -> VGPR copies
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = reinterpret_cast<int*>(smem);   // the one LDS array
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int ticket = __hip_atomic_fetch_add(
          cnt + blockIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = ticket == static_cast<int>(gridDim.y) - 1;
      if (is_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
    // the reducer adds its own and the other slice's partial tile by tile
    // in the epilogue below (two K slices only: the host launches the
    // fused path for splits == 2)
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    // m is the same for lanes l and l ^ 16, so a skipped row skips both
    // partners of every exchange below
    const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nb = n0 + wn * (TN * 16) + j * 16 + g * 4;
      if (EPI == EPI_PARTIAL) {
        float* P = reinterpret_cast<float*>(C) +
                   static_cast<size_t>(split) * M * N;
        *reinterpret_cast<float4*>(P + static_cast<size_t>(m) * N + nb) =
            float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      }
    }
    if (EPI == EPI_PARTIAL) continue;
#pragma unroll
    for (int jp = 0; jp < TN; jp += 2) {
      const int base = n0 + wn * (TN * 16) + jp * 16;
      float v0[4], v1[4];
      if constexpr (kFused == 1) {
        // the reducer re-reads its own partial (L2-warm) instead of
        // keeping 256 accumulators live across the ticket
        const size_t own = static_cast<size_t>(split) * M * N +
                           static_cast<size_t>(m) * N;
        const float4 p0 = *reinterpret_cast<const float4*>(P + own + base +
                                                           g * 4);
        const float4 p1 = *reinterpret_cast<const float4*>(P + own + base +
                                                           16 + g * 4);
        finish(m, base + g * 4, jp, f32x4{p0.x, p0.y, p0.z, p0.w}, v0);
        finish(m, base + 16 + g * 4, jp + 1, f32x4{p1.x, p1.y, p1.z, p1.w},
               v1);
      } else {
        finish(m, base + g * 4, jp, acc[i][jp], v0);
        finish(m, base + 16 + g * 4, jp + 1, acc[i][jp + 1], v1);
      }
      // v_permlane16_swap(X, Y) swaps the odd 16-lane rows of X with the
      // even rows of Y.  With X = this lane's tile-jp half and Y = its
      // tile-(jp+1) half, even rows end with {own jp, partner's jp} and odd
      // rows with {partner's jp+1, own jp+1}: both are {X', Y'}.
      const auto x0 = __builtin_amdgcn_permlane16_swap(
          pack2(v0[0], v0[1]), pack2(v1[0], v1[1]), false, false);
      const auto x1 = __builtin_amdgcn_permlane16_swap(
          pack2(v0[2], v0[3]), pack2(v1[2], v1[3]), false, false);
      const uint4 out = uint4{x0[0], x1[0], x0[1], x1[1]};
      const int col = odd ? base + 16 + (g - 1) * 4 : base + g * 4;
      *reinterpret_cast<uint4*>(C + static_cast<size_t>(m) * N + col) = out;
    }
  }
  if constexpr (!kPersist) {
    break;
  } else {
    tile += static_cast<int>(gridDim.x);
    if (tile >= ntiles) {
      // the last prefetch must land before the workgroup's LDS is freed
      __builtin_amdgcn_s_waitcnt(kWaitAll);
      break;
    }
    m0 = m0_next;
    n0 = n0_next;
  }
  }  // tile loop
}

// tile rows per group of the 256-row kernels' tile order (gemm_set_group_m)
int g_group_m = 4;


// ---------------------------------------------------------------------------
// 4-wave 256x256 tile on v_mfma_f32_32x32x16_bf16 (gemm_set_mfma32).  The
// ring, the DMA rate (8 pieces per half-step), the swizzle and the counted
// waits are the 4-wave kernel's above; a half-step
// runs 32 MFMAs of 32x32x16 instead of 64 of 16x16x32.  Each keeps the
// matrix pipe busy for 32 cycles, so a wave held by an LDS-DMA issue stalls
// the pipe for less of it (profiles/r4_mfma_dma: the same schedule on
// register operands runs 7 % faster).  Per wave a 128x128 output in 4x4
// tiles of 32x32 (16 AGPRs each); per 32-deep half-step two k-substeps of
// 16.  Operands swapped as in the 4-wave kernel (C^T in the accumulators):
// lane l holds, of tile (i, j), output row (l & 31) and the columns
// 8b + 4(l >> 5) + 0..3, b = 0..3, of the tile's 32.  Fragment reads:
// row (l & 31), 16-B chunk 2ks + (l >> 5) (+4 in a step's upper half):
// 16 distinct bank groups in every ds_read_b128 lane group under the
// ring's (r >> 1) & 7 swizzle.
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ void mfma32_agpr(f32x16& acc, const bf16x8& a,
                                            const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
               : "+a"(acc)
               : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma32_agpr_first(f32x16& acc,
                                                  const bf16x8& a,
                                                  const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0"
               : "=a"(acc)
               : "v"(a), "v"(b));
}

template <int EPI>
__global__ __launch_bounds__(256, 1) void gemm256m32_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
    uint16_t* __restrict__ C, const float* __restrict__ bias,
    const uint16_t* __restrict__ R, int M, int N, int K, int lda,
    int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int split = static_cast<int>(blockIdx.y);
  A += static_cast<size_t>(split) * K;
  B += static_cast<size_t>(split) * K;
  const int tiles_n = N / 256;
  const int tiles_m = (M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  int m0 = 0, n0 = 0;
  {
    const int wg = xcd_remap(static_cast<int>(blockIdx.x), ntiles);
    const int per_group = group_m * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * group_m;
    const int gsize = min(tiles_m - first_m, group_m);
    const int in_group = wg - group * per_group;
    m0 = (first_m + in_group % gsize) * BM;
    n0 = (in_group / gsize) * 256;
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int lane = static_cast<int>(threadIdx.x & 63);
  constexpr int kUnit = BM * 128;
  const int steps = K / 64;
  f32x16 acc[4][4];

  int voff_a[8], voff_b[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const int r = (wave * 8 + p) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int ra = m0 + r < M ? m0 + r : M - 1;
    const int rb = n0 + r < N ? n0 + r : N - 1;
    voff_a[p] = (ra * lda + c * 8) * 2;
    voff_b[p] = (rb * lda + c * 8) * 2;
  }
  const auto rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(A), 0, 0x7fffffff, 0x00020000);
  const auto rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(B), 0, 0x7fffffff, 0x00020000);
  // piece p of group g = operand (g & 1: B) of 64-deep step g >> 1, clamped
  // to the last step past the end (same pipeline shape every step)
  auto dma = [&](int g, int p) {
    const int t = min(g >> 1, steps - 1);
    char* lds = smem + (g % 5) * kUnit + (wave * 8 + p) * 1024;
    if (g & 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void_t*)lds, 16,
                                               voff_b[p], t * 128, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)lds, 16,
                                               voff_a[p], t * 128, 0, 0);
  };
  const int fr = lane & 31;
  const int sw = (fr >> 1) & 7;
  const int hk = lane >> 5;
  const int row_a = (wm * 128 + fr) * 128, row_b = (wn * 128 + fr) * 128;
  // [upper half][k-substep] -> this lane's byte offset in a unit
  int off_a[2][2], off_b[2][2];
#pragma unroll
  for (int hi = 0; hi < 2; ++hi)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ((hi * 4 + ks * 2 + hk) ^ sw) << 4;
      off_a[hi][ks] = row_a + chunk;
      off_b[hi][ks] = row_b + chunk;
    }
  // fragment r of a half: r < 8 -> B (k-substep r >> 2, tile r & 3), else A
  auto read = [&](auto hh, int t, int r, bf16x8 (&wb)[2][4],
                  bf16x8 (&xa)[2][4]) {
    constexpr int kHi = decltype(hh)::value;
    const int ks = (r >> 2) & 1, idx = r & 3;
    if (r < 8) {
      const char* base = smem + __builtin_amdgcn_readfirstlane(
                                    ((2 * t + 1) % 5) * kUnit) +
                         off_b[kHi][ks];
      wb[ks][idx] = *reinterpret_cast<const bf16x8*>(base + idx * 4096);
    } else {
      const char* base = smem + __builtin_amdgcn_readfirstlane(
                                    ((2 * t) % 5) * kUnit) +
                         off_a[kHi][ks];
      xa[ks][idx] = *reinterpret_cast<const bf16x8*>(base + idx * 4096);
    }
  };
  auto half = [&](auto first, auto odd, int t, const bf16x8 (&wb)[2][4],
                  const bf16x8 (&xa)[2][4], bf16x8 (&wb_next)[2][4],
                  bf16x8 (&xa_next)[2][4]) {
    constexpr bool kOdd = decltype(odd)::value;
    const int h = 2 * t + kOdd;
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(kOdd ? 8 : 16));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int tn = kOdd ? t + 1 : t;
    using HH = std::integral_constant<int, kOdd ? 0 : 1>;
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int ks = u >> 4, i = (u >> 2) & 3, j = u & 3;
      if constexpr (decltype(first)::value) {
        if (ks == 0)
          mfma32_agpr_first(acc[i][j], wb[ks][j], xa[ks][i]);
        else
          mfma32_agpr(acc[i][j], wb[ks][j], xa[ks][i]);
      } else {
        mfma32_agpr(acc[i][j], wb[ks][j], xa[ks][i]);
      }
      // a DMA piece every 4 MFMAs; the 16 reads of the next half-step in
      // the first 24 MFMAs (two of every three), so the last one has 8
      // MFMAs (~256 cycles) to land before the next half's lgkmcnt(0)
      if (u % 4 == 1) dma(h + 4, u / 4);
      if (u < 24 && u % 3 != 2) read(HH(), tn, (u / 3) * 2 + u % 3, wb_next,
                                     xa_next);
    }
  };
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int p = 0; p < 8; ++p) dma(g, p);
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(16));
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  bf16x8 wb0[2][4], xa0[2][4], wb1[2][4], xa1[2][4];
#pragma unroll
  for (int r = 0; r < 16; ++r)
    read(std::integral_constant<int, 0>(), 0, r, wb0, xa0);
  half(std::true_type(), std::false_type(), 0, wb0, xa0, wb1, xa1);
  half(std::false_type(), std::true_type(), 0, wb1, xa1, wb0, xa0);
  for (int t = 1; t < steps; ++t) {
    half(std::false_type(), std::false_type(), t, wb0, xa0, wb1, xa1);
    half(std::false_type(), std::true_type(), t, wb1, xa1, wb0, xa0);
  }
  // drain the tail DMAs before the workgroup's LDS can be released
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  mfma_drain();
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+a"(acc[i][j]));

  auto pack2 = [](float lo, float hi) {
    return f32_to_bf16(lo) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
  };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 128 + i * 32 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int n = n0 + wn * 128 + j * 32 + b * 8 + hk * 4;
        float v[4] = {acc[i][j][4 * b], acc[i][j][4 * b + 1],
                      acc[i][j][4 * b + 2], acc[i][j][4 * b + 3]};
        if (EPI == EPI_PARTIAL) {
          float* P = reinterpret_cast<float*>(C) +
                     static_cast<size_t>(split) * M * N;
          *reinterpret_cast<float4*>(P + static_cast<size_t>(m) * N + n) =
              float4{v[0], v[1], v[2], v[3]};
          continue;
        }
        if (EPI != EPI_NONE) {
          const float4 bb = *reinterpret_cast<const float4*>(bias + n);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        }
        if (EPI == EPI_BIAS_GELU) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
        }
        if (EPI == EPI_BIAS_RESIDUAL) {
          const uint2 res = *reinterpret_cast<const uint2*>(
              R + static_cast<size_t>(m) * N + n);
          v[0] += bf16_to_f32(res.x & 0xffff);
          v[1] += bf16_to_f32(res.x >> 16);
          v[2] += bf16_to_f32(res.y & 0xffff);
          v[3] += bf16_to_f32(res.y >> 16);
        }
        *reinterpret_cast<uint2*>(C + static_cast<size_t>(m) * N + n) =
            uint2{pack2(v[0], v[1]), pack2(v[2], v[3])};
      }
    }
    // one row of tiles at a time: bounds the AGPR -> VGPR copies
    __builtin_amdgcn_sched_barrier(0);
  }
}

// 0: the 16x16x32 4-wave kernel; 1: gemm256m32_kernel wherever the 4-wave
// one-tile kernel runs (plain, fused epilogues, split-K partials)
int g_mfma32 = 0;

template <int EPI>
hipError_t configure_m32() {
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm256m32_kernel<EPI>),
      hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256, 4>::kLdsBytes);
  return err == hipSuccess ? prepare_kernel(&gemm256m32_kernel<EPI>) : err;
}

hipError_t launch_m32(const uint16_t* A, const uint16_t* B, uint16_t* C,
                      const float* bias, const uint16_t* R, int M, int N,
                      int K, int lda, int splits, int epilogue,
                      hipStream_t stream) {
  const int blocks = ((M + BM - 1) / BM) * (N / 256);
  const dim3 grid(blocks, splits), block(256);
  constexpr int lds = Geo<256, 4>::kLdsBytes;
  switch (epilogue) {
    case EPI_NONE:
      return launch_kernel(&gemm256m32_kernel<EPI_NONE>, grid, block, lds,
                           stream, A, B, C, bias, R, M, N, K, lda, g_group_m);
    case EPI_BIAS_GELU:
      return launch_kernel(&gemm256m32_kernel<EPI_BIAS_GELU>, grid, block,
                           lds, stream, A, B, C, bias, R, M, N, K, lda,
                           g_group_m);
    case EPI_BIAS_RESIDUAL:
      return launch_kernel(&gemm256m32_kernel<EPI_BIAS_RESIDUAL>, grid, block,
                           lds, stream, A, B, C, bias, R, M, N, K, lda,
                           g_group_m);
    case EPI_PARTIAL:
      return launch_kernel(&gemm256m32_kernel<EPI_PARTIAL>, grid, block, lds,
                           stream, A, B, C, bias, R, M, N, K, lda, g_group_m);
    default:
      return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// Two waves per SIMD (gemm_set_pair): the 4-wave
// kernel's 256x256 tile, ring, swizzle and counted waits with 8 waves of
// 128x64 outputs each (2 x 4 waves, 8 x 4 tiles of v_mfma_f32_16x16x32_bf16,
// 128 AGPRs).  The 4-wave kernel loses ~20 % of the matrix pipe to its own
// LDS-DMA issue: one wave per SIMD has nothing to run while its DMA issue
// holds it (profiles/r4_mfma_dma, the ablation's +21 % without in-loop
// DMA).  Here a wave issues half the DMA pieces (4 per half-step) and its
// SIMD partner's MFMAs run while it is held.  The partners are staggered
// (waves 4-7 issue their DMA later in the half-step, MI355X_MICROARCH.md
// "Two waves per SIMD" item 9) so they are not both held at once.  LDS
// reads per CU rise from 64 to 96 KiB per half-step (384 of the 1024
// cycles at 256 B/clk) -- within the array's budget.
template <int EPI, int kStagger, int kPrio>
__global__ __launch_bounds__(512, 1) void gemm256p_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
    uint16_t* __restrict__ C, const float* __restrict__ bias,
    const uint16_t* __restrict__ R, int M, int N, int K, int lda,
    int group_m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int TM = 8, TN = 4;            // 16x16 tiles per wave
  const int split = static_cast<int>(blockIdx.y);
  A += static_cast<size_t>(split) * K;
  B += static_cast<size_t>(split) * K;
  const int tiles_n = N / 256;
  const int tiles_m = (M + BM - 1) / BM;
  const int ntiles = tiles_m * tiles_n;
  int m0 = 0, n0 = 0;
  {
    const int wg = xcd_remap(static_cast<int>(blockIdx.x), ntiles);
    const int per_group = group_m * tiles_n;
    const int group = wg / per_group;
    const int first_m = group * group_m;
    const int gsize = min(tiles_m - first_m, group_m);
    const int in_group = wg - group * per_group;
    m0 = (first_m + in_group % gsize) * BM;
    n0 = (in_group / gsize) * 256;
  }
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int lane = static_cast<int>(threadIdx.x & 63);
  constexpr int kUnit = BM * 128;
  const int steps = K / 64;
  f32x4 acc[TM][TN];

  // a group (one operand of one 64-deep step) is 32 pieces of 8 rows x
  // 128 B; wave w issues pieces 4w .. 4w + 3 (the 4-wave kernel's LDS image)
  int voff_a[4], voff_b[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = (wave * 4 + p) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int ra = m0 + r < M ? m0 + r : M - 1;
    const int rb = n0 + r < N ? n0 + r : N - 1;
    voff_a[p] = (ra * lda + c * 8) * 2;
    voff_b[p] = (rb * lda + c * 8) * 2;
  }
  const auto rsrc_a = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(A), 0, 0x7fffffff, 0x00020000);
  const auto rsrc_b = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(B), 0, 0x7fffffff, 0x00020000);
  auto dma = [&](int g, int p) {
    const int t = min(g >> 1, steps - 1);
    char* lds = smem + (g % 5) * kUnit + (wave * 4 + p) * 1024;
    if (g & 1)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_b, (lds_void_t*)lds, 16,
                                               voff_b[p], t * 128, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc_a, (lds_void_t*)lds, 16,
                                               voff_a[p], t * 128, 0, 0);
  };
  const int fr = lane & 15;
  const int sw = (fr >> 1) & 7;
  const int lane_a = (wm * 128 + fr) * 128, lane_b = (wn * 64 + fr) * 128;
  const int lane_a0 = lane_a + (((lane >> 4) ^ sw) << 4);
  const int lane_a1 = lane_a + (((4 + (lane >> 4)) ^ sw) << 4);
  const int lane_b0 = lane_b + (((lane >> 4) ^ sw) << 4);
  const int lane_b1 = lane_b + (((4 + (lane >> 4)) ^ sw) << 4);
  // fragment r of half h: r < TN -> B tile r, else A tile r - TN
  auto read = [&](auto hh, int t, int r, bf16x8 (&wb)[TN],
                  bf16x8 (&xa)[TM]) {
    constexpr bool kHi = decltype(hh)::value != 0;
    if (r < TN) {
      const char* base = smem + __builtin_amdgcn_readfirstlane(
                                    ((2 * t + 1) % 5) * kUnit) +
                         (kHi ? lane_b1 : lane_b0);
      wb[r] = *reinterpret_cast<const bf16x8*>(base + r * 2048);
    } else {
      const char* base = smem + __builtin_amdgcn_readfirstlane(
                                    ((2 * t) % 5) * kUnit) +
                         (kHi ? lane_a1 : lane_a0);
      xa[r - TN] = *reinterpret_cast<const bf16x8*>(base + (r - TN) * 2048);
    }
  };
  // half-step h = 2t + odd: 32 MFMAs; the 4 DMA pieces of group h + 4 at
  // MFMAs kOff + 0, 5, 10, 15 (waves 4-7 later than 0-3); the 12 reads of
  // half h + 1 in the first 24 MFMAs (every other one)
  auto half = [&](auto first, auto odd, auto off, int t,
                  const bf16x8 (&wb)[TN], const bf16x8 (&xa)[TM],
                  bf16x8 (&wb_next)[TN], bf16x8 (&xa_next)[TM]) {
    constexpr bool kOdd = decltype(odd)::value;
    constexpr int kOff = decltype(off)::value;
    const int h = 2 * t + kOdd;
    __builtin_amdgcn_sched_barrier(0);
    // (lgkmcnt 0 too: every LDS read of this wave has returned before
    // the barrier lets another wave's DMA reuse a unit)
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(kOdd ? 4 : 8));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    const int tn = kOdd ? t + 1 : t;
    using HH = std::integral_constant<int, kOdd ? 0 : 1>;
#pragma unroll
    for (int u = 0; u < TM * TN; ++u) {
      if constexpr (decltype(first)::value)
        mfma_agpr_first(acc[u / TN][u % TN], wb[u % TN], xa[u / TN]);
      else
        mfma_agpr(acc[u / TN][u % TN], wb[u % TN], xa[u / TN]);
      if (u >= kOff && (u - kOff) % 5 == 0 && (u - kOff) < 20)
        dma(h + 4, (u - kOff) / 5);
      if (u % 2 == 0 && u < 24) read(HH(), tn, u / 2, wb_next, xa_next);
    }
  };
  auto mainloop = [&](auto off) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int p = 0; p < 4; ++p) dma(g, p);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(8));
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    bf16x8 wb0[TN], xa0[TM], wb1[TN], xa1[TM];
#pragma unroll
    for (int r = 0; r < TM + TN; ++r)
      read(std::integral_constant<int, 0>(), 0, r, wb0, xa0);
    half(std::true_type(), std::false_type(), off, 0, wb0, xa0, wb1, xa1);
    half(std::false_type(), std::true_type(), off, 0, wb1, xa1, wb0, xa0);
    for (int t = 1; t < steps; ++t) {
      half(std::false_type(), std::false_type(), off, t, wb0, xa0, wb1, xa1);
      half(std::false_type(), std::true_type(), off, t, wb1, xa1, wb0, xa0);
    }
  };
  if (wave >= 4) {
    // static priority for the later-dispatched half (MI355X_MICROARCH.md
    // "Two waves per SIMD" item 4): one s_setprio before the loop
    if constexpr (kPrio) __builtin_amdgcn_s_setprio(1);
    mainloop(std::integral_constant<int, kStagger>());
  } else {
    mainloop(std::integral_constant<int, 0>());
  }
  // drain the tail DMAs before the workgroup's LDS can be released
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
  mfma_drain();
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+a"(acc[i][j]));

  // Epilogue: the 4-wave kernel's (lane l: row l & 15, columns 4(l >> 4)..
  // +3 of each 16x16 tile; v_permlane16_swap pairs -> 16-B stores)
  auto pack2 = [](float lo, float hi) {
    return f32_to_bf16(lo) | (static_cast<uint32_t>(f32_to_bf16(hi)) << 16);
  };
  const int g = lane >> 4;
  const bool odd = (g & 1) != 0;
  auto finish = [&](int m, int nb, const f32x4& a, float (&v)[4]) {
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    if (EPI != EPI_NONE) {
      const float4 b = *reinterpret_cast<const float4*>(bias + nb);
      v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
    }
    if (EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
    }
    if (EPI == EPI_BIAS_RESIDUAL) {
      const uint2 res = *reinterpret_cast<const uint2*>(
          R + static_cast<size_t>(m) * N + nb);
      v[0] += bf16_to_f32(res.x & 0xffff);
      v[1] += bf16_to_f32(res.x >> 16);
      v[2] += bf16_to_f32(res.y & 0xffff);
      v[3] += bf16_to_f32(res.y >> 16);
    }
  };
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
    if (m >= M) continue;
    if (EPI == EPI_PARTIAL) {
      float* P = reinterpret_cast<float*>(C) +
                 static_cast<size_t>(split) * M * N;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nb = n0 + wn * (TN * 16) + j * 16 + g * 4;
        *reinterpret_cast<float4*>(P + static_cast<size_t>(m) * N + nb) =
            float4{acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      }
      __builtin_amdgcn_sched_barrier(0);
      continue;
    }
#pragma unroll
    for (int jp = 0; jp < TN; jp += 2) {
      const int base = n0 + wn * (TN * 16) + jp * 16;
      float v0[4], v1[4];
      finish(m, base + g * 4, acc[i][jp], v0);
      finish(m, base + 16 + g * 4, acc[i][jp + 1], v1);
      const auto x0 = __builtin_amdgcn_permlane16_swap(
          pack2(v0[0], v0[1]), pack2(v1[0], v1[1]), false, false);
      const auto x1 = __builtin_amdgcn_permlane16_swap(
          pack2(v0[2], v0[3]), pack2(v1[2], v1[3]), false, false);
      const uint4 out = uint4{x0[0], x1[0], x0[1], x1[1]};
      const int col = odd ? base + 16 + (g - 1) * 4 : base + g * 4;
      *reinterpret_cast<uint4*>(C + static_cast<size_t>(m) * N + col) = out;
    }
    // one row of tiles at a time: bounds the AGPR -> VGPR copies
    __builtin_amdgcn_sched_barrier(0);
  }
}

// 0: one wave per SIMD (gemm256_kernel<., 256, 4>); 1: gemm256p_kernel
// wherever the 4-wave one-tile kernel runs -- an A/B arm, off: it measured
// 0.6 % faster on the plain up-projection and 2.5-4 % slower everywhere
// else (profiles/r6_gemm_pair/)
int g_pair = 0;
// the best of the five stagger / priority arms measured: waves 4-7 start
// their DMA at MFMA 12 of a half-step and run at s_setprio 1
constexpr int kPairStagger = 12, kPairPrio = 1;

template <int EPI>
hipError_t configure_pair() {
  constexpr auto k = &gemm256p_kernel<EPI, kPairStagger, kPairPrio>;
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(k),
      hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256, 4>::kLdsBytes);
  return err == hipSuccess ? prepare_kernel(k) : err;
}

template <int EPI>
hipError_t launch_pair_epi(const uint16_t* A, const uint16_t* B, uint16_t* C,
                           const float* bias, const uint16_t* R, int M, int N,
                           int K, int lda, int splits, hipStream_t stream) {
  const int blocks = ((M + BM - 1) / BM) * (N / 256);
  const dim3 grid(blocks, splits), block(512);
  constexpr int lds = Geo<256, 4>::kLdsBytes;
  return launch_kernel(&gemm256p_kernel<EPI, kPairStagger, kPairPrio>, grid,
                       block, lds, stream, A, B, C, bias, R, M, N, K, lda,
                       g_group_m);
}

hipError_t launch_pair(const uint16_t* A, const uint16_t* B, uint16_t* C,
                       const float* bias, const uint16_t* R, int M, int N,
                       int K, int lda, int splits, int epilogue,
                       hipStream_t stream) {
  switch (epilogue) {
    case EPI_NONE:
      return launch_pair_epi<EPI_NONE>(A, B, C, bias, R, M, N, K, lda, splits,
                                       stream);
    case EPI_BIAS_GELU:
      return launch_pair_epi<EPI_BIAS_GELU>(A, B, C, bias, R, M, N, K, lda,
                                            splits, stream);
    case EPI_BIAS_RESIDUAL:
      return launch_pair_epi<EPI_BIAS_RESIDUAL>(A, B, C, bias, R, M, N, K,
                                                lda, splits, stream);
    case EPI_PARTIAL:
      return launch_pair_epi<EPI_PARTIAL>(A, B, C, bias, R, M, N, K, lda,
                                          splits, stream);
    default:
      return hipErrorInvalidValue;
  }
}

template <int EPI, int BN, int W>
hipError_t configure256() {
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm256_kernel<EPI, BN, W>),
      hipFuncAttributeMaxDynamicSharedMemorySize, Geo<BN, W>::kLdsBytes);
  return err == hipSuccess ? prepare_kernel(&gemm256_kernel<EPI, BN, W>)
                           : err;
}

template <int BN, int W>
hipError_t configure256_all() {
  hipError_t err = configure256<EPI_NONE, BN, W>();
  if (err == hipSuccess) err = configure256<EPI_BIAS_GELU, BN, W>();
  if (err == hipSuccess) err = configure256<EPI_BIAS_RESIDUAL, BN, W>();
  if (err == hipSuccess) err = configure256<EPI_PARTIAL, BN, W>();
  return err;
}

template <int BN, int W>
hipError_t launch256(const uint16_t* A, const uint16_t* B, uint16_t* C,
                     const float* bias, const uint16_t* R, int M, int N,
                     int K, int lda, int splits, int epilogue,
                     hipStream_t stream) {
  if constexpr (BN == 256 && W == 4) {
    if (g_pair)
      return launch_pair(A, B, C, bias, R, M, N, K, lda, splits, epilogue,
                         stream);
    if (g_mfma32)
      return launch_m32(A, B, C, bias, R, M, N, K, lda, splits, epilogue,
                        stream);
  }
  const int blocks = ((M + BM - 1) / BM) * (N / BN);
  const dim3 grid(blocks, splits), block(64 * W);
  const int lds = Geo<BN, W>::kLdsBytes;
  switch (epilogue) {
    case EPI_NONE:
      return launch_kernel(&gemm256_kernel<EPI_NONE, BN, W>, grid, block, lds,
                         stream, A, B, C, bias, R, M, N, K, lda, nullptr, nullptr, g_group_m);
    case EPI_BIAS_GELU:
      return launch_kernel(&gemm256_kernel<EPI_BIAS_GELU, BN, W>, grid, block,
                         lds, stream, A, B, C, bias, R, M, N, K, lda, nullptr, nullptr, g_group_m);
    case EPI_BIAS_RESIDUAL:
      return launch_kernel(&gemm256_kernel<EPI_BIAS_RESIDUAL, BN, W>, grid,
                         block, lds, stream, A, B, C, bias, R, M, N, K, lda, nullptr, nullptr, g_group_m);
    case EPI_PARTIAL:
      return launch_kernel(&gemm256_kernel<EPI_PARTIAL, BN, W>, grid, block,
                         lds, stream, A, B, C, bias, R, M, N, K, lda, nullptr, nullptr, g_group_m);
    default:
      return hipErrorInvalidValue;
  }
}

// persistent 4-wave kernel: one workgroup per CU (its 160 KiB of LDS allow
// no more), each walking ceil(tiles / CUs) tiles
int g_cu_count = 256;

template <int EPI>
hipError_t configure_persist() {
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm256_kernel<EPI, 256, 4, 0, 1>),
      hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256, 4>::kLdsBytes);
  return err == hipSuccess
             ? prepare_kernel(&gemm256_kernel<EPI, 256, 4, 0, 1>)
             : err;
}

template <int EPI>
hipError_t launch_persist_epi(const uint16_t* A, const uint16_t* B, uint16_t* C,
                        const float* bias, const uint16_t* R, int M, int N,
                        int K, int grid, hipStream_t stream) {
  constexpr int lds = Geo<256, 4>::kLdsBytes;
  return launch_kernel(&gemm256_kernel<EPI, 256, 4, 0, 1>, dim3(grid),
                     dim3(256), lds, stream, A, B, C, bias, R, M, N, K, K,
                     nullptr, nullptr, g_group_m);
}

template <int EPI, int kMode>
hipError_t launch_fused4(const uint16_t* A, const uint16_t* B, uint16_t* C,
                         const float* bias, const uint16_t* R, int M, int N,
                         int K, int lda, int splits, float* P, int* cnt,
                         hipStream_t stream) {
  const int blocks = ((M + BM - 1) / BM) * (N / 256);
  constexpr int lds = Geo<256, 4>::kLdsBytes;
  return launch_kernel(&gemm256_kernel<EPI, 256, 4, kMode>,
                     dim3(blocks, splits), dim3(256), lds, stream, A, B, C,
                     bias, R, M, N, K, lda, P, cnt, g_group_m);
}

template <int EPI>
hipError_t configure_fused4() {
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm256_kernel<EPI, 256, 4, 1>),
      hipFuncAttributeMaxDynamicSharedMemorySize, Geo<256, 4>::kLdsBytes);
  return err == hipSuccess ? prepare_kernel(&gemm256_kernel<EPI, 256, 4, 1>)
                           : err;
}

template <int kMode>
hipError_t launch_fused4_epi(const uint16_t* A, const uint16_t* B,
                             uint16_t* C, const float* bias, const uint16_t* R,
                             int M, int N, int K, int lda, int splits,
                             float* P, int* cnt, int epilogue,
                             hipStream_t stream) {
  switch (epilogue) {
    case EPI_NONE:
      return launch_fused4<EPI_NONE, kMode>(A, B, C, bias, R, M, N, K, lda,
                                            splits, P, cnt, stream);
    case EPI_BIAS_GELU:
      return launch_fused4<EPI_BIAS_GELU, kMode>(A, B, C, bias, R, M, N, K,
                                                 lda, splits, P, cnt, stream);
    case EPI_BIAS_RESIDUAL:
      return launch_fused4<EPI_BIAS_RESIDUAL, kMode>(
          A, B, C, bias, R, M, N, K, lda, splits, P, cnt, stream);
    default:
      return hipErrorInvalidValue;
  }
}

// out = epi(sum_s P[s]) over `splits` fp32 partial planes of M x N; each
// thread owns 8 consecutive columns (two float4 per plane, one 16-B bf16
// store).  N % 8 == 0 (N is a multiple of 128 here).
template <int EPI>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(
    const float* __restrict__ P, int splits, int M, int N,
    const float* __restrict__ bias, const uint16_t* __restrict__ R,
    uint16_t* __restrict__ out) {
  const size_t total = static_cast<size_t>(M) * N / 8;
  const size_t plane = static_cast<size_t>(M) * N;
  for (size_t c = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
       c < total; c += static_cast<size_t>(gridDim.x) * blockDim.x) {
    const size_t off = c * 8;
    float v[8];
    {
      const float4 a = *reinterpret_cast<const float4*>(P + off);
      const float4 b = *reinterpret_cast<const float4*>(P + off + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
      v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    for (int s = 1; s < splits; ++s) {
      const float4 a = *reinterpret_cast<const float4*>(P + s * plane + off);
      const float4 b =
          *reinterpret_cast<const float4*>(P + s * plane + off + 4);
      v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
      v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
    }
    if (EPI != EPI_NONE) {
      const int n = static_cast<int>(off % N);
      const float4 b0 = *reinterpret_cast<const float4*>(bias + n);
      const float4 b1 = *reinterpret_cast<const float4*>(bias + n + 4);
      v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
      v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = gelu_tanh(v[r]);
    }
    if (EPI == EPI_BIAS_RESIDUAL) {
      const uint4 res = *reinterpret_cast<const uint4*>(R + off);
      const uint32_t w[4] = {res.x, res.y, res.z, res.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[2 * r] += bf16_to_f32(w[r] & 0xffff);
        v[2 * r + 1] += bf16_to_f32(w[r] >> 16);
      }
    }
    uint32_t o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      o[r] = f32_to_bf16(v[2 * r]) |
             (static_cast<uint32_t>(f32_to_bf16(v[2 * r + 1])) << 16);
    *reinterpret_cast<uint4*>(out + off) = uint4{o[0], o[1], o[2], o[3]};
  }
}

hipError_t launch_reduce(const float* P, int splits, int M, int N,
                         const float* bias, const uint16_t* R, uint16_t* out,
                         int epilogue, hipStream_t stream) {
  const size_t chunks = static_cast<size_t>(M) * N / 8;
  const int blocks = static_cast<int>(
      std::min<size_t>((chunks + 255) / 256, 256 * 16));
  switch (epilogue) {
    case EPI_NONE:
      return launch_kernel(&splitk_reduce_kernel<EPI_NONE>, dim3(blocks),
                         dim3(256), 0, stream, P, splits, M, N, bias, R, out);
    case EPI_BIAS_GELU:
      return launch_kernel(&splitk_reduce_kernel<EPI_BIAS_GELU>, dim3(blocks),
                         dim3(256), 0, stream, P, splits, M, N, bias, R, out);
    case EPI_BIAS_RESIDUAL:
      return launch_kernel(&splitk_reduce_kernel<EPI_BIAS_RESIDUAL>,
                         dim3(blocks), dim3(256), 0, stream, P, splits, M, N,
                         bias, R, out);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace

hipError_t gemm256_prepare() {
  int device = 0, cus = 0;
  if (hipGetDevice(&device) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                            device) == hipSuccess && cus > 0)
    g_cu_count = cus;
  hipError_t err = configure256_all<256, 8>();
  if (err == hipSuccess) err = configure_persist<EPI_NONE>();
  if (err == hipSuccess) err = configure_persist<EPI_BIAS_RESIDUAL>();
  if (err == hipSuccess) err = configure256_all<128, 8>();
  if (err == hipSuccess) err = configure256_all<256, 4>();
  if (err == hipSuccess) err = configure_m32<EPI_NONE>();
  if (err == hipSuccess) err = configure_m32<EPI_BIAS_GELU>();
  if (err == hipSuccess) err = configure_m32<EPI_BIAS_RESIDUAL>();
  if (err == hipSuccess) err = configure_m32<EPI_PARTIAL>();
  if (err == hipSuccess) err = configure_pair<EPI_NONE>();
  if (err == hipSuccess) err = configure_pair<EPI_BIAS_GELU>();
  if (err == hipSuccess) err = configure_pair<EPI_BIAS_RESIDUAL>();
  if (err == hipSuccess) err = configure_pair<EPI_PARTIAL>();
  if (err == hipSuccess) err = configure_fused4<EPI_NONE>();
  if (err == hipSuccess) err = configure_fused4<EPI_BIAS_GELU>();
  if (err == hipSuccess) err = configure_fused4<EPI_BIAS_RESIDUAL>();
  if (err == hipSuccess) err = prepare_kernel(&splitk_reduce_kernel<EPI_NONE>);
  if (err == hipSuccess)
    err = prepare_kernel(&splitk_reduce_kernel<EPI_BIAS_GELU>);
  if (err == hipSuccess)
    err = prepare_kernel(&splitk_reduce_kernel<EPI_BIAS_RESIDUAL>);
  return err;
}

bool gemm256_shape_ok(int M, int N, int K, int bn) {
  return (bn == 256 || bn == 128) && M >= 1 && N % bn == 0 && N >= bn &&
         K % BKH == 0 && K >= BKH;
}

// The 4-wave kernel consumes K in 64-deep steps and addresses A and B
// through buffer descriptors with 32-bit byte offsets.
bool gemm256w4_shape_ok(int M, int N, int K) {
  return gemm256_shape_ok(M, N, K, 256) && K % 64 == 0 &&
         static_cast<size_t>(M > N ? M : N) * K * 2 < 0x7fff0000ull;
}

hipError_t launch_gemm256(const uint16_t* A, const uint16_t* B, uint16_t* C,
                          const float* bias, const uint16_t* R, int M, int N,
                          int K, int epilogue, hipStream_t stream, int bn,
                          int waves) {
  if (!gemm256_shape_ok(M, N, K, bn) || epilogue == EPI_PARTIAL ||
      (waves != 8 && !(waves == 4 && bn == 256)) ||
      (waves == 4 && !gemm256w4_shape_ok(M, N, K)))
    return hipErrorInvalidValue;
  if (waves == 4)
    return launch256<256, 4>(A, B, C, bias, R, M, N, K, K, 1, epilogue,
                             stream);
  if (bn == 128)
    return launch256<128, 8>(A, B, C, bias, R, M, N, K, K, 1, epilogue,
                             stream);
  return launch256<256, 8>(A, B, C, bias, R, M, N, K, K, 1, epilogue,
                           stream);
}

hipError_t launch_gemm256_persist(const uint16_t* A, const uint16_t* B,
                                  uint16_t* C, const float* bias,
                                  const uint16_t* R, int M, int N, int K,
                                  int epilogue, hipStream_t stream) {
  if (!gemm256w4_shape_ok(M, N, K)) return hipErrorInvalidValue;
  const int tiles = ((M + BM - 1) / BM) * (N / 256);
  const int grid = tiles < g_cu_count ? tiles : g_cu_count;
  switch (epilogue) {
    case EPI_NONE:
      return launch_persist_epi<EPI_NONE>(A, B, C, bias, R, M, N, K, grid,
                                          stream);
    case EPI_BIAS_GELU:
      // the persistent bias+GELU kernel carried the next tile's address
      // state across the GELU epilogue and spilled a VGPR; it also ran
      // 1-2 % slower than the one-tile kernel (round 3): the GELU epilogue
      // runs the one-tile grid
      return launch256<256, 4>(A, B, C, bias, R, M, N, K, K, 1,
                               EPI_BIAS_GELU, stream);
    case EPI_BIAS_RESIDUAL:
      return launch_persist_epi<EPI_BIAS_RESIDUAL>(A, B, C, bias, R, M, N, K,
                                                   grid, stream);
    default:
      return hipErrorInvalidValue;
  }
}

int gemm256_splits(int M, int N, int K) {
  // split K for the 256x256 kernel only while its grid leaves CUs idle,
  // each slice keeps >= 2048 of K, and the slices stay 32-aligned
  const int tiles = ((M + BM - 1) / BM) * (N / 256);
  if (tiles >= 256 || N % 256 || K % BKH) return 1;
  int s = 1;
  while (s < 4 && tiles * s < 256 && K % (2 * s * BKH) == 0 &&
         K / (2 * s) >= 2048)
    s *= 2;
  return s;
}

// Split-K combine: 0 = partial planes + the reduce kernel; 1 = in-launch,
// last arriver re-reads both planes (6 % slower than 0 at 2048x4096x16384,
// profiles/r1_gemm/gemm_w4_splitk_fused_ab.jsonl).
int g_splitk_fused = 0;

void gemm_set_group_m(int rows) { g_group_m = rows < 1 ? 1 : rows; }
int gemm_group_m() { return g_group_m; }

void gemm_set_splitk_fused(int mode) { g_splitk_fused = mode ? 1 : 0; }

void gemm_set_mfma32(int on) { g_mfma32 = on ? 1 : 0; }
void gemm_set_pair(int on) { g_pair = on ? 1 : 0; }
int gemm_pair() { return g_pair; }
int gemm_mfma32() { return g_mfma32; }
int gemm_splitk_fused() { return g_splitk_fused; }

// the fused 4-wave split-K path: two 64-deep-aligned slices, 32-bit
// operand offsets
bool splitk_w4(int M, int N, int K, int splits) {
  return splits == 2 && (K / splits) % 64 == 0 &&
         static_cast<size_t>(M > N ? M : N) * K * 2 < 0x7fff0000ull;
}

// fp32 partial planes, then (4-wave path) one ticket counter per tile
size_t splitk_counter_offset(int M, int N, int splits) {
  return static_cast<size_t>(splits) * M * N * sizeof(float);
}

size_t gemm256_splitk_workspace(int M, int N, int K) {
  const int s = gemm256_splits(M, N, K);
  if (s <= 1) return 0;
  const size_t tiles = static_cast<size_t>((M + BM - 1) / BM) * (N / 256);
  return splitk_counter_offset(M, N, s) + ((tiles * 4 + 255) / 256) * 256;
}

hipError_t launch_gemm256_splitk(const uint16_t* A, const uint16_t* B,
                                 uint16_t* C, const float* bias,
                                 const uint16_t* R, int M, int N, int K,
                                 int epilogue, int splits, float* workspace,
                                 size_t workspace_bytes, hipStream_t stream) {
  if (splits < 2 || K % (splits * BKH) || M < 1 || N % 256 ||
      workspace == nullptr ||
      workspace_bytes < static_cast<size_t>(splits) * M * N * sizeof(float))
    return hipErrorInvalidValue;
  if (splitk_w4(M, N, K, splits) && !g_splitk_fused) {
    // A/B reference: 4-wave partial planes + the separate reduce kernel
    hipError_t err = launch256<256, 4>(
        A, B, reinterpret_cast<uint16_t*>(workspace), nullptr, nullptr, M, N,
        K / splits, K, splits, EPI_PARTIAL, stream);
    if (err != hipSuccess) return err;
    return launch_reduce(workspace, splits, M, N, bias, R, C, epilogue,
                         stream);
  }
  if (splitk_w4(M, N, K, splits)) {
    // 4-wave kernel, combined in-launch by each tile's last K-slice block
    const size_t tiles = static_cast<size_t>((M + BM - 1) / BM) * (N / 256);
    const size_t off = splitk_counter_offset(M, N, splits);
    if (workspace_bytes < off + tiles * 4) return hipErrorInvalidValue;
    int* cnt = reinterpret_cast<int*>(reinterpret_cast<char*>(workspace) + off);
    hipError_t err = hipMemsetAsync(cnt, 0, tiles * 4, stream);
    if (err != hipSuccess) return err;
    return launch_fused4_epi<1>(A, B, C, bias, R, M, N, K / splits, K, splits,
                                workspace, cnt, epilogue, stream);
  }
  hipError_t err = launch256<256, 8>(A, B, reinterpret_cast<uint16_t*>(workspace),
                                     nullptr, nullptr, M, N, K / splits, K,
                                     splits, EPI_PARTIAL, stream);
  if (err != hipSuccess) return err;
  return launch_reduce(workspace, splits, M, N, bias, R, C, epilogue, stream);
}

}  // namespace kiosk
