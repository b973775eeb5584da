// Host-side launchers for the gfx950 kernels in csrc/kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace kiosk {

enum Epilogue {
  EPI_NONE = 0,           // C = A.B^T
  EPI_BIAS_GELU = 1,      // C = gelu_tanh(A.B^T + bias)
  EPI_BIAS_RESIDUAL = 2,  // C = A.B^T + bias + R
  EPI_PARTIAL = 3,        // internal: fp32 split-K partial planes
};

// GEMM tile geometry (shared with the warm-start kernel, which
// pre-allocates and zeroes the same LDS footprint).
constexpr int kGemmBM = 128;
constexpr int kGemmBN = 128;
constexpr int kGemmBK = 64;
constexpr int kGemmThreads = 256;
constexpr int kGemmLdsBytes = 2 * 2 * kGemmBM * kGemmBK * 2;  // 64 KiB
constexpr int kGemmBlocksPerCU = 2;
// LDS of the largest GEMM block (the 4-wave 256x256 kernel's 5-unit ring):
// the warm-start kernel pre-allocates and zeroes this much per CU
constexpr int kGemmRingLdsBytes = 5 * 256 * 128;  // 160 KiB

// C[M,N] (bf16) = epilogue(A[M,K] . B[N,K]^T); fp32 accumulate.
// Requires N % 128 == 0, K % 64 == 0; any M >= 1.
hipError_t launch_gemm(const uint16_t* A, const uint16_t* B, uint16_t* C,
                       const float* bias, const uint16_t* R, int M, int N,
                       int K, int epilogue, hipStream_t stream);
bool gemm_shape_ok(int M, int N, int K);
hipError_t gemm_prepare();  // call once before launching / capturing
// Code-object loads without a launch (no hardware queue, no HBM beyond the
// code itself): what a `context` standby pre-pays.
hipError_t misc_prepare();
hipError_t warmstart_prepare();

// Kernel variants: 0 = auto (256x256 ring kernel -- the 4-wave one where
// its 32-bit offsets reach -- when it yields >= 256 tiles, else split-K 256x256 when a workspace is given, else the 256x128
// ring when that fills the chip, else 128x128), 1 = 128x128 two-barrier,
// 2 = 256x256 LDS ring, 3 = 256x128 LDS ring, 4 = split-K 256x256 (fp32
// partials in `workspace` + one fused reduce/epilogue kernel), 5 = 256x256
// ring with 4 waves of 128x128 outputs (accumulators in AGPRs), 6 = the
// same as a persistent grid (one workgroup per CU walks the tiles; the next
// tile's first DMA groups overlap the epilogue).
enum GemmVariant {
  GEMM_AUTO = 0, GEMM_128 = 1, GEMM_256 = 2, GEMM_256x128 = 3,
  GEMM_256_SPLITK = 4, GEMM_256W4 = 5, GEMM_256W4P = 6
};
hipError_t launch_gemm_variant(const uint16_t* A, const uint16_t* B,
                               uint16_t* C, const float* bias,
                               const uint16_t* R, int M, int N, int K,
                               int epilogue, int variant, hipStream_t stream,
                               float* workspace = nullptr,
                               size_t workspace_bytes = 0);
int gemm_pick_variant(int M, int N, int K, bool have_workspace = false);
// bytes of fp32 workspace the split-K path needs for this shape (0: none)
size_t gemm_workspace_bytes(int M, int N, int K);
// 256 x bn ring kernel (gemm256.hip), bn = 256 or 128
bool gemm256_shape_ok(int M, int N, int K, int bn = 256);
bool gemm256w4_shape_ok(int M, int N, int K);
hipError_t gemm256_prepare();
hipError_t launch_gemm256(const uint16_t* A, const uint16_t* B, uint16_t* C,
                          const float* bias, const uint16_t* R, int M, int N,
                          int K, int epilogue, hipStream_t stream,
                          int bn = 256, int waves = 8);
hipError_t launch_gemm256_persist(const uint16_t* A, const uint16_t* B,
                                  uint16_t* C, const float* bias,
                                  const uint16_t* R, int M, int N, int K,
                                  int epilogue, hipStream_t stream);
int gemm256_splits(int M, int N, int K);
size_t gemm256_splitk_workspace(int M, int N, int K);
// split-K on the 4-wave kernel: combine in-launch by each tile's last
// slice, or (default, faster here) partial planes + the reduce kernel
void gemm_set_splitk_fused(int mode);   // 0 reduce kernel, 1 in-launch
int gemm_splitk_fused();
// 1: the 4-wave one-tile kernel runs on v_mfma_f32_32x32x16_bf16
// (gemm256m32_kernel, profiles/r4_mfma_dma); 0: on 16x16x32
void gemm_set_mfma32(int on);
int gemm_mfma32();
// 1: the 4-wave one-tile GEMM path runs gemm256p_kernel (8 waves, two per
// SIMD, 128x64 AGPR tiles; an A/B arm, profiles/r6_gemm_pair)
void gemm_set_pair(int on);
int gemm_pair();
// tile rows per group in the 256-row kernels' tile order (default 4)
void gemm_set_group_m(int rows);
int gemm_group_m();
hipError_t launch_gemm256_splitk(const uint16_t* A, const uint16_t* B,
                                 uint16_t* C, const float* bias,
                                 const uint16_t* R, int M, int N, int K,
                                 int epilogue, int splits, float* workspace,
                                 size_t workspace_bytes, hipStream_t stream);

// Uniform [lo, hi) init, counter-based (reproducible for a seed).
hipError_t launch_init_uniform_bf16(uint16_t* p, size_t n, uint64_t seed,
                                    float lo, float hi, hipStream_t stream);
hipError_t launch_init_uniform_f32(float* p, size_t n, uint64_t seed,
                                   float lo, float hi, hipStream_t stream);
// Same, but the seed is read from device memory (graph-capturable).
hipError_t launch_init_uniform_bf16_devseed(uint16_t* p, size_t n,
                                            const uint64_t* seed, float lo,
                                            float hi, hipStream_t stream);

// Deterministic fp32 partial sums of a bf16 buffer (one per block).
constexpr int kSumBlocks = 1024;
hipError_t launch_partial_sums(const uint16_t* p, size_t n, float* partials,
                               hipStream_t stream);

// Bounded GPU stall for fault injection: one wave sleeping `ms`
// (clamped to kSpinMaxMs) of wall clock, then *done = 1 (if non-null).
constexpr double kSpinMaxMs = 30000.0;
hipError_t launch_spin(double ms, unsigned int* done, hipStream_t stream);

// N1 warm-start: one workgroup per CU (LDS request > half the CU's LDS
// keeps two from sharing a CU); zeroes `lds_bytes` of LDS, streams a slice
// of `w` (n elements), runs `iters` MFMA steps and records per-WG
// {HW_ID, XCC_ID, t0, t1, checksum bits, ...} into record[8 * wg].
constexpr int kWarmRecordWords = 8;
hipError_t launch_warmstart(const uint16_t* w, size_t n, uint32_t* record,
                            int nblocks, int iters, int lds_bytes,
                            hipStream_t stream);

}  // namespace kiosk
