// What an LDS-DMA issue costs the matrix pipe, per MFMA shape (gfx950).
//
// The 4-wave 256x256 GEMM issues 16 LDS-DMA pieces per wave per 64-deep
// k-step among 128 v_mfma_f32_16x16x32_bf16 (profiles/r3_mfma_util: the
// down-projection keeps the pipe 68.7 % busy; dropping the in-loop DMA
// in an ablation build runs +21 %).  A DMA issue holds the wave; the MFMA
// in flight keeps the pipe busy only for its own issue interval, 16
// cycles for 16x16x32 and 32 for 32x32x16.  This probe runs the same
// schedule -- one workgroup of 4 waves per CU, 256 accumulators per wave
// in AGPRs, the same MFMA cycles per step (2048 per SIMD) and the same 16
// DMA pieces (1 KiB each, buffer_load ... lds) per wave per step -- with
// either MFMA shape, with and without the DMA, and prints the time per
// step.  Operands come from registers (no LDS reads), so the DMA issue is
// the only thing competing with the MFMAs.
//
//   hipcc -O3 --offload-arch=gfx950 -I csrc/kernels \
//     tools/probes/mfma_dma_probe.hip -o build/mfma_dma_probe
//   build/mfma_dma_probe [steps]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "common.hpp"

using kiosk::bf16x8;
using kiosk::f32x4;
using kiosk::lds_void_t;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,               \
              hipGetErrorString(e_));                                 \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

namespace {

constexpr int kWaves = 4;
constexpr int kPieces = 16;            // DMA pieces per wave per step
constexpr int kSliceBytes = kPieces * 1024;
constexpr int kLdsBytes = 128 * 1024;

__device__ __forceinline__ void mfma16(f32x4& acc, const bf16x8& a,
                                       const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
               : "+a"(acc)
               : "v"(a), "v"(b));
}

__device__ __forceinline__ void mfma32(f32x16& acc, const bf16x8& a,
                                       const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
               : "+a"(acc)
               : "v"(a), "v"(b));
}

// vmcnt(16) | expcnt(7) | lgkmcnt(0): at most one step of DMA in flight
constexpr int kWaitVm16 = (16 & 15) | (7 << 4) | (0 << 8) | ((16 >> 4) << 14);

template <int kShape, bool kDma>
__global__ __launch_bounds__(64 * kWaves, 1) void probe_kernel(
    const uint16_t* __restrict__ src, float* __restrict__ out, int steps) {
  extern __shared__ __attribute__((aligned(1024))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t*>(src), 0, 0x7fffffff, 0x00020000);
  // this wave's 16 KiB slice of the source; lane l moves bytes
  // [16 l, 16 l + 16) of each 1 KiB piece
  const int voff = (blockIdx.x * kWaves + wave) * kSliceBytes + lane * 16;
  bf16x8 a, b;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = static_cast<__bf16>(0.001f * ((lane + i) & 7));
    b[i] = static_cast<__bf16>(0.002f * ((lane * 3 + i) & 7));
  }
  auto dma = [&](int p) {
    if constexpr (kDma) {
      char* lds = smem + ((wave * kPieces + p) % (kLdsBytes / 1024)) * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void_t*)lds, 16,
                                               voff + p * 1024, 0, 0, 0);
    }
  };
  float total = 0.f;
  if constexpr (kShape == 16) {
    f32x4 acc[64];
#pragma unroll
    for (int t = 0; t < 64; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < steps; ++s) {
      // 128 MFMAs (64 tiles x 2 k-substeps), a DMA piece after every 8th
#pragma unroll
      for (int u = 0; u < 128; ++u) {
        mfma16(acc[u & 63], a, b);
        if ((u & 7) == 7) dma(u >> 3);
      }
      __builtin_amdgcn_s_waitcnt(kWaitVm16);
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int t = 0; t < 64; ++t) total += acc[t][0] + acc[t][3];
  } else {
    f32x16 acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;
    for (int s = 0; s < steps; ++s) {
      // 64 MFMAs (16 tiles x 4 k-substeps), a DMA piece after every 4th
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        mfma32(acc[u & 15], a, b);
        if ((u & 3) == 3) dma(u >> 2);
      }
      __builtin_amdgcn_s_waitcnt(kWaitVm16);
      __builtin_amdgcn_s_barrier();
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int t = 0; t < 16; ++t) total += acc[t][0] + acc[t][15];
  }
  // drain the DMA before the workgroup (and its LDS) ends
  __builtin_amdgcn_s_waitcnt(0);
  out[blockIdx.x * blockDim.x + threadIdx.x] = total;
}

template <int kShape, bool kDma>
float run(const uint16_t* src, float* out, int blocks, int steps) {
  auto k = probe_kernel<kShape, kDma>;
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                            hipFuncAttributeMaxDynamicSharedMemorySize,
                            kLdsBytes));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * kWaves), kLdsBytes, 0, src,
                     out, 2);                         // warm-up
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * kWaves), kLdsBytes, 0, src,
                     out, steps);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms;
}

}  // namespace

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 4000;
  if (steps < 1 || steps > 1000000) {
    fprintf(stderr, "steps out of range\n");
    return 2;
  }
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                              0));
  const int blocks = cus;
  const size_t src_bytes = static_cast<size_t>(blocks) * kWaves * kSliceBytes;
  uint16_t* src = nullptr;
  float* out = nullptr;
  CHECK(hipMalloc(&src, src_bytes));
  CHECK(hipMemset(src, 0, src_bytes));
  CHECK(hipMalloc(&out, static_cast<size_t>(blocks) * 64 * kWaves * 4));
  for (int round = 0; round < 3; ++round) {
    const float m16 = run<16, false>(src, out, blocks, steps);
    const float m16d = run<16, true>(src, out, blocks, steps);
    const float m32 = run<32, false>(src, out, blocks, steps);
    const float m32d = run<32, true>(src, out, blocks, steps);
    // per step: 2048 MFMA-busy cycles per SIMD in every variant
    printf("{\"round\": %d, \"steps\": %d, \"cus\": %d, "
           "\"us_per_step\": {\"16x16x32\": %.4f, \"16x16x32+dma\": %.4f, "
           "\"32x32x16\": %.4f, \"32x32x16+dma\": %.4f}, "
           "\"dma_slowdown\": {\"16x16x32\": %.4f, \"32x32x16\": %.4f}, "
           "\"implied_ghz_no_dma\": {\"16x16x32\": %.3f, \"32x32x16\": "
           "%.3f}}\n",
           round, steps, cus, 1e3f * m16 / steps, 1e3f * m16d / steps,
           1e3f * m32 / steps, 1e3f * m32d / steps, m16d / m16, m32d / m32,
           2048.0 * steps / (m16 * 1e6), 2048.0 * steps / (m32 * 1e6));
  }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
