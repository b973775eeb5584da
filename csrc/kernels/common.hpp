// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//  * wave64; block sizes are multiples of 64; lane = threadIdx.x & 63.
//  * bf16 tensors are passed as uint16_t* and loaded 16 B per lane
//    (8 x bf16) -- hipcc does not vectorise scalar bf16 loads.
//  * all LDS is one `extern __shared__` array aligned to 16 B (no static
//    __shared__ objects: they shift the dynamic base and add waits).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.hpp"

namespace kiosk {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

constexpr int kWave = 64;

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// Round-to-nearest-even via the hardware convert (hipcc -O3 emits
// v_cvt_pk_bf16_f32, which keeps NaN a NaN).
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  __bf16 b = static_cast<__bf16>(f);
  return __builtin_bit_cast(uint16_t, b);
}

// 16-byte global -> LDS DMA (global_load_lds_dwordx4).  The LDS
// destination is the wave-uniform `lds_wave_base` + lane * 16.
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((gbl_void_t*)gsrc,
                                   (lds_void_t*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt0() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// tanh-approximated GELU: 0.5 x (1 + tanh u) = x * sigmoid(2u)
// = x / (1 + exp(-2u)), u = sqrt(2/pi) (x + 0.044715 x^3).  With log2(e)
// folded into the polynomial, -2u log2(e) = x (k0 + k1 x^2): 3 VALU, one
// v_exp_f32 (2^z), one add, one v_rcp_f32 (~1 ulp), one mul -- no IEEE
// division, no separate scaling multiply.  Limits are exact (2^z -> inf
// gives x * 0, 2^z -> 0 gives x).
__device__ __forceinline__ float gelu_tanh(float x) {
  constexpr float k0 = -2.0f * 0.7978845608028654f * 1.4426950408889634f;
  constexpr float k1 = k0 * 0.044715f;
  const float z = x * __builtin_fmaf(x * x, k1, k0);
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
}

// Bijective XCD-aware remap of a linear workgroup id: consecutive remapped
// ids run on the same XCD (blockIdx % 8 labels the XCD a block lands on
// under round-robin dispatch).  Speed only -- never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nxcd = 8;
  if (nwg < nxcd) return bid;
  const int xcd = bid % nxcd, q = nwg / nxcd, r = nwg % nxcd;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / nxcd;
}

// splitmix64: counter-based generator for reproducible on-device init.
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

}  // namespace kiosk
