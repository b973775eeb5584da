// Memory-bound helper kernels: on-device random init and checksums.
//
// Weight init runs on the device so a scale-up never generates or copies a
// GB of host-side random numbers: at the HBM rate the
// 1 GiB default model initialises in well under a millisecond.
#include <mutex>
#include <utility>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

namespace kiosk {
namespace {

constexpr int kInitThreads = 256;
constexpr int kInitMaxBlocks = 2048;   // 256 CUs x 8, grid-stride the rest

__device__ __forceinline__ void random8(uint64_t key, size_t chunk,
                                        float lo, float scale, float (&v)[8]) {
  const uint64_t r0 = splitmix64(key + 2 * chunk);
  const uint64_t r1 = splitmix64(key + 2 * chunk + 1);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = lo + scale * ((static_cast<float>((r0 >> (16 * k)) & 0xffff) + 0.5f)
                         * (1.0f / 65536.0f));
    v[4 + k] = lo + scale *
               ((static_cast<float>((r1 >> (16 * k)) & 0xffff) + 0.5f)
                * (1.0f / 65536.0f));
  }
}

__global__ __launch_bounds__(kInitThreads) void init_bf16_kernel(
    uint16_t* __restrict__ p, size_t n, uint64_t seed,
    const uint64_t* __restrict__ seed_dev, float lo, float scale) {
  const uint64_t key = splitmix64(seed_dev != nullptr ? *seed_dev : seed);
  const size_t chunks = (n + 7) / 8;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t c = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
       c < chunks; c += stride) {
    float v[8];
    random8(key, c, lo, scale, v);
    if (c * 8 + 8 <= n) {
      uint4 out;
      out.x = f32_to_bf16(v[0]) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      out.y = f32_to_bf16(v[2]) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      out.z = f32_to_bf16(v[4]) | (static_cast<uint32_t>(f32_to_bf16(v[5])) << 16);
      out.w = f32_to_bf16(v[6]) | (static_cast<uint32_t>(f32_to_bf16(v[7])) << 16);
      *reinterpret_cast<uint4*>(p + c * 8) = out;
    } else {
      for (size_t k = 0; c * 8 + k < n; ++k) p[c * 8 + k] = f32_to_bf16(v[k]);
    }
  }
}

__global__ __launch_bounds__(kInitThreads) void init_f32_kernel(
    float* __restrict__ p, size_t n, uint64_t seed, float lo, float scale) {
  const uint64_t key = splitmix64(seed);
  const size_t chunks = (n + 7) / 8;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t c = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
       c < chunks; c += stride) {
    float v[8];
    random8(key, c, lo, scale, v);
    for (size_t k = 0; k < 8 && c * 8 + k < n; ++k) p[c * 8 + k] = v[k];
  }
}

__global__ __launch_bounds__(256) void partial_sums_kernel(
    const uint16_t* __restrict__ p, size_t n, float* __restrict__ partials) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* wave_sums = reinterpret_cast<float*>(smem);
  float acc = 0.f;
  const size_t chunks = n / 8;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t c = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
       c < chunks; c += stride) {
    const uint4 v = *reinterpret_cast<const uint4*>(p + c * 8);
    acc += bf16_to_f32(v.x & 0xffff) + bf16_to_f32(v.x >> 16) +
           bf16_to_f32(v.y & 0xffff) + bf16_to_f32(v.y >> 16) +
           bf16_to_f32(v.z & 0xffff) + bf16_to_f32(v.z >> 16) +
           bf16_to_f32(v.w & 0xffff) + bf16_to_f32(v.w >> 16);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    for (size_t k = chunks * 8; k < n; ++k) acc += bf16_to_f32(p[k]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) wave_sums[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float total = 0.f;
    for (int w = 0; w < static_cast<int>(blockDim.x) / 64; ++w)
      total += wave_sums[w];
    partials[blockIdx.x] = total;
  }
}

// Fault injection (utils/faults.py "hang_key"): one wave that sleeps until
// `ticks` of the 100 MHz s_memrealtime clock have passed -- a stuck kernel
// as the manager's watchdog sees it, but one that always terminates (the
// host clamps ticks), so the grid drains even if nobody kills the process.
__global__ __launch_bounds__(64) void spin_kernel(unsigned long long ticks,
                                                  unsigned int* done) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(127);
  }
  if (threadIdx.x == 0 && done) *done = 1u;
}

int init_blocks(size_t n) {
  const size_t chunks = (n + 7) / 8;
  size_t blocks = (chunks + kInitThreads - 1) / kInitThreads;
  if (blocks > kInitMaxBlocks) blocks = kInitMaxBlocks;
  return blocks < 1 ? 1 : static_cast<int>(blocks);
}

}  // namespace

hipError_t launch_init_uniform_bf16(uint16_t* p, size_t n, uint64_t seed,
                                    float lo, float hi, hipStream_t stream) {
  return launch_kernel(&init_bf16_kernel, dim3(init_blocks(n)),
                     dim3(kInitThreads), 0, stream, p, n, seed,
                     static_cast<const uint64_t*>(nullptr), lo, hi - lo);
}

hipError_t launch_init_uniform_bf16_devseed(uint16_t* p, size_t n,
                                            const uint64_t* seed, float lo,
                                            float hi, hipStream_t stream) {
  return launch_kernel(&init_bf16_kernel, dim3(init_blocks(n)),
                     dim3(kInitThreads), 0, stream, p, n, uint64_t(0), seed,
                     lo, hi - lo);
}

hipError_t launch_init_uniform_f32(float* p, size_t n, uint64_t seed,
                                   float lo, float hi, hipStream_t stream) {
  return launch_kernel(&init_f32_kernel, dim3(init_blocks(n)),
                     dim3(kInitThreads), 0, stream, p, n, seed, lo, hi - lo);
}

hipError_t launch_partial_sums(const uint16_t* p, size_t n, float* partials,
                               hipStream_t stream) {
  return launch_kernel(&partial_sums_kernel, dim3(kSumBlocks), dim3(256),
                     4 * sizeof(float), stream, p, n, partials);
}

hipError_t launch_spin(double ms, unsigned int* done, hipStream_t stream) {
  if (!(ms >= 0.0)) return hipErrorInvalidValue;
  ms = ms > kSpinMaxMs ? kSpinMaxMs : ms;
  const unsigned long long ticks =
      static_cast<unsigned long long>(ms * 1e5);   // 100 MHz
  return launch_kernel(&spin_kernel, dim3(1), dim3(64), 0, stream, ticks, done);
}

// Loads this file's code object (first use of any of its kernels does;
// querying attributes does it without a launch, so no hardware queue) and
// resolves every kernel's launch handle.
hipError_t misc_prepare() {
  static std::atomic<unsigned long long> done{0};
  return prepare_per_device(done, [] {
    hipFuncAttributes attr;
    hipError_t err = hipFuncGetAttributes(
        &attr, reinterpret_cast<const void*>(&init_bf16_kernel));
    if (err == hipSuccess) err = prepare_kernel(&init_bf16_kernel);
    if (err == hipSuccess) err = prepare_kernel(&init_f32_kernel);
    if (err == hipSuccess) err = prepare_kernel(&partial_sums_kernel);
    if (err == hipSuccess) err = prepare_kernel(&spin_kernel);
    return err;
  });
}

namespace {

// (stub, device) -> handle; a handful of kernels, looked up on every launch
struct KernelCache {
  struct Entry {
    const void* stub;
    int device;
    hipFunction_t f;
  };
  std::mutex mu;
  std::vector<Entry> entries;
};

KernelCache& kernel_cache() {
  static KernelCache* cache = new KernelCache();   // never destroyed
  return *cache;
}

}  // namespace

hipFunction_t resolve_kernel(const void* stub) {
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return nullptr;
  KernelCache& cache = kernel_cache();
  {
    std::lock_guard<std::mutex> lock(cache.mu);
    for (const auto& e : cache.entries) {
      if (e.stub == stub && e.device == device) return e.f;
    }
  }
  // outside our mutex: this call may wait on the runtime's registry lock
  hipFunction_t f = nullptr;
  if (hipGetFuncBySymbol(&f, stub) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lock(cache.mu);
  cache.entries.push_back({stub, device, f});
  return f;
}

}  // namespace kiosk
