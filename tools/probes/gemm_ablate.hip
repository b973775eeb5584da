// Diagnostic: time the 4-wave 256x256 ring GEMM with parts of its k-loop
// removed (-DKIOSK_GEMM_ABLATE=<bits>, see gemm256.hip).  Numerics are
// meaningless in ablated builds; only the timing is reported.
//   hipcc -O3 --offload-arch=gfx950 -DKIOSK_GEMM_ABLATE=1 \
//     -I csrc/kernels tools/probes/gemm_ablate.hip -o build/gemm_ablate_1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <cstring>
#include <vector>

#include "../../csrc/kernels/gemm256.hip"

#define CHECK(x)                                                      \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,               \
              hipGetErrorString(e_));                                 \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 8192;
  const int N = argc > 2 ? atoi(argv[2]) : 8192;
  const int K = argc > 3 ? atoi(argv[3]) : 8192;
  const int waves = argc > 4 ? atoi(argv[4]) : 4;
  // epilogue (0 none, 1 bias+GELU, 2 bias+residual) and split-K slices
  // (>= 2: the 4-wave partial kernel + the reduce, as the worker's
  // down-projection runs)
  const int epi = argc > 5 ? atoi(argv[5]) : 0;
  const int splits = argc > 6 ? atoi(argv[6]) : 1;
  const int iters = 20;
  std::vector<uint16_t> h(static_cast<size_t>(std::max(M, N)) * K);
  uint32_t x = 12345;
  for (auto& v : h) {  // uniform-ish bf16 in [-1, 1): random operands
    x = x * 1664525u + 1013904223u;
    const float f = ((x >> 8) * (1.0f / 16777216.0f)) * 2.0f - 1.0f;
    uint32_t u;
    std::memcpy(&u, &f, 4);
    v = static_cast<uint16_t>(u >> 16);
  }
  uint16_t *A, *B, *C;
  CHECK(hipMalloc(&A, static_cast<size_t>(M) * K * 2));
  CHECK(hipMalloc(&B, static_cast<size_t>(N) * K * 2));
  CHECK(hipMalloc(&C, static_cast<size_t>(M) * N * 2));
  CHECK(hipMemcpy(A, h.data(), static_cast<size_t>(M) * K * 2,
                  hipMemcpyHostToDevice));
  CHECK(hipMemcpy(B, h.data(), static_cast<size_t>(N) * K * 2,
                  hipMemcpyHostToDevice));
  float* bias = nullptr;
  uint16_t* R = nullptr;
  float* ws = nullptr;
  const size_t ws_bytes =
      splits > 1 ? static_cast<size_t>(splits) * M * N * 4 + 65536 : 0;
  CHECK(hipMalloc(&bias, static_cast<size_t>(N) * 4));
  CHECK(hipMemset(bias, 0, static_cast<size_t>(N) * 4));
  CHECK(hipMalloc(&R, static_cast<size_t>(M) * N * 2));
  CHECK(hipMemset(R, 0, static_cast<size_t>(M) * N * 2));
  if (ws_bytes) CHECK(hipMalloc(&ws, ws_bytes));
  CHECK(kiosk::gemm256_prepare());
  hipEvent_t t0, t1;
  CHECK(hipEventCreate(&t0));
  CHECK(hipEventCreate(&t1));
  float best = 1e30f;
  for (int r = 0; r < 7; ++r) {
    CHECK(hipEventRecord(t0, 0));
    for (int i = 0; i < iters; ++i)
      CHECK(splits > 1
                ? kiosk::launch_gemm256_splitk(A, B, C, bias, R, M, N, K, epi,
                                               splits, ws, ws_bytes, 0)
                : kiosk::launch_gemm256(A, B, C, bias, R, M, N, K, epi, 0,
                                        256, waves));
    CHECK(hipEventRecord(t1, 0));
    CHECK(hipEventSynchronize(t1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, t0, t1));
    ms /= iters;
    if (r > 0 && ms < best) best = ms;
  }
  // FNV-1a over every output bit: variants of the same math must agree
  std::vector<uint16_t> out(static_cast<size_t>(M) * N);
  CHECK(hipMemcpy(out.data(), C, out.size() * 2, hipMemcpyDeviceToHost));
  uint64_t hash = 1469598103934665603ull;
  for (uint16_t v : out) hash = (hash ^ v) * 1099511628211ull;
  printf("{\"ablate\": %d, \"waves\": %d, \"epi\": %d, \"splits\": %d, "
         "\"shape\": [%d, %d, %d], \"ms\": %.4f, \"tflops\": %.1f, "
         "\"hash\": \"%016llx\"}\n",
         KIOSK_GEMM_ABLATE, waves, epi, splits, M, N, K, best,
         2.0 * M * N * K / (best * 1e-3) / 1e12,
         static_cast<unsigned long long>(hash));
  return 0;
}
