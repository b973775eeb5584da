// bf16 "TN" GEMM for gfx950 with fused epilogues (the worker MLP, N2).
//
//   C[M,N] = epi(A[M,K] . B[N,K]^T)      A, B, C bf16; fp32 accumulation
//
// Structure (cdna_hip_programming.md §5, "Minimum 2-phase"):
//  * 128x128x64 block tile, 256 threads = 4 waves as 2x2, each wave owns a
//    64x64 output = 4x4 tiles of v_mfma_f32_16x16x32_bf16.
//  * A and B tiles staged global->LDS by global_load_lds_dwordx4 (LDS-DMA,
//    no VGPR round trip), double-buffered: the DMA of k-tile t+1 is issued
//    before the MFMAs of tile t, one vmcnt(0)+barrier per k-tile.
//  * LDS image: [128 rows][128 B]; 16-B chunk c of row r lives at chunk
//    c ^ ((r >> 1) & 7).  LDS-DMA writes lane-linearly, so the swizzle is
//    applied to the per-lane *source* address and undone on the ds_read
//    (rule 21): 16 consecutive lanes reading 16 rows at one k-chunk hit 16
//    distinct 16-B bank groups -> conflict-free ds_read_b128.
//  * Operands are fed to the MFMA swapped (W fragment as "A", X fragment as
//    "B"), so the accumulator holds C^T: each lane ends with 4 consecutive
//    output columns of one row -> 8-byte packed bf16 stores, float4 bias
//    loads and 8-byte residual loads in the epilogue.
//  * Workgroup ids are remapped XCD-aware (bijective) and then walked in
//    8-tile-row groups so blocks sharing A/B panels share an XCD's L2.
#include "common.hpp"
#include "kernels.hpp"

namespace kiosk {
namespace {

constexpr int BM = kGemmBM, BN = kGemmBN, BK = kGemmBK;
constexpr int kTileBytes = BM * BK * 2;          // 16 KiB per operand tile
constexpr int kStageBytes = 2 * kTileBytes;      // A + B
static_assert(kGemmLdsBytes == 2 * kStageBytes, "LDS budget mismatch");
static_assert(BM == BN, "staging assumes square tiles");
constexpr int kGroupM = 8;

__device__ __forceinline__ int tile_off(int r, int c) {
  return r * 128 + ((c ^ ((r >> 1) & 7)) << 4);
}

// Each wave DMAs 4 x 1 KiB (8 rows x 128 B each) of one operand tile.
__device__ __forceinline__ void stage_tile(const uint16_t* __restrict__ g,
                                           int ld, int row0, int rows,
                                           int k0, char* lds, int wave,
                                           int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int group = wave * 4 + i;
    const int r = group * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    int grow = row0 + r;
    grow = grow < rows ? grow : rows - 1;   // clamp: rows >= M are masked
    glds16(g + static_cast<size_t>(grow) * ld + k0 + c * 8,
           lds + group * 1024);
  }
}

__device__ __forceinline__ void mma_tile(const char* __restrict__ la,
                                         const char* __restrict__ lb,
                                         int wm, int wn, int lane,
                                         f32x4 (&acc)[4][4]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = s * 4 + (lane >> 4);
    bf16x8 xa[4], wb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[i] = *reinterpret_cast<const bf16x8*>(
          la + tile_off(wm * 64 + i * 16 + (lane & 15), c));
      wb[i] = *reinterpret_cast<const bf16x8*>(
          lb + tile_off(wn * 64 + i * 16 + (lane & 15), c));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            wb[j], xa[i], acc[i][j], 0, 0, 0);
  }
}

template <int EPI>
__global__ __launch_bounds__(kGemmThreads, 2) void gemm_bf16_tn_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B,
    uint16_t* __restrict__ C, const float* __restrict__ bias,
    const uint16_t* __restrict__ R, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = N / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int wg = xcd_remap(static_cast<int>(blockIdx.x), tiles_m * tiles_n);
  const int per_group = kGroupM * tiles_n;
  const int group = wg / per_group;
  const int first_m = group * kGroupM;
  const int gsize = min(tiles_m - first_m, kGroupM);
  const int in_group = wg - group * per_group;
  const int m0 = (first_m + in_group % gsize) * BM;
  const int n0 = (in_group / gsize) * BN;

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  char* buf0 = smem;
  char* buf1 = smem + kStageBytes;
  const int kt_count = K / BK;
  stage_tile(A, K, m0, M, 0, buf0, wave, lane);
  stage_tile(B, K, n0, N, 0, buf0 + kTileBytes, wave, lane);
  wait_vmcnt0();
  __syncthreads();
  for (int kt = 0; kt < kt_count; ++kt) {
    char* cur = (kt & 1) ? buf1 : buf0;
    char* nxt = (kt & 1) ? buf0 : buf1;
    if (kt + 1 < kt_count) {
      stage_tile(A, K, m0, M, (kt + 1) * BK, nxt, wave, lane);
      stage_tile(B, K, n0, N, (kt + 1) * BK, nxt + kTileBytes, wave, lane);
    }
    mma_tile(cur, cur + kTileBytes, wm, wn, lane, acc);
    wait_vmcnt0();
    __syncthreads();
  }

  // Epilogue: acc[i][j][r] = C[m][nb + r], m on the lane, 4 columns per lane.
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nb = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      if (EPI != EPI_NONE) {
        const float4 b = *reinterpret_cast<const float4*>(bias + nb);
        v[0] += b.x; v[1] += b.y; v[2] += b.z; v[3] += b.w;
      }
      if (EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      }
      const size_t off = static_cast<size_t>(m) * N + nb;
      if (EPI == EPI_BIAS_RESIDUAL) {
        const uint2 res = *reinterpret_cast<const uint2*>(R + off);
        v[0] += bf16_to_f32(res.x & 0xffff);
        v[1] += bf16_to_f32(res.x >> 16);
        v[2] += bf16_to_f32(res.y & 0xffff);
        v[3] += bf16_to_f32(res.y >> 16);
      }
      uint2 out;
      out.x = f32_to_bf16(v[0]) | (static_cast<uint32_t>(f32_to_bf16(v[1])) << 16);
      out.y = f32_to_bf16(v[2]) | (static_cast<uint32_t>(f32_to_bf16(v[3])) << 16);
      *reinterpret_cast<uint2*>(C + off) = out;
    }
  }
}

template <int EPI>
hipError_t configure_epi() {
  hipError_t err = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&gemm_bf16_tn_kernel<EPI>),
      hipFuncAttributeMaxDynamicSharedMemorySize, kGemmLdsBytes);
  return err == hipSuccess ? prepare_kernel(&gemm_bf16_tn_kernel<EPI>) : err;
}

template <int EPI>
hipError_t launch_epi(const uint16_t* A, const uint16_t* B, uint16_t* C,
                      const float* bias, const uint16_t* R, int M, int N,
                      int K, hipStream_t stream) {
  const int blocks = ((M + BM - 1) / BM) * (N / BN);
  return launch_kernel(&gemm_bf16_tn_kernel<EPI>, dim3(blocks),
                     dim3(kGemmThreads), kGemmLdsBytes, stream, A, B, C, bias,
                     R, M, N, K);
}

}  // namespace

// Raise the dynamic-LDS limits and resolve every launch handle once,
// outside any graph capture (once per device that succeeded: these runtime
// calls take the registry lock, see launch.hpp).
hipError_t gemm_prepare() {
  static std::atomic<unsigned long long> done{0};
  return prepare_per_device(done, [] {
    hipError_t err = configure_epi<EPI_NONE>();
    if (err == hipSuccess) err = configure_epi<EPI_BIAS_GELU>();
    if (err == hipSuccess) err = configure_epi<EPI_BIAS_RESIDUAL>();
    if (err == hipSuccess) err = gemm256_prepare();
    return err;
  });
}

int gemm_pick_variant(int M, int N, int K, bool have_workspace) {
  // the 256-row ring kernels run one block per CU: use the 256x256 one
  // when its grid fills the 256 CUs, else split K across the idle CUs
  // (needs a workspace), else the 256x128 ring, else the 128x128 kernel
  const int rows = (M + 255) / 256;
  if (gemm256_shape_ok(M, N, K, 256) && rows * (N / 256) >= 256)
    return gemm256w4_shape_ok(M, N, K) ? GEMM_256W4 : GEMM_256;
  if (have_workspace && gemm256_shape_ok(M, N, K, 256) &&
      gemm256_splits(M, N, K) > 1)
    return GEMM_256_SPLITK;
  if (gemm256_shape_ok(M, N, K, 128) && rows * (N / 128) >= 256)
    return GEMM_256x128;
  return GEMM_128;
}

size_t gemm_workspace_bytes(int M, int N, int K) {
  return gemm256_splitk_workspace(M, N, K);
}

hipError_t launch_gemm_variant(const uint16_t* A, const uint16_t* B,
                               uint16_t* C, const float* bias,
                               const uint16_t* R, int M, int N, int K,
                               int epilogue, int variant, hipStream_t stream,
                               float* workspace, size_t workspace_bytes) {
  if ((epilogue != EPI_NONE && bias == nullptr) ||
      (epilogue == EPI_BIAS_RESIDUAL && R == nullptr) ||
      epilogue < EPI_NONE || epilogue > EPI_BIAS_RESIDUAL)
    return hipErrorInvalidValue;
  if (variant == GEMM_AUTO)
    variant = gemm_pick_variant(
        M, N, K, workspace != nullptr &&
                     workspace_bytes >= gemm_workspace_bytes(M, N, K));
  if (variant == GEMM_256_SPLITK) {
    return launch_gemm256_splitk(A, B, C, bias, R, M, N, K, epilogue,
                                 gemm256_splits(M, N, K), workspace,
                                 workspace_bytes, stream);
  }
  if (variant == GEMM_256 || variant == GEMM_256x128) {
    return launch_gemm256(A, B, C, bias, R, M, N, K, epilogue, stream,
                          variant == GEMM_256 ? 256 : 128);
  }
  if (variant == GEMM_256W4)
    return launch_gemm256(A, B, C, bias, R, M, N, K, epilogue, stream, 256,
                          4);
  if (variant == GEMM_256W4P)
    return launch_gemm256_persist(A, B, C, bias, R, M, N, K, epilogue,
                                  stream);
  return launch_gemm(A, B, C, bias, R, M, N, K, epilogue, stream);
}

bool gemm_shape_ok(int M, int N, int K) {
  return M >= 1 && N >= BN && K >= BK && N % BN == 0 && K % BK == 0;
}

hipError_t launch_gemm(const uint16_t* A, const uint16_t* B, uint16_t* C,
                       const float* bias, const uint16_t* R, int M, int N,
                       int K, int epilogue, hipStream_t stream) {
  if (!gemm_shape_ok(M, N, K)) return hipErrorInvalidValue;
  switch (epilogue) {
    case EPI_NONE:
      return launch_epi<EPI_NONE>(A, B, C, bias, R, M, N, K, stream);
    case EPI_BIAS_GELU:
      if (bias == nullptr) return hipErrorInvalidValue;
      return launch_epi<EPI_BIAS_GELU>(A, B, C, bias, R, M, N, K, stream);
    case EPI_BIAS_RESIDUAL:
      if (bias == nullptr || R == nullptr) return hipErrorInvalidValue;
      return launch_epi<EPI_BIAS_RESIDUAL>(A, B, C, bias, R, M, N, K, stream);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace kiosk
