// CDNA4 (gfx950) fp8 GEMM for the node validator workload -- the shipped dispatch.
//
//   C[M,N] (bf16) = A[M,K] (fp8 e4m3fn, K-major) * Bt[N,K]^T (fp8 e4m3fn, K-major), fp32 accumulation.
//
// Kernels and design: gemm_fp8_kernels.h (block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 with unit
// scales = the matrix cores' fp8 rate). Only the measured production kernels are reachable; the
// variant is an API argument, never read from the environment (placement sweeps live in the
// tools-only gemm_fp8_lab.hip).
//   0 = automatic (default): v9 (v4 schedule + serpentine K + loop rotation); v10 (persistent) for
//       K <= 2048 with >= 2 tiles per CU; v13 (v9 + square cross-XCD raster) for >= 16 dispatch waves
//       with K >= 16384 on 16x16-tile multiples; v7 / v4 on devices without 256 CUs.
//   4 / 7 / 9 / 10 / 13 = that kernel pinned (no automatic switch; falls back when the shape or the
//       device cannot run it).
// Fast path: M % 256 == 0, N % 256 == 0, K % 128 == 0, K >= 256; otherwise the generic kernel.

#include "gemm_fp8_kernels.h"

static int g_fp8_variant = 0;

static int resolve_fp8_variant(int M, int N, int K) {
  if (M % F8_BM || N % F8_BN || K % F8_BK || K < 2 * F8_BK) return 0;
  const int nwg = (M / F8_BM) * (N / F8_BN);
  const int cus = device_cu_count();
  const int pgrid = ((nwg < cus ? nwg : cus) / NXCD) * NXCD;     // persistent grid: one WG per CU
  const bool sq = (M / F8_BM) % 16 == 0 && (N / F8_BN) % 16 == 0;
  int v = g_fp8_variant;
  if (v == 0) {
    v = 9;
    // Short K (<= 16 K-tiles) with several tiles per CU: the persistent kernel hides each tile's
    // prologue and epilogue under the neighbouring K-loops.
    if (K <= 16 * F8_BK && nwg >= 2 * cus) v = 10;
    // The square cross-XCD raster (as bf16 v45) only pays for fp8 on the biggest grids: at
    // 16384^3 +4.3 %, but 12288^3, 16384x8192x8192 and 16384^2x8192 ran 1-3 % behind v9
    // (profiles/r1_s6_sq). fp8 panels are half the bytes, so the panel traffic it saves matters less.
    else if (sq && nwg >= 16 * cus && K >= 128 * F8_BK) v = 13;
  }
  if (v == 13 && !sq) v = 9;
  if (v == 10 && pgrid < NXCD) v = 9;
  if ((v == 9 || v == 13) && cus != 256) v = 7;
  return v;
}

extern "C" {

// 0 on success; hipErrorInvalidValue for a variant outside the production set.
int amdgo_gemm_fp8_set_variant(int v) {
  if (v != 0 && v != 4 && v != 7 && v != 9 && v != 10 && v != 13) return (int)hipErrorInvalidValue;
  g_fp8_variant = v;
  return 0;
}
int amdgo_gemm_fp8_get_variant() { return g_fp8_variant; }
int amdgo_gemm_fp8_resolve_variant(int M, int N, int K) { return resolve_fp8_variant(M, N, K); }

// Returns 0 on success, a hipError_t value otherwise. `stream` may be null.
int amdgo_gemm_fp8(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const uint8_t*)A;
  const auto* b = (const uint8_t*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / F8_BM) * (N / F8_BN);
  const int cus = device_cu_count();
  const int pgrid = ((nwg < cus ? nwg : cus) / NXCD) * NXCD;
  switch (resolve_fp8_variant(M, N, K)) {
    case 4:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4s<6, 7, 16, 24, 6>), dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 7:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 0, true>), dim3(nwg), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 9:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 32, true>), dim3(nwg), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 10:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4sp<6, 7, 16, 24, 6>), dim3(pgrid), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 13:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 32, true, true>), dim3(nwg), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    default: {
      dim3 grid((N + G8 - 1) / G8, (M + G8 - 1) / G8);
      hipLaunchKernelGGL(gemm_fp8_generic, grid, dim3(256), 0, s, a, b, c, M, N, K);
    }
  }
  return (int)hipGetLastError();
}

int amdgo_gemm_fp8_generic(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + G8 - 1) / G8, (M + G8 - 1) / G8);
  hipLaunchKernelGGL(gemm_fp8_generic, grid, dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)A, (const uint8_t*)Bt, (__bf16*)C, M, N, K);
  return (int)hipGetLastError();
}

int amdgo_gemm_fp8_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out,
                            int N, int K, void* stream) {
  dim3 grid((N + 255) / 256, nrows);
  hipLaunchKernelGGL(gemm_fp8_ref_rows, grid, dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)A, (const uint8_t*)Bt, rows, nrows, out, N, K);
  return (int)hipGetLastError();
}

int amdgo_fill_uniform_fp8(void* p, size_t n, uint32_t seed, void* stream) {
  hipLaunchKernelGGL(fill_uniform_fp8, dim3(2048), dim3(256), 0, (hipStream_t)stream,
                     (uint8_t*)p, n, seed);
  return (int)hipGetLastError();
}

int amdgo_gemm_fp8_tile_m() { return F8_BM; }
int amdgo_gemm_fp8_tile_n() { return F8_BN; }
int amdgo_gemm_fp8_tile_k() { return F8_BK; }

}  // extern "C"
