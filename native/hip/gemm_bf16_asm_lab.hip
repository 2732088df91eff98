// Tools-only A/B library for the hand-scheduled bf16 K pipeline (gemm_bf16_256x256_w4a): the
// production v44 next to the asm-loop schedules, in one code object so tools/asm_lab.py can
// interleave them with hipBLASLt in one process. Never loaded by the validator.
//   44  = w4s v44 (production: serpentine K, loop rotation, VK)
//   100 + SC = w4a with schedule SC (gemm_bf16_asm_loop.h lists them), serpentine K
//   120 = w4a schedule 0 without serpentine K
//   25  = w4sp v25 (production for short K: persistent, VK)
//   45  = w4s v45 (production for big square grids: v44 + square cross-XCD raster)
//   130 + SC = w4ap (persistent) with persistent schedule SC, serpentine K; 133 = schedule 0 without
//   150 / 151 = w4ap square raster (SQ) with persistent schedule 5 / 9; 152 = 150 without serpentine K
#include "gemm_bf16_kernels.h"

extern "C" {

int amdgo_asmlab_gemm_bf16(int v, const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M % BM || N % BN || K % (2 * BK) || K < 4 * BK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const __bf16*)A;
  const auto* b = (const __bf16*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / BM) * (N / BN);
  switch (v) {
    case 44:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
#define W4A_CASE(V, SC, SERP)                                                                             \
    case V:                                                                                               \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4a<SC, SERP, false>), dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, \
                         M, N, K);                                                                        \
      break;
    case 25: {
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40, false, true>), dim3(g), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    }
    case 45:
      if ((M / BM) % 16 || (N / BN) % 16) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    W4A_CASE(100, 0, 32)
    W4A_CASE(101, 1, 32)
    W4A_CASE(102, 2, 32)
    W4A_CASE(103, 3, 32)
    W4A_CASE(104, 4, 32)
    W4A_CASE(105, 5, 32)
    W4A_CASE(106, 6, 32)
    W4A_CASE(107, 7, 32)
    W4A_CASE(108, 8, 32)
    W4A_CASE(109, 9, 32)
    W4A_CASE(110, 10, 32)
    W4A_CASE(111, 11, 32)
    W4A_CASE(112, 12, 32)
    W4A_CASE(120, 0, 0)
#define W4AP_CASE(V, SC, SERP)                                                                             \
    case V: {                                                                                             \
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;                   \
      if (g < NXCD) return (int)hipErrorInvalidValue;                                                     \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<SC, SERP>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K); \
      break;                                                                                              \
    }
    W4AP_CASE(130, 0, true)
    W4AP_CASE(131, 1, true)
    W4AP_CASE(132, 2, true)
    W4AP_CASE(133, 0, false)
    W4AP_CASE(134, 3, true)
    W4AP_CASE(135, 4, true)
    W4AP_CASE(136, 5, true)
    W4AP_CASE(137, 6, true)
    W4AP_CASE(138, 7, true)
    W4AP_CASE(139, 8, true)
    W4AP_CASE(140, 9, true)
    W4AP_CASE(141, 10, true)
    W4AP_CASE(142, 11, true)
    W4AP_CASE(143, 12, true)
#define W4APSQ_CASE(V, SC, SERP)                                                                           \
    case V:                                                                                               \
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;    \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<SC, SERP, true>), dim3(256), dim3(W4_THREADS), 0, s, a, b, c, \
                         M, N, K);                                                                        \
      break;
    W4APSQ_CASE(150, 5, true)
    W4APSQ_CASE(151, 9, true)
    W4APSQ_CASE(152, 5, false)
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
