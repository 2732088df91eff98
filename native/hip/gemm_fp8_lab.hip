// Tools-only fp8 experiment dispatch (libamdgo_gemm_lab.so; see gemm_bf16_lab.hip): every schedule
// placement of the fp8 kernels under its variant number, without automatic switches.
//   1 .. 4 = schedule placements, 5 / 6 = 4 / 3 with serpentine K, 7 / 8 = 4 / 3 with the loop
//   rotated at slot B1, 9 = 4 with both, 10 / 11 = persistent with the schedules of 4 / 3,
//   12 = 10 with serpentine K, 13 = 9 with the square cross-XCD raster; 20-37 = q16 placements;
//   40 / 41 = persistent q16 (41: serpentine K).
#include "gemm_fp8_asm_loop_lab.h"  // every schedule (masks the production header)
#include "gemm_fp8_kernels.h"

extern "C" {

int amdgo_lab_gemm_fp8(int v, const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % F8_BM || N % F8_BN || K % F8_BK || K < 2 * F8_BK)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const uint8_t*)A;
  const auto* b = (const uint8_t*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / F8_BM) * (N / F8_BN);
  const int cus = device_cu_count();
  const int pgrid = ((nwg < cus ? nwg : cus) / NXCD) * NXCD;
  if (v >= 10 && v <= 12 && pgrid >= NXCD) {
    auto kern = v == 10 ? gemm_fp8_256x256_w4sp<6, 7, 16, 24, 6>
              : v == 11 ? gemm_fp8_256x256_w4sp<4, 5, 20, 22, 8>
                        : gemm_fp8_256x256_w4sp<6, 7, 16, 24, 6, true>;
    hipLaunchKernelGGL(kern, dim3(pgrid), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
  } else if ((v == 40 || v == 41) && pgrid >= NXCD) {   // persistent q16 (41: serpentine K)
    auto kern = v == 40 ? gemm_fp8_256x256_q16p<> : gemm_fp8_256x256_q16p<16, 18, 3, 34, 35, 43, true>;
    hipLaunchKernelGGL(kern, dim3(pgrid), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v == 13 && (M / F8_BM) % 16 == 0 && (N / F8_BN) % 16 == 0) {
    hipLaunchKernelGGL((gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 32, true, true>), dim3(nwg), dim3(F8_THREADS), 0, s,
                       a, b, c, M, N, K);
  } else if (v >= 20 && v <= 37) {                   // q16: unscaled 16x16x128 f8f6f4 MFMA
    // 20-22: one DMA piece per slot; 23: pieces every other slot; 24: landing wait right after the
    // free barrier, reads as soon as each fragment dies; 25: mid landing wait; 26/27 = 24/25 with the
    // serpentine K and the square raster; 28-30: pieces every third slot, landing wait at 34 / 42 /
    // 26; 31 / 32 = 27 / 28 without the square raster; 33 = 28 with the free barrier one slot
    // earlier; 34 = 28 with reads every third slot between the DMA pieces, 35 = 34 unsquared;
    // 36 / 37 = 28 / 32 with the K offset in the lane offset (VK)
    auto kern = v == 20 ? gemm_fp8_256x256_q16<>
              : v == 21 ? gemm_fp8_256x256_q16<16, 18, 1, 34, 36, 48, 32>
              : v == 22 ? gemm_fp8_256x256_q16<16, 18, 1, 34, 36, 48, 32, true>
              : v == 23 ? gemm_fp8_256x256_q16<16, 18, 2, 49, 51, 52, 32, true, 2, 3>
              : v == 24 ? gemm_fp8_256x256_q16<16, 21, 2, 18, 20, 36, 0, false, 4, 4, true>
              : v == 25 ? gemm_fp8_256x256_q16<16, 18, 2, 34, 35, 43, 0, false, 2, 2, true>
              : v == 26 ? gemm_fp8_256x256_q16<16, 21, 2, 18, 20, 36, 32, true, 4, 4, true>
              : v == 27 ? gemm_fp8_256x256_q16<16, 18, 2, 34, 35, 43, 32, true, 2, 2, true>
              : v == 28 ? gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, true, 2, 2, true>
              : v == 29 ? gemm_fp8_256x256_q16<16, 18, 3, 42, 43, 44, 32, true, 2, 2, true>
              : v == 30 ? gemm_fp8_256x256_q16<16, 18, 3, 26, 27, 36, 32, true, 2, 4, true>
              : v == 31 ? gemm_fp8_256x256_q16<16, 18, 2, 34, 35, 43, 32, false, 2, 2, true>
              : v == 32 ? gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, false, 2, 2, true>
              : v == 33 ? gemm_fp8_256x256_q16<15, 17, 3, 34, 35, 43, 32, true, 2, 2, true>
              : v == 34 ? gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 46, 32, true, 3, 3, true>
              : v == 35 ? gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 46, 32, false, 3, 3, true>
              : v == 36 ? gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, true, 2, 2, true, true>
                        : gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, false, 2, 2, true, true>;
    if ((v == 22 || v == 23 || (v >= 26 && v <= 30) || v == 33 || v == 34 || v == 36) && ((M / F8_BM) % 16 || (N / F8_BN) % 16))
      return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 1 && v <= 9) {
    auto kern = v == 1 ? gemm_fp8_256x256_w4s<5, 5, 16, 20, 10>
              : v == 2 ? gemm_fp8_256x256_w4s<5, 6, 12, 18, 12>
              : v == 3 ? gemm_fp8_256x256_w4s<4, 5, 20, 22, 8>
              : v == 4 ? gemm_fp8_256x256_w4s<6, 7, 16, 24, 6>
              : v == 5 ? gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 32>
              : v == 6 ? gemm_fp8_256x256_w4s<4, 5, 20, 22, 8, 32>
              : v == 7 ? gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 0, true>
              : v == 8 ? gemm_fp8_256x256_w4s<4, 5, 20, 22, 8, 0, true>
                       : gemm_fp8_256x256_w4s<6, 7, 16, 24, 6, 32, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
