// CDNA4 (gfx950) bf16 GEMM for the node validator workload -- the shipped dispatch.
//
//   C[M,N] (bf16) = A[M,K] (bf16, K-major) * Bt[N,K]^T (bf16, K-major), fp32 accumulation.
//
// This replaces the reference operator's only GPU code, the prebuilt CUDA-samples
// `vectorAdd` binary that its validator image copies in (validator/Dockerfile:33-35,
// validator/cuda-workload-validation.yaml:20). There the kernel was a pass/fail
// check; here it is a throughput probe that exercises the matrix cores, LDS and HBM.
//
// Design (MI355X-first, see docs/validator-gemm.md; kernels in gemm_bf16_kernels.h):
//   * 256x256 output tile per 256-thread workgroup: one wave64 per SIMD, each owning a 128x128
//     sub-tile = 8x8 MFMA 16x16x32 accumulators pinned in all 256 AGPRs (inline-asm MFMAs).
//   * K-step BK=64, two LDS buffers staged by `buffer_load ... lds` (LDS-DMA, no VGPR round trip),
//     XOR-swizzled on the source address; the v18 K-tile schedule interleaves fragment reads,
//     DMA pieces and two barriers into the 128-MFMA stream of each K-tile.
//   * XCD-aware rasters (8 XCDs with private L2): a bijective XCD-contiguous remap plus grouped
//     raster, serpentine K across dispatch waves, and a square cross-XCD super-tile raster.
//
// Only numerically exact, measured production kernels are reachable from here. The variant is an
// API argument (amdgo_gemm_set_variant), never read from the environment; superseded generations
// and knock-out timings live in the tools-only gemm_bf16_lab.hip.
//   0  = automatic (default): on the 256-CU MI355X with a power-of-two K >= 256, the persistent asm
//        K pipeline -- v50, v51 (square raster: >= 8 dispatch waves, K >= 8192, 16x16-tile
//        multiples), v52 (one or two dispatch waves, K >= 32768), v56 (16x16-tile multiples with K <= 2048
//        or one dispatch wave), v55 (other one-wave grids); otherwise v44, v25 for K <= 4096
//        with >= 2 tiles per CU, v45 for >= 8 dispatch waves with K >= 8192 on 16x16-tile
//        multiples; v42 / v18 on devices without 256 CUs.
//   53 / 54 = the asm pipeline (g4) in the VP DMA form (gemm_w4ap.h DM 1), linear / square raster: the
//        default when K is not a power of two (an even number of K-tiles, >= 4).
//   47 / 48 = v44 / v45 with permuted A-panel DMA rows (PA), the default for other K not a power of two.
//   50 / 51 / 52 = the asm pipeline: w4ap (gemm_bf16_kernels.h) with the g4 schedule, g4 on the square
//        raster, the g6d6 schedule (tools/gen_bf16_asm_loop.py generates gemm_bf16_asm_loop.h).
//   55 / 56 (round 4) = v53 / v54 with the A-panel pieces reading rows 32 apart (PA, DM 2) and the LEAN
//        epilogue (EPI 15: conflict-free staging, saddr C stores; v56 pipelines it over 8 half-passes and
//        interleaves each half-pass's stores into the next one's staging, EPI 17 LEAN_ILV: 16384^2x1024
//        +2.2 %, 8192^2x2048 +1.2 % over the plain pipeline, profiles/r4_sweep/lab_ilv_*.jsonl;
//        gemm_w4ap.h): the power-of-two-K default for short K or one dispatch wave.
//   18 / 25 / 42 / 44 / 45 / 47 / 48 / 50 / 51 / 52 / 53 / 54 / 55 / 56 = that kernel pinned (no automatic switch; still falls back to a kernel
//        that can run the shape or the device).
// Every w4s / w4sp kernel here carries the K offset of its LDS-DMA pieces in the lane offset (VK: one VALU
// add per K-tile, loop-invariant soffsets; 17 fewer SALU per K-tile, +0.6-0.8 % at 8192^3 and
// 16384^3, profiles/r2_sched/sweep_vk.jsonl).
// A bounds-checked generic kernel handles shapes that are not multiples of the tile.

#include "gemm_bf16_kernels.h"

// K-tile schedules of the persistent asm pipeline (gemm_bf16_asm_loop.h, tools/gen_bf16_asm_loop.py):
// g4 waits for the last R1 fragment read 4 MFMAs after it is issued (not 1), which takes the
// lgkmcnt stall out of the free barrier; g6d6 also spaces the DMA pieces 6 MFMAs apart, which
// spreads the HBM requests of a one-wave grid whose workgroups run in lockstep.
// profiles/r3_asm/asm8_summary.jsonl, asm9_summary.jsonl
// Every tile's first K-tile starts its accumulators with src C = 0 (the *_zc schedules, EPI 8), so the
// epilogue reads the accumulators without writing zeros back: 8192^3 +0.8 %, 8192^2x2048 +1.4 %
// (profiles/r3_s2/zc_bf16.jsonl).
// The C tile leaves through nontemporal (streaming) stores: the next tile's first landing wait and
// the end-of-kernel release no longer wait on C lines allocated in L2 (8192^3 +1.1 %, one dispatch
// wave 4096^2x16384 +6.3 %; profiles/r3_s2/nt_*.jsonl).
#define W4AP_SC_MAIN W4AP_SC_G4_ZC
#define W4AP_SC_LONGK W4AP_SC_G6D6_ZC

static int g_variant = 0;

// Persistent grid: one workgroup per CU (the 160 KiB LDS admits one), a multiple of the 8 XCDs,
// never more workgroups than tiles. 0 when the device or the tile count is too small.
static int persistent_grid(int nwg, hipStream_t s) {
  const int cus = device_cu_count(s);
  const int g = nwg < cus ? nwg : cus;
  return (g / NXCD) * NXCD;
}

// The kernel amdgo_gemm_bf16 runs for this shape on the device of stream `s` (0 = generic).
static int resolve_variant(int M, int N, int K, hipStream_t s) {
  if (M % BM || N % BN || K % BK || K < 2 * BK) return 0;
  const int nwg = (M / BM) * (N / BN);
  const int cus = device_cu_count(s);
  const bool sq = (M / BM) % 16 == 0 && (N / BN) % 16 == 0;
  int v = g_variant;
  const bool pow2k = (K & (K - 1)) == 0;
  if (v == 0 && cus == 256 && !pow2k && K % (2 * BK) == 0 && K >= 4 * BK && persistent_grid(nwg, s) >= NXCD) {
    // K not a power of two: the asm pipeline in the VP DMA form (per-piece VGPR lane offsets, the K
    // offset in one SGPR): 12288^3 1.02x hipBLASLt (v48 0.98x, the DM-0 asm form 0.88x),
    // 8192^2x12288 1.07x (v47 1.02x), 12288^2x10240 1.03x (v48 1.03x); profiles/r3_s2/vp_bf16.jsonl.
    // v54 = the same on the square cross-XCD raster for >= 8 dispatch waves on 16x16-tile multiples:
    // 12288^3 1.05x (v53 1.03x), 12288^2x10240 1.07x (v53 1.04x); profiles/r3_s2/vpsq_bf16.jsonl
    v = (sq && nwg >= 8 * cus) ? 54 : 53;
  } else if (v == 0 && cus == 256 && pow2k && K >= 4 * BK && persistent_grid(nwg, s) >= NXCD) {
    // The hand-scheduled asm K pipeline, persistent (profiles/r3_asm/): v50 everywhere it runs,
    // ahead of v44 and v25 on every measured shape (8192^3 +2-3 %, 8192^2x2048 +7 %,
    // 16384^2x1024 +14 % over v44); its square-raster form v51 for >= 8 dispatch waves with long K
    // (16384^3 1.01x hipBLASLt, v45 0.98x); the DMA-spaced schedule v52 for one or two dispatch
    // waves with very long K (with nontemporal C stores: 4096^2x32768 +1.0 % over v50, but v50 ahead
    // at 4096^2x16384 by 1.9 % and at 4096x8192x8192 by 0.5 %; profiles/r3_s2/longk_bf16.jsonl).
    v = 50;
    if (sq && nwg >= 8 * cus && K >= 128 * BK) v = 51;
    else if (nwg <= 2 * cus && K >= 512 * BK) v = 52;
    // Round 4 (profiles/r4_lean/, r4_prod/): on 16x16-tile multiples with short K (<= 2048) or one
    // dispatch wave, v56 (VP + PA DMA, pipelined LEAN epilogue, square raster): 16384^2x1024 1440 TF/s =
    // 1.08x hipBLASLt (v50 1.06x), 8192^2x1024 1.09x (1.02x), 8192^2x2048 1.05x (1.03x), 4096^2x2048
    // 1.03x (1.00x); other one-wave grids v55 (VP + PA, LEAN, linear raster).
    else if (sq && (K <= 32 * BK || nwg <= cus)) v = 56;
    else if (nwg <= cus) v = 55;
  } else if (v == 0) {
    v = 44;
    // Short K (K-loop of <= 64 K-tiles) with several tiles per CU: the persistent v25 hides each
    // tile's prologue and epilogue under the neighbouring K-loops (16384x16384x1024: +10 %;
    // K = 3072 +1.2 %, K = 4096 +0.3-0.7 %: profiles/r2_sched/sweep_persistent_midk.jsonl).
    if (K <= 64 * BK && nwg >= 2 * cus) v = 25;
    // Big grids (>= 8 dispatch waves) with long K: the square cross-XCD raster (v45) streams fewer
    // distinct panels per wave (profiles/r1_s6_sq: 12288^3 +5.5 %, 16384x8192x8192 +2.9 %,
    // 16384^3 +3.4 %; at 4 waves or K = 4096 it measured 1 % behind v44, so those stay on v44).
    else if (sq && nwg >= 8 * cus && K >= 128 * BK) v = 45;
  }
  if (v == 45 && !sq) v = 44;                           // square raster needs 16x16 super-tiles
  if (v == 48 && !sq) v = 47;
  if ((v == 47 || v == 48) && cus != 256) v = 42;
  if (v == 25 && persistent_grid(nwg, s) < NXCD) v = 44;
  // w4ap runs an even number of K-tiles (>= 4) on a grid of whole XCD groups; its square raster
  // (v51) needs exactly 256 workgroups over 16x16 super-tiles
  if ((v == 50 || v == 51 || v == 52 || v == 53 || v == 54 || v == 55 || v == 56) &&
      (K % (2 * BK) != 0 || K < 4 * BK || persistent_grid(nwg, s) < NXCD))
    v = 44;
  if (v == 54 && (!sq || cus != 256)) v = 53;
  if (v == 56 && (!sq || cus != 256)) v = 55;
  if (v == 51 && (!sq || cus != 256)) v = 50;
  if ((v == 44 || v == 45) && cus != 256) v = 42;       // serpentine K assumes 32 co-resident WGs / XCD
  // K not a power of two: A-panel DMA instructions read rows 32 apart (PA, v47 / v48). At a 24 KiB
  // row stride adjacent rows cost 8-11 % (12288^3 1405 -> 1557 TF, 8192^2x12288 1457 -> 1579,
  // 12288^2x10240 +5 %); at power-of-two K it is neutral (8192) or worse (16384: -8 %).
  // profiles/r2_sched/sweep_pa.jsonl
  if (g_variant == 0 && !pow2k) {
    if (v == 44) v = 47;
    else if (v == 45) v = 48;
  }
  return v;
}

extern "C" {

// 0 on success; hipErrorInvalidValue for a variant outside the production set.
int amdgo_gemm_set_variant(int v) {
  if (v != 0 && v != 18 && v != 25 && v != 42 && v != 44 && v != 45 && v != 47 && v != 48 && v != 50 &&
      v != 51 && v != 52 && v != 53 && v != 54 && v != 55 && v != 56)
    return (int)hipErrorInvalidValue;
  g_variant = v;
  return 0;
}
int amdgo_gemm_get_variant() { return g_variant; }
int amdgo_gemm_resolve_variant(int M, int N, int K) { return resolve_variant(M, N, K, nullptr); }

// Returns 0 on success, a hipError_t value otherwise. `stream` may be null.
int amdgo_gemm_bf16(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const __bf16*)A;
  const auto* b = (const __bf16*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / BM) * (N / BN);
  switch (resolve_variant(M, N, K, s)) {
    case 18:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 0, false, false, true>), dim3(nwg), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 25:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40, false, true>), dim3(persistent_grid(nwg, s)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 42:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 0, true, false, true>), dim3(nwg), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 44:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true>), dim3(nwg), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 47:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 48:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 45:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true>), dim3(nwg), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 50:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_MAIN, true, false, W4AP_EPI_STAGED_ZC>), dim3(persistent_grid(nwg, s)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 51:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_MAIN, true, true, W4AP_EPI_STAGED_ZC>), dim3(256), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 53:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_STAGED_ZC, 1>), dim3(persistent_grid(nwg, s)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 54:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_STAGED_ZC, 1>), dim3(256), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 55:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_LEAN, 2>), dim3(persistent_grid(nwg, s)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 56:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN_ILV, 2>), dim3(256), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 52:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_LONGK, true, false, W4AP_EPI_STAGED_ZC>), dim3(persistent_grid(nwg, s)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    default: {
      dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
      hipLaunchKernelGGL(gemm_bf16_generic, grid, dim3(256), 0, s, a, b, c, M, N, K);
    }
  }
  return (int)hipGetLastError();
}

// Force the generic kernel (independent implementation used by tests).
int amdgo_gemm_bf16_generic(const void* A, const void* Bt, void* C, int M, int N, int K,
                            void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
  hipLaunchKernelGGL(gemm_bf16_generic, grid, dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
  return (int)hipGetLastError();
}

int amdgo_gemm_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out,
                        int N, int K, void* stream) {
  dim3 grid((N + 255) / 256, nrows);
  hipLaunchKernelGGL(gemm_ref_rows, grid, dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)A, (const __bf16*)Bt, rows, nrows, out, N, K);
  return (int)hipGetLastError();
}

int amdgo_fill_uniform_bf16(void* p, size_t n, uint32_t seed, void* stream) {
  hipLaunchKernelGGL(fill_uniform_bf16, dim3(2048), dim3(256), 0, (hipStream_t)stream,
                     (__bf16*)p, n, seed);
  return (int)hipGetLastError();
}

// Tile constraints of the fast path (for host-side shape checks).
int amdgo_gemm_tile_m() { return BM; }
int amdgo_gemm_tile_n() { return BN; }
int amdgo_gemm_tile_k() { return BK; }

}  // extern "C"
