// CDNA4 (gfx950) fp8 GEMM for the node validator workload -- the shipped dispatch.
//
//   C[M,N] (bf16) = A[M,K] (fp8 e4m3fn, K-major) * Bt[N,K]^T (fp8 e4m3fn, K-major), fp32 accumulation.
//
// Kernels and design: gemm_fp8_kernels.h. Only the measured production kernels are reachable; the
// variant is an API argument, never read from the environment (placement sweeps live in the
// tools-only gemm_fp8_lab.hip).
//   0 = automatic (default): v15 (q16: unscaled double-rate v_mfma_f32_16x16x128_f8f6f4, DMA pieces
//       every third MFMA slot, serpentine K); v16 (v15 + square cross-XCD raster) on 16x16-tile
//       multiples; v10 (persistent, block-scaled 32x32x64) for K <= 2048 with >= 2 tiles per CU;
//       v17 (q16 without serpentine K) on devices without 256 CUs; v18 (persistent q16: the next
//       tile's prologue DMA under the current tile's last K-tiles) for 2048 <= K <= 8192 with >= 4
//       tiles per CU (8192^3 +0.7-1.2 %, 16384^2x4096 +2.9 %; profiles/r2_fp8_q16/sweep_q16p*.jsonl).
//   20 / 21 (round 3, the default on the 256-CU MI355X for K a multiple of 256, K >= 512): q16ap, the
//       q16 K-tile body as one hand-scheduled asm block per output tile in the persistent frame of
//       the bf16 v50 (gemm_w4ap.h, tools/gen_fp8_asm_loop.py), nontemporal C stores (4096^3 +4.9 %,
//       16384^2x1024 +6.6 %): v20 schedule p, linear K; v21 the same
//       on the square cross-XCD raster with serpentine K, for >= 2 dispatch waves on 16x16-tile
//       multiples (8192^2x2048 1.03x vs v20 0.98x, 16384^2x4096 1.01x vs 0.99x; profiles/r3_s2/zc_fp8.jsonl).
//       Both start each tile's accumulators with src C = 0 (the p_zc schedule, EPI 8; 8192^2x2048 +3.9 %). Against hipBLASLt fp8 on MI355X (profiles/r3_s2/): 8192^3 1.005-1.021x (q16p
//       0.974-0.981x), 4096^3 1.04x, 16384^3 1.03x (v21), 16384^2x2048 1.05x (v21), 16384^2x1024
//       1.09x (v21), 16384x8192x8192 1.00x.
//   22 / 23 (round 4): v21 / v20 in the VP DMA form with the A-panel pieces reading rows 32 apart (PA,
//       DM 2; the p_zc schedule, gen_fp8_asm_loop.py VP) and the LEAN epilogue (v22: its pipelined,
//       store-interleaved form EPI 17, +0.4-0.5 % over EPI 15/16; v23: EPI 15 -- conflict-free
//       staging, saddr C stores, gemm_w4ap.h). v22 replaces v21 as the default on the square raster
//       when both sides have >= 32 tiles (v21 stays ahead with a 16-tile side at short K):
//       16384^2x1024 1.19x hipBLASLt (v21 1.13x), 12288^3 1.02x (v21 1.00x), 8192^2x2048 1.10x (1.08x),
//       16384^3 1.035x (1.031x), 8192^3 1.035x (1.023x); profiles/r4_lean/. One dispatch wave: v22 (v23 off the
//       16x16-tile multiples).
//   60 / 61 (round 5): the 128x128 small-grid kernel of the bf16 v60 / v61 (gemm_small.h) on the
//       double-rate v_mfma_f32_16x16x128_f8f6f4, whole-tile or split-K, for grids the 256x256 tiling
//       leaves mostly idle (and shapes only 128-tileable).
//   62 (round 5): the same frame in 256x128 tiles for 256-tile grids of a quarter to a half of the CUs.
//   24 (round 6): v23 in the split-K form of the asm frame (gemm_w4ap.h SPLIT): one (tile, K piece) per
//       workgroup, two pieces, the tile's last arrival sums; the default over v62 for 65-128-tile grids
//       with K >= 8192 (2560^2x16384 1.19x v62, 1.17x hipBLASLt; profiles/r6_splitk/band_fp8.jsonl).
//   10 / 15 / 16 / 17 / 18 / 20 / 21 / 22 / 23 / 24 / 60 / 61 / 62 = that kernel pinned (no automatic switch; falls back when the
//       shape or the device cannot run it).
// q16 vs the round-1 default (block-scaled 32x32x64, lab v9), same process, 4 boxes
// (profiles/r2_fp8_q16/): 8192^3 +5.3 %, 16384^3 +3.1 %, 4096^3 +4.1 %, 16384x8192x8192 +2.2 %.
// Fast path: M % 256 == 0, N % 256 == 0, K % 128 == 0, K >= 256; otherwise the generic kernel.

#include "gemm_fp8_kernels.h"
#include "gemm_raster_host.h"
#include "gemm_small_host.h"

// The variant a caller pinned (amdgo_gemm_fp8_set_variant): per host thread (see gemm_bf16.hip).
static thread_local int g_fp8_variant = 0;

// q16 schedule (lab v28 / v32): free barrier after slot 17, DMA pieces at slots 18, 21, .., 63,
// landing wait at 34, B0' reads from slot 35, A0' reads from 43 (block 2 walks A0 slowly).
#define Q16(SERP, SQ, REC) (gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, SERP, SQ, 2, 2, true, false, REC>)

// What the dispatch knows about a shape on a device.
struct Fp8Shape {
  int M, N, K, cus;
  bool tiles;      // M, N multiples of 256, K of 128, K >= 256: the 256x256 kernels can run it
  bool tiles128;   // M, N multiples of 128, K of 128: the 128x128 kernels (v60 / v61, gemm_small.h)
  int nwg, pgrid;  // 256x256 output tiles; the persistent grid (one WG per CU, whole XCD groups)
  bool sq;         // 16x16-tile multiples (the square cross-XCD raster)
  bool wide;       // >= 32 tiles on both sides
  bool ap;         // the q16ap asm frame can run it: the 256-CU MI355X, an even K-tile count >= 4
};

static Fp8Shape fp8_shape(int M, int N, int K, int cus) {
  Fp8Shape c{M, N, K, cus};
  c.tiles = M % F8_BM == 0 && N % F8_BN == 0 && K % F8_BK == 0 && K >= 2 * F8_BK;
  c.tiles128 = M % S_BM == 0 && N % S_BN == 0 && K % 128 == 0 && K >= 128;
  c.nwg = (M / F8_BM) * (N / F8_BN);
  c.pgrid = ((c.nwg < cus ? c.nwg : cus) / NXCD) * NXCD;
  c.sq = (M / F8_BM) % 16 == 0 && (N / F8_BN) % 16 == 0;
  c.wide = M / F8_BM >= 32 && N / F8_BN >= 32;
  c.ap = cus == 256 && K % (2 * F8_BK) == 0 && K >= 4 * F8_BK && c.pgrid >= NXCD;
  return c;
}

// The automatic dispatch, first match wins; each row names the sweep that put it there.
struct Fp8Rule {
  int variant;
  bool (*match)(const Fp8Shape&);
  const char* evidence;
};
static constexpr Fp8Rule kFp8Rules[] = {
    // a 256x256 grid of at most a quarter of the CUs (or a shape only 128-tileable): the 128x128
    // kernel, split-K when the 128x128 grid is under the CU count (the bf16 rows' rule, same kernel frame)
    // 33-64 256x256 tiles with K >= 32768: the asm frame split in four K pieces
    {24, [](const Fp8Shape& c) { return c.ap && c.tiles && 8 * c.nwg > c.cus && 4 * c.nwg <= c.cus && c.K >= 256 * F8_BK; },
     "profiles/r6_splitk/fp8_s34.jsonl (2048^2x32768 2357 vs 2004 TF/s, 1024x4096x32768 2466 vs 1762; 1.5x hipBLASLt)"},
    {61, [](const Fp8Shape& c) {
       return c.tiles128 && (!c.tiles || 4 * c.nwg <= c.cus) &&
              small_splits((c.M / S_BM) * (c.N / S_BN), c.K / 128, c.cus) > 1; },
     "profiles/r5_small/ (fp8 128x128 split-K)"},
    {60, [](const Fp8Shape& c) { return c.tiles128 && (!c.tiles || 4 * c.nwg <= c.cus); },
     "profiles/r5_small/ (fp8 128x128)"},
    {0, [](const Fp8Shape& c) { return !c.tiles; }, "generic bounds-checked kernel"},
    // a quarter to a half of the CUs in 256x256 tiles with K >= 8192: the asm frame split in two K pieces
    {24, [](const Fp8Shape& c) { return c.ap && 4 * c.nwg > c.cus && 2 * c.nwg <= c.cus && c.K >= 64 * F8_BK; },
     "profiles/r6_splitk/band_fp8.jsonl (2560^2x8192 1.02x v62, 2560^2x16384 1.19x, 2048x4096x16384 1.16x)"},
    // a quarter to a half of the CUs in 256x256 tiles: 256x128 tiles fill the chip in one wave
    {62, [](const Fp8Shape& c) { return 4 * c.nwg > c.cus && 2 * c.nwg <= c.cus; },
     "profiles/r5_small/sweep_tile256x128_mid_fp8.jsonl (2560^3 1591 vs 1412, 2560^2x8192 2032 vs 1713)"},
    // one dispatch wave: v22 (v23 off the 16x16-tile multiples)
    {22, [](const Fp8Shape& c) { return c.ap && c.nwg <= c.cus && c.sq; },
     "profiles/r4_sweep/onewave_fp8.jsonl (4096^3 2996 vs v20 2957)"},
    {23, [](const Fp8Shape& c) { return c.ap && c.nwg <= c.cus; },
     "profiles/r4_sweep/onewave_fp8.jsonl (2048x4096x4096 1.010x vs 0.997x)"},
    // multi-wave square grids: v22 needs >= 32 tiles on both sides or K >= 4096, else v21
    {22, [](const Fp8Shape& c) { return c.ap && c.sq && c.nwg >= 2 * c.cus && (c.wide || c.K >= 4096); },
     "profiles/r4_lean/ (16384^2x1024 1.19x, 12288^3 1.02x)"},
    {21, [](const Fp8Shape& c) { return c.ap && c.sq && c.nwg >= 2 * c.cus; },
     "profiles/r4_sweep/rules2_fp8.jsonl (12288x4096x1024 2253 vs v22 2129)"},
    {20, [](const Fp8Shape& c) { return c.ap; }, "profiles/r3_s2/zc_fp8.jsonl (4096^3 1.04x)"},
    // off the asm frame (other devices, K not an even K-tile count): the C++ q16 family
    {10, [](const Fp8Shape& c) { return c.K <= 12 * F8_BK && c.nwg >= 2 * c.cus && c.pgrid >= NXCD; },
     "profiles/r2_fp8_q16/ (persistent block-scaled kernel, short K)"},
    {18, [](const Fp8Shape& c) { return c.K <= 64 * F8_BK && c.nwg >= 4 * c.cus && c.pgrid >= NXCD; },
     "profiles/r2_fp8_q16/sweep_q16p*.jsonl (8192^3 +0.7-1.2 %, 16384^2x4096 +2.9 %)"},
    {16, [](const Fp8Shape& c) { return c.sq && c.cus == 256; }, "profiles/r2_fp8_q16/ (square raster)"},
    {15, [](const Fp8Shape& c) { return c.cus == 256; }, "profiles/r2_fp8_q16/ (q16 vs block-scaled +3-5 %)"},
    {17, [](const Fp8Shape&) { return true; }, "devices without 256 CUs: q16 without serpentine K"},
};

// What a kernel needs, and where a pinned variant goes when it cannot run.
struct Fp8Need {
  int variant;
  bool (*ok)(const Fp8Shape&);
  int fallback;   // -1: 16 on the square raster, else 15
};
static constexpr Fp8Need kFp8Needs[] = {
    {60, [](const Fp8Shape& c) { return c.tiles128; }, 0},
    {61, [](const Fp8Shape& c) { return c.tiles128; }, 0},
    {62, [](const Fp8Shape& c) { return c.tiles128 && c.M % 256 == 0; }, 0},
    {20, [](const Fp8Shape& c) { return c.ap; }, -1},
    {21, [](const Fp8Shape& c) { return c.ap; }, -1},
    {22, [](const Fp8Shape& c) { return c.ap; }, -1},
    {23, [](const Fp8Shape& c) { return c.ap; }, -1},
    {24, [](const Fp8Shape& c) { return c.ap && asm_splits(c.nwg, c.K / F8_BK, c.cus) > 1; }, 23},
    {21, [](const Fp8Shape& c) { return c.sq; }, 20},
    {22, [](const Fp8Shape& c) { return c.sq; }, 23},
    {16, [](const Fp8Shape& c) { return c.sq; }, 15},
    {10, [](const Fp8Shape& c) { return c.pgrid >= NXCD; }, 15},
    {18, [](const Fp8Shape& c) { return c.pgrid >= NXCD; }, 15},
    // serpentine K assumes 32 co-resident tiles per XCD
    {15, [](const Fp8Shape& c) { return c.cus == 256; }, 17},
    {16, [](const Fp8Shape& c) { return c.cus == 256; }, 17},
};

// The kernel for a shape on a device with `cus` CUs (0 = generic): the pinned variant walked down its
// fallbacks, or the first matching row of kFp8Rules.
static int plan_fp8(int M, int N, int K, int cus, int pinned) {
  const Fp8Shape c = fp8_shape(M, N, K, cus);
  if (!c.tiles && !c.tiles128) return 0;
  if (pinned == 0) {
    for (const auto& r : kFp8Rules)
      if (r.match(c)) return r.variant;
    return 0;
  }
  if (!c.tiles && pinned != 60 && pinned != 61 && pinned != 62) return 0;
  int v = pinned;
  for (bool moved = true; moved;) {
    moved = false;
    for (const auto& n : kFp8Needs)
      if (n.variant == v && !n.ok(c)) {
        v = n.fallback < 0 ? (c.sq ? 16 : 15) : n.fallback;
        moved = true;
        break;
      }
  }
  return v;
}

static int resolve_fp8_variant(int M, int N, int K, hipStream_t s) {
  return plan_fp8(M, N, K, device_cu_count(s), g_fp8_variant);
}

extern "C" {

int amdgo_ref_rows(int dtype, const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                   void* stream);

// 0 on success; hipErrorInvalidValue for a variant outside the production set.
int amdgo_gemm_fp8_set_variant(int v) {
  if (v != 0 && v != 10 && v != 15 && v != 16 && v != 17 && v != 18 && v != 20 && v != 21 && v != 22 && v != 23 && v != 24 &&
      v != 60 && v != 61 && v != 62)
    return (int)hipErrorInvalidValue;
  g_fp8_variant = v;
  return 0;
}
int amdgo_gemm_fp8_get_variant() { return g_fp8_variant; }
int amdgo_gemm_fp8_resolve_variant(int M, int N, int K) { return resolve_fp8_variant(M, N, K, nullptr); }
int amdgo_gemm_plan_fp8(int M, int N, int K, int cus, int pinned) { return plan_fp8(M, N, K, cus, pinned); }
const char* amdgo_gemm_plan_fp8_evidence(int M, int N, int K, int cus) {
  const Fp8Shape c = fp8_shape(M, N, K, cus);
  for (const auto& r : kFp8Rules)
    if (r.match(c)) return r.evidence;
  return "";
}

}  // extern "C"

// The dispatch of one GEMM; REC: the placement-recording instantiations (see gemm_bf16.hip).
template <Rec REC>
static int gemm_fp8_dispatch(const void* A, const void* Bt, void* C, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  const auto* a = (const uint8_t*)A;
  const auto* b = (const uint8_t*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / F8_BM) * (N / F8_BN);
  const int cus = device_cu_count(s);
  const int pgrid = persistent_launch_grid(nwg, cus);
  const int variant_now = resolve_fp8_variant(M, N, K, s);
  switch (variant_now) {
    case 60:
    case 61:
      launch_small<true, 128, REC>(a, b, c, M, N, K, s, cus, variant_now == 61);
      break;
    case 62:
      launch_small<true, 256, REC>(a, b, c, M, N, K, s, cus, false);
      break;
    case 10:
      hipLaunchKernelGGL((gemm_fp8_256x256_w4sp<6, 7, 16, 24, 6, false, REC>), dim3(pgrid), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 18:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16p<16, 18, 3, 34, 35, 43, false, 2, 2, true, REC>), dim3(pgrid),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 20:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, false, false, W4AP_EPI_STAGED_ZC, 0, REC>), dim3(pgrid),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 21:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, true, true, W4AP_EPI_STAGED_ZC, 0, REC>), dim3(256),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 22:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_LEAN_ILV, 2, REC>), dim3(256),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 23:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, false, false, W4AP_EPI_LEAN, 2, REC>), dim3(pgrid),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 24: {
      const int splits = asm_splits(nwg, K / F8_BK, cus);   // > 1: kFp8Needs
      SmallWorkspace* w = small_workspace(s, (size_t)nwg * splits * kAsmSlabFloats, nwg * 2);
      if (!w) return (int)hipErrorOutOfMemory;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap_sk<F8VP_SC_P_ZC, W4AP_EPI_LEAN, 2, REC>), dim3(nwg * splits),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K, splits, w->ws, w->cnt,
                         asm_last_pairs(K / F8_BK, splits), asm_piece_major());
      (void)hipEventRecord(w->done, s);
      break;
    }
    case 15:
      hipLaunchKernelGGL(Q16(32, false, REC), dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 16:
      hipLaunchKernelGGL(Q16(32, true, REC), dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 17:
      hipLaunchKernelGGL(Q16(0, false, REC), dim3(nwg), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    default: {
      dim3 grid((N + G8 - 1) / G8, (M + G8 - 1) / G8);
      hipLaunchKernelGGL(gemm_fp8_generic<REC>, grid, dim3(256), 0, s, a, b, c, M, N, K);
    }
  }
  return (int)hipGetLastError();
}

// The raster of the kernel the dispatch picks for a shape on the current device (gemm_raster_host.h).
static GemmRaster raster_fp8(int M, int N, int K, int cus) {
  const int v = plan_fp8(M, N, K, cus, g_fp8_variant);
  const int nwg = (M / F8_BM) * (N / F8_BN);
  switch (v) {
    case 60:
    case 61: {
      const int tiles = (M / S_BM) * (N / S_BN);
      const int nk = K / 128;
      const int splits = v == 61 ? small_splits(tiles, nk, cus) : 1;
      return GemmRaster::small(v, S_BM, S_BN, splits, small_piece_major(nk, splits));
    }
    case 62:
      return GemmRaster::small(v, 256, S_BN, 1, 0);
    case 15: case 17:
      return GemmRaster::grid_of(v, F8_BM, F8_BN, nwg, false);
    case 16:
      return GemmRaster::grid_of(v, F8_BM, F8_BN, nwg, true);
    case 10: case 18: case 20: case 23:
      return GemmRaster::persistent(v, F8_BM, F8_BN, persistent_launch_grid(nwg, cus), false);
    case 21: case 22:
      return GemmRaster::persistent(v, F8_BM, F8_BN, 256, true);
    case 24:
      return GemmRaster::split(v, asm_splits(nwg, K / F8_BK, cus), asm_piece_major());
    default:
      return GemmRaster::generic(v, G8, G8);
  }
}

extern "C" {

// Returns 0 on success, a hipError_t value otherwise. `stream` may be null.
int amdgo_gemm_fp8(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  return gemm_fp8_dispatch<kTimed>(A, Bt, C, M, N, K, (hipStream_t)stream);
}

// The placement-recording dispatch (amdgo_gemm_bf16_placed).
int amdgo_gemm_fp8_placed(const void* A, const void* Bt, void* C, int M, int N, int K, uint32_t* placement,
                          void* stream) {
  const hipError_t e = set_placement_record((hipStream_t)stream, placement);
  if (e != hipSuccess) return (int)e;
  return gemm_fp8_dispatch<kRecord>(A, Bt, C, M, N, K, (hipStream_t)stream);
}

int amdgo_gemm_fp8_placement_init() { return (int)set_placement_record(nullptr, nullptr); }

// The dispatch's raster (amdgo_gemm_bf16_raster).
int amdgo_gemm_fp8_raster(int M, int N, int K, int* info, int* owners, int* rounds, int cap) {
  return raster_fill(raster_fp8(M, N, K, device_cu_count(nullptr)), M, N, info, owners, rounds, cap);
}
// The same for a device with `cus` CUs (no GPU needed: the CPU tests check every raster is a bijection).
int amdgo_gemm_fp8_raster_for(int M, int N, int K, int cus, int* info, int* owners, int* rounds, int cap) {
  return raster_fill(raster_fp8(M, N, K, cus), M, N, info, owners, rounds, cap);
}

int amdgo_gemm_fp8_generic(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + G8 - 1) / G8, (M + G8 - 1) / G8);
  hipLaunchKernelGGL(gemm_fp8_generic<kTimed>, grid, dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)A, (const uint8_t*)Bt, (__bf16*)C, M, N, K);
  return (int)hipGetLastError();
}

// fp32 reference of sampled rows (gemm_abft.hip, software e4m3 decode).
int amdgo_gemm_fp8_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                            void* stream) {
  return amdgo_ref_rows(1, A, Bt, rows, nrows, out, N, K, stream);
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
