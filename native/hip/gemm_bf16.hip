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
//   60 (round 5) = 128x128 output tiles (gemm_small.h) for grids the 256x256 kernels leave mostly idle
//        (a 256-tile grid of at most a quarter of the CUs) and for shapes only 128-tileable; 61 = its
//        split-K form when the 128x128 grid is under the CU count and K leaves pieces of >= 16
//        K-tiles; 62 = 256x128 tiles for 256-tile grids of a quarter to a half of the CUs.
//   57 (round 6) = v55 in the split-K form of the asm frame (gemm_w4ap.h SPLIT): one (tile, K piece) per
//        workgroup, two pieces (the last 52 % of K), a tile's pieces on one XCD, the tile's last arrival
//        sums; the default over v62 for 65-128-tile grids with K >= 4096 (2560^2x8192 1.12x v62,
//        2048x4096x16384 1.27x; profiles/r6_splitk/band_bf16.jsonl).
//   18 / 25 / 42 / 44 / 45 / 47 / 48 / 50 / 51 / 52 / 53 / 54 / 55 / 56 / 57 / 60 / 61 / 62 = that kernel pinned (no automatic switch; still falls back to a
//        kernel that can run the shape or the device).
// The automatic choice is the first matching row of the declarative table kBf16Rules below (each row
// cites its sweep); what each kernel needs, and where a pinned one falls back, is kBf16Needs. Both are
// checked against the round-4 rule code they replaced in tests/test_gemm_dispatch.py.
// Every w4s / w4sp kernel here carries the K offset of its LDS-DMA pieces in the lane offset (VK: one VALU
// add per K-tile, loop-invariant soffsets; 17 fewer SALU per K-tile, +0.6-0.8 % at 8192^3 and
// 16384^3, profiles/r2_sched/sweep_vk.jsonl).
// A bounds-checked generic kernel handles shapes that are not multiples of the tile.

#include <map>
#include <mutex>

#include "gemm_bf16_kernels.h"
#include "gemm_raster_host.h"
#include "gemm_small_host.h"

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

// The variant a caller pinned (amdgo_gemm_set_variant): per host thread, so threads driving
// different GPUs (amd-gemm-validate --launch threads) never see each other's pin.
static thread_local int g_variant = 0;

// Persistent grid as the dispatch rules see it: one workgroup per CU (the 160 KiB LDS admits one), a
// multiple of the 8 XCDs, never more workgroups than tiles. 0 when the device or the tile count is too
// small. (The launch rounds up instead: persistent_launch_grid, gemm_tile_common.h.)
static int persistent_grid(int nwg, int cus) {
  const int g = nwg < cus ? nwg : cus;
  return (g / NXCD) * NXCD;
}

// What the dispatch knows about a shape on a device.
struct Bf16Shape {
  int M, N, K, cus;
  bool tiles256;   // M, N multiples of 256, K of 64, K >= 128: the 256x256 kernels can run it
  bool tiles128;   // M, N multiples of 128, K of 64: the 128x128 kernel (v60) can run it
  int nwg;         // 256x256 output tiles
  int pgrid;       // persistent grid of the 256x256 kernels
  bool sq;         // 16x16-tile multiples (the square cross-XCD raster)
  bool pow2k;
  bool mi355;      // the 256-CU MI355X every w4ap / serpentine schedule was measured on
};

static Bf16Shape bf16_shape(int M, int N, int K, int cus) {
  Bf16Shape c{M, N, K, cus};
  c.tiles256 = M % BM == 0 && N % BN == 0 && K % BK == 0 && K >= 2 * BK;
  c.tiles128 = M % S_BM == 0 && N % S_BN == 0 && K % S_BK == 0 && K >= S_BK;
  c.nwg = (M / BM) * (N / BN);
  c.pgrid = persistent_grid(c.nwg, cus);
  c.sq = (M / BM) % 16 == 0 && (N / BN) % 16 == 0;
  c.pow2k = (K & (K - 1)) == 0;
  c.mi355 = cus == 256;
  return c;
}

// The automatic dispatch, one row per shape class, first match wins. Each row names the sweep that
// put it there (every number: our kernel against hipBLASLt in the same process on MI355X).
struct Bf16Rule {
  int variant;
  bool (*match)(const Bf16Shape&);
  const char* evidence;
};
static constexpr Bf16Rule kBf16Rules[] = {
    // a 256x256 grid of at most a quarter of the CUs (or a shape only 128-tileable): 128x128 tiles, 4x
    // the workgroups; split-K too when the 128x128 grid is still far below the chip and K is long
    // 33-64 256x256 tiles with K >= 16384: the asm frame split in up to four K pieces
    {57, [](const Bf16Shape& c) { return c.mi355 && c.tiles256 && 8 * c.nwg > c.cus && 4 * c.nwg <= c.cus &&
                                         c.K % (2 * BK) == 0 && c.K >= 256 * BK; },
     "profiles/r6_splitk/tree_s34.jsonl (2048^2x16384 1189 vs v60 1012 TF/s, 1.07x hipBLASLt)"},
    {61, [](const Bf16Shape& c) {
       return c.tiles128 && (!c.tiles256 || 4 * c.nwg <= c.cus) &&
              small_splits((c.M / S_BM) * (c.N / S_BN), c.K / S_BK, c.cus) > 1; },
     "profiles/r5_small/sweep_v62.jsonl (1024^2x8192 458 vs 207 TF/s unsplit)"},
    {60, [](const Bf16Shape& c) { return c.tiles128 && (!c.tiles256 || 4 * c.nwg <= c.cus); },
     "profiles/r5_small/sweep_v62.jsonl (1024^3 1.36x, 1536^3 1.01x, 2048^2x1024 1.35x hipBLASLt)"},
    {0, [](const Bf16Shape& c) { return !c.tiles256; }, "generic bounds-checked kernel"},
    // a quarter to a half of the CUs in 256x256 tiles with K >= 4096: the asm frame split in two K pieces
    {57, [](const Bf16Shape& c) { return c.mi355 && 4 * c.nwg > c.cus && 2 * c.nwg <= c.cus && c.K % (2 * BK) == 0 &&
                                         c.K >= 64 * BK; },
     "profiles/r6_splitk/band_bf16.jsonl (2560^2x8192 1.12x v62, 2048x4096x16384 1.27x, 2304^2x4096 1.06x)"},
    // a quarter to a half of the CUs in 256x256 tiles: 256x128 tiles fill the chip in one wave
    {62, [](const Bf16Shape& c) { return 4 * c.nwg > c.cus && 2 * c.nwg <= c.cus; },
     "profiles/r5_small/sweep_tile256x128.jsonl, sweep_tile256x128_mid.jsonl (2560^3 878 vs 773, 2816^3 1060 vs 969)"},
    // K not a power of two (even K-tile count >= 4): the asm pipeline in the VP DMA form
    {54, [](const Bf16Shape& c) { return c.mi355 && !c.pow2k && c.K % (2 * BK) == 0 && c.K >= 4 * BK &&
                                         c.pgrid >= NXCD && c.sq && c.nwg >= 8 * c.cus; },
     "profiles/r3_s2/vpsq_bf16.jsonl (12288^3 1.05x, 12288^2x10240 1.07x)"},
    {53, [](const Bf16Shape& c) { return c.mi355 && !c.pow2k && c.K % (2 * BK) == 0 && c.K >= 4 * BK &&
                                         c.pgrid >= NXCD; },
     "profiles/r3_s2/vp_bf16.jsonl (12288^3 1.02x, 8192^2x12288 1.07x)"},
    // power-of-two K: the persistent asm K pipeline and its forms
    {51, [](const Bf16Shape& c) { return c.mi355 && c.pow2k && c.K >= 4 * BK && c.pgrid >= NXCD && c.sq &&
                                         c.nwg >= 8 * c.cus && c.K >= 128 * BK; },
     "profiles/r3_asm/ (16384^3 1.01x)"},
    {52, [](const Bf16Shape& c) { return c.mi355 && c.pow2k && c.K >= 4 * BK && c.pgrid >= NXCD &&
                                         c.nwg <= 2 * c.cus && c.K >= 512 * BK; },
     "profiles/r3_s2/longk_bf16.jsonl (4096^2x32768 +1.0 %)"},
    {56, [](const Bf16Shape& c) { return c.mi355 && c.pow2k && c.K >= 4 * BK && c.pgrid >= NXCD && c.sq &&
                                         (c.K <= 32 * BK || c.nwg <= c.cus); },
     "profiles/r4_lean/, r4_sweep/ (16384^2x1024 1.08x, 8192^2x2048 1.05x)"},
    {55, [](const Bf16Shape& c) { return c.mi355 && c.pow2k && c.K >= 4 * BK && c.pgrid >= NXCD && c.nwg <= c.cus; },
     "profiles/r4_lean/ (one-wave grids off the 16x16-tile multiples)"},
    {50, [](const Bf16Shape& c) { return c.mi355 && c.pow2k && c.K >= 4 * BK && c.pgrid >= NXCD; },
     "profiles/r3_asm/asm8_summary.jsonl (8192^3 +2-3 % over v44)"},
    // the C++ w4s family (short K without a persistent asm grid, other devices)
    {25, [](const Bf16Shape& c) { return c.K <= 64 * BK && c.nwg >= 2 * c.cus && c.pgrid >= NXCD; },
     "profiles/r2_sched/sweep_persistent_midk.jsonl (16384^2x1024 +10 %)"},
    {48, [](const Bf16Shape& c) { return c.mi355 && !c.pow2k && c.sq && c.nwg >= 8 * c.cus && c.K >= 128 * BK; },
     "profiles/r2_sched/sweep_pa.jsonl (PA rows, K not a power of two)"},
    {45, [](const Bf16Shape& c) { return c.mi355 && c.sq && c.nwg >= 8 * c.cus && c.K >= 128 * BK; },
     "profiles/r1_s6_sq (12288^3 +5.5 %, 16384^3 +3.4 %)"},
    {47, [](const Bf16Shape& c) { return c.mi355 && !c.pow2k; }, "profiles/r2_sched/sweep_pa.jsonl (12288^3 +11 %)"},
    {44, [](const Bf16Shape& c) { return c.mi355; }, "profiles/r1_* (serpentine K + loop rotation)"},
    {42, [](const Bf16Shape&) { return true; }, "devices without 256 CUs: rotation only"},
};

// What a kernel needs from the shape and device, and where a pinned variant goes when it cannot run.
struct Bf16Need {
  int variant;
  bool (*ok)(const Bf16Shape&);
  int fallback;
};
static constexpr Bf16Need kBf16Needs[] = {
    {60, [](const Bf16Shape& c) { return c.tiles128; }, 0},
    {61, [](const Bf16Shape& c) { return c.tiles128; }, 0},
    {62, [](const Bf16Shape& c) { return c.tiles128 && c.M % 256 == 0; }, 0},

    {45, [](const Bf16Shape& c) { return c.sq; }, 44},
    {48, [](const Bf16Shape& c) { return c.sq; }, 47},
    {47, [](const Bf16Shape& c) { return c.mi355; }, 42},
    {48, [](const Bf16Shape& c) { return c.mi355; }, 42},
    {25, [](const Bf16Shape& c) { return c.pgrid >= NXCD; }, 44},
    // w4ap runs an even number of K-tiles (>= 4) on a grid of whole XCD groups
    {50, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {51, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {52, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {53, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {54, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {55, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    {56, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && c.K >= 4 * BK && c.pgrid >= NXCD; }, 44},
    // the split-K asm form: even K-tile pieces of >= 16, at least 2 of them per tile within the CUs
    {57, [](const Bf16Shape& c) { return c.K % (2 * BK) == 0 && asm_splits(c.nwg, c.K / BK, c.cus) > 1; }, 55},
    // the square raster needs 16x16 super-tiles and exactly 256 workgroups
    {54, [](const Bf16Shape& c) { return c.sq && c.mi355; }, 53},
    {56, [](const Bf16Shape& c) { return c.sq && c.mi355; }, 55},
    {51, [](const Bf16Shape& c) { return c.sq && c.mi355; }, 50},
    // serpentine K assumes 32 co-resident workgroups per XCD
    {44, [](const Bf16Shape& c) { return c.mi355; }, 42},
    {45, [](const Bf16Shape& c) { return c.mi355; }, 42},
};


// The kernel for a shape on a device with `cus` CUs: the pinned variant (walked down its fallbacks
// until it can run), or the first matching row of kBf16Rules. 0 = the generic kernel.
static int plan_bf16(int M, int N, int K, int cus, int pinned) {
  const Bf16Shape c = bf16_shape(M, N, K, cus);
  int v = pinned;
  if (v == 0) {
    for (const auto& r : kBf16Rules)
      if (r.match(c)) {
        v = r.variant;
        break;
      }
    return v;
  }
  if (v < 60 && !c.tiles256) return 0;
  for (bool moved = true; moved && v;) {
    moved = false;
    for (const auto& n : kBf16Needs)
      if (n.variant == v && !n.ok(c)) {
        v = n.fallback;
        moved = true;
        break;
      }
  }
  return v;
}

static int resolve_variant(int M, int N, int K, hipStream_t s) {
  return plan_bf16(M, N, K, device_cu_count(s), g_variant);
}

extern "C" {

int amdgo_ref_rows(int dtype, const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                   void* stream);

// 0 on success; hipErrorInvalidValue for a variant outside the production set.
int amdgo_gemm_set_variant(int v) {
  if (v != 0 && v != 18 && v != 25 && v != 42 && v != 44 && v != 45 && v != 47 && v != 48 && v != 50 &&
      v != 51 && v != 52 && v != 53 && v != 54 && v != 55 && v != 56 && v != 57 && v != 60 && v != 61 && v != 62)
    return (int)hipErrorInvalidValue;
  g_variant = v;
  return 0;
}
int amdgo_gemm_get_variant() { return g_variant; }
// v61: split-K workgroups per CU to aim for (1 = one wave of the chip); per host thread like the pin.
int amdgo_gemm_set_split_target(int t) {
  if (t < 1 || t > 8) return (int)hipErrorInvalidValue;
  small_split_target() = t;
  return 0;
}
// v57 / fp8 v24 sweep knobs for the calling host thread: a forced piece count (0 = automatic) and the
// last piece's share of K in permille (0 = default), and the item order (1 = piece-major). gemm_small_host.h
// AsmSplitKnobs.
int amdgo_gemm_set_asm_split(int splits, int last_permille, int piece_major) {
  if (splits < 0 || splits > 64 || last_permille < 0 || last_permille >= 1000 || piece_major < 0 || piece_major > 1)
    return (int)hipErrorInvalidValue;
  asm_split_knobs() = AsmSplitKnobs{splits, last_permille, piece_major};
  return 0;
}
int amdgo_gemm_small_splits(int M, int N, int K, int cus) {
  return small_splits((M / S_BM) * (N / S_BN), K / S_BK, cus);
}
// v61 split-K workspace sets held for device `dev` (at most kSmallWorkspaces; gemm_small_host.h).
int amdgo_gemm_small_workspace_count(int dev) { return small_workspace_count(dev); }
// The launch grid of the persistent 256x256 kernels for `nwg` tiles on `cus` CUs (gemm_tile_common.h).
int amdgo_gemm_persistent_launch_grid(int nwg, int cus) { return persistent_launch_grid(nwg, cus); }
int amdgo_gemm_resolve_variant(int M, int N, int K) { return resolve_variant(M, N, K, nullptr); }
// The dispatch as a pure function of the shape, the device's CU count and a pinned variant (no GPU
// needed: the CPU tests check the table against the rules it replaced).
int amdgo_gemm_plan_bf16(int M, int N, int K, int cus, int pinned) { return plan_bf16(M, N, K, cus, pinned); }
// The evidence row behind the automatic choice (the sweep file that put it there).
const char* amdgo_gemm_plan_bf16_evidence(int M, int N, int K, int cus) {
  const Bf16Shape c = bf16_shape(M, N, K, cus);
  for (const auto& r : kBf16Rules)
    if (r.match(c)) return r.evidence;
  return "";
}

}  // extern "C"

// The dispatch of one GEMM. REC: the placement-recording instantiations of the same kernels (the
// checked dispatch of amd-gemm-validate, gemm_tile_common.h note_placement); REC = kTimed is every
// other launch, and its kernels carry no record code.
template <Rec REC>
static int gemm_bf16_dispatch(const void* A, const void* Bt, void* C, int M, int N, int K, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  const auto* a = (const __bf16*)A;
  const auto* b = (const __bf16*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / BM) * (N / BN);
  const int cus = device_cu_count(s);
  auto persistent = [&](int n) { return persistent_launch_grid(n, cus); };
  const int variant_now = resolve_variant(M, N, K, s);
  switch (variant_now) {
    case 60:
    case 61:
      launch_small<false, 128, REC>(a, b, c, M, N, K, s, cus, variant_now == 61);
      break;
    case 62:
      launch_small<false, 256, REC>(a, b, c, M, N, K, s, cus, false);
      break;
    case 18:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 0, false, false, true, false, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 25:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40, false, true, REC>), dim3(persistent(nwg)),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 42:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 0, true, false, true, false, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 44:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true, false, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 47:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true, true, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 48:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true, true, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 45:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true, false, REC>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 50:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_MAIN, true, false, W4AP_EPI_STAGED_ZC, 0, REC>),
                         dim3(persistent(nwg)), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 51:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_MAIN, true, true, W4AP_EPI_STAGED_ZC, 0, REC>), dim3(256),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 53:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_STAGED_ZC, 1, REC>),
                         dim3(persistent(nwg)), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 54:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_STAGED_ZC, 1, REC>), dim3(256),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 55:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_LEAN, 2, REC>),
                         dim3(persistent(nwg)), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 56:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN_ILV, 2, REC>), dim3(256),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 52:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_LONGK, true, false, W4AP_EPI_STAGED_ZC, 0, REC>),
                         dim3(persistent(nwg)), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 57: {
      const int splits = asm_splits(nwg, K / BK, cus);   // > 1: kBf16Needs
      SmallWorkspace* w = small_workspace(s, (size_t)nwg * splits * kAsmSlabFloats, nwg * 2);
      if (!w) return (int)hipErrorOutOfMemory;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap_sk<W4VP_SC_G4_ZC, W4AP_EPI_LEAN, 2, REC>), dim3(nwg * splits),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K, splits, w->ws, w->cnt,
                         asm_last_pairs(K / BK, splits), asm_piece_major());
      (void)hipEventRecord(w->done, s);
      break;
    }
    default: {
      dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
      hipLaunchKernelGGL(gemm_bf16_generic<REC>, grid, dim3(256), 0, s, a, b, c, M, N, K);
    }
  }
  return (int)hipGetLastError();
}

// The raster of the kernel the dispatch picks for a shape on the current device: output tile, launch
// grid and how workgroups walk the tiles (gemm_raster_host.h) -- what the ABFT check needs to name the
// workgroup behind a bad tile.
static GemmRaster raster_bf16(int M, int N, int K, int cus) {
  const int v = plan_bf16(M, N, K, cus, g_variant);
  const int nwg = (M / BM) * (N / BN);
  switch (v) {
    case 60:
    case 61: {
      const int tiles = (M / S_BM) * (N / S_BN);
      const int nk = K * 2 / 128;
      const int splits = v == 61 ? small_splits(tiles, nk, cus) : 1;
      return GemmRaster::small(v, S_BM, S_BN, splits, small_piece_major(nk, splits));
    }
    case 62:
      return GemmRaster::small(v, 256, S_BN, 1, 0);
    case 18: case 42: case 44: case 47:
      return GemmRaster::grid_of(v, BM, BN, nwg, false);
    case 45: case 48:
      return GemmRaster::grid_of(v, BM, BN, nwg, true);
    case 25: case 50: case 52: case 53: case 55:
      return GemmRaster::persistent(v, BM, BN, persistent_launch_grid(nwg, cus), false);
    case 51: case 54: case 56:
      return GemmRaster::persistent(v, BM, BN, 256, true);
    case 57:
      return GemmRaster::split(v, asm_splits(nwg, K / BK, cus), asm_piece_major());
    default:
      return GemmRaster::generic(v, GBM, GBN);
  }
}

extern "C" {

// Returns 0 on success, a hipError_t value otherwise. `stream` may be null.
int amdgo_gemm_bf16(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  return gemm_bf16_dispatch<kTimed>(A, Bt, C, M, N, K, (hipStream_t)stream);
}

// The same GEMM through the placement-recording kernels: workgroup b of the dispatch writes
// {HW_REG_XCC_ID, HW_REG_HW_ID} to placement[2b], [2b+1] (device memory, room for the raster's grid).
int amdgo_gemm_bf16_placed(const void* A, const void* Bt, void* C, int M, int N, int K, uint32_t* placement,
                           void* stream) {
  const hipError_t e = set_placement_record((hipStream_t)stream, placement);
  if (e != hipSuccess) return (int)e;
  return gemm_bf16_dispatch<kRecord>(A, Bt, C, M, N, K, (hipStream_t)stream);
}

// One-time setup of the placement record on the current device (the first hipMemcpyToSymbol of a
// process resolves the symbol: ~9 ms, which the first checked dispatch paid inside the probe).
int amdgo_gemm_bf16_placement_init() { return (int)set_placement_record(nullptr, nullptr); }

// The dispatch's raster for a shape on the current device: fills `info` (GemmRasterInfo fields, see
// gemm_raster_host.h) and, when `owners` is non-null, the owning workgroup and round of every
// (tile, piece) -- `cap` ints per array. Returns the tile count, or -1 when `cap` is too small.
int amdgo_gemm_bf16_raster(int M, int N, int K, int* info, int* owners, int* rounds, int cap) {
  return raster_fill(raster_bf16(M, N, K, device_cu_count(nullptr)), M, N, info, owners, rounds, cap);
}
// The same for a device with `cus` CUs (no GPU needed: the CPU tests check every raster is a bijection).
int amdgo_gemm_bf16_raster_for(int M, int N, int K, int cus, int* info, int* owners, int* rounds, int cap) {
  return raster_fill(raster_bf16(M, N, K, cus), M, N, info, owners, rounds, cap);
}

// Force the generic kernel (independent implementation used by tests).
int amdgo_gemm_bf16_generic(const void* A, const void* Bt, void* C, int M, int N, int K,
                            void* stream) {
  if (M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
  hipLaunchKernelGGL(gemm_bf16_generic<kTimed>, grid, dim3(256), 0, (hipStream_t)stream,
                     (const __bf16*)A, (const __bf16*)Bt, (__bf16*)C, M, N, K);
  return (int)hipGetLastError();
}

// fp32 reference of sampled rows (gemm_abft.hip, one wave per output column).
int amdgo_gemm_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                        void* stream) {
  return amdgo_ref_rows(0, A, Bt, rows, nrows, out, N, K, stream);
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
