// The persistent asm-pipeline GEMM frame shared by the bf16 kernel gemm_bf16_256x256_w4ap (v50-v52,
// gemm_bf16_kernels.h) and the fp8 kernel gemm_fp8_256x256_q16ap (gemm_fp8_kernels.h).
//
// Both stage 256x256 output tiles from 128-byte K-rows: a K-tile is 64 bf16 or 128 fp8 elements,
// so the LDS image (two 64 KiB buffers of A and B panels), the 16 LDS-DMA pieces per K-tile, the
// XOR swizzle, the fragment addresses and the 8x8 grid of 16x16 accumulators per wave are the same
// bytes. Only the K-tile body differs -- 128 `v_mfma_f32_16x16x32_bf16` over two fragment sets
// (tools/gen_bf16_asm_loop.py) or 64 `v_mfma_f32_16x16x128_f8f6f4` over one
// (tools/gen_fp8_asm_loop.py) -- and that is generated asm text selected by SC.
//
// gridDim = one workgroup per CU (a multiple of 8); XCD x owns a contiguous run of output tiles that
// its workgroups walk in strides of gridDim / 8, so the 32 co-resident tiles of an XCD are
// neighbours in the grouped raster. SQ: the square cross-XCD raster instead -- gridDim is exactly
// 256, workgroup b's i-th tile is dispatch-wave index i * 256 + b of tile_coords_sq, so every round
// of 256 co-resident tiles is one 16x16 super-tile (host: tiles_m, tiles_n multiples of 16).
// The K stream runs on across tiles: the last two K-tiles of a tile DMA the next tile's K-tiles 0
// and 1 into the buffers they free (drain with %[nA] / %[nB] / %[nvoff]), and the epilogue stages
// each wave's 128x128 sub-tile through a private 8 KiB slice of the 32 KiB of LDS beyond the K
// buffers -- no workgroup barrier, overlapping the in-flight DMA; its vmcnt(0) before the first C
// store retires those DMAs, so the next tile starts with a barrier and its fragment reads. SERP:
// odd tiles of a workgroup walk K backwards (they start on the K-slices the previous tile left in
// L2). Host guarantees: M, N multiples of 256, an even number (>= 4) of K-tiles, gridDim % 8 == 0.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_tile_common.h"
#include "gemm_bf16_asm_loop.h"
#include "gemm_fp8_asm_loop.h"
#ifndef F8EF_LOOP_SELECT
#define F8EF_LOOP_SELECT(SC) static_assert(SC < 0, "no fp8 fused-epilogue schedule generated");
#endif

namespace {

#define W4A_VCLOBBERS                                                                                       \
  "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", \
  "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31",   \
  "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46",   \
  "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61",   \
  "v62", "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", "v76",   \
  "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", "v89", "v90", "v91",   \
  "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105",    \
  "v106", "v107", "v108", "v109", "v110", "v111", "v112", "v113", "v114", "v115", "v116", "v117", "v118",    \
  "v119", "v120", "v121", "v122", "v123", "v124", "v125", "v126", "v127"

#define W4EF_VCLOBBERS                                                                                      \
  "v224", "v225", "v226", "v227", "v228", "v229", "v230", "v231", "v232", "v233", "v234", "v235", "v236",     \
  "v237", "v238", "v239", "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249",     \
  "v250", "v251", "v252", "v253", "v254", "v255"

typedef uint32_t w4a_u32x4 __attribute__((ext_vector_type(4)));

// The deferred-store form (EPI 7; tools/gen_*_asm_loop.py kloop_persistent_ds): the previous tile's
// C quarters 1-2 in h0..h15, quarter 3 in the wave's staging LDS (stgl: this lane's 16-byte slot), stored
// through vcur (advanced by s8N = 4 C rows per store) from the previous tile's corner sCp.
#define W4DS_LOOP(TEXT)                                                                                       \
  asm volatile("s_mov_b32 %[m0save], m0\n\t" TEXT "s_mov_b32 m0, %[m0save]"                                   \
               : [voff] "+v"(voff_k), [nvoff] "+v"(nvoff), [cnt] "+s"(trips), [m0save] "=&s"(m0save),          \
                 [vcur] "+v"(vcur)                                                                             \
               : [ra00] "v"(ra00), [rb00] "v"(rb00), [ra01] "v"(ra01), [rb01] "v"(rb01), [ra10] "v"(ra10),       \
                 [rb10] "v"(rb10), [ra11] "v"(ra11), [rb11] "v"(rb11), [kstep] "s"(kstep), [s0] "s"(so[0]),      \
                 [s1] "s"(so[1]), [s2] "s"(so[2]), [s3] "s"(so[3]), [s4] "s"(so[4]), [s5] "s"(so[5]),            \
                 [s6] "s"(so[6]), [s7] "s"(so[7]), [rA] "s"(sA), [rB] "s"(sB), [nA] "s"(nA), [nB] "s"(nB),       \
                 [nkstep] "s"(nkstep), [m0b0] "s"(m0b0), [m0b1] "s"(m0b1), [flags] "s"(flags), [h0] "v"(held[0]), \
                 [h1] "v"(held[1]), [h2] "v"(held[2]), [h3] "v"(held[3]), [h4] "v"(held[4]), [h5] "v"(held[5]),  \
                 [h6] "v"(held[6]), [h7] "v"(held[7]), [h8] "v"(held[8]), [h9] "v"(held[9]),                     \
                 [h10] "v"(held[10]), [h11] "v"(held[11]), [h12] "v"(held[12]), [h13] "v"(held[13]),             \
                 [h14] "v"(held[14]), [h15] "v"(held[15]), [stgl] "v"(stgl), [s8N] "s"(s8N), [sCp] "s"(sCp)      \
               : "memory", "scc", W4A_VCLOBBERS, W4DS_VCLOBBERS, W4_AGPR_CLOBBERS)
#define W4DS_VCLOBBERS                                                                                      \
  "v240", "v241", "v242", "v243", "v244", "v245", "v246", "v247", "v248", "v249", "v250", "v251", "v252",     \
  "v253", "v254", "v255"

// The VP DMA form (DM >= 1; tools/gen_*_asm_loop.py to_vp): piece p's lane offset is its own VGPR
// vp[p] and the DMA'd K-tile's byte offset one SGPR (koff, nkoff for the next tile).
#define W4VP_LOOP(TEXT)                                                                                       \
  asm volatile("s_mov_b32 %[m0save], m0\n\t" TEXT "s_mov_b32 m0, %[m0save]"                                   \
               : [koff] "+s"(koff), [nkoff] "+s"(nkoff), [cnt] "+s"(trips), [m0save] "=&s"(m0save)              \
               : [ra00] "v"(ra00), [rb00] "v"(rb00), [ra01] "v"(ra01), [rb01] "v"(rb01), [ra10] "v"(ra10),       \
                 [rb10] "v"(rb10), [ra11] "v"(ra11), [rb11] "v"(rb11), [kstep] "s"(kstep), [vp0] "v"(vp[0]),     \
                 [vp1] "v"(vp[1]), [vp2] "v"(vp[2]), [vp3] "v"(vp[3]), [vp4] "v"(vp[4]), [vp5] "v"(vp[5]),        \
                 [vp6] "v"(vp[6]), [vp7] "v"(vp[7]), [vp8] "v"(vp[8]), [vp9] "v"(vp[9]), [vp10] "v"(vp[10]),      \
                 [vp11] "v"(vp[11]), [vp12] "v"(vp[12]), [vp13] "v"(vp[13]), [vp14] "v"(vp[14]),                 \
                 [vp15] "v"(vp[15]), [rA] "s"(sA), [rB] "s"(sB), [nA] "s"(nA), [nB] "s"(nB), [nkstep] "s"(nkstep), \
                 [m0b0] "s"(m0b0), [m0b1] "s"(m0b1), [flags] "s"(flags)                                          \
               : "memory", "scc", W4A_VCLOBBERS, W4_AGPR_CLOBBERS)

// LEAN staging layout (EPI 15 / 16): 8-byte half h of 16-byte chunk c of a staged 256-byte C row r
// sits at chunk c ^ ((r & 15) >> 1), half h ^ (r & 1). A ds_write_b64 lane group (16 lanes = 16 rows,
// one chunk half; banks mod 32) lands on 16 distinct 8-byte slots of 128 bytes -- every bank once --
// and each half-wave of a ds_read_b64 (2 rows x 16 chunks, one half each; banks mod 64) covers all 64
// banks once, so neither side conflicts and a 16-byte row piece comes back as two 8-byte reads in
// order (no lane-dependent swap). MI355X_MICROARCH.md, LDS banking table.
__device__ __forceinline__ uint32_t lean_off(int r, int c, int h) {
  return (uint32_t)(r * 256 + ((c ^ ((r & 15) >> 1)) << 4) + ((h ^ (r & 1)) << 3));
}
typedef uint32_t w4a_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ w4a_u32x4 lean_read(const char* stg, int r, int c) {
  const w4a_u32x2 lo = *reinterpret_cast<const w4a_u32x2*>(stg + lean_off(r, c, 0));
  const w4a_u32x2 hi = *reinterpret_cast<const w4a_u32x2*>(stg + lean_off(r, c, 1));
  return w4a_u32x4{lo[0], lo[1], hi[0], hi[1]};
}

constexpr int W4AP_TILE = 256;                     // output tile edge
constexpr int W4AP_ROW = 128;                      // bytes per staged K-row (one K-tile)
constexpr int W4AP_PANEL = W4AP_TILE * W4AP_ROW;   // 32 KiB per operand per K-tile
constexpr int W4AP_BUF = 2 * W4AP_PANEL;           // A + B
constexpr int W4AP_EPI_WAVE = 8192;                // 32 C rows x 128 cols x bf16 per wave
constexpr int W4AP_LDS = 2 * W4AP_BUF + 4 * W4AP_EPI_WAVE;   // 160 KiB

#define W4AP_LOOP(TEXT)                                                                                       \
  asm volatile("s_mov_b32 %[m0save], m0\n\t" TEXT "s_mov_b32 m0, %[m0save]"                                   \
               : [voff] "+v"(voff_k), [nvoff] "+v"(nvoff), [cnt] "+s"(trips), [m0save] "=&s"(m0save)           \
               : [ra00] "v"(ra00), [rb00] "v"(rb00), [ra01] "v"(ra01), [rb01] "v"(rb01), [ra10] "v"(ra10),       \
                 [rb10] "v"(rb10), [ra11] "v"(ra11), [rb11] "v"(rb11), [kstep] "s"(kstep), [s0] "s"(so[0]),      \
                 [s1] "s"(so[1]), [s2] "s"(so[2]), [s3] "s"(so[3]), [s4] "s"(so[4]), [s5] "s"(so[5]),            \
                 [s6] "s"(so[6]), [s7] "s"(so[7]), [rA] "s"(sA), [rB] "s"(sB), [nA] "s"(nA), [nB] "s"(nB),       \
                 [nkstep] "s"(nkstep), [m0b0] "s"(m0b0), [m0b1] "s"(m0b1), [flags] "s"(flags)                    \
               : "memory", "scc", W4A_VCLOBBERS, W4_AGPR_CLOBBERS)

// The fused-epilogue pipeline (EPI=2, tools/gen_bf16_asm_loop.py EF): permuted B-fragment lane offsets
// (rbe / rbo), the per-row-block C lane offsets cv0..cv7 and the tile's C corner sC; v[224:255] are its
// epilogue temps.
#define W4EF_LOOP(TEXT)                                                                                       \
  asm volatile("s_mov_b32 %[m0save], m0\n\t" TEXT "s_mov_b32 m0, %[m0save]"                                   \
               : [voff] "+v"(voff_k), [nvoff] "+v"(nvoff), [cnt] "+s"(trips), [m0save] "=&s"(m0save)           \
               : [ra00] "v"(ra00), [ra01] "v"(ra01), [ra10] "v"(ra10), [ra11] "v"(ra11), [rbe00] "v"(rbe00),    \
                 [rbo00] "v"(rbo00), [rbe01] "v"(rbe01), [rbo01] "v"(rbo01), [rbe10] "v"(rbe10),                \
                 [rbo10] "v"(rbo10), [rbe11] "v"(rbe11), [rbo11] "v"(rbo11), [kstep] "s"(kstep), [s0] "s"(so[0]), \
                 [s1] "s"(so[1]), [s2] "s"(so[2]), [s3] "s"(so[3]), [s4] "s"(so[4]), [s5] "s"(so[5]),            \
                 [s6] "s"(so[6]), [s7] "s"(so[7]), [rA] "s"(sA), [rB] "s"(sB), [nA] "s"(nA), [nB] "s"(nB),       \
                 [nkstep] "s"(nkstep), [m0b0] "s"(m0b0), [m0b1] "s"(m0b1), [flags] "s"(flags), [cv0] "v"(cv[0]), \
                 [cv1] "v"(cv[1]), [cv2] "v"(cv[2]), [cv3] "v"(cv[3]), [cv4] "v"(cv[4]), [cv5] "v"(cv[5]),       \
                 [cv6] "v"(cv[6]), [cv7] "v"(cv[7]), [sC] "s"(sC)                                               \
               : "memory", "scc", W4A_VCLOBBERS, W4EF_VCLOBBERS, W4_AGPR_CLOBBERS)

// Epilogue forms (EPI template argument of w4ap_run and its kernels).
constexpr int W4AP_EPI_STAGED = 0;      // LDS-staged row stores
constexpr int W4AP_EPI_FUSED = 2;       // C stored from the last K-tile's MFMA gaps (generated asm)
constexpr int W4AP_EPI_STAGED_NT = 4;   // staged, nontemporal stores (profiles/r3_s2/)
constexpr int W4AP_EPI_DEFERRED = 7;    // staged nt, quarters 1-3 of C stored during the next tile's K-loop
constexpr int W4AP_EPI_DIRECT = 9;      // EF fragment layout, src C = 0 first K-tile, C stored straight from the
                                        // accumulators after the K-loop (no LDS staging; bf16)
constexpr int W4AP_EPI_WG512 = 10;      // ZC; the workgroup stages 512-byte C rows (both column halves) through
                                        // the shared 32 KiB, 2 barriers per pass: one store = 2 full rows
constexpr int W4AP_EPI_STAGED_ZC = 8;   // staged nt; the K-loop's first K-tile starts accumulators with src C = 0,
                                        // so the epilogue only reads them (generated *_zc schedules)
constexpr int W4AP_EPI_LEAN = 15;       // ZC, staged through conflict-free swizzled LDS rows read back in 8-byte
                                        // halves (lean_off: no lane-dependent half swap) and stored with global saddr stores: one
                                        // per-lane 32-bit offset for the whole tile, the row step in an SGPR base.
                                        // Removes the ~320 per-tile VALU ops (v_cndmask, 64-bit address math)
                                        // that the STAGED_ZC store loop compiles to
constexpr int W4AP_EPI_LEAN_PIPE = 16;  // LEAN in 8 software-pipelined half-passes (double-buffered staging)
constexpr int W4AP_EPI_LEAN_ILV = 17;   // LEAN_PIPE with each half-pass's stores interleaved into the next staging
constexpr int W4AP_EPI_LEAN_ILVB = 18;  // LEAN_ILV reading a half-pass's accumulators in one burst (lab)

// What the staged epilogue does for an EPI value. The tools-only lab library specialises this for its
// knock-out forms (native/hip/gemm_bf16_asm_lab.hip); the production forms are the primary template.
template <int EPI>
struct W4apEpi {
  static constexpr bool run = true;                         // run the staged epilogue at all
  static constexpr bool zc = EPI == W4AP_EPI_STAGED_ZC || EPI == W4AP_EPI_WG512 || EPI == W4AP_EPI_LEAN ||
                             EPI == W4AP_EPI_LEAN_PIPE || EPI == W4AP_EPI_LEAN_ILV ||
                             EPI == W4AP_EPI_LEAN_ILVB;                            // K-loop zeroes (src C = 0)
  template <int S>                                          // pass S's 16-byte C store
  static __device__ __forceinline__ void store(__bf16* dst, uint4 v) {
    if constexpr (EPI == W4AP_EPI_STAGED) *reinterpret_cast<uint4*>(dst) = v;
    else store_c16(dst, v);
  }
};

// The split-K form (SPLIT, v57 / fp8 v24): one (tile, K piece) item per workgroup, gridDim = tiles x
// splits <= the CU count, so the 65-128-tile and the long-K 64-tile grids fill the chip in 256x256
// tiles instead of falling to the smaller tiles of the small-grid frame (gemm_small.h). Items are
// piece-major through xcd_remap: an XCD runs neighbouring tiles (tile_coords) at one K range, so its
// workgroups share A and B panel slices in its L2. Piece p runs K-tile pairs [p P / S, (p + 1) P / S)
// (P = K-tiles / 2: every piece an even count, host: >= 4), or with `last_pairs` the last piece that
// many pairs and the others the rest evenly.
// The reduction, per tile on two counters (arrivals, done): a workgroup draws an arrival ticket first.
// Every arrival but the last stores its fp32 partial as lane-major slabs (per wave 64 accumulator quads
// x 64 lanes x 16 B, one contiguous KiB per store) with plain stores, drains them, meets its waves at a
// barrier, releases ONCE at agent scope and counts itself done; the last arrival keeps its partial in
// its accumulators, waits for the done count of the S - 1 workgroups that arrived before it, acquires
// (agent scope) and sums every piece in a fixed tree of commutative two-input adds -- its own partial
// from its accumulators -- so the result does not depend on arrival order (cdna_hip_programming.md §5 "In-launch split-K reduction",
// §6 Guideline 16). The wait is only ever for workgroups that have already arrived, i.e. are running
// and owe nothing but their stores: no co-residency is assumed. The last arrival resets both counters
// for the next launch, then runs the ordinary epilogue. Only S - 1 of S partials travel, and each writer
// workgroup releases once: the first form of this reduction stored all S partials and released every
// wave's separately (4 L2 write-backs per workgroup), 490 TF/s at 2560^3 (profiles/r6_splitk/).
struct W4Split {
  int splits = 1;
  float* ws = nullptr;   // tiles x splits x 4 waves x 64 KiB
  int* cnt = nullptr;    // tiles x 2 (arrivals, done), zero between launches
  int last_pairs = 0;    // K-tile pairs of the last piece; 0 = even pieces (gemm_small_host.h asm_last_pairs)
  int pmajor = 1;        // item order: 1 piece-major, 0 tile-major (a tile's pieces adjacent, on one XCD)
};

// SPLIT: this workgroup's reduction (every wave calls it). False: the workgroup stored its partial and
// is finished. True: it was the tile's last arrival and its accumulators now hold the sum over every
// piece. `flag`: two LDS words no wave touches until the epilogue (wave 0's epilogue staging).
// SKO: knock-outs for timing in the tools-only lab library (gemm_bf16_asm_lab.hip), wrong results by
// design -- 1: the writers' release, 2: the reducer's slab reads, 4: the writers' slab stores. Every
// production instantiation has SKO = 0.
template <int SKO = 0>
__device__ __forceinline__ bool w4ap_split_reduce(const W4Split& sp, int tile, int piece, int wid, int lane,
                                                  int* flag) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int WAVE_F4 = 64 * 64;   // 64 accumulator quads x 64 lanes
  const int S = sp.splits;
  int* const arrive = sp.cnt + tile * 2;
  int* const done = arrive + 1;
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // the last MFMAs' results
  if (wid == 0 && lane == 0) *flag = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int ticket = __builtin_amdgcn_readfirstlane(*flag);
  // piece p's slab of this wave: quad i of lane l at float4 index ((tile S + p) 4 + wid) 4096 + 64 i + l
  auto slab = [&](int p) { return ((tile * S + p) * 4 + wid) * WAVE_F4 + lane; };
  f4* const ws4 = (f4*)sp.ws;
  auto own = [&](auto I) {
    constexpr int i = decltype(I)::value;
    float x0, x1, x2, x3;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                 "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                 : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                 : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
    return f4{x0, x1, x2, x3};
  };
  if (ticket < S - 1) {
    f4* const mine = ws4 + slab(piece);
    if constexpr (!(SKO & 4)) static_for<0, 64>([&](auto I) { mine[decltype(I)::value * 64] = own(I); });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wid == 0 && lane == 0) {
      if constexpr (!(SKO & 1)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return false;
  }
  if (wid == 0 && lane == 0) {
    // every workgroup counted here has arrived and owes only its stores; bounded all the same (~1 s)
    bool seen = false;
    for (unsigned spins = 0; !(seen = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= S - 1) &&
                             spins < (1u << 24); ++spins)
      __builtin_amdgcn_s_sleep(2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    *arrive = 0;                       // ready for the next launch on this stream
    *done = 0;
    flag[1] = seen;                    // (flag[0] holds the ticket the other waves may still be reading)
  }
  __syncthreads();
  auto put = [&](auto I, f4 t) {
    constexpr int i = decltype(I)::value;
    asm volatile("v_accvgpr_write_b32 a%c0, %4\n\tv_accvgpr_write_b32 a%c1, %5\n\t"
                 "v_accvgpr_write_b32 a%c2, %6\n\tv_accvgpr_write_b32 a%c3, %7"
                 :: "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3),
                    "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3]));
  };
  if (!__builtin_amdgcn_readfirstlane(flag[1])) {
    // the wait gave up (a writer that never counted itself done): a NaN tile, never a silent partial sum
    const float nan = __builtin_nanf("");
    static_for<0, 64>([&](auto I) { put(I, f4{nan, nan, nan, nan}); });
    return true;
  }
  // The sum is a fixed tree of two-input adds -- S = 2: p0 + p1; 3: (p0 + p1) + p2; 4: (p0 + p1) + (p2 + p3)
  // -- and a two-input add is commutative, so whichever piece reduces, holding its own partial in its
  // accumulators, computes the same bits. add_slab: accumulators += slab p (32 quads, 128 VGPRs, in flight
  // at once); add_pair: accumulators += (slab a + slab b), both slabs' 16-quad chunks in flight together.
  auto add_slab = [&](int p) {
    const f4* const src = ws4 + slab(p);
    static_for<0, 2>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      f4 t[32];
#pragma unroll
      for (int j = 0; j < 32; ++j) t[j] = src[(q * 32 + j) * 64];
      static_for<0, 32>([&](auto J) {
        constexpr int i = q * 32 + decltype(J)::value;
        const f4 tj = t[decltype(J)::value];   // (a generic lambda does not capture a name used only in asm operands)
        put(std::integral_constant<int, i>{}, own(std::integral_constant<int, i>{}) + tj);
      });
    });
  };
  auto add_pair = [&](int pa, int pb) {
    const f4* const sa = ws4 + slab(pa);
    const f4* const sb = ws4 + slab(pb);
    static_for<0, 4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      f4 ta[16], tb[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        ta[j] = sa[(q * 16 + j) * 64];
        tb[j] = sb[(q * 16 + j) * 64];
      }
      static_for<0, 16>([&](auto J) {
        constexpr int i = q * 16 + decltype(J)::value;
        const f4 pj = ta[decltype(J)::value] + tb[decltype(J)::value];
        put(std::integral_constant<int, i>{}, own(std::integral_constant<int, i>{}) + pj);
      });
    });
  };
  if constexpr (SKO & 2) {
  } else if (S == 2) {
    add_slab(1 - piece);
  } else if (S == 3) {
    if (piece == 2) {
      add_pair(0, 1);
    } else {
      add_slab(1 - piece);
      add_slab(2);
    }
  } else if (S == 4) {
    add_slab(piece ^ 1);
    add_pair(piece < 2 ? 2 : 0, piece < 2 ? 3 : 1);
  } else {
    // more pieces (forced only): piece order, 16 quads at a time
    static_for<0, 4>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      f4 acc[16];
      for (int p = 0; p < S; ++p) {
        f4 t[16];
        if (p == piece) {
          static_for<0, 16>([&](auto J) { t[decltype(J)::value] = own(std::integral_constant<int, q * 16 + decltype(J)::value>{}); });
        } else {
          const f4* const src = ws4 + slab(p);
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = src[(q * 16 + j) * 64];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) acc[j] = p == 0 ? t[j] : acc[j] + t[j];
      }
      static_for<0, 16>([&](auto J) {
        const f4 aj = acc[decltype(J)::value];
        put(std::integral_constant<int, q * 16 + decltype(J)::value>{}, aj);
      });
    });
  }
  return true;
}

// A, Bt: K-major operands (element size 1 for F8, else 2); C: bf16; smem: W4AP_LDS bytes.
// DM (DMA form): 0 = one lane offset + per-row-block SGPR soffsets, SC indexes W4AP/F8AP schedules;
// 1 = VP (per-piece VGPR lane offsets, SGPR K offset), SC indexes the VP schedules; 2 = VP with the
// A-panel pieces reading rows 32 apart (PA; the epilogue maps LDS slot s to C row 32 (s & 7) + (s >> 3)).
// EPI: the W4AP_EPI_* forms above (W4apEpi says what the staged epilogue does for each).
template <int SC, bool SERP, bool SQ, bool F8, int EPI = 0, int DM = 0, bool SPLIT = false, int SKO = 0>
__device__ __forceinline__ void w4ap_run(const char* __restrict__ A, const char* __restrict__ Bt,
                                         __bf16* __restrict__ C, int M, int N, int K, char* smem,
                                         W4Split sp = W4Split{}) {
  constexpr int ESZ = F8 ? 1 : 2;
  const int tiles_m = M / W4AP_TILE;
  const int tiles_n = N / W4AP_TILE;
  const int nwg = tiles_m * tiles_n;
  int tile, per, t_end, piece = 0;
  if constexpr (SPLIT) {
    const int items = nwg * sp.splits;                    // gridDim == items
    const int item = xcd_remap((int)blockIdx.x, items);
    piece = sp.pmajor ? item / nwg : item % sp.splits;
    tile = sp.pmajor ? item - piece * nwg : item / sp.splits;
    per = items;                                          // one item per workgroup: no next tile
    t_end = nwg;
  } else if constexpr (SQ) {
    tile = (int)blockIdx.x;
    per = (int)gridDim.x;
    t_end = nwg;
  } else {
    const int xcd = blockIdx.x % NXCD;
    per = gridDim.x / NXCD;
    const int q = nwg / NXCD, rem = nwg % NXCD;
    const int t_begin = (xcd < rem) ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
    t_end = t_begin + q + (xcd < rem ? 1 : 0);
    tile = t_begin + (int)(blockIdx.x / NXCD);
  }
  if (tile >= t_end) return;                              // uniform over the workgroup
  auto coords = [&](int t, int& m, int& n) {
    if constexpr (SQ) tile_coords_sq(t, tiles_n, m, n);
    else tile_coords(t, tiles_m, tiles_n, m, n);
  };

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const uint32_t row_bytes = (uint32_t)K * ESZ;
  const uint32_t panel_bytes = (uint32_t)W4AP_TILE * row_bytes;
  auto mk_rs = [&](const char* base) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    w4a_u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    r[2] = panel_bytes;
    r[3] = 0x00020000u;
    return r;
  };
  const int par = wid & 1;
  int ktiles = (int)(row_bytes / W4AP_ROW);
  size_t kbyte0 = 0;                                      // SPLIT: the piece's first K-tile, in bytes
  if constexpr (SPLIT) {
    const int pairs = ktiles >> 1;
    int p0 = piece * pairs / sp.splits, p1 = (piece + 1) * pairs / sp.splits;
    if (sp.last_pairs > 0) {            // the first S - 1 pieces share pairs - last_pairs evenly
      const int rest = pairs - sp.last_pairs, n = sp.splits - 1;
      p0 = piece < n ? piece * rest / n : rest;
      p1 = piece < n ? (piece + 1) * rest / n : pairs;
    }
    kbyte0 = (size_t)(2 * p0) * W4AP_ROW;
    ktiles = 2 * (p1 - p0);
  }
  const uint32_t lane_dma = (uint32_t)(lane >> 3) * row_bytes +
                            (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  // the lane offset of a tile's first DMA K-tile, and its K step, by walking direction
  auto voff0 = [&](bool rev) { return lane_dma + (uint32_t)((rev ? ktiles - 1 : 0) * W4AP_ROW); };
  auto kst = [&](bool rev) { return rev ? -W4AP_ROW : W4AP_ROW; };
  uint32_t so[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    so[i] = __builtin_amdgcn_readfirstlane((uint32_t)((i << 2) + wid) * 8u * row_bytes);
  static_assert(DM == 0 || (EPI != W4AP_EPI_FUSED && EPI != W4AP_EPI_DEFERRED), "EPI 2 / 7 use the DM 0 DMA form");
  uint32_t vp[16] = {};
  if constexpr (DM >= 1) {
    const uint32_t chunk = (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const uint32_t rblk = (uint32_t)(((p & 7) << 2) + wid);
      vp[p] = (DM == 2 && p < 8) ? (uint32_t)(lane >> 3) * 32u * row_bytes + chunk + rblk * row_bytes
                                 : (uint32_t)(lane >> 3) * row_bytes + chunk + rblk * 8u * row_bytes;
    }
  }
  auto koff0 = [&](bool rev) { return __builtin_amdgcn_readfirstlane((uint32_t)((rev ? ktiles - 1 : 0) * W4AP_ROW)); };
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  const uint32_t m0b0 = lds0 + (uint32_t)wid * 1024u, m0b1 = m0b0 + (uint32_t)W4AP_BUF;
  // a lane's two 16-byte chunks of row (lane & 15) of a 16-row fragment: kk*4 + g for bf16 k-half
  // kk, g + 4h for fp8 half h (F8Q_CHUNK) -- the same address; chunk c of row R sits at c ^ ((R>>1)&7)
  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * W4AP_ROW + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const uint32_t a_base = lds0 + (uint32_t)(wr * 128 * W4AP_ROW);
  const uint32_t b_base = lds0 + (uint32_t)(W4AP_PANEL + wc * 128 * W4AP_ROW);
  const uint32_t ra00 = a_base + lane_off[0], rb00 = b_base + lane_off[0];
  const uint32_t ra01 = a_base + lane_off[1], rb01 = b_base + lane_off[1];
  const uint32_t ra10 = ra00 + W4AP_BUF, rb10 = rb00 + W4AP_BUF;
  const uint32_t ra11 = ra01 + W4AP_BUF, rb11 = rb01 + W4AP_BUF;
  // EF (EPI=2): B fragment x, row rho reads panel row 32(x>>1) + 4(x&1) + 8(rho>>2) + (rho&3); even and
  // odd fragments differ in bit 1 of the chunk swizzle, so each has its own lane offset (the fragment's
  // 4 KiB step is the read's immediate offset). Lane (g, r) of accumulator pair (m, 2p), (m, 2p+1) then
  // holds C row 16m + r, columns 32p + 8g .. +7: cv[m] is that row's byte offset from the wave's corner.
  uint32_t rbe00 = 0, rbo00 = 0, rbe01 = 0, rbo01 = 0, rbe10 = 0, rbo10 = 0, rbe11 = 0, rbo11 = 0;
  uint32_t cv[8] = {};
  constexpr bool EFL = EPI == W4AP_EPI_FUSED || EPI == W4AP_EPI_DIRECT;   // the EF fragment layout
  static_assert(!(EPI == W4AP_EPI_DIRECT && F8), "EPI 9 is generated for bf16 only");
  if constexpr (EFL) {
    const int rho = lane & 15;
    const int re = 8 * (rho >> 2) + (rho & 3);
    uint32_t pe[2], po[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int c = kk * 4 + (lane >> 4);
      pe[kk] = b_base + (uint32_t)(re * W4AP_ROW + ((c ^ ((re >> 1) & 7)) << 4));
      po[kk] = b_base + (uint32_t)((re + 4) * W4AP_ROW + ((c ^ (((re + 4) >> 1) & 7)) << 4));
    }
    rbe00 = pe[0]; rbo00 = po[0]; rbe01 = pe[1]; rbo01 = po[1];
    rbe10 = pe[0] + W4AP_BUF; rbo10 = po[0] + W4AP_BUF; rbe11 = pe[1] + W4AP_BUF; rbo11 = po[1] + W4AP_BUF;
#pragma unroll
    for (int m = 0; m < 8; ++m)
      cv[m] = (uint32_t)(16 * m + rho) * (uint32_t)N * 2u + (uint32_t)(16 * (lane >> 4));
  }
  char* const stg = smem + 2 * W4AP_BUF + wid * W4AP_EPI_WAVE;
  // EPI 7: the held C quarters, the lane's LDS slot of the staged quarter, the store offset walker
  w4a_u32x4 held[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) held[i] = w4a_u32x4{0u, 0u, 0u, 0u};
  const uint32_t stgl = (uint32_t)(uintptr_t)stg + (uint32_t)lane * 16u;
  const uint32_t s8N = __builtin_amdgcn_readfirstlane((uint32_t)N * 8u);
  const uint32_t vcur0 = (uint32_t)(32 + (lane >> 4)) * (uint32_t)N * 2u + (uint32_t)(lane & 15) * 16u;
  auto corner = [&](int tm_, int tn_) {
    const uint64_t cc = (uint64_t)(uintptr_t)(C + (size_t)(tm_ * W4AP_TILE + wr * 128) * N + tn_ * W4AP_TILE + wc * 128);
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cc >> 32)) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cc);
  };

  int tm, tn;
  coords(tile, tm, tn);
  bool rev = false;
  w4a_u32x4 sA = mk_rs(A + (size_t)tm * panel_bytes + kbyte0), sB = mk_rs(Bt + (size_t)tn * panel_bytes + kbyte0);
  uint32_t voff_k = voff0(rev);
  uint32_t koff = koff0(rev);
  int kstep = kst(rev);
  uint32_t first = 1;
  uint64_t sCp = corner(tm, tn);    // the first tile's deferred stores write its own corner (overwritten later)

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  if constexpr (!EFL && !W4apEpi<EPI>::zc)   // EF / direct / ZC: the first K-tile uses src C = 0
    static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });
  for (;;) {
    const int next = tile + per;
    const uint32_t hasnext = __builtin_amdgcn_readfirstlane(next < t_end ? 1u : 0u);
    const bool nrev = SERP && !rev;
    int ntm = tm, ntn = tn;
    w4a_u32x4 nA = sA, nB = sB;
    if (hasnext) {
      coords(next, ntm, ntn);
      nA = mk_rs(A + (size_t)ntm * panel_bytes);
      nB = mk_rs(Bt + (size_t)ntn * panel_bytes);
    }
    uint32_t nvoff = voff0(nrev);
    uint32_t nkoff = koff0(nrev);
    const int nkstep = kst(nrev);
    uint32_t trips = __builtin_amdgcn_readfirstlane((uint32_t)((ktiles - 2) >> 1));
    uint32_t m0save;
    const uint32_t flags = __builtin_amdgcn_readfirstlane(first | (hasnext << 1));
    if constexpr (EFL) {
      // this tile's C corner for the fused epilogue's stores (wave-uniform)
      const uint64_t cc = (uint64_t)(uintptr_t)(C + (size_t)(tm * W4AP_TILE + wr * 128) * N + tn * W4AP_TILE + wc * 128);
      // readfirstlane returns int: widen through uint32_t, or bit 31 of the low word sign-extends
      const uint64_t sC = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cc >> 32)) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cc);
      if constexpr (F8) {
        F8EF_LOOP_SELECT(SC)
      } else {
        W4EF_LOOP_SELECT(SC)
      }
    } else if constexpr (EPI == W4AP_EPI_DEFERRED) {
      uint32_t vcur = vcur0;
      if constexpr (F8) {
        F8DS_LOOP_SELECT(SC)
      } else {
        W4DS_LOOP_SELECT(SC)
      }
    } else if constexpr (DM >= 1 && F8) {
      F8VP_LOOP_SELECT(SC)
    } else if constexpr (DM >= 1) {
      W4VP_LOOP_SELECT(SC)
    } else if constexpr (F8) {
      F8AP_LOOP_SELECT(SC)
    } else {
      W4AP_LOOP_SELECT(SC)
    }

    if constexpr (SPLIT) {
      if (sp.splits > 1 && !w4ap_split_reduce<SKO>(sp, tile, piece, wid, lane, (int*)(smem + 2 * W4AP_BUF))) return;
    }

    // wave-private epilogue (the K buffers may be receiving the next tile's DMA): 4 passes of
    // 2 fragment rows = 32 C rows x 128 columns through this wave's 8 KiB, accumulators zeroed
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    if constexpr (EPI == 2) {
      // the asm block stored C; its stores and the next tile's DMA are waited for by count in the next block
    } else if constexpr (EPI == W4AP_EPI_DIRECT) {
      // accumulator pair (m, 2p), (m, 2p+1): lane (g, r) holds C row 16m + r, columns 32p + 8g .. +7
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");          // the next tile's DMA landed
      __bf16* const cw = C + (size_t)(tm * W4AP_TILE + wr * 128 + (lane & 15)) * N + tn * W4AP_TILE + wc * 128 +
                         8 * (lane >> 4);
      static_for<0, 32>([&](auto Q) {
        constexpr int m = decltype(Q)::value >> 2, p = decltype(Q)::value & 3;
        constexpr int a0 = 4 * (m * 8 + 2 * p);
        float x[8];
        asm volatile("v_accvgpr_read_b32 %0, a%c8\n\tv_accvgpr_read_b32 %1, a%c9\n\t"
                     "v_accvgpr_read_b32 %2, a%c10\n\tv_accvgpr_read_b32 %3, a%c11\n\t"
                     "v_accvgpr_read_b32 %4, a%c12\n\tv_accvgpr_read_b32 %5, a%c13\n\t"
                     "v_accvgpr_read_b32 %6, a%c14\n\tv_accvgpr_read_b32 %7, a%c15"
                     : "=v"(x[0]), "=v"(x[1]), "=v"(x[2]), "=v"(x[3]), "=v"(x[4]), "=v"(x[5]), "=v"(x[6]), "=v"(x[7])
                     : "i"(a0), "i"(a0 + 1), "i"(a0 + 2), "i"(a0 + 3), "i"(a0 + 4), "i"(a0 + 5), "i"(a0 + 6),
                       "i"(a0 + 7));
        typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
        bf16x8 b;
#pragma unroll
        for (int e = 0; e < 8; ++e) b[e] = (__bf16)x[e];
        store_c16(cw + (size_t)(16 * m) * N + 32 * p, __builtin_bit_cast(uint4, b));
      });
    } else if constexpr (EPI == W4AP_EPI_LEAN) {
      // 4 passes of 32 C rows x 128 columns through this wave's 8 KiB. Lane (r, j) of accumulator m*8+n
      // holds row 16m + r, columns 16n + 4j .. +3: the 8-byte half j & 1 of 16-byte chunk 2n + (j >> 1).
      // Staged through lean_off (bank-conflict free on both sides, no half swap on the way back).
      const int lr = lane & 15, lj = lane >> 4;
      const uint32_t vst = DM == 2 ? (uint32_t)lj * 64u * (uint32_t)N + (uint32_t)lr * 16u    // PA: rows 32 apart
                                   : (uint32_t)lj * 2u * (uint32_t)N + (uint32_t)lr * 16u;
      const uint64_t cb = (uint64_t)(uintptr_t)(C + (size_t)tm * W4AP_TILE * N + tn * W4AP_TILE + wc * 128);
      const uint64_t cbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cb >> 32)) << 32) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cb);
      const uint64_t rowb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)N * 2u);
      // the wave-uniform part of a store's C row, walked by one SGPR pointer (laundered so the compiler
      // cannot fold every store's row into a hoisted 64-bit constant: 32 of them spill the SGPR file).
      // DM 0/1: row 128 wr + 32 s + 4 k, +4 rows a store. DM 2 maps LDS slot wr*128 + s*32 + r to panel
      // row 32 (slot & 7) + (slot >> 3) = 32 lj + [128 (k & 1) + 16 wr + 4 s + (k >> 1)]: even k at the
      // pointer, odd k 128 rows on, +1 row a pair
      uint64_t cp = cbase + (uint64_t)(DM == 2 ? 16 * wr : 128 * wr) * rowb;
      const uint64_t cstep = DM == 2 ? rowb : 4 * rowb;
      const uint64_t codd = 128 * rowb;
      static_for<0, 4>([&](auto S) {
        constexpr int s = decltype(S)::value;
        static_for<0, 16>([&](auto I) {
          constexpr int u = decltype(I)::value;
          constexpr int mm = u >> 3, n = u & 7;
          constexpr int i = (2 * s + mm) * 8 + n;
          float x0, x1, x2, x3;
          asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                       "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                       : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                       : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
          bf16x4 v;
          v[0] = (__bf16)x0;
          v[1] = (__bf16)x1;
          v[2] = (__bf16)x2;
          v[3] = (__bf16)x3;
          const int c = 2 * n + (lj >> 1);
          *reinterpret_cast<bf16x4*>(stg + lean_off(mm * 16 + lr, c, lj & 1)) = v;
        });
        asm volatile("" ::: "memory");     // a wave's LDS ops execute in order: no wait, no barrier
        if constexpr (s == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's DMA landed
        const uint32_t vs = vst;           // (a generic lambda does not capture a name used only in asm operands)
        // all 8 row reads in flight before the first store (the stores' memory clobber orders them)
        w4a_u32x4 rows[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = k * 4 + lj;
          rows[k] = lean_read(stg, r, lr);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t base = (DM == 2 && (k & 1)) ? cp + codd : cp;
          // s_nop: a VALU write of a > 8-byte store's data VGPRs needs one wait state after the store,
          // which the compiler cannot see inside the asm
          asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 0" :: "v"(vs), "v"(rows[k]), "s"(base) : "memory");
          if (DM != 2 || (k & 1)) {
            cp += cstep;
            asm volatile("" : "+s"(cp));
          }
        }
        asm volatile("" ::: "memory");
      });
    } else if constexpr (EPI == W4AP_EPI_LEAN_PIPE || EPI == W4AP_EPI_LEAN_ILV || EPI == W4AP_EPI_LEAN_ILVB) {
      constexpr bool ILV = EPI != W4AP_EPI_LEAN_PIPE;
      // LEAN in 8 half-passes of 16 rows (one accumulator row block each) through two 4 KiB halves of
      // the wave's staging, software-pipelined: half-pass h + 1's accumulator reads, cvts and LDS writes
      // run while half-pass h's row reads land, then h's 4 stores go out (order W0 R0 | W1 R1 S0 | W2 R2
      // S1 | ...): the LDS round trip and the store issue hide under VALU work instead of stalling it.
      const int lr = lane & 15, lj = lane >> 4;
      const uint32_t vst = DM == 2 ? (uint32_t)lj * 64u * (uint32_t)N + (uint32_t)lr * 16u
                                   : (uint32_t)lj * 2u * (uint32_t)N + (uint32_t)lr * 16u;
      const uint64_t cb = (uint64_t)(uintptr_t)(C + (size_t)tm * W4AP_TILE * N + tn * W4AP_TILE + wc * 128);
      const uint64_t cbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cb >> 32)) << 32) |
                             (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cb);
      const uint64_t rowb = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)N * 2u);
      // DM 0/1: half-pass h, read k (row 4k + lj of the block) is tile row 128 wr + 16 h + 4 k: +4 rows a
      // store. DM 2: LDS slot wr*128 + 16 h + 4 k + lj -> panel row 32 lj + [128 (k & 1) + 16 wr + 2 h +
      // (k >> 1)]: the pointer walks 16 wr + 2 h, read k adds 128 (k & 1) + (k >> 1) rows
      uint64_t cp = cbase + (uint64_t)(DM == 2 ? 16 * wr : 128 * wr) * rowb;
      const uint64_t c1 = rowb, c128 = 128 * rowb, c129 = 129 * rowb, c4 = 4 * rowb, c2 = 2 * rowb;
      auto stage = [&](auto H, auto&& after) {
        constexpr int h = decltype(H)::value;
        char* const buf = stg + (h & 1) * 4096;
        if constexpr (EPI == W4AP_EPI_LEAN_ILVB) {
          // ILVB: the half-pass's 32 accumulator registers in one read burst, then the cvts and LDS
          // writes -- no accvgpr-read -> VALU wait state per accumulator
          float x[32];
          static_for<0, 8>([&](auto I) {
            constexpr int i = h * 8 + decltype(I)::value;
            constexpr int q = 4 * decltype(I)::value;
            float a0, a1, a2, a3;        // (asm operands cannot name the enclosing lambda's array)
            asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                         "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                         : "=v"(a0), "=v"(a1), "=v"(a2), "=v"(a3)
                         : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
            x[q] = a0;
            x[q + 1] = a1;
            x[q + 2] = a2;
            x[q + 3] = a3;
          });
          static_for<0, 8>([&](auto I) {
            constexpr int n = decltype(I)::value;
            bf16x4 v;
            v[0] = (__bf16)x[4 * n];
            v[1] = (__bf16)x[4 * n + 1];
            v[2] = (__bf16)x[4 * n + 2];
            v[3] = (__bf16)x[4 * n + 3];
            const int c = 2 * n + (lj >> 1);
            *reinterpret_cast<bf16x4*>(buf + lean_off(lr, c, lj & 1)) = v;
            after(I);
          });
          return;
        }
        static_for<0, 8>([&](auto I) {
          constexpr int n = decltype(I)::value;
          constexpr int i = h * 8 + n;
          float x0, x1, x2, x3;
          asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                       "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                       : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                       : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
          bf16x4 v;
          v[0] = (__bf16)x0;
          v[1] = (__bf16)x1;
          v[2] = (__bf16)x2;
          v[3] = (__bf16)x3;
          const int c = 2 * n + (lj >> 1);
          *reinterpret_cast<bf16x4*>(buf + lean_off(lr, c, lj & 1)) = v;
          after(I);
        });
      };
      auto nothing = [](auto) {};
      auto load = [&](auto H, w4a_u32x4* rows) {
        constexpr int h = decltype(H)::value;
        const char* const buf = stg + (h & 1) * 4096;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int r = k * 4 + lj;
          rows[k] = lean_read(buf, r, lr);
        }
      };
      auto store_one = [&](const w4a_u32x4* rows, int k) {
        const uint32_t vs = vst;
        uint64_t base = cp;
        if (DM == 2) base = cp + (k == 0 ? 0 : k == 1 ? c128 : k == 2 ? c1 : c129);
        // s_nop: the store's data VGPRs may be rewritten by the next VALU (one wait state)
        asm volatile("global_store_dwordx4 %0, %1, %2 nt\n\ts_nop 0" :: "v"(vs), "v"(rows[k]), "s"(base) : "memory");
        if (DM != 2 || k == 3) {
          cp += DM == 2 ? c2 : c4;
          asm volatile("" : "+s"(cp));
        }
      };
      auto store = [&](const w4a_u32x4* rows) {
#pragma unroll
        for (int k = 0; k < 4; ++k) store_one(rows, k);
      };
      w4a_u32x4 ra[4], rb[4];
      stage(std::integral_constant<int, 0>{}, nothing);
      load(std::integral_constant<int, 0>{}, ra);
      static_for<0, 8>([&](auto H) {
        constexpr int h = decltype(H)::value;
        const w4a_u32x4* const cur = (h & 1) ? rb : ra;
        if constexpr (ILV && h + 1 < 8) {
          // ILV: half-pass h's 4 stores ride between half-pass h + 1's accumulator stagings (one after
          // every second ds_write), so no store burst stalls the VALU stream
          if constexpr (h == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          stage(std::integral_constant<int, h + 1>{}, [&](auto I) {
            if constexpr (decltype(I)::value & 1) store_one(cur, decltype(I)::value >> 1);
          });
          load(std::integral_constant<int, h + 1>{}, (h & 1) ? ra : rb);
        } else {
          if constexpr (h + 1 < 8) {
            stage(std::integral_constant<int, h + 1>{}, nothing);
            load(std::integral_constant<int, h + 1>{}, (h & 1) ? ra : rb);
          }
          // the next tile's DMA landed before any C store (its K-loop's landing waits count only its
          // own pieces); waiting here, not before half-pass 1, gives the DMA two half-passes of cover
          if constexpr (h == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          store(cur);
        }
      });
      asm volatile("" ::: "memory");
    } else if constexpr (!W4apEpi<EPI>::run) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
    // last MFMA D -> accvgpr reads. ZC reads in pass order, whose first accumulators took their last
    // MFMA >= 16 MFMAs before the end of the K-tile (g4 / p orders), so it needs no pad
    if constexpr (W4apEpi<EPI>::zc) {
    } else if constexpr (F8) asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    else asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    static_for<0, 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      static_for<0, 16>([&](auto I) {
        constexpr int u = decltype(I)::value;
        constexpr int mm = u >> 3, n = u & 7;
        constexpr int i = (2 * s + mm) * 8 + n;                    // accumulator index m*8+n
        float x0, x1, x2, x3;
        if constexpr (W4apEpi<EPI>::zc)
          asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                       "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                       : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                       : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
        else
          asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                       "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7\n\t"
                       "v_accvgpr_write_b32 a%c4, 0\n\tv_accvgpr_write_b32 a%c5, 0\n\t"
                       "v_accvgpr_write_b32 a%c6, 0\n\tv_accvgpr_write_b32 a%c7, 0"
                       : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                       : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
        const int r = mm * 16 + (lane & 15);
        const int g = n * 4 + (lane >> 4);
        bf16x4 v;
        v[0] = (__bf16)x0;
        v[1] = (__bf16)x1;
        v[2] = (__bf16)x2;
        v[3] = (__bf16)x3;
        if constexpr (EPI == W4AP_EPI_WG512) {
          // shared staging [wr][32 rows][512 B]: column group c (8 B) of row r at c ^ (r & 31)
          const int c = wc * 32 + g;
          *reinterpret_cast<bf16x4*>(smem + 2 * W4AP_BUF + wr * 16384 + r * 512 + ((c ^ (r & 31)) << 3)) = v;
        } else {
          *reinterpret_cast<bf16x4*>(stg + r * 256 + ((g ^ (r & 15)) << 3)) = v;
        }
      });
      asm volatile("" ::: "memory");     // a wave's LDS ops execute in order: no wait, no barrier
      if constexpr (s == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the next tile's DMA landed
      if constexpr (EPI == W4AP_EPI_WG512) {
        __syncthreads();                  // both column halves of every row staged
        // wave w stores rows (w & 1) * 16 .. +15 of row block w >> 1: one store = 2 rows x 512 B
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = (wid & 1) * 16 + 2 * k + (lane >> 5);
          const int sw = r & 31;
          const int pg = (2 * (lane & 31)) ^ sw;
          const uint4 raw = *reinterpret_cast<const uint4*>(smem + 2 * W4AP_BUF + (wid >> 1) * 16384 + r * 512 +
                                                            ((pg & ~1) << 3));
          uint4 v = raw;
          if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
          store_c16(C + (size_t)(tm * W4AP_TILE + (wid >> 1) * 128 + s * 32 + r) * N + tn * W4AP_TILE + (lane & 31) * 8, v);
        }
        __syncthreads();                  // the staging is free for the next pass
      } else if constexpr (EPI == W4AP_EPI_DEFERRED) {
        // quarter 0 now; with a next tile, quarters 1-2 stay in registers (held) and quarter 3 in this
        // wave's staging LDS, lane-linear, for the next tile's K-loop to store (W4DS_LOOP)
        uint4 vv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = k * 4 + (lane >> 4);
          const int sw = r & 15;
          const int pg = (2 * (lane & 15)) ^ sw;
          const uint4 raw = *reinterpret_cast<const uint4*>(stg + r * 256 + ((pg & ~1) << 3));
          vv[k] = raw;
          if (sw & 1) { vv[k].x = raw.z; vv[k].y = raw.w; vv[k].z = raw.x; vv[k].w = raw.y; }
        }
        if (s == 0 || !hasnext) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int r = k * 4 + (lane >> 4);
            store_c16(C + (size_t)(tm * W4AP_TILE + wr * 128 + s * 32 + r) * N + tn * W4AP_TILE + wc * 128 +
                          (lane & 15) * 8, vv[k]);
          }
        } else if constexpr (s == 1 || s == 2) {
#pragma unroll
          for (int k = 0; k < 8; ++k)
            held[(s - 1) * 8 + k] = w4a_u32x4{vv[k].x, vv[k].y, vv[k].z, vv[k].w};
        } else {
          asm volatile("" ::: "memory");   // every read of the staging above is issued before these writes
#pragma unroll
          for (int k = 0; k < 8; ++k) *reinterpret_cast<uint4*>(stg + k * 1024 + lane * 16) = vv[k];
        }
      } else
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = k * 4 + (lane >> 4);
        const int ch = lane & 15;
        const int sw = r & 15;
        const int pg = (2 * ch) ^ sw;
        const uint4 raw = *reinterpret_cast<const uint4*>(stg + r * 256 + ((pg & ~1) << 3));
        uint4 v = raw;
        if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
        const int slot = wr * 128 + s * 32 + r;                        // the tile row's LDS slot
        const int crow = DM == 2 ? 32 * (slot & 7) + (slot >> 3) : slot; // PA: slot -> panel row
        __bf16* const dst = C + (size_t)(tm * W4AP_TILE + crow) * N + tn * W4AP_TILE + wc * 128 + ch * 8;
        W4apEpi<EPI>::template store<s>(dst, v);
      }
      asm volatile("" ::: "memory");
    });
    }
    if constexpr (EPI == W4AP_EPI_DEFERRED) sCp = corner(tm, tn);   // the next tile stores this tile's rest
    if (!hasnext) break;
    tile = next;
    tm = ntm;
    tn = ntn;
    sA = nA;
    sB = nB;
    rev = nrev;
    voff_k = nvoff;                 // the drain advanced it past the next tile's K-tiles 0 and 1
    koff = nkoff;
    kstep = nkstep;
    first = 0;
  }
}

}  // namespace
