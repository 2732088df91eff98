// Tools-only experiment library (libamdgo_gemm_lab.so, built by `python -m gpu_operator_amd._build
// --lab`): every superseded bf16 GEMM generation (v1-v19, the v30-v35 barrier sweep, the v20-v24
// knock-out timings whose results are WRONG on purpose) plus the production kernels under pinned
// variant numbers, for A/B sweeps (tools/gemm_sweep.py) and rocprofv3 knock-out profiling.
// Never loaded by the validator: the shipped libamdgo_hip.so (gemm_bf16.hip) dispatches only the
// production set and ignores environment variables.
//
// Variants: 1 = double-buffered baseline, 2 = fragment pipelined, 3 = ping-pong (two wave groups
// one barrier apart, half-tile LDS ring), 4 = v3 with buffer_load...lds staging, 5 = v4 with an
// LDS-staged, fully coalesced epilogue, 6-9 = v5 phase/knob variants; 10-14 = one wave per SIMD with
// a 128x128 wave tile; 15-17 = half-tile ring; 18/19 = the K-tile schedule; 20-24 = knock-outs;
// (the v44 knock-outs 80-89 and the row-grouping timings 95-97 were retired once priced:
// profiles/r2_sched/README.md);
// 25-27 = persistent; 30-35 = barrier-placement sweep; 40/41 = serpentine K, 42/43 = loop rotation,
// 44 = both (production default), 45 = 44 + square raster. Measured: profiles/r1_gemm_v4/,
// profiles/r1_s2_gemm/, profiles/r1_s6_sq/.
#include <stdlib.h>

#include "gemm_bf16_asm_loop_lab.h"  // every schedule (masks the production header)
#include "gemm_bf16_kernels.h"

namespace {

// smallest j in [0, n] with j*span/n >= q: items j of a span placed at group j*span/n, so the
// items of group q are [lab_span_lo(q), lab_span_lo(q+1))
constexpr int lab_span_lo(int q, int span, int n) {
  for (int j = 0; j < n; ++j)
    if (j * span / n >= q) return j;
  return n;
}

// Stage one 256-row x 64-k panel (32 KiB) of a K-major operand into LDS.
// 32 wave-instructions of 1 KiB (8 rows each); wave w issues rows blocks {w, w+8, w+16, w+24}.
__device__ __forceinline__ void stage_panel(const __bf16* __restrict__ g, int ld, int k0,
                                            char* lds_panel, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rblk = i * 8 + wid;           // 8-row block index 0..31
    const int r = rblk * 8 + (lane >> 3);   // row inside the panel
    const int pc = lane & 7;                // physical 16-B chunk this lane writes
    const int c = pc ^ ((r >> 1) & 7);      // logical chunk it must fetch (XOR involution)
    const __bf16* src = g + (size_t)r * ld + k0 + c * 8;
    char* dst = lds_panel + rblk * 1024;    // wave-uniform base; HW adds lane*16
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)dst, 16, 0, 0);
  }
}

__global__ void __launch_bounds__(NTHREADS)
gemm_bf16_256x256(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                  __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2;   // 0..1  -> 128-row half of the tile
  const int wc = wid & 3;    // 0..3  -> 64-col quarter of the tile

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;

  // Per-lane LDS read offsets for the two 32-deep k-steps of a BK=64 tile.
  // Row within a 16-row fragment = lane&15; logical chunk = kk*4 + (lane>>4);
  // swizzle term ((row>>1)&7) only depends on lane because fragment bases are 16-row aligned.
  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * ROW_BYTES + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_row0 = wr * 128;   // first A row (panel-local) this wave reads
  const int b_row0 = wc * 64;    // first Bt row (panel-local) this wave reads

  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int ktiles = K / BK;

  stage_panel(gA, K, 0, smem, wid, lane);
  stage_panel(gB, K, 0, smem + PANEL_BYTES, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  for (int t = 0; t < ktiles; ++t) {
    char* cur = smem + (t & 1) * BUF_BYTES;
    if (t + 1 < ktiles) {
      char* nxt = smem + ((t + 1) & 1) * BUF_BYTES;
      stage_panel(gA, K, (t + 1) * BK, nxt, wid, lane);
      stage_panel(gB, K, (t + 1) * BK, nxt + PANEL_BYTES, wid, lane);
    }
    const char* la = cur + a_row0 * ROW_BYTES;
    const char* lb = cur + PANEL_BYTES + b_row0 * ROW_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[8], bfr[4];
#pragma unroll
      for (int n = 0; n < 4; ++n)
        bfr[n] = *reinterpret_cast<const bf16x8*>(lb + n * 16 * ROW_BYTES + lane_off[kk]);
#pragma unroll
      for (int m = 0; m < 8; ++m)
        af[m] = *reinterpret_cast<const bf16x8*>(la + m * 16 * ROW_BYTES + lane_off[kk]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n], af[m], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // Epilogue: lane holds C[row = m*16 + (lane&15)][col = n*16 + 4*(lane>>4) + j], j = 0..3.
  const int row_base = tm * BM + wr * 128 + (lane & 15);
  const int col_base = tn * BN + wc * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    __bf16* crow = C + (size_t)(row_base + m * 16) * N + col_base;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 v;
      v[0] = (__bf16)acc[m][n][0];
      v[1] = (__bf16)acc[m][n][1];
      v[2] = (__bf16)acc[m][n][2];
      v[3] = (__bf16)acc[m][n][3];
      *reinterpret_cast<bf16x4*>(crow + n * 16) = v;
    }
  }
}

// v2: same tile/LDS image as v1, software-pipelined at the fragment level.
//   Two fragment register sets R0/R1 (k-steps kk=0/1 of a BK=64 tile). Per tile t:
//     issue ds_read (t,kk1)->R1 ; MFMA R0 ; [vmcnt(0) lgkmcnt(0) ; barrier]
//     issue LDS-DMA of tile t+2 into the buffer tile t used ; ds_read (t+1,kk0)->R0 ; MFMA R1
//   The single barrier per tile sits mid-tile: the next tile's first fragment reads are
//   in flight under the current tile's second MFMA cluster, and each LDS-DMA has a full
//   tile of MFMAs (64 per wave) to land. WAR on the refilled buffer is covered by the
//   lgkmcnt(0) + barrier (every wave's reads of tile t have completed).
__global__ void __launch_bounds__(NTHREADS)
gemm_bf16_256x256_v2(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                     __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2;
  const int wc = wid & 3;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;

  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * ROW_BYTES + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_off = wr * 128 * ROW_BYTES;
  const int b_off = PANEL_BYTES + wc * 64 * ROW_BYTES;

  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 a0[8], b0[4], a1[8], b1[4];
  auto read_frags = [&](const char* buf, int kk, bf16x8 (&af)[8], bf16x8 (&bfr)[4]) {
#pragma unroll
    for (int n = 0; n < 4; ++n)
      bfr[n] = *reinterpret_cast<const bf16x8*>(buf + b_off + n * 16 * ROW_BYTES + lane_off[kk]);
#pragma unroll
    for (int m = 0; m < 8; ++m)
      af[m] = *reinterpret_cast<const bf16x8*>(buf + a_off + m * 16 * ROW_BYTES + lane_off[kk]);
  };
  auto mfma_all = [&](const bf16x8 (&af)[8], const bf16x8 (&bfr)[4]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[n], af[m], acc[m][n], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int ktiles = K / BK;

  // prologue: tile 0 resident, tile 1 in flight, (0,kk0) fragments loaded
  stage_panel(gA, K, 0, smem, wid, lane);
  stage_panel(gB, K, 0, smem + PANEL_BYTES, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (ktiles > 1) {
    stage_panel(gA, K, BK, smem + BUF_BYTES, wid, lane);
    stage_panel(gB, K, BK, smem + BUF_BYTES + PANEL_BYTES, wid, lane);
  }
  read_frags(smem, 0, a0, b0);

  for (int t = 0; t < ktiles; ++t) {
    char* cur = smem + (t & 1) * BUF_BYTES;
    char* nxt = smem + ((t + 1) & 1) * BUF_BYTES;
    read_frags(cur, 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_all(a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + 2 < ktiles) {
      stage_panel(gA, K, (t + 2) * BK, cur, wid, lane);
      stage_panel(gB, K, (t + 2) * BK, cur + PANEL_BYTES, wid, lane);
    }
    if (t + 1 < ktiles) read_frags(nxt, 0, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mfma_all(a1, b1);
    __builtin_amdgcn_sched_barrier(0);
  }

  const int row_base = tm * BM + wr * 128 + (lane & 15);
  const int col_base = tn * BN + wc * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    __bf16* crow = C + (size_t)(row_base + m * 16) * N + col_base;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 v;
      v[0] = (__bf16)acc[m][n][0];
      v[1] = (__bf16)acc[m][n][1];
      v[2] = (__bf16)acc[m][n][2];
      v[3] = (__bf16)acc[m][n][3];
      *reinterpret_cast<bf16x4*>(crow + n * 16) = v;
    }
  }
}

// v3: ping-pong schedule. Same 256x256x64 tile, 8 waves (2 groups of 4: one wave of each
// group per SIMD), but the LDS image is cut into four 16 KiB half-tiles per K-tile that line
// up with the waves' register quadrants:
//     A_lo = A rows {0-63, 128-191}   A_hi = A rows {64-127, 192-255}
//     B_lo = Bt rows {64w+0..31}      B_hi = Bt rows {64w+32..63}      (w = 0..3)
// A K-tile is 4 phases, one output quadrant (4x2 fragments x K=64 = 16 MFMAs) each:
//     P1 (lo,lo) reads A_lo+B_lo, P2 (lo,hi) reads B_hi, P3 (hi,hi) reads A_hi, P4 (hi,lo)
//     reads nothing (B_lo kept in registers) — 24 ds_read_b128 per K-tile, the minimum.
// Each phase: [ds_reads ; one half-tile of LDS-DMA prefetch] s_barrier [MFMA x16] s_barrier.
// Group 1 runs one barrier behind group 0, so on every SIMD one wave issues MFMAs while the
// other issues its reads and DMA: the matrix pipe never waits on LDS latency.
// Two K-tile buffers (even/odd) = 128 KiB; a half-tile is restaged >= 2 phases after its last
// read, and vmcnt(4) (two half-tiles in flight, never 0 in the steady loop) at P4/P8 retires
// the buffer the next four phases read. See docs/validator-gemm.md for the full table.
constexpr int HALF_BYTES = 128 * ROW_BYTES;   // 16 KiB
constexpr int HB_A_LO = 0, HB_A_HI = HALF_BYTES, HB_B_LO = 2 * HALF_BYTES, HB_B_HI = 3 * HALF_BYTES;

// LDS row r (0..127) of a half-tile -> row of the 256-row global panel.
__device__ __forceinline__ int a_half_row(int r, int hi) { return (r & 63) + ((r >> 6) << 7) + (hi << 6); }
__device__ __forceinline__ int b_half_row(int r, int hi) { return (r & 31) + ((r >> 5) << 6) + (hi << 5); }

template <bool IS_A>
__device__ __forceinline__ void stage_half(const __bf16* __restrict__ g, int ld, int k0, char* lds_half,
                                           int hi, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rblk = i * 8 + wid;            // 8-row block 0..15
    const int r = rblk * 8 + (lane >> 3);    // LDS row 0..127
    const int pc = lane & 7;
    const int c = pc ^ ((r >> 1) & 7);
    const int gr = IS_A ? a_half_row(r, hi) : b_half_row(r, hi);
    const __bf16* src = g + (size_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds_half + rblk * 1024), 16, 0, 0);
  }
}

// BUF=true (v4): the half-tile DMA is `buffer_load_dwordx4 ... lds` with a per-lane voffset fixed
// for the whole kernel and the K offset in an SGPR — no per-load 64-bit VALU address math.
// EPI_LDS (v5): the epilogue goes through LDS (the K loop's buffers are free by then): each wave
// writes its bf16 128x64 sub-tile with ds_write_b64 (8-byte granules XOR-swizzled by row so the
// 16 rows a lane group writes hit distinct banks), then every thread stores whole 16-byte
// chunks, 32 lanes per 512-byte output row — fully coalesced global_store_dwordx4.
// PH = 4: four 16-MFMA phases per K-tile (v3-v5). PH = 2 (v6): two 32-MFMA phases per K-tile
// (P_a: A_lo x {B_lo,B_hi}, reads A_lo+B_lo+B_hi; P_b: A_hi x {B_hi,B_lo}, reads A_hi), halving
// the group hand-offs. Staging: {A_lo,B_lo,B_hi} of a buffer 2 phases after their read, A_hi
// likewise; every phase ends with a counted vmcnt (2 or 6) retiring what the next phase reads.
// KNOB (A/B experiments on the PH=4 schedule): 1 = no s_setprio around the MFMA blocks,
// 2 = issue each phase's half-tile DMA before its ds_reads.
template <bool BUF, bool EPI_LDS, int PH = 4, int KNOB = 0>
__global__ void __launch_bounds__(NTHREADS)
gemm_bf16_256x256_pp(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                     __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 2;   // group: 0 or 1 (also the 128-row half of the output tile)
  const int wc = wid & 3;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  // per-lane byte offsets inside the panel: [A/B][hi][i]
  uint32_t voff[2][2][2];
#pragma unroll
  for (int ab = 0; ab < 2; ++ab)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = (i * 8 + wid) * 8 + (lane >> 3);
        const int c = (lane & 7) ^ ((r >> 1) & 7);
        const int gr = ab == 0 ? a_half_row(r, hi) : b_half_row(r, hi);
        voff[ab][hi][i] = (uint32_t)gr * (uint32_t)K * 2u + (uint32_t)c * 16u;
      }
  auto stage = [&](int ab, int hi, int k0, char* lds_half) {
    if constexpr (BUF) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ab == 0 ? rA : rB, (lds_void*)(lds_half + (i * 8 + wid) * 1024), 16,
                                                 voff[ab][hi][i], k0 * 2, 0, 0);
    } else {
      if (ab == 0) stage_half<true>(gA, K, k0, lds_half, hi, wid, lane);
      else stage_half<false>(gB, K, k0, lds_half, hi, wid, lane);
    }
  };

  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * ROW_BYTES + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_off = wr * 64 * ROW_BYTES;   // this wave's 64 rows inside A_lo / A_hi
  const int b_off = wc * 32 * ROW_BYTES;   // this wave's 32 rows inside B_lo / B_hi

  f32x4 acc[8][4];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  bf16x8 af[4][2];        // A quadrant: 4 fragments x 2 k-steps
  bf16x8 bq[2][2][2];     // B: [lo/hi][2 fragments][2 k-steps]

  auto read_a = [&](const char* half) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        af[m][kk] = *reinterpret_cast<const bf16x8*>(half + a_off + m * 16 * ROW_BYTES + lane_off[kk]);
  };
  auto read_b = [&](const char* half, int q) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int n = 0; n < 2; ++n)
        bq[q][n][kk] = *reinterpret_cast<const bf16x8*>(half + b_off + n * 16 * ROW_BYTES + lane_off[kk]);
  };
  auto mfma_q = [&](int qm, int qn) {
    if constexpr (KNOB != 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[qm * 4 + m][qn * 2 + n] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[qn][n][kk], af[m][kk], acc[qm * 4 + m][qn * 2 + n], 0, 0, 0);
    if constexpr (KNOB != 1) __builtin_amdgcn_s_setprio(0);
  };

  const int ktiles = K / BK;            // even (host guarantees K % 128 == 0)
  char* const E = smem;
  char* const O = smem + BUF_BYTES;

  if constexpr (PH == 2) {
    stage(0, 0, 0, E + HB_A_LO);
    stage(0, 1, 0, E + HB_A_HI);
    stage(1, 0, 0, E + HB_B_LO);
    stage(1, 1, 0, E + HB_B_HI);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();
    if (wr == 1) bar();
    for (int t = 0; t < ktiles; t += 2) {
      const bool more = t + 2 < ktiles;
      const int k1 = (t + 1) * BK, k2 = (t + 2) * BK;
      // P1: tile t (even), A_lo x {B_lo, B_hi}; stage odd {A_lo, B_lo, B_hi} <- t+1
      read_b(E + HB_B_LO, 0);
      read_b(E + HB_B_HI, 1);
      __builtin_amdgcn_sched_barrier(0);
      read_a(E + HB_A_LO);
      stage(0, 0, k1, O + HB_A_LO);
      stage(1, 0, k1, O + HB_B_LO);
      stage(1, 1, k1, O + HB_B_HI);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      bar();
      mfma_q(0, 0);
      mfma_q(0, 1);
      bar();
      // P2: A_hi x {B_hi, B_lo}; stage odd A_hi <- t+1
      read_a(E + HB_A_HI);
      stage(0, 1, k1, O + HB_A_HI);
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      bar();
      mfma_q(1, 1);
      mfma_q(1, 0);
      bar();
      // P3: tile t+1 (odd); stage even {A_lo, B_lo, B_hi} <- t+2
      read_b(O + HB_B_LO, 0);
      read_b(O + HB_B_HI, 1);
      __builtin_amdgcn_sched_barrier(0);
      read_a(O + HB_A_LO);
      if (more) {
        stage(0, 0, k2, E + HB_A_LO);
        stage(1, 0, k2, E + HB_B_LO);
        stage(1, 1, k2, E + HB_B_HI);
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      bar();
      mfma_q(0, 0);
      mfma_q(0, 1);
      bar();
      // P4: stage even A_hi <- t+2
      read_a(O + HB_A_HI);
      if (more) {
        stage(0, 1, k2, E + HB_A_HI);
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      }
      bar();
      mfma_q(1, 1);
      mfma_q(1, 0);
      bar();
    }
  } else if constexpr (PH == 8) {
    // v7: v5's phases and staging order, but a counted wait before every phase that reads
    // (vmcnt(8): four half-tiles in flight instead of two) — every half-tile gets >= 4
    // phases between its DMA issue and the wait that retires it.
#define VMWAIT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
    stage(0, 0, 0, E + HB_A_LO);
    stage(1, 0, 0, E + HB_B_LO);
    stage(1, 1, 0, E + HB_B_HI);
    stage(0, 1, 0, E + HB_A_HI);
    stage(0, 0, BK, O + HB_A_LO);
    stage(1, 0, BK, O + HB_B_LO);
    VMWAIT(8);
    bar();
    if (wr == 1) bar();
    for (int t = 0; t < ktiles; t += 2) {
      const bool more = t + 2 < ktiles;
      const int k1 = (t + 1) * BK, k2 = (t + 2) * BK, k3 = (t + 3) * BK;
      // P1
      read_b(E + HB_B_LO, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(E + HB_A_LO);
      stage(1, 1, k1, O + HB_B_HI);
      VMWAIT(8);
      bar();
      mfma_q(0, 0);
      bar();
      // P2
      read_b(E + HB_B_HI, 1);
      stage(0, 1, k1, O + HB_A_HI);
      VMWAIT(8);
      bar();
      mfma_q(0, 1);
      bar();
      // P3
      read_a(E + HB_A_HI);
      if (more) stage(0, 0, k2, E + HB_A_LO);
      bar();
      mfma_q(1, 1);
      bar();
      // P4
      if (more) {
        stage(1, 0, k2, E + HB_B_LO);
        VMWAIT(8);
      } else {
        VMWAIT(4);
      }
      bar();
      mfma_q(1, 0);
      bar();
      // P5
      read_b(O + HB_B_LO, 0);
      __builtin_amdgcn_sched_barrier(0);
      read_a(O + HB_A_LO);
      if (more) {
        stage(1, 1, k2, E + HB_B_HI);
        VMWAIT(8);
      } else {
        VMWAIT(2);
      }
      bar();
      mfma_q(0, 0);
      bar();
      // P6
      read_b(O + HB_B_HI, 1);
      if (more) {
        stage(0, 1, k2, E + HB_A_HI);
        VMWAIT(8);
      } else {
        VMWAIT(0);
      }
      bar();
      mfma_q(0, 1);
      bar();
      // P7
      read_a(O + HB_A_HI);
      if (more) stage(0, 0, k3, O + HB_A_LO);
      bar();
      mfma_q(1, 1);
      bar();
      // P8
      if (more) {
        stage(1, 0, k3, O + HB_B_LO);
        VMWAIT(8);
      }
      bar();
      mfma_q(1, 0);
      bar();
    }
#undef VMWAIT
  } else if constexpr (KNOB == 2) {
  // prologue: even buffer <- tile 0 (complete), odd A_lo/B_lo <- tile 1 (in flight)
  stage(0, 0, 0, E + HB_A_LO);
  stage(0, 1, 0, E + HB_A_HI);
  stage(1, 0, 0, E + HB_B_LO);
  stage(1, 1, 0, E + HB_B_HI);
  stage(0, 0, BK, O + HB_A_LO);
  stage(1, 0, BK, O + HB_B_LO);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bar();
  if (wr == 1) bar();   // stagger: group 1 runs one barrier behind group 0

  for (int t = 0; t < ktiles; t += 2) {
    const bool more = t + 2 < ktiles;
    const int k1 = (t + 1) * BK, k2 = (t + 2) * BK, k3 = (t + 3) * BK;
    // ---- even buffer (tile t) ----
    // P1
    stage(1, 1, k1, O + HB_B_HI);
    read_b(E + HB_B_LO, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(E + HB_A_LO);
    bar();
    mfma_q(0, 0);
    bar();
    // P2
    stage(0, 1, k1, O + HB_A_HI);
    read_b(E + HB_B_HI, 1);
    bar();
    mfma_q(0, 1);
    bar();
    // P3
    if (more) stage(0, 0, k2, E + HB_A_LO);
    read_a(E + HB_A_HI);
    bar();
    mfma_q(1, 1);
    bar();
    // P4
    if (more) {
      stage(1, 0, k2, E + HB_B_LO);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    mfma_q(1, 0);
    bar();
    // ---- odd buffer (tile t+1) ----
    // P5
    if (more) stage(1, 1, k2, E + HB_B_HI);
    read_b(O + HB_B_LO, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(O + HB_A_LO);
    bar();
    mfma_q(0, 0);
    bar();
    // P6
    if (more) stage(0, 1, k2, E + HB_A_HI);
    read_b(O + HB_B_HI, 1);
    bar();
    mfma_q(0, 1);
    bar();
    // P7
    if (more) stage(0, 0, k3, O + HB_A_LO);
    read_a(O + HB_A_HI);
    bar();
    mfma_q(1, 1);
    bar();
    // P8
    if (more) {
      stage(1, 0, k3, O + HB_B_LO);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    bar();
    mfma_q(1, 0);
    bar();
  }
  } else {
  // prologue: even buffer <- tile 0 (complete), odd A_lo/B_lo <- tile 1 (in flight)
  stage(0, 0, 0, E + HB_A_LO);
  stage(0, 1, 0, E + HB_A_HI);
  stage(1, 0, 0, E + HB_B_LO);
  stage(1, 1, 0, E + HB_B_HI);
  stage(0, 0, BK, O + HB_A_LO);
  stage(1, 0, BK, O + HB_B_LO);
  asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  bar();
  if (wr == 1) bar();   // stagger: group 1 runs one barrier behind group 0

  for (int t = 0; t < ktiles; t += 2) {
    const bool more = t + 2 < ktiles;
    const int k1 = (t + 1) * BK, k2 = (t + 2) * BK, k3 = (t + 3) * BK;
    // ---- even buffer (tile t) ----
    // P1
    read_b(E + HB_B_LO, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(E + HB_A_LO);
    stage(1, 1, k1, O + HB_B_HI);
    bar();
    mfma_q(0, 0);
    bar();
    // P2
    read_b(E + HB_B_HI, 1);
    stage(0, 1, k1, O + HB_A_HI);
    bar();
    mfma_q(0, 1);
    bar();
    // P3
    read_a(E + HB_A_HI);
    if (more) stage(0, 0, k2, E + HB_A_LO);
    bar();
    mfma_q(1, 1);
    bar();
    // P4
    if (more) {
      stage(1, 0, k2, E + HB_B_LO);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    bar();
    mfma_q(1, 0);
    bar();
    // ---- odd buffer (tile t+1) ----
    // P5
    read_b(O + HB_B_LO, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(O + HB_A_LO);
    if (more) stage(1, 1, k2, E + HB_B_HI);
    bar();
    mfma_q(0, 0);
    bar();
    // P6
    read_b(O + HB_B_HI, 1);
    if (more) stage(0, 1, k2, E + HB_A_HI);
    bar();
    mfma_q(0, 1);
    bar();
    // P7
    read_a(O + HB_A_HI);
    if (more) stage(0, 0, k3, O + HB_A_LO);
    bar();
    mfma_q(1, 1);
    bar();
    // P8
    if (more) {
      stage(1, 0, k3, O + HB_B_LO);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    bar();
    mfma_q(1, 0);
    bar();
  }
  }  // PH
  if (wr == 0) bar();   // re-align the groups' barrier counts

  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  if constexpr (EPI_LDS) {
    bar();                // every wave is past its last ds_read of the K loop
    constexpr int CROW = BN * 2;                     // 512-byte LDS row
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int r = wr * 128 + m * 16 + (lane & 15);
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int g = (wc * 64 + n * 16 + 4 * (lane >> 4)) >> 2;   // 8-byte granule 0..63
        bf16x4 v;
        v[0] = (__bf16)acc[m][n][0];
        v[1] = (__bf16)acc[m][n][1];
        v[2] = (__bf16)acc[m][n][2];
        v[3] = (__bf16)acc[m][n][3];
        *reinterpret_cast<bf16x4*>(smem + r * CROW + ((g ^ (r & 15)) << 3)) = v;
      }
    }
    bar();
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < (BM * BN * 2) / (NTHREADS * 16); ++i) {      // 16 chunks per thread
      const int r = i * (NTHREADS / 32) + (tid >> 5);
      const int ch = tid & 31;                                        // 16-byte chunk in the row
      const int s = r & 15;
      const int pg = (2 * ch) ^ s;                                    // physical granule of the even half
      const uint4 raw = *reinterpret_cast<const uint4*>(smem + r * CROW + ((pg & ~1) << 3));
      uint4 v = raw;
      if (s & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
      *reinterpret_cast<uint4*>(C + (size_t)(tm * BM + r) * N + tn * BN + ch * 8) = v;
    }
    return;
  }

  const int row_base = tm * BM + wr * 128 + (lane & 15);
  const int col_base = tn * BN + wc * 64 + 4 * (lane >> 4);
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    __bf16* crow = C + (size_t)(row_base + m * 16) * N + col_base;
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      bf16x4 v;
      v[0] = (__bf16)acc[m][n][0];
      v[1] = (__bf16)acc[m][n][1];
      v[2] = (__bf16)acc[m][n][2];
      v[3] = (__bf16)acc[m][n][3];
      *reinterpret_cast<bf16x4*>(crow + n * 16) = v;
    }
  }
}

// v10: one wave per SIMD. 4 waves (2x2), each owning a 128x128 sub-tile: 8x8 MFMA 16x16x32
// accumulators = the wave's 256 AGPRs; its fragments (2 x 16 x bf16x8 = 128 VGPRs) and addresses
// fit the 256 VGPRs. A 128x128 wave tile halves the LDS bytes per MFMA against v5's 128x64
// (256 B vs 384 B): per K-tile the CU reads 128 KiB of fragments + 64 KiB of DMA writes in 2048
// MFMA cycles (96 B/clk of LDS's 128) where v5 needed 128 B/clk, i.e. sat on the LDS port.
// Each SIMD's matrix pipe is fed by its single wave, which interleaves its own LDS fragment reads
// (1 ds_read_b128 per 4 MFMAs) and LDS-DMA pieces (1 per 4 MFMAs) into the MFMA stream. Per K-tile:
//   block(t, kk0): MFMA with R0, read R1 <- frags(t, kk1)
//   wait lgkmcnt(0) + vmcnt(0) (tile t+1 landed) ; barrier (tile t fully read by every wave)
//   block(t, kk1): MFMA with R1, read R0 <- frags(t+1, kk0), DMA tile t+2 into tile t's buffer
// One barrier per K-tile; the DMA of a tile has a full K-tile (128 MFMAs) to land.
//
template <int RSPAN = 16, int DSPAN = 16, int KO = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                     __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  // wave w issues pieces p = 4i + w (A row blocks 0..31, then B); every piece it issues has
  // row-block parity w & 1, so one per-lane voffset serves all of them.
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K * 2u +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, int k0, char* buf) {
    const int p = i * 4 + wid;                     // 0..63
    const int rblk = p & 31;
    char* lds = buf + (p >= 32 ? PANEL_BYTES : 0) + rblk * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(p >= 32 ? rB : rA, (lds_void*)lds, 16, voff,
                                             (uint32_t)rblk * 8u * (uint32_t)K * 2u + (uint32_t)k0 * 2u, 0, 0);
  };

  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * ROW_BYTES + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_off = wr * 128 * ROW_BYTES;
  const int b_off = PANEL_BYTES + wc * 128 * ROW_BYTES;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  W4Frags R0, R1;
  char* const buf0 = smem;
  char* const buf1 = smem + BUF_BYTES;

  auto read_frag = [&](W4Frags& F, const char* buf, int kk, auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int x = w4_idx(j);
    if constexpr (w4_isb(j))
      F.b[x] = *reinterpret_cast<const bf16x8*>(buf + b_off + x * 16 * ROW_BYTES + lane_off[kk]);
    else
      F.a[x] = *reinterpret_cast<const bf16x8*>(buf + a_off + x * 16 * ROW_BYTES + lane_off[kk]);
  };
  // 64 MFMAs with Fc; optionally 16 fragment reads into Fn (from nbuf, step nkk) and 16 DMA
  // pieces (tile at column dk into dbuf) placed after groups of 4 MFMAs; sched_barrier pins it.
  auto block = [&](const W4Frags& Fc, W4Frags& Fn, const char* nbuf, int nkk, auto RD, char* dbuf, int dk,
                   auto DM) {
    static_for<0, 16>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      static_for<0, 4>([&](auto U) {
        constexpr int i = q * 4 + decltype(U)::value;
        w4_mfma<i>(Fc.b[i & 7], Fc.a[i >> 3]);
      });
      // the reads / pieces j with j*SPAN/16 == q: a contiguous range, instantiated alone
      if constexpr (decltype(RD)::value && !(KO & 4))
        static_for<lab_span_lo(q, RSPAN, 16), lab_span_lo(q + 1, RSPAN, 16)>([&](auto J) { read_frag(Fn, nbuf, nkk, J); });
      if constexpr (decltype(DM)::value && !(KO & 2))
        static_for<lab_span_lo(q, DSPAN, 16), lab_span_lo(q + 1, DSPAN, 16)>([&](auto J) {
          dma_piece(decltype(J)::value, dk, dbuf);
        });
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  auto sync_tile = [&]() {
    if constexpr (!(KO & 1)) {
      __builtin_amdgcn_s_waitcnt(0x0070);           // vmcnt(0) lgkmcnt(0), visible to hipcc's counters
      bar();
    }
  };

  const int ktiles = K / BK;        // >= 2 (host guarantees)
  // prologue: tile 0 -> buf0 (waited), tile 1 -> buf1 (in flight), R0 <- (0, kk0)
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, 0, buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, BK, buf1);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): tile 0 landed, tile 1 in flight
  bar();
  static_for<0, 16>([&](auto J) { read_frag(R0, buf0, 0, J); });

  char* cur = buf0;
  char* nxt = buf1;
  for (int t = 0; t < ktiles - 2; ++t) {
    block(R0, R1, cur, 1, T_{}, nullptr, 0, F_{});
    sync_tile();
    block(R1, R0, nxt, 0, T_{}, cur, (t + 2) * BK, T_{});
    char* tmp = cur; cur = nxt; nxt = tmp;
  }
  // second-to-last tile: prefetch fragments, no DMA; then the last tile
  block(R0, R1, cur, 1, T_{}, nullptr, 0, F_{});
  sync_tile();
  block(R1, R0, nxt, 0, T_{}, nullptr, 0, F_{});
  block(R0, R1, nxt, 1, T_{}, nullptr, 0, F_{});
  block(R1, R0, nullptr, 0, F_{}, nullptr, 0, F_{});

  // epilogue through LDS (every wave is past its last ds_read once all reach this barrier);
  // pad the last MFMA's D before the accumulator reads.
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  bar();
  constexpr int CROW = BN * 2;
  static_for<0, 64>([&](auto I) {
    constexpr int i = decltype(I)::value;
    constexpr int m = i >> 3, n = i & 7;
    float x0, x1, x2, x3;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                 "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                 : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                 : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
    const int r = wr * 128 + m * 16 + (lane & 15);
    const int g = (wc * 128 + n * 16 + 4 * (lane >> 4)) >> 2;
    bf16x4 v;
    v[0] = (__bf16)x0;
    v[1] = (__bf16)x1;
    v[2] = (__bf16)x2;
    v[3] = (__bf16)x3;
    *reinterpret_cast<bf16x4*>(smem + r * CROW + ((g ^ (r & 15)) << 3)) = v;
  });
  bar();
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < (BM * BN * 2) / (W4_THREADS * 16); ++i) {      // 32 chunks per thread
    const int r = i * (W4_THREADS / 32) + (tid >> 5);
    const int ch = tid & 31;
    const int sw = r & 15;
    const int pg = (2 * ch) ^ sw;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + r * CROW + ((pg & ~1) << 3));
    uint4 v = raw;
    if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
    *reinterpret_cast<uint4*>(C + (size_t)(tm * BM + r) * N + tn * BN + ch * 8) = v;
  }
}
// v15: v10's wave layout over a 5-slot ring of K-half-tiles (32 k-columns: A 16 KiB + B 16 KiB
// per slot = all 160 KiB of LDS). v10 syncs once per K-tile but the DMA it waits for was issued
// only one 64-MFMA block earlier (~1000 cycles: less than a loaded L2-miss round trip). Here block
// h (64 MFMAs on half h) reads the fragments of half h+1 and DMAs half h+4 into the slot of half
// h-1; its closing barrier needs half h+2, issued two blocks earlier (vmcnt(16): halves h+3, h+4
// stay in flight). One barrier per 64 MFMAs instead of per 128.
// Slot layout: 256 rows x 64 B per operand, 16-B chunk c of row r at ((c ^ ((r >> 2) & 3)) << 4):
// the 16 lanes of a ds_read_b128 phase (16 rows, one chunk) cover all 64 banks. LDS-DMA writes a
// 1-KiB piece (16 rows) lane-contiguous, so each lane fetches the global chunk its LDS slot holds.
constexpr int RH_ROW = 64;                          // bytes per row per half
constexpr int RH_OP = BM * RH_ROW;                  // 16 KiB per operand per half
constexpr int RH_SLOT = 2 * RH_OP;                  // 32 KiB
constexpr int RH_NSLOT = 5;                         // 160 KiB

template <int RSPAN = 12, int DSPAN = 8>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4r(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[RH_NSLOT * RH_SLOT];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  // piece = 16 rows x 64 B; lane L -> row L>>2, LDS chunk L&3 holding global chunk (L&3)^((L>>4)&3)
  const uint32_t voff = (uint32_t)(lane >> 2) * (uint32_t)K * 2u +
                        (uint32_t)(((lane & 3) ^ ((lane >> 4) & 3)) * 16);
  // half h: 32 pieces (A row blocks 0..15, B 0..15); wave w issues p = 4i + w, i = 0..7
  // slot indices are carried incrementally (sl = h mod 5): no division in the loop
  auto m5 = [](int x) { return x >= RH_NSLOT ? x - RH_NSLOT : x; };
  auto dma_piece = [&](int i, int h, int sl) {
    const int p = i * 4 + wid;
    const int rblk = p & 15;
    char* lds = smem + sl * RH_SLOT + (p >= 16 ? RH_OP : 0) + rblk * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(p >= 16 ? rB : rA, (lds_void*)lds, 16, voff,
                                             (uint32_t)rblk * 16u * (uint32_t)K * 2u + (uint32_t)h * 64u, 0, 0);
  };
  const int r16 = lane & 15;
  const int lane_off = r16 * RH_ROW + (((lane >> 4) ^ ((r16 >> 2) & 3)) << 4);
  const int a_off = wr * 128 * RH_ROW + lane_off;
  const int b_off = RH_OP + wc * 128 * RH_ROW + lane_off;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  W4Frags R0, R1;
  auto read_frag = [&](W4Frags& F, int sl, auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int x = w4_idx(j);
    const char* slot = smem + sl * RH_SLOT;
    if constexpr (w4_isb(j))
      F.b[x] = *reinterpret_cast<const bf16x8*>(slot + b_off + x * 16 * RH_ROW);
    else
      F.a[x] = *reinterpret_cast<const bf16x8*>(slot + a_off + x * 16 * RH_ROW);
  };
  // one block: 64 MFMAs on Fc; reads from slot rs into Fn; DMA of half dh into slot ds
  auto block = [&](const W4Frags& Fc, W4Frags& Fn, int rs, auto RD, int dh, int ds, auto DM) {
    static_for<0, 16>([&](auto Q) {
      constexpr int q = decltype(Q)::value;
      static_for<0, 4>([&](auto U) {
        constexpr int i = q * 4 + decltype(U)::value;
        w4_mfma<i>(Fc.b[i & 7], Fc.a[i >> 3]);
      });
      if constexpr (decltype(RD)::value)
        static_for<lab_span_lo(q, RSPAN, 16), lab_span_lo(q + 1, RSPAN, 16)>([&](auto J) { read_frag(Fn, rs, J); });
      if constexpr (decltype(DM)::value)
        static_for<lab_span_lo(q, DSPAN, 8), lab_span_lo(q + 1, DSPAN, 8)>([&](auto J) {
          dma_piece(decltype(J)::value, dh, ds);
        });
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int H = K / 32;             // >= 4 (host guarantees K >= 128)
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) dma_piece(i, h, h);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): halves 0, 1 landed
  bar();
  static_for<0, 16>([&](auto J) { read_frag(R0, 0, J); });

  // steady state, two halves per trip so R0/R1 keep their roles
  int h = 0, sl = 0;
  for (; h + 5 < H; h += 2, sl = m5(sl + 2)) {
    block(R0, R1, m5(sl + 1), T_{}, h + 4, m5(sl + 4), T_{});
    __builtin_amdgcn_s_waitcnt(0x4070);             // vmcnt(16) lgkmcnt(0): half h+2 landed
    bar();
    block(R1, R0, m5(sl + 2), T_{}, h + 5, sl, T_{});
    __builtin_amdgcn_s_waitcnt(0x4070);             // half h+3 landed
    bar();
  }
  // H is even, so exactly 4 halves are left: h .. H-1
  block(R0, R1, m5(sl + 1), T_{}, 0, 0, F_{});
  __builtin_amdgcn_s_waitcnt(0x0078);             // vmcnt(8): half h+2 landed, h+3 in flight
  bar();
  block(R1, R0, m5(sl + 2), T_{}, 0, 0, F_{});
  __builtin_amdgcn_s_waitcnt(0x0070);             // vmcnt(0): half h+3 landed
  bar();
  block(R0, R1, m5(sl + 3), T_{}, 0, 0, F_{});
  block(R1, R0, 0, F_{}, 0, 0, F_{});

  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  bar();
  constexpr int CROW = BN * 2;
  static_for<0, 64>([&](auto I) {
    constexpr int i = decltype(I)::value;
    constexpr int m = i >> 3, n = i & 7;
    float x0, x1, x2, x3;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                 "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                 : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                 : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
    const int r = wr * 128 + m * 16 + (lane & 15);
    const int g = (wc * 128 + n * 16 + 4 * (lane >> 4)) >> 2;
    bf16x4 v;
    v[0] = (__bf16)x0;
    v[1] = (__bf16)x1;
    v[2] = (__bf16)x2;
    v[3] = (__bf16)x3;
    *reinterpret_cast<bf16x4*>(smem + r * CROW + ((g ^ (r & 15)) << 3)) = v;
  });
  bar();
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < (BM * BN * 2) / (W4_THREADS * 16); ++i) {
    const int r = i * (W4_THREADS / 32) + (tid >> 5);
    const int ch = tid & 31;
    const int sw = r & 15;
    const int pg = (2 * ch) ^ sw;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + r * CROW + ((pg & ~1) << 3));
    uint4 v = raw;
    if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
    *reinterpret_cast<uint4*>(C + (size_t)(tm * BM + r) * N + tn * BN + ch * 8) = v;
  }
}
}  // namespace

extern "C" {

// Returns 0 on success, a hipError_t value otherwise (hipErrorInvalidValue for a variant or a shape
// the variant cannot run). No automatic switches: the lab runs exactly what it is asked.
int amdgo_lab_gemm_bf16(int v, const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int nwg = (M / BM) * (N / BN);
  const auto* a = (const __bf16*)A;
  const auto* b = (const __bf16*)Bt;
  auto* c = (__bf16*)C;
  const bool k2 = K % (2 * BK) == 0, kk = K >= 2 * BK;
  const int cus = device_cu_count();
  const int pgrid = ((nwg < cus ? nwg : cus) / NXCD) * NXCD;
  if (v == 1)
    hipLaunchKernelGGL(gemm_bf16_256x256, dim3(nwg), dim3(NTHREADS), 0, s, a, b, c, M, N, K);
  else if (v == 2)
    hipLaunchKernelGGL(gemm_bf16_256x256_v2, dim3(nwg), dim3(NTHREADS), 0, s, a, b, c, M, N, K);
  else if (v >= 3 && v <= 9 && k2) {
    auto kern = v == 3 ? gemm_bf16_256x256_pp<false, false>
              : v == 4 ? gemm_bf16_256x256_pp<true, false>
              : v == 5 ? gemm_bf16_256x256_pp<true, true>
              : v == 6 ? gemm_bf16_256x256_pp<true, true, 2>
              : v == 7 ? gemm_bf16_256x256_pp<true, true, 8>
              : v == 8 ? gemm_bf16_256x256_pp<true, true, 4, 1>
                       : gemm_bf16_256x256_pp<true, true, 4, 2>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(NTHREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 10 && v <= 14 && kk) {
    auto kern = v == 10 ? gemm_bf16_256x256_w4<16, 16>
              : v == 11 ? gemm_bf16_256x256_w4<12, 16>
              : v == 12 ? gemm_bf16_256x256_w4<12, 8>
              : v == 13 ? gemm_bf16_256x256_w4<8, 8>
                        : gemm_bf16_256x256_w4<12, 4>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 15 && v <= 17 && kk) {
    auto kern = v == 15 ? gemm_bf16_256x256_w4r<12, 8>
              : v == 16 ? gemm_bf16_256x256_w4r<16, 16>
                        : gemm_bf16_256x256_w4r<12, 4>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if ((v == 18 || v == 19) && kk) {
    auto kern = v == 18 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40> : gemm_bf16_256x256_w4s<17, 19, 4, 72, 48>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 20 && v <= 24 && kk) {            // knock-out timings (WRONG results by design)
    auto kern = v == 20 ? gemm_bf16_256x256_w4<16, 16, 1>
              : v == 21 ? gemm_bf16_256x256_w4<16, 16, 2>
              : v == 22 ? gemm_bf16_256x256_w4<16, 16, 4>
              : v == 23 ? gemm_bf16_256x256_w4<16, 16, 7>
                        : gemm_bf16_256x256_w4<16, 16, 3>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 25 && v <= 27 && kk && pgrid >= NXCD) {
    auto kern = v == 25 ? gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40>
              : v == 26 ? gemm_bf16_256x256_w4sp<17, 19, 4, 72, 48>
                        : gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40, true>;
    hipLaunchKernelGGL(kern, dim3(pgrid), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 30 && v <= 35 && kk) {
    auto kern = v == 30 ? gemm_bf16_256x256_w4s<24, 26, 5, 80, 40>
              : v == 31 ? gemm_bf16_256x256_w4s<32, 34, 5, 80, 40>
              : v == 32 ? gemm_bf16_256x256_w4s<40, 42, 5, 96, 24>
              : v == 33 ? gemm_bf16_256x256_w4s<32, 34, 5, 96, 24>
              : v == 34 ? gemm_bf16_256x256_w4s<24, 26, 4, 72, 48>
                        : gemm_bf16_256x256_w4s<48, 50, 4, 100, 24>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 40 && v <= 44 && kk) {
    auto kern = v == 40 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32>
              : v == 41 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 64>
              : v == 42 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 0, true>
              : v == 43 ? gemm_bf16_256x256_w4s<17, 19, 4, 72, 48, 0, true>
                        : gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v == 45 && kk && (M / BM) % 16 == 0 && (N / BN) % 16 == 0) {
    hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true>), dim3(nwg), dim3(W4_THREADS),
                       0, s, a, b, c, M, N, K);
  } else if (v >= 90 && v <= 94 && kk) {            // v44 + VK (90); DMA spacing 6 / 7 slots (91-94)
    auto kern = v == 90 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true>
              : v == 91 ? gemm_bf16_256x256_w4s<17, 19, 6, 80, 40, 32, true, false, true>
              : v == 92 ? gemm_bf16_256x256_w4s<17, 19, 7, 80, 40, 32, true, false, true>
              : v == 93 ? gemm_bf16_256x256_w4s<17, 19, 6, 96, 24, 32, true, false, true>
                        : gemm_bf16_256x256_w4s<17, 18, 6, 64, 48, 32, true, false, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if ((v == 98 && kk && (M / BM) % 16 == 0 && (N / BN) % 16 == 0) || (v == 99 && kk)) {   // + PA
    auto kern = v == 98 ? gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true, true>
                        : gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if ((v == 70 || v == 71) && kk) {            // w4t, B-outer MFMA operand order
    auto kern = v == 70 ? gemm_bf16_256x256_w4t<W4SchedV18, 32, true, false, false, 0, true>
                        : gemm_bf16_256x256_w4t<W4SchedSplit, 32, true, false, false, 0, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 67 && v <= 69 && kk) {            // w4t v18 schedule + K-start stagger
    auto kern = v == 67 ? gemm_bf16_256x256_w4t<W4SchedV18, 0, true, false, false, 8>
              : v == 68 ? gemm_bf16_256x256_w4t<W4SchedV18, 32, true, false, false, 4>
                        : gemm_bf16_256x256_w4t<W4SchedV18, 0, true, false, false, 32>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if ((v == 65 || v == 66) && kk) {            // w4t + fused MFMA/LDS-DMA asm (no s_nop per piece)
    auto kern = v == 65 ? gemm_bf16_256x256_w4t<W4SchedV18, 32, true, false, true>
                        : gemm_bf16_256x256_w4t<W4SchedSplit, 32, true, false, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else if (v >= 60 && v <= 64 && kk) {            // w4t schedules, all with v44's serpentine K + rotation
    auto kern = v == 60 ? gemm_bf16_256x256_w4t<W4SchedV18, 32, true>
              : v == 61 ? gemm_bf16_256x256_w4t<W4SchedSplit, 32, true>
              : v == 62 ? gemm_bf16_256x256_w4t<W4SchedSpread, 32, true>
              : v == 63 ? gemm_bf16_256x256_w4t<W4SchedSplitEarly, 32, true>
                        : gemm_bf16_256x256_w4t<W4SchedSplitTight, 32, true>;
    hipLaunchKernelGGL(kern, dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// 1 if variant v produces correct results (everything except the knock-out timings 20-24).
int amdgo_lab_variant_is_exact(int v) { return !(v >= 20 && v <= 24); }

}  // extern "C"
