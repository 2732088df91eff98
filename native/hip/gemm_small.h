// gfx950 bf16 GEMM for small output grids (v60):
//
//   C[M,N] (bf16) = A[M,K] (bf16, K-major) * Bt[N,K]^T (bf16, K-major), fp32 accumulation.
//
// The 256x256 kernels own one output tile per CU: on a grid of 16 such tiles (1024^3) 16 of the 256
// CUs work and each runs a 134 MFLOP tile alone (~14 us at one CU's matrix rate), so the dispatch is
// bound by the per-CU MFMA time of a few CUs, not by the chip. This kernel cuts the work 4x finer:
//
//   * 128x128 output tile per 256-thread workgroup, 4 waves as 2x2, each wave a 64x64 sub-tile =
//     4x4 v_mfma_f32_16x16x32_bf16 accumulators (64 AGPRs);
//   * K-step 64: one K-tile of A and of B is 16 KiB each, in a ring of 3 LDS buffers (below);
//   * LDS rows of 128 B hold 8 16-B chunks XOR-swizzled by (row & 7): the ds_read_b128 fragment reads
//     (16 rows, one chunk column) spread over the banks -- 2-way at worst, the minimum for a 16-row
//     b128 read;
//   * XCD-aware tile order (bijective remap): the tiles one XCD runs are contiguous row-major, so
//     they share A row panels in that XCD's L2.
//
// Shapes: M % 128 == 0, N % 128 == 0, K % 64 == 0 (host checks). v60 runs the whole K per tile;
// v61 splits K over several workgroups per tile (below).
//
// (launch_bounds(256, 1): the 96 KiB ring admits one workgroup per CU.)
#pragma once

#include "gemm_tile_common.h"

constexpr int S_BM = 128, S_BN = 128, S_BK = 64, S_THREADS = 256;

typedef __bf16 s_bf16x8 __attribute__((ext_vector_type(8)));
typedef float s_floatx4 __attribute__((ext_vector_type(4)));

// byte offset of 16-B chunk q (0..7) of row r in a [rows][64] bf16 panel (128-B rows), swizzled
__device__ __forceinline__ int s_swz(int r, int q) { return r * 128 + ((q ^ (r & 7)) << 4); }

// The in-launch split-K combine (cdna_hip_programming.md "Projection GEMM at M = 256" item 2): every
// split stores its fp32 slab with plain 16-B stores, drains them, and after a workgroup barrier ONE
// lane releases at agent scope and draws a ticket from the tile's counter; the split that draws the
// last ticket acquires (one lane, agent scope) and sums ALL the tile's slabs in split order -- its own
// included, re-read -- so the result does not depend on which split finished last. Returns true in the
// reducing workgroup (acc then holds the full sum), false in the others. `flag` is LDS scratch.
template <class Acc>
__device__ __forceinline__ bool small_split_reduce(Acc& acc, float* __restrict__ ws, int* __restrict__ cnt, int item,
                                                   int tile, int splits, int tid, int* flag) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4* slab = (f4*)(ws + (size_t)item * (128 * 128));
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) slab[(i * 4 + j) * 256 + tid] = acc[i][j];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int ticket = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = ticket == splits - 1;
    if (ticket == splits - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!*flag) return false;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < splits; ++s) {
    const f4* part = (const f4*)(ws + ((size_t)tile * splits + s) * (128 * 128));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] += part[(i * 4 + j) * 256 + tid];
  }
  if (tid == 0) cnt[tile] = 0;   // ready for the next launch on this stream
  return true;
}

// Staging: LDS-DMA (global_load_lds_dwordx4): each wave-instruction writes 1 KiB (8 rows of 128 B)
// straight to LDS, lane-linear, so the XOR swizzle goes on the SOURCE address (lane L of a chunk loads
// global chunk (L & 7) ^ (L >> 3) of its row; the fragment reads use s_swz). A ring of 3 K-tile buffers
// (96 KiB) keeps two K-tiles in flight: at K-tile t a counted vmcnt retires tile t only, a raw s_barrier
// (no __syncthreads, whose fence would drain the DMA) publishes it, and the DMA of tile t + 2 goes into
// the buffer every wave finished reading at t - 1. The loads' latency hides under two K-tiles of MFMA
// work instead of one -- these grids have one workgroup per CU and no other wave to hide it. Against
// register staging (one tile ahead, ds_write_b128 pass) the same tile measured 1024^3 +6 %, 1536^3
// +9 %, 2048^3 +9 %, 2048^2x1024 +8 % (profiles/r5_small/sweep_v62.jsonl).
//
// SPLIT (v61): split-K for grids far below the chip. The grid is tiles x `splits` workgroups; item
// (tile, s) runs K-tiles [s nk / splits, (s + 1) nk / splits), stores its fp32 partial (thread-major
// float4s: one coalesced KiB per wave and accumulator) and the last split of the tile sums them
// (small_split_reduce) and writes the bf16 tile. The splits of a tile are adjacent items, so the
// bijective XCD remap keeps them on one XCD and the partials in one L2. Splits keep >= 16 K-tiles each:
// at 4 K-tiles (1024^3 in 4 splits) the reduction costs more than the idle CUs (110 vs 167 TF/s), at 32
// (1024^2x8192 in 4 splits) it pays 2.2x (458 vs 207 TF/s).
typedef __attribute__((address_space(3))) void* s_lds_ptr;

template <bool SPLIT>
__global__ void __launch_bounds__(S_THREADS, 1)
gemm_bf16_128x128(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C, int M,
                    int N, int K, int splits, float* __restrict__ ws, int* __restrict__ cnt) {
  constexpr int NBUF = 3, OPB = S_BM * S_BK * 2, TILEB = 2 * OPB;     // 16 KiB per operand, 32 KiB per K-tile
  __shared__ __attribute__((aligned(16))) char lds[NBUF * TILEB];     // the only LDS object (trap 4a)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / S_BN, ntiles = (M / S_BM) * tiles_n;
  const int item = xcd_remap(blockIdx.x, ntiles * (SPLIT ? splits : 1));
  const int tile = SPLIT ? item / splits : item, split = SPLIT ? item % splits : 0;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int nk_all = K / S_BK;
  const int kt0 = SPLIT ? split * nk_all / splits : 0;
  const int nk = SPLIT ? (split + 1) * nk_all / splits - kt0 : nk_all;

  // DMA sources: wave w issues the 8-row chunks c = w + 4 i (i = 0..3) of each operand
  const int lr = lane >> 3, lq = (lane & 7) ^ lr;
  const __bf16* srcA = A + ((size_t)tm * S_BM + 8 * wave + lr) * K + (size_t)kt0 * S_BK + lq * 8;
  const __bf16* srcB = Bt + ((size_t)tn * S_BN + 8 * wave + lr) * K + (size_t)kt0 * S_BK + lq * 8;
  const size_t chunk_step = (size_t)32 * K;        // 4 chunks of 8 rows further
#define S_DMA(kt, buf)                                                                                         \
  do {                                                                                                        \
    char* base_ = lds + (buf) * TILEB + wave * 1024;                                                          \
    const size_t ko_ = (size_t)(kt) * S_BK;                                                                   \
    __builtin_amdgcn_global_load_lds((const void*)(srcA + ko_), (s_lds_ptr)(base_), 16, 0, 0);                \
    __builtin_amdgcn_global_load_lds((const void*)(srcA + chunk_step + ko_), (s_lds_ptr)(base_ + 4096), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(srcA + 2 * chunk_step + ko_), (s_lds_ptr)(base_ + 8192), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(srcA + 3 * chunk_step + ko_), (s_lds_ptr)(base_ + 12288), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(srcB + ko_), (s_lds_ptr)(base_ + OPB), 16, 0, 0);          \
    __builtin_amdgcn_global_load_lds((const void*)(srcB + chunk_step + ko_), (s_lds_ptr)(base_ + OPB + 4096), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(srcB + 2 * chunk_step + ko_), (s_lds_ptr)(base_ + OPB + 8192), 16, 0, 0); \
    __builtin_amdgcn_global_load_lds((const void*)(srcB + 3 * chunk_step + ko_), (s_lds_ptr)(base_ + OPB + 12288), 16, 0, 0); \
  } while (0)

  s_floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = s_floatx4{0.f, 0.f, 0.f, 0.f};

  S_DMA(0, 0);
  if (nk > 1) S_DMA(1, 1);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire K-tile kt (8 DMAs per thread per tile; tile kt + 1's stay in flight), then publish it
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // every wave is past K-tile kt - 1's reads: its buffer takes tile kt + 2
    if (kt + 2 < nk) S_DMA(kt + 2, buf == 0 ? 2 : buf - 1);
    const char* la = lds + buf * TILEB;
    const char* lb = la + OPB;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int q = kk * 4 + (lane >> 4);
      s_bf16x8 af[4], bf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *(const s_bf16x8*)(la + s_swz(wm * 64 + i * 16 + (lane & 15), q));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *(const s_bf16x8*)(lb + s_swz(wn * 64 + j * 16 + (lane & 15), q));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    buf = buf == 2 ? 0 : buf + 1;
  }
#undef S_DMA
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();     // every wave done with the ring (the split reduce reuses lds)
  if constexpr (SPLIT) {
    if (splits > 1 && !small_split_reduce(acc, ws, cnt, item, tile, splits, tid, (int*)lds)) return;
  }
  const int row0 = tm * S_BM + wm * 64 + (lane >> 4) * 4, col0 = tn * S_BN + wn * 64 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        C[(size_t)(row0 + i * 16 + e) * N + col0 + j * 16] = (__bf16)acc[i][j][e];
}
