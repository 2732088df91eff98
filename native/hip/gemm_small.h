// gfx950 bf16 GEMM for small output grids (v60):
//
//   C[M,N] (bf16) = A[M,K] (bf16, K-major) * Bt[N,K]^T (bf16, K-major), fp32 accumulation.
//
// The 256x256 kernels own one output tile per CU: on a grid of 16 such tiles (1024^3) 16 of the 256
// CUs work and each runs a 134 MFLOP tile alone (~14 us at one CU's matrix rate), so the dispatch is
// bound by the per-CU MFMA time of a few CUs, not by the chip. This kernel cuts the work 4x finer:
//
//   * 128x128 output tile per 256-thread workgroup, 4 waves as 2x2, each wave a 64x64 sub-tile =
//     4x4 v_mfma_f32_16x16x32_bf16 accumulators (64 VGPRs); launch_bounds(256, 2): two workgroups
//     share a CU when the grid is larger than the chip;
//   * K-step 64: one K-tile of A and of B is 16 KiB each, double-buffered in 64 KiB of LDS;
//   * the next K-tile's global loads (16 B per lane, 4 per operand per thread) are issued before the
//     current K-tile's 32 MFMAs per wave and written to the other LDS buffer after them: one barrier
//     per K-tile, the HBM/L2 latency under the matrix work;
//   * LDS rows of 128 B hold 8 16-B chunks XOR-swizzled by (row & 7): the ds_write_b128 of a wave (8
//     rows x 8 chunks) and the ds_read_b128 fragment reads (16 rows, one chunk column) spread over
//     the banks -- 2-way at worst on the reads, the minimum for a 16-row b128 read;
//   * XCD-aware tile order (bijective remap): the tiles one XCD runs are contiguous row-major, so
//     they share A row panels in that XCD's L2.
//
// Shapes: M % 128 == 0, N % 128 == 0, K % 64 == 0 (host checks). v60 runs the whole K per tile;
// v61 splits K over several workgroups per tile (below).
#pragma once

#include "gemm_tile_common.h"

constexpr int S_BM = 128, S_BN = 128, S_BK = 64, S_THREADS = 256;

typedef __bf16 s_bf16x8 __attribute__((ext_vector_type(8)));
typedef float s_floatx4 __attribute__((ext_vector_type(4)));

// byte offset of 16-B chunk q (0..7) of row r in a [rows][64] bf16 panel (128-B rows), swizzled
__device__ __forceinline__ int s_swz(int r, int q) { return r * 128 + ((q ^ (r & 7)) << 4); }

// SPLIT (v61): split-K for grids smaller than the chip. The grid is tiles x `splits` workgroups; item
// (tile, s) runs K-tiles [s nk / splits, (s + 1) nk / splits). Every workgroup stores its fp32 partial
// tile to `ws` (thread-major float4s: one coalesced KiB per wave and accumulator), releases it
// (__threadfence, device scope) and counts itself in `cnt[tile]`; the workgroup that arrives last
// acquires, adds the other partials to its registers, writes the bf16 tile and resets the counter for
// the next launch (stream order). The splits of a tile are adjacent items, so the bijective XCD remap
// keeps them on one XCD and the partials in one L2.
template <bool SPLIT>
__global__ void __launch_bounds__(S_THREADS, 2)
gemm_bf16_128x128_t(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C, int M,
                    int N, int K, int splits, float* __restrict__ ws, int* __restrict__ cnt) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * S_BM * S_BK * 2];   // [buf][A|B] 64 KiB
  __shared__ int arrived;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / S_BN, ntiles = (M / S_BM) * tiles_n;
  const int item = xcd_remap(blockIdx.x, ntiles * (SPLIT ? splits : 1));
  const int tile = SPLIT ? item / splits : item, split = SPLIT ? item % splits : 0;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const __bf16* Ab = A + (size_t)tm * S_BM * K;
  const __bf16* Bb = Bt + (size_t)tn * S_BN * K;

  // global -> register staging: chunk c = tid + 256 i covers row c >> 3, 16-B chunk c & 7
  // (straight-line code, no lambdas: an array a lambda captures by reference lives in scratch)
  const int r0 = tid >> 3, q0 = tid & 7;        // chunk i: row r0 + 32 i, chunk q0
  const __bf16* ga = Ab + (size_t)r0 * K + q0 * 8;
  const __bf16* gb = Bb + (size_t)r0 * K + q0 * 8;
  const size_t rstep = (size_t)32 * K;
  int soff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) soff[i] = s_swz(r0 + 32 * i, q0);
  uint4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
#define S_GLOAD(kt)                                                   \
  do {                                                                \
    const size_t k0_ = (size_t)(kt) * S_BK;                           \
    ra0 = *(const uint4*)(ga + k0_);                                  \
    ra1 = *(const uint4*)(ga + rstep + k0_);                          \
    ra2 = *(const uint4*)(ga + 2 * rstep + k0_);                      \
    ra3 = *(const uint4*)(ga + 3 * rstep + k0_);                      \
    rb0 = *(const uint4*)(gb + k0_);                                  \
    rb1 = *(const uint4*)(gb + rstep + k0_);                          \
    rb2 = *(const uint4*)(gb + 2 * rstep + k0_);                      \
    rb3 = *(const uint4*)(gb + 3 * rstep + k0_);                      \
  } while (0)
#define S_LSTORE(buf)                                                 \
  do {                                                                \
    char* la_ = lds + (buf) * (2 * S_BM * S_BK * 2);                  \
    char* lb_ = la_ + S_BM * S_BK * 2;                                \
    *(uint4*)(la_ + soff[0]) = ra0;                                   \
    *(uint4*)(la_ + soff[1]) = ra1;                                   \
    *(uint4*)(la_ + soff[2]) = ra2;                                   \
    *(uint4*)(la_ + soff[3]) = ra3;                                   \
    *(uint4*)(lb_ + soff[0]) = rb0;                                   \
    *(uint4*)(lb_ + soff[1]) = rb1;                                   \
    *(uint4*)(lb_ + soff[2]) = rb2;                                   \
    *(uint4*)(lb_ + soff[3]) = rb3;                                   \
  } while (0)

  s_floatx4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = s_floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = K / S_BK;
  const int kt0 = SPLIT ? split * nk_all / splits : 0;
  const int nk = SPLIT ? (split + 1) * nk_all / splits - kt0 : nk_all;
  S_GLOAD(kt0);
  S_LSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) S_GLOAD(kt0 + kt + 1);
    const char* la = lds + buf * (2 * S_BM * S_BK * 2);
    const char* lb = la + S_BM * S_BK * 2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      // lane l: row (l & 15) of its 16-row block, k = 32 kk + 8 (l >> 4) .. + 7 = chunk 4 kk + (l >> 4)
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
    if (kt + 1 < nk) S_LSTORE(buf ^ 1);
    __syncthreads();
  }
  if constexpr (SPLIT) {
    if (splits > 1) {
      s_floatx4* part = (s_floatx4*)(ws + (size_t)item * (S_BM * S_BN));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) part[(i * 4 + j) * S_THREADS + tid] = acc[i][j];
      __threadfence();                     // release: the partial is visible device-wide
      __syncthreads();
      if (tid == 0) arrived = atomicAdd(&cnt[tile], 1);
      __syncthreads();
      if (arrived != splits - 1) return;   // not the last of the tile's splits
      __threadfence();                     // acquire: every other split's partial
      for (int s2 = 0; s2 < splits; ++s2) {
        if (s2 == split) continue;
        const s_floatx4* other = (const s_floatx4*)(ws + ((size_t)tile * splits + s2) * (S_BM * S_BN));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] += other[(i * 4 + j) * S_THREADS + tid];
      }
      if (tid == 0) cnt[tile] = 0;         // ready for the next launch on this stream
    }
  }
  // epilogue: D of block (i, j): column l & 15, rows 4 (l >> 4) + e
  const int row0 = tm * S_BM + wm * 64 + (lane >> 4) * 4, col0 = tn * S_BN + wn * 64 + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        C[(size_t)(row0 + i * 16 + e) * N + col0 + j * 16] = (__bf16)acc[i][j][e];
#undef S_GLOAD
#undef S_LSTORE
}
