// gfx950 bf16 / fp8 GEMM for small output grids (v60, v61, v62):
//
//   C[M,N] (bf16) = A[M,K] * Bt[N,K]^T, A and Bt K-major, both bf16 or both fp8 e4m3fn, fp32 accumulation.
//
// A K-tile is 128 bytes of every row -- 64 bf16 or 128 fp8 elements -- so the LDS image, the DMA and the
// fragment reads are the same bytes for both dtypes: a lane reads 16-byte chunks g and g + 4 of a row
// (g = lane >> 4). bf16 runs them as two k-steps of v_mfma_f32_16x16x32_bf16; fp8 feeds both chunks to
// one v_mfma_f32_16x16x128_f8f6f4 (the unscaled double-rate form; any lane -> k map gives the same sums
// when A and B share it, as in gemm_fp8_kernels.h F8Q_CHUNK). The accumulator layout is the same.
//
// The 256x256 kernels own one output tile per CU: on a grid of 16 such tiles (1024^3) 16 of the 256
// CUs work and each runs a 134 MFLOP tile alone (~14 us at one CU's matrix rate), so the dispatch is
// bound by the per-CU MFMA time of a few CUs, not by the chip. This frame cuts the work finer:
//
//   * BMT x 128 output tiles (BMT = 128: v60 / v61; 256: v62), one 512-thread workgroup each, 8 waves
//     (two per SIMD) of 64 x TN (SmallCfg below);
//   * K-step 128 bytes, in an LDS ring of 4 K-tiles (128 rows) or 3 (256 rows);
//   * LDS rows of 128 B hold 8 16-B chunks XOR-swizzled by (row & 7): the ds_read_b128 fragment reads
//     (16 rows, one chunk column) spread over the banks (SQ_LDS_BANK_CONFLICT 0, profiles/r5_small/);
//   * XCD-aware tile order (bijective remap): the tiles one XCD runs are contiguous row-major, so
//     they share A row panels in that XCD's L2.
//
// Shapes: M % BMT == 0, N % 128 == 0, K a multiple of one K-tile (host checks). v60 / v62 run the whole
// K per tile; v61 splits K over several workgroups per tile (below). One workgroup per CU (the ring is
// 128 or 144 KiB of the CU's 160).
#pragma once

#include "gemm_tile_common.h"

constexpr int S_BM = 128, S_BN = 128, S_BK = 64, S_WAVES = 8, S_THREADS = S_WAVES * 64;

typedef __bf16 s_bf16x8 __attribute__((ext_vector_type(8)));
typedef int s_i32x4 __attribute__((ext_vector_type(4)));
typedef int s_i32x8 __attribute__((ext_vector_type(8)));
typedef float s_floatx4 __attribute__((ext_vector_type(4)));

// byte offset of 16-B chunk q (0..7) of row r in a panel of 128-B rows, swizzled
__device__ __forceinline__ int s_swz(int r, int q) { return r * 128 + ((q ^ (r & 7)) << 4); }

// Staging: LDS-DMA (buffer_load_dwordx4 ... lds): each wave-instruction writes 1 KiB (8 rows of 128 B)
// straight to LDS, lane-linear, so the XOR swizzle goes on the SOURCE address (lane L of a chunk loads
// global chunk (L & 7) ^ (L >> 3) of its row; the fragment reads use s_swz). One buffer descriptor per
// operand panel; the lane's byte offset is one VGPR for the whole K loop and the K-tile / chunk offsets
// are SGPRs, so a DMA costs no address VALU -- every VALU op sits in the MFMA issue stream: buffer
// loads against global_load_lds with 64-bit lane addresses measured +10-12 % on every shape
// (2048^2x8192 838 -> 937 TF/s, 9.6e6 -> 7.4e6 VALU instructions; profiles/r5_small/).
// A ring of 4 K-tile buffers (128 KiB) keeps three K-tiles in flight: at K-tile t a counted vmcnt
// retires tile t only, a raw s_barrier (no __syncthreads, whose fence would drain the DMA) publishes it,
// and the DMA of tile t + 3 goes into the buffer every wave finished reading at t - 1.
//
// Waves: 8 (two per SIMD, 2x4 of 64x32) against 4 (one per SIMD, 2x2 of 64x64): +4-10 % on every
// shape (2048^3 802 -> 834, 1536^3 450 -> 490 TF/s) -- a SIMD's second wave issues MFMAs while the
// first waits on its fragment reads or at the barrier.
//
// Fragments: a K-tile's A reads and its first k-step's B reads go out at once, then the first k-step's
// MFMAs (each waits only for its own operands: counted lgkmcnt), then the second k-step's B reads and
// MFMAs (+2-5 % over one k-step at a time). The kernel arguments are read into SGPRs before the loop:
// a scalar load still pending at the loop header turns every counted fragment wait into lgkmcnt(0).
typedef __attribute__((address_space(3))) void* s_lds_ptr;

// Tile shapes: BMT x 128 output tiles (BMT = 128: v60 / v61; 256: v62, for 256x256 grids of a quarter
// to a half of the CUs, where 256x128 tiles fill the chip in one wave: 2560^3 878 vs 773 TF/s, 2816^3
// 1060 vs 969, 4096x2048x4096 1145 vs 1074; fp8 2560^3 1591 vs 1412 -- profiles/r5_small/),
// 8 waves as WM x WN of 64 x TN each; a ring of NBUF K-tiles of OPA (A: BMT rows) + OPB (B: 128 rows)
// bytes: 4 x 32 KiB for 128, 3 x 48 KiB for 256.
template <int BMT>
struct SmallCfg {
  static_assert(BMT == 128 || BMT == 256, "128- or 256-row tiles");
  static constexpr int WM = BMT / 64, WN = S_WAVES / WM, TN = S_BN / WN, NJ = TN / 16;
  static constexpr int NBUF = BMT == 128 ? 4 : 3;
  static constexpr int OPA = BMT * 128, OPB = S_BN * 128, TILEB = OPA + OPB;
  static constexpr int LDS = NBUF * TILEB + 16;                // the ring + the split reduction's flag
  static constexpr int CPA = BMT / 8 / S_WAVES, CPB = S_BN / 8 / S_WAVES;   // 8-row DMA chunks per wave
  static constexpr int PT = CPA + CPB;                         // DMAs per thread per K-tile
  static constexpr int NACC = 4 * NJ;                          // 16x16 accumulators per thread
  static_assert(LDS <= 160 * 1024, "one CU's LDS");
};
template <int BMT>
using SmallAcc = s_floatx4[4][SmallCfg<BMT>::NJ];

// wait until at most `ahead` K-tiles (PT DMAs each) of this thread are in flight; ahead <= 2
template <int PT>
__device__ __forceinline__ void s_wait_tiles(int ahead) {
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PT) : "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PT) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// acc = A[tile rows, K-tiles kt0 .. kt0 + nk) * Bt[...]^T for output tile (tm, tn); row_b = bytes per
// operand row. Ends with every wave past its last fragment read (the ring is free again).
template <bool F8, int BMT>
__device__ __forceinline__ void small_mainloop(const char* __restrict__ A, const char* __restrict__ Bt, uint32_t row_b,
                                               int tm, int tn, int kt0, int nk, char* lds, SmallAcc<BMT>& acc) {
  using Cfg = SmallCfg<BMT>;
  constexpr int NBUF = Cfg::NBUF, WAVES = S_WAVES, NJ = Cfg::NJ, TN = Cfg::TN;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform: LDS-DMA bases stay scalar
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  // DMA pieces: wave w issues the 8-row chunks c = w + WAVES i of each operand
  const int lr = lane >> 3, lq = (lane & 7) ^ lr;
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)(A + (size_t)tm * BMT * row_b), 0, (int)(BMT * row_b), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)(Bt + (size_t)tn * S_BN * row_b), 0, (int)(S_BN * row_b), 0x00020000);
  const uint32_t voff = (uint32_t)(8 * wave + lr) * row_b + (uint32_t)kt0 * 128u + (uint32_t)lq * 16u;
  const uint32_t cstep = 8u * WAVES * row_b;
  auto dma = [&](int kt, int b) {
    char* base = lds + b * Cfg::TILEB + wave * 1024;
    const uint32_t kb = (uint32_t)kt * 128u;
#pragma unroll
    for (int i = 0; i < Cfg::CPA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (s_lds_ptr)(base + i * WAVES * 1024), 16, voff, kb + i * cstep, 0, 0);
#pragma unroll
    for (int i = 0; i < Cfg::CPB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (s_lds_ptr)(base + Cfg::OPA + i * WAVES * 1024), 16, voff,
                                               kb + i * cstep, 0, 0);
  };
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = s_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < NBUF - 1; ++t)
    if (t < nk) dma(t, t);
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // retire K-tile kt (the younger tiles stay in flight), then publish it
    s_wait_tiles<Cfg::PT>(min(NBUF - 2, nk - 1 - kt));
    __builtin_amdgcn_s_barrier();
    // every wave is past K-tile kt - 1's reads: its buffer takes tile kt + NBUF - 1
    if (kt + NBUF - 1 < nk) dma(kt + NBUF - 1, buf == 0 ? NBUF - 1 : buf - 1);
    const char* la = lds + buf * Cfg::TILEB;
    const char* lb = la + Cfg::OPA;
    s_i32x4 af[2][4], bf[2][NJ];
    const int q0 = lane >> 4, q1 = 4 + (lane >> 4);
    auto rd = [&](const char* base, int row, int q) { return *(const s_i32x4*)(base + s_swz(row + (lane & 15), q)); };
    if constexpr (F8) {
      // one 16x16x128 MFMA per accumulator over both chunks. Reads in the order the MFMAs (B column
      // j outer, A row i inner) first need them -- A0, B0, A1, A2, A3, B1.. -- so each MFMA waits
      // only for its own operands' reads
      auto rda = [&](int i) { af[0][i] = rd(la, wm * 64 + i * 16, q0); af[1][i] = rd(la, wm * 64 + i * 16, q1); };
      auto rdb = [&](int j) { bf[0][j] = rd(lb, wn * TN + j * 16, q0); bf[1][j] = rd(lb, wn * TN + j * 16, q1); };
      rda(0);
      rdb(0);
      __builtin_amdgcn_sched_barrier(0);     // (pins the read order: the scheduler would reorder them)
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        rda(i);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 1; j < NJ; ++j) {
        rdb(j);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const s_i32x8 b8 = __builtin_shufflevector(bf[0][j], bf[1][j], 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const s_i32x8 a8 = __builtin_shufflevector(af[0][i], af[1][i], 0, 1, 2, 3, 4, 5, 6, 7);
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc[i][j], 0, 0, 0, 0, 0, 0);
        }
      }
    } else {
      af[0][0] = rd(la, wm * 64, q0);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[0][j] = rd(lb, wn * TN + j * 16, q0);
#pragma unroll
      for (int i = 1; i < 4; ++i) af[0][i] = rd(la, wm * 64 + i * 16, q0);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) af[1][i] = rd(la, wm * 64 + i * 16, q1);
#pragma unroll
      for (int j = 0; j < NJ; ++j) bf[1][j] = rd(lb, wn * TN + j * 16, q1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((s_bf16x8)af[0][i], (s_bf16x8)bf[0][j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16((s_bf16x8)af[1][i], (s_bf16x8)bf[1][j], acc[i][j], 0, 0, 0);
    }
    buf = buf == NBUF - 1 ? 0 : buf + 1;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();     // every wave done with the ring
}

template <int BMT>
__device__ __forceinline__ void small_store_c(__bf16* __restrict__ C, int N, int tm, int tn, const SmallAcc<BMT>& acc) {
  using Cfg = SmallCfg<BMT>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  const int row0 = tm * BMT + wm * 64 + (lane >> 4) * 4, col0 = tn * S_BN + wn * Cfg::TN + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < Cfg::NJ; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        C[(size_t)(row0 + i * 16 + e) * N + col0 + j * 16] = (__bf16)acc[i][j][e];
}

// v60 (BMT = 128) / v62 (BMT = 256): one workgroup per BMT x 128 output tile,
// the whole K. F8: A, Bt are fp8 e4m3fn bytes.
template <bool F8, int BMT = 128, Rec REC = kTimed>
__global__ void __launch_bounds__(S_THREADS, 1) __attribute__((amdgpu_waves_per_eu(S_WAVES / 4, S_WAVES / 4)))
gemm_mfma_small(const void* __restrict__ A, const void* __restrict__ Bt, __bf16* __restrict__ C, int M, int N,
                  int K) {
  __shared__ __attribute__((aligned(16))) char lds[SmallCfg<BMT>::LDS];     // the only LDS object (trap 4a)
  note_placement<REC>();
  const int tiles_n = N / S_BN, ntiles = (M / BMT) * tiles_n;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const uint32_t row_b = (uint32_t)K * (F8 ? 1u : 2u);
  asm volatile("" ::"s"(C), "s"(N));   // kernel arguments in SGPRs before the loop (see "Fragments")
  SmallAcc<BMT> acc;
  small_mainloop<F8, BMT>((const char*)A, (const char*)Bt, row_b, tm, tn, 0, (int)(row_b / 128u), lds, acc);
  small_store_c<BMT>(C, N, tm, tn, acc);
}

// v61, split-K: `splits` workgroups per output tile; piece s of a tile runs K-tiles
// [s nk / splits, (s + 1) nk / splits), so every tile is cut at the same K offsets and the workgroups
// sharing an A or B panel stream the same K-slices at the same time (L2 hits). A piece stores its fp32
// slab (thread-major float4s: one coalesced KiB per wave and accumulator) -- round 6: only the pieces
// that draw an arrival ticket before the last one do (cdna_hip_programming.md "Projection GEMM at M =
// 256" item 2: plain 16-B stores, drain, barrier, ONE lane releases at agent scope and counts itself
// done); the last arrival waits for their done count, acquires, and sums the pieces in piece order with
// its own from its registers, so the result does not depend on arrival order, and writes the bf16 tile. Nobody waits for anybody: the grid needs no
// co-residency. Item order: pieces of >= 32 K-tiles go piece-major (item = piece x tiles + tile), so
// the XCD remap gives an XCD a run of neighbouring tiles at ONE K range -- 1024^2x16384 in 4 pieces
// streams 6 MiB of A and B per XCD instead of 18 (tile-major, every XCD read all of B): bf16 617 ->
// 709 TF/s (1.07x hipBLASLt), 1024^2x8192 485 -> 518, fp8 1024^2x16384 974 -> 1048; the slabs then
// cross XCDs (the agent-scope release / acquire covers that), which costs more than it saves on
// shorter pieces (1024^2x4096, 16 K-tiles: 327 -> 316), so those stay tile-major (the pieces of a
// tile adjacent, on one XCD; profiles/r5_small/sweep_piece_major.jsonl). Pieces keep >= 16 K-tiles (gemm_small_host.h): at 4 K-tiles (1024^3 in 4 pieces)
// the reduction costs more than the idle CUs (110 vs 167 TF/s), at 32 (1024^2x8192 in 4) it pays 2.2x
// (458 vs 207). A stream-K even share of grids larger than the chip (pieces cut at offsets that differ
// from workgroup to workgroup) lost the panel sharing and ran 35-40 % below v60
// (profiles/r5_small/sweep_streamk.jsonl).
template <bool F8, int BMT = 128, Rec REC = kTimed>
__global__ void __launch_bounds__(S_THREADS, 1) __attribute__((amdgpu_waves_per_eu(S_WAVES / 4, S_WAVES / 4)))
gemm_mfma_small_sk(const void* __restrict__ A, const void* __restrict__ Bt, __bf16* __restrict__ C, int M, int N,
                     int K, int splits, int pmajor, float* __restrict__ ws, int* __restrict__ cnt) {
  typedef float f4 __attribute__((ext_vector_type(4)));
  using Cfg = SmallCfg<BMT>;
  __shared__ __attribute__((aligned(16))) char lds[Cfg::LDS];     // the only LDS object (trap 4a)
  note_placement<REC>();
  int* flag = (int*)(lds + Cfg::NBUF * Cfg::TILEB);
  const int tid = threadIdx.x;
  const int tiles_n = N / S_BN, ntiles = (M / BMT) * tiles_n;
  const uint32_t row_b = (uint32_t)K * (F8 ? 1u : 2u);
  const int nk = (int)(row_b / 128u);
  const int item = xcd_remap(blockIdx.x, ntiles * splits);
  const int piece = pmajor ? item / ntiles : item % splits;      // item order: see v61 above
  const int tile = pmajor ? item - piece * ntiles : item / splits;
  const int kt0 = piece * nk / splits, kt1 = (piece + 1) * nk / splits;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  asm volatile("" ::"s"(C), "s"(N), "s"(ws), "s"(cnt), "s"(splits));   // see "Fragments"
  SmallAcc<BMT> acc;
  small_mainloop<F8, BMT>((const char*)A, (const char*)Bt, row_b, tm, tn, kt0, kt1 - kt0, lds, acc);
  if (splits > 1) {
    // ticket first (the asm frame's protocol, gemm_w4ap.h SPLIT): only the earlier arrivals store their
    // slab and release; the last arrival keeps its partial in registers, waits for their done count (they
    // have arrived: they owe only their stores), acquires, and sums the pieces in piece order with its
    // own at its place -- the same bits whichever piece reduces.
    constexpr size_t SLAB = (size_t)BMT * S_BN;     // floats per tile
    f4* flat = (f4*)&acc[0][0];
    int* const arrive = cnt + 2 * tile;
    int* const done = arrive + 1;
    if (tid == 0) flag[0] = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int ticket = flag[0];
    if (ticket < splits - 1) {
      f4* slab = (f4*)(ws + ((size_t)tile * splits + piece) * SLAB);
#pragma unroll
      for (int a = 0; a < Cfg::NACC; ++a) slab[a * S_THREADS + tid] = flat[a];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    if (tid == 0) {
      bool seen = false;       // bounded (~1 s) although every awaited workgroup is running
      for (unsigned spins = 0;
           !(seen = __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= splits - 1) &&
           spins < (1u << 24);
           ++spins)
        __builtin_amdgcn_s_sleep(2);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      *arrive = 0;             // ready for the next launch on this stream
      *done = 0;
      flag[1] = seen;          // (flag[0] holds the ticket the other waves may still be reading)
    }
    __syncthreads();
    if (!flag[1]) {            // the wait gave up: a NaN tile, never a silent partial sum
#pragma unroll
      for (int a = 0; a < Cfg::NACC; ++a) flat[a] = f4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                                                      __builtin_nanf("")};
    } else {
      f4 mine[Cfg::NACC];
#pragma unroll
      for (int a = 0; a < Cfg::NACC; ++a) mine[a] = flat[a];
      for (int p = 0; p < splits; ++p) {
        const f4* part = (const f4*)(ws + ((size_t)tile * splits + p) * SLAB);
#pragma unroll
        for (int a = 0; a < Cfg::NACC; ++a) {
          const f4 x = p == piece ? mine[a] : part[a * S_THREADS + tid];
          flat[a] = p == 0 ? x : flat[a] + x;
        }
      }
    }
  }
  small_store_c<BMT>(C, N, tm, tn, acc);
}
