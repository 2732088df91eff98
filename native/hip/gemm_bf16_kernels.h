// Production gfx950 bf16 GEMM kernels of the node validator (shared by the validator library
// gemm_bf16.hip and the tools-only experiment library gemm_bf16_lab.hip):
//
//   C[M,N] (bf16) = A[M,K] (bf16, K-major) * Bt[N,K]^T (bf16, K-major), fp32 accumulation.
//
//   * gemm_bf16_256x256_w4s  -- v18 schedule; v44 = + serpentine K + loop rotation (the default),
//                               v45 = v44 + square cross-XCD raster, v42 = rotation only (devices
//                               without 256 CUs), v18 = neither;
//   * gemm_bf16_256x256_w4sp -- v25: v18 made persistent (short K, several tiles per CU);
//   * gemm_bf16_generic      -- bounds-checked 64x64-tile MFMA kernel for every other shape;
//   * fill_uniform_bf16 -- the operand filler (the fp32 reference rows live in gemm_abft.hip).
// Design notes and measurements: docs/validator-gemm.md, profiles/r1_*.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_tile_common.h"
#include "gemm_w4ap.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256;
constexpr int BN = 256;
constexpr int BK = 64;
constexpr int NTHREADS = 512;
constexpr int ROW_BYTES = BK * 2;             // 128 B per staged row
constexpr int PANEL_BYTES = BM * ROW_BYTES;   // 32 KiB per operand per K-tile
constexpr int BUF_BYTES = 2 * PANEL_BYTES;    // A + B
constexpr int LDS_BYTES = 2 * BUF_BYTES;      // double buffered: 128 KiB

// The accumulators are pinned: hipcc's greedy allocator, given 64 tuples that fill all 256 AGPRs,
// cannot keep them in place across the loop back-edge and shuffles them through a[0:3] with
// ~600 v_accvgpr moves per K-tile. So the MFMAs are inline asm on literal a[4i:4i+3] (the kernel
// owns every AGPR via W4_AGPR_CLOBBERS; the compiler has no AGPR values of its own -- audited in
// tests/test_gemm_build.py: no compiler v_accvgpr_* outside the asm blocks). Hazards handled by
// hand (cdna_hip_programming.md §5.7 item 2): zeroing writes -> first MFMA reading them as C are
// separated by the prologue; the last MFMA's D -> v_accvgpr_read is covered by an explicit s_nop
// pad; an accumulate chain MFMA -> MFMA (same C) needs none. A/B operands come from compiler
// ds_reads whose lgkmcnt waits hipcc inserts before each asm statement that names them.
constexpr int W4_THREADS = 256;

struct W4Frags {
  bf16x8 a[8];
  bf16x8 b[8];
};

template <int I>
__device__ __forceinline__ void w4_mfma(const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]"
               :: "i"(4 * I), "i"(4 * I + 3), "v"(b), "v"(a));
}

// fragment read order j -> (A or B, index): the order the next block consumes them
// (i = 0..7 uses a0 with b0..b7, then a1 ...), so hipcc's lgkmcnt ladder releases MFMAs early.
__device__ __forceinline__ constexpr int w4_isb(int j) { return j >= 1 && j <= 8; }
__device__ __forceinline__ constexpr int w4_idx(int j) { return j == 0 ? 0 : (j <= 8 ? j - 1 : j - 8); }

// the R0 read (j in w4_isb order) issued at slot i of a w4s iteration, or -1: read j sits at
// slot B2 + 1 + j*RS/16 (a constexpr lookup keeps the compile time of a variant at seconds)
__host__ __device__ constexpr int w4s_r0_at(int b2, int rs, int i) {
  for (int j = 0; j < 16; ++j)
    if (b2 + 1 + (j * rs) / 16 == i) return j;
  return -1;
}

// RSPAN / DSPAN: the 16 fragment reads / DMA pieces of a block are spread over its first
// RSPAN / DSPAN groups of 4 MFMAs (16 = evenly; smaller = earlier, more latency slack).

// v18: v10's data layout with the schedule reshaped around the K-tile instead of two halves.
// Knock-out cycle accounting of v10 (profiles/r1_gemm_v10/README.md) priced its DMA at 13 % of
// the wave cycles and its wait+barrier at 4 %, with fragment reads nearly free. Here, in MFMA
// slots 0..127 of iteration t (0..63 on R0 = tile t kk0, 64..127 on R1 = tile t kk1):
//   slots 0..15      read R1 <- tile t kk1 (one per MFMA)
//   slot B1          lgkmcnt(0) one MFMA earlier, then a barrier: every wave is done with tile t
//   slots D0 + j*DS  DMA tile t+2 into tile t's buffer (16 pieces), starting ~40 slots earlier
//                    than v10 so a piece has ~80 MFMAs to land
//   slot B2          vmcnt(pieces issued so far this iteration) one MFMA earlier -- tile t+1 (last
//                    iteration's pieces) landed, this iteration's stay in flight -- then a barrier
//   slots B2+1 ..    read R0 <- tile t+1 kk0, spread over RS slots
// Barriers sit between two MFMAs so the matrix pipe has queued work while the wave waits.
// (The round-2 knock-out timings that priced each of these parts are recorded in
// profiles/r2_sched/README.md; the knock-out builds themselves were retired from the tree.)
template <int B1 = 17, int D0 = 19, int DS = 5, int B2 = 80, int RS = 40, int SERP = 0, bool ROT = false,
          bool SQ = false, bool VK = false, bool PA = false, Rec REC = kTimed>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4s(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  static_assert(B1 >= 16 && D0 > B1 && D0 + 15 * DS < 127 && B2 > B1 && B2 + RS < 127, "schedule");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  note_placement<REC>();

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  if constexpr (SQ) tile_coords_sq(blockIdx.x, tiles_n, tm, tn);
  else tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K * 2u +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  const uint32_t voff_p = (uint32_t)(lane >> 3) * 32u * (uint32_t)K * 2u +
                          (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, int k0, char* buf) {
    // piece p = 4i + wid; p >= 32 (the B panel) <=> i >= 8, a compile-time fact once unrolled
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? PANEL_BYTES : 0) + rblk * 1024;
    // PA: an A-panel DMA instruction reads panel rows rblk + 32 g (g = lane >> 3) into LDS slots
    // 8 rblk + g, so its 8 rows are 32 rows apart instead of adjacent (at a 24 KiB row stride,
    // K = 12288, adjacent rows cost 10 %); LDS slot s then holds panel row 32 (s & 7) + (s >> 3),
    // which the epilogue's row mapping undoes. B keeps adjacent rows: its slots are C columns.
    if (PA && i < 8) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff_p + (uint32_t)k0 * 2u,
                                               (uint32_t)rblk * (uint32_t)K * 2u, 0, 0);
      return;
    }
    if constexpr (VK)   // K offset in the lane offset (one VALU add per K-tile), loop-invariant soffset
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff + (uint32_t)k0 * 2u,
                                               (uint32_t)rblk * 8u * (uint32_t)K * 2u, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff,
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
  // DM: DMA tile t+2; NX: tile t+1 exists (wait for it, read its kk0 into R0); LAST_DMA: the
  // previous iteration issued no DMA (vmcnt target 0 instead of this iteration's count)
  // slots [LO, HI) of one K-tile iteration; the slots before B1 depend on no flag (ROT splits there)
  auto iter = [&](char* cur, char* nxt, int dk, auto DM, auto NX, auto LO, auto HI) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value;
    static_for<decltype(LO)::value, decltype(HI)::value>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 64) w4_mfma<i>(R0.b[i & 7], R0.a[i >> 3]);
      else w4_mfma<i - 64>(R1.b[i & 7], R1.a[(i - 64) >> 3]);
      if constexpr (i < 16) read_frag(R1, cur, 1, std::integral_constant<int, i>{});
      if constexpr (i == B1 - 1) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      if constexpr (dm && i == B1) __builtin_amdgcn_s_barrier();
      if constexpr (dm && i >= D0 && (i - D0) % DS == 0 && (i - D0) / DS < 16) dma_piece((i - D0) / DS, dk, cur);
      if constexpr (nx && i == B2 - 1) {
        constexpr int issued = !dm ? 0 : (B2 - 1 < D0 ? 0 : ((B2 - 1 - D0) / DS + 1 > 16 ? 16 : (B2 - 1 - D0) / DS + 1));
        // vmcnt(issued) lgkmcnt(0): vmcnt low 4 bits [3:0], high 2 bits [15:14]; expcnt 7
        __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == B2) __builtin_amdgcn_s_barrier();
      constexpr int jr0 = w4s_r0_at(B2, RS, i);
      if constexpr (nx && jr0 >= 0) read_frag(R0, nxt, 0, std::integral_constant<int, jr0>{});
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int ktiles = K / BK;        // >= 2 (host guarantees)
  // SERP > 0 (serpentine K): with SERP co-resident workgroups per XCD, every other wave of tiles
  // walks K backwards, so it starts on the K-slices of the A panels the previous wave just left
  // in the XCD's L2.
  const bool rev = SERP > 0 && (((int)blockIdx.x / NXCD) / (SERP > 0 ? SERP : 1)) & 1;
  auto kof = [&](int kt) { return (rev ? ktiles - 1 - kt : kt) * BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(0), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(1), buf1);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): tile 0 landed, tile 1 in flight
  bar();
  static_for<0, 16>([&](auto J) { read_frag(R0, buf0, 0, J); });

  using S0 = std::integral_constant<int, 0>;
  using SB = std::integral_constant<int, B1>;
  using SE = std::integral_constant<int, 128>;
  char* cur = buf0;
  char* nxt = buf1;
  if constexpr (ROT) {
    // Loop rotation (v42/v43): an iteration runs slots B1..127 of tile t, then 0..B1-1 of tile
    // t+1, so the back-edge follows the explicit lgkmcnt(0) at slot B1-1 instead of the R0 reads,
    // where hipcc's merged loop-header state is a blanket lgkmcnt(0) before the first MFMA.
    iter(cur, nxt, 0, T_{}, T_{}, S0{}, SB{});
    for (int t = 0; t < ktiles - 2; ++t) {
      iter(cur, nxt, kof(t + 2), T_{}, T_{}, SB{}, SE{});
      char* tmp = cur; cur = nxt; nxt = tmp;
      iter(cur, nxt, 0, T_{}, T_{}, S0{}, SB{});
    }
    iter(cur, nxt, 0, F_{}, T_{}, SB{}, SE{});
    iter(nxt, nullptr, 0, F_{}, F_{}, S0{}, SE{});
  } else {
    for (int t = 0; t < ktiles - 2; ++t) {
      iter(cur, nxt, kof(t + 2), T_{}, T_{}, S0{}, SE{});
      char* tmp = cur; cur = nxt; nxt = tmp;
    }
    iter(cur, nxt, 0, F_{}, T_{}, S0{}, SE{});
    iter(nxt, nullptr, 0, F_{}, F_{}, S0{}, SE{});
  }

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
    const int gr = PA ? 32 * (r & 7) + (r >> 3) : r;           // LDS slot -> panel row (PA)
    store_c16(C + (size_t)(tm * BM + gr) * N + tn * BN + ch * 8, v);
  }
}
// w4t: the w4s kernel with the whole K-tile schedule taken from a schedule class SC, so the
// read/DMA/barrier placement can differ per operand panel. SC provides, in MFMA slots 0..127
// (an op "at slot i" issues right after MFMA i):
//   r1(j)   read of R1 <- tile t kk1, j < 8: A fragment j, j >= 8: B fragment j-8
//   wa, ba  lgkmcnt(0) and barrier after which tile t's A panel is free (A DMA pieces may start)
//   wb, bb  the same for the B panel (wa == wb and ba == bb: one barrier for both)
//   dma(p)  DMA piece p of tile t+2 (p < 8: A panel, p >= 8: B panel)
//   w2, b2  vmcnt(pieces issued so far) + lgkmcnt(0), then a barrier: tile t+1 landed
//   r0(j)   read of R0 <- tile t+1 kk0, j in w4_isb order
// With split panels, A's kk1 fragments are read first and A's DMA overlaps B's kk1 reads, so
// the fragment reads run at one per two MFMAs instead of the v18 burst of one per MFMA (a
// 64 KiB burst per CU that the LDS serves at 128 B/clk while the burst itself spans only 17
// MFMAs).
template <class SC>
__host__ __device__ constexpr int w4t_issued_by_w2() {
  int n = 0;
  for (int p = 0; p < 16; ++p) n += SC::dma(p) <= SC::w2 ? 1 : 0;
  return n;
}
// inverse lookups (the op of a kind issued at slot i, or -1): constexpr loops instead of a
// 16-way static_for per slot keep the compile time of a schedule at a few seconds
template <class SC>
__host__ __device__ constexpr int w4t_r1_at(int i) {
  for (int j = 0; j < 16; ++j)
    if (SC::r1(j) == i) return j;
  return -1;
}
template <class SC>
__host__ __device__ constexpr int w4t_dma_at(int i) {
  for (int j = 0; j < 16; ++j)
    if (SC::dma(j) == i) return j;
  return -1;
}
template <class SC>
__host__ __device__ constexpr int w4t_r0_at(int i) {
  for (int j = 0; j < 16; ++j)
    if (SC::r0(j) == i) return j;
  return -1;
}
template <class SC>
__host__ __device__ constexpr bool w4t_valid() {
  for (int j = 0; j < 16; ++j) {
    for (int q = 0; q < j; ++q)                          // at most one op of a kind per slot
      if (SC::r1(q) == SC::r1(j) || SC::dma(q) == SC::dma(j) || SC::r0(q) == SC::r0(j)) return false;
    if (SC::r1(j) < 0 || SC::r1(j) >= (j < 8 ? SC::wa : SC::wb)) return false;
    if (SC::r0(j) <= SC::b2 || SC::r0(j) > 127) return false;
    if (SC::dma(j) <= (j < 8 ? SC::ba : SC::bb) || SC::dma(j) > 127) return false;
    for (int q = 0; q < j; ++q)
      if (SC::r0(q) > SC::r0(j)) return false;          // R0 reads in consumption order
  }
  const bool one = SC::wa == SC::wb && SC::ba == SC::bb;
  return SC::wa < SC::ba && SC::wb < SC::bb && (one || SC::wb > SC::ba) && SC::w2 > SC::bb && SC::b2 == SC::w2 + 1 &&
         SC::ba >= 1;
}

// v18's schedule (B1=17, D0=19, DS=5, B2=80, RS=40) in w4t form: the parity reference.
struct W4SchedV18 {
  static constexpr int r1(int j) { return j; }
  static constexpr int wa = 16, ba = 17, wb = 16, bb = 17, w2 = 79, b2 = 80;
  static constexpr int dma(int p) { return 19 + 5 * p; }
  static constexpr int r0(int j) { return 81 + (j * 40) / 16; }
};
// hipBLASLt's gfx950 MT256x256x64 custom kernel places its loop this way (disassembled from the
// shipped code object, docs/validator-gemm.md): A kk1 reads every other MFMA, A-panel barrier,
// A DMA interleaved with B kk1 reads, B-panel barrier, the rest of the DMA, landing barrier,
// kk0 reads every other MFMA.
struct W4SchedSplit {
  static constexpr int r1(int j) {
    constexpr int b[8] = {23, 26, 29, 32, 35, 38, 40, 42};
    return j < 8 ? 2 * j : b[j - 8];
  }
  static constexpr int wa = 20, ba = 21, wb = 50, bb = 51, w2 = 91, b2 = 92;
  static constexpr int dma(int p) {
    constexpr int s[16] = {22, 25, 28, 31, 34, 52, 55, 58, 61, 64, 85, 87, 89, 96, 100, 124};
    return s[p];
  }
  static constexpr int r0(int j) { return 93 + 2 * j; }
};
// One barrier, but the 16 kk1 reads spread over 32 MFMAs and the DMA behind them.
struct W4SchedSpread {
  static constexpr int r1(int j) { return 2 * j; }
  static constexpr int wa = 33, ba = 34, wb = 33, bb = 34, w2 = 91, b2 = 92;
  static constexpr int dma(int p) { return 35 + (p * 7) / 2; }
  static constexpr int r0(int j) { return 93 + 2 * j; }
};
// Split panels with every DMA piece issued early and evenly (long landing time).
struct W4SchedSplitEarly {
  static constexpr int r1(int j) { return j < 8 ? 2 * j : 23 + 3 * (j - 8); }
  static constexpr int wa = 16, ba = 17, wb = 46, bb = 47, w2 = 91, b2 = 92;
  static constexpr int dma(int p) { return p < 8 ? 18 + 3 * p + 1 : 48 + 4 * (p - 8); }
  static constexpr int r0(int j) { return 93 + 2 * j; }
};
// Split panels, tighter: B reads right behind the A barrier, landing barrier at v18's slot 80.
struct W4SchedSplitTight {
  static constexpr int r1(int j) { return j < 8 ? 2 * j : 18 + 2 * (j - 8); }
  static constexpr int wa = 16, ba = 17, wb = 34, bb = 35, w2 = 79, b2 = 80;
  static constexpr int dma(int p) { return p < 8 ? 19 + 2 * p : 36 + 3 * (p - 8); }
  static constexpr int r0(int j) { return 81 + (j * 40) / 16; }
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ADMA: an LDS-DMA piece and the MFMA of its slot in ONE asm statement, M0 written first: the
// MFMA is the wait state the M0 -> LDS-DMA hazard needs, where hipcc (blind to what an asm MFMA
// is) pads every piece with an s_nop of its own. hipcc does not count asm loads: every vmcnt
// the kernel relies on is explicit (prologue, w2).
template <int I>
__device__ __forceinline__ void w4_mfma_dma(const bf16x8& b, const bf16x8& a, uint32_t m0v, uint32_t voff,
                                            u32x4 rs, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %4\n\tv_mfma_f32_16x16x32_bf16 a[%c0:%c1], %2, %3, a[%c0:%c1]\n\t"
               "buffer_load_dwordx4 %5, %6, %7 offen lds"
               :: "i"(4 * I), "i"(4 * I + 3), "v"(b), "v"(a), "s"(m0v), "v"(voff), "s"(rs), "s"(soff) : "memory");
}
__device__ __forceinline__ void w4_dma(uint32_t m0v, uint32_t voff, u32x4 rs, uint32_t soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(m0v), "v"(voff), "s"(rs), "s"(soff) : "memory");
}

// STAG > 0: K-start stagger (hipBLASLt's StaggerU idea): co-resident workgroup j of an XCD starts
// its K walk at K-tile (j % STAG) * ktiles / STAG and wraps, so the chip's simultaneous DMA
// requests spread over STAG K-columns instead of one.
// BOUT: B-outer MFMA order -- the B fragment (srcA) stays for 8 consecutive MFMAs while the A
// fragment (srcB) changes, hipBLASLt's operand order; the kk0 reads follow (b0, a0..a7, b1..b7).
template <class SC, int SERP = 0, bool ROT = false, bool SQ = false, bool ADMA = false, int STAG = 0,
          bool BOUT = false>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4t(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  static_assert(w4t_valid<SC>(), "schedule");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  if constexpr (SQ) tile_coords_sq(blockIdx.x, tiles_n, tm, tn);
  else tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K * 2u +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto mk_rs = [&](const __bf16* base) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    r[2] = panel_bytes;
    r[3] = 0x00020000u;
    return r;
  };
  const u32x4 sA = mk_rs(gA), sB = mk_rs(gB);
  auto dma_m0 = [&](int i, char* buf) -> uint32_t {
    const int rblk = ((i & 7) << 2) + wid;
    // the low 32 bits of a generic LDS address are the LDS offset (the shared aperture is the
    // high half): no addrspacecast, whose null check would cost a compare and select per piece
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)buf) + (uint32_t)((i >= 8 ? PANEL_BYTES : 0) + rblk * 1024);
  };
  auto dma_soff = [&](int i, int k0) -> uint32_t {
    const int rblk = ((i & 7) << 2) + wid;
    return (uint32_t)rblk * 8u * (uint32_t)K * 2u + (uint32_t)k0 * 2u;
  };
  auto dma_piece = [&](int i, int k0, char* buf) {
    if constexpr (ADMA) {
      w4_dma(dma_m0(i, buf), voff, i >= 8 ? sB : sA, dma_soff(i, k0));
    } else {
      const int rblk = ((i & 7) << 2) + wid;
      char* lds = buf + (i >= 8 ? PANEL_BYTES : 0) + rblk * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff,
                                               (uint32_t)rblk * 8u * (uint32_t)K * 2u + (uint32_t)k0 * 2u, 0, 0);
    }
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
  auto read_frag = [&](W4Frags& F, const char* buf, int kk, auto J) {      // consumption order
    constexpr int j = decltype(J)::value;
    // A-outer (w4_isb): a0, b0..b7, a1..a7; B-outer: b0, a0..a7, b1..b7
    constexpr bool isb = BOUT ? (j == 0 || j >= 9) : w4_isb(j);
    constexpr int x = BOUT ? (j == 0 ? 0 : (j <= 8 ? j - 1 : j - 8)) : w4_idx(j);
    if constexpr (isb)
      F.b[x] = *reinterpret_cast<const bf16x8*>(buf + b_off + x * 16 * ROW_BYTES + lane_off[kk]);
    else
      F.a[x] = *reinterpret_cast<const bf16x8*>(buf + a_off + x * 16 * ROW_BYTES + lane_off[kk]);
  };
  auto read_r1 = [&](const char* buf, auto J) {                             // A first, then B
    constexpr int j = decltype(J)::value;
    if constexpr (j >= 8)
      R1.b[j - 8] = *reinterpret_cast<const bf16x8*>(buf + b_off + (j - 8) * 16 * ROW_BYTES + lane_off[1]);
    else
      R1.a[j] = *reinterpret_cast<const bf16x8*>(buf + a_off + j * 16 * ROW_BYTES + lane_off[1]);
  };
  constexpr int issued = w4t_issued_by_w2<SC>();
  constexpr bool split = SC::ba != SC::bb;
  auto iter = [&](char* cur, char* nxt, int dk, auto DM, auto NX, auto LO, auto HI) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value;
    static_for<decltype(LO)::value, decltype(HI)::value>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int jr1 = w4t_r1_at<SC>(i), jdma = w4t_dma_at<SC>(i), jr0 = w4t_r0_at<SC>(i);
      constexpr bool fused = ADMA && dm && jdma >= 0;
      constexpr int s64 = i & 63;
      constexpr int ai = BOUT ? (s64 & 7) : (s64 >> 3), bi = BOUT ? (s64 >> 3) : (s64 & 7);
      constexpr int acc = ai * 8 + bi;                     // accumulator m*8+n (the epilogue's order)
      W4Frags& F = i < 64 ? R0 : R1;
      if constexpr (fused)
        w4_mfma_dma<acc>(F.b[bi], F.a[ai], dma_m0(jdma, cur), voff, jdma >= 8 ? sB : sA, dma_soff(jdma, dk));
      else
        w4_mfma<acc>(F.b[bi], F.a[ai]);
      if constexpr (jr1 >= 0) read_r1(cur, std::integral_constant<int, jr1>{});
      if constexpr (i == SC::wa || (split && i == SC::wb)) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      if constexpr (dm && (i == SC::ba || (split && i == SC::bb))) __builtin_amdgcn_s_barrier();
      if constexpr (!fused && dm && jdma >= 0) dma_piece(jdma, dk, cur);
      if constexpr (nx && i == SC::w2) {
        constexpr int n = dm ? issued : 0;
        __builtin_amdgcn_s_waitcnt((n & 15) | ((n >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == SC::b2) __builtin_amdgcn_s_barrier();
      if constexpr (nx && jr0 >= 0) read_frag(R0, nxt, 0, std::integral_constant<int, jr0>{});
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int ktiles = K / BK;        // >= 2 (host guarantees)
  const bool rev = SERP > 0 && (((int)blockIdx.x / NXCD) / (SERP > 0 ? SERP : 1)) & 1;
  const int kst = STAG > 0 ? ((((int)blockIdx.x / NXCD) % (STAG > 0 ? STAG : 1)) * ktiles) / (STAG > 0 ? STAG : 1) : 0;
  auto kof = [&](int kt) {
    int k = (rev ? ktiles - 1 - kt : kt) + kst;
    if (STAG > 0 && k >= ktiles) k -= ktiles;
    return k * BK;
  };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(0), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(1), buf1);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): tile 0 landed, tile 1 in flight
  bar();
  static_for<0, 16>([&](auto J) { read_frag(R0, buf0, 0, J); });

  using S0 = std::integral_constant<int, 0>;
  using SB = std::integral_constant<int, SC::ba>;
  using SE = std::integral_constant<int, 128>;
  char* cur = buf0;
  char* nxt = buf1;
  if constexpr (ROT) {
    iter(cur, nxt, 0, T_{}, T_{}, S0{}, SB{});
    for (int t = 0; t < ktiles - 2; ++t) {
      iter(cur, nxt, kof(t + 2), T_{}, T_{}, SB{}, SE{});
      char* tmp = cur; cur = nxt; nxt = tmp;
      iter(cur, nxt, 0, T_{}, T_{}, S0{}, SB{});
    }
    iter(cur, nxt, 0, F_{}, T_{}, SB{}, SE{});
    iter(nxt, nullptr, 0, F_{}, F_{}, S0{}, SE{});
  } else {
    for (int t = 0; t < ktiles - 2; ++t) {
      iter(cur, nxt, kof(t + 2), T_{}, T_{}, S0{}, SE{});
      char* tmp = cur; cur = nxt; nxt = tmp;
    }
    iter(cur, nxt, 0, F_{}, T_{}, S0{}, SE{});
    iter(nxt, nullptr, 0, F_{}, F_{}, S0{}, SE{});
  }

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
    store_c16(C + (size_t)(tm * BM + r) * N + tn * BN + ch * 8, v);
  }
}

// w4a: the w4s kernel (v44 configuration: serpentine K, VK) with its whole K pipeline -- prologue
// DMA, steady-state loop unrolled over the two LDS buffers, two-tile drain -- as ONE hand-scheduled
// asm block generated by tools/gen_bf16_asm_loop.py (native/hip/gemm_bf16_asm_loop.h; the header
// comment there has the register map and the wait/barrier protocol). Same MFMA order, operands and
// accumulators as w4s: the results are bitwise those of v44. SC selects the schedule (the index list
// is in gemm_bf16_asm_loop.h). Host guarantees: K % 128 == 0 and K >= 256 (an even number of
// K-tiles, at least one loop trip).
#define W4A_LOOP(TEXT)                                                                                       \
  asm volatile("s_mov_b32 %[m0save], m0\n\t" TEXT "s_mov_b32 m0, %[m0save]"                                  \
               : [voff] "+v"(voff_k), [cnt] "+s"(trips), [m0save] "=&s"(m0save)                               \
               : [ra00] "v"(ra00), [rb00] "v"(rb00), [ra01] "v"(ra01), [rb01] "v"(rb01), [ra10] "v"(ra10),      \
                 [rb10] "v"(rb10), [ra11] "v"(ra11), [rb11] "v"(rb11), [kstep] "s"(kstep), [s0] "s"(so[0]),     \
                 [s1] "s"(so[1]), [s2] "s"(so[2]), [s3] "s"(so[3]), [s4] "s"(so[4]), [s5] "s"(so[5]),           \
                 [s6] "s"(so[6]), [s7] "s"(so[7]), [rA] "s"(sA), [rB] "s"(sB), [m0b0] "s"(m0b0), [m0b1] "s"(m0b1) \
               : "memory", "scc", W4A_VCLOBBERS, W4_AGPR_CLOBBERS)

template <int SC = 0, int SERP = 32, bool SQ = false>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4a(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  if constexpr (SQ) tile_coords_sq(blockIdx.x, tiles_n, tm, tn);
  else tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const __bf16* gA = A + (size_t)tm * BM * K;
  const __bf16* gB = Bt + (size_t)tn * BN * K;
  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  auto mk_rs = [&](const __bf16* base) {
    const uint64_t p = (uint64_t)(uintptr_t)base;
    w4a_u32x4 r;
    r[0] = __builtin_amdgcn_readfirstlane((uint32_t)p);
    r[1] = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
    r[2] = panel_bytes;
    r[3] = 0x00020000u;
    return r;
  };
  const w4a_u32x4 sA = mk_rs(gA), sB = mk_rs(gB);
  const int par = wid & 1;
  const int ktiles = K / BK;
  // serpentine K (v44): every other dispatch wave of an XCD walks K backwards
  const bool rev = SERP > 0 && (((int)blockIdx.x / NXCD) / (SERP > 0 ? SERP : 1)) & 1;
  const int kstep = rev ? -2 * BK : 2 * BK;                       // bytes per K-tile
  uint32_t voff_k = (uint32_t)(lane >> 3) * (uint32_t)K * 2u +
                    (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16) +
                    (uint32_t)((rev ? ktiles - 1 : 0) * BK * 2);   // K offset of tile 0
  uint32_t so[8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
    so[i] = __builtin_amdgcn_readfirstlane((uint32_t)((i << 2) + wid) * 8u * (uint32_t)K * 2u);
  // the low 32 bits of a generic LDS address are the LDS offset
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)smem);
  const uint32_t m0b0 = lds0 + (uint32_t)wid * 1024u, m0b1 = m0b0 + (uint32_t)BUF_BYTES;

  int lane_off[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int r = lane & 15;
    const int c = kk * 4 + (lane >> 4);
    lane_off[kk] = r * ROW_BYTES + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const uint32_t a_base = lds0 + (uint32_t)(wr * 128 * ROW_BYTES);
  const uint32_t b_base = lds0 + (uint32_t)(PANEL_BYTES + wc * 128 * ROW_BYTES);
  const uint32_t ra00 = a_base + lane_off[0], rb00 = b_base + lane_off[0];
  const uint32_t ra01 = a_base + lane_off[1], rb01 = b_base + lane_off[1];
  const uint32_t ra10 = ra00 + BUF_BYTES, rb10 = rb00 + BUF_BYTES;
  const uint32_t ra11 = ra01 + BUF_BYTES, rb11 = rb01 + BUF_BYTES;
  uint32_t trips = __builtin_amdgcn_readfirstlane((uint32_t)((ktiles - 2) >> 1));
  uint32_t m0save;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });
  W4A_LOOP_SELECT(SC)

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
    store_c16(C + (size_t)(tm * BM + r) * N + tn * BN + ch * 8, v);
  }
}

// w4ap (v50-v52): w4a made persistent; the frame is shared with the fp8 kernel (gemm_w4ap.h).
template <int SC = 0, bool SERP = true, bool SQ = false, int EPI = 0, int DM = 0, Rec REC = kTimed>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4ap(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                       __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[W4AP_LDS];
  note_placement<REC>();
  w4ap_run<SC, SERP, SQ, false, EPI, DM>((const char*)A, (const char*)Bt, C, M, N, K, smem);
}

// w4ap split-K (v57): one (tile, K piece) per workgroup, the piece sums reduced by each tile's last
// arriving waves (gemm_w4ap.h SPLIT). ws / cnt: gemm_small_host.h's per-(device, stream) workspace.
template <int SC, int EPI, int DM, Rec REC = kTimed, int SKO = 0>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4ap_sk(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt, __bf16* __restrict__ C,
                          int M, int N, int K, int splits, float* __restrict__ ws, int* __restrict__ cnt,
                          int last_pairs, int pmajor) {
  __shared__ __attribute__((aligned(16))) char smem[W4AP_LDS];
  note_placement<REC>();
  w4ap_run<SC, false, false, false, EPI, DM, true, SKO>((const char*)A, (const char*)Bt, C, M, N, K, smem,
                                                   W4Split{splits, ws, cnt, last_pairs, pmajor});
}

// v25/v26: v18 made persistent. gridDim = one workgroup per CU; XCD x (= blockIdx % 8) owns a
// contiguous run of output tiles (the bijective split of xcd_remap) that its gridDim/8
// workgroups walk in strides. The K-tile stream runs on across tile boundaries: the last two
// K-iterations of a tile DMA the NEXT tile's K-tiles 0 and 1 into the freed buffers and the last
// one already reads its first fragments, so the next tile starts without a cold HBM prologue.
// The epilogue no longer needs the K buffers: each wave stages its own 128x128 sub-tile through a
// private 8 KiB slice of the 32 KiB of LDS the K buffers leave free (2 fragment rows = 32 C rows
// per pass, XOR-swizzled, read back as full 256-B row segments), so it needs no workgroup barrier
// and overlaps the in-flight DMA; the accumulators are zeroed as they are read.
constexpr int W4P_EPI_WAVE = 8192;                       // 32 rows x 128 cols x bf16
constexpr int W4P_LDS = LDS_BYTES + 4 * W4P_EPI_WAVE;     // 160 KiB

template <int B1 = 17, int D0 = 19, int DS = 5, int B2 = 80, int RS = 40, bool SERP = false, bool VK = false,
          Rec REC = kTimed>
__global__ void __launch_bounds__(W4_THREADS, 1)
gemm_bf16_256x256_w4sp(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                       __bf16* __restrict__ C, int M, int N, int K) {
  static_assert(B1 >= 16 && D0 > B1 && D0 + 15 * DS < 127 && B2 > B1 && B2 + RS < 127, "schedule");
  __shared__ __attribute__((aligned(16))) char smem[W4P_LDS];
  note_placement<REC>();

  const int tiles_m = M / BM;
  const int tiles_n = N / BN;
  const int nwg = tiles_m * tiles_n;
  const int xcd = blockIdx.x % NXCD;
  const int per = gridDim.x / NXCD;                       // workgroups per XCD (host: gridDim % 8 == 0)
  const int q = nwg / NXCD, rem = nwg % NXCD;
  const int t_begin = (xcd < rem) ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q;
  const int t_end = t_begin + q + (xcd < rem ? 1 : 0);
  int tile = t_begin + (int)(blockIdx.x / NXCD);
  if (tile >= t_end) return;                              // uniform over the workgroup

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const uint32_t panel_bytes = (uint32_t)BM * (uint32_t)K * 2u;
  auto rsrc = [&](const __bf16* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, panel_bytes, 0x00020000);
  };
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, tm, tn);
  __amdgpu_buffer_rsrc_t rA = rsrc(A + (size_t)tm * BM * K);
  __amdgpu_buffer_rsrc_t rB = rsrc(Bt + (size_t)tn * BN * K);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K * 2u +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int k0, char* buf) {
    // piece p = 4i + wid; p >= 32 (the B panel) <=> i >= 8, a compile-time fact once unrolled
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? PANEL_BYTES : 0) + rblk * 1024;
    if constexpr (VK)   // K offset in the lane offset, loop-invariant soffsets (as w4s VK)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rb : ra, (lds_void*)lds, 16, voff + (uint32_t)k0 * 2u,
                                               (uint32_t)rblk * 8u * (uint32_t)K * 2u, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rb : ra, (lds_void*)lds, 16, voff,
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
  // The v18 iteration; the DMA target (operand panels and K offset) is a runtime argument so the
  // same body serves this tile's K-tile t+2 and the next tile's K-tiles 0 and 1.
  // FRESH: a tile's first iteration. The vmcnt(0) before it (prologue or previous epilogue) already
  // retired this tile's K-tile 1, so its B2 does not wait again: the epilogue's C stores are older
  // than this iteration's DMA, and a counted vmcnt would wait for them too.
  auto iter = [&](char* cur, char* nxt, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int dk, auto FR,
                  auto DM, auto NX) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value, fresh = decltype(FR)::value;
    static_for<0, 128>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 64) w4_mfma<i>(R0.b[i & 7], R0.a[i >> 3]);
      else w4_mfma<i - 64>(R1.b[i & 7], R1.a[(i - 64) >> 3]);
      if constexpr (i < 16) read_frag(R1, cur, 1, std::integral_constant<int, i>{});
      if constexpr (dm && i == B1 - 1) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      if constexpr (dm && i == B1) __builtin_amdgcn_s_barrier();
      if constexpr (dm && i >= D0 && (i - D0) % DS == 0 && (i - D0) / DS < 16) dma_piece((i - D0) / DS, ra, rb, dk, cur);
      if constexpr (nx && i == B2 - 1) {
        constexpr int issued = !dm ? 0 : (B2 - 1 < D0 ? 0 : ((B2 - 1 - D0) / DS + 1 > 16 ? 16 : (B2 - 1 - D0) / DS + 1));
        if constexpr (fresh) __builtin_amdgcn_s_waitcnt(0xC07F);             // lgkmcnt(0) only
        else __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == B2) __builtin_amdgcn_s_barrier();
      constexpr int jr0 = w4s_r0_at(B2, RS, i);
      if constexpr (nx && jr0 >= 0) read_frag(R0, nxt, 0, std::integral_constant<int, jr0>{});
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  // Wave-private epilogue: 4 passes of 2 fragment rows (32 C rows x 128 cols).
  char* const stg = smem + LDS_BYTES + wid * W4P_EPI_WAVE;
  auto epilogue = [&](int tm_, int tn_) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // last MFMA D -> accvgpr reads
    static_for<0, 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      static_for<0, 16>([&](auto I) {
        constexpr int u = decltype(I)::value;
        constexpr int mm = u >> 3, n = u & 7;
        constexpr int i = (2 * s + mm) * 8 + n;                    // accumulator index m*8+n
        float x0, x1, x2, x3;
        asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                     "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7\n\t"
                     "v_accvgpr_write_b32 a%c4, 0\n\tv_accvgpr_write_b32 a%c5, 0\n\t"
                     "v_accvgpr_write_b32 a%c6, 0\n\tv_accvgpr_write_b32 a%c7, 0"
                     : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                     : "i"(4 * i), "i"(4 * i + 1), "i"(4 * i + 2), "i"(4 * i + 3));
        const int r = mm * 16 + (lane & 15);                       // 0..31
        const int g = n * 4 + (lane >> 4);                         // 8-byte group 0..31
        bf16x4 v;
        v[0] = (__bf16)x0;
        v[1] = (__bf16)x1;
        v[2] = (__bf16)x2;
        v[3] = (__bf16)x3;
        *reinterpret_cast<bf16x4*>(stg + r * 256 + ((g ^ (r & 15)) << 3)) = v;
      });
      asm volatile("" ::: "memory");     // a wave's LDS ops execute in order: no wait, no barrier
      // retire the next tile's K-tile DMAs before the first C store (see `fresh`)
      if constexpr (s == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = k * 4 + (lane >> 4);
        const int ch = lane & 15;
        const int sw = r & 15;
        const int pg = (2 * ch) ^ sw;
        const uint4 raw = *reinterpret_cast<const uint4*>(stg + r * 256 + ((pg & ~1) << 3));
        uint4 v = raw;
        if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
        store_c16(C + (size_t)(tm_ * BM + wr * 128 + s * 32 + r) * N + tn_ * BN + wc * 128 + ch * 8, v);
      }
      asm volatile("" ::: "memory");
    });
  };

  const int ktiles = K / BK;        // >= 2 (host guarantees)
  // SERP (v27): a workgroup's i-th tile belongs to wave i of its XCD; odd waves walk K backwards
  // and start on the A-panel K-slices the previous wave left in the XCD's L2.
  bool rev = false;
  auto kof = [&](int kt, bool r) { return (r ? ktiles - 1 - kt : kt) * BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(0, rev), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(1, rev), buf1);
  __builtin_amdgcn_s_waitcnt(0x0070);               // vmcnt(0): K-tiles 0 and 1 landed (FRESH iteration)
  bar();
  static_for<0, 16>([&](auto J) { read_frag(R0, buf0, 0, J); });

  char* cur = buf0;
  char* nxt = buf1;
  for (;;) {
    const int next = tile + per;
    const bool has_next = next < t_end;
    int ntm = tm, ntn = tn;
    __amdgpu_buffer_rsrc_t nA = rA, nB = rB;
    if (has_next) {
      tile_coords(next, tiles_m, tiles_n, ntm, ntn);
      nA = rsrc(A + (size_t)ntm * BM * K);
      nB = rsrc(Bt + (size_t)ntn * BN * K);
    }
    const int nsteady = has_next ? ktiles : ktiles - 2;
    auto dma_of = [&](int t, __amdgpu_buffer_rsrc_t& ra, __amdgpu_buffer_rsrc_t& rb) {
      const bool nt = t + 2 >= ktiles;               // DMA the next tile's K-tile t+2-ktiles
      ra = nt ? nA : rA;
      rb = nt ? nB : rB;
      return nt ? kof(t + 2 - ktiles, SERP && !rev) : kof(t + 2, rev);
    };
    __amdgpu_buffer_rsrc_t ra, rb;
    if (nsteady > 0) {
      const int dk = dma_of(0, ra, rb);
      iter(cur, nxt, ra, rb, dk, T_{}, T_{}, T_{});
      char* tmp = cur; cur = nxt; nxt = tmp;
    }
    for (int t = 1; t < nsteady; ++t) {
      const int dk = dma_of(t, ra, rb);
      iter(cur, nxt, ra, rb, dk, F_{}, T_{}, T_{});
      char* tmp = cur; cur = nxt; nxt = tmp;
    }
    if (!has_next) {
      iter(cur, nxt, rA, rB, 0, F_{}, F_{}, T_{});
      iter(nxt, nullptr, rA, rB, 0, F_{}, F_{}, F_{});
    }
    epilogue(tm, tn);
    if (!has_next) break;
    tile = next;
    rev = SERP && !rev;
    tm = ntm;
    tn = ntn;
    rA = nA;
    rB = nB;
  }
}
// Generic bounds-checked MFMA kernel (64x64 tile, 4 waves of 32x32), register-staged.
// Used for shapes that are not multiples of 256/256/64 and as a second, independent
// implementation for cross-checking the fast path.
constexpr int GBM = 64, GBN = 64, GBK = 32;

template <Rec REC = kTimed>
__global__ void __launch_bounds__(256)
gemm_bf16_generic(const __bf16* __restrict__ A, const __bf16* __restrict__ Bt,
                  __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) __bf16 sa[GBM][GBK + 8];
  __shared__ __attribute__((aligned(16))) __bf16 sb[GBN][GBK + 8];
  note_placement<REC>();
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // 256 threads x 8 elements = 64 rows x 32 k per operand.
  const int lr = threadIdx.x >> 2;        // row 0..63
  const int lk = (threadIdx.x & 3) * 8;   // k offset 0,8,16,24
  for (int k0 = 0; k0 < K; k0 += GBK) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = k0 + lk + e;
      const int ra = m0 + lr, rb = n0 + lr;
      sa[lr][lk + e] = (ra < M && k < K) ? A[(size_t)ra * K + k] : (__bf16)0.f;
      sb[lr][lk + e] = (rb < N && k < K) ? Bt[(size_t)rb * K + k] : (__bf16)0.f;
    }
    __syncthreads();
    bf16x8 af[2], bfr[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        af[i][e] = sa[wr * 32 + i * 16 + (lane & 15)][8 * (lane >> 4) + e];
        bfr[i][e] = sb[wc * 32 + i * 16 + (lane & 15)][8 * (lane >> 4) + e];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wr * 32 + i * 16 + (lane & 15);
        const int col = n0 + wc * 32 + j * 16 + 4 * (lane >> 4) + e;
        if (row < M && col < N) C[(size_t)row * N + col] = (__bf16)acc[i][j][e];
      }
}

// Deterministic uniform [-1,1) bf16 fill (counter-based hash), so validator runs on
// random data (zero-filled operands inflate MFMA clocks and hide layout bugs).
__global__ void fill_uniform_bf16(__bf16* p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const float u = (float)(x >> 8) * (1.0f / 16777216.0f);
    p[i] = (__bf16)(2.0f * u - 1.0f);
  }
}

}  // namespace
