// CDNA4 (gfx950) fp8 GEMM for the node validator workload: the matrix cores at their fp8 rate.
//
//   C[M,N] (bf16) = A[M,K] (fp8 e4m3fn, K-major) * Bt[N,K]^T (fp8 e4m3fn, K-major), fp32 accumulation.
//
// gfx950 runs fp8 at twice the bf16 rate through the f8f6f4 MFMA family, scaled
// (`v_mfma_scale_f32_32x32x64_f8f6f4`) or not (`v_mfma_f32_16x16x128_f8f6f4`); the older
// `*_fp8_fp8` forms run at the bf16 rate. OCP e4m3fn encoding (not MI300's fnuz).
//   * gemm_fp8_256x256_q16  -- the production kernel (gemm_fp8.hip v15/v16/v17): unscaled
//                              16x16x128, described at its definition below;
//   * gemm_fp8_256x256_w4sp -- persistent, block-scaled with unit E8M0 scales (v10, short K);
//   * gemm_fp8_256x256_w4s  -- the round-1 block-scaled kernel (lab only), described next.
//
// w4s design: the bf16 v18 kernel's schedule (gemm_bf16.hip, docs/validator-gemm.md) carried over in
// bytes. A K-tile is 128 fp8 = the same 128-byte LDS row as 64 bf16, so the LDS image, the
// buffer_load...lds DMA pieces, the XOR swizzle and the 2x2 wave grid (4 wave64s, one per SIMD,
// each owning a 128x128 sub-tile of the 256x256 workgroup tile) are unchanged. What changes:
//   * a wave's 128x128 sub-tile is 4x4 MFMAs of 32x32 (16 AGPRs each, all 256 AGPRs), so a K-tile
//     is 32 MFMA slots -- 16 on k-half 0 (register set R0), 16 on k-half 1 (R1) -- each 4x the
//     matrix-pipe time of a bf16 16x16x32 slot: the same time per K-tile for twice the FLOPs;
//   * a fragment is 32 bytes per lane (8 VGPRs = two ds_read_b128): lane l holds row l & 31 and
//     the two 16-byte chunks 2(l >> 5), 2(l >> 5) + 1 of its k-half. Which k the hardware assigns
//     to each byte does not matter: A and B use the same lane->k map, so any consistent
//     permutation of k inside a k-half sums the same products;
//   * the epilogue reads the 32x32 C/D layout (col = lane & 31, row = (reg & 3) + 8 (reg >> 2) +
//     4 (lane >> 5)); with Bt as the MFMA's "A" operand each lane holds 4 consecutive N columns of
//     one output row, staged through LDS for fully coalesced 16-byte row stores as in v18.
// Schedule per K-tile t (slots = MFMA issue positions 0..31, template parameters):
//   slots 0..3        read R1 <- tile t k-half 1 (two fragments per slot)
//   slot  B1          lgkmcnt(0) one slot earlier, then a barrier: every wave is done with tile t
//   slots D0..        DMA tile t+2 into tile t's buffer (16 1-KiB pieces spread over DSPAN slots)
//   slot  B2          vmcnt(pieces issued so far) one slot earlier -- tile t+1 landed -- then a barrier
//   slots B2+1..      read R0 <- tile t+1 k-half 0, spread over RS slots
// A bounds-checked generic kernel (software e4m3 decode, fp32 FMA) handles other shapes and is
// the independent implementation the tests compare against.

#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gemm_tile_common.h"
#include "gemm_w4ap.h"

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

constexpr int F8_BM = 256;
constexpr int F8_BN = 256;
constexpr int F8_BK = 128;                       // elements = bytes
constexpr int F8_ROW = F8_BK;                    // 128 B per staged row
constexpr int F8_PANEL = F8_BM * F8_ROW;         // 32 KiB per operand per K-tile
constexpr int F8_BUF = 2 * F8_PANEL;             // A + B
constexpr int F8_LDS = 2 * F8_BUF;               // double buffered: 128 KiB
constexpr int F8_THREADS = 256;
constexpr int E8M0_ONE = 127;                    // block scale 2^0

struct F8Frags {
  i32x8 a[4];
  i32x8 b[4];
};

// acc q (a[16q .. 16q+15]) += Bt fragment (as "A") x A fragment (as "B"), both e4m3, unit scales.
template <int Q>
__device__ __forceinline__ void f8_mfma(const i32x8& b, const i32x8& a, int scale) {
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 a[%c0:%c1], %2, %3, a[%c0:%c1], %4, %4 op_sel_hi:[0,0,0]"
               :: "i"(16 * Q), "i"(16 * Q + 15), "v"(b), "v"(a), "v"(scale));
}

// Fragment read order j -> (A or B, index). The registers overwritten first are the ones whose
// last MFMA use is oldest (a0..a2 before b0..b2, a3/b3 last): reads of a k-half start right after
// the previous k-half's final MFMAs, which still name a3 and b3.
__device__ __forceinline__ constexpr int f8_isb(int j) { return j >= 3 && j != 6; }
__device__ __forceinline__ constexpr int f8_idx(int j) {
  return j < 3 ? j : (j < 6 ? j - 3 : 3);
}

template <int B1 = 5, int D0 = 5, int DSPAN = 16, int B2 = 20, int RS = 10, int SERP = 0, bool ROT = false,
          bool SQ = false>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_w4s(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                     __bf16* __restrict__ C, int M, int N, int K) {
  constexpr int SLOTS = 32;
  static_assert(B1 >= 4 && D0 >= B1 && D0 + DSPAN <= SLOTS && B2 >= 16 && B2 > B1 && B2 + RS < SLOTS,
                "schedule");
  __shared__ __attribute__((aligned(16))) char smem[F8_LDS];

  const int tiles_m = M / F8_BM;
  const int tiles_n = N / F8_BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  if constexpr (SQ) tile_coords_sq(blockIdx.x, tiles_n, tm, tn);   // square cross-XCD raster (v13)
  else tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const uint8_t* gA = A + (size_t)tm * F8_BM * K;
  const uint8_t* gB = Bt + (size_t)tn * F8_BN * K;
  const uint32_t panel_bytes = (uint32_t)F8_BM * (uint32_t)K;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  // wave w issues pieces p = 4i + w: A row blocks 0..31 (i < 8), then B. Every piece it issues has
  // row-block parity w & 1, so one per-lane voffset (row lane>>3, swizzled chunk) serves them all.
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, int k0, char* buf) {
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? F8_PANEL : 0) + rblk * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff,
                                             (uint32_t)rblk * 8u * (uint32_t)K + (uint32_t)k0, 0, 0);
  };

  // lane_off[kh][s]: byte offset of the lane's 16-byte chunk s of k-half kh in a 32-row fragment
  int lane_off[2][2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = lane & 31;
      const int c = kh * 4 + 2 * (lane >> 5) + s;
      lane_off[kh][s] = r * F8_ROW + ((c ^ ((r >> 1) & 7)) << 4);
    }
  const int a_off = wr * 128 * F8_ROW;
  const int b_off = F8_PANEL + wc * 128 * F8_ROW;
  const int scale = E8M0_ONE;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  F8Frags R0, R1;
  char* const buf0 = smem;
  char* const buf1 = smem + F8_BUF;
  auto read_frag = [&](F8Frags& F, const char* buf, int kh, auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int x = f8_idx(j);
    const char* base = buf + (f8_isb(j) ? b_off : a_off) + x * 32 * F8_ROW;
    const i32x4 lo = *reinterpret_cast<const i32x4*>(base + lane_off[kh][0]);
    const i32x4 hi = *reinterpret_cast<const i32x4*>(base + lane_off[kh][1]);
    const i32x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    if constexpr (f8_isb(j)) F.b[x] = v;
    else F.a[x] = v;
  };
  // slots [LO, HI) of one K-tile iteration; the slots before B1 depend on no flag (ROT splits there)
  auto iter = [&](char* cur, char* nxt, int dk, auto DM, auto NX, auto LO, auto HI) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value;
    static_for<decltype(LO)::value, decltype(HI)::value>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 16) f8_mfma<i>(R0.b[i & 3], R0.a[i >> 2], scale);
      else f8_mfma<i - 16>(R1.b[i & 3], R1.a[(i - 16) >> 2], scale);
      if constexpr (i < 4) {
        read_frag(R1, cur, 1, std::integral_constant<int, 2 * i>{});
        read_frag(R1, cur, 1, std::integral_constant<int, 2 * i + 1>{});
      }
      if constexpr (i == B1 - 1) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      if constexpr (dm && i == B1) __builtin_amdgcn_s_barrier();
      if constexpr (dm) {
        static_for<0, 16>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (D0 + (j * DSPAN) / 16 == i) dma_piece(j, dk, cur);
        });
      }
      if constexpr (nx && i == B2 - 1) {
        constexpr int issued = [] {
          int n = 0;
          for (int j = 0; j < 16; ++j) n += (dm && D0 + (j * DSPAN) / 16 <= B2 - 1) ? 1 : 0;
          return n;
        }();
        // vmcnt(issued) lgkmcnt(0): vmcnt low 4 bits [3:0], high 2 bits [15:14]; expcnt 7
        __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == B2) __builtin_amdgcn_s_barrier();
      if constexpr (nx && i > B2) {
        static_for<0, 8>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (B2 + 1 + (j * RS) / 8 == i) read_frag(R0, nxt, 0, J);
        });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int ktiles = K / F8_BK;     // >= 2 (host guarantees)
  // SERP > 0 (serpentine K): with SERP co-resident workgroups per XCD, every other wave of tiles
  // walks K backwards, starting on the A-panel K-slices the previous wave left in the XCD's L2.
  const bool rev = SERP > 0 && (((int)blockIdx.x / NXCD) / (SERP > 0 ? SERP : 1)) & 1;
  auto kof = [&](int kt) { return (rev ? ktiles - 1 - kt : kt) * F8_BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(0), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(1), buf1);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): tile 0 landed, tile 1 in flight
  bar();
  static_for<0, 8>([&](auto J) { read_frag(R0, buf0, 0, J); });

  using S0 = std::integral_constant<int, 0>;
  using SB = std::integral_constant<int, B1>;
  using SE = std::integral_constant<int, SLOTS>;
  char* cur = buf0;
  char* nxt = buf1;
  if constexpr (ROT) {
    // Loop rotation: an iteration runs slots B1..31 of tile t, then slots 0..B1-1 of tile t+1, so
    // the back-edge sits right after the explicit lgkmcnt(0) at slot B1-1. Unrotated, the
    // back-edge falls just after the R0 reads and hipcc's merged wait state at the loop header
    // is a blanket lgkmcnt(0) before the first MFMA, which stalls on the newest read.
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

  // epilogue through LDS; pad the last MFMA's D before the accumulator reads
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  bar();
  constexpr int CROW = F8_BN * 2;
  static_for<0, 64>([&](auto I) {
    constexpr int i = decltype(I)::value;
    constexpr int q = i >> 2, g = i & 3;              // accumulator q = 4 i_m + i_n, register group g
    constexpr int im = q >> 2, in = q & 3;
    float x0, x1, x2, x3;
    asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                 "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7"
                 : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                 : "i"(16 * q + 4 * g), "i"(16 * q + 4 * g + 1), "i"(16 * q + 4 * g + 2),
                   "i"(16 * q + 4 * g + 3));
    const int r = wr * 128 + im * 32 + (lane & 31);
    const int gc = (wc * 128 + in * 32 + 8 * g + 4 * (lane >> 5)) >> 2;
    bf16x4 v;
    v[0] = (__bf16)x0;
    v[1] = (__bf16)x1;
    v[2] = (__bf16)x2;
    v[3] = (__bf16)x3;
    *reinterpret_cast<bf16x4*>(smem + r * CROW + ((gc ^ (r & 15)) << 3)) = v;
  });
  bar();
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < (F8_BM * F8_BN * 2) / (F8_THREADS * 16); ++i) {
    const int r = i * (F8_THREADS / 32) + (tid >> 5);
    const int ch = tid & 31;
    const int sw = r & 15;
    const int pg = (2 * ch) ^ sw;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + r * CROW + ((pg & ~1) << 3));
    uint4 v = raw;
    if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
    store_c16(C + (size_t)(tm * F8_BM + r) * N + tn * F8_BN + ch * 8, v);
  }
}

// q16: fp8 on the UNSCALED double-rate `v_mfma_f32_16x16x128_f8f6f4` (gfx950's f8f6f4 family runs
// fp8 at twice the bf16 rate with or without the block scales; the older `*_fp8_fp8` forms are
// the bf16-rate ones). hipBLASLt's gfx950 fp8 kernel (MT256x256x128, MI 16x16x128) is built on
// it. The 16x16 output shape is also the one that holds clocks better under the power limit
// (MI355X_MICROARCH.md, DVFS give-back item 7).
// A wave's 128x128 sub-tile is 8x8 MFMAs of 16x16 (the bf16 w4s accumulator layout, so the bf16
// epilogue applies as is). A fragment is 16 rows x 128 k = 32 B per lane (8 VGPRs, two
// ds_read_b128: chunks g and g+4 of the 128-B row for lane group g = lane >> 4). A K-tile needs
// 8 A + 8 B fragments = 128 VGPRs -- exactly one set, no double buffer -- because the 64 MFMAs run
// in quarter blocks that free half of the fragments early:
//   slots  0..15  B0 x A0      B0 = b0..3, B1 = b4..7, A0 = a0..3, A1 = a4..7
//   slots 16..31  B0 x A1      B0 is dead after slot 31
//   slots 32..47  B1 x A0      A0 is dead after slot 47
//   slots 48..63  B1 x A1
// and the reads: A1, B1 of tile t at slots 0..15 (their registers died at the previous tile's
// slot 63); B0, A0 of tile t+1 after their last use (slots RB0.., RA0..). Barriers: after the A1/B1
// reads every wave is done with tile t (DMA of tile t+2 may overwrite it); before B0' the
// landing wait for tile t+1.
// Which two 16-byte chunks of a 128-byte K-row lane group g (= lane >> 4) holds, h = 0 / 1.
// Any lane -> k map gives the same sums as long as A and B use the same one, so it is chosen
// for the LDS banks: gfx950 serves a ds_read_b128 32 lanes at a time from 128 banks (512 B), so
// the two lane groups of a pass (g = 0, 1 or 2, 3) must read chunks of opposite parity -- under the
// (R >> 1) & 7 row swizzle, chunks 2g / 2g+1 (0 and 2 in one pass) put two lanes on every bank
// (SQ_LDS_BANK_CONFLICT = half of SQ_LDS_IDX_ACTIVE, profiles/r3_pmc), chunks g / g+4 none (the
// bf16 kernels' kk*4 + g pattern).
#define F8Q_CHUNK(g, h) ((g) + 4 * (h))

template <int I>
__device__ __forceinline__ void f8q_mfma(const i32x8& b, const i32x8& a) {
  asm volatile("v_mfma_f32_16x16x128_f8f6f4 a[%c0:%c1], %2, %3, a[%c0:%c1]"
               :: "i"(4 * I), "i"(4 * I + 3), "v"(b), "v"(a));
}

// Schedule parameters: W1 = lgkmcnt(0) slot (barrier at W1 + 1: tile t's buffer is free); DMA piece
// j of tile t+2 at slot D0 + j DS; W2 = landing wait for tile t+1 (barrier at W2 + 1); B0' fragment j
// read at RB0 + j RBS, A0' fragment j at RA0 + j RAS. ASLOW: block 2 (B1 x A0) walks A0 slowly, so
// a0 dies at slot 35, a1 at 39, ... (else every A0 fragment lives to slot 47). Block 1 always walks
// B0 slowly (b0 dies at slot 19, b1 at 23, ...).
template <int W1 = 16, int D0 = 18, int DS = 1, int W2 = 34, int RB0 = 36, int RA0 = 48, int SERP = 0,
          bool SQ = false, int RBS = 2, int RAS = 2, bool ASLOW = false, bool VK = false, Rec REC = kTimed>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_q16(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                     __bf16* __restrict__ C, int M, int N, int K) {
  note_placement<REC>();
  constexpr int SLOTS = 64;
  constexpr auto rb_ok = [] {
    for (int j = 0; j < 4; ++j) {
      if (RB0 + j * RBS <= 19 + 4 * j || RB0 + j * RBS >= SLOTS) return false;     // b_j dead, in range
      const int ra = RA0 + j * RAS;
      if (ra <= (ASLOW ? 35 + 4 * j : 47) || ra >= SLOTS) return false;             // a_j dead, in range
    }
    return true;
  }();
  static_assert(W1 >= 15 && D0 > W1 && D0 + 15 * DS < SLOTS && W2 > W1 && RB0 > W2 && RA0 > W2 && rb_ok,
                "schedule");
  __shared__ __attribute__((aligned(16))) char smem[F8_LDS];

  const int tiles_m = M / F8_BM;
  const int tiles_n = N / F8_BN;
  const int nwg = tiles_m * tiles_n;
  int tm, tn;
  if constexpr (SQ) tile_coords_sq(blockIdx.x, tiles_n, tm, tn);
  else tile_coords(xcd_remap(blockIdx.x, nwg), tiles_m, tiles_n, tm, tn);

  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wid >> 1, wc = wid & 1;

  const uint8_t* gA = A + (size_t)tm * F8_BM * K;
  const uint8_t* gB = Bt + (size_t)tn * F8_BN * K;
  const uint32_t panel_bytes = (uint32_t)F8_BM * (uint32_t)K;
  __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)gA, 0, panel_bytes, 0x00020000);
  __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)gB, 0, panel_bytes, 0x00020000);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, int k0, char* buf) {
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? F8_PANEL : 0) + rblk * 1024;
    if constexpr (VK)   // K offset in the lane offset: loop-invariant soffsets (as bf16 w4s VK)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff + (uint32_t)k0,
                                               (uint32_t)rblk * 8u * (uint32_t)K, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rB : rA, (lds_void*)lds, 16, voff,
                                               (uint32_t)rblk * 8u * (uint32_t)K + (uint32_t)k0, 0, 0);
  };

  // the lane's two 16-byte chunks (g, g + 4) of row (lane & 15) of a 16-row fragment, swizzled as
  // the DMA wrote them (chunk c of row R at c ^ ((R >> 1) & 7)); see F8Q_CHUNK
  int lane_off[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = lane & 15;
    const int c = F8Q_CHUNK(lane >> 4, h);
    lane_off[h] = r * F8_ROW + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_off = wr * 128 * F8_ROW;
  const int b_off = F8_PANEL + wc * 128 * F8_ROW;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  i32x8 FA[8], FB[8];
  char* const buf0 = smem;
  char* const buf1 = smem + F8_BUF;
  // read j of a set: j = 0..3 -> fragment base + j, one ds_read_b128 per half h
  auto read = [&](bool isb, int x, int h, const char* buf) {
    const char* base = buf + (isb ? b_off : a_off) + x * 16 * F8_ROW + lane_off[h];
    return *reinterpret_cast<const i32x4*>(base);
  };
  auto read_frag = [&](i32x8& F, bool isb, int x, const char* buf) {
    const i32x4 lo = read(isb, x, 0, buf);
    const i32x4 hi = read(isb, x, 1, buf);
    F = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto iter = [&](char* cur, char* nxt, int dk, auto DM, auto NX) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value;
    static_for<0, SLOTS>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int blk = i >> 4, w = i & 15;
      constexpr bool aslow = ASLOW && blk == 2;
      constexpr int bi = (blk >> 1) * 4 + (aslow ? (w & 3) : (w >> 2));
      constexpr int ai = (blk & 1) * 4 + (aslow ? (w >> 2) : (w & 3));
      f8q_mfma<ai * 8 + bi>(FB[bi], FA[ai]);                      // accumulator m*8+n
      // A1 (a4..7) at slots 0..7, B1 (b4..7) at 8..15: one fragment per two slots
      if constexpr (i < 8 && (i & 1) == 0) read_frag(FA[4 + i / 2], false, 4 + i / 2, cur);
      if constexpr (i >= 8 && i < 16 && (i & 1) == 0) read_frag(FB[4 + (i - 8) / 2], true, 4 + (i - 8) / 2, cur);
      if constexpr (i == W1) __builtin_amdgcn_s_waitcnt(0xC07F);                 // lgkmcnt(0)
      if constexpr (dm && i == W1 + 1) __builtin_amdgcn_s_barrier();
      if constexpr (dm && i >= D0 && (i - D0) % DS == 0 && (i - D0) / DS < 16) dma_piece((i - D0) / DS, dk, cur);
      if constexpr (nx && i == W2) {
        constexpr int issued = !dm || W2 < D0 ? 0 : ((W2 - D0) / DS + 1 > 16 ? 16 : (W2 - D0) / DS + 1);
        __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);   // vmcnt(n) lgkmcnt(0)
      }
      if constexpr (nx && i == W2 + 1) __builtin_amdgcn_s_barrier();
      if constexpr (nx && i >= RB0 && i <= RB0 + 3 * RBS && (i - RB0) % RBS == 0)
        read_frag(FB[(i - RB0) / RBS], true, (i - RB0) / RBS, nxt);
      if constexpr (nx && i >= RA0 && i <= RA0 + 3 * RAS && (i - RA0) % RAS == 0)
        read_frag(FA[(i - RA0) / RAS], false, (i - RA0) / RAS, nxt);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  const int ktiles = K / F8_BK;     // >= 2 (host guarantees)
  const bool rev = SERP > 0 && (((int)blockIdx.x / NXCD) / (SERP > 0 ? SERP : 1)) & 1;
  auto kof = [&](int kt) { return (rev ? ktiles - 1 - kt : kt) * F8_BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(0), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, kof(1), buf1);
  __builtin_amdgcn_s_waitcnt(0x4F70);               // vmcnt(16): tile 0 landed, tile 1 in flight
  bar();
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    read_frag(FB[x], true, x, buf0);
    read_frag(FA[x], false, x, buf0);
  }

  char* cur = buf0;
  char* nxt = buf1;
  for (int t = 0; t < ktiles - 2; ++t) {
    iter(cur, nxt, kof(t + 2), T_{}, T_{});
    char* tmp = cur; cur = nxt; nxt = tmp;
  }
  iter(cur, nxt, 0, F_{}, T_{});
  iter(nxt, nullptr, 0, F_{}, F_{});

  // epilogue: the bf16 w4s one (same 16x16 accumulator layout)
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
  bar();
  constexpr int CROW = F8_BN * 2;
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
  for (int i = 0; i < (F8_BM * F8_BN * 2) / (F8_THREADS * 16); ++i) {
    const int r = i * (F8_THREADS / 32) + (tid >> 5);
    const int ch = tid & 31;
    const int sw = r & 15;
    const int pg = (2 * ch) ^ sw;
    const uint4 raw = *reinterpret_cast<const uint4*>(smem + r * CROW + ((pg & ~1) << 3));
    uint4 v = raw;
    if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
    store_c16(C + (size_t)(tm * F8_BM + r) * N + tn * F8_BN + ch * 8, v);
  }
}

// Persistent fp8 kernel (variants 10/11): the bf16 v25 structure (gemm_bf16.hip) on the fp8 body.
// gridDim = one workgroup per CU (a multiple of 8); XCD x (= blockIdx % 8) owns the contiguous run
// of tiles xcd_remap gives it and its gridDim/8 workgroups walk it in strides. The K-tile stream
// runs across tile boundaries: a tile's last two K-iterations DMA the next tile's K-tiles 0 and 1
// into the freed buffers, so the next tile starts without a cold HBM prologue. Each wave stages its
// own 128x128 C sub-tile through a private 8 KiB LDS slice (32 rows per pass: one row of 32x32
// accumulators), so the epilogue needs no workgroup barrier and overlaps the in-flight DMA; the
// accumulators are zeroed as they are read. Pays off when the K-loop is short (16384x16384x1024).
constexpr int F8P_EPI_WAVE = 8192;                        // 32 rows x 128 cols x bf16
constexpr int F8P_LDS = F8_LDS + 4 * F8P_EPI_WAVE;        // 160 KiB

template <int B1 = 6, int D0 = 7, int DSPAN = 16, int B2 = 24, int RS = 6, bool SERP = false, Rec REC = kTimed>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_w4sp(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  note_placement<REC>();
  constexpr int SLOTS = 32;
  static_assert(B1 >= 4 && D0 >= B1 && D0 + DSPAN <= SLOTS && B2 >= 16 && B2 > B1 && B2 + RS < SLOTS,
                "schedule");
  __shared__ __attribute__((aligned(16))) char smem[F8P_LDS];

  const int tiles_m = M / F8_BM;
  const int tiles_n = N / F8_BN;
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

  const uint32_t panel_bytes = (uint32_t)F8_BM * (uint32_t)K;
  auto rsrc = [&](const uint8_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, panel_bytes, 0x00020000);
  };
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, tm, tn);
  __amdgpu_buffer_rsrc_t rA = rsrc(A + (size_t)tm * F8_BM * K);
  __amdgpu_buffer_rsrc_t rB = rsrc(Bt + (size_t)tn * F8_BN * K);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int k0, char* buf) {
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? F8_PANEL : 0) + rblk * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rb : ra, (lds_void*)lds, 16, voff,
                                             (uint32_t)rblk * 8u * (uint32_t)K + (uint32_t)k0, 0, 0);
  };

  int lane_off[2][2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = lane & 31;
      const int c = kh * 4 + 2 * (lane >> 5) + s;
      lane_off[kh][s] = r * F8_ROW + ((c ^ ((r >> 1) & 7)) << 4);
    }
  const int a_off = wr * 128 * F8_ROW;
  const int b_off = F8_PANEL + wc * 128 * F8_ROW;
  const int scale = E8M0_ONE;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  F8Frags R0, R1;
  char* const buf0 = smem;
  char* const buf1 = smem + F8_BUF;
  auto read_frag = [&](F8Frags& F, const char* buf, int kh, auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int x = f8_idx(j);
    const char* base = buf + (f8_isb(j) ? b_off : a_off) + x * 32 * F8_ROW;
    const i32x4 lo = *reinterpret_cast<const i32x4*>(base + lane_off[kh][0]);
    const i32x4 hi = *reinterpret_cast<const i32x4*>(base + lane_off[kh][1]);
    const i32x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    if constexpr (f8_isb(j)) F.b[x] = v;
    else F.a[x] = v;
  };
  // The w4s iteration with the DMA target (panels, K offset) a runtime argument. FRESH = a tile's
  // first iteration: the vmcnt(0) before it (prologue or previous epilogue) already retired its
  // K-tile 1, and a counted vmcnt would also wait for the epilogue's C stores.
  auto iter = [&](char* cur, char* nxt, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int dk, auto FR,
                  auto DM, auto NX) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value, fresh = decltype(FR)::value;
    static_for<0, SLOTS>([&](auto I) {
      constexpr int i = decltype(I)::value;
      if constexpr (i < 16) f8_mfma<i>(R0.b[i & 3], R0.a[i >> 2], scale);
      else f8_mfma<i - 16>(R1.b[i & 3], R1.a[(i - 16) >> 2], scale);
      if constexpr (i < 4) {
        read_frag(R1, cur, 1, std::integral_constant<int, 2 * i>{});
        read_frag(R1, cur, 1, std::integral_constant<int, 2 * i + 1>{});
      }
      if constexpr (i == B1 - 1) __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
      if constexpr (dm && i == B1) __builtin_amdgcn_s_barrier();
      if constexpr (dm) {
        static_for<0, 16>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (D0 + (j * DSPAN) / 16 == i) dma_piece(j, ra, rb, dk, cur);
        });
      }
      if constexpr (nx && i == B2 - 1) {
        constexpr int issued = [] {
          int n = 0;
          for (int j = 0; j < 16; ++j) n += (dm && D0 + (j * DSPAN) / 16 <= B2 - 1) ? 1 : 0;
          return n;
        }();
        if constexpr (fresh) __builtin_amdgcn_s_waitcnt(0xC07F);             // lgkmcnt(0) only
        else __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == B2) __builtin_amdgcn_s_barrier();
      if constexpr (nx && i > B2) {
        static_for<0, 8>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (B2 + 1 + (j * RS) / 8 == i) read_frag(R0, nxt, 0, J);
        });
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  // Wave-private epilogue: 4 passes, one per accumulator row i_m (32 C rows x 128 cols).
  char* const stg = smem + F8_LDS + wid * F8P_EPI_WAVE;
  auto epilogue = [&](int tm_, int tn_) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // MFMA D -> reads
    static_for<0, 4>([&](auto S) {
      constexpr int im = decltype(S)::value;
      static_for<0, 16>([&](auto I) {
        constexpr int u = decltype(I)::value;
        constexpr int in = u >> 2, g = u & 3;
        constexpr int a0 = 16 * (4 * im + in) + 4 * g;
        float x0, x1, x2, x3;
        asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                     "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7\n\t"
                     "v_accvgpr_write_b32 a%c4, 0\n\tv_accvgpr_write_b32 a%c5, 0\n\t"
                     "v_accvgpr_write_b32 a%c6, 0\n\tv_accvgpr_write_b32 a%c7, 0"
                     : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                     : "i"(a0), "i"(a0 + 1), "i"(a0 + 2), "i"(a0 + 3));
        const int r = lane & 31;                                   // C row inside the pass
        const int gi = 8 * in + 2 * g + (lane >> 5);               // 8-byte column group 0..31
        bf16x4 v;
        v[0] = (__bf16)x0;
        v[1] = (__bf16)x1;
        v[2] = (__bf16)x2;
        v[3] = (__bf16)x3;
        *reinterpret_cast<bf16x4*>(stg + r * 256 + ((gi ^ (r & 15)) << 3)) = v;
      });
      asm volatile("" ::: "memory");     // a wave's LDS ops execute in order: no wait, no barrier
      if constexpr (im == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // see FRESH
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = k * 4 + (lane >> 4);
        const int ch = lane & 15;
        const int sw = r & 15;
        const int pg = (2 * ch) ^ sw;
        const uint4 raw = *reinterpret_cast<const uint4*>(stg + r * 256 + ((pg & ~1) << 3));
        uint4 v = raw;
        if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
        store_c16(C + (size_t)(tm_ * F8_BM + wr * 128 + im * 32 + r) * N + tn_ * F8_BN +
                                  wc * 128 + ch * 8, v);
      }
      asm volatile("" ::: "memory");
    });
  };

  const int ktiles = K / F8_BK;     // >= 2 (host guarantees)
  // SERP: the workgroups of an XCD reach their i-th tile together, so tile i of every workgroup is
  // one wave of co-resident tiles; odd waves walk K backwards and start on the A-panel K-slices
  // the previous wave left in the XCD's L2.
  bool rev = false;
  auto kof = [&](int kt, bool r) { return (r ? ktiles - 1 - kt : kt) * F8_BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(0, rev), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(1, rev), buf1);
  __builtin_amdgcn_s_waitcnt(0x0070);               // vmcnt(0): K-tiles 0 and 1 landed (FRESH iteration)
  bar();
  static_for<0, 8>([&](auto J) { read_frag(R0, buf0, 0, J); });

  char* cur = buf0;
  char* nxt = buf1;
  for (;;) {
    const int next = tile + per;
    const bool has_next = next < t_end;
    int ntm = tm, ntn = tn;
    __amdgpu_buffer_rsrc_t nA = rA, nB = rB;
    if (has_next) {
      tile_coords(next, tiles_m, tiles_n, ntm, ntn);
      nA = rsrc(A + (size_t)ntm * F8_BM * K);
      nB = rsrc(Bt + (size_t)ntn * F8_BN * K);
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

// Persistent q16 (fp8 v18): the w4sp frame (one workgroup per CU, K-stream across tiles, the next
// tile's K-tiles 0 and 1 DMA'd by the current tile's last two iterations, wave-private epilogue
// that zeroes the accumulators as it reads them) around the q16 iteration (unscaled 16x16x128,
// quarter-block slot order, the production placement). For short K with several tiles per CU.
template <int W1 = 16, int D0 = 18, int DS = 3, int W2 = 34, int RB0 = 35, int RA0 = 43, bool SERP = false,
          int RBS = 2, int RAS = 2, bool ASLOW = true, Rec REC = kTimed>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_q16p(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                      __bf16* __restrict__ C, int M, int N, int K) {
  note_placement<REC>();
  constexpr int SLOTS = 64;
  static_assert(W1 >= 15 && D0 > W1 && D0 + 15 * DS < SLOTS && W2 > W1 && RB0 > W2 && RA0 > W2, "schedule");
  __shared__ __attribute__((aligned(16))) char smem[F8P_LDS];

  const int tiles_m = M / F8_BM;
  const int tiles_n = N / F8_BN;
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

  const uint32_t panel_bytes = (uint32_t)F8_BM * (uint32_t)K;
  auto rsrc = [&](const uint8_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, panel_bytes, 0x00020000);
  };
  int tm, tn;
  tile_coords(tile, tiles_m, tiles_n, tm, tn);
  __amdgpu_buffer_rsrc_t rA = rsrc(A + (size_t)tm * F8_BM * K);
  __amdgpu_buffer_rsrc_t rB = rsrc(Bt + (size_t)tn * F8_BN * K);
  const int par = wid & 1;
  const uint32_t voff = (uint32_t)(lane >> 3) * (uint32_t)K +
                        (uint32_t)(((lane & 7) ^ ((par * 4 + (lane >> 4)) & 7)) * 16);
  auto dma_piece = [&](int i, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int k0, char* buf) {
    const int rblk = ((i & 7) << 2) + wid;
    char* lds = buf + (i >= 8 ? F8_PANEL : 0) + rblk * 1024;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(i >= 8 ? rb : ra, (lds_void*)lds, 16, voff,
                                             (uint32_t)rblk * 8u * (uint32_t)K + (uint32_t)k0, 0, 0);
  };
  int lane_off[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = lane & 15;
    const int c = F8Q_CHUNK(lane >> 4, h);                 // (g, g + 4): conflict-free, see F8Q_CHUNK
    lane_off[h] = r * F8_ROW + ((c ^ ((r >> 1) & 7)) << 4);
  }
  const int a_off = wr * 128 * F8_ROW;
  const int b_off = F8_PANEL + wc * 128 * F8_ROW;

  asm volatile("" ::: W4_AGPR_CLOBBERS);
  static_for<0, 256>([&](auto R) { asm volatile("v_accvgpr_write_b32 a%c0, 0" :: "i"(decltype(R)::value)); });

  i32x8 FA[8], FB[8];
  char* const buf0 = smem;
  char* const buf1 = smem + F8_BUF;
  auto read_frag = [&](i32x8& F, bool isb, int x, const char* buf) {
    const char* base = buf + (isb ? b_off : a_off) + x * 16 * F8_ROW;
    const i32x4 lo = *reinterpret_cast<const i32x4*>(base + lane_off[0]);
    const i32x4 hi = *reinterpret_cast<const i32x4*>(base + lane_off[1]);
    F = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  // FRESH = a tile's first iteration: the epilogue's vmcnt(0) already retired its K-tile 1, and a
  // counted vmcnt would also wait for the epilogue's C stores.
  auto iter = [&](char* cur, char* nxt, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int dk, auto FR,
                  auto DM, auto NX) {
    constexpr bool dm = decltype(DM)::value, nx = decltype(NX)::value, fresh = decltype(FR)::value;
    static_for<0, SLOTS>([&](auto I) {
      constexpr int i = decltype(I)::value;
      constexpr int blk = i >> 4, w = i & 15;
      constexpr bool aslow = ASLOW && blk == 2;
      constexpr int bi = (blk >> 1) * 4 + (aslow ? (w & 3) : (w >> 2));
      constexpr int ai = (blk & 1) * 4 + (aslow ? (w >> 2) : (w & 3));
      f8q_mfma<ai * 8 + bi>(FB[bi], FA[ai]);
      if constexpr (i < 8 && (i & 1) == 0) read_frag(FA[4 + i / 2], false, 4 + i / 2, cur);
      if constexpr (i >= 8 && i < 16 && (i & 1) == 0) read_frag(FB[4 + (i - 8) / 2], true, 4 + (i - 8) / 2, cur);
      if constexpr (i == W1) __builtin_amdgcn_s_waitcnt(0xC07F);                 // lgkmcnt(0)
      if constexpr (dm && i == W1 + 1) __builtin_amdgcn_s_barrier();
      if constexpr (dm && i >= D0 && (i - D0) % DS == 0 && (i - D0) / DS < 16) dma_piece((i - D0) / DS, ra, rb, dk, cur);
      if constexpr (nx && i == W2) {
        constexpr int issued = !dm || W2 < D0 ? 0 : ((W2 - D0) / DS + 1 > 16 ? 16 : (W2 - D0) / DS + 1);
        if constexpr (fresh) __builtin_amdgcn_s_waitcnt(0xC07F);             // lgkmcnt(0) only
        else __builtin_amdgcn_s_waitcnt((issued & 15) | ((issued >> 4) << 14) | 0x70);
      }
      if constexpr (nx && i == W2 + 1) __builtin_amdgcn_s_barrier();
      if constexpr (nx && i >= RB0 && i <= RB0 + 3 * RBS && (i - RB0) % RBS == 0)
        read_frag(FB[(i - RB0) / RBS], true, (i - RB0) / RBS, nxt);
      if constexpr (nx && i >= RA0 && i <= RA0 + 3 * RAS && (i - RA0) % RAS == 0)
        read_frag(FA[(i - RA0) / RAS], false, (i - RA0) / RAS, nxt);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  using T_ = std::true_type;
  using F_ = std::false_type;

  // Wave-private epilogue: 4 passes of 32 C rows (accumulator rows m = 2p, 2p+1) x 128 cols.
  char* const stg = smem + F8_LDS + wid * F8P_EPI_WAVE;
  auto epilogue = [&](int tm_, int tn_) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");   // MFMA D -> reads
    static_for<0, 4>([&](auto P) {
      constexpr int p = decltype(P)::value;
      static_for<0, 16>([&](auto I) {
        constexpr int u = decltype(I)::value;
        constexpr int m = 2 * p + (u >> 3), n = u & 7;
        constexpr int a0 = 4 * (m * 8 + n);
        float x0, x1, x2, x3;
        asm volatile("v_accvgpr_read_b32 %0, a%c4\n\tv_accvgpr_read_b32 %1, a%c5\n\t"
                     "v_accvgpr_read_b32 %2, a%c6\n\tv_accvgpr_read_b32 %3, a%c7\n\t"
                     "v_accvgpr_write_b32 a%c4, 0\n\tv_accvgpr_write_b32 a%c5, 0\n\t"
                     "v_accvgpr_write_b32 a%c6, 0\n\tv_accvgpr_write_b32 a%c7, 0"
                     : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)
                     : "i"(a0), "i"(a0 + 1), "i"(a0 + 2), "i"(a0 + 3));
        const int r = (u >> 3) * 16 + (lane & 15);                 // C row inside the pass
        const int gi = 4 * n + (lane >> 4);                        // 8-byte column group 0..31
        bf16x4 v;
        v[0] = (__bf16)x0;
        v[1] = (__bf16)x1;
        v[2] = (__bf16)x2;
        v[3] = (__bf16)x3;
        *reinterpret_cast<bf16x4*>(stg + r * 256 + ((gi ^ (r & 15)) << 3)) = v;
      });
      asm volatile("" ::: "memory");     // a wave's LDS ops execute in order: no wait, no barrier
      if constexpr (p == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // see FRESH
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int r = k * 4 + (lane >> 4);
        const int ch = lane & 15;
        const int sw = r & 15;
        const int pg = (2 * ch) ^ sw;
        const uint4 raw = *reinterpret_cast<const uint4*>(stg + r * 256 + ((pg & ~1) << 3));
        uint4 v = raw;
        if (sw & 1) { v.x = raw.z; v.y = raw.w; v.z = raw.x; v.w = raw.y; }
        store_c16(C + (size_t)(tm_ * F8_BM + wr * 128 + p * 32 + r) * N + tn_ * F8_BN +
                                  wc * 128 + ch * 8, v);
      }
      asm volatile("" ::: "memory");
    });
  };

  const int ktiles = K / F8_BK;     // >= 2 (host guarantees)
  bool rev = false;
  auto kof = [&](int kt, bool r) { return (r ? ktiles - 1 - kt : kt) * F8_BK; };
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(0, rev), buf0);
#pragma unroll
  for (int i = 0; i < 16; ++i) dma_piece(i, rA, rB, kof(1, rev), buf1);
  __builtin_amdgcn_s_waitcnt(0x0070);               // vmcnt(0): K-tiles 0 and 1 landed (FRESH iteration)
  bar();
#pragma unroll
  for (int x = 0; x < 4; ++x) {
    read_frag(FB[x], true, x, buf0);
    read_frag(FA[x], false, x, buf0);
  }

  char* cur = buf0;
  char* nxt = buf1;
  for (;;) {
    const int next = tile + per;
    const bool has_next = next < t_end;
    int ntm = tm, ntn = tn;
    __amdgpu_buffer_rsrc_t nA = rA, nB = rB;
    if (has_next) {
      tile_coords(next, tiles_m, tiles_n, ntm, ntn);
      nA = rsrc(A + (size_t)ntm * F8_BM * K);
      nB = rsrc(Bt + (size_t)ntn * F8_BN * K);
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

// q16ap (fp8 v20-v22): the persistent asm-pipeline frame of the bf16 v50 (gemm_w4ap.h) around the
// q16 K-tile body as one hand-scheduled asm block per output tile (tools/gen_fp8_asm_loop.py,
// gemm_fp8_asm_loop.h): the same MFMAs, operands and accumulators as q16p, waits computed per
// fragment instead of hipcc's, no per-piece SALU address arithmetic or s_nop.
template <int SC = 0, bool SERP = false, bool SQ = false, int EPI = 0, int DM = 0, Rec REC = kTimed>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_q16ap(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                       __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem[W4AP_LDS];
  note_placement<REC>();
  w4ap_run<SC, SERP, SQ, true, EPI, DM>((const char*)A, (const char*)Bt, C, M, N, K, smem);
}

// q16ap split-K (fp8 v24): one (tile, K piece) per workgroup, the piece sums reduced by each tile's last
// arriving waves (gemm_w4ap.h SPLIT; the bf16 v57's frame with the fp8 K-tile body).
template <int SC, int EPI, int DM, Rec REC = kTimed>
__global__ void __launch_bounds__(F8_THREADS, 1)
gemm_fp8_256x256_q16ap_sk(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt, __bf16* __restrict__ C,
                          int M, int N, int K, int splits, float* __restrict__ ws, int* __restrict__ cnt,
                          int last_pairs, int pmajor) {
  __shared__ __attribute__((aligned(16))) char smem[W4AP_LDS];
  note_placement<REC>();
  w4ap_run<SC, false, false, true, EPI, DM, true>((const char*)A, (const char*)Bt, C, M, N, K, smem,
                                                  W4Split{splits, ws, cnt, last_pairs, pmajor});
}

// OCP e4m3fn -> f32 in software (independent of the matrix cores): bias 7, no infinities,
// S.1111.111 = NaN, exponent 0 = subnormal m/8 * 2^-6.
__device__ __forceinline__ float e4m3_to_f32(uint8_t v) {
  const int e = (v >> 3) & 15, m = v & 7;
  float f;
  if (e == 15 && m == 7) f = __builtin_nanf("");
  else if (e == 0) f = ldexpf((float)m, -9);
  else f = ldexpf((float)(8 + m), e - 10);
  return (v & 0x80) ? -f : f;
}

constexpr int G8 = 64, G8K = 32;

// Bounds-checked 64x64 tiles, operands decoded to fp32 in LDS, 4x4 outputs per thread.
template <Rec REC = kTimed>
__global__ void __launch_bounds__(256)
gemm_fp8_generic(const uint8_t* __restrict__ A, const uint8_t* __restrict__ Bt,
                 __bf16* __restrict__ C, int M, int N, int K) {
  __shared__ float sa[G8K][G8 + 1];
  __shared__ float sb[G8K][G8 + 1];
  note_placement<REC>();
  const int m0 = blockIdx.y * G8, n0 = blockIdx.x * G8;
  const int tr = threadIdx.x >> 4, tc = threadIdx.x & 15;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < K; k0 += G8K) {
    for (int e = threadIdx.x; e < G8 * G8K; e += 256) {
      const int r = e / G8K, k = e % G8K;
      const int gk = k0 + k;
      sa[k][r] = (m0 + r < M && gk < K) ? e4m3_to_f32(A[(size_t)(m0 + r) * K + gk]) : 0.f;
      sb[k][r] = (n0 + r < N && gk < K) ? e4m3_to_f32(Bt[(size_t)(n0 + r) * K + gk]) : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int k = 0; k < G8K; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i] = sa[k][tr * 4 + i];
        bv[i] = sb[k][tc * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = m0 + tr * 4 + i, c = n0 + tc * 4 + j;
      if (r < M && c < N) C[(size_t)r * N + c] = (__bf16)acc[i][j];
    }
}

// Deterministic uniform [-1,1) fill, rounded to e4m3fn by the hardware converter (OCP on gfx950).
__global__ void fill_uniform_fp8(uint8_t* p, size_t n, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) {
    uint32_t x = (uint32_t)i * 0x9E3779B1u ^ seed;
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    const float u = 2.0f * ((float)(x >> 8) * (1.0f / 16777216.0f)) - 1.0f;
    p[i] = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(u, u, 0, false) & 0xFF);
  }
}

}  // namespace
