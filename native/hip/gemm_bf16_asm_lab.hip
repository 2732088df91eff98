// Tools-only A/B library for the hand-scheduled bf16 K pipeline (gemm_bf16_256x256_w4a): the
// production v44 next to the asm-loop schedules, in one code object so tools/asm_lab.py can
// interleave them with hipBLASLt in one process. Never loaded by the validator.
//   44  = w4s v44 (production: serpentine K, loop rotation, VK)
//   100 + SC = w4a with schedule SC (gemm_bf16_asm_loop.h lists them), serpentine K
//   120 = w4a schedule 0 without serpentine K
//   25  = w4sp v25 (production for short K: persistent, VK)
//   45  = w4s v45 (production for big square grids: v44 + square cross-XCD raster)
// (every w4ap / q16ap case below uses the production nontemporal-store epilogue unless it says otherwise)
//   130 + SC = w4ap (persistent) with persistent schedule SC, serpentine K; 133 = schedule 0 without
//   170 / 171 / 172 / 173 = w4ap with the fused epilogue (EPI=2): g4 serpentine K, g6d6 serpentine, g4 linear,
//   g4 square raster
//   180 / 181 / 182 = relaxed first landing wait (_rw): g4 (= v50 + rw), g6d6 (v52 + rw), g4 square raster (v51 + rw)
//   190 / 191 / 192 / 193 = VP DMA form: g4 (= v50 in VP form), g4 + PA, g6d6 VP, g4 + PA linear K
//   194 / 195 = VP DMA form on the square raster (g4), without / with PA
//   197 / 198 / 265 / 266 = ZC (EPI 8, src C = 0 first K-tile): bf16 v50 / v51, fp8 v20 / v21 forms
//   200 / 267 / 268 = WG512 epilogue (EPI 10: workgroup-shared staging, 2 x 512-byte rows per store): bf16 v50, fp8 v20 / v21
//   199 = direct epilogue (EPI 9: EF layout, stores from the accumulators, no LDS staging)
//   215 / 216 / 217 = LEAN epilogue (EPI 15: chunk-swizzled staging, saddr stores): 197 / 198 / VP G4_ZC;
//   218 / 219 = VP + PA G4_ZC with LEAN / STAGED_ZC, 222 = 218 on the square raster; 223 / 224 = VP
//   G4_ZC square raster with LEAN / STAGED_ZC (224 = production v54); 225 / 226 / 227 = LEAN_PIPE (EPI 16,
//   pipelined half-passes): 197 / 218 / 222 with it; fp8 274 = 272 with it, 275 = 265 with it; 228 / 229 /
//   fp8 276 = LEAN_ILV (EPI 17, stores interleaved into the next staging): 227 / 225 / 274 with it; 238 /
//   fp8 277 = 228 / 276 with LEAN_ILVB (EPI 18, burst accumulator reads);
//   fp8 269 / 270 = 265 / 266 with it; 271 = VP + PA p_zc square raster (262 + ZC), 272 = 271 + LEAN,
//   273 = VP + PA p_zc linear raster + LEAN
//   211-214 = 197 with store cache policy sc1 nt / sc0 sc1 / sc0 sc1 nt / sc0 nt
//   196 / 264 = deferred C stores (EPI 7): bf16 g4 serpentine (v50 + DS), fp8 p linear (v20 + DS); K >= 8 K-tiles
//   163 / 164 = knock-outs: production epilogue storing only the first quarter / half of C; 233 = fp8 quarter
//   162 = v50 (136) with nontemporal C stores; 174 = 170 with nontemporal stores
//   160 / 161 = knock-outs (wrong C): 136 without its epilogue / without the epilogue's global stores
//   150 / 151 = w4ap square raster (SQ) with persistent schedule 5 / 9; 152 = 150 without serpentine K
// amdgo_asmlab_gemm_fp8 (fp8 e4m3 operands):
//   15 / 16 / 18 = production q16 (serpentine K), q16 square raster, persistent q16p
//   200 + SC = q16ap (persistent asm pipeline) with fp8 schedule SC (gemm_fp8_asm_loop.h), linear K
//   210 + SC = q16ap with serpentine K; 220 + SC = q16ap square raster, serpentine K
//   240 / 241 / 242 / 243 = q16ap with the fused epilogue (EPI=2): p linear, s1d3 serpentine, p serpentine,
//   p square raster
//   250 / 251 / 252 / 253 = q16ap relaxed first landing wait: p linear (v20 + rw), s1d3 serpentine, p square
//   raster (v21 + rw), p serpentine
//   260 / 261 / 262 / 263 = q16ap VP form: p linear (= v20 in VP form), p + PA, p + PA square raster, s1d3 + PA serp
//   232 = 200 with nontemporal C stores; 244 = 240 with nontemporal stores
//   230 / 231 = knock-outs: 200 without its epilogue / without the epilogue's global stores
#include "gemm_bf16_asm_loop_lab.h"  // every schedule (masks the production header)
#include "gemm_fp8_asm_loop_lab.h"  // every schedule (masks the production header)
#include "gemm_bf16_kernels.h"
#include "gemm_fp8_kernels.h"
#include "gemm_small_host.h"

namespace {

// Lab: a 16-byte C store with explicit gfx950 cache-policy bits (POL: 1 = "sc1 nt", 2 = "sc0 sc1",
// 3 = "sc0 sc1 nt", 4 = "sc0 nt"), to price the store path against store_c16's plain "nt".
template <int POL>
__device__ __forceinline__ void store_c16_pol(void* p, uint4 v) {
  typedef unsigned int u32x4_p __attribute__((ext_vector_type(4)));
  u32x4_p x;
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(p), "v"(x) : "memory");
  else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(x) : "memory");
  else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" :: "v"(p), "v"(x) : "memory");
  else asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" :: "v"(p), "v"(x) : "memory");
}

// Lab epilogue forms of the persistent frame (W4apEpi, gemm_w4ap.h): knock-outs that price the
// epilogue (wrong C) and store-policy variants. Production kernels never instantiate these.
constexpr int EPI_KO_NONE = 1;      // no epilogue at all
constexpr int EPI_KO_NOSTORE = 3;   // staged epilogue without the global stores
constexpr int EPI_KO_QUARTER = 5;   // nt stores of only the first quarter of C
constexpr int EPI_KO_HALF = 6;      // ... the first half

template <int EPI, int STORED_PASSES, bool ZC>
struct W4apEpiLab {
  static constexpr bool run = STORED_PASSES >= 0;
  static constexpr bool zc = ZC;
  template <int S>
  static __device__ __forceinline__ void store(__bf16* dst, uint4 v) {
    if constexpr (S < STORED_PASSES) store_c16(dst, v);
    else asm volatile("" :: "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));   // keep the value live
  }
};
template <> struct W4apEpi<EPI_KO_NONE> : W4apEpiLab<EPI_KO_NONE, -1, false> {};
template <> struct W4apEpi<EPI_KO_NOSTORE> : W4apEpiLab<EPI_KO_NOSTORE, 0, false> {};
template <> struct W4apEpi<EPI_KO_QUARTER> : W4apEpiLab<EPI_KO_QUARTER, 1, false> {};
template <> struct W4apEpi<EPI_KO_HALF> : W4apEpiLab<EPI_KO_HALF, 2, false> {};
template <int P>
struct W4apEpiPol {                 // ZC with the store cache-policy bits of store_c16_pol<P>
  static constexpr bool run = true, zc = true;
  template <int S>
  static __device__ __forceinline__ void store(__bf16* dst, uint4 v) { store_c16_pol<P>(dst, v); }
};
template <> struct W4apEpi<11> : W4apEpiPol<1> {};
template <> struct W4apEpi<12> : W4apEpiPol<2> {};
template <> struct W4apEpi<13> : W4apEpiPol<3> {};
template <> struct W4apEpi<14> : W4apEpiPol<4> {};

}  // namespace

extern "C" {

int amdgo_asmlab_gemm_bf16(int v, const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M % BM || N % BN || K % (2 * BK) || K < 4 * BK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const __bf16*)A;
  const auto* b = (const __bf16*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / BM) * (N / BN);
  // 300-307: the production split-K form (v57) with its reduction knocked out piece by piece
  // (gemm_w4ap.h w4ap_split_reduce SKO = v - 300: 1 no release, 2 no slab reads, 4 no slab stores);
  // the pieces, last-piece share and item order are the production defaults
  auto split_ko = [&](auto KO) -> int {
    const int splits = asm_splits(nwg, K / BK, device_cu_count(s));
    if (splits < 2) return (int)hipErrorInvalidValue;
    SmallWorkspace* w = small_workspace(s, (size_t)nwg * splits * kAsmSlabFloats, nwg * 2);
    if (!w) return (int)hipErrorOutOfMemory;
    hipLaunchKernelGGL((gemm_bf16_256x256_w4ap_sk<W4VP_SC_G4_ZC, W4AP_EPI_LEAN, 2, kTimed, decltype(KO)::value>),
                       dim3(nwg * splits), dim3(W4_THREADS), 0, s, a, b, c, M, N, K, splits, w->ws, w->cnt,
                       asm_last_pairs(K / BK, splits), asm_piece_major());
    (void)hipEventRecord(w->done, s);
    return (int)hipGetLastError();
  };
  switch (v) {
    case 300: return split_ko(std::integral_constant<int, 0>{});
    case 301: return split_ko(std::integral_constant<int, 1>{});
    case 302: return split_ko(std::integral_constant<int, 2>{});
    case 303: return split_ko(std::integral_constant<int, 3>{});
    case 305: return split_ko(std::integral_constant<int, 5>{});
    case 307: return split_ko(std::integral_constant<int, 7>{});
    case 44:
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, false, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
#define W4A_CASE(V, SC, SERP)                                                                             \
    case V:                                                                                               \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4a<SC, SERP, false>), dim3(nwg), dim3(W4_THREADS), 0, s, a, b, c, \
                         M, N, K);                                                                        \
      break;
    case 25: {
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4sp<17, 19, 5, 80, 40, false, true>), dim3(g), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    }
    case 45:
      if ((M / BM) % 16 || (N / BN) % 16) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4s<17, 19, 5, 80, 40, 32, true, true, true>), dim3(nwg),
                         dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    W4A_CASE(100, 0, 32)
    W4A_CASE(101, 1, 32)
    W4A_CASE(102, 2, 32)
    W4A_CASE(103, 3, 32)
    W4A_CASE(104, 4, 32)
    W4A_CASE(105, 5, 32)
    W4A_CASE(106, 6, 32)
    W4A_CASE(107, 7, 32)
    W4A_CASE(108, 8, 32)
    W4A_CASE(109, 9, 32)
    W4A_CASE(110, 10, 32)
    W4A_CASE(111, 11, 32)
    W4A_CASE(112, 12, 32)
    W4A_CASE(120, 0, 0)
#define W4AP_CASE(V, SC, SERP)                                                                             \
    case V: {                                                                                             \
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;                   \
      if (g < NXCD) return (int)hipErrorInvalidValue;                                                     \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<SC, SERP, false, W4AP_EPI_STAGED_NT>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K); \
      break;                                                                                              \
    }
    W4AP_CASE(130, 0, true)
    W4AP_CASE(131, 1, true)
    W4AP_CASE(132, 2, true)
    W4AP_CASE(133, 0, false)
    W4AP_CASE(134, 3, true)
    W4AP_CASE(135, 4, true)
    W4AP_CASE(136, 5, true)
    W4AP_CASE(137, 6, true)
    W4AP_CASE(138, 7, true)
    W4AP_CASE(139, 8, true)
    W4AP_CASE(140, 9, true)
    W4AP_CASE(141, 10, true)
    W4AP_CASE(142, 11, true)
    W4AP_CASE(143, 12, true)
    W4AP_CASE(144, 13, true)
    W4AP_CASE(145, 14, true)
    W4AP_CASE(146, 15, true)
    W4AP_CASE(147, 16, true)
    W4AP_CASE(180, W4AP_SC_G4_RW, true)
#define W4VP_CASE(V, SC, SERP, DM)                                                                         \
    case V: {                                                                                             \
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;                   \
      if (g < NXCD) return (int)hipErrorInvalidValue;                                                     \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<SC, SERP, false, W4AP_EPI_STAGED_NT, DM>), dim3(g), dim3(W4_THREADS), 0, s, \
                         a, b, c, M, N, K);                                                               \
      break;                                                                                              \
    }
    W4VP_CASE(190, W4VP_SC_G4, true, 1)
    W4VP_CASE(191, W4VP_SC_G4, true, 2)
    W4VP_CASE(192, W4VP_SC_G6D6, true, 1)
    W4VP_CASE(193, W4VP_SC_G4, false, 2)
    W4AP_CASE(181, W4AP_SC_G6D6_RW, true)
#define W4APSQ_CASE(V, SC, SERP)                                                                           \
    case V:                                                                                               \
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;    \
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<SC, SERP, true, W4AP_EPI_STAGED_NT>), dim3(256), dim3(W4_THREADS), 0, s, a, b, c, \
                         M, N, K);                                                                        \
      break;
    W4APSQ_CASE(150, 5, true)
    W4APSQ_CASE(151, 9, true)
    W4APSQ_CASE(152, 5, false)
    W4APSQ_CASE(182, W4AP_SC_G4_RW, true)
    case 194:     // VP DMA form on the square raster (g4, serpentine K); 195 = the same with PA
    case 195:
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      if (v == 194)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4, true, true, W4AP_EPI_STAGED_NT, 1>), dim3(256), dim3(W4_THREADS), 0,
                           s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4, true, true, W4AP_EPI_STAGED_NT, 2>), dim3(256), dim3(W4_THREADS), 0,
                           s, a, b, c, M, N, K);
      break;
    case 173:     // EF square raster, g4, serpentine K
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G4, true, true, 2>), dim3(256), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 160: {   // knock-out: v50 (schedule g4, serpentine K) without the epilogue's C stores
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<5, true, false, 1>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 170:     // EF: fused epilogue (EPI=2), schedule g4, serpentine K
    case 171:     // EF: schedule g6d6
    case 174:     // EF g4 with nontemporal stores
    case 172: {   // EF: g4, linear K
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 170)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G4, true, false, 2>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      else if (v == 171)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G6D6, true, false, 2>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      else if (v == 174)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G4_NT, true, false, 2>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G4, false, false, 2>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 162: {   // v50 with nontemporal C stores in the staged epilogue
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<5, true, false, 4>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 163:     // knock-outs of the production epilogue: only the first quarter (163) / half (164) of C stored
    case 164: {
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 163)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<5, true, false, 5>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<5, true, false, 6>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 196: {   // deferred C stores (EPI 7): v50 (g4, serpentine K) storing quarters 1-3 in the next K-loop
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD || K < 8 * 2 * BK) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4DS_SC_G4, true, false, W4AP_EPI_DEFERRED>), dim3(g), dim3(W4_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    }
    case 197: {   // ZC (EPI 8): v50 with src C = 0 in each tile's first K-tile, epilogue without zeroing writes
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, W4AP_EPI_STAGED_ZC>), dim3(g), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    }
    case 211: case 212: case 213: case 214: {   // 197 with store policy sc1 nt / sc0 sc1 / sc0 sc1 nt / sc0 nt
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 211) hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, 11>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      if (v == 212) hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, 12>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      if (v == 213) hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, 13>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      if (v == 214) hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, 14>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 199: {   // direct epilogue (EPI 9): EF fragment layout, C stored from the accumulators after the loop
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4EF_SC_G4_POST, true, false, W4AP_EPI_DIRECT>), dim3(g), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    }
    case 200: {   // WG512 epilogue (EPI 10): ZC, workgroup-shared staging, 2 x 512 B rows per store
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, W4AP_EPI_WG512>), dim3(g), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    }
    case 215: case 217: {   // LEAN epilogue (EPI 15): 197 / the VP G4_ZC form (DM 1) with it
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 215)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, W4AP_EPI_LEAN>), dim3(g), dim3(W4_THREADS), 0,
                           s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_LEAN, 1>), dim3(g), dim3(W4_THREADS),
                           0, s, a, b, c, M, N, K);
      break;
    }
    case 218: case 219: {   // VP + PA (DM 2) G4_ZC, serpentine K, linear raster: LEAN / STAGED_ZC epilogue
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 218)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_LEAN, 2>), dim3(g), dim3(W4_THREADS),
                           0, s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_STAGED_ZC, 2>), dim3(g),
                           dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 222:     // VP + PA G4_ZC + LEAN on the square raster
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN, 2>), dim3(256), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    case 223: case 224:     // VP (DM 1) G4_ZC on the square raster: LEAN / STAGED_ZC (= production v54)
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      if (v == 223)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN, 1>), dim3(256), dim3(W4_THREADS),
                           0, s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_STAGED_ZC, 1>), dim3(256),
                           dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 225: case 226: {   // LEAN_PIPE epilogue (EPI 16): 197 with it / VP + PA G4_ZC with it, linear raster
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      if (v == 225)
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, W4AP_EPI_LEAN_PIPE>), dim3(g), dim3(W4_THREADS),
                           0, s, a, b, c, M, N, K);
      else
        hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, false, W4AP_EPI_LEAN_PIPE, 2>), dim3(g),
                           dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    case 227:     // VP + PA G4_ZC + LEAN_PIPE on the square raster
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN_PIPE, 2>), dim3(256), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 228:     // LEAN_ILV (EPI 17: stores interleaved into the next staging): 227 with it
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN_ILV, 2>), dim3(256), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 229: {   // 225 (v50 + LEAN_PIPE) with LEAN_ILV
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, false, W4AP_EPI_LEAN_ILV>), dim3(g), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    }
    case 238:     // 228 with LEAN_ILVB (EPI 18: a half-pass's accumulators read in one burst)
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4VP_SC_G4_ZC, true, true, W4AP_EPI_LEAN_ILVB, 2>), dim3(256), dim3(W4_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 216:     // LEAN epilogue on the square raster (198 + EPI 15)
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, true, W4AP_EPI_LEAN>), dim3(256), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    case 198:     // ZC on the square raster (v51 + ZC)
      if ((M / BM) % 16 || (N / BN) % 16 || device_cu_count() != 256) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<W4AP_SC_G4_ZC, true, true, W4AP_EPI_STAGED_ZC>), dim3(256), dim3(W4_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    case 161: {   // knock-out: v50 with the epilogue but without its global C stores
      const int g = ((nwg < device_cu_count() ? nwg : device_cu_count()) / NXCD) * NXCD;
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_bf16_256x256_w4ap<5, true, false, 3>), dim3(g), dim3(W4_THREADS), 0, s, a, b, c, M, N, K);
      break;
    }
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

int amdgo_asmlab_gemm_fp8(int v, const void* A, const void* Bt, void* C, int M, int N, int K, void* stream) {
  if (M % F8_BM || N % F8_BN || K % (2 * F8_BK) || K < 4 * F8_BK) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const auto* a = (const uint8_t*)A;
  const auto* b = (const uint8_t*)Bt;
  auto* c = (__bf16*)C;
  const int nwg = (M / F8_BM) * (N / F8_BN);
  const int cus = device_cu_count();
  const int g = ((nwg < cus ? nwg : cus) / NXCD) * NXCD;
  const bool sq = (M / F8_BM) % 16 == 0 && (N / F8_BN) % 16 == 0 && cus == 256;
  switch (v) {
    case 15:
      hipLaunchKernelGGL((gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, false, 2, 2, true>), dim3(nwg),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 16:
      if (!sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16<16, 18, 3, 34, 35, 43, 32, true, 2, 2, true>), dim3(nwg),
                         dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 18:
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16p<>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
#define F8AP_CASE(V, SC, SERP, SQ)                                                                         \
    case V:                                                                                               \
      if (g < NXCD || (SQ && !sq)) return (int)hipErrorInvalidValue;                                      \
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<SC, SERP, SQ, W4AP_EPI_STAGED_NT>), dim3(SQ ? 256 : g), dim3(F8_THREADS), 0, s, \
                         a, b, c, M, N, K);                                                               \
      break;
    F8AP_CASE(200, 0, false, false)
    F8AP_CASE(201, 1, false, false)
    F8AP_CASE(202, 2, false, false)
    F8AP_CASE(203, 3, false, false)
    F8AP_CASE(204, 4, false, false)
    F8AP_CASE(205, 5, false, false)
    F8AP_CASE(206, 6, false, false)
    F8AP_CASE(210, 0, true, false)
    F8AP_CASE(211, 1, true, false)
    F8AP_CASE(212, 2, true, false)
    F8AP_CASE(213, 3, true, false)
    F8AP_CASE(214, 4, true, false)
    F8AP_CASE(215, 5, true, false)
    F8AP_CASE(216, 6, true, false)
    F8AP_CASE(220, 0, true, true)
    F8AP_CASE(221, 1, true, true)
    F8AP_CASE(222, 2, true, true)
    F8AP_CASE(223, 3, true, true)
    F8AP_CASE(224, 4, true, true)
    F8AP_CASE(225, 5, true, true)
    F8AP_CASE(226, 6, true, true)
    F8AP_CASE(250, F8AP_SC_P_RW, false, false)
#define F8VP_CASE(V, SC, SERP, SQ, DM)                                                                     \
    case V:                                                                                               \
      if (g < NXCD || (SQ && !sq)) return (int)hipErrorInvalidValue;                                      \
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<SC, SERP, SQ, W4AP_EPI_STAGED_NT, DM>), dim3(SQ ? 256 : g), dim3(F8_THREADS), \
                         0, s, a, b, c, M, N, K);                                                         \
      break;
    F8VP_CASE(260, F8VP_SC_P, false, false, 1)
    F8VP_CASE(261, F8VP_SC_P, false, false, 2)
    F8VP_CASE(262, F8VP_SC_P, true, true, 2)
    F8VP_CASE(263, F8VP_SC_S1D3, true, false, 2)
    F8AP_CASE(251, F8AP_SC_S1D3_RW, true, false)
    F8AP_CASE(252, F8AP_SC_P_RW, true, true)
    F8AP_CASE(253, F8AP_SC_P_RW, true, false)
    case 240:     // EF: fused epilogue (EPI=2), schedule p, linear K
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8EF_SC_P, false, false, 2>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 241:     // EF: schedule s1d3, serpentine K
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8EF_SC_S1D3, true, false, 2>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 242:     // EF: schedule p, serpentine K
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8EF_SC_P, true, false, 2>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 243:     // EF: schedule p, square raster, serpentine K
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8EF_SC_P, true, true, 2>), dim3(256), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 232:     // 200 with nontemporal C stores
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<0, false, false, 4>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 244:     // EF p with nontemporal stores
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8EF_SC_P_NT, false, false, 2>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 233:     // knock-out: 200 with nontemporal stores of only the first quarter of C
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<0, false, false, 5>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 264:     // deferred C stores (EPI 7): v20 (p, linear K)
      if (g < NXCD || K < 8 * 2 * F8_BK) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8DS_SC_P, false, false, W4AP_EPI_DEFERRED>), dim3(g), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 265:     // ZC (EPI 8): v20 with src C = 0 in each tile's first K-tile
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, false, false, W4AP_EPI_STAGED_ZC>), dim3(g), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 266:     // ZC square raster (v21 + ZC)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, true, true, W4AP_EPI_STAGED_ZC>), dim3(256), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 271:     // VP + PA form of p_zc (ZC, EPI 8) on the square raster, serpentine K (262 + ZC)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_STAGED_ZC, 2>), dim3(256), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 272:     // 271 with the LEAN epilogue (EPI 15, PA row map)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_LEAN, 2>), dim3(256), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 273:     // VP + PA p_zc, linear raster and K, LEAN epilogue
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, false, false, W4AP_EPI_LEAN, 2>), dim3(g), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 274:     // 272 with the LEAN_PIPE epilogue (EPI 16)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_LEAN_PIPE, 2>), dim3(256), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 275:     // v20 (p_zc, linear) with the LEAN_PIPE epilogue
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, false, false, W4AP_EPI_LEAN_PIPE>), dim3(g), dim3(F8_THREADS), 0,
                         s, a, b, c, M, N, K);
      break;
    case 276:     // 274 with LEAN_ILV (EPI 17)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_LEAN_ILV, 2>), dim3(256), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 277:     // 276 with LEAN_ILVB (EPI 18)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8VP_SC_P_ZC, true, true, W4AP_EPI_LEAN_ILVB, 2>), dim3(256), dim3(F8_THREADS),
                         0, s, a, b, c, M, N, K);
      break;
    case 269:     // LEAN epilogue (EPI 15) for v20 (p_zc, linear K)
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, false, false, W4AP_EPI_LEAN>), dim3(g), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 270:     // LEAN epilogue for v21 (square raster)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, true, true, W4AP_EPI_LEAN>), dim3(256), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 267:     // WG512 epilogue (EPI 10) for v20 (p_zc, linear K)
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, false, false, W4AP_EPI_WG512>), dim3(g), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 268:     // WG512 epilogue for v21 (square raster)
      if (g < NXCD || !sq) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<F8AP_SC_P_ZC, true, true, W4AP_EPI_WG512>), dim3(256), dim3(F8_THREADS), 0, s,
                         a, b, c, M, N, K);
      break;
    case 231:     // knock-out: 200 with the epilogue but without its global C stores
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<0, false, false, 3>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    case 230:     // knock-out: q16ap schedule p, linear K, without the epilogue
      if (g < NXCD) return (int)hipErrorInvalidValue;
      hipLaunchKernelGGL((gemm_fp8_256x256_q16ap<0, false, false, 1>), dim3(g), dim3(F8_THREADS), 0, s, a, b, c, M, N, K);
      break;
    default:
      return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // extern "C"
