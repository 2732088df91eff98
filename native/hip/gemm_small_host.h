// Host side of the 128x128 small-grid kernels (gemm_small.h), shared by the bf16 and fp8 dispatches:
// the split-K piece count, the per-(device, stream) workspace, and the launch.
#pragma once

#include <map>
#include <mutex>
#include <utility>

#include "gemm_small.h"

// The split-K target (workgroups per CU) a caller set (amdgo_gemm_set_split_target): per host thread.
inline int& small_split_target() {
  static thread_local int t = 1;
  return t;
}

// v61's K pieces per tile: target x CUs / tiles, at most one per 16 K-tiles; 1 = no split (v60).
inline int small_splits(int tiles, int nk, int cus) {
  if (tiles <= 0) return 1;
  int splits = small_split_target() * cus / tiles;
  if (splits > nk / 16) splits = nk / 16;
  // pieces as short as 16 K-tiles only while that keeps the grid within half the chip: their
  // reduction outweighs the extra CUs (1024^2x4096: 4 pieces of 16 on 256 CUs 330 TF/s, 2 of 32 on
  // 128 CUs 355; fp8 1024^2x8192 661 -> 724; 512^2x8192 keeps 8 of 16 on 128 CUs;
  // profiles/r5_small/sweep_piece32.jsonl)
  if (splits > 1 && nk / splits <= 16) {
    const int half = small_split_target() * cus / 2 / tiles;
    if (half < splits) splits = half;
  }
  return splits > 1 ? splits : 1;
}

// v61's fp32 partials (one 128x128 slab per workgroup) and per-tile arrival counters, one set per
// (device, stream): two GEMMs in flight on different streams never share them; a launch on one stream
// resets its counters before it ends, so the next launch there finds them zero. Allocated on first
// use, never shrunk.
struct SmallWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;
  size_t floats = 0;
  int counters = 0;
};

inline SmallWorkspace* small_workspace(hipStream_t s, size_t floats, int tiles) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, SmallWorkspace> all;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(mu);
  SmallWorkspace& w = all[{dev, s}];
  if (w.floats < floats) {
    // a larger partial buffer: the old one may still be read by a launch in flight on this stream
    if (w.ws && hipStreamSynchronize(s) != hipSuccess) return nullptr;
    if (w.ws) (void)hipFree(w.ws);
    w.ws = nullptr;
    w.floats = 0;
    if (hipMalloc(&w.ws, floats * sizeof(float)) != hipSuccess) return nullptr;
    w.floats = floats;
  }
  if (w.counters < tiles) {
    if (w.cnt && hipStreamSynchronize(s) != hipSuccess) return nullptr;
    if (w.cnt) (void)hipFree(w.cnt);
    w.cnt = nullptr;
    w.counters = 0;
    const int n = tiles < 1024 ? 1024 : tiles;
    if (hipMalloc(&w.cnt, n * sizeof(int)) != hipSuccess) return nullptr;
    if (hipMemsetAsync(w.cnt, 0, n * sizeof(int), s) != hipSuccess) return nullptr;
    w.counters = n;
  }
  return &w;
}

// v60 (split = false) or v61: split-K when the grid has pieces to give, else v60. Host guarantees M, N multiples
// of 128 and K a whole number of 128-byte K-tiles.
template <bool F8, int BMT = 128>
inline void launch_small(const void* a, const void* b, __bf16* c, int M, int N, int K, hipStream_t s, int cus, bool split) {
  const int tiles = (M / BMT) * (N / S_BN);
  const int nk = (int)((size_t)K * (F8 ? 1 : 2) / 128);
  const int splits = split ? small_splits(tiles, nk, cus) : 1;
  SmallWorkspace* w = splits > 1 ? small_workspace(s, (size_t)tiles * splits * BMT * S_BN, tiles) : nullptr;
  if (w)
    hipLaunchKernelGGL((gemm_mfma_small_sk<F8, BMT>), dim3(tiles * splits), dim3(S_THREADS), 0, s, a, b, c, M, N, K,
                       splits, nk / splits >= 32 ? 1 : 0, w->ws, w->cnt);
  else
    hipLaunchKernelGGL((gemm_mfma_small<F8, BMT>), dim3(tiles), dim3(S_THREADS), 0, s, a, b, c, M, N, K);
}
