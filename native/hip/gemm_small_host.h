// Host side of the 128x128 small-grid kernels (gemm_small.h), shared by the bf16 and fp8 dispatches:
// the split-K piece count, the per-(device, stream) workspace, and the launch.
#pragma once

#include <map>
#include <mutex>
#include <thread>
#include <tuple>
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

// The split-K form of the 256x256 asm frame (bf16 v57, fp8 v24; gemm_w4ap.h SPLIT): K pieces per
// tile -- as many as fit the CUs in one wave (cus / tiles), each of at least kAsmPieceMinKt K-tiles (an
// even count); 1 = no split. At most 2 for grids of more than a quarter of the CUs (the measured band),
// at most 4 below that: four pieces of a 64-tile grid win at K 16384 (2048^2x16384 1189 vs 1012 TF/s
// for the 128x128 kernel, 1.07x hipBLASLt) and lose at 8192 (900-918 vs 977; three pieces tie),
// profiles/r6_splitk/tree_s34.jsonl, order_s34.jsonl.
constexpr int kAsmPieceMinKt = 16;
constexpr int kAsmMaxSplits = 4;
// The last piece's default share of K: 52 % (profiles/r6_splitk/band_bf16.jsonl, band_fp8.jsonl: +1-5 %
// over even pieces at K 4096-8192; the first piece's slab stores and release run under the last one's
// K-loop).
constexpr int kAsmLastPermille = 520;
// Sweep knobs of the split-K asm form, per host thread (amdgo_gemm_set_asm_split): a forced piece count
// (0 = the automatic one below; forced pieces keep >= 4 K-tiles), the last piece's share of K in
// permille (0 = kAsmLastPermille; 500 = even pieces) and the item order.
struct AsmSplitKnobs {
  int splits = 0;
  int last_permille = 0;
  int piece_major = 0;   // 1: piece-major items; 0 (default): a tile's pieces adjacent, on one XCD, so the
                         // last arrival reads the other slab from its own L2 (2048x4096x8192 1309 -> 1329,
                         // 2560^3 735 -> 811 TF/s; profiles/r6_splitk/order_s2.jsonl)
};
inline AsmSplitKnobs& asm_split_knobs() {
  static thread_local AsmSplitKnobs k;
  return k;
}
inline int asm_splits(int tiles, int nk, int cus) {
  if (tiles <= 0) return 1;
  if (const int forced = asm_split_knobs().splits) {
    const int s = forced < nk / 4 ? forced : nk / 4;
    return s > 1 ? s : 1;
  }
  int s = cus / tiles;
  const int most = nk / kAsmPieceMinKt;
  if (s > most) s = most;
  const int cap = 4 * tiles > cus ? 2 : kAsmMaxSplits;
  if (s > cap) s = cap;
  return s > 1 ? s : 1;
}
inline int asm_piece_major() { return asm_split_knobs().piece_major; }
// K-tile pairs of the last piece (0 = even pieces). The tile's last arrival sums the others' slabs; a
// longer last piece lets the other pieces' slab stores and release run under its K-loop instead of
// after it. Every piece keeps >= 2 pairs.
inline int asm_last_pairs(int nk, int splits) {
  // the longer last piece is measured for two pieces; three and four run even (2048^2x16384: 4 even
  // 1189, the last 28 % 1179, 31 % 1118 TF/s)
  const int pm = asm_split_knobs().last_permille ? asm_split_knobs().last_permille
                                                 : (splits == 2 ? kAsmLastPermille : 0);
  if (splits < 2 || pm <= 0) return 0;
  const int pairs = nk / 2;
  const int last = (pairs * pm + 500) / 1000;
  if (last < 2 || pairs - last < 2 * (splits - 1)) return 0;
  return last;
}
constexpr size_t kAsmSlabFloats = 256 * 256;   // one 256x256 fp32 partial per (tile, piece)

// v61's item order: piece-major for pieces of >= 32 K-tiles (gemm_small.h, gemm_mfma_small_sk).
inline int small_piece_major(int nk, int splits) { return nk / splits >= 32 ? 1 : 0; }

// v61's fp32 partials (one 128x128 slab per workgroup) and per-tile arrival counters, one set per
// (device, stream): two GEMMs in flight on different streams never share them; a launch on one stream
// resets its counters before it ends, so the next launch there finds them zero. The device is the
// stream's (hipStreamGetDevice), not the caller's current one, and the allocation is made on it: a
// launch on a cuda:1 stream while the current device is 0 must not get GPU 0 memory. The per-thread
// stream handle names a different stream in every host thread, so its key includes the thread.
// At most kSmallWorkspaces sets per device, least recently used evicted: a process that cycles streams
// (torch side streams, a stream per request) would otherwise grow HBM use without bound. Each set
// carries an event recorded after its last launch; eviction waits on that event, never on the stream
// (which the caller may have destroyed).
struct SmallWorkspace {
  float* ws = nullptr;
  int* cnt = nullptr;
  size_t floats = 0;
  int counters = 0;
  hipEvent_t done = nullptr;   // after the last launch that used this set
  uint64_t used = 0;           // LRU clock
};

constexpr int kSmallWorkspaces = 16;   // per device

struct SmallWorkspaceKey {
  int dev;
  hipStream_t s;
  std::thread::id tid;   // only for the per-thread stream handle
  bool operator<(const SmallWorkspaceKey& o) const { return std::tie(dev, s, tid) < std::tie(o.dev, o.s, o.tid); }
};

// Runs `f` with `dev` current, then restores the caller's device.
template <class F>
inline auto on_device(int dev, F&& f) {
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != dev) (void)hipSetDevice(dev);
  auto r = f();
  if (prev != dev && prev >= 0) (void)hipSetDevice(prev);
  return r;
}

inline void small_workspace_release(SmallWorkspace& w) {
  if (w.done) (void)hipEventSynchronize(w.done);
  if (w.ws) (void)hipFree(w.ws);
  if (w.cnt) (void)hipFree(w.cnt);
  if (w.done) (void)hipEventDestroy(w.done);
  w = SmallWorkspace{};
}

struct SmallWorkspaces {
  std::mutex mu;
  std::map<SmallWorkspaceKey, SmallWorkspace> all;
  uint64_t clock = 0;
};

inline SmallWorkspaces& small_workspaces() {
  static SmallWorkspaces* w = new SmallWorkspaces();   // never destroyed: no teardown-order hazard at exit
  return *w;
}

// Workspace sets currently held for `dev` (the GPU test of the LRU cap reads it).
inline int small_workspace_count(int dev) {
  SmallWorkspaces& W = small_workspaces();
  std::lock_guard<std::mutex> lk(W.mu);
  int n = 0;
  for (const auto& kv : W.all) n += kv.first.dev == dev;
  return n;
}

inline SmallWorkspace* small_workspace(hipStream_t s, size_t floats, int tiles) {
  int dev = 0;
  if (s != nullptr && s != hipStreamPerThread) {
    if (hipStreamGetDevice(s, &dev) != hipSuccess) return nullptr;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return nullptr;
  }
  const SmallWorkspaceKey key{dev, s, s == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id()};
  SmallWorkspaces& W = small_workspaces();
  std::lock_guard<std::mutex> lk(W.mu);
  auto it = W.all.find(key);
  if (it == W.all.end()) {
    // a new set: evict this device's least recently used one at the cap
    int held = 0;
    auto lru = W.all.end();
    for (auto j = W.all.begin(); j != W.all.end(); ++j)
      if (j->first.dev == dev) {
        ++held;
        if (lru == W.all.end() || j->second.used < lru->second.used) lru = j;
      }
    if (held >= kSmallWorkspaces && lru != W.all.end()) {
      on_device(dev, [&] { small_workspace_release(lru->second); return 0; });
      W.all.erase(lru);
    }
    it = W.all.emplace(key, SmallWorkspace{}).first;
  }
  SmallWorkspace& w = it->second;
  w.used = ++W.clock;
  const bool ok = on_device(dev, [&] {
    if (!w.done && hipEventCreateWithFlags(&w.done, hipEventDisableTiming) != hipSuccess) return false;
    if (w.floats < floats) {
      // a larger partial buffer: the old one may still be read by a launch in flight on this stream
      if (w.ws && hipEventSynchronize(w.done) != hipSuccess) return false;
      if (w.ws) (void)hipFree(w.ws);
      w.ws = nullptr;
      w.floats = 0;
      if (hipMalloc(&w.ws, floats * sizeof(float)) != hipSuccess) return false;
      w.floats = floats;
    }
    if (w.counters < tiles) {
      if (w.cnt && hipEventSynchronize(w.done) != hipSuccess) return false;
      if (w.cnt) (void)hipFree(w.cnt);
      w.cnt = nullptr;
      w.counters = 0;
      const int n = tiles < 1024 ? 1024 : tiles;
      if (hipMalloc(&w.cnt, n * sizeof(int)) != hipSuccess) return false;
      if (hipMemsetAsync(w.cnt, 0, n * sizeof(int), s) != hipSuccess) return false;
      w.counters = n;
    }
    return true;
  });
  return ok ? &w : nullptr;
}

// v60 (split = false) or v61: split-K when the grid has pieces to give, else v60. Host guarantees M, N multiples
// of 128 and K a whole number of 128-byte K-tiles.
// REC: the placement-recording instantiations (gemm_tile_common.h note_placement).
template <bool F8, int BMT = 128, Rec REC = kTimed>
inline void launch_small(const void* a, const void* b, __bf16* c, int M, int N, int K, hipStream_t s, int cus, bool split) {
  const int tiles = (M / BMT) * (N / S_BN);
  const int nk = (int)((size_t)K * (F8 ? 1 : 2) / 128);
  const int splits = split ? small_splits(tiles, nk, cus) : 1;
  SmallWorkspace* w = splits > 1 ? small_workspace(s, (size_t)tiles * splits * BMT * S_BN, 2 * tiles) : nullptr;
  if (w) {
    hipLaunchKernelGGL((gemm_mfma_small_sk<F8, BMT, REC>), dim3(tiles * splits), dim3(S_THREADS), 0, s, a, b, c, M, N,
                       K, splits, small_piece_major(nk, splits), w->ws, w->cnt);
    (void)hipEventRecord(w->done, s);
  } else {
    hipLaunchKernelGGL((gemm_mfma_small<F8, BMT, REC>), dim3(tiles), dim3(S_THREADS), 0, s, a, b, c, M, N, K);
  }
}
