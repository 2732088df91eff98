// Shared pieces of the validator's CDNA4 (gfx950) GEMM kernels (gemm_bf16.hip, gemm_fp8.hip):
// address-space casts for LDS-DMA, the XCD-aware workgroup remap and grouped raster, the raw
// workgroup barrier and a compile-time loop. Everything lives in an anonymous namespace: each
// kernel TU gets its own copy, nothing is exported from the shared library.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>

// Every AGPR, for inline-asm kernels that pin their accumulators in a0..a255 by hand.
#define W4_AGPR_CLOBBERS \
  "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", \
  "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", \
  "a31", "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", \
  "a46", "a47", "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", \
  "a61", "a62", "a63", "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", \
  "a76", "a77", "a78", "a79", "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", \
  "a91", "a92", "a93", "a94", "a95", "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", \
  "a105", "a106", "a107", "a108", "a109", "a110", "a111", "a112", "a113", "a114", "a115", "a116", "a117", \
  "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127", "a128", "a129", "a130", \
  "a131", "a132", "a133", "a134", "a135", "a136", "a137", "a138", "a139", "a140", "a141", "a142", "a143", \
  "a144", "a145", "a146", "a147", "a148", "a149", "a150", "a151", "a152", "a153", "a154", "a155", "a156", \
  "a157", "a158", "a159", "a160", "a161", "a162", "a163", "a164", "a165", "a166", "a167", "a168", "a169", \
  "a170", "a171", "a172", "a173", "a174", "a175", "a176", "a177", "a178", "a179", "a180", "a181", "a182", \
  "a183", "a184", "a185", "a186", "a187", "a188", "a189", "a190", "a191", "a192", "a193", "a194", "a195", \
  "a196", "a197", "a198", "a199", "a200", "a201", "a202", "a203", "a204", "a205", "a206", "a207", "a208", \
  "a209", "a210", "a211", "a212", "a213", "a214", "a215", "a216", "a217", "a218", "a219", "a220", "a221", \
  "a222", "a223", "a224", "a225", "a226", "a227", "a228", "a229", "a230", "a231", "a232", "a233", "a234", \
  "a235", "a236", "a237", "a238", "a239", "a240", "a241", "a242", "a243", "a244", "a245", "a246", "a247", \
  "a248", "a249", "a250", "a251", "a252", "a253", "a254", "a255"

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int GROUP_M = 8;   // tile rows per raster group (L2 panel reuse)
constexpr int NXCD = 8;      // MI355X: 8 XCDs, each with a private 4 MiB L2

// Bijective for any nwg: blocks b and b+8 share an XCD (observed round-robin dispatch); give
// each XCD a contiguous run of logical tiles so co-resident tiles share A/B panels in its L2.
__host__ __device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid % NXCD;
  const int q = nwg / NXCD;
  const int r = nwg % NXCD;
  const int start = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return start + bid / NXCD;
}

// Launch grid of the persistent 256x256 kernels: one workgroup per CU, a multiple of 8 (whole XCD
// groups), and every tile in the first round when the grid has fewer tiles than CUs -- rounding
// down instead (100 tiles on 96 workgroups) ran 4 tiles in a second round at half the chip's
// throughput (2560^3 416 TF/s; profiles/r5_small/). Workgroups past their XCD's tiles exit at once.
__host__ inline int persistent_launch_grid(int nwg, int cus) {
  const int whole = (cus / NXCD) * NXCD;
  if (nwg >= whole) return whole;
  const int up = (nwg + NXCD - 1) / NXCD * NXCD;
  return up <= whole ? up : whole;
}

// Grouped raster: GROUP_M tile rows walk the N tiles together.
__host__ __device__ __forceinline__ void tile_coords(int wgid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int per_group = GROUP_M * tiles_n;
  const int group = wgid / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = tiles_m - first_m < GROUP_M ? tiles_m - first_m : GROUP_M;
  const int in_group = wgid - group * per_group;
  tm = first_m + in_group % gsize;
  tn = in_group / gsize;
}

// Square cross-XCD raster (v45): one dispatch wave of 256 workgroups (32 per XCD, one per CU)
// covers a 16x16-tile super-tile; XCD x owns its 8x4 sub-block (rows 8*(x&1), cols 4*(x>>1)).
// Per wave the chip then streams 16 A + 16 B panels instead of 64 A + 4 B (16384^3) or
// 32 A + 8 B (8192^3) for the XCD-contiguous raster, and XCD pairs / quads read the same B / A
// panel K-slices at the same time (MALL hits). Consecutive waves walk N inside a super-row (an
// XCD keeps its A panels, so serpentine K still finds their K-slices in L2); super-rows snake.
// Host guarantees tiles_m % 16 == 0 and tiles_n % 16 == 0, so the map is a bijection.
__host__ __device__ __forceinline__ void tile_coords_sq(int bid, int tiles_n, int& tm, int& tn) {
  const int wave = bid >> 8;
  const int xcd = bid & (NXCD - 1);
  const int slot = (bid & 255) >> 3;
  const int sn = tiles_n >> 4;
  const int sr = wave / sn;
  int sc = wave - sr * sn;
  if (sr & 1) sc = sn - 1 - sc;
  tm = (sr << 4) + ((xcd & 1) << 3) + (slot & 7);
  tn = (sc << 4) + ((xcd >> 1) << 2) + (slot >> 3);
}

// The rasters above are __host__ too: the host mirrors a dispatch's tile -> workgroup map with the very
// functions the kernels run (gemm_raster_host.h), so amd-gemm-validate can name the workgroup behind a
// bad output tile.

// Placement record (REC instantiations only, amd-gemm-validate's checked dispatch): workgroup b stores
// the XCD it ran on (HW_REG_XCC_ID) and its hardware id (HW_REG_HW_ID: CU, SH and SE) at
// g_wg_placement[2b], [2b+1]. blockIdx % 8 only says which workgroups share an XCD, not which XCD
// (MI355X_MICROARCH.md, "Workgroup dispatch"); the record says which one, and which CU. One lane, two
// plain vector stores, before anything else -- the REC=false kernels (every timed dispatch) do not
// contain it. One copy of the pointer per TU and device; set from the host before a REC launch.
__device__ uint32_t* g_wg_placement = nullptr;

// A kernel's instantiation: timed (every production launch) or placement-recording. An enum, not a
// bool, so the two are told apart by name in the code object (tests/test_gemm_build.py).
enum Rec : int { kTimed = 0, kRecord = 1 };

template <Rec REC>
__device__ __forceinline__ void note_placement() {
  if constexpr (REC == kRecord) {
    if (threadIdx.x == 0 && g_wg_placement != nullptr) {
      uint32_t xcc, hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      const uint32_t b = blockIdx.x + blockIdx.y * gridDim.x;
      g_wg_placement[2 * b] = xcc;
      g_wg_placement[2 * b + 1] = hw;
    }
  }
}

// Raw s_barrier pinned in place (no implicit vmcnt(0) as __syncthreads() would emit).
__device__ __forceinline__ void bar() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// Host: compute units of the device a launch on `stream` runs on (cached per device; 256 on MI355X,
// 32 on a CPX partition). The stream's device, not the calling thread's current one: a process that
// drives several devices (or an SPX GPU next to CPX partitions) launches on streams of devices other
// than the current one, and a grid sized for the wrong device over- or under-fills by up to 8x. A null
// stream is the current device's. The serpentine-K variants assume NXCD x 32 co-resident workgroups
// (one per CU) and are only picked at 256.
inline int device_cu_count(hipStream_t stream = nullptr) {
  static int cus[64] = {0};
  int dev = 0;
  if (stream != nullptr) {
    if (hipStreamGetDevice(stream, &dev) != hipSuccess) return 0;
  } else if (hipGetDevice(&dev) != hipSuccess) {
    return 0;
  }
  if (dev < 0 || dev >= 64) return 0;
  int n = __atomic_load_n(&cus[dev], __ATOMIC_RELAXED);
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    __atomic_store_n(&cus[dev], n, __ATOMIC_RELAXED);
  }
  return n;
}

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// A 16-byte C store with the nontemporal (streaming) hint: `global_store_dwordx4 ... nt`. The C tile is
// written once and never re-read by the kernel; streaming it keeps the write-allocated lines from
// filling L2 under the operand panels and shortens the wait on the stores (the next tile's landing
// wait, the end-of-kernel release): persistent asm pipeline +1.1 % at 8192^3, +6.3 % with one
// dispatch wave (4096^2x16384), fp8 +4.9 % at 4096^3 (profiles/r3_s2/nt_*.jsonl).
__device__ __forceinline__ void store_c16(void* p, uint4 v) {
  typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
  u32x4_nt x;
  x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4_nt*>(p));
}

}  // namespace
