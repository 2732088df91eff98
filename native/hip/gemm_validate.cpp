// amd-gemm-validate: the validator's matrix-core probe (replaces the reference's vectorAdd,
// validator/cuda-workload-validation.yaml:20; the reference gates only on its exit code,
// validator/main.go:1176-1211 -- this probe also gates on throughput).
//
// Runs the hand-written CDNA4 MFMA GEMMs -- bf16 (gemm_bf16.hip) and/or fp8 e4m3fn on the
// double-rate matrix-core path (gemm_fp8.hip) -- concurrently on the selected GPUs on uniform
// [-1,1) operands; checks every output element (ABFT tile checksums, below) and sampled rows against an
// independent fp32 reference kernel; prints
// one JSON line per (dtype, GPU, shape) and an aggregate line.
//
// One process per GPU (--launch processes, the default): this process never
// touches the GPU. It enumerates the GPU agents this container may use from KFD sysfs (the HIP order),
// starts one worker per GPU -- itself with `--worker`, HIP_VISIBLE_DEVICES naming that one GPU --
// and meets the workers of each GPU set at a rendezvous over their stdin/stdout pipes. No HIP runtime
// is shared between GPUs, so no host-side lock of one runtime serialises eight GPUs' launches.
// --launch threads keeps the whole run in one process, one host thread per GPU (it is what runs
// under a profiler: rocprofv3 initialises the GPU in the process it starts, which must then not
// spawn programs).
//
// Timing protocol (the same as bench.py's, so the pod's number and the bench's agree):
//   1. --warmup untimed dispatches;
//   2. clock stabilisation, untimed: batches of 10 dispatches with an event between each, until
//      at least 50 dispatches ran and the last 10 per-dispatch times spread by < 2 % of their
//      median, capped at --stabilise-max-s (MI355X ramps its clock over the first ~25
//      back-to-back GEMMs; timing that transient under-reports steady state by 8-19 %);
//   3. every GPU of the set meets at the rendezvous -- a GPU that stabilised early idles there
//      until the slowest one arrives, and its clock drops while it waits;
//   4. the re-ramp, untimed: at least 10 dispatches and --ramp-ms of work, enqueued back to back
//      right after the rendezvous, with no host sync between them and the timed loop -- on sets of
//      2+ GPUs (a 1-GPU set waits for nobody); with --no-stabilise neither step 2 nor this one runs:
//      exactly --iters dispatches are issued;
//   5. the timed loop: at least --iters dispatches and at least --min-window-ms of work (sized from
//      the stabilised per-dispatch time), between two events -- a residual ramp is a small part of
//      a 100 ms window, not half of a 30 ms one.
// --pre-timed-idle-ms T inserts T ms of host-side idle after the rendezvous (the test of step 4).
//
// --scaling 1,2,4,8 runs the probe on N GPUs for each N (concurrently within one N) and adds
// `efficiency` = aggregate / (N x the 1-GPU figure) to each aggregate line; an N above the visible
// GPU count prints a `skipped` line instead of failing. A set of N takes one
// agent per PHYSICAL GPU first (agents grouped by PCI function: a CPX GPU shows one agent per
// partition); a set that must put two agents of one GPU together is measured and marked
// `shared_gpu`, and the efficiency gate does not apply to it (partitions of one GPU share its power
// and HBM, they are not independent GPUs).
//
// --min-efficiency E fails every scaling N > 1 whose efficiency is below E: independent GEMMs on
// separate GPUs should scale at ~1.0, so a shortfall is a GPU, power or cooling problem.
//
// --min-relative R compares the GPUs of this run with each other: per (dtype, shape) each GPU's best
// TFLOP/s against the node median (upper median), one `uniformity` line each; a GPU below R x median
// fails. Boxes differ by ~6 % in absolute terms, so absolute floors cannot be tight; a sick GPU next to
// 7 healthy siblings stands out here.
//
// Memory: before allocating, each GPU's free HBM (hipMemGetInfo) is compared with what the shape needs;
// a shortfall (or an allocation failure) is reported as `"oom":true` with need / free bytes and no
// kernel is launched -- on a GPU a tenant holds, the validator maps that to "skipped: busy".
//
// Every failing line carries a structured `kind`: "correctness" (a wrong result, a failed launch or
// allocation, a lost worker), "oom", "floor", "efficiency" or "uniformity" -- the validator decides
// what a failure means from it, never from the wording of `error`.
//
// Exit status 0 only if every check passed and every GPU reached its floor (--min-tflops for
// bf16, --min-tflops-fp8 for fp8; 0 = no floor) and the two gates above. The floors are fractions of
// the dense peak, so they apply to shapes that can reach it: at least one full dispatch wave of
// 256x256 tiles (M*N >= 256 * 256^2) and K >= 4096; smaller shapes are checked for correctness.
//
//   amd-gemm-validate [--shapes 8192,4096,16384x16384x1024] [--dtype bf16|fp8|both] [--iters 50]
//                     [--warmup 5] [--devices all|0,1,...] [--scaling 1,2,4,8] [--check-rows 32]
//                     [--min-tflops X] [--min-tflops-fp8 Y] [--min-efficiency E] [--min-relative R]
//                     [--stabilise-max-s 6] [--no-stabilise] [--smoke] [--launch processes|threads]
//                     [--min-window-ms 100] [--ramp-ms 60] [--pre-timed-idle-ms 0] [--inject-fault TM,TN[,DELTA]]
//
// Correctness (every set, every GPU): after the timed loop, C is poisoned with NaN and one more dispatch
// runs through the placement-recording instantiation of the same kernel (each workgroup stores the XCD
// and CU it ran on); the ABFT check (gemm_abft.hip) then verifies every output element through per-tile
// row and column checksums and names each bad tile, the workgroup that computed it (the dispatch's raster,
// gemm_raster_host.h), its XCD and CU: {"kind":"correctness","tile":[TM,TN],"xcd":X,"cu":{..}}. The
// --check-rows sampled rows against an independent fp32 reference stay as a second opinion.
// --inject-fault TM,TN[,DELTA] adds DELTA (default 64) to one element of tile (TM, TN) of that C, between
// the dispatch and the check (the GPU test of the naming).
//
// --smoke first runs hip-smoke (smoke.hip: the vectorAdd analogue, every element checked on the
// host) on each selected GPU and prints its `hip-smoke` line -- in the workers, so the validator's
// critical path starts one HIP runtime per GPU, not two.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <poll.h>
#include <csignal>
#include <spawn.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "amdnode.h"
#include "validate_protocol.h"

using namespace vproto;

extern char** environ;

extern "C" {
int amdgo_gemm_bf16(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream);
int amdgo_gemm_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out, int N, int K,
                        void* stream);
int amdgo_fill_uniform_bf16(void* p, size_t n, uint32_t seed, void* stream);
int amdgo_gemm_fp8(const void* A, const void* Bt, void* C, int M, int N, int K, void* stream);
int amdgo_gemm_fp8_ref_rows(const void* A, const void* Bt, const int* rows, int nrows, float* out, int N,
                            int K, void* stream);
int amdgo_fill_uniform_fp8(void* p, size_t n, uint32_t seed, void* stream);
int amdgo_vector_add_f32(const float* a, const float* b, float* c, size_t n, void* stream);
int amdgo_gemm_bf16_placed(const void* A, const void* Bt, void* C, int M, int N, int K, uint32_t* placement,
                           void* stream);
int amdgo_gemm_fp8_placed(const void* A, const void* Bt, void* C, int M, int N, int K, uint32_t* placement,
                          void* stream);
int amdgo_gemm_bf16_raster(int M, int N, int K, int* info, int* owners, int* rounds, int cap);
int amdgo_gemm_fp8_raster(int M, int N, int K, int* info, int* owners, int* rounds, int cap);
long long amdgo_abft_workspace_bytes(int M, int N, int K, int TM, int TN);
int amdgo_abft_check(int dtype, const void* A, const void* Bt, const void* C, int M, int N, int K, int TM, int TN,
                     void* ws, long long ws_bytes, int* tile_flags, float* worst_ratio, void* stream);
int amdgo_abft_inject(void* C, int M, int N, int row, int col, float delta, void* stream);
int amdgo_gemm_bf16_placement_init();
int amdgo_gemm_fp8_placement_init();
int amdgo_rows_max_rel_err(const void* C, const int* rows, int nrows, const float* ref, int N, void* scratch,
                           float* max_rel_err, void* stream);
}

static constexpr size_t kSmokeElements = 50000;

// hip-smoke on each device (the amd-hip-smoke binary's check, in this process): fp32 C = A + B over
// 50,000 elements, every element verified on the host. Returns the number of failing devices.
static int smoke_failures(const std::vector<int>& devs) {
  constexpr size_t n = kSmokeElements;
  std::vector<float> a(n), b(n), c(n);
  for (size_t i = 0; i < n; ++i) {
    a[i] = (float)(i % 1000) / 7.0f;
    b[i] = (float)((i * 7) % 1000) / 13.0f;
  }
  int failures = 0;
  for (int d : devs) {
    float *da = nullptr, *db = nullptr, *dc = nullptr;
    bool ok = hipSetDevice(d) == hipSuccess && hipMalloc(&da, n * 4) == hipSuccess &&
              hipMalloc(&db, n * 4) == hipSuccess && hipMalloc(&dc, n * 4) == hipSuccess &&
              hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess &&
              hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess &&
              amdgo_vector_add_f32(da, db, dc, n, nullptr) == 0 &&
              hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost) == hipSuccess;
    for (size_t i = 0; ok && i < n; ++i) ok = c[i] == a[i] + b[i];
    for (float* p : {da, db, dc})
      if (p) (void)hipFree(p);
    failures += !ok;
  }
  return failures;
}

static void print_smoke(size_t devices, int failures) {
  std::printf("{\"event\":\"hip-smoke\",\"devices\":%zu,\"elements\":%zu,\"ok\":%s%s}\n", devices, kSmokeElements,
              failures ? "false" : "true", failures ? ",\"kind\":\"correctness\"" : "");
  std::fflush(stdout);
}

// One operand precision: element size plus its GEMM, reference and fill entry points, the
// placement-recording dispatch and raster of the checked dispatch, and its ABFT operand code.
struct DType {
  const char* name;
  size_t esize;
  int (*gemm)(const void*, const void*, void*, int, int, int, void*);
  int (*ref_rows)(const void*, const void*, const int*, int, float*, int, int, void*);
  int (*fill)(void*, size_t, uint32_t, void*);
  int (*placed)(const void*, const void*, void*, int, int, int, uint32_t*, void*);
  int (*raster)(int, int, int, int*, int*, int*, int);
  int abft_dtype;
};
static const DType kBf16{"bf16", 2, amdgo_gemm_bf16, amdgo_gemm_ref_rows, amdgo_fill_uniform_bf16,
                         amdgo_gemm_bf16_placed, amdgo_gemm_bf16_raster, 0};
static const DType kFp8{"fp8_e4m3fn", 1, amdgo_gemm_fp8, amdgo_gemm_fp8_ref_rows, amdgo_fill_uniform_fp8,
                        amdgo_gemm_fp8_placed, amdgo_gemm_fp8_raster, 1};

static const DType* dtype_by_name(const std::string& n) {
  if (n == kBf16.name) return &kBf16;
  if (n == kFp8.name) return &kFp8;
  return nullptr;
}

// Record the failing call in r.error and return false from run_one; the Resources destructor
// frees whatever was allocated before the failure.
#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      r.error = std::string(#x) + ": " + hipGetErrorString(e_);                           \
      return false;                                                                       \
    }                                                                                     \
  } while (0)

// Reusable thread rendezvous (std::barrier is C++20 and clashes with HIP's __barrier).
class Rendezvous {
 public:
  explicit Rendezvous(size_t n) : n_(n) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(m_);
    const size_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != gen; });
  }

 private:
  std::mutex m_;
  std::condition_variable cv_;
  size_t n_, count_ = 0, gen_ = 0;
};

// Every device object of one run_one call; freed on every return path.
struct Resources {
  void *A = nullptr, *B = nullptr, *C = nullptr, *abft_ws = nullptr, *scratch = nullptr;
  float* ref = nullptr;
  int* rows = nullptr;
  uint32_t* placement = nullptr;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> events;
  ~Resources() {
    if (st) (void)hipStreamSynchronize(st);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    for (void* p : {A, B, C, abft_ws, scratch, (void*)ref, (void*)rows, (void*)placement})
      if (p) (void)hipFree(p);
    if (st) (void)hipStreamDestroy(st);
  }
};

// Whether the per-GPU floors apply to this shape (see the header).
static bool floor_applies(const Shape& s) { return (double)s.m * s.n >= 256.0 * 65536.0 && s.k >= 4096; }

static std::string json_safe(std::string s) {
  for (char& c : s)
    if (c == '"' || c == '\\' || c == '\n' || c == '\r') c = '\'';
  return s;
}

// Clock stabilisation (see the header): returns false on a launch/event error. r.stab_ms is the
// median per-dispatch time of the last window (what the re-ramp and the timed window are sized from).
static bool stabilise(const DType& dt, const Shape& s, Resources& res, const Options& o, Result& r) {
  constexpr int kBatch = 10, kMin = 50, kWindow = 10;
  constexpr double kTol = 0.02;
  std::vector<hipEvent_t> ev(kBatch + 1);
  for (auto& e : ev) {
    CHECK(hipEventCreate(&e));
    res.events.push_back(e);
  }
  std::vector<float> times;
  const auto t_end = std::chrono::steady_clock::now() +
                     std::chrono::microseconds((long long)(o.stabilise_max_s * 1e6));
  for (;;) {
    CHECK(hipEventRecord(ev[0], res.st));
    for (int i = 0; i < kBatch; ++i) {
      const int err = dt.gemm(res.A, res.B, res.C, s.m, s.n, s.k, res.st);
      if (err) {
        r.error = std::string("gemm launch: ") + hipGetErrorString((hipError_t)err);
        return false;
      }
      CHECK(hipEventRecord(ev[i + 1], res.st));
    }
    CHECK(hipEventSynchronize(ev[kBatch]));
    for (int i = 0; i < kBatch; ++i) {
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
      times.push_back(ms);
    }
    std::vector<float> last(times.end() - kWindow, times.end());
    std::sort(last.begin(), last.end());
    const double med = last[kWindow / 2];
    r.stab_ms = med;
    r.stab_spread = med > 0 ? (last.back() - last.front()) / med : 0.0;
    r.stab_dispatches = (int)times.size();
    if (((int)times.size() >= kMin && r.stab_spread < kTol) || std::chrono::steady_clock::now() > t_end) return true;
  }
}

// One GPU's probe of one (dtype, shape). `barrier` is the set's rendezvous; it is reached exactly once
// on every path, also when setup fails early, or the other GPUs of the set would wait forever.
static bool run_one(const DType& dt, int dev, const Shape& s, const Options& o, const std::function<void()>& barrier,
                    int set_size, Result& r) {
  r.device = dev;
  r.s = s;
  struct Arrive {
    const std::function<void()>& b;
    bool done = false;
    void now() {
      if (!done && b) b();
      done = true;
    }
    ~Arrive() { now(); }
  } arrive{barrier};
  CHECK(hipSetDevice(dev));
  Resources res;  // declared after Arrive: freed (and the stream drained) before the rendezvous
  CHECK(hipStreamCreateWithFlags(&res.st, hipStreamNonBlocking));
  const auto t_probe = std::chrono::steady_clock::now();
  const size_t na = (size_t)s.m * s.k, nb = (size_t)s.n * s.k, nc = (size_t)s.m * s.n;
  const int check_rows = std::max(1, std::min(o.check_rows, s.m));
  // the checked dispatch's raster: its output tile (the ABFT strips), launch grid (the placement
  // record's size) and the ABFT workspace
  int info[8] = {0};
  dt.raster(s.m, s.n, s.k, info, nullptr, nullptr, 0);
  const int tile_m = info[2], tile_n = info[3], tiles_m = info[4], tiles_n = info[5], grid = info[6],
            pieces = info[7];
  const long long abft_bytes = amdgo_abft_workspace_bytes(s.m, s.n, s.k, tile_m, tile_n);
  if (abft_bytes < 0 || grid <= 0) {
    r.error = "no ABFT layout for this shape";
    return false;
  }
  r.abft.variant = info[0];
  r.abft.tile_m = tile_m;
  r.abft.tile_n = tile_n;
  // what this shape needs against what the GPU has free: a tenant may hold most of the HBM
  // (+ the reference rows' pool scratch: the gathered rows and up to 8 K-slices of 2 x rows x N floats)
  r.need_bytes = na * dt.esize + nb * dt.esize + nc * 2 + (size_t)check_rows * s.n * 4 + (size_t)check_rows * 4 +
                 (size_t)abft_bytes + (size_t)grid * 8 + 256 + (size_t)check_rows * s.k * 4 +
                 (size_t)16 * check_rows * s.n * 4;
  size_t total = 0;
  CHECK(hipMemGetInfo(&r.free_bytes, &total));
  if (r.need_bytes > r.free_bytes) {
    r.oom = true;
    char buf[160];
    std::snprintf(buf, sizeof buf, "out of memory: the shape needs %.2f GiB, %.2f GiB of %.2f GiB free",
                  r.need_bytes / 1073741824.0, r.free_bytes / 1073741824.0, total / 1073741824.0);
    r.error = buf;
    return false;
  }
  auto alloc = [&](void** p, size_t bytes, const char* what) {
    const hipError_t e = hipMalloc(p, bytes);
    if (e == hipSuccess) return true;
    r.oom = e == hipErrorOutOfMemory;
    r.error = std::string(r.oom ? "out of memory: " : "") + "hipMalloc(" + what + "): " + hipGetErrorString(e);
    return false;
  };
  if (!alloc(&res.A, na * dt.esize, "A") || !alloc(&res.B, nb * dt.esize, "B") || !alloc(&res.C, nc * 2, "C") ||
      !alloc((void**)&res.ref, (size_t)check_rows * s.n * 4, "ref") || !alloc((void**)&res.rows, check_rows * 4, "rows") ||
      !alloc(&res.abft_ws, (size_t)abft_bytes, "abft") || !alloc((void**)&res.placement, (size_t)grid * 8, "placement") ||
      !alloc(&res.scratch, 256, "scratch"))
    return false;
  if (dt.fill(res.A, na, 1000 + dev, res.st) || dt.fill(res.B, nb, 2000 + dev, res.st)) {
    r.error = "fill failed";
    return false;
  }
  auto launch = [&](int n) {
    for (int i = 0; i < n; ++i) {
      const int err = dt.gemm(res.A, res.B, res.C, s.m, s.n, s.k, res.st);
      if (err) {
        r.error = std::string("gemm launch: ") + hipGetErrorString((hipError_t)err);
        return false;
      }
    }
    return true;
  };
  if (!launch(o.warmup)) return false;
  CHECK(hipStreamSynchronize(res.st));
  if (o.stabilise && !stabilise(dt, s, res, o, r)) return false;
  // the re-ramp and the timed window, sized from the stabilised dispatch time; without the clock
  // protocol (--no-stabilise: a correctness probe, a profiled single dispatch) exactly --iters. A
  // one-GPU set waits for nobody at its rendezvous (tens of microseconds through the pipes): no idle,
  // no re-ramp -- unless the test hook injects one.
  const bool ramp = o.stabilise && (set_size > 1 || o.pre_idle_ms > 0);
  r.ramp = ramp ? 10 : 0;
  r.iters = o.iters;
  if (o.stabilise && r.stab_ms > 0) {
    if (ramp) r.ramp = std::max(r.ramp, (int)std::ceil(o.ramp_ms / r.stab_ms));
    // +5 %: the stabilisation median runs a little above the steady state the timed loop reaches (a
    // 100 ms target timed 98.9 ms: 149 x 0.664 ms)
    r.iters = std::max(r.iters, (int)std::ceil(1.05 * o.min_window_ms / r.stab_ms));
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  res.events.push_back(e0);
  CHECK(hipEventCreate(&e1));
  res.events.push_back(e1);
  arrive.now();  // all GPUs of the set start together
  if (o.pre_idle_ms > 0) std::this_thread::sleep_for(std::chrono::microseconds((long long)(o.pre_idle_ms * 1e3)));
  if (!launch(r.ramp)) return false;  // back to the steady clock after the idle at the rendezvous
  CHECK(hipEventRecord(e0, res.st));  // no host sync between the re-ramp and the timed loop
  if (!launch(r.iters)) return false;
  CHECK(hipEventRecord(e1, res.st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  r.ms = ms / r.iters;
  r.tflops = 2.0 * s.m * s.n * (double)s.k / (r.ms * 1e-3) / 1e12;
  r.launched = true;
  // The checked dispatch: C poisoned with NaN (a tile nobody writes fails, a stale one cannot pass
  // for fresh), one dispatch through the placement-recording instantiation of the same kernel, then
  // the ABFT check of every output element; the sampled fp32 rows are a second opinion on that C.
  const auto t_check = std::chrono::steady_clock::now();
  CHECK(hipMemsetAsync(res.C, 0xFF, nc * 2, res.st));
  CHECK(hipMemsetAsync(res.placement, 0xFF, (size_t)grid * 8, res.st));
  if (const int err = dt.placed(res.A, res.B, res.C, s.m, s.n, s.k, res.placement, res.st)) {
    r.error = std::string("checked dispatch: ") + hipGetErrorString((hipError_t)err);
    return false;
  }
  CHECK(hipStreamSynchronize(res.st));
  if (o.inject_tm >= 0 && o.inject_tn >= 0) {
    const int row = std::min(s.m - 1, o.inject_tm * tile_m + tile_m / 2);
    const int col = std::min(s.n - 1, o.inject_tn * tile_n + tile_n / 3);
    if (amdgo_abft_inject(res.C, s.m, s.n, row, col, (float)o.inject_delta, res.st)) {
      r.error = "inject failed";
      return false;
    }
  }
  std::vector<int> flags((size_t)tiles_m * tiles_n, 0);
  float worst = 0.f;
  const auto t_abft = std::chrono::steady_clock::now();
  if (const int err = amdgo_abft_check(dt.abft_dtype, res.A, res.B, res.C, s.m, s.n, s.k, tile_m, tile_n, res.abft_ws,
                                       abft_bytes, flags.data(), &worst, res.st)) {
    r.error = std::string("ABFT check: ") + hipGetErrorString((hipError_t)err);
    return false;
  }
  const auto ms_since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  AbftOut& ab = r.abft;
  ab.abft_ms = ms_since(t_abft);
  ab.dispatch_ms = std::chrono::duration<double, std::milli>(t_abft - t_check).count();
  ab.ran = true;
  ab.worst_ratio = worst;
  ab.checked_fraction = 1.0;   // every element is in one row sum and one column sum (gemm_abft.hip)
  for (int f : flags) ab.bad_tiles += f != 0;
  if (ab.bad_tiles) {
    // name the bad tiles: raster -> workgroup (per piece) -> that workgroup's placement record
    std::vector<int> owners((size_t)tiles_m * tiles_n * pieces), rounds(owners.size());
    std::vector<uint32_t> place((size_t)grid * 2);
    dt.raster(s.m, s.n, s.k, info, owners.data(), rounds.data(), (int)owners.size());
    CHECK(hipMemcpy(place.data(), res.placement, place.size() * 4, hipMemcpyDeviceToHost));
    int listed = 0;
    for (int t = 0; t < tiles_m * tiles_n; ++t) {
      if (!flags[t]) continue;
      int xcd = -2, wg = -1, round = -1;
      uint32_t hw = 0xFFFFFFFFu;
      for (int p = 0; p < pieces; ++p) {
        const int b = owners[(size_t)t * pieces + p];
        const int x = b >= 0 && b < grid && place[2 * b] != 0xFFFFFFFFu ? (int)(place[2 * b] & 0xF) : -1;
        if (p == 0) wg = b, round = rounds[(size_t)t * pieces], hw = b >= 0 && b < grid ? place[2 * b + 1] : hw;
        xcd = xcd == -2 ? x : (xcd == x ? xcd : -1);
      }
      if (ab.tm < 0) {
        ab.tm = t / tiles_n, ab.tn = t % tiles_n, ab.wg = wg, ab.round = round, ab.xcd = xcd;
        if (hw != 0xFFFFFFFFu) ab.cu = (hw >> 8) & 0xF, ab.sh = (hw >> 12) & 1, ab.se = (hw >> 13) & 7;
      }
      if (listed++ < 8)
        ab.list += (ab.list.empty() ? "" : ";") + std::to_string(t / tiles_n) + "." + std::to_string(t % tiles_n) + "." +
                   std::to_string(xcd);
    }
  }
  if (ab.list.empty()) ab.list = "-";
  // second opinion: sampled rows against the independent fp32 reference kernel
  const auto t_rows = std::chrono::steady_clock::now();
  std::vector<int> hrows(check_rows);
  for (int i = 0; i < check_rows; ++i) hrows[i] = (int)(((uint64_t)i * 2654435761u + dev) % s.m);
  CHECK(hipMemcpyAsync(res.rows, hrows.data(), check_rows * 4, hipMemcpyHostToDevice, res.st));
  if (dt.ref_rows(res.A, res.B, res.rows, check_rows, res.ref, s.n, s.k, res.st)) {
    r.error = "reference launch failed";
    return false;
  }
  float worst_rel_f = 0.f;
  if (const int err = amdgo_rows_max_rel_err(res.C, res.rows, check_rows, res.ref, s.n, res.scratch, &worst_rel_f,
                                             res.st)) {
    r.error = std::string("sampled-row compare: ") + hipGetErrorString((hipError_t)err);
    return false;
  }
  const double worst_rel = worst_rel_f;
  r.max_rel_err = worst_rel;
  ab.rows_ms = ms_since(t_rows);
  ab.check_ms = ms_since(t_check);
  const bool rows_ok = std::isfinite(worst_rel) && worst_rel <= 1.0 / 128;
  r.ok = rows_ok && ab.bad_tiles == 0;
  if (ab.bad_tiles) {
    char buf[192];
    std::snprintf(buf, sizeof buf, "ABFT: %d bad tile(s), first [%d,%d] (workgroup %d, XCD %d)%s", ab.bad_tiles, ab.tm,
                  ab.tn, ab.wg, ab.xcd, rows_ok ? "" : "; sampled rows also wrong");
    r.error = buf;
  } else if (!rows_ok) {
    r.error = "check failed: max_rel_err " + std::to_string(worst_rel);
  }
  r.probe_ms = ms_since(t_probe);
  return true;
}

// ---------------------------------------------------------------------------------------------
// The plan: every (dtype, shape, GPU set) in order, identical in every launch mode.
// ---------------------------------------------------------------------------------------------
struct Set {
  int id = 0;
  const DType* dt = nullptr;
  Shape s{};
  int scaling_n = 0;         // 0: no --scaling (every selected GPU)
  std::vector<int> slots;    // positions in the selected device list
  bool skipped = false;      // N above the visible GPUs
  bool shared_gpu = false;   // two agents of one physical GPU in the set
};

// `bdf[i]`: the PCI function of selected device i (empty: unknown, every device its own GPU).
static std::vector<Set> make_plan(const std::vector<const DType*>& dtypes, const std::vector<Shape>& shapes,
                                  const std::vector<int>& counts, size_t ndev, const std::vector<std::string>& bdf) {
  // scaling order: the first agent of each physical GPU, then the other agents
  std::vector<int> order, rest;
  std::set<std::string> seen;
  for (size_t i = 0; i < ndev; ++i) {
    const std::string key = i < bdf.size() && !bdf[i].empty() ? bdf[i] : "#" + std::to_string(i);
    (seen.insert(key).second ? order : rest).push_back((int)i);
  }
  order.insert(order.end(), rest.begin(), rest.end());
  std::vector<Set> plan;
  for (const DType* dt : dtypes)
    for (const auto& s : shapes) {
      if (counts.empty()) {
        Set st;
        st.dt = dt, st.s = s;
        for (size_t i = 0; i < ndev; ++i) st.slots.push_back((int)i);
        plan.push_back(st);
        continue;
      }
      // the 1-GPU figure every efficiency divides by: the N=1 run when the sweep has one, else a
      // 1-GPU run first
      std::vector<int> ns = counts;
      if (std::find(ns.begin(), ns.end(), 1) == ns.end()) ns.insert(ns.begin(), 1);
      std::stable_sort(ns.begin(), ns.end());
      for (int n : ns) {
        if (n < 1) continue;
        Set st;
        st.dt = dt, st.s = s, st.scaling_n = n;
        if ((size_t)n > ndev) {
          st.skipped = true;
        } else {
          st.slots.assign(order.begin(), order.begin() + n);
          std::set<std::string> gpus;
          for (int i : st.slots) gpus.insert(i < (int)bdf.size() && !bdf[i].empty() ? bdf[i] : "#" + std::to_string(i));
          st.shared_gpu = gpus.size() < st.slots.size();
        }
        plan.push_back(st);
      }
    }
  for (size_t i = 0; i < plan.size(); ++i) plan[i].id = (int)i;
  return plan;
}

struct Aggregate {
  double total = 0, per_gpu = 0, min_gpu = 0;
  bool ok = true;
};

// (dtype, m, n, k) -> device -> best TFLOP/s over every set it ran in (the --min-relative gate)
static std::map<std::tuple<std::string, int, int, int>, std::map<int, double>> g_best;

static const char* failure_kind(const Result& r, bool floor_ok) {
  if (r.oom) return "oom";
  if (!r.launched || !r.ok) return "correctness";
  if (!floor_ok) return "floor";
  return "";
}

// The ABFT fields of a gemm line: coverage, margin, cost, and the first bad tile named by workgroup,
// XCD and CU (gemm_abft.hip; the placement record of the checked dispatch).
static std::string abft_json(const Result& r) {
  const AbftOut& a = r.abft;
  if (!a.ran) return "";
  char buf[512];
  std::snprintf(buf, sizeof buf,
                ",\"checked_fraction\":%.3f,\"abft_worst_ratio\":%.4f,\"bad_tiles\":%d,\"variant\":%d,\"tile_m\":%d,"
                "\"tile_n\":%d,\"check_ms\":%.3f,\"check_dispatch_ms\":%.3f,\"abft_ms\":%.3f,\"check_rows_ms\":%.3f,"
                "\"probe_ms\":%.1f",
                a.checked_fraction, std::isfinite(a.worst_ratio) ? a.worst_ratio : 1e30, a.bad_tiles, a.variant, a.tile_m,
                a.tile_n, a.check_ms, a.dispatch_ms, a.abft_ms, a.rows_ms, r.probe_ms);
  std::string out = buf;
  if (a.bad_tiles > 0) {
    std::snprintf(buf, sizeof buf, ",\"tile\":[%d,%d],\"workgroup\":%d,\"round\":%d,\"xcd\":", a.tm, a.tn, a.wg,
                  a.round);
    out += buf;
    out += a.xcd >= 0 ? std::to_string(a.xcd) : "null";
    if (a.cu >= 0) {
      std::snprintf(buf, sizeof buf, ",\"cu\":{\"se\":%d,\"sh\":%d,\"cu\":%d}", a.se, a.sh, a.cu);
      out += buf;
    }
    // "tm.tn.xcd;..." -> [[tm,tn,xcd],...]
    std::string lst = ",\"bad_tile_list\":[";
    size_t pos = 0;
    bool first = true;
    while (a.list != "-" && pos < a.list.size()) {
      size_t e = a.list.find(';', pos);
      std::string item = a.list.substr(pos, e == std::string::npos ? std::string::npos : e - pos);
      pos = e == std::string::npos ? a.list.size() : e + 1;
      int tm = 0, tn = 0, x = 0;
      if (std::sscanf(item.c_str(), "%d.%d.%d", &tm, &tn, &x) != 3) continue;
      lst += (first ? "[" : ",[") + std::to_string(tm) + "," + std::to_string(tn) + "," +
             (x >= 0 ? std::to_string(x) : std::string("null")) + "]";
      first = false;
    }
    out += lst + "]";
  }
  return out;
}

// The per-GPU lines and the aggregate of one set (results in slot order).
static Aggregate report_set(const Set& set, std::vector<Result>& res, double floor, double single, double min_eff) {
  const DType& dt = *set.dt;
  const Shape& s = set.s;
  Aggregate agg;
  const std::string scal = set.scaling_n > 0 ? ",\"gpus\":" + std::to_string(set.scaling_n) : std::string();
  for (size_t i = 0; i < res.size(); ++i) {
    auto& r = res[i];
    const bool floor_ok = !floor_applies(s) || r.tflops >= floor;
    const bool ok = r.launched && r.ok && floor_ok;
    agg.ok = agg.ok && ok;
    agg.total += r.tflops;
    agg.min_gpu = i == 0 ? r.tflops : std::min(agg.min_gpu, r.tflops);
    std::string err = r.error;
    if (err.empty() && !ok && !floor_ok) {
      char buf[128];
      std::snprintf(buf, sizeof buf, "below floor: %.1f < %.1f TFLOP/s", r.tflops, floor);
      err = buf;
    }
    if (err.empty() && !ok) err = "check failed";
    err = json_safe(err);
    char oom[96] = "";
    if (r.oom)
      std::snprintf(oom, sizeof oom, ",\"oom\":true,\"need_bytes\":%zu,\"free_bytes\":%zu", r.need_bytes, r.free_bytes);
    const std::string kind = ok ? "" : std::string(",\"kind\":\"") + failure_kind(r, floor_ok) + "\"";
    std::printf("{\"event\":\"gemm\",\"dtype\":\"%s\",\"device\":%d%s,\"m\":%d,\"n\":%d,\"k\":%d,\"ms\":%.4f,"
                "\"tflops\":%.1f,\"max_rel_err\":%.3e,\"stabilise_dispatches\":%d,\"stabilise_spread\":%.4f,"
                "\"iters\":%d,\"ramp_dispatches\":%d,\"min_tflops\":%.1f%s,\"ok\":%s%s%s%s%s%s}\n",
                dt.name, r.device, scal.c_str(), s.m, s.n, s.k, r.ms, r.tflops,
                std::isfinite(r.max_rel_err) ? r.max_rel_err : 1e30, r.stab_dispatches, r.stab_spread, r.iters, r.ramp,
                floor_applies(s) ? floor : 0.0, abft_json(r).c_str(), ok ? "true" : "false", kind.c_str(), oom,
                err.empty() ? "" : ",\"error\":\"", err.c_str(), err.empty() ? "" : "\"");
    if (r.launched && r.ok) {
      double& best = g_best[{dt.name, s.m, s.n, s.k}][r.device];
      best = std::max(best, r.tflops);
    }
  }
  agg.per_gpu = res.empty() ? 0 : agg.total / res.size();
  std::string eff;
  if (set.scaling_n == 1 && agg.total > 0) single = agg.total;   // the 1-GPU run is its own reference
  if (set.scaling_n > 0 && single > 0) {
    const double e = agg.total / (set.scaling_n * single);
    const bool gated = set.scaling_n > 1 && min_eff > 0 && !set.shared_gpu;
    const bool eff_ok = !gated || e >= min_eff;
    char buf[160];
    std::snprintf(buf, sizeof buf, ",\"efficiency\":%.4f,\"min_efficiency\":%.2f%s%s", e, min_eff,
                  set.shared_gpu ? ",\"shared_gpu\":true,\"efficiency_gated\":false" : "",
                  eff_ok ? "" : ",\"efficiency_ok\":false");
    eff = buf;
    agg.ok = agg.ok && eff_ok;
  }
  // the aggregate's own kind: a failed GPU line carries the cause, the aggregate adds efficiency
  std::string kind;
  if (!agg.ok) {
    bool any_gpu_bad = false;
    for (const auto& r : res) any_gpu_bad = any_gpu_bad || !(r.launched && r.ok && (!floor_applies(s) || r.tflops >= floor));
    kind = any_gpu_bad ? "" : ",\"kind\":\"efficiency\"";
  }
  std::printf("{\"event\":\"aggregate\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%zu,\"total_tflops\":%.1f,"
              "\"per_gpu_tflops\":%.1f,\"min_gpu_tflops\":%.1f,\"min_tflops\":%.1f%s%s,\"ok\":%s%s}\n",
              dt.name, s.m, s.n, s.k, res.size(), agg.total, agg.per_gpu, agg.min_gpu, floor_applies(s) ? floor : 0.0,
              set.scaling_n > 0 ? ",\"scaling\":true" : "", eff.c_str(), agg.ok ? "true" : "false", kind.c_str());
  std::fflush(stdout);
  return agg;
}

static void print_skipped(const Set& set, size_t ndev) {
  std::printf("{\"event\":\"scaling\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%d,"
              "\"skipped\":\"%zu GPU(s) visible\"}\n",
              set.dt->name, set.s.m, set.s.n, set.s.k, set.scaling_n, ndev);
  std::fflush(stdout);
}

// Runs every set of the plan through `run` (which fills the set's results) and reports it; then the
// uniformity lines. Returns whether everything passed.
static bool run_plan(const std::vector<Set>& plan, size_t ndev, double min_tflops, double min_tflops_fp8,
                     double min_eff, double min_rel,
                     const std::function<void(const Set&, std::vector<Result>&)>& run) {
  bool all_ok = true;
  double single = 0;
  for (const Set& set : plan) {
    if (set.skipped) {
      print_skipped(set, ndev);
      continue;
    }
    if (set.scaling_n <= 1) single = 0;       // a new (dtype, shape): its 1-GPU figure comes first
    std::vector<Result> res(set.slots.size());
    run(set, res);
    const double floor = set.dt == &kFp8 ? min_tflops_fp8 : min_tflops;
    Aggregate a = report_set(set, res, floor, single, min_eff);
    if (set.scaling_n == 1) single = a.per_gpu;
    all_ok = a.ok && all_ok;
  }
  // uniformity: every GPU's best against the node's (upper) median, per dtype and shape
  for (const auto& [key, per_dev] : g_best) {
    if (per_dev.size() < 2) continue;
    std::vector<double> v;
    for (const auto& kv : per_dev) v.push_back(kv.second);
    std::sort(v.begin(), v.end());
    const double med = v[v.size() / 2];
    double worst = 1e30;
    std::string slow;
    for (const auto& [dev, t] : per_dev) {
      const double ratio = med > 0 ? t / med : 0;
      worst = std::min(worst, ratio);
      if (min_rel > 0 && ratio < min_rel) slow += (slow.empty() ? "" : ",") + std::to_string(dev);
    }
    const bool ok = slow.empty();
    all_ok = all_ok && ok;
    std::printf("{\"event\":\"uniformity\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%zu,"
                "\"median_tflops\":%.1f,\"min_ratio\":%.4f,\"min_relative\":%.2f,\"slow_devices\":[%s],\"ok\":%s%s}\n",
                std::get<0>(key).c_str(), std::get<1>(key), std::get<2>(key), std::get<3>(key), per_dev.size(), med,
                worst, min_rel, slow.c_str(), ok ? "true" : "false", ok ? "" : ",\"kind\":\"uniformity\"");
  }
  return all_ok;
}

// ---------------------------------------------------------------------------------------------
// One worker process per GPU
// ---------------------------------------------------------------------------------------------
// Worker -> launcher lines (the worker's stdout; its stderr is the launcher's):
//   S <hip device count> <bdf> <gcn arch> <cus> <lds per block>   after HIP init
//   H <0|1>                                                       hip-smoke result (--smoke)
//   W <set>                                                       at the set's rendezvous
//   R <set> <launched> <ok> <oom> <tflops> <ms> <max_rel_err> <stab dispatches> <stab spread>
//     <need bytes> <free bytes> <iters> <ramp> <error...>         the set's result
// Launcher -> worker: "P <sets>\n" once, after the start (and smoke) lines -- the worker's part of the
// plan, built over the workers that saw their GPU -- then "g\n" releases each rendezvous. EOF on stdin
// ends the worker.
struct Worker {
  int slot = 0;
  pid_t pid = -1;
  int to = -1, from = -1;
  std::string buf;
  bool alive = false;
  std::string why;

  // The next line from the worker within timeout_s; false (and the worker killed) on EOF or timeout.
  bool line(std::string& out, double timeout_s) {
    const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds((long long)(timeout_s * 1e6));
    while (alive) {
      const size_t nl = buf.find('\n');
      if (nl != std::string::npos) {
        out = buf.substr(0, nl);
        buf.erase(0, nl + 1);
        return true;
      }
      const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(end - std::chrono::steady_clock::now());
      if (left.count() <= 0) {
        fail("no reply within " + std::to_string((int)timeout_s) + " s");
        break;
      }
      pollfd p{from, POLLIN, 0};
      const int n = ::poll(&p, 1, (int)std::min<long long>(left.count(), 1000));
      if (n < 0 && errno != EINTR) {
        fail(std::string("poll: ") + std::strerror(errno));
        break;
      }
      if (n <= 0) continue;
      char tmp[4096];
      const ssize_t got = ::read(from, tmp, sizeof tmp);
      if (got > 0) {
        buf.append(tmp, (size_t)got);
      } else if (got == 0 || errno != EINTR) {
        fail("exited");
        break;
      }
    }
    return false;
  }
  void send(const char* s) {
    if (alive && ::write(to, s, std::strlen(s)) < 0) fail(std::string("write: ") + std::strerror(errno));
  }
  void fail(const std::string& w) {
    if (!alive) return;
    alive = false;
    int st = 0;
    if (::waitpid(pid, &st, WNOHANG) == 0) {
      ::kill(pid, SIGKILL);
      (void)::waitpid(pid, &st, 0);
    }
    char code[64] = "";
    if (WIFEXITED(st)) std::snprintf(code, sizeof code, " (exit %d)", WEXITSTATUS(st));
    else if (WIFSIGNALED(st)) std::snprintf(code, sizeof code, " (signal %d)", WTERMSIG(st));
    why = "worker for GPU " + std::to_string(slot) + " " + w + code;
    pid = -1;
  }
};

// The GPU agents this process may use, in HIP order, from KFD sysfs (no HIP call: the launcher
// must not initialise the GPU). KFD hides the properties of agents the device cgroup denies, so the
// list is what the HIP runtime will enumerate; ROCR_VISIBLE_DEVICES then HIP_VISIBLE_DEVICES narrow it
// the way the runtime does. `hip_index[i]` is agent i's index under ROCR_VISIBLE_DEVICES (what a
// worker's HIP_VISIBLE_DEVICES names). False when a visibility list is not numeric (UUIDs).
static bool visible_agents(std::vector<std::string>& bdf, std::vector<int>& hip_index) {
  const auto gpus = amdnode::enumerate_gpus("/");
  std::vector<int> idx;
  for (size_t i = 0; i < gpus.size(); ++i) idx.push_back((int)i);
  std::vector<int> sel;
  if (const char* r = std::getenv("ROCR_VISIBLE_DEVICES"); r && *r) {
    if (!parse_index_list(r, sel)) return false;
    std::vector<int> k;
    for (int x : sel)
      if (x >= 0 && x < (int)idx.size()) k.push_back(idx[x]);
    idx = k;
  }
  std::vector<int> under_rocr(idx.size());
  for (size_t i = 0; i < idx.size(); ++i) under_rocr[i] = (int)i;
  for (const char* var : {"HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"}) {
    const char* h = std::getenv(var);
    if (!h || !*h) continue;
    if (!parse_index_list(h, sel)) return false;
    std::vector<int> k, u;
    for (int x : sel)
      if (x >= 0 && x < (int)idx.size()) k.push_back(idx[x]), u.push_back(under_rocr[x]);
    idx = k, under_rocr = u;
    break;
  }
  bdf.clear();
  hip_index.clear();
  for (size_t i = 0; i < idx.size(); ++i) {
    bdf.push_back(gpus[idx[i]].pci_bdf);
    hip_index.push_back(under_rocr[i]);
  }
  return true;
}

static bool spawn_worker(Worker& w, int hip_index, const std::vector<std::string>& args) {
  int in[2], out[2];
  if (::pipe2(in, O_CLOEXEC) || ::pipe2(out, O_CLOEXEC)) return false;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, in[0], 0);
  posix_spawn_file_actions_adddup2(&fa, out[1], 1);
  std::vector<std::string> env_s;
  for (char** e = environ; *e; ++e)
    if (std::strncmp(*e, "HIP_VISIBLE_DEVICES=", 20) && std::strncmp(*e, "CUDA_VISIBLE_DEVICES=", 21)) env_s.push_back(*e);
  env_s.push_back("HIP_VISIBLE_DEVICES=" + std::to_string(hip_index));
  std::vector<char*> envp, argv;
  for (auto& s : env_s) envp.push_back(s.data());
  envp.push_back(nullptr);
  std::vector<std::string> a = args;
  for (auto& s : a) argv.push_back(s.data());
  argv.push_back(nullptr);
  pid_t pid = -1;
  const int rc = posix_spawn(&pid, "/proc/self/exe", &fa, nullptr, argv.data(), envp.data());
  posix_spawn_file_actions_destroy(&fa);
  ::close(in[0]);
  ::close(out[1]);
  if (rc != 0) {
    ::close(in[1]);
    ::close(out[0]);
    w.why = std::string("posix_spawn: ") + std::strerror(rc);
    return false;
  }
  w.pid = pid, w.to = in[1], w.from = out[0], w.alive = true;
  return true;
}

// --worker: one GPU (HIP device 0 under the HIP_VISIBLE_DEVICES the launcher set). After its start
// (and smoke) line it reads its part of the plan from stdin, "P <id>:<dtype>:<m>x<n>x<k>:<gpus>;..." --
// the sets it takes part in, in plan order, with their sizes -- or "Q" (no part: the launcher dropped it).
static int worker_main(const Options& o, bool run_smoke) {
  std::signal(SIGPIPE, SIG_IGN);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    std::printf("%s\n", fmt_start_line({0, "-", "-", 0, 0}).c_str());
    std::fflush(stdout);
    return 3;
  }
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  char bus[64] = "-";
  if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) std::strcpy(bus, "-");
  for (char* c = bus; *c; ++c) *c = (char)std::tolower(*c);
  std::printf("%s\n", fmt_start_line({ndev, bus, prop.gcnArchName, prop.multiProcessorCount,
                                       (size_t)prop.sharedMemPerBlock}).c_str());
  std::fflush(stdout);
  (void)hipSetDevice(0);
  (void)amdgo_gemm_bf16_placement_init();   // process setup of the checked dispatch, not the probe's
  (void)amdgo_gemm_fp8_placement_init();
  if (run_smoke) {
    std::printf("H %d\n", smoke_failures({0}) == 0 ? 1 : 0);
    std::fflush(stdout);
  }
  std::vector<PlanItem> items;
  {
    std::vector<char> line(1 << 16);
    if (!std::fgets(line.data(), (int)line.size(), stdin) || line[0] != 'P') return 0;
    if (!parse_plan_line(line.data(), items)) return 2;
  }
  for (const PlanItem& it : items) {
    const int id = it.id, set_size = it.set_size;
    const Shape s = it.s;
    const DType* dt = dtype_by_name(it.dtype);
    if (!dt) return 2;
    const std::function<void()> barrier = [&] {
      std::printf("W %d\n", id);
      std::fflush(stdout);
      char go[8];
      if (!std::fgets(go, sizeof go, stdin)) std::_Exit(4);   // the launcher is gone
    };
    Result r;
    run_one(*dt, 0, s, o, barrier, set_size, r);
    std::printf("%s\n", fmt_result_line(id, r).c_str());
    std::fflush(stdout);
  }
  return 0;
}

static constexpr double kWorkerReplyS = 600.0;   // one set's worst case is seconds; a GPU hang is not

// The launcher: one worker per selected GPU, the plan driven through their pipes. `all`: the
// device list is every agent sysfs showed (no --devices); an agent whose worker then sees no GPU
// (a container whose device cgroup hides it from the runtime but not from sysfs) is dropped and
// reported, not failed. With an explicit --devices it is a failure.
static int launch_processes(const std::vector<int>& devs_in, bool all, const std::vector<std::string>& bdf,
                            const std::vector<int>& hip_index, const std::vector<const DType*>& dtypes,
                            const std::vector<Shape>& shapes, const std::vector<int>& counts, const Options& o,
                            bool run_smoke, double min_tflops, double min_tflops_fp8, double min_eff, double min_rel) {
  std::signal(SIGPIPE, SIG_IGN);
  std::vector<Worker> spawned(devs_in.size());
  for (size_t i = 0; i < devs_in.size(); ++i) {
    spawned[i].slot = devs_in[i];
    std::vector<std::string> args = {"amd-gemm-validate", "--worker", "--worker-opts", fmt_opts(o)};
    if (run_smoke) args.push_back("--smoke");
    if (!spawn_worker(spawned[i], hip_index[devs_in[i]], args))
      spawned[i].why = "worker for GPU " + std::to_string(devs_in[i]) + ": " + spawned[i].why;
  }
  // start lines: the runtime's view of each worker's GPU, checked against the sysfs agent
  std::string arch = "unknown", dropped;
  int cus = 0;
  size_t lds = 0;
  std::vector<Worker> ws;
  for (auto& w : spawned) {
    std::string ln;
    if (w.line(ln, 300.0)) {
      StartLine sl;
      const bool parsed = parse_start_line(ln, sl);
      const int n = sl.ndev, c = sl.cus;
      const size_t l = sl.lds;
      const std::string bus = sl.bus, a = sl.arch;
      if (parsed && n < 1 && all) {
        dropped += (dropped.empty() ? "" : ",") + std::to_string(w.slot);
        w.fail("dropped: the runtime sees no GPU there");
        continue;
      }
      if (!parsed || n < 1) w.fail("saw no GPU (" + ln + ")");
      else if (!bdf[w.slot].empty() && std::string(bus) != "-" && bdf[w.slot] != bus)
        w.fail(std::string("opened ") + bus + ", not " + bdf[w.slot]);
      else if (arch == "unknown") arch = a, cus = c, lds = l;
    }
    ws.push_back(w);
  }
  if (ws.empty()) {
    std::printf("{\"error\":\"no AMD GPU visible to the runtime (sysfs agents %s)\"}\n", dropped.c_str());
    return 3;
  }
  std::vector<int> devs;
  std::vector<std::string> sel_bdf;
  for (const auto& w : ws) devs.push_back(w.slot), sel_bdf.push_back(bdf[w.slot]);
  const std::vector<Set> plan = make_plan(dtypes, shapes, counts, devs.size(), sel_bdf);
  std::printf("{\"event\":\"start\",\"devices\":%zu,\"visible\":%zu,\"gcn_arch\":\"%s\",\"cus\":%d,"
              "\"lds_per_block\":%zu,\"iters\":%d,\"stabilise\":%s,\"launch\":\"processes\",\"min_window_ms\":%.0f%s%s%s}\n",
              devs.size(), bdf.size(), arch.c_str(), cus, lds, o.iters, o.stabilise ? "true" : "false", o.min_window_ms,
              dropped.empty() ? "" : ",\"dropped\":[", dropped.c_str(), dropped.empty() ? "" : "]");
  std::fflush(stdout);
  bool all_ok = true;
  if (run_smoke) {
    int failures = 0;
    for (auto& w : ws) {
      std::string ln;
      failures += !(w.line(ln, 120.0) && ln == "H 1");
    }
    print_smoke(devs.size(), failures);
    all_ok = failures == 0;
  }
  // each worker's part of the plan
  for (size_t i = 0; i < ws.size(); ++i) {
    std::string sets;
    for (const Set& st : plan)
      if (std::find(st.slots.begin(), st.slots.end(), (int)i) != st.slots.end()) {
        sets += (sets.empty() ? "" : ";") + fmt_plan_item({st.id, st.dt->name, st.s, (int)st.slots.size()});
      }
    ws[i].send(("P " + sets + "\n").c_str());
  }
  auto lost = [&](Result& r, const Worker& w) {
    r.launched = false;
    r.error = w.why.empty() ? "worker for GPU " + std::to_string(w.slot) + " lost" : w.why;
  };
  all_ok = run_plan(plan, devs.size(), min_tflops, min_tflops_fp8, min_eff, min_rel,
                    [&](const Set& set, std::vector<Result>& res) {
                      const std::string want_w = "W " + std::to_string(set.id);
                      for (int slot : set.slots) {
                        std::string ln;
                        while (ws[slot].line(ln, kWorkerReplyS) && ln != want_w) {
                        }
                      }
                      for (int slot : set.slots) ws[slot].send("g\n");
                      for (size_t i = 0; i < set.slots.size(); ++i) {
                        Worker& w = ws[set.slots[i]];
                        res[i].device = w.slot;
                        res[i].s = set.s;
                        std::string ln;
                        int id = -1;
                        bool got = false;
                        while (w.line(ln, kWorkerReplyS))
                          if (ln.rfind("R ", 0) == 0 && parse_result_line(ln, id, res[i]) && id == set.id) {
                            got = true;
                            break;
                          }
                        if (!got) lost(res[i], w);
                      }
                    }) && all_ok;
  // the last line: every result is out; the workers' exits (the runtime's and the driver's teardown
  // of their GPU state, ~0.1 s on MI355X) are not waited for before it (workload_main.stream_run)
  std::printf("{\"event\":\"done\",\"ok\":%s}\n", all_ok ? "true" : "false");
  std::fflush(stdout);
  for (auto& w : ws) {
    if (w.to >= 0) ::close(w.to);
    if (w.pid > 0) (void)::waitpid(w.pid, nullptr, 0);
    if (w.from >= 0) ::close(w.from);
  }
  return all_ok ? 0 : 1;
}

// Launched under a profiler, the process already holds the GPU (rocprofv3's preloaded tool
// initialises it): it must not start other programs.
static bool under_profiler() {
  const char* p = std::getenv("LD_PRELOAD");
  return (p && std::strstr(p, "rocprof")) || std::getenv("ROCPROFILER_LIBRARY_CTOR") != nullptr;
}

int main(int argc, char** argv) {
  std::string shapes = "8192", devices = "all", dtype = "bf16", scaling, launch = "processes";
  std::string worker_opts;
  bool worker = false;
  Options o;
  double min_tflops = 0, min_tflops_fp8 = 0, min_eff = 0, min_rel = 0;
  bool run_smoke = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--shapes") shapes = next();
    else if (a == "--iters") o.iters = std::max(1, std::atoi(next().c_str()));
    else if (a == "--warmup") o.warmup = std::max(0, std::atoi(next().c_str()));
    else if (a == "--devices") devices = next();
    else if (a == "--dtype") dtype = next();
    else if (a == "--scaling") scaling = next();
    else if (a == "--check-rows") o.check_rows = std::atoi(next().c_str());
    else if (a == "--min-tflops") min_tflops = std::atof(next().c_str());
    else if (a == "--min-tflops-fp8") min_tflops_fp8 = std::atof(next().c_str());
    else if (a == "--min-efficiency") min_eff = std::atof(next().c_str());
    else if (a == "--min-relative") min_rel = std::atof(next().c_str());
    else if (a == "--stabilise-max-s") o.stabilise_max_s = std::atof(next().c_str());
    else if (a == "--no-stabilise") o.stabilise = false;
    else if (a == "--min-window-ms") o.min_window_ms = std::max(0.0, std::atof(next().c_str()));
    else if (a == "--ramp-ms") o.ramp_ms = std::max(0.0, std::atof(next().c_str()));
    else if (a == "--pre-timed-idle-ms") o.pre_idle_ms = std::max(0.0, std::atof(next().c_str()));
    else if (a == "--inject-fault") {
      const std::string v = next();
      double d = o.inject_delta;
      const int got = std::sscanf(v.c_str(), "%d,%d,%lf", &o.inject_tm, &o.inject_tn, &d);
      if (got < 2 || o.inject_tm < 0 || o.inject_tn < 0) {
        std::printf("{\"error\":\"--inject-fault wants TM,TN[,DELTA], got %s\"}\n", json_safe(v).c_str());
        return 2;
      }
      o.inject_delta = d;
    }
    else if (a == "--launch") launch = next();
    else if (a == "--smoke") run_smoke = true;
    else if (a == "--worker") worker = true;
    else if (a == "--worker-opts") worker_opts = next();
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-gemm-validate [--shapes 8192,4096,MxNxK] [--dtype bf16|fp8|both] [--iters N] "
                  "[--warmup N] [--devices all|0,1] [--scaling 1,2,4,8] [--check-rows N] [--min-tflops X] "
                  "[--min-tflops-fp8 Y] [--min-efficiency E] [--min-relative R] [--stabilise-max-s S] [--no-stabilise] "
                  "[--smoke] [--launch processes|threads] [--min-window-ms MS] [--ramp-ms MS] [--pre-timed-idle-ms MS] "
                  "[--inject-fault TM,TN[,DELTA]]\n");
      return 0;
    } else {
      std::printf("{\"error\":\"unknown argument %s\"}\n", json_safe(a).c_str());
      return 2;
    }
  }
  if (worker) {
    if (!worker_opts.empty() && !parse_opts(worker_opts, o)) return 2;
    return worker_main(o, run_smoke);
  }
  if (launch != "processes" && launch != "threads") {
    std::printf("{\"error\":\"unknown --launch %s (processes or threads)\"}\n", json_safe(launch).c_str());
    return 2;
  }
  std::vector<const DType*> dtypes;
  if (dtype == "bf16" || dtype == "both") dtypes.push_back(&kBf16);
  if (dtype == "fp8" || dtype == "both") dtypes.push_back(&kFp8);
  if (dtypes.empty()) {
    std::printf("{\"error\":\"unknown --dtype %s (bf16, fp8 or both)\"}\n", json_safe(dtype).c_str());
    return 2;
  }
  std::vector<Shape> shape_list;
  if (!parse_shapes_strict(shapes, shape_list)) {
    std::printf("{\"error\":\"bad --shapes %s (N or MxNxK, comma separated)\"}\n", json_safe(shapes).c_str());
    return 2;
  }
  for (const auto& s : shape_list)
    if (s.m <= 0 || s.n <= 0 || s.k <= 0) {
      std::printf("{\"error\":\"bad shape %dx%dx%d\"}\n", s.m, s.n, s.k);
      return 2;
    }
  const std::vector<int> counts = parse_ints(scaling);
  // the device list: from sysfs in the launcher (no HIP call), from the runtime with threads
  std::vector<std::string> bdf;
  std::vector<int> hip_index;
  if (launch == "processes" && (under_profiler() || !visible_agents(bdf, hip_index))) launch = "threads";
  int ndev = 0;
  if (launch == "processes") {
    ndev = (int)bdf.size();
  } else if (hipGetDeviceCount(&ndev) != hipSuccess) {
    ndev = 0;
  }
  if (ndev == 0) {
    std::printf("{\"error\":\"no AMD GPU visible\"}\n");
    return 3;
  }
  std::vector<int> devs;
  if (devices == "all") {
    for (int d = 0; d < ndev; ++d) devs.push_back(d);
  } else {
    for (int d : parse_ints(devices)) {
      if (d < 0 || d >= ndev) {
        std::printf("{\"error\":\"--devices names GPU %d but %d are visible\"}\n", d, ndev);
        return 2;
      }
      devs.push_back(d);
    }
  }
  if (devs.empty()) {
    std::printf("{\"error\":\"no device selected\"}\n");
    return 2;
  }
  if (launch == "processes")
    return launch_processes(devs, devices == "all", bdf, hip_index, dtypes, shape_list, counts, o, run_smoke, min_tflops,
                            min_tflops_fp8, min_eff, min_rel);

  // --launch threads: one process, one host thread per GPU
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, devs[0]);
  std::printf("{\"event\":\"start\",\"devices\":%zu,\"visible\":%d,\"gcn_arch\":\"%s\",\"cus\":%d,"
              "\"lds_per_block\":%zu,\"iters\":%d,\"stabilise\":%s,\"launch\":\"threads\",\"min_window_ms\":%.0f}\n",
              devs.size(), ndev, prop.gcnArchName, prop.multiProcessorCount, (size_t)prop.sharedMemPerBlock,
              o.iters, o.stabilise ? "true" : "false", o.min_window_ms);
  bool all_ok = true;
  for (int d : devs)
    if (hipSetDevice(d) == hipSuccess) (void)amdgo_gemm_bf16_placement_init(), (void)amdgo_gemm_fp8_placement_init();
  if (run_smoke) {
    const int failures = smoke_failures(devs);
    print_smoke(devs.size(), failures);
    all_ok = failures == 0;
  }
  std::vector<std::string> sel_bdf;
  for (int d : devs) {
    char bus[64] = "";
    sel_bdf.push_back(hipDeviceGetPCIBusId(bus, sizeof bus, d) == hipSuccess ? std::string(bus) : std::string());
  }
  const std::vector<Set> plan = make_plan(dtypes, shape_list, counts, devs.size(), sel_bdf);
  all_ok = run_plan(plan, devs.size(), min_tflops, min_tflops_fp8, min_eff, min_rel,
                    [&](const Set& set, std::vector<Result>& res) {
                      Rendezvous sync(set.slots.size());
                      const std::function<void()> barrier = [&] { sync.arrive_and_wait(); };
                      std::vector<std::thread> th;
                      for (size_t i = 0; i < set.slots.size(); ++i)
                        th.emplace_back([&, i] {
                          run_one(*set.dt, devs[set.slots[i]], set.s, o, barrier, (int)set.slots.size(), res[i]);
                        });
                      for (auto& t : th) t.join();
                    }) && all_ok;
  // the last line: every result is out and every device synchronised. The validator reads up to
  // here and lets the process exit on its own (the runtime's and the driver's teardown of this
  // process's GPU state takes ~0.1 s on MI355X after the last line; workload_main.stream_run).
  std::printf("{\"event\":\"done\",\"ok\":%s}\n", all_ok ? "true" : "false");
  std::fflush(stdout);
  return all_ok ? 0 : 1;
}
