// amd-gemm-validate: the validator's matrix-core probe (replaces the reference's vectorAdd,
// validator/cuda-workload-validation.yaml:20; the reference gates only on its exit code,
// validator/main.go:1176-1211 -- this probe also gates on throughput).
//
// Runs the hand-written CDNA4 MFMA GEMMs -- bf16 (gemm_bf16.hip) and/or fp8 e4m3fn on the
// double-rate matrix-core path (gemm_fp8.hip) -- concurrently on the selected GPUs, one host
// thread per GPU, on uniform [-1,1) operands; checks sampled output rows against an independent
// fp32 reference kernel; prints one JSON line per (dtype, GPU, shape) and an aggregate line.
//
// Timing protocol (the same as bench.py's, so the pod's number and the bench's agree):
//   1. --warmup untimed dispatches;
//   2. clock stabilisation, untimed: batches of 10 dispatches with an event between each, until
//      at least 50 dispatches ran and the last 10 per-dispatch times spread by < 2 % of their
//      median, capped at --stabilise-max-s (MI355X ramps its clock over the first ~25
//      back-to-back GEMMs; timing that transient under-reports steady state by 8-19 %);
//   3. every GPU's thread meets at a rendezvous, then --iters dispatches are timed between two
//      events.
//
// --scaling 1,2,4,8 runs the probe on GPUs 0..N-1 for each N (concurrently within one N) and adds
// `efficiency` = aggregate / (N x the 1-GPU figure) to each aggregate line; an N above the visible
// GPU count prints a `skipped` line instead of failing.
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
// Exit status 0 only if every check passed and every GPU reached its floor (--min-tflops for
// bf16, --min-tflops-fp8 for fp8; 0 = no floor) and the two gates above. The floors are fractions of
// the dense peak, so they apply to shapes that can reach it: at least one full dispatch wave of
// 256x256 tiles (M*N >= 256 * 256^2) and K >= 4096; smaller shapes are checked for correctness.
//
//   amd-gemm-validate [--shapes 8192,4096,16384x16384x1024] [--dtype bf16|fp8|both] [--iters 50]
//                     [--warmup 5] [--devices all|0,1,...] [--scaling 1,2,4,8] [--check-rows 32]
//                     [--min-tflops X] [--min-tflops-fp8 Y] [--min-efficiency E] [--min-relative R]
//                     [--stabilise-max-s 6] [--no-stabilise] [--smoke]
//
// --smoke first runs hip-smoke (smoke.hip: the vectorAdd analogue, every element checked on the
// host) on each selected GPU in this process and prints its `hip-smoke` line -- one HIP runtime
// start for both checks on the validator's critical path instead of two processes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

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
}

// hip-smoke on each device (the amd-hip-smoke binary's check, in this process): fp32 C = A + B over
// 50,000 elements, every element verified on the host.
static bool smoke(const std::vector<int>& devs) {
  constexpr size_t n = 50000;
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
  std::printf("{\"event\":\"hip-smoke\",\"devices\":%zu,\"elements\":%zu,\"ok\":%s}\n", devs.size(), n,
              failures ? "false" : "true");
  std::fflush(stdout);
  return failures == 0;
}

// One operand precision: element size plus its GEMM, reference and fill entry points.
struct DType {
  const char* name;
  size_t esize;
  int (*gemm)(const void*, const void*, void*, int, int, int, void*);
  int (*ref_rows)(const void*, const void*, const int*, int, float*, int, int, void*);
  int (*fill)(void*, size_t, uint32_t, void*);
};
static const DType kBf16{"bf16", 2, amdgo_gemm_bf16, amdgo_gemm_ref_rows, amdgo_fill_uniform_bf16};
static const DType kFp8{"fp8_e4m3fn", 1, amdgo_gemm_fp8, amdgo_gemm_fp8_ref_rows, amdgo_fill_uniform_fp8};

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

struct Shape {
  int m, n, k;
};

struct Options {
  int iters = 50, warmup = 5, check_rows = 32;
  double stabilise_max_s = 6.0;
  bool stabilise = true;
};

struct Result {
  int device = 0;
  Shape s{};
  double tflops = 0, ms = 0, max_rel_err = 0, stab_spread = -1;
  int stab_dispatches = 0;
  bool ok = false, oom = false;
  size_t need_bytes = 0, free_bytes = 0;
  std::string error;
};

// Every device object of one run_one call; freed on every return path.
struct Resources {
  void *A = nullptr, *B = nullptr, *C = nullptr;
  float* ref = nullptr;
  int* rows = nullptr;
  hipStream_t st = nullptr;
  std::vector<hipEvent_t> events;
  ~Resources() {
    if (st) (void)hipStreamSynchronize(st);
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    for (void* p : {A, B, C, (void*)ref, (void*)rows})
      if (p) (void)hipFree(p);
    if (st) (void)hipStreamDestroy(st);
  }
};

static std::vector<Shape> parse_shapes(const std::string& spec) {
  std::vector<Shape> out;
  size_t pos = 0;
  while (pos <= spec.size()) {
    size_t c = spec.find(',', pos);
    std::string t = spec.substr(pos, c == std::string::npos ? std::string::npos : c - pos);
    if (!t.empty()) {
      int m, n, k;
      if (std::sscanf(t.c_str(), "%dx%dx%d", &m, &n, &k) == 3) out.push_back({m, n, k});
      else out.push_back({std::atoi(t.c_str()), std::atoi(t.c_str()), std::atoi(t.c_str())});
    }
    if (c == std::string::npos) break;
    pos = c + 1;
  }
  return out;
}

static std::vector<int> parse_ints(const std::string& spec) {
  std::vector<int> out;
  for (const auto& s : parse_shapes(spec)) out.push_back(s.m);
  return out;
}

static float bf16_to_f32(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

// Whether the per-GPU floors apply to this shape (see the header).
static bool floor_applies(const Shape& s) { return (double)s.m * s.n >= 256.0 * 65536.0 && s.k >= 4096; }

// Clock stabilisation (see the header): returns false on a launch/event error.
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
    r.stab_spread = med > 0 ? (last.back() - last.front()) / med : 0.0;
    r.stab_dispatches = (int)times.size();
    if (((int)times.size() >= kMin && r.stab_spread < kTol) || std::chrono::steady_clock::now() > t_end) return true;
  }
}

static bool run_one(const DType& dt, int dev, const Shape& s, const Options& o, Rendezvous* sync, Result& r) {
  r.device = dev;
  r.s = s;
  // Every thread must reach the rendezvous exactly once, also when setup fails early,
  // or the other GPUs' threads would wait forever.
  struct Arrive {
    Rendezvous* r;
    bool done = false;
    void now() {
      if (r && !done) r->arrive_and_wait();
      done = true;
    }
    ~Arrive() { now(); }
  } arrive{sync};
  CHECK(hipSetDevice(dev));
  Resources res;  // declared after Arrive: freed (and the stream drained) before the rendezvous
  CHECK(hipStreamCreateWithFlags(&res.st, hipStreamNonBlocking));
  const size_t na = (size_t)s.m * s.k, nb = (size_t)s.n * s.k, nc = (size_t)s.m * s.n;
  const int check_rows = std::max(1, std::min(o.check_rows, s.m));
  // what this shape needs against what the GPU has free: a tenant may hold most of the HBM
  r.need_bytes = na * dt.esize + nb * dt.esize + nc * 2 + (size_t)check_rows * s.n * 4 + (size_t)check_rows * 4;
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
      !alloc((void**)&res.ref, (size_t)check_rows * s.n * 4, "ref") || !alloc((void**)&res.rows, check_rows * 4, "rows"))
    return false;
  if (dt.fill(res.A, na, 1000 + dev, res.st) || dt.fill(res.B, nb, 2000 + dev, res.st)) {
    r.error = "fill failed";
    return false;
  }
  for (int i = 0; i < o.warmup; ++i) {
    const int err = dt.gemm(res.A, res.B, res.C, s.m, s.n, s.k, res.st);
    if (err) {
      r.error = std::string("gemm launch: ") + hipGetErrorString((hipError_t)err);
      return false;
    }
  }
  CHECK(hipStreamSynchronize(res.st));
  if (o.stabilise && !stabilise(dt, s, res, o, r)) return false;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  res.events.push_back(e0);
  CHECK(hipEventCreate(&e1));
  res.events.push_back(e1);
  arrive.now();  // all GPUs start the timed loop together
  CHECK(hipEventRecord(e0, res.st));
  for (int i = 0; i < o.iters; ++i) {
    const int err = dt.gemm(res.A, res.B, res.C, s.m, s.n, s.k, res.st);
    if (err) {
      r.error = std::string("gemm launch: ") + hipGetErrorString((hipError_t)err);
      return false;
    }
  }
  CHECK(hipEventRecord(e1, res.st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  r.ms = ms / o.iters;
  r.tflops = 2.0 * s.m * s.n * (double)s.k / (r.ms * 1e-3) / 1e12;
  // correctness on sampled rows against the independent fp32 reference kernel
  std::vector<int> hrows(check_rows);
  for (int i = 0; i < check_rows; ++i) hrows[i] = (int)(((uint64_t)i * 2654435761u + dev) % s.m);
  CHECK(hipMemcpyAsync(res.rows, hrows.data(), check_rows * 4, hipMemcpyHostToDevice, res.st));
  if (dt.ref_rows(res.A, res.B, res.rows, check_rows, res.ref, s.n, s.k, res.st)) {
    r.error = "reference launch failed";
    return false;
  }
  std::vector<float> href((size_t)check_rows * s.n);
  std::vector<uint16_t> hc((size_t)s.n);
  CHECK(hipMemcpyAsync(href.data(), res.ref, href.size() * 4, hipMemcpyDeviceToHost, res.st));
  CHECK(hipStreamSynchronize(res.st));
  double worst = 0;
  for (int i = 0; i < check_rows; ++i) {
    CHECK(hipMemcpy(hc.data(), (uint16_t*)res.C + (size_t)hrows[i] * s.n, s.n * 2, hipMemcpyDeviceToHost));
    for (int j = 0; j < s.n; ++j) {
      const double got = bf16_to_f32(hc[j]), want = href[(size_t)i * s.n + j];
      const double rel = std::fabs(got - want) / std::max(1.0, std::fabs(want));
      worst = std::max(worst, rel);
    }
  }
  r.max_rel_err = worst;
  r.ok = std::isfinite(worst) && worst <= 1.0 / 128;
  return true;
}

struct Aggregate {
  double total = 0, per_gpu = 0, min_gpu = 0;
  bool ok = true;
};

// (dtype, m, n, k) -> device -> best TFLOP/s over every set it ran in (the --min-relative gate)
static std::map<std::tuple<std::string, int, int, int>, std::map<int, double>> g_best;

// One (dtype, shape) on a device set, concurrently; prints the per-GPU lines and the aggregate.
static Aggregate run_set(const DType& dt, const Shape& s, const std::vector<int>& devs, const Options& o,
                         double floor, int scaling_n, double single, double min_eff) {
  std::vector<Result> res(devs.size());
  Rendezvous sync(devs.size());
  std::vector<std::thread> th;
  std::vector<char> launched(devs.size(), 0);
  for (size_t i = 0; i < devs.size(); ++i)
    th.emplace_back([&, i] { launched[i] = run_one(dt, devs[i], s, o, &sync, res[i]); });
  for (auto& t : th) t.join();
  Aggregate agg;
  const std::string scal = scaling_n > 0 ? ",\"gpus\":" + std::to_string(scaling_n) : std::string();
  for (size_t i = 0; i < devs.size(); ++i) {
    const auto& r = res[i];
    const bool floor_ok = !floor_applies(s) || r.tflops >= floor;
    const bool ok = launched[i] && r.ok && floor_ok;
    agg.ok = agg.ok && ok;
    agg.total += r.tflops;
    agg.min_gpu = i == 0 ? r.tflops : std::min(agg.min_gpu, r.tflops);
    std::string err = r.error;
    if (err.empty() && launched[i] && r.ok && !floor_ok) {
      char buf[128];
      std::snprintf(buf, sizeof buf, "below floor: %.1f < %.1f TFLOP/s", r.tflops, floor);
      err = buf;
    }
    for (char& c : err)
      if (c == '"' || c == '\\') c = '\'';
    char oom[96] = "";
    if (r.oom)
      std::snprintf(oom, sizeof oom, ",\"oom\":true,\"need_bytes\":%zu,\"free_bytes\":%zu", r.need_bytes, r.free_bytes);
    std::printf("{\"event\":\"gemm\",\"dtype\":\"%s\",\"device\":%d%s,\"m\":%d,\"n\":%d,\"k\":%d,\"ms\":%.4f,"
                "\"tflops\":%.1f,\"max_rel_err\":%.3e,\"stabilise_dispatches\":%d,\"stabilise_spread\":%.4f,"
                "\"min_tflops\":%.1f,\"ok\":%s%s%s%s%s}\n",
                dt.name, r.device, scal.c_str(), s.m, s.n, s.k, r.ms, r.tflops, r.max_rel_err, r.stab_dispatches,
                r.stab_spread, floor_applies(s) ? floor : 0.0, ok ? "true" : "false", oom, err.empty() ? "" : ",\"error\":\"", err.c_str(),
                err.empty() ? "" : "\"");
    if (launched[i] && r.ok) {
      double& best = g_best[{dt.name, s.m, s.n, s.k}][r.device];
      best = std::max(best, r.tflops);
    }
  }
  agg.per_gpu = agg.total / devs.size();
  std::string eff;
  if (scaling_n == 1 && agg.total > 0) single = agg.total;   // the 1-GPU run is its own reference
  if (scaling_n > 0 && single > 0) {
    const double e = agg.total / (scaling_n * single);
    const bool eff_ok = scaling_n == 1 || min_eff <= 0 || e >= min_eff;
    char buf[96];
    std::snprintf(buf, sizeof buf, ",\"efficiency\":%.4f,\"min_efficiency\":%.2f%s", e, min_eff,
                  eff_ok ? "" : ",\"efficiency_ok\":false");
    eff = buf;
    agg.ok = agg.ok && eff_ok;
  }
  std::printf("{\"event\":\"aggregate\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%zu,\"total_tflops\":%.1f,"
              "\"per_gpu_tflops\":%.1f,\"min_gpu_tflops\":%.1f,\"min_tflops\":%.1f%s%s,\"ok\":%s}\n",
              dt.name, s.m, s.n, s.k, devs.size(), agg.total, agg.per_gpu, agg.min_gpu, floor_applies(s) ? floor : 0.0,
              scaling_n > 0 ? ",\"scaling\":true" : "", eff.c_str(), agg.ok ? "true" : "false");
  std::fflush(stdout);
  return agg;
}

int main(int argc, char** argv) {
  std::string shapes = "8192", devices = "all", dtype = "bf16", scaling;
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
    else if (a == "--smoke") run_smoke = true;
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-gemm-validate [--shapes 8192,4096,MxNxK] [--dtype bf16|fp8|both] [--iters N] "
                  "[--warmup N] [--devices all|0,1] [--scaling 1,2,4,8] [--check-rows N] [--min-tflops X] "
                  "[--min-tflops-fp8 Y] [--min-efficiency E] [--min-relative R] [--stabilise-max-s S] [--no-stabilise] "
                  "[--smoke]\n");
      return 0;
    } else {
      std::printf("{\"error\":\"unknown argument %s\"}\n", a.c_str());
      return 2;
    }
  }
  std::vector<const DType*> dtypes;
  if (dtype == "bf16" || dtype == "both") dtypes.push_back(&kBf16);
  if (dtype == "fp8" || dtype == "both") dtypes.push_back(&kFp8);
  if (dtypes.empty()) {
    std::printf("{\"error\":\"unknown --dtype %s (bf16, fp8 or both)\"}\n", dtype.c_str());
    return 2;
  }
  const std::vector<Shape> shape_list = parse_shapes(shapes);
  for (const auto& s : shape_list)
    if (s.m <= 0 || s.n <= 0 || s.k <= 0) {
      std::printf("{\"error\":\"bad shape %dx%dx%d\"}\n", s.m, s.n, s.k);
      return 2;
    }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
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
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, devs[0]);
  std::printf("{\"event\":\"start\",\"devices\":%zu,\"visible\":%d,\"gcn_arch\":\"%s\",\"cus\":%d,"
              "\"lds_per_block\":%zu,\"iters\":%d,\"stabilise\":%s}\n",
              devs.size(), ndev, prop.gcnArchName, prop.multiProcessorCount, (size_t)prop.sharedMemPerBlock,
              o.iters, o.stabilise ? "true" : "false");
  bool all_ok = true;
  if (run_smoke) all_ok = smoke(devs);
  const std::vector<int> counts = parse_ints(scaling);
  for (const DType* dt : dtypes) {
    const double floor = dt == &kFp8 ? min_tflops_fp8 : min_tflops;
    for (const auto& s : shape_list) {
      if (counts.empty()) {
        all_ok = run_set(*dt, s, devs, o, floor, 0, 0, 0).ok && all_ok;
        continue;
      }
      // the 1-GPU figure every efficiency divides by: the N=1 run when the sweep has one, else
      // a 1-GPU run first
      double single = 0;
      std::vector<int> order = counts;
      if (std::find(order.begin(), order.end(), 1) == order.end()) order.insert(order.begin(), 1);
      std::stable_sort(order.begin(), order.end());
      for (int n : order) {
        if (n < 1) continue;
        if ((size_t)n > devs.size()) {
          std::printf("{\"event\":\"scaling\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%d,"
                      "\"skipped\":\"%zu GPU(s) visible\"}\n",
                      dt->name, s.m, s.n, s.k, n, devs.size());
          continue;
        }
        std::vector<int> sub(devs.begin(), devs.begin() + n);
        Aggregate a = run_set(*dt, s, sub, o, floor, n, single, min_eff);
        if (n == 1) single = a.per_gpu;
        all_ok = a.ok && all_ok;
      }
    }
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
                "\"median_tflops\":%.1f,\"min_ratio\":%.4f,\"min_relative\":%.2f,\"slow_devices\":[%s],\"ok\":%s}\n",
                std::get<0>(key).c_str(), std::get<1>(key), std::get<2>(key), std::get<3>(key), per_dev.size(), med,
                worst, min_rel, slow.c_str(), ok ? "true" : "false");
  }
  // the last line: every result is out and every device synchronised. The validator reads up to
  // here and lets the process exit on its own (the runtime's and the driver's teardown of this
  // process's GPU state takes ~0.1 s on MI355X after the last line; workload_main.stream_run).
  std::printf("{\"event\":\"done\",\"ok\":%s}\n", all_ok ? "true" : "false");
  std::fflush(stdout);
  return all_ok ? 0 : 1;
}
