// amd-gemm-validate: the validator's matrix-core probe (replaces the reference's vectorAdd,
// validator/cuda-workload-validation.yaml:20).
//
// Runs the hand-written CDNA4 MFMA GEMMs -- bf16 (gemm_bf16.hip) and/or fp8 e4m3fn on the
// double-rate matrix-core path (gemm_fp8.hip) -- concurrently on every selected GPU, one host
// thread per GPU, on uniform [-1,1) operands; checks sampled output rows against an independent
// fp32 reference kernel; prints one JSON line per (dtype, GPU, shape) and an aggregate line.
// Exit status 0 only if every check passed.
//
//   amd-gemm-validate [--shapes 8192,4096,16384x16384x1024] [--dtype bf16|fp8|both] [--iters 20]
//                     [--warmup 5] [--devices all|0,1,...] [--check-rows 32] [--min-tflops X]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
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

#define CHECK(x)                                                                          \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
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

struct Result {
  int device = 0;
  Shape s{};
  double tflops = 0, ms = 0, max_rel_err = 0;
  bool ok = false;
  std::string error;
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

static float bf16_to_f32(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

static bool run_one(const DType& dt, int dev, const Shape& s, int iters, int warmup, int check_rows,
                    Rendezvous* sync, Result& r) {
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
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  void *A, *B, *C;
  float* ref;
  int* rows;
  const size_t na = (size_t)s.m * s.k, nb = (size_t)s.n * s.k, nc = (size_t)s.m * s.n;
  CHECK(hipMalloc(&A, na * dt.esize));
  CHECK(hipMalloc(&B, nb * dt.esize));
  CHECK(hipMalloc(&C, nc * 2));
  CHECK(hipMalloc(&ref, (size_t)check_rows * s.n * 4));
  CHECK(hipMalloc(&rows, check_rows * 4));
  if (dt.fill(A, na, 1000 + dev, st) || dt.fill(B, nb, 2000 + dev, st)) {
    r.error = "fill failed";
    return false;
  }
  for (int i = 0; i < warmup; ++i) dt.gemm(A, B, C, s.m, s.n, s.k, st);
  CHECK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  arrive.now();   // all GPUs start the timed loop together
  CHECK(hipEventRecord(e0, st));
  for (int i = 0; i < iters; ++i) {
    int err = dt.gemm(A, B, C, s.m, s.n, s.k, st);
    if (err) {
      r.error = std::string("gemm launch: ") + hipGetErrorString((hipError_t)err);
      return false;
    }
  }
  CHECK(hipEventRecord(e1, st));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  r.ms = ms / iters;
  r.tflops = 2.0 * s.m * s.n * (double)s.k / (r.ms * 1e-3) / 1e12;
  // correctness on sampled rows against the independent fp32 reference kernel
  std::vector<int> hrows(check_rows);
  for (int i = 0; i < check_rows; ++i) hrows[i] = (int)(((uint64_t)i * 2654435761u + dev) % s.m);
  CHECK(hipMemcpyAsync(rows, hrows.data(), check_rows * 4, hipMemcpyHostToDevice, st));
  if (dt.ref_rows(A, B, rows, check_rows, ref, s.n, s.k, st)) {
    r.error = "reference launch failed";
    return false;
  }
  std::vector<float> href((size_t)check_rows * s.n);
  std::vector<uint16_t> hc((size_t)s.n);
  CHECK(hipMemcpyAsync(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost, st));
  CHECK(hipStreamSynchronize(st));
  double worst = 0;
  for (int i = 0; i < check_rows; ++i) {
    CHECK(hipMemcpy(hc.data(), (uint16_t*)C + (size_t)hrows[i] * s.n, s.n * 2, hipMemcpyDeviceToHost));
    for (int j = 0; j < s.n; ++j) {
      const double got = bf16_to_f32(hc[j]), want = href[(size_t)i * s.n + j];
      const double rel = std::fabs(got - want) / std::max(1.0, std::fabs(want));
      worst = std::max(worst, rel);
    }
  }
  r.max_rel_err = worst;
  r.ok = std::isfinite(worst) && worst <= 1.0 / 128;
  hipFree(A);
  hipFree(B);
  hipFree(C);
  hipFree(ref);
  hipFree(rows);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipStreamDestroy(st);
  return true;
}

int main(int argc, char** argv) {
  std::string shapes = "8192", devices = "all", dtype = "bf16";
  int iters = 20, warmup = 5, check_rows = 32;
  double min_tflops = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : ""); };
    if (a == "--shapes") shapes = next();
    else if (a == "--iters") iters = std::atoi(next().c_str());
    else if (a == "--warmup") warmup = std::atoi(next().c_str());
    else if (a == "--devices") devices = next();
    else if (a == "--dtype") dtype = next();
    else if (a == "--check-rows") check_rows = std::atoi(next().c_str());
    else if (a == "--min-tflops") min_tflops = std::atof(next().c_str());
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-gemm-validate [--shapes 8192,4096,MxNxK] [--dtype bf16|fp8|both] [--iters N] "
                  "[--warmup N] [--devices all|0,1] [--check-rows N] [--min-tflops X]\n");
      return 0;
    }
  }
  std::vector<const DType*> dtypes;
  if (dtype == "bf16" || dtype == "both") dtypes.push_back(&kBf16);
  if (dtype == "fp8" || dtype == "both") dtypes.push_back(&kFp8);
  if (dtypes.empty()) {
    std::printf("{\"error\":\"unknown --dtype %s (bf16, fp8 or both)\"}\n", dtype.c_str());
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
    for (auto& s : parse_shapes(devices)) devs.push_back(s.m);
  }
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, devs[0]);
  std::printf("{\"event\":\"start\",\"devices\":%zu,\"gcn_arch\":\"%s\",\"cus\":%d,\"lds_per_block\":%zu}\n",
              devs.size(), prop.gcnArchName, prop.multiProcessorCount, (size_t)prop.sharedMemPerBlock);
  bool all_ok = true;
  for (const DType* dt : dtypes) {
    for (const auto& s : parse_shapes(shapes)) {
      std::vector<Result> res(devs.size());
      Rendezvous sync(devs.size());
      std::vector<std::thread> th;
      std::vector<char> launched(devs.size(), 0);
      for (size_t i = 0; i < devs.size(); ++i)
        th.emplace_back([&, i] { launched[i] = run_one(*dt, devs[i], s, iters, warmup, check_rows, &sync, res[i]); });
      for (auto& t : th) t.join();
      double total = 0;
      for (size_t i = 0; i < devs.size(); ++i) {
        const auto& r = res[i];
        const bool ok = launched[i] && r.ok && r.tflops >= min_tflops;
        all_ok = all_ok && ok;
        total += r.tflops;
        std::printf("{\"event\":\"gemm\",\"dtype\":\"%s\",\"device\":%d,\"m\":%d,\"n\":%d,\"k\":%d,\"ms\":%.4f,\"tflops\":%.1f,"
                    "\"max_rel_err\":%.3e,\"ok\":%s%s%s%s}\n",
                    dt->name, r.device, s.m, s.n, s.k, r.ms, r.tflops, r.max_rel_err, ok ? "true" : "false",
                    r.error.empty() ? "" : ",\"error\":\"", r.error.c_str(), r.error.empty() ? "" : "\"");
      }
      std::printf("{\"event\":\"aggregate\",\"dtype\":\"%s\",\"m\":%d,\"n\":%d,\"k\":%d,\"gpus\":%zu,\"total_tflops\":%.1f,"
                  "\"per_gpu_tflops\":%.1f}\n",
                  dt->name, s.m, s.n, s.k, devs.size(), total, total / devs.size());
      std::fflush(stdout);
    }
  }
  return all_ok ? 0 : 1;
}
