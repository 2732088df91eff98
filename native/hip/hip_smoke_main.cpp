// amd-hip-smoke: fp32 vector add on every visible GPU with full host verification — the
// functional analogue of the CUDA-samples vectorAdd the reference validator runs
// (validator/cuda-workload-validation.yaml:20). Prints one JSON line; exit 0 on success.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" int amdgo_vector_add_f32(const float* a, const float* b, float* c, size_t n, void* stream);

int main(int argc, char** argv) {
  size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 50000;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    std::printf("{\"event\":\"hip-smoke\",\"ok\":false,\"error\":\"no AMD GPU visible\"}\n");
    return 3;
  }
  std::vector<float> a(n), b(n), c(n);
  for (size_t i = 0; i < n; ++i) {
    a[i] = (float)(rand() % 1000) / 7.0f;
    b[i] = (float)(rand() % 1000) / 13.0f;
  }
  int failures = 0;
  for (int d = 0; d < ndev; ++d) {
    float *da, *db, *dc;
    if (hipSetDevice(d) != hipSuccess || hipMalloc(&da, n * 4) != hipSuccess || hipMalloc(&db, n * 4) != hipSuccess ||
        hipMalloc(&dc, n * 4) != hipSuccess) {
      ++failures;
      continue;
    }
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
    int err = amdgo_vector_add_f32(da, db, dc, n, nullptr);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i) bad += (c[i] != a[i] + b[i]);
    if (err || bad) ++failures;
    hipFree(da);
    hipFree(db);
    hipFree(dc);
  }
  std::printf("{\"event\":\"hip-smoke\",\"devices\":%d,\"elements\":%zu,\"ok\":%s}\n", ndev, n,
              failures ? "false" : "true");
  return failures ? 1 : 0;
}
