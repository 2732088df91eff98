// amd-rccl-validate: prove the xGMI fabric of a node with RCCL all-reduces.
//
// New in this framework: the reference never exercises the GPU interconnect (SURVEY.md
// §2.7). One process drives every visible GPU (ncclCommInitAll), sum-reduces fp32 or bf16
// buffers over a message-size sweep and reports algorithm and bus bandwidth
// (busBW = algBW * 2(n-1)/n) against the per-link (~153 GB/s) and 7-link mesh bounds of an
// MI355X. Every result buffer is checked exactly (rank r contributes r+1, so the sum is
// n(n+1)/2). With --sizes the sweep is explicit; otherwise 8 B ... --max-bytes in x2 steps.
//
//   amd-rccl-validate [--ranks N] [--min-bytes 8] [--max-bytes 1073741824] [--iters 20]
//                     [--warmup 5] [--dtype float|bf16] [--min-busbw GBPS]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define HIPCHECK(x)                                                                        \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("{\"error\":\"%s: %s\"}\n", #x, hipGetErrorString(e_));                  \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)
#define NCCLCHECK(x)                                                                       \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) {                                                               \
      std::printf("{\"error\":\"%s: %s\"}\n", #x, ncclGetErrorString(r_));                 \
      return 2;                                                                            \
    }                                                                                      \
  } while (0)

__global__ void fill_kernel(float* p, size_t n, float v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = v;
}
__global__ void fill_bf16_kernel(__bf16* p, size_t n, float v) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = (__bf16)v;
}
// counts elements != expect (exact compare)
__global__ void check_kernel(const float* p, size_t n, float expect, unsigned long long* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) c += (p[i] != expect);
  if (c) atomicAdd(bad, c);
}
__global__ void check_bf16_kernel(const __bf16* p, size_t n, float expect, unsigned long long* bad) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long c = 0;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) c += ((float)p[i] != expect);
  if (c) atomicAdd(bad, c);
}

int main(int argc, char** argv) {
  int ranks = 0, iters = 20, warmup = 5;
  size_t min_bytes = 8, max_bytes = (size_t)1 << 30;
  std::string dtype = "float";
  double min_busbw = 0;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : "0"); };
    if (a == "--ranks") ranks = std::atoi(next().c_str());
    else if (a == "--min-bytes") min_bytes = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--max-bytes") max_bytes = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--iters") iters = std::atoi(next().c_str());
    else if (a == "--warmup") warmup = std::atoi(next().c_str());
    else if (a == "--dtype") dtype = next();
    else if (a == "--min-busbw") min_busbw = std::atof(next().c_str());
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-rccl-validate [--ranks N] [--min-bytes B] [--max-bytes B] [--iters N] "
                  "[--warmup N] [--dtype float|bf16] [--min-busbw GBPS]\n");
      return 0;
    }
  }
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (ranks <= 0 || ranks > ndev) ranks = ndev;
  if (ranks < 1) {
    std::printf("{\"error\":\"no AMD GPU visible\"}\n");
    return 3;
  }
  const bool bf16 = dtype == "bf16";
  const size_t esz = bf16 ? 2 : 4;
  std::vector<int> devs(ranks);
  for (int r = 0; r < ranks; ++r) devs[r] = r;
  std::vector<ncclComm_t> comms(ranks);
  NCCLCHECK(ncclCommInitAll(comms.data(), ranks, devs.data()));
  int ver = 0;
  ncclGetVersion(&ver);
  std::printf("{\"event\":\"start\",\"ranks\":%d,\"rccl_version\":%d,\"dtype\":\"%s\"}\n", ranks, ver,
              dtype.c_str());
  std::vector<void*> buf(ranks);
  std::vector<hipStream_t> st(ranks);
  std::vector<hipEvent_t> e0(ranks), e1(ranks);
  std::vector<unsigned long long*> bad(ranks);
  for (int r = 0; r < ranks; ++r) {
    HIPCHECK(hipSetDevice(r));
    HIPCHECK(hipMalloc(&buf[r], max_bytes));
    HIPCHECK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
    HIPCHECK(hipEventCreate(&e0[r]));
    HIPCHECK(hipEventCreate(&e1[r]));
    HIPCHECK(hipMalloc(&bad[r], sizeof(unsigned long long)));
  }
  const double bus_factor = ranks > 1 ? 2.0 * (ranks - 1) / ranks : 1.0;
  const float expect = ranks * (ranks + 1) / 2.0f;
  bool all_ok = true;
  double peak_busbw = 0;
  for (size_t bytes = std::max(min_bytes, esz); bytes <= max_bytes; bytes *= 2) {
    const size_t count = bytes / esz;
    const ncclDataType_t dt = bf16 ? ncclBfloat16 : ncclFloat;
    auto allreduce = [&]() -> int {
      NCCLCHECK(ncclGroupStart());
      for (int r = 0; r < ranks; ++r) NCCLCHECK(ncclAllReduce(buf[r], buf[r], count, dt, ncclSum, comms[r], st[r]));
      NCCLCHECK(ncclGroupEnd());
      return 0;
    };
    for (int w = 0; w < warmup; ++w)
      if (allreduce()) return 2;
    for (int r = 0; r < ranks; ++r) {
      HIPCHECK(hipSetDevice(r));
      HIPCHECK(hipStreamSynchronize(st[r]));
      HIPCHECK(hipEventRecord(e0[r], st[r]));
    }
    for (int it = 0; it < iters; ++it)
      if (allreduce()) return 2;
    double worst_ms = 0;
    for (int r = 0; r < ranks; ++r) {
      HIPCHECK(hipSetDevice(r));
      HIPCHECK(hipEventRecord(e1[r], st[r]));
      HIPCHECK(hipEventSynchronize(e1[r]));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0[r], e1[r]));
      worst_ms = std::max(worst_ms, (double)ms);
    }
    const double t = worst_ms / iters * 1e-3;
    const double algbw = bytes / t / 1e9, busbw = algbw * bus_factor;
    // correctness: one fresh reduction of rank+1
    for (int r = 0; r < ranks; ++r) {
      HIPCHECK(hipSetDevice(r));
      if (bf16) fill_bf16_kernel<<<256, 256, 0, st[r]>>>((__bf16*)buf[r], count, (float)(r + 1));
      else fill_kernel<<<256, 256, 0, st[r]>>>((float*)buf[r], count, (float)(r + 1));
      HIPCHECK(hipMemsetAsync(bad[r], 0, sizeof(unsigned long long), st[r]));
    }
    if (allreduce()) return 2;
    unsigned long long nbad = 0;
    for (int r = 0; r < ranks; ++r) {
      HIPCHECK(hipSetDevice(r));
      if (bf16) check_bf16_kernel<<<256, 256, 0, st[r]>>>((const __bf16*)buf[r], count, expect, bad[r]);
      else check_kernel<<<256, 256, 0, st[r]>>>((const float*)buf[r], count, expect, bad[r]);
      unsigned long long h = 0;
      HIPCHECK(hipMemcpyAsync(&h, bad[r], sizeof(h), hipMemcpyDeviceToHost, st[r]));
      HIPCHECK(hipStreamSynchronize(st[r]));
      nbad += h;
    }
    const bool ok = nbad == 0;
    all_ok = all_ok && ok;
    peak_busbw = std::max(peak_busbw, busbw);
    std::printf("{\"event\":\"allreduce\",\"ranks\":%d,\"bytes\":%zu,\"time_us\":%.2f,\"algbw_gbps\":%.2f,"
                "\"busbw_gbps\":%.2f,\"errors\":%llu,\"ok\":%s}\n",
                ranks, bytes, t * 1e6, algbw, busbw, nbad, ok ? "true" : "false");
    std::fflush(stdout);
  }
  const bool bw_ok = peak_busbw >= min_busbw;
  std::printf("{\"event\":\"summary\",\"ranks\":%d,\"peak_busbw_gbps\":%.2f,\"link_bound_gbps\":153.0,"
              "\"mesh_bound_gbps\":%.1f,\"ok\":%s}\n",
              ranks, peak_busbw, 153.0 * std::max(1, std::min(ranks - 1, 7)),
              (all_ok && bw_ok) ? "true" : "false");
  for (int r = 0; r < ranks; ++r) {
    hipSetDevice(r);
    hipFree(buf[r]);
    hipFree(bad[r]);
    ncclCommDestroy(comms[r]);
  }
  return (all_ok && bw_ok) ? 0 : 1;
}
