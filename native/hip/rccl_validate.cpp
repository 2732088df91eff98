// amd-rccl-validate: prove the xGMI fabric of a node with RCCL all-reduces.
//
// New in this framework: the reference never exercises the GPU interconnect (SURVEY.md §2.7,
// §5.8, §7.5.3). Three parts, one JSON line per event:
//
//  1. Topology (no HIP call, also runs without a GPU): every GPU agent KFD exposes, its xGMI hive
//     and the xGMI io_links of its KFD node (libamdnode). The fabric check requires one hive id
//     across the visible GPUs and, on a full 8-GPU MI355X node, 7 xGMI links per GPU (a fully
//     connected mesh). A split hive or a missing link fails the run before any collective.
//  2. A rank sweep (--ranks 2,4,8): for every rank count N one process drives GPUs 0..N-1
//     (ncclCommInitAll), sum-reduces fp32 or bf16 buffers over a message-size sweep and reports
//     algorithm and bus bandwidth (busBW = algBW * 2(N-1)/N) against the per-link (~153 GB/s)
//     and N-1-link bounds. Every result is checked exactly (rank r contributes r+1, the sum is
//     N(N+1)/2). A rank count above the visible GPUs is reported as skipped, not failed.
//  3. Multi-process mode (--mp-rank R --mp-nranks N --mp-id-file F): one process per GPU, the
//     deployment shape of a training job; rank 0 publishes the ncclUniqueId through F (atomic
//     rename), every rank joins with ncclCommInitRank. The launcher (amd-validator-workload
//     rccl --processes N) starts the ranks from a parent that never touches the GPU.
//
// `ok` also requires the peak bus bandwidth of the largest rank count to reach --min-busbw
// (the validator passes spec.validator.rccl.env RCCL_MIN_BUSBW_GBPS).
//
// Hang guard (--timeout-s T): a watchdog thread bounds every blocking step -- communicator init, each
// message size's all-reduces, each result check -- by T seconds and polls ncclCommGetAsyncError on the
// live communicators every 100 ms. A faulted or missing peer otherwise blocks inside
// ncclCommInitAll / ncclAllReduce until the pod's timeout and the failure reads "timed out". On a
// deadline or an async error it prints one structured line
//   {"event":"timeout"|"async_error","phase":"init|allreduce|check","ranks":N,"rank":R,"bytes":B,...}
// aborts the communicators (ncclCommAbort, bounded) and exits 124 (timeout) / 125 (async error).
//
//   amd-rccl-validate [--ranks 2,4,8] [--min-bytes 8] [--max-bytes 1073741824] [--iters 20]
//                     [--warmup 5] [--dtype float|bf16] [--min-busbw GBPS] [--topology-only]
//                     [--timeout-s T] [--sys-root /]
//                     [--mp-rank R --mp-nranks N --mp-id-file F [--device D]]
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "amdnode.h"

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

namespace {

constexpr double kLinkGBps = 153.0;   // MI355X xGMI, per link per direction
constexpr int kXgmiPeersFullNode = 7;

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

// --- hang guard ------------------------------------------------------------------------------
class Watchdog {
 public:
  enum Phase { kIdle = 0, kInit, kAllreduce, kCheck };

  void start(double timeout_s, int rank) {
    timeout_s_ = timeout_s;
    rank_ = rank;
    th_ = std::thread([this] { loop(); });
  }
  ~Watchdog() {
    stop_ = true;
    if (th_.joinable()) th_.join();
  }
  // (Re)start the clock of one blocking step.
  void arm(Phase p, int ranks, size_t bytes) {
    ranks_ = ranks;
    bytes_ = (long long)bytes;
    phase_ = p;
    deadline_ns_ = timeout_s_ > 0 ? now_ns() + (long long)(timeout_s_ * 1e9) : 0;
  }
  void disarm() {
    deadline_ns_ = 0;
    phase_ = kIdle;
  }
  void watch(const std::vector<ncclComm_t>& comms) {
    std::lock_guard<std::mutex> lk(mu_);
    comms_ = comms;
  }
  void unwatch() {
    std::lock_guard<std::mutex> lk(mu_);
    comms_.clear();
  }

 private:
  static long long now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
  }
  static const char* phase_name(int p) {
    return p == kInit ? "init" : p == kAllreduce ? "allreduce" : p == kCheck ? "check" : "idle";
  }
  void loop() {
    while (!stop_) {
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
      std::string async;
      {
        std::lock_guard<std::mutex> lk(mu_);
        for (ncclComm_t c : comms_) {
          ncclResult_t ae = ncclSuccess;
          if (ncclCommGetAsyncError(c, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
            async = ncclGetErrorString(ae);
            break;
          }
        }
      }
      if (!async.empty()) fail("async_error", async, 125);
      const long long d = deadline_ns_;
      if (d && now_ns() > d) fail("timeout", "", 124);
    }
  }
  [[noreturn]] void fail(const char* event, const std::string& what, int code) {
    for (char& ch : const_cast<std::string&>(what))
      if (ch == '"' || ch == '\\') ch = '\'';
    std::printf("{\"event\":\"%s\",\"phase\":\"%s\",\"ranks\":%d,\"rank\":%d,\"bytes\":%lld,\"timeout_s\":%.1f%s%s%s,"
                "\"ok\":false}\n",
                event, phase_name(phase_), (int)ranks_, rank_, (long long)bytes_, timeout_s_,
                what.empty() ? "" : ",\"error\":\"", what.c_str(), what.empty() ? "" : "\"");
    std::fflush(stdout);
    // abort the communicators so peers blocked on this rank see the failure; bounded, since an abort
    // can itself wait on a wedged peer
    std::vector<ncclComm_t> comms;
    {
      std::lock_guard<std::mutex> lk(mu_);
      comms = comms_;
    }
    std::atomic<bool> done{false};
    std::thread([comms, &done] {
      for (ncclComm_t c : comms) ncclCommAbort(c);
      done = true;
    }).detach();
    for (int i = 0; i < 100 && !done; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(100));
    _exit(code);
  }

  double timeout_s_ = 0;
  int rank_ = 0;
  std::atomic<bool> stop_{false};
  std::atomic<int> phase_{kIdle}, ranks_{0};
  std::atomic<long long> bytes_{0}, deadline_ns_{0};
  std::mutex mu_;
  std::vector<ncclComm_t> comms_;
  std::thread th_;
};

Watchdog g_watchdog;

struct Opts {
  std::vector<int> ranks;          // empty = all visible GPUs
  int iters = 20, warmup = 5;
  double timeout_s = 0;
  size_t min_bytes = 8, max_bytes = (size_t)1 << 30;
  std::string dtype = "float";
  double min_busbw = 0;
  bool topology_only = false;
  std::string sys_root = "/";
  int mp_rank = -1, mp_nranks = 0, device = -1;
  std::string id_file;
};

std::vector<int> parse_list(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ','))
    if (!tok.empty()) out.push_back(std::atoi(tok.c_str()));
  return out;
}

// --- 1. topology ----------------------------------------------------------------------------
bool fabric_check(const std::string& root) {
  const auto gpus = amdnode::enumerate_gpus(root);
  std::set<std::string> phys;
  std::set<uint64_t> hives;
  std::ostringstream js;
  js << "{\"event\":\"topology\",\"gpus\":[";
  for (size_t i = 0; i < gpus.size(); ++i) {
    const auto& g = gpus[i];
    phys.insert(g.pci_bdf);
    hives.insert(g.xgmi_hive_id);
    js << (i ? "," : "") << "{\"index\":" << g.index << ",\"bdf\":\"" << g.pci_bdf << "\",\"kfd_node\":" << g.kfd_node
       << ",\"hive\":\"" << std::hex << g.xgmi_hive_id << std::dec << "\",\"xgmi_links\":" << g.xgmi_links
       << ",\"xgmi_peers\":[";
    bool first = true;
    for (const auto& l : g.links) {
      if (l.type != 11) continue;
      js << (first ? "" : ",") << l.node_to;
      first = false;
    }
    js << "],\"compute_partition\":\"" << g.compute_partition << "\"}";
  }
  js << "]}";
  std::printf("%s\n", js.str().c_str());
  // A full node is one where every GPU's io_links reach 7 xGMI peers, or where 8 physical GPUs are
  // visible; there the mesh must be complete. With fewer GPUs only hive consistency is checkable.
  const int n = (int)phys.size();
  int max_links = 0, min_links = 1 << 30;
  for (const auto& g : gpus) {
    max_links = std::max(max_links, g.xgmi_links);
    min_links = std::min(min_links, g.xgmi_links);
  }
  const bool single_hive = n >= 1 && hives.size() == 1 && !hives.count(0);
  const bool full_node = n == 8 || max_links >= kXgmiPeersFullNode;
  std::string why;
  bool ok = true;
  if (n == 0) {
    ok = false;
    why = "no GPU agent visible";
  } else if (n >= 2 && !single_hive) {
    ok = false;
    why = "GPUs span " + std::to_string(hives.size()) + " xGMI hives";
  } else if (full_node && min_links < kXgmiPeersFullNode) {
    ok = false;
    why = "a GPU has " + std::to_string(min_links) + " xGMI links, a full MI355X node needs 7";
  }
  std::printf("{\"event\":\"fabric\",\"physical_gpus\":%d,\"single_hive\":%s,\"full_node\":%s,"
              "\"min_xgmi_links\":%d,\"ok\":%s%s%s%s}\n",
              n, single_hive ? "true" : "false", full_node ? "true" : "false", n ? min_links : 0,
              ok ? "true" : "false", why.empty() ? "" : ",\"reason\":\"", why.c_str(), why.empty() ? "" : "\"");
  std::fflush(stdout);
  return ok;
}

// --- 2. one rank count in one process ---------------------------------------------------------
struct SweepResult {
  bool ok = true;
  double peak_busbw = 0;
};

int sweep(const Opts& o, const std::vector<ncclComm_t>& comms, const std::vector<int>& devs, int rank_base,
          int world, SweepResult& res) {
  const int local = (int)comms.size();
  const bool bf16 = o.dtype == "bf16";
  const size_t esz = bf16 ? 2 : 4;
  const ncclDataType_t dt = bf16 ? ncclBfloat16 : ncclFloat;
  std::vector<void*> buf(local);
  std::vector<hipStream_t> st(local);
  std::vector<hipEvent_t> e0(local), e1(local);
  std::vector<unsigned long long*> bad(local);
  for (int r = 0; r < local; ++r) {
    HIPCHECK(hipSetDevice(devs[r]));
    HIPCHECK(hipMalloc(&buf[r], o.max_bytes));
    HIPCHECK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
    HIPCHECK(hipEventCreate(&e0[r]));
    HIPCHECK(hipEventCreate(&e1[r]));
    HIPCHECK(hipMalloc(&bad[r], sizeof(unsigned long long)));
  }
  const double bus_factor = world > 1 ? 2.0 * (world - 1) / world : 1.0;
  const float expect = world * (world + 1) / 2.0f;
  for (size_t bytes = std::max(o.min_bytes, esz); bytes <= o.max_bytes; bytes *= 2) {
    const size_t count = bytes / esz;
    auto allreduce = [&]() -> int {
      NCCLCHECK(ncclGroupStart());
      for (int r = 0; r < local; ++r) NCCLCHECK(ncclAllReduce(buf[r], buf[r], count, dt, ncclSum, comms[r], st[r]));
      NCCLCHECK(ncclGroupEnd());
      return 0;
    };
    g_watchdog.arm(Watchdog::kAllreduce, world, bytes);
    for (int w = 0; w < o.warmup; ++w)
      if (allreduce()) return 2;
    for (int r = 0; r < local; ++r) {
      HIPCHECK(hipSetDevice(devs[r]));
      HIPCHECK(hipStreamSynchronize(st[r]));
      HIPCHECK(hipEventRecord(e0[r], st[r]));
    }
    for (int it = 0; it < o.iters; ++it)
      if (allreduce()) return 2;
    double worst_ms = 0;
    for (int r = 0; r < local; ++r) {
      HIPCHECK(hipSetDevice(devs[r]));
      HIPCHECK(hipEventRecord(e1[r], st[r]));
      HIPCHECK(hipEventSynchronize(e1[r]));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0[r], e1[r]));
      worst_ms = std::max(worst_ms, (double)ms);
    }
    const double t = worst_ms / o.iters * 1e-3;
    const double algbw = bytes / t / 1e9, busbw = algbw * bus_factor;
    // correctness: one fresh reduction of rank+1
    g_watchdog.arm(Watchdog::kCheck, world, bytes);
    for (int r = 0; r < local; ++r) {
      HIPCHECK(hipSetDevice(devs[r]));
      const float v = (float)(rank_base + r + 1);
      if (bf16) fill_bf16_kernel<<<256, 256, 0, st[r]>>>((__bf16*)buf[r], count, v);
      else fill_kernel<<<256, 256, 0, st[r]>>>((float*)buf[r], count, v);
      HIPCHECK(hipMemsetAsync(bad[r], 0, sizeof(unsigned long long), st[r]));
    }
    if (allreduce()) return 2;
    unsigned long long nbad = 0;
    for (int r = 0; r < local; ++r) {
      HIPCHECK(hipSetDevice(devs[r]));
      if (bf16) check_bf16_kernel<<<256, 256, 0, st[r]>>>((const __bf16*)buf[r], count, expect, bad[r]);
      else check_kernel<<<256, 256, 0, st[r]>>>((const float*)buf[r], count, expect, bad[r]);
      unsigned long long h = 0;
      HIPCHECK(hipMemcpyAsync(&h, bad[r], sizeof(h), hipMemcpyDeviceToHost, st[r]));
      HIPCHECK(hipStreamSynchronize(st[r]));
      nbad += h;
    }
    const bool ok = nbad == 0;
    res.ok = res.ok && ok;
    res.peak_busbw = std::max(res.peak_busbw, busbw);
    std::printf("{\"event\":\"allreduce\",\"ranks\":%d,\"rank\":%d,\"bytes\":%zu,\"time_us\":%.2f,"
                "\"algbw_gbps\":%.2f,\"busbw_gbps\":%.2f,\"errors\":%llu,\"ok\":%s}\n",
                world, rank_base, bytes, t * 1e6, algbw, busbw, nbad, ok ? "true" : "false");
    std::fflush(stdout);
  }
  g_watchdog.disarm();
  for (int r = 0; r < local; ++r) {
    hipSetDevice(devs[r]);
    hipFree(buf[r]);
    hipFree(bad[r]);
    hipStreamDestroy(st[r]);
    hipEventDestroy(e0[r]);
    hipEventDestroy(e1[r]);
  }
  return 0;
}

void print_rank_summary(int n, const SweepResult& r, double min_busbw, bool gate) {
  const bool bw_ok = !gate || r.peak_busbw >= min_busbw;
  std::printf("{\"event\":\"ranks_summary\",\"ranks\":%d,\"peak_busbw_gbps\":%.2f,\"link_bound_gbps\":%.1f,"
              "\"mesh_bound_gbps\":%.1f,\"min_busbw_gbps\":%.1f,\"bw_gated\":%s,\"ok\":%s}\n",
              n, r.peak_busbw, kLinkGBps, kLinkGBps * std::max(1, std::min(n - 1, 7)), min_busbw,
              gate ? "true" : "false", (r.ok && bw_ok) ? "true" : "false");
  std::fflush(stdout);
}

// --- 3. one rank of a multi-process run --------------------------------------------------------
int run_mp(const Opts& o) {
  ncclUniqueId id;
  const std::string tmp = o.id_file + ".tmp";
  if (o.mp_rank == 0) {
    NCCLCHECK(ncclGetUniqueId(&id));
    {
      std::ofstream f(tmp, std::ios::binary);
      f.write(reinterpret_cast<const char*>(&id), sizeof(id));
    }
    if (std::rename(tmp.c_str(), o.id_file.c_str()) != 0) {
      std::printf("{\"error\":\"cannot publish the unique id at %s\"}\n", o.id_file.c_str());
      return 2;
    }
  } else {
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(120);
    for (;;) {
      std::ifstream f(o.id_file, std::ios::binary);
      if (f && f.read(reinterpret_cast<char*>(&id), sizeof(id)) && f.gcount() == (std::streamsize)sizeof(id)) break;
      if (std::chrono::steady_clock::now() > deadline) {
        std::printf("{\"error\":\"rank %d: no unique id at %s after 120 s\"}\n", o.mp_rank, o.id_file.c_str());
        return 2;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
  }
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    std::printf("{\"error\":\"no AMD GPU visible\"}\n");
    return 3;
  }
  const int dev = o.device >= 0 ? o.device : o.mp_rank % ndev;
  HIPCHECK(hipSetDevice(dev));
  ncclComm_t comm;
  g_watchdog.start(o.timeout_s, o.mp_rank);
  g_watchdog.arm(Watchdog::kInit, o.mp_nranks, 0);
  NCCLCHECK(ncclCommInitRank(&comm, o.mp_nranks, id, o.mp_rank));
  g_watchdog.disarm();
  g_watchdog.watch({comm});
  int ver = 0;
  ncclGetVersion(&ver);
  std::printf("{\"event\":\"start\",\"mode\":\"multi-process\",\"ranks\":%d,\"rank\":%d,\"device\":%d,"
              "\"rccl_version\":%d,\"dtype\":\"%s\"}\n", o.mp_nranks, o.mp_rank, dev, ver, o.dtype.c_str());
  SweepResult res;
  std::vector<ncclComm_t> comms{comm};
  std::vector<int> devs{dev};
  const int rc = sweep(o, comms, devs, o.mp_rank, o.mp_nranks, res);
  g_watchdog.unwatch();
  ncclCommDestroy(comm);
  if (rc) return rc;
  const bool bw_ok = res.peak_busbw >= o.min_busbw;
  if (o.mp_rank == 0) print_rank_summary(o.mp_nranks, res, o.min_busbw, true);
  std::printf("{\"event\":\"summary\",\"mode\":\"multi-process\",\"rank\":%d,\"ranks\":%d,\"peak_busbw_gbps\":%.2f,"
              "\"ok\":%s}\n", o.mp_rank, o.mp_nranks, res.peak_busbw, (res.ok && bw_ok) ? "true" : "false");
  return (res.ok && bw_ok) ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
  Opts o;
  if (const char* e = std::getenv("AMD_SYSFS_ROOT")) o.sys_root = e;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() { return std::string(i + 1 < argc ? argv[++i] : "0"); };
    if (a == "--ranks") o.ranks = parse_list(next());
    else if (a == "--min-bytes") o.min_bytes = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--max-bytes") o.max_bytes = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--iters") o.iters = std::atoi(next().c_str());
    else if (a == "--warmup") o.warmup = std::atoi(next().c_str());
    else if (a == "--dtype") o.dtype = next();
    else if (a == "--min-busbw") o.min_busbw = std::atof(next().c_str());
    else if (a == "--topology-only") o.topology_only = true;
    else if (a == "--sys-root") o.sys_root = next();
    else if (a == "--mp-rank") o.mp_rank = std::atoi(next().c_str());
    else if (a == "--mp-nranks") o.mp_nranks = std::atoi(next().c_str());
    else if (a == "--mp-id-file") o.id_file = next();
    else if (a == "--device") o.device = std::atoi(next().c_str());
    else if (a == "--timeout-s") o.timeout_s = std::atof(next().c_str());
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-rccl-validate [--ranks 2,4,8] [--min-bytes B] [--max-bytes B] [--iters N] "
                  "[--warmup N] [--dtype float|bf16] [--min-busbw GBPS] [--topology-only] [--timeout-s T] [--sys-root DIR] "
                  "[--mp-rank R --mp-nranks N --mp-id-file F [--device D]]\n");
      return 0;
    } else {
      std::printf("{\"error\":\"unknown argument %s\"}\n", a.c_str());
      return 2;
    }
  }
  if (o.dtype != "float" && o.dtype != "bf16") {
    std::printf("{\"error\":\"unknown --dtype %s\"}\n", o.dtype.c_str());
    return 2;
  }
  if (o.mp_rank >= 0) {
    if (o.mp_nranks < 1 || o.mp_rank >= o.mp_nranks || o.id_file.empty()) {
      std::printf("{\"error\":\"multi-process mode needs --mp-rank < --mp-nranks and --mp-id-file\"}\n");
      return 2;
    }
    return run_mp(o);
  }
  const bool fabric_ok = fabric_check(o.sys_root);
  if (o.topology_only) return fabric_ok ? 0 : 1;
  if (!fabric_ok) {
    std::printf("{\"event\":\"summary\",\"ok\":false,\"reason\":\"fabric check failed\"}\n");
    return 1;
  }
  int ndev = 0;
  HIPCHECK(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    std::printf("{\"error\":\"no AMD GPU visible\"}\n");
    return 3;
  }
  std::vector<int> counts = o.ranks.empty() ? std::vector<int>{ndev} : o.ranks;
  int ver = 0;
  ncclGetVersion(&ver);
  std::printf("{\"event\":\"start\",\"mode\":\"single-process\",\"visible_gpus\":%d,\"rccl_version\":%d,"
              "\"dtype\":\"%s\",\"timeout_s\":%.1f}\n", ndev, ver, o.dtype.c_str(), o.timeout_s);
  g_watchdog.start(o.timeout_s, 0);
  bool all_ok = true;
  int largest = 0;
  double largest_peak = 0;
  std::vector<int> run;
  for (int n : counts) {
    if (n < 1 || n > ndev) {
      std::printf("{\"event\":\"skipped\",\"ranks\":%d,\"reason\":\"%d GPU(s) visible\"}\n", n, ndev);
      continue;
    }
    std::vector<int> devs(n);
    for (int r = 0; r < n; ++r) devs[r] = r;
    std::vector<ncclComm_t> comms(n);
    g_watchdog.arm(Watchdog::kInit, n, 0);
    NCCLCHECK(ncclCommInitAll(comms.data(), n, devs.data()));
    g_watchdog.disarm();
    g_watchdog.watch(comms);
    SweepResult res;
    const int rc = sweep(o, comms, devs, 0, n, res);
    g_watchdog.unwatch();
    for (auto c : comms) ncclCommDestroy(c);
    if (rc) return rc;
    const bool gate = n == *std::max_element(counts.begin(), counts.end()) || o.ranks.empty();
    print_rank_summary(n, res, o.min_busbw, gate);
    all_ok = all_ok && res.ok && (!gate || res.peak_busbw >= o.min_busbw);
    run.push_back(n);
    if (n >= largest) {
      largest = n;
      largest_peak = res.peak_busbw;
    }
  }
  // Nothing multi-GPU to prove (e.g. a 1-GPU node asked for 2,4,8): a clean skip, not a failure.
  const bool skipped = largest < 2;
  std::ostringstream rs;
  for (size_t i = 0; i < run.size(); ++i) rs << (i ? "," : "") << run[i];
  std::printf("{\"event\":\"summary\",\"mode\":\"single-process\",\"ranks\":%d,\"ranks_run\":[%s],"
              "\"peak_busbw_gbps\":%.2f,\"link_bound_gbps\":%.1f,\"mesh_bound_gbps\":%.1f,\"skipped\":%s,\"ok\":%s}\n",
              largest, rs.str().c_str(), largest_peak, kLinkGBps, kLinkGBps * std::max(1, std::min(largest - 1, 7)),
              skipped ? "true" : "false", all_ok ? "true" : "false");
  return all_ok ? 0 : 1;
}
