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
//  4. The link matrix (before the rank sweep, 2+ GPUs): every ordered GPU pair (src -> dst) with
//     peer access enabled, timed with a pull kernel on dst that reads src's HBM over xGMI (16 B per
//     lane, wide enough to fill a link), first one pair at a time ("isolated"), then all N(N-1)
//     pairs at once ("concurrent": ONE kernel per destination GPU pulls from every peer, its blocks
//     split among the sources, a rate per source from its blocks' wall-clock stamps -- one stream per
//     GPU, within the 4 hardware queues a process gets; --link-plan N prints the launch plan). Every copy is
//     checked (a link that corrupts data fails). A pair below --min-link-relative (0.8) x the node
//     median of its mode fails and is NAMED (`slow_links`: "3->5"): an all-reduce over 8 ranks can
//     hide one degraded link, this cannot. One compact `xgmi_matrix` line carries both 8x8 matrices
//     (GB/s) and the per-GPU measured aggregate (the mesh bound the validator's busBW gate uses).
//     1 GPU: a clean skip. --link-self-test times GPU 0 -> GPU 0 (the kernels on a 1-GPU box);
//     --virtual-peers V pulls V buffers of GPU 0 with one kernel (the concurrent phase's shape on one
//     GPU), and --throttle-peer P gives source P an eighth of the blocks: the proof that the naming
//     names the slow source and only it.
//
// `ok` also requires the peak bus bandwidth of the largest rank count to reach --min-busbw (an explicit
// spec.validator.rccl.env RCCL_MIN_BUSBW_GBPS) or, without one, --min-busbw-mesh-fraction x the
// measured mesh bound (the smallest per-GPU ingress of the concurrent link matrix).
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
//                     [--timeout-s T] [--sys-root /] [--link-bytes B] [--link-iters N]
//                     [--min-link-relative R] [--no-links] [--links-only] [--link-self-test]
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
#include <iomanip>
#include <map>
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

// The link probe: dst[i] = src[i] where src is a peer GPU's buffer (read over xGMI) -- launched on
// the destination GPU, so the bytes cross the src -> dst direction of the link.
__global__ void __launch_bounds__(256) peer_read_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                        size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}
// src pattern of GPU g: word i = (g + 1) * 0x9E3779B1 ^ i
__global__ void pattern_kernel(uint32_t* p, size_t n, uint32_t g) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (g + 1u) * 0x9E3779B1u ^ (uint32_t)i;
}
__global__ void pattern_check_kernel(const uint32_t* p, size_t n, uint32_t g, unsigned long long* bad) {
  unsigned long long c = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    c += p[i] != ((g + 1u) * 0x9E3779B1u ^ (uint32_t)i);
  if (c) atomicAdd(bad, c);
}

// --- hang guard ------------------------------------------------------------------------------
class Watchdog {
 public:
  enum Phase { kIdle = 0, kInit, kAllreduce, kCheck, kLinks };

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
    return p == kInit ? "init" : p == kAllreduce ? "allreduce" : p == kCheck ? "check" : p == kLinks ? "links" : "idle";
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
  size_t link_bytes = (size_t)256 << 20;
  int link_iters = 5;
  double min_link_relative = 0.8;
  double mesh_fraction = 0;        // busBW floor as a fraction of the measured mesh bound (no --min-busbw)
  bool links = true, links_only = false, link_self_test = false;
  int virtual_peers = 0;           // 1-GPU self-test: this many source buffers on GPU 0, pulled by one kernel
  int throttle_peer = -1;          // the source given 1/throttle_factor of the pull blocks (the naming test)
  int throttle_factor = 8;
  int link_plan = 0;               // print the plan for this many GPUs and exit (no GPU call)
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

// --- 4. the link matrix -------------------------------------------------------------------------
// One pull kernel per destination GPU: its blocks are split among the sources it reads (block table
// first_block[s] .. first_block[s+1]), each block copies its share of its source's buffer over the link
// and stamps the 100 MHz wall clock around its work; a source's rate is its bytes over the span of its
// blocks' stamps. So the concurrent phase -- every destination pulling from every peer at once -- needs
// one stream per GPU, not one per ordered pair: with GPU_MAX_HW_QUEUES=4, 7 streams per GPU shared 3
// hardware queues two by two, each pair's event window held its queue partner's copies, and a slow link
// slowed (and could get named instead of) its partner. The isolated phase runs the
// same kernel with one source.
struct LinkResult {
  bool ok = true, skipped = false;
  double min_aggregate = 0;   // smallest per-GPU concurrent ingress (GB/s): the measured mesh bound
};

constexpr int kMaxPullSources = 16;
constexpr int kPullThreads = 256;

struct PullArgs {
  const uint4* src[kMaxPullSources];
  uint4* dst[kMaxPullSources];
  int blocks[kMaxPullSources];      // blocks per source
};

// Block -> (source, index among that source's blocks): `table` (device memory, one int2 per block)
// deals each source's blocks evenly over the grid. Contiguous ranges ran source 0's blocks as the
// oldest waves of every CU: the sequencer's age priority let them finish first, and 7 equal sources
// measured 462 down to 361 GB/s in block order (one MI355X, --virtual-peers 7).
__global__ void __launch_bounds__(kPullThreads)
multi_pull_kernel(PullArgs a, const int2* __restrict__ table, size_t vecs, int iters,
                  unsigned long long* __restrict__ stamps) {
  const int2 t = table[blockIdx.x];
  const int s = t.x, b = t.y, nb = a.blocks[s];
  const uint4* __restrict__ src = a.src[s];
  uint4* __restrict__ dst = a.dst[s];
  __syncthreads();
  const unsigned long long t0 = (unsigned long long)wall_clock64();
  for (int it = 0; it < iters; ++it)
    for (size_t i = (size_t)b * kPullThreads + threadIdx.x; i < vecs; i += (size_t)nb * kPullThreads) dst[i] = src[i];
  __syncthreads();
  const unsigned long long t1 = (unsigned long long)wall_clock64();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = t1;
  }
}

// What the link matrix will launch, computed without touching the GPU (--link-plan prints it; the
// run executes exactly this). A source is a buffer on a GPU: GPU s itself on a multi-GPU node, or one of
// --virtual-peers buffers on GPU 0 in the 1-GPU self-test ("v3"). `blocks[p]`: the pull blocks of pair p
// (source si -> destination di) -- --throttle-peer gives one source 1/--throttle-factor (8) of them.
struct LinkPlan {
  struct Src {
    int dev;
    std::string name;
    uint32_t pattern;
  };
  std::vector<Src> srcs;
  std::vector<int> dsts;                                // destination devices
  std::vector<std::pair<int, int>> pairs;               // (source index, destination index)
  std::vector<int> iso_blocks, conc_blocks;             // per pair
  std::vector<int> devices;                             // every device involved: one stream each
};

LinkPlan plan_links(const Opts& o, const std::vector<int>& devs) {
  LinkPlan pl;
  const bool virt = o.virtual_peers > 0;
  if (virt) {
    for (int v = 0; v < o.virtual_peers; ++v) pl.srcs.push_back({devs[0], "v" + std::to_string(v), (uint32_t)(100 + v)});
    pl.dsts = {devs[0]};
  } else {
    for (int d : devs) pl.srcs.push_back({d, std::to_string(d), (uint32_t)d});
    pl.dsts = devs;
  }
  for (int di = 0; di < (int)pl.dsts.size(); ++di)
    for (int si = 0; si < (int)pl.srcs.size(); ++si)
      if (virt || pl.srcs[si].dev != pl.dsts[di] || o.link_self_test) pl.pairs.push_back({si, di});
  std::set<int> dv;
  for (const auto& s : pl.srcs) dv.insert(s.dev);
  for (int d : pl.dsts) dv.insert(d);
  pl.devices.assign(dv.begin(), dv.end());
  std::vector<int> per_dst(pl.dsts.size(), 0);
  for (auto [si, di] : pl.pairs) ++per_dst[di];
  for (auto [si, di] : pl.pairs) {
    const bool slow = o.throttle_peer >= 0 && si == o.throttle_peer;
    const int f = slow ? std::max(1, o.throttle_factor) : 1;
    pl.iso_blocks.push_back(std::max(8, 2048 / f));
    // concurrent: ~2048 blocks per destination kernel (8 per CU), split evenly over its sources
    pl.conc_blocks.push_back(std::max(8, std::max(128, 2048 / std::max(1, per_dst[di])) / f));
  }
  return pl;
}

// The block table of one pull kernel: each block goes to the source furthest behind its share
// (assigned / wanted), so every source's blocks are spread evenly over the grid's dispatch order.
std::vector<std::pair<int, int>> deal_blocks(const std::vector<int>& want) {
  int total = 0;
  for (int w : want) total += w;
  std::vector<int> got(want.size(), 0);
  std::vector<std::pair<int, int>> out;
  out.reserve(total);
  for (int b = 0; b < total; ++b) {
    int best = -1;
    double key = 1e30;
    for (size_t s = 0; s < want.size(); ++s) {
      if (got[s] >= want[s]) continue;
      const double k = (got[s] + 0.5) / want[s];
      if (k < key) key = k, best = (int)s;
    }
    out.push_back({best, got[best]++});
  }
  return out;
}

void print_plan(const LinkPlan& pl) {
  std::ostringstream k;
  for (int di = 0; di < (int)pl.dsts.size(); ++di) {
    int nsrc = 0, blocks = 0;
    std::string b;
    for (size_t p = 0; p < pl.pairs.size(); ++p)
      if (pl.pairs[p].second == di) {
        ++nsrc;
        blocks += pl.conc_blocks[p];
        b += (b.empty() ? "" : ",") + std::to_string(pl.conc_blocks[p]);
      }
    k << (di ? "," : "") << "{\"dst\":" << pl.dsts[di] << ",\"sources\":" << nsrc << ",\"blocks\":" << blocks
      << ",\"blocks_per_source\":[" << b << "]}";
  }
  std::printf("{\"event\":\"link_plan\",\"devices\":%zu,\"streams_per_device\":1,\"pairs\":%zu,"
              "\"concurrent_kernels\":[%s]}\n",
              pl.devices.size(), pl.pairs.size(), k.str().c_str());
  std::fflush(stdout);
}

static double median_of(std::vector<double> v) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

// Times every pair of the plan (isolated, then concurrent) and prints the `xgmi_matrix` line.
int link_matrix(const Opts& o, const std::vector<int>& devs, LinkResult& res) {
  const LinkPlan pl = plan_links(o, devs);
  const int ns = (int)pl.srcs.size(), nd = (int)pl.dsts.size();
  const size_t bytes = o.link_bytes & ~(size_t)15, words = bytes / 4, vecs = bytes / 16;
  // peer access for every cross-GPU pair (the pull kernel on dst dereferences src's memory)
  std::vector<std::string> no_peer;
  std::vector<bool> usable(pl.pairs.size(), true);
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    const int sd = pl.srcs[pl.pairs[p].first].dev, dd = pl.dsts[pl.pairs[p].second];
    if (sd == dd) continue;
    int can = 0;
    HIPCHECK(hipDeviceCanAccessPeer(&can, dd, sd));
    if (!can) {
      no_peer.push_back(pl.srcs[pl.pairs[p].first].name + "->" + std::to_string(dd));
      usable[p] = false;
      continue;
    }
    HIPCHECK(hipSetDevice(dd));
    const hipError_t e = hipDeviceEnablePeerAccess(sd, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHECK(e);
    (void)hipGetLastError();
  }
  // one stream per device; a patterned buffer per source; a destination buffer per pair
  std::map<int, hipStream_t> st;
  std::map<int, unsigned long long*> bad;
  std::map<int, double> tick_hz;
  for (int d : pl.devices) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamCreateWithFlags(&st[d], hipStreamNonBlocking));
    HIPCHECK(hipMalloc(&bad[d], sizeof(unsigned long long)));
    int khz = 0;
    HIPCHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d));
    tick_hz[d] = khz > 0 ? khz * 1e3 : 1e8;
  }
  std::vector<void*> src(ns, nullptr), dst(pl.pairs.size(), nullptr);
  for (int si = 0; si < ns; ++si) {
    HIPCHECK(hipSetDevice(pl.srcs[si].dev));
    HIPCHECK(hipMalloc(&src[si], bytes));
    pattern_kernel<<<1024, 256, 0, st[pl.srcs[si].dev]>>>((uint32_t*)src[si], words, pl.srcs[si].pattern);
    HIPCHECK(hipGetLastError());
  }
  int max_grid = 0;
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    HIPCHECK(hipSetDevice(pl.dsts[pl.pairs[p].second]));
    HIPCHECK(hipMalloc(&dst[p], bytes));
    max_grid = std::max(max_grid, pl.iso_blocks[p]);
  }
  std::vector<int> grid_of(nd, 0);
  for (size_t p = 0; p < pl.pairs.size(); ++p) grid_of[pl.pairs[p].second] += usable[p] ? pl.conc_blocks[p] : 0;
  for (int g : grid_of) max_grid = std::max(max_grid, g);
  std::map<int, unsigned long long*> stamps;
  for (int d : pl.dsts) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMalloc(&stamps[d], (size_t)max_grid * 2 * sizeof(unsigned long long)));
  }
  for (int d : pl.devices) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamSynchronize(st[d]));
  }
  // one launch of destination di's kernel over `which` pairs with their block counts; `deal` gets the
  // block table (block -> source slot, index) for the rates
  // the block table of a launch, uploaded before anything is timed: the isolated launches of a
  // destination share the single-source table (block b -> source 0, index b), the concurrent launch
  // has its own
  std::vector<int2*> iso_table(nd, nullptr), conc_table(nd, nullptr);
  auto upload = [&](int di, const std::vector<std::pair<int, int>>& deal, int2** out) -> int {
    std::vector<int2> ht(deal.size());
    for (size_t b = 0; b < deal.size(); ++b) ht[b] = make_int2(deal[b].first, deal[b].second);
    HIPCHECK(hipSetDevice(pl.dsts[di]));
    HIPCHECK(hipMalloc(out, std::max<size_t>(1, ht.size()) * sizeof(int2)));
    HIPCHECK(hipMemcpy(*out, ht.data(), ht.size() * sizeof(int2), hipMemcpyHostToDevice));
    return 0;
  };
  // one launch of destination di's kernel over `which` pairs with their block counts and block table
  auto launch = [&](int di, const std::vector<size_t>& which, const std::vector<int>& blocks, int iters,
                    const int2* table, int grid) -> int {
    PullArgs a{};
    int k = 0;
    for (size_t p : which) {
      a.src[k] = (const uint4*)src[pl.pairs[p].first];
      a.dst[k] = (uint4*)dst[p];
      a.blocks[k] = blocks[p];
      ++k;
    }
    const int d = pl.dsts[di];
    HIPCHECK(hipSetDevice(d));
    multi_pull_kernel<<<grid, kPullThreads, 0, st[d]>>>(a, table, vecs, iters, stamps[d]);
    HIPCHECK(hipGetLastError());
    return 0;
  };
  // per pair: bytes x iters over the span of its blocks' stamps
  auto rates = [&](int di, const std::vector<size_t>& which, const std::vector<std::pair<int, int>>& deal,
                   int iters, std::vector<double>& out) -> int {
    const int d = pl.dsts[di];
    std::vector<unsigned long long> h(deal.size() * 2);
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMemcpyAsync(h.data(), stamps[d], h.size() * 8, hipMemcpyDeviceToHost, st[d]));
    HIPCHECK(hipStreamSynchronize(st[d]));
    std::vector<unsigned long long> lo(which.size(), ~0ull), hi(which.size(), 0);
    for (size_t b = 0; b < deal.size(); ++b) {
      const int q = deal[b].first;
      lo[q] = std::min(lo[q], h[2 * b]);
      hi[q] = std::max(hi[q], h[2 * b + 1]);
    }
    for (size_t q = 0; q < which.size(); ++q) {
      const double s = hi[q] > lo[q] ? (double)(hi[q] - lo[q]) / tick_hz[d] : 0;
      out[which[q]] = s > 0 ? (double)bytes * iters / s / 1e9 : 0;
    }
    return 0;
  };
  std::vector<double> iso(pl.pairs.size(), 0.0), conc(pl.pairs.size(), 0.0);
  std::vector<unsigned long long> errs(pl.pairs.size(), 0);
  g_watchdog.arm(Watchdog::kLinks, nd, bytes);
  std::vector<std::vector<size_t>> by_dst(nd);
  for (size_t p = 0; p < pl.pairs.size(); ++p)
    if (usable[p]) by_dst[pl.pairs[p].second].push_back(p);
  std::vector<std::vector<std::pair<int, int>>> conc_deal(nd);
  for (int di = 0; di < nd; ++di) {
    int most = 0;
    std::vector<int> want;
    for (size_t p : by_dst[di]) most = std::max(most, pl.iso_blocks[p]), want.push_back(pl.conc_blocks[p]);
    if (upload(di, deal_blocks({most}), &iso_table[di])) return 2;
    conc_deal[di] = deal_blocks(want);
    if (upload(di, conc_deal[di], &conc_table[di])) return 2;
  }
  // isolated: one pair at a time (a warm-up pass, then the timed launch of link_iters passes)
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    if (!usable[p]) continue;
    const int di = pl.pairs[p].second;
    std::vector<std::pair<int, int>> deal(pl.iso_blocks[p]);
    for (int b = 0; b < pl.iso_blocks[p]; ++b) deal[b] = {0, b};
    if (launch(di, {p}, pl.iso_blocks, 1, iso_table[di], pl.iso_blocks[p]) ||
        launch(di, {p}, pl.iso_blocks, o.link_iters, iso_table[di], pl.iso_blocks[p]) ||
        rates(di, {p}, deal, o.link_iters, iso))
      return 2;
  }
  // concurrent: every destination's kernel over all its sources, all destinations at once
  for (int di = 0; di < nd; ++di)
    if (!by_dst[di].empty() &&
        launch(di, by_dst[di], pl.conc_blocks, 1, conc_table[di], (int)conc_deal[di].size()))
      return 2;
  for (int d : pl.dsts) {
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipStreamSynchronize(st[d]));
  }
  for (int di = 0; di < nd; ++di)
    if (!by_dst[di].empty() &&
        launch(di, by_dst[di], pl.conc_blocks, o.link_iters, conc_table[di], (int)conc_deal[di].size()))
      return 2;
  for (int di = 0; di < nd; ++di)
    if (!by_dst[di].empty() && rates(di, by_dst[di], conc_deal[di], o.link_iters, conc)) return 2;
  // correctness: every destination buffer holds its source's pattern
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    if (!usable[p]) continue;
    const int d = pl.dsts[pl.pairs[p].second];
    HIPCHECK(hipSetDevice(d));
    HIPCHECK(hipMemsetAsync(bad[d], 0, sizeof(unsigned long long), st[d]));
    pattern_check_kernel<<<1024, 256, 0, st[d]>>>((const uint32_t*)dst[p], words, pl.srcs[pl.pairs[p].first].pattern,
                                                   bad[d]);
    unsigned long long h = 0;
    HIPCHECK(hipMemcpyAsync(&h, bad[d], sizeof h, hipMemcpyDeviceToHost, st[d]));
    HIPCHECK(hipStreamSynchronize(st[d]));
    errs[p] = h;
  }
  g_watchdog.disarm();
  // the relative gate, per mode, against the node median of that mode
  std::vector<double> iv, cv;
  for (size_t p = 0; p < pl.pairs.size(); ++p)
    if (usable[p]) iv.push_back(iso[p]), cv.push_back(conc[p]);
  const double imed = median_of(iv), cmed = median_of(cv);
  std::vector<std::string> slow, corrupt;
  double worst = 1e30;
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    if (!usable[p]) continue;
    const double ri = imed > 0 ? iso[p] / imed : 0, rc = cmed > 0 ? conc[p] / cmed : 0;
    worst = std::min(worst, std::min(ri, rc));
    const std::string name = pl.srcs[pl.pairs[p].first].name + "->" + std::to_string(pl.dsts[pl.pairs[p].second]);
    if (errs[p]) corrupt.push_back(name);
    if (o.min_link_relative > 0 && (ri < o.min_link_relative || rc < o.min_link_relative)) {
      slow.push_back(name);
      const std::string& sn = pl.srcs[pl.pairs[p].first].name;     // a GPU index, or "v3" (virtual peer)
      const std::string sj = o.virtual_peers > 0 ? "\"" + sn + "\"" : sn;
      std::printf("{\"event\":\"xgmi_link\",\"src\":%s,\"dst\":%d,\"isolated_gbps\":%.1f,\"concurrent_gbps\":%.1f,"
                  "\"isolated_ratio\":%.3f,\"concurrent_ratio\":%.3f,\"ok\":false,\"kind\":\"link\"}\n",
                  sj.c_str(), pl.dsts[pl.pairs[p].second], iso[p], conc[p], ri, rc);
    }
  }
  // per-GPU measured ingress with every peer pulling at once: the mesh bound of a collective
  std::vector<double> agg(nd, 0.0);
  for (size_t p = 0; p < pl.pairs.size(); ++p) agg[pl.pairs[p].second] += conc[p];
  res.min_aggregate = nd ? *std::min_element(agg.begin(), agg.end()) : 0;
  res.ok = slow.empty() && corrupt.empty() && no_peer.empty();
  auto matrix = [&](const std::vector<double>& v) {   // rows = sources, columns = destinations
    std::vector<std::vector<double>> m(ns, std::vector<double>(nd, 0.0));
    for (size_t p = 0; p < pl.pairs.size(); ++p) m[pl.pairs[p].first][pl.pairs[p].second] = v[p];
    std::ostringstream js;
    js << "[";
    for (int r = 0; r < ns; ++r) {
      js << (r ? "," : "") << "[";
      for (int c = 0; c < nd; ++c) {
        char b[24];
        std::snprintf(b, sizeof b, "%.1f", m[r][c]);
        js << (c ? "," : "") << b;
      }
      js << "]";
    }
    js << "]";
    return js.str();
  };
  auto list = [](const std::vector<std::string>& v) {
    std::string out;
    for (const auto& x : v) out += (out.empty() ? "\"" : ",\"") + x + "\"";
    return out;
  };
  std::ostringstream ag, names;
  for (int g = 0; g < nd; ++g) ag << (g ? "," : "") << std::fixed << std::setprecision(1) << agg[g];
  for (int si = 0; si < ns; ++si) names << (si ? ",\"" : "\"") << pl.srcs[si].name << "\"";
  std::printf("{\"event\":\"xgmi_matrix\",\"gpus\":%d,\"sources\":[%s],\"bytes\":%zu,\"iters\":%d,"
              "\"isolated_gbps\":%s,\"concurrent_gbps\":%s,\"median_isolated_gbps\":%.1f,\"median_concurrent_gbps\":%.1f,"
              "\"gpu_ingress_gbps\":[%s],\"min_gpu_ingress_gbps\":%.1f,\"min_ratio\":%.3f,\"min_link_relative\":%.2f,"
              "\"slow_links\":[%s],\"corrupt_links\":[%s],\"no_peer_access\":[%s],\"self_test\":%s,"
              "\"virtual_peers\":%d,\"throttle_peer\":%d,\"streams_per_device\":1,"
              "\"concurrent_method\":\"one pull kernel per destination, per-source block stamps\",\"ok\":%s%s}\n",
              nd, names.str().c_str(), bytes, o.link_iters, matrix(iso).c_str(), matrix(conc).c_str(), imed, cmed,
              ag.str().c_str(), res.min_aggregate, pl.pairs.empty() ? 0.0 : worst, o.min_link_relative,
              list(slow).c_str(), list(corrupt).c_str(), list(no_peer).c_str(),
              (o.link_self_test || o.virtual_peers > 0) ? "true" : "false", o.virtual_peers, o.throttle_peer,
              res.ok ? "true" : "false", res.ok ? "" : ",\"kind\":\"link\"");
  std::fflush(stdout);
  for (size_t p = 0; p < pl.pairs.size(); ++p) {
    (void)hipSetDevice(pl.dsts[pl.pairs[p].second]);
    (void)hipFree(dst[p]);
  }
  for (int si = 0; si < ns; ++si) {
    (void)hipSetDevice(pl.srcs[si].dev);
    (void)hipFree(src[si]);
  }
  for (int di = 0; di < nd; ++di) {
    (void)hipSetDevice(pl.dsts[di]);
    if (iso_table[di]) (void)hipFree(iso_table[di]);
    if (conc_table[di]) (void)hipFree(conc_table[di]);
  }
  for (int d : pl.devices) {
    (void)hipSetDevice(d);
    (void)hipFree(bad[d]);
    if (stamps.count(d)) (void)hipFree(stamps[d]);
    (void)hipStreamDestroy(st[d]);
  }
  return 0;
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
    else if (a == "--link-bytes") o.link_bytes = std::strtoull(next().c_str(), nullptr, 10);
    else if (a == "--link-iters") o.link_iters = std::max(1, std::atoi(next().c_str()));
    else if (a == "--min-link-relative") o.min_link_relative = std::atof(next().c_str());
    else if (a == "--min-busbw-mesh-fraction") o.mesh_fraction = std::atof(next().c_str());
    else if (a == "--no-links") o.links = false;
    else if (a == "--links-only") o.links_only = true;
    else if (a == "--link-self-test") o.link_self_test = true;
    else if (a == "--virtual-peers") o.virtual_peers = std::max(0, std::min(kMaxPullSources, std::atoi(next().c_str())));
    else if (a == "--throttle-peer") o.throttle_peer = std::atoi(next().c_str());
    else if (a == "--throttle-factor") o.throttle_factor = std::max(1, std::atoi(next().c_str()));
    else if (a == "--link-plan") o.link_plan = std::max(1, std::atoi(next().c_str()));
    else if (a == "-h" || a == "--help") {
      std::printf("usage: amd-rccl-validate [--ranks 2,4,8] [--min-bytes B] [--max-bytes B] [--iters N] "
                  "[--warmup N] [--dtype float|bf16] [--min-busbw GBPS] [--topology-only] [--timeout-s T] [--sys-root DIR] "
                  "[--mp-rank R --mp-nranks N --mp-id-file F [--device D]] [--link-bytes B] [--link-iters N] "
                  "[--min-link-relative R] [--min-busbw-mesh-fraction F] [--no-links] [--links-only] [--link-self-test] "
                  "[--virtual-peers V] [--throttle-peer P] [--throttle-factor F] [--link-plan N]\n");
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
  if (o.link_plan > 0) {            // what the link matrix launches on N GPUs (no GPU call; CPU tests)
    std::vector<int> devs(o.virtual_peers > 0 ? 1 : o.link_plan);
    for (int d = 0; d < (int)devs.size(); ++d) devs[d] = d;
    print_plan(plan_links(o, devs));
    return 0;
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
  // the link matrix over every visible GPU (one process: peer access between its devices)
  LinkResult links;
  if (o.links || o.links_only) {
    const bool self = o.link_self_test || o.virtual_peers > 0;
    std::vector<int> all(self ? 1 : ndev);
    for (int d = 0; d < (int)all.size(); ++d) all[d] = d;
    if ((int)all.size() >= 2 || self) {
      if (link_matrix(o, all, links)) return 2;
      all_ok = links.ok;
    } else {
      links.skipped = true;
      std::printf("{\"event\":\"xgmi_matrix\",\"gpus\":%d,\"skipped\":\"%d GPU visible: no link to measure\","
                  "\"ok\":true}\n", ndev, ndev);
    }
    if (o.links_only) {
      std::printf("{\"event\":\"summary\",\"mode\":\"links-only\",\"skipped\":%s,\"min_gpu_ingress_gbps\":%.1f,"
                  "\"ok\":%s}\n", links.skipped ? "true" : "false", links.min_aggregate, all_ok ? "true" : "false");
      return all_ok ? 0 : 1;
    }
  }
  // the busBW floor: --min-busbw when given, else --min-busbw-mesh-fraction of the measured mesh bound
  Opts gated = o;
  if (gated.min_busbw <= 0 && o.mesh_fraction > 0 && links.min_aggregate > 0 && !o.link_self_test)
    gated.min_busbw = o.mesh_fraction * links.min_aggregate;
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
    print_rank_summary(n, res, gated.min_busbw, gate);
    all_ok = all_ok && res.ok && (!gate || res.peak_busbw >= gated.min_busbw);
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
  // both bounds: the model's (one link / N-1 links of kLinkGBps) and the measured mesh
  // bound (the smallest per-GPU ingress with every peer pulling at once, from the link matrix)
  std::printf("{\"event\":\"summary\",\"mode\":\"single-process\",\"ranks\":%d,\"ranks_run\":[%s],"
              "\"peak_busbw_gbps\":%.2f,\"link_bound_gbps\":%.1f,\"mesh_bound_gbps\":%.1f,"
              "\"measured_mesh_bound_gbps\":%.1f,\"links_ok\":%s,\"skipped\":%s,\"ok\":%s}\n",
              largest, rs.str().c_str(), largest_peak, kLinkGBps, kLinkGBps * std::max(1, std::min(largest - 1, 7)),
              links.min_aggregate, links.ok ? "true" : "false", skipped ? "true" : "false", all_ok ? "true" : "false");
  return all_ok ? 0 : 1;
}
