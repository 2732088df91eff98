// libamdnode implementation. See amdnode.h for the interfaces read.
#include "amdnode.h"

#include <dirent.h>
#include <errno.h>
#include <poll.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <set>
#include <sstream>
#include <thread>

namespace amdnode {

namespace {

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

bool is_dir(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0 && S_ISDIR(st.st_mode);
}

std::string read_file(const std::string& p) {
  std::ifstream f(p);
  if (!f) return "";
  std::stringstream ss;
  ss << f.rdbuf();
  std::string s = ss.str();
  while (!s.empty() && (s.back() == '\n' || s.back() == '\r' || s.back() == ' ' || s.back() == '\0'))
    s.pop_back();
  return s;
}

bool write_file(const std::string& p, const std::string& v, std::string* err) {
  FILE* f = std::fopen(p.c_str(), "w");
  if (!f) {
    if (err) *err = "open " + p + ": " + std::strerror(errno);
    return false;
  }
  size_t n = std::fwrite(v.data(), 1, v.size(), f);
  int rc = std::fclose(f);
  if (n != v.size() || rc != 0) {
    if (err) *err = "write " + p + ": " + std::strerror(errno);
    return false;
  }
  return true;
}

std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = ::opendir(p.c_str());
  if (!d) return out;
  while (dirent* e = ::readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.emplace_back(e->d_name);
  }
  ::closedir(d);
  std::sort(out.begin(), out.end(), [](const std::string& a, const std::string& b) {
    // numeric-aware ordering for KFD node / hwmon directories
    bool an = !a.empty() && std::all_of(a.begin(), a.end(), ::isdigit);
    bool bn = !b.empty() && std::all_of(b.begin(), b.end(), ::isdigit);
    if (an && bn) return std::stoll(a) < std::stoll(b);
    return a < b;
  });
  return out;
}

uint64_t to_u64(const std::string& s, int base = 10) {
  if (s.empty()) return 0;
  try {
    return std::stoull(s, nullptr, base);
  } catch (...) {
    return 0;
  }
}

int64_t to_i64(const std::string& s) {
  if (s.empty()) return -1;
  try {
    return std::stoll(s);
  } catch (...) {
    return -1;
  }
}

uint64_t kv_u64(const std::map<std::string, std::string>& kv, const char* k) {
  auto it = kv.find(k);
  return it == kv.end() ? 0 : to_u64(it->second);
}

std::vector<std::string> split_modes(const std::string& s) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : s + ",") {
    if (c == ',' || c == ' ' || c == '\n') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur.push_back((char)::toupper((unsigned char)c));
    }
  }
  return out;
}

std::string gfx_name(uint32_t v) {
  // gfx_target_version = major*10000 + minor*100 + stepping; printed as gfx<major><minor:x><step:x>
  if (!v) return "";
  char b[32];
  std::snprintf(b, sizeof(b), "gfx%u%x%x", v / 10000, (v / 100) % 100, v % 100);
  return b;
}

std::string product_from_id(uint16_t dev) {
  switch (dev) {
    case 0x75a0: return "AMD Instinct MI350X";
    case 0x75a3: return "AMD Instinct MI355X";
    case 0x74a0: return "AMD Instinct MI300A";
    case 0x74a1: return "AMD Instinct MI300X";
    case 0x74a2: return "AMD Instinct MI308X";
    case 0x74a5: return "AMD Instinct MI325X";
    case 0x740f: return "AMD Instinct MI210";
    case 0x740c: return "AMD Instinct MI250X";
    default: return "";
  }
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    if (c == '"' || c == '\\') {
      o.push_back('\\');
      o.push_back(c);
    } else if ((unsigned char)c < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      o += b;
    } else {
      o.push_back(c);
    }
  }
  return o;
}

double hwmon_value(const std::string& hwdir, const std::string& file, double scale) {
  std::string v = read_file(hwdir + "/" + file);
  if (v.empty()) return -1;
  return (double)to_i64(v) * scale;
}

double current_dpm_mhz(const std::string& p) {
  // lines like "1: 2100Mhz *"
  std::ifstream f(p);
  std::string line;
  while (std::getline(f, line)) {
    if (line.find('*') == std::string::npos) continue;
    auto c = line.find(':');
    if (c == std::string::npos) continue;
    return (double)to_i64(line.substr(c + 1));
  }
  return -1;
}

}  // namespace

std::string join(const std::string& root, const std::string& path) {
  if (root.empty() || root == "/") return path;
  std::string r = root;
  while (!r.empty() && r.back() == '/') r.pop_back();
  return r + path;
}

std::map<std::string, std::string> read_kv(const std::string& path) {
  std::map<std::string, std::string> kv;
  std::ifstream f(path);
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream ls(line);
    std::string k, v;
    if (ls >> k >> v) kv[k] = v;
  }
  return kv;
}

std::vector<Gpu> enumerate_gpus(const std::string& root) {
  std::vector<Gpu> gpus;
  const std::string topo = join(root, "/sys/class/kfd/kfd/topology/nodes");
  int index = 0;
  std::map<int, int> node_to_index;
  std::set<int> cpu_nodes;
  for (const auto& n : list_dir(topo)) {
    const std::string nd = topo + "/" + n;
    auto kv = read_kv(nd + "/properties");
    if (kv_u64(kv, "simd_count") == 0) {
      // CPU agent -- or a GPU agent this cgroup may not access: KFD refuses to show its
      // properties (EPERM, empty read), so only a node with CPU cores counts as a CPU.
      if (kv_u64(kv, "cpu_cores_count") > 0) cpu_nodes.insert((int)to_u64(n));
      continue;
    }
    Gpu g;
    g.kfd_node = (int)to_u64(n);
    g.gpu_id = (uint32_t)to_u64(read_file(nd + "/gpu_id"));
    g.unique_id = kv_u64(kv, "unique_id");
    g.gfx_target_version = (uint32_t)kv_u64(kv, "gfx_target_version");
    g.gfx_target = gfx_name(g.gfx_target_version);
    g.simd_count = (int)kv_u64(kv, "simd_count");
    g.simd_per_cu = (int)kv_u64(kv, "simd_per_cu");
    g.cu_count = g.simd_per_cu ? g.simd_count / g.simd_per_cu : 0;
    g.max_waves_per_simd = (int)kv_u64(kv, "max_waves_per_simd");
    g.lds_size_kib = kv_u64(kv, "lds_size_in_kb");
    g.drm_render_minor = kv.count("drm_render_minor") ? (int)to_i64(kv["drm_render_minor"]) : -1;
    g.vendor_id = (uint16_t)kv_u64(kv, "vendor_id");
    g.device_id = (uint16_t)kv_u64(kv, "device_id");
    g.xgmi_hive_id = kv_u64(kv, "hive_id");
    const uint64_t loc = kv_u64(kv, "location_id");
    const uint64_t dom = kv_u64(kv, "domain");
    char bdf[32];
    std::snprintf(bdf, sizeof(bdf), "%04llx:%02llx:%02llx.%llx", (unsigned long long)dom,
                  (unsigned long long)((loc >> 8) & 0xff), (unsigned long long)((loc >> 3) & 0x1f),
                  (unsigned long long)(loc & 0x7));
    g.pci_bdf = bdf;
    // io links
    const std::string ld = nd + "/io_links";
    for (const auto& l : list_dir(ld)) {
      auto lk = read_kv(ld + "/" + l + "/properties");
      IoLink il;
      il.type = (int)kv_u64(lk, "type");
      il.node_from = (int)kv_u64(lk, "node_from");
      il.node_to = (int)kv_u64(lk, "node_to");
      il.weight = (int)kv_u64(lk, "weight");
      il.min_bandwidth = kv_u64(lk, "min_bandwidth");
      il.max_bandwidth = kv_u64(lk, "max_bandwidth");
      g.links.push_back(il);
    }
    // PCI device directory
    std::string dev = join(root, "/sys/bus/pci/devices/" + g.pci_bdf);
    if (!is_dir(dev) && g.drm_render_minor >= 0) {
      dev = join(root, "/sys/class/drm/renderD" + std::to_string(g.drm_render_minor) + "/device");
    }
    g.device_path = dev;
    if (is_dir(dev)) {
      if (!g.vendor_id) g.vendor_id = (uint16_t)to_u64(read_file(dev + "/vendor"), 16);
      if (!g.device_id) g.device_id = (uint16_t)to_u64(read_file(dev + "/device"), 16);
      g.subsystem_device = (uint16_t)to_u64(read_file(dev + "/subsystem_device"), 16);
      g.pci_class = read_file(dev + "/class");
      g.numa_node = (int)to_i64(read_file(dev + "/numa_node"));
      char buf[4096];
      ssize_t n = ::readlink((dev + "/driver").c_str(), buf, sizeof(buf) - 1);
      if (n > 0) {
        buf[n] = 0;
        std::string s(buf);
        g.driver = s.substr(s.find_last_of('/') + 1);
      }
      g.vram_total = to_u64(read_file(dev + "/mem_info_vram_total"));
      g.vram_used = to_u64(read_file(dev + "/mem_info_vram_used"));
      g.product_name = read_file(dev + "/product_name");
      g.vbios_version = read_file(dev + "/vbios_version");
      g.compute_partition = read_file(dev + "/current_compute_partition");
      g.memory_partition = read_file(dev + "/current_memory_partition");
      g.available_compute_partitions = split_modes(read_file(dev + "/available_compute_partition"));
      g.available_memory_partitions = split_modes(read_file(dev + "/available_memory_partition"));
      std::transform(g.compute_partition.begin(), g.compute_partition.end(), g.compute_partition.begin(), ::toupper);
      std::transform(g.memory_partition.begin(), g.memory_partition.end(), g.memory_partition.begin(), ::toupper);
      const std::string hive = read_file(dev + "/xgmi_hive_info/xgmi_hive_id");
      if (!hive.empty()) g.xgmi_hive_id = to_u64(hive);
      for (const auto& c : list_dir(dev + "/drm")) {
        if (c.rfind("card", 0) == 0) g.drm_card = (int)to_i64(c.substr(4));
      }
    }
    if (g.product_name.empty()) g.product_name = product_from_id(g.device_id);
    g.index = index;
    node_to_index[g.kfd_node] = index++;
    gpus.push_back(g);
  }
  // count xGMI/PCIe links. An xGMI io_link whose peer agent is not enumerated here (a GPU this
  // container's cgroup hides from KFD) still is a physical GPU-to-GPU link: count all but CPU peers.
  for (auto& g : gpus) {
    for (const auto& l : g.links) {
      if (l.type == 11 && !cpu_nodes.count(l.node_to)) g.xgmi_links++;
      if (l.type == 2) g.pcie_links++;
    }
  }
  return gpus;
}

std::vector<PciFunction> scan_pci(const std::string& root, uint16_t vendor, bool gpu_classes_only) {
  std::vector<PciFunction> out;
  const std::string base = join(root, "/sys/bus/pci/devices");
  for (const auto& bdf : list_dir(base)) {
    const std::string d = base + "/" + bdf;
    PciFunction f;
    f.bdf = bdf;
    f.vendor_id = (uint16_t)to_u64(read_file(d + "/vendor"), 16);
    if (vendor && f.vendor_id != vendor) continue;
    f.device_id = (uint16_t)to_u64(read_file(d + "/device"), 16);
    f.pci_class = read_file(d + "/class");
    if (gpu_classes_only) {
      const std::string c = f.pci_class.size() >= 6 ? f.pci_class.substr(0, 6) : f.pci_class;
      if (c != "0x0300" && c != "0x0380" && c != "0x1200") continue;
    }
    char buf[4096];
    ssize_t n = ::readlink((d + "/driver").c_str(), buf, sizeof(buf) - 1);
    if (n > 0) {
      buf[n] = 0;
      std::string s(buf);
      f.driver = s.substr(s.find_last_of('/') + 1);
    }
    n = ::readlink((d + "/iommu_group").c_str(), buf, sizeof(buf) - 1);
    if (n > 0) {
      buf[n] = 0;
      std::string s(buf);
      f.iommu_group = (int)to_i64(s.substr(s.find_last_of('/') + 1));
    }
    f.sriov_totalvfs = (int)to_i64(read_file(d + "/sriov_totalvfs"));
    f.sriov_numvfs = (int)to_i64(read_file(d + "/sriov_numvfs"));
    if (f.sriov_totalvfs < 0) f.sriov_totalvfs = 0;
    if (f.sriov_numvfs < 0) f.sriov_numvfs = 0;
    n = ::readlink((d + "/physfn").c_str(), buf, sizeof(buf) - 1);
    if (n > 0) {
      buf[n] = 0;
      std::string s(buf);
      f.is_virtfn = true;
      f.physfn = s.substr(s.find_last_of('/') + 1);
    }
    out.push_back(f);
  }
  return out;
}

DriverState driver_state(const std::string& root, const std::string& dev_root) {
  DriverState s;
  const std::string mod = join(root, "/sys/module/amdgpu");
  s.module_loaded = is_dir(mod);
  s.live = read_file(mod + "/initstate") == "live";
  s.version = read_file(mod + "/version");
  s.kfd_present = exists(join(dev_root, "/dev/kfd"));
  const std::string topo = join(root, "/sys/class/kfd/kfd/topology/nodes");
  for (const auto& n : list_dir(topo)) {
    auto kv = read_kv(topo + "/" + n + "/properties");
    if (kv_u64(kv, "simd_count") > 0) s.kfd_gpu_nodes++;
  }
  return s;
}

std::vector<Telemetry> read_telemetry(const std::string& root) {
  std::vector<Telemetry> out;
  for (const auto& g : enumerate_gpus(root)) {
    Telemetry t;
    t.index = g.index;
    t.vram_total = g.vram_total;
    t.vram_used = g.vram_used;
    const std::string dev = g.device_path;
    for (const auto& h : list_dir(dev + "/hwmon")) {
      const std::string hd = dev + "/hwmon/" + h;
      double p = hwmon_value(hd, "power1_average", 1e-6);
      if (p < 0) p = hwmon_value(hd, "power1_input", 1e-6);
      if (p >= 0) t.power_w = p;
      for (int i = 1; i <= 8; ++i) {
        const std::string label = read_file(hd + "/temp" + std::to_string(i) + "_label");
        double v = hwmon_value(hd, "temp" + std::to_string(i) + "_input", 1e-3);
        if (v < 0) continue;
        if (label == "edge") t.temp_edge_c = v;
        else if (label == "junction" || label == "hotspot") t.temp_junction_c = v;
        else if (label == "mem") t.temp_mem_c = v;
      }
    }
    const std::string busy = read_file(dev + "/gpu_busy_percent");
    if (!busy.empty()) t.gpu_busy_pct = (double)to_i64(busy);
    const std::string mbusy = read_file(dev + "/mem_busy_percent");
    if (!mbusy.empty()) t.mem_busy_pct = (double)to_i64(mbusy);
    t.sclk_mhz = current_dpm_mhz(dev + "/pp_dpm_sclk");
    t.mclk_mhz = current_dpm_mhz(dev + "/pp_dpm_mclk");
    // RAS: "ue: N" / "ce: M" per block; the HBM (umc) counts are the ECC fields
    auto ras = read_kv(dev + "/ras/umc_err_count");
    if (ras.count("ue:")) t.ecc_uncorrectable = to_i64(ras["ue:"]);
    if (ras.count("ce:")) t.ecc_correctable = to_i64(ras["ce:"]);
    for (const auto& f : list_dir(dev + "/ras")) {
      const std::string suffix = "_err_count";
      if (f.size() <= suffix.size() || f.compare(f.size() - suffix.size(), suffix.size(), suffix) != 0) continue;
      auto kv = read_kv(dev + "/ras/" + f);
      if (!kv.count("ue:") && !kv.count("ce:")) continue;
      const int64_t ue = kv.count("ue:") ? std::max<int64_t>(0, to_i64(kv["ue:"])) : 0;
      const int64_t ce = kv.count("ce:") ? std::max<int64_t>(0, to_i64(kv["ce:"])) : 0;
      t.ras_ue_total = std::max<int64_t>(0, t.ras_ue_total) + ue;
      t.ras_ce_total = std::max<int64_t>(0, t.ras_ce_total) + ce;
      if (ue > 0) t.ras_ue_blocks += (t.ras_ue_blocks.empty() ? "" : ",") + f.substr(0, f.size() - suffix.size());
    }
    // "0x<page> : 0x<size> : R|P|F" per line (retired / pending / failed to retire)
    const std::string bp = dev + "/ras/gpu_vram_bad_pages";
    if (exists(bp)) {
      t.bad_pages_retired = t.bad_pages_pending = 0;
      std::istringstream in(read_file(bp));
      for (std::string line; std::getline(in, line);) {
        const size_t c = line.find_last_of(':');
        if (c == std::string::npos) continue;
        std::string flag = line.substr(c + 1);
        flag.erase(0, flag.find_first_not_of(" \t"));
        if (flag.rfind("R", 0) == 0) ++t.bad_pages_retired;
        else if (flag.rfind("P", 0) == 0) ++t.bad_pages_pending;
      }
    }
    const std::string bw = read_file(dev + "/pcie_bw");
    if (!bw.empty()) {
      // "<received> <sent> <max payload>": packets in the last second
      std::istringstream ss(bw);
      uint64_t rx = 0, tx = 0, mps = 0;
      ss >> rx >> tx >> mps;
      t.pcie_bw_bytes = (double)(rx + tx) * (double)mps;
    }
    out.push_back(t);
  }
  return out;
}

namespace {

template <typename T>
T rd(const std::string& b, size_t off) {
  T v{};
  if (off + sizeof(T) <= b.size()) std::memcpy(&v, b.data() + off, sizeof(T));
  return v;
}

double na16(uint16_t v) { return v == 0xFFFF ? -1.0 : (double)v; }
int na16i(uint16_t v) { return v == 0xFFFF ? -1 : (int)v; }
uint64_t na64(uint64_t v) { return v == ~0ull ? 0 : v; }
uint64_t na32(uint32_t v) { return v == ~0u ? 0 : v; }

// gpu_metrics format 1 content 8 (MI355X PMFW, 3872 bytes). Offsets pinned against amd-smi's
// decoding of the same blob on an MI355X (tools/gpu_metrics_probe.py, tests/fixtures/gpu_metrics).
struct LayoutV18 {
  static constexpr size_t temp_hotspot = 4, temp_mem = 6, temp_vrsoc = 8, socket_power = 10;
  static constexpr size_t gfx_activity = 12, umc_activity = 14, mem_max_bw = 16, energy = 24, sysclk = 32;
  static constexpr size_t accum = 40, ppt_res = 48;
  static constexpr size_t pcie_width = 68, pcie_speed = 70, xgmi_width = 72, xgmi_speed = 74;
  static constexpr size_t pcie_bw_acc = 88, pcie_bw_inst = 96;
  static constexpr size_t xgmi_read = 136, xgmi_write = 200, xgmi_status = 264;   // 8 links each
  static constexpr size_t fw_ts = 288, gfxclk = 296, uclk = 336;
  static constexpr int links = 8, xccs = 8;
  static constexpr size_t min_size = 338;
};

}  // namespace

GpuMetrics parse_gpu_metrics(const std::string& blob) {
  GpuMetrics m;
  if (blob.size() < 4) {
    m.error = "gpu_metrics too short";
    return m;
  }
  m.structure_size = rd<uint16_t>(blob, 0);
  m.format_revision = (uint8_t)blob[2];
  m.content_revision = (uint8_t)blob[3];
  if (m.format_revision != 1 || m.content_revision != 8) {
    m.error = "unsupported gpu_metrics v" + std::to_string(m.format_revision) + "." +
              std::to_string(m.content_revision);
    return m;
  }
  using L = LayoutV18;
  if (blob.size() < L::min_size || m.structure_size < L::min_size) {
    m.error = "gpu_metrics v1.8 truncated";
    return m;
  }
  m.temp_hotspot_c = na16(rd<uint16_t>(blob, L::temp_hotspot));
  m.temp_mem_c = na16(rd<uint16_t>(blob, L::temp_mem));
  m.temp_vrsoc_c = na16(rd<uint16_t>(blob, L::temp_vrsoc));
  m.socket_power_w = na16(rd<uint16_t>(blob, L::socket_power));
  m.gfx_activity_pct = na16(rd<uint16_t>(blob, L::gfx_activity));
  m.umc_activity_pct = na16(rd<uint16_t>(blob, L::umc_activity));
  m.mem_max_bandwidth = na64(rd<uint64_t>(blob, L::mem_max_bw));
  m.energy_acc = na64(rd<uint64_t>(blob, L::energy));
  m.system_clock_ns = na64(rd<uint64_t>(blob, L::sysclk));
  m.accumulation_counter = na32(rd<uint32_t>(blob, L::accum));
  m.ppt_residency_acc = na32(rd<uint32_t>(blob, L::ppt_res));
  m.pcie_link_width = na16i(rd<uint16_t>(blob, L::pcie_width));
  m.pcie_link_speed = na16i(rd<uint16_t>(blob, L::pcie_speed));
  m.xgmi_link_width = na16i(rd<uint16_t>(blob, L::xgmi_width));
  m.xgmi_link_speed = na16i(rd<uint16_t>(blob, L::xgmi_speed));
  m.pcie_bandwidth_acc = na64(rd<uint64_t>(blob, L::pcie_bw_acc));
  m.pcie_bandwidth_inst = na64(rd<uint64_t>(blob, L::pcie_bw_inst));
  m.firmware_timestamp = na64(rd<uint64_t>(blob, L::fw_ts));
  for (int i = 0; i < L::links; ++i) {
    m.xgmi_read_kb.push_back(na64(rd<uint64_t>(blob, L::xgmi_read + 8 * i)));
    m.xgmi_write_kb.push_back(na64(rd<uint64_t>(blob, L::xgmi_write + 8 * i)));
    m.xgmi_link_status.push_back(na16i(rd<uint16_t>(blob, L::xgmi_status + 2 * i)));
  }
  for (int i = 0; i < L::xccs; ++i) m.gfxclk_mhz.push_back(na16i(rd<uint16_t>(blob, L::gfxclk + 2 * i)));
  m.uclk_mhz = na16i(rd<uint16_t>(blob, L::uclk));
  m.valid = true;
  return m;
}

std::vector<GpuMetrics> read_gpu_metrics(const std::string& root) {
  std::vector<GpuMetrics> out;
  for (const auto& g : enumerate_gpus(root)) {
    std::ifstream f(g.device_path + "/gpu_metrics", std::ios::binary);
    GpuMetrics m;
    if (!f) {
      m.error = "no gpu_metrics";
    } else {
      std::string blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      m = parse_gpu_metrics(blob);
    }
    m.index = g.index;
    m.pci_bdf = g.pci_bdf;
    out.push_back(m);
  }
  return out;
}

std::string set_partition(const std::string& root, const std::string& bdf, const std::string& kind,
                          const std::string& mode) {
  if (kind != "compute" && kind != "memory") return "kind must be compute or memory";
  const std::string dev = join(root, "/sys/bus/pci/devices/" + bdf);
  if (!is_dir(dev)) return "no such PCI device " + bdf;
  std::string want = mode;
  std::transform(want.begin(), want.end(), want.begin(), ::toupper);
  auto avail = split_modes(read_file(dev + "/available_" + kind + "_partition"));
  if (std::find(avail.begin(), avail.end(), want) == avail.end()) {
    std::string a;
    for (auto& x : avail) a += (a.empty() ? "" : ",") + x;
    return "mode " + want + " not in available_" + kind + "_partition [" + a + "]";
  }
  std::string cur = read_file(dev + "/current_" + kind + "_partition");
  std::transform(cur.begin(), cur.end(), cur.begin(), ::toupper);
  if (cur == want) return "";
  std::string err;
  if (!write_file(dev + "/current_" + kind + "_partition", want, &err)) return err;
  return "";
}

std::vector<std::string> wait_files(const std::string& dir, const std::vector<std::string>& names,
                                    bool any_of, int64_t timeout_ms) {
  using clock = std::chrono::steady_clock;
  const auto deadline = clock::now() + std::chrono::milliseconds(timeout_ms < 0 ? 0 : timeout_ms);
  auto present = [&]() {
    std::vector<std::string> have;
    for (const auto& n : names)
      if (exists(dir + "/" + n)) have.push_back(n);
    return have;
  };
  auto satisfied = [&](const std::vector<std::string>& have) {
    return any_of ? !have.empty() : have.size() == names.size();
  };
  auto remaining_ms = [&]() -> int {
    if (timeout_ms < 0) return 1000;
    auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - clock::now()).count();
    return left < 0 ? 0 : (int)std::min<int64_t>(left, 1000);
  };
  // the directory may not exist yet (hostPath created by another pod): poll for it
  while (!is_dir(dir)) {
    if (timeout_ms >= 0 && clock::now() >= deadline) return {};
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  int fd = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  int wd = fd >= 0 ? inotify_add_watch(fd, dir.c_str(), IN_CREATE | IN_MOVED_TO | IN_CLOSE_WRITE | IN_ATTRIB |
                                                           IN_DELETE_SELF | IN_MOVE_SELF)
                   : -1;
  std::vector<std::string> have = present();  // check after arming the watch: no lost event
  while (!satisfied(have)) {
    int ms = remaining_ms();
    if (timeout_ms >= 0 && ms == 0) {
      have.clear();
      break;
    }
    if (wd >= 0) {
      struct pollfd p = {fd, POLLIN, 0};
      int r = ::poll(&p, 1, ms);
      if (r > 0) {
        char buf[4096];
        while (::read(fd, buf, sizeof(buf)) > 0) {
        }
      }
    } else {
      std::this_thread::sleep_for(std::chrono::milliseconds(std::min(ms, 50)));
    }
    have = present();
  }
  if (fd >= 0) ::close(fd);
  return have;
}

std::string to_json(const std::vector<Gpu>& gpus, const DriverState& drv) {
  std::ostringstream o;
  o << "{\"driver\":{\"module_loaded\":" << (drv.module_loaded ? "true" : "false")
    << ",\"live\":" << (drv.live ? "true" : "false") << ",\"kfd\":" << (drv.kfd_present ? "true" : "false")
    << ",\"version\":\"" << json_escape(drv.version) << "\",\"kfd_gpu_nodes\":" << drv.kfd_gpu_nodes
    << "},\"gpus\":[";
  for (size_t i = 0; i < gpus.size(); ++i) {
    const Gpu& g = gpus[i];
    if (i) o << ",";
    o << "{\"index\":" << g.index << ",\"kfd_node\":" << g.kfd_node << ",\"gpu_id\":" << g.gpu_id
      << ",\"unique_id\":" << g.unique_id << ",\"gfx\":\"" << g.gfx_target << "\",\"cu_count\":" << g.cu_count
      << ",\"simd_count\":" << g.simd_count << ",\"lds_kib\":" << g.lds_size_kib
      << ",\"render_minor\":" << g.drm_render_minor << ",\"card\":" << g.drm_card
      << ",\"numa_node\":" << g.numa_node << ",\"bdf\":\"" << g.pci_bdf << "\",\"vendor\":" << g.vendor_id
      << ",\"device\":" << g.device_id << ",\"driver\":\"" << json_escape(g.driver)
      << "\",\"vram_total\":" << g.vram_total << ",\"product\":\"" << json_escape(g.product_name)
      << "\",\"compute_partition\":\"" << g.compute_partition << "\",\"memory_partition\":\""
      << g.memory_partition << "\",\"xgmi_hive_id\":" << g.xgmi_hive_id << ",\"xgmi_links\":" << g.xgmi_links
      << ",\"available_compute_partitions\":[";
    for (size_t j = 0; j < g.available_compute_partitions.size(); ++j)
      o << (j ? "," : "") << "\"" << g.available_compute_partitions[j] << "\"";
    o << "],\"available_memory_partitions\":[";
    for (size_t j = 0; j < g.available_memory_partitions.size(); ++j)
      o << (j ? "," : "") << "\"" << g.available_memory_partitions[j] << "\"";
    o << "]}";
  }
  o << "]}";
  return o.str();
}

}  // namespace amdnode
