// libamdnode: host-side view of the AMD GPUs of one node, read from the kernel interfaces
// the amdgpu/KFD drivers expose (no ROCm runtime, no GPU context needed):
//
//   /sys/class/kfd/kfd/topology/nodes/<n>/properties     KFD agents (CUs, SIMDs, gfx target,
//   /sys/class/kfd/kfd/topology/nodes/<n>/io_links/*     drm render minor, unique id) and
//                                                         their links (xGMI / PCIe, weight)
//   /sys/class/drm/renderD<minor>/device -> PCI device   vendor/device, VRAM, partitions,
//                                                         hwmon, RAS, xGMI hive
//   /sys/bus/pci/devices/*                                 vendor 0x1002 functions, driver
//                                                         binding (amdgpu / vfio-pci), SR-IOV
//   /sys/module/amdgpu/{initstate,version}, /dev/kfd      driver liveness
//
// Every path is resolved under a caller-supplied root so the same code runs against the
// host (root "/" or "/host" inside a container) and against fake sysfs trees in tests.
// Used by the validator, device plugin, node labeller, partition manager and exporter.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace amdnode {

struct IoLink {
  int type = 0;             // KFD io_link type: 2 = PCIe, 11 = xGMI
  int node_from = -1;
  int node_to = -1;
  int weight = 0;
  uint64_t min_bandwidth = 0;   // MB/s as reported
  uint64_t max_bandwidth = 0;
};

struct Gpu {
  int index = 0;                // dense index over GPU agents, in KFD node order
  int kfd_node = -1;
  uint32_t gpu_id = 0;
  uint64_t unique_id = 0;
  std::string gfx_target;       // e.g. "gfx950"
  uint32_t gfx_target_version = 0;
  int simd_count = 0;
  int cu_count = 0;
  int simd_per_cu = 0;
  int max_waves_per_simd = 0;
  uint64_t lds_size_kib = 0;
  int drm_render_minor = -1;
  int drm_card = -1;
  int numa_node = -1;
  std::string pci_bdf;          // 0000:xx:yy.z
  uint16_t vendor_id = 0;
  uint16_t device_id = 0;
  uint16_t subsystem_device = 0;
  std::string pci_class;        // "0x038000"
  std::string driver;           // bound kernel driver (amdgpu, vfio-pci, ...)
  uint64_t vram_total = 0;      // bytes
  uint64_t vram_used = 0;
  std::string product_name;
  std::string vbios_version;
  std::string compute_partition;          // SPX/DPX/QPX/CPX (empty if unsupported)
  std::string memory_partition;           // NPS1/NPS2/NPS4
  std::vector<std::string> available_compute_partitions;
  std::vector<std::string> available_memory_partitions;
  uint64_t xgmi_hive_id = 0;
  int xgmi_links = 0;                     // xGMI links to other GPUs (from io_links)
  int pcie_links = 0;
  std::vector<IoLink> links;
  std::string device_path;                // resolved sysfs PCI device dir
  bool partition_capable() const { return available_compute_partitions.size() > 1; }
};

struct PciFunction {
  std::string bdf;
  uint16_t vendor_id = 0;
  uint16_t device_id = 0;
  std::string pci_class;
  std::string driver;
  int iommu_group = -1;
  int sriov_totalvfs = 0;
  int sriov_numvfs = 0;
  bool is_virtfn = false;
  std::string physfn;           // BDF of the PF for a VF
};

struct DriverState {
  bool module_loaded = false;   // /sys/module/amdgpu exists
  bool live = false;            // initstate == live
  bool kfd_present = false;     // /dev/kfd exists
  std::string version;          // /sys/module/amdgpu/version (DKMS) or empty (inbox)
  int kfd_gpu_nodes = 0;
};

struct Telemetry {
  int index = 0;
  double power_w = -1, temp_edge_c = -1, temp_junction_c = -1, temp_mem_c = -1;
  double gpu_busy_pct = -1, mem_busy_pct = -1;
  uint64_t vram_used = 0, vram_total = 0;
  double sclk_mhz = -1, mclk_mhz = -1;
  int64_t ecc_correctable = -1, ecc_uncorrectable = -1;
  double pcie_bw_bytes = -1;
  // RAS over every block the driver reports (ras/<block>_err_count: umc, gfx, sdma, mmhub, xgmi_wafl,
  // ...; -1 when the device has no RAS directory), the blocks with uncorrectable errors, and the HBM
  // pages the driver retired or holds pending retirement (ras/gpu_vram_bad_pages: R / P entries).
  int64_t ras_ue_total = -1, ras_ce_total = -1;
  std::string ras_ue_blocks;            // comma list, e.g. "umc,gfx"
  int64_t bad_pages_retired = -1, bad_pages_pending = -1;
};

// Decoded sysfs `gpu_metrics` (the PMFW metrics table the amdgpu driver exports per device).
// Only layouts verified byte-for-byte against amd-smi on real hardware are decoded (format 1,
// content 8 = MI355X; tests/fixtures/gpu_metrics/); any other revision sets `error` and leaves
// every value at its N/A default rather than guessing offsets.
struct GpuMetrics {
  int index = 0;
  std::string pci_bdf;
  bool valid = false;
  std::string error;
  int format_revision = 0, content_revision = 0;
  uint32_t structure_size = 0;
  double temp_hotspot_c = -1, temp_mem_c = -1, temp_vrsoc_c = -1;
  double socket_power_w = -1, gfx_activity_pct = -1, umc_activity_pct = -1;
  uint64_t energy_acc = 0;              // 15.259 uJ (2^-16 J) units
  uint64_t system_clock_ns = 0;         // driver timestamp of the sample
  uint64_t firmware_timestamp = 0;      // PMFW timestamp, 10 ns units
  uint64_t accumulation_counter = 0;
  uint64_t ppt_residency_acc = 0;       // power-limit (PPT) throttle residency, accumulated
  int pcie_link_width = -1, pcie_link_speed = -1;    // lanes, 0.1 GT/s
  int xgmi_link_width = -1, xgmi_link_speed = -1;    // lanes, Gbps per lane
  uint64_t pcie_bandwidth_acc = 0, pcie_bandwidth_inst = 0;   // GB/s (accumulated / instantaneous)
  uint64_t mem_max_bandwidth = 0;       // GB/s
  std::vector<uint64_t> xgmi_read_kb;   // per xGMI link: accumulated KiB read
  std::vector<uint64_t> xgmi_write_kb;  // per xGMI link: accumulated KiB written
  std::vector<int> xgmi_link_status;    // per link: 1 up, 0 down, -1 not applicable
  std::vector<int> gfxclk_mhz;          // per XCC
  int uclk_mhz = -1;
};

// --- discovery -------------------------------------------------------------------------
std::vector<Gpu> enumerate_gpus(const std::string& root = "/");
std::vector<PciFunction> scan_pci(const std::string& root = "/", uint16_t vendor = 0x1002,
                                  bool gpu_classes_only = true);
DriverState driver_state(const std::string& root = "/", const std::string& dev_root = "/");
std::vector<Telemetry> read_telemetry(const std::string& root = "/");
GpuMetrics parse_gpu_metrics(const std::string& blob);
std::vector<GpuMetrics> read_gpu_metrics(const std::string& root = "/");

// --- partitioning ------------------------------------------------------------------------
// Write current_{compute,memory}_partition of one GPU (by PCI BDF). Returns "" on success or
// an error message (mode not in available_* list, write rejected, ...).
std::string set_partition(const std::string& root, const std::string& bdf, const std::string& kind,
                          const std::string& mode);

// --- barriers -----------------------------------------------------------------------------
// Block until `names` exist in `dir` (all of them, or any one when any_of), event-driven via
// inotify (falls back to 50 ms polling if inotify is unavailable). timeout_ms < 0 waits
// forever. Returns the names that exist when it returns (empty on timeout).
std::vector<std::string> wait_files(const std::string& dir, const std::vector<std::string>& names,
                                    bool any_of, int64_t timeout_ms);

// --- helpers ------------------------------------------------------------------------------
std::string join(const std::string& root, const std::string& path);
std::map<std::string, std::string> read_kv(const std::string& path);
std::string to_json(const std::vector<Gpu>& gpus, const DriverState& drv);

}  // namespace amdnode
