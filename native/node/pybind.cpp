// Python bindings of libamdnode (module gpu_operator_amd._native._amdnode).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "amdnode.h"

namespace py = pybind11;
using namespace amdnode;

PYBIND11_MODULE(_amdnode, m) {
  m.doc() = "AMD GPU node discovery, partitioning, telemetry and inotify barrier waits";

  py::class_<IoLink>(m, "IoLink")
      .def_readonly("type", &IoLink::type)
      .def_readonly("node_from", &IoLink::node_from)
      .def_readonly("node_to", &IoLink::node_to)
      .def_readonly("weight", &IoLink::weight)
      .def_readonly("min_bandwidth", &IoLink::min_bandwidth)
      .def_readonly("max_bandwidth", &IoLink::max_bandwidth);

  py::class_<Gpu>(m, "Gpu")
      .def_readonly("index", &Gpu::index)
      .def_readonly("kfd_node", &Gpu::kfd_node)
      .def_readonly("gpu_id", &Gpu::gpu_id)
      .def_readonly("unique_id", &Gpu::unique_id)
      .def_readonly("gfx_target", &Gpu::gfx_target)
      .def_readonly("gfx_target_version", &Gpu::gfx_target_version)
      .def_readonly("simd_count", &Gpu::simd_count)
      .def_readonly("cu_count", &Gpu::cu_count)
      .def_readonly("simd_per_cu", &Gpu::simd_per_cu)
      .def_readonly("max_waves_per_simd", &Gpu::max_waves_per_simd)
      .def_readonly("lds_size_kib", &Gpu::lds_size_kib)
      .def_readonly("drm_render_minor", &Gpu::drm_render_minor)
      .def_readonly("drm_card", &Gpu::drm_card)
      .def_readonly("numa_node", &Gpu::numa_node)
      .def_readonly("pci_bdf", &Gpu::pci_bdf)
      .def_readonly("vendor_id", &Gpu::vendor_id)
      .def_readonly("device_id", &Gpu::device_id)
      .def_readonly("subsystem_device", &Gpu::subsystem_device)
      .def_readonly("pci_class", &Gpu::pci_class)
      .def_readonly("driver", &Gpu::driver)
      .def_readonly("vram_total", &Gpu::vram_total)
      .def_readonly("vram_used", &Gpu::vram_used)
      .def_readonly("product_name", &Gpu::product_name)
      .def_readonly("vbios_version", &Gpu::vbios_version)
      .def_readonly("compute_partition", &Gpu::compute_partition)
      .def_readonly("memory_partition", &Gpu::memory_partition)
      .def_readonly("available_compute_partitions", &Gpu::available_compute_partitions)
      .def_readonly("available_memory_partitions", &Gpu::available_memory_partitions)
      .def_readonly("xgmi_hive_id", &Gpu::xgmi_hive_id)
      .def_readonly("xgmi_links", &Gpu::xgmi_links)
      .def_readonly("pcie_links", &Gpu::pcie_links)
      .def_readonly("links", &Gpu::links)
      .def_readonly("device_path", &Gpu::device_path)
      .def_property_readonly("partition_capable", &Gpu::partition_capable);

  py::class_<PciFunction>(m, "PciFunction")
      .def_readonly("bdf", &PciFunction::bdf)
      .def_readonly("vendor_id", &PciFunction::vendor_id)
      .def_readonly("device_id", &PciFunction::device_id)
      .def_readonly("pci_class", &PciFunction::pci_class)
      .def_readonly("driver", &PciFunction::driver)
      .def_readonly("iommu_group", &PciFunction::iommu_group)
      .def_readonly("sriov_totalvfs", &PciFunction::sriov_totalvfs)
      .def_readonly("sriov_numvfs", &PciFunction::sriov_numvfs)
      .def_readonly("is_virtfn", &PciFunction::is_virtfn)
      .def_readonly("physfn", &PciFunction::physfn);

  py::class_<DriverState>(m, "DriverState")
      .def_readonly("module_loaded", &DriverState::module_loaded)
      .def_readonly("live", &DriverState::live)
      .def_readonly("kfd_present", &DriverState::kfd_present)
      .def_readonly("version", &DriverState::version)
      .def_readonly("kfd_gpu_nodes", &DriverState::kfd_gpu_nodes);

  py::class_<Telemetry>(m, "Telemetry")
      .def_readonly("index", &Telemetry::index)
      .def_readonly("power_w", &Telemetry::power_w)
      .def_readonly("temp_edge_c", &Telemetry::temp_edge_c)
      .def_readonly("temp_junction_c", &Telemetry::temp_junction_c)
      .def_readonly("temp_mem_c", &Telemetry::temp_mem_c)
      .def_readonly("gpu_busy_pct", &Telemetry::gpu_busy_pct)
      .def_readonly("mem_busy_pct", &Telemetry::mem_busy_pct)
      .def_readonly("vram_used", &Telemetry::vram_used)
      .def_readonly("vram_total", &Telemetry::vram_total)
      .def_readonly("sclk_mhz", &Telemetry::sclk_mhz)
      .def_readonly("mclk_mhz", &Telemetry::mclk_mhz)
      .def_readonly("ecc_correctable", &Telemetry::ecc_correctable)
      .def_readonly("ecc_uncorrectable", &Telemetry::ecc_uncorrectable)
      .def_readonly("pcie_bw_bytes", &Telemetry::pcie_bw_bytes)
      .def_readonly("ras_ue_total", &Telemetry::ras_ue_total)
      .def_readonly("ras_ce_total", &Telemetry::ras_ce_total)
      .def_readonly("ras_ue_blocks", &Telemetry::ras_ue_blocks)
      .def_readonly("bad_pages_retired", &Telemetry::bad_pages_retired)
      .def_readonly("bad_pages_pending", &Telemetry::bad_pages_pending);

  py::class_<GpuMetrics>(m, "GpuMetrics")
      .def_readonly("index", &GpuMetrics::index)
      .def_readonly("pci_bdf", &GpuMetrics::pci_bdf)
      .def_readonly("valid", &GpuMetrics::valid)
      .def_readonly("error", &GpuMetrics::error)
      .def_readonly("format_revision", &GpuMetrics::format_revision)
      .def_readonly("content_revision", &GpuMetrics::content_revision)
      .def_readonly("structure_size", &GpuMetrics::structure_size)
      .def_readonly("temp_hotspot_c", &GpuMetrics::temp_hotspot_c)
      .def_readonly("temp_mem_c", &GpuMetrics::temp_mem_c)
      .def_readonly("temp_vrsoc_c", &GpuMetrics::temp_vrsoc_c)
      .def_readonly("socket_power_w", &GpuMetrics::socket_power_w)
      .def_readonly("gfx_activity_pct", &GpuMetrics::gfx_activity_pct)
      .def_readonly("umc_activity_pct", &GpuMetrics::umc_activity_pct)
      .def_readonly("energy_acc", &GpuMetrics::energy_acc)
      .def_readonly("system_clock_ns", &GpuMetrics::system_clock_ns)
      .def_readonly("firmware_timestamp", &GpuMetrics::firmware_timestamp)
      .def_readonly("accumulation_counter", &GpuMetrics::accumulation_counter)
      .def_readonly("ppt_residency_acc", &GpuMetrics::ppt_residency_acc)
      .def_readonly("pcie_link_width", &GpuMetrics::pcie_link_width)
      .def_readonly("pcie_link_speed", &GpuMetrics::pcie_link_speed)
      .def_readonly("xgmi_link_width", &GpuMetrics::xgmi_link_width)
      .def_readonly("xgmi_link_speed", &GpuMetrics::xgmi_link_speed)
      .def_readonly("pcie_bandwidth_acc", &GpuMetrics::pcie_bandwidth_acc)
      .def_readonly("pcie_bandwidth_inst", &GpuMetrics::pcie_bandwidth_inst)
      .def_readonly("mem_max_bandwidth", &GpuMetrics::mem_max_bandwidth)
      .def_readonly("xgmi_read_kb", &GpuMetrics::xgmi_read_kb)
      .def_readonly("xgmi_write_kb", &GpuMetrics::xgmi_write_kb)
      .def_readonly("xgmi_link_status", &GpuMetrics::xgmi_link_status)
      .def_readonly("gfxclk_mhz", &GpuMetrics::gfxclk_mhz)
      .def_readonly("uclk_mhz", &GpuMetrics::uclk_mhz);

  m.def("enumerate_gpus", &enumerate_gpus, py::arg("root") = "/");
  m.def("scan_pci", &scan_pci, py::arg("root") = "/", py::arg("vendor") = 0x1002,
        py::arg("gpu_classes_only") = true);
  m.def("driver_state", &driver_state, py::arg("root") = "/", py::arg("dev_root") = "/");
  m.def("read_telemetry", &read_telemetry, py::arg("root") = "/");
  m.def("read_gpu_metrics", &read_gpu_metrics, py::arg("root") = "/");
  m.def("parse_gpu_metrics", [](const py::bytes& b) { return parse_gpu_metrics(std::string(b)); });
  m.def("set_partition", &set_partition, py::arg("root"), py::arg("bdf"), py::arg("kind"), py::arg("mode"));
  m.def(
      "wait_files",
      [](const std::string& dir, const std::vector<std::string>& names, bool any_of, int64_t timeout_ms) {
        py::gil_scoped_release release;   // let other Python threads run while blocked
        return wait_files(dir, names, any_of, timeout_ms);
      },
      py::arg("dir"), py::arg("names"), py::arg("any_of") = false, py::arg("timeout_ms") = -1);
  m.def("to_json", &to_json);
}
