"""Native decoding of the PMFW metrics table (sysfs ``gpu_metrics``) and the exporter's xGMI
metrics built on it.

The fixture ``tests/fixtures/gpu_metrics/mi355x_v1_8.bin`` is a raw table read from an MI355X;
``mi355x_v1_8.amdsmi.json`` is amd-smi's decoding of the same device taken right after it
(tools/gpu_metrics_probe.py). The native decoder must agree with amd-smi field by field.
"""

import json
import os

import pytest

from gpu_operator_amd import devices as D
from gpu_operator_amd.devices import fakesys
from gpu_operator_amd.operands import metrics_exporter as ME

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "gpu_metrics")


def _na(v):
    return -1 if v == "N/A" else v


def test_real_mi355x_table_matches_amdsmi():
    m = D.parse_gpu_metrics(open(os.path.join(FIX, "mi355x_v1_8.bin"), "rb").read())
    smi = json.load(open(os.path.join(FIX, "mi355x_v1_8.amdsmi.json")))["amdsmi"]
    assert m["valid"] and (m["format_revision"], m["content_revision"], m["structure_size"]) == (1, 8, 3872)
    for ours, theirs in (("pcie_link_width", "pcie_link_width"), ("pcie_link_speed", "pcie_link_speed"),
                         ("xgmi_link_width", "xgmi_link_width"), ("xgmi_link_speed", "xgmi_link_speed"),
                         ("uclk_mhz", "current_uclk"), ("mem_max_bandwidth", "vram_max_bandwidth")):
        assert m[ours] == smi[theirs], ours
    assert m["temp_hotspot_c"] == smi["temperature_hotspot"] and m["temp_mem_c"] == smi["temperature_mem"]
    assert m["socket_power_w"] == smi["current_socket_power"]
    assert m["xgmi_read_kb"] == smi["xgmi_read_data_acc"]
    assert m["xgmi_write_kb"] == smi["xgmi_write_data_acc"]
    assert m["xgmi_link_status"] == [_na(x) for x in smi["xgmi_link_status"]]
    # accumulators/clocks drift between the two reads: same magnitude, ours not newer
    for ours, theirs in (("energy_acc", "energy_accumulator"), ("system_clock_ns", "system_clock_counter"),
                         ("firmware_timestamp", "firmware_timestamp"), ("pcie_bandwidth_acc", "pcie_bandwidth_acc"),
                         ("accumulation_counter", "accumulation_counter")):
        assert 0 < m[ours] <= smi[theirs] and m[ours] > 0.999 * smi[theirs], ours
    assert all(abs(a - b) <= 25 for a, b in zip(m["gfxclk_mhz"], smi["current_gfxclks"]))
    assert sum(1 for s in m["xgmi_link_status"] if s == 1) == 7      # 7 xGMI peers of an 8-GPU hive


def test_unknown_revision_is_not_guessed():
    raw = bytearray(open(os.path.join(FIX, "mi355x_v1_8.bin"), "rb").read())
    raw[3] = 6                                    # content revision 6 (MI300-era layout)
    m = D.parse_gpu_metrics(bytes(raw))
    assert not m["valid"] and "v1.6" in m["error"] and m["xgmi_read_kb"] == []
    assert not D.parse_gpu_metrics(b"\x01")["valid"]
    assert "truncated" in D.parse_gpu_metrics(bytes(raw[:4]).replace(b"\x06", b"\x08", 1) + b"\0" * 40)["error"]


def test_encoder_round_trip():
    blob = fakesys.encode_gpu_metrics_v18(xgmi_read_kb=range(8), xgmi_write_kb=range(10, 18), clock_ns=123456789,
                                          xgmi_link_status=(-1, 1, 0, 1, 1, 1, 1, 1), energy_acc=65536)
    m = D.parse_gpu_metrics(blob)
    assert m["valid"] and m["xgmi_read_kb"] == list(range(8)) and m["xgmi_write_kb"] == list(range(10, 18))
    assert m["xgmi_link_status"] == [-1, 1, 0, 1, 1, 1, 1, 1] and m["system_clock_ns"] == 123456789
    assert m["energy_acc"] * D.ENERGY_UNIT_J == pytest.approx(1.0, rel=1e-3)


def _samples(reg, name):
    out = {}
    for fam in reg.collect():
        for s in fam.samples:
            if s.name == name:
                out[(s.labels["gpu"], s.labels.get("link"))] = s.value
    return out


def test_exporter_xgmi_counters_and_throughput(tmp_path):
    root = fakesys.make_node(tmp_path, n_gpus=2)
    gpus = D.enumerate_gpus(str(root))
    bdf0 = gpus[0]["pci_bdf"]
    reg = ME.build_registry(ME.load_fields(None), root=str(root), hostname="n0")
    fakesys.write_gpu_metrics(root, bdf0, fakesys.encode_gpu_metrics_v18(
        xgmi_read_kb=[0] + [1000] * 7, xgmi_write_kb=[0] + [2000] * 7, clock_ns=10 ** 12))
    first = _samples(reg, "amd_gpu_xgmi_read_bytes_total")
    assert first[("0", "1")] == 1000 * 1024 and ("0", "0") not in first      # slot 0 is N/A: no link
    assert _samples(reg, "amd_gpu_xgmi_read_throughput_bytes_per_second") == {}    # needs two samples
    # 0.5 s later link 3 moved 64 MiB each way
    rd = [0] + [1000] * 7
    wr = [0] + [2000] * 7
    rd[3] += 64 * 1024
    wr[3] += 64 * 1024
    fakesys.write_gpu_metrics(root, bdf0, fakesys.encode_gpu_metrics_v18(
        xgmi_read_kb=rd, xgmi_write_kb=wr, clock_ns=10 ** 12 + 5 * 10 ** 8))
    thr = _samples(reg, "amd_gpu_xgmi_read_throughput_bytes_per_second")
    assert thr[("0", "3")] == pytest.approx(64 * 2 ** 20 / 0.5)
    assert thr[("0", "2")] == 0.0
    assert _samples(reg, "amd_gpu_xgmi_write_throughput_bytes_per_second")[("0", "3")] == pytest.approx(2 ** 27)
    up = _samples(reg, "amd_gpu_xgmi_link_up")
    assert sum(v for (g, _), v in up.items() if g == "0") == 7
    assert _samples(reg, "amd_gpu_energy_joules_total")[("0", None)] > 0
    assert _samples(reg, "amd_gpu_xgmi_link_speed_gbps")[("0", None)] == 38


def test_exporter_skips_counter_reset_and_unsupported_tables(tmp_path):
    root = fakesys.make_node(tmp_path, n_gpus=1)
    bdf = D.enumerate_gpus(str(root))[0]["pci_bdf"]
    reg = ME.build_registry(ME.load_fields(None), root=str(root))
    fakesys.write_gpu_metrics(root, bdf, fakesys.encode_gpu_metrics_v18(xgmi_read_kb=[0] + [5000] * 7, clock_ns=10 ** 12))
    _samples(reg, "amd_gpu_xgmi_read_bytes_total")
    fakesys.write_gpu_metrics(root, bdf, fakesys.encode_gpu_metrics_v18(xgmi_read_kb=[0] + [10] * 7,
                                                                        clock_ns=2 * 10 ** 12))
    assert _samples(reg, "amd_gpu_xgmi_read_throughput_bytes_per_second") == {}      # reset: no negative rate
    raw = bytearray(fakesys.encode_gpu_metrics_v18())
    raw[3] = 5
    fakesys.write_gpu_metrics(root, bdf, bytes(raw))
    assert _samples(reg, "amd_gpu_xgmi_read_bytes_total") == {}
    assert _samples(reg, "amd_gpu_power_watts")                                      # hwmon path unaffected


def test_field_csv_selects_link_metrics(tmp_path):
    csv = tmp_path / "fields.csv"
    csv.write_text("# field\ngpu_xgmi_read_bytes_total\ngpu_power_watts\nnot_a_field\n")
    assert ME.load_fields(str(csv)) == ["gpu_xgmi_read_bytes_total", "gpu_power_watts"]


def test_default_field_configmap_lists_only_known_fields(tmp_path):
    import yaml
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    doc = yaml.safe_load(open(os.path.join(here, "gpu_operator_amd/assets/state-metrics-exporter/0800_configmap.yaml")))
    csv = tmp_path / "f.csv"
    csv.write_text(doc["data"]["fields.csv"])
    assert sorted(ME.load_fields(str(csv))) == sorted(ME.ALL_FIELDS)
