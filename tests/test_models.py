"""GPU model catalog."""

from gpu_operator_amd import models


def test_catalog_lookup():
    m, vf = models.by_device_id(0x75A3)
    assert m.name == "MI355X" and not vf and m.gfx == "gfx950" and m.family == "cdna4"
    assert m.hbm_gib == 288 and m.cus == 256 and m.lds_kib == 160 and m.xgmi_links == 7
    assert m.partition_capable and "CPX" in m.compute_partitions and "NPS2" in m.memory_partitions
    assert models.by_device_id(0x75B3) == (m, True)
    assert models.by_device_id(0x1234) is None
    assert models.by_name("MI300X").gfx == "gfx942"
    assert models.family_of_gfx("gfx950") == "cdna4" and models.family_of_gfx("gfx000") == "unknown"
    assert models.PARTITION_CAPABLE_FAMILIES == {"cdna3", "cdna4"}


def test_dense_peaks_exclude_sparsity():
    m = models.by_name("MI355X")
    # dense bf16 ~2.5 PF, fp8 2x bf16 (no 2:1 sparsity factor)
    assert 2400 < m.bf16_dense_tflops < 2600 and m.fp8_dense_tflops == 2 * m.bf16_dense_tflops
    assert m.gemm_floor_tflops() < 1000
    ids = [d for g in models.CATALOG for d in g.device_ids + g.vf_device_ids]
    assert len(ids) == len(set(ids))
