"""Static audit of the gfx950 GEMM code object (CPU-only: hipcc cross-compiles).

The v10 kernel keeps its 256 accumulators in literal AGPRs written by inline-asm MFMAs
(native/hip/gemm_bf16.hip, "v10" comment). That is only sound if hipcc never touches an AGPR
itself, so every build is audited here: no compiler-emitted ``v_accvgpr_*`` outside the asm
blocks, no scratch, occupancy 1, and the main loop carries exactly one barrier and no
hipcc-inserted ``s_nop`` hazard padding (which would mean an unmodelled dependency)."""

import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _compile(tmp_path_factory, src: str) -> str:
    out = tmp_path_factory.mktemp("gemm_asm") / "gemm.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT}/native/include",
                    "--cuda-device-only", "-S", os.path.join(ROOT, "native/hip", src), "-o", str(out)],
                   check=True, capture_output=True, timeout=600)
    return out.read_text()


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    return _compile(tmp_path_factory, "gemm_bf16.hip")


@pytest.fixture(scope="module")
def asm_fp8(tmp_path_factory):
    return _compile(tmp_path_factory, "gemm_fp8.hip")


def _kernels(asm: str, name: str, rec: bool = False):
    """The kernels whose mangled name contains `name`: the timed instantiations, or with `rec` the
    placement-recording ones (test_placement_record_only_in_rec_kernels audits those)."""
    starts = [m for m in re.finditer(rf"^(_Z\w*{name}\w*):", asm, re.M) if _is_rec(m.group(1)) == rec]
    assert starts, name
    return [_kernel_at(asm, m) for m in starts]


def _kernel_at(asm: str, start):
    body = asm[start.start():asm.index(".end_amdhsa_kernel", start.start())]
    tail = asm[start.start():]
    stats = {k: int(v) for k, v in re.findall(r"^; (NumVgprs|NumAgprs|ScratchSize|Occupancy): (\d+)", tail,
                                                re.M)[:4]}
    return body, stats


@pytest.fixture(scope="module")
def asm_lab(tmp_path_factory):
    return _compile(tmp_path_factory, "gemm_bf16_lab.hip")


@pytest.fixture(scope="module", params=["production", "lab"])
def w4(request):
    asm = request.getfixturevalue("asm" if request.param == "production" else "asm_lab")
    # the hand-scheduled asm K pipeline (w4a/w4ap) has no compiler loop: audited separately below
    return [k for k in _kernels(asm, "gemm_bf16_256x256_w4") if not re.match(r"\w*w4ap?(?:_sk)?I", k[0])]


def test_production_library_kernel_set(asm):
    """The shipped code object holds exactly the production kernels: w4s for v18/v42/v44/v45, the
    persistent w4sp (v25) and the generic kernel -- no superseded generation, no knock-out build."""
    names = re.findall(r"^(_Z\w+):", asm, re.M)
    # every production kernel twice: the timed instantiation and the placement-recording one (REC,
    # the last template argument) that amd-gemm-validate's checked dispatch runs
    assert len([x for x in names if "w4sI" in x]) == 2 * 6     # v18, v42, v44, v45, v47, v48
    assert len([x for x in names if "w4spI" in x]) == 2 * 1
    assert not [x for x in names if re.search(r"w4I|w4rI|_ppI|256x256_v2|256x256P", x)], names
    assert "AMDGO_GEMM" not in asm


def test_production_sources_read_no_environment():
    for f in ("gemm_bf16.hip", "gemm_fp8.hip", "gemm_bf16_kernels.h", "gemm_fp8_kernels.h"):
        text = open(os.path.join(ROOT, "native/hip", f)).read()
        assert "getenv" not in text, f


def _no_compiler_agpr_access(body: str):
    outside = []
    in_asm = False
    for line in body.splitlines():
        if ";;#ASMSTART" in line:
            in_asm = True
        elif ";;#ASMEND" in line:
            in_asm = False
        elif not in_asm and "v_accvgpr" in line:
            outside.append(line.strip())
    assert not outside, outside[:5]


def _audit_q16(kernels):
    for body, st in kernels:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        assert st["NumVgprs"] <= 160, st
        _no_compiler_agpr_access(body)
        assert "v_mfma_scale" not in body
        loop = re.search(r"; =>\s*This Inner Loop Header.*?\n(.*?)s_cbranch_scc\d \.LBB", body, re.S)
        assert loop, "main loop not found"
        text = loop.group(1)
        assert text.count("v_mfma_f32_16x16x128_f8f6f4") == 64
        assert text.count("ds_read_b128") == 32
        assert len(re.findall(r"buffer_load_dwordx4 .* lds", text)) == 16
        assert text.count("s_barrier") == 2
        # fragments are loaded straight into the 8-VGPR operand tuples: no VALU copies before MFMAs
        assert "v_mov_b32" not in text


def test_fp8_kernel_audit(asm_fp8):
    """fp8 production q16 (unscaled v_mfma_f32_16x16x128_f8f6f4): 256 pinned AGPRs, one 128-VGPR
    fragment set (no spills into AGPRs), 64 MFMAs / 32 ds_read_b128 / 16 LDS-DMA pieces per
    K-tile, two barriers per K-tile (buffer free, next tile landed)."""
    kernels = _kernels(asm_fp8, "gemm_fp8_256x256_q16I")
    assert len(kernels) == 3    # production: v15, v16 (square raster), v17 (no serpentine K)
    _audit_q16(kernels)
    assert "gemm_fp8_256x256_w4sI" not in asm_fp8     # superseded: lab only


def test_fp8_w4s_lab_kernel_audit(asm_fp8_lab):
    """fp8 w4s (block-scaled 32x32x64, the round-1 default, now lab v1-v9/v13): 256 pinned AGPRs,
    no scratch, 32 scaled MFMAs per K-tile, 2 barriers, 16 DMA pieces."""
    kernels = _kernels(asm_fp8_lab, "gemm_fp8_256x256_w4sI")
    assert len(kernels) == 10
    for body, st in kernels:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        _no_compiler_agpr_access(body)
        assert "v_mfma_f32" not in body.replace("v_mfma_scale_f32", "")
        loop = re.search(r"; =>\s*This Inner Loop Header.*?\n(.*?)s_cbranch_scc\d \.LBB", body, re.S)
        assert loop, "main loop not found"
        text = loop.group(1)
        assert text.count("v_mfma_scale") == 32
        assert text.count("ds_read_b128") == 32
        assert len(re.findall(r"buffer_load_dwordx4 .* lds", text)) == 16
        assert text.count("s_barrier") == 2
        assert "v_mov_b32" not in text


def test_fp8_persistent_q16_kernel_audit(asm_fp8):
    """Persistent q16 (v18): pinned AGPRs, one fragment set, unscaled 16x16x128 only; the fresh,
    steady, last-with-read and last iterations are each one 64-MFMA body."""
    kernels = _kernels(asm_fp8, "gemm_fp8_256x256_q16pI")
    assert len(kernels) == 1
    for body, st in kernels:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        assert st["NumVgprs"] <= 192, st
        _no_compiler_agpr_access(body)
        assert "v_mfma_scale" not in body
        assert len(re.findall(r"v_mfma_f32_16x16x128_f8f6f4", body)) == 4 * 64


def test_fp8_persistent_kernel_audit(asm_fp8):
    kernels = _kernels(asm_fp8, "gemm_fp8_256x256_w4spI")
    assert len(kernels) == 1    # production: v10
    for body, st in kernels:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        _no_compiler_agpr_access(body)
        # fresh + steady iterations of every tile, plus the two tail iterations of the last one
        assert len(re.findall(r"v_mfma_scale_f32_32x32x64_f8f6f4", body)) == 4 * 32


def test_w4_accumulators_pinned(w4):
    for body, st in w4:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        assert st["NumVgprs"] <= 256
        _no_compiler_agpr_access(body)
        # 3 instances of the 128-MFMA iteration (steady, last-with-read, last); the persistent
        # w4sp adds its peeled first iteration of every tile
        name = body.split(":", 1)[0]
        assert len(re.findall(r"v_mfma_f32_16x16x32_bf16", body)) == (8 if "w4sp" in name else 6) * 64


def _audit_asm_pipeline(body, st):
    assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
    assert st["NumVgprs"] <= 256, st
    _no_compiler_agpr_access(body)
    mfma = len(re.findall(r"v_mfma_f32_16x16x32_bf16", body))
    # 16-byte reads: fragment reads, and the staged epilogue's C rows (the LEAN forms read those as
    # 8-byte halves, which hipcc may pair into ds_read2st64_b64)
    reads = (body.count("ds_read_b128") + len(re.findall(r"\bds_read_b64\b", body)) // 2 +
             len(re.findall(r"\bds_read2(?:st64)?_b64\b", body)))
    dma = len(re.findall(r"buffer_load_dwordx4 .* lds", body))
    # every K-tile in the asm block is 128 MFMAs fed by 32 fragment reads and 16 LDS-DMA pieces;
    # the persistent form adds the epilogue reads of the next tile's prologue
    assert mfma % 128 == 0 and mfma >= 3 * 128, mfma
    name = body.split(":", 1)[0]
    if re.search(r"w4apILi\d+ELb\dELb\dELi9E", name):
        # direct epilogue (EPI 9): the EF fragment layout with standard bodies; C stored after the block
        # straight from the accumulators (32 pair stores, 256 accumulator reads, no LDS staging)
        assert mfma == 8 * 128 and reads == 16 + 6 * 32 + 2 * 16, (mfma, reads)
        assert body.count("global_store_dwordx4") == 32 and body.count("v_accvgpr_read_b32") == 256
        return mfma
    if re.search(r"w4apILi\d+ELb\dELb\dELi2E", name):
        # fused epilogue (EPI=2): peeled first K-tile pair, loop, two drains whose last K-tiles read
        # only k-half 1 and store the C tile (32 pair stores each); no compiler epilogue
        assert mfma == 8 * 128 and reads == 16 + 6 * 32 + 2 * 16, (mfma, reads)
        assert body.count("global_store_dwordx4") == 2 * 32, body.count("global_store_dwordx4")
        assert body.count("v_accvgpr_read_b32") == 2 * 256
        return mfma
    assert reads >= 32 * (mfma // 128) and dma >= 16 * (mfma // 128 - 2), (reads, dma)
    # the loop itself is one asm block: hipcc inserted no hazard padding into it
    for blk in re.findall(r";;#ASMSTART(.*?);;#ASMEND", body, re.S):
        if blk.count("v_mfma") >= 128:
            assert "s_cbranch" in blk and "s_barrier" in blk
    return mfma


def test_w4ap_production_pipeline(asm):
    """Production v50 / v51 / v52 / v53 / v54 / v55 / v56: the persistent asm K pipeline (main schedule,
    its square-raster form, the long-K schedule, the VP DMA form, linear and square raster, and the
    VP + PA form with the LEAN epilogue, linear and square raster)."""
    kernels = _kernels(asm, "gemm_bf16_256x256_w4apI")
    assert len(kernels) == 7
    for body, st in kernels:
        # the zc schedules (every production form) peel the first K-tile pair (src C = 0): 8 bodies
        assert _audit_asm_pipeline(body, st) == 8 * 128
        assert "v_accvgpr_write" not in body      # src C = 0 instead of zeroing writes


def test_w4ap_split_k_pipeline(asm):
    """Production v57: the asm K pipeline of v55 (VP + PA, LEAN epilogue) in its split-K form -- the same
    8 K-tile bodies, plus the reduction (gemm_w4ap.h SPLIT): an arrival ticket and a done count per
    tile (two agent atomics), the partial slab as 64 16-byte stores per wave, one release per writing
    workgroup and one acquire per reducing one, and the last arrival's sum written back into the 256
    accumulators (the two-piece path and the general one)."""
    kernels = _kernels(asm, "gemm_bf16_256x256_w4ap_skI")
    assert len(kernels) == 1
    for body, st in kernels:
        assert _audit_asm_pipeline(body, st) == 8 * 128
        writes = body.count("v_accvgpr_write_b32")
        assert writes % 256 == 0 and writes >= 2 * 256, writes
        assert len(re.findall(r"global_atomic_add\b", body)) == 2
        assert len(re.findall(r"global_store_dwordx4\b", body)) >= 64
        assert body.count("buffer_wbl2") == 1 and body.count("buffer_inv") == 1


def test_w4a_lab_pipelines(tmp_path_factory):
    """Every lab schedule of the asm K pipeline keeps the same register/occupancy contract."""
    asm = _compile(tmp_path_factory, "gemm_bf16_asm_lab.hip")
    kernels = _kernels(asm, "gemm_bf16_256x256_w4a")
    assert len(kernels) >= 10
    for body, st in kernels:
        if re.search(r"w4apILi\d+ELb\dELb\dELi[13]E", body.split(":", 1)[0]):
            continue                        # knock-out builds (EPI 1 / 3) drop the epilogue on purpose
        _audit_asm_pipeline(body, st)
    # the fused-epilogue fp8 kernels: 4 K-tile pairs of 64 MFMAs, C stored from the asm block
    ef8 = [k for k in _kernels(asm, "gemm_fp8_256x256_q16apI") if re.search(r"Lb\dELb\dELi2E", k[0].split(":", 1)[0])]
    assert len(ef8) >= 3
    for body, st in ef8:
        assert st["NumAgprs"] == 256 and st["ScratchSize"] == 0 and st["Occupancy"] == 1, st
        _no_compiler_agpr_access(body)
        assert len(re.findall(r"v_mfma_f32_16x16x128_f8f6f4", body)) == 8 * 64
        assert body.count("global_store_dwordx4") == 2 * 32 and body.count("v_accvgpr_read_b32") == 2 * 256


def test_w4_main_loop_shape(w4):
    for body, _ in w4:
        ko = re.match(r"\w*w4ILi\d+ELi\d+ELi(\d+)E", body)
        if ko and int(ko.group(1)):
            continue                        # knock-out profiling builds drop parts on purpose
        loop = re.search(r"; =>\s*This Inner Loop Header.*?\n(.*?)s_cbranch_scc\d \.LBB", body, re.S)
        assert loop, "main loop not found"
        text = loop.group(1)
        assert text.count("v_mfma") == 128
        assert text.count("ds_read_b128") == 32
        assert len(re.findall(r"buffer_load_dwordx4 .* lds", text)) == 16
        # v10 syncs once per K-tile; the v15 half-tile ring once per 64-MFMA block; v18 twice per
        # K-tile (buffer free for DMA, next tile landed)
        name = body.split(":", 1)[0]
        if "w4t" in name:        # lab schedule classes: split A/B panel barriers add one
            expected = 3 if "SchedSplit" in name else 2
        else:
            expected = 2 if ("w4r" in name or "w4s" in name) else 1
        assert text.count("s_barrier") == expected, name
        assert "scratch_" not in text
        # the only padding hipcc may add is the M0 write -> LDS-DMA nop; anything else means it
        # found a dependency the asm MFMAs hide from it
        ins = [x.strip() for x in text.splitlines() if x.strip() and not x.strip().startswith((";", "."))]
        for i, x in enumerate(ins):
            if x.startswith("s_nop"):
                assert ins[i + 1].startswith("buffer_load") and ins[i + 1].endswith(" lds"), ins[i - 3:i + 2]


def test_no_kernel_spills(asm):
    for m in re.finditer(r"^; ScratchSize: (\d+)", asm, re.M):
        assert int(m.group(1)) == 0


def test_shipped_library_exports_no_lab_entry_points():
    """libamdgo_hip.so (validator + ops) carries only the production dispatch: no lab symbols, no
    environment switch, and the variant API refuses everything outside the production set."""
    lib = os.path.join(ROOT, "gpu_operator_amd", "_native", "libamdgo_hip.so")
    if not os.path.exists(lib):
        pytest.skip("native library not built")
    syms = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    assert "amdgo_gemm_bf16" in syms and "lab" not in syms
    assert b"AMDGO_GEMM" not in open(lib, "rb").read()
    from gpu_operator_amd.ops import gemm as G
    for bad in (1, 20, 24, 46, 14):
        with pytest.raises(ValueError):
            G.set_variant(bad)
    for bad in (1, 5, 11, 14):
        with pytest.raises(ValueError):
            G.set_fp8_variant(bad)
    G.set_variant(0)
    G.set_fp8_variant(0)


@pytest.fixture(scope="module")
def asm_fp8_lab(tmp_path_factory):
    return _compile(tmp_path_factory, "gemm_fp8_lab.hip")


def test_fp8_q16_kernel_audit(asm_fp8_lab):
    """q16 lab placements (v20-v37): the same invariants as the production q16 kernels."""
    kernels = _kernels(asm_fp8_lab, "gemm_fp8_256x256_q16I")
    assert len(kernels) == 18
    _audit_q16(kernels)


@pytest.mark.parametrize("gen,headers", [
    ("gen_bf16_asm_loop.py", ["gemm_bf16_asm_loop.h", "gemm_bf16_asm_loop_lab.h"]),
    ("gen_fp8_asm_loop.py", ["gemm_fp8_asm_loop.h", "gemm_fp8_asm_loop_lab.h"]),
])
def test_generated_asm_headers_match_generator(tmp_path, gen, headers):
    """The checked-in K-pipeline headers are exactly what their generator emits today: a generator
    edit committed without regenerating (or a hand-edited header) fails here."""
    subprocess.run(["python3", os.path.join(ROOT, "tools", gen), "--out-dir", str(tmp_path)], check=True,
                   capture_output=True, timeout=300)
    for h in headers:
        want = (tmp_path / h).read_bytes()
        have = open(os.path.join(ROOT, "native", "hip", h), "rb").read()
        assert have == want, f"native/hip/{h} differs from tools/{gen} output: regenerate it"


def test_production_asm_headers_carry_only_shipped_schedules():
    """Production builds (libamdgo_hip.so, amd-gemm-validate) read the small headers; only the lab
    sources include the *_lab.h headers (which carry every schedule)."""
    hip = os.path.join(ROOT, "native", "hip")
    prod = [open(os.path.join(hip, h)).read() for h in ("gemm_bf16_asm_loop.h", "gemm_fp8_asm_loop.h")]
    assert sum(p.count("\n") for p in prod) < 10000
    asm_defs = sorted(re.findall(r"^#define (\w+_ASM_\w+) \\", "\n".join(prod), re.M))
    assert asm_defs == ["F8AP_ASM_P_ZC", "F8VP_ASM_P_ZC", "W4AP_ASM_G4_ZC", "W4AP_ASM_G6D6_ZC", "W4VP_ASM_G4_ZC"]
    for f in os.listdir(hip):
        text = open(os.path.join(hip, f), errors="replace").read()
        if "_asm_loop_lab.h\"" in text and not f.endswith("_lab.h"):
            assert f.endswith("_lab.hip"), f"{f} includes a lab header"


def _is_rec(name: str) -> bool:
    """A placement-recording instantiation: template argument Rec::kRecord (gemm_tile_common.h)."""
    return "3RecE1E" in name


@pytest.mark.parametrize("which", ["asm", "asm_fp8"])
def test_placement_record_only_in_rec_kernels(request, which):
    """The placement record (HW_REG_XCC_ID / HW_REG_HW_ID read, two vector stores by one lane) is in the
    REC instantiations only: the timed kernels are the code they were before it existed."""
    asm = request.getfixturevalue(which)
    names = [n for n in re.findall(r"^(_Z\w*gemm_\w+):", asm, re.M) if "ref_rows" not in n and "fill_" not in n]
    rec = [n for n in names if _is_rec(n)]
    timed = [n for n in names if "3RecE0E" in n]
    assert rec and len(rec) == len(timed) == len(names) // 2, (len(rec), len(timed), len(names))
    for n in names:
        body = asm[asm.index(n + ":"):asm.index(".end_amdhsa_kernel", asm.index(n + ":"))]
        has = "hwreg(HW_REG_XCC_ID" in body
        assert has == _is_rec(n), n
        if _is_rec(n):
            # the record costs no scratch and leaves the pinned accumulators to the asm blocks
            tail = asm[asm.index(n + ":"):]
            assert "scratch_" not in body and re.search(r"ScratchSize: (\d+)", tail).group(1) == "0", n
            if "256x256" in n:      # the asm-pinned families (the small kernels' accumulators are hipcc's)
                _no_compiler_agpr_access(body)
