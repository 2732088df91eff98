#!/usr/bin/env python3
"""Generate the hand-scheduled K-loop of the bf16 256x256 GEMM (native/hip/gemm_bf16_asm_loop.h).

The production w4s kernel's K-tile schedule (v18: 128 MFMA slots per K-tile, fragment reads,
16 LDS-DMA pieces, two barriers) is written as C++ that hipcc schedules; what hipcc adds
around it -- SALU address arithmetic per DMA piece, an ``s_nop 0`` before each piece, lgkmcnt
ladders, register moves at the back-edge -- is the part of the instruction stream the source
cannot control (profiles/r2_sched/README.md). Here the whole K pipeline of one workgroup tile
(prologue DMA of K-tiles 0 and 1, the steady-state loop unrolled over the two LDS buffers, the
two-tile drain) is one ``asm volatile`` block with physical registers:

  a[0:255]   accumulators (acc m*8+n = a[4(m*8+n) : +3], the w4s layout, read by its epilogue)
  v[0:63]    R0 = A fragments a0..a7 (v[0:31]) and B fragments b0..b7 (v[32:63]), k-half 0
  v[64:127]  R1 = the same for k-half 1
  M0         LDS-DMA destination, advanced 4 KiB per piece (piece p of a wave lands at
             buffer + p * 4096 + wid * 1024: A pieces 0-7, B pieces 8-15)

and the schedule is data (SCHEDULES below): in MFMA slot i of a K-tile the gap after MFMA i holds
the ops listed for i. Every gap is kept to <= 2 single-issue instructions (one wave per SIMD: a
16x16x32 bf16 MFMA leaves 8 of its 16 issue cycles, ~4 per instruction; MI355X_MICROARCH.md).
Waits are explicit and counted:
  * lgkmcnt(0) before the "free" barrier: this wave's reads of tile t are done;
  * vmcnt(n) before the "landed" barrier, n = pieces this K-tile has issued so far: tile t+1's 16
    pieces (issued one K-tile earlier) have landed in LDS for this wave, the barrier makes that
    true for all four waves;
  * lgkmcnt(0) at the end of the K-tile: the next tile's k-half-0 fragments are in registers.
The MFMA order, operands and accumulators are those of w4s, so results are bitwise identical to
it (tests/test_gemm_gpu.py checks that).

    python tools/gen_bf16_asm_loop.py               # rewrites both headers in native/hip/
    python tools/gen_bf16_asm_loop.py --out-dir D   # writes them to D (tests/test_gemm_build.py drift check)

Two headers: ``gemm_bf16_asm_loop.h`` carries only the shipped schedules (SHIPPED below, the ones
gemm_bf16.hip dispatches), ``gemm_bf16_asm_loop_lab.h`` every schedule, for the tools-only lab
libraries (which include it before gemm_bf16_kernels.h; it then masks the production header). A
schedule keeps its SC index in both, so production kernel names do not change.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "native", "hip", "gemm_bf16_asm_loop.h")
LAB_OUT = os.path.join(ROOT, "native", "hip", "gemm_bf16_asm_loop_lab.h")
LAB_GUARD = "AMDGO_BF16_ASM_LOOP_LAB"

SLOTS = 128
PIECE_STRIDE = 0x1000


def frag_regs(r: int, isb: bool, x: int) -> str:
    base = 64 * r + (32 if isb else 0) + 4 * x
    return f"v[{base}:{base + 3}]"


def read_order(j: int):
    """Read j of a fragment set in consumption order: a0, b0..b7, a1..a7 -> (isb, index)."""
    if j == 0:
        return False, 0
    if j <= 8:
        return True, j - 1
    return False, j - 8


def mfma(i: int, bout: bool = False, zero_c: bool = False) -> str:
    """MFMA slot i: k-half i >> 6; A-outer (m = s >> 3, n = s & 7: the A fragment stays in srcB for
    8 MFMAs) or B-outer (n = s >> 3, m = s & 7: the B fragment stays in srcA for 8 MFMAs). Each
    accumulator m*8+n gets the same k sequence either way, so the results are identical."""
    r, s = (0, i) if i < 64 else (1, i - 64)
    m, n = (s & 7, s >> 3) if bout else (s >> 3, s & 7)
    acc = m * 8 + n
    c = "0" if zero_c and r == 0 else f"a[{4 * acc}:{4 * acc + 3}]"     # zero_c: a tile's first k-half
    return (f"v_mfma_f32_16x16x32_bf16 a[{4 * acc}:{4 * acc + 3}], {frag_regs(r, True, n)}, "
            f"{frag_regs(r, False, m)}, {c}")


class Schedule:
    """Slot positions of one K-tile (see the module docstring)."""

    def __init__(self, name, r1, w1, b1, dma, m0_lead, w2, b2, r0, vk, w3, bout=False):
        self.name = name
        self.bout = bout        # B-outer MFMA order (see mfma())
        self.r1 = r1            # slot of R1 read j (k-half 1 of tile t), j = 0..15
        self.w1, self.b1 = w1, b1   # lgkmcnt(0) slot, free barrier slot
        self.dma = dma          # slot of DMA piece p (p = 0..15)
        self.m0_lead = m0_lead  # the M0 update for piece p goes this many slots before it (>= 1)
        self.w2, self.b2 = w2, b2   # landing vmcnt slot, landing barrier slot
        self.r0 = r0            # slot of R0 read j (k-half 0 of tile t+1)
        self.vk = vk            # slot of the K-offset add after the last piece
        self.w3 = w3            # lgkmcnt(0) slot (the next tile's R0 landed)

    @property
    def merged(self) -> bool:
        return self.w2 is None

    def issued_before_w2(self) -> int:
        return sum(1 for s in self.dma if s <= self.w2)


def make(name, r1=(0, 1), dma=(19, 5), w2=79, r0=(81, 2), w3=126, vk=None, bout=False, w1_gap=1):
    """A schedule from arithmetic progressions: R1 reads j at r1[0] + j*r1[1] (then lgkmcnt(0) and
    the free barrier right after the last one), DMA piece p at dma[0] + p*dma[1], the landing wait at
    w2 and its barrier at w2 + 1, R0 reads j at r0[0] + j*r0[1].
    w2 = None: ONE barrier per K-tile -- the free wait becomes vmcnt(0) lgkmcnt(0), so the barrier
    after it also publishes tile t+1 (DMA'd during the previous K-tile) and R0 of tile t+1 may be
    read any time after MFMA 63."""
    r1s = [r1[0] + j * r1[1] for j in range(16)]
    w1 = r1s[-1] + w1_gap                  # lgkmcnt(0): w1_gap MFMAs after the last R1 read
    ds = [dma[0] + p * dma[1] for p in range(16)]
    r0s = [r0[0] + j * r0[1] for j in range(16)]
    sc = Schedule(name, r1=r1s, w1=w1, b1=w1 + 1, dma=ds, m0_lead=1, w2=w2, b2=None if w2 is None else w2 + 1, r0=r0s,
                  vk=vk if vk is not None else ds[-1] + 2, w3=w3, bout=bout)
    validate(sc)
    return sc


def validate(sc: "Schedule") -> None:
    """The protocol's ordering constraints (module docstring) and <= 2 fillers per gap."""
    land = [] if sc.merged else [sc.w2, sc.b2]
    assert all(0 <= x < SLOTS for x in sc.r1 + sc.dma + sc.r0 + [sc.w1, sc.b1, sc.vk, sc.w3] + land), sc.name
    assert sc.w1 > max(sc.r1) and sc.w1 < 64 and sc.b1 > sc.w1, sc.name           # R1 in before MFMA 64
    assert min(sc.dma) - sc.m0_lead >= 0 and min(sc.dma) > sc.b1, sc.name          # DMA after the free barrier
    assert min(sc.r0) >= 64, sc.name                                                # R0 regs dead after MFMA 63
    assert sc.merged or (sc.b2 > sc.w2 and min(sc.r0) > sc.b2), sc.name
    assert max(sc.r0) < sc.w3 < SLOTS and sc.vk > max(sc.dma), sc.name
    load = {i: 0 for i in range(SLOTS)}
    for x in sc.r1 + sc.r0 + sc.dma + [d - sc.m0_lead for d in sc.dma] + [sc.w1, sc.b1, sc.vk, sc.w3] + land:
        load[x] += 1
    assert max(load.values()) <= 2, (sc.name, {k: v for k, v in load.items() if v > 2})


SCHEDULES = {
    # v18's placement (the production w4s kernel): R1 burst at slots 0-15, barrier at 17, DMA every
    # 5th slot from 19, landing barrier at 80, R0 reads every 2nd slot from 81.
    "v18": make("v18"),
    # R1 reads every other slot (half the LDS read burst), DMA from slot 35 every 4th
    "spread": make("spread", r1=(0, 2), dma=(35, 4), w2=99, r0=(101, 1)),
    # DMA pieces early and dense after the free barrier (more landing time), R0 reads late
    "early": make("early", dma=(18, 3), w2=68, r0=(71, 3)),
    "spread3": make("spread3", r1=(0, 3), dma=(48, 4), w2=100, r0=(102, 1)),
    "spread_d5": make("spread_d5", r1=(0, 2), dma=(34, 5), w2=96, r0=(98, 1)),
    "v18_r1": make("v18_r1", r0=(81, 1)),
    "v18_d4": make("v18_d4", dma=(19, 4), w2=80, r0=(82, 2)),
    "late_land": make("late_land", dma=(18, 3), w2=100, r0=(102, 1)),
    "v18_d6": make("v18_d6", dma=(19, 6), w2=98, r0=(100, 1)),
    "v18_d6b": make("v18_d6b", dma=(19, 6), w2=80, r0=(82, 2)),
    "v18_d5_late": make("v18_d5_late", w2=96, r0=(98, 1)),
    # the same placements with the B fragment held in srcA across 8 MFMAs (hipBLASLt's order)
    "v18_d6b_bout": make("v18_d6b_bout", dma=(19, 6), w2=80, r0=(82, 2), bout=True),
    "v18_d5_late_bout": make("v18_d5_late_bout", w2=96, r0=(98, 1), bout=True),
    # the R1 reads' lgkmcnt(0) a few MFMAs after the last read (the LDS latency under the read
    # burst of all four waves), then the free barrier and the DMA
    "g4": make("g4", w1_gap=4, dma=(22, 5), w2=98, r0=(100, 1)),
    "g6": make("g6", w1_gap=6, dma=(24, 5), w2=100, r0=(102, 1)),
    "g8": make("g8", w1_gap=8, dma=(26, 5), w2=102, r0=(104, 1)),
    "sp2g6": make("sp2g6", r1=(0, 2), w1_gap=6, dma=(39, 4), w2=100, r0=(102, 1)),
    "g6d6": make("g6d6", w1_gap=6, dma=(24, 6), w2=86, r0=(88, 2)),
    "g4d6": make("g4d6", w1_gap=4, dma=(22, 6), w2=86, r0=(88, 2)),
    "g2d6": make("g2d6", w1_gap=2, dma=(20, 6), w2=84, r0=(86, 2)),
    "sp2g4d5": make("sp2g4d5", r1=(0, 2), w1_gap=4, dma=(37, 5), w2=100, r0=(102, 1)),
    # one barrier per K-tile (w2=None): the landing of tile t+1 is published by the free barrier
    "m4": make("m4", w1_gap=4, dma=(22, 5), w2=None, r0=(100, 1)),
    "m4d4": make("m4d4", w1_gap=4, dma=(22, 4), w2=None, r0=(88, 1)),
    "m4d3": make("m4d3", w1_gap=4, dma=(22, 3), w2=None, r0=(72, 1)),
    "m6d4": make("m6d4", w1_gap=6, dma=(24, 4), w2=None, r0=(90, 1)),
}


# schedules the persistent kernel is generated for (its SC index = position here)
PERSISTENT = ["v18", "v18_d6b", "v18_d5_late", "v18_d6b_bout", "v18_d5_late_bout", "g4", "g6", "g8", "sp2g6",
              "g6d6", "g4d6", "g2d6", "sp2g4d5", "m4", "m4d4", "m4d3", "m6d4", "g4_rw", "g6d6_rw", "g4_zc",
              "g6d6_zc"]
# a name ending in _zc: kloop_persistent_zc (first K-tile with src C = 0; frame EPI 8)
# a name ending in _rw: that schedule in kloop_persistent_rw (relaxed first landing wait)


def body(sc: Schedule, cur: int, dma: bool, nx: bool, nxt_tile: bool = False, w2_extra: int = 0,
         extra: Dict[int, List[str]] = None, zero_c: bool = False) -> List[str]:
    """One K-tile: MFMAs on tile t (buffer ``cur``), R1 reads from ``cur``, DMA of tile t+2 into
    ``cur``, R0 reads of tile t+1 from the other buffer. ``nxt_tile``: the DMA fetches the next
    output tile's K-tile instead (persistent kernel drain: operands nA / nB / nvoff / nkstep)."""
    rA, rB, voff, kstep = ("%[nA]", "%[nB]", "%[nvoff]", "%[nkstep]") if nxt_tile else \
        ("%[rA]", "%[rB]", "%[voff]", "%[kstep]")
    nxt = 1 - cur
    gap: Dict[int, List[str]] = {i: [] for i in range(SLOTS)}
    for j, s in enumerate(sc.r1):
        isb, x = read_order(j)
        gap[s].append(f"ds_read_b128 {frag_regs(1, isb, x)}, %[{'rb' if isb else 'ra'}{cur}1] offset:{x * 2048}")
    gap[sc.w1].append("s_waitcnt vmcnt(0) lgkmcnt(0)" if sc.merged else "s_waitcnt lgkmcnt(0)")
    gap[sc.b1].append("s_barrier")
    if dma:
        for p, s in enumerate(sc.dma):
            lead = s - sc.m0_lead
            gap[lead].append(f"s_mov_b32 m0, %[m0b{cur}]" if p == 0 else f"s_add_u32 m0, m0, {PIECE_STRIDE:#x}")
            gap[s].append(f"buffer_load_dwordx4 {voff}, {rB if p >= 8 else rA}, %[s{p & 7}] offen lds")
        gap[sc.vk].append(f"v_add_u32_e32 {voff}, {kstep}, {voff}")
    if nx:
        if not sc.merged:
            n = (sc.issued_before_w2() if dma else 0) + w2_extra
            gap[sc.w2].append(f"s_waitcnt vmcnt({n})")
            gap[sc.b2].append("s_barrier")
        for j, s in enumerate(sc.r0):
            isb, x = read_order(j)
            gap[s].append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}{nxt}0] offset:{x * 2048}")
        gap[sc.w3].append("s_waitcnt lgkmcnt(0)")
    for i, ops in (extra or {}).items():
        gap[i] += ops
    out = []
    for i in range(SLOTS):
        out.append(mfma(i, sc.bout, zero_c))
        out += gap[i]
    return out


def prologue() -> List[str]:
    """DMA K-tiles 0 and 1 into buffers 0 and 1, wait for tile 0, read its k-half 0."""
    out = ["s_nop 4"]                 # SGPR operands fresh from readfirstlane -> buffer descriptor use
    for buf in (0, 1):
        for p in range(16):
            out.append(f"s_mov_b32 m0, %[m0b{buf}]" if p == 0 else f"s_add_u32 m0, m0, {PIECE_STRIDE:#x}")
            out.append("s_nop 0")     # M0 write -> LDS-DMA
            out.append(f"buffer_load_dwordx4 %[voff], %[{'rB' if p >= 8 else 'rA'}], %[s{p & 7}] offen lds")
        out.append("v_add_u32_e32 %[voff], %[kstep], %[voff]")
    out += ["s_waitcnt vmcnt(16)", "s_barrier"]
    for j in range(16):
        isb, x = read_order(j)
        out.append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def kloop(sc: Schedule) -> List[str]:
    out = prologue()
    out.append(".Lw4a_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4a_loop_%="]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    return out


def kloop_persistent_rw(sc: Schedule, stores: int = 32) -> List[str]:
    """kloop_persistent() for the staged epilogue with a relaxed first landing wait ("_rw"): the
    previous tile's epilogue issued ``stores`` C stores after waiting for this tile's K-tiles 0 and 1
    (vmcnt(0)), so the first K-tile's landing wait (K-tile 1) skips them -- vmcnt(16 + stores) -- and
    the stores have until the second K-tile's landing wait to complete. The first tile of a workgroup
    waits for both prologue K-tiles (vmcnt(0)), so the relaxed count is exact there too."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4rw_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier" and not x.startswith("s_waitcnt vmcnt")]
    out.append("s_waitcnt vmcnt(0)")
    out.append(".Lw4rw_entry_%=:")
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    out += body(sc, 0, dma=True, nx=True, w2_extra=stores)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4rw_drain_%="]
    out.append(".Lw4rw_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4rw_loop_%="]
    out.append(".Lw4rw_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4rw_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lw4rw_done_%=", ".Lw4rw_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lw4rw_done_%=:")
    return out


# Deferred C stores (frame EPI 7, gemm_w4ap.h): the staged epilogue stores only the first quarter of
# the tile (8 stores per wave); the other 24 go out from the next tile's first 6 K-tiles, 4 at the
# start of each (before its DMA pieces, so the next landing wait but one is the first to need them):
# 16 from VGPRs the epilogue left in %[h0..h15], 8 from the wave's staging LDS, read into v[240:255]
# at the end of the K-tile before. Knock-outs priced the burst: storing a quarter of C at the tile
# boundary costs 0.2 %, all of it 1.5 % (bf16 8192^3; fp8 0.4 % / 3.3 %; profiles/r3_s2/).
DS_PEEL = 6                          # K-tiles carrying deferred stores (3 loop pairs)
DS_STORE_SLOTS = (1, 3, 5, 7)        # store slots in a carrying K-tile (add of %[vcur] one slot later)
DS_LDS_SLOTS = (116, 117, 118, 119)  # ds_reads for the next K-tile's LDS-held stores (w3 covers them)
DS_EPI_STORES = 8                    # stores the staged epilogue itself issues (pass 0)


def ds_ops(j: int, store_slots=DS_STORE_SLOTS, lds_slots=DS_LDS_SLOTS) -> Dict[int, List[str]]:
    """Deferred-store ops of carrying K-tile j (0-based within the tile)."""
    ops: Dict[int, List[str]] = {}
    for n, sl in enumerate(store_slots):
        item = 4 * j + n
        data = f"%[h{item}]" if item < 16 else f"v[{240 + 4 * n}:{243 + 4 * n}]"
        ops.setdefault(sl, []).append(f"global_store_dwordx4 %[vcur], {data}, %[sCp] nt")
        ops.setdefault(sl + 1, []).append("v_add_u32_e32 %[vcur], %[s8N], %[vcur]")
    if j + 1 < DS_PEEL and 4 * (j + 1) >= 16:        # the next K-tile stores from LDS: read it now
        for n, sl in enumerate(lds_slots):
            k = 4 * (j + 1) - 16 + n
            ops.setdefault(sl, []).append(f"ds_read_b128 v[{240 + 4 * n}:{243 + 4 * n}], %[stgl] offset:{k * 1024}")
    return ops


def kloop_persistent_ds(sc: Schedule) -> List[str]:
    """kloop_persistent() with the deferred stores in the first DS_PEEL K-tiles (host: >= 8 K-tiles).
    Landing waits: the first K-tile's skips the epilogue's 8 stores and its own 4 (the first tile of a
    workgroup waits for both prologue K-tiles instead), every carrying K-tile's skips its own 4."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4ds_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier" and not x.startswith("s_waitcnt vmcnt")]
    out.append("s_waitcnt vmcnt(0)")
    out.append(".Lw4ds_entry_%=:")
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    for j in range(DS_PEEL):
        extra = len(DS_STORE_SLOTS) + (DS_EPI_STORES if j == 0 else 0)
        out += body(sc, j % 2, dma=True, nx=True, w2_extra=extra, extra=ds_ops(j))
    out += [f"s_sub_u32 %[cnt], %[cnt], {DS_PEEL // 2}", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4ds_drain_%="]
    out.append(".Lw4ds_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4ds_loop_%="]
    out.append(".Lw4ds_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4ds_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lw4ds_done_%=", ".Lw4ds_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lw4ds_done_%=:")
    assert sum(ln.startswith("global_store") for ln in out) == 24
    return out


DS = ["g4"]


def kloop_persistent_zc(sc: Schedule) -> List[str]:
    """kloop_persistent() whose first K-tile issues its k-half-0 MFMAs with src C = 0 (frame EPI 8): the
    epilogue reads the accumulators without writing 256 zeros back, and nothing zeroes them at start."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4zc_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier"]
    out.append(".Lw4zc_entry_%=:")
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    out += body(sc, 0, dma=True, nx=True, zero_c=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4zc_drain_%="]
    out.append(".Lw4zc_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4zc_loop_%="]
    out.append(".Lw4zc_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4zc_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lw4zc_done_%=", ".Lw4zc_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lw4zc_done_%=:")
    return out


def kloop_persistent(sc: Schedule) -> List[str]:
    """The K pipeline of one output tile of the persistent kernel (w4ap). Uniform branches on
    %[flags] bit 0 (this workgroup's first tile: issue K-tiles 0 and 1 here; later tiles had them
    issued by the previous tile's drain and retired by its epilogue) and bit 1 (a next tile: drain
    with its K-tiles 0 and 1 DMA'd into the buffers as they free up, else the plain drain)."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4ap_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier"]
    out.append(".Lw4ap_entry_%=:")
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(f"ds_read_b128 {frag_regs(0, isb, x)}, %[{'rb' if isb else 'ra'}00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    out.append(".Lw4ap_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4ap_loop_%="]
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4ap_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lw4ap_done_%=", ".Lw4ap_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lw4ap_done_%=:")
    return out


# ---------------------------------------------------------------------------------------------------
# Fused epilogue (w4ap EPI=2, "EF"): the C tile leaves through the last K-tile's MFMA shadow.
#
# The staged epilogue (gemm_w4ap.h, EPI=0) runs after the K pipeline: 256 accvgpr reads, 256 zeroing
# writes, an LDS round trip and 32 row stores per wave, none of it under an MFMA -- the lab prices it
# at 4-5 % of an 8192^3 GEMM (profiles/r3_s2). Here:
#   * B fragment x reads Bt rows 32(x>>1) + 4(x&1) + 8(rho>>2) + (rho&3) for fragment row rho (even /
#     odd fragments through their own lane offsets rbe / rbo), so a lane of accumulator pair
#     (m, 2p), (m, 2p+1) holds 8 consecutive C columns 32p + 8g .. +7 of row 16m + (lane & 15):
#     one 16-byte global store per pair, straight from registers;
#   * the last K-tile runs its MFMAs so the finals (k-half 1) spread over slots 20..127 -- k-half 0
#     of accumulators 0..19 first, then k-half 1 interleaved with the rest of k-half 0 (each
#     accumulator still gets k-half 0 before k-half 1: bitwise the same sums) -- and each final is
#     followed (>= 3 MFMAs later: the XDL-write -> VALU-read distance) by 4 v_accvgpr_read, 2
#     v_cvt_pk_bf16_f32 and, per pair, one global_store_dwordx4 in the gaps;
#   * the next tile's first K-tile issues its k-half-0 MFMAs with src C = 0 (no zeroing writes);
#   * waits: the entry waits vmcnt(16 + stores) (K-tile 0 landed: younger are K-tile 1's 16 pieces and
#     this tile's stores), the first K-tile's landing wait counts the stores issued after the last
#     K-tile-1 piece, so stores have the rest of that K-tile to complete.
# Physical temps: v[224:239] accumulator reads (4 sets), v[240:255] packed pairs (4 sets).
EF_T, EF_NT = 224, 4
EF_P, EF_NP = 240, 4
EF_FIRST_KH1 = 20          # first slot of a k-half-1 MFMA in the last K-tile (R1 landed at w1 <= 19)
EF_HAZ = 3                 # accvgpr reads of an accumulator >= this many MFMAs after its final


def b_read(r: int, x: int, buf: int) -> str:
    """EF: B fragment x of k-half r from buffer buf through the permuted lane offsets."""
    par = "e" if x % 2 == 0 else "o"
    return f"ds_read_b128 {frag_regs(r, True, x)}, %[rb{par}{buf}{r}] offset:{(x >> 1) * 4096}"


def ef_last_order() -> List[tuple]:
    """(k-half, acc) per slot of the last K-tile: finals spread over slots 20..127."""
    order = [(0, i) for i in range(EF_FIRST_KH1)]
    n0, n1 = EF_FIRST_KH1, 0
    span = SLOTS - EF_FIRST_KH1
    for s in range(EF_FIRST_KH1, SLOTS):
        want1 = -(-(s - EF_FIRST_KH1 + 1) * 64 // span)        # ceil: k-half-1 MFMAs due by slot s
        if (n1 < want1 and n1 < n0) or n0 == 64:
            order.append((1, n1))
            n1 += 1
        else:
            order.append((0, n0))
            n0 += 1
    assert n0 == 64 and n1 == 64 and len(order) == SLOTS
    first = {}
    for s, (kh, acc) in enumerate(order):
        if kh == 0:
            first[acc] = s
        else:
            assert first[acc] < s, acc
    return order


def mfma_op(kh: int, acc: int, zero_c: bool = False) -> str:
    m, n = acc >> 3, acc & 7
    c = "0" if zero_c else f"a[{4 * acc}:{4 * acc + 3}]"
    return f"v_mfma_f32_16x16x32_bf16 a[{4 * acc}:{4 * acc + 3}], {frag_regs(kh, True, n)}, {frag_regs(kh, False, m)}, {c}"


def ef_epilogue(order: List[tuple], load: Dict[int, int], cap: int):
    """Place the epilogue of the last K-tile: returns ({slot: [ops]}, tail ops). Greedy: each op goes
    to the earliest gap at or after it is ready with fewer than ``cap`` instructions (existing fillers
    counted by ``load``); what does not fit before the last MFMA runs after it."""
    final = {acc: s for s, (kh, acc) in enumerate(order) if kh == 1}
    gaps: Dict[int, List[str]] = {i: [] for i in range(SLOTS)}
    tail: List[str] = []
    used = dict(load)
    where = {}                                   # op id -> position (slot, or SLOTS + tail index)

    def put(op: str, ready: int, key) -> int:
        for s in range(max(ready, 0), SLOTS):
            if used.get(s, 0) < cap:
                gaps[s].append(op)
                used[s] = used.get(s, 0) + 1
                where[key] = s
                return s
        tail.append(op)
        where[key] = SLOTS + len(tail)
        return SLOTS + len(tail)

    accs = sorted(final, key=lambda a: final[a])
    pair_done = {}
    tset = 0
    pset_of = {}
    npairs = 0
    last_store_pos = {}                          # P set -> position of its last store
    last_cvt_pos = {}                            # T set -> position of its last cvt
    for acc in accs:
        t = EF_T + 4 * (tset % EF_NT)
        ready = max(final[acc] + EF_HAZ, last_cvt_pos.get(tset % EF_NT, -1))
        for k in range(4):
            ready = put(f"v_accvgpr_read_b32 v{t + k}, a{4 * acc + k}", ready, ("r", acc, k))
        pair = acc >> 1
        if pair not in pset_of:
            pset_of[pair] = npairs % EF_NP
            npairs += 1
        ps = pset_of[pair]
        pbase = EF_P + 4 * ps + 2 * (acc & 1)
        ready = max(ready, last_store_pos.get(ps, -1))
        for k in range(2):
            ready = put(f"v_cvt_pk_bf16_f32 v{pbase + k}, v{t + 2 * k}, v{t + 2 * k + 1}", ready, ("c", acc, k))
        last_cvt_pos[tset % EF_NT] = ready
        tset += 1
        pair_done.setdefault(pair, []).append(ready)
        if len(pair_done[pair]) == 2:
            m, p = pair >> 2, pair & 3
            pos = put(f"global_store_dwordx4 %[cv{m}], v[{EF_P + 4 * ps}:{EF_P + 4 * ps + 3}], %[sC] offset:{64 * p}",
                      max(pair_done[pair]), ("s", pair))
            last_store_pos[ps] = pos + 1             # the next cvt into this set at least one op later
    return gaps, tail


def ef_check(lines: List[str]) -> None:
    """Static audit of the EF last K-tile text: every accumulator read >= EF_HAZ MFMAs (or a
    16-wait-state pad) after its final MFMA, read -> cvt -> store register flow without a clobber
    in between, every pair stored exactly once."""
    import re
    mf = 0
    final_at = {}
    pad = {}
    treg = {}          # v reg -> (acc, k) last written by an accvgpr read
    pword = {}         # v reg -> acc of its last cvt
    stored = set()
    for ln in lines:
        if ln.startswith("v_mfma"):
            mf += 1
            mm = re.match(r"v_mfma_f32_16x16x32_bf16 a\[(\d+):\d+\], v\[(\d+):", ln)
            acc = int(mm.group(1)) // 4
            kh = 1 if int(mm.group(2)) >= 64 else 0
            if kh == 1:
                final_at[acc] = mf
            continue
        if ln.startswith("s_nop"):
            pad[mf] = pad.get(mf, 0) + int(ln.split()[1]) + 1
            continue
        mm = re.match(r"v_accvgpr_read_b32 v(\d+), a(\d+)", ln)
        if mm:
            acc = int(mm.group(2)) // 4
            assert acc in final_at, ("read before final", acc)
            dist = mf - final_at[acc]
            assert dist >= EF_HAZ or pad.get(mf, 0) >= 16, ("hazard", acc, dist)
            treg[int(mm.group(1))] = (acc, int(mm.group(2)) % 4)
            continue
        mm = re.match(r"v_cvt_pk_bf16_f32 v(\d+), v(\d+), v(\d+)", ln)
        if mm:
            d, s0, s1 = (int(x) for x in mm.groups())
            (a0, k0), (a1, k1) = treg[s0], treg[s1]
            assert a0 == a1 and k1 == k0 + 1 and k0 % 2 == 0, ln
            assert (d - EF_P) % 4 == 2 * (a0 & 1) + k0 // 2, ln
            pword[d] = a0
            continue
        mm = re.match(r"global_store_dwordx4 %\[cv(\d)\], v\[(\d+):\d+\], %\[sC\] offset:(\d+)", ln)
        if mm:
            m, base, off = int(mm.group(1)), int(mm.group(2)), int(mm.group(3))
            accs = [pword[base + k] for k in range(4)]
            p = off // 64
            want = [m * 8 + 2 * p, m * 8 + 2 * p, m * 8 + 2 * p + 1, m * 8 + 2 * p + 1]
            assert accs == want, (ln, accs, want)
            stored.add((m, p))
    assert len(stored) == 32, len(stored)


def body_ef(sc: Schedule, cur: int, dma: bool, nx: bool, nxt_tile: bool = False, zero_c: bool = False,
            w2_extra: int = 0, last: bool = False, cap: int = 5):
    """body() for the EF kernel: permuted B reads, optional src-C-zero first K-tile, extra landing-wait
    count, and (last) the fused epilogue with the spread-final MFMA order. Returns (lines, stores issued
    after the last DMA piece)."""
    assert not sc.bout
    rA, rB, voff, kstep = ("%[nA]", "%[nB]", "%[nvoff]", "%[nkstep]") if nxt_tile else \
        ("%[rA]", "%[rB]", "%[voff]", "%[kstep]")
    nxt = 1 - cur
    gap: Dict[int, List[str]] = {i: [] for i in range(SLOTS)}
    for j, s in enumerate(sc.r1):
        isb, x = read_order(j)
        gap[s].append(b_read(1, x, cur) if isb else f"ds_read_b128 {frag_regs(1, False, x)}, %[ra{cur}1] offset:{x * 2048}")
    gap[sc.w1].append("s_waitcnt vmcnt(0) lgkmcnt(0)" if sc.merged else "s_waitcnt lgkmcnt(0)")
    gap[sc.b1].append("s_barrier")
    if dma:
        for p, s in enumerate(sc.dma):
            lead = s - sc.m0_lead
            gap[lead].append(f"s_mov_b32 m0, %[m0b{cur}]" if p == 0 else f"s_add_u32 m0, m0, {PIECE_STRIDE:#x}")
            gap[s].append(f"buffer_load_dwordx4 {voff}, {rB if p >= 8 else rA}, %[s{p & 7}] offen lds")
        gap[sc.vk].append(f"v_add_u32_e32 {voff}, {kstep}, {voff}")
    if nx:
        assert not last
        if not sc.merged:
            n = (sc.issued_before_w2() if dma else 0) + w2_extra
            gap[sc.w2].append(f"s_waitcnt vmcnt({n})")
            gap[sc.b2].append("s_barrier")
        for j, s in enumerate(sc.r0):
            isb, x = read_order(j)
            gap[s].append(b_read(0, x, nxt) if isb else f"ds_read_b128 {frag_regs(0, False, x)}, %[ra{nxt}0] offset:{x * 2048}")
        gap[sc.w3].append("s_waitcnt lgkmcnt(0)")
    if last:
        order = ef_last_order()
        load = {i: len(gap[i]) for i in range(SLOTS)}
        egap, tail = ef_epilogue(order, load, cap)
        for i in range(SLOTS):
            gap[i] += egap[i]
    else:
        order = [(i >> 6, i & 63) for i in range(SLOTS)]
        tail = []
    out = []
    for i in range(SLOTS):
        kh, acc = order[i]
        out.append(mfma_op(kh, acc, zero_c and kh == 0))
        out += gap[i]
    if tail:
        out += ["s_nop 7", "s_nop 7"] + tail
    late = 0
    if last and dma:
        seen_last_piece = False
        for ln in out:
            if ln.startswith("buffer_load"):
                seen_last_piece = True
                late = 0
            elif ln.startswith("global_store") and seen_last_piece:
                late += 1
    elif last:
        late = sum(ln.startswith("global_store") for ln in out)
    return out, late


def kloop_persistent_ef(sc: Schedule, cap: int = 5) -> List[str]:
    """kloop_persistent() with the fused epilogue (EPI=2). %[flags] bit 0: first tile of this
    workgroup (prologue DMA, then vmcnt(0): nothing older is in flight); bit 1: a next tile (the drain
    DMAs its K-tiles 0 and 1)."""
    last_nx, late_nx = body_ef(sc, 1, dma=True, nx=False, nxt_tile=True, last=True, cap=cap)
    last_no, late_no = body_ef(sc, 1, dma=False, nx=False, last=True, cap=cap)
    ef_check(last_nx)
    ef_check(last_no)
    stores = sum(ln.startswith("global_store") for ln in last_nx)
    assert stores == 32 and 16 + stores <= 63
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4ef_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier" and not x.startswith("s_waitcnt vmcnt")]
    out.append("s_waitcnt vmcnt(0)")
    out.append(".Lw4ef_entry_%=:")
    out.append(f"s_waitcnt vmcnt({16 + stores})")        # K-tile 0 landed (K-tile 1 + the stores younger)
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(b_read(0, x, 0) if isb else f"ds_read_b128 {frag_regs(0, False, x)}, %[ra00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    out += body_ef(sc, 0, dma=True, nx=True, zero_c=True, w2_extra=late_nx)[0]
    out += body_ef(sc, 1, dma=True, nx=True)[0]
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4ef_drain_%="]
    out.append(".Lw4ef_loop_%=:")
    out += body_ef(sc, 0, dma=True, nx=True)[0]
    out += body_ef(sc, 1, dma=True, nx=True)[0]
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4ef_loop_%="]
    out.append(".Lw4ef_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4ef_last_%="]
    out += body_ef(sc, 0, dma=True, nx=True, nxt_tile=True)[0]
    out += last_nx
    out += ["s_branch .Lw4ef_done_%=", ".Lw4ef_last_%=:"]
    out += body_ef(sc, 0, dma=False, nx=True)[0]
    out += last_no
    out.append(".Lw4ef_done_%=:")
    return out


def kloop_persistent_efp(sc: Schedule) -> List[str]:
    """The EF fragment layout (permuted B reads: a lane of an accumulator pair holds 8 consecutive C
    columns) with the standard K-tile bodies and src C = 0 in each tile's first K-tile; the C tile
    is stored after the block straight from the accumulators, no LDS staging (frame EPI 9)."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lw4efp_entry_%="]
    out += [x for x in prologue() if not x.startswith("ds_read") and x != "s_waitcnt lgkmcnt(0)"
            and x != "s_barrier"]
    out.append(".Lw4efp_entry_%=:")
    out.append("s_barrier")
    for j in range(16):
        isb, x = read_order(j)
        out.append(b_read(0, x, 0) if isb else f"ds_read_b128 {frag_regs(0, False, x)}, %[ra00] offset:{x * 2048}")
    out.append("s_waitcnt lgkmcnt(0)")
    out += body_ef(sc, 0, dma=True, nx=True, zero_c=True)[0]
    out += body_ef(sc, 1, dma=True, nx=True)[0]
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4efp_drain_%="]
    out.append(".Lw4efp_loop_%=:")
    out += body_ef(sc, 0, dma=True, nx=True)[0]
    out += body_ef(sc, 1, dma=True, nx=True)[0]
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lw4efp_loop_%="]
    out.append(".Lw4efp_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lw4efp_last_%="]
    out += body_ef(sc, 0, dma=True, nx=True, nxt_tile=True)[0]
    out += body_ef(sc, 1, dma=True, nx=False, nxt_tile=True)[0]
    out += ["s_branch .Lw4efp_done_%=", ".Lw4efp_last_%=:"]
    out += body_ef(sc, 0, dma=False, nx=True)[0]
    out += body_ef(sc, 1, dma=False, nx=False)[0]
    out.append(".Lw4efp_done_%=:")
    assert not any(ln.startswith("global_store") for ln in out)
    return out


# schedules the fused-epilogue kernel is generated for (index = EF SC)
EF = ["g4", "g6d6", "g4_nt", "g4_post"]   # _post: kloop_persistent_efp (frame EPI 9)
# a name ending in _nt: the same schedule with nontemporal C stores (global_store ... nt)


# ---------------------------------------------------------------------------------------------------
# VP DMA form (frame DM >= 1, gemm_w4ap.h): piece p's whole lane offset (row block, row, chunk) is its
# own VGPR %[vp<p>], fixed for the kernel, and the K byte offset of the DMA'd K-tile is one SGPR
# (%[koff], %[nkoff] for the next tile) used as the soffset: one SALU add per K-tile instead of a VALU
# add, no per-piece row-block SGPRs, and A and B pieces may use different row maps -- DM = 2 reads each
# A-panel DMA instruction's 8 rows 32 apart (PA: K not a power of two, see gemm_bf16.hip v47).
VP = ["g4", "g6d6", "g4_zc"]   # _zc: from kloop_persistent_zc (frame EPI 8)


def to_vp(lines: List[str]) -> List[str]:
    out = []
    for ln in lines:
        m = re.match(r"buffer_load_dwordx4 %\[(n?)voff\], %\[([rn])([AB])\], %\[s(\d)\] offen lds", ln)
        if m:
            piece = int(m.group(4)) + (8 if m.group(3) == "B" else 0)
            assert (m.group(1) == "n") == (m.group(2) == "n"), ln
            out.append(f"buffer_load_dwordx4 %[vp{piece}], %[{m.group(2)}{m.group(3)}], %[{m.group(1)}koff] offen lds")
            continue
        m = re.match(r"v_add_u32_e32 %\[(n?)voff\], %\[(n?)kstep\], %\[(n?)voff\]", ln)
        if m:
            n = m.group(1)
            out.append(f"s_add_u32 %[{n}koff], %[{n}koff], %[{n}kstep]")
            continue
        assert "voff" not in ln and "%[s" not in ln, ln
        out.append(ln)
    return out


def audit(lines: List[str]) -> Dict[str, int]:
    gaps, cur, worst = [], 0, 0
    for ln in lines:
        if ln.startswith("v_mfma"):
            gaps.append(cur)
            cur = 0
        elif not ln.startswith("."):
            cur += 1
    return {"max_fillers_per_gap": max(gaps[1:]), "mfmas": sum(ln.startswith("v_mfma") for ln in lines)}


def render() -> str:
    parts = ["// GENERATED by tools/gen_bf16_asm_loop.py -- do not edit by hand.",
             "// LAB header: every schedule of the hand-scheduled K pipeline of gemm_bf16_256x256_w4a / w4ap",
             "// (gemm_bf16_kernels.h, gemm_w4ap.h), one asm string per schedule. Only the tools-only lab",
             "// libraries include it (before gemm_bf16_kernels.h); production builds gemm_bf16_asm_loop.h.",
             "#pragma once", f"#define {LAB_GUARD} 1", ""]
    sel = []
    for idx, (name, sc) in enumerate(SCHEDULES.items()):
        sel.append(f"if constexpr (SC == {idx}) W4A_LOOP(W4A_ASM_{name.upper()});")
    parts.append("// schedule index -> asm text (SC template parameter of gemm_bf16_256x256_w4a)")
    parts.append("#define W4A_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(sel))
    parts.append("")
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(SCHEDULES)))
    parts.append("")
    psel = [f"if constexpr (SC == {i}) W4AP_LOOP(W4AP_ASM_{n.upper()});" for i, n in enumerate(PERSISTENT)]
    parts.append("// persistent kernel (gemm_bf16_256x256_w4ap): schedule index -> asm text")
    parts.append("#define W4AP_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(psel))
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(PERSISTENT)))
    parts.append("// by name (the production dispatch refers to schedules this way)")
    for i, n in enumerate(PERSISTENT):
        parts.append(f"#define W4AP_SC_{n.upper()} {i}")
    parts.append("")
    esel = [f"if constexpr (SC == {i}) W4EF_LOOP(W4EF_ASM_{n.upper()});" for i, n in enumerate(EF)]
    parts.append("// fused-epilogue persistent kernel (w4ap EPI=2): schedule index -> asm text")
    parts.append("#define W4EF_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(esel))
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(EF)))
    for i, n in enumerate(EF):
        parts.append(f"#define W4EF_SC_{n.upper()} {i}")
    parts.append("")
    for name in EF:
        lines = (kloop_persistent_efp(SCHEDULES[name.split("_")[0]]) if name.endswith("_post") else
                 kloop_persistent_ef(SCHEDULES[name.split("_")[0]]))
        if name.endswith("_nt"):
            lines = [ln + " nt" if ln.startswith("global_store") else ln for ln in lines]
        parts.append(f"#define W4EF_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    dsel = [f"if constexpr (SC == {i}) W4DS_LOOP(W4DS_ASM_{n.upper()});" for i, n in enumerate(DS)]
    parts.append("// deferred-store form (frame EPI 7): schedule index -> asm text (W4DS_LOOP)")
    parts.append("#define W4DS_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(dsel))
    for i, n in enumerate(DS):
        parts.append(f"#define W4DS_SC_{n.upper()} {i}")
    parts.append("")
    for name in DS:
        lines = kloop_persistent_ds(SCHEDULES[name])
        parts.append(f"#define W4DS_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    vsel = [f"if constexpr (SC == {i}) W4VP_LOOP(W4VP_ASM_{n.upper()});" for i, n in enumerate(VP)]
    parts.append("// VP DMA form (frame DM >= 1): schedule index -> asm text (W4VP_LOOP)")
    parts.append("#define W4VP_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(vsel))
    for i, n in enumerate(VP):
        parts.append(f"#define W4VP_SC_{n.upper()} {i}")
    parts.append("")
    for name in VP:
        lines = vp_lines(name)
        parts.append(f"#define W4VP_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    for name in PERSISTENT:
        lines = ap_lines(name)
        parts.append(f"#define W4AP_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    for name, sc in SCHEDULES.items():
        lines = kloop(sc)
        a = audit(lines)
        parts.append(f"// {name}: {a['mfmas']} MFMAs per tile pipeline text, <= {a['max_fillers_per_gap']} "
                     f"instructions per MFMA gap")
        parts.append(f"#define W4A_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    return "\n".join(parts)


# The schedules gemm_bf16.hip dispatches: v50 / v51 W4AP g4_zc, v52 W4AP g6d6_zc, v53 / v54 W4VP g4_zc.
SHIPPED = {"W4AP": ["g4_zc", "g6d6_zc"], "W4VP": ["g4_zc"]}


def ap_lines(name: str) -> List[str]:
    return (kloop_persistent_rw(SCHEDULES[name[:-3]]) if name.endswith("_rw") else
            kloop_persistent_zc(SCHEDULES[name[:-3]]) if name.endswith("_zc") else kloop_persistent(SCHEDULES[name]))


def vp_lines(name: str) -> List[str]:
    return to_vp(kloop_persistent_zc(SCHEDULES[name[:-3]]) if name.endswith("_zc") else kloop_persistent(SCHEDULES[name]))


def _asm_define(macro: str, lines: List[str]) -> List[str]:
    return [f"#define {macro} \\"] + [f'  "{ln}\\n\\t" \\' for ln in lines] + ['  ""', ""]


def render_production() -> str:
    """The shipped schedules only, at their lab SC indices; every other family or index is a
    compile-time error naming the lab header."""
    lab_only = 'static_assert(SC < 0, "lab-only schedule: include gemm_bf16_asm_loop_lab.h first");'
    parts = ["// GENERATED by tools/gen_bf16_asm_loop.py -- do not edit by hand.",
             "// PRODUCTION header: the K-pipeline schedules gemm_bf16.hip dispatches (SHIPPED in the generator),",
             "// at the SC indices they have in the lab header gemm_bf16_asm_loop_lab.h, which carries every",
             "// schedule and, when included first, masks this one.",
             "#pragma once", f"#ifndef {LAB_GUARD}", ""]
    for fam in ("W4A", "W4EF", "W4DS"):
        parts.append(f"#define {fam}_LOOP_SELECT(SC) {lab_only}")
    parts.append("")
    for fam, names in (("W4AP", PERSISTENT), ("W4VP", VP)):
        sel = [f"if constexpr (SC == {names.index(n)}) {fam}_LOOP({fam}_ASM_{n.upper()});" for n in SHIPPED[fam]]
        parts.append(f"#define {fam}_LOOP_SELECT(SC) \\")
        parts.append("  " + " else \\\n  ".join(sel + [lab_only]))
        for n in SHIPPED[fam]:
            parts.append(f"#define {fam}_SC_{n.upper()} {names.index(n)}")
        parts.append("")
    for n in SHIPPED["W4AP"]:
        parts += _asm_define(f"W4AP_ASM_{n.upper()}", ap_lines(n))
    for n in SHIPPED["W4VP"]:
        parts += _asm_define(f"W4VP_ASM_{n.upper()}", vp_lines(n))
    parts.append(f"#endif  // {LAB_GUARD}")
    return "\n".join(parts) + "\n"


def write_all(out_dir: str = "") -> List[str]:
    outs = []
    for path, text in ((OUT, render_production()), (LAB_OUT, render())):
        if out_dir:
            path = os.path.join(out_dir, os.path.basename(path))
        with open(path, "w") as f:
            f.write(text)
        outs.append(path)
    return outs


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--out-dir", default="", help="write the headers here instead of native/hip/")
    for p in write_all(ap.parse_args().out_dir):
        print(f"wrote {p}")
