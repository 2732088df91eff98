#!/usr/bin/env python3
"""Generate the hand-scheduled K pipeline of the fp8 256x256 GEMM (native/hip/gemm_fp8_asm_loop.h).

The fp8 production kernel q16 (gemm_fp8_kernels.h) runs the unscaled double-rate
``v_mfma_f32_16x16x128_f8f6f4``: a K-tile is 128 fp8 = one 128-byte LDS row, so its LDS image,
LDS-DMA pieces and XOR swizzle are byte-for-byte those of the bf16 w4ap kernel, and a wave's
128x128 sub-tile is the same 8x8 grid of 16x16 accumulators. What differs is the K-tile body:

  * 64 MFMA slots of 32 cycles (not 128 of 16) in four quarter blocks over ONE fragment set
    (FA = A fragments a0..a7 in v[0:63], FB = B fragments b0..b7 in v[64:127], 8 VGPRs each):
        slots  0..15  B0 x A0      B0 = b0..3, B1 = b4..7, A0 = a0..3, A1 = a4..7
        slots 16..31  B0 x A1      (b_j last used at slot 19 + 4j)
        slots 32..47  B1 x A0      ASLOW: a_j last used at slot 35 + 4j
        slots 48..63  B1 x A1
  * A1 / B1 of tile t are read at the start of K-tile t (their registers died in the previous
    K-tile's last block); B0' / A0' of tile t+1 after their last use in this one;
  * a fragment is two ds_read_b128 (16-byte chunks g and g + 4 of its 128-byte row for lane group
    g = lane >> 4: conflict-free, see F8Q_CHUNK).

Waits: the lgkmcnt before an MFMA whose operand was read in this K-tile is computed here
(``lgkmcnt(n)``, n = LDS reads issued after that fragment's), so a schedule only places reads,
the free barrier (lgkmcnt(0) + s_barrier: every wave is done with tile t, whose buffer the DMA
of tile t+2 then overwrites), the DMA pieces, and the landing wait (vmcnt(pieces issued so far)
+ s_barrier: tile t+1 is in LDS). The persistent frame (operands, drain into the next output
tile, flags) is the bf16 one: gemm_w4ap.h runs both.

    python tools/gen_fp8_asm_loop.py               # rewrites both headers in native/hip/
    python tools/gen_fp8_asm_loop.py --out-dir D   # writes them to D (tests/test_gemm_build.py drift check)

Two headers, as for bf16 (tools/gen_bf16_asm_loop.py): ``gemm_fp8_asm_loop.h`` with the shipped
schedules only (SHIPPED below), ``gemm_fp8_asm_loop_lab.h`` with every schedule for the lab libraries.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "native", "hip", "gemm_fp8_asm_loop.h")
LAB_OUT = os.path.join(ROOT, "native", "hip", "gemm_fp8_asm_loop_lab.h")
LAB_GUARD = "AMDGO_FP8_ASM_LOOP_LAB"

SLOTS = 64
PIECE_STRIDE = 0x1000
MAX_FILLERS = 4          # per 32-cycle MFMA gap (one wave per SIMD)


def frag(isb: bool, x: int) -> str:
    base = (64 if isb else 0) + 8 * x
    return f"v[{base}:{base + 7}]"


def half(isb: bool, x: int, h: int) -> str:
    base = (64 if isb else 0) + 8 * x + 4 * h
    return f"v[{base}:{base + 3}]"


def operands(i: int, aslow: bool):
    """(bi, ai) of MFMA slot i: the q16 quarter-block order (gemm_fp8_kernels.h)."""
    blk, w = i >> 4, i & 15
    sl = aslow and blk == 2
    bi = (blk >> 1) * 4 + ((w & 3) if sl else (w >> 2))
    ai = (blk & 1) * 4 + ((w >> 2) if sl else (w & 3))
    return bi, ai


def mfma(i: int, aslow: bool, zero_c: bool = False) -> str:
    bi, ai = operands(i, aslow)
    q = ai * 8 + bi
    c = "0" if zero_c else f"a[{4 * q}:{4 * q + 3}]"
    return f"v_mfma_f32_16x16x128_f8f6f4 a[{4 * q}:{4 * q + 3}], {frag(True, bi)}, {frag(False, ai)}, {c}"


def last_use(aslow: bool) -> Dict[tuple, int]:
    out = {}
    for i in range(SLOTS):
        bi, ai = operands(i, aslow)
        out[(True, bi)] = i
        out[(False, ai)] = i
    return out


def first_use(aslow: bool) -> Dict[tuple, int]:
    out = {}
    for i in reversed(range(SLOTS)):
        bi, ai = operands(i, aslow)
        out[(True, bi)] = i
        out[(False, ai)] = i
    return out


# read order of the two halves of each set: R1 = A1 then B1 of tile t, R0 = B0 then A0 of tile t+1
R1_ORDER = [(False, 4 + j // 2, j % 2) for j in range(8)] + [(True, 4 + j // 2, j % 2) for j in range(8)]
R0_ORDER = [(True, j // 2, j % 2) for j in range(8)] + [(False, j // 2, j % 2) for j in range(8)]


class Schedule:
    def __init__(self, name, r1, w1, dma, w2, r0, aslow=True, w3=SLOTS - 1):
        self.name, self.r1, self.w1, self.b1 = name, r1, w1, w1 + 1
        self.dma, self.w2, self.b2, self.r0 = dma, w2, None if w2 is None else w2 + 1, r0
        self.aslow, self.w3 = aslow, w3
        self.vk = dma[-1]                   # the K-offset add right after the last piece

    @property
    def merged(self) -> bool:
        """One barrier per K-tile: the free wait is vmcnt(0) lgkmcnt(0), so its barrier also
        publishes tile t+1 (DMA'd during the previous K-tile)."""
        return self.w2 is None

    def issued_before_w2(self) -> int:
        return sum(1 for s in self.dma if s <= self.w2)


def validate(sc: Schedule) -> None:
    lu, fu = last_use(sc.aslow), first_use(sc.aslow)
    assert len(sc.r1) == 16 and len(sc.r0) == 16 and len(sc.dma) == 16, sc.name
    land = [] if sc.merged else [sc.w2, sc.b2]
    assert all(0 <= x < SLOTS for x in sc.r1 + sc.r0 + sc.dma + [sc.w1, sc.b1, sc.w3] + land), sc.name
    assert sc.r1 == sorted(sc.r1) and sc.r0 == sorted(sc.r0) and sc.dma == sorted(sc.dma), sc.name
    # R1 of tile t: read before its first use (the generator then inserts the lgkmcnt)
    for (isb, x, _), s in zip(R1_ORDER, sc.r1):
        assert s < fu[(isb, x)], (sc.name, "R1", isb, x, s)
    assert sc.w1 > max(sc.r1) and min(sc.dma) > sc.b1, sc.name      # DMA after the free barrier
    if sc.merged:
        assert min(sc.r0) > sc.b1, sc.name                           # R0' after the (only) barrier
    else:
        assert sc.b2 > sc.w2 > sc.b1 and min(sc.r0) >= sc.b2, sc.name   # R0' after the landing barrier
    # R0' of tile t+1 overwrites a fragment only after this K-tile's last MFMA on it
    for (isb, x, _), s in zip(R0_ORDER, sc.r0):
        assert s >= lu[(isb, x)], (sc.name, "R0", isb, x, s, lu[(isb, x)])
    assert sc.w3 >= max(sc.r0), sc.name
    load = {i: 0 for i in range(SLOTS)}
    for x in sc.r1 + sc.r0 + sc.dma + [d - 1 for d in sc.dma] + [sc.w1, sc.b1, sc.w3] + land:
        load[x] += 1
    assert max(load.values()) <= MAX_FILLERS, (sc.name, {k: v for k, v in load.items() if v > MAX_FILLERS})


def pairs(start, step, n=8):
    """Two reads (one fragment) per slot, a fragment every `step` slots."""
    return [start + (j // 2) * step for j in range(2 * n)]


def make(name, r1, w1, dma, w2, r0, aslow=True):
    sc = Schedule(name, r1=r1, w1=w1, dma=dma, w2=w2, r0=r0, aslow=aslow)
    validate(sc)
    return sc


SCHEDULES = {
    # the production q16 placement (v15/v18): a fragment every 2nd slot from 0, free barrier after
    # slot 17, DMA every 3rd slot from 18, landing wait at 34, B0' from 35 and A0' from 43 in pairs
    "p": make("p", r1=pairs(0, 2), w1=16, dma=[18 + 3 * p for p in range(16)], w2=34,
              r0=pairs(35, 2, 4) + pairs(43, 2, 4)),
    # one read per slot; the free wait 4 MFMAs after the last R1 read (the bf16 g4 lesson)
    "s1": make("s1", r1=list(range(16)), w1=19, dma=[21 + 2 * p for p in range(16)], w2=36,
               r0=list(range(38, 46)) + list(range(46, 54))),
    # as s1, DMA every 3rd slot (to 66 would overflow: pieces 0..13 every 3rd, the last two every 2nd)
    "s1d3": make("s1d3", r1=list(range(16)), w1=19, dma=[21 + 3 * p for p in range(14)] + [61, 63], w2=36,
                 r0=list(range(38, 46)) + list(range(46, 54))),
    # dense DMA right after the free barrier, landing wait late
    "s1early": make("s1early", r1=list(range(16)), w1=19, dma=list(range(21, 37)), w2=44,
                    r0=list(range(45, 53)) + list(range(53, 61))),
    # production's pairs with the free wait moved 4 MFMAs after the last read
    "pg": make("pg", r1=pairs(0, 2), w1=18, dma=[20 + 3 * p for p in range(14)] + [61, 63], w2=35,
               r0=pairs(37, 2, 4) + pairs(45, 2, 4)),
}

# one barrier per K-tile: B0' / A0' of tile t+1 as soon as their registers are dead
_M_R0 = [22, 23, 24, 25, 28, 29, 32, 33, 36, 37, 40, 41, 44, 45, 48, 49]
SCHEDULES["m"] = make("m", r1=list(range(16)), w1=19, dma=[21 + 2 * p for p in range(16)], w2=None, r0=_M_R0)
SCHEDULES["md3"] = make("md3", r1=list(range(16)), w1=19, dma=[21 + 3 * p for p in range(14)] + [61, 63],
                        w2=None, r0=_M_R0)

PERSISTENT = list(SCHEDULES) + ["p_rw", "s1d3_rw", "p_zc"]
# a name ending in _zc: kloop_persistent_zc (first K-tile with src C = 0; frame EPI 8)
# a name ending in _rw: that schedule in kloop_persistent_rw (relaxed first landing wait)


def rd(isb: bool, x: int, h: int, buf: int, ef: bool) -> str:
    """ds_read of fragment half (isb, x, h) from buffer buf; ef: B through the permuted lane offsets
    (gemm_w4ap.h EPI=2: fragment x reads Bt rows 32(x>>1) + 4(x&1) + 8(rho>>2) + (rho&3))."""
    if ef and isb:
        return f"ds_read_b128 {half(isb, x, h)}, %[rb{'e' if x % 2 == 0 else 'o'}{buf}{h}] offset:{(x >> 1) * 4096}"
    return f"ds_read_b128 {half(isb, x, h)}, %[{'rb' if isb else 'ra'}{buf}{h}] offset:{x * 2048}"


def body(sc: Schedule, cur: int, dma: bool, nx: bool, nxt_tile: bool = False, ef: bool = False,
         zero_c: bool = False, w2_extra: int = 0, last: bool = False, cap: int = 7,
         extra: Dict[int, List[str]] = None) -> List[str]:
    """One K-tile. EF kernel (ef): permuted B reads; zero_c: src C = 0 (the tile's first K-tile);
    w2_extra: stores younger than the landing pieces; last: the fused epilogue in the gaps."""
    rA, rB, voff, kstep = ("%[nA]", "%[nB]", "%[nvoff]", "%[nkstep]") if nxt_tile else \
        ("%[rA]", "%[rB]", "%[voff]", "%[kstep]")
    nxt = 1 - cur
    gap: Dict[int, List[tuple]] = {i: [] for i in range(SLOTS)}
    for (isb, x, h), s in zip(R1_ORDER, sc.r1):
        gap[s].append(("read", (isb, x), rd(isb, x, h, cur, ef)))
    gap[sc.w1].append(("lgk0", None, "s_waitcnt vmcnt(0) lgkmcnt(0)" if sc.merged else "s_waitcnt lgkmcnt(0)"))
    gap[sc.b1].append(("op", None, "s_barrier"))
    if dma:
        for p, s in enumerate(sc.dma):
            gap[s - 1].append(("op", None, f"s_mov_b32 m0, %[m0b{cur}]" if p == 0 else
                               f"s_add_u32 m0, m0, {PIECE_STRIDE:#x}"))
            gap[s].append(("op", None, f"buffer_load_dwordx4 {voff}, {rB if p >= 8 else rA}, %[s{p & 7}] offen lds"))
        gap[sc.vk].append(("op", None, f"v_add_u32_e32 {voff}, {kstep}, {voff}"))
    if nx:
        if not sc.merged:
            n = (sc.issued_before_w2() if dma else 0) + w2_extra
            gap[sc.w2].append(("op", None, f"s_waitcnt vmcnt({n})"))
            gap[sc.b2].append(("op", None, "s_barrier"))
        for (isb, x, h), s in zip(R0_ORDER, sc.r0):
            gap[s].append(("read", None, rd(isb, x, h, nxt, ef)))
    gap[sc.w3].append(("lgk0", None, "s_waitcnt lgkmcnt(0)"))
    for i, ops in (extra or {}).items():
        gap[i] += [("read", None, t) if t.startswith("ds_read") else ("op", None, t) for t in ops]
    tail: List[str] = []
    if last:
        assert ef and not nx
        load = {i: len(gap[i]) for i in range(SLOTS)}
        egap, tail = ef_epilogue([operands(i, sc.aslow) for i in range(SLOTS)], load, cap)
        for i in range(SLOTS):
            gap[i] += [("op", None, t) for t in egap[i]]
    # simulate the LDS queue: before each MFMA, wait for the reads of this K-tile it consumes
    out: List[str] = []
    queue: List[object] = []           # in-flight LDS reads in issue order (fragment key or None)
    for i in range(SLOTS):
        bi, ai = operands(i, sc.aslow)
        need = [k for k in ((True, bi), (False, ai)) if k in queue]
        if need:
            last = max(idx for idx, k in enumerate(queue) if k in need)
            n = len(queue) - last - 1
            out.append(f"s_waitcnt lgkmcnt({n})")
            queue = queue[last + 1:]
        out.append(mfma(i, sc.aslow, zero_c))
        for kind, key, text in gap[i]:
            out.append(text)
            if kind == "read":
                queue.append(key)
            elif kind == "lgk0":
                queue = []
    if tail:
        out += ["s_nop 7", "s_nop 7"] + tail
    return out


def prologue() -> List[str]:
    out = ["s_nop 4"]
    for buf in (0, 1):
        for p in range(16):
            out.append(f"s_mov_b32 m0, %[m0b{buf}]" if p == 0 else f"s_add_u32 m0, m0, {PIECE_STRIDE:#x}")
            out.append("s_nop 0")
            out.append(f"buffer_load_dwordx4 %[voff], %[{'rB' if p >= 8 else 'rA'}], %[s{p & 7}] offen lds")
        out.append("v_add_u32_e32 %[voff], %[kstep], %[voff]")
    return out


def r0_reads(buf: int) -> List[str]:
    return [f"ds_read_b128 {half(isb, x, h)}, %[{'rb' if isb else 'ra'}{buf}{h}] offset:{x * 2048}"
            for isb, x, h in R0_ORDER]


def kloop_persistent_rw(sc: Schedule, stores: int = 32) -> List[str]:
    """kloop_persistent() with the relaxed first landing wait (tools/gen_bf16_asm_loop.py
    kloop_persistent_rw): the previous tile's staged-epilogue stores are skipped by the first K-tile's
    landing wait; the first tile waits for both prologue K-tiles."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lf8rw_entry_%="]
    out += prologue()
    out += ["s_waitcnt vmcnt(0)"]
    out.append(".Lf8rw_entry_%=:")
    out.append("s_barrier")
    out += r0_reads(0)
    out.append("s_waitcnt lgkmcnt(0)")
    out += body(sc, 0, dma=True, nx=True, w2_extra=stores)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8rw_drain_%="]
    out.append(".Lf8rw_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8rw_loop_%="]
    out.append(".Lf8rw_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lf8rw_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lf8rw_done_%=", ".Lf8rw_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lf8rw_done_%=:")
    return out


# Deferred C stores (frame EPI 7; the bf16 generator documents the protocol). fp8 K-tile: stores at
# the odd slots 1..7 (no R1 reads there, before the first DMA piece at 18), the LDS reads for the next
# K-tile at 51..57 (after the R0 reads; the K-tile's closing lgkmcnt(0) covers them).
DS_PEEL = 6
DS_STORE_SLOTS = (1, 3, 5, 7)
DS_ADD_SLOTS = (9, 11, 13, 15)
DS_LDS_SLOTS = (51, 53, 55, 57)
DS_EPI_STORES = 8


def ds_ops(j: int) -> Dict[int, List[str]]:
    ops: Dict[int, List[str]] = {}
    for n, (sl, al) in enumerate(zip(DS_STORE_SLOTS, DS_ADD_SLOTS)):
        item = 4 * j + n
        data = f"%[h{item}]" if item < 16 else f"v[{240 + 4 * n}:{243 + 4 * n}]"
        ops.setdefault(sl, []).append(f"global_store_dwordx4 %[vcur], {data}, %[sCp] nt")
        ops.setdefault(sl + 1, []).append("v_add_u32_e32 %[vcur], %[s8N], %[vcur]")
    if j + 1 < DS_PEEL and 4 * (j + 1) >= 16:
        for n, sl in enumerate(DS_LDS_SLOTS):
            k = 4 * (j + 1) - 16 + n
            ops.setdefault(sl, []).append(f"ds_read_b128 v[{240 + 4 * n}:{243 + 4 * n}], %[stgl] offset:{k * 1024}")
    return ops


def kloop_persistent_ds(sc: Schedule) -> List[str]:
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lf8ds_entry_%="]
    out += prologue()
    out += ["s_waitcnt vmcnt(0)"]
    out.append(".Lf8ds_entry_%=:")
    out.append("s_barrier")
    out += r0_reads(0)
    out.append("s_waitcnt lgkmcnt(0)")
    for j in range(DS_PEEL):
        extra = len(DS_STORE_SLOTS) + (DS_EPI_STORES if j == 0 else 0)
        out += body(sc, j % 2, dma=True, nx=True, w2_extra=extra, extra=ds_ops(j))
    out += [f"s_sub_u32 %[cnt], %[cnt], {DS_PEEL // 2}", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8ds_drain_%="]
    out.append(".Lf8ds_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8ds_loop_%="]
    out.append(".Lf8ds_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lf8ds_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lf8ds_done_%=", ".Lf8ds_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lf8ds_done_%=:")
    assert sum(ln.startswith("global_store") for ln in out) == 24
    return out


DS = ["p"]


def kloop_persistent_zc(sc: Schedule) -> List[str]:
    """kloop_persistent() whose first K-tile starts every accumulator with src C = 0 (frame EPI 8)."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lf8zc_entry_%="]
    out += prologue()
    out += ["s_waitcnt vmcnt(16)"]
    out.append(".Lf8zc_entry_%=:")
    out.append("s_barrier")
    out += r0_reads(0)
    out.append("s_waitcnt lgkmcnt(0)")
    out += body(sc, 0, dma=True, nx=True, zero_c=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8zc_drain_%="]
    out.append(".Lf8zc_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8zc_loop_%="]
    out.append(".Lf8zc_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lf8zc_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lf8zc_done_%=", ".Lf8zc_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lf8zc_done_%=:")
    return out


def kloop_persistent(sc: Schedule) -> List[str]:
    """One output tile's K pipeline (the w4ap frame: flags bit 0 = first tile of this workgroup,
    bit 1 = a next tile whose K-tiles 0 and 1 the drain DMAs)."""
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lf8ap_entry_%="]
    out += prologue()
    out += ["s_waitcnt vmcnt(16)"]
    out.append(".Lf8ap_entry_%=:")
    out.append("s_barrier")
    out += r0_reads(0)
    out.append("s_waitcnt lgkmcnt(0)")
    out.append(".Lf8ap_loop_%=:")
    out += body(sc, 0, dma=True, nx=True)
    out += body(sc, 1, dma=True, nx=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8ap_loop_%="]
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lf8ap_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True)
    out += body(sc, 1, dma=True, nx=False, nxt_tile=True)
    out += ["s_branch .Lf8ap_done_%=", ".Lf8ap_last_%=:"]
    out += body(sc, 0, dma=False, nx=True)
    out += body(sc, 1, dma=False, nx=False)
    out.append(".Lf8ap_done_%=:")
    return out


# ---------------------------------------------------------------------------------------------------
# Fused epilogue (w4ap EPI=2, "EF"; the bf16 design in tools/gen_bf16_asm_loop.py). In the fp8 K-tile
# every accumulator gets exactly one MFMA, so in the last K-tile each slot finalises one accumulator:
# its 4 accvgpr reads (>= EF_HAZ MFMAs later: 16x16x128 f8 is an 8-pass XDL op), 2 cvts and, per
# accumulator pair (bi even / odd, same ai), one 16-byte store go into the following gaps.
EF_T, EF_NT = 224, 4
EF_P, EF_NP = 240, 4
EF_HAZ = 2


def ef_epilogue(order: List[tuple], load: Dict[int, int], cap: int):
    """order: (bi, ai) per slot. Same greedy placement as the bf16 generator."""
    final = {ai * 8 + bi: s for s, (bi, ai) in enumerate(order)}
    gaps: Dict[int, List[str]] = {i: [] for i in range(SLOTS)}
    tail: List[str] = []
    used = dict(load)

    def put(op: str, ready: int) -> int:
        for s in range(max(ready, 0), SLOTS):
            if used.get(s, 0) < cap:
                gaps[s].append(op)
                used[s] = used.get(s, 0) + 1
                return s
        tail.append(op)
        return SLOTS + len(tail)

    pair_done, pset_of, last_store, last_cvt = {}, {}, {}, {}
    for n_acc, acc in enumerate(sorted(final, key=lambda a: final[a])):
        ts = n_acc % EF_NT
        t = EF_T + 4 * ts
        ready = max(final[acc] + EF_HAZ, last_cvt.get(ts, -1))
        for k in range(4):
            ready = put(f"v_accvgpr_read_b32 v{t + k}, a{4 * acc + k}", ready)
        pair = acc >> 1
        if pair not in pset_of:
            pset_of[pair] = len(pset_of) % EF_NP
        ps = pset_of[pair]
        pbase = EF_P + 4 * ps + 2 * (acc & 1)
        ready = max(ready, last_store.get(ps, -1))
        for k in range(2):
            ready = put(f"v_cvt_pk_bf16_f32 v{pbase + k}, v{t + 2 * k}, v{t + 2 * k + 1}", ready)
        last_cvt[ts] = ready
        pair_done.setdefault(pair, []).append(ready)
        if len(pair_done[pair]) == 2:
            m, p = pair >> 2, pair & 3
            pos = put(f"global_store_dwordx4 %[cv{m}], v[{EF_P + 4 * ps}:{EF_P + 4 * ps + 3}], %[sC] offset:{64 * p}",
                      max(pair_done[pair]))
            last_store[ps] = pos + 1
    return gaps, tail


def ef_check(lines: List[str]) -> None:
    """Static audit of an EF last K-tile (see the bf16 generator's ef_check)."""
    import re
    mf, final_at, pad, treg, pword, stored = 0, {}, {}, {}, {}, set()
    for ln in lines:
        if ln.startswith("v_mfma"):
            mf += 1
            final_at[int(re.match(r"v_mfma\S* a\[(\d+):", ln).group(1)) // 4] = mf
            continue
        if ln.startswith("s_nop"):
            pad[mf] = pad.get(mf, 0) + int(ln.split()[1]) + 1
            continue
        mm = re.match(r"v_accvgpr_read_b32 v(\d+), a(\d+)", ln)
        if mm:
            acc = int(mm.group(2)) // 4
            assert acc in final_at and (mf - final_at[acc] >= EF_HAZ or pad.get(mf, 0) >= 16), ("hazard", acc)
            treg[int(mm.group(1))] = (acc, int(mm.group(2)) % 4)
            continue
        mm = re.match(r"v_cvt_pk_bf16_f32 v(\d+), v(\d+), v(\d+)", ln)
        if mm:
            d, s0, s1 = (int(x) for x in mm.groups())
            (a0, k0), (a1, k1) = treg[s0], treg[s1]
            assert a0 == a1 and k1 == k0 + 1 and k0 % 2 == 0 and (d - EF_P) % 4 == 2 * (a0 & 1) + k0 // 2, ln
            pword[d] = a0
            continue
        mm = re.match(r"global_store_dwordx4 %\[cv(\d)\], v\[(\d+):\d+\], %\[sC\] offset:(\d+)", ln)
        if mm:
            m, base, p = int(mm.group(1)), int(mm.group(2)), int(mm.group(3)) // 64
            q = m * 8 + 2 * p
            assert [pword[base + k] for k in range(4)] == [q, q, q + 1, q + 1], ln
            stored.add((m, p))
    assert len(stored) == 32, len(stored)


def late_stores(lines: List[str]) -> int:
    """Stores issued after the last DMA piece of a K-tile text."""
    late = 0
    for ln in lines:
        if ln.startswith("buffer_load"):
            late = 0
        elif ln.startswith("global_store"):
            late += 1
    return late


def kloop_persistent_ef(sc: Schedule, cap: int = 7) -> List[str]:
    last_nx = body(sc, 1, dma=True, nx=False, nxt_tile=True, ef=True, last=True, cap=cap)
    last_no = body(sc, 1, dma=False, nx=False, ef=True, last=True, cap=cap)
    ef_check(last_nx)
    ef_check(last_no)
    stores = sum(ln.startswith("global_store") for ln in last_nx)
    assert stores == 32
    out = ["s_nop 4", "s_bitcmp0_b32 %[flags], 0", "s_cbranch_scc1 .Lf8ef_entry_%="]
    out += prologue()
    out += ["s_waitcnt vmcnt(0)"]
    out.append(".Lf8ef_entry_%=:")
    out.append(f"s_waitcnt vmcnt({16 + stores})")
    out.append("s_barrier")
    out += [rd(isb, x, h, 0, True) for isb, x, h in R0_ORDER]
    out.append("s_waitcnt lgkmcnt(0)")
    out += body(sc, 0, dma=True, nx=True, ef=True, zero_c=True, w2_extra=late_stores(last_nx))
    out += body(sc, 1, dma=True, nx=True, ef=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_eq_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8ef_drain_%="]
    out.append(".Lf8ef_loop_%=:")
    out += body(sc, 0, dma=True, nx=True, ef=True)
    out += body(sc, 1, dma=True, nx=True, ef=True)
    out += ["s_sub_u32 %[cnt], %[cnt], 1", "s_cmp_lg_u32 %[cnt], 0", "s_cbranch_scc1 .Lf8ef_loop_%="]
    out.append(".Lf8ef_drain_%=:")
    out += ["s_bitcmp0_b32 %[flags], 1", "s_cbranch_scc1 .Lf8ef_last_%="]
    out += body(sc, 0, dma=True, nx=True, nxt_tile=True, ef=True)
    out += last_nx
    out += ["s_branch .Lf8ef_done_%=", ".Lf8ef_last_%=:"]
    out += body(sc, 0, dma=False, nx=True, ef=True)
    out += last_no
    out.append(".Lf8ef_done_%=:")
    return out


# schedules the fused-epilogue kernel is generated for (index = EF SC)
EF = ["p", "s1d3", "p_nt"]
# a name ending in _nt: the same schedule with nontemporal C stores (global_store ... nt)


# ---------------------------------------------------------------------------------------------------
# VP DMA form (frame DM >= 1, gemm_w4ap.h): piece p's whole lane offset (row block, row, chunk) is its
# own VGPR %[vp<p>], fixed for the kernel, and the K byte offset of the DMA'd K-tile is one SGPR
# (%[koff], %[nkoff] for the next tile) used as the soffset: one SALU add per K-tile instead of a VALU
# add, no per-piece row-block SGPRs, and A and B pieces may use different row maps -- DM = 2 reads each
# A-panel DMA instruction's 8 rows 32 apart (PA: K not a power of two, see gemm_bf16.hip v47).
VP = ["p", "s1d3", "p_zc"]   # p_zc: the ZC first K-tile (src C = 0) in VP form


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
    gaps, cur = [], 0
    for ln in lines:
        if ln.startswith("v_mfma"):
            gaps.append(cur)
            cur = 0
        elif not ln.startswith("."):
            cur += 1
    return {"max_fillers_per_gap": max(gaps[1:]), "mfmas": sum(ln.startswith("v_mfma") for ln in lines)}


def render() -> str:
    parts = ["// GENERATED by tools/gen_fp8_asm_loop.py -- do not edit by hand.",
             "// LAB header: every schedule of the hand-scheduled K pipeline of the persistent fp8 GEMM",
             "// (gemm_fp8_256x256_q16ap, gemm_fp8_kernels.h; frame and operands in gemm_w4ap.h, W4AP_LOOP).",
             "// Only the tools-only lab libraries include it; production builds gemm_fp8_asm_loop.h.",
             "#pragma once", f"#define {LAB_GUARD} 1", ""]
    sel = [f"if constexpr (SC == {i}) W4AP_LOOP(F8AP_ASM_{n.upper()});" for i, n in enumerate(PERSISTENT)]
    parts.append("#define F8AP_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(sel))
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(PERSISTENT)))
    for i, n in enumerate(PERSISTENT):
        parts.append(f"#define F8AP_SC_{n.upper()} {i}")
    parts.append("")
    esel = [f"if constexpr (SC == {i}) W4EF_LOOP(F8EF_ASM_{n.upper()});" for i, n in enumerate(EF)]
    parts.append("// fused-epilogue persistent kernel (q16ap EPI=2): schedule index -> asm text (W4EF_LOOP)")
    parts.append("#define F8EF_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(esel))
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(EF)))
    for i, n in enumerate(EF):
        parts.append(f"#define F8EF_SC_{n.upper()} {i}")
    parts.append("")
    for name in EF:
        lines = kloop_persistent_ef(SCHEDULES[name.split("_")[0]])
        if name.endswith("_nt"):
            lines = [ln + " nt" if ln.startswith("global_store") else ln for ln in lines]
        parts.append(f"#define F8EF_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    dsel = [f"if constexpr (SC == {i}) W4DS_LOOP(F8DS_ASM_{n.upper()});" for i, n in enumerate(DS)]
    parts.append("// deferred-store form (frame EPI 7): schedule index -> asm text (W4DS_LOOP)")
    parts.append("#define F8DS_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(dsel))
    for i, n in enumerate(DS):
        parts.append(f"#define F8DS_SC_{n.upper()} {i}")
    parts.append("")
    for name in DS:
        lines = kloop_persistent_ds(SCHEDULES[name])
        parts.append(f"#define F8DS_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    vsel = [f"if constexpr (SC == {i}) W4VP_LOOP(F8VP_ASM_{n.upper()});" for i, n in enumerate(VP)]
    parts.append("// VP DMA form (frame DM >= 1): schedule index -> asm text (W4VP_LOOP)")
    parts.append("#define F8VP_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(vsel))
    for i, n in enumerate(VP):
        parts.append(f"#define F8VP_SC_{n.upper()} {i}")
    parts.append("")
    for name in VP:
        lines = to_vp(ap_lines(name))
        parts.append(f"#define F8VP_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    for name in PERSISTENT:
        lines = ap_lines(name)
        a = audit(lines)
        parts.append(f"// {name}: {a['mfmas']} MFMAs, <= {a['max_fillers_per_gap']} instructions per MFMA gap")
        parts.append(f"#define F8AP_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    return "\n".join(parts)


# The schedules gemm_fp8.hip dispatches: v20 / v21 F8AP p_zc, v22 / v23 F8VP p_zc (VP + PA DMA form).
SHIPPED = {"F8AP": ["p_zc"], "F8VP": ["p_zc"]}


def ap_lines(name: str) -> List[str]:
    return (kloop_persistent_rw(SCHEDULES[name[:-3]]) if name.endswith("_rw") else
            kloop_persistent_zc(SCHEDULES[name[:-3]]) if name.endswith("_zc") else kloop_persistent(SCHEDULES[name]))


def render_production() -> str:
    """The shipped schedule only, at its lab SC index; every other family or index is a
    compile-time error naming the lab header."""
    lab_only = 'static_assert(SC < 0, "lab-only schedule: include gemm_fp8_asm_loop_lab.h first");'
    parts = ["// GENERATED by tools/gen_fp8_asm_loop.py -- do not edit by hand.",
             "// PRODUCTION header: the K-pipeline schedule gemm_fp8.hip dispatches (SHIPPED in the generator),",
             "// at the SC index it has in the lab header gemm_fp8_asm_loop_lab.h, which carries every",
             "// schedule and, when included first, masks this one.",
             "#pragma once", f"#ifndef {LAB_GUARD}", ""]
    for fam in ("F8EF", "F8DS"):
        parts.append(f"#define {fam}_LOOP_SELECT(SC) {lab_only}")
    for fam, names, macro, lines_of in (("F8AP", PERSISTENT, "W4AP_LOOP", ap_lines),
                                        ("F8VP", VP, "W4VP_LOOP", lambda n: to_vp(ap_lines(n)))):
        sel = [f"if constexpr (SC == {names.index(n)}) {macro}({fam}_ASM_{n.upper()});" for n in SHIPPED[fam]]
        parts.append(f"#define {fam}_LOOP_SELECT(SC) \\")
        parts.append("  " + " else \\\n  ".join(sel + [lab_only]))
        for n in SHIPPED[fam]:
            parts.append(f"#define {fam}_SC_{n.upper()} {names.index(n)}")
        parts.append("")
        for n in SHIPPED[fam]:
            parts.append(f"#define {fam}_ASM_{n.upper()} \\")
            parts += [f'  "{ln}\\n\\t" \\' for ln in lines_of(n)] + ['  ""', ""]
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
        print("wrote", p)
