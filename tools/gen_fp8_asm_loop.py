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

    python tools/gen_fp8_asm_loop.py          # rewrites native/hip/gemm_fp8_asm_loop.h
"""
from __future__ import annotations

import os
from typing import Dict, List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "native", "hip", "gemm_fp8_asm_loop.h")

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


def mfma(i: int, aslow: bool) -> str:
    bi, ai = operands(i, aslow)
    q = ai * 8 + bi
    return f"v_mfma_f32_16x16x128_f8f6f4 a[{4 * q}:{4 * q + 3}], {frag(True, bi)}, {frag(False, ai)}, a[{4 * q}:{4 * q + 3}]"


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

PERSISTENT = list(SCHEDULES)


def body(sc: Schedule, cur: int, dma: bool, nx: bool, nxt_tile: bool = False) -> List[str]:
    rA, rB, voff, kstep = ("%[nA]", "%[nB]", "%[nvoff]", "%[nkstep]") if nxt_tile else \
        ("%[rA]", "%[rB]", "%[voff]", "%[kstep]")
    nxt = 1 - cur
    gap: Dict[int, List[tuple]] = {i: [] for i in range(SLOTS)}
    for (isb, x, h), s in zip(R1_ORDER, sc.r1):
        gap[s].append(("read", (isb, x), f"ds_read_b128 {half(isb, x, h)}, %[{'rb' if isb else 'ra'}{cur}{h}] "
                                         f"offset:{x * 2048}"))
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
            n = sc.issued_before_w2() if dma else 0
            gap[sc.w2].append(("op", None, f"s_waitcnt vmcnt({n})"))
            gap[sc.b2].append(("op", None, "s_barrier"))
        for (isb, x, h), s in zip(R0_ORDER, sc.r0):
            gap[s].append(("read", None, f"ds_read_b128 {half(isb, x, h)}, %[{'rb' if isb else 'ra'}{nxt}{h}] "
                                         f"offset:{x * 2048}"))
    gap[sc.w3].append(("lgk0", None, "s_waitcnt lgkmcnt(0)"))
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
        out.append(mfma(i, sc.aslow))
        for kind, key, text in gap[i]:
            out.append(text)
            if kind == "read":
                queue.append(key)
            elif kind == "lgk0":
                queue = []
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
             "// The hand-scheduled K pipeline of the persistent fp8 GEMM (gemm_fp8_256x256_q16ap,",
             "// gemm_fp8_kernels.h; frame and operands in gemm_w4ap.h, W4AP_LOOP).",
             "#pragma once", ""]
    sel = [f"if constexpr (SC == {i}) W4AP_LOOP(F8AP_ASM_{n.upper()});" for i, n in enumerate(PERSISTENT)]
    parts.append("#define F8AP_LOOP_SELECT(SC) \\")
    parts.append("  " + " else \\\n  ".join(sel))
    parts.append("// " + ", ".join(f"{i} = {n}" for i, n in enumerate(PERSISTENT)))
    for i, n in enumerate(PERSISTENT):
        parts.append(f"#define F8AP_SC_{n.upper()} {i}")
    parts.append("")
    for name in PERSISTENT:
        lines = kloop_persistent(SCHEDULES[name])
        a = audit(lines)
        parts.append(f"// {name}: {a['mfmas']} MFMAs, <= {a['max_fillers_per_gap']} instructions per MFMA gap")
        parts.append(f"#define F8AP_ASM_{name.upper()} \\")
        for ln in lines:
            parts.append(f'  "{ln}\\n\\t" \\')
        parts.append('  ""')
        parts.append("")
    return "\n".join(parts)


if __name__ == "__main__":
    with open(OUT, "w") as f:
        f.write(render())
    print("wrote", OUT)
