"""The LEAN epilogue's LDS staging layout is bank-conflict free (CPU check of gemm_w4ap.h lean_off).

Banking model (MI355X_MICROARCH.md, LDS table): a ds_write_b64 is serviced in 4 groups of 16
contiguous lanes with banks (a/4) mod 32; a ds_read_b64 in 2 groups of 32 lanes with banks (a/4)
mod 64. A group is conflict free when no bank receives two different dword addresses.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lean_off(r, c, h):
    return r * 256 + ((c ^ ((r & 15) >> 1)) << 4) + ((h ^ (r & 1)) << 3)


def _conflict_free(addrs, nbanks):
    seen = {}
    for a in addrs:
        for d in (a // 4, a // 4 + 1):          # an 8-byte access touches two dwords
            b = d % nbanks
            if seen.setdefault(b, d) != d:
                return False
    return True


def test_header_carries_the_checked_formula():
    text = open(os.path.join(ROOT, "native", "hip", "gemm_w4ap.h")).read()
    body = re.search(r"uint32_t lean_off\(int r, int c, int h\) \{\s*return (.*?);\s*\}", text, re.S).group(1)
    assert re.sub(r"\s+", "", body) == "(uint32_t)(r*256+((c^((r&15)>>1))<<4)+((h^(r&1))<<3))"


def test_staging_writes_are_conflict_free():
    # lane (lr, lj) of accumulator n writes row 16*mm + lr, chunk 2n + (lj >> 1), half lj & 1
    for mm in range(2):
        for n in range(8):
            addrs = [lean_off(16 * mm + (lane & 15), 2 * n + ((lane >> 4) >> 1), (lane >> 4) & 1) for lane in range(64)]
            for g in range(4):
                assert _conflict_free(addrs[16 * g:16 * g + 16], 32), (mm, n, g)


def test_staging_reads_are_conflict_free_and_in_order():
    # lane (lr, lj) reads row 4k + lj (+ 16 for the second half of a 32-row pass), chunk lr, both halves
    for base in (0, 16):
        for k in range(4):
            for h in range(2):
                addrs = [lean_off(base + 4 * k + (lane >> 4), lane & 15, h) for lane in range(64)]
                for g in range(2):
                    assert _conflict_free(addrs[32 * g:32 * g + 32], 64), (base, k, h, g)
    # the layout is a bijection of each 256-byte row's 32 eight-byte slots
    for r in range(32):
        slots = {lean_off(r, c, h) for c in range(16) for h in range(2)}
        assert slots == set(range(r * 256, r * 256 + 256, 8))
