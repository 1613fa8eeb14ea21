#!/usr/bin/env python3
"""Bank-conflict model of the P1 tile image (the C2 kernel's SQ_LDS_BANK_CONFLICT is 66 % of
SQ_LDS_IDX_ACTIVE), the same model DESIGN.md §4.2f used for the Q1 image:

  * LDS: 64 banks of 4 bytes; a ds_write_b64 is serviced in 16-lane groups, each lane's 8-byte value occupying the
    bank pair (addr / 8) mod 32; a ds_read_b128 in 16-lane groups over the 64 banks (4 banks per lane);
  * the cycles of one group = the largest number of lanes that hit the same bank (pair);
  * P1 tile image: lane l owns element l of the tile, its row block of RB = 36 doubles (3 rows x 4 blocks x 3) at
    double offset off_l; the closed form writes it with 36 ds_write_b64 (value j of every lane in one instruction);
    the store phase reads the tile's contiguous CSR range with 18 ds_read_b128 per lane (lane l, chunk l + 64 k).

Prints cycles per instruction for the production layout (full tiles: off_l = 36 l, the alignment slot d in {0, 1})
and for alternatives: an odd row stride (37, padding), and a per-element rotation of the value slots like Q1's.
usage: python scripts/study/lds_banks_p1.py
"""
from collections import Counter


def write_cycles(addr_dw):
    """addr_dw: 64 dword addresses of one ds_write_b64 -> cycles (16-lane groups over 32 bank pairs)"""
    cyc = 0
    for g in range(4):
        c = Counter((a // 2) % 32 for a in addr_dw[16 * g:16 * g + 16])
        cyc += max(c.values())
    return cyc


def read_cycles(addr_dw):
    """addr_dw: 64 dword addresses of one ds_read_b128 (16-byte aligned) -> cycles (16-lane groups, 64 banks)"""
    cyc = 0
    for g in range(4):
        c = Counter()
        for a in addr_dw[16 * g:16 * g + 16]:
            for k in range(4):
                c[(a + k) % 64] += 1
        cyc += max(c.values())
    return cyc


def layout(stride, rot, d):
    """double offset of value j of lane l's row block"""
    def at(l, j):
        jj = (j + (2 * (l % 8) if rot else 0)) % 36
        return stride * l + jj + d
    return at


def main():
    RB = 36
    print("P1 tile image, 64 lanes x %d doubles; cycles per instruction (ideal: 4 per 64-lane instruction)" % RB)
    for name, stride, rot in (("production (stride 36)", 36, False), ("padded (stride 37)", 37, False),
                              ("rotated slots (stride 36, 2 (l mod 8))", 36, True)):
        for d in (0, 1):
            at = layout(stride, rot, d)
            w = [write_cycles([2 * at(l, j) for l in range(64)]) for j in range(RB)]
            # reader: 16-byte chunk c of the tile's CSR range = values 2c, 2c + 1 (CSR order = lane-major, value-minor)
            r = []
            for k in range(18):
                addrs = []
                for l in range(64):
                    c = l + 64 * k
                    v0 = 2 * c - d if d else 2 * c          # (d = 1: the odd first value is stored alone)
                    lane, j = divmod(max(v0, 0), RB)
                    a = at(min(lane, 63), j)
                    addrs.append(2 * (a - a % 2))           # the 16-byte aligned pair holding it
                r.append(read_cycles(addrs))
            aligned = all(at(l, j) % 2 == (j + d) % 2 for l in range(64) for j in range(RB))
            print("  %-42s d=%d  writes %.2f (x36)  reads %.2f (x18)  per tile %4d cycles  reader pairs contiguous: %s"
                  % (name, d, sum(w) / len(w), sum(r) / len(r), sum(w) + sum(r),
                     "yes" if (stride == 36 and not rot) else "no (needs per-value gathers)"))


if __name__ == "__main__":
    main()
