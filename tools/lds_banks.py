"""Bank-conflict count of solve2_kernel's LDS accesses (dev tool; see solve2_kernel.h).

ds_read_b32 / ds_write_b32 are serviced in two 32-lane groups, bank = dword index mod 32,
identical addresses broadcast (MI355X_MICROARCH.md, LDS).  One half of the wave = one group.
Prints the extra LDS cycles per round for the row-major unit order and for the digit-class
order of G(r,c) = (3(r%3) + 2(r/3) + c) mod 9 that the kernel uses.
"""


def unit_cells(j):
    if j < 9:
        return [9 * j + q for q in range(9)]
    if j < 18:
        return [9 * q + (j - 9) for q in range(9)]
    b = j - 18
    return [((b // 3) * 3 + q // 3) * 9 + (b % 3) * 3 + q % 3 for q in range(9)]


def G(cell):
    r, c = divmod(cell, 9)
    return (3 * (r % 3) + 2 * (r // 3) + c) % 9


def extra_cycles(addrs):
    """Extra cycles of one 32-lane group: max distinct addresses on one bank, minus 1."""
    banks = {}
    for a in set(addrs):
        banks.setdefault(a % 32, set()).add(a)
    return max(len(v) for v in banks.values()) - 1


def reads(order):
    total = 0
    for k in range(9):
        addrs = []
        for lane in range(32):
            j = lane if lane < 27 else 0          # spare lanes mirror lane 0
            addrs.append(order(j)[k])
        total += extra_cycles(addrs)
    return total


def main():
    rowmajor = unit_cells
    digit = lambda j: sorted(unit_cells(j), key=G)
    # the kernel's spare lanes used to read cells 81+k (row-major build)
    print("unit reads, row-major order : extra cycles per round =", reads(rowmajor))
    print("unit reads, digit-class order: extra cycles per round =", reads(digit))
    for d in range(9):
        cells = [c for c in range(81) if G(c) == d]
        assert len({c % 32 for c in cells}) == 9, d
    print("every digit class of G occupies 9 distinct banks: ok")


if __name__ == "__main__":
    main()


# ------------------------------------------------------------------ solve4_kernel
# 8-byte (X, S) words.  ds_read_b64: 2 x 32-lane groups, bank = dword mod 64, a lane uses 2 banks.
# ds_write_b64 (and each half of ds_read2/write2_b64): 4 x 16 contiguous lanes, bank = dword mod 32.
def extra_b64(slots, groups, banks):
    """Extra LDS cycles of one b64 access: per lane group, max distinct addresses on a bank - 1."""
    total = 0
    for g in groups:
        per = {}
        for s in {slots[l] for l in g}:
            for dw in (2 * s, 2 * s + 1):
                per.setdefault(dw % banks, set()).add(s)
        total += max(len(v) for v in per.values()) - 1
    return total


R64 = [range(0, 32), range(32, 64)]
W64 = [range(0, 16), range(16, 32), range(32, 48), range(48, 64)]


def solve4_round():
    digit = lambda j: sorted(unit_cells(j), key=G)
    half_base = lambda lane: (lane >> 5) * 150
    hl = lambda lane: lane & 31
    act = lambda lane: hl(lane) < 27
    c0 = lambda lane: hl(lane) if act(lane) else 91 + hl(lane) - 27
    rep = {}
    for k in range(3):                                        # cell stores
        rep[f"cell store +{27 * k}"] = extra_b64([half_base(l) + c0(l) + 27 * k for l in range(64)], W64, 32)
    rep["gather reads"] = sum(extra_b64([half_base(l) + digit(hl(l) if act(l) else 0)[q] for l in range(64)],
                                        R64, 64) for q in range(9))
    ubase = lambda lane: 300 + (lane >> 5) * 32               # s_unit follows s_cell (2 x 150 slots)
    rep["unit store"] = extra_b64([ubase(l) + hl(l) for l in range(64)], W64, 32)
    j = lambda lane: hl(lane) if act(lane) else 0
    reads = {"ucol": lambda l: 9 + j(l) % 9}
    for k in range(3):
        reads[f"row+{3 * k}"] = lambda l, k=k: j(l) // 9 + 3 * k
        reads[f"box+{3 * k}"] = lambda l, k=k: 18 + (j(l) % 9) // 3 + 3 * k
    for name, f in reads.items():
        rep[f"unit read {name}"] = extra_b64([ubase(l) + f(l) for l in range(64)], R64, 64)
    return rep


if __name__ == "__main__":
    print("solve4_kernel, extra LDS cycles per round (b64 model):")
    for k, v in solve4_round().items():
        print(f"  {k:20s} {v}")
