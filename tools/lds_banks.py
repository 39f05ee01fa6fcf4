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
