"""LDS bank-conflict model of k_fir_pfft's accesses (MI355X_MICROARCH.md §LDS): per instruction,
the LDS array cycles = sum over its lane groups of the largest number of distinct entries on one
bank (pair). Models (8-B entries):
  ds_read_b64                 2 groups of 32 lanes, bank pair = entry mod 32
  ds_read2_b64, ds_write_b64, ds_write2_b64   4 groups of 16 contiguous lanes, entry mod 16
Checks the exchange layouts e1/e2 and the ring stores (with and without the slot permutation
row_slot), and searches additive paddings e(i) = i + sum_k c_k (i >> k) for exchange 1.
Usage: python tools/probe/lds_banks.py  (CPU only)"""
import itertools

import numpy as np

J = np.arange(64)


def cycles(e, kind):
    e = np.asarray(e)
    if kind == "rd64":
        groups = [e[:32] % 32, e[32:] % 32]
    else:
        groups = [e[k * 16:(k + 1) * 16] % 16 for k in range(4)]
    return int(sum(np.bincount(g).max() for g in groups)), len(groups)


def exchange(e, store_idx, kind_rd):
    """(store cycles, ideal), (load cycles, ideal) over r = 0..7; loads at j + 64 r."""
    st = [cycles(e(store_idx(r)), "wr") for r in range(8)]
    ld = [cycles(e(J + 64 * r), kind_rd) for r in range(8)]
    return (sum(c for c, _ in st), sum(n for _, n in st)), (sum(c for c, _ in ld), sum(n for _, n in ld))


X1 = lambda r: 8 * J + r                                  # pass-1 stores
X2 = lambda r: 64 * (J >> 3) + (J & 7) + 8 * r            # pass-2 stores
E1_OLD = lambda i: i + (i >> 5)
E1 = lambda i: i + (i >> 4)
E2 = lambda i: i + 3 * (i >> 5) + 2 * (i >> 6)


def row_slot(l, P):
    g = l >> 4
    if P == 16:
        return (4 * (g >> 1) + (g & 1) + 2 * ((l >> 3) & 1)) * 8 + (l & 7)
    h = (l >> 2) & 3
    return (8 * (g >> 1) + 2 * (g & 1) + (h & 1) + 4 * (h >> 1)) * 4 + (l & 3)


def ring_stores(P, perm):
    sw = lambda s: (s // (32 // P)) & (P - 1)
    tot = ideal = 0
    for base in range(0, 512, 7):
        for w in range(P):
            pos = np.array([w * 64 + (row_slot(l, P) if perm else l) for l in range(64)])
            s = (base + (2 * pos) // P) % 512
            ph = (2 * pos) % P
            for off in (0, 1):
                c, n = cycles(s * P + ((ph + off) ^ sw(s)), "wr")
                tot += c
                ideal += n
    return tot, ideal


if __name__ == "__main__":
    for name, e, st in (("e1 old", E1_OLD, X1), ("e1", E1, X1), ("e2", E2, X2)):
        for kind in ("rd2", "rd64"):
            print(name, "loads as", kind, "stores/ideal, loads/ideal:", exchange(e, st, kind))
    for P in (16, 8):
        print("ring stores P=%d wave order" % P, ring_stores(P, False), "row_slot", ring_stores(P, True))
    best = []
    for c in itertools.product(range(9), range(9), range(9), range(5)):
        e = lambda i, c=c: i + c[0] * (i >> 3) + c[1] * (i >> 4) + c[2] * (i >> 5) + c[3] * (i >> 6)
        (sc, si), (lc, li) = exchange(e, X1, "rd2")
        if sc == si and lc == li:
            best.append((int(e(np.arange(512)).max()), c))
    print("exchange-1 paddings conflict-free with read2 loads (max index, (c3, c4, c5, c6)):", sorted(best)[:4])
