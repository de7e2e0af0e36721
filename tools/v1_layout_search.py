"""LDS layout searches behind csrc/conv_v1r.hip (v_conv1, dense K).

1. A-fragment reads (compute waves): ds_read2_b32 per dword, lane groups of 32, bank = (addr / 4) % 32.
   Window copies: 10-byte pixels, row pitch RP, copy 1 shifted by 2 bytes at C1 (mod 128); group 15 reads the
   column-major frame-4 plane (column pitch CP, copies at P0 / P1 mod 128).  For every (RP, CP, P0, P1) the
   16 k-groups are paired (the two 16-lane k-groups sharing a 32-lane bank group) by an exact minimum-cost
   perfect matching; cost = sum over waves, blocks, dwords of the worst bank multiplicity.
   Result used: RP 208, C1 = P0 = P1 = 0 mod 128, CP 48, pairing V1_GMAP (cost 576 vs 512 conflict-free: only
   group 15's half-wave is 2-way).
2. Loader stores: each parity's 200 window pixels into 8 groups of 25 (one 32-lane ds_write group each),
   annealed so that the window-copy dword stores and the frame-4-plane b16 stores of a group have few distinct
   addresses per bank -> kLoaderPix (C++ table printed with --emit).

    python tools/v1_layout_search.py [--reads] [--loader [--emit]]
"""
import argparse
import random
import sys
from collections import defaultdict
from functools import lru_cache

RP, C1 = 208, 0


def pix(l, w, i):
    q, dy, dx = l >> 2, (l >> 1) & 1, l & 1
    return 4 * w + 2 * (q >> 1) + dy, 4 * i + 2 * (q & 1) + dx


def addr(g, py, px, CP, P0, P1):
    if g < 15:
        ky, r = g // 3, g % 3
        b = (py + ky) * RP + 10 * px + 16 * r
        return b if px % 2 == 0 else C1 + b - 2
    b = (px + 4) * CP + 2 * py
    return (P0 + b) if py % 2 == 0 else (P1 + b - 2)


def pair_cost(g1, g2, CP, P0, P1):
    tot = 0
    for w in range(4):
        for i in range(4):
            for d in range(4):
                A = [addr(g1, *pix(l, w, i), CP, P0, P1) + 4 * d for l in range(16)] + \
                    [addr(g2, *pix(l, w, i), CP, P0, P1) + 4 * d for l in range(16)]
                banks = defaultdict(set)
                for a in A:
                    banks[(a // 4) % 32].add(a)
                tot += max(len(v) for v in banks.values())
    return tot


def best_matching(cost):
    n = len(cost)

    @lru_cache(None)
    def f(mask):
        if mask == (1 << n) - 1:
            return (0, ())
        i = next(k for k in range(n) if not mask >> k & 1)
        best = None
        for j in range(i + 1, n):
            if not mask >> j & 1:
                c, m = f(mask | 1 << i | 1 << j)
                c += cost[i][j]
                if best is None or c < best[0]:
                    best = (c, ((i, j),) + m)
        return best
    return f(0)


def search_reads():
    wcost = [[pair_cost(a, b, 48, 0, 0) if a != b and a < 15 and b < 15 else 0 for b in range(16)] for a in range(16)]
    res = None
    for CP in range(48, 48 + 129, 4):
        for P0 in range(0, 128, 8):
            for P1 in range(0, 128, 8):
                cm = [row[:] for row in wcost]
                for g in range(15):
                    cm[g][15] = cm[15][g] = pair_cost(g, 15, CP, P0, P1)
                c, m = best_matching(cm)
                if res is None or c < res[0]:
                    res = (c, CP, P0, P1, m)
                    print(res, flush=True)
    return res


def search_loader(emit):
    def addr_a(wy, u, par):
        return wy * 52 + 5 * u + (2 if par else 0)   # window dword (copy 0)

    def addr_b(wy, u, par):
        return (2 * u + par) * 12 + (wy >> 1)        # frame-4 plane dword

    def gcost(g, par):
        c = 0
        for f in (addr_a, addr_b):
            banks = defaultdict(set)
            for (wy, u) in g:
                a = f(wy, u, par)
                banks[a % 32].add(a)
            c += max(len(v) for v in banks.values())
        return c

    random.seed(2)
    tables = []
    for par in (0, 1):
        px = [(wy, u) for wy in range(20) for u in range(10)]
        random.shuffle(px)
        groups = [px[i::8] for i in range(8)]
        cur = [gcost(g, par) for g in groups]
        T = 2.0
        for _ in range(600000):
            g1, g2 = random.sample(range(8), 2)
            i1, i2 = random.randrange(25), random.randrange(25)
            groups[g1][i1], groups[g2][i2] = groups[g2][i2], groups[g1][i1]
            n1, n2 = gcost(groups[g1], par), gcost(groups[g2], par)
            d = n1 + n2 - cur[g1] - cur[g2]
            if d <= 0 or random.random() < 2.718 ** (-d / T):
                cur[g1], cur[g2] = n1, n2
            else:
                groups[g1][i1], groups[g2][i2] = groups[g2][i2], groups[g1][i1]
            T = max(0.05, T * 0.99997)
        print("parity", par, "group costs (2 = conflict-free)", cur, file=sys.stderr)
        vals = []
        for g in groups:
            vals += [wy | ((2 * u + par) << 8) for wy, u in g] + [0xFFFF] * (32 - len(g))
        tables.append(vals)
    if emit:
        print("__device__ const unsigned short kLoaderPix[2][256] = {")
        for vals in tables:
            print("    {" + ", ".join(f"0x{v:04x}" for v in vals) + "},")
        print("};")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", action="store_true")
    ap.add_argument("--loader", action="store_true")
    ap.add_argument("--emit", action="store_true")
    a = ap.parse_args()
    if a.reads:
        search_reads()
    if a.loader:
        search_loader(a.emit)
