#!/usr/bin/env python3
"""LDS bank-conflict model of one LED step of k_fused_s90 (fused_s90.hip,
dft90.hpp) for a choice of exchange-tile stride / row pitch and T row pitch,
using the gfx950 lane-group table of tools/lds_banks.py.

  python3 tools/lds_s90.py            # current layout and a search over pitches
"""
import itertools
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lds_banks import total  # noqa: E402

NP, N2, GPW, NW = 90, 10, 6, 16
R = 30
NB = 2 * R + 1


def fold(n):
    return n if n < NP // 2 else n - NP


def lanes():
    """per lane of a wave: (group-in-wave, lane-in-group) or None"""
    out = []
    for ln in range(64):
        gw = ln // N2
        out.append((gw, ln - N2 * gw) if gw < GPW else None)
    return out


DENSE = (600, [100 * g for g in range(6)], 91)
FAST = (704, [0, 122, 230, 356, 478, 602], 106)  # fused_s90.hip XW_FAST / XG_FAST / TLD_FAST


def sites(xw, xg, tld, w=1, xp=10):
    """(kind, byte addresses, repeat) of the wave's LDS instructions per LED.
    xw: wave slot of the exchange tiles, xg: tile offset of each group in it,
    xp: exchange row pitch, tld: T row pitch (all complex).  Wave w."""
    L = lanes()
    th = NW * xw  # T after the tiles (complex)
    rowoff = [(fold(y) + R) * tld if -R <= fold(y) <= R else NB * tld for y in range(NP)]
    out = []

    def addr(f):
        return [None if x is None else 8 * f(*x) for x in L]

    def gidx(gw):
        return w * GPW + gw

    def tb(gw):
        return w * xw + xg[gw]

    # exchange: write rows m (9 or 10), read lane's row l
    for nrows, nread in ((9, 5), (10, 4)):  # ab: 9 rows written, 10 read (5 x b128); ba: 10 written, 9 read
        for m in range(nrows):
            out.append(("write_b64", addr(lambda gw, l: tb(gw) + m * xp + l), 1))
        for i in range(nread):
            out.append(("read_b128", addr(lambda gw, l: tb(gw) + l * xp + 2 * i), 1))
        if nread == 4:
            out.append(("read_b64", addr(lambda gw, l: tb(gw) + l * xp + 8), 1))
    # each LED runs ab twice (A, B) and ba twice (B, C)
    ex = [(k, a, 2) for k, a, _ in out]
    # T: A writes row g: th[g tld + l + 9 m], l < 9
    tl = []
    for m in range(10):
        tl.append(("write_b64", [None if x is None or x[1] >= 9 else 8 * (th + gidx(x[0]) * tld + x[1] + 9 * m) for x in L], 1))
    # B reads / writes column g at rows rowoff[l + 10 k]
    for k in range(9):
        tl.append(("read_b64", [None if x is None else 8 * (th + rowoff[x[1] + 10 * k] + gidx(x[0])) for x in L], 2))
    # C reads row g like A writes it
    for m in range(10):
        tl.append(("read_b64", [None if x is None or x[1] >= 9 else 8 * (th + gidx(x[0]) * tld + x[1] + 9 * m) for x in L], 1))
    # numerators: th[g tld + k 10 + l] written and read
    for k in range(9):
        tl.append(("write_b64", addr(lambda gw, l: th + gidx(gw) * tld + 10 * k + l), 1))
        tl.append(("read_b64", addr(lambda gw, l: th + gidx(gw) * tld + 10 * k + l), 1))
    return ex, tl


def report(xw, xg, tld):
    ce = ie = ct = it = 0
    for w in range(NW):
        ex, tl = sites(xw, xg, tld, w)
        a, b, _ = total(ex)
        c, d, _ = total(tl)
        ce, ie, ct, it = ce + a, ie + b, ct + c, it + d
    return ce, ie, ct, it


if __name__ == "__main__":
    for name, lay in (("dense", DENSE), ("fast", FAST)):
        ce, ie, ct, it = report(*lay)
        print(f"{name} {lay}: exchange {ce} LDS cycles (conflict-free {ie}), T {ct} ({it}); "
              f"conflict share {(ce + ct - ie - it) / (ce + ct):.2f}")
