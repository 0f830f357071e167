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


def sites(xt, xp, tld, w=1):
    """(kind, byte addresses, repeat) of the wave's LDS instructions per LED.
    xt: exchange-tile stride per group (complex), xp: exchange row pitch
    (complex), tld: T row pitch (complex).  Wave w (groups 6w..6w+5)."""
    L = lanes()
    tiles = 0
    th = NW * GPW * xt  # T after the tiles (complex)
    rowoff = [(fold(y) + R) * tld if -R <= fold(y) <= R else NB * tld for y in range(NP)]
    out = []

    def addr(f):
        return [None if x is None else 8 * f(*x) for x in L]

    def gidx(gw):
        return w * GPW + gw

    # exchange: write rows m (9 or 10), read lane's row l
    for nrows, nread in ((9, 5), (10, 4)):  # ab: 9 rows written, 10 read (5 x b128); ba: 10 written, 9 read
        for m in range(nrows):
            out.append(("write_b64", addr(lambda gw, l: tiles + gidx(gw) * xt + m * xp + l), 1))
        for i in range(nread):
            out.append(("read_b128", addr(lambda gw, l: tiles + gidx(gw) * xt + l * xp + 2 * i), 1))
        if nread == 4:
            out.append(("read_b64", addr(lambda gw, l: tiles + gidx(gw) * xt + l * xp + 8), 1))
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


def report(xt, xp, tld):
    res = []
    for w in range(NW):
        ex, tl = sites(xt, xp, tld, w)
        res.append((total(ex), total(tl)))
    ce = sum(r[0][0] for r in res)
    ie = sum(r[0][1] for r in res)
    ct = sum(r[1][0] for r in res)
    it = sum(r[1][1] for r in res)
    return ce, ie, ct, it


if __name__ == "__main__":
    ce, ie, ct, it = report(100, 10, 91)
    print(f"current xt 100 xp 10 tld 91: exchange {ce} cyc (ideal {ie}, {1 - ie / ce:.2f} conflict), "
          f"T {ct} (ideal {it}, {1 - it / ct:.2f}); total share {(ce + ct - ie - it) / (ce + ct):.2f}")
    best = []
    for xp in (10, 11, 12):
        for xt in range(10 * xp, 10 * xp + 40, 2):
            ce, ie, ct, it = report(xt, xp, 91)
            best.append((ce, xt, xp, ie))
    best.sort()
    for ce, xt, xp, ie in best[:8]:
        print(f"exchange xt {xt} xp {xp}: {ce} cyc (ideal {ie})")
    bt = []
    for tld in range(91, 110):
        ce, ie, ct, it = report(100, 10, tld)
        bt.append((ct, tld, it))
    bt.sort()
    for ct, tld, it in bt[:6]:
        print(f"T tld {tld}: {ct} cyc (ideal {it})")
