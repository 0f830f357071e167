"""The ePIE object update and pupil numerator (fpmMain.cpp:405-471) exactly as
the fused kernels evaluate them -- update.hpp slot_update, the one function
every fused kernel calls, run through include/fpm_hip_debug.h
fpm_debug_slot_update -- and the general path's coefficient (fpm_state.hpp
upd_coef_div through fpm_debug_update_coef), against float64 numpy.

With D = F - O P:
  O' = O + D conj(P) |P| / ((|P|^2 + delta2 + i d2im) max|P|)
  num = D conj(O) |O| / (|O|^2 + delta1 + i d1im)
(d1im / d2im = delta1 / delta2: OpenCV's scalar unrolling; 0 in
the re-only reading).  The kernels take the complex reciprocal scale-safely:
with a = |X|^2 + delta and q = c / a, (1 - iq) / (a (1 + q^2) m).  Round 2's
(a - ic) / ((a^2 + c^2) m) squared a, i.e. |O|^4, which overflows fp32 once
|O| ~ 3e9 (a ~ 1e19); no valid uint16 stack reaches that (|objF| <=
Np^2 max sqrt(I) ~ 2.7e8 at Np 1024), so it is pinned here on synthetic
inputs up to |O| = 1e15, a = 1e30."""
import ctypes as C

import numpy as np
import pytest

import fpm_amd

pytestmark = pytest.mark.gpu

fp = C.POINTER(C.c_float)


def _c(x):
    return np.ascontiguousarray(np.stack([x.real, x.imag], -1).astype(np.float32))


def _slot_update(f, o, p, pm, d1, d2, d1im, d2im):
    lib = fpm_amd.load_library()
    fn = lib.fpm_debug_slot_update
    fn.argtypes = [fp, fp, fp, fp, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, fp, fp, fp]
    n = len(f)
    fa, oa_, pa = _c(f), _c(o), _c(p)
    pma = np.ascontiguousarray(pm, dtype=np.float32)
    nv = np.zeros((n, 2), np.float32)
    num = np.zeros((n, 2), np.float32)
    oa = np.zeros(n, np.float32)
    rc = fn(*[x.ctypes.data_as(fp) for x in (fa, oa_, pa, pma)], n, d1, d2, d1im, d2im,
            *[x.ctypes.data_as(fp) for x in (nv, num, oa)])
    assert rc == 0, lib.fpm_last_error()
    as64 = lambda x: x[:, 0].astype(np.float64) + 1j * x[:, 1].astype(np.float64)  # noqa: E731
    return as64(nv), as64(num), oa.astype(np.float64)


def _logmag(rng, n, lo, hi):
    return 10.0 ** rng.uniform(lo, hi, n) * np.exp(1j * rng.uniform(-np.pi, np.pi, n))


@pytest.mark.parametrize("all_channels", [True, False], ids=["complex_denominators", "re_only"])
def test_slot_update_matches_float64_up_to_1e30(all_channels):
    rng = np.random.default_rng(3)
    n = 4096
    # one of |O|, |P| up to 1e15 (|X|^2 + delta up to 1e30), the other <= 1e3,
    # so the products D conj(P), D conj(O) stay inside fp32 (as any real stack's do)
    h = n // 2
    o = np.concatenate([_logmag(rng, h, -3, 15), _logmag(rng, n - h, -3, 3)])
    p = np.concatenate([_logmag(rng, h, -3, 3), _logmag(rng, n - h, -3, 15)])
    # |F| of the order of |O P| (no cancellation in D), max|P| >= |P|
    f = o * p * _logmag(rng, n, -0.5, 0.5)
    pm = np.abs(p) * 10.0 ** rng.uniform(0, 2, n)
    d1, d2 = 10.0, 3.0
    d1im, d2im = (d1, d2) if all_channels else (0.0, 0.0)
    # the float32 inputs the kernel sees
    o, p, f = (np.complex128(np.complex64(x)) for x in (o, p, f))
    pm = pm.astype(np.float32).astype(np.float64)
    nv, num, oa = _slot_update(f, o, p, pm, d1, d2, d1im, d2im)
    D = f - o * p
    dO = D * np.conj(p) * np.abs(p) / ((np.abs(p) ** 2 + d2 + 1j * d2im) * pm)
    ref_nv = o + dO
    ref_num = D * np.conj(o) * np.abs(o) / (np.abs(o) ** 2 + d1 + 1j * d1im)
    assert np.isfinite(nv).all() and np.isfinite(num).all()
    # nv = fl(O + dO): an error of a few ulp of the larger term
    scale = np.abs(o) + np.abs(dO)
    assert (np.abs(nv - ref_nv) / scale).max() < 4e-6
    assert (np.abs(num - ref_num) / np.abs(ref_num)).max() < 4e-6
    assert (np.abs(oa - np.abs(o)) / np.abs(o)).max() < 1e-6
    big = np.maximum(np.abs(o), np.abs(p)) ** 2
    assert (big > 1e20).sum() > 400  # the range round 2's squared form overflowed


def test_general_path_update_coefficient():
    lib = fpm_amd.load_library()
    fn = lib.fpm_debug_update_coef
    fn.argtypes = [fp, fp, fp, fp, fp, C.c_int]
    rng = np.random.default_rng(3)
    a = np.concatenate([10.0 ** np.linspace(-3, 30, 200), rng.uniform(1, 1e6, 56)])
    c = np.where(np.arange(a.size) % 2 == 0, 5.0, 0.0)      # delta im part, and the re-only reading
    m = 10.0 ** rng.uniform(0, 7, a.size)                    # max|P| / max|objF| factor
    f = 10.0 ** rng.uniform(0, 15, a.size)                   # |P| / |O|
    arrs = [np.ascontiguousarray(x, dtype=np.float32) for x in (a, c, m, f)]
    out = np.zeros(2 * len(a), dtype=np.float32)
    assert fn(*[x.ctypes.data_as(fp) for x in arrs], out.ctypes.data_as(fp), len(a)) == 0
    got = out[0::2].astype(np.float64) + 1j * out[1::2].astype(np.float64)
    a32, c32, m32, f32 = (x.astype(np.float64) for x in arrs)
    ref = f32 / ((a32 + 1j * c32) * m32)
    ok = np.isfinite(ref) & (np.abs(ref) > 1e-36)            # fp32 normal range of the result
    assert np.isfinite(got[ok]).all()
    rel = np.abs(got[ok] - ref[ok]) / np.abs(ref[ok])
    assert rel.max() < 4e-6, (rel.max(), a[ok][np.argmax(rel)])
    assert (a[ok] > 1e20).sum() > 20
