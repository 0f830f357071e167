"""The ePIE update coefficient f / ((a + i c) m) (fpmMain.cpp:417-419 object,
:469-471 pupil numerator; a = |X|^2 + delta, c = the imaginary part OpenCV's
scalar unrolling adds) as the kernels evaluate it
(include/fpm_hip_debug.h fpm_debug_update_coef), against float64 numpy.

The kernels form it scale-safely: with q = c / a, (1 - iq) / (a (1 + q^2) m).
Round 2's (a - ic) / ((a^2 + c^2) m) squared a = |O|^2 + delta1, i.e. |O|^4,
which overflows fp32 once |O| ~ 3e9 (a ~ 1e19); no valid uint16 stack reaches
that (|objF| <= Np^2 max sqrt(I) ~ 2.7e8 at Np 1024), so it is pinned here on
synthetic inputs up to a = 1e30."""
import ctypes as C

import numpy as np
import pytest

import fpm_amd

pytestmark = pytest.mark.gpu


def _coef(a, c, m, f, form):
    lib = fpm_amd.load_library()
    fn = lib.fpm_debug_update_coef
    fp = C.POINTER(C.c_float)
    fn.argtypes = [fp, fp, fp, fp, fp, C.c_int, C.c_int]
    arrs = [np.ascontiguousarray(x, dtype=np.float32) for x in (a, c, m, f)]
    out = np.zeros(2 * len(a), dtype=np.float32)
    rc = fn(*[x.ctypes.data_as(fp) for x in arrs], out.ctypes.data_as(fp), len(a), form)
    assert rc == 0, fpm_amd.load_library().fpm_last_error()
    return out[0::2].astype(np.float64) + 1j * out[1::2].astype(np.float64)


def _case():
    rng = np.random.default_rng(3)
    a = np.concatenate([10.0 ** np.linspace(-3, 30, 200), rng.uniform(1, 1e6, 56)])
    c = np.where(np.arange(a.size) % 2 == 0, 5.0, 0.0)      # delta im part, and the re-only reading
    m = 10.0 ** rng.uniform(0, 7, a.size)                    # max|P| / max|objF| factor
    f = 10.0 ** rng.uniform(0, 15, a.size)                   # |P| / |O|
    return a, c, m, f


@pytest.mark.parametrize("form", [0, 1, 2], ids=["fused_upd_coef_safe", "upd_coef", "upd_coef_div"])
def test_update_coefficient_scale_safe(form):
    a, c, m, f = _case()
    if form:  # upd_coef / upd_coef_div return the coefficient; their callers apply |X|
        f = np.ones_like(f)
    a32, c32, m32, f32 = (x.astype(np.float32).astype(np.float64) for x in (a, c, m, f))
    ref = f32 / ((a32 + 1j * c32) * m32)
    got = _coef(a, c, m, f, form)
    ok = np.isfinite(ref) & (np.abs(ref) > 1e-36)            # fp32 normal range of the result
    assert np.isfinite(got[ok]).all()
    rel = np.abs(got[ok] - ref[ok]) / np.abs(ref[ok])
    assert rel.max() < 4e-6, (form, rel.max(), a[ok][np.argmax(rel)])
    assert (a[ok] > 1e20).sum() > 20                          # the range round 2 overflowed
