"""ctypes loader for oracle/liboracle.so (the C++ fp64 restatement).
Test infrastructure: used by tests/, smoke() and bench.py's cpu_baseline."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
        lib = C.CDLL(ORACLE_SO)
        ip, dp, u16p = C.POINTER(C.c_int), C.POINTER(C.c_double), C.POINTER(C.c_uint16)
        lib.oracle_run_fpm.argtypes = [C.c_int, C.c_int, C.c_int, u16p, C.c_int, ip, ip, ip, C.c_int,
                                       C.c_double, C.c_double, C.c_double, C.c_int, C.c_int, dp, dp, dp]
        lib.oracle_run_fpm_batch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, u16p, C.c_int, ip, ip, ip,
                                             C.c_int, C.c_double, C.c_double, C.c_double, C.c_int, C.c_int,
                                             C.c_int, dp, dp, dp]
        lib.oracle_fft2.argtypes = [dp, C.c_int, C.c_int, C.c_int]
        _lib = lib
    return _lib


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int))


def run_fpm(stack, order, x0, y0, np_, L, r, d1, d2, iters, eps=float(np.float32(1e-10)), all_channels=True):
    """One patch; stack uint16 [n_stack][Np][Np]. Returns complex128 outputs.
    all_channels=False restates FPM_FLAG_SCALAR_RE_ONLY (fpm_oracle.cpp header)."""
    lib = load()
    st = np.ascontiguousarray(stack, np.uint16)
    order, x0, y0 = (np.ascontiguousarray(v, np.int32) for v in (order, x0, y0))
    objF = np.zeros((L, L), np.complex128)
    objCrop = np.zeros((L, L), np.complex128)
    pupil = np.zeros((np_, np_), np.complex128)
    dp = C.POINTER(C.c_double)
    rc = lib.oracle_run_fpm(np_, L, len(x0), st.ctypes.data_as(C.POINTER(C.c_uint16)), len(order), _ip(order),
                            _ip(x0), _ip(y0), r, d1, d2, eps, iters, int(all_channels), objF.ctypes.data_as(dp),
                            objCrop.ctypes.data_as(dp), pupil.ctypes.data_as(dp))
    assert rc == 0, rc
    return dict(objF=objF, objCrop=objCrop, pupil=pupil)


def run_fpm_batch(stack, order, x0, y0, np_, L, r, d1, d2, iters, threads, outputs=True,
                  eps=float(np.float32(1e-10)), all_channels=True, pupil=False, objF=False):
    """stack uint16 [n_stack][B][Np][Np]; B patches on `threads` threads.
    Returns objCrop [B][L][L] (None when outputs=False), or with pupil=True
    (objF=True) a dict of objCrop and pupil [B][Np][Np] (centred, like
    run_fpm) (and objF [B][L][L])."""
    lib = load()
    st = np.ascontiguousarray(stack, np.uint16)
    B = st.shape[1]
    order, x0, y0 = (np.ascontiguousarray(v, np.int32) for v in (order, x0, y0))
    dp = C.POINTER(C.c_double)
    objCrop = np.zeros((B, L, L), np.complex128) if outputs else None
    pupil = pupil or objF
    pup = np.zeros((B, np_, np_), np.complex128) if (outputs and pupil) else None
    oF = np.zeros((B, L, L), np.complex128) if (outputs and objF) else None
    rc = lib.oracle_run_fpm_batch(np_, L, len(x0), B, st.ctypes.data_as(C.POINTER(C.c_uint16)), len(order),
                                  _ip(order), _ip(x0), _ip(y0), r, d1, d2, eps, iters, int(all_channels), threads,
                                  oF.ctypes.data_as(dp) if oF is not None else None,
                                  objCrop.ctypes.data_as(dp) if outputs else None,
                                  pup.ctypes.data_as(dp) if pup is not None else None)
    assert rc == 0, rc
    if pupil and outputs:
        return dict(objCrop=objCrop, pupil=pup, **({"objF": oF} if objF else {}))
    return objCrop


def fft2(a, inverse=False):
    lib = load()
    b = np.ascontiguousarray(a, np.complex128).copy()
    rc = lib.oracle_fft2(b.ctypes.data_as(C.POINTER(C.c_double)), b.shape[0], b.shape[1], int(inverse))
    assert rc == 0
    return b
