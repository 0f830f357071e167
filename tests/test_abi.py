"""The C-ABI libraries load and export every symbol their headers declare;
argument validation fails loudly with the documented codes.  CPU only: no
compute call is made without a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import fpm_amd
from fpm_amd import host

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    return set(re.findall(r"\b(fpm_\w+)\s*\(", text))


@pytest.mark.parametrize("header,lib", [("fpm_hip.h", fpm_amd.HIP_LIB), ("fpm_hip_debug.h", fpm_amd.HIP_LIB),
                                        ("fpm_host.h", fpm_amd.HOST_LIB)])
def test_library_exports_every_declared_symbol(header, lib):
    names = _declared(header)
    assert names, header
    so = C.CDLL(lib)
    missing = [n for n in sorted(names) if not hasattr(so, n)]
    assert not missing, missing


def test_python_mirror_covers_header():
    assert _declared("fpm_hip.h") == set(fpm_amd.HIP_SYMBOLS)
    assert _declared("fpm_hip_debug.h") == set(fpm_amd.HIP_DEBUG_SYMBOLS)
    assert _declared("fpm_host.h") == set(host.HOST_SYMBOLS)


def test_version_string():
    assert b"gfx950" in fpm_amd.load_library().fpm_version()


@pytest.mark.parametrize("change,match", [
    (dict(np_=33), "even"),
    (dict(np_=14, L=42), "2\\^a 3\\^b 5\\^c"),
    (dict(radius=20), "2r\\+1"),
    (dict(delta2=0.0), "delta2"),
    (dict(x0=np.array([0, 200])), "leaves"),
])
def test_create_rejects_bad_problems(change, match):
    base = dict(np_=32, L=96, order=[0, 1], x0=np.array([32, 30]), y0=np.array([32, 34]), radius=6,
                delta1=5, delta2=10)
    base.update(change)
    with pytest.raises(fpm_amd.FpmError, match=match) as e:
        fpm_amd.Solver(fpm_amd.Problem(**base))
    assert e.value.code == fpm_amd.FPM_ERR_INVAL


def test_flag_and_path_constants_match_header():
    text = open(os.path.join(ROOT, "include", "fpm_hip.h")).read()
    defs = dict(re.findall(r"#define\s+(FPM_(?:FLAG|PATH)_\w+)\s+(\d+)u?", text))
    assert int(defs["FPM_FLAG_OBJCROP_LAST_ONLY"]) == fpm_amd.FLAG_OBJCROP_LAST_ONLY
    assert int(defs["FPM_FLAG_SPEC_FP16"]) == fpm_amd.FLAG_SPEC_FP16
    assert (int(defs["FPM_PATH_AUTO"]), int(defs["FPM_PATH_GENERAL"]), int(defs["FPM_PATH_FUSED"])) == \
        (fpm_amd.PATH_AUTO, fpm_amd.PATH_GENERAL, fpm_amd.PATH_FUSED)
    kern = dict(re.findall(r"#define\s+FPM_KERNEL_(\w+)\s+(\d+)", text))
    assert {k: int(v) for k, v in kern.items()} == {
        "GENERAL": fpm_amd.KERNEL_GENERAL, "FUSED_NP256": fpm_amd.KERNEL_FUSED_NP256,
        "FUSED_NP200": fpm_amd.KERNEL_FUSED_NP200, "FUSED_SMALL": fpm_amd.KERNEL_FUSED_SMALL,
        "FUSED_NP256_DIST": fpm_amd.KERNEL_FUSED_NP256_DIST, "FUSED_NP90": fpm_amd.KERNEL_FUSED_NP90}
