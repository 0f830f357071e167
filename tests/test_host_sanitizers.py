"""The host front-end (JSON reader, geometry, LED order, loader, TIFF reader:
fpm-opencv_amd/host/*.cpp) built with AddressSanitizer + UndefinedBehavior-
Sanitizer and driven over well-formed and malformed inputs (SURVEY.md §5:
sanitizer builds of the CPU side).  CPU only; the GPU kernels are not part of
this build (GPU ASan is not available on the pool)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from dataset_fixture import make_dataset
from fpm_amd import host

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "fpm-opencv_amd", "host")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "host_driver")
    srcs = [os.path.join(HOST, f) for f in sorted(os.listdir(HOST)) if f.endswith(".cpp") and f != "fpmMain.cpp"]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"), "-I", HOST,
           os.path.join(ROOT, "tests", "sanitize", "host_driver.cpp"), *srcs, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


def _run(driver, mode, files):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([driver, mode, *files], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "ERROR" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert f"host_driver ok {len(files)} files" in r.stdout


def _json_variants(base_text):
    """The reference-schema text plus truncations, trailing garbage, deleted
    keys and numeric edge cases (jsoncpp 1.6.5 recovery paths)."""
    v = [base_text, base_text[: len(base_text) // 2], base_text[:17], base_text + "}}}]]",
         base_text.replace("holeCoordinates", "holeCoordinatez"),
         base_text.replace('"cropSizeX" : 32', '"cropSizeX" : 1e9'),
         base_text.replace('"cropSizeX" : 32', '"cropSizeX" : -4'),
         base_text.replace('"lambda" : 0.6292', '"lambda" : 0'),
         base_text.replace(",", ",,", 5), "", "{", "[1,2,3]", '{"cropSizeX": "x"}',
         '{"a": "\\u12"}', '{"a": 1.7976931348623157e309}', "\x00\xff{" * 50]
    return v


def test_json_geometry_loader_under_asan_ubsan(driver, tmp_path):
    ds = make_dataset(str(tmp_path / "ds"))
    base = open(ds["json"]).read()
    files = []
    for i, text in enumerate(_json_variants(base)):
        p = tmp_path / f"v{i}.json"
        p.write_bytes(text.encode("latin-1", "replace"))
        files.append(str(p))
    _run(driver, "json", files)


def test_tiff_reader_under_asan_ubsan(driver, tmp_path):
    rng = np.random.default_rng(3)
    good = tmp_path / "good.tif"
    host.write_tiff16(str(good), rng.integers(0, 65535, (40, 52)).astype(np.uint16))
    raw = good.read_bytes()
    files = [str(good)]
    cases = [raw[:8], raw[: len(raw) // 2], raw[:-3], b"II*\x00" + b"\xff" * 64, b"MM\x00*" + raw[4:],
             raw[:4] + (2 ** 31).to_bytes(4, "little") + raw[8:], b"", os.urandom(512)]
    big = tmp_path / "big.tif"   # more pixels than the driver's buffer
    host.write_tiff16(str(big), rng.integers(0, 65535, (300, 300)).astype(np.uint16))
    files.append(str(big))
    for i, c in enumerate(cases):
        p = tmp_path / f"t{i}.tif"
        p.write_bytes(c)
        files.append(str(p))
    _run(driver, "tiff", files)
