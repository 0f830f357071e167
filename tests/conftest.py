"""pytest configuration: the `gpu` marker and shared import paths.

`-m "not gpu"` runs on any CPU box (oracle vs golden vectors, host logic,
C-ABI symbol checks); `-m gpu` needs an MI355X and calls the HIP library
through its C ABI.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "fpm-opencv_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")

# Import torch (if present) before anything loads libfpm_hip.so: torch ships
# its own HIP/HSA runtime, and libfpm_hip.so then binds to that already-loaded
# libamdhip64.so.7 (same SONAME) -- the configuration bench.py runs in.  Two
# HIP runtimes in one process do not work (torch then sees no GPU).
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    pass
