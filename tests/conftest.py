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
