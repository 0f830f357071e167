"""libfpm_hip.so in a process WITHOUT torch (ROCm 7.2 runtime from
/opt/rocm, like the fpmMain CLI) -- the pytest process itself runs on torch's
bundled runtime (conftest.py), so this case runs in a child process."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path[:0] = [%r, %r, %r]
import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import grid_geometry, make_stack
assert 'torch' not in sys.modules
Np, L, r = 32, 96, 6
x0, y0, order = grid_geometry(Np, L, 5, 4)
st = make_stack(Np, L, r, x0, y0, n_patch=1, seed=4)
import oracle_lib
ref = oracle_lib.run_fpm(st[:, 0], order, x0, y0, Np, L, r, 5, 10, 2)
out = fpm_amd.run_fpm(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10), st, 2)
e = rel_l2(out['objCrop'][0], ref['objCrop'])
assert e < 5e-5, e
print('OK', e)
""" % (ROOT, os.path.join(ROOT, "fpm-opencv_amd", "python"), os.path.join(ROOT, "oracle"))


def test_library_without_torch():
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "tests"))
    p = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "OK" in p.stdout
