"""Bit-identity of two builds of libfpm_hip.so on the same inputs (same-box
checks of changes that must not move a bit, e.g. a reduction rewritten with
DPP moves).  Each library runs in its own process (FPM_HIP_LIB is read at
import); the outputs are compared exactly.

usage: python tools/gpu/cmp_libs.py <lib_a.so> <lib_b.so>
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

CASES = [  # (name, environment): Np 256 metric-like geometry, r 33 (tail rows and tail pixels)
    ("one_workgroup", {"FPM_NO_DIST": "1", "FPM_NO_SPLIT": "1"}),
    ("split_ks2", {"FPM_NO_DIST": "1", "FPM_SPLIT": "2"}),
    ("dist_ks4", {"FPM_DIST": "4"}),
    ("dist_ks8", {"FPM_DIST": "8"}),
]

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, 'fpm-opencv_amd/python'); sys.path.insert(0, '.')
import fpm_amd
from tools.synth import grid_geometry, make_stack
Np, L, r = 256, 768, 33
x0, y0, order = grid_geometry(Np, L, 3, 60)
stack = make_stack(Np, L, r, x0, y0, n_patch=4, seed=7)
prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=4)
out = fpm_amd.run_fpm(prob, stack, 2)
np.savez(sys.argv[1], **{k: np.asarray(out[k]) for k in ("objF", "objCrop", "pupil")})
"""


def run(lib, env, path):
    e = dict(os.environ, FPM_HIP_LIB=os.path.abspath(lib), **env)
    subprocess.run([sys.executable, "-c", CHILD, path], check=True, env=e, timeout=300)


def main():
    a, b = sys.argv[1], sys.argv[2]
    ok = True
    with tempfile.TemporaryDirectory() as d:
        for name, env in CASES:
            pa, pb = os.path.join(d, f"{name}_a.npz"), os.path.join(d, f"{name}_b.npz")
            run(a, env, pa)
            run(b, env, pb)
            za, zb = np.load(pa), np.load(pb)
            same = all(np.array_equal(za[k], zb[k]) for k in za.files)
            ok = ok and same
            print(f"{name}: {'bit-identical' if same else 'DIFFERENT'}")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
