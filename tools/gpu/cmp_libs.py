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

G256 = (256, 768, 33, 3, 60)  # Np, L, r, LED grid side, step: metric-like, tail rows and tail pixels
CASES = [  # (name, environment, geometry)
    ("one_workgroup", {"FPM_NO_DIST": "1", "FPM_NO_SPLIT": "1"}, G256),
    ("split_ks2", {"FPM_NO_DIST": "1", "FPM_SPLIT": "2"}, G256),
    ("dist_ks4", {"FPM_DIST": "4"}, G256),
    ("dist_ks8", {"FPM_DIST": "8"}, G256),
    ("np90_s90", {}, (90, 360, 30, 5, 24)),       # k_fused_s90 (configs 1 / 2)
    ("np200_mr", {}, (200, 600, 26, 5, 40)),      # k_fused_mr (config 3)
    # the general path's Np 1024 register kernels + K4 + the L 4096 objCrop
    # passes (config 5 shape at L 2048 / 4096, fp16 spectrum storage: flag 2)
    ("np1024_fp16", {"CMP_FLAGS": "2", "CMP_NPATCH": "1"}, (1024, 4096, 333, 3, 200)),
    ("np1024_fp32", {"CMP_NPATCH": "2"}, (1024, 2048, 120, 3, 100)),
]

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, 'fpm-opencv_amd/python'); sys.path.insert(0, '.')
import fpm_amd
from tools.synth import grid_geometry, make_stack
Np, L, r, nside, step = (int(v) for v in sys.argv[2:7])
x0, y0, order = grid_geometry(Np, L, nside, step)
import os
npatch = int(os.environ.get("CMP_NPATCH", "4"))
stack = make_stack(Np, L, r, x0, y0, n_patch=npatch, seed=7)
prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=npatch, flags=int(os.environ.get("CMP_FLAGS", "0")))
out = fpm_amd.run_fpm(prob, stack, 2)
np.savez(sys.argv[1], **{k: np.asarray(out[k]) for k in ("objF", "objCrop", "pupil")})
"""


def run(lib, env, geo, path):
    e = dict(os.environ, FPM_HIP_LIB=os.path.abspath(lib), **env)
    subprocess.run([sys.executable, "-c", CHILD, path, *map(str, geo)], check=True, env=e, timeout=300)


def main():
    a, b = sys.argv[1], sys.argv[2]
    ok = True
    with tempfile.TemporaryDirectory() as d:
        for name, env, geo in CASES:
            pa, pb = os.path.join(d, f"{name}_a.npz"), os.path.join(d, f"{name}_b.npz")
            run(a, env, geo, pa)
            run(b, env, geo, pb)
            za, zb = np.load(pa), np.load(pb)
            same = all(np.array_equal(za[k], zb[k]) for k in za.files)
            ok = ok and same
            if same:
                print(f"{name}: bit-identical")
            else:  # which outputs moved, by how much (relative L2)
                rel = {k: float(np.linalg.norm(za[k] - zb[k]) / max(np.linalg.norm(za[k]), 1e-30))
                       for k in za.files if not np.array_equal(za[k], zb[k])}
                print(f"{name}: DIFFERENT " + " ".join(f"{k} rel {v:.2e}" for k, v in rel.items()))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
