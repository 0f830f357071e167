"""Generate tests/golden/solver_*.npz: seeded synthetic stacks (tools/synth.py)
run through the numpy oracle (oracle/fpm_oracle.py, complex128).

Each file holds the runFPM inputs (stack, order, crop offsets, radius,
delta1/2, iterations) and its outputs (objF, objCrop, centred pupil) stored as
complex64 to keep the fixtures small.  They pin the oracles (numpy and C++)
against regression and are the fixed target of the GPU golden test.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
from fpm_oracle import run_fpm  # noqa: E402
from tools.synth import grid_geometry, make_stack  # noqa: E402

CASES = {
    # name: Np, L, r, n_side, step, iters, delta1, delta2, seed, all_channels
    # all_channels = 1: cv::add / cv::multiply(UMat c2, double) act on both
    # channels (OpenCV's published scalar unrolling, the default); 0: the
    # real-channel-only restatement kept as FPM_FLAG_SCALAR_RE_ONLY
    "np32_r6_it2": (32, 96, 6, 5, 4, 2, 5, 10, 11, 1),
    "np30_r5_it2": (30, 90, 5, 5, 4, 2, 10, 3, 12, 1),
    "np40_r7_it1": (40, 120, 7, 3, 9, 1, 1000, 70, 13, 1),
    "np32_r6_it2_reonly": (32, 96, 6, 5, 4, 2, 5, 10, 11, 0),
}


def main():
    for name, (Np, L, r, ns, step, iters, d1, d2, seed, allc) in CASES.items():
        x0, y0, order = grid_geometry(Np, L, ns, step)
        stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=seed)[:, 0]
        out = run_fpm(stack, order, x0, y0, Np, L, r, d1, d2, iters, all_channels=bool(allc))
        np.savez_compressed(os.path.join(HERE, f"solver_{name}.npz"), stack=stack, order=np.array(order),
                            x0=x0, y0=y0, params=np.array([Np, L, r, iters, d1, d2]), all_channels=np.array(allc),
                            objF=out["objF"].astype(np.complex64), objCrop=out["objCrop"].astype(np.complex64),
                            pupil=out["pupil"].astype(np.complex64))
        print("wrote", name)


if __name__ == "__main__":
    main()
