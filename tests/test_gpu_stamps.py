"""FPM_STAMPS=1 (the phase-cycle diagnostic every DESIGN.md stamp table comes
from) only adds s_memtime reads to the fused kernels: results are
bit-identical to a run without it, and fpm_run prints the per-phase cycles
for the one-workgroup, split and distributed instances and the Np 90 / Np 200
kernels."""
import os

import numpy as np
import pytest

import fpm_amd
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu

CASES = [  # Np, L, r, B, env
    (256, 512, 20, 2, {"FPM_NO_SPLIT": "1", "FPM_NO_DIST": "1"}),
    (256, 512, 20, 2, {"FPM_SPLIT": "2", "FPM_NO_DIST": "1"}),
    (256, 512, 20, 2, {"FPM_DIST": "4"}),
    (200, 600, 20, 2, {}),
    (90, 360, 20, 2, {}),
]


@pytest.mark.parametrize("Np,L,r,B,env", CASES, ids=["np256", "split2", "dist4", "np200", "np90"])
def test_stamps_do_not_change_results(Np, L, r, B, env, capfd):
    x0, y0, order = grid_geometry(Np, L, 3, 20)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=23)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=B, path=fpm_amd.PATH_FUSED)
    outs = []
    for stamps in (False, True):
        e = dict(env, **({"FPM_STAMPS": "1"} if stamps else {}))
        os.environ.update(e)
        try:
            outs.append(fpm_amd.run_fpm(prob, stack, 1))
        finally:
            for k in e:
                os.environ.pop(k, None)
    for k in ("objF", "objCrop", "pupil"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
    assert "[fpm stamps]" in capfd.readouterr().err
