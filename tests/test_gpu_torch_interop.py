"""The HIP library inside a process that imported torch first (bench.py's
situation: torch's bundled HIP runtime, device pointers from torch's
allocator handed across the C ABI)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_upload_from_torch_tensor_and_download_to_torch():
    import torch
    import fpm_amd
    from fpm_oracle import rel_l2
    from tools.synth import grid_geometry, make_stack
    Np, L, r = 32, 96, 6
    x0, y0, order = grid_geometry(Np, L, 5, 4)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=9)
    dev = torch.from_numpy(stack.view(np.int16)).cuda()
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=2)
    with fpm_amd.Solver(prob) as s:
        s.upload_device(dev.data_ptr())
        s.init()
        s.run(2)
        host = s.download()
        out = torch.empty((2, L, L, 2), dtype=torch.float32, device="cuda")
        s.download_objcrop_device(out.data_ptr())
        torch.cuda.synchronize()
    ref = fpm_amd.run_fpm(prob, stack, 2)
    got = out.cpu().numpy().view(np.complex64)[..., 0]
    assert rel_l2(got, host["objCrop"]) == 0.0
    assert rel_l2(host["objCrop"], ref["objCrop"]) == 0.0


@pytest.mark.parametrize("np_,L,r", [(256, 768, 33), (200, 600, 26)])
def test_device_upload_layout_pass_matches_host_upload(np_, L, r):
    """fpm_upload_stack_device on the fused Np 256 / Np 200 paths copies and
    permutes the stack in one out-of-place pass (preprocess.hip
    k_meas_layout_copy); the host upload copies and permutes in place.  Both
    must leave the same stack (fpm_download_stack un-permutes it) and the
    same solution, bit for bit."""
    import torch
    import fpm_amd
    from tools.synth import grid_geometry
    x0, y0, order = grid_geometry(np_, L, 3, 40)
    rng = np.random.default_rng(5)
    stack = rng.integers(0, 40000, (len(x0), 3, np_, np_)).astype(np.uint16)
    prob = fpm_amd.Problem(np_, L, order, x0, y0, r, 10, 3, n_patch=3, path=fpm_amd.PATH_FUSED)
    dev = torch.from_numpy(stack.view(np.int16)).cuda()
    outs = []
    for device_upload in (True, False):
        with fpm_amd.Solver(prob) as s:
            if device_upload:
                s.upload_device(dev.data_ptr())
            else:
                s.upload(stack)
            np.testing.assert_array_equal(s.download_stack(), stack)
            s.init()
            s.run(1)
            outs.append(s.download(objF=False, support=False))
    for k in ("objCrop", "pupil"):
        np.testing.assert_array_equal(outs[0][k], outs[1][k])
