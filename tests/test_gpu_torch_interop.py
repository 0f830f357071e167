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
