"""Two co-resident grids on one device, and the frozen fpm_get_info (GPU only).

Split and distributed modes launch grids whose workgroups wait on each other,
so every block must be resident at once (fused_sync.hpp launch_coresident).
Two such grids from two contexts on two streams of the same GPU could each get
only part of their blocks resident and wait for the rest until the ~1 s
timeout; launch_coresident_raw (api.cpp) orders every co-resident grid of the
process on a device after the previous one.  The test runs two 64-patch
contexts (k_fused_dist<4>: 256 workgroups each, one per CU) from two host
threads at once and checks both against the same runs made one after the
other -- bit for bit, since the kernels are deterministic.
"""
import ctypes as C
import threading

import numpy as np
import pytest

import fpm_amd
from tools.synth import grid_geometry, make_stack

pytestmark = pytest.mark.gpu


def _problem(B, seed):
    Np, L, r = 256, 512, 20
    x0, y0, order = grid_geometry(Np, L, 3, 24)
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=seed)
    return fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=B, path=fpm_amd.PATH_FUSED), stack


def test_two_coresident_contexts_on_two_streams():
    import torch
    B, iters = 64, 3
    cases = [_problem(B, 71), _problem(B, 72)]
    solvers = [fpm_amd.Solver(p) for p, _ in cases]
    try:
        for s, (_, st) in zip(solvers, cases):
            info = s.info()
            assert info.fused_kernel == fpm_amd.KERNEL_FUSED_NP256_DIST and info.wg_per_patch * B == 256
            s.upload(st)
        # one after the other: the expected results
        want = []
        for s in solvers:
            s.init()
            s.run(iters)
            want.append(s.download(objF=False, support=False))
        # both at once, each context on its own stream, from two host threads
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for s, cs in zip(solvers, streams):
            s.set_stream(cs.cuda_stream)
            s.init()
        torch.cuda.synchronize()
        errs = [None, None]
        go = threading.Barrier(2)

        def work(i):
            try:
                go.wait()
                solvers[i].run(iters)
            except Exception as e:  # noqa: BLE001 -- reported below
                errs[i] = e

        th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th)
        assert errs == [None, None], errs
        for s, w in zip(solvers, want):
            got = s.download(objF=False, support=False)
            for k in ("objCrop", "pupil"):
                assert np.array_equal(got[k], w[k]), k
    finally:
        for s in solvers:
            s.close()


def test_get_info_writes_only_the_abi3_struct():
    """fpm_get_info is frozen at the ABI-3 layout (path .. fused_kernel): a
    caller built against that header has a struct of that size, so nothing
    past it may be written; fpm_get_info_sized reports the rest."""
    lib = fpm_amd.load_library()
    prob, st = _problem(2, 5)
    v3 = fpm_amd.fpm_info.fused_kernel.offset + 4
    assert v3 == 32
    with fpm_amd.Solver(prob) as s:
        buf = (C.c_uint8 * 64)(*([0xAB] * 64))
        assert lib.fpm_get_info(s._h, C.cast(buf, C.POINTER(fpm_amd.fpm_info))) == 0
        assert bytes(buf[v3:]) == b"\xab" * (64 - v3)
        full = s.info()
        head = bytes(C.string_at(C.addressof(full), v3))
        assert bytes(buf[:v3]) == head
        assert full.threads_per_wg == 512
