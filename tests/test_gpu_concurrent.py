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


@pytest.mark.filterwarnings("ignore:The CUDA Graph is empty")  # the refused capture records nothing
def test_run_on_a_capturing_stream_is_refused():
    """fpm_run is blocking and, in distributed / split mode, launches grids
    whose workgroups must all be resident at once; a replayed graph could not
    keep them ordered against other co-resident grids, so a capturing caller
    stream is refused with FPM_ERR_INVAL before anything is enqueued
    (fpm_hip.h).  The capture stays valid and the context
    runs normally afterwards."""
    import torch
    B = 64
    prob, st = _problem(B, 73)
    with fpm_amd.Solver(prob) as s:
        info = s.info()
        assert info.fused_kernel == fpm_amd.KERNEL_FUSED_NP256_DIST and info.wg_per_patch * B == 256
        s.upload(st)
        s.init()
        s.run(1)
        want = s.download(objF=False, support=False)
        s.init()
        cs = torch.cuda.Stream()
        s.set_stream(cs.cuda_stream)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with pytest.raises(fpm_amd.FpmError) as ei:
            with torch.cuda.graph(g, stream=cs, capture_error_mode="relaxed"):
                s.run(1)
        assert ei.value.code == fpm_amd.FPM_ERR_INVAL and "capturing" in str(ei.value)
        s.set_stream(None)
        s.run(1)  # the refused call left the context usable
        got = s.download(objF=False, support=False)
        for k in ("objCrop", "pupil"):
            assert np.array_equal(got[k], want[k]), k


def test_clock_probe_reports_the_launch():
    """fpm_get_clock (ABI 5): block 0's shader cycles and real time over each
    LED-update launch; the clock they give is a plausible MI355X shader clock
    and the probed time fits inside the HIP-event time around the launch
    (which also holds the launch's flag resets and start-up: on this tiny
    problem the kernel itself is ~0.1 ms of ~0.2)."""
    prob, st = _problem(8, 74)
    with fpm_amd.Solver(prob) as s:
        s.upload(st)
        s.init()
        s.run(3)
        k, t = s.clock(), s.timing()
        assert k.launches == 3
        assert 500.0 < k.clock_mhz < 2600.0, k.clock_mhz
        assert k.cycles_per_launch > 0
        assert 0.0 < k.ms_per_launch <= 1.05 * t.led_launch_ms, (k.ms_per_launch, t.led_launch_ms)
        assert abs(k.cycles_per_launch / (k.ms_per_launch * 1e-3) / 1e6 - k.clock_mhz) < 1e-3 * k.clock_mhz


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
