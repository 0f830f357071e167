"""BASELINE.json configs 1-5 as parity cases (GPU only).

  config 1: dataset_mono optics with the 508-LED dome table (SURVEY.md 8(c)
            fallback; geometry and LED order from the reference's own jsoncpp
            probe, tests/golden/geometry_mono_dome.json): Np 90, L 360,
            naRadius 30, 193 LEDs, 1 patch, 5 iterations, vs the C++ fp64
            oracle, for both readings of cv::add(UMat c2, double)
  config 2: the same geometry, 64 patches batched, 2 iterations; sampled
            patches vs the oracle
  config 3: dataset_dogStomach.json literal (tests/golden/
            geometry_dogStomach_literal.json: 157 LEDs in the reference's
            tie-ordered std::sort order, Np 200, L 600, naRadius 26,
            delta1/delta2 = 10/3), 256 patches, 2 iterations; patches
            0/128/255 vs the oracle
  config 4: one GPU's shard of the 1024-patch metric field (128 patches x
            293 LEDs, Np 256, L 768), 1 iteration; sampled patches vs oracle
  config 5: Np 1024, L 4096 (fp32 and fp16 spectrum storage)
Tolerance: relative L2 <= 1e-4 after 5 iterations (SURVEY.md 8(c) proposes
1e-3), <= 1e-5 after 1 iteration, <= 5e-5 after 2.
"""
import json
import os

import numpy as np
import pytest

import fpm_amd
from fpm_oracle import rel_l2
from tools.synth import make_stack

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(__file__), "golden", "geometry_mono_dome.json")


def _geometry():
    p = json.load(open(FIX))["probe"]
    leds = {l["led"]: l for l in p["leds"]}
    order = p["sorted_indices"]
    x0 = np.array([leds[n]["crop_x0"] for n in order], np.int32)
    y0 = np.array([leds[n]["crop_y0"] for n in order], np.int32)
    return p, x0, y0


@pytest.mark.parametrize("all_channels", [True, False], ids=["opencv_scalar", "re_only"])
def test_config1_mono_dome_single_patch_5_iterations(all_channels):
    import oracle_lib
    p, x0, y0 = _geometry()
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    assert (Np, L, r, len(x0)) == (90, 360, 30, 193)
    order = np.arange(len(x0))
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=11)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, p["delta1"], p["delta2"], 5,
                             all_channels=all_channels)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=1,
                           flags=0 if all_channels else fpm_amd.FLAG_SCALAR_RE_ONLY)
    out = fpm_amd.run_fpm(prob, stack, 5)
    for k in ("objCrop", "objF", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        assert e < 1e-4, (k, e)


def test_config2_mono_dome_64_patches_batched():
    import oracle_lib
    p, x0, y0 = _geometry()
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    order = np.arange(len(x0))
    B = 64
    stack = make_stack(Np, L, r, x0, y0, n_patch=B, seed=12)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=B)
    out = fpm_amd.run_fpm(prob, stack, 2)
    assert np.isfinite(out["objCrop"]).all()
    sample = (0, 37, 63)
    refs = oracle_lib.run_fpm_batch(stack[:, sample], order, x0, y0, Np, L, r, p["delta1"], p["delta2"], 2,
                                    threads=3, pupil=True)
    for i, b in enumerate(sample):
        for k in ("objCrop", "pupil"):
            e = rel_l2(out[k][b], refs[k][i])
            print(f"config2 patch {b} {k} rel L2 {e:.2e}")
            assert e < 5e-5, (k, b, e)


def _probe_geometry(name):
    p = json.load(open(os.path.join(os.path.dirname(__file__), "golden", name)))["probe"]
    leds = {l["led"]: l for l in p["leds"]}
    order = p["sorted_indices"]
    x0 = np.array([leds[n]["crop_x0"] for n in order], np.int32)
    y0 = np.array([leds[n]["crop_y0"] for n in order], np.int32)
    return p, x0, y0


def _tiled_stack(Np, L, r, x0, y0, B, n_distinct, seed):
    """[nLED][B][Np][Np]: n_distinct forward-model patches, patch b = base[b % n_distinct]
    (a prime n_distinct keeps the sampled patches 0/128/255 distinct)."""
    base = make_stack(Np, L, r, x0, y0, n_patch=n_distinct, seed=seed)
    idx = np.arange(B) % n_distinct
    return base[:, idx], idx


def test_config2_geometry_at_np256_r84_64_patches():
    """BASELINE.md 3's "dataset_mono geometry (Np = 90 / 256)" at Np 256: the
    dome fallback at cropSizeX 256 (tests/golden/geometry_mono_dome_np256.json
    from the reference's own jsoncpp probe) gives L 1024 and naRadius 84
    (fpmMain.cpp:305-306), beyond the fused Np 256 kernels' r <= 34, so the
    general path runs it (fpm_info); 64 patches, 2 iterations, sampled patches
    vs the C++ fp64 oracle."""
    import oracle_lib
    p, x0, y0 = _probe_geometry("geometry_mono_dome_np256.json")
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    assert (Np, L, r, len(x0)) == (256, 1024, 84, 193)
    order = np.arange(len(x0))
    B = 64
    stack, idx = _tiled_stack(Np, L, r, x0, y0, B, 5, seed=212)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=B)
    with fpm_amd.Solver(prob) as s:
        info = s.info()
        assert info.path == fpm_amd.PATH_GENERAL and info.fused_kernel == fpm_amd.KERNEL_GENERAL
        assert info.box == 169
        s.upload(stack)
        s.init()
        s.run(2)
        out = s.download(objF=False, support=False)
    sample = (0, 31, 63)
    assert len({int(idx[b]) for b in sample}) == 3
    refs = oracle_lib.run_fpm_batch(stack[:, sample], order, x0, y0, Np, L, r, p["delta1"], p["delta2"], 2,
                                    threads=3, pupil=True)
    for i, b in enumerate(sample):
        for k in ("objCrop", "pupil"):
            e = rel_l2(out[k][b], refs[k][i])
            print(f"config2 at Np 256 (r 84) patch {b} {k} rel L2 {e:.2e}")
            assert e < 5e-5, (k, b, e)


def test_config3_dogstomach_literal_256_patches():
    """Config 3 as dataset_dogStomach.json states it: 157 LEDs (maxNA 0.4) in
    the reference's own unstable std::sort order, Np 200 / L 600 / r 26,
    delta1 10 / delta2 3, 256 patches on one GPU, 2 iterations."""
    import oracle_lib
    p, x0, y0 = _probe_geometry("geometry_dogStomach_literal.json")
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    assert (Np, L, r, len(x0), p["delta1"], p["delta2"]) == (200, 600, 26, 157, 10, 3)
    order = np.arange(len(x0))
    B = 256
    stack, idx = _tiled_stack(Np, L, r, x0, y0, B, 7, seed=301)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=B)
    out = fpm_amd.run_fpm(prob, stack, 2)
    sample = (0, 128, 255)
    assert len({int(idx[b]) for b in sample}) == 3
    refs = oracle_lib.run_fpm_batch(stack[:, sample], order, x0, y0, Np, L, r, p["delta1"], p["delta2"], 2,
                                    threads=3, pupil=True)
    for i, b in enumerate(sample):
        for k in ("objCrop", "pupil"):
            e = rel_l2(out[k][b], refs[k][i])
            print(f"config3 patch {b} {k} rel L2 {e:.2e}")
            assert e < 5e-5, (k, b, e)
    # identical inputs give identical bits whatever the patch slot
    np.testing.assert_array_equal(out["objCrop"][0], out["objCrop"][7])
    np.testing.assert_array_equal(out["pupil"][128], out["pupil"][2])


def test_config4_single_gpu_shard_128_patches():
    """Config 4 on one GPU: the 128-patch shard one of 8 ranks owns of the
    1024-patch field (parallel.shard_range), metric geometry (dogStomach
    optics, maxNA 0.6: 293 LEDs, Np 256, L 768, r 33), 1 iteration."""
    import oracle_lib
    from fpm_amd import parallel
    p, x0, y0 = _probe_geometry("geometry_dogStomach_metric.json")
    Np, L, r = p["np"], p["nlarge"], p["na_radius"]
    assert (Np, L, r, len(x0)) == (256, 768, 33, 293)
    lo, hi = parallel.shard_range(1024, 8, 3)
    assert hi - lo == 128
    order = np.arange(len(x0))
    stack, idx = _tiled_stack(Np, L, r, x0, y0, hi - lo, 5, seed=401)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, p["delta1"], p["delta2"], n_patch=hi - lo)
    out = fpm_amd.run_fpm(prob, stack, 1)
    sample = (0, 63, 127)
    assert len({int(idx[b]) for b in sample}) == 3
    refs = oracle_lib.run_fpm_batch(stack[:, sample], order, x0, y0, Np, L, r, p["delta1"], p["delta2"], 1,
                                    threads=3, pupil=True)
    for i, b in enumerate(sample):
        for k in ("objCrop", "pupil"):
            e = rel_l2(out[k][b], refs[k][i])
            print(f"config4 patch {b} {k} rel L2 {e:.2e}")
            assert e < 1e-5, (k, b, e)


def test_config5_geometry_np1024_l4096():
    """BASELINE config 5 geometry (Np 1024, L 4096, naRadius 333 -- mono
    optics at Np 1024): the general path and the batched L = 4096 objCrop
    transform at full size, 6 LEDs of a synthetic grid, 1 iteration, fp32
    storage (the fp16-storage variant is the next test)."""
    import oracle_lib
    from tools.synth import grid_geometry
    Np, L, r = 1024, 4096, 333
    x0, y0, order = grid_geometry(Np, L, 3, 40)
    x0, y0 = x0[:6], y0[:6]
    order = np.arange(6, dtype=np.int32)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=13)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 1)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1)
    out = fpm_amd.run_fpm(prob, stack, 1)
    for k in ("objCrop", "objF", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        assert e < 1e-5, (k, e)


# fp16 spectrum storage (FPM_FLAG_SPEC_FP16, config 5 "fp16 storage / fp32
# accumulate"): SURVEY.md 8(c) states <= 1e-2 relative L2 for the fp16-storage
# variant; one fp16 rounding per spectrum store (2^-11 relative) measured
# ~1e-3 after 3 iterations, so the bound below keeps a ~5x margin while
# catching any scale or conversion error (those give O(1) errors).
FP16_TOL = 1e-2


def test_fp16_storage_small_vs_oracle():
    import oracle_lib
    from tools.synth import grid_geometry
    Np, L, r, iters = 64, 192, 10, 3
    x0, y0, order = grid_geometry(Np, L, 7, 6)
    stack = make_stack(Np, L, r, x0, y0, n_patch=2, seed=41)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2, flags=fpm_amd.FLAG_SPEC_FP16)
    with fpm_amd.Solver(prob) as s:
        assert s.info().path == fpm_amd.PATH_GENERAL
        s.upload(stack)
        s.init()
        s.run(iters)
        out = s.download()
    f32 = fpm_amd.run_fpm(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, n_patch=2), stack, iters)
    for b in range(2):
        ref = oracle_lib.run_fpm(stack[:, b], order, x0, y0, Np, L, r, 10, 3, iters)
        for k in ("objCrop", "objF", "pupil"):
            e16 = rel_l2(out[k][b], ref[k])
            assert e16 < FP16_TOL, (k, b, e16)
            # fp16 storage is measurably coarser than fp32 but not broken
            assert e16 > rel_l2(f32[k][b], ref[k]), k


def test_fp16_storage_rejected_on_fused_path():
    from tools.synth import grid_geometry
    Np, L, r = 256, 512, 33
    x0, y0, order = grid_geometry(Np, L, 3, 24)
    with pytest.raises(fpm_amd.FpmError, match="fp16") as e:
        fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 10, 3, path=fpm_amd.PATH_FUSED,
                                       flags=fpm_amd.FLAG_SPEC_FP16))
    assert e.value.code == fpm_amd.FPM_ERR_INVAL


def test_config5_fp16_storage_65_leds_2_iterations():
    """Config 5 at scale: Np 1024, L 4096, naRadius 333, fp16 spectrum storage,
    65 LEDs spread over the bench's whole 512-LED grid (every 8th LED of its
    centre-out order plus the outermost one, so the outermost sub-apertures and
    the spectrum edge are exercised), 2 iterations vs the fp64 oracle."""
    import bench
    import oracle_lib
    geo = bench.config_geometry("c5")
    Np, L, r = geo["np_"], geo["L"], geo["r"]
    pick = list(range(0, geo["n_led"], 8)) + [geo["n_led"] - 1]
    x0, y0 = np.asarray(geo["x0"])[pick], np.asarray(geo["y0"])[pick]
    assert len(pick) == 65 and max(np.abs(x0 - (L // 2 - Np // 2)).max(), np.abs(y0 - (L // 2 - Np // 2)).max()) > 1000
    order = np.arange(len(pick), dtype=np.int32)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=15)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, geo["d1"], geo["d2"], 2)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, geo["d1"], geo["d2"], n_patch=1, flags=fpm_amd.FLAG_SPEC_FP16)
    out = fpm_amd.run_fpm(prob, stack, 2)
    for k in ("objCrop", "objF", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        print(f"config5 fp16 65 LEDs 2 it {k} rel L2 {e:.2e}")
        assert e < FP16_TOL, (k, e)


def test_config5_fp16_storage_np1024_l4096():
    """Config 5 as BASELINE.json names it: Np 1024, L 4096 spectrum held in
    fp16 (half the bytes of fp32 complex), fp32 arithmetic; 6 LEDs, 1
    iteration vs the fp64 oracle, and the device-memory saving."""
    import oracle_lib
    from tools.synth import grid_geometry
    Np, L, r = 1024, 4096, 333
    x0, y0, order = grid_geometry(Np, L, 3, 40)
    x0, y0 = x0[:6], y0[:6]
    order = np.arange(6, dtype=np.int32)
    stack = make_stack(Np, L, r, x0, y0, n_patch=1, seed=13)
    ref = oracle_lib.run_fpm(stack[:, 0], order, x0, y0, Np, L, r, 5, 10, 1)
    prob = fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1, flags=fpm_amd.FLAG_SPEC_FP16)
    with fpm_amd.Solver(prob) as s:
        full = fpm_amd.Solver(fpm_amd.Problem(Np, L, order, x0, y0, r, 5, 10, n_patch=1))
        # the spectrum is the one L^2 buffer that shrinks (8 -> 4 bytes per
        # pixel); the Np 1024 row / column scratch T goes fp16 with it (8 -> 4
        # bytes per element of [nb][Np]) plus its row and column scales
        nb = 2 * r + 1
        assert full.info().device_bytes - s.info().device_bytes == 4 * L * L + 4 * nb * Np - 4 * (nb + Np)
        full.close()
        s.upload(stack)
        s.init()
        s.run(1)
        out = s.download()
    for k in ("objCrop", "objF", "pupil"):
        e = rel_l2(out[k][0], ref[k])
        assert e < FP16_TOL, (k, e)
