"""Host front-end (libfpm_host.so) vs golden geometry from the reference's
own jsoncpp (tests/golden/geometry_*.json, made by make_golden_geometry.py
with oracle/_ref/ref_probe).  CPU only.

Pins: JSON defaults / asInt truncation / trailing-comma recovery
(fpmMain.cpp:512-575), LED NA filter and k-space crop offsets
(fpmMain.cpp:77-168), and the unstable std::sort LED order including ties
(fpmMain.cpp:246-258, fpmMain.h:103-115) -- bit-exact.
"""
import glob
import json
import os

import numpy as np
import pytest

from fpm_amd import host

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _fixtures():
    return sorted(glob.glob(os.path.join(GOLDEN, "geometry_*.json")))


def _load(path):
    with open(path) as f:
        return json.load(f)


@pytest.mark.parametrize("path", _fixtures(), ids=lambda p: os.path.basename(p)[9:-5])
def test_host_geometry_matches_reference_jsoncpp_probe(path):
    fx = _load(path)
    probe = fx["probe"]
    keys = dict(fx["keys"])
    if "leds" not in probe:
        # no holeCoordinates: the reference throws Json::LogicError; the host
        # refuses instead of guessing (dome fallback must be explicit)
        ds = host.Dataset(json_text=json.dumps(keys))
        ds.set_present(range(1, fx["n_present"] + 1))
        with pytest.raises(host.HostError, match="holeCoordinates"):
            ds.geometry()
        return
    if fx["max_na_override"] is not None:
        keys["maxIlluminationNA"] = fx["max_na_override"]
    if fx["np_override"] is not None:
        keys["cropSizeX"] = fx["np_override"]
    xyz = [(l["x"], l["y"], l["z"]) for l in probe["leds"]]
    text = host.dataset_json(keys, xyz, trailing_comma=fx["trailing_comma"])
    ds = host.Dataset(json_text=text)
    cfg = ds.config()
    assert cfg.json_ok == (not fx["trailing_comma"])
    assert cfg.hole_coordinates_count == probe["hole_coordinates_size"]
    assert cfg.np == probe["np"]
    assert cfg.nlarge == probe["nlarge"]
    assert cfg.res_improvement_factor == probe["rif"]
    assert cfg.na_radius == probe["na_radius"]
    assert np.float32(cfg.du) == np.float32(probe["du"])
    assert cfg.delta1 == probe["delta1"] and cfg.delta2 == probe["delta2"]
    assert cfg.led_count == probe["led_count"]
    ds.set_present(range(1, fx["n_present"] + 1))
    used = ds.geometry()
    assert used == probe["led_used_count"]
    leds = ds.leds()
    assert len(leds) == len(probe["leds"])
    for got, want in zip(leds, probe["leds"]):
        assert got.led == want["led"]
        assert np.float32(got.illumination_na) == np.float32(want["na"])
        assert got.used == want["used"]
        if want["used"]:
            assert (got.idx_u, got.idx_v) == (want["idx_u"], want["idx_v"])
            assert (got.crop_x0, got.crop_y0) == (want["crop_x0"], want["crop_y0"])
    np.testing.assert_array_equal(ds.order(), probe["sorted_indices"])


def test_dogstomach_table_is_procedural():
    """The 293 dogStomach LED coordinates are a 4 mm grid within 38 mm."""
    fx = _load(os.path.join(GOLDEN, "geometry_dogStomach_metric.json"))
    want = np.array([(l["x"], l["y"], l["z"]) for l in fx["probe"]["leds"]], np.float32)
    np.testing.assert_array_equal(host.dogstomach_led_table(), want)


def test_led_order_matches_survey_probe():
    """maxNA 0.4 -> 147,166,128,146,148 (init 166);
    maxNA 0.6 -> 147,148,128,146,166 (init 148)."""
    lit = _load(os.path.join(GOLDEN, "geometry_dogStomach_literal.json"))["probe"]
    met = _load(os.path.join(GOLDEN, "geometry_dogStomach_metric.json"))["probe"]
    assert lit["sorted_indices"][:5] == [147, 166, 128, 146, 148]
    assert met["sorted_indices"][:5] == [147, 148, 128, 146, 166]
    assert (lit["na_radius"], met["na_radius"]) == (26, 33)
    assert (lit["nlarge"], met["nlarge"]) == (600, 768)


def test_defaults_when_json_missing(tmp_path):
    """The reference ignores a failed parse and uses every default (:517-575)."""
    ds = host.Dataset(json_path=str(tmp_path / "does_not_exist.json"))
    c = ds.config()
    assert (c.np, c.led_count, c.center_led) == (90, 508, 249)
    assert np.float32(c.objective_na) == np.float32(0.2)
    assert c.delta1 == 5 and c.delta2 == 10 and c.bg_threshold == 1000
    assert c.json_ok == 0


def test_asint_truncates_and_override_rederives():
    ds = host.Dataset(json_text='{"delta1": 7.9, "delta2": -2.5, "cropSizeX": 64.7, "arrayRotation": 3.9}')
    c = ds.config()
    assert (c.delta1, c.delta2, c.np, c.array_rotation) == (7, -2, 64, 3.0)
    ds.override("cropSizeX", 256)
    assert ds.config().np == 256
