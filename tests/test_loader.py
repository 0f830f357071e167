"""Host loader (libfpm_host.so: scan + TIFF + preprocessing, fpmMain.cpp:59-144)
vs the oracle's numpy restatement of the preprocessing, bit-exact.  CPU only.

The dataset is synthetic (tests/dataset_fixture.py): the reference ships no
images, so the loader is pinned by the restatement of fpmMain.cpp:124-144 and
by the geometry fixtures of the reference's own jsoncpp (test_geometry.py).
"""
import numpy as np
import pytest

import fpm_oracle as oracle
from dataset_fixture import make_dataset
from fpm_amd import host


@pytest.fixture(scope="module")
def dataset(tmp_path_factory):
    root = tmp_path_factory.mktemp("ds")
    return make_dataset(str(root))


def _loaded(ds):
    d = host.Dataset(ds["json"])
    d.scan()
    n = d.geometry()
    assert n >= 2
    assert d.load_images() == n
    return d


def test_loader_preprocessing_matches_oracle(dataset):
    k = dataset["keys"]
    d = _loaded(dataset)
    stack = d.stack()
    leds = {l.led: l for l in d.leds()}
    order = d.order()
    npx = k["cropSizeX"]
    n_dark = n_clamped = 0
    for s, led in enumerate(order):
        dark = leds[led].illumination_na > k["objectiveNA"]
        want, bg = oracle.preprocess_frame(dataset["frames"][led], npx, (k["cropX"], k["cropY"]),
                                           (k["bk1cropX"], k["bk1cropY"]), (k["bk2cropX"], k["bk2cropY"]),
                                           k["bgThresh"], k["darkfieldExpMultiplier"], dark)
        np.testing.assert_array_equal(stack[s], want, err_msg=f"LED {led}")
        assert leds[led].bg_val == bg
        n_dark += dark
        n_clamped += bg == k["bgThresh"]
    # the fixture exercises every branch of fpmMain.cpp:128-140
    assert 0 < n_dark < len(order)
    assert 0 < n_clamped < len(order)


def test_loader_rejects_window_outside_frame(tmp_path):
    ds = make_dataset(str(tmp_path), keys={"bk2cropX": 80})
    d = host.Dataset(ds["json"])
    d.scan()
    d.geometry()
    with pytest.raises(Exception, match="outside"):
        d.load_images()


def test_tiff_round_trip(tmp_path):
    a = np.random.default_rng(3).integers(0, 65535, (17, 29)).astype(np.uint16)
    p = str(tmp_path / "x.tif")
    host.write_tiff16(p, a)
    np.testing.assert_array_equal(host.read_tiff(p), a)
