"""ctypes mirror of libfpm_host.so (include/fpm_host.h): the dataset-JSON
contract, LED geometry / order and the TIFF loader of the reference's
main()/loadFPMDataset (fpmMain.cpp:36-271, 500-592)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import HOST_LIB

_lib = None

HOST_SYMBOLS = (
    "fpm_host_open", "fpm_host_open_text", "fpm_host_close", "fpm_host_get_config",
    "fpm_host_override", "fpm_host_set_led_table", "fpm_host_set_present", "fpm_host_scan",
    "fpm_host_geometry", "fpm_host_n_present", "fpm_host_n_used", "fpm_host_get_leds",
    "fpm_host_get_order", "fpm_host_get_crops", "fpm_host_load_images", "fpm_host_get_stack",
    "fpm_host_load_frames", "fpm_host_read_tiff", "fpm_host_write_tiff16", "fpm_host_last_error",
)


class HostError(RuntimeError):
    pass


class fpm_host_config(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "np", "nlarge", "res_improvement_factor", "na_radius", "led_count", "crop_x", "crop_y",
        "bk1_crop_x", "bk1_crop_y", "bk2_crop_x", "bk2_crop_y", "center_led",
        "darkfield_exp_multiplier", "color", "flip_x", "flip_y", "debug",
        "hole_coordinates_present", "hole_coordinates_count", "json_ok")] + \
        [(n, C.c_float) for n in (
            "pixel_size", "objective_mag", "objective_na", "max_illumination_na", "lambda_",
            "ps_eff", "du", "ps", "bg_threshold", "delta1", "delta2")] + \
        [("array_rotation", C.c_double), ("dataset_root", C.c_char * 1024),
         ("file_prefix", C.c_char * 128), ("file_extension", C.c_char * 32)]


class fpm_host_led(C.Structure):
    _fields_ = [("led", C.c_int32), ("used", C.c_int32), ("pos", C.c_float * 3),
                ("sin_theta_x", C.c_double), ("sin_theta_y", C.c_double),
                ("illumination_na", C.c_float), ("uled", C.c_float), ("vled", C.c_float),
                ("idx_u", C.c_int32), ("idx_v", C.c_int32), ("crop_x0", C.c_int32),
                ("crop_y0", C.c_int32), ("crop_x1", C.c_int32), ("crop_y1", C.c_int32),
                ("bg_val", C.c_int32)]


def load_host_library(path: str = HOST_LIB):
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `make -C fpm-opencv_amd host`")
    lib = C.CDLL(path)
    vp, i32p = C.c_void_p, C.POINTER(C.c_int32)
    sig = {
        "fpm_host_open": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
        "fpm_host_open_text": (C.c_int, [C.c_char_p, C.POINTER(vp)]),
        "fpm_host_close": (None, [vp]),
        "fpm_host_get_config": (C.c_int, [vp, C.POINTER(fpm_host_config)]),
        "fpm_host_override": (C.c_int, [vp, C.c_char_p, C.c_double]),
        "fpm_host_set_led_table": (C.c_int, [vp, C.POINTER(C.c_float), C.c_int]),
        "fpm_host_set_present": (C.c_int, [vp, i32p, C.c_int]),
        "fpm_host_scan": (C.c_int, [vp]),
        "fpm_host_geometry": (C.c_int, [vp]),
        "fpm_host_n_present": (C.c_int, [vp]),
        "fpm_host_n_used": (C.c_int, [vp]),
        "fpm_host_get_leds": (C.c_int, [vp, C.POINTER(fpm_host_led), C.c_int]),
        "fpm_host_get_order": (C.c_int, [vp, i32p, C.c_int]),
        "fpm_host_get_crops": (C.c_int, [vp, i32p, i32p, C.c_int]),
        "fpm_host_load_images": (C.c_int, [vp]),
        "fpm_host_get_stack": (C.c_int, [vp, C.POINTER(C.c_uint16), C.c_size_t]),
        "fpm_host_load_frames": (C.c_int, [vp, C.POINTER(C.c_uint16), C.c_size_t, i32p, i32p]),
        "fpm_host_read_tiff": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint16), C.c_size_t, i32p, i32p]),
        "fpm_host_write_tiff16": (C.c_int, [C.c_char_p, C.POINTER(C.c_uint16), C.c_int32, C.c_int32]),
        "fpm_host_last_error": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _chk(rc):
    if rc < 0:
        raise HostError(f"fpm_host error {rc}: {_lib.fpm_host_last_error().decode()}")
    return rc


class Dataset:
    """Host-side FPM_Dataset: JSON config + LED geometry + (optionally) images."""

    def __init__(self, json_path: str | None = None, json_text: str | None = None):
        lib = load_host_library()
        h = C.c_void_p()
        if json_text is not None:
            _chk(lib.fpm_host_open_text(json_text.encode(), C.byref(h)))
        else:
            _chk(lib.fpm_host_open(json_path.encode(), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.fpm_host_close(self._h)
            self._h = None

    __del__ = close

    def config(self) -> fpm_host_config:
        c = fpm_host_config()
        _chk(_lib.fpm_host_get_config(self._h, C.byref(c)))
        return c

    def override(self, key: str, value: float):
        _chk(_lib.fpm_host_override(self._h, key.encode(), float(value)))

    def set_led_table(self, xyz):
        a = np.ascontiguousarray(np.asarray(xyz, np.float32).reshape(-1, 3))
        _chk(_lib.fpm_host_set_led_table(self._h, a.ctypes.data_as(C.POINTER(C.c_float)), len(a)))

    def set_present(self, leds):
        a = np.ascontiguousarray(np.asarray(leds, np.int32))
        _chk(_lib.fpm_host_set_present(self._h, a.ctypes.data_as(C.POINTER(C.c_int32)), len(a)))

    def scan(self) -> int:
        return _chk(_lib.fpm_host_scan(self._h))

    def geometry(self) -> int:
        return _chk(_lib.fpm_host_geometry(self._h))

    def leds(self):
        n = _lib.fpm_host_n_present(self._h)
        arr = (fpm_host_led * max(n, 1))()
        k = _chk(_lib.fpm_host_get_leds(self._h, arr, n))
        return [arr[i] for i in range(k)]

    def order(self) -> np.ndarray:
        n = _lib.fpm_host_n_used(self._h)
        a = np.zeros(n, np.int32)
        _chk(_lib.fpm_host_get_order(self._h, a.ctypes.data_as(C.POINTER(C.c_int32)), n))
        return a

    def crops(self):
        n = _lib.fpm_host_n_used(self._h)
        x0, y0 = np.zeros(n, np.int32), np.zeros(n, np.int32)
        _chk(_lib.fpm_host_get_crops(self._h, x0.ctypes.data_as(C.POINTER(C.c_int32)),
                                     y0.ctypes.data_as(C.POINTER(C.c_int32)), n))
        return x0, y0

    def load_images(self) -> int:
        return _chk(_lib.fpm_host_load_images(self._h))

    def stack(self) -> np.ndarray:
        c = self.config()
        n = _lib.fpm_host_n_used(self._h)
        a = np.zeros((n, c.np, c.np), np.uint16)
        _chk(_lib.fpm_host_get_stack(self._h, a.ctypes.data_as(C.POINTER(C.c_uint16)), a.size))
        return a

    def frames(self) -> np.ndarray:
        """Raw full frames of the used LEDs, uint16 [n_used][H][W], stack order."""
        w, h = C.c_int32(), C.c_int32()
        _chk(_lib.fpm_host_load_frames(self._h, None, 0, C.byref(w), C.byref(h)))
        n = _lib.fpm_host_n_used(self._h)
        a = np.zeros((n, h.value, w.value), np.uint16)
        _chk(_lib.fpm_host_load_frames(self._h, a.ctypes.data_as(C.POINTER(C.c_uint16)), a.size, None, None))
        return a


def write_tiff16(path: str, img: np.ndarray):
    load_host_library()
    a = np.ascontiguousarray(img, np.uint16)
    _chk(_lib.fpm_host_write_tiff16(path.encode(), a.ctypes.data_as(C.POINTER(C.c_uint16)),
                                    a.shape[1], a.shape[0]))


def read_tiff(path: str) -> np.ndarray:
    load_host_library()
    w, h = C.c_int32(), C.c_int32()
    _chk(_lib.fpm_host_read_tiff(path.encode(), None, 0, C.byref(w), C.byref(h)))
    a = np.zeros((h.value, w.value), np.uint16)
    _chk(_lib.fpm_host_read_tiff(path.encode(), a.ctypes.data_as(C.POINTER(C.c_uint16)), a.size,
                                 C.byref(w), C.byref(h)))
    return a


def dogstomach_led_table():
    """The 293-LED planar array of dataset_dogStomach.json (holeCoordinates,
    :28-320), regenerated procedurally: 4 mm grid points with x^2+y^2 <= 38^2
    mm^2, ordered by x then y, at z = 67.5 mm (checked against the
    reference-probe fixture in tests/test_geometry.py)."""
    pts = [(float(x), float(y), 67.5) for x in range(-36, 37, 4) for y in range(-36, 37, 4)
           if x * x + y * y <= 38 * 38]
    return np.array(pts, np.float32)


def dataset_json(keys: dict, xyz, trailing_comma: bool = False) -> str:
    """A dataset JSON in the reference's schema (scalar keys + holeCoordinates
    as [{"x":..},{"y":..},{"z":..}] triples)."""
    import json
    parts = [f'  {json.dumps(k)} : {json.dumps(v)}' for k, v in keys.items()]
    rows = ",\n".join('   [{"x":%.9g},{"y":%.9g},{"z":%.9g}]' % tuple(map(float, p)) for p in xyz)
    hc = '  "holeCoordinates":[\n' + rows + (",\n" if trailing_comma else "\n") + "]"
    return "{\n" + ",\n".join(parts + [hc]) + "\n}\n"
