"""ctypes mirror of the libfpm_hip.so C ABI (include/fpm_hip.h).

This is the Python face of the reference's ``runFPM(FPM_Dataset*)``
(fpmMain.cpp:274): ``Solver`` owns one ``fpm_ctx`` on one GPU and exposes
create / upload / init / run / download with numpy arrays, and ``run_fpm`` is
the one-shot call.  Errors raise ``FpmError`` carrying the library's negative
code and ``fpm_last_error()`` text.  There is no CPU fallback: if the HIP
library cannot be loaded, ``load_library`` raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(_HERE))          # fpm-opencv_amd/
LIB_DIR = os.path.join(PKG_ROOT, "lib")
# FPM_HIP_LIB: an alternative build of the same library (compiler-flag A/B
# experiments under tools/gpu/); the default is the in-tree build
HIP_LIB = os.environ.get("FPM_HIP_LIB") or os.path.join(LIB_DIR, "libfpm_hip.so")
HOST_LIB = os.path.join(LIB_DIR, "libfpm_host.so")

FPM_OK = 0
FPM_ERR_INVAL = -22
FPM_ERR_NOMEM = -12
FPM_ERR_DEVICE = -5
FPM_ERR_STATE = -71
FPM_ERR_NODEV = -19

PATH_AUTO, PATH_GENERAL, PATH_FUSED = 0, 1, 2
FLAG_OBJCROP_LAST_ONLY = 1
FLAG_SPEC_FP16 = 2          # fp16 spectrum storage, fp32 arithmetic (config 5)
FLAG_SCALAR_RE_ONLY = 4     # legacy: cv::add(UMat c2, double) on the real channel only (fpm_hip.h)

# fpm_info.fused_kernel: the LED-update kernel of the context (fpm_hip.h FPM_KERNEL_*)
KERNEL_GENERAL, KERNEL_FUSED_NP256, KERNEL_FUSED_NP200, KERNEL_FUSED_SMALL, KERNEL_FUSED_NP256_DIST = 0, 1, 2, 3, 4
KERNEL_FUSED_NP90 = 5
KERNEL_NAMES = {KERNEL_GENERAL: "general_led_step", KERNEL_FUSED_NP256: "k_fused_iteration",
                KERNEL_FUSED_NP200: "k_fused_mr", KERNEL_FUSED_SMALL: "k_fused_small",
                KERNEL_FUSED_NP256_DIST: "k_fused_dist", KERNEL_FUSED_NP90: "k_fused_s90"}

# every symbol include/fpm_hip.h declares
HIP_SYMBOLS = (
    "fpm_create", "fpm_destroy", "fpm_upload_stack", "fpm_upload_stack_device",
    "fpm_init", "fpm_run", "fpm_synchronize", "fpm_download",
    "fpm_download_objcrop_device", "fpm_set_stream", "fpm_get_info",
    "fpm_get_timing", "fpm_runFPM", "fpm_last_error", "fpm_version",
    "fpm_upload_frames", "fpm_download_stack", "fpm_get_info_sized", "fpm_abi_version",
    "fpm_get_clock",
)
# test-only entry points (include/fpm_hip_debug.h)
HIP_DEBUG_SYMBOLS = ("fpm_debug_slot_update", "fpm_debug_update_coef", "fpm_debug_set_stall")
ABI_VERSION = 5  # include/fpm_hip.h FPM_ABI_VERSION this mirror follows


class FpmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fpm error {code}: {msg}")
        self.code = code


class fpm_problem(C.Structure):
    _fields_ = [
        ("np", C.c_int32), ("nlarge", C.c_int32), ("n_stack", C.c_int32),
        ("n_order", C.c_int32), ("order", C.POINTER(C.c_int32)),
        ("crop_x0", C.POINTER(C.c_int32)), ("crop_y0", C.POINTER(C.c_int32)),
        ("na_radius", C.c_int32), ("init_pos", C.c_int32),
        ("delta1", C.c_double), ("delta2", C.c_double), ("eps", C.c_double),
        ("n_patch", C.c_int32), ("path", C.c_int32), ("flags", C.c_uint32),
    ]


class fpm_frames(C.Structure):
    _fields_ = [
        ("height", C.c_int32), ("width", C.c_int32),
        ("patch_x0", C.POINTER(C.c_int32)), ("patch_y0", C.POINTER(C.c_int32)),
        ("bk1_x", C.c_int32), ("bk1_y", C.c_int32), ("bk2_x", C.c_int32), ("bk2_y", C.c_int32),
        ("bg_threshold", C.c_double), ("darkfield_exp_multiplier", C.c_double),
        ("darkfield", C.POINTER(C.c_uint8)),
    ]


class fpm_info(C.Structure):
    _fields_ = [("path", C.c_int32), ("box", C.c_int32), ("support_px", C.c_int32),
                ("device", C.c_int32), ("device_bytes", C.c_size_t), ("wg_per_patch", C.c_int32),
                ("fused_kernel", C.c_int32), ("threads_per_wg", C.c_int32)]


class fpm_timing(C.Structure):
    _fields_ = [("run_ms", C.c_double), ("led_ms", C.c_double),
                ("led_launch_ms", C.c_double), ("led_launches", C.c_int32),
                ("objcrop_ms", C.c_double)]


class fpm_clock(C.Structure):
    _fields_ = [("clock_mhz", C.c_double), ("cycles_per_launch", C.c_double),
                ("ms_per_launch", C.c_double), ("launches", C.c_int32)]


_lib = None


def load_library(path: str = HIP_LIB):
    """Load libfpm_hip.so (raises OSError when it is missing -- no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `make -C fpm-opencv_amd` "
                      "(or __graft_entry__.build())")
    lib = C.CDLL(path)
    vp = C.c_void_p
    f32p = C.POINTER(C.c_float)
    u16p = C.POINTER(C.c_uint16)
    sig = {
        "fpm_create": (C.c_int, [C.POINTER(fpm_problem), C.c_int, C.POINTER(vp)]),
        "fpm_destroy": (None, [vp]),
        "fpm_upload_stack": (C.c_int, [vp, u16p]),
        "fpm_upload_stack_device": (C.c_int, [vp, vp]),
        "fpm_init": (C.c_int, [vp]),
        "fpm_run": (C.c_int, [vp, C.c_int]),
        "fpm_synchronize": (C.c_int, [vp]),
        "fpm_download": (C.c_int, [vp, f32p, f32p, f32p, f32p]),
        "fpm_download_objcrop_device": (C.c_int, [vp, vp]),
        "fpm_set_stream": (C.c_int, [vp, vp]),
        "fpm_get_info": (C.c_int, [vp, C.POINTER(fpm_info)]),
        "fpm_get_info_sized": (C.c_int, [vp, C.POINTER(fpm_info), C.c_size_t]),
        "fpm_abi_version": (C.c_int, []),
        "fpm_debug_set_stall": (C.c_int, [vp, C.c_int]),
        "fpm_get_timing": (C.c_int, [vp, C.POINTER(fpm_timing)]),
        "fpm_get_clock": (C.c_int, [vp, C.POINTER(fpm_clock)]),
        "fpm_runFPM": (C.c_int, [C.POINTER(fpm_problem), C.c_int, u16p, C.c_int,
                                 f32p, f32p, f32p, f32p]),
        "fpm_upload_frames": (C.c_int, [vp, C.POINTER(fpm_frames), vp, C.c_int, C.POINTER(C.c_int16)]),
        "fpm_download_stack": (C.c_int, [vp, u16p]),
        "fpm_last_error": (C.c_char_p, []),
        "fpm_version": (C.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fpm_abi_version() != ABI_VERSION:
        raise OSError(f"{path}: ABI {lib.fpm_abi_version()}, this mirror follows ABI {ABI_VERSION}: rebuild")
    _lib = lib
    return lib


def _check(rc: int):
    if rc != FPM_OK:
        raise FpmError(rc, _lib.fpm_last_error().decode())


def _i32(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def _f32p(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_float))


@dataclass
class Problem:
    """Flattened ``FPM_Dataset`` fields runFPM reads."""
    np_: int
    L: int
    order: np.ndarray
    x0: np.ndarray
    y0: np.ndarray
    radius: int
    delta1: float
    delta2: float
    n_patch: int = 1
    init_pos: int = 1
    eps: float = float(np.float32(1e-10))
    path: int = PATH_AUTO
    flags: int = 0
    _keep: list = field(default_factory=list, repr=False)

    def to_c(self) -> fpm_problem:
        order, x0, y0 = _i32(self.order), _i32(self.x0), _i32(self.y0)
        self._keep[:] = [order, x0, y0]
        p = fpm_problem()
        p.np = self.np_
        p.nlarge = self.L
        p.n_stack = len(x0)
        p.n_order = len(order)
        p.order = order.ctypes.data_as(C.POINTER(C.c_int32))
        p.crop_x0 = x0.ctypes.data_as(C.POINTER(C.c_int32))
        p.crop_y0 = y0.ctypes.data_as(C.POINTER(C.c_int32))
        p.na_radius = self.radius
        p.init_pos = self.init_pos
        p.delta1 = float(self.delta1)
        p.delta2 = float(self.delta2)
        p.eps = float(self.eps)
        p.n_patch = self.n_patch
        p.path = self.path
        p.flags = self.flags
        return p


class Solver:
    """One fpm_ctx on one GPU."""

    def __init__(self, prob: Problem, device: int = 0):
        lib = load_library()
        self.prob = prob
        self._cprob = prob.to_c()
        h = C.c_void_p()
        _check(lib.fpm_create(C.byref(self._cprob), device, C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.fpm_destroy(self._h)
            self._h = None

    __del__ = close

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def upload(self, stack: np.ndarray):
        """stack: uint16 [n_stack][n_patch][Np][Np] (or [n_stack][Np][Np] if n_patch == 1)."""
        p = self.prob
        a = np.ascontiguousarray(stack, dtype=np.uint16)
        want = (len(p.x0), p.n_patch, p.np_, p.np_)
        if a.ndim == 3 and p.n_patch == 1:
            a = a[:, None]
        if a.shape != want:
            raise ValueError(f"stack shape {a.shape} != {want}")
        _check(_lib.fpm_upload_stack(self._h, a.ctypes.data_as(C.POINTER(C.c_uint16))))

    def upload_frames(self, frames, patch_x0, patch_y0, bk1=(1, 1), bk2=(1, 1), bg_threshold=1000.0,
                      darkfield_exp_multiplier=1.0, darkfield=None, device_ptr: int | None = None,
                      shape=None):
        """Loader preprocessing on the GPU (fpmMain.cpp:124-144): `frames` is
        uint16 [n_stack][H][W] on the host, or pass device_ptr (+ shape=(H, W))
        for frames already in device memory.  Returns the int16 bg_val per image."""
        p = self.prob
        n = len(p.x0)
        if device_ptr is None:
            a = np.ascontiguousarray(frames, dtype=np.uint16)
            if a.ndim != 3 or a.shape[0] != n:
                raise ValueError(f"frames shape {a.shape}: want [{n}][H][W]")
            H, W = a.shape[1:]
            data = a.ctypes.data_as(C.c_void_p)
        else:
            H, W = shape
            data = C.c_void_p(device_ptr)
        px, py = _i32(patch_x0), _i32(patch_y0)
        if len(px) != p.n_patch or len(py) != p.n_patch:
            raise ValueError("one (x0, y0) per patch")
        dark = np.ascontiguousarray(np.zeros(n, np.uint8) if darkfield is None else np.asarray(darkfield, np.uint8))
        f = fpm_frames(int(H), int(W), px.ctypes.data_as(C.POINTER(C.c_int32)), py.ctypes.data_as(C.POINTER(C.c_int32)),
                       int(bk1[0]), int(bk1[1]), int(bk2[0]), int(bk2[1]), float(bg_threshold),
                       float(darkfield_exp_multiplier), dark.ctypes.data_as(C.POINTER(C.c_uint8)))
        bg = np.zeros(n, np.int16)
        _check(_lib.fpm_upload_frames(self._h, C.byref(f), data, 0 if device_ptr is None else 1,
                                      bg.ctypes.data_as(C.POINTER(C.c_int16))))
        return bg

    def download_stack(self) -> np.ndarray:
        p = self.prob
        out = np.empty((len(p.x0), p.n_patch, p.np_, p.np_), np.uint16)
        _check(_lib.fpm_download_stack(self._h, out.ctypes.data_as(C.POINTER(C.c_uint16))))
        return out

    def upload_device(self, ptr: int):
        _check(_lib.fpm_upload_stack_device(self._h, C.c_void_p(ptr)))

    def set_stream(self, stream_ptr: int | None):
        _check(_lib.fpm_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def init(self):
        _check(_lib.fpm_init(self._h))

    def run(self, iters: int):
        _check(_lib.fpm_run(self._h, int(iters)))

    def synchronize(self):
        _check(_lib.fpm_synchronize(self._h))

    def download(self, objF=True, objCrop=True, pupil=True, support=True):
        p = self.prob
        B, L, N = p.n_patch, p.L, p.np_
        oF = np.empty((B, L, L), np.complex64) if objF else None
        oC = np.empty((B, L, L), np.complex64) if objCrop else None
        pu = np.empty((B, N, N), np.complex64) if pupil else None
        su = np.empty((B, N, N), np.float32) if support else None
        _check(_lib.fpm_download(self._h, _f32p(oF), _f32p(oC), _f32p(pu), _f32p(su)))
        return dict(objF=oF, objCrop=oC, pupil=pu, support=su)

    def download_objcrop_device(self, ptr: int):
        _check(_lib.fpm_download_objcrop_device(self._h, C.c_void_p(ptr)))

    def info(self) -> fpm_info:
        i = fpm_info()
        _check(_lib.fpm_get_info_sized(self._h, C.byref(i), C.sizeof(i)))
        return i

    def debug_set_stall(self, led: int):
        """Test-only fault injection (include/fpm_hip_debug.h): from LED
        position `led` on, the last workgroup of each patch stops publishing
        its split / distributed-mode handoffs; -1 switches it off."""
        _check(_lib.fpm_debug_set_stall(self._h, int(led)))

    def timing(self) -> fpm_timing:
        t = fpm_timing()
        _check(_lib.fpm_get_timing(self._h, C.byref(t)))
        return t

    def clock(self) -> fpm_clock:
        """Shader clock and cycles of the last run's LED-update launches
        (fused path; launches == 0 on the general path)."""
        k = fpm_clock()
        _check(_lib.fpm_get_clock(self._h, C.byref(k)))
        return k


def run_fpm(prob: Problem, stack: np.ndarray, iters: int, device: int = 0):
    """One-shot runFPM equivalent (create, upload, init, run, download)."""
    with Solver(prob, device) as s:
        s.upload(stack)
        s.init()
        s.run(iters)
        return s.download()
