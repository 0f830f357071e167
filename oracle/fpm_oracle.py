"""CPU oracle for the FPM per-patch phase-retrieval loop -- TEST INFRASTRUCTURE ONLY.

This module is the parity *checker*.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``fpm-opencv_amd/``) never does and fails loudly when its HIP library is missing.

It restates, in numpy complex128, what ``runFPM`` in the reference computes
(``/root/reference/fpmMain.cpp:274-498``), operation for operation, including
the wasteful full-spectrum ``fftShift`` round trips, so that it can be read
side by side with the reference:

* pupil / support init ............ fpmMain.cpp:302-313
* spectrum init from LED order[1] . fpmMain.cpp:319-343
* per-LED update .................. fpmMain.cpp:348-476
* per-iteration objCrop IDFT ...... fpmMain.cpp:481
* pupil re-centred at exit ........ fpmMain.cpp:496
* loader preprocessing ............ fpmMain.cpp:124-144 (``preprocess_frame``)

Semantics of the un-vendored ``cvComplex`` helpers are *assumed* as listed in
SURVEY.md section 8(c) (i)-(vii): ``fft2`` = unscaled forward DFT, ``ifft2`` =
inverse DFT scaled by 1/N, ``complexAbs`` returns (|z|, 0), ``fftShift`` is a
quadrant swap (even sizes only), the filled ``cv::circle`` is the Euclidean
disk.  ``cv::add`` / ``cv::multiply(UMat CV_64FC2, double)`` (fpmMain.cpp:390,
417-418, 469-470) follow OpenCV's published ``arithm_op``: the double becomes
a 1x1 array (``_InputArray(const double&)``), ``checkScalar`` accepts it as a
scalar and ``convertAndUnrollScalar`` copies it into EVERY channel, so eps is
added to Re and Im and both update denominators are complex
(``all_channels=True``, the default).  ``all_channels=False`` restates the
round-1 assumption (real channel only), kept as FPM_FLAG_SCALAR_RE_ONLY.  The reference
cannot be built here (OpenCV 3 + cvComplex absent), so these semantics are
"parity unpinned" at the cvComplex boundary; see DESIGN.md "Oracle".
"""
from __future__ import annotations

import numpy as np


def fftshift2(a: np.ndarray) -> np.ndarray:
    """cvComplex ``fftShift`` on an even-sized 2-D array: quadrant swap.

    Used at fpmMain.cpp:310,327,343,358,361,427,432,447,496.  For even sizes
    fftshift == ifftshift, which is why the reference can use one routine for
    both directions.
    """
    h, w = a.shape[-2:]
    if h % 2 or w % 2:
        raise ValueError("fftShift restatement only defined for even sizes")
    return np.roll(np.roll(a, h // 2, axis=-2), w // 2, axis=-1)


def disk_support(np_: int, radius: int) -> np.ndarray:
    """Pupil support, fpmMain.cpp:302-313.

    ``cv::circle(planes[0], (Np/2, Np/2), naRadius, 1.0, -1 /*filled*/, 8, 0)``
    then ``fftShift``.  The filled LINE_8 circle is the Euclidean disk
    (x-c)^2 + (y-c)^2 <= r^2.  Returned un-centred (DC at
    [0,0]) as float64 0/1.
    """
    c = np_ // 2
    y, x = np.mgrid[0:np_, 0:np_]
    s = (((x - c) ** 2 + (y - c) ** 2) <= radius * radius).astype(np.float64)
    return fftshift2(s)


def _fft2(a):
    # cvComplex fft2: unscaled forward DFT (fpmMain.cpp:325,394)
    return np.fft.fft2(a)


def _ifft2(a):
    # cvComplex ifft2: inverse DFT scaled by 1/(rows*cols) (fpmMain.cpp:365)
    return np.fft.ifft2(a)


def run_fpm(stack, order, x0, y0, np_: int, L: int, radius: int,
            delta1: float, delta2: float, iters: int,
            eps: float = float(np.float32(1e-10)), record=None,
            all_channels: bool = True):
    """Restatement of ``runFPM`` (fpmMain.cpp:274-498) for ONE patch.

    Parameters mirror the ``FPM_Dataset`` fields runFPM reads
    (SURVEY.md 8(b)):

    stack   : uint16 array [n_stack][Np][Np] -- ``imageStack[led].Image``
              (already background-subtracted by the loader).
    order   : sequence of stack indices -- ``sortedIndicies[0:ledUsedCount]``.
    x0, y0  : per stack index crop start (``cropXStart`` / ``cropYStart``),
              in the *centred* L x L spectrum.
    radius  : ``naRadius`` (fpmMain.cpp:305-306).
    delta1/2: JSON ``asInt`` values (fpmMain.cpp:567-568).
    eps     : ``float eps = 1e-10`` (fpmMain.h:99).
    all_channels : OpenCV scalar unrolling (module docstring): a double added
              to / multiplied into a CV_64FC2 array acts on both channels.

    Returns dict(objF=un-centred L x L spectrum, objCrop=IDFT(objF)/L^2,
    pupil=centred Np x Np pupil (fpmMain.cpp:496), support=un-centred S).
    """
    stack = np.asarray(stack)
    order = [int(i) for i in order]
    # cv::add(c2, s) with s a double: (re + s, im + s) when unrolled to every
    # channel, (re + s, im) under the real-channel-only assumption
    cs = (1 + 1j) if all_channels else 1.0
    S = disk_support(np_, radius)                       # :302-313
    pupil = S.astype(np.complex128)                     # mergeUMat(planes)
    support = pupil.copy()                              # :313

    # :319-327  A = sqrt(I[sortedIndicies[1]]); O = fftShift(fft2(A) * S)
    amp0 = np.sqrt(stack[order[1]].astype(np.float64))
    complex_i = _fft2(amp0.astype(np.complex128))
    complex_i = complex_i * support
    complex_i = fftshift2(complex_i)

    # :330-343 place in the centre of an L x L zero spectrum, then un-centre
    objF = np.zeros((L, L), np.complex128)
    c0 = L // 2 - np_ // 2
    objF[c0:c0 + np_, c0:c0 + np_] = complex_i
    objF = fftshift2(objF)

    objCrop = None
    for _itr in range(iters):                           # :345
        for led in order:                               # :348
            xs, ys = int(x0[led]), int(y0[led])
            objF_c = fftshift2(objF)                                    # :358
            objfcrop = fftshift2(objF_c[ys:ys + np_, xs:xs + np_])      # :361
            objfcropP = objfcrop * pupil                                # :364
            objcropP = _ifft2(objfcropP)                                # :365
            object_amp = np.sqrt(stack[led].astype(np.float64))         # :378-387
            tmp1 = objcropP + eps * cs                                  # :390
            tmp3 = np.abs(tmp1)                                         # :391
            tmp1 = objcropP / tmp3                                      # :392
            tmp3 = tmp1 * object_amp                                    # :393
            objfup = _fft2(tmp3)                                        # :394

            # object update :405-447
            pupil_abs = np.abs(pupil)
            numerator = (objfup - objfcropP) * (pupil_abs * np.conj(pupil))
            pupil_abs_max = pupil_abs.max()                             # :415
            denom = (pupil_abs * pupil_abs + delta2 * cs) * pupil_abs_max  # :417-418
            tmp2 = numerator / denom                                    # :419
            objF_c = fftshift2(objF)                                    # :427
            upd = fftshift2(tmp2) + objF_c[ys:ys + np_, xs:xs + np_]    # :432-433
            objF_c[ys:ys + np_, xs:xs + np_] = upd                      # :444
            objF = fftshift2(objF_c)                                    # :447

            # pupil update :457-475 (uses the PRE-update objfcrop)
            objfcrop_abs = np.abs(objfcrop)
            objf_abs_max = np.abs(objF).max()                           # :460,467
            numerator = (objfup - objfcropP) * (objfcrop_abs * np.conj(objfcrop))
            denom = (objfcrop_abs * objfcrop_abs + delta1 * cs) * objf_abs_max  # :469-470
            tmp2 = (numerator / denom) * support                        # :471-472
            pupil = pupil + tmp2                                        # :475
            if record is not None:
                record.append((led, objF.copy(), pupil.copy()))
        objCrop = np.fft.ifft2(objF)                    # :481 DFT_INVERSE|DFT_SCALE
    if objCrop is None:
        objCrop = np.fft.ifft2(objF)
    return dict(objF=objF, objCrop=objCrop, pupil=fftshift2(pupil),
                support=support)


def rel_l2(a, b) -> float:
    """Relative L2 error ||a-b|| / ||b|| used by every parity test."""
    a = np.asarray(a, np.complex128)
    b = np.asarray(b, np.complex128)
    den = np.linalg.norm(b.ravel())
    return float(np.linalg.norm((a - b).ravel()) / (den if den > 0 else 1.0))


def preprocess_frame(frame, np_: int, crop, bk1, bk2, bg_threshold: float, dark_mult: float = 1.0,
                     darkfield: bool = False):
    """loadFPMDataset's per-image preprocessing (fpmMain.cpp:124-144) for one
    patch window ``crop`` = (x, y) of a full uint16 frame [H][W]:

    * crop ``Image = fullImg(Rect(cropX, cropY, Np, Np))``           (:124-125)
    * darkfield ``cv::divide(Image, mult)`` when the LED NA > objective NA and
      mult != 1: saturate_cast<ushort> of the quotient, round half to even (:128-129)
    * ``bg = (mean(bk2 window) + mean(bk1 window)) / 2`` of the UNDIVIDED frame,
      clamped to bgThresh, ``(int16_t)round(bg)``                    (:131-140)
    * saturating ``cv::subtract(Image, bg)``                         (:143-144)

    Returns (uint16 [Np][Np], bg_val)."""
    f = np.asarray(frame)
    x, y = crop
    img = f[y:y + np_, x:x + np_].astype(np.int64)
    if darkfield and dark_mult != 1:
        img = np.clip(np.rint(img / float(dark_mult)), 0, 65535).astype(np.int64)

    def mean(w):
        wx, wy = w
        return float(f[wy:wy + np_, wx:wx + np_].astype(np.int64).sum()) / (np_ * np_)

    bg = (mean(bk2) + mean(bk1)) / 2
    if bg > bg_threshold:
        bg = float(bg_threshold)
    bg_val = int(np.floor(bg + 0.5))                       # std::round, bg >= 0
    bg_val = (bg_val + 32768) % 65536 - 32768               # (int16_t) conversion
    return np.clip(img - bg_val, 0, 65535).astype(np.uint16), bg_val
