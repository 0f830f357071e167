"""Seeded synthetic FPM measurement stacks (SURVEY.md 8(d) "Synthetic input").

The reference ships no images, so every test and bench
input is produced by the FPM forward model:

    o      = a * exp(i*phi)            HR object, L x L, per patch
             a   = 0.5 + 0.5*U(0,1),   phi = 0.5*U(-pi, pi), both Gaussian
             smoothed (sigma = 1 px, periodic)
    O      = fftshift(fft2(o))         centred HR spectrum
    P_true = S * exp(i*0.3*(2 rho^2 - 1))   defocus (Zernike Z4) pupil
    I_k    = | ifft2( ifftshift(O[y0:y0+Np, x0:x0+Np]) * P_true ) |^2

scaled so that the brightest LED image peaks at ~40000 counts, Poisson noise
added and quantised to uint16 -- this is the background-subtracted
``imageStack[led].Image`` that ``runFPM`` consumes (fpmMain.cpp:378-387).
Seeds: ``numpy.random.default_rng(seed + patch_index)``.
"""
from __future__ import annotations

import math

import numpy as np


def _smooth_periodic(a: np.ndarray, sigma: float = 1.0) -> np.ndarray:
    n0, n1 = a.shape
    f0 = np.fft.fftfreq(n0)[:, None]
    f1 = np.fft.fftfreq(n1)[None, :]
    g = np.exp(-2.0 * (math.pi * sigma) ** 2 * (f0 * f0 + f1 * f1))
    return np.real(np.fft.ifft2(np.fft.fft2(a) * g))


def hr_object(L: int, rng: np.random.Generator) -> np.ndarray:
    amp = _smooth_periodic(0.5 + 0.5 * rng.random((L, L)))
    phase = _smooth_periodic(0.5 * rng.uniform(-math.pi, math.pi, (L, L)))
    return amp * np.exp(1j * phase)


def true_pupil(np_: int, radius: int, defocus: float = 0.3) -> np.ndarray:
    """Un-centred pupil: disk support * exp(i * defocus * Z4)."""
    k = np.fft.fftfreq(np_, 1.0 / np_)
    ky, kx = np.meshgrid(k, k, indexing="ij")
    rho2 = (kx * kx + ky * ky) / float(max(radius, 1) ** 2)
    s = (kx * kx + ky * ky) <= radius * radius
    return s * np.exp(1j * defocus * (2.0 * rho2 - 1.0))


def forward_intensities(o: np.ndarray, np_: int, radius: int, x0, y0):
    """|ifft2(crop_k(O) * P_true)|^2 for every LED, float64 [nLED][Np][Np]."""
    O = np.fft.fftshift(np.fft.fft2(o))
    P = true_pupil(np_, radius)
    out = np.empty((len(x0), np_, np_), np.float64)
    for k, (xs, ys) in enumerate(zip(x0, y0)):
        crop = np.fft.ifftshift(O[ys:ys + np_, xs:xs + np_])
        out[k] = np.abs(np.fft.ifft2(crop * P)) ** 2
    return out


def make_stack(np_: int, L: int, radius: int, x0, y0, n_patch: int = 1,
               seed: int = 20261015, peak: float = 40000.0, noise: bool = True):
    """uint16 stack, LED-major: [nLED][n_patch][Np][Np] (the C-ABI layout)."""
    x0 = [int(v) for v in x0]
    y0 = [int(v) for v in y0]
    n = len(x0)
    stack = np.empty((n, n_patch, np_, np_), np.uint16)
    for b in range(n_patch):
        rng = np.random.default_rng(seed + b)
        o = hr_object(L, rng)
        inten = forward_intensities(o, np_, radius, x0, y0)
        scale = peak / max(float(inten.max()), 1e-30)
        lam = inten * scale
        if noise:
            lam = rng.poisson(lam).astype(np.float64)
        stack[:, b] = np.clip(np.rint(lam), 0, 65535).astype(np.uint16)
    return stack


def grid_geometry(np_: int, L: int, n_side: int, step: int):
    """Small synthetic LED grid: crop starts around the spectrum centre.

    Returns (x0, y0, order): ``order`` sorts LEDs by distance from the centre
    (ties by index, i.e. a stable order) -- the runFPM boundary takes the order
    as an input, so any order is a valid parity case.
    """
    c = L // 2 - np_ // 2
    h = n_side // 2
    x0, y0, d = [], [], []
    for iy in range(-h, n_side - h):
        for ix in range(-h, n_side - h):
            x0.append(c + ix * step)
            y0.append(c + iy * step)
            d.append(ix * ix + iy * iy)
    for xs, ys in zip(x0, y0):
        if not (0 <= xs <= L - np_ and 0 <= ys <= L - np_):
            raise ValueError("LED grid leaves the HR spectrum")
    order = sorted(range(len(d)), key=lambda i: (d[i], i))
    return np.array(x0), np.array(y0), order
