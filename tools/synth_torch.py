"""GPU version of tools/synth.py for bench-sized stacks (256 patches x 293
LEDs x 256^2 = 4.9 GB of uint16): the same FPM forward model evaluated with
torch.fft on the device.  This only MAKES the synthetic input; the solver under
test never touches torch.

Model: per patch o = a*exp(i*phi), a = 0.5 + 0.5*U(0,1),
phi = 0.5*U(-pi,pi), both Gaussian smoothed (sigma 1 px, periodic);
P_true = S*exp(0.3i*(2 rho^2 - 1)); I_k = |ifft2(crop_k(fftshift(fft2 o)) P)|^2
scaled per patch so the brightest LED image peaks at 40000, Poisson noise,
uint16.  Seeded with torch.Generator(seed); patches come from one stream, so
values differ from the numpy generator (which seeds per patch) -- tests use
the numpy one, the bench this one.
"""
from __future__ import annotations

import math

import torch


def _smooth(a: torch.Tensor, sigma: float = 1.0) -> torch.Tensor:
    n = a.shape[-1]
    f = torch.fft.fftfreq(n, device=a.device)
    g = torch.exp(-2.0 * (math.pi * sigma) ** 2 * (f[:, None] ** 2 + f[None, :] ** 2))
    return torch.fft.ifft2(torch.fft.fft2(a) * g).real


def true_pupil(np_: int, radius: int, device) -> torch.Tensor:
    k = torch.fft.fftfreq(np_, 1.0 / np_, device=device)
    ky, kx = torch.meshgrid(k, k, indexing="ij")
    r2 = kx * kx + ky * ky
    s = (r2 <= radius * radius).to(torch.float32)
    ph = 0.3 * (2.0 * r2 / float(max(radius, 1) ** 2) - 1.0)
    return torch.polar(s, ph.to(torch.float32))


@torch.no_grad()
def make_stack(np_: int, L: int, radius: int, x0, y0, n_patch: int, seed: int = 20261015,
               peak: float = 40000.0, device="cuda", chunk: int = 64) -> torch.Tensor:
    """uint16 [nLED][n_patch][Np][Np] on `device` (LED-major, the C-ABI layout)."""
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    n_led = len(x0)
    out = torch.empty((n_led, n_patch, np_, np_), dtype=torch.int32, device=device)
    P = true_pupil(np_, radius, device)
    for b0 in range(0, n_patch, chunk):
        nb = min(chunk, n_patch - b0)
        amp = _smooth(0.5 + 0.5 * torch.rand((nb, L, L), generator=gen, device=device))
        ph = _smooth(0.5 * (2 * torch.rand((nb, L, L), generator=gen, device=device) - 1) * math.pi)
        O = torch.fft.fftshift(torch.fft.fft2(torch.polar(amp, ph)), dim=(-2, -1))
        del amp, ph
        inten = []
        peak_b = torch.zeros(nb, device=device)
        for k in range(n_led):
            xs, ys = int(x0[k]), int(y0[k])
            crop = torch.fft.ifftshift(O[:, ys:ys + np_, xs:xs + np_], dim=(-2, -1))
            I = torch.fft.ifft2(crop * P).abs() ** 2
            peak_b = torch.maximum(peak_b, I.amax(dim=(-2, -1)))
            inten.append(I)
        scale = (peak / peak_b.clamp_min(1e-30))[:, None, None]
        for k in range(n_led):
            lam = inten[k] * scale
            noisy = torch.poisson(lam, generator=gen)
            out[k, b0:b0 + nb] = noisy.round().clamp_(0, 65535).to(torch.int32)
            inten[k] = None
        del O
    # int32 -> int16 keeps the uint16 bit pattern (two's-complement wrap)
    return out.to(torch.int16)  # uint16 bit pattern in an int16 tensor
