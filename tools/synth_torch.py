"""GPU version of tools/synth.py for bench-sized stacks (256 patches x 293
LEDs x 256^2 = 4.9 GB of uint16): the same FPM forward model evaluated with
torch.fft on the device.  This only MAKES the synthetic input; the solver under
test never touches torch.

Model: per patch o = a*exp(i*phi), a = 0.5 + 0.5*U(0,1),
phi = 0.5*U(-pi,pi), both Gaussian smoothed (sigma 1 px, periodic);
P_true = S*exp(0.3i*(2 rho^2 - 1)); I_k = |ifft2(crop_k(fftshift(fft2 o)) P)|^2
scaled per patch so the brightest LED image peaks at 40000, Poisson noise,
uint16.  Seeded per patch with torch.Generator(seed + patch index); the
values differ from the numpy generator's (same seeding rule, different
streams) -- tests use the numpy one, the bench this one.
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
               peak: float = 40000.0, device="cuda", chunk: int = 64, patch_offset: int = 0) -> torch.Tensor:
    """uint16 [nLED][n_patch][Np][Np] on `device` (LED-major, the C-ABI layout).

    Patch b of this call is global patch patch_offset + b and draws all of its
    random numbers (object amplitude, phase, Poisson noise) from its own
    generator seeded seed + patch_offset + b, so a rank's shard of a field is
    the same data whatever the shard layout (bench.py --patches-total)."""
    n_led = len(x0)
    out = torch.empty((n_led, n_patch, np_, np_), dtype=torch.int32, device=device)
    P = true_pupil(np_, radius, device)
    for b0 in range(0, n_patch, chunk):
        nb = min(chunk, n_patch - b0)
        gens = [torch.Generator(device=device) for _ in range(nb)]
        for i, g in enumerate(gens):
            g.manual_seed(seed + patch_offset + b0 + i)
        amp = _smooth(0.5 + 0.5 * torch.stack([torch.rand((L, L), generator=g, device=device) for g in gens]))
        ph = _smooth(0.5 * (2 * torch.stack([torch.rand((L, L), generator=g, device=device) for g in gens]) - 1)
                     * math.pi)
        O = torch.fft.fftshift(torch.fft.fft2(torch.polar(amp, ph)), dim=(-2, -1))
        del amp, ph
        inten = torch.empty((nb, n_led, np_, np_), dtype=torch.float32, device=device)
        for k in range(n_led):
            xs, ys = int(x0[k]), int(y0[k])
            crop = torch.fft.ifftshift(O[:, ys:ys + np_, xs:xs + np_], dim=(-2, -1))
            inten[:, k] = torch.fft.ifft2(crop * P).abs() ** 2
        del O
        scale = peak / inten.amax(dim=(1, 2, 3)).clamp_min(1e-30)
        for i, g in enumerate(gens):
            noisy = torch.poisson(inten[i] * scale[i], generator=g)
            out[:, b0 + i] = noisy.round().clamp_(0, 65535).to(torch.int32)
        del inten
    # int32 -> int16 keeps the uint16 bit pattern (two's-complement wrap)
    return out.to(torch.int16)  # uint16 bit pattern in an int16 tensor
