// tilemax.hpp -- exact max|objF| over the whole spectrum after every object
// update (fpmMain.cpp:460,467) for the fused kernels, from the band-tile
// maxima those kernels keep incrementally (fpm_fused.hip: an LDS atomicMax
// raises a tile's maximum, a tile whose maximum pixel decreased is marked
// dirty and its value becomes an upper bound).
//
// An LED's update changes only the tiles its window (the (2r+1)^2 box)
// touches, at most 7 x 7.  So the maxima over every OTHER band tile are known
// before the update: the waves that own no box row (idle in the row DFT and
// the update) form them meanwhile, and after the update's barrier ONE wave
// folds in the window tiles (one per lane) and hands the result to the block
// through the barrier the old per-wave partials needed anyway.  (Every wave
// scanning a share of all band tiles after the update, as in rounds 1-4, or
// every wave folding the window tiles itself, costs the SIMDs the kernels
// share among four waves several times over: DESIGN.md 4.2c.)
#pragma once
#include <hip/hip_runtime.h>

#include "fft_lds.hpp"

namespace fpm {

// band-tile rectangle of an LED window (band coordinates, inclusive)
struct TileWin {
    int y0, y1, x0, x1;
    __device__ __forceinline__ int nx() const { return x1 - x0 + 1; }
    __device__ __forceinline__ int count() const { return nx() * (y1 - y0 + 1); }
    __device__ __forceinline__ bool has(int dy, int dx) const { return dy >= y0 && dy <= y1 && dx >= x0 && dx <= x1; }
};

// window of the LED centred at (yc, xc) of the spectrum, radius r
__device__ __forceinline__ TileWin tile_window(int yc, int xc, int r, int bty0, int btx0) {
    return TileWin{((yc - r) >> 4) - bty0, ((yc + r) >> 4) - bty0, ((xc - r) >> 4) - btx0, ((xc + r) >> 4) - btx0};
}

__device__ __forceinline__ bool tile_dirty(const unsigned *dirty, int k) { return (dirty[k >> 5] >> (k & 31)) & 1u; }

// Clean maximum / dirty bound over the band tiles OUTSIDE the window, tiles
// k = k0, k0 + stride, ... (the lanes of the scanning waves), reduced over the
// wave: valid in every lane.  The tiles must be final (behind the previous
// update's barrier) and the window known; the result stays valid through the
// window's update, which never touches these tiles.
__device__ __forceinline__ void outside_max(const float *tmx, const unsigned *dirty, int nbt, int nbx, float rnbx,
                                            const TileWin &wn, int k0, int stride, float &c, float &d) {
    float cc = 0.f, dd = 0.f;
    for (int k = k0; k < nbt; k += stride) {
        const int dy = (int)(((float)k + 0.5f) * rnbx);  // exact for k < 2^16 (fpm_fused.hip band_dy)
        if (wn.has(dy, k - dy * nbx)) continue;
        const float v = tmx[k];
        if (tile_dirty(dirty, k)) dd = fmaxf(dd, v);
        else cc = fmaxf(cc, v);
    }
    c = wave_max_nonneg(cc);
    d = wave_max_nonneg(dd);
}

// After the update (tiles final): the band's clean maximum cm and dirty
// bound dm in every lane, from the window tiles and the maxima c0 / d0 of
// the tiles outside it.  Lane 8 dy + dx takes window tile (dy, dx): the
// window spans at most 8 x 8 tiles (2r + 1 <= 113 pixels; every fused kernel
// has r <= 44).
__device__ __forceinline__ void window_max(const float *tmx, const unsigned *dirty, int nbx, const TileWin &wn,
                                           int lane, float c0, float d0, float &cm, float &dm) {
    float cc = c0, dd = d0;
    const int dy = lane >> 3, dx = lane & 7;
    if (dy <= wn.y1 - wn.y0 && dx < wn.nx()) {
        const int k = (wn.y0 + dy) * nbx + wn.x0 + dx;
        const float v = tmx[k];
        if (tile_dirty(dirty, k)) dd = fmaxf(dd, v);
        else cc = fmaxf(cc, v);
    }
    cm = wave_max_nonneg(cc);
    dm = wave_max_nonneg(dd);
}

}  // namespace fpm
