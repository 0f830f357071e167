// tilemax.hpp -- exact max|objF| over the whole spectrum after every object
// update (fpmMain.cpp:460,467) for the fused kernels, from the band-tile
// maxima those kernels keep incrementally (fpm_fused.hip: an LDS atomicMax
// raises a tile's maximum, a tile whose maximum pixel decreased is marked
// dirty and its value becomes an upper bound).
//
// Per-tile-row maxima on top of the tiles: rc[ty] = max over the clean tiles
// of band tile row ty, rd[ty] = max over its dirty bounds.  An LED's update
// changes only the tiles of its window, i.e. the 5-7 tile rows [t0, t1], so
// after the update every wave forms the band's clean / dirty maxima on its
// own -- the untouched rows from rc / rd, the touched rows from their tiles --
// with no barrier and no cross-wave reduction (identical in every wave: the
// same LDS values, max is exact), and the first waves refresh rc / rd of the
// touched rows, which no wave reads in that phase.  The full pass over every
// band tile (plus a barrier and a per-wave partial exchange) of rounds 1-4 is
// left to the rare re-scan of dirty tiles whose bound exceeds the clean
// maximum, which rebuilds every row.
#pragma once
#include <hip/hip_runtime.h>

#include "fft_lds.hpp"

namespace fpm {

constexpr int kMaxBandRows = 64;  // band tile rows: L <= 1024 (fused kernels)

struct TileRows {
    const float *tmx;        // [nby][nbx] band-tile maxima (upper bound if dirty)
    const unsigned *dirty;   // band-tile dirty bits
    float *rc, *rd;          // [nby] per-row clean maximum / dirty bound
    int nbx, nby;

    __device__ __forceinline__ bool isdirty(int k) const { return (dirty[k >> 5] >> (k & 31)) & 1u; }

    // clean / dirty maxima of band tile row ty, in every lane of the wave
    __device__ __forceinline__ void row_of(int ty, int lane, float &c, float &d) const {
        c = 0.f;
        d = 0.f;
        for (int x = lane; x < nbx; x += 64) {
            const int k = ty * nbx + x;
            const float v = tmx[k];
            if (isdirty(k)) d = fmaxf(d, v);
            else c = fmaxf(c, v);
        }
        c = wave_max(c);
        d = wave_max(d);
    }

    // every row (waves take rows w, w + nw, ...); the caller brackets it with
    // barriers: after the tiles are final, before rc / rd are read
    __device__ __forceinline__ void rebuild(int w, int nw, int lane) const {
        for (int ty = w; ty < nby; ty += nw) {
            float c, d;
            row_of(ty, lane, c, d);
            if (lane == 0) {
                rc[ty] = c;
                rd[ty] = d;
            }
        }
    }

    // After an update confined to band tile rows [t0, t1] (tiles final, i.e.
    // behind the update's barrier): the band's clean maximum cm and dirty
    // bound dm, in every lane of every wave; waves w < t1 - t0 + 1 also
    // refresh rc / rd of row t0 + w.
    __device__ __forceinline__ void band_max(int t0, int t1, int w, int nw, int lane, float &cm, float &dm) const {
        float c = 0.f, d = 0.f;
        for (int ty = lane; ty < nby; ty += 64)
            if (ty < t0 || ty > t1) {
                c = fmaxf(c, rc[ty]);
                d = fmaxf(d, rd[ty]);
            }
        const int k0 = t0 * nbx, nk = (t1 - t0 + 1) * nbx;
        for (int i = lane; i < nk; i += 64) {
            const float v = tmx[k0 + i];
            if (isdirty(k0 + i)) d = fmaxf(d, v);
            else c = fmaxf(c, v);
        }
        cm = wave_max(c);
        dm = wave_max(d);
        for (int ty = t0 + w; ty <= t1; ty += nw) {
            float rc_, rd_;
            row_of(ty, lane, rc_, rd_);
            if (lane == 0) {
                rc[ty] = rc_;
                rd[ty] = rd_;
            }
        }
    }

    // max over the rows' clean maxima (after a rebuild), in every lane
    __device__ __forceinline__ float clean_max(int lane) const {
        float c = 0.f;
        for (int ty = lane; ty < nby; ty += 64) c = fmaxf(c, rc[ty]);
        return wave_max(c);
    }
};

}  // namespace fpm
