// ledtab.hpp -- the LED order of one fused-kernel launch as an LDS table:
// order position -> LED index and window centre (yc, xc) in the spectrum
// (fpmMain.cpp:348-357: sortedIndicies, then the LED's crop offsets).
//
// Read from the global tables, every LED step paid two dependent loads
// (order[it], then x0 / y0 of that LED) before the measurement pointer and
// the window offsets were known, and the next window's loads waited for the
// same chain: two memory round trips on the per-LED critical path.  The
// table is filled once per launch; a lookup is one LDS read.  When it does
// not fit beside a kernel's own LDS the kernel reads the global tables.
#pragma once
#include <hip/hip_runtime.h>

namespace fpm {

struct LedPos {
    int led, yc, xc;
};

struct LedTab {
    const int2 *lds;  // [n_order] {led, yc << 16 | xc}, or null
    const int *order, *x0, *y0;
    int half;         // Np / 2

    // block-wide; the caller's next barrier publishes the table
    __device__ __forceinline__ void fill(int2 *t, int n_order, int tid, int nt) const {
        for (int i = tid; i < n_order; i += nt) {
            const int led = order[i];
            t[i] = make_int2(led, ((y0[led] + half) << 16) | (x0[led] + half));
        }
    }
    __device__ __forceinline__ LedPos at(int it) const {
        if (lds) {
            const int2 e = lds[it];
            // centres are in [0, L): unsigned 16-bit fields (ledtab_offset
            // refuses the table for L > 65536)
            return LedPos{e.x, (int)((unsigned)e.y >> 16), (int)((unsigned)e.y & 0xffffu)};
        }
        const int led = order[it];
        return LedPos{led, y0[led] + half, x0[led] + half};
    }
};

// Host: byte offset of the table after `lds` bytes of a kernel's own LDS
// (8-byte aligned), or -1 when it does not fit in `cap` bytes; `total`
// becomes the launch's dynamic LDS size.  A centre (yc, xc) lies in [0, L)
// (fpm_create keeps every crop window inside the spectrum) and is packed as
// two unsigned 16-bit fields, so the table is used only for L <= 65536.
inline int ledtab_offset(size_t lds, int n_order, int L, size_t cap, size_t &total) {
    const size_t off = (lds + 7) & ~(size_t)7;
    if (n_order > 0 && L <= 65536 && off + (size_t)n_order * 8 <= cap) {
        total = off + (size_t)n_order * 8;
        return (int)off;
    }
    total = lds;
    return -1;
}

}  // namespace fpm
