// dft16.hpp -- register-resident 16-point DFTs and the 16x16 four-step
// exchange shared by the fused LED-update kernel (fpm_fused.hip) and the
// objCrop transform (objcrop.hip).
//
// Layout: a 16-lane group holds 16 complex values per lane; a 256-point
// transform is two register 16-point DFTs with one LDS exchange between them.
#pragma once
#include <hip/hip_runtime.h>

#include "fft_lds.hpp"

namespace fpm {

// ---------------------------------------------------------------- 16-pt DFTs
// W16^j for the forward transform; the inverse uses the conjugate.
template <bool INV>
__device__ __forceinline__ float2 w16(float2 a, int j) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    float c, s;  // W16^j = c - i s (forward)
    switch (j & 15) {
        case 1: c = C1; s = S1; break;
        case 2: c = R2; s = R2; break;
        case 3: c = S1; s = C1; break;
        case 6: c = -R2; s = R2; break;
        case 9: c = -C1; s = -S1; break;
        default: c = 1.f; s = 0.f; break;
    }
    if (j == 4) return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
    const float si = INV ? -s : s;
    // (a.x + i a.y)(c - i si)
    return make_float2(a.x * c + a.y * si, a.y * c - a.x * si);
}

template <bool INV>
__device__ __forceinline__ void bf4(float2 &a0, float2 &a1, float2 &a2, float2 &a3) {
    float2 q[4] = {a0, a1, a2, a3};
    dft4<INV>(q);
    a0 = q[0];
    a1 = q[1];
    a2 = q[2];
    a3 = q[3];
}

// twiddles between the two radix-4 stages: position k1 + 4 m1 *= W16^{k1 m1}
template <bool INV>
__device__ __forceinline__ void mid_tw(float2 (&v)[16]) {
    v[5] = w16<INV>(v[5], 1);
    v[6] = w16<INV>(v[6], 2);
    v[7] = w16<INV>(v[7], 3);
    v[9] = w16<INV>(v[9], 2);
    v[10] = w16<INV>(v[10], 4);
    v[11] = w16<INV>(v[11], 6);
    v[13] = w16<INV>(v[13], 3);
    v[14] = w16<INV>(v[14], 6);
    v[15] = w16<INV>(v[15], 9);
}

// dense 16-point DFT: in v[k], out r[m] = sum_k v[k] W16^{+-km}
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&v)[16], float2 (&r)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) bf4<INV>(v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    mid_tw<INV>(v);
#pragma unroll
    for (int m1 = 0; m1 < 4; ++m1) bf4<INV>(v[4 * m1], v[4 * m1 + 1], v[4 * m1 + 2], v[4 * m1 + 3]);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// ------------------------------------------------------- four-step exchange
// Lane t of a 16-lane group holds y[m1] (m1 = 0..15); afterwards lane t holds
// z[j] = y_of_lane_j[t].  The 16x16 tile is padded (row pitch XP complex):
// the write (16 lanes, one row) and the read are bank-conflict free, and every
// access is one base register plus an immediate offset (an XOR swizzle would
// need 32 per-lane address registers).  Pitch 17 (odd) suits 8-byte reads;
// pitch 18 (below) allows 16-byte reads.
//
// Ordering: LDS instructions of one wave execute in issue order, so the reads
// see every lane's writes as long as the COMPILER keeps them in program
// order.  Alias analysis could otherwise prove that read j only overlaps
// this lane's own write j (17*m1 + t == 17*t + j needs m1 == j) and hoist the
// others, so the read base `xrd` (= t*XP) is laundered through an empty asm
// once per kernel: every read may alias every write and stays after them,
// while unrelated loads and stores remain free to move across the exchange
// (a wave_barrier/fence pair here pinned them and cost 7% of the kernel).
//
// With an even pitch (18 complex = 144 B, every row 16-B aligned) each lane
// reads its row as eight ds_read_b128 instead of sixteen 8-byte reads (which
// the compiler pairs into ds_read2_b64, half the LDS bytes per clock). Banks:
// row t starts at dword 36 t = 4 (9 t mod 16) (mod 64), a distinct 16-byte
// slot for each t, and every ds_read_b128 lane group holds 16 distinct t, so
// the wide reads are conflict-free; the 16-lane row writes stay contiguous.
constexpr int XP = 18;                      // exchange-tile row pitch
constexpr int XTILE = 16 * XP;              // complex per group tile
__device__ __forceinline__ int opaque_int(int v) {
    asm volatile("" : "+v"(v));
    return v;
}
// read base of lane t, laundered (see above); computed once per kernel
__device__ __forceinline__ int exch_rbase(int t) { return opaque_int(t * XP); }
// (a lane-major tile with eight 16-byte writes per lane was measured: pass B
// +3%, the strided reads cost more than the halved write count saves)
__device__ __forceinline__ void exchange16(float2 *scr, int t, int xrd, const float2 (&y)[16], float2 (&z)[16]) {
#pragma unroll
    for (int m1 = 0; m1 < 16; ++m1) scr[m1 * XP + t] = y[m1];
    const float4 *rp = (const float4 *)(scr + xrd);  // 16-B aligned: XTILE and XP even
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const float4 q = rp[j];
        z[2 * j] = make_float2(q.x, q.y);
        z[2 * j + 1] = make_float2(q.z, q.w);
    }
}

// Half-tile exchange: the same result through an 8-row tile (8 x XP complex,
// half of XTILE) in two rounds -- rows y[0..7] written, lanes t < 8 read
// theirs; rows y[8..15] written over them, lanes t >= 8 read.  The second
// round's writes stay behind the first round's reads because the read base
// (exch_rbase_half) is laundered like exch_rbase's.
constexpr int XTILE_H = 8 * XP;
__device__ __forceinline__ int exch_rbase_half(int t) { return opaque_int((t & 7) * XP); }
__device__ __forceinline__ void exchange16_half(float2 *scr, int t, int xrdh, const float2 (&y)[16],
                                                float2 (&z)[16]) {
    const float4 *rp = (const float4 *)(scr + xrdh);  // 16-B aligned: XP even
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int m1 = 0; m1 < 8; ++m1) scr[m1 * XP + t] = y[8 * h + m1];
        if ((t >> 3) == h) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float4 q = rp[j];
                z[2 * j] = make_float2(q.x, q.y);
                z[2 * j + 1] = make_float2(q.z, q.w);
            }
        }
    }
}

}  // namespace fpm
