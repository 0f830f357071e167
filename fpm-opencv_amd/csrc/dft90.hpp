// dft90.hpp -- register-resident 90-point DFT of a 10-lane group (9 x 10
// four-step, packed FP32) for the Np 90 fused LED-update kernel
// (fused_s90.hip; BASELINE configs 1 and 2, dataset_mono: Np 90).
//
// Two layouts of a 90-point sequence over the ten lanes of a group:
//   A: lane l < 10 holds x[l + 10 k], k = 0..8  (nine registers)
//   B: lane j <  9 holds x[j +  9 k], k = 0..9  (ten registers; lane 9 idle)
// dft90_ab maps A -> B:  X[m1 + 9 m2] = sum_l W10^{l m2} W90^{l m1} U_l[m1],
//   U_l = DFT9 over lane l's registers; lane j = m1 then runs the DFT10.
// dft90_ba maps B -> A (the transposed algorithm):
//   X[m + 10 q] = sum_j W9^{j q} W90^{j m} Z_j[m], Z_j = DFT10 of lane j;
//   lane m runs the DFT9.
// So an inverse A -> B followed by a forward B -> A needs no reordering: the
// column pass of the fused kernel transforms, replaces amplitudes in layout B
// and transforms back into the box rows of layout A.  One LDS exchange per
// transform through a 10 x 10 tile of the group (row pitch kXP90).
#pragma once
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "dft200.hpp"

namespace fpm {

constexpr int kXP90 = 10;  // exchange-tile row pitch (complex); a tile is 10 rows

// 3-point DFT in place, packed: y1 = m + W4 h d, y2 = m - W4 h d (W4 = -i forward)
template <bool INV>
__device__ __forceinline__ void pdft3(pf2 &a0, pf2 &a1, pf2 &a2) {
    constexpr float h = 0.86602540378443864676f;  // sqrt(3) / 2
    const pf2 t = a1 + a2, d = (a1 - a2) * h;
    const pf2 m = __builtin_elementwise_fma(t, (pf2){-0.5f, -0.5f}, a0);
    a0 = a0 + t;
    a1 = padd_w4<INV>(m, d);
    a2 = psub_w4<INV>(m, d);
}

// 9-point DFT, natural order in and out: n = 3 n1 + n2, k = k1 + 3 k2
template <bool INV>
__device__ __forceinline__ void dft9(pf2 (&v)[9]) {
    pf2 u[3][3];  // u[n2][k1], then u[k2][k1]
#pragma unroll
    for (int n2 = 0; n2 < 3; ++n2) {
        u[n2][0] = v[n2];
        u[n2][1] = v[3 + n2];
        u[n2][2] = v[6 + n2];
        pdft3<INV>(u[n2][0], u[n2][1], u[n2][2]);
    }
    u[1][1] = twc<INV, 1, 9>(u[1][1]);
    u[1][2] = twc<INV, 2, 9>(u[1][2]);
    u[2][1] = twc<INV, 2, 9>(u[2][1]);
    u[2][2] = twc<INV, 4, 9>(u[2][2]);
#pragma unroll
    for (int k1 = 0; k1 < 3; ++k1) {
        pdft3<INV>(u[0][k1], u[1][k1], u[2][k1]);
        v[k1] = u[0][k1];
        v[k1 + 3] = u[1][k1];
        v[k1 + 6] = u[2][k1];
    }
}

// layout A (v[0..8]) -> layout B (v[0..9], lanes 0..8).  tw[a * 10 + b] =
// W90^{a b} (forward), a, b < 10, read per use from LDS; xrd = l * kXP90,
// laundered (opaque_i) so the reads stay behind the writes.
template <bool INV>
__device__ __forceinline__ void dft90_ab(float2 (&v)[10], float2 *tile, const float2 *tw, int l, int xrd) {
    pf2 p[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) p[k] = pin(v[k]);
    dft9<INV>(p);
#pragma unroll
    for (int m1 = 1; m1 < 9; m1 += 2) {
        const pf2 w[2] = {pin(tw[m1 * 10 + l]), pin(tw[(m1 + 1) * 10 + l])};
        ptw_block<INV, 2>(&p[m1], w);
    }
#pragma unroll
    for (int m1 = 0; m1 < 9; ++m1) tile[m1 * kXP90 + l] = pout(p[m1]);
    // lane j reads row j (lane 9: row 9, never written -- its output is unused)
    const float4 *rp = (const float4 *)(tile + xrd);
    pf2 z[10];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const float4 q = rp[i];
        z[2 * i] = (pf2){q.x, q.y};
        z[2 * i + 1] = (pf2){q.z, q.w};
    }
    dft10<INV>(z);
#pragma unroll
    for (int m2 = 0; m2 < 10; ++m2) v[m2] = pout(z[m2]);
}

// layout B (v[0..9], lanes 0..8; lane 9's registers are ignored) -> layout A
// (v[0..8], lanes 0..9)
template <bool INV>
__device__ __forceinline__ void dft90_ba(float2 (&v)[10], float2 *tile, const float2 *tw, int l, int xrd) {
    pf2 p[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) p[k] = pin(v[k]);
    dft10<INV>(p);
#pragma unroll
    for (int m = 1; m < 9; m += 2) {
        const pf2 w[2] = {pin(tw[m * 10 + l]), pin(tw[(m + 1) * 10 + l])};
        ptw_block<INV, 2>(&p[m], w);
    }
    p[9] = INV ? pmulc(p[9], pin(tw[90 + l])) : pmul(p[9], pin(tw[90 + l]));
    // row m, column j; lane 9 writes the pad column (never read)
#pragma unroll
    for (int m = 0; m < 10; ++m) tile[m * kXP90 + l] = pout(p[m]);
    const float4 *rp = (const float4 *)(tile + xrd);
    pf2 z[9];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float4 q = rp[i];
        z[2 * i] = (pf2){q.x, q.y};
        z[2 * i + 1] = (pf2){q.z, q.w};
    }
    {
        const float2 q = *(const float2 *)(tile + xrd + 8);
        z[8] = (pf2){q.x, q.y};
    }
    dft9<INV>(z);
#pragma unroll
    for (int q = 0; q < 9; ++q) v[q] = pout(z[q]);
}

}  // namespace fpm
