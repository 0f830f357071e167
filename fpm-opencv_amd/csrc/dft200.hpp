// dft200.hpp -- register-resident 200-point DFT of a 10-lane group (20 x 10
// four-step, packed FP32), shared by the Np 200 fused LED-update kernel
// (fused_mr.hip) and the L = 600 objCrop transform (objcrop.hip).
//
//   lane l holds x[l + 10 k], k = 0..19 (the "slot layout").  Stage 1 is a
//   20-point DFT over the registers (5 x 4), then the twiddles W200^{l m1}, one
//   LDS exchange in two rounds (m1 < 10, then m1 >= 10: lane l' reads row l' of
//   a 10 x 10 tile each time), and stage 2 is two 10-point DFTs (5 x 2) per
//   lane (m1 = l' and m1 = l' + 10).  Their outputs X[m1 + 20 m2] land in
//   register k = 2 m2 (+1 for m1 = l' + 10): the slot layout again.
#pragma once
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "fft_lds.hpp"

namespace fpm {

constexpr int kXP10 = 10;  // exchange-tile row pitch (complex) of xchg10

// ----------------------------------------------------- compile-time twiddles
constexpr double kPi = 3.14159265358979323846;
constexpr double ct_sin(double x) {  // |x| <= pi/2 after reduction below
    double term = x, sum = x;
    for (int n = 1; n < 14; ++n) {
        term *= -x * x / ((2.0 * n) * (2.0 * n + 1.0));
        sum += term;
    }
    return sum;
}
// exp(-2 pi i j / n) for the forward transform (angle reduced to [0, 2 pi))
struct CW {
    float re, im;
};
constexpr CW cw(int j, int n) {
    j %= n;
    if (j < 0) j += n;
    double a = 2.0 * kPi * j / n;  // [0, 2 pi)
    double s = 0, c = 0;
    if (a <= kPi / 2) {
        s = ct_sin(a);
        c = ct_sin(kPi / 2 - a);
    } else if (a <= kPi) {
        s = ct_sin(kPi - a);
        c = -ct_sin(a - kPi / 2);
    } else if (a <= 3 * kPi / 2) {
        s = -ct_sin(a - kPi);
        c = -ct_sin(3 * kPi / 2 - a);
    } else {
        s = -ct_sin(2 * kPi - a);
        c = ct_sin(a - 3 * kPi / 2);
    }
    return CW{(float)c, (float)-s};
}
// a * W_n^{+-j} with a compile-time twiddle (forward: W = exp(-2 pi i/n)),
// packed FP32 (cpk.hpp): (a.x wr - a.y wi, a.x wi + a.y wr) = a wr + a.yx (-wi, wi)
template <bool INV, int J, int N>
__device__ __forceinline__ pf2 twc(pf2 a) {
    constexpr CW w = cw(J, N);
    constexpr float wr = w.re, wi = INV ? -w.im : w.im;
    if constexpr (J % N == 0) return a;
    return __builtin_elementwise_fma(a.yx, (pf2){-wi, wi}, a * wr);
}

// ------------------------------------------------------- register DFTs (packed)
// 5-point DFT in place (the scalar dft5 of fft_lds.hpp)
template <bool INV>
__device__ __forceinline__ void pdft5(pf2 *v) {
    constexpr float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    constexpr float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const pf2 t1 = v[1] + v[4], d1 = v[1] - v[4];
    const pf2 t2 = v[2] + v[3], d2 = v[2] - v[3];
    const pf2 a0 = v[0];
    const pf2 r1 = __builtin_elementwise_fma(t2, (pf2){c2, c2}, __builtin_elementwise_fma(t1, (pf2){c1, c1}, a0));
    const pf2 r2 = __builtin_elementwise_fma(t2, (pf2){c1, c1}, __builtin_elementwise_fma(t1, (pf2){c2, c2}, a0));
    const pf2 q1 = __builtin_elementwise_fma(d2, (pf2){s2, s2}, d1 * s1);
    const pf2 q2 = __builtin_elementwise_fma(d2, (pf2){-s1, -s1}, d1 * s2);
    v[0] = a0 + (t1 + t2);
    v[1] = padd_w4<INV>(r1, q1);
    v[4] = psub_w4<INV>(r1, q1);
    v[2] = padd_w4<INV>(r2, q2);
    v[3] = psub_w4<INV>(r2, q2);
}

// 10-point DFT, natural order in and out: k = k1 + 2 k2, m = j2 + 5 j1
template <bool INV>
__device__ __forceinline__ void dft10(pf2 (&v)[10]) {
    pf2 e[5] = {v[0], v[2], v[4], v[6], v[8]}, o[5] = {v[1], v[3], v[5], v[7], v[9]};
    pdft5<INV>(e);
    pdft5<INV>(o);
    o[1] = twc<INV, 1, 10>(o[1]);
    o[2] = twc<INV, 2, 10>(o[2]);
    o[3] = twc<INV, 3, 10>(o[3]);
    o[4] = twc<INV, 4, 10>(o[4]);
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        v[j] = e[j] + o[j];
        v[j + 5] = e[j] - o[j];
    }
}

// 20-point DFT, natural order in and out: k = k1 + 4 k2 (DFT5 over k2), then
// W20^{k1 j2}, then DFT4 over k1: m = j2 + 5 j1
template <bool INV>
__device__ __forceinline__ void dft20(pf2 (&v)[20]) {
    pf2 u[4][5];
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
#pragma unroll
        for (int k2 = 0; k2 < 5; ++k2) u[k1][k2] = v[k1 + 4 * k2];
        pdft5<INV>(u[k1]);
    }
    u[1][1] = twc<INV, 1, 20>(u[1][1]);
    u[1][2] = twc<INV, 2, 20>(u[1][2]);
    u[1][3] = twc<INV, 3, 20>(u[1][3]);
    u[1][4] = twc<INV, 4, 20>(u[1][4]);
    u[2][1] = twc<INV, 2, 20>(u[2][1]);
    u[2][2] = twc<INV, 4, 20>(u[2][2]);
    u[2][3] = twc<INV, 6, 20>(u[2][3]);
    u[2][4] = twc<INV, 8, 20>(u[2][4]);
    u[3][1] = twc<INV, 3, 20>(u[3][1]);
    u[3][2] = twc<INV, 6, 20>(u[3][2]);
    u[3][3] = twc<INV, 9, 20>(u[3][3]);
    u[3][4] = twc<INV, 12, 20>(u[3][4]);
#pragma unroll
    for (int j2 = 0; j2 < 5; ++j2) {
        pbf4<INV>(u[0][j2], u[1][j2], u[2][j2], u[3][j2]);
        v[j2] = u[0][j2];
        v[j2 + 5] = u[1][j2];
        v[j2 + 10] = u[2][j2];
        v[j2 + 15] = u[3][j2];
    }
}

// the same with only v[0,1,2,17,18,19] non-zero (k1,k2) = (0,0),(1,0),(2,0),
// (1,4),(2,4),(3,4): the DFT5s collapse to one or two terms
template <bool INV>
__device__ __forceinline__ void dft20_in6(pf2 (&v)[20]) {
    const pf2 a0 = v[0], a1 = v[1], a2 = v[2], b1 = v[17], b2 = v[18], b3 = v[19];
    pf2 u[4][5];
    // DFT5 of (x, 0, 0, 0, y): U[j] = x + y W5^{4 j}
#pragma unroll
    for (int j = 0; j < 5; ++j) u[0][j] = a0;
    u[1][0] = a1 + b1;
    u[1][1] = a1 + twc<INV, 4, 5>(b1);
    u[1][2] = a1 + twc<INV, 8, 5>(b1);
    u[1][3] = a1 + twc<INV, 12, 5>(b1);
    u[1][4] = a1 + twc<INV, 16, 5>(b1);
    u[2][0] = a2 + b2;
    u[2][1] = a2 + twc<INV, 4, 5>(b2);
    u[2][2] = a2 + twc<INV, 8, 5>(b2);
    u[2][3] = a2 + twc<INV, 12, 5>(b2);
    u[2][4] = a2 + twc<INV, 16, 5>(b2);
    u[1][1] = twc<INV, 1, 20>(u[1][1]);
    u[1][2] = twc<INV, 2, 20>(u[1][2]);
    u[1][3] = twc<INV, 3, 20>(u[1][3]);
    u[1][4] = twc<INV, 4, 20>(u[1][4]);
    u[2][1] = twc<INV, 2, 20>(u[2][1]);
    u[2][2] = twc<INV, 4, 20>(u[2][2]);
    u[2][3] = twc<INV, 6, 20>(u[2][3]);
    u[2][4] = twc<INV, 8, 20>(u[2][4]);
    // u[3][j] = b3 W5^{4j} W20^{3j} = b3 W20^{16j + 3j} = b3 W20^{19 j}
    u[3][0] = b3;
    u[3][1] = twc<INV, 19, 20>(b3);
    u[3][2] = twc<INV, 38, 20>(b3);
    u[3][3] = twc<INV, 57, 20>(b3);
    u[3][4] = twc<INV, 76, 20>(b3);
#pragma unroll
    for (int j2 = 0; j2 < 5; ++j2) {
        pbf4<INV>(u[0][j2], u[1][j2], u[2][j2], u[3][j2]);
        v[j2] = u[0][j2];
        v[j2 + 5] = u[1][j2];
        v[j2 + 10] = u[2][j2];
        v[j2 + 15] = u[3][j2];
    }
}

__device__ __forceinline__ int opaque_i(int v) {
    asm volatile("" : "+v"(v));
    return v;
}

// Four-step exchange of a 10-lane group: lane n2 holds U[m1], m1 = 0..19; lane
// l' receives U_of_lane_j[l'] (za) and U_of_lane_j[l' + 10] (zb), j = 0..9.
// Two rounds through a 10 x 10 tile (row m1 mod 10 written by all lanes, row
// l' read by lane l'); LDS operations of one wave execute in issue order and
// the laundered read base `xrd` keeps the compiler from moving the second
// round's writes above the first round's reads (see dft16.hpp exchange16).
__device__ __forceinline__ void xchg10(float2 *tile, int l, int xrd, const float2 (&u)[20], float2 (&za)[10],
                                       float2 (&zb)[10]) {
    const float4 *rp = (const float4 *)(tile + xrd);
#pragma unroll
    for (int m = 0; m < 10; ++m) tile[m * kXP10 + l] = u[m];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float4 q = rp[j];
        za[2 * j] = make_float2(q.x, q.y);
        za[2 * j + 1] = make_float2(q.z, q.w);
    }
#pragma unroll
    for (int m = 0; m < 10; ++m) tile[m * kXP10 + l] = u[10 + m];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const float4 q = rp[j];
        zb[2 * j] = make_float2(q.x, q.y);
        zb[2 * j + 1] = make_float2(q.z, q.w);
    }
}

// 200-point DFT in the slot layout (in and out: register k <-> index l + 10 k).
// INV: inverse (unscaled); IN6: only the input registers {0,1,2,17,18,19} are
// non-zero (the fused kernel's support-pruned inverse).
// tw2[m1 * 10 + l] = W200^{l m1} (forward), read per use from LDS.
template <bool INV, bool IN6>
__device__ __forceinline__ void dft200(float2 (&v)[20], float2 *tile, const float2 *tw2, int l, int xrd) {
    pf2 p[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) p[k] = pin(v[k]);
    if (IN6) dft20_in6<INV>(p);
    else dft20<INV>(p);
    {
        pf2 w[20];
#pragma unroll
        for (int m1 = 1; m1 < 20; ++m1) w[m1] = pin(tw2[m1 * 10 + l]);
        w[0] = w[1];
        ptw_range<INV, 20>(p, w);  // cpk.hpp: blocks of products, then fmas
    }
    float2 u[20];
#pragma unroll
    for (int k = 0; k < 20; ++k) u[k] = pout(p[k]);
    float2 za[10], zb[10];
    xchg10(tile, l, xrd, u, za, zb);
    pf2 pa[10], pb[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        pa[k] = pin(za[k]);
        pb[k] = pin(zb[k]);
    }
    dft10<INV>(pa);
    dft10<INV>(pb);
    // X[m1 + 20 m2]: m1 = l' -> register 2 m2, m1 = l' + 10 -> register 2 m2 + 1
#pragma unroll
    for (int m2 = 0; m2 < 10; ++m2) {
        v[2 * m2] = pout(pa[m2]);
        v[2 * m2 + 1] = pout(pb[m2]);
    }
}

}  // namespace fpm
