// fused256.hpp -- register 256-point DFT building blocks of the Np 256 fused
// LED-update kernel (fpm_fused.hip): support-pruned 16-point DFTs, the
// four-step exchange variants and the twiddle holders.  Layout and pruning:
// see the fpm_fused.hip header.
#pragma once
#include <hip/hip_runtime.h>

#include "cpk.hpp"
#include "dft16.hpp"

namespace fpm {

// The register 16-point DFTs below compute in packed FP32 (cpk.hpp): every
// complex add/sub is one v_pk_add_f32, every twiddle multiply two VOP3P ops.
// Arrays are float2 at the interfaces (LDS and global memory) and pf2 inside;
// the conversions are bit casts of the same VGPR pairs.
template <int N>
__device__ __forceinline__ void to_pk(const float2 (&a)[N], pf2 (&p)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) p[i] = pin(a[i]);
}
template <int N>
__device__ __forceinline__ void from_pk(const pf2 (&p)[N], float2 (&a)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) a[i] = pout(p[i]);
}

// 16-point DFT whose input is zero except v[0,1,2,13,14,15]
template <bool INV>
__device__ __forceinline__ void pdft16_in6(const pf2 (&in)[16], pf2 (&r)[16]) {
    // stage 1, butterfly k1 over positions (k1, k1+4, k1+8, k1+12)
    const pf2 a0 = in[0], b1 = in[1], b13 = in[13], c2 = in[2], c14 = in[14], d15 = in[15];
    pf2 v[16];
    // k1 = 0: (a0,0,0,0)
    v[0] = a0; v[4] = a0; v[8] = a0; v[12] = a0;
    // k1 = 1: (b1,0,0,b13): U[m] = b1 + b13 W4^{3m};  W4^3 = conj(W4) = -W4
    v[1] = b1 + b13;
    v[5] = psub_w4<INV>(b1, b13);
    v[9] = b1 - b13;
    v[13] = padd_w4<INV>(b1, b13);
    v[2] = c2 + c14;
    v[6] = psub_w4<INV>(c2, c14);
    v[10] = c2 - c14;
    v[14] = padd_w4<INV>(c2, c14);
    // k1 = 3: (0,0,0,d15): U[m] = d15 W4^{3m}
    const pf2 z = {0.f, 0.f};
    v[3] = d15;
    v[7] = psub_w4<INV>(z, d15);
    v[11] = -d15;
    v[15] = padd_w4<INV>(z, d15);
    pmid_tw<INV>(v);
    pstage2<INV>(v);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// 16-point DFT returning only outputs m in {0,1,2,13,14,15} as o[0..5]
template <bool INV>
__device__ __forceinline__ void pdft16_out6(pf2 (&v)[16], pf2 (&o)[6]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) pbf4<INV>(v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    pmid_tw<INV>(v);
    // stage 2 over k1 for fixed m1 (positions 4 m1 + k1): y0 = sum, y3 = (a0-a2) - W4(a1-a3);
    // m1 = 2 carries the W16^4 twiddle of position 10 (a2 -> W4 a2)
    o[0] = (v[0] + v[2]) + (v[1] + v[3]);                          // m = 0  (m1 0, m2 0)
    o[1] = (v[4] + v[6]) + (v[5] + v[7]);                          // m = 1  (m1 1, m2 0)
    o[2] = padd_w4<INV>(v[8], v[10]) + (v[9] + v[11]);             // m = 2
    o[3] = psub_w4<INV>(v[4] - v[6], v[5] - v[7]);                 // m = 13 (m1 1, m2 3)
    o[4] = psub_w4<INV>(psub_w4<INV>(v[8], v[10]), v[9] - v[11]);  // m = 14
    o[5] = psub_w4<INV>(v[12] - v[14], v[13] - v[15]);             // m = 15
}

// 16-point DFT whose input is zero outside v[8H .. 8H+7] (one half of a row)
template <bool INV, int H>
__device__ __forceinline__ void pdft16_inhalf(pf2 (&v)[16], pf2 (&r)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        if (H == 0) {  // (a0, a1, 0, 0)
            const pf2 a0 = v[k1], a1 = v[k1 + 4];
            v[k1] = a0 + a1;
            v[k1 + 4] = padd_w4<INV>(a0, a1);
            v[k1 + 8] = a0 - a1;
            v[k1 + 12] = psub_w4<INV>(a0, a1);
        } else {       // (0, 0, a2, a3): W4^2 = -1, W4^3 = -W4
            const pf2 a2 = v[k1 + 8], a3 = v[k1 + 12];
            v[k1] = a2 + a3;
            v[k1 + 4] = -padd_w4<INV>(a2, a3);
            v[k1 + 8] = a2 - a3;
            v[k1 + 12] = -psub_w4<INV>(a2, a3);
        }
    }
    pmid_tw<INV>(v);
    pstage2<INV>(v);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// first radix-4 butterfly of a 16-point DFT with one non-zero input a in
// position Q of (k1, k1+4, k1+8, k1+12): a -> (a, W4^Q a, W4^2Q a, W4^3Q a)
template <bool INV, int Q>
__device__ __forceinline__ void pbf4_one(pf2 a, pf2 &y0, pf2 &y1, pf2 &y2, pf2 &y3) {
    const pf2 z = {0.f, 0.f};
    if constexpr (Q == 0) {
        y0 = a; y1 = a; y2 = a; y3 = a;
    } else if constexpr (Q == 1) {   // pbf4 of (0, a, 0, 0)
        y0 = a; y1 = padd_w4<INV>(z, a); y2 = -a; y3 = psub_w4<INV>(z, a);
    } else if constexpr (Q == 2) {   // (0, 0, a, 0)
        y0 = a; y1 = -a; y2 = a; y3 = -a;
    } else {                         // (0, 0, 0, a)
        y0 = a; y1 = psub_w4<INV>(z, a); y2 = -a; y3 = padd_w4<INV>(z, a);
    }
}

// 16-point DFT whose input is zero outside v[4Q .. 4Q+3] (one quarter of a
// row, split mode with four workgroups per patch): the first radix-4 stage
// sees one non-zero input per butterfly
template <bool INV, int Q>
__device__ __forceinline__ void pdft16_inquarter(pf2 (&v)[16], pf2 (&r)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) {
        const pf2 a = v[k1 + 4 * Q];
        pbf4_one<INV, Q>(a, v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    }
    pmid_tw<INV>(v);
    pstage2<INV>(v);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

// Four-step twiddles W256^{m t} (m = 0..15) of lane t, held in 32 VGPRs for a
// whole pass: a table read per use serialised on LDS latency at two waves per
// SIMD.
struct Tw {
    float2 w[16];
    __device__ __forceinline__ void load(const float2 *tw2, int t) {
#pragma unroll
        for (int m = 0; m < 16; ++m) w[m] = tw2[m * 16 + t];
    }
    __device__ __forceinline__ float2 operator[](int m) const { return w[m]; }
};

// inverse 256-point DFT (unscaled), input v[k] = X[t + 16 k] (only the six
// SK registers may be non-zero), output r[m2] = x[t + 16 m2]
template <class TW>
__device__ __forceinline__ void idft256_in6(float2 (&v)[16], float2 (&r)[16], float2 *scr, const TW &wt, int t,
                                            int xrd) {
    pf2 pv[16], py[16];
    to_pk(v, pv);
    pdft16_in6<true>(pv, py);
    ptwiddle15<true>(py, wt);
    float2 y[16];
    from_pk(py, y);
    exchange16(scr, t, xrd, y, v);
    to_pk(v, pv);
    pdft16<true>(pv, py);
    from_pk(py, r);
}

// forward 256-point DFT, input v[n2] = x[t + 16 n2], output o[s] = X[t + 16 SK[s]]
template <class TW>
__device__ __forceinline__ void dft256_out6(float2 (&v)[16], float2 (&o)[6], float2 *scr, const TW &wt, int t,
                                            int xrd) {
    pf2 pv[16], py[16], po[6];
    to_pk(v, pv);
    pdft16<false>(pv, py);
    ptwiddle15<false>(py, wt);
    float2 y[16];
    from_pk(py, y);
    exchange16(scr, t, xrd, y, v);
    to_pk(v, pv);
    pdft16_out6<false>(pv, po);
    from_pk(po, o);
}

// forward 256-point DFT of a half row (x = t + 16 n2, n2 in [8H, 8H+8), zero
// elsewhere), output o[s] = X[t + 16 SK[s]]
template <int H, class TW>
__device__ __forceinline__ void dft256_inhalf_out6(float2 (&v)[16], float2 (&o)[6], float2 *scr, const TW &wt, int t,
                                                   int xrd) {
    pf2 pv[16], py[16], po[6];
    to_pk(v, pv);
    pdft16_inhalf<false, H>(pv, py);
    ptwiddle15<false>(py, wt);
    float2 y[16];
    from_pk(py, y);
    exchange16(scr, t, xrd, y, v);
    to_pk(v, pv);
    pdft16_out6<false>(pv, po);
    from_pk(po, o);
}

// forward 256-point DFT of part P of NPARTS (x = t + 16 n2, n2 in
// [P 16/NPARTS, (P+1) 16/NPARTS), zero elsewhere), output o[s] = X[t + 16 SK[s]]
template <int NPARTS, int P, class TW>
__device__ __forceinline__ void dft256_inpart_out6(float2 (&v)[16], float2 (&o)[6], float2 *scr, const TW &wt,
                                                   int t, int xrd) {
    if constexpr (NPARTS == 2) {
        dft256_inhalf_out6<P>(v, o, scr, wt, t, xrd);
    } else {
        static_assert(NPARTS == 4, "two or four column parts");
        pf2 pv[16], py[16], po[6];
        to_pk(v, pv);
        pdft16_inquarter<false, P>(pv, py);
        ptwiddle15<false>(py, wt);
        float2 y[16];
        from_pk(py, y);
        exchange16(scr, t, xrd, y, v);
        to_pk(v, pv);
        pdft16_out6<false>(pv, po);
        from_pk(po, o);
    }
}

// pruned forward row DFT of column part h (block-uniform, 0 <= h < NPARTS):
// input row[16 m'] = x[t + 16 (h MPP + m')], m' < MPP = 16 / NPARTS, output
// o[s] = the part's contribution to X[t + 16 SK[s]].  One unrolled branch per
// part keeps every register index static.
template <int NPARTS, class TW, int HH = 0>
__device__ __forceinline__ void row_dft_part(const float2 *row, float2 (&v)[16], float2 (&o)[6], float2 *scr,
                                             const TW &wt, int t, int xrd, int h) {
    constexpr int MPP = 16 / NPARTS;
    if constexpr (HH < NPARTS) {
        if (HH == h) {
#pragma unroll
            for (int k = 0; k < 16; ++k) v[k] = make_float2(0.f, 0.f);
#pragma unroll
            for (int m = 0; m < MPP; ++m) v[HH * MPP + m] = row[16 * m];
            dft256_inpart_out6<NPARTS, HH>(v, o, scr, wt, t, xrd);
        } else {
            row_dft_part<NPARTS, TW, HH + 1>(row, v, o, scr, wt, t, xrd, h);
        }
    }
}

}  // namespace fpm
