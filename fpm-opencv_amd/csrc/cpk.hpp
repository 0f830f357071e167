// cpk.hpp -- packed-FP32 complex arithmetic for the register-resident DFTs.
//
// A complex value lives in one VGPR pair (re, im) and every complex add,
// subtract, multiply and W4 rotation is one or two VOP3P instructions
// (v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32) instead of two to four scalar
// ones.  Why it pays on gfx950 (tools/gpu/micro/valu_rate.hip, measured on
// MI355X): at two waves per SIMD -- the occupancy the fused LED-update kernel
// runs at -- the SIMD issues a scalar f32 instruction every 3.0-3.4 cycles
// (each wave issues one every ~6.9), but a packed one every 4.4 cycles, i.e.
// 2.2 cycles per f32 operation: the per-wave issue rate, not the f32 pipe, is
// the limit there, and a packed instruction does twice the work per issue.
// (At four waves per SIMD both forms approach the pipe's 2 cycles per f32
// operation, which is why a high-occupancy throughput test shows no gain.)
//
// Rounding is the scalar code's: packed f32 add/mul/fma are IEEE single
// operations on each half.  Swizzles the compiler folds into op_sel (a.yx,
// broadcasts a.xx / a.yy) are written as vector expressions; the W4 rotation
// "a + (-+i) b" needs a swap plus a one-lane negation, which the compiler
// does not fold (it emits v_xor + v_mov), so it is written as one VOP3P
// instruction with explicit op_sel / neg modifiers.
#pragma once
#include <hip/hip_runtime.h>

namespace fpm {

typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pf2 pin(float2 a) { return __builtin_bit_cast(pf2, a); }
__device__ __forceinline__ float2 pout(pf2 a) { return __builtin_bit_cast(float2, a); }

// Amplitude-replacement scale sqrt(I) / sqrt(mag2) (fpmMain.cpp:378-394, with
// mag2 = |psi + eps (1 + i)|^2 on the unscaled transform) for an integer
// measurement I >= 0: I * rsq(mag2 I + FLT_MIN), ONE transcendental (v_rsq_f32
// issues in 8 cycles, a plain VALU op in 4; MI355X_MICROARCH.md constants
// table) where rsq(mag2 * rcp(I)) needed two; the fma costs what the mul did.
// FLT_MIN keeps I = 0 finite: 0 * rsq(FLT_MIN) = 0, the reference's sqrt(0)
// factor (it is below the rounding of mag2 I for any I >= 1 and mag2 the
// solver meets).  -DFPM_AMP_RCP builds the two-transcendental form for A/B runs.
__device__ __forceinline__ float amp_scale(float mag2, float I) {
#ifdef FPM_AMP_RCP
    return __builtin_amdgcn_rsqf(mag2 * __builtin_amdgcn_rcpf(I));
#else
    return I * __builtin_amdgcn_rsqf(__builtin_fmaf(mag2, I, 1.17549435e-38f));
#endif
}

// a + W4 b with W4 = -i (forward) or +i (inverse):
//   -i b = (b.y, -b.x) -> (a.x + b.y, a.y - b.x);  +i b = (-b.y, b.x) -> (a.x - b.y, a.y + b.x)
// op_sel / op_sel_hi pick b.y for the low lane and b.x for the high lane.
template <bool INV>
__device__ __forceinline__ pf2 padd_w4(pf2 a, pf2 b) {
    pf2 r;
    if constexpr (INV)
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    else
        asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// a - W4 b = a + conj(W4) b
template <bool INV>
__device__ __forceinline__ pf2 psub_w4(pf2 a, pf2 b) {
    return padd_w4<!INV>(a, b);
}

// a * w:  (a.x w.x - a.y w.y, a.x w.y + a.y w.x) = a.xx * w + a.yy * (-w.y, w.x)
__device__ __forceinline__ pf2 pmul(pf2 a, pf2 w) {
    const pf2 r = a.xx * w;
    pf2 d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
        : "=v"(d)
        : "v"(a), "v"(w), "v"(r));
    return d;
}
// a * conj(w):  (a.x w.x + a.y w.y, a.y w.x - a.x w.y) = a * w.xx + a.yx * (w.y, -w.y)
__device__ __forceinline__ pf2 pmulc(pf2 a, pf2 w) {
    const pf2 r = a * w.xx;
    pf2 d;
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
        : "=v"(d)
        : "v"(a), "v"(w), "v"(r));
    return d;
}

// Twiddle multiplies of a 16-register column, py[m] *= w[m] (CONJ: by
// conj(w[m])) for m = 1..15, in three asm blocks of five: the five partial
// products first, then the five fmas, so no VOP3P read directly follows the
// VALU write it depends on.  With one pmul / pmulc per asm fma the compiler
// places each fma right after its mul and pays the hazard's wait state as an
// `s_nop 0` per twiddle (it cannot see into the asm, so it also pads the
// boundary of every block: fewer, larger blocks).
//   pmulc: t = a * w.xx, a = a.yx * (w.y, -w.y) + t
//   pmul:  t = a.xx * w, a = a.yy * (-w.y, w.x) + t
template <bool CONJ>
__device__ __forceinline__ void ptw5(pf2 &a0, pf2 &a1, pf2 &a2, pf2 &a3, pf2 &a4, pf2 w0, pf2 w1, pf2 w2, pf2 w3,
                                     pf2 w4) {
    pf2 t0, t1, t2, t3, t4;
    if constexpr (CONJ)
        asm("v_pk_mul_f32 %0, %5, %10 op_sel_hi:[1,0]\n\t"
            "v_pk_mul_f32 %1, %6, %11 op_sel_hi:[1,0]\n\t"
            "v_pk_mul_f32 %2, %7, %12 op_sel_hi:[1,0]\n\t"
            "v_pk_mul_f32 %3, %8, %13 op_sel_hi:[1,0]\n\t"
            "v_pk_mul_f32 %4, %9, %14 op_sel_hi:[1,0]\n\t"
            "v_pk_fma_f32 %5, %5, %10, %0 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]\n\t"
            "v_pk_fma_f32 %6, %6, %11, %1 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]\n\t"
            "v_pk_fma_f32 %7, %7, %12, %2 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]\n\t"
            "v_pk_fma_f32 %8, %8, %13, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]\n\t"
            "v_pk_fma_f32 %9, %9, %14, %4 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4)
            : "v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(w4));
    else
        asm("v_pk_mul_f32 %0, %5, %10 op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %1, %6, %11 op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %2, %7, %12 op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %3, %8, %13 op_sel_hi:[0,1]\n\t"
            "v_pk_mul_f32 %4, %9, %14 op_sel_hi:[0,1]\n\t"
            "v_pk_fma_f32 %5, %5, %10, %0 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
            "v_pk_fma_f32 %6, %6, %11, %1 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
            "v_pk_fma_f32 %7, %7, %12, %2 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
            "v_pk_fma_f32 %8, %8, %13, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
            "v_pk_fma_f32 %9, %9, %14, %4 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]"
            : "=&v"(t0), "=&v"(t1), "=&v"(t2), "=&v"(t3), "=&v"(t4), "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4)
            : "v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(w4));
}
template <bool CONJ, class TW>
__device__ __forceinline__ void ptwiddle15(pf2 (&py)[16], const TW &wt) {
#ifndef FPM_TW_SINGLE  // A/B: one asm fma per twiddle (round 2)
#pragma unroll
    for (int m = 1; m < 16; m += 5)
        ptw5<CONJ>(py[m], py[m + 1], py[m + 2], py[m + 3], py[m + 4], pin(wt[m]), pin(wt[m + 1]), pin(wt[m + 2]),
                   pin(wt[m + 3]), pin(wt[m + 4]));
#else
#pragma unroll
    for (int m = 1; m < 16; ++m) py[m] = CONJ ? pmulc(py[m], pin(wt[m])) : pmul(py[m], pin(wt[m]));
#endif
}

// radix-4 butterfly in place (the scalar dft4 of fft_lds.hpp, packed)
template <bool INV>
__device__ __forceinline__ void pbf4(pf2 &a0, pf2 &a1, pf2 &a2, pf2 &a3) {
    const pf2 s02 = a0 + a2, d02 = a0 - a2, s13 = a1 + a3, e13 = a1 - a3;
    a0 = s02 + s13;
    a2 = s02 - s13;
    a1 = padd_w4<INV>(d02, e13);
    a3 = psub_w4<INV>(d02, e13);
}
// the same with a2 pre-multiplied by W4 (the W16^4 mid twiddle folded in)
template <bool INV>
__device__ __forceinline__ void pbf4_w2(pf2 &a0, pf2 &a1, pf2 &a2, pf2 &a3) {
    // a2' = W4 a2; s02 = a0 + W4 a2, d02 = a0 - W4 a2
    const pf2 s02 = padd_w4<INV>(a0, a2), d02 = psub_w4<INV>(a0, a2), s13 = a1 + a3, e13 = a1 - a3;
    a0 = s02 + s13;
    a2 = s02 - s13;
    a1 = padd_w4<INV>(d02, e13);
    a3 = psub_w4<INV>(d02, e13);
}

// a * W16^{+-j} for the constant mid twiddles of the 16-point DFT
// (forward W16^j = c - i s; the inverse conjugates); j = 4 is folded into
// pbf4_w2 by the callers
template <bool INV, int J>
__device__ __forceinline__ pf2 pw16(pf2 a) {
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    if constexpr (J == 2) {  // (1 -+ i) R2: forward (a.x + a.y, a.y - a.x) R2
        return padd_w4<INV>(a, a) * R2;
    } else if constexpr (J == 6) {  // (-1 -+ i) R2 = -(1 +- i) R2
        return padd_w4<!INV>(a, a) * (-R2);
    } else {
        constexpr float c = J == 1 ? C1 : J == 3 ? S1 : -C1;  // J = 9: W16^9 = -W16^1
        constexpr float s = J == 1 ? S1 : J == 3 ? C1 : -S1;
        constexpr float si = INV ? -s : s;
        // (a.x c + a.y si, a.y c - a.x si)
        return __builtin_elementwise_fma(a.yx, (pf2){si, -si}, a * c);
    }
}

// twiddles between the two radix-4 stages of the 16-point DFT:
// position k1 + 4 m1 *= W16^{k1 m1}; position 10 (W16^4) is left to pbf4_w2
template <bool INV>
__device__ __forceinline__ void pmid_tw(pf2 (&v)[16]) {
    v[5] = pw16<INV, 1>(v[5]);
    v[6] = pw16<INV, 2>(v[6]);
    v[7] = pw16<INV, 3>(v[7]);
    v[9] = pw16<INV, 2>(v[9]);
    v[11] = pw16<INV, 6>(v[11]);
    v[13] = pw16<INV, 3>(v[13]);
    v[14] = pw16<INV, 6>(v[14]);
    v[15] = pw16<INV, 9>(v[15]);
}
// second radix-4 stage over positions 4 m1 + k1 (k1 = 0..3), m1 = 2 with the
// W16^4 twiddle of position 10 folded in
template <bool INV>
__device__ __forceinline__ void pstage2(pf2 (&v)[16]) {
    pbf4<INV>(v[0], v[1], v[2], v[3]);
    pbf4<INV>(v[4], v[5], v[6], v[7]);
    pbf4_w2<INV>(v[8], v[9], v[10], v[11]);
    pbf4<INV>(v[12], v[13], v[14], v[15]);
}

// dense 16-point DFT: in v[k], out r[m] = sum_k v[k] W16^{+-km}
template <bool INV>
__device__ __forceinline__ void pdft16(pf2 (&v)[16], pf2 (&r)[16]) {
#pragma unroll
    for (int k1 = 0; k1 < 4; ++k1) pbf4<INV>(v[k1], v[k1 + 4], v[k1 + 8], v[k1 + 12]);
    pmid_tw<INV>(v);
    pstage2<INV>(v);
#pragma unroll
    for (int m = 0; m < 16; ++m) r[m] = v[4 * (m & 3) + (m >> 2)];
}

}  // namespace fpm
