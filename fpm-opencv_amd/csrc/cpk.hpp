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
// solver meets).
__device__ __forceinline__ float amp_scale(float mag2, float I) {
    return I * __builtin_amdgcn_rsqf(__builtin_fmaf(mag2, I, 1.17549435e-38f));
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
// one partial product / one fma of a twiddle multiply in asm text (operand
// numbers are literal tokens); C: conjugate twiddle (pmulc), F: pmul
#define FPM_TWMUL_C(t, a, w) "v_pk_mul_f32 %" #t ", %" #a ", %" #w " op_sel_hi:[1,0]\n\t"
#define FPM_TWFMA_C(a, w, t) "v_pk_fma_f32 %" #a ", %" #a ", %" #w ", %" #t " op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]\n\t"
#define FPM_TWMUL_F(t, a, w) "v_pk_mul_f32 %" #t ", %" #a ", %" #w " op_sel_hi:[0,1]\n\t"
#define FPM_TWFMA_F(a, w, t) "v_pk_fma_f32 %" #a ", %" #a ", %" #w ", %" #t " op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]\n\t"
// blocks of N = 2 .. 5 twiddles: operands t0..t(N-1), a0..a(N-1), w0..w(N-1)
#define FPM_TW2(K) FPM_TWMUL_##K(0, 2, 4) FPM_TWMUL_##K(1, 3, 5) FPM_TWFMA_##K(2, 4, 0) FPM_TWFMA_##K(3, 5, 1)
#define FPM_TW3(K) FPM_TWMUL_##K(0, 3, 6) FPM_TWMUL_##K(1, 4, 7) FPM_TWMUL_##K(2, 5, 8) \
    FPM_TWFMA_##K(3, 6, 0) FPM_TWFMA_##K(4, 7, 1) FPM_TWFMA_##K(5, 8, 2)
#define FPM_TW4(K) FPM_TWMUL_##K(0, 4, 8) FPM_TWMUL_##K(1, 5, 9) FPM_TWMUL_##K(2, 6, 10) FPM_TWMUL_##K(3, 7, 11) \
    FPM_TWFMA_##K(4, 8, 0) FPM_TWFMA_##K(5, 9, 1) FPM_TWFMA_##K(6, 10, 2) FPM_TWFMA_##K(7, 11, 3)
#define FPM_TW5(K) FPM_TWMUL_##K(0, 5, 10) FPM_TWMUL_##K(1, 6, 11) FPM_TWMUL_##K(2, 7, 12) FPM_TWMUL_##K(3, 8, 13) \
    FPM_TWMUL_##K(4, 9, 14) FPM_TWFMA_##K(5, 10, 0) FPM_TWFMA_##K(6, 11, 1) FPM_TWFMA_##K(7, 12, 2)                \
    FPM_TWFMA_##K(8, 13, 3) FPM_TWFMA_##K(9, 14, 4)
// a[i] *= w[i] (CONJ: conj(w[i])) for i < N, N = 2..5, in one asm block
template <bool CONJ, int N>
__device__ __forceinline__ void ptw_block(pf2 *a, const pf2 *w) {
    static_assert(N >= 2 && N <= 5, "block of 2..5 twiddles");
    pf2 t[N];
    if constexpr (N == 2) {
        if constexpr (CONJ)
            asm(FPM_TW2(C) : "=&v"(t[0]), "=&v"(t[1]), "+v"(a[0]), "+v"(a[1]) : "v"(w[0]), "v"(w[1]));
        else
            asm(FPM_TW2(F) : "=&v"(t[0]), "=&v"(t[1]), "+v"(a[0]), "+v"(a[1]) : "v"(w[0]), "v"(w[1]));
    } else if constexpr (N == 3) {
        if constexpr (CONJ)
            asm(FPM_TW3(C) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "+v"(a[0]), "+v"(a[1]), "+v"(a[2])
                : "v"(w[0]), "v"(w[1]), "v"(w[2]));
        else
            asm(FPM_TW3(F) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "+v"(a[0]), "+v"(a[1]), "+v"(a[2])
                : "v"(w[0]), "v"(w[1]), "v"(w[2]));
    } else if constexpr (N == 4) {
        if constexpr (CONJ)
            asm(FPM_TW4(C) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]),
                "+v"(a[3]) : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
        else
            asm(FPM_TW4(F) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "+v"(a[0]), "+v"(a[1]), "+v"(a[2]),
                "+v"(a[3]) : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
    } else {
        if constexpr (CONJ)
            asm(FPM_TW5(C) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "+v"(a[0]), "+v"(a[1]),
                "+v"(a[2]), "+v"(a[3]), "+v"(a[4]) : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]));
        else
            asm(FPM_TW5(F) : "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]), "+v"(a[0]), "+v"(a[1]),
                "+v"(a[2]), "+v"(a[3]), "+v"(a[4]) : "v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]), "v"(w[4]));
    }
}
// a[i] *= w[i] for i in [1, M) (a[0] has no twiddle) in blocks of 3..5
template <bool CONJ, int M>
__device__ __forceinline__ void ptw_range(pf2 (&a)[M > 0 ? M : 1], const pf2 (&w)[M > 0 ? M : 1]) {
    constexpr int n = M - 1;                          // twiddles
    constexpr int nb = (n + 4) / 5;                   // blocks
#pragma unroll
    for (int b = 0, i = 1; b < nb; ++b) {
        const int len = (n - (i - 1)) / (nb - b);     // spread evenly: every block 3..5
        if (len == 5) ptw_block<CONJ, 5>(&a[i], &w[i]);
        else if (len == 4) ptw_block<CONJ, 4>(&a[i], &w[i]);
        else ptw_block<CONJ, 3>(&a[i], &w[i]);
        i += len;
    }
}
template <bool CONJ, class TW>
__device__ __forceinline__ void ptwiddle15(pf2 (&py)[16], const TW &wt) {
    pf2 w[16];
#pragma unroll
    for (int m = 1; m < 16; ++m) w[m] = pin(wt[m]);
    w[0] = w[1];
    ptw_range<CONJ, 16>(py, w);
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
    // the same operations, first steps of all eight twiddles before the
    // second steps (no VOP3P read right after the write it depends on; the
    // four W4 rotations in one asm block: no padding between blocks)
    constexpr float C1 = 0.92387953251128675613f, S1 = 0.38268343236508977173f, R2 = 0.70710678118654752440f;
    constexpr float s1 = INV ? -S1 : S1, s3 = INV ? -C1 : C1;  // J = 1: (C1, S1); J = 3: (S1, C1); J = 9: -(C1, S1)
    const pf2 t5 = v[5] * C1, t7 = v[7] * S1, t13 = v[13] * S1, t15 = v[15] * (-C1);
    pf2 u6, u9, u11, u14;  // (1 -+ i) a for J = 2, (1 +- i) a for J = 6
    if constexpr (INV)
        asm("v_pk_add_f32 %0, %4, %4 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
            "v_pk_add_f32 %1, %5, %5 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
            "v_pk_add_f32 %2, %6, %6 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %3, %7, %7 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]"
            : "=&v"(u6), "=&v"(u9), "=&v"(u11), "=v"(u14)
            : "v"(v[6]), "v"(v[9]), "v"(v[11]), "v"(v[14]));
    else
        asm("v_pk_add_f32 %0, %4, %4 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %1, %5, %5 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
            "v_pk_add_f32 %2, %6, %6 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
            "v_pk_add_f32 %3, %7, %7 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
            : "=&v"(u6), "=&v"(u9), "=&v"(u11), "=v"(u14)
            : "v"(v[6]), "v"(v[9]), "v"(v[11]), "v"(v[14]));
    v[5] = __builtin_elementwise_fma(v[5].yx, (pf2){s1, -s1}, t5);
    v[7] = __builtin_elementwise_fma(v[7].yx, (pf2){s3, -s3}, t7);
    v[13] = __builtin_elementwise_fma(v[13].yx, (pf2){s3, -s3}, t13);
    v[15] = __builtin_elementwise_fma(v[15].yx, (pf2){-s1, s1}, t15);
    v[6] = u6 * R2;
    v[9] = u9 * R2;
    v[11] = u11 * (-R2);
    v[14] = u14 * (-R2);
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
