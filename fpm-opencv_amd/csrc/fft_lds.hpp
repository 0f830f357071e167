// fft_lds.hpp -- mixed-radix (2/3/4/5/8) Stockham FFT over LDS-resident
// sequences, plus the complex helpers shared by every FPM kernel.
//
// Replaces the reference's cvComplex fft2/ifft2 and cv::dft calls
// (fpmMain.cpp:325,365,394,481) for arbitrary sizes N = 2^a 3^b 5^c: this is
// the general path.  The metric-config hot loop uses the register-resident
// 16x16 four-step transform in fpm_fused.hip instead.
//
// Stockham autosort (no bit reversal): pass p with radix R and current
// sub-transform length Ns maps butterfly j to
//     v[r] = src[j + r*N/R] * w^(r*(j mod Ns)),   w = exp(-+2 pi i/(Ns R))
//     dst[(j/Ns)*Ns*R + (j mod Ns) + r*Ns] = DFT_R(v)[r]
// Twiddles come from a host-computed (double precision) table
// tw[k] = exp(-2 pi i k/N); the inverse uses the conjugate.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace fpm {

struct FftPlan {
    int n;
    int nstages;
    int radix[24];
};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cconj(float2 a) { return make_float2(a.x, -a.y); }
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
// multiply by -i (forward) or +i (inverse)
template <bool INV>
__device__ __forceinline__ float2 mul_mi(float2 a) {
    return INV ? make_float2(-a.y, a.x) : make_float2(a.y, -a.x);
}
// |a|^2 with an explicit fma so every kernel rounds it identically (the fused
// path compares tile maxima bit for bit with freshly computed magnitudes)
__device__ __forceinline__ float cabs2(float2 a) { return __builtin_fmaf(a.x, a.x, a.y * a.y); }
// |a| as stored in the tile maxima: every kernel that writes or compares a
// tile maximum uses this one function (raw v_sqrt_f32, no denormal fix-up)
__device__ __forceinline__ float cmag(float2 a) { return __builtin_amdgcn_sqrtf(cabs2(a)); }

template <bool INV>
__device__ __forceinline__ void dft2(float2 *v) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b);
    v[1] = csub(a, b);
}

template <bool INV>
__device__ __forceinline__ void dft4(float2 *v) {
    float2 s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
    float2 s13 = cadd(v[1], v[3]), d13 = mul_mi<INV>(csub(v[1], v[3]));
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    v[1] = cadd(d02, d13);
    v[3] = csub(d02, d13);
}

// radix 8 as two radix-4 DFTs (even / odd inputs) and one radix-2 stage with
// the W8^k twiddles (k = 1, 3 cost 2 adds + 2 muls each, k = 2 is a swap)
template <bool INV>
__device__ __forceinline__ void dft8(float2 *v) {
    constexpr float R2 = 0.70710678118654752440f;
    float2 e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    dft4<INV>(e);
    dft4<INV>(o);
    // W8 = (1 - i)/sqrt2 forward, (1 + i)/sqrt2 inverse
    const float2 o1 = INV ? make_float2((o[1].x - o[1].y) * R2, (o[1].x + o[1].y) * R2)
                          : make_float2((o[1].x + o[1].y) * R2, (o[1].y - o[1].x) * R2);
    const float2 o2 = mul_mi<INV>(o[2]);
    // W8^3 = (-1 - i)/sqrt2 forward, (-1 + i)/sqrt2 inverse
    const float2 o3 = INV ? make_float2((-o[3].x - o[3].y) * R2, (o[3].x - o[3].y) * R2)
                          : make_float2((o[3].y - o[3].x) * R2, (-o[3].x - o[3].y) * R2);
    v[0] = cadd(e[0], o[0]);
    v[4] = csub(e[0], o[0]);
    v[1] = cadd(e[1], o1);
    v[5] = csub(e[1], o1);
    v[2] = cadd(e[2], o2);
    v[6] = csub(e[2], o2);
    v[3] = cadd(e[3], o3);
    v[7] = csub(e[3], o3);
}

template <bool INV>
__device__ __forceinline__ void dft3(float2 *v) {
    const float h = 0.86602540378443864676f;  // sqrt(3)/2
    float2 t = cadd(v[1], v[2]);
    float2 d = csub(v[1], v[2]);
    float2 m = make_float2(v[0].x - 0.5f * t.x, v[0].y - 0.5f * t.y);
    // forward: y1 = m - i h d, y2 = m + i h d
    float2 ihd = INV ? make_float2(-h * d.y, h * d.x) : make_float2(h * d.y, -h * d.x);  // (-+i) h d
    v[0] = cadd(v[0], t);
    v[1] = cadd(m, ihd);
    v[2] = csub(m, ihd);
}

template <bool INV>
__device__ __forceinline__ void dft5(float2 *v) {
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    float2 t1 = cadd(v[1], v[4]), d1 = csub(v[1], v[4]);
    float2 t2 = cadd(v[2], v[3]), d2 = csub(v[2], v[3]);
    float2 a0 = v[0];
    float2 r1 = make_float2(a0.x + c1 * t1.x + c2 * t2.x, a0.y + c1 * t1.y + c2 * t2.y);
    float2 r2 = make_float2(a0.x + c2 * t1.x + c1 * t2.x, a0.y + c2 * t1.y + c1 * t2.y);
    float2 q1 = make_float2(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y);
    float2 q2 = make_float2(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y);
    float2 iq1 = mul_mi<INV>(q1), iq2 = mul_mi<INV>(q2);
    v[0] = cadd(a0, cadd(t1, t2));
    v[1] = cadd(r1, iq1);
    v[4] = csub(r1, iq1);
    v[2] = cadd(r2, iq2);
    v[3] = csub(r2, iq2);
}

// ---- composite radices R = A*B (A, B in {2, 3, 4, 5}) in registers --------
// One Stockham pass of radix 6/9/10/12/15 replaces two passes of its factors
// (half the LDS round trips and barriers of the small-patch kernel, whose
// Np = 90 = 2*3*3*5 otherwise takes four passes per transform: stockham_t).
// X[k1 + A k2] = sum_n2 W_B^{n2 k2} W_R^{n2 k1} sum_n1 v[B n1 + n2] W_A^{n1 k1}
// with compile-time twiddles W_R^m.
namespace cwt {
constexpr double kPi = 3.14159265358979323846;
// cos / sin by Taylor series of |x| <= pi after reduction (compile time only)
constexpr double csin(double x) {
    double t = x, s = x;
    for (int i = 1; i < 20; ++i) {
        t *= -x * x / ((2 * i) * (2 * i + 1));
        s += t;
    }
    return s;
}
constexpr double ccos(double x) {
    double t = 1, s = 1;
    for (int i = 1; i < 20; ++i) {
        t *= -x * x / ((2 * i - 1) * (2 * i));
        s += t;
    }
    return s;
}
// W_R^m = exp(-2 pi i m / R) as (cos, sin) of the reduced angle
constexpr double wang(int R, int m) {
    const int q = ((m % R) + R) % R;
    const double a = -2.0 * kPi * q / R;
    return a < -kPi ? a + 2.0 * kPi : a;
}
}  // namespace cwt

template <int R, bool INV>
__device__ __forceinline__ void dft_prime(float2 *v) {
    if constexpr (R == 2) dft2<INV>(v);
    if constexpr (R == 3) dft3<INV>(v);
    if constexpr (R == 4) dft4<INV>(v);
    if constexpr (R == 5) dft5<INV>(v);
}

template <int A, int B, bool INV>
__device__ __forceinline__ void dft_ab(float2 *v) {
    constexpr int R = A * B;
    float2 y[R];
#pragma unroll
    for (int n2 = 0; n2 < B; ++n2) {
        float2 t[A];
#pragma unroll
        for (int n1 = 0; n1 < A; ++n1) t[n1] = v[B * n1 + n2];
        dft_prime<A, INV>(t);
#pragma unroll
        for (int k1 = 0; k1 < A; ++k1) {
            if ((n2 * k1) % R == 0) {
                y[k1 * B + n2] = t[k1];
            } else {
                const float c = (float)cwt::ccos(cwt::wang(R, n2 * k1));
                const float sn = (float)cwt::csin(cwt::wang(R, n2 * k1)) * (INV ? -1.f : 1.f);
                y[k1 * B + n2] = cmul(t[k1], make_float2(c, sn));
            }
        }
    }
#pragma unroll
    for (int k1 = 0; k1 < A; ++k1) {
        float2 u[B];
#pragma unroll
        for (int n2 = 0; n2 < B; ++n2) u[n2] = y[k1 * B + n2];
        dft_prime<B, INV>(u);
#pragma unroll
        for (int k2 = 0; k2 < B; ++k2) v[k1 + A * k2] = u[k2];
    }
}

// a / d for 0 <= a < 2^22 via the float reciprocal rd = 1/d and one
// correction step (an integer division by a runtime value costs ~40 VALU
// instructions on CDNA; this is 6)
__device__ __forceinline__ int udiv(int a, int d, float rd) {
    int q = (int)((float)a * rd);
    const int r = a - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

template <int R, bool INV>
__device__ __forceinline__ void stockham_pass(const float2 *__restrict__ a, float2 *__restrict__ b,
                                              int n, int C, int Ns, const float2 *__restrict__ tw,
                                              int tid, int nthr) {
    const int nR = n / R;
    const int tmul = n / (Ns * R);
    const float rNs = 1.0f / (float)Ns, rnR = 1.0f / (float)nR;
    const bool pow2 = (Ns & (Ns - 1)) == 0;
    const int lNs = 31 - __builtin_clz(Ns);
    for (int jj = tid; jj < C * nR; jj += nthr) {
        const int s = (C == 1) ? 0 : udiv(jj, nR, rnR);
        const int j = jj - s * nR;
        const float2 *src = a + s * n;
        float2 *dst = b + s * n;
        const int jq = pow2 ? (j >> lNs) : udiv(j, Ns, rNs);
        const int k = j - jq * Ns;
        float2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = src[j + r * nR];
        if (Ns > 1) {
            const int ts = tmul * k;
#pragma unroll
            for (int r = 1; r < R; ++r) {
                float2 w = tw[r * ts];
                if (INV) w.y = -w.y;
                v[r] = cmul(v[r], w);
            }
        }
        if (R == 2) dft2<INV>(v);
        if (R == 3) dft3<INV>(v);
        if (R == 4) dft4<INV>(v);
        if (R == 5) dft5<INV>(v);
        if (R == 8) dft8<INV>(v);
        if constexpr (R == 6) dft_ab<2, 3, INV>(v);
        if constexpr (R == 9) dft_ab<3, 3, INV>(v);
        if constexpr (R == 10) dft_ab<2, 5, INV>(v);
        if constexpr (R == 12) dft_ab<4, 3, INV>(v);
        if constexpr (R == 15) dft_ab<3, 5, INV>(v);
        const int base = jq * Ns * R + k;
#pragma unroll
        for (int r = 0; r < R; ++r) dst[base + r * Ns] = v[r];
    }
}

// Transforms C sequences of length pl.n stored contiguously (sequence s at
// a + s*n) in LDS; `b` is an equally sized ping-pong buffer.  Unscaled.
// Returns the buffer that holds the result.  All threads of the block must
// call it; it ends with a barrier.
template <bool INV>
__device__ float2 *stockham(float2 *a, float2 *b, int C, const FftPlan &pl,
                            const float2 *__restrict__ tw, int tid, int nthr) {
    int Ns = 1;
    const int n = pl.n;
    for (int st = 0; st < pl.nstages; ++st) {
        const int R = pl.radix[st];
        switch (R) {
            case 8: stockham_pass<8, INV>(a, b, n, C, Ns, tw, tid, nthr); break;
            case 4: stockham_pass<4, INV>(a, b, n, C, Ns, tw, tid, nthr); break;
            case 2: stockham_pass<2, INV>(a, b, n, C, Ns, tw, tid, nthr); break;
            case 3: stockham_pass<3, INV>(a, b, n, C, Ns, tw, tid, nthr); break;
            default: stockham_pass<5, INV>(a, b, n, C, Ns, tw, tid, nthr); break;
        }
        __syncthreads();
        float2 *t = a; a = b; b = t;
        Ns *= R;
    }
    return a;
}

// stockham() with the transform length N and the radices fixed at compile
// time (the small-patch kernel's Np 90 = 10 x 9 instance): no radix switch,
// constant strides and divisors.  Ends with a barrier; returns the result buffer.
template <bool INV, int N, int NS, int R, int... REST>
__device__ __forceinline__ float2 *stockham_t(float2 *a, float2 *b, int C, const float2 *__restrict__ tw, int tid,
                                              int nthr) {
    stockham_pass<R, INV>(a, b, N, C, NS, tw, tid, nthr);
    __syncthreads();
    if constexpr (sizeof...(REST) == 0) {
        return b;
    } else {
        return stockham_t<INV, N, NS * R, REST...>(b, a, C, tw, tid, nthr);
    }
}

// any supported radix in registers
template <int R, bool INV>
__device__ __forceinline__ void dft_any(float2 *v) {
    if constexpr (R == 2 || R == 3 || R == 4 || R == 5) dft_prime<R, INV>(v);
    if constexpr (R == 8) dft8<INV>(v);
    if constexpr (R == 6) dft_ab<2, 3, INV>(v);
    if constexpr (R == 9) dft_ab<3, 3, INV>(v);
    if constexpr (R == 10) dft_ab<2, 5, INV>(v);
    if constexpr (R == 12) dft_ab<4, 3, INV>(v);
    if constexpr (R == 15) dft_ab<3, 5, INV>(v);
}

// stockham_t whose first pass (Ns = 1: no twiddles) takes its inputs from a
// loader ld(s, i) = element i of sequence s instead of an LDS buffer, so a
// gather or a transpose folds into the transform; the first pass writes `a`.
template <bool INV, int N, int R, int... REST, class LD>
__device__ __forceinline__ float2 *stockham_t_ld(const LD &ld, float2 *a, float2 *b, int C,
                                                 const float2 *__restrict__ tw, int tid, int nthr) {
    constexpr int NR = N / R;
    for (int jj = tid; jj < C * NR; jj += nthr) {
        const int s = jj / NR, j = jj - s * NR;
        float2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = ld(s, j + r * NR);
        dft_any<R, INV>(v);
        float2 *dst = a + s * N + j * R;
#pragma unroll
        for (int r = 0; r < R; ++r) dst[r] = v[r];
    }
    __syncthreads();
    if constexpr (sizeof...(REST) == 0) {
        return a;
    } else {
        return stockham_t<INV, N, R, REST...>(a, b, C, tw, tid, nthr);
    }
}

// ---- block reductions -------------------------------------------------------
// Max over the 64 lanes, in every lane; the wave must be fully active.  DPP
// moves within each row of 16 (xor 1 and 2 as quad permutes, then the
// half-row and row mirrors), then the four row maxima by v_readlane: four VALU
// moves instead of six ds_bpermute round trips through the LDS crossbar (the
// __shfl_xor form).  max is exact, so the result is the same in any order.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
// Sum over each row of 16 lanes, in every lane of the row, with exactly the
// association of the xor butterfly o = 8, 4, 2, 1 (after the first step the
// row is 8-periodic, so row_ror:4 reads the value lane ^ 4 holds, and so on):
// bit-identical to the __shfl_xor form.  Each row must be fully active.
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0x128>(v);  // row_ror:8
    v += dpp_f<0x124>(v);  // row_ror:4
    v += dpp_f<0x122>(v);  // row_ror:2
    v += dpp_f<0x121>(v);  // row_ror:1
    return v;
}
// For values >= +0 only (magnitudes, |z|^2, tile maxima -- every caller),
// whose IEEE bits order as unsigned integers: the steps are v_max_u32 (fmaxf
// costs a canonicalising v_max per operand in IEEE mode: three VALU per step
// instead of one) and the four row maxima fold on the scalar unit.  The sign
// bit is cleared on entry, so a misuse with a negative input (or -0) reduces
// |x| -- a bounded result, never a negative value winning as a huge unsigned
// one.  A NaN would win here where fmaxf drops it -- it never reaches a
// maximum of a finite run.
__device__ __forceinline__ float wave_max_nonneg(float x) {
    unsigned v = __float_as_uint(x) & 0x7fffffffu;
    auto dpp_u = [](unsigned u, auto ctrl) {
        // old = 0, the identity of unsigned max: the DPP combiner folds the
        // move into the v_max_u32 that uses it
        return (unsigned)__builtin_amdgcn_update_dpp(0, (int)u, decltype(ctrl)::value, 0xF, 0xF, false);
    };
    v = max(v, dpp_u(v, std::integral_constant<int, 0xB1>{}));   // quad_perm [1,0,3,2]: lane ^ 1
    v = max(v, dpp_u(v, std::integral_constant<int, 0x4E>{}));   // quad_perm [2,3,0,1]: lane ^ 2
    v = max(v, dpp_u(v, std::integral_constant<int, 0x141>{}));  // row_half_mirror: the other quad of the 8
    v = max(v, dpp_u(v, std::integral_constant<int, 0x140>{}));  // row_mirror: the other 8 of the row
    const unsigned r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const unsigned r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return __uint_as_float(max(max(r0, r1), max(r2, r3)));
}

// Max over the block of values >= +0 (wave_max_nonneg); `red` is LDS scratch
// of >= nwaves floats. Result valid in every thread. Contains two barriers.
__device__ __forceinline__ float block_max_nonneg(float v, float *red) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nw = (blockDim.x + 63) >> 6;
    v = wave_max_nonneg(v);
    if (lane == 0) red[w] = v;
    __syncthreads();
    float r = red[0];
    for (int i = 1; i < nw; ++i) r = fmaxf(r, red[i]);
    __syncthreads();
    return r;
}

}  // namespace fpm
